"""Keep-bit producer (attn7 dmask_kernel) alone: one launch writing 6 sites (the step's per-launch count) at the C2 and
C4 decoder shapes, HIP events over 50 launches. The library comes from FDDM_HIP_LIB (A/B against an abl/*.so).
  python tools/dmask_time.py [tag]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fddm-asr_amd"))
from fddm_hip import ops  # noqa: E402

SHAPES = [("C2 self", 32, 8, 256, 256), ("C2 cross", 32, 8, 256, 499), ("C4 self", 16, 12, 512, 512),
          ("C4 cross", 16, 12, 512, 499)]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.environ.get("FDDM_HIP_LIB", "default"))
    dev = torch.device("cuda:0")
    for name, B, H, Lq, Lk in SHAPES:
        words = ops.drop_words(B, H, Lq, Lk)
        out = torch.empty(6, words, device=dev, dtype=torch.int64)
        run = lambda: ops.attn_drop_bits(out, 6, B, H, Lq, Lk, 0.1, 1, 1, 6)  # noqa: E731
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 50
        nbytes = out.numel() * 8
        print(f"{tag:12s} {name:9s} {us:7.1f} us per 6-site launch  ({nbytes / us / 1e6:.2f} TB/s written, "
              f"{6 * B * H * Lq * Lk / us / 1e6:.2f} T scores/s)", flush=True)


if __name__ == "__main__":
    main()
