"""Micro-benchmark: token-embedding backward (dE scatter-add + time-bias sums) at the C2 shapes
(8192 tokens, d 512, V 8000, L 256), HIP-event timing."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, L, d, V = 32, 256, 512, 8000
    tok = torch.randint(0, V, (B * L,), device=dev)
    dx = torch.randn(B * L, d, device=dev)
    dE = torch.zeros(V, d, device=dev)
    dtb = torch.zeros(B, d, device=dev)
    f = lambda: ops.embed_bwd(tok, dx, dE, dtb, L, 0)  # noqa: E731
    for _ in range(5):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        f()
    e.record()
    torch.cuda.synchronize()
    print(f"embed_bwd {s.elapsed_time(e) / 50 * 1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
