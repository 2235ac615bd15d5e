"""bf16 GEMM micro-benchmark at the train step's shapes: libfddm_hip (ops.linear) vs torch's library GEMM
(F.linear -> hipBLASLt) as a yardstick. HIP-event timing, 20 back-to-back launches after 3 warm-ups."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    M = 32 * 499
    cases = [("wavlm qkv+gate", M, 2400, 768), ("wavlm out", M, 768, 768), ("wavlm ff1", M, 3072, 768),
             ("wavlm ff2", M, 768, 3072), ("wavlm featproj", M, 768, 512),
             ("dec qkv", 32 * 256, 1536, 512), ("dec ff1", 32 * 256, 2048, 512), ("dec ff2", 32 * 256, 512, 2048),
             ("dec head", 32 * 256, 8000, 512), ("dec cross kv", M, 1024, 512)]
    for name, m, n, k in cases:
        x = torch.randn(m, k, device=dev, dtype=bf)
        w = torch.randn(n, k, device=dev, dtype=bf) * 0.02
        b = torch.randn(n, device=dev, dtype=torch.float32)
        bb = b.to(bf)
        fl = 2.0 * m * n * k
        t_ours = timeit(lambda: ops.linear(x, w, b, out_dtype=bf))
        t_lib = timeit(lambda: F.linear(x, w, bb))
        print(f"{name:16s} M={m:6d} N={n:5d} K={k:5d} | ours {t_ours:7.1f} us {fl/t_ours/1e6:6.0f} TF/s | "
              f"hipBLASLt {t_lib:7.1f} us {fl/t_lib/1e6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
