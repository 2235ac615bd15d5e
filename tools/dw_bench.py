"""Weight-gradient GEMMs of one decoder block (dW = dY^T X, both operands token-major): the grouped launch as the
train step issues it, each problem alone through ops.linear_dw, and hipBLASLt (torch.matmul on the transposed
views) for the same shapes. HIP-event timing (tools/g128_bench.py's timer). Library from FDDM_HIP_LIB."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from g128_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
M, Me = 32 * 256, 32 * 499
SHAPES = [(M, 1536, 512), (M, 512, 512), (M, 512, 512), (M, 512, 512), (M, 2048, 512), (M, 512, 2048), (Me, 1024, 512)]


def main():
    tag = os.path.basename(os.environ.get("FDDM_HIP_LIB", "in-tree"))
    jobs, fl = [], 0.0
    for (m, a, b) in SHAPES:
        jobs.append((torch.randn(m, a, device=dev, dtype=bf), torch.randn(m, b, device=dev, dtype=bf),
                     torch.zeros(a, b, device=dev), torch.zeros(a, device=dev)))
        fl += 2.0 * m * a * b
    t = timeit(lambda: ops.linear_dw_grouped(jobs))
    print(f"[{tag}] grouped dW ({fl / 1e9:.1f} GFLOP): {t:7.1f} us {fl / t / 1e6:6.0f} TF/s", flush=True)
    if os.environ.get("DW_ALONE"):
        for (dy, x, dW, db) in jobs[:1] + jobs[4:]:
            f = 2.0 * dy.shape[0] * dy.shape[1] * x.shape[1]
            t = timeit(lambda: ops.linear_dw(dy, x, out=dW, accumulate=True, db=db))
            o = torch.empty(dy.shape[1], x.shape[1], device=dev, dtype=bf)
            tl = timeit(lambda: torch.matmul(dy.t(), x, out=o))
            print(f"[{tag}] dW {dy.shape[1]}x{x.shape[1]} over {dy.shape[0]}: ours {t:6.1f} us {f / t / 1e6:5.0f} TF/s"
                  f" | hipBLASLt (bf16 out) {tl:6.1f} us {f / tl / 1e6:5.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
