"""Run one 256x256-path GEMM shape a few times (for rocprofv3 PMC passes): g256_one.py M N K [iters]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

M, N, K = (int(a) for a in sys.argv[1:4])
it = int(sys.argv[4]) if len(sys.argv) > 4 else 5
os.environ.setdefault("FDDM_GEMM_PATH", "256")
dev = torch.device("cuda:0")
A = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) / 30
o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for _ in range(it):
    ops.gemm(A, W, o, M, N, K, lda=K, ldb=K, ldc=N)
torch.cuda.synchronize()
print("done", M, N, K)
