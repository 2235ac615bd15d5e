"""Diagnostic: a few launches of one weight-gradient GEMM (dW[N,K] += dy^T x over M tokens, both operands token-major)
and one forward NT GEMM of the same size, for counter passes (tools/pmc_generic.sh)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
M, N, K = 8192, 2048, 512
dy = torch.randn(M, N, device=dev, dtype=bf)
x = torch.randn(M, K, device=dev, dtype=bf)
dW = torch.zeros(N, K, device=dev)
w = torch.randn(N, K, device=dev, dtype=bf)
for _ in range(5):
    ops.linear_dw(dy, x, out=dW, accumulate=True)
    ops.linear(x, w, out_dtype=bf)
torch.cuda.synchronize()
