"""Diagnostic: per-K-tile cycles (s_memtime stamps, library built with -DG128_STAMPS=48) of the weight-gradient
GEMM (both operands token-major) over output sizes and token counts, to see what sets the K-loop rate."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from fddm_hip._lib import lib  # noqa: E402

NS = 48
dev = torch.device("cuda:0")
bf = torch.bfloat16
os.environ["FDDM_GEMM_PATH"] = "128"
cases = [("dW", 512, 512, 8192), ("dW", 2048, 512, 8192), ("dX", 512, 2048, 8192), ("dX", 2048, 512, 8192),
         ("fwd", 512, 2048, 8192), ("fwd", 2048, 512, 8192)]
for (kind, N, K, M) in cases:
    if kind == "dW":     # dW[N, K] += dy[M, N]^T x[M, K]: both operands token-major (MC x MC)
        dy = torch.randn(M, N, device=dev, dtype=bf)
        x = torch.randn(M, K, device=dev, dtype=bf)
        dW = torch.zeros(N, K, device=dev)
        fn = lambda: ops.linear_dw(dy, x, out=dW, accumulate=True)  # noqa: E731
    elif kind == "dX":   # dX[M, K] = dy[M, N] W[N, K]: W as stored (KC x MC)
        dy = torch.randn(M, N, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf)
        o = torch.empty(M, K, device=dev)
        fn = lambda: ops.linear_dx(dy, w, out=o)  # noqa: E731
    else:                # y[M, N] = x[M, K] W[N, K]^T (KC x KC)
        x = torch.randn(M, K, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf)
        fn = lambda: ops.linear(x, w, out_dtype=bf)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (2048 * NS))()
    assert lib().fddm_gemm128_stamps(buf, ctypes.c_long(2048 * NS)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(2048, NS).astype(np.int64)
    a = a[a[:, 0] > 0]
    d = np.diff(a[:, 3:20], axis=1)
    d = d[(d > 0) & (d < 100000)]
    print(f"{kind} N={N} K={K} M={M}: ~{len(a)} blocks, K-tile cycles med {np.median(d):.0f} p10 {np.percentile(d, 10):.0f} "
          f"p90 {np.percentile(d, 90):.0f}", flush=True)
    buf2 = (ctypes.c_ulonglong * (2048 * NS))()   # clear for the next case
    ctypes.memset(buf2, 0, ctypes.sizeof(buf2))
