"""Diagnostic: per-K-tile cycle stamps of the 256x256 GEMM (library built with -DG256_STAMPS=64, loaded via
FDDM_HIP_LIB). Prints, per K-tile index, the median over workgroups of the cycles that K-tile took."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fddm_hip import _lib, ops  # noqa: E402

NS = 64
M, N, K = (int(a) for a in sys.argv[1:4])
EPI = int(sys.argv[4]) if len(sys.argv) > 4 else 0
__import__("fddm_hip.ops", fromlist=["ops"]).gemm_force_path("256")
dev = torch.device("cuda:0")
A = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) / 30
o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
cap = int(os.environ.get("G256_CAP", "0"))
if cap:
    _lib.lib().fddm_gemm_persistent_cap(cap)
C2 = torch.empty_like(o) if EPI == 1 else None  # EPI_GELU writes a second output
for _ in range(5):
    ops.gemm(A, W, o, M, N, K, lda=K, ldb=K, ldc=N, epi=EPI, C2=C2)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (256 * NS))()
f = _lib.lib().fddm_gemm256_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_long]
assert f(buf, 256 * NS) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(256, NS).astype(np.int64)
d = np.diff(st, axis=1)
ok = (st[:, 1:] > 0) & (st[:, :-1] > 0)
nk = K // 64
print(f"M{M} N{N} K{K} epi{EPI} nk={nk} cap={cap}: median cycles per K-tile (column = K-tile index within the workgroup)")
med = [int(np.median(d[ok[:, j], j])) if ok[:, j].any() else -1 for j in range(NS - 1)]
for j in range(0, NS - 1, 8):
    print(" ".join(f"{v:7d}" for v in med[j:j + 8]))
