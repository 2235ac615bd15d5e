"""Per-tile time of the persistent 256x256 GEMM against its workgroup cap (32 .. 256 CUs) at the encoder shapes:
with tools/g256_stamps.py (cycles per K-tile, identical at every cap) it separates clock from cycles — the wall time
per tile rises with the number of busy CUs while the cycle count does not (power-limited clock)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fddm-asr_amd"))
import torch
from fddm_hip import ops, _lib
dev = torch.device("cuda:0"); bf = torch.bfloat16
def timeit(fn, iters=20):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3
ops.gemm_force_path("256")
for (M, N, K, epi) in [(15968, 3072, 768, 0), (15968, 3072, 768, 3), (15968, 768, 3072, 0), (15968, 3072, 3072, 0)]:
    A = torch.randn(M, K, device=dev, dtype=bf); W = torch.randn(N, K, device=dev, dtype=bf) / 30
    o = torch.empty(M, N, device=dev, dtype=bf)
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    line = f"M{M} N{N} K{K} epi{epi} tiles {tiles}:"
    for cap in (32, 64, 128, 192, 256):
        _lib.lib().fddm_gemm_persistent_cap(cap)
        us = timeit(lambda: ops.gemm(A, W, o, M, N, K, lda=K, ldb=K, ldc=N, epi=epi))
        line += f" | cap {cap}: {us:7.1f} us, {us * cap / tiles:5.2f} us/tile, {2*M*N*K/us/1e6*256/cap:5.0f} TF/s-eq"
    print(line, flush=True)
