"""K-sweep of the 256x256 GEMM (fixed overhead per tile vs per-K-tile cost); library from FDDM_HIP_LIB."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

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
    return s.elapsed_time(e) / iters


tag = os.path.basename(os.environ.get("FDDM_HIP_LIB", "base"))
__import__("fddm_hip.ops", fromlist=["ops"]).gemm_force_path("256")
for (M, N, K, epi) in [(15968, 3072, 256, 0), (15968, 3072, 768, 0), (15968, 3072, 1536, 0), (15968, 3072, 3072, 0),
                       (15968, 3072, 768, 3), (15968, 2304, 768, 0), (15968, 768, 3072, 0), (8192, 8192, 8192, 0),
                       (4096, 4096, 4096, 0)]:
    A = torch.randn(M, K, device=dev, dtype=bf)
    W = torch.randn(N, K, device=dev, dtype=bf) / 30
    o = torch.empty(M, N, device=dev, dtype=bf)
    f = lambda: ops.gemm(A, W, o, M, N, K, lda=K, ldb=K, ldc=N, epi=epi)  # noqa: E731
    ms = timeit(f)
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    print(f"{tag:14s} M{M} N{N} K{K} epi{epi} tiles {tiles:5d}: {ms*1e3:8.1f} us {2*M*N*K/ms/1e9:7.1f} TF/s "
          f"per-round {ms*1e3/((tiles+255)//256):7.2f} us", flush=True)
