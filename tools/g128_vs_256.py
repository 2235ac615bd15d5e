"""The decoder's backward dX GEMM shapes (C2: 8192 tokens, d 512, ff 2048) on the 128x128 kernel (all CUs) against
the persistent 256x256 kernel at 256 / 128 / 64 workgroups (the CUs the encoder's side stream leaves the decoder),
NT layout, f32 output. HIP-event timing, 20 launches after 3 warm-ups."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import _lib, ops  # noqa: E402

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


for (M, N, K) in [(8192, 512, 2048), (8192, 512, 1536), (8192, 2048, 512), (8192, 512, 512), (8192, 768, 3072),
                  (8192, 768, 768)]:
    A = torch.randn(M, K, device=dev, dtype=bf)
    W = torch.randn(N, K, device=dev, dtype=bf) / 30
    o = torch.empty(M, N, device=dev, dtype=torch.float32)
    f = lambda: ops.gemm(A, W, o, M, N, K, lda=K, ldb=K, ldc=N)  # noqa: E731
    fl = 2.0 * M * N * K
    ops.gemm_force_path("128")
    t128 = timeit(f)
    line = f"M{M} N{N} K{K}: g128 {t128:6.1f} us {fl / t128 / 1e6:5.0f} TF/s"
    ops.gemm_force_path("256")
    for cap in (256, 128, 64):
        _lib.lib().fddm_gemm_persistent_cap(cap)
        t = timeit(f)
        line += f" | g256@{cap} {t:6.1f} us {fl / t / 1e6:5.0f}"
    _lib.lib().fddm_gemm_persistent_cap(0)
    ops.gemm_force_path("auto")
    print(line, flush=True)
