"""Round-4 experiment: the one-wave-per-SIMD 256x256 GEMM (csrc/gemm1w.hip, fddm_gemm1w_probe) against the production
persistent 256x256 kernel (gemm256, forced via ops.gemm_force_path("256")) at the encoder's GEMM shapes; checks the
probe's result against torch first. HIP-event timing, 20 back-to-back launches after 3 warm-ups.
   python tools/g1w_bench.py [grid ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from fddm_hip._lib import call  # noqa: E402

dev = torch.device("cuda:0")
VARIANTS = (1, 2, 3)   # 3: K-loop without DMA (timing only)
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


def g1w(x, w, out, bias, grid, variant=0):
    M, K = x.shape
    N = w.shape[0]
    call("fddm_gemm1w_probe", x.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N,
         None if bias is None else bias.data_ptr(), M, N, K, grid, variant, torch.cuda.current_stream().cuda_stream)


def main():
    grids = [int(a) for a in sys.argv[1:]] or [256]
    M = 32 * 499
    cases = [("ff1", M, 3072, 768), ("qkv+gate", M, 2304, 768), ("out", M, 768, 768), ("ff2", M, 768, 3072),
             ("8192^3", 8192, 8192, 8192)]
    torch.manual_seed(0)
    for name, m, n, k in cases:
        x = torch.randn(m, k, device=dev, dtype=bf)
        w = torch.randn(n, k, device=dev, dtype=bf) * 0.05
        b = torch.randn(n, device=dev, dtype=torch.float32)
        ref = (x.float() @ w.float().t() + b)
        for bias, var in ((None, 0), (b, 0), (b, 1), (None, 2), (b, 2)):
            out = torch.empty(m, n, device=dev, dtype=bf)
            g1w(x, w, out, bias, grids[0], var)
            torch.cuda.synchronize()
            r = ref if bias is not None else ref - b
            err = ((out.float() - r).abs().max() / r.abs().max()).item()
            print(f"{name:9s} bias={bias is not None} variant {var} max rel err {err:.2e}", flush=True)
            assert err < 1e-2, (name, err)
        fl = 2.0 * m * n * k
        out = torch.empty(m, n, device=dev, dtype=bf)
        old = ops.gemm_force_path("256")
        t256 = timeit(lambda: ops.linear(x, w, b, out=out))
        ops.gemm_force_path(old)
        line = f"{name:9s} M={m:6d} N={n:5d} K={k:5d} | gemm256 {t256:7.1f} us {fl/t256/1e6:5.0f} TF/s"
        for gr in grids:
            for var in VARIANTS:
                t0 = timeit(lambda: g1w(x, w, out, None, gr, var))
                t1 = timeit(lambda: g1w(x, w, out, b, gr, var))
                line += f" | v{var}[{gr}] {fl/t0/1e6:5.0f} TF/s, +bias {fl/t1/1e6:5.0f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
