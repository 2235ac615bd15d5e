"""Micro-benchmark of the libfddm_hip GEMM at the train step's shapes (HIP-event timing, bf16)."""
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


def report(name, flops, ms):
    print(f"{name:48s} {ms*1e3:9.1f} us  {flops/ms/1e9:8.1f} TF/s", flush=True)


def report_paths(name, flops, fn, paths=("auto", "256", "big")):
    """time fn under each FDDM_GEMM_PATH (read per launch by the library)"""
    cells = []
    for p in paths:
        if p == "auto":
            os.environ.pop("FDDM_GEMM_PATH", None)
        else:
            os.environ["FDDM_GEMM_PATH"] = p
        ms = timeit(fn)
        cells.append(f"{p}:{ms*1e3:8.1f} us {flops/ms/1e9:7.1f} TF/s")
    os.environ.pop("FDDM_GEMM_PATH", None)
    print(f"{name:40s} " + " | ".join(cells), flush=True)


def main():
    only = sys.argv[1] if len(sys.argv) > 1 else ""
    B, T0, C = 32, 31999, 512
    T1 = (T0 - 3) // 2 + 1
    if not only or only == "conv":
        x = torch.randn(B, T0, C, device=dev, dtype=bf)
        W = torch.randn(C, 3 * C, device=dev, dtype=bf) / 40
        out = torch.empty(B, T1, C, device=dev, dtype=bf)
        f = lambda: ops.conv1d_gemm(x, W, out, lda=C, sAb=T0 * C, Tin=T0, Cg=C, cstride=2, cpad=0, Bn=B, Tout=T1,  # noqa
                                    N=C, K=3 * C, gelu=True)
        report_paths("conv1 implicit GEMM 511968x512x1536", 2 * B * T1 * C * 3 * C, f)
    shapes = [("square 8192^3", 8192, 8192, 8192, ops.EPI_STORE),
              ("enc FF1 15968x3072x768 GELU", 15968, 3072, 768, ops.EPI_GELU_ONLY),
              ("enc QKV 15968x2304x768", 15968, 2304, 768, ops.EPI_STORE),
              ("enc FF2 15968x768x3072", 15968, 768, 3072, ops.EPI_STORE),
              ("dec FF1 8192x2048x512", 8192, 2048, 512, ops.EPI_STORE),
              ("dec out 8192x512x512", 8192, 512, 512, ops.EPI_STORE),
              ("dec head 8192x8000x512 f32out", 8192, 8000, 512, -1)]
    for name, M, N, K, epi in shapes:
        if only and only != "fwd":
            break
        A = torch.randn(M, K, device=dev, dtype=bf)
        Wt = torch.randn(N, K, device=dev, dtype=bf) / 30
        o = torch.empty(M, N, device=dev, dtype=torch.float32 if epi < 0 else bf)
        e = ops.EPI_STORE if epi < 0 else epi
        f = lambda: ops.gemm(A, Wt, o, M, N, K, lda=K, ldb=K, ldc=N, epi=e)  # noqa: E731
        report_paths(name, 2 * M * N * K, f, paths=("auto", "256", "128", "big"))
    dws = [("dW dec FF1 2048x512 (K=8192)", 2048, 512, 8192), ("dW dec out 512x512 (K=8192)", 512, 512, 8192),
           ("dW head 8000x512 (K=8192)", 8000, 512, 8192), ("dW cross kv 1024x512 (K=15968)", 1024, 512, 15968)]
    for name, M, N, K in dws:
        if only and only != "dw":
            break
        dy = torch.randn(K, M, device=dev, dtype=bf)
        x = torch.randn(K, N, device=dev, dtype=bf)
        o = torch.empty(M, N, device=dev)
        db = torch.empty(M, device=dev)
        f = lambda: ops.linear_dw(dy, x, out=o, db=db)  # noqa: E731
        report_paths(name, 2 * M * N * K, f, paths=("auto", "small"))
    if not only or only == "dw":
        # the 8 weight-gradient GEMMs of one C2 decoder block in one grouped launch
        T, d, FF, TS = 8192, 512, 2048, 15968
        specs = [(T, d, FF), (T, FF, d), (T, d, d), (T, d, d), (TS, 2 * d, d), (T, d, d), (T, 2 * d, d), (T, d, d)]
        jobs, fl = [], 0
        for K, M, N in specs:
            jobs.append((torch.randn(K, M, device=dev, dtype=bf), torch.randn(K, N, device=dev, dtype=bf),
                         torch.zeros(M, N, device=dev), torch.zeros(M, device=dev)))
            fl += 2 * M * N * K
        for kc in (0, 8192, 4096):
            f = lambda: ops.linear_dw_grouped(jobs, kchunk=kc)  # noqa: E731
            report(f"dW grouped block (8 GEMMs) kchunk {kc}", fl, timeit(f))

        def seq():
            for dy, x, o, db in jobs:
                ops.linear_dw(dy, x, out=o, accumulate=True, db=db)
        report("dW block as 8 split-K launches", fl, timeit(seq))
    dxs = [("dX dec FF1 8192x512 (K=2048)", 8192, 512, 2048), ("dX dec out 8192x512 (K=512)", 8192, 512, 512),
           ("dX dec qkv 8192x512 (K=1536)", 8192, 512, 1536), ("dX cross kv 15968x512 (K=1024)", 15968, 512, 1024),
           ("dX dec FF2 8192x2048 (K=512)", 8192, 2048, 512), ("dX head 8192x512 (K=8000, f32 A)", 8192, 512, 8000)]
    for name, M, N, K in dxs:
        if only and only != "dx":
            break
        dy = torch.randn(M, K, device=dev, dtype=torch.float32 if "f32" in name else bf)
        w = torch.randn(K, N, device=dev, dtype=bf)
        o = torch.empty(M, N, device=dev)
        f = lambda: ops.linear_dx(dy, w, out=o)  # noqa: E731
        report_paths(name, 2 * M * N * K, f, paths=("auto", "small"))


if __name__ == "__main__":
    main()
