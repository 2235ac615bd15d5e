"""Diagnostic: s_memtime stamps of the 128x128 GEMM (library variant built with -DG128_STAMPS=48, loaded via
FDDM_HIP_LIB): kernel start skew, prologue (first K-tile landed), per-K-tile cycles, epilogue, per workgroup."""
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
__import__("fddm_hip.ops", fromlist=["ops"]).gemm_force_path("128")


def run(name, fn, nblk):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (2048 * NS))()
    assert lib().fddm_gemm128_stamps(buf, ctypes.c_long(2048 * NS)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(2048, NS)[:nblk].astype(np.int64)
    t0 = a[:, 0].min()
    start = a[:, 0] - t0
    pro = a[:, 1] - a[:, 0]
    epi = a[:, NS - 1] - a[:, NS - 2]
    end = a[:, NS - 1] - t0
    print(f"{name}: blocks {nblk}  start skew med {np.median(start):.0f} max {start.max()}  prologue med "
          f"{np.median(pro):.0f}  epilogue med {np.median(epi):.0f}  end med {np.median(end):.0f} max {end.max()}")
    return a


def t0s(a):
    return a[:, 0].min()


def grouped():
    """one decoder block's weight-gradient group (tools/g128_bench.py shapes): per-block durations (cycles)"""
    bf = torch.bfloat16
    M, Me = 32 * 256, 32 * 499
    shapes = [(M, 1536, 512), (M, 512, 512), (M, 512, 512), (M, 512, 512), (M, 2048, 512), (M, 512, 2048),
              (Me, 1024, 512)]
    jobs = [(torch.randn(m, a, device=dev, dtype=bf), torch.randn(m, b, device=dev, dtype=bf),
             torch.zeros(a, b, device=dev), torch.zeros(a, device=dev)) for (m, a, b) in shapes]
    for _ in range(3):
        ops.linear_dw_grouped(jobs)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (2048 * NS))()
    assert lib().fddm_gemm128_stamps(buf, ctypes.c_long(2048 * NS)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(2048, NS).astype(np.int64)
    a = a[a[:, 0] > 0]
    if os.environ.get("G128_FINE"):
        f = a[:, 2:42].reshape(-1, 8, 5)
        d = np.diff(f, axis=2)
        nxt = f[:, 1:, 0] - f[:, :-1, 4]
        ok = (d > 0).all(axis=(1, 2)) & (d < 100000).all(axis=(1, 2))
        d, nxt = d[ok], nxt[ok]
        print("grouped fine (median cycles over %d blocks): reads+lgkm %.0f | vmcnt %.0f | bar1 %.0f | mfma %.0f | "
              "bar2 %.0f" % (ok.sum(), np.median(d[:, :, 0]), np.median(d[:, :, 1]), np.median(d[:, :, 2]),
                             np.median(d[:, :, 3]), np.median(nxt)))
        print("   vmcnt p90 %.0f, reads p90 %.0f" % (np.percentile(d[:, :, 1], 90), np.percentile(d[:, :, 0], 90)))
        return
    tot = a[:, NS - 1] - a[:, 0]
    pro = a[:, 1] - a[:, 0]
    epi = a[:, NS - 1] - a[:, NS - 2]
    print(f"grouped dW: {len(a)} blocks stamped; block cycles med {np.median(tot):.0f} min {tot.min()} max {tot.max()}; "
          f"prologue med {np.median(pro):.0f}; epilogue med {np.median(epi):.0f} p90 {np.percentile(epi, 90):.0f}")
    d = np.diff(a[:, 2:NS - 4], axis=1)
    d = d[(d > 0) & (d < 100000)]
    print(f"   K-tile cycles: med {np.median(d):.0f} p10 {np.percentile(d, 10):.0f} p90 {np.percentile(d, 90):.0f}")


def main():
    if os.environ.get("G128_GROUPED"):
        return grouped()
    bf = torch.bfloat16
    if os.environ.get("G128_FWD"):  # forward-type NT GEMMs with a bf16 STORE epilogue (V / out / cross-Q projections)
        for (M, N, K) in [(8192, 512, 512), (8192, 512, 64), (8192, 2048, 64)]:
            x = torch.randn(M, K, device=dev, dtype=bf)
            w = torch.randn(N, K, device=dev, dtype=bf)
            o = torch.empty(M, N, device=dev, dtype=bf)
            a = run(f"fwd {M}x{N}x{K}", lambda: ops.linear(x, w, out=o), (M // 128) * (N // 128))
            kt = min(K // 64, NS - 4)
            d = np.diff(a[:, 1:2 + kt], axis=1)
            print("   per-K-tile cycles (median over blocks):", " ".join(f"{int(x)}" for x in np.median(d, axis=0)))
            e = a[:, NS - 1] - t0s(a)
            print("   end time per round of 256 blocks (median):",
                  " ".join(f"{int(np.median(e[r:r + 256]))}" for r in range(0, len(a), 256)))
        return
    for (M, N, K) in [(8192, 512, 2048), (8192, 512, 512), (8192, 2048, 512)]:
        dy = torch.randn(M, K, device=dev, dtype=bf)
        w = torch.randn(K, N, device=dev, dtype=bf)
        o = torch.empty(M, N, device=dev)
        a = run(f"dX {M}x{N}x{K}", lambda: ops.linear_dx(dy, w, out=o), (M // 128) * (N // 128))
        if os.environ.get("G128_DW"):  # weight gradient of the same shapes: dW[K, N] += dy^T x (MC x MC)
            x = torch.randn(M, N, device=dev, dtype=bf)
            dW = torch.zeros(K, N, device=dev)
            a = run(f"dW {K}x{N} over {M} tokens", lambda: ops.linear_dw(dy, x, out=dW, accumulate=True),
                    min(2048, (K // 128) * (N // 128) * 8))
        nk = K // 64
        if os.environ.get("G128_FINE"):
            f = a[:, 2:42].reshape(-1, 8, 5)
            st = np.concatenate([np.diff(f, axis=2), (f[:, 1:, :1] - f[:, :-1, 4:5])], axis=None) if False else None
            d = np.diff(f, axis=2)                     # read->lgkm, lgkm->vm, vm->bar1, bar1->mma end
            nxt = f[:, 1:, 0] - f[:, :-1, 4]            # mma end -> bar2 -> next top
            print("   fine (median cycles): reads+lgkm %.0f | vmcnt %.0f | bar1 %.0f | mfma %.0f | bar2 %.0f" %
                  (np.median(d[:, :, 0]), np.median(d[:, :, 1]), np.median(d[:, :, 2]), np.median(d[:, :, 3]),
                   np.median(nxt)))
            continue
        kt = min(nk, NS - 4)
        d = np.diff(a[:, 2:2 + kt], axis=1)
        print("   per-K-tile cycles (median over blocks):", " ".join(f"{int(x)}" for x in np.median(d, axis=0)))
        last = a[:, NS - 2] - a[:, 2 + kt - 1]
        print(f"   last stamped K-tile -> epilogue start: med {np.median(last):.0f} ({nk - kt + 1} K-tiles)")


if __name__ == "__main__":
    main()
