"""WavLM conv feature extractor layers 1..6 at the C2 batch (32 x 10 s) on the persistent gemm256 implicit-GEMM path:
HIP-event time per launch (random bf16 activations, GELU epilogue) at a workgroup cap of 128 (the train step's conv
cap beside the decoder) and 256 (whole chip), with TFLOP/s and the fraction of the 2.5 PF/s dense bf16 peak.
  python tools/conv_bench.py [iters]     (FDDM_HIP_LIB=<variant .so> to time another build)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops, _lib  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    B, C = 32, 512
    T = (160000 - 10) // 5 + 1
    g = torch.Generator(device=dev).manual_seed(0)
    tot = {128: 0.0, 256: 0.0}
    for i, (k, s) in enumerate(((3, 2), (3, 2), (3, 2), (3, 2), (2, 2), (2, 2)), start=1):
        Tout = (T - k) // s + 1
        x = torch.randn(B, T, C, device=dev, dtype=bf, generator=g)
        W = (torch.randn(C, k * C, device=dev, dtype=bf, generator=g) / (k * C) ** 0.5).to(bf)
        out = torch.empty(B, Tout, C, device=dev, dtype=bf)
        fl = 2.0 * B * Tout * C * k * C
        line = f"conv{i} T{T}->{Tout} K{k * C}:"
        for cap in (128, 256):
            _lib.lib().fddm_gemm_persistent_cap(cap)
            us = timeit(lambda: ops.conv1d_gemm(x, W, out, lda=C, sAb=T * C, Tin=T, Cg=C, cstride=s, cpad=0, Bn=B,
                                                Tout=Tout, N=C, K=k * C, gelu=True), iters)
            tot[cap] += us
            tf = fl / us / 1e6
            line += f" | cap {cap}: {us:8.1f} us {tf:6.0f} TF/s {tf / 2500:.3f}"
        print(line, flush=True)
        T = Tout
        del x, W, out
    _lib.lib().fddm_gemm_persistent_cap(0)
    print(f"layers 1-6 total: cap 128 {tot[128]:.1f} us, cap 256 {tot[256]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
