"""The decoder block's dX GEMMs at C2 (B 32 x L 256, d 512, FF 2048) as DecoderBlockFn.backward issues them
(functions.py), each timed alone (HIP events, 20 launches after 3 warm-ups) next to its FLOP rate and its HBM floor
(operand + output bytes at 6.3 TB/s achievable). Library from FDDM_HIP_LIB.
   python tools/dx_bench.py [gemm path]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from g128_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
bf, f32 = torch.bfloat16, torch.float32


def main():
    if len(sys.argv) > 1:   # a GEMM family forced for every case (ops.GEMM_PATHS), e.g. "small"
        ops.gemm_force_path(sys.argv[1])
    N, d, FF = 32 * 256, 512, 2048
    r = lambda *s, dt=bf: torch.randn(*s, device=dev, dtype=dt)  # noqa: E731
    dy3, hpre, dh = r(N, d), r(N, FF), torch.empty(N, FF, device=dev, dtype=bf)
    wf3, wf0, wco, wca, wsa = r(d, FF) * 0.02, r(FF, d) * 0.02, r(d, d) * 0.02, r(d, d) * 0.02, r(3 * d, d) * 0.02
    dx = torch.zeros(N, d, device=dev)
    dqk, dqc = r(N, 2 * d), r(N, d)
    cases = [
        ("FF2 dX, dGELU + dropout epilogue -> bf16", lambda: ops.linear_dx(dy3, wf3, out=dh, epi=ops.EPI_DGELU, C2=hpre,
                                                                          drop_p=0.1, seed=1, rng_stream=5),
         N * FF * d, (N * d + d * FF + 2 * N * FF) * 2),
        ("FF2 dX shape, plain bf16 store (no epilogue)", lambda: ops.linear_dx(dy3, wf3, out=dh), N * FF * d,
         (N * d + d * FF + N * FF) * 2),
        ("FF2 dX shape, dGELU without dropout", lambda: ops.linear_dx(dy3, wf3, out=dh, epi=ops.EPI_DGELU, C2=hpre),
         N * FF * d, (N * d + d * FF + 2 * N * FF) * 2),
        ("FF1 dX, f32 accumulate (K 2048)", lambda: ops.linear_dx(dh, wf0, out=dx, accumulate=True),
         N * d * FF, (N * FF + FF * d) * 2 + 2 * N * d * 4),
        ("cross out-proj dX -> bf16", lambda: ops.linear_dx(dy3, wco, out_dtype=bf), N * d * d, (2 * N * d + d * d) * 2 + N * d * 2),
        ("cross Q dX, f32 accumulate", lambda: ops.linear_dx(dqc, wca, out=dx, accumulate=True), N * d * d,
         (N * d + d * d) * 2 + 2 * N * d * 4),
        ("self QK dX (K 1024) -> f32", lambda: ops.linear_dx(dqk, wsa[:2 * d]), N * d * 2 * d,
         (N * 2 * d + 2 * d * d) * 2 + N * d * 4),
    ]
    for name, fn, mnk, byt in cases:
        t = timeit(fn)
        print(f"{name:44s} {t:6.1f} us  {2.0 * mnk / t / 1e6:6.0f} TF/s  HBM floor {byt / 6.3e6:5.1f} us", flush=True)


if __name__ == "__main__":
    main()
