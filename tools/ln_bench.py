"""LayerNorm micro-benchmark at the train step's shapes (HIP-event timing): decoder residual+dropout+LN(+FiLM)
forward / fused backward (N = 8192, d = 512, f32 residual) and the WavLM post-LN forward (N = 15968, d = 768,
bf16). Prints us per launch and the achieved rate of the algorithmic bytes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    bf, f32 = torch.bfloat16, torch.float32
    N, d, L = 8192, 512, 256
    x = torch.randn(N, d, device=dev)
    y = torch.randn(N, d, device=dev, dtype=bf)
    g, b = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    fs, fh = torch.zeros(N // L, d, device=dev), torch.zeros(N // L, d, device=dev)
    s, out, m, r = torch.empty_like(x), torch.empty_like(x), torch.empty(N, device=dev), torch.empty(N, device=dev)
    ot = torch.empty(N, d, device=dev, dtype=bf)
    t = timeit(lambda: ops.ln_fwd(x, y, g, b, out_f32=out, out_t=ot, save_s=s, mean=m, rstd=r, film=(fs, fh),
                                  rows_per_batch=L, drop_p=0.1, seed=1, rng_stream=2))
    byt = N * d * (4 + 2 + 4 + 4 + 2)
    print(f"decoder LN fwd (FiLM, dropout)  {t:6.1f} us  {byt / t / 1e3:6.0f} GB/s", flush=True)
    dout = torch.randn(N, d, device=dev)
    dres, dy = torch.empty_like(x), torch.empty(N, d, device=dev, dtype=bf)
    dg, db = torch.zeros(d, device=dev), torch.zeros(d, device=dev)
    dfs, dfh = torch.zeros(N // L, d, device=dev), torch.zeros(N // L, d, device=dev)
    t = timeit(lambda: ops.ln_bwd(dout, s, m, r, g, b, dres=dres, dy_t=dy, dgamma=dg, dbeta=db, film_scale=fs,
                                  dfilm=(dfs, dfh), rows_per_batch=L, drop_p=0.1, seed=1, rng_stream=2))
    byt = N * d * (4 + 4 + 4 + 2)
    print(f"decoder LN bwd (FiLM, dropout)  {t:6.1f} us  {byt / t / 1e3:6.0f} GB/s", flush=True)
    t = timeit(lambda: ops.ln_bwd(dout, s, m, r, g, b, dres=dres, dy_t=dy, dgamma=dg, dbeta=db, drop_p=0.1, seed=1,
                                  rng_stream=2))
    print(f"decoder LN bwd (no FiLM)        {t:6.1f} us  {byt / t / 1e3:6.0f} GB/s", flush=True)
    # the train step's form: slab sums to partials (one ln_fold per block afterwards) instead of atomics
    lp = ops.LnPartials()
    part = lp.add(N, d, dg, db, (dfs, dfh), L)

    def bwd_part():
        ops.call("fddm_ln_bwd", ops.BF16, ops.ptr(dout), ops.ptr(s), ops.ptr(m), ops.ptr(r), ops.ptr(g), ops.ptr(b),
                 ops.ptr(fs), ops.ptr(dres), ops.ptr(dy), ops.ptr(dg), ops.ptr(db), ops.ptr(dfs), ops.ptr(dfh), N, d, L,
                 0.1, 1, 2, ops.ptr(part), ops.stream())
    t = timeit(bwd_part)
    print(f"decoder LN bwd (FiLM, partials) {t:6.1f} us  {byt / t / 1e3:6.0f} GB/s  (the step's form)", flush=True)
    job = lp.jobs[0]

    def fold():
        lp.jobs = [job]
        lp.fold()
    t = timeit(fold)
    print(f"  + ln_fold of its slab sums    {t:6.1f} us", flush=True)
    N4, d4, L4 = 8192, 768, 512   # C4 decoder LN (d 768): FiLM form and the plain f32 -> f32 + bf16 form
    x4 = torch.randn(N4, d4, device=dev)
    y4 = torch.randn(N4, d4, device=dev, dtype=bf)
    g4, b4 = torch.ones(d4, device=dev), torch.zeros(d4, device=dev)
    fs4, fh4 = torch.zeros(N4 // L4, d4, device=dev), torch.zeros(N4 // L4, d4, device=dev)
    s4, o4, m4, r4 = torch.empty_like(x4), torch.empty_like(x4), torch.empty(N4, device=dev), torch.empty(N4, device=dev)
    ot4 = torch.empty(N4, d4, device=dev, dtype=bf)
    t = timeit(lambda: ops.ln_fwd(x4, y4, g4, b4, out_f32=o4, out_t=ot4, save_s=s4, mean=m4, rstd=r4,
                                  film=(fs4, fh4), rows_per_batch=L4, drop_p=0.1, seed=1, rng_stream=2))
    byt = N4 * d4 * (4 + 2 + 4 + 4 + 2)
    print(f"C4 decoder LN fwd (FiLM, drop)  {t:6.1f} us  {byt / t / 1e3:6.0f} GB/s", flush=True)
    t = timeit(lambda: ops.ln_fwd(x4, y4, g4, b4, out_f32=o4, out_t=ot4, save_s=s4, mean=m4, rstd=r4,
                                  drop_p=0.1, seed=1, rng_stream=2))
    print(f"C4 decoder LN fwd (drop)        {t:6.1f} us  {byt / t / 1e3:6.0f} GB/s", flush=True)
    N2, d2 = 15968, 768
    xb = torch.randn(N2, d2, device=dev, dtype=bf)
    yb = torch.randn(N2, d2, device=dev, dtype=bf)
    ob = torch.empty_like(xb)
    g2, b2 = torch.ones(d2, device=dev), torch.zeros(d2, device=dev)
    t = timeit(lambda: ops.ln_fwd(xb, yb, g2, b2, out_t=ob, eps=1e-5))
    byt = N2 * d2 * 6
    print(f"WavLM LN fwd (bf16)             {t:6.1f} us  {byt / t / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
