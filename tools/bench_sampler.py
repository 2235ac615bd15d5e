"""C5 benchmark (BASELINE.json configs[4]): jumpy-sampler inference RTF on one MI355X.

B=64 x 10 s synthetic audio, WavLM-base encoder + 6-layer d512/H8 decoder (random init), V=8000,
T_train=200, T_infer=20, r=5, exact posterior, greedy, seq_len 256; the denoise loop is replayed from
a HIP graph. RTF = (encoder + sampler wall time) / audio seconds (lower is better). Prints one JSON
line. The reference's CPU figure: RTF 0.0637 on 8 host cores.

  python tools/bench_sampler.py [--batch 64] [--iters 5] [--no-graph]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--seq-len", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--precision", default="bf16")
    args = ap.parse_args()
    import train as T_
    from fddm_hip import runtime as rt
    from sampler.jumpy_sampler import DiffusionJumpySampler
    dev = torch.device("cuda:0")
    rt.set_precision(args.precision)
    torch.manual_seed(1337)
    cfg = T_.Config(seed=1337, data={"pad_id": 0, "vocab_size": 8000},
                    model={"d_model": 512, "nhead": 8, "num_layers": 6, "dim_ff": 2048, "dropout": 0.1,
                           "encoder": {"wavlm_name": {}, "freeze": True, "proj": "linear", "pooling": "none"},
                           "projector": {"d_proj": 256}},
                    diffusion={"T": 200, "beta_max": 0.2}, inference={}, optim={}, lfd={}, log={})
    enc, dec, sp, te, tp, sch = T_.build_models(cfg, dev)
    enc.eval()
    dec.eval()
    smp = DiffusionJumpySampler(sch.sch, dec, K=8000, T_train=200, T_infer=20, r=5, greedy=True, posterior_mode="map",
                                sampling_mode="exact", device=dev)
    wave = 0.1 * torch.randn(args.batch, int(16000 * args.seconds), device=dev)
    graph = not args.no_graph

    def run():
        with torch.no_grad():
            c, _, _ = enc(wave)
            x0, _ = smp.sample(c, seq_len=args.seq_len, graph=graph, return_probs=False)
        return c, x0

    run()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_enc = t_smp = 0.0
    t0 = time.perf_counter()
    for _ in range(args.iters):
        e[0].record()
        with torch.no_grad():
            c, _, _ = enc(wave)
        e[1].record()
        with torch.no_grad():
            x0, _ = smp.sample(c, seq_len=args.seq_len, graph=graph, return_probs=False)
        e[2].record()
        torch.cuda.synchronize()
        t_enc += e[0].elapsed_time(e[1])
        t_smp += e[1].elapsed_time(e[2])
    wall = (time.perf_counter() - t0) / args.iters
    audio = args.batch * args.seconds
    print(json.dumps({
        "metric": "jumpy-sampler RTF (C5: B=64 x 10 s, T_infer=20, r=5, exact, greedy, seq 256)",
        "value": round(wall / audio, 6), "unit": "RTF (s compute / s audio)", "higher_is_better": False,
        "ms_per_batch": round(1000 * wall, 3), "encoder_ms": round(t_enc / args.iters, 3),
        "sampler_ms": round(t_smp / args.iters, 3), "graph": graph, "dtype": args.precision,
        "vs_reference_cpu_rtf": 0.0637, "data": "synthetic (random-init weights)",
        "config": {"workload": "C5", "batch": args.batch, "audio_seconds": args.seconds, "seq_len": args.seq_len}}),
        flush=True)


if __name__ == "__main__":
    main()
