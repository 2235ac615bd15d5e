"""Per-phase GPU timeline of the overlapped C2 train step (bench.py's build, no profiler): HIP events on the main
stream around the decoder forward, KL, backward and clip+AdamW, and on the side stream around each encoder replay.
Prints the average offsets (ms) of every phase boundary from the start of step i's decoder forward, and where
batch i+1's encoder starts and ends on that clock."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from fddm_hip import graphs as G  # noqa: E402


def main():
    dec_only = "--dec-only" in sys.argv
    sys.argv = [a for a in sys.argv if a != "--dec-only"]
    args = bench.parse()
    dev = torch.device("cuda:0")
    T_, cfg, models, opt = bench.build(args, dev)
    enc, dec, sp, te, tp, sch = models
    n = 16
    batches = bench.synthetic_batches(args, dev, 4, 1000)
    ev = []

    def mark(tag):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append((tag, e))

    run0 = G.GraphedEncoder.run

    def run(self, wave, slot, cap=0):
        mark("enc0")
        out = run0(self, wave, slot, cap)
        mark("enc1")
        return out
    G.GraphedEncoder.run = run
    f0 = dec.forward

    def fwd(*a, **k):
        mark("dec0")
        out = f0(*a, **k)
        mark("dec1")
        return out
    dec.forward = fwd
    k0 = sch.kl_term

    def kl(*a, **k):
        out = k0(*a, **k)
        mark("kl1")
        return out
    sch.kl_term = kl
    c0 = opt.clip_and_step

    def step(*a, **k):
        mark("bwd1")
        out = c0(*a, **k)
        mark("opt1")
        return out
    opt.clip_and_step = step
    if dec_only:      # the decoder step alone on the whole chip: the condition precomputed (no encoder stream)
        with torch.no_grad():
            cs = [enc(b[0])[0].clone() for b in batches]

        def fake_encoded(encoder, loader, device, optimizer):
            for k, (wave, x0) in enumerate(loader):
                mark("enc0")
                mark("enc1")
                yield cs[k % 4], None, x0
        T_._encoded = fake_encoded
    gs = 4
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, [batches[j % 4] for j in range(4)], opt, dev, cfg, gs, None,
                               0, False)
    torch.cuda.synchronize()
    ev.clear()
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, [batches[j % 4] for j in range(n)], opt, dev, cfg, gs, None,
                               0, False)
    torch.cuda.synchronize()
    # group: encoder marks pair up in order; decoder marks per step
    encs = [e for t, e in ev if t == "enc0"], [e for t, e in ev if t == "enc1"]
    steps = []
    cur = {}
    for t, e in ev:
        if t.startswith("enc"):
            continue
        cur[t] = e
        if t == "opt1":
            steps.append(cur)
            cur = {}
    acc = {}
    cnt = 0
    for i in range(2, len(steps) - 1):
        s = steps[i]
        base = s["dec0"]
        row = {k: base.elapsed_time(v) for k, v in s.items()}
        row["enc(i+1)0"] = base.elapsed_time(encs[0][i + 1])
        row["enc(i+1)1"] = base.elapsed_time(encs[1][i + 1])
        row["next dec0"] = base.elapsed_time(steps[i + 1]["dec0"])
        for k, v in row.items():
            acc[k] = acc.get(k, 0.0) + v
        cnt += 1
    for k in ("dec0", "dec1", "kl1", "bwd1", "opt1", "enc(i+1)0", "enc(i+1)1", "next dec0"):
        print(f"{k:10s} {acc[k] / cnt:8.3f} ms")


if __name__ == "__main__":
    main()
