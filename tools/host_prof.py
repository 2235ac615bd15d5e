"""cProfile of the host side of the C2 train step (bench.py's build): where the Python time per step goes."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "full"
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda:0")
    T_, cfg, models, opt = bench.build(args, dev)
    enc, dec, sp, te, tp, sch = models
    batches = bench.synthetic_batches(args, dev, 4, 1000)
    n = 16
    loader = [batches[i % 4] for i in range(n)]
    T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader[:4], opt, dev, cfg, 1, None, 0, False)
    torch.cuda.synchronize()
    # one step at a time from an idle GPU: host time of the enqueue vs the step's completion
    hs, ws = [], []
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader[:1], opt, dev, cfg, 5 + i, None, 0, False)
        hs.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        ws.append(time.perf_counter() - t0)
    print("single step from idle: host enqueue ms", [round(1e3 * h, 2) for h in hs], "complete ms",
          [round(1e3 * w, 2) for w in ws])
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader, opt, dev, cfg, 9, None, 0, False)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumtime").print_stats(30)


if __name__ == "__main__":
    main()
