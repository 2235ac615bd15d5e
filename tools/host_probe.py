"""Is the train step host-bound? Times the host enqueue of one step against its GPU completion, and lists
the device->host synchronisations inside a step (torch sync-debug warnings).

  python tools/host_probe.py [--steps 5]
"""
import os
import sys
import time
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "--no-cpu-baseline"] + sys.argv[1:]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    T_, cfg, models, opt = bench.build(args, dev)
    enc, dec, sp, te, tp, sch = models
    batches = bench.synthetic_batches(args, dev, 4, 7)
    gs = 1
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, batches[:4], opt, dev, cfg, gs, None, 0, False)
    torch.cuda.synchronize()
    cpu, ev = [], []

    def loader():
        for i in range(args.steps + 1):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            cpu.append(time.perf_counter())
            ev.append(e)
            if i < args.steps:
                yield batches[i % 4]
    gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, loader(), opt, dev, cfg, gs, None, 1, False)
    torch.cuda.synchronize()
    for i in range(1, len(ev)):
        c = 1e3 * (cpu[i] - cpu[0])
        g = ev[0].elapsed_time(ev[i])
        print(f"after step {i}: host {c:8.2f} ms  GPU {g:8.2f} ms  GPU behind host by {g - c:7.2f} ms "
              f"(host step {1e3 * (cpu[i] - cpu[i - 1]):6.2f}, GPU step {ev[i - 1].elapsed_time(ev[i]):6.2f})", flush=True)
    torch.cuda.set_sync_debug_mode("warn")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        for i in range(4):
            gs, _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, [batches[i]], opt, dev, cfg, gs, None, 1, False)
        torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode(0)
    print(f"{len(w)} synchronising ops in 4 steps")
    import traceback
    seen = set()
    for x in w:
        key = str(x.message)[:80] + str(x.filename) + str(x.lineno)
        if key in seen:
            continue
        seen.add(key)
        print(" ", x.filename, x.lineno, str(x.message)[:100])


if __name__ == "__main__":
    main()
