"""Times the two halves of the C2 train step alone on the whole chip and the overlapped step (bench.py's build):
(a) the frozen encoder forward per batch, (b) the decoder step (q_sample .. AdamW) on a precomputed condition,
(c) train_one_epoch with the encoder of batch i+1 on the side stream. HIP-event timing, bf16."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda:0")
    T_, cfg, models, opt = bench.build(args, dev)
    enc, dec, sp, te, tp, sch = models
    batches = bench.synthetic_batches(args, dev, 4, 1000)
    n = 12

    def timed(fn, k):
        fn(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(k):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / k

    with torch.no_grad():
        t_enc = timed(lambda i: enc(batches[i % 4][0]), n)
    cs = [enc(b[0])[0] for b in batches]

    class Pre:
        def __init__(self):
            self.i = 0

    # decoder step alone: the encoder replaced by the precomputed condition
    real_encoded = T_._encoded

    def fake_encoded(encoder, loader, device, optimizer):
        for k, (wave, x0) in enumerate(loader):
            yield cs[k % 4], None, x0

    T_._encoded = fake_encoded
    gs = [4]

    def dec_step(i):
        gs[0], _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, [batches[i % 4]], opt, dev, cfg, gs[0], None, 0, False)
    t_dec = timed(dec_step, n)
    T_._encoded = real_encoded

    def full(i):
        gs[0], _ = T_.train_one_epoch(enc, dec, sp, te, tp, sch, [batches[j % 4] for j in range(n)], opt, dev, cfg,
                                      gs[0], None, 0, False)
    full(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    full(0)
    t_host = (time.perf_counter() - t0) * 1e3 / n          # host enqueue time (no wait inside the loop)
    torch.cuda.synchronize()
    t_full = (time.perf_counter() - t0) * 1e3 / n
    T_._encoded = fake_encoded
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        dec_step(i)
    t_dhost = (time.perf_counter() - t0) * 1e3 / n
    torch.cuda.synchronize()
    T_._encoded = real_encoded
    print(f"host enqueue: overlapped step {t_host:.3f} ms, decoder step {t_dhost:.3f} ms")
    print(f"encoder alone {t_enc:.3f} ms/batch | decoder step alone {t_dec:.3f} ms | overlapped step {t_full:.3f} ms "
          f"| sum {t_enc + t_dec:.3f}")


if __name__ == "__main__":
    main()
