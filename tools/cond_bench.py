"""Micro-benchmark of the decoder's conditioning path at C2 (B 32, d 512, 6 blocks): the time MLP + FiLM small
row-batch launches (forward) and their backward, HIP-event timing per launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402


def timeit(f, n=50):
    for _ in range(5):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    B, d, NL = 32, 512, 6
    x = torch.randn(B, d, device=dev)
    Ws = [torch.randn(d, d, device=dev) / 23 for _ in range(2 * NL)]
    bs = [torch.randn(d, device=dev) for _ in range(2 * NL)]
    outs = [torch.empty(B, d, device=dev) for _ in range(2 * NL)]
    import os
    for tag in ("v4", "v1"):
        if tag == "v1":
            os.environ["FDDM_SMALL_LIN1"] = "1"
        print(tag)
        run(dev, B, d, NL)


def run(dev, B, d, NL):
    import os
    x = torch.randn(B, d, device=dev)
    Ws = [torch.randn(d, d, device=dev) / 23 for _ in range(2 * NL)]
    bs = [torch.randn(d, device=dev) for _ in range(2 * NL)]
    outs = [torch.empty(B, d, device=dev) for _ in range(2 * NL)]
    print(f"FiLM forward (12 x [32,512]x[512,512]) {timeit(lambda: ops.small_linear(x, Ws, bs, outs)):7.1f} us")
    print(f"one Linear [32,512]x[512,512]          {timeit(lambda: ops.small_linear(x, Ws[:1], bs[:1], outs[:1])):7.1f} us")
    dW = [torch.zeros(d, d, device=dev) for _ in range(2 * NL)]
    db = [torch.zeros(d, device=dev) for _ in range(2 * NL)]
    jobs = [(outs[i], x, dW[i], db[i]) for i in range(2 * NL)]
    print(f"FiLM weight grads (12 jobs)            {timeit(lambda: ops.small_dw(jobs)):7.1f} us")
    print(f"transposed Linear (input grad)          {timeit(lambda: ops.small_linear(x, Ws[:1], None, outs[:1], transpose_w=True)):7.1f} us")


if __name__ == "__main__":
    main()
