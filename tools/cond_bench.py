"""The decoder's conditioning Linears alone (csrc/small.hip, HIP-event timing): the 12 FiLM projections in one launch,
the time-MLP Linears, their input gradients (transposed weights) and the weight gradients (small_dw), at C2's shapes
(B 32, d 512, time-MLP hidden 2048). Prints us per launch.
  python tools/cond_bench.py"""
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
    B, d, hid, nf = 32, 512, 2048, 12
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, d, device=dev, generator=g)
    Wf = [torch.randn(d, d, device=dev, generator=g) / 20 for _ in range(nf)]
    bf = [torch.randn(d, device=dev, generator=g) for _ in range(nf)]
    of = [torch.empty(B, d, device=dev) for _ in range(nf)]
    print(f"FiLM x12 [32,512]x[512,512]^T      {timeit(lambda: ops.small_linear(x, Wf, bf, of)):6.1f} us", flush=True)
    W1 = torch.randn(hid, d, device=dev, generator=g) / 20
    b1 = torch.randn(hid, device=dev, generator=g)
    pre, h = torch.empty(B, hid, device=dev), torch.empty(B, hid, device=dev)
    print(f"MLP 1 [32,512]x[2048,512]^T + SiLU {timeit(lambda: ops.small_linear(x, [W1], [b1], [pre], [h], act=1)):6.1f} us",
          flush=True)
    W2 = torch.randn(d, hid, device=dev, generator=g) / 40
    o2 = torch.empty(B, d, device=dev)
    print(f"MLP 2 [32,2048]x[512,2048]^T       {timeit(lambda: ops.small_linear(h, [W2], [bf[0]], [o2])):6.1f} us", flush=True)
    dx = torch.empty(B, hid, device=dev)
    print(f"MLP 2 input grad (in @ W, SiLU')   "
          f"{timeit(lambda: ops.small_linear(o2, [W2], None, [dx], act=2, aux=pre, transpose_w=True)):6.1f} us", flush=True)
    dW = [torch.zeros(d, d, device=dev) for _ in range(nf)]
    db = [torch.zeros(d, device=dev) for _ in range(nf)]
    jobs = [(of[i], x, dW[i], db[i]) for i in range(nf)]
    print(f"FiLM x12 weight grads (small_dw)   {timeit(lambda: ops.small_dw(jobs)):6.1f} us", flush=True)


if __name__ == "__main__":
    main()
