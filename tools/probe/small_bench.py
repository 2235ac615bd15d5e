"""The decoder's conditioning Linears (csrc/small.hip) at the C2 / C4 shapes, HIP events: us per launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from attn7_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
for name, B, d, nf in (("C2", 32, 512, 12), ("C4", 16, 768, 24)):
    x = torch.randn(B, d, device=dev)
    Ws = [torch.randn(d, d, device=dev) * 0.02 for _ in range(nf)]
    bs = [torch.randn(d, device=dev) for _ in range(nf)]
    outs = [torch.empty(B, d, device=dev) for _ in range(nf)]
    t = timeit(lambda: ops.small_linear(x, Ws, bs, outs), 50)
    W1 = torch.randn(4 * d, d, device=dev) * 0.02
    pre, h = torch.empty(B, 4 * d, device=dev), torch.empty(B, 4 * d, device=dev)
    t1 = timeit(lambda: ops.small_linear(x, [W1], [bs[0].new_zeros(4 * d)], [pre], [h], act=1), 50)
    dx = torch.empty(B, d, device=dev)
    t2 = timeit(lambda: ops.small_linear(pre, [W1], None, [dx], transpose_w=True), 50)
    print(f"{name}: FiLM {nf} x [{B},{d}]x[{d},{d}] {t*1e3:6.1f} us | [{B},{d}]x[{d},{4*d}]+SiLU {t1*1e3:6.1f} us | "
          f"transposed [{B},{4*d}]x[{4*d},{d}] {t2*1e3:6.1f} us", flush=True)
