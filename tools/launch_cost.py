"""GPU-side cost per kernel launch: N back-to-back launches captured in one HIP graph (no host launch cost in the
timing), for a 1-element fill (one workgroup), a 256-workgroup fill, and the 128x128 GEMM at 8192x512xK (K = 64
and 512: one round of 256 workgroups), against the same GEMMs launched eagerly."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
N = 200


def graph_time(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(N):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 5 / N * 1e3


def eager_time(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(N):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / N * 1e3


x1 = torch.zeros(1, device=dev)
x256 = torch.zeros(256 * 1024, device=dev)
print(f"fill 1 elem:      graph {graph_time(lambda: x1.fill_(1.0)):6.2f} us/launch  eager {eager_time(lambda: x1.fill_(1.0)):6.2f}")
print(f"fill 256 blocks:  graph {graph_time(lambda: x256.fill_(1.0)):6.2f} us/launch  eager {eager_time(lambda: x256.fill_(1.0)):6.2f}")
__import__("fddm_hip.ops", fromlist=["ops"]).gemm_force_path("128")
bf = torch.bfloat16
for K in (64, 512):
    x = torch.randn(8192, K, device=dev, dtype=bf)
    w = torch.randn(512, K, device=dev, dtype=bf) * 0.02
    o = torch.empty(8192, 512, device=dev, dtype=bf)
    f = lambda: ops.linear(x, w, out=o)  # noqa: E731
    print(f"gemm128 8192x512x{K}: graph {graph_time(f):6.2f} us/launch  eager {eager_time(f):6.2f}")
