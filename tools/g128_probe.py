"""Time the 128x128 LDS-DMA kernel at the decoder's shapes (HIP events); run once per library variant
(FDDM_HIP_LIB) to A/B kernel experiments.   python tools/g128_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
__import__("fddm_hip.ops", fromlist=["ops"]).gemm_force_path("128")
res = []
for (M, N, K) in [(8192, 512, 2048), (8192, 512, 512), (15968, 512, 1024)]:
    dy = torch.randn(M, K, device=dev, dtype=bf)
    w = torch.randn(K, N, device=dev, dtype=bf)
    o = torch.empty(M, N, device=dev)
    ms = timeit(lambda: ops.linear_dx(dy, w, out=o))
    res.append(f"dX {M}x{N}x{K}: {ms*1e3:6.1f} us {2*M*N*K/ms/1e9:6.0f} TF/s")
T, d, FF, TS = 8192, 512, 2048, 15968
specs = [(T, d, FF), (T, FF, d), (T, d, d), (T, d, d), (TS, 2 * d, d), (T, d, d), (T, 2 * d, d), (T, d, d)]
jobs, fl = [], 0
for K, M, N in specs:
    jobs.append((torch.randn(K, M, device=dev, dtype=bf), torch.randn(K, N, device=dev, dtype=bf),
                 torch.zeros(M, N, device=dev), torch.zeros(M, device=dev)))
    fl += 2 * M * N * K
__import__("fddm_hip.ops", fromlist=["ops"]).gemm_force_path("auto")
ms = timeit(lambda: ops.linear_dw_grouped(jobs))
res.append(f"dW grouped: {ms*1e3:6.1f} us {fl/ms/1e9:6.0f} TF/s")
print(os.path.basename(os.environ.get("FDDM_HIP_LIB", "in-tree")), " | ".join(res), flush=True)
