"""WavLM Q|K|V projection at C2 (15968 x 768 -> 2304, or 2400 with the 96 gate columns) on the persistent gemm256 at
the encoder's transformer cap (192 CUs), and the separate gate kernel (fddm_wavlm_gate) on the same rows."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "fddm-asr_amd"))
import torch
from fddm_hip import ops, _lib
dev = torch.device("cuda:0"); bf = torch.bfloat16
def timeit(fn, iters=20):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3
M, K, H = 15968, 768, 12
x = torch.randn(M, K, device=dev, dtype=bf)
for cap in (192, 256):
    _lib.lib().fddm_gemm_persistent_cap(cap)
    for N in (2304, 2400):
        W = torch.randn(N, K, device=dev, dtype=bf) / 30
        b = torch.randn(N, device=dev)
        o = torch.empty(M, N, device=dev, dtype=bf)
        print(f"cap {cap} N {N}: {timeit(lambda: ops.linear(x, W, b, out=o)):.1f} us", flush=True)
_lib.lib().fddm_gemm_persistent_cap(0)
Wg = torch.randn(8, 64, device=dev); bg = torch.randn(8, device=dev); cst = torch.randn(H, device=dev)
print(f"wavlm_gate bf16: {timeit(lambda: ops.wavlm_gate(x, Wg, bg, cst, 32, 499, H)):.1f} us", flush=True)
