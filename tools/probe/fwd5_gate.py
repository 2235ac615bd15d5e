"""WavLM attention at C2 (B 32, S 499, H 12, bf16): gate from 96 extra projection columns (fddm_attn_fwd_relgate) vs
from the attention input (fddm_attn_fwd_relgate_x), HIP events, same box."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "fddm-asr_amd"))
import torch
from fddm_hip import ops
from models.wavlm import _fold_gate
dev = torch.device("cuda:0"); bf = torch.bfloat16
def timeit(fn, iters=60):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3
B, S, H, E = 32, 499, 12, 768
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B * S, E, device=dev, generator=g).to(bf)
buf = torch.randn(B * S, 3 * E + 8 * H, device=dev, generator=g).to(bf)
qkv = buf[:, :3 * E].contiguous()
lin = torch.nn.Linear(64, 8).to(dev)
gw = _fold_gate(lin)
cst = torch.rand(H, device=dev) + 0.5
table = torch.randn(H, 2 * S - 1, device=dev)
o = torch.empty(B * S, E, device=dev, dtype=bf)
for r in range(6):
    t1 = timeit(lambda: ops.attn_fwd_relgate(buf, buf[:, E:], buf[:, 2 * E:], o, buf[:, 3 * E:], cst, table, B, H, S))
    t2 = timeit(lambda: ops.attn_fwd_relgate_x(qkv, qkv[:, E:], qkv[:, 2 * E:], o, x, gw, cst, table, B, H, S))
    print(f"round {r}: relgate (cols) {t1:.1f} us, relgate_x {t2:.1f} us", flush=True)
