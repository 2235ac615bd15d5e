import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch
from fddm_hip.optim import FusedAdamW
dev = torch.device("cuda:0")
ps = [torch.nn.Parameter(torch.randn(n, device=dev)) for n in [512 * 2048] * 30 + [8000 * 512] * 2 + [512] * 60]
for p in ps:
    p.grad = torch.randn_like(p)
opt = FusedAdamW(ps, lr=1e-4)
for _ in range(3):
    opt.clip_and_step(max_norm=5.0)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    opt.clip_and_step(max_norm=5.0)
e.record(); torch.cuda.synchronize()
print("clip_and_step", round(s.elapsed_time(e) / 20 * 1e3, 1), "us for", sum(p.numel() for p in ps) / 1e6, "M params")
