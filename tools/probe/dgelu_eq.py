import math, os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "fddm-asr_amd"))
import torch
from fddm_hip import ops as o
dev = torch.device("cuda:0")
gen = torch.Generator(device=dev).manual_seed(21)
M, N, K = 8192, 2048, 512
dy = torch.randn(M, K, device=dev, generator=gen).bfloat16()
W = (torch.randn(K, N, device=dev, generator=gen) / math.sqrt(K)).bfloat16()
pre = torch.randn(M, N, device=dev, generator=gen).bfloat16()
outs = {}
for path in ("128", "small"):
    o.gemm_force_path(path)
    dh = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    o.linear_dx(dy, W, out=dh, epi=o.EPI_DGELU, C2=pre, drop_p=0.1, seed=9, rng_stream=4)
    outs[path] = dh
torch.cuda.synchronize()
a, b = outs["128"], outs["small"]
d = (a == 0) != (b == 0)
print("mismatch zeros", int(d.sum()), "nonfinite", int((~torch.isfinite(a.float())).sum()), int((~torch.isfinite(b.float())).sum()))
if d.any():
    idx = d.nonzero()[:5]
    for m, n in idx.tolist():
        print(m, n, float(a[m, n]), float(b[m, n]), float(pre[m, n]))
