import os, sys, math
sys.path.insert(0, "/root/repo/fddm-asr_amd")
import torch
import torch.nn.functional as F
from fddm_hip import ops as o
dev = torch.device("cuda:0")
os.environ["FDDM_GEMM_PATH"] = "256"
for (M, N, K) in [(15968, 768, 3072), (1024, 768, 3072), (512, 512, 128), (256, 256, 128)]:
    gen = torch.Generator(device=dev).manual_seed(3)
    A = torch.randn(M, K, device=dev, generator=gen).bfloat16()
    W = (torch.randn(N, K, device=dev, generator=gen) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev, generator=gen)
    ref = A.float() @ W.float().T + b
    out = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    act = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    o.gemm(A, W, out, M, N, K, lda=K, ldb=K, ldc=N, bias=b, epi=1, C2=act)
    bad = ((out.float() - ref).abs() > 0.05 * ref.abs().max()) | out.float().isnan()
    badp = ((act.float() - F.gelu(ref)).abs() > 0.05 * ref.abs().max()) | act.float().isnan()
    idx = bad.nonzero()
    print(M, N, K, "bad pre:", int(bad.sum()), "bad post:", int(badp.sum()))
    if len(idx):
        r = idx[:, 0]; c = idx[:, 1]
        print("  rows", r.min().item(), r.max().item(), "unique rows mod 256:", sorted(set((r % 256).tolist()))[:20])
        print("  cols mod 64:", sorted(set((c % 64).tolist()))[:40], "n-tiles", sorted(set((c // 256).tolist())))
        print("  sample", idx[:8].tolist())
