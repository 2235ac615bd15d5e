import os, sys
sys.path.insert(0, "fddm-asr_amd")
import torch
from fddm_hip import ops
dev = torch.device("cuda:0"); bf = torch.bfloat16
def timeit(fn, it=20):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3
for (Mt, n, k) in [(64, 128, 128), (512, 128, 128), (512, 512, 512), (4096, 128, 128)]:
    A = torch.randn(Mt, n, device=dev, dtype=bf)
    B = torch.randn(Mt, k, device=dev, dtype=bf)
    W = torch.zeros(n, k, device=dev)
    t = timeit(lambda: ops.linear_dw(A, B, out=W, accumulate=True))
    print(f"dW {n}x{k} over {Mt}: {t:6.1f} us", flush=True)
x = torch.empty(1, device=dev)
print(f"torch fill of 1 float: {timeit(lambda: x.fill_(1.0)):6.1f} us", flush=True)
M = 8192
for (n, k, lda, ldb) in [(512, 512, 512, 512), (512, 512, 2048, 2048), (512, 512, 520, 520), (512, 512, 576, 576), (2048, 512, 2048, 512), (2048, 512, 2048, 576)]:
    A = torch.randn(M, lda, device=dev, dtype=bf)[:, :n]
    B = torch.randn(M, ldb, device=dev, dtype=bf)[:, :k]
    W = torch.zeros(n, k, device=dev)
    t = timeit(lambda: ops.linear_dw(A, B, out=W, accumulate=True))
    print(f"dW {n}x{k} over {M}: lda {lda} ldb {ldb}: {t:6.1f} us {2*M*n*k/t/1e6:5.0f} TF/s", flush=True)
