import torch
dev = torch.device("cuda:0")
for n in (1 << 28, 524_236_800 // 1):
    x = torch.empty(n, device=dev, dtype=torch.bfloat16)
    for f, name in ((lambda: x.fill_(1.0), "fill"), (lambda: x.zero_(), "zero")):
        for _ in range(3): f()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20): f()
        e.record(); torch.cuda.synchronize()
        t = s.elapsed_time(e) / 20 * 1e3
        print(name, n * 2 / 1e9, "GB", round(t, 1), "us", round(n * 2 / t / 1e3), "GB/s", flush=True)
