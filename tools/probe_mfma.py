"""GPU probe: checks the MFMA fragment maps and the ds_read_b64_tr_b16 semantics the kernels rely on."""
import ctypes, os, sys
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "libprobe.so"))
dev = torch.device("cuda:0")
s = torch.cuda.current_stream().cuda_stream
torch.manual_seed(0)

A = torch.randint(-3, 4, (16, 32)).float()
B = torch.randint(-3, 4, (32, 16)).float()
Ab = A.bfloat16().to(dev).view(torch.int16)
Bb = B.bfloat16().to(dev).view(torch.int16)
C = torch.zeros(16, 16, device=dev)
assert lib.probe_bf16(ctypes.c_void_p(Ab.data_ptr()), ctypes.c_void_p(Bb.data_ptr()), ctypes.c_void_p(C.data_ptr()), ctypes.c_void_p(s)) == 0
torch.cuda.synchronize()
ok1 = torch.equal(C.cpu(), A @ B)
print("bf16 16x16x32 layout ok:", ok1)

A = torch.randint(-3, 4, (16, 4)).float()
B = torch.randint(-3, 4, (4, 16)).float()
C = torch.zeros(16, 16, device=dev)
Ad, Bd = A.to(dev), B.to(dev)
assert lib.probe_f32(ctypes.c_void_p(Ad.data_ptr()), ctypes.c_void_p(Bd.data_ptr()), ctypes.c_void_p(C.data_ptr()), ctypes.c_void_p(s)) == 0
torch.cuda.synchronize()
ok2 = torch.equal(C.cpu(), A @ B)
print("f32 16x16x4 layout ok:", ok2)

t = torch.arange(256, dtype=torch.int16).to(dev)
out = torch.zeros(256, dtype=torch.int16, device=dev)
assert lib.probe_tr(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s)) == 0
torch.cuda.synchronize()
o = out.cpu().view(64, 4)
# expected: lane l (group g, i=l&15) gets column i of rows 4g..4g+3 of the [16][16] tile
exp = torch.zeros(64, 4, dtype=torch.int16)
for l in range(64):
    g, i = l >> 4, l & 15
    for e in range(4):
        exp[l, e] = (4 * g + e) * 16 + i
ok3 = torch.equal(o, exp)
print("tr_b16 ok:", ok3)
if not ok3:
    print(o[:20])
sys.exit(0 if (ok1 and ok2 and ok3) else 1)
