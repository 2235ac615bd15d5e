"""Per-phase cycle stamps of the decoder attention kernels (fwd3 / dq3 / dkv3) at the C2 shapes. Needs the stamps
build of the library: `bash tools/build_variant.sh attnst attention -DATTN_STAMPS` then
`FDDM_HIP_LIB=vlib/attnst.so python tools/attn_stamps.py`. Per kernel: median over workgroups of the cycles of each
phase of wave 0 (entry -> loads issued -> data landed + barrier -> each tile -> stores issued -> stores done), the
workgroups' start skew and the kernel span from the 100 MHz real-time stamps, and the core clock they imply. The
stamps' own cost (~40 cycles each) and their lgkmcnt(0) fences make this build slower: read the shares."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fddm_hip import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
NS = 16
LIB = _lib.lib()
LIB.fddm_attn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_long]


def stamps(nblk):
    buf = (ctypes.c_ulonglong * (8192 * NS))()
    assert LIB.fddm_attn_stamps(buf, 8192 * NS) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(8192, NS)[:nblk].astype(np.int64)


def report(name, fn, nblk, ntiles):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    assert LIB.fddm_attn_stamps_clear() == 0
    fn()
    torch.cuda.synchronize()
    st = stamps(nblk)
    ok = st[:, 13] > 0
    st = st[ok]
    rt0, rt1 = st[:, 14], st[:, 15]
    cyc = st[:, 13] - st[:, 0]
    us = (rt1 - rt0) / 100.0
    clk = np.median(cyc / np.maximum(us, 1e-3)) / 1e3
    cols = [("loads issued", 0, 1), ("wait + barrier", 1, 2)]
    prev = 2
    for t in range(ntiles):
        cols.append((f"tile {t}", prev, 3 + t))
        prev = 3 + t
    cols += [("stores issued", prev, 12), ("stores done", 12, 13)]
    span = (rt1.max() - rt0.min()) / 100.0
    skew = (rt0.max() - rt0.min()) / 100.0
    print(f"\n### {name}: {len(st)} workgroups, span {span:.1f} us (start skew {skew:.1f} us), per-workgroup "
          f"{np.median(us):.1f} us median, clock ~{clk:.2f} GHz\n")
    print("| phase | median cycles | share |")
    print("|---|---|---|")
    tot = np.median(cyc)
    for lab, a, b in cols:
        d = np.median(st[:, b] - st[:, a])
        print(f"| {lab} | {int(d)} | {d / tot:.2f} |")
    print(f"| total (wave 0) | {int(tot)} | 1.00 |")


def main():
    B, H, L, S = 32, 8, 256, 499
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B * L, H * 64, device=dev, dtype=bf, generator=g)
    kq = torch.randn(B * L, H * 64, device=dev, dtype=bf, generator=g)
    v = torch.randn(B * L, H * 64, device=dev, dtype=bf, generator=g)
    kc = torch.randn(B * S, H * 64, device=dev, dtype=bf, generator=g)
    vc = torch.randn(B * S, H * 64, device=dev, dtype=bf, generator=g)
    # every key valid (no fully padded tile is skipped, so every workgroup stamps every tile); the mask path runs
    keep = torch.ones(B, L, device=dev, dtype=torch.uint8)
    o = torch.empty_like(q)
    lse = torch.empty(B * H, L, device=dev)
    bits = ops.drop_bits(B, H, L, L, dev)
    ops.attn_fwd(q, kq, v, o, lse, B, H, L, L, key_keep=keep, drop_p=0.1, seed=5, rng_stream=1, dbits=bits)
    report("fwd3 self (B32 H8 L256, key padding, dropout 0.1)",
           lambda: ops.attn_fwd(q, kq, v, o, lse, B, H, L, L, key_keep=keep, drop_p=0.1, seed=5, rng_stream=1,
                                dbits=bits), B * H, 4)
    oc = torch.empty_like(q)
    lsec = torch.empty(B * H, L, device=dev)
    bitsc = ops.drop_bits(B, H, L, S, dev)
    report("fwd3 cross (B32 H8 256 x 499, dropout 0.1)",
           lambda: ops.attn_fwd(q, kc, vc, oc, lsec, B, H, L, S, drop_p=0.1, seed=5, rng_stream=3, dbits=bitsc),
           B * H, 8)
    do = torch.randn_like(q)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    delta = torch.empty(B * H, L, device=dev)

    def dq3():
        ops.call("fddm_attn_bwd", ops.BF16, q.data_ptr(), q.stride(0), kq.data_ptr(), kq.stride(0), v.data_ptr(),
                 v.stride(0), o.data_ptr(), o.stride(0), do.data_ptr(), do.stride(0), lse.data_ptr(), dq.data_ptr(),
                 dq.stride(0), dk.data_ptr(), dk.stride(0), dv.data_ptr(), dv.stride(0), delta.data_ptr(),
                 keep.data_ptr(), B, H, L, L, 0.125, 0.1, 5, 1, bits.data_ptr(), ops.stream())

    # fddm_attn_bwd launches dq3 then dkv3: the stamps buffer holds the LAST one (dkv3); dq3 alone via FDDM env
    os.environ["FDDM_ATTN_DKV2"] = "1"        # dK/dV on the streamed kernel (not stamped): the buffer keeps dq3's
    report("dq3 self (B32 H8 L256, key padding, recorded dropout bits)", dq3, B * H, 4)
    del os.environ["FDDM_ATTN_DKV2"]
    report("dkv3 self (B32 H8 L256, key padding, recorded dropout bits)", dq3, B * H, 4)


if __name__ == "__main__":
    main()
