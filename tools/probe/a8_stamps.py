"""Phase timing of fwd8 from in-kernel s_memtime stamps (timing-only build: tools/build_variant.sh a8st attn8
-fno-slp-vectorize -DA8_STAMPS, then FDDM_HIP_LIB=abl/a8st.so python tools/probe/a8_stamps.py). Stamps of wave 0 of
every workgroup overwrite the first output row of its query block: 0 start, 1 tile 0 landed (after the prologue's
barrier), 2 first half-tile done, 3..10 mid-tile barriers, 12 loop end, 13 DMA drained (epilogue start), 14 stores
drained;
15 key mask done (before the Q loads), 11 prologue fills issued.
Prints, per shape, the median cycles between consecutive stamps over the workgroups and the spread of start times."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16


def main():
    ops.attn_force_kernels("fwd8")     # every shape on fwd8 (auto takes fwd7 at C4)
    cases = [("C2 self", 32, 8, 256, 256, True), ("C2 cross", 32, 8, 256, 499, False),
             ("C4 self", 16, 12, 512, 512, True), ("C4 cross", 16, 12, 512, 499, False)]
    for name, B, H, Lq, Lk, kpm in cases:
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B * Lq, H * 64, device=dev, dtype=bf, generator=g)
        k = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
        v = torch.randn(B * Lk, H * 64, device=dev, dtype=bf, generator=g)
        keep = None
        if kpm:
            lens = torch.randint(Lk // 2, Lk + 1, (B,), device=dev, generator=g)
            keep = (torch.arange(Lk, device=dev)[None] < lens[:, None]).to(torch.uint8).contiguous()
        db = ops.drop_bits(B, H, Lq, Lk, dev)
        ops.attn_drop_bits(db.view(1, -1), 1, B, H, Lq, Lk, 0.1, 1, 1, 0)
        o = torch.empty(B * Lq, H * 64, device=dev, dtype=bf)
        lse = torch.empty(B * H, Lq, device=dev)
        for _ in range(5):
            ops.attn_fwd(q, k, v, o, lse, B, H, Lq, Lk, key_keep=keep, drop_p=0.1, seed=1, rng_stream=1, dbits=db,
                         bits_ready=True)
        torch.cuda.synchronize()
        rows = o.view(B, Lq, H, 64)
        st = []
        for b in range(B):
            for qb in range(0, Lq, 256):
                for h in range(H):
                    st.append(rows[b, qb, h].contiguous().view(torch.int64)[:16])
        st = torch.stack(st).cpu().double()                       # [WGs, 16]
        t0 = st[:, 0].min()
        print(f"{name}: {st.shape[0]} WGs, start spread {float(st[:, 0].max() - t0):.0f} cyc, "
              f"end spread {float(st[:, 14].max() - st[:, 14].min()):.0f}, kernel span {float(st[:, 14].max() - t0):.0f}")
        pro = [0, 15, 11, 1] if (st[:, 15] > 0).all() else [0, 11, 1]
        pts = pro + [2] + [i for i in range(3, 11) if (st[:, i] > 0).all()] + [12, 13, 14]
        seg = []
        for a_, b_ in zip(pts[:-1], pts[1:]):
            seg.append(f"{a_}->{b_} {float((st[:, b_] - st[:, a_]).median()):.0f}")
        print("   median cycles: " + ", ".join(seg), flush=True)
        if os.environ.get("A8_FINE"):   # -DA8_FINE build: chunk ends of one phase call in the second row
            fs = []
            for b in range(B):
                for qb in range(0, Lq, 256):
                    for h in range(H):
                        fs.append(rows[b, qb + 1, h].contiguous().view(torch.int64)[:16])
            fs = torch.stack(fs).cpu().double()
            d = [f"c{k} {float((fs[:, k + 1] - fs[:, k]).median()):.0f}" for k in range(9)]
            print(f"   phase {os.environ['A8_FINE']} chunk cycles: " + ", ".join(d) +
                  f" | total {float((fs[:, 9] - fs[:, 0]).median()):.0f}", flush=True)


if __name__ == "__main__":
    main()
