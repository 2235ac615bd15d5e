// Decoder attention on 32x32x16 bf16 MFMAs (gfx950): forward (fwd7).
//
// The decoder's self- and cross-attention (models/denoise_decoder.py:129-130,164,169-176 -> nn.MultiheadAttention:
// key-padding mask, dropout p on the attention probabilities, head_dim 64), bf16 in / out, fp32 softmax statistics.
//
// Why a second kernel family next to attention.hip's fwd6 (16x16x32 MFMAs): at head_dim 64 the forward is bound by
// vector-instruction issue, not by the matrix cores (profiles/r04_summary.md: fwd6's tile loop issues
// ~263 VALU instructions against 32 MFMAs per wave and 64-key tile). Per wave and tile fwd7 issues half the MFMA
// instructions for the same work (16 x 32x32x16 instead of 32 x 16x16x32: the SIMD's vector issue is held 8 cycles
// per MFMA either way), reduces each query's row over 2 lanes instead of 4 (one v_permlane32_swap), and skips the
// tile maximum on every tile after a query block's first unless the tile's probabilities exceed 2^8 (checked on the
// lane's row sum it needs anyway), which leaves the exponent, its FMA, the row sum, the keep-bit AND and the bf16 pack
// per score. The prologue issues the first K / V tile's LDS-DMA, the Q fragments and the key-mask bytes together,
// and the output goes out through LDS as whole 128-B rows.
//
// Layout (per workgroup: 4 waves x 32 queries = 128 queries of one (b, h)):
//   S^T = K Q^T per 32-key block kb: A = K rows (LDS, KC swizzle, ds_read_b128), B = the lane's own query fragment
//   (registers). Accumulator register r of lane l holds key 32 kb + 8 (r >> 2) + 4 (l >> 5) + (r & 3), query l & 31:
//   a query's 64 keys of a tile sit in lanes l and l ^ 32.
//   O^T += V^T P^T per k-step (kb, s): B = the lane's P values r = 8 s .. 8 s + 7 packed to bf16 (k position j <-> key
//   32 kb + 16 s + 8 (j >> 2) + 4 (l >> 5) + (j & 3): the reduction order is permuted consistently on both operands);
//   A = V^T from two ds_read_b64_tr_b16 of 4 keys each (V image swizzle vsw: the 4 rows a 32-lane half reads are
//   conflict-free).
// The key mask (0 / -inf per key) is the S accumulator's initial value (no add per score).
#include "attn7_common.h"

namespace fddm {
namespace attn {

typedef __attribute__((address_space(4))) const uint64_t* cu64p;
// v_writelane_b32 through the LLVM intrinsic (this clang has no builtin for it), so the hazard recognizer inserts the
// wait states a VALU-written SGPR needs before v_writelane reads it (an inline-asm writelane got none: stale ballots)
__device__ int amdgcn_writelane_i32(int v, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
// lane L of x := the wave-uniform value v (the ballot of one slot goes to the lane that stores it)
template <int L>
__device__ __forceinline__ void writelane(unsigned& x, unsigned v) {
  x = (unsigned)amdgcn_writelane_i32((int)v, L, (int)x);
}

struct DmArgs {
  uint64_t* out;
  long site_words;  // words per site
  int BH, Lq, Lk;
  uint64_t seed, stream0, stream_step;
  unsigned thr16;
  const uint64_t* seed_off;
};

// One workgroup per (b, h, site): the site's three 4096-entry draw tables in LDS (one splitmix64 per 4 entries, as
// dbits_kernel), each followed by a copy of its first 64 entries so that a tile's 64 keys never wrap; then each wave
// takes 32-query groups. Per group and key tile, lane l draws the 4 keys 64 t + 32 kb + 8 m + 4 (l >> 5) + 0..3 of
// query 32 qg + (l & 31) from one 8-byte entry of each table (one base address per table and tile, the rest immediate
// offsets; single ds_read_b64, see below) and builds its layout-v5 dword directly: per dword of draws one XOR of the
// three tables (v_bitop3), a saturating packed u16 subtract of thr - 1 and a packed min with 1 (keep as 0 / 1 in bits
// 0 and 16), shifted to the pair's bits. The lane-mask words (layout v3) are the transpose of those dwords over each
// 32-lane half: a 32 x 32 bit transpose in five lane-exchange (DPP / v_permlane16_swap) / rotate / bit-select stages
// leaves in lane j of half h the keep bits of lanes 32 h .. 32 h + 31 for bit position j, i.e. one 32-bit half of the
// word of the slot whose bit is j, stored straight to it. Per tile and wave ~106 VALU and 24 LDS gathers instead of
// ~230 VALU (a ballot and two v_writelane per draw); the random gathers' bank conflicts bound it
// (profiles/r06i_dmask.md).
__device__ __forceinline__ int lb_slot(int j) {  // the slot 16 kb + r whose layout-v5 bit position is j (lb_bit^-1)
  const int odd = j >> 4, P = odd ? 31 - j : 15 - j;
  return 16 * (P >> 3) + 2 * (P & 7) + odd;
}
constexpr int DM_TABW = ATTN_R / 4 + 16;  // 8-byte words per table: 4096 entries + the first 64 again
typedef unsigned dm_u32x2 __attribute__((ext_vector_type(2)));
template <int OFF>
__device__ __forceinline__ dm_u32x2 lds_read64_at(unsigned a) {  // not tracked by hipcc: the caller waits lgkmcnt
  dm_u32x2 v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}

__global__ void __launch_bounds__(256) dmask_kernel(DmArgs d) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[3 * DM_TABW];
  const int bh = blockIdx.x, site = blockIdx.y, tid = threadIdx.x;
  const uint64_t stream = d.stream0 + (uint64_t)site * d.stream_step;
  const uint64_t seed = eff_seed(d.seed, d.seed_off);
  for (int wi = tid; wi < 3 * ATTN_R / 4; wi += 256) {
    const int tau = wi / (ATTN_R / 4), jw = wi % (ATTN_R / 4);
    const uint64_t v = mix64(seed, stream, ATTN_TAB0 + ((uint64_t)bh * 3 + tau) * (ATTN_R / 4) + jw);
    tab[tau * DM_TABW + jw] = v;
    if (jw < 16) tab[tau * DM_TABW + ATTN_R / 4 + jw] = v;
  }
  __syncthreads();
  const int ntiles = (d.Lk + 63) >> 6, nqg = (d.Lq + 31) >> 5;
  const int lane = tid & 63, w = tid >> 6, qi = lane & 31, hh = lane >> 5;
  uint64_t* out = d.out + (long)site * d.site_words;
  const unsigned char* tb = (const unsigned char*)tab;
  unsigned* lbits = (unsigned*)(out + (long)d.BH * nqg * ntiles * 32);  // the per-lane dwords after the lane masks
  // transpose stage constants: stage s pairs lane l with l ^ s; the lane's partner word rotated right by rot[i] and
  // merged under msk[i] (kept bits of its own word)
  unsigned rot[5], msk[5];
  static_for<0, 5>([&](auto ic) {
    constexpr int i = decltype(ic)::value, s = 16 >> i;
    constexpr unsigned ms = i == 0 ? 0x0000FFFFu : i == 1 ? 0x00FF00FFu : i == 2 ? 0x0F0F0F0Fu : i == 3 ? 0x33333333u
                                                                                                        : 0x55555555u;
    const bool up = (lane & s) != 0;
    rot[i] = up ? s : 32 - s;
    msk[i] = up ? ~ms : ms;
  });
  const int wslot = 2 * lb_slot(qi) + hh;  // the dword of the lane-mask words this lane stores
  const unsigned thm1 = ((d.thr16 - 1) & 0xFFFFu) * 0x00010001u;  // both u16 halves thr16 - 1: keep iff draw > it
  for (int qg = w; qg < nqg; qg += 4) {
    const uint64_t off = mix64(seed, stream, ATTN_OFF0 + (uint64_t)bh * d.Lq + 32 * qg + qi);
    const unsigned o0 = (unsigned)(off & 0xFFCu), o1 = (unsigned)((off >> 16) & 0xFFCu),
                   o2 = (unsigned)((off >> 32) & 0xFFCu);
    for (int t = 0; t < ntiles; ++t) {
      const unsigned kq = 64 * t + 4 * hh;
      // the tile's 24 table reads as single ds_read_b64 by hand: hipcc pairs them into ds_read2_b64, which the LDS
      // serves at half the rate with 32-bank conflict groups (MI355X_MICROARCH.md, LDS table) -- on these random
      // gathers the bank conflicts, not the VALU, bound the kernel
      const unsigned tl = lds_addr(tb);
      const unsigned a0 = tl + (((o0 + kq) & (ATTN_R - 1)) << 1);
      const unsigned a1 = tl + DM_TABW * 8 + (((o1 + kq) & (ATTN_R - 1)) << 1);
      const unsigned a2 = tl + DM_TABW * 16 + (((o2 + kq) & (ATTN_R - 1)) << 1);
      dm_u32x2 rd[3][8];  // [table][4 kb + m]
      static_for<0, 8>([&](auto jc) {
        constexpr int j = decltype(jc)::value, ob = 64 * (j >> 2) + 16 * (j & 3);
        rd[0][j] = lds_read64_at<ob>(a0);
        rd[1][j] = lds_read64_at<ob>(a1);
        rd[2][j] = lds_read64_at<ob>(a2);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(rd[0][j]), "+v"(rd[1][j]), "+v"(rd[2][j]));
      // dword h of the (kb, m) entry holds the draws of registers r = 4 m + 2 h (low half) and r + 1 (high half): score
      // pair p = 8 kb + 2 m + h, whose bits are 15 - p and 31 - p. Saturating u16 subtract of thr - 1 and a min with 1
      // (two packed ops) leave keep as 0 / 1 in bits 0 and 16; shifted left by 15 - p they are the pair's two bits.
      unsigned lw = 0;
      static_for<0, 16>([&](auto ic) {
        constexpr int i = decltype(ic)::value, j = i >> 1, h = i & 1, p = 8 * (j >> 2) + 2 * (j & 3) + h;
        unsigned k;  // as packed VALU by hand (hipcc turns the builtins into two compares and selects)
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96\n\tv_pk_sub_u16 %0, %0, %4 clamp\n\tv_pk_min_u16 %0, %0, %5"
            : "=&v"(k)
            : "v"(rd[0][j][h]), "v"(rd[1][j][h]), "v"(rd[2][j][h]), "s"(thm1), "s"(0x00010001u));
        lw |= k << (15 - p);
      });
      if (d.thr16 == 0) lw = 0xFFFFFFFFu;  // p < 2^-17: every score kept
      lbits[lb_dword(bh, nqg, ntiles, qg, t) + lane] = lw;
      unsigned x = lw;
      static_for<0, 5>([&](auto ic) {
        constexpr int i = decltype(ic)::value, s = 16 >> i;
        unsigned y;  // x of lane l ^ s: cross-lane moves on the VALU (no LDS round trip in the chain)
        if constexpr (s == 16) {
          const auto sw = __builtin_amdgcn_permlane16_swap(x, x, false, false);
          y = (lane & 16) ? sw[0] : sw[1];
        } else if constexpr (s == 8) {
          y = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
        } else if constexpr (s == 4) {  // lanes with bit 2 clear read l + 4 (row_ror:12), the others l - 4 (row_ror:4)
          y = (unsigned)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x12C, 0xF, 0x5, false);
          y = (unsigned)__builtin_amdgcn_update_dpp((int)y, (int)x, 0x124, 0xF, 0xA, false);
        } else {
          y = (unsigned)__builtin_amdgcn_mov_dpp((int)x, s == 2 ? 0x4E : 0xB1, 0xF, 0xF, false);  // quad_perm
        }
        x = (msk[i] & x) | (~msk[i] & __builtin_rotateright32(y, rot[i]));
      });
      ((unsigned*)(out + lm_word(bh, nqg, ntiles, qg, t)))[wslot] = x;
    }
  }
}

int attn7_drop_bits(uint64_t* out, long site_words, int nsites, int BH, int Lq, int Lk, uint64_t seed,
                    uint64_t stream0, uint64_t stream_step, unsigned thr16, const uint64_t* seed_off, hipStream_t s) {
  DmArgs d{out, site_words, BH, Lq, Lk, seed, stream0, stream_step, thr16, seed_off};
  hipLaunchKernelGGL(dmask_kernel, dim3(BH, nsites), dim3(256), 0, s, d);
  return (int)hipGetLastError();
}
long attn7_drop_words(int B, int H, int Lq, int Lk) {  // lane masks + per-lane dwords
  return (long)B * H * ((Lq + 31) / 32) * ((Lk + 63) / 64) * 64;
}

// DM: 0 no dropout, 1 keep bits from the words fddm_attn_drop_bits wrote (word (bh, t, q), bit = key - 64 t).
// MK: 0 no mask, 1 the ragged last tile only (Lk % 64 != 0, no key-padding mask), 2 key-padding mask on every tile.
// REL: WavLM's gated relative-position bias (HF modeling_wavlm.py:474-513, 569-596; round 6, replacing fwd5 of
// attention.hip): score += gate(q) * table[h][k - q + Lk - 1], added in log2 units (g2 = gate log2 e) to the score
// accumulators before the softmax. The workgroup's slice of the table row (keys 0 .. LkP + 127 relative to its 128
// queries) is staged in LDS as two copies shifted by 0 / 1 entries, so that a lane's 4 consecutive keys of an
// accumulator quad are two aligned ds_read_b64 (copy jq & 1 of lane offset jq = qbase + 127 - q); copies are
// LkP + 160 floats apart (= 128 B mod 256), which spreads a 32-lane read group over all 64 banks, and the workgroup
// fits 40 KB of LDS (no keep-bit stage without dropout): four workgroups per CU (four copies and ds_read_b128: three,
// 46-47 us at the C2 encoder shape; v_pk_fma_f32 / v_pk_add_f32 for the bias and the row sums measured 2-3 % slower than
// scalar f32, here and in the decoder's fwd7, tools/r06_t48.sh). The gate per query
// comes from a precomputed row, from the Q|K|V projection's 8 extra columns, or from the attention input x through
// the folded GRU weights (lanes l and l ^ 32 each take 32 of the head's 64 inputs).
#ifndef A7_FWD_WPS
#define A7_FWD_WPS 3  // waves per SIMD the forward's register allocation targets
#endif
template <int DM, int MK, bool REL = false>
__global__ void __launch_bounds__(256, A7_FWD_WPS) fwd7_kernel(AttnArgs a) {
  constexpr bool DROP = DM != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm7[];
  const int ntiles = (a.Lk + 63) >> 6, LkP = ntiles * 64;
  unsigned char* kst = sm7;                             // [2][64 rows][128 B] K, KC swizzle
  unsigned char* vst = sm7 + 2 * A7_TB;                 // [2][64 rows][128 B] V, vsw swizzle
  constexpr int KBL = DROP ? 2048 : 0;                   // the keep-bit stage only with dropout (REL: 4 WGs per CU)
  unsigned* kbl = (unsigned*)(sm7 + 4 * A7_TB);         // [2][4 waves][64 lanes] keep bits of the tile (v4 dwords)
  unsigned* tact = (unsigned*)(sm7 + 4 * A7_TB + KBL);   // [4] active-tile nibbles per wave (MK 2)
  unsigned* mpk = (unsigned*)(sm7 + 4 * A7_TB + KBL + 16);  // [LkP] bf16 pair (1, mask): the key's fifth-k-step operand
  float* bcp = (float*)(sm7 + 4 * A7_TB + KBL + 16 + LkP * 4);  // REL: [2][LkP + 160] bias slices shifted by 0 / 1
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, qi = lane & 31;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const int qw0 = bxi * 128 + 32 * w;
  const int q = qw0 + qi;
  const bool qv = q < a.Lq;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;

  // one tile's stream: wave w brings rows 16 w .. 16 w + 15 of K and V (2 + 2 KB pieces, XOR swizzles applied to the
  // per-lane source addresses); byte offsets from the (b, h) bases (row * stride * 2 < 2^31 for Lk <= 1024)
  const unsigned sk2 = (unsigned)a.sk * 2u, sv2 = (unsigned)a.sv * 2u;
  const int nqg = (a.Lq + 31) >> 5, qg = 4 * bxi + w;  // the wave's 32-query group (keep bits)
  const unsigned* lbits = (const unsigned*)(a.dbits + (long)a.B * a.H * nqg * ntiles * 32);
  auto fill = [&](int tt, int st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int R = 16 * w + 8 * u;
      const int r = 64 * tt + R + (lane >> 3), pch = lane & 7;
      const unsigned rr = (unsigned)min(r, a.Lk - 1);
      dma16_sv(Kb, rr * sk2 + (unsigned)((pch ^ ((r >> 1) & 7)) << 4), kst + st * A7_TB + R * 128);
      dma16_sv(Vb, rr * sv2 + (unsigned)((pch ^ vsw(r)) << 4), vst + st * A7_TB + R * 128);
    }
    if constexpr (DROP)
      dma4_sv(lbits, (unsigned)(lb_dword(bh, nqg, ntiles, min(qg, nqg - 1), tt) + lane) * 4u,
              (const unsigned char*)(kbl + st * 256 + w * 64));
  };

  // ---- prologue: tile 0's stream, the Q fragments (pre-scaled by sl2: scores come out in log2 units) and the key
  // mask in flight together; rows past Lq read row Lq - 1 and are zeroed (never stored)
  fill(0, 0);
  const float sl2 = a.scale * 1.4426950408889634f;
  uint4 qf[4];
  {
    const long qc = min(q, a.Lq - 1);
    const unsigned zm = qv ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const uint4 x = *(const uint4*)(Qb + qc * a.sq + 16 * ks + 8 * hh);
      qf[ks] = scale_frag(make_uint4(x.x & zm, x.y & zm, x.z & zm, x.w & zm), sl2);
    }
  }
  float g2 = 0.f;  // REL: the query's gate in log2 units
  int boff = 0;    // REL: the lane's float offset of its bias quads in the shifted copies (key offset 0)
  if constexpr (REL) {
    float gate = 0.f;
    if (a.gate) {
      gate = qv ? a.gate[(long)bh * a.Lq + q] : 0.f;
    } else if (a.graw) {  // gate from the 8 pre-activations the Q|K|V projection appended (HF modeling_wavlm.py:177-186)
      const long qc = min(q, a.Lq - 1);
      const uint4 u = *(const uint4*)((const bf16_t*)a.graw + ((long)b * a.Lq + qc) * a.sgr + h * 8);
      const float ra = __uint_as_float(u.x << 16) + __uint_as_float(u.x & 0xFFFF0000u) + __uint_as_float(u.y << 16) +
                       __uint_as_float(u.y & 0xFFFF0000u);
      const float rb = __uint_as_float(u.z << 16) + __uint_as_float(u.z & 0xFFFF0000u) + __uint_as_float(u.w << 16) +
                       __uint_as_float(u.w & 0xFFFF0000u);
      const float ga = 1.f / (1.f + __expf(-ra)), gb = 1.f / (1.f + __expf(-rb));
      gate = ga * (gb * a.gconst[h] - 1.f) + 2.f;
    } else {  // gate from the attention input x through the folded GRU weights: lane half hh takes inputs 32 hh ..
      const long qc = min(q, a.Lq - 1);
      const bf16_t* xr = (const bf16_t*)a.gx + ((long)b * a.Lq + qc) * a.sgx + h * DH + 32 * hh;
      const float4* wa = (const float4*)(a.gw + 32 * hh);
      const float4* wb = (const float4*)(a.gw + 64 + 32 * hh);
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint4 xv = *(const uint4*)(xr + 8 * c);
        const unsigned xs[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float4 A = wa[2 * c + j], Bw = wb[2 * c + j];
          const float e0 = __uint_as_float(xs[2 * j] << 16), e1 = __uint_as_float(xs[2 * j] & 0xFFFF0000u);
          const float e2 = __uint_as_float(xs[2 * j + 1] << 16), e3 = __uint_as_float(xs[2 * j + 1] & 0xFFFF0000u);
          sa = fmaf(e0, A.x, fmaf(e1, A.y, fmaf(e2, A.z, fmaf(e3, A.w, sa))));
          sb = fmaf(e0, Bw.x, fmaf(e1, Bw.y, fmaf(e2, Bw.z, fmaf(e3, Bw.w, sb))));
        }
      }
      sa = xsum32(sa) + a.gw[128];
      sb = xsum32(sb) + a.gw[129];
      const float ga = 1.f / (1.f + __expf(-sa)), gb = 1.f / (1.f + __expf(-sb));
      gate = qv ? ga * (gb * a.gconst[h] - 1.f) + 2.f : 0.f;
    }
    g2 = gate * 1.4426950408889634f;
    // copy c, entry i = table[h][off0 + i + c], off0 = (Lk - 1) - (qbase + 127); zero outside the row
    const int CL = LkP + 160, qbase = bxi * 128;
    const float* tabh = a.table + (long)h * (2 * a.Lk - 1);
    const long off0 = (long)(a.Lk - 1) - (qbase + 127);
    for (int i = tid; i < 2 * CL; i += 256) {
      const int c = i >= CL ? 1 : 0;
      const long ti = off0 + (i - c * CL) + c;
      bcp[i] = (ti >= 0 && ti < 2L * a.Lk - 1) ? tabh[ti] : 0.f;
    }
    const int jq = qbase + 127 - q;  // key k of this query sits at slice entry k + jq
    boff = (jq & 1) * CL + (jq & ~1) + 4 * hh;
  }
  unsigned tmask = ntiles >= 32 ? 0xFFFFFFFFu : ((1u << ntiles) - 1u);
  if constexpr (MK != 0) {
    // thread tid owns keys 4 tid .. 4 tid + 3 (LkP <= 1024)
    bool any = false;
    if (4 * tid < LkP) {
      unsigned mv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 4 * tid + j;
        const bool ok = k < a.Lk && (MK == 1 || a.key_keep[(long)b * a.Lk + k] != 0);
        mv[j] = pk_bf16(1.f, ok ? 0.f : -INFINITY);
        any |= ok;
      }
      *(uint4*)(mpk + 4 * tid) = make_uint4(mv[0], mv[1], mv[2], mv[3]);
    }
    if constexpr (MK == 2) {
      const unsigned long long bal = __ballot(any);  // lanes 16 j .. 16 j + 15 of wave w: the keys of tile 4 w + j
      if (lane == 0) {
        unsigned nib = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) nib |= ((bal >> (16 * j)) & 0xFFFFull) ? (1u << j) : 0u;
        tact[w] = nib;
      }
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) pin16(qf[ks]);  // hipcc waits for the Q loads here, not inside the stream loop
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (MK == 2) tmask &= tact[0] | (tact[1] << 4) | (tact[2] << 8) | (tact[3] << 12);

  // per-lane LDS offsets: K row reads (row qi of a 32-key block, chunk 2 ks + hh), V transposed reads (16-lane group
  // G = lane >> 4 reads rows 4 hh + (i >> 2) of a 16-key step, 8-B units 8 db + 4 (G & 1) + (i & 3), i = lane & 15)
  int koff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) koff[ks] = qi * 128 + (((2 * ks + hh) ^ ((qi >> 1) & 7)) << 4);
  const int vi = lane & 15, vrow = 4 * hh + (vi >> 2);
  int voff[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
    voff[db] = vrow * 128 + (((8 * db + 4 * ((lane >> 4) & 1) + (vi & 3)) ^ ((vrow & 2) << 2)) << 3);

  // online softmax in log2 units: m = running maximum (-inf until a finite score), rf = the reference subtracted
  // inside the score MFMA (bf16-exact, 0 while m = -inf): p = 2^(s sl2 - rf); O and l are kept relative to rf
  float m = -INFINITY, rf = 0.f, l = 0.f;
  f32x16_t o0 = {}, o1 = {};
  bool first = true;
  // the query's fifth-k-step operand: (-rf, 1, 0, ...) on the lanes of the first 8 k positions
  uint4 q5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(0.f, 1.f), 0u, 0u, 0u);

  // one 64-key tile as two 32-key halves, each an online-softmax step of its own (S, exponentials, PV), so that only
  // one half's 16 scores and 8 packed probabilities are live next to O and Q
  auto tile = [&](const int t, const int st) {
    const bool mt = MK == 2 || (MK == 1 && t == ntiles - 1);  // this tile's keys carry a mask
    const unsigned char* kimg = kst + st * A7_TB;
    const unsigned char* vimg = vst + st * A7_TB;
    unsigned kw = 0xFFFFFFFFu;
    if constexpr (DROP) kw = kbl[st * 256 + w * 64 + lane];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // S''^T = K Q'^T + (1, mask) . (-rf, 1): the key's operand (1, mask) on the lanes of the first 8 k positions
      unsigned mk = pk_bf16(1.f, 0.f);
      if (MK != 0 && mt) mk = mpk[64 * t + 32 * kb + qi];
      const uint4 k5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(mk, 0u, 0u, 0u);
      f32x16_t sc = mfma32(k5, q5, f32x16_t{});
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) sc = mfma32(*(const uint4*)(kimg + koff[ks] + kb * 32 * 128), qf[ks], sc);
      if constexpr (REL) {  // + g2 * bias: register r is key 32 kb + 8 (r >> 2) + 4 hh + (r & 3) of tile t
        // the 8 bias pairs as single ds_read_b64 by hand: hipcc pairs them into ds_read2_b64 (16-lane groups over 32
        // banks, where the two shifted copies collide), the same trap as the keep-bit producer's gathers
        const unsigned bl = lds_addr(bcp) + 4u * (unsigned)(boff + 64 * t + 32 * kb);
        dm_u32x2 bw[8];
        bw[0] = lds_read64_at<0>(bl);
        bw[1] = lds_read64_at<8>(bl);
        bw[2] = lds_read64_at<32>(bl);
        bw[3] = lds_read64_at<40>(bl);
        bw[4] = lds_read64_at<64>(bl);
        bw[5] = lds_read64_at<72>(bl);
        bw[6] = lds_read64_at<96>(bl);
        bw[7] = lds_read64_at<104>(bl);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(bw[j]));
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {  // scalar FMAs: v_pk_fma_f32 measured 2-3 % slower
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sc[4 * rq + e] = fmaf(g2, __uint_as_float(bw[2 * rq + (e >> 1)][e & 1]), sc[4 * rq + e]);
        }
      }
      // exponentials 2^(sc - d), the lane's row sum (before dropout), the keep-mask select and the bf16 pack into
      // the PV operands bq[s]
      uint4 bq[2];
      float ls;
      auto expall = [&](float d) {
        float la = 0.f, lb = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          unsigned bw[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int r = 8 * s + 2 * jj;
            float x = __builtin_amdgcn_exp2f(sc[r] - d);
            float y = __builtin_amdgcn_exp2f(sc[r + 1] - d);
            la += x;
            lb += y;
            if constexpr (DROP) {  // keep bit lb_bit(kb, r) of the lane's dword as an AND mask (v_bfe_i32)
              x = __uint_as_float(__float_as_uint(x) & (unsigned)__builtin_amdgcn_sbfe((int)kw, lb_bit(kb, r), 1));
              y = __uint_as_float(__float_as_uint(y) & (unsigned)__builtin_amdgcn_sbfe((int)kw, lb_bit(kb, r + 1), 1));
            }
            bw[jj] = pk_bf16(x, y);
          }
          bq[s] = make_uint4(bw[0], bw[1], bw[2], bw[3]);
        }
        ls = la + lb;
      };
      // fast path: 2^sc against the current reference; slow path (a query block's first half-tile, or a lane sum
      // above 2^8 / inf / NaN): the half's maximum, a new bf16 reference, O and l rescaled, 2^(sc - (rf' - rf))
      // (also while a row has no finite reference yet, m = -inf: the fast path bounds the sum only from above, so a
      // row whose first keys were all masked and whose later scores sit below 2^-126 of rf = 0 would sum to 0)
      bool slow = first;
      if (!first) {
        expall(0.f);
        slow = __any(!(ls <= 256.f) || m == -INFINITY);
      }
      if (slow) {
        float tm = fmaxf(sc[0], sc[1]);
#pragma unroll
        for (int r = 2; r < 16; r += 2) tm = fmaxf(tm, fmaxf(sc[r], sc[r + 1]));
        tm = xmax32(tm) + rf;                       // absolute (log2 units)
        const float mn = fmaxf(m, tm);
        float rn = rf;
        if (mn != -INFINITY) rn = __uint_as_float(((unsigned)pk_bf16(mn, 0.f)) << 16);
        const float alpha = (m == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(rf - rn);
        l *= alpha;
        o0 *= alpha;
        o1 *= alpha;
        expall(rn - rf);
        m = mn;
        rf = rn;
        q5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(-rf, 1.f), 0u, 0u, 0u);
      }
      l += ls;
      first = false;
      // O^T += V^T P^T over the half's two 16-key steps
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int rb = (32 * kb + 16 * s) * 128;
        const uint4 v0 = join_tr(tr_read(vimg + voff[0] + rb), tr_read(vimg + voff[0] + rb + 8 * 128));
        const uint4 v1 = join_tr(tr_read(vimg + voff[1] + rb), tr_read(vimg + voff[1] + rb + 8 * 128));
        o0 = mfma32(v0, bq[s], o0);
        o1 = mfma32(v1, bq[s], o1);
      }
    }
  };

  // ---- the stream: tile t sits in stage st; the next active tile is filled into st ^ 1 before t is computed
  int t = 0, st = 0;
  bool act = (tmask & 1u) != 0;
  while (true) {
    const unsigned rest = t + 1 < 32 ? (tmask & ~((2u << t) - 1u)) : 0u;
    const int tn = rest ? __builtin_ctz(rest) : -1;
    if (tn >= 0) fill(tn, st ^ 1);
    if (act) tile(t, st);
    if (tn < 0) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile tn landed
    __builtin_amdgcn_s_barrier();                      // every wave's pieces landed; every wave finished tile t
    t = tn;
    st ^= 1;
    act = true;
  }

  // ---- epilogue: normalise, stage the wave's 32 output rows in LDS (K ring, free after the barrier), store rows
  __syncthreads();
  const float lt = xsum32(l);
  const float inv = (lt > 0.f) ? (DROP ? a.drop_scale : 1.f) / lt : NAN;
  unsigned char* ost = kst + w * 4096;
#pragma unroll
  for (int db = 0; db < 2; ++db) {
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      const f32x16_t& oo = db ? o1 : o0;
      uint2 u2;
      u2.x = pk_bf16(oo[4 * mm] * inv, oo[4 * mm + 1] * inv);
      u2.y = pk_bf16(oo[4 * mm + 2] * inv, oo[4 * mm + 3] * inv);
      *(uint2*)(ost + qi * 128 + (((4 * db + mm) ^ (qi & 7)) << 4) + 8 * hh) = u2;
    }
  }
  if (a.lse && hh == 0 && qv)
    a.lse[(long)bh * a.Lq + q] = (lt > 0.f) ? (rf + __log2f(lt)) * 0.69314718055994531f : NAN;
  bf16_t* Ob = (bf16_t*)a.Out + (long)b * a.Lq * a.so + h * DH;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (lane >> 3) + 8 * i, c = lane & 7;
    const uint4 v = *(const uint4*)(ost + row * 128 + ((c ^ (row & 7)) << 4));
    if (qw0 + row < a.Lq) *(uint4*)(Ob + (long)(qw0 + row) * a.so + c * 8) = v;
  }
}

// dQ, query-owned (4 waves x 32 queries per workgroup, K / V tiles of 64 keys streamed through a 2-stage LDS-DMA
// ring). Per 32-key half: S''^T = K Q'^T over 4 k-steps plus a fifth k-step that adds -LSE (log2 units, hi + lo bf16)
// and the key mask, so p = exp2(S'') is one instruction; dP^T = V dO^T; dS = p (keep dscale dP - delta);
// dQ^T += K^T dS^T (K^T by transposed reads of the same K image). Also writes the backward's per-query row terms for
// dkv7: nlse2 = -LSE log2(e) (-inf past Lq) and delta = rowsum(dO O) (0 past Lq), both [B*H][LqP], then the
// pre-scaled Q' = bf16(Q scale log2(e)) (0 past Lq) as [B*H][LqP][64] bf16.
template <int DM, int MK>
__global__ void __launch_bounds__(256, 3) dq7_kernel(AttnArgs a) {
  constexpr bool DROP = DM != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smq7[];
  const int ntiles = (a.Lk + 63) >> 6, LkP = ntiles * 64, LqP = (a.Lq + 63) & ~63;
  unsigned char* kst = smq7;                      // [2][64 rows][128 B] K, dsw swizzle (row + transposed reads)
  unsigned char* vst = smq7 + 2 * A7_TB;          // [2][64 rows][128 B] V, KC swizzle (row reads)
  unsigned* kbl = (unsigned*)(smq7 + 4 * A7_TB);         // [2][4 waves][64 lanes] keep bits of the tile (v4 dwords)
  unsigned* tact = (unsigned*)(smq7 + 4 * A7_TB + 2048);  // [4] active-tile nibbles per wave (MK 2)
  unsigned* mpk = (unsigned*)(smq7 + 4 * A7_TB + 2064);   // [LkP] bf16 pair (mask, 0): the key's fifth-k-step operand
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, qi = lane & 31;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const int qw0 = bxi * 128 + 32 * w;
  const int q = qw0 + qi;
  const bool qv = q < a.Lq;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Ob = (const bf16_t*)a.O + (long)b * a.Lq * a.so + h * DH;
  const bf16_t* dOb = (const bf16_t*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  const unsigned sk2 = (unsigned)a.sk * 2u, sv2 = (unsigned)a.sv * 2u;
  const int nqg = (a.Lq + 31) >> 5, qg = 4 * bxi + w;
  const unsigned* lbits = (const unsigned*)(a.dbits + (long)a.B * a.H * nqg * ntiles * 32);
  auto fill = [&](int tt, int st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int R = 16 * w + 8 * u;
      const int r = 64 * tt + R + (lane >> 3), pch = lane & 7;
      const unsigned rr = (unsigned)min(r, a.Lk - 1);
      dma16_sv(Kb, rr * sk2 + (unsigned)((pch ^ dsw(r)) << 4), kst + st * A7_TB + R * 128);
      dma16_sv(Vb, rr * sv2 + (unsigned)((pch ^ ((r >> 1) & 7)) << 4), vst + st * A7_TB + R * 128);
    }
    if constexpr (DROP)
      dma4_sv(lbits, (unsigned)(lb_dword(bh, nqg, ntiles, min(qg, nqg - 1), tt) + lane) * 4u,
              (const unsigned char*)(kbl + st * 256 + w * 64));
  };

  // ---- prologue: tile 0's stream; Q (pre-scaled), dO, O fragments; the key mask; delta and the row terms
  fill(0, 0);
  const float sl2 = a.scale * 1.4426950408889634f;
  uint4 qf[4], dof[4];
  float dl = 0.f;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    // rows past Lq read row Lq - 1 (valid memory) and are zeroed: no contribution, never stored
    const long c = 16 * ks + 8 * hh, qc = min(q, a.Lq - 1);
    const unsigned zm = qv ? 0xFFFFFFFFu : 0u;
    const uint4 x = *(const uint4*)(Qb + qc * a.sq + c);
    const uint4 xo = *(const uint4*)(dOb + qc * a.sdo + c);
    const uint4 y = *(const uint4*)(Ob + qc * a.so + c);
    dof[ks] = make_uint4(xo.x & zm, xo.y & zm, xo.z & zm, xo.w & zm);
    qf[ks] = scale_frag(make_uint4(x.x & zm, x.y & zm, x.z & zm, x.w & zm), sl2);
    const u32x4v_t xd = __builtin_bit_cast(u32x4v_t, dof[ks]), yo = __builtin_bit_cast(u32x4v_t, y);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      dl += __uint_as_float(xd[j] << 16) * __uint_as_float(yo[j] << 16) +
            __uint_as_float(xd[j] & 0xFFFF0000u) * __uint_as_float(yo[j] & 0xFFFF0000u);
  }
  dl = xsum32(dl);  // delta = rowsum(dO * O) over the query's 64 columns (lanes l, l ^ 32)
  const float lse2 = qv ? a.lse[(long)bh * a.Lq + q] * 1.4426950408889634f : 0.f;
  if (hh == 0 && q < LqP) {
    a.delta[(long)bh * LqP + q] = qv ? dl : 0.f;
    a.delta[(long)a.B * a.H * LqP + (long)bh * LqP + q] = qv ? -lse2 : -INFINITY;
  }
  // the query's fifth-k-step operand: (-lse2 hi, -lse2 lo, 1, 0, ...) on the lanes of the first 8 k positions
  const uint4 q5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(neg_split(lse2), pk_bf16(1.f, 0.f), 0u, 0u);
  unsigned tmask = ntiles >= 32 ? 0xFFFFFFFFu : ((1u << ntiles) - 1u);
  if constexpr (MK != 0) {
    bool any = false;
    if (4 * tid < LkP) {
      unsigned mv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 4 * tid + j;
        const bool ok = k < a.Lk && (MK == 1 || a.key_keep[(long)b * a.Lk + k] != 0);
        mv[j] = pk_bf16(ok ? 0.f : -INFINITY, 0.f);
        any |= ok;
      }
      *(uint4*)(mpk + 4 * tid) = make_uint4(mv[0], mv[1], mv[2], mv[3]);
    }
    if constexpr (MK == 2) {
      const unsigned long long bal = __ballot(any);
      if (lane == 0) {
        unsigned nib = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) nib |= ((bal >> (16 * j)) & 0xFFFFull) ? (1u << j) : 0u;
        tact[w] = nib;
      }
    }
  }
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    pin16(qf[ks]);
    pin16(dof[ks]);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (MK == 2) tmask &= tact[0] | (tact[1] << 4) | (tact[2] << 8) | (tact[3] << 12);

  int koff[4], voffr[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    koff[ks] = qi * 128 + (((2 * ks + hh) ^ dsw(qi)) << 4);
    voffr[ks] = qi * 128 + (((2 * ks + hh) ^ ((qi >> 1) & 7)) << 4);
  }
  // K^T transposed reads: 16-lane group G reads rows kb0 + 4 hh + (i >> 2) (+ 8 for the hi half), units 8 db + 4 (G &
  // 1) + (i & 3); the row's dsw depends only on hh, the hi half and i >> 3 (kb0 is a multiple of 16)
  const int vi = lane & 15;
  int ktr[2][2];
#pragma unroll
  for (int hi = 0; hi < 2; ++hi) {
    const int row = 4 * hh + 8 * hi + (vi >> 2);
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int u = 8 * db + 4 * ((lane >> 4) & 1) + (vi & 3);
      ktr[hi][db] = row * 128 + ((((u >> 1) ^ dsw(row)) << 1 | (u & 1)) << 3);
    }
  }
  f32x16_t g0 = {}, g1 = {};  // dQ^T, d-blocks 0 / 1

  auto tile = [&](const int t, const int st) {
    const bool mt = MK == 2 || (MK == 1 && t == ntiles - 1);  // this tile's keys carry a mask
    const unsigned char* kimg = kst + st * A7_TB;
    const unsigned char* vimg = vst + st * A7_TB;
    unsigned kw = 0xFFFFFFFFu;
    if constexpr (DROP) kw = kbl[st * 256 + w * 64 + lane];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // the key's fifth-k-step operand: (1, 1, mask, 0, ...) on the lanes of the first 8 k positions
      unsigned mk = 0u;
      if (MK != 0 && mt) mk = mpk[64 * t + 32 * kb + qi];
      const uint4 k5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(1.f, 1.f), mk, 0u, 0u);
      f32x16_t sc = mfma32(k5, q5, f32x16_t{});
      f32x16_t dp = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        sc = mfma32(*(const uint4*)(kimg + koff[ks] + kb * 32 * 128), qf[ks], sc);
        dp = mfma32(*(const uint4*)(vimg + voffr[ks] + kb * 32 * 128), dof[ks], dp);
      }
      uint4 bs[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        unsigned bw[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int r = 8 * s + 2 * jj;
          float d0 = dp[r], d1 = dp[r + 1];
          if constexpr (DROP) {  // keep ? dscale dP - delta : -delta (keep bit lb_bit(kb, r) as an AND mask)
            d0 = fmaf(__uint_as_float(__float_as_uint(d0) & (unsigned)__builtin_amdgcn_sbfe((int)kw, lb_bit(kb, r), 1)),
                      a.drop_scale, -dl);
            d1 = fmaf(__uint_as_float(__float_as_uint(d1) & (unsigned)__builtin_amdgcn_sbfe((int)kw, lb_bit(kb, r + 1), 1)),
                      a.drop_scale, -dl);
          } else {
            d0 -= dl;
            d1 -= dl;
          }
          bw[jj] = pk_bf16(__builtin_amdgcn_exp2f(sc[r]) * d0, __builtin_amdgcn_exp2f(sc[r + 1]) * d1);
        }
        bs[s] = make_uint4(bw[0], bw[1], bw[2], bw[3]);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int rb = (32 * kb + 16 * s) * 128;
        const uint4 k0 = join_tr(tr_read(kimg + ktr[0][0] + rb), tr_read(kimg + ktr[1][0] + rb));
        const uint4 k1 = join_tr(tr_read(kimg + ktr[0][1] + rb), tr_read(kimg + ktr[1][1] + rb));
        g0 = mfma32(k0, bs[s], g0);
        g1 = mfma32(k1, bs[s], g1);
      }
    }
  };

  int t = 0, st = 0;
  bool act = (tmask & 1u) != 0;
  while (true) {
    const unsigned rest = t + 1 < 32 ? (tmask & ~((2u << t) - 1u)) : 0u;
    const int tn = rest ? __builtin_ctz(rest) : -1;
    if (tn >= 0) fill(tn, st ^ 1);
    if (act) tile(t, st);
    if (tn < 0) break;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    t = tn;
    st ^= 1;
    act = true;
  }

  if (q < LqP) {  // the pre-scaled Q dkv7 streams: the same bf16 scores as the forward and this kernel
    uint4* qs = (uint4*)(a.delta + 2L * a.B * a.H * LqP) + ((long)bh * LqP + q) * 8 + hh;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) qs[2 * ks] = qf[ks];
  }
  // ---- epilogue: dQ = scale * dQ^T, staged per wave in LDS (K ring, free after the barrier), stored as rows
  __syncthreads();
  unsigned char* ost = kst + w * 4096;
#pragma unroll
  for (int db = 0; db < 2; ++db) {
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
      const f32x16_t& gg = db ? g1 : g0;
      uint2 u2;
      u2.x = pk_bf16(gg[4 * mm] * a.scale, gg[4 * mm + 1] * a.scale);
      u2.y = pk_bf16(gg[4 * mm + 2] * a.scale, gg[4 * mm + 3] * a.scale);
      *(uint2*)(ost + qi * 128 + (((4 * db + mm) ^ (qi & 7)) << 4) + 8 * hh) = u2;
    }
  }
  bf16_t* dQb = (bf16_t*)a.dQ + (long)b * a.Lq * a.sdq + h * DH;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (lane >> 3) + 8 * i, c = lane & 7;
    const uint4 v = *(const uint4*)(ost + row * 128 + ((c ^ (row & 7)) << 4));
    if (qw0 + row < a.Lq) *(uint4*)(dQb + (long)(qw0 + row) * a.sdq + c * 8) = v;
  }
}

// dK / dV, key-owned (4 waves x 32 keys per workgroup, Q / dO tiles of 64 queries streamed through a 2-stage LDS-DMA
// ring with the tiles' row terms nlse2 / delta from dq7 and the forward's keep words). Per 32-query half:
// S'' = Q' K^T over 4 k-steps (Q' = the pre-scaled Q dq7 wrote, bf16-identical to the forward's and dq7's register
// operand, so p is the forward's probability; K in registers) plus a fifth k-step that adds the row's -LSE (log2
// units, hi + lo bf16), p = exp2(S''); dP = dO V^T; dS = p (keep dscale dP - delta); dV^T += dO^T (p keep) and
// dK^T += Q'^T dS (x ln 2 = scale / sl2 at the end) with the key on the MFMA lane: the score accumulators are the B
// operands (no LDS round trip), and the Q' / dO images serve both the row reads and the transposed reads. Keys that
// are padding get zero gradients.
template <int DM, bool MASK>
__global__ void __launch_bounds__(256, 2) dkv7_kernel(AttnArgs a) {
  constexpr bool DROP = DM != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smk7[];
  const int ntiles = (a.Lk + 63) >> 6, nqt = (a.Lq + 63) >> 6, LqP = nqt * 64;
  unsigned char* qst = smk7;                      // [2][64 rows][128 B] Q, dsw swizzle
  unsigned char* dost = smk7 + 2 * A7_TB;         // [2][64 rows][128 B] dO, dsw swizzle
  float* rowt = (float*)(smk7 + 4 * A7_TB);       // [2][nlse2 64 | delta 64]
  unsigned* kwd = (unsigned*)(smk7 + 4 * A7_TB + 1024);  // [2][4 waves][2 query groups][16 words] keep masks
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, qi = lane & 31;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh - b * a.H;
  const int kw0 = bxi * 128 + 32 * w;
  const int kk = kw0 + qi;
  const bool kv = kk < a.Lk && (!MASK || a.key_keep[(long)b * a.Lk + min(kk, a.Lk - 1)] != 0);
  const bf16_t* Qb = (const bf16_t*)(a.delta + 2L * a.B * a.H * LqP) + (long)bh * LqP * DH;  // Q' rows, 128 B
  const bf16_t* dOb = (const bf16_t*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  const float* nlse_g = a.delta + (long)a.B * a.H * LqP + (long)bh * LqP;
  const float* dlt_g = a.delta + (long)bh * LqP;
  const unsigned sq2 = (unsigned)DH * 2u, sdo2 = (unsigned)a.sdo * 2u;
  // the keep masks (layout v3) of the wave's 32 keys: slots 16 kbw .. 16 kbw + 15 of key tile tw, for both 32-query
  // groups of a 64-query tile (one 256-B piece per wave and tile); the lane's word is slot rpk of its key
  const int nqg = (a.Lq + 31) >> 5, tw = min(kw0 >> 6, ntiles - 1), kbw = (kw0 >> 5) & 1;
  const int kt = kk & 63, rpk = 4 * ((kt >> 3) & 3) + (kt & 3), ksh = 4 * hh + 32 * ((kt >> 2) & 1);
  auto fill = [&](int uu, int st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int R = 16 * w + 8 * u;
      const int r = 64 * uu + R + (lane >> 3), pch = lane & 7;
      const unsigned rr = (unsigned)min(r, a.Lq - 1);
      dma16_sv(Qb, rr * sq2 + (unsigned)((pch ^ dsw(r)) << 4), qst + st * A7_TB + R * 128);
      dma16_sv(dOb, rr * sdo2 + (unsigned)((pch ^ dsw(r)) << 4), dost + st * A7_TB + R * 128);
    }
    if (w == 0) dma4_sv(nlse_g, (unsigned)(64 * uu + lane) * 4u, (const unsigned char*)(rowt + st * 128));
    if (w == 1) dma4_sv(dlt_g, (unsigned)(64 * uu + lane) * 4u, (const unsigned char*)(rowt + st * 128 + 64));
    if constexpr (DROP) {
      const int qgl = min(2 * uu + (lane >> 5), nqg - 1);
      dma4_sv(a.dbits, (unsigned)((lm_word(bh, nqg, ntiles, qgl, tw) + 16 * kbw) * 8 + (lane & 31) * 4),
              (const unsigned char*)(kwd + st * 256 + w * 64));
    }
  };

  fill(0, 0);
  const int kc = min(kk, a.Lk - 1);
  uint4 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const long c = 16 * ks + 8 * hh;
    kf[ks] = *(const uint4*)(Kb + (long)kc * a.sk + c);
    vf[ks] = *(const uint4*)(Vb + (long)kc * a.sv + c);
  }
  // the key's fifth-k-step operand (1, 1, 0, ...) on the lanes of the first 8 k positions
  const uint4 b5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(1.f, 1.f), 0u, 0u, 0u);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    pin16(kf[ks]);
    pin16(vf[ks]);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  int qoff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qoff[ks] = qi * 128 + (((2 * ks + hh) ^ dsw(qi)) << 4);
  const int vi = lane & 15;
  int ttr[2][2];
#pragma unroll
  for (int hi = 0; hi < 2; ++hi) {
    const int row = 4 * hh + 8 * hi + (vi >> 2);
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int u = 8 * db + 4 * ((lane >> 4) & 1) + (vi & 3);
      ttr[hi][db] = row * 128 + ((((u >> 1) ^ dsw(row)) << 1 | (u & 1)) << 3);
    }
  }
  f32x16_t gk0 = {}, gk1 = {}, gv0 = {}, gv1 = {};  // dK^T, dV^T, d-blocks 0 / 1

  auto tile = [&](const int st) {
    const unsigned char* qimg = qst + st * A7_TB;
    const unsigned char* doimg = dost + st * A7_TB;
    const float* nl = rowt + st * 128;
    const float* dl = nl + 64;
    const unsigned* kd = kwd + st * 256 + w * 64;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      // register r of this half is query 32 qb + 8 (r >> 2) + 4 hh + (r & 3): bit 8 (r >> 2) + (r & 3) of kbits
      unsigned kbits = 0xFFFFFFFFu;
      if constexpr (DROP) kbits = (unsigned)(*(const uint64_t*)(kd + 32 * qb + 2 * rpk) >> ksh);
      // the query row's fifth-k-step operand (-LSE log2(e) as hi + lo bf16) on the lanes of the first 8 k positions
      const float x = nl[32 * qb + qi];
      const float xh = __uint_as_float(((unsigned)pk_bf16(x, 0.f)) << 16);
      const float xl = (x == -INFINITY) ? 0.f : x - xh;
      const uint4 a5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(xh, xl), 0u, 0u, 0u);
      f32x16_t sc = mfma32(a5, b5, f32x16_t{});
      f32x16_t dp = {};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        sc = mfma32(*(const uint4*)(qimg + qoff[ks] + qb * 32 * 128), kf[ks], sc);
        dp = mfma32(*(const uint4*)(doimg + qoff[ks] + qb * 32 * 128), vf[ks], dp);
      }
      uint4 bp[2], bs[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        unsigned pw[4], sw[4];
#pragma unroll
        for (int mh = 0; mh < 2; ++mh) {
          // registers r = 8 s + 4 mh .. + 3: queries 32 qb + 8 (2 s + mh) + 4 hh + 0 .. 3
          const int r0 = 8 * s + 4 * mh, qr = 32 * qb + 8 * (2 * s + mh) + 4 * hh;
          const f32x4_t d4 = *(const f32x4_t*)(dl + qr);
          float pv[4], dv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pr = __builtin_amdgcn_exp2f(sc[r0 + e]);
            float dd = dp[r0 + e];
            if constexpr (DROP) {
              const unsigned m = (unsigned)__builtin_amdgcn_sbfe((int)kbits, 8 * (2 * s + mh) + e, 1);
              pv[e] = __uint_as_float(__float_as_uint(pr) & m);
              dd = fmaf(__uint_as_float(__float_as_uint(dd) & m), a.drop_scale, -d4[e]);
            } else {
              pv[e] = pr;
              dd -= d4[e];
            }
            dv[e] = pr * dd;
          }
          pw[2 * mh] = pk_bf16(pv[0], pv[1]);
          pw[2 * mh + 1] = pk_bf16(pv[2], pv[3]);
          sw[2 * mh] = pk_bf16(dv[0], dv[1]);
          sw[2 * mh + 1] = pk_bf16(dv[2], dv[3]);
        }
        bp[s] = make_uint4(pw[0], pw[1], pw[2], pw[3]);
        bs[s] = make_uint4(sw[0], sw[1], sw[2], sw[3]);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int rb = (32 * qb + 16 * s) * 128;
        const uint4 o0 = join_tr(tr_read(doimg + ttr[0][0] + rb), tr_read(doimg + ttr[1][0] + rb));
        const uint4 o1 = join_tr(tr_read(doimg + ttr[0][1] + rb), tr_read(doimg + ttr[1][1] + rb));
        gv0 = mfma32(o0, bp[s], gv0);
        gv1 = mfma32(o1, bp[s], gv1);
        const uint4 q0 = join_tr(tr_read(qimg + ttr[0][0] + rb), tr_read(qimg + ttr[1][0] + rb));
        const uint4 q1 = join_tr(tr_read(qimg + ttr[0][1] + rb), tr_read(qimg + ttr[1][1] + rb));
        gk0 = mfma32(q0, bs[s], gk0);
        gk1 = mfma32(q1, bs[s], gk1);
      }
    }
  };

  int st = 0;
  for (int uu = 0; uu < nqt; ++uu) {
    if (uu + 1 < nqt) fill(uu + 1, st ^ 1);
    tile(st);
    if (uu + 1 < nqt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      st ^= 1;
    }
  }

  // ---- epilogue: dV = dscale dV^T, dK = scale dK^T = ln 2 (Q'^T dS) (zero for padding keys), staged per wave in
  // LDS, stored as rows
  __syncthreads();
  unsigned char* ost = qst + w * 4096;
  const float fv = kv ? (DROP ? a.drop_scale : 1.f) : 0.f, fk = kv ? 0.6931471805599453f : 0.f;
#pragma unroll
  for (int which = 0; which < 2; ++which) {
    const float f = which ? fk : fv;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        const f32x16_t& gg = which ? (db ? gk1 : gk0) : (db ? gv1 : gv0);
        uint2 u2;
        u2.x = pk_bf16(gg[4 * mm] * f, gg[4 * mm + 1] * f);
        u2.y = pk_bf16(gg[4 * mm + 2] * f, gg[4 * mm + 3] * f);
        *(uint2*)(ost + qi * 128 + (((4 * db + mm) ^ (qi & 7)) << 4) + 8 * hh) = u2;
      }
    }
    bf16_t* Gb = which ? (bf16_t*)a.dK + (long)b * a.Lk * a.sdk + h * DH : (bf16_t*)a.dV + (long)b * a.Lk * a.sdv + h * DH;
    const long sg = which ? a.sdk : a.sdv;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (lane >> 3) + 8 * i, c = lane & 7;
      const uint4 v = *(const uint4*)(ost + row * 128 + ((c ^ (row & 7)) << 4));
      if (kw0 + row < a.Lk) *(uint4*)(Gb + (long)(kw0 + row) * sg + c * 8) = v;
    }
  }
}

// Fused backward for Lk <= 512: one workgroup of 8 waves x 32 keys holds 256 keys of one (b, h) at a time (one pass
// per 256 keys), so P and dP are computed once (dq7 + dkv7 compute them twice). Per 64-query tile: dkv7's body
// (S'' = Q' K^T with the key on the lane, dP, dS; dV^T and dK^T accumulated), each wave writing its dS^T slice into
// an LDS image ([256 keys][64 queries] bf16, dsw swizzle, zero for padding keys); after the tile's barrier the 4
// waves of the tile's parity compute dQ^T = K^T dS^T over the pass's keys (one 32x32 block each; K^T and dS^T by
// transposed reads of the K image and the dS^T image, dq7's addressing). With one pass dQ is stored at once; with two,
// the first pass leaves each block's f32 partial in the workspace (written and read back by the same lane, no
// synchronisation) and the second adds it. The row terms come one tile ahead from the waves themselves: each thread
// loads 16 B of the next tile's Q, dO and O (8 lanes per query row), writes Q' = bf16(Q scale log2 e) (the forward's
// operand, bit for bit) and dO into the ring, and the row's delta = rowsum(dO O) (8-lane reduction) and -LSE log2 e
// into the row-term slots.
template <int DM, bool MASK, int NP>
__global__ void __launch_bounds__(512, 1) bwdf7_kernel(AttnArgs a) {
  constexpr bool DROP = DM != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smf7[];
  const int ntiles = (a.Lk + 63) >> 6, nqt = (a.Lq + 63) >> 6;  // NP = (Lk + 255) / 256 key passes
  unsigned char* qst = smf7;                              // [2][64 rows][128 B] Q', dsw swizzle
  unsigned char* dost = smf7 + 2 * A7_TB;                 // [2][64 rows][128 B] dO, dsw swizzle
  unsigned char* kim = smf7 + 4 * A7_TB;                  // [256 keys][128 B] K of the pass, dsw swizzle
  unsigned char* dsi = smf7 + 8 * A7_TB;                  // [2][256 keys][128 B] dS^T (64 queries), dsw swizzle
  float* rowt = (float*)(smf7 + 16 * A7_TB);              // [2][nlse2 64 | delta 64]
  unsigned* kwd = (unsigned*)(smf7 + 16 * A7_TB + 1024);  // [2][8 waves][64 dwords] keep masks
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, qi = lane & 31;
  const int bh = blockIdx.x, b = bh / a.H, h = bh - b * a.H;
  const int kr = 32 * w + qi;  // the lane's key within a pass (and its LDS row)
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  const int nqg = (a.Lq + 31) >> 5, kbw = (kr >> 5) & 1;
  const int kt = kr & 63, rpk = 4 * ((kt >> 3) & 3) + (kt & 3), ksh = 4 * hh + 32 * ((kt >> 2) & 1);
  int kk = kr, tw = 0;  // the pass's key of the lane and the wave's 64-key tile

  // ---- row terms of query tile uu into stage st: thread = (row tid >> 3, 16-B chunk tid & 7)
  const int pr_r = tid >> 3, pr_c = tid & 7;
  const float sl2 = a.scale * 1.4426950408889634f;
  uint4 nx, nxo, ny;
  float nlse = 0.f;
  auto pload = [&](int uu) {
    const long qc = min(64 * uu + pr_r, a.Lq - 1);
    const long c = h * DH + pr_c * 8;
    nx = *(const uint4*)((const bf16_t*)a.Q + ((long)b * a.Lq + qc) * a.sq + c);
    nxo = *(const uint4*)((const bf16_t*)a.dO + ((long)b * a.Lq + qc) * a.sdo + c);
    ny = *(const uint4*)((const bf16_t*)a.O + ((long)b * a.Lq + qc) * a.so + c);
    nlse = a.lse[(long)bh * a.Lq + qc];
  };
  auto pstore = [&](int uu, int st) {
    const bool qv = 64 * uu + pr_r < a.Lq;
    const unsigned zm = qv ? 0xFFFFFFFFu : 0u;
    const uint4 xd = make_uint4(nxo.x & zm, nxo.y & zm, nxo.z & zm, nxo.w & zm);
    const u32x4v_t xv = __builtin_bit_cast(u32x4v_t, xd), yv = __builtin_bit_cast(u32x4v_t, ny);
    float dl = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      dl += __uint_as_float(xv[j] << 16) * __uint_as_float(yv[j] << 16) +
            __uint_as_float(xv[j] & 0xFFFF0000u) * __uint_as_float(yv[j] & 0xFFFF0000u);
    dl += __shfl_xor(dl, 1);
    dl += __shfl_xor(dl, 2);
    dl += __shfl_xor(dl, 4);
    const int off = st * A7_TB + pr_r * 128 + ((pr_c ^ dsw(pr_r)) << 4);
    *(uint4*)(qst + off) = scale_frag(make_uint4(nx.x & zm, nx.y & zm, nx.z & zm, nx.w & zm), sl2);
    *(uint4*)(dost + off) = xd;
    if (pr_c == 0) {
      rowt[st * 128 + pr_r] = qv ? -(nlse * 1.4426950408889634f) : -INFINITY;
      rowt[st * 128 + 64 + pr_r] = qv ? dl : 0.f;
    }
  };
  auto kmask = [&](int uu, int st) {  // the keep masks of the wave's 32 keys for query tile uu (as dkv7)
    if constexpr (DROP) {
      const int qgl = min(2 * uu + (lane >> 5), nqg - 1);
      dma4_sv(a.dbits, (unsigned)((lm_word(bh, nqg, ntiles, qgl, tw) + 16 * kbw) * 8 + (lane & 31) * 4),
              (const unsigned char*)(kwd + st * 512 + w * 64));
    }
  };

  int qoff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qoff[ks] = qi * 128 + (((2 * ks + hh) ^ dsw(qi)) << 4);
  const int vi = lane & 15;
  int ttr[2][2];
#pragma unroll
  for (int hi = 0; hi < 2; ++hi) {
    const int row = 4 * hh + 8 * hi + (vi >> 2);
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int u = 8 * db + 4 * ((lane >> 4) & 1) + (vi & 3);
      ttr[hi][db] = row * 128 + ((((u >> 1) ^ dsw(row)) << 1 | (u & 1)) << 3);
    }
  }
  // the dQ block of this wave (when its parity group runs dQ): d-block w & 1, query half (w >> 1) & 1
  const int dqd = w & 1, dqq = (w >> 1) & 1;
  const int ka0 = dqd ? ttr[0][1] : ttr[0][0], ka1 = dqd ? ttr[1][1] : ttr[1][0];
  const int sb0 = dqq ? ttr[0][1] : ttr[0][0], sb1 = dqq ? ttr[1][1] : ttr[1][0];
  const uint4 b5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(1.f, 1.f), 0u, 0u, 0u);
  bf16_t* dQb = (bf16_t*)a.dQ + (long)b * a.Lq * a.sdq + h * DH;
  const int dsw_k = dsw(kr);

#pragma unroll
  for (int pass = 0; pass < NP; ++pass) {
    kk = 256 * pass + kr;
    tw = min(kk >> 6, ntiles - 1);
    const bool kv = kk < a.Lk && (!MASK || a.key_keep[(long)b * a.Lk + min(kk, a.Lk - 1)] != 0);
    const unsigned kvm = kv ? 0xFFFFFFFFu : 0u;
    const int nks = (min(256, a.Lk - 256 * pass) + 15) >> 4;  // 16-key steps holding a key < Lk
    const bool first = NP == 1 || pass == 0, last = NP == 1 || pass == NP - 1;

    // ---- prologue: the lane's K / V rows (registers) and the K image; tile 0's row terms and keep masks
    const int kc = min(kk, a.Lk - 1);
    uint4 kf[4], vf[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const long c = 16 * ks + 8 * hh;
      kf[ks] = *(const uint4*)(Kb + (long)kc * a.sk + c);
      vf[ks] = *(const uint4*)(Vb + (long)kc * a.sv + c);
    }
    kmask(0, 0);
    pload(0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) *(uint4*)(kim + kr * 128 + (((2 * ks + hh) ^ dsw_k) << 4)) = kf[ks];
    pstore(0, 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      pin16(kf[ks]);
      pin16(vf[ks]);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    f32x16_t gk0 = {}, gk1 = {}, gv0 = {}, gv1 = {};  // dK^T, dV^T, d-blocks 0 / 1

    auto tile = [&](const int st) {
      const unsigned char* qimg = qst + st * A7_TB;
      const unsigned char* doimg = dost + st * A7_TB;
      unsigned char* dsimg = dsi + st * 4 * A7_TB + kr * 128;
      const float* nl = rowt + st * 128;
      const float* dl = nl + 64;
      const unsigned* kd = kwd + st * 512 + w * 64;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        unsigned kbits = 0xFFFFFFFFu;
        if constexpr (DROP) kbits = (unsigned)(*(const uint64_t*)(kd + 32 * qb + 2 * rpk) >> ksh);
        const float x = nl[32 * qb + qi];
        const float xh = __uint_as_float(((unsigned)pk_bf16(x, 0.f)) << 16);
        const float xl = (x == -INFINITY) ? 0.f : x - xh;
        const uint4 a5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(xh, xl), 0u, 0u, 0u);
        f32x16_t sc = mfma32(a5, b5, f32x16_t{});
        f32x16_t dp = {};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          sc = mfma32(*(const uint4*)(qimg + qoff[ks] + qb * 32 * 128), kf[ks], sc);
          dp = mfma32(*(const uint4*)(doimg + qoff[ks] + qb * 32 * 128), vf[ks], dp);
        }
        uint4 bp[2], bs[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          unsigned pw[4], sw[4];
#pragma unroll
          for (int mh = 0; mh < 2; ++mh) {
            const int r0 = 8 * s + 4 * mh, qr = 32 * qb + 8 * (2 * s + mh) + 4 * hh;
            const f32x4_t d4 = *(const f32x4_t*)(dl + qr);
            float pv[4], dv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float pr = __builtin_amdgcn_exp2f(sc[r0 + e]);
              float dd = dp[r0 + e];
              if constexpr (DROP) {
                const unsigned m = (unsigned)__builtin_amdgcn_sbfe((int)kbits, 8 * (2 * s + mh) + e, 1);
                pv[e] = __uint_as_float(__float_as_uint(pr) & m);
                dd = fmaf(__uint_as_float(__float_as_uint(dd) & m), a.drop_scale, -d4[e]);
              } else {
                pv[e] = pr;
                dd -= d4[e];
              }
              dv[e] = pr * dd;
            }
            pw[2 * mh] = pk_bf16(pv[0], pv[1]);
            pw[2 * mh + 1] = pk_bf16(pv[2], pv[3]);
            sw[2 * mh] = pk_bf16(dv[0], dv[1]);
            sw[2 * mh + 1] = pk_bf16(dv[2], dv[3]);
            // dS^T for dQ: queries 32 qb + 16 s + 8 mh + 4 hh + 0..3 of the key's row (zero for padding keys)
            *(uint2*)(dsimg + (((4 * qb + 2 * s + mh) ^ dsw_k) << 4) + 8 * hh) =
                make_uint2(sw[2 * mh] & kvm, sw[2 * mh + 1] & kvm);
          }
          bp[s] = make_uint4(pw[0], pw[1], pw[2], pw[3]);
          bs[s] = make_uint4(sw[0], sw[1], sw[2], sw[3]);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int rb = (32 * qb + 16 * s) * 128;
          const uint4 o0 = join_tr(tr_read(doimg + ttr[0][0] + rb), tr_read(doimg + ttr[1][0] + rb));
          const uint4 o1 = join_tr(tr_read(doimg + ttr[0][1] + rb), tr_read(doimg + ttr[1][1] + rb));
          gv0 = mfma32(o0, bp[s], gv0);
          gv1 = mfma32(o1, bp[s], gv1);
          const uint4 q0 = join_tr(tr_read(qimg + ttr[0][0] + rb), tr_read(qimg + ttr[1][0] + rb));
          const uint4 q1 = join_tr(tr_read(qimg + ttr[0][1] + rb), tr_read(qimg + ttr[1][1] + rb));
          gk0 = mfma32(q0, bs[s], gk0);
          gk1 = mfma32(q1, bs[s], gk1);
        }
      }
    };
    // dQ of query tile uu (dS^T image st): this wave's 32x32 block over the pass's 16-key steps; the f32 partial of
    // an earlier pass comes back from the workspace (this lane wrote it), the last pass stores bf16 dQ
    auto dq_tile = [&](const int uu, const int st) {
      const unsigned char* ds = dsi + st * 4 * A7_TB;
      float4* part = (float4*)(a.delta + (((long)bh * nqt + uu) * 4 + 2 * dqq + dqd) * 1024) + lane * 4;
      f32x16_t g = {};
      if (!first) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 v = part[i];
          g[4 * i] = v.x;
          g[4 * i + 1] = v.y;
          g[4 * i + 2] = v.z;
          g[4 * i + 3] = v.w;
        }
      }
#pragma unroll 4
      for (int j = 0; j < nks; ++j) {
        const int rb = j * 16 * 128;
        const uint4 ka = join_tr(tr_read(kim + ka0 + rb), tr_read(kim + ka1 + rb));
        const uint4 sb = join_tr(tr_read(ds + sb0 + rb), tr_read(ds + sb1 + rb));
        g = mfma32(ka, sb, g);
      }
      if (!last) {
#pragma unroll
        for (int i = 0; i < 4; ++i) part[i] = make_float4(g[4 * i], g[4 * i + 1], g[4 * i + 2], g[4 * i + 3]);
        return;
      }
      // register r: d = 32 dqd + 8 (r >> 2) + 4 hh + (r & 3), query 64 uu + 32 dqq + qi
      const int q = 64 * uu + 32 * dqq + qi;
      if (q < a.Lq) {
        bf16_t* row = dQb + (long)q * a.sdq + 32 * dqd + 4 * hh;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          *(uint2*)(row + 8 * rr) = make_uint2(pk_bf16(g[4 * rr] * a.scale, g[4 * rr + 1] * a.scale),
                                               pk_bf16(g[4 * rr + 2] * a.scale, g[4 * rr + 3] * a.scale));
      }
    };

    for (int uu = 0; uu < nqt; ++uu) {
      const int st = uu & 1;
      const bool more = uu + 1 < nqt;
      if (more) {
        kmask(uu + 1, st ^ 1);
        pload(uu + 1);
      }
      tile(st);
      if (more) pstore(uu + 1, st ^ 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // tile uu's dS^T image complete; tile uu + 1's ring stage and row terms in place
      if ((w >> 2) == st) dq_tile(uu, st);
    }

    // ---- the pass's keys: dV = dscale dV^T, dK = ln 2 (Q'^T dS) (zero for padding keys), staged per wave in the
    // Q' / dO ring (every wave is past its last ring read after the barrier), stored as rows
    __syncthreads();
    unsigned char* ost = qst + w * 4096;
    const float fv = kv ? (DROP ? a.drop_scale : 1.f) : 0.f, fk = kv ? 0.6931471805599453f : 0.f;
    const int kw0 = 256 * pass + 32 * w;
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      const float f = which ? fk : fv;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
          const f32x16_t& gg = which ? (db ? gk1 : gk0) : (db ? gv1 : gv0);
          uint2 u2;
          u2.x = pk_bf16(gg[4 * mm] * f, gg[4 * mm + 1] * f);
          u2.y = pk_bf16(gg[4 * mm + 2] * f, gg[4 * mm + 3] * f);
          *(uint2*)(ost + qi * 128 + (((4 * db + mm) ^ (qi & 7)) << 4) + 8 * hh) = u2;
        }
      }
      bf16_t* Gb = which ? (bf16_t*)a.dK + (long)b * a.Lk * a.sdk + h * DH : (bf16_t*)a.dV + (long)b * a.Lk * a.sdv + h * DH;
      const long sg = which ? a.sdk : a.sdv;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (lane >> 3) + 8 * i, c = lane & 7;
        const uint4 v = *(const uint4*)(ost + row * 128 + ((c ^ (row & 7)) << 4));
        if (kw0 + row < a.Lk) *(uint4*)(Gb + (long)(kw0 + row) * sg + c * 8) = v;
      }
    }
    if (!last) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();  // the staging reads are done before the next pass's K image and ring stage 0 are written
    }
  }
}

int attn7_fwd(AttnArgs& a, hipStream_t s) {
  const int dm = a.thr16 == 0 ? 0 : 1;
  const int mk = a.key_keep != nullptr ? 2 : (a.Lk % 64) != 0 ? 1 : 0;
  const int ntiles = (a.Lk + 63) / 64;
  const bool rel = a.table != nullptr;  // the caller checked a gate source (fddm_attn_fwd dispatch)
  if (ntiles > 16 || (rel && dm)) return (int)hipErrorInvalidValue;  // LkP <= 1024; WavLM has no dropout
  const size_t lds = (size_t)4 * A7_TB + (dm ? 2048 : 0) + 16 + (size_t)ntiles * 64 * 4 +
                     (rel ? (size_t)2 * (ntiles * 64 + 160) * 4 : 0);
  dim3 grid((a.Lq + 127) / 128, a.B * a.H);
#define FWD7(D, M) hipLaunchKernelGGL((fwd7_kernel<D, M>), grid, dim3(256), lds, s, a)
#define FWD7R(M) hipLaunchKernelGGL((fwd7_kernel<0, M, true>), grid, dim3(256), lds, s, a)
  if (rel) { if (mk == 2) FWD7R(2); else if (mk == 1) FWD7R(1); else FWD7R(0); }
  else if (dm) { if (mk == 2) FWD7(1, 2); else if (mk == 1) FWD7(1, 1); else FWD7(1, 0); }
  else { if (mk == 2) FWD7(0, 2); else if (mk == 1) FWD7(0, 1); else FWD7(0, 0); }
#undef FWD7R
#undef FWD7
  return (int)hipGetLastError();
}

int attn7_dq(AttnArgs& a, hipStream_t s) {
  const int dm = a.thr16 == 0 ? 0 : 1;
  const int mk = a.key_keep != nullptr ? 2 : (a.Lk % 64) != 0 ? 1 : 0;
  const int ntiles = (a.Lk + 63) / 64;
  const size_t lds = (size_t)4 * A7_TB + 2064 + (size_t)ntiles * 64 * 4;
  dim3 grid((a.Lq + 127) / 128, a.B * a.H);
#define DQ7(D, M) hipLaunchKernelGGL((dq7_kernel<D, M>), grid, dim3(256), lds, s, a)
  if (dm) { if (mk == 2) DQ7(1, 2); else if (mk == 1) DQ7(1, 1); else DQ7(1, 0); }
  else { if (mk == 2) DQ7(0, 2); else if (mk == 1) DQ7(0, 1); else DQ7(0, 0); }
#undef DQ7
  return (int)hipGetLastError();
}

int attn7_dkv(AttnArgs& a, hipStream_t s) {
  const int dm = a.thr16 == 0 ? 0 : 1;
  const size_t lds = (size_t)4 * A7_TB + 1024 + 2048;
  dim3 grid((a.Lk + 127) / 128, a.B * a.H);
#define DKV7(D, M) hipLaunchKernelGGL((dkv7_kernel<D, M>), grid, dim3(256), lds, s, a)
  if (dm) { if (a.key_keep) DKV7(1, true); else DKV7(1, false); }
  else { if (a.key_keep) DKV7(0, true); else DKV7(0, false); }
#undef DKV7
  return (int)hipGetLastError();
}

int attn7_bwdf(AttnArgs& a, hipStream_t s) {
  // two key passes keep a per-lane f32 dQ partial of 64 floats per query row in the workspace (fddm_attn_bwd_ws_floats)
  if (a.Lk > 512 || (a.Lk > 256 && a.delta == nullptr)) return (int)hipErrorInvalidValue;
  const int dm = a.thr16 == 0 ? 0 : 1;
  const size_t lds = (size_t)16 * A7_TB + 1024 + 4096;
  dim3 grid(a.B * a.H);
#define BWF7(D, M, P) hipLaunchKernelGGL((bwdf7_kernel<D, M, P>), grid, dim3(512), lds, s, a)
  if (a.Lk <= 256) {
    if (dm) { if (a.key_keep) BWF7(1, true, 1); else BWF7(1, false, 1); }
    else { if (a.key_keep) BWF7(0, true, 1); else BWF7(0, false, 1); }
  } else {
    if (dm) { if (a.key_keep) BWF7(1, true, 2); else BWF7(1, false, 2); }
    else { if (a.key_keep) BWF7(0, true, 2); else BWF7(0, false, 2); }
  }
#undef BWF7
  return (int)hipGetLastError();
}

}  // namespace attn
}  // namespace fddm
