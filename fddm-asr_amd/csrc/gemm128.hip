// 128x128 bf16 GEMM for gfx950 (MI355X) with an LDS-DMA ring:  C[m][n] = alpha * sum_k A(m,k) * B(n,k) (+ epilogue)
//
// The GEMMs of the decoder whose output is too small for the 256x256 kernel (gemm256.hip) to fill 256 CUs:
// d_model-wide outputs (8192 tokens x 512: 64 tiles of 256x256, 256 tiles of 128x128), their input gradients
// (dX = dY W, W read as stored, [out][in] = M/N-contiguous) and the weight gradients (dW = dY^T X, both operands
// token-major). Each operand is K-contiguous ("KC", [rows][K]) or row-contiguous ("MC", [K][rows]); a
// workgroup computes one 128x128 tile (split-K slice) in one pass, so its whole K walk is pipelined:
//
//   4 waves (2 x 2), 64x64 outputs each = 4 x 4 MFMA 16x16x32 blocks (64 f32 accumulators per lane).
//   LDS: a 4-stage ring of K-tiles (BK = 64), 16 KB per operand per stage, filled by LDS-DMA
//   (buffer_load ... lds, 16 B per lane, 8 instructions per wave per K-tile), three K-tiles in flight.
//     KC image: [128 rows][128 B], 16-B chunk c of row r at r*128 + ((c ^ ((r>>1)&7))<<4)   -> ds_read_b128
//     MC image: [64 k][256 B],    16-B chunk c of k-row k at k*256 + ((c ^ sw(k))<<4),
//               sw(k) = ((k&3)<<1) | (((k>>3)&1)<<3)                                        -> ds_read_b64_tr_b16
//     (the swizzle is applied to the DMA's per-lane SOURCE address; both reads are bank-conflict-free)
//   K-tile t:  wait fragments(t, k-half 0) | read fragments(t, k-half 1) | 16 MFMAs (t, 0) |
//              wait reads; vmcnt: K-tile t+1 landed | s_barrier | LDS-DMA K-tile t+4 into t's stage |
//              read fragments(t+1, 0) | 16 MFMAs (t, 1)
//   Every vmcnt is a compile-time count (8 DMA instructions per K-tile; past the end the last K-tile is re-read).
//   MFMA operands are swapped (C^T fragments): a lane owns 4 consecutive columns of one row, so the epilogue
//   stores 8 B (bf16) / 16 B (f32) per block straight from the accumulators; the f32-accumulate epilogue
//   (weight gradients, split-K) goes through LDS so every atomic instruction adds 256 contiguous bytes.
//   Ragged M / N: the last tile is the full tile ending at M (N) — recomputed overlap is masked only where it
//   would be added twice (f32 accumulate). Ragged K (token counts): MC operands read zeros past their end
//   (buffer range checking); KC operands need K % 64 == 0.
//   Optional fused bias gradient for an MC A operand: colsum[m] += sum_k A(m,k), accumulated from the A
//   fragments with v_dot2_f32_bf16 by the waves of the first column of tiles.
#include "gemm.h"
#include "lds_dma.h"

namespace fddm {
namespace g128 {
using namespace ldsdma;

#ifndef G128_NST
#define G128_NST 4
#endif
constexpr int BM = 128, BN = 128, OPB = 16384, STAGE = 2 * OPB, NST = G128_NST, LDS_BYTES = NST * STAGE;
constexpr int DPW = 4;  // LDS-DMA instructions per K-tile per wave (2 A + 2 B)

#ifdef G128_STAMPS
// diagnostic build only: s_memtime stamps per workgroup (fddm_gemm128_stamps reads them)
constexpr int NSTAMP = G128_STAMPS;
__device__ unsigned long long g128_stamps[2048 * NSTAMP];
#define STAMP(slot) do { if (threadIdx.x == 0 && blockIdx.x < 2048) g128_stamps[blockIdx.x * NSTAMP + (slot)] = __builtin_amdgcn_s_memtime(); } while (0)
#ifdef G128_FINE
// fine mode: wave 0's steps inside K-tiles 8..15: slot 2 + (t-8)*5 + e
#define FSTAMP(t, e) do { if ((t) >= 8 && (t) < 16) STAMP(2 + ((t) - 8) * 5 + (e)); } while (0)
#else
#define FSTAMP(t, e) do {} while (0)
#endif
#else
#define STAMP(slot) do {} while (0)
#define FSTAMP(t, e) do {} while (0)
#endif

__device__ __forceinline__ int mc_sw(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }

// per-lane DMA source byte offsets (tile origin r0 included) of a wave's 2 instructions for one operand image
// (16 wave-instructions of 1 KB fill a 16-KB image: wave w issues numbers 2w, 2w+1)
// rope: the MC image's 128 columns are 64 of the first half of the output and their RoPE partners 64 further in the
// second half (rh = N / 2): logical chunk 8 wc + q holds columns r0 + 32 wc + 8 q (q < 4) or r0 + rh + 32 wc + 8 (q - 4)
template <bool KC>
__device__ __forceinline__ void dma_offsets(int (&v)[2], int wid, int lane, int r0, int ld, int rh = 0) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int gi = wid * 2 + u;
    if (KC) {
      const int R = gi * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((R >> 1) & 7);
      v[u] = ((r0 + R) * ld + c * 8) * 2;
    } else {
      const int k = gi * 4 + (lane >> 4);
      const int c = (lane & 15) ^ mc_sw(k);
      const int col = rh ? r0 + ((c >> 3) << 5) + ((c >> 2) & 1) * rh + ((c & 3) << 3) : r0 + c * 8;
      v[u] = (k * ld + col) * 2;
    }
  }
}

// fragment of block I (rows/cols rb + 16*I of the image) of a KC image (base: lane address of block 0, k-half
// included) or an MC image (base: lane address of block I, k-half included)
template <int I>
__device__ __forceinline__ u32x4_t frag_kc(unsigned base) {
  return ds_read128_at<I * 2048>(base);
}
__device__ __forceinline__ u32x4_t frag_mc(unsigned base) {
  const u32x2_t lo = ds_read_tr16_at<0>(base);
  const u32x2_t hi = ds_read_tr16_at<1024>(base);
  return u32x4_t{lo[0], lo[1], hi[0], hi[1]};
}

template <bool AKC, bool BKC, int EPI, typename OT>
__device__ __forceinline__ void tile128(const GemmArgs& g, unsigned char* smem, int bx, int by, int bz, int nz) {
  STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2, w4 = wid & 3, wr = w4 >> 1, wc = w4 & 1;  // grp = k-half of every K-tile
  const int fr = lane & 15, fg = lane >> 4;
  const int M = (int)g.M, N = (int)g.N;
  constexpr bool ROPE = EPI == EPI_ROPE_ACC;
  const int m0 = min(by * BM, M - BM), n0 = ROPE ? bx * (BN / 2) : min(bx * BN, N - BN);
  const int lda = (int)g.lda, ldb = (int)g.ldb;
  int kbeg = 0, kend = (int)g.K;
  if (nz > 1) {
    kbeg = bz * (int)g.ksplit;
    kend = min(kend, kbeg + (int)g.ksplit);
  }
  const int nk = (kend - kbeg + 63) / 64;

  // operand buffers: MC operands are range-checked at their last k-row (the ragged tail is masked below)
  const unsigned recA = AKC ? 0x7fffffffu : (unsigned)(((long)(g.K - 1) * lda + M) * 2);
  const unsigned recB = BKC ? 0x7fffffffu : (unsigned)(((long)(g.K - 1) * ldb + N) * 2);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, (int)recA, SRD_W3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, (int)recB, SRD_W3);
  int va[2], vb[2];
  dma_offsets<AKC>(va, wid, lane, m0, lda);
  dma_offsets<BKC>(vb, wid, lane, n0, ldb, ROPE ? N / 2 : 0);
  auto issue = [&](int kt, int st) {
    const int kk = kbeg + kt * 64;
    const int sa = AKC ? kk * 2 : kk * lda * 2, sb = BKC ? kk * 2 : kk * ldb * 2;
    unsigned char* d = smem + st * STAGE + wid * 2048;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lptr_t)d, 16, va[0], sa, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lptr_t)(d + 1024), 16, va[1], sa, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lptr_t)(d + OPB), 16, vb[0], sb, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lptr_t)(d + OPB + 1024), 16, vb[1], sb, 0, 0);
  };

  // fragment lane addresses in stage 0, this wave's k-half (k = 32*grp + 8*fg + 0..7)
  const unsigned lds0 = lds_addr(smem);
  unsigned fa_kc, fb_kc, fa_mc[4], fb_mc[4];
  {
    const int q = fr >> 2, p = fr & 3, sw = (q << 1) | ((fg & 1) << 3);
    fa_kc = lds0 + wr * 64 * 128 + swz_kc(fr, grp * 4 + fg);
    fb_kc = lds0 + OPB + wc * 64 * 128 + swz_kc(fr, grp * 4 + fg);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ca = (wr * 64 + 16 * i) / 8 + (p >> 1), cb = (wc * 64 + 16 * i) / 8 + (p >> 1);
      fa_mc[i] = lds0 + grp * 8192 + (8 * fg + q) * 256 + ((ca ^ sw) << 4) + 8 * (p & 1);
      fb_mc[i] = lds0 + OPB + grp * 8192 + (8 * fg + q) * 256 + ((cb ^ sw) << 4) + 8 * (p & 1);
    }
  }
  auto read_set = [&](int st, u32x4_t(&a)[4], u32x4_t(&b)[4]) {
    const unsigned so = (unsigned)(st * STAGE);
    if constexpr (AKC) {
      const unsigned ba = fa_kc + so;
      a[0] = frag_kc<0>(ba);
      a[1] = frag_kc<1>(ba);
      a[2] = frag_kc<2>(ba);
      a[3] = frag_kc<3>(ba);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag_mc(fa_mc[i] + so);
    }
    if constexpr (BKC) {
      const unsigned bb = fb_kc + so;
      b[0] = frag_kc<0>(bb);
      b[1] = frag_kc<1>(bb);
      b[2] = frag_kc<2>(bb);
      b[3] = frag_kc<3>(bb);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i] = frag_mc(fb_mc[i] + so);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // fused bias gradient (MC A): the wc == 0 waves of the first column of tiles sum their A fragments
  const bool do_cs = !AKC && g.colsum != nullptr && bx == 0 && wc == 0;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const u32x4_t(&a)[4], const u32x4_t(&b)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, b[j]),
                                                            __builtin_bit_cast(bf16x8_t, a[i]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (!AKC && do_cs) {
      // v_dot2_f32_bf16 against (1, 1) as inline asm (hipcc 7.2 lowered the builtin to the same source dword for
      // every element of a fragment)
      const unsigned one = 0x3f803f80u;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int w = 0; w < 4; ++w)
          asm volatile("v_dot2_f32_bf16 %0, %1, %2, %0" : "+v"(cs[i]) : "v"(a[i][w]), "v"(one));
    }
  };

  // ragged K (token-major operands only; KC operands have K % 64 == 0): the last K-tile's fragments are masked
  // to zero past kv, whatever the range-checked DMA left in the image rows beyond the operand's end
  const int kv = kend - kbeg - (nk - 1) * 64;
  auto mask_set = [&](u32x4_t(&a)[4], u32x4_t(&b)[4]) {
    const int k0 = grp * 32 + 8 * fg;
    u32x4_t mk;
#pragma unroll
    for (int w = 0; w < 4; ++w)
      mk[w] = (k0 + 2 * w < kv ? 0xffffu : 0u) | (k0 + 2 * w + 1 < kv ? 0xffff0000u : 0u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] &= mk;
      b[i] &= mk;
    }
  };

  // K loop. The two wave groups (k-halves) run one barrier apart, so that on every SIMD one wave issues its
  // 16 MFMAs while its partner reads the next fragments, issues its share of the LDS-DMA and waits:
  //   read phase of K-tile t: fragments (t) | DMA K-tile t+NST-1 into the stage of t-1 (read by both groups
  //   before the last barrier) | lgkmcnt(0) | vmcnt: own share of t+1 landed | barrier
  //   MFMA phase: 16 MFMAs | barrier
  // (Issuing the 4 DMA instructions between the MFMAs instead of in the read phase — gemm256's placement — measured
  // slower here: grouped weight gradients 115 -> 129 us; fine stamps: read phase 532 -> 448 cycles, MFMA phase
  // 376 -> 516. The read phase is bound by its 16 transposed reads and their latency, not by the DMA issue.)
  u32x4_t fa[4], fb[4];
  constexpr int AHEAD = NST - 1;
#pragma unroll
  for (int u = 0; u < AHEAD; ++u) issue(min(u, nk - 1), u);
  vmcnt<(AHEAD - 1) * DPW>();
  bar();
  STAMP(1);
  if (grp == 1) bar();
  for (int t = 0; t < nk; ++t) {
#if defined(G128_STAMPS) && !defined(G128_FINE)
    if (t < NSTAMP - 4) STAMP(2 + t);
#endif
    FSTAMP(t, 0);
    read_set(t % NST, fa, fb);
    issue(min(t + AHEAD, nk - 1), (t + AHEAD) % NST);
    lgkmcnt0();
    __builtin_amdgcn_sched_barrier(0);
    if (kv < 64 && t == nk - 1) mask_set(fa, fb);
    FSTAMP(t, 1);
    vmcnt<(AHEAD - 1) * DPW>();
    FSTAMP(t, 2);
    bar();
    FSTAMP(t, 3);
    mma(fa, fb);
    FSTAMP(t, 4);
    bar();
  }
  if (grp == 0) bar();
  vmcnt<0>();  // no LDS-DMA may land after this point
  bar();       // ... for every wave: the ring is free
  STAMP(NSTAMP - 2);

  // ------------------------------------------------------------------ k-half reduction, epilogue
  // Each group finalises half of its wave tile's rows (group g: row blocks 2g, 2g+1): it parks the partial
  // sums of the other half in LDS for its partner, and adds the partner's parked half of its own rows. The
  // epilogue's global loads (bias, dGELU pre-activation) are issued before the exchange barrier.
  const int mw = m0 + wr * 64, nw = n0 + wc * 64;
  if (!AKC && do_cs) {
    // lanes fr, fr+16, fr+32, fr+48 hold partial sums of row 16i + fr (each group its k-half)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = cs[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int m = mw + 16 * i + fr;
      if (fg == 0 && m >= by * BM) atomicAdd(g.colsum + m, v);
    }
  }
  f32x4_t* red = (f32x4_t*)smem + w4 * 1024;  // [i][j][lane], 16 KB per wave pair
  const float alpha = g.alpha;
  const long ldc = g.ldc;
  auto finish = [&](auto gc) {
    constexpr int G = decltype(gc)::value, I0 = 2 * G, P0 = 2 - 2 * G;  // own / partner's row blocks
    f32x4_t bv[4];
    uint2 pre[2][4];
    if constexpr (EPI != EPI_ACC_F32 && !ROPE) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bv[j] = g.bias ? *(const f32x4_t*)(g.bias + nw + 16 * j + 4 * fg) : f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (EPI == EPI_DGELU) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          pre[ii][j] = *(const uint2*)((const OT*)g.C2 + (long)(mw + 16 * (I0 + ii) + fr) * ldc + nw + 16 * j + 4 * fg);
    }
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[((P0 + ii) * 4 + j) * 64 + lane] = acc[P0 + ii][j];
    bar();
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[I0 + ii][j] += red[((I0 + ii) * 4 + j) * 64 + lane];
    if constexpr (ROPE) {
      // column block j < 2 holds columns jj = n0 + 32 wc + 16 j + 4 fg + e of the first half, block j + 2 their
      // partners jj + N/2: dx[m][2 jj] += a cs[p][2 jj] + b sn[p][2 jj], dx[m][2 jj + 1] += -a sn[p][2 jj + 1] +
      // b cs[p][2 jj + 1] (p = m % rL): 8 consecutive f32 outputs per lane and block pair
      const int mlo = by * BM;
      float* C = (float*)g.C;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int m = mw + 16 * (I0 + ii) + fr;
        const long p = m % (int)g.rL;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c2 = 2 * (n0 + 32 * wc + 16 * j + 4 * fg);
          const f32x4_t a = acc[I0 + ii][j] * alpha, b = acc[I0 + ii][j + 2] * alpha;
          const f32x4_t c0 = *(const f32x4_t*)(g.rcs + p * N + c2), c1 = *(const f32x4_t*)(g.rcs + p * N + c2 + 4);
          const f32x4_t s0 = *(const f32x4_t*)(g.rsn + p * N + c2), s1 = *(const f32x4_t*)(g.rsn + p * N + c2 + 4);
          f32x4_t* cp = (f32x4_t*)(C + (long)m * ldc + c2);
          if (m >= mlo) {
            f32x4_t u = cp[0], v = cp[1];
            u[0] += a[0] * c0[0] + b[0] * s0[0];
            u[1] += -a[0] * s0[1] + b[0] * c0[1];
            u[2] += a[1] * c0[2] + b[1] * s0[2];
            u[3] += -a[1] * s0[3] + b[1] * c0[3];
            v[0] += a[2] * c1[0] + b[2] * s1[0];
            v[1] += -a[2] * s1[1] + b[2] * c1[1];
            v[2] += a[3] * c1[2] + b[3] * s1[2];
            v[3] += -a[3] * s1[3] + b[3] * c1[3];
            cp[0] = u;
            cp[1] = v;
          }
        }
      }
    } else if constexpr (EPI == EPI_ACC_F32) {
      // park the finished 32x64 f32 rows in LDS (chunk c of row r at c ^ (r & 15)), then add one 256-B row per
      // instruction: split-K slices atomically, a single slice by read-modify-write
      float* tl = (float*)(smem + 65536) + wid * 2048;
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 16 * ii + fr, c = 4 * j + fg;
          *(f32x4_t*)(tl + r * 64 + ((c ^ (r & 15)) << 2)) = acc[I0 + ii][j];
        }
      const int n = nw + lane;
      const int mlo = by * BM;
      const bool nok = n >= bx * BN;
      float* C = (float*)g.C;
      if (nz > 1) {
        for (int r = 0; r < 32; ++r) {
          const int m = mw + 32 * G + r;
          const float v = tl[r * 64 + ((((lane >> 2) ^ (r & 15)) << 2) | (lane & 3))] * alpha;
          if (nok && m >= mlo) atomicAdd(C + (long)m * ldc + n, v);
        }
      } else {
        // read-modify-write, 8 rows' loads in flight before their adds (a load behind each store was one memory
        // round trip per row: epilogue p90 25.8k cycles in the grouped weight gradients)
        float* crow = C + (long)(mw + 32 * G) * ldc + n;
#pragma unroll 1
        for (int r0 = 0; r0 < 32; r0 += 8) {
          float old[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) old[r] = (nok && mw + 32 * G + r0 + r >= mlo) ? crow[(r0 + r) * ldc] : 0.f;
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int rr = r0 + r;
            const float v = tl[rr * 64 + ((((lane >> 2) ^ (rr & 15)) << 2) | (lane & 3))] * alpha;
            if (nok && mw + 32 * G + rr >= mlo) crow[rr * ldc] = old[r] + v;
          }
        }
      }
    } else {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = mw + 16 * (I0 + ii) + fr, n = nw + 16 * j + 4 * fg;
          f32x4_t v = acc[I0 + ii][j] * alpha + bv[j];
          OT* cp = (OT*)g.C + (long)m * ldc + n;
          if constexpr (sizeof(OT) == 4) {
            *(f32x4_t*)cp = v;
          } else {
            if constexpr (EPI == EPI_GELU) {
              *(uint2*)cp = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));  // pre-activation
              const unsigned keep =
                  g.thr16 ? drop_keep4(eff_seed(g.seed, g.seed_off), g.stream, ((uint64_t)m * (uint64_t)N + n) >> 2, g.thr16) : 0xfu;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float a = gelu_f(v[e]);
                v[e] = (keep >> e) & 1u ? (g.thr16 ? a * g.drop_scale : a) : 0.f;
              }
              cp = (OT*)g.C2 + (long)m * ldc + n;
            } else if constexpr (EPI == EPI_GELU_ONLY) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = gelu_f(v[e]);
            } else if constexpr (EPI == EPI_DGELU) {
              const uint2 pu = pre[ii][j];
              const float pv[4] = {__uint_as_float(pu.x << 16), __uint_as_float(pu.x & 0xffff0000u),
                                   __uint_as_float(pu.y << 16), __uint_as_float(pu.y & 0xffff0000u)};
              const unsigned keep =
                  g.thr16 ? drop_keep4(eff_seed(g.seed, g.seed_off), g.stream, ((uint64_t)m * (uint64_t)N + n) >> 2, g.thr16) : 0xfu;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float a = v[e] * gelu_grad(pv[e]);
                v[e] = (keep >> e) & 1u ? (g.thr16 ? a * g.drop_scale : a) : 0.f;
              }
            }
            *(uint2*)cp = make_uint2(pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]));
          }
        }
    }
  };
  if (grp == 0) finish(IC<0>{});
  else finish(IC<1>{});
  STAMP(NSTAMP - 1);
}

// XCD-aware unit order: workgroup w runs on XCD w % 8, so within every round of 256 workgroups (one per CU,
// dispatched in order) each XCD is given a contiguous range of that round's units (tile column fastest): tiles
// that share an A row panel, and the B column panels, meet in one L2, and the rounds keep the unit order
// (the grouped launch lists its longest units first)
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int base = b & ~255, size = min(256, nb - base);
  const int x = b & 7, j = (b - base) >> 3, q = size >> 3, r = size & 7;
  return base + (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
}

template <bool AKC, bool BKC, int EPI, typename OT>
__global__ void __launch_bounds__(512) gemm128_kernel(GemmArgs g, int nz) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tn = (int)((g.N + BN - 1) / BN), tm = (int)((g.M + BM - 1) / BM);
  const int u = xcd_remap(blockIdx.x, gridDim.x), per = tn * tm;
  const int bz = u / per, rem = u - bz * per;
  tile128<AKC, BKC, EPI, OT>(g, smem, rem % tn, rem / tn, bz, nz);
}

// grouped launch (weight gradients of a decoder block): unit u (XCD-remapped workgroup id) is unit u - start[p] of
// problem p, units ordered (split, tile row, tile column)
template <bool AKC, bool BKC, int EPI, typename OT>
__global__ void __launch_bounds__(512) gemm128_grouped_kernel(G128Group ga) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  int p = 0;
  while (p + 1 < ga.np && b >= ga.start[p + 1]) ++p;
  const int local = b - ga.start[p], per = ga.tn[p] * ga.tm[p];
  const int bz = local / per, rem = local - bz * per;
  tile128<AKC, BKC, EPI, OT>(ga.g[p], smem, rem % ga.tn[p], rem / ga.tn[p], bz, ga.nz[p]);
}

template <bool AKC, bool BKC, int EPI, typename OT>
static int launch(const GemmArgs& g, int nz, hipStream_t s) {
  const long nb = ((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM) * nz;
  hipLaunchKernelGGL((gemm128_kernel<AKC, BKC, EPI, OT>), dim3((unsigned)nb), dim3(512), LDS_BYTES, s, g, nz);
  return (int)hipGetLastError();
}

}  // namespace g128

long gemm128_tiles(long M, long N) { return ((M + 127) / 128) * ((N + 127) / 128); }

bool gemm128_ok(const GemmArgs& g, bool akc, bool bkc, int epi, int out_dtype) {
  if (g.M < 128 || g.N < 128 || g.K <= 0 || g.N % 8 || g.lda % 8 || g.ldb % 8 || g.ldc % 8) return false;
  if ((akc || bkc) && g.K % 64) return false;
  if (!akc && g.M % 8) return false;
  if ((((uintptr_t)g.A) | ((uintptr_t)g.B) | ((uintptr_t)g.C) | ((uintptr_t)g.C2) | ((uintptr_t)g.bias)) & 15)
    return false;
  if (g.Mi < g.M || g.geo.cstride != 0) return false;  // no implicit conv
  // 31-bit byte offsets
  const long aext = akc ? (g.M - 1) * g.lda + g.K : (g.K - 1 + 64) * g.lda + g.M;
  const long bext = bkc ? (g.N - 1) * g.ldb + g.K : (g.K - 1 + 64) * g.ldb + g.N;
  if (aext * 2 >= (1L << 31) || bext * 2 >= (1L << 31)) return false;
  if (((g.M - 1) * g.ldc + g.N) * 4 >= (1L << 31)) return false;
  if (!akc && bkc) return false;
  if (epi == EPI_ROPE_ACC)  // whole 128-column tiles of partner pairs, tables and output 16-B aligned
    return akc && !bkc && out_dtype == FDDM_F32 && g.N % 128 == 0 && g.ldc % 4 == 0 && g.rL > 0 && g.rcs && g.rsn &&
           !(((uintptr_t)g.rcs | (uintptr_t)g.rsn) & 15);
  if (out_dtype == FDDM_F32) return epi == EPI_STORE || epi == EPI_ACC_F32;
  if (!akc) return false;
  if (!bkc) return epi == EPI_STORE || epi == EPI_DGELU;
  return epi == EPI_STORE || epi == EPI_GELU || epi == EPI_GELU_ONLY || epi == EPI_DGELU;
}

int gemm128_launch(const GemmArgs& g, bool akc, bool bkc, int epi, int out_dtype, int nz, hipStream_t s) {
  using namespace g128;
  if (!gemm128_ok(g, akc, bkc, epi, out_dtype)) return (int)hipErrorInvalidValue;
  if (nz > 1 && epi != EPI_ACC_F32) return (int)hipErrorInvalidValue;
  if (akc && bkc) {
    if (out_dtype == FDDM_F32) return epi == EPI_ACC_F32 ? launch<true, true, EPI_ACC_F32, float>(g, nz, s)
                                                         : launch<true, true, EPI_STORE, float>(g, nz, s);
    if (epi == EPI_GELU) return launch<true, true, EPI_GELU, bf16_t>(g, nz, s);
    if (epi == EPI_GELU_ONLY) return launch<true, true, EPI_GELU_ONLY, bf16_t>(g, nz, s);
    if (epi == EPI_DGELU) return launch<true, true, EPI_DGELU, bf16_t>(g, nz, s);
    return launch<true, true, EPI_STORE, bf16_t>(g, nz, s);
  }
  if (akc && !bkc) {
    if (epi == EPI_ROPE_ACC) return nz == 1 ? launch<true, false, EPI_ROPE_ACC, float>(g, nz, s) : (int)hipErrorInvalidValue;
    if (out_dtype == FDDM_F32) return epi == EPI_ACC_F32 ? launch<true, false, EPI_ACC_F32, float>(g, nz, s)
                                                         : launch<true, false, EPI_STORE, float>(g, nz, s);
    if (epi == EPI_DGELU) return launch<true, false, EPI_DGELU, bf16_t>(g, nz, s);
    if (epi == EPI_STORE) return launch<true, false, EPI_STORE, bf16_t>(g, nz, s);
    return (int)hipErrorInvalidValue;
  }
  if (!akc && !bkc && out_dtype == FDDM_F32)
    return epi == EPI_ACC_F32 ? launch<false, false, EPI_ACC_F32, float>(g, nz, s)
                              : launch<false, false, EPI_STORE, float>(g, nz, s);
  return (int)hipErrorInvalidValue;
}

#ifdef G128_STAMPS
FDDM_API int fddm_gemm128_stamps(unsigned long long* host, long n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fddm::g128::g128_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif

int gemm128_grouped_dw(const G128Group& ga, int total, hipStream_t s) {
  hipLaunchKernelGGL((g128::gemm128_grouped_kernel<false, false, EPI_ACC_F32, float>), dim3((unsigned)total),
                     dim3(512), g128::LDS_BYTES, s, ga);
  return (int)hipGetLastError();
}

}  // namespace fddm
