// Decoder attention forward with two query chains per wave (gfx950): fwd8.
//
// The decoder's self- and cross-attention (models/denoise_decoder.py:129-130,164,169-176 -> nn.MultiheadAttention:
// key-padding mask, dropout p on the attention probabilities, head_dim 64), bf16 in / out, fp32 softmax statistics.
// Score operands as fwd7 (attn7.hip): pre-scaled Q' = bf16(Q scale log2 e), the softmax reference and the key mask
// folded into the score MFMA as a fifth k-step, bf16 P into the PV MFMA. Unlike fwd7, each chain's reference is fixed
// after its first half-tile (no rescale branch in the loop; a guard on the final row sums sends a wave to an exact
// online-softmax fallback), the keep bits are layout v5 (a score pair's mask by one shift + v_perm), and the row sums
// come from row-selector MFMAs on the undropped packed probabilities.
//
// Why a new structure (profiles/r05e_pmc_attn7_c2.md): fwd7 runs one 32-query chain per wave, so
// each half-tile is a serial chain — score MFMAs, then ~70 VALU + 16 v_exp on their results, then the PV MFMAs — and
// its waves sat parked 34-44 % of their cycles with the matrix pipe busy 8-14 %. Here each wave owns TWO independent
// 32-query chains A and B and software-pipelines them against each other: while the VALU works on one chain's
// exponentials, the matrix pipe runs the other chain's PV MFMAs and next score MFMAs. One phase = 9 (+2 row-sum) MFMAs:
//   alpha_j: MFMA { S_B(j) [5], PV_B(j-1) [4] }   VALU { softmax_A(j) }   LDS { K fragments of half j + 1 }
//   beta_j : MFMA { S_A(j+1) [5], PV_A(j) [4] }   VALU { softmax_B(j) }   LDS { V fragments of half j + 1 }
// (j = 32-key half-tile). Each phase is written as 9 chunks {one MFMA, three stages of score-pair softmax VALU, an
// LDS read or DMA piece} fenced by sched_barrier, so the placement is ours, not the scheduler's. Both chains share
// every K / V fragment (half the LDS reads per MFMA of fwd7). DESIGN.md §4.7 has the measurements.
//
// Layout: one workgroup = 4 waves x 64 queries = 256 queries of one (b, h) (C2's Lq 256: one workgroup per (b, h),
// K / V read once). K / V tiles (64 keys) and the chains' keep dwords stream through a 4-stage LDS-DMA ring, two tiles
// ahead; one counted vmcnt + barrier per tile, placed mid-tile (after the last read of the previous tile's stage,
// before the first read of the next tile). Each wave also owns 16 KB past the ring: its Q rows' staging in the
// prologue, the fallback's tile staging in the epilogue.
#include "attn7_common.h"

namespace fddm {
namespace attn {

constexpr int A8_NS = 4;  // ring stages (tiles in flight: 2 ahead of the one being read)
// Row sums: A8_RSMFMA 1 = by 32x32x16 MFMAs of a row-selector operand against the undropped packed probabilities (two
// per phase) into ONE accumulator shared by the chains (rows 0-15: chain A's sums, rows 16-31: chain B's), 0 = f32
// adds (16 per phase)
#ifndef A8_RSMFMA
#define A8_RSMFMA 1
#endif
#ifndef A8_WPS
#define A8_WPS 2  // waves per SIMD the register allocation targets (<= 256 registers: no accumulator-file split)
#endif

// pin a value to this point of the instruction stream: its computation cannot sink past the chunk's sched_barrier
__device__ __forceinline__ void pinv(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pinv(unsigned& x) { asm volatile("" : "+v"(x)); }
// a score pair's keep mask and bf16 pack in one statement (the fallback's f32 path): x & sext(bit B0 of kw),
// y & sext(bit B1 of kw), then v_cvt_pk_bf16_f32 (low half = x); one asm statement, so hipcc pads no state between
template <int B0, int B1>
__device__ __forceinline__ unsigned keep_pack(float x, float y, unsigned kw) {
  unsigned r, t;
  asm volatile(
      "v_bfe_i32 %1, %3, %5, 1\n\t"
      "v_and_b32 %1, %1, %2\n\t"
      "v_bfe_i32 %0, %3, %6, 1\n\t"
      "v_and_b32 %0, %0, %4\n\t"
      "v_cvt_pk_bf16_f32 %0, %1, %0"
      : "=&v"(r), "=&v"(t)
      : "v"(x), "v"(kw), "v"(y), "i"(B0), "i"(B1));
  return r;
}
#define A8_FENCE() __builtin_amdgcn_sched_barrier(0)

// Diagnostic build only (-DA8_STAMPS, tools/probe/a8_stamps.py; outputs are overwritten): s_memtime of wave 0 at the
// kernel's phase points, written over the first output row of the workgroup's query block (16 x 8 B = 128 B)
#ifdef A8_STAMPS
#define A8ST(k)                                 \
  do {                                          \
    a8st_[k] = __builtin_amdgcn_s_memtime(); /* uniform: SGPRs */ \
  } while (0)
#else
#define A8ST(k) \
  do {          \
  } while (0)
#endif
// diagnostic: -DA8_FINE=n (with A8_STAMPS) stamps the start and every chunk end of the workgroup's n-th phase call into
// the second output row (tools/probe/a8_stamps.py --fine)
#if defined(A8_STAMPS) && defined(A8_FINE)
#define A8FS(k)                                                  \
  do {                                                           \
    if (a8pc_ == A8_FINE) a8fs_[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define A8FS(k) \
  do {          \
  } while (0)
#endif

// LDS: K ring, V ring, keep dwords, 16 B, the key operands [LkP]; then (16-B aligned) 16 KB per wave for the
// fallback's private tile staging
__host__ __device__ __forceinline__ int attn8_fwd_fb_off(int Lk) {
  const int LkP = (Lk + 63) / 64 * 64;
  return (2 * A8_NS * A7_TB + A8_NS * 512 * 4 + 16 + LkP * 4 + 15) / 16 * 16;
}

template <int DM, int MK>
__global__ void __launch_bounds__(256, A8_WPS) fwd8_kernel(AttnArgs a) {
  constexpr bool DROP = DM != 0;
  constexpr int NP = DROP ? 6 : 4;  // LDS-DMA instructions per wave and tile (K 2, V 2, keep dwords 2)
  extern __shared__ __attribute__((aligned(16))) unsigned char sm8[];
  const int ntiles = (a.Lk + 63) >> 6, LkP = ntiles * 64;
  unsigned char* kst = sm8;                                     // [NS][64 rows][128 B] K, KC swizzle
  unsigned char* vst = sm8 + A8_NS * A7_TB;                     // [NS][64 rows][128 B] V, vsw swizzle
  unsigned* kbl = (unsigned*)(sm8 + 2 * A8_NS * A7_TB);         // [NS][4 waves][2 chains][64 lanes] keep dwords
  unsigned* mpk = kbl + A8_NS * 512 + 4;                        // [LkP] bf16 pair (1, mask): the key's fifth k-step
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, qi = lane & 31;
  int bxi, bh;
  xcd_tile(bxi, bh);
#ifdef A8_STAMPS
  unsigned long long a8st_[16] = {};
#endif
#if defined(A8_STAMPS) && defined(A8_FINE)
  unsigned long long a8fs_[16] = {};
  int a8pc_ = 0;
#endif
  A8ST(0);
  const int b = bh / a.H, h = bh - b * a.H;
  const int qw0 = bxi * 256 + 64 * w;  // chain c: queries qw0 + 32 c + (lane & 31)
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  const unsigned sk2 = (unsigned)a.sk * 2u, sv2 = (unsigned)a.sv * 2u;
  const int nqg = (a.Lq + 31) >> 5, qg0 = 8 * bxi + 2 * w;  // the chains' 32-query groups qg0, qg0 + 1
  const unsigned* lbits = (const unsigned*)(a.dbits + (long)a.B * a.H * nqg * ntiles * 32);

  // ---- prologue. The loads are issued in the order they are needed and the prologue fetches no more than the
  // pipeline's start needs (key mask, Q, tiles 0 and 1), all untracked by hipcc and waited for by ONE counted vmcnt:
  // with every workgroup issuing at once, an instruction that finds the memory queue full blocks its wave, so a deeper
  // up-front prefetch only delays the first MFMA (stamps: issuing Q + three tiles took 3.9k-8.6k cycles). Later tiles
  // are fetched one per mid-tile span, their pieces spread over the phases' chunks. Every key tile is computed (no
  // skipping of fully masked tiles: with one workgroup per (b, h) and CU, the kernel lasts as long as its longest
  // workgroup anyway, and the key mask need not be known before the first fills).
  // key-padding bytes (MK 2): thread tid's keys 4 tid .. 4 tid + 3, one global_load_ubyte each
  unsigned kb8[4] = {1u, 1u, 1u, 1u};
  if constexpr (MK == 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = min(4 * tid + j, a.Lk - 1);
      asm volatile("global_load_ubyte %0, %1, off" : "=v"(kb8[j]) : "v"(a.key_keep + (long)b * a.Lk + k) : "memory");
    }
  }
  // Q rows of the wave's two chains by LDS-DMA into the wave's private 16 KB past the ring (the fallback's staging,
  // unused until the epilogue): whole 128-B rows per lane group, and no barrier before the reads, since each wave reads
  // only the rows it brought (its own counted vmcnt covers them). Row r of the wave's 64, chunk c at c ^ (r & 7).
  // (Direct global loads of the fragments into registers measured slower: each wave-instruction touches 32 rows in
  // 32-B pieces, and the prologue's fills queued behind them, +2k cycles.)
  const int qA = qw0 + qi, qB = qw0 + 32 + qi;
  unsigned char* qst = sm8 + attn8_fwd_fb_off(a.Lk) + w * 16384;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int r = 8 * u + (lane >> 3), pch = lane & 7;   // row within the wave's 64 queries
    const unsigned qr = (unsigned)min(qw0 + r, a.Lq - 1);
    dma16_sv(Qb, qr * (unsigned)a.sq * 2u + (unsigned)((pch ^ (r & 7)) << 4), qst + 8 * u * 128);
  }
  const unsigned tmask = ntiles >= 32 ? 0xFFFFFFFFu : ((1u << ntiles) - 1u);
  const int nact = ntiles;
  A8ST(15);

  // tile fills by pieces (K rows 16 w .. + 7 and + 8 .. + 15, V the same, the chains' keep dwords): piece k of tile
  // tt into stage st. Wave w brings rows 16 w .. 16 w + 15; XOR swizzles applied to the per-lane source addresses.
  // Addressing: the swizzles depend on the row mod 16 only (tile-invariant); LDS destinations as integer byte
  // addresses (no pointer conversion per piece); source offsets by 24-bit multiplies (rows < 2^24, strides < 2^23).
  const unsigned kst_a = lds_addr(kst), vst_a = lds_addr(vst), kbl_a = lds_addr(kbl);
  auto piece = [&](int tt, int st, int k) {
    if (k < 4) {
      const int u = k >> 1, R = 16 * w + 8 * u;
      const int r0 = R + (lane >> 3), pch = lane & 7;
      const unsigned rr = (unsigned)min(64 * tt + r0, a.Lk - 1);
      if ((k & 1) == 0)
        dma16_so(Kb, __umul24(rr, sk2) + (unsigned)((pch ^ ((r0 >> 1) & 7)) << 4), kst_a + st * A7_TB + R * 128);
      else
        dma16_so(Vb, __umul24(rr, sv2) + (unsigned)((pch ^ vsw(r0)) << 4), vst_a + st * A7_TB + R * 128);
    } else {
      const int c = k - 4;
      dma4_so(lbits, (unsigned)(lb_dword(bh, nqg, ntiles, min(qg0 + c, nqg - 1), tt) + lane) * 4u,
              kbl_a + (st * 512 + (2 * w + c) * 64) * 4);
    }
  };
  // fill cursor over the active tiles; active tile i goes to stage i % NS. Every span issues exactly NP pieces (past
  // the last active tile: the last one again, into the stage nobody reads), so each wait below is vmcnt(NP).
  unsigned fmask = tmask;
  int flast = 0;
  auto next_fill_tile = [&]() {
    if (fmask) {
      flast = __builtin_ctz(fmask);
      fmask &= fmask - 1u;
    }
    return flast;
  };
  {
    const int t0 = next_fill_tile(), t1 = next_fill_tile();
#pragma unroll
    for (int k = 0; k < NP; ++k) piece(t0, 0, k);
#pragma unroll
    for (int k = 0; k < NP; ++k) piece(t1, 1, k);
  }
  A8ST(11);
  // key bytes, Q and tile 0 landed; tile 1 in flight (the loaded registers named, so no use moves above the wait)
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(kb8[0]), "+v"(kb8[1]), "+v"(kb8[2]), "+v"(kb8[3]) : "n"(NP) : "memory");
  // the keys' fifth-k-step operands (1, 0 or -inf)
  if constexpr (MK != 0) {
    if (4 * tid < LkP) {
      unsigned mv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = 4 * tid + j < a.Lk && (MK == 1 || (kb8[j] & 0xFFu) != 0);
        mv[j] = pk_bf16(1.f, ok ? 0.f : -INFINITY);
      }
      *(uint4*)(mpk + 4 * tid) = make_uint4(mv[0], mv[1], mv[2], mv[3]);
    }
  }
  __builtin_amdgcn_s_barrier();                                 // every wave's pieces; the key operands in LDS
  A8ST(1);
  // the chains' Q fragments (lane: row qi of chain c, chunk 2 ks + hh) from the wave's own staging, pre-scaled by sl2
  // (scores in log2 units); rows past Lq are zeroed (never stored)
  const float sl2 = a.scale * 1.4426950408889634f;
  uint4 qa[4], qb[4];
  {
    const unsigned zA = qA < a.Lq ? 0xFFFFFFFFu : 0u, zB = qB < a.Lq ? 0xFFFFFFFFu : 0u;
    const int rA = qi, rB = qi + 32;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const uint4 x = *(const uint4*)(qst + rA * 128 + (((2 * ks + hh) ^ (rA & 7)) << 4));
      const uint4 y = *(const uint4*)(qst + rB * 128 + (((2 * ks + hh) ^ (rB & 7)) << 4));
      qa[ks] = scale_frag(make_uint4(x.x & zA, x.y & zA, x.z & zA, x.w & zA), sl2);
      qb[ks] = scale_frag(make_uint4(y.x & zB, y.y & zB, y.z & zB, y.w & zB), sl2);
    }
  }

  // per-lane LDS offsets: K row reads (row qi of a 32-key half, chunk 2 ks + hh), V transposed reads
  int koff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) koff[ks] = qi * 128 + (((2 * ks + hh) ^ ((qi >> 1) & 7)) << 4);
  const int vi = lane & 15, vrow = 4 * hh + (vi >> 2);
  int voff[2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
    voff[db] = vrow * 128 + (((8 * db + 4 * ((lane >> 4) & 1) + (vi & 3)) ^ ((vrow & 2) << 2)) << 3);

  // chain state, softmax in log2 units: rf = the chain's bf16 reference, fixed after its first half-tile (the lane
  // pair's row maximum there, 0 while that is -inf), subtracted inside the score MFMA; O^T accumulators; q5 = the
  // fifth-k-step operand (-rf, 1); p = packed probabilities; ls = the lane's row sum of its keys (f32 adds).
  // With a fixed reference the fast loop has no rescale branch (no phi copies of O). A row sum that ends above 2^64
  // (or inf / NaN) could have overflowed on the way, and one below 2^-40 (a first half-tile fully masked, then scores
  // far below 0) lost its precision: such waves recompute their chains in the wave-local fallback (online softmax with
  // rescaling, fwd7's algorithm), exact but slow — not reached by softmax inputs of sane range.
  float rfA = 0.f, rfB = 0.f;
  f32x16_t oA0 = {}, oA1 = {}, oB0 = {}, oB1 = {};
  constexpr bool RSM = A8_RSMFMA != 0;
  float lsA = 0.f, lsB = 0.f;  // add row sums (relative to rf): the lane's keys
  f32x16_t lsum = {};           // MFMA row sums: row r of the accumulator = chain (r >> 4)'s sum for the lane's query
  uint4 ucar = make_uint4(0, 0, 0, 0);  // MFMA row sums: the previous phase's second packed half, summed a phase late
  // selector A operands (lane: row l & 31, k 8 hh .. + 7): ones in rows 0-15 (chain A) or 16-31 (chain B)
  const unsigned one2 = 0x3F803F80u, selA1 = qi < 16 ? one2 : 0u, selB1 = qi < 16 ? 0u : one2;
  const uint4 selA = make_uint4(selA1, selA1, selA1, selA1), selB = make_uint4(selB1, selB1, selB1, selB1);
  f32x16_t sA, sB;
  uint4 pA[2], pB[2];
  pB[0] = pB[1] = make_uint4(0, 0, 0, 0);
  const uint4 q5init = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(0.f, 1.f), 0u, 0u, 0u);
  uint4 q5A = q5init, q5B = q5init;
  unsigned kwA = 0xFFFFFFFFu, kwB = 0xFFFFFFFFu;
  // fragments, one buffer each (reads are placed after the last MFMA that used the previous contents): K of a half
  // (4 x ds_read_b128), its fifth-k-step operand k5, V of a half (2 steps x 2 d-blocks, each two tr reads)
  uint4 kf[4], vf[2][2];
  uint4 k5 = make_uint4(0, 0, 0, 0);
  const unsigned lo32 = hh ? 0u : 0xFFFFFFFFu;  // lanes 0-31 hold the first 8 k positions of the fifth k-step
  auto mk5 = [&](int key0) {
    unsigned mk = pk_bf16(1.f, 0.f);
    if constexpr (MK != 0) mk = mpk[key0 + qi];  // every lane reads (no exec-masked branch), lanes 32-63 drop it
    return make_uint4(mk & lo32, 0u, 0u, 0u);
  };
  // in the phases the key operand's LDS read (chunk 1) and its use (chunk 8) are apart, so its wait finds it landed
  unsigned mkr = 0;
  auto mk5_read = [&](int key0) {
    if constexpr (MK != 0) mkr = mpk[key0 + qi];
  };
  auto mk5_set = [&]() {
    unsigned mk = pk_bf16(1.f, 0.f);
    if constexpr (MK != 0) mk = mkr;
    k5 = make_uint4(mk & lo32, 0u, 0u, 0u);
  };
  // V fragment c (= 2 s + db) of the half at vimg
  auto rdv = [&](const unsigned char* vimg, int c) {
    const int o = voff[c & 1] + 16 * (c >> 1) * 128;
    vf[c >> 1][c & 1] = join_tr(tr_read(vimg + o), tr_read(vimg + o + 1024));
  };
  auto pset = [&](uint4 (&p)[2], auto ic, unsigned v) {
    constexpr int i = decltype(ic)::value;
    if constexpr ((i & 3) == 0) p[i >> 2].x = v;
    if constexpr ((i & 3) == 1) p[i >> 2].y = v;
    if constexpr ((i & 3) == 2) p[i >> 2].z = v;
    if constexpr ((i & 3) == 3) p[i >> 2].w = v;
  };
  auto pand = [&](uint4 (&p)[2], auto ic, unsigned m) {
    constexpr int i = decltype(ic)::value;
    if constexpr ((i & 3) == 0) p[i >> 2].x &= m;
    if constexpr ((i & 3) == 1) p[i >> 2].y &= m;
    if constexpr ((i & 3) == 2) p[i >> 2].z &= m;
    if constexpr ((i & 3) == 3) p[i >> 2].w &= m;
  };

  // the fallback's softmax pair (f32 row sums, keep bits tested one by one): registers 2 i, 2 i + 1 of half kb
  auto sm_pair_f32 = [&](const f32x16_t& s, float d, unsigned kw, uint4 (&p)[2], float& la, float& lb, auto kbc,
                         auto ic) {
    constexpr int kb = decltype(kbc)::value, i = decltype(ic)::value;
    const float x = __builtin_amdgcn_exp2f(s[2 * i] - d);
    const float y = __builtin_amdgcn_exp2f(s[2 * i + 1] - d);
    la += x;
    lb += y;
    unsigned v;
    if constexpr (DROP) v = keep_pack<lb_bit(kb, 2 * i), lb_bit(kb, 2 * i + 1)>(x, y, kw);
    else v = pk_bf16(x, y);
    pset(p, ic, v);
  };
  // the reference of a chain's first half-tile (scores computed against 0): bf16 of the lane pair's row maximum
  auto first_ref = [&](const f32x16_t& s, float& rf, uint4& q5) {
    float tm = fmaxf(s[0], s[1]);
#pragma unroll
    for (int r = 2; r < 16; r += 2) tm = fmaxf(tm, fmaxf(s[r], s[r + 1]));
    tm = xmax32(tm);
    rf = (tm == -INFINITY) ? 0.f : __uint_as_float(((unsigned)pk_bf16(tm, 0.f)) << 16);
    q5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(-rf, 1.f), 0u, 0u, 0u);
  };

  // One phase: 9 chunks {an MFMA, one score pair of the other chain's softmax, LDS reads}, fenced. MFMA order: the
  // score chain first (its result feeds the next phase's VALU), then the PV chain (its operand came from the previous
  // phase). A score pair's work is pipelined over two chunks so a chunk's VALU instructions do not wait on each other:
  // chunk i issues pair i's two v_exp, chunk i + 1 its two row-sum adds, the v_cvt_pk and (dropout) the pair mask
  // (shift + v_perm) and one v_and. Measured against an MFMA row sum (a 16x16x32 ones-selector product of the packed
  // probabilities): that cost 3.4 us at C2 cross in stalls around the 16x16 MFMAs (profiles/r06_attn8_ablations.md).
  //   SX: score accumulator (written) from qX / q5X and the current kf / k5
  //   oY0 / oY1 += V^T pY with the current vf; sZ - dZ -> pZ, lsZ: the softmax chain (half KB of the tile: keep bits of
  //   kwZ at lb_bit(KB, .)); rd(c): the LDS reads of chunk c; dm(c): its LDS-DMA pieces of the span's tile fill
  auto phase = [&](f32x16_t& SX, const uint4 (&qX)[4], const uint4& q5X, f32x16_t& oY0, f32x16_t& oY1,
                   const uint4 (&pY)[2], const f32x16_t& sZ, float dZ, uint4 (&pZ)[2], float& lZ,
                   const uint4& selZ, const uint4& selP, unsigned kwZ, auto kbc, auto&& rd, auto&& dm) {
    constexpr int KB = decltype(kbc)::value;
    float ex[8], ey[8], la, lb;
    unsigned sh[8], u[8], mk[8];
    // stage 1 of score pair i (chunk i): the two exponentials and the keep word shifted to the pair's bits (layout
    // v5, attn7_common.h lb_bit: bits 15 - P and 31 - P, P = 8 KB + i, moved to bits 15 and 31)
    auto expo = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
#ifndef A8_NOEXP  // timing-only ablation: no exponentials (wrong results)
      ex[i] = __builtin_amdgcn_exp2f(sZ[2 * i] - dZ);
      ey[i] = __builtin_amdgcn_exp2f(sZ[2 * i + 1] - dZ);
#else
      ex[i] = sZ[2 * i] - dZ;
      ey[i] = sZ[2 * i + 1] - dZ;
#endif
      pinv(ex[i]);
      pinv(ey[i]);
      if constexpr (DROP) {
        sh[i] = kwZ << (8 * KB + i);
        pinv(sh[i]);
      }
    };
    // stage 2 (chunk i + 1): the row sums, the bf16 pack, the pair's 32-bit keep mask (v_perm: the signs of bits 15 and
    // 31 replicated into the low and high halves)
    auto fin = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (!RSM) {
        if constexpr (i == 0) {
          la = ex[0];
          lb = ey[0];
        } else {
          la += ex[i];
          lb += ey[i];
        }
        pinv(la);
        pinv(lb);
      }
      u[i] = pk_bf16(ex[i], ey[i]);
      pinv(u[i]);
      if constexpr (DROP) {
#ifndef A8_NODROPMASK
        mk[i] = __builtin_amdgcn_perm(sh[i], sh[i], 0x09090808u);
#else
        mk[i] = 0xFFFFFFFFu;
#endif
        pinv(mk[i]);
      } else {
        pset(pZ, ic, u[i]);
      }
    };
    // stage 3 (chunk i + 2): the mask applied -> the PV operand
    auto apply = [&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (DROP) {
        unsigned v = u[i] & mk[i];
        pinv(v);
        pset(pZ, ic, v);
      }
    };
    // chunk c: stage 1 of pair c, stage 2 of pair c - 1, stage 3 of pair c - 2 (pair 7's stage 3 in chunk 8 as well):
    // the chunk's VALU instructions are independent of each other
    auto stages = [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if constexpr (c < 8) expo(std::integral_constant<int, c>{});
      if constexpr (c >= 1) fin(std::integral_constant<int, c - 1>{});
      if constexpr (c >= 2) apply(std::integral_constant<int, c - 2>{});
      if constexpr (c == 8) {
        apply(std::integral_constant<int, 7>{});
        if constexpr (!RSM) lZ += la + lb;
      }
    };
    // MFMA row sums (every row of the accumulator = the query's sum over the 16 keys of the k-step): the previous
    // phase's second half (its packs written in that phase's last chunk) in chunk 1, this phase's first half (packs of
    // chunks 1-4) in chunk 6, the second half carried to the next phase
    auto rsum = [&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if constexpr (RSM && c == 1) lsum = mfma32(selP, ucar, lsum);
      if constexpr (RSM && c == 6) lsum = mfma32(selZ, make_uint4(u[0], u[1], u[2], u[3]), lsum);
    };
#if defined(A8_STAMPS) && defined(A8_FINE)
    ++a8pc_;
#endif
    A8FS(0);
    f32x16_t acc = mfma32(k5, q5X, f32x16_t{});
    stages(std::integral_constant<int, 0>{});
    rd(std::integral_constant<int, 0>{});
    dm(std::integral_constant<int, 0>{});
    A8_FENCE();
    A8FS(1);
    static_for<0, 4>([&](auto kc) {
      constexpr int ks = decltype(kc)::value;
      acc = mfma32(kf[ks], qX[ks], acc);
      rsum(std::integral_constant<int, ks + 1>{});
      stages(std::integral_constant<int, ks + 1>{});
      rd(std::integral_constant<int, ks + 1>{});
      dm(std::integral_constant<int, ks + 1>{});
      A8_FENCE();
      A8FS(ks + 2);
    });
    SX = acc;
    static_for<0, 4>([&](auto pc) {
      constexpr int pi = decltype(pc)::value;  // PV step s = pi >> 1, d-block pi & 1
      if constexpr ((pi & 1) == 0) oY0 = mfma32(vf[pi >> 1][0], pY[pi >> 1], oY0);
      else oY1 = mfma32(vf[pi >> 1][1], pY[pi >> 1], oY1);
      rsum(std::integral_constant<int, 5 + pi>{});
      stages(std::integral_constant<int, 5 + pi>{});
      rd(std::integral_constant<int, 5 + pi>{});
      dm(std::integral_constant<int, 5 + pi>{});
      A8_FENCE();
      A8FS(pi + 6);
    });
    if constexpr (RSM) ucar = make_uint4(u[4], u[5], u[6], u[7]);
  };

  // the stream of active tiles: active tile i = tile t in stage i % NS; half 0 = keys 64 t .. + 31, half 1 = + 32 ..
  unsigned cmask = tmask;
  int t = __builtin_ctz(cmask);
  cmask &= cmask - 1u;
  int st = 0;
  if (nact > 0) {  // (every key masked: NaN rows, torch's softmax over -inf)
  {
    // pipeline start: K (+ k5) of half 0 and S_A(half 0) against reference 0; V of half 0 for PV_B(-1), which runs
    // with pB = 0 (finite data, zero contribution); keep bits of tile 0
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) kf[ks] = *(const uint4*)(kst + koff[ks]);
    k5 = mk5(64 * t);
    if constexpr (DROP) {
      kwA = kbl[(2 * w) * 64 + lane];
      kwB = kbl[(2 * w + 1) * 64 + lane];
    }
    f32x16_t acc = mfma32(k5, q5A, f32x16_t{});
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) acc = mfma32(kf[ks], qa[ks], acc);
    sA = acc;
#pragma unroll
    for (int c = 0; c < 4; ++c) rdv(vst, c);
  }
  // ---- tile 0, half 0: each chain's reference comes from this half's scores (computed against 0). This span fills
  // active tile 2 (stage 2): pieces in chunks 1, 4, 7 of both phases
  int fidx = 2, ftile = next_fill_tile();
  auto dm_first = [&](auto base, auto cc) {
    constexpr int c = decltype(cc)::value, k = decltype(base)::value + c / 3;
    if constexpr (c % 3 == 1 && k < NP) piece(ftile, fidx & 3, k);
  };
  auto dm_none = [&](auto) {};
  first_ref(sA, rfA, q5A);
  phase(sB, qb, q5B, oB0, oB1, pB, sA, rfA, pA, lsA, selA, selB, kwA, std::integral_constant<int, 0>{},
        [&](auto cc) {  // alpha (see below)
          constexpr int c = decltype(cc)::value;
          if constexpr (c == 1) mk5_read(64 * t + 32);
          if constexpr (c == 8) mk5_set();
          if constexpr (c >= 5) kf[c - 5] = *(const uint4*)(kst + koff[c - 5] + 32 * 128);
        },
        [&](auto cc) { dm_first(std::integral_constant<int, 0>{}, cc); });
  first_ref(sB, rfB, q5B);
  phase(sA, qa, q5A, oA0, oA1, pA, sB, rfB, pB, lsB, selB, selA, kwB, std::integral_constant<int, 0>{},
        [&](auto cc) {  // beta
          constexpr int c = decltype(cc)::value;
          if constexpr (c < 4) rdv(vst, c);
        },
        [&](auto cc) { dm_first(std::integral_constant<int, 3>{}, cc); });
  A8ST(2);
  // the other spans (mid-tile i to mid-tile i + 1: the current tile's half 1, the next tile's half 0) fill active tile
  // i + 3 into the stage of tile i - 1 (read out before mid-tile i): pieces in chunks 2 and 6 of the first 3 phases
  auto dm_span = [&](auto base, auto cc) {
    constexpr int c = decltype(cc)::value, k = decltype(base)::value + (c == 6 ? 1 : 0);
    if constexpr ((c == 2 || c == 6) && k < NP) piece(ftile, fidx & 3, k);
  };
  for (int i = 0;; ++i) {
    const bool more = cmask != 0u;
    // ---- mid-tile: the previous tile's stage is read out by every wave; the next active tile must have landed (own
    // pieces, then every wave's by the barrier; the span's fill of the tile after it stays in flight)
    int tn = t, stn = st;
    unsigned kwAn = 0xFFFFFFFFu, kwBn = 0xFFFFFFFFu;
    if (more) {
      tn = __builtin_ctz(cmask);
      cmask &= cmask - 1u;
      stn = st == A8_NS - 1 ? 0 : st + 1;
#ifndef A8_NOWAIT  // timing-only ablation: no wait for the next tile's DMA (wrong results)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NP) : "memory");
#else
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
      __builtin_amdgcn_s_barrier();
#ifdef A8_STAMPS  // constant indices only (a register array indexed at run time would go to scratch)
      if (i == 0) A8ST(3);
      if (i == 1) A8ST(4);
      if (i == 2) A8ST(5);
      if (i == 3) A8ST(6);
      if (i == 4) A8ST(7);
      if (i == 5) A8ST(8);
      if (i == 6) A8ST(9);
      if (i == 7) A8ST(10);
#endif
      if constexpr (DROP) {
        kwAn = kbl[stn * 512 + (2 * w) * 64 + lane];
        kwBn = kbl[stn * 512 + (2 * w + 1) * 64 + lane];
      }
    }
    ++fidx;
    ftile = next_fill_tile();
    {
      const unsigned char* kimn = kst + stn * A7_TB;
      const unsigned char* vimg = vst + st * A7_TB;
      // ---- half 1. alpha: S_B(h1), PV_B(h0); softmax A(h1); reads: k5 and K of the next tile's h0
      phase(sB, qb, q5B, oB0, oB1, pB, sA, 0.f, pA, lsA, selA, selB, kwA, std::integral_constant<int, 1>{},
            [&](auto cc) {
              constexpr int c = decltype(cc)::value;
              if constexpr (c == 1) mk5_read(64 * tn);
              if constexpr (c == 8) mk5_set();
              if constexpr (c >= 5) kf[c - 5] = *(const uint4*)(kimn + koff[c - 5]);
            },
            [&](auto cc) { dm_span(std::integral_constant<int, 0>{}, cc); });
      // beta: V of h1 (chunks 0-3, before its PV in chunks 5-8), S_A(next h0), PV_A(h1); softmax B(h1)
      phase(sA, qa, q5A, oA0, oA1, pA, sB, 0.f, pB, lsB, selB, selA, kwB, std::integral_constant<int, 1>{},
            [&](auto cc) {
              constexpr int c = decltype(cc)::value;
              if constexpr (c < 4) rdv(vimg + 32 * 128, c);
            },
            [&](auto cc) { dm_span(std::integral_constant<int, 2>{}, cc); });
    }
    if (!more) break;
    t = tn;
    st = stn;
    kwA = kwAn;
    kwB = kwBn;
    {
      const unsigned char* kimg = kst + st * A7_TB;
      const unsigned char* vimg = vst + st * A7_TB;
      // ---- half 0. alpha: S_B(h0), PV_B(previous h1); softmax A(h0); reads: k5 and K of h1 (after S_B's last K use)
      phase(sB, qb, q5B, oB0, oB1, pB, sA, 0.f, pA, lsA, selA, selB, kwA, std::integral_constant<int, 0>{},
            [&](auto cc) {
              constexpr int c = decltype(cc)::value;
              if constexpr (c == 1) mk5_read(64 * t + 32);
              if constexpr (c == 8) mk5_set();
              if constexpr (c >= 5) kf[c - 5] = *(const uint4*)(kimg + koff[c - 5] + 32 * 128);
            },
            [&](auto cc) { dm_span(std::integral_constant<int, 4>{}, cc); });
      // beta: V of h0, S_A(h1), PV_A(h0); softmax B(h0)
      phase(sA, qa, q5A, oA0, oA1, pA, sB, 0.f, pB, lsB, selB, selA, kwB, std::integral_constant<int, 0>{},
            [&](auto cc) {
              constexpr int c = decltype(cc)::value;
              if constexpr (c < 4) rdv(vimg, c);
            },
            dm_none);
    }
  }
  // pipeline end: PV_B of the last half (and its second half's row sum)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    oB0 = mfma32(vf[s][0], pB[s], oB0);
    oB1 = mfma32(vf[s][1], pB[s], oB1);
  }
  if constexpr (RSM) lsum = mfma32(selB, ucar, lsum);
  }  // nact > 0

  A8ST(12);
  // no LDS-DMA may land after the workgroup retires (the fills past the last tile are the only ones left)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  A8ST(13);
  // the row sums (adds: the query's keys sit in lanes l and l ^ 32; MFMA: accumulator rows 0 + 4 hh / 16 + 4 hh)
  float ltA = RSM ? lsum[0] : xsum32(lsA), ltB = RSM ? lsum[8] : xsum32(lsB);
#ifdef A8_NOFALLBACK  // timing-only ablations below skip the fallback (their sums are not softmax sums)
  if (false) {
#else
  if (nact > 0 && __any(!(ltA <= 0x1p64f && ltA >= 0x1p-40f) || !(ltB <= 0x1p64f && ltB >= 0x1p-40f))) {
#endif
    // ---- fallback (guard tripped): both chains again, online softmax with rescaling (fwd7's algorithm), each
    // active tile staged by this wave alone into its own 16 KB past the ring (K image 8 KB, V image 8 KB; no other
    // wave touches it, so no barrier), keep dwords from memory
    unsigned char* kp = sm8 + attn8_fwd_fb_off(a.Lk) + w * 16384;
    unsigned char* vp = kp + 8192;
    auto redo = [&](int c, const uint4 (&qX)[4], f32x16_t& o0, f32x16_t& o1, float& l, float& rf) {
      const int qg = min(qg0 + c, nqg - 1);
      float m = -INFINITY;
      rf = 0.f;
      l = 0.f;
      o0 = f32x16_t{};
      o1 = f32x16_t{};
      uint4 q5 = q5init;
      unsigned tm_ = tmask;
      while (tm_) {
        const int tt = __builtin_ctz(tm_);
        tm_ &= tm_ - 1u;
        const int r = 64 * tt + lane, rr = min(r, a.Lk - 1);
#pragma unroll
        for (int ch = 0; ch < 8; ++ch) {
          const uint4 kx = *(const uint4*)(Kb + (long)rr * a.sk + 8 * ch);
          const uint4 vx = *(const uint4*)(Vb + (long)rr * a.sv + 8 * ch);
          *(uint4*)(kp + lane * 128 + ((ch ^ ((lane >> 1) & 7)) << 4)) = kx;
          *(uint4*)(vp + lane * 128 + ((ch ^ vsw(lane)) << 4)) = vx;
        }
        unsigned kw = 0xFFFFFFFFu;
        if constexpr (DROP) kw = lbits[lb_dword(bh, nqg, ntiles, qg, tt) + lane];
        static_for<0, 2>([&](auto kbc) {
          constexpr int kb = decltype(kbc)::value;
          const uint4 k5_ = mk5(64 * tt + 32 * kb);
          f32x16_t sc = mfma32(k5_, q5, f32x16_t{});
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) sc = mfma32(*(const uint4*)(kp + koff[ks] + kb * 32 * 128), qX[ks], sc);
          float tmx = fmaxf(sc[0], sc[1]);
#pragma unroll
          for (int rr2 = 2; rr2 < 16; rr2 += 2) tmx = fmaxf(tmx, fmaxf(sc[rr2], sc[rr2 + 1]));
          tmx = xmax32(tmx) + rf;
          const float mn = fmaxf(m, tmx);
          float rn = rf;
          if (mn != -INFINITY) rn = __uint_as_float(((unsigned)pk_bf16(mn, 0.f)) << 16);
          const float alpha = (m == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(rf - rn);
          l *= alpha;
          o0 *= alpha;
          o1 *= alpha;
          uint4 pp[2];
          float la = 0.f, lb = 0.f;
          static_for<0, 8>([&](auto ic) { sm_pair_f32(sc, rn - rf, kw, pp, la, lb, kbc, ic); });
          l += la + lb;
          m = mn;
          rf = rn;
          q5 = hh ? make_uint4(0, 0, 0, 0) : make_uint4(pk_bf16(-rf, 1.f), 0u, 0u, 0u);
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const int rb = (32 * kb + 16 * s) * 128;
            o0 = mfma32(join_tr(tr_read(vp + voff[0] + rb), tr_read(vp + voff[0] + rb + 1024)), pp[s], o0);
            o1 = mfma32(join_tr(tr_read(vp + voff[1] + rb), tr_read(vp + voff[1] + rb + 1024)), pp[s], o1);
          }
        });
      }
      l = xsum32(l);
    };
    redo(0, qa, oA0, oA1, ltA, rfA);
    redo(1, qb, oB0, oB1, ltB, rfB);
  }
  // ---- normalise and store straight from the O^T accumulators: lane (qi, hh) holds d = 8 g + 4 hh + 0..3 of its
  // query for g = 0..3 (per 32-d half); one v_permlane32_swap per dword pair gives lane hh = 0 the 8 consecutive d
  // 16 g' .. 16 g' + 7 and lane hh = 1 16 g' + 8 .. + 15 (g' = 0, 1): 16-B stores, the two lanes of a query filling
  // 32 contiguous bytes (no LDS staging, no barrier)
  bf16_t* Ob = (bf16_t*)a.Out + (long)b * a.Lq * a.so + h * DH;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float lt = c ? ltB : ltA;
    const float rf = c ? rfB : rfA;
    const float inv = (lt > 0.f) ? (DROP ? a.drop_scale : 1.f) / lt : NAN;
    const int q = qw0 + 32 * c + qi;
    bf16_t* orow = Ob + (long)min(q, a.Lq - 1) * a.so;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const f32x16_t& oo = c ? (db ? oB1 : oB0) : (db ? oA1 : oA0);
#pragma unroll
      for (int gp = 0; gp < 2; ++gp) {
        unsigned p0[2], p1[2];  // d groups 2 gp and 2 gp + 1, packed bf16 pairs
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          p0[j] = pk_bf16(oo[8 * gp + 2 * j] * inv, oo[8 * gp + 2 * j + 1] * inv);
          p1[j] = pk_bf16(oo[8 * gp + 4 + 2 * j] * inv, oo[8 * gp + 4 + 2 * j + 1] * inv);
        }
        const auto s0 = __builtin_amdgcn_permlane32_swap(p0[0], p1[0], false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(p0[1], p1[1], false, false);
        const uint4 v = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        if (q < a.Lq) *(uint4*)(orow + 32 * db + 16 * gp + 8 * hh) = v;
      }
    }
    if (a.lse && hh == 0 && q < a.Lq)
      a.lse[(long)bh * a.Lq + q] = (lt > 0.f) ? (rf + __log2f(lt)) * 0.69314718055994531f : NAN;
  }
#ifdef A8_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  A8ST(14);
  if (threadIdx.x == 0) {
    unsigned long long* dst = (unsigned long long*)(Ob + (long)(bxi * 256) * a.so);
#pragma unroll
    for (int k = 0; k < 16; ++k) dst[k] = a8st_[k];
#ifdef A8_FINE
    unsigned long long* dst2 = (unsigned long long*)(Ob + (long)(bxi * 256 + 1) * a.so);
#pragma unroll
    for (int k = 0; k < 16; ++k) dst2[k] = a8fs_[k];
#endif
  }
#endif
}

#ifndef A8_LDS_FLOOR
#define A8_LDS_FLOOR 0  // timing probe: a larger LDS request limits the workgroups per CU (tools/build_variant.sh)
#endif
size_t attn8_fwd_lds(int Lk) {
  const size_t n = (size_t)attn8_fwd_fb_off(Lk) + 4 * 16384;  // + the 4 waves' fallback staging
  return n > (size_t)A8_LDS_FLOOR ? n : (size_t)A8_LDS_FLOOR;
}

int attn8_fwd(AttnArgs& a, hipStream_t s) {
  if (a.Lk > 1024 || a.Lk <= 0 || a.Lq <= 0) return (int)hipErrorInvalidValue;
  const int dm = a.thr16 == 0 ? 0 : 1;
  const int mk = a.key_keep != nullptr ? 2 : (a.Lk % 64) != 0 ? 1 : 0;
  const size_t lds = attn8_fwd_lds(a.Lk);
  dim3 grid((a.Lq + 255) / 256, a.B * a.H);
#define FWD8(D, M) hipLaunchKernelGGL((fwd8_kernel<D, M>), grid, dim3(256), lds, s, a)
  if (dm) { if (mk == 2) FWD8(1, 2); else if (mk == 1) FWD8(1, 1); else FWD8(1, 0); }
  else { if (mk == 2) FWD8(0, 2); else if (mk == 1) FWD8(0, 1); else FWD8(0, 0); }
#undef FWD8
  return (int)hipGetLastError();
}

}  // namespace attn
}  // namespace fddm
