// 256x256 bf16 NT GEMM for gfx950 (MI355X):  C[m][n] = sum_k A(m,k) * B(n,k) + bias[n]  (+ epilogue)
//
// The large forward GEMMs of the train step run here: the WavLM conv feature extractor (layers 1..6 as
// implicit GEMMs over channels-last windows), the WavLM Q|K|V / FF projections, the decoder FF1 and head.
//
// Persistent: one 512-thread workgroup per CU walks its tiles back to back through ONE continuous LDS-DMA
// pipeline — the first K-tiles of tile i+1 are in flight while tile i finishes, and tile i's results are
// stored from registers in phase 1 of tile i+1's first K-tile, so neither the prologue
// latency nor the store drain is exposed per tile. Tile order: each XCD owns a contiguous range of a
// grouped (4 M-rows x all N-tiles) ordering, so the ~32 tiles an XCD runs at once share A and B panels in
// its L2.
//
// Geometry: 8 waves as 2 (M) x 4 (N); each wave owns a 128x64 output sub-tile = 8 x 4 MFMA 16x16x32 blocks
// (128 f32 accumulators per lane, seeded with the bias). BK = 64.
// LDS: 2 stages x 4 half-tile images of 16 KB = 128 KB, one `extern __shared__` array:
//   A0 / A1 = the A rows a wave group reads in phase 1 / 3 (rows wr*128 + {0..63} / {64..127}),
//   B0 / B1 = the B rows (output columns) read in phase 4 of the previous K-tile / phase 2 (cols wc*64 +
//   {0..31} / {32..63}). Every image is [128 rows][128 B] with the XOR chunk swizzle swz_kc (conflict-free
//   ds_read_b128), filled by global_load_lds_dwordx4 (1 KB = 8 rows per wave instruction; the swizzle is
//   applied to the SOURCE address).
// K-tile = 4 phases; each phase = [the previous tile's epilogue (phase 1 of the first K-tile only), fragment
// reads, one half-tile LDS-DMA, counted vmcnt] -> s_barrier -> 16 MFMAs (one 64x32 quadrant, K = 64) ->
// s_barrier. The wave groups wr = 0 / 1 run one barrier apart: on every SIMD one wave issues MFMAs while its
// partner reads LDS and issues DMA. A half-tile is re-staged >= 2 phases after its last read and read >= 4
// phases after its DMA. Every vmcnt is exact: the wave counts each vector-memory instruction it issues
// (DMA, bias loads, stores — all explicit, none compiler-generated) and waits for "issued since X".
// The MFMAs compute C^T fragments (operands swapped) so a lane owns 4 consecutive columns of one row: the
// epilogue writes 16-B buffer stores of whole 128-B lines from the accumulators after two lane exchanges.
#include "gemm.h"
#include <type_traits>

namespace fddm {
namespace g256 {

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));

#ifndef G256_GM
#define G256_GM 4
#endif
// Both LDS-DMA instructions of a half-tile are issued between the MFMAs of the compute segment that follows the
// load segment which used to issue them (steady K-tile at the WavLM FF1 shape: 3256 cycles with both in the load
// segment, 3080 with one deferred, 2972-2984 with both; tools/g256_stamps.py). -DG256_DEFER1 keeps one in the
// load segment.
#ifndef G256_DEFER1
#define G256_DEFER2
#endif
constexpr int BM = 256, BN = 256, HALF = 16384, STAGE = 4 * HALF, LDS_BYTES = 2 * STAGE, GM = G256_GM;
constexpr unsigned SRD_W3 = 0x00020000u;  // buffer resource word 3 (raw dword access) on gfx9xx
enum { HA0 = 0, HA1 = 1, HB0 = 2, HB1 = 3 };

// LDS fragment read as inline asm: hipcc's waitcnt pass would make a plain ds_read wait for every
// outstanding LDS-DMA (vmcnt(0)); the kernel waits lgkmcnt itself before the MFMAs.
__device__ __forceinline__ u32x4_t ds_read128(const unsigned char* p) {
  const unsigned a = (unsigned)(size_t)(lptr_t)(void*)p;
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

template <int OFF>
__device__ __forceinline__ u32x4_t ds_read128_at(unsigned a) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF) : "memory");
  return v;
}
template <int V> using IC = std::integral_constant<int, V>;

// leave at most N vector-memory instructions of this wave in flight (N is always a compile-time count)
template <int N> __device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 63 ? N : 63) : "memory");
}

// 16-B buffer store as inline asm with the wait state gfx950 needs before the store-data VGPRs may be
// rewritten (a wide store reads its data late: the builtin let hipcc overwrite them in the next instruction,
// corrupting the last lanes' data)
__device__ __forceinline__ void store16(const u32x4_t& d, const i32x4_t& srd, int voff, int soff) {
#ifdef G256_NOSTORE  // timing diagnostic only (tools/g256_stamps.py): no output, so no MFMA survives either
  if (soff == -1)
#endif
  asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen\n\ts_nop 1" ::"v"(d), "v"(voff), "s"(srd), "s"(soff)
               : "memory");
}
__device__ __forceinline__ i32x4_t make_srd(const void* base) {
  const unsigned long a = (unsigned long)base;
  return i32x4_t{(int)(unsigned)a, (int)(unsigned)(a >> 32), 0x7fffffff, (int)SRD_W3};
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

#ifdef G256_STAMPS
// diagnostic build only: s_memtime at the start of each K-tile of each workgroup (fddm_gemm256_stamps reads it)
__device__ unsigned long long g256_stamps[256 * G256_STAMPS];
#endif

template <int EPI, typename OT, bool CONV>
__global__ void __launch_bounds__(512) gemm256_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int fr = lane & 15, fg = lane >> 4;

  // ---------------------------------------------------------------- persistent schedule
  const int nN = (int)((g.N + BN - 1) / BN), nM = (int)((g.M + BM - 1) / BM), tiles = nN * nM;
  const int G = gridDim.x, wg = blockIdx.x, x = wg & 7, jx = wg >> 3;
  int Wx = 0;  // workgroups on the XCDs before this one (workgroup w runs on XCD w % 8)
  for (int y = 0; y < x; ++y) Wx += (G - 1 - y) / 8 + 1;
  const int Px = (G - 1 - x) / 8 + 1;
  const int s0 = (int)((long)tiles * Wx / G), s1 = (int)((long)tiles * (Wx + Px) / G);
  const int nmine = (s1 - s0 > jx) ? (s1 - s0 - jx + Px - 1) / Px : 0;
  if (nmine == 0) return;
  // i-th tile of this workgroup (clamped to its last one: loads past the end re-read valid data). A ragged
  // last tile is computed as the full tile ending at M (N): it recomputes some rows (columns) of its
  // neighbour bit-identically and writes the same values, so no load or store needs a bounds check.
  auto coords = [&](int i, int& m0, int& n0) {
    const int s = s0 + jx + min(i, nmine - 1) * Px;
    const int per = GM * nN, grp = s / per, first = grp * GM, gsz = min(GM, nM - first), rr = s - grp * per;
    m0 = min((first + rr % gsz) * BM, (int)g.M - BM);
    n0 = min((rr / gsz) * BN, (int)g.N - BN);
  };

  // ---------------------------------------------------------------- operand sources
  // Buffer resources over A and B; per-lane byte offsets of the rows a lane fills relative to the tile
  // origin (half h, instruction i fills image rows (wid*2+i)*8 + lane/8, physical chunk lane%8, which holds
  // logical chunk (lane%8) ^ ((row>>1)&7)); tile origin, half shift and K offset go in the scalar soffset.
  // Implicit conv: A rows are (utterance, frame) windows, so their offsets are per tile and per half.
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, 0x7fffffff, SRD_W3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, 0x7fffffff, SRD_W3);
  const int lda = (int)g.lda, ldb = (int)g.ldb, ldc = (int)g.ldc, Nc = (int)g.N;
  int va[2], vb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wid * 2 + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    va[i] = (((row >> 6) * 128 + (row & 63)) * lda + c * 8) * 2;  // A0 rows; A1 = +64 rows
    vb[i] = (((row >> 5) * 64 + (row & 31)) * ldb + c * 8) * 2;   // B0 rows; B1 = +32 rows
  }
  int vcc[2][2] = {{0, 0}, {0, 0}}, vcn[2][2] = {{0, 0}, {0, 0}};  // conv: [half][i] of current / next tile
  auto conv_rows = [&](int (&v)[2][2], int m0) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (wid * 2 + i) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        const int m = m0 + (row >> 6) * 128 + h * 64 + (row & 63);
        const int b = m / (int)g.Mi, tt = m - b * (int)g.Mi;
        v[h][i] = (b * (int)g.sAb + tt * (int)(g.geo.cstride * g.lda) + c * 8) * 2;
      }
  };
  // A half-tile is 2 LDS-DMA instructions per wave. In the K loop (split = true) they are left pending and issued
  // between the MFMAs of the following compute segment (mma) — G256_DEFER1: only the second — so the load segment,
  // which bounds each barrier interval (fragment reads + wait), carries no DMA issue.
  int pd_v = 0, pd_so = 0;
  lptr_t pd_d = nullptr;
#ifdef G256_DEFER2
  int pd0_v = 0;
  lptr_t pd0_d = nullptr;
#endif
  bool pd_b = false;
  auto issue = [&](int h, int buf, int v0, int v1, int so, bool split = false) {  // so: scalar byte offset
#ifdef G256_NODMA  // timing diagnostic only: operand tiles never loaded (garbage results)
    if (so != -12345) return;
#endif
    lptr_t d = (lptr_t)(smem + buf * STAGE + h * HALF + wid * 2048);
    const __amdgpu_buffer_rsrc_t& r = h < 2 ? rA : rB;
#ifdef G256_DEFER2
    if (split) {
      pd0_d = d;
      pd0_v = v0;
    } else
#endif
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, d, 16, v0, so, 0, 0);
    if (split) {
      pd_d = (lptr_t)((unsigned char*)d + 1024);
      pd_v = v1;
      pd_so = so;
      pd_b = h >= 2;
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr_t)((unsigned char*)d + 1024), 16, v1, so, 0, 0);
    }
  };
  auto issue_pending = [&]() {
#ifdef G256_NODMA
    if (pd_so != -12345) return;
#endif
    if (pd_b) __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, pd_d, 16, pd_v, pd_so, 0, 0);
    else __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, pd_d, 16, pd_v, pd_so, 0, 0);
  };
  const int nk = (int)(g.K / 64);
  const int cshift = CONV ? __builtin_ctz((unsigned)(g.geo.Cg / 64)) : 0;  // K-tiles per conv tap = 2^cshift
  auto koffA = [&](int kt) -> int {  // byte offset of K-tile kt in an A row
    if (!CONV) return kt * 128;
    return ((kt >> cshift) * lda + (kt & ((1 << cshift) - 1)) * 64) * 2;
  };
  // tile origins: current tile (cm0, cn0) and this workgroup's next tile (nm0, nn0)
  int cm0, cn0, nm0, nn0;
  coords(0, cm0, cn0);
  coords(1, nm0, nn0);
  if (CONV) {
    conv_rows(vcc, cm0);
    conv_rows(vcn, nm0);
  }
  // half h of K-tile kt of the tile at (m0, n0) [conv: lane offsets vc]
  auto issueA = [&](int h, int buf, int kt, int m0, const int (&vc)[2][2], bool split = false) {
    if (CONV) issue(h, buf, vc[h][0], vc[h][1], koffA(kt), split);
    else issue(h, buf, va[0], va[1], m0 * lda * 2 + h * 64 * lda * 2 + koffA(kt), split);
  };
  auto issueB = [&](int h, int buf, int kt, int n0, bool split = false) {
    issue(h, buf, vb[0], vb[1], n0 * ldb * 2 + (h - 2) * 32 * ldb * 2 + kt * 128, split);
  };

  // ---------------------------------------------------------------- bias
  // each wave's 64 columns n0 + wc*64 + 0..63 come into its own 256-B LDS slot (one 4-byte LDS-DMA, one tile
  // ahead) and seed the accumulators; without a bias the DMA reads A (any valid address) and the seed is 0
  // Every K-tile issues one such DMA (phase 1); only a tile's last K-tile aims it at the real slot, the others
  // at a dummy slot, so that all K-tiles issue the same vector-memory sequence.
  const bool has_bias = g.bias != nullptr;
  unsigned char* bslot = smem + LDS_BYTES + wid * 256;
  auto load_bias = [&](int n0, bool real) {
    const float* src = has_bias ? g.bias + n0 + wc * 64 + lane : (const float*)g.A + lane;
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(real ? bslot : bslot + 2048), 4, 0, 0);
  };
  // the 4 bias values of block columns jb, jb+1 for this lane (columns j*16 + 4*fg .. +3); the slot's DMA
  // has been covered by a vmcnt of this wave
  auto bias_pair = [&](int jb, f32x4_t& v0, f32x4_t& v1) {
    const u32x4_t a = ds_read128(bslot + (jb * 16 + 4 * fg) * 4);
    const u32x4_t b = ds_read128(bslot + ((jb + 1) * 16 + 4 * fg) * 4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    v0 = __builtin_bit_cast(f32x4_t, a);
    v1 = __builtin_bit_cast(f32x4_t, b);
    asm volatile("" : "+v"(v0), "+v"(v1));
    if (!has_bias) {
      v0 = f32x4_t{0.f, 0.f, 0.f, 0.f};
      v1 = v0;
    }
  };

  // ---------------------------------------------------------------- stores
  // buffer stores: lane offset fixed, tile origin and block offset in soffset
  const i32x4_t rc = make_srd(g.C);
  const i32x4_t rc2 = make_srd(EPI == EPI_GELU ? g.C2 : g.C);
  constexpr int ESZ = (int)sizeof(OT);
  // store instructions per half (4 row blocks x 64 columns): f32 16; bf16 8 per output
  constexpr int SPH = sizeof(OT) == 4 ? 16 : (EPI == EPI_GELU ? 16 : 8);
  // Every store instruction writes 8 whole rows x 128 B (full cache lines), and each group of 4 consecutive
  // lanes 2 rows: a wave's 16 x 64 row block leaves in 2 (bf16) or 4 (f32) instructions, even rows in the
  // first, odd rows in the second. Lane (fr, fg) writes row (fr & ~1) (+1 in the second register); fr & 1
  // selects the column half (bf16: 32 of the wave's 64 columns, f32: 16 of a 32-column pair); cc = the 16-B
  // chunk within it. Epilogue K-tile at the WavLM FF1 shape (tools/g256_stamps.py): 16 rows x 64 B per
  // instruction and 4 rows per lane group, one quadrant per phase: 11.9k cycles; whole lines but 4 rows per
  // lane group: 11.7k; whole lines, 2 rows per lane group, one half-tile per odd phase: 9.9k; the same with
  // the whole tile in phase 1: 9.2k (steady K-tile 2956).
  const int cc = sizeof(OT) == 4 ? 4 * fg : 4 * fg + ((fg & 1) ? 12 : 0);
  const int vst = ((wr * 128 + (fr & ~1)) * ldc + wc * 64 + (fr & 1) * (sizeof(OT) == 4 ? 16 : 32) + cc) * ESZ;
  const bool odd_r = fr & 1;

  u32x4_t af[4][2], b0[2][2], b1[2][2];
  f32x4_t acc[8][4];

  // x0 / x1 hold row fr of column group 0 / 1; after the exchange (lane bit 0 <-> register) x0 holds the even
  // and x1 the odd rows of the block, lane bit 0 selecting the column group. Lanes fr and fr ^ 1 trade through
  // DPP quad_perm [1,0,3,2].
  // (each select reads its partner's register through DPP: hipcc folds the quad_perm into the v_cndmask, two VALU per
  // dword instead of a select, a DPP move and two selects)
  auto xchg1 = [&](u32x4_t& x0, u32x4_t& x1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned a = x0[e], b = x1[e];
      const unsigned pb = (unsigned)__builtin_amdgcn_mov_dpp((int)b, 0xb1, 0xf, 0xf, false);  // x1 of lane ^ 1
      const unsigned pa = (unsigned)__builtin_amdgcn_mov_dpp((int)a, 0xb1, 0xf, 0xf, false);  // x0 of lane ^ 1
      x0[e] = odd_r ? pb : a;
      x1[e] = odd_r ? b : pa;
    }
  };
  // bf16: the two lanes 16 apart (fg, fg^1) trade packed halves (v_permlane16_swap) so that each lane holds 8
  // consecutive columns (16 B) of a 32-column pair; odd-fg lanes hold the second block of the pair.
  // v_permlane16_swap(pa, pb) swaps the odd 16-lane rows of pa with the even rows of pb: an even-row lane keeps its pa
  // and gets the pa of lane + 16 in pb's place, an odd-row lane gets the pb of lane - 16 in pa's place and keeps its pb
  // — exactly {pa, pa'} / {pb', pb}, no lane-parity selects
  auto chunk16 = [&](const f32x4_t& a, const f32x4_t& b) -> u32x4_t {
    const auto s0 = __builtin_amdgcn_permlane16_swap(pk_bf16(a[0], a[1]), pk_bf16(b[0], b[1]), false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(pk_bf16(a[2], a[3]), pk_bf16(b[2], b[3]), false, false);
    return u32x4_t{s0[0], s1[0], s0[1], s1[1]};
  };
  // one bf16 row block (4 column blocks v) -> 2 whole-line stores
  auto emit_bf16 = [&](const f32x4_t (&v)[4], const i32x4_t& r, int so) {
    u32x4_t x0 = chunk16(v[0], v[1]), x1 = chunk16(v[2], v[3]);
    xchg1(x0, x1);
    store16(x0, r, vst, so);
    store16(x1, r, vst, so + ldc * ESZ);
  };

  // half hh of the finished tile at (em0, en0): row blocks 4*hh .. 4*hh+3, all 4 column blocks; then (reseed)
  // seed them with the bias of the tile that follows
  auto epi_rows = [&](auto ibc, auto nc, int em0, int en0, bool reseed) {
    constexpr int ib = decltype(ibc)::value, NR = decltype(nc)::value;
    f32x4_t bq[4];
    if (reseed) {
      bias_pair(0, bq[0], bq[1]);
      bias_pair(2, bq[2], bq[3]);
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int so = ((em0 + (ib + i) * 16) * ldc + en0) * ESZ;
      if constexpr (sizeof(OT) == 4) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          u32x4_t x0 = __builtin_bit_cast(u32x4_t, acc[ib + i][2 * p]);
          u32x4_t x1 = __builtin_bit_cast(u32x4_t, acc[ib + i][2 * p + 1]);
          xchg1(x0, x1);
          store16(x0, rc, vst, so + 32 * p * ESZ);
          store16(x1, rc, vst, so + (ldc + 32 * p) * ESZ);
        }
      } else {
        f32x4_t v[4] = {acc[ib + i][0], acc[ib + i][1], acc[ib + i][2], acc[ib + i][3]};
        if constexpr (EPI == EPI_GELU) {
          emit_bf16(v, rc, so);
          const unsigned thr = g.thr16;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            unsigned keep = 0xfu;
            if (thr) {  // 4 consecutive columns (N % 8 == 0): one hash
              const unsigned m = (unsigned)(em0 + wr * 128 + (ib + i) * 16 + fr);
              const unsigned n = (unsigned)(en0 + wc * 64 + j * 16 + 4 * fg);
              keep = drop_keep4(eff_seed(g.seed, g.seed_off), g.stream, ((uint64_t)m * (uint64_t)Nc + n) >> 2, thr);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float a = gelu_f(v[j][e]);
              v[j][e] = thr ? ((keep >> e) & 1u ? a * g.drop_scale : 0.f) : a;
            }
          }
          emit_bf16(v, rc2, so);
        } else {
          if constexpr (EPI == EPI_GELU_ONLY) {  // the frozen encoder's conv layers / FF1: bf16-output GELU
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e) v[j][e] = gelu_bf16out(v[j][e]);
          }
          emit_bf16(v, rc, so);
        }
      }
      if (reseed) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[ib + i][j] = bq[j];
      }
      __builtin_amdgcn_sched_barrier(0);  // one row block at a time: bounds the epilogue's live registers
    }
  };

  // fragment addresses: swz_kc(base16 + i*16 + fr, s*4 + fg) = (base16 + i*16)*128 + swz_kc(fr, s*4 + fg) for a
  // 16-aligned base, so one lane address per k-half s plus immediate offsets (half image, row block)
  const unsigned lds0 = (unsigned)(size_t)(lptr_t)(void*)smem;
  const unsigned aadr[2] = {lds0 + wr * 8192 + swz_kc(fr, fg), lds0 + wr * 8192 + swz_kc(fr, 4 + fg)};
  const unsigned badr[2] = {lds0 + wc * 4096 + swz_kc(fr, fg), lds0 + wc * 4096 + swz_kc(fr, 4 + fg)};
  auto readA = [&](int buf, auto hc) {
    constexpr int h = decltype(hc)::value;
#ifdef G256_NOREAD  // timing diagnostic only: no fragment reads (MFMAs on stale registers)
    asm volatile("" : "+v"(af[0][0]), "+v"(af[1][0]), "+v"(af[2][0]), "+v"(af[3][0]), "+v"(af[0][1]), "+v"(af[1][1]),
                 "+v"(af[2][1]), "+v"(af[3][1]));
    if (buf >= 0) return;
#endif
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const unsigned a = aadr[s] + buf * STAGE;
      af[0][s] = ds_read128_at<h * HALF + 0 * 2048>(a);
      af[1][s] = ds_read128_at<h * HALF + 1 * 2048>(a);
      af[2][s] = ds_read128_at<h * HALF + 2 * 2048>(a);
      af[3][s] = ds_read128_at<h * HALF + 3 * 2048>(a);
    }
  };
  auto readB = [&](int buf, auto hc, u32x4_t(&bf)[2][2]) {
    constexpr int h = decltype(hc)::value;
#ifdef G256_NOREAD
    asm volatile("" : "+v"(bf[0][0]), "+v"(bf[1][0]), "+v"(bf[0][1]), "+v"(bf[1][1]));
    if (buf >= 0) return;
#endif
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const unsigned a = badr[s] + buf * STAGE;
      bf[0][s] = ds_read128_at<h * HALF + 0 * 2048>(a);
      bf[1][s] = ds_read128_at<h * HALF + 1 * 2048>(a);
    }
  };
  // one quadrant: rows ib..ib+3 (A fragments af) x cols jb..jb+1 (bf), K = 64; operands swapped -> C^T
  auto mma = [&](int ib, int jb, const u32x4_t(&bf)[2][2]) {
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[ib + i][jb + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, bf[j][s]), __builtin_bit_cast(bf16x8_t, af[i][s]), acc[ib + i][jb + j], 0, 0,
              0);
#ifdef G256_DEFER2
      if (i == 0) {
        __builtin_amdgcn_sched_barrier(0);
        if (pd_b) __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, pd0_d, 16, pd0_v, pd_so, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, pd0_d, 16, pd0_v, pd_so, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (i == 2) {
#else
      if (i == 1) {  // the load segment's second DMA instruction, behind 8 MFMAs
#endif
        __builtin_amdgcn_sched_barrier(0);
        issue_pending();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    bar();
  };

  // ---------------------------------------------------------------- prologue
  // VMEM issue order (= the steady-state order of the K loop): bias(tile 0), A0 B0 B1 A1 of K-tile 0,
  // A0 B0 of K-tile 1
  load_bias(cn0, true);
  {
    const int kt1 = 1 % nk;
    const int m1 = nk > 1 ? cm0 : nm0, n1 = nk > 1 ? cn0 : nn0;
    issueA(HA0, 0, 0, cm0, vcc);
    issueB(HB0, 0, 0, cn0);
    issueB(HB1, 0, 0, cn0);
    issueA(HA1, 0, 0, cm0, vcc);
    issueA(HA0, 1, kt1, m1, nk > 1 ? vcc : vcn);
    issueB(HB0, 1, kt1, n1);
  }
  vmcnt<8>();  // bias(0), A0(0), B0(0) landed
  bar();
#pragma unroll
  for (int jb = 0; jb < 4; jb += 2) {
    f32x4_t v0, v1;
    bias_pair(jb, v0, v1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i][jb] = v0;
      acc[i][jb + 1] = v1;
    }
  }
  readB(0, IC<HB0>{}, b0);
  if (wr == 1) bar();  // stagger the wave groups by one barrier

  // ---------------------------------------------------------------- flattened K loop over all my tiles
  // One K-tile T (kt within tile ti). Issues, in order: phase 1 bias DMA (real slot on a tile's last K-tile),
  // B1(T+1); phase 2 A1(T+1); phase 3 A0(T+2); phase 4 B0(T+2) — K-tiles past the end re-read valid data.
  // Each phase then waits for the half its successor reads; the count of younger vector-memory instructions
  // is exact and compile-time per mode: EP (kt 0 of tiles >= 1) stores the whole previous tile in phase 1,
  // after its wait, so phases 2-4 of EP count those stores too; the stores precede the next K-tile's awaited
  // halves, so no later count sees them. Requires nk >= 2.
  int em0 = 0, en0 = 0, kt = 0, ti = 0;
  const int NT = nmine * nk;
  // one body for steady and EP K-tiles; only the s_waitcnt immediate depends on the mode
  auto wait2 = [&](bool EP, auto n0c, auto nec) {
    if (EP) vmcnt<decltype(nec)::value>();
    else vmcnt<decltype(n0c)::value>();
  };
#ifdef G256_DEFER2
  constexpr int D2 = 1;  // both DMA instructions of a half deferred: one fewer issued before each wait
#else
  constexpr int D2 = 0;
#endif
  auto ktile = [&](int T, bool EP) {
    const int bc = T & 1, bn = bc ^ 1;
    // K-tile T+1 is in the next tile iff LAST; T+2 iff kt >= nk-2
    const bool n1b = kt == nk - 1, n2 = kt >= nk - 2;
    const int kt1 = n1b ? 0 : kt + 1;
    const int kt2 = n2 ? kt + 2 - nk : kt + 2;
    const int m1 = n1b ? nm0 : cm0, n1 = n1b ? nn0 : cn0;
    const int m2 = n2 ? nm0 : cm0, n2c = n2 ? nn0 : cn0;
    // ---- phase 1: A rows 0..63 x B cols 0..31
    readA(bc, IC<HA0>{});
    load_bias(nn0, n1b);
    issueB(HB1, bn, kt1, n1, true);
    // counts: VMEM instructions issued after the awaited half's second (pending) instruction
    vmcnt<8 - D2>();  // B1(T)
    if (EP) epi_rows(IC<0>{}, IC<8>{}, em0, en0, true);
    mma(0, 0, b0);
    // ---- phase 2: A rows 0..63 x B cols 32..63
    readB(bc, IC<HB1>{}, b1);
    if (CONV) issueA(HA1, bn, kt1, m1, n1b ? vcn : vcc, true);
    else issueA(HA1, bn, kt1, m1, vcc, true);
    wait2(EP, IC<8 - D2>{}, IC<8 - D2 + 2 * SPH>{});  // A1(T)
    mma(0, 2, b1);
    // ---- phase 3: A rows 64..127 x B cols 0..31
    readA(bc, IC<HA1>{});
    if (CONV) issueA(HA0, bc, kt2, m2, n2 ? vcn : vcc, true);
    else issueA(HA0, bc, kt2, m2, vcc, true);
    wait2(EP, IC<6 - D2>{}, IC<6 - D2 + 2 * SPH>{});  // B0(T+1)
    mma(4, 0, b0);
    // ---- phase 4: A rows 64..127 x B cols 32..63; B0 fragments of K-tile T+1
    readB(bn, IC<HB0>{}, b0);
    issueB(HB0, bc, kt2, n2c, true);
    wait2(EP, IC<10 - D2>{}, IC<10 - D2 + 2 * SPH>{});  // A0(T+1)
    mma(4, 2, b1);
  };
  // after a tile's last K-tile: its results move to the epilogue slot, the workgroup's next tile becomes current
  auto next_tile = [&]() {
    em0 = cm0;
    en0 = cn0;
    cm0 = nm0;
    cn0 = nn0;
    coords(ti + 2, nm0, nn0);
    if (CONV) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) vcc[h][i] = vcn[h][i];
      conv_rows(vcn, nm0);
    }
    ++ti;
  };
  for (int T = 0; T < NT; ++T) {
    const bool later = ti > 0;
#ifdef G256_STAMPS
    if (tid == 0 && T < G256_STAMPS) g256_stamps[blockIdx.x * G256_STAMPS + T] = __builtin_amdgcn_s_memtime();
#endif
    ktile(T, later && kt == 0);
    if (kt == nk - 1) {
      next_tile();
      kt = 0;
    } else {
      ++kt;
    }
  }
  if (wr == 0) bar();
  // the last tile (its successor "tile" was a clamped re-read: nothing to seed)
  epi_rows(IC<0>{}, IC<8>{}, em0, en0, false);
  vmcnt<0>();  // no LDS-DMA may land after the workgroup retires
}

// Workgroup cap of the persistent grid (0 = one per CU). Set around launches that share the chip with another
// stream (train.py runs the frozen encoder of the next step beside the decoder): fewer persistent workgroups
// leave whole CUs to the other stream's short launches instead of making them queue behind 132 KB-LDS tiles.
static int g_grid_cap = 0;

template <int EPI, typename OT, bool CONV>
static int launch(const GemmArgs& g, hipStream_t s) {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  const long tiles = gemm256_tiles(g.M, g.N);
#ifdef G256_NOPERSIST
  const long grid = tiles;
#else
  const long cap = (g_grid_cap > 0 && g_grid_cap < ncu) ? g_grid_cap : ncu;
  // as few workgroups as give the same number of tile rounds (e.g. 630 tiles on 256 CUs: 3 rounds either
  // way, 216 workgroups instead of 256): the launch takes as long, and the spare CUs go to the other stream
  const long rounds = (tiles + cap - 1) / cap;
  const long need = ((tiles + rounds - 1) / rounds + 7) & ~7L;
  const long grid = tiles < cap ? tiles : (need < cap ? need : cap);
#endif
  hipLaunchKernelGGL((gemm256_kernel<EPI, OT, CONV>), dim3((unsigned)grid), dim3(512), LDS_BYTES + 4096, s, g);
  return (int)hipGetLastError();
}

}  // namespace g256

long gemm256_tiles(long M, long N) { return ((M + 255) / 256) * ((N + 255) / 256); }

bool gemm256_ok(const GemmArgs& g, int epi, int out_dtype, bool conv) {
  if (g.K % 64 || g.K < 128 || g.M <= 0 || g.N <= 0 || g.N % 8 || g.lda % 8 || g.ldb % 8 || g.ldc % 8) return false;
  if (g.alpha != 1.f) return false;
  if ((((uintptr_t)g.A) | ((uintptr_t)g.B) | ((uintptr_t)g.C) | ((uintptr_t)g.C2) | ((uintptr_t)g.bias)) & 15)
    return false;
  if (g.M < 256 || g.N < 256) return false;  // ragged tiles are shifted full tiles
  // 31-bit byte offsets into A, B and C
  const long aext = conv ? ((g.M / g.Mi) * g.sAb + g.geo.Tin * g.lda) : ((g.M - 1) * g.lda + g.K);
  if (aext * 2 >= (1L << 31) || ((g.N - 1) * g.ldb + g.K) * 2 >= (1L << 31)) return false;
  if (conv && (g.M % g.Mi || g.geo.cstride * g.lda >= (1L << 31))) return false;
  const long esz = out_dtype == FDDM_F32 ? 4 : 2;
  if (((g.M - 1) * g.ldc + g.N) * esz >= (1L << 31)) return false;  // 32-bit buffer offsets
  if (conv && (g.geo.cpad != 0 || g.geo.Cg % 64 || ((g.geo.Cg / 64) & (g.geo.Cg / 64 - 1)))) return false;
  if (out_dtype == FDDM_F32) return epi == EPI_STORE && !conv;
  if (conv) return epi == EPI_STORE || epi == EPI_GELU_ONLY;
  return epi == EPI_STORE || epi == EPI_GELU || epi == EPI_GELU_ONLY;
}

int gemm256_launch(const GemmArgs& g, int epi, int out_dtype, bool conv, hipStream_t s) {
  if (!gemm256_ok(g, epi, out_dtype, conv)) return (int)hipErrorInvalidValue;
  if (out_dtype == FDDM_F32) return g256::launch<EPI_STORE, float, false>(g, s);
  if (conv) {
    if (epi == EPI_GELU_ONLY) return g256::launch<EPI_GELU_ONLY, bf16_t, true>(g, s);
    return g256::launch<EPI_STORE, bf16_t, true>(g, s);
  }
  if (epi == EPI_GELU) return g256::launch<EPI_GELU, bf16_t, false>(g, s);
  if (epi == EPI_GELU_ONLY) return g256::launch<EPI_GELU_ONLY, bf16_t, false>(g, s);
  return g256::launch<EPI_STORE, bf16_t, false>(g, s);
}

}  // namespace fddm

FDDM_API int fddm_gemm_persistent_cap(int cap) {
  const int prev = fddm::g256::g_grid_cap;
  fddm::g256::g_grid_cap = cap > 0 ? (cap & ~7) : 0;  // multiple of 8: the tile order is XCD-chunked
  return prev;
}

#ifdef G256_STAMPS
FDDM_API int fddm_gemm256_stamps(unsigned long long* host, long n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fddm::g256::g256_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
#endif
