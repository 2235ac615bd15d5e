// 256x256 bf16 NT GEMM for gfx950 (MI355X):  C[m][n] = sum_k A(m,k) * B(n,k) + bias[n]  (+ epilogue)
//
// The large forward GEMMs of the train step run here: the WavLM conv feature extractor (layers 1..6 as
// implicit GEMMs over channels-last windows), the WavLM Q|K|V / FF projections, the decoder FF1 and head.
//
// Persistent: one 512-thread workgroup per CU walks its tiles back to back through ONE continuous LDS-DMA
// pipeline — the first K-tiles of tile i+1 are in flight while tile i finishes, and tile i's results are
// stored from registers one quadrant per phase during tile i+1's first K-tile, so neither the prologue
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
// K-tile = 4 phases; each phase = [epilogue quadrant of the previous tile (first K-tile only), fragment
// reads, one half-tile LDS-DMA, counted vmcnt] -> s_barrier -> 16 MFMAs (one 64x32 quadrant, K = 64) ->
// s_barrier. The wave groups wr = 0 / 1 run one barrier apart: on every SIMD one wave issues MFMAs while its
// partner reads LDS and issues DMA. A half-tile is re-staged >= 2 phases after its last read and read >= 4
// phases after its DMA. Every vmcnt is exact: the wave counts each vector-memory instruction it issues
// (DMA, bias loads, stores — all explicit, none compiler-generated) and waits for "issued since X".
// The MFMAs compute C^T fragments (operands swapped) so a lane owns 4 consecutive columns of one row: the
// epilogue writes 8-B (bf16) / 16-B (f32) bounds-checked buffer stores straight from the accumulators.
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

// leave at most n (rounded down to a coded step) vector-memory instructions of this wave in flight
template <int N> __device__ __forceinline__ void vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void wait_vm(int n) {
  if (n >= 32) {
    if (n >= 63) vmcnt<63>();
    else if (n >= 56) vmcnt<56>();
    else if (n >= 48) vmcnt<48>();
    else if (n >= 40) vmcnt<40>();
    else vmcnt<32>();
  } else if (n >= 12) {
    if (n >= 28) vmcnt<28>();
    else if (n >= 24) vmcnt<24>();
    else if (n >= 20) vmcnt<20>();
    else if (n >= 16) vmcnt<16>();
    else vmcnt<12>();
  } else {
    if (n >= 10) vmcnt<10>();
    else if (n >= 8) vmcnt<8>();
    else if (n >= 6) vmcnt<6>();
    else if (n >= 4) vmcnt<4>();
    else if (n >= 2) vmcnt<2>();
    else vmcnt<0>();
  }
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

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
  // A ragged last tile is computed as the full tile ending at M (N): it recomputes some rows (columns) of
  // its neighbour bit-identically and writes the same values, so no load or store needs a bounds check.
  auto coords = [&](int i, int& m0, int& n0) {  // i-th tile of this workgroup
    const int s = s0 + jx + i * Px;
    const int per = GM * nN, grp = s / per, first = grp * GM, gsz = min(GM, nM - first), rr = s - grp * per;
    m0 = min((first + rr % gsz) * BM, (int)g.M - BM);
    n0 = min((rr / gsz) * BN, (int)g.N - BN);
  };

  // LDS-DMA sources: buffer resources over A and B; per-lane byte offsets of the rows a lane fills relative
  // to the tile origin (half h, instruction i fills image rows (wid*2+i)*8 + lane/8, physical chunk lane%8,
  // which holds logical chunk (lane%8) ^ ((row>>1)&7)); tile origin, half shift and K offset go in the
  // scalar soffset. Implicit conv: A rows are (utterance, frame) windows, so their offsets are per tile.
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
  int vc1[2] = {0, 0}, vc2[2] = {0, 0};  // conv: A1 rows of stream 1's tile, A0 rows of stream 2's tile
  auto conv_rows = [&](int (&v)[2], int m0, int h) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (wid * 2 + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int m = m0 + (row >> 6) * 128 + h * 64 + (row & 63);
      const int b = m / (int)g.Mi, tt = m - b * (int)g.Mi;
      v[i] = (b * (int)g.sAb + tt * (int)(g.geo.cstride * g.lda) + c * 8) * 2;
    }
  };
  int vm = 0;  // vector-memory instructions issued by this wave so far
  auto issue = [&](int h, int buf, const int (&v)[2], int so) {  // so: scalar byte offset
    lptr_t d = (lptr_t)(smem + buf * STAGE + h * HALF + wid * 2048);
    const __amdgpu_buffer_rsrc_t& r = h < 2 ? rA : rB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, d, 16, v[0], so, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr_t)((unsigned char*)d + 1024), 16, v[1], so, 0, 0);
    vm += 2;
  };
  // issue streams: K-tile T+1 (halves B1, A1) and T+2 (A0, B0); each tracks its tile, K-tile, tile origin
  // (scalar byte offsets into A and B) and, for conv, the (tap, channel) of the K-tile
  struct Cursor { int ti, kt, tap, c, sa, sb; };
  const int nk = (int)(g.K / 64), NT = nmine * nk;
  const int Cg = CONV ? (int)g.geo.Cg : 64;
  auto advance = [&](Cursor& u) {
    if (++u.kt == nk) { u.kt = 0; ++u.ti; u.tap = 0; u.c = 0; }
    else if (CONV) { u.c += 64; if (u.c == Cg) { u.c = 0; ++u.tap; } }
  };
  auto koffA = [&](const Cursor& u) -> int { return (CONV ? u.tap * lda + u.c : u.sa + u.kt * 64) * 2; };
  auto koffB = [&](const Cursor& u) -> int { return (u.sb + u.kt * 64) * 2; };
  // at a tile start: the stream's tile origin (and conv row offsets of its A half)
  auto enter = [&](Cursor& u, int (&vc)[2], int ha) {
    if (u.kt == 0) {
      int mm, nn;
      coords(u.ti, mm, nn);
      u.sa = mm * lda;
      u.sb = nn * ldb;
      if (CONV) conv_rows(vc, mm, ha);
    }
  };
  auto issueA = [&](int h, int buf, const Cursor& u, const int (&vc)[2]) {
    if (CONV) issue(h, buf, vc, koffA(u));
    else issue(h, buf, va, koffA(u) + (h == HA1 ? 64 * lda * 2 : 0));
  };
  auto issueB = [&](int h, int buf, const Cursor& u) { issue(h, buf, vb, koffB(u) + (h == HB1 ? 32 * ldb * 2 : 0)); };

  // bias: each wave's 64 columns n0 + wc*64 + 0..63 are brought into its own 256-B LDS slot (one 4-byte
  // LDS-DMA, one tile ahead) and seed the accumulators
  const bool has_bias = g.bias != nullptr;
  unsigned char* bslot = smem + LDS_BYTES + wid * 256;
  int pos_bias = 0;
  auto load_bias = [&](int n0) {
    if (has_bias) {
      const int n = n0 + wc * 64 + lane;
      __builtin_amdgcn_global_load_lds((gptr_t)(g.bias + n), (lptr_t)bslot, 4, 0, 0);
      vm += 1;
    }
    pos_bias = vm;
  };
  // the 4 bias values of block column j for this lane (columns j*16 + 4*fg .. +3); the caller has waited
  // for the slot's LDS-DMA (vm - pos_bias)
  auto bias_pair = [&](int jb, f32x4_t& v0, f32x4_t& v1) {
    if (has_bias) {
      const u32x4_t a = ds_read128(bslot + (jb * 16 + 4 * fg) * 4);
      const u32x4_t b = ds_read128(bslot + ((jb + 1) * 16 + 4 * fg) * 4);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      v0 = __builtin_bit_cast(f32x4_t, a);
      v1 = __builtin_bit_cast(f32x4_t, b);
      asm volatile("" : "+v"(v0), "+v"(v1));
    } else {
      v0 = f32x4_t{0.f, 0.f, 0.f, 0.f};
      v1 = v0;
    }
  };

  // stores: buffer stores, lane offset fixed, tile origin and block offset in soffset
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(g.C, 0, 0x7fffffff, SRD_W3);
  const __amdgpu_buffer_rsrc_t rc2 =
      __builtin_amdgcn_make_buffer_rsrc(EPI == EPI_GELU ? g.C2 : g.C, 0, 0x7fffffff, SRD_W3);
  constexpr int ESZ = (int)sizeof(OT);
  const int vst = ((wr * 128 + fr) * ldc + wc * 64 + 4 * fg) * ESZ;
  constexpr int SPQ = EPI == EPI_GELU ? 16 : 8;  // store instructions per quadrant

  u32x4_t af[4][2], b0[2][2], b1[2][2];
  f32x4_t acc[8][4];

  // quadrant q of the finished tile at (em0, en0): blocks i in 4*(q>>1).., j in 2*(q&1)..; then re-seed it
  auto epi_quadrant = [&](int q, int em0, int en0, bool reseed) {
    const int ib = (q >> 1) * 4, jb = (q & 1) * 2;
    f32x4_t bq[2];
    if (reseed) bias_pair(jb, bq[0], bq[1]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int so = ((em0 + (ib + i) * 16) * ldc + en0 + (jb + j) * 16) * ESZ;
        const int off = vst;
        f32x4_t v = acc[ib + i][jb + j];
        if constexpr (sizeof(OT) == 4) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), rc, off, so, 0);
        } else {
          if constexpr (EPI == EPI_GELU) {
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])}, rc, off, so, 0);
            const unsigned thr = g.thr16;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float a = gelu_f(v[e]);
              if (thr) {
                const unsigned m = (unsigned)(em0 + wr * 128 + (ib + i) * 16 + fr);
                const unsigned n = (unsigned)(en0 + wc * 64 + (jb + j) * 16 + 4 * fg + e);
                a = drop_keep(g.seed, g.stream, (uint64_t)m * (uint64_t)Nc + n, thr) ? a * g.drop_scale : 0.f;
              }
              v[e] = a;
            }
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])}, rc2, off, so, 0);
          } else {
            if constexpr (EPI == EPI_GELU_ONLY) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = gelu_f(v[e]);
            }
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])}, rc, off, so, 0);
          }
        }
        if (reseed) acc[ib + i][jb + j] = bq[j];
        __builtin_amdgcn_sched_barrier(0);  // one block at a time: bounds the epilogue's live registers
      }
    vm += SPQ;
  };

  // fragment addresses: swz_kc(base16 + i*16 + fr, s*4 + fg) = (base16 + i*16)*128 + swz_kc(fr, s*4 + fg) for a
  // 16-aligned base, so one lane address per k-half s plus immediate offsets (half image, row block)
  const unsigned lds0 = (unsigned)(size_t)(lptr_t)(void*)smem;
  const unsigned aadr[2] = {lds0 + wr * 8192 + swz_kc(fr, fg), lds0 + wr * 8192 + swz_kc(fr, 4 + fg)};
  const unsigned badr[2] = {lds0 + wc * 4096 + swz_kc(fr, fg), lds0 + wc * 4096 + swz_kc(fr, 4 + fg)};
  auto readA = [&](int buf, auto hc) {
    constexpr int h = decltype(hc)::value;
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
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[ib + i][jb + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(bf16x8_t, bf[j][s]), __builtin_bit_cast(bf16x8_t, af[i][s]), acc[ib + i][jb + j], 0, 0,
              0);
    __builtin_amdgcn_s_setprio(0);
    bar();
  };

  // ---------------------------------------------------------------- prologue
  int m0, n0;
  coords(0, m0, n0);
  load_bias(n0);
  Cursor c1{0, 0, 0, 0, 0, 0}, c2{0, 0, 0, 0, 0, 0};  // both at K-tile 0; c2 moves to K-tile 1 below
  enter(c1, vc1, HA1);
  enter(c2, vc2, HA0);
  int pos_A0, pos_A0_prev, pos_B0, pos_B1, pos_A1;
  issueA(HA0, 0, c2, vc2);
  issueB(HB0, 0, c2);
  const int pos_first = vm;
  issueB(HB1, 0, c1);
  pos_B1 = vm;
  issueA(HA1, 0, c1, vc1);
  pos_A1 = vm;
  pos_A0 = pos_B0 = pos_first;
  advance(c2);  // K-tile 1
  if (NT > 1) {
    enter(c2, vc2, HA0);
    issueA(HA0, 1, c2, vc2);
    pos_A0 = vm;
    issueB(HB0, 1, c2);
    pos_B0 = vm;
  }
  wait_vm(vm - pos_first);  // bias, A0(0), B0(0)
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
  // c1 -> K-tile T+1, c2 -> K-tile T+2 at the top of iteration T
  advance(c1);
  advance(c2);

  // ---------------------------------------------------------------- flattened K loop over all my tiles
  bool ep = false;  // the previous tile's results are still in acc (stored during this K-tile)
  int em0 = 0, en0 = 0;
  int kt = 0, ti = 0;
  for (int T = 0; T < NT; ++T) {
    const int bc = T & 1, bn = bc ^ 1;
    const bool last = kt == nk - 1;
    const bool more1 = T + 1 < NT, more2 = T + 2 < NT;
    int nm0 = 0, nn0 = 0;  // next tile of this workgroup (for its bias)
    if (last && more1) coords(ti + 1, nm0, nn0);
    // ---- phase 1: A rows 0..63 x B cols 0..31
    if (ep) {
      wait_vm(vm - pos_bias);  // this tile's bias slot (loaded during the previous K-tile)
      epi_quadrant(0, em0, en0, true);
    }
    readA(bc, IC<HA0>{});
    if (last && nk > 1 && more1) load_bias(nn0);
    {
      const int prev = pos_B1;  // B1(T), read in phase 2
      if (more1) {
        enter(c1, vc1, HA1);
        issueB(HB1, bn, c1);
        pos_B1 = vm;
      }
      wait_vm(vm - prev);
    }
    mma(0, 0, b0);
    // ---- phase 2: A rows 0..63 x B cols 32..63
    if (ep) epi_quadrant(1, em0, en0, true);
    readB(bc, IC<HB1>{}, b1);
    {
      const int prev = pos_A1;  // A1(T), read in phase 3
      if (more1) {
        issueA(HA1, bn, c1, vc1);
        pos_A1 = vm;
      }
      wait_vm(vm - prev);
    }
    mma(0, 2, b1);
    // ---- phase 3: A rows 64..127 x B cols 0..31
    if (ep) epi_quadrant(2, em0, en0, true);
    readA(bc, IC<HA1>{});
    pos_A0_prev = pos_A0;
    if (more2) {
      enter(c2, vc2, HA0);
      issueA(HA0, bc, c2, vc2);
      pos_A0 = vm;
    }
    if (more1) wait_vm(vm - pos_B0);  // B0(T+1), read in phase 4
    mma(4, 0, b0);
    // ---- phase 4: A rows 64..127 x B cols 32..63; B0 fragments of K-tile T+1
    if (ep) {
      epi_quadrant(3, em0, en0, true);
      ep = false;
    }
    if (more1) readB(bn, IC<HB0>{}, b0);
    if (last && nk == 1 && more1) load_bias(nn0);
    if (more2) {
      issueB(HB0, bc, c2);
      pos_B0 = vm;
    }
    if (more1) wait_vm(vm - pos_A0_prev);  // A0(T+1), read in phase 1 of T+1
    mma(4, 2, b1);
    // ---- advance
    advance(c1);
    advance(c2);
    if (last) {
      ep = true;
      em0 = m0;
      en0 = n0;
      m0 = nm0;
      n0 = nn0;
      kt = 0;
      ++ti;
    } else {
      ++kt;
    }
  }
  if (wr == 0) bar();
  // the last tile
#pragma unroll
  for (int q = 0; q < 4; ++q) epi_quadrant(q, em0, en0, false);
}

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
  const long grid = tiles < ncu ? tiles : ncu;
#endif
  hipLaunchKernelGGL((gemm256_kernel<EPI, OT, CONV>), dim3((unsigned)grid), dim3(512), LDS_BYTES + 2048, s, g);
  return (int)hipGetLastError();
}

}  // namespace g256

long gemm256_tiles(long M, long N) { return ((M + 255) / 256) * ((N + 255) / 256); }

bool gemm256_ok(const GemmArgs& g, int epi, int out_dtype, bool conv) {
  if (g.K % 64 || g.K <= 0 || g.M <= 0 || g.N <= 0 || g.N % 8 || g.lda % 8 || g.ldb % 8 || g.ldc % 8) return false;
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
  if (conv && (g.geo.cpad != 0 || g.geo.Cg % 64)) return false;
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
