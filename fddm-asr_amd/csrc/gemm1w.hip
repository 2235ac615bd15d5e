// 256x256 bf16 NT GEMM with ONE wave per SIMD (round-4 experiment): C[m][n] = sum_k A(m,k) B(n,k) + bias[n].
//
// gemm256 runs 8 waves (2 per SIMD) of 128x64 outputs: its per-wave tile reads 24 KB of LDS fragments per 64-K
// step for 64 MFMAs, so LDS bandwidth ~ MFMA time, and its 128 accumulators per lane leave no room to hold a tile's
// results while the next tile computes (the epilogue is ~21 % of a K = 768 tile). Here a workgroup is 4 waves, one
// per SIMD, each owning a 128x128 output block = 4 x 4 blocks of v_mfma_f32_32x32x16_bf16 (256 f32 accumulators in
// AGPRs): 32 KB of fragment reads per 64-K step for 64 MFMAs of twice the work, i.e. LDS at half the MFMA time.
// Operands arrive by LDS-DMA into a 2-stage ring (one 64-K step = A [256][128 B] + B [256][128 B] per stage, KC
// swizzle); a wave software-pipelines its own fragment reads one 16-K step ahead of its MFMAs and issues its share
// of the next stage's DMA between them; one barrier per 64-K step.
// C^T blocks are computed (operands swapped) so that a lane owns one output row and 4 x 4 consecutive columns.
#include "gemm.h"

namespace fddm {
namespace g1w {

typedef __attribute__((address_space(3))) void* lptr_t;
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
constexpr unsigned SRD_W3 = 0x00020000u;
constexpr int BM = 256, BN = 256, IMG = 256 * 128, STAGE = 2 * IMG, GM = 4;

__device__ __forceinline__ u32x4_t ds_read128(unsigned a) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

template <bool BIAS, int EARLY>
__global__ void __launch_bounds__(256, 1) gemm1w_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int r32 = lane & 31, h = lane >> 5;

  // persistent schedule (gemm256's): each XCD owns a contiguous range of a grouped tile order
  const int nN = (int)((g.N + BN - 1) / BN), nM = (int)((g.M + BM - 1) / BM), tiles = nN * nM;
  const int G = gridDim.x, wg = blockIdx.x, x = wg & 7, jx = wg >> 3;
  int Wx = 0;
  for (int y = 0; y < x; ++y) Wx += (G - 1 - y) / 8 + 1;
  const int Px = (G - 1 - x) / 8 + 1;
  const int s0 = (int)((long)tiles * Wx / G), s1 = (int)((long)tiles * (Wx + Px) / G);
  const int nmine = (s1 - s0 > jx) ? (s1 - s0 - jx + Px - 1) / Px : 0;
  auto coords = [&](int i, int& m0, int& n0) {
    const int s = s0 + jx + i * Px;
    const int per = GM * nN, grp = s / per, first = grp * GM, gsz = min(GM, nM - first), rr = s - grp * per;
    m0 = min((first + rr % gsz) * BM, (int)g.M - BM);
    n0 = min((rr / gsz) * BN, (int)g.N - BN);
  };

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, 0x7fffffff, SRD_W3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, 0x7fffffff, SRD_W3);
  const int lda = (int)g.lda, ldb = (int)g.ldb, ldc = (int)g.ldc;
  // DMA: wave w fills rows 64w .. 64w+63 of the A and of the B image (8 pieces of 8 rows each); lane -> row
  // base + lane/8, physical chunk lane%8 holding logical chunk (lane%8) ^ ((row>>1)&7)
  int voffA[8], voffB[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int row = 64 * wid + 8 * p + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    voffA[p] = (row * lda + c * 8) * 2;
    voffB[p] = (row * ldb + c * 8) * 2;
  }
  const unsigned lbase = (unsigned)(size_t)(lptr_t)(void*)smem;
  auto dma = [&](int p, int st, int m0, int n0, int kt) {  // piece p (0..15) of this wave for K-step kt
    if (p < 8) {
      lptr_t d = (lptr_t)(smem + st * STAGE + (64 * wid + 8 * p) * 128);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, d, 16, voffA[p], (m0 * lda + kt * 64) * 2, 0, 0);
    } else {
      lptr_t d = (lptr_t)(smem + st * STAGE + IMG + (64 * wid + 8 * (p - 8)) * 128);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, d, 16, voffB[p - 8], (n0 * ldb + kt * 64) * 2, 0, 0);
    }
  };
  // fragment addresses: A block bi rows wr*128 + 32 bi + r32, B block bj rows wc*128 + 32 bj + r32; 16-K step s reads
  // logical chunk 2s + h
  auto frag_addr = [&](int img, int row, int s) -> unsigned {
    return lbase + img + row * 128 + (((2 * s + h) ^ ((row >> 1) & 7)) << 4);
  };

  const int nk = (int)(g.K / 64);
  const bf16_t* Cb = (const bf16_t*)g.C;
  for (int it = 0; it < nmine; ++it) {
    int m0, n0;
    coords(it, m0, n0);
    // accumulators start at the bias (C^T register 4q + e is column 8q + 4h + e of its 32-column block)
    f32x16_t acc[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x16_t b0{};
      if constexpr (BIAS) {
        const float* bp = g.bias + n0 + wc * 128 + 32 * j + 4 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 bb = *(const float4*)(bp + 8 * q);
          b0[4 * q] = bb.x;
          b0[4 * q + 1] = bb.y;
          b0[4 * q + 2] = bb.z;
          b0[4 * q + 3] = bb.w;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = b0;
    }
    // prologue: K-step 0 into stage 0
#pragma unroll
    for (int p = 0; p < 16; ++p) dma(p, 0, m0, n0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
      const int st = kt & 1;
      const bool more = kt + 1 < nk;
      u32x4_t fa[2][4], fb[2][4];
      auto rd = [&](int buf, int s) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          fa[buf][b] = ds_read128(frag_addr(st * STAGE, wr * 128 + 32 * b + r32, s));
          fb[buf][b] = ds_read128(frag_addr(st * STAGE + IMG, wc * 128 + 32 * b + r32, s));
        }
      };
      if constexpr (EARLY) {  // the whole next K-step's DMA right after the barrier: ~2048 MFMA cycles to land
        if (more) {
#pragma unroll
          for (int p = 0; p < 16; ++p) dma(p, st ^ 1, m0, n0, kt + 1);
        }
      }
      rd(0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int cur = s & 1;
        if (s < 3) {
          rd(cur ^ 1, s + 1);
          asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          asm volatile("" : "+v"(fa[cur][b]), "+v"(fb[cur][b]));
        }
        // next K-step's DMA, 4 pieces per 16-K step, between the MFMA blocks
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (!EARLY && more) dma(4 * s + i, st ^ 1, m0, n0, kt + 1);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[cur][j]),
                                                                 __builtin_bit_cast(bf16x8_t, fa[cur][i]), acc[i][j],
                                                                 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    // epilogue: acc[i][j] = C^T block (n = wc*128 + 32 j + 8 q + 4 h + e, m = wr*128 + 32 i + r32) at register 4q + e
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wc * 128 + 32 * j;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wr * 128 + 32 * i + r32;
        float v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = acc[i][j][e];
        // lane (r32, h) holds columns 8q + 4h .. +3 for q = 0..3: trade with lane ^ 32 so that each lane gets 8
        // consecutive columns of two q's: h = 0 keeps q = 0, 2 and receives their upper halves; h = 1 keeps q = 1, 3
        unsigned pk4[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pk4[q][0] = pk_bf16(v[4 * q], v[4 * q + 1]);
          pk4[q][1] = pk_bf16(v[4 * q + 2], v[4 * q + 3]);
        }
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
          // h = 0 sends q = 2qq+1's lower... exchange: lane h=0 gives (q=2qq+1, its 4 cols), gets (q=2qq, cols 4..7)
          const unsigned s0_ = h ? pk4[2 * qq][0] : pk4[2 * qq + 1][0];
          const unsigned s1_ = h ? pk4[2 * qq][1] : pk4[2 * qq + 1][1];
          const auto x0 = __builtin_amdgcn_permlane32_swap(s0_, s0_, false, false);
          const auto x1 = __builtin_amdgcn_permlane32_swap(s1_, s1_, false, false);
          // after the swap lane l holds the partner's value in x[0] (h = 1) / x[1] (h = 0)
          const unsigned r0 = h ? x0[0] : x0[1], r1 = h ? x1[0] : x1[1];
          uint4 out;
          int col;
          if (!h) {  // q = 2qq: own cols 8q..8q+3, partner's 8q+4..+7
            out = make_uint4(pk4[2 * qq][0], pk4[2 * qq][1], r0, r1);
            col = nb + 16 * qq;
          } else {   // q = 2qq+1: partner's 8q..8q+3, own 8q+4..+7
            out = make_uint4(r0, r1, pk4[2 * qq + 1][0], pk4[2 * qq + 1][1]);
            col = nb + 16 * qq + 8;
          }
          *(uint4*)((bf16_t*)Cb + (long)m * ldc + col) = out;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}


// Variant 2: one flat stream of (tile, K-step) steps per workgroup. The DMA runs two steps ahead across tile
// boundaries (the next tile's first K-steps land while this tile's epilogue runs), and the last 16-K MFMA group of a
// step is issued after the barrier that opens the next step, so the next step's first fragment reads overlap MFMAs
// instead of an idle pipe. Bias: loaded into registers at a tile's first K-step, added in the epilogue.
template <bool BIAS, bool NODMA = false>
__global__ void __launch_bounds__(256, 1) gemm1w_flat_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int r32 = lane & 31, h = lane >> 5;

  const int nN = (int)((g.N + BN - 1) / BN), nM = (int)((g.M + BM - 1) / BM), tiles = nN * nM;
  const int G = gridDim.x, wg = blockIdx.x, x = wg & 7, jx = wg >> 3;
  int Wx = 0;
  for (int y = 0; y < x; ++y) Wx += (G - 1 - y) / 8 + 1;
  const int Px = (G - 1 - x) / 8 + 1;
  const int s0 = (int)((long)tiles * Wx / G), s1 = (int)((long)tiles * (Wx + Px) / G);
  const int nmine = (s1 - s0 > jx) ? (s1 - s0 - jx + Px - 1) / Px : 0;
  if (nmine == 0) return;
  auto coords = [&](int i, int& m0, int& n0) {
    const int s = s0 + jx + i * Px;
    const int per = GM * nN, grp = s / per, first = grp * GM, gsz = min(GM, nM - first), rr = s - grp * per;
    m0 = min((first + rr % gsz) * BM, (int)g.M - BM);
    n0 = min((rr / gsz) * BN, (int)g.N - BN);
  };

  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, 0x7fffffff, SRD_W3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, 0x7fffffff, SRD_W3);
  const int lda = (int)g.lda, ldb = (int)g.ldb, ldc = (int)g.ldc;
  int voffA[8], voffB[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int row = 64 * wid + 8 * p + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    voffA[p] = (row * lda + c * 8) * 2;
    voffB[p] = (row * ldb + c * 8) * 2;
  }
  const unsigned lbase = (unsigned)(size_t)(lptr_t)(void*)smem;
  const __amdgpu_buffer_rsrc_t rBias = __builtin_amdgcn_make_buffer_rsrc((void*)g.bias, 0, 0x7fffffff, SRD_W3);
  const int nk = (int)(g.K / 64), total = nmine * nk;
  // prefetch cursor: the (tile, K-step) whose operands the next DMA issue loads
  int pt = 0, pk = 0, pm0, pn0;
  coords(0, pm0, pn0);
  auto pf_issue = [&](int st) {
    const int soA = (pm0 * lda + pk * 64) * 2, soB = (pn0 * ldb + pk * 64) * 2;
#pragma unroll
    for (int p = 0; p < 8; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lptr_t)(smem + st * STAGE + (64 * wid + 8 * p) * 128), 16,
                                               voffA[p], soA, 0, 0);
#pragma unroll
    for (int p = 0; p < 8; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lptr_t)(smem + st * STAGE + IMG + (64 * wid + 8 * p) * 128), 16,
                                               voffB[p], soB, 0, 0);
    if (++pk == nk) {
      pk = 0;
      if (++pt < nmine) coords(pt, pm0, pn0);
    }
  };
  auto frag_addr = [&](int img, int row, int s) -> unsigned {
    return lbase + img + row * 128 + (((2 * s + h) ^ ((row >> 1) & 7)) << 4);
  };
  u32x4_t fa[2][4], fb[2][4];
  auto rd = [&](int buf, int st, int s) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      fa[buf][b] = ds_read128(frag_addr(st * STAGE, wr * 128 + 32 * b + r32, s));
      fb[buf][b] = ds_read128(frag_addr(st * STAGE + IMG, wc * 128 + 32 * b + r32, s));
    }
  };
  auto mfma_group = [&](f32x16_t (&acc)[4][4], int buf) {
#pragma unroll
    for (int b = 0; b < 4; ++b) asm volatile("" : "+v"(fa[buf][b]), "+v"(fb[buf][b]));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, fb[buf][j]),
                                                             __builtin_bit_cast(bf16x8_t, fa[buf][i]), acc[i][j], 0, 0,
                                                             0);
  };

  pf_issue(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (total > 1) pf_issue(1);
  rd(0, 0, 0);
  const bf16_t* Cb = (const bf16_t*)g.C;
  int gs = 0;
  for (int tile = 0; tile < nmine; ++tile) {
    int m0, n0;
    coords(tile, m0, n0);
    // the tile's 256 bias values: one LDS-DMA per wave into its own 1 KB slot (two slots by tile parity); the
    // K-loop's vmcnt(0) lands it, the epilogue reads it
    unsigned char* bslot = smem + 2 * STAGE + ((tile & 1) * 4 + wid) * 1024;
    if constexpr (BIAS) __builtin_amdgcn_raw_ptr_buffer_load_lds(rBias, (lptr_t)bslot, 16, lane * 16, n0 * 4, 0, 0);
    f32x16_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x16_t{};
    for (int kt = 0; kt < nk; ++kt, ++gs) {
      const int st = gs & 1;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        rd((s + 1) & 1, st, s + 1);
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        mfma_group(acc, s & 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (gs + 1 < total) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (!NODMA && gs + 2 < total) pf_issue(st);
        rd(0, st ^ 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_group(acc, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue (see gemm1w_kernel): C^T register 4q + e = column 8q + 4h + e of block j, row 32 i + r32
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wc * 128 + 32 * j;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wr * 128 + 32 * i + r32;
        float v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = acc[i][j][e];
        if constexpr (BIAS) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 bb = *(const float4*)(bslot + (wc * 128 + 32 * j + 8 * q + 4 * h) * 4);
            v[4 * q] += bb.x;
            v[4 * q + 1] += bb.y;
            v[4 * q + 2] += bb.z;
            v[4 * q + 3] += bb.w;
          }
        }
        unsigned pk4[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pk4[q][0] = pk_bf16(v[4 * q], v[4 * q + 1]);
          pk4[q][1] = pk_bf16(v[4 * q + 2], v[4 * q + 3]);
        }
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
          const unsigned x0s = h ? pk4[2 * qq][0] : pk4[2 * qq + 1][0];
          const unsigned x1s = h ? pk4[2 * qq][1] : pk4[2 * qq + 1][1];
          const auto x0 = __builtin_amdgcn_permlane32_swap(x0s, x0s, false, false);
          const auto x1 = __builtin_amdgcn_permlane32_swap(x1s, x1s, false, false);
          const unsigned r0 = h ? x0[0] : x0[1], r1 = h ? x1[0] : x1[1];
          const uint4 out = h ? make_uint4(r0, r1, pk4[2 * qq + 1][0], pk4[2 * qq + 1][1])
                              : make_uint4(pk4[2 * qq][0], pk4[2 * qq][1], r0, r1);
          *(uint4*)((bf16_t*)Cb + (long)m * ldc + nb + 16 * qq + 8 * h) = out;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

}  // namespace g1w
}  // namespace fddm

using namespace fddm;

// Probe entry (round-4 experiment, tools/g1w_bench.py): bf16 A [M][lda], B [N][ldb] (K-contiguous), bf16 C [M][ldc],
// optional f32 bias [N]; M, N >= 256 (the edge tiles overlap their neighbours), K % 64 == 0.
FDDM_API int fddm_gemm1w_probe(const void* A, long lda, const void* B, long ldb, void* C, long ldc, const float* bias,
                               long M, long N, long K, int ncu, int variant, void* hs) {
  if (M < 256 || N < 256 || K % 64 || lda % 8 || ldb % 8 || ldc % 8) return (int)hipErrorInvalidValue;
  GemmArgs g{};
  g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.C = C; g.ldc = ldc; g.bias = bias; g.M = M; g.N = N; g.K = K;
  const size_t lds = 2 * g1w::STAGE;
  const int grid = ncu > 0 ? ncu : 256;
#define G1W_LAUNCH(E)                                                                                        \
  if (bias) hipLaunchKernelGGL((g1w::gemm1w_kernel<true, E>), dim3(grid), dim3(256), lds, (hipStream_t)hs, g); \
  else hipLaunchKernelGGL((g1w::gemm1w_kernel<false, E>), dim3(grid), dim3(256), lds, (hipStream_t)hs, g);
  if (variant == 3) {  // timing probe only: the K-loop without its DMA (wrong results)
    hipLaunchKernelGGL((g1w::gemm1w_flat_kernel<false, true>), dim3(grid), dim3(256), lds, (hipStream_t)hs, g);
  } else if (variant == 2) {
    if (bias)
      hipLaunchKernelGGL(g1w::gemm1w_flat_kernel<true>, dim3(grid), dim3(256), lds + 8192, (hipStream_t)hs, g);
    else hipLaunchKernelGGL(g1w::gemm1w_flat_kernel<false>, dim3(grid), dim3(256), lds, (hipStream_t)hs, g);
  } else if (variant == 1) {
    G1W_LAUNCH(1)
  } else {
    G1W_LAUNCH(0)
  }
#undef G1W_LAUNCH
  return (int)hipGetLastError();
}
