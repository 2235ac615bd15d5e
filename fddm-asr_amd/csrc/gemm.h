// Shared declarations of the MFMA GEMM kernels (gemm.hip: 128x128 general kernel; gemm256.hip: 256x256
// 8-phase kernel for the large NT shapes).
#pragma once
#include "common.h"

namespace fddm {

// EPI_ROPE_ACC (gemm128, A KC + B MC, f32 out): C += rope_bwd(A B) with the decoder's RoPE pairing (column j with
// j + N/2, written to columns 2j, 2j+1; misc.hip rope_bwd_kernel), rope tables rcs / rsn [rL][N]
enum { EPI_STORE = 0, EPI_GELU = 1, EPI_ACC_F32 = 2, EPI_GELU_ONLY = 3, EPI_DGELU = 4, EPI_ROPE_ACC = 5 };

// implicit-conv addressing of a KC A operand: A(m,k) = A + (m/Mi)*sAb + (t*cstride - cpad + k/Cg)*lda + k%Cg,
// t = m%Mi, zero outside 0 <= time < Tin (WavLM conv feature extractor and grouped positional conv)
struct ConvGeo { long Cg, cstride, cpad, Tin; };

struct GemmArgs {
  const void* A; long lda, Mi, sAb;
  const void* B; long ldb;
  void* C; long ldc; void* C2;
  const float* bias; float alpha;
  long M, N, K;
  uint64_t seed, stream; unsigned thr16; float drop_scale;
  ConvGeo geo;
  long sAz, sBz, sCz, sbiasz;  // per-blockIdx.z offsets (grouped conv)
  long ksplit;                 // K elements per split-K slice (plain GEMM)
  float* colsum;               // optional: colsum[m] += sum_k A(m,k) (MC A operand) — fused bias gradient
  const uint64_t* seed_off;    // graph-replay seed offset (common.h eff_seed) or null
  const float* rcs = nullptr;  // EPI_ROPE_ACC: cos / sin tables [rL][N] (row m uses position m % rL)
  const float* rsn = nullptr;
  long rL = 0;
};

// KC LDS image: 16-B chunk c of 128-B row r at r*128 + ((c ^ ((r>>1)&7))<<4) — conflict-free ds_read_b128 of
// MFMA fragments (16 rows x one chunk per lane group)
__device__ __forceinline__ int swz_kc(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

// 256x256 8-phase bf16 NT GEMM (gemm256.hip). Preconditions: bf16 A/B, both K-contiguous, K % 64 == 0,
// 16-B aligned rows, N % 8 == 0, conv without padding taps and Cg % 64 == 0. epi: STORE, GELU, GELU_ONLY;
// out_dtype: FDDM_BF16 or FDDM_F32 (STORE only). Returns hipError_t.
int gemm256_launch(const GemmArgs& g, int epi, int out_dtype, bool conv, hipStream_t s);
bool gemm256_ok(const GemmArgs& g, int epi, int out_dtype, bool conv);
long gemm256_tiles(long M, long N);

// 128x128 LDS-DMA ring GEMM (gemm128.hip) for outputs with too few 256x256 tiles. Layouts: A KC + B KC (STORE
// bf16/f32, GELU, GELU_ONLY, DGELU, ACC_F32), A KC + B MC (STORE bf16/f32, DGELU, ACC_F32), A MC + B MC (ACC_F32, with
// colsum). nz > 1: split-K slices of g.ksplit (ACC_F32 only, f32 atomics).
bool gemm128_ok(const GemmArgs& g, bool akc, bool bkc, int epi, int out_dtype);
int gemm128_launch(const GemmArgs& g, bool akc, bool bkc, int epi, int out_dtype, int nz, hipStream_t s);
long gemm128_tiles(long M, long N);
constexpr int G128_GROUP_MAX = 12;
struct G128Group {
  int np;
  int start[G128_GROUP_MAX + 1];
  int tn[G128_GROUP_MAX], tm[G128_GROUP_MAX], nz[G128_GROUP_MAX];
  GemmArgs g[G128_GROUP_MAX];
};
// A MC + B MC, ACC_F32 (weight gradients): `total` workgroups over the problems of ga
int gemm128_grouped_dw(const G128Group& ga, int total, hipStream_t s);

}  // namespace fddm
