// WavLM positional convolution embedding on gfx950:
//   pos[b][t][g*Cg + n] = GELU( bias[g*Cg + n] + sum_{tap < kp} sum_{c < Cg} x[b][t + tap - kp/2][g*Cg + c] * W[g][n][tap*Cg + c] )
// for t < S (HF modeling_wavlm.py:37-90: Conv1d(E, E, kp, padding=kp/2, groups=G) + SamePad (drop the last
// frame) + GELU). x, W, pos: bf16, channels-last; bias f32.
//
// A grouped conv with N = Cg = 48 output channels per group and K = kp*Cg = 6144 is a poor fit for 128/256-wide
// GEMM tiles. Here one workgroup owns (b, g, 256 consecutive frames): the whole input window those frames
// touch — 256 + kp - 1 frames x Cg channels, 37 KB — is loaded into LDS once, laid out [frame][Cg] so that the
// implicit-GEMM row of frame t is the contiguous run window[(t - t0)*Cg ...] (tap-major K = tap*Cg + c); only
// the weights W[g] (Cg x 6144) stream through a double-buffered LDS-DMA ring, 128 K per step. 4 waves x 64
// frames; MFMA 16x16x32 with operands swapped so each lane owns 4 consecutive channels of one frame.
#include "common.h"

namespace fddm {
namespace posconv {

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

constexpr int TR = 256;   // frames per workgroup
constexpr int KS = 128;   // K per weight stage
constexpr int MAXNB = 4;  // Cg <= 64

// LDS read as inline asm: a compiler-visible read would wait for every outstanding LDS-DMA (vmcnt(0))
__device__ __forceinline__ u32x4_t lds_read128(unsigned a) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

struct Args {
  const bf16_t* x; const bf16_t* W; const float* bias; bf16_t* out;
  int S, E, kp, nwin;  // nwin = TR + kp - 1 window frames
};

template <int NB>
__global__ void __launch_bounds__(256, 2) posconv_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int Cg = NB * 16;
  constexpr int WST = Cg * KS * 2;  // bytes per weight stage: Cg rows x 256 B
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int t0 = blockIdx.x * TR, g = blockIdx.y, b = blockIdx.z;
  const int half = a.kp / 2, K = a.kp * Cg, nks = K / KS;
  unsigned char* wst = smem;            // 2 weight stages
  unsigned char* win = smem + 2 * WST;  // window [nwin][Cg] bf16
  const bf16_t* Wg = a.W + (long)g * Cg * K;

  // weight stage: wave instruction r (NB per wave) fills rows 4r..4r+3 (256 B each); the lane at physical
  // 16-B chunk p of row n brings logical chunk p ^ (n & 15) (conflict-free B fragment reads)
  auto issue = [&](int ks, int buf) {
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int r = w * NB + u, n = r * 4 + (lane >> 4), p = lane & 15;
      const bf16_t* src = Wg + (long)n * K + ks * KS + ((p ^ (n & 15)) * 8);
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(wst + buf * WST + r * 1024), 16, 0, 0);
    }
  };
  issue(0, 0);

  // input window: frames t0 - half .. t0 - half + nwin - 1 (zero outside [0, S)), Cg channels each
  {
    constexpr int cpf = Cg / 8;  // 16-B chunks per frame
    const int nch = a.nwin * cpf;
    const bf16_t* xb = a.x + (long)b * a.S * a.E + g * Cg;
    for (int c = tid; c < nch; c += 256) {
      const int f = c / cpf, q = c - f * cpf, t = t0 - half + f;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (t >= 0 && t < a.S) v = *(const uint4*)(xb + (long)t * a.E + q * 8);
      *(uint4*)(win + (f * Cg + q * 8) * 2) = v;
    }
  }

  f32x4_t acc[4][NB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const unsigned wbase = (unsigned)(size_t)(lptr_t)(void*)wst;
  const unsigned xbase = (unsigned)(size_t)(lptr_t)(void*)win + ((w * 64 + fr) * Cg + 8 * fg) * 2;
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage ks
    __syncthreads();                                   // everyone's (and the window); stage ks-1 retired
    if (ks + 1 < nks) issue(ks + 1, buf ^ 1);
#pragma unroll
    for (int s = 0; s < KS / 32; ++s) {
      u32x4_t af[4], bfr[NB];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_read128(xbase + (i * 16 * Cg + ks * KS + s * 32) * 2);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int n = j * 16 + fr, c = s * 4 + fg;
        bfr[j] = lds_read128(wbase + buf * WST + n * 256 + ((c ^ (n & 15)) << 4));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, bfr[j]),
                                                              __builtin_bit_cast(bf16x8_t, af[i]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // epilogue: acc[i][j][e] = pre-activation of frame t0 + w*64 + i*16 + fr, channel j*16 + 4*fg + e
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int n = g * Cg + j * 16 + 4 * fg;
    const float4 bv = *(const float4*)(a.bias + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + w * 64 + i * 16 + fr;
      if (t < a.S) {
        const f32x4_t v = acc[i][j];
        uint2 u;
        u.x = pk_bf16(gelu_f(v[0] + bv.x), gelu_f(v[1] + bv.y));
        u.y = pk_bf16(gelu_f(v[2] + bv.z), gelu_f(v[3] + bv.w));
        *(uint2*)(a.out + ((long)b * a.S + t) * a.E + n) = u;
      }
    }
  }
}

}  // namespace posconv
}  // namespace fddm

using namespace fddm;

// x [B][S][E] bf16, W [G][Cg][kp*Cg] bf16 (tap-major K), bias [E] f32, out [B][S][E] bf16.
FDDM_API int fddm_posconv_gelu(const void* x, const void* W, const float* bias, void* out, long B, long S, long E,
                               int G, int kp, void* hip_stream) {
  if (B <= 0 || S <= 0) return 0;
  if (G <= 0 || E % G || E % 8) return (int)hipErrorInvalidValue;
  const int Cg = (int)(E / G);
  if (Cg % 16 || Cg / 16 > posconv::MAXNB || kp <= 0 || kp % 2 || (kp * Cg) % posconv::KS)
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)x) | ((uintptr_t)W) | ((uintptr_t)out) | ((uintptr_t)bias)) & 15) return (int)hipErrorInvalidValue;
  posconv::Args a{(const bf16_t*)x, (const bf16_t*)W, bias, (bf16_t*)out, (int)S, (int)E, kp, posconv::TR + kp - 1};
  const size_t lds = 2 * (size_t)Cg * posconv::KS * 2 + (size_t)a.nwin * Cg * 2;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((S + posconv::TR - 1) / posconv::TR), (unsigned)G, (unsigned)B);
  hipStream_t s = (hipStream_t)hip_stream;
  switch (Cg / 16) {
    case 1: hipLaunchKernelGGL(posconv::posconv_kernel<1>, grid, dim3(256), lds, s, a); break;
    case 2: hipLaunchKernelGGL(posconv::posconv_kernel<2>, grid, dim3(256), lds, s, a); break;
    case 3: hipLaunchKernelGGL(posconv::posconv_kernel<3>, grid, dim3(256), lds, s, a); break;
    default: hipLaunchKernelGGL(posconv::posconv_kernel<4>, grid, dim3(256), lds, s, a); break;
  }
  return (int)hipGetLastError();
}
