// WavLM-specific kernels (forward only; the encoder is frozen):
//  * conv layer 0 + GroupNorm(C groups) + exact GELU (HF modeling_wavlm.py:723-744, "group" norm):
//      y[b][t][c] = sum_k w[c][k] * x[b][5t + k]     (1 -> 512 channels, k = 10, stride 5, no bias)
//    two launches: per-(b,c) statistics over the whole utterance (fp64 accumulation), then a
//    recompute + normalise + GELU pass that writes the channels-last activation once (bf16/f32).
//    The conv itself is ~10 MACs per output, so recomputing it is cheaper than re-reading y.
//  * gated relative-position gate (HF modeling_wavlm.py:166-180):
//      (a, b) = sigmoid(sum4(Linear_64->8(x[b,s,h*64:(h+1)*64])));  gate = a*(b*const[h] - 1) + 2
#include "common.h"

namespace fddm {

constexpr int C0_FRAMES = 64;         // frames per apply block
constexpr int C0_MAXK = 16;

// GroupNorm statistics without materialising y: per utterance the K sums S1[k] = sum_t x[S t + k] and
// the K x K Gram G[k][k'] = sum_t x[S t + k] x[S t + k'] (fp64) give, per channel c,
//   sum_t y = w_c . S1      sum_t y^2 = w_c^T G w_c.
// Each block of C0_GRAM_FRAMES frames stores its partial [S1 (K), upper triangle of G (K(K+1)/2)] with plain stores
// (ws: [B][nb][NQ]); the affine kernel sums the nb partials of its utterance in a fixed order (deterministic, and
// no zero-fill: the double atomics of 8 blocks per utterance made the statistics ~33 us).
constexpr int C0_GRAM_FRAMES = 4096;  // 1024 per block measured slower (50 vs 29 us)
template <int K> constexpr int c0_nq() { return K + K * (K + 1) / 2; }
template <int K>
__global__ void __launch_bounds__(256) conv0_gram_kernel(const float* __restrict__ x, double* __restrict__ part,
                                                         long nsamp, long T0, int S) {
  constexpr int NQ = c0_nq<K>();
  const long b = blockIdx.y;
  const long f0 = (long)blockIdx.x * C0_GRAM_FRAMES;
  const long f1 = min(T0, f0 + C0_GRAM_FRAMES);
  double s1[K], g[K * (K + 1) / 2];
#pragma unroll
  for (int k = 0; k < K; ++k) s1[k] = 0.0;
#pragma unroll
  for (int k = 0; k < K * (K + 1) / 2; ++k) g[k] = 0.0;
#pragma unroll 4
  for (long f = f0 + threadIdx.x; f < f1; f += 256) {
    float xv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) xv[k] = x[b * nsamp + f * S + k];
    int q = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      s1[k] += (double)xv[k];
#pragma unroll
      for (int j = k; j < K; ++j) g[q++] += (double)xv[k] * (double)xv[j];
    }
  }
  __shared__ double red[NQ][4];
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    double v = q < K ? s1[q] : g[q - K];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[q][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < NQ) {
    const int q = threadIdx.x;
    part[(b * gridDim.x + blockIdx.x) * NQ + q] = (red[q][0] + red[q][1]) + (red[q][2] + red[q][3]);
  }
}

// per (b, c): mean/var from (S1, G) -> fused GroupNorm affine  sc = gamma*rstd, sh = beta - mean*sc; one block
// per utterance sums its nb partials once into LDS
template <int K>
__global__ void __launch_bounds__(512) conv0_gn_affine_kernel(const double* __restrict__ part, int nb,
                                                              const float* __restrict__ w, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float* __restrict__ scsh,
                                                              long T0, int C, float eps) {
  constexpr int NQ = c0_nq<K>();
  __shared__ double tot[NQ];
  const long b = blockIdx.x;
  if (threadIdx.x < NQ) {
    double t = 0.0;
    for (int i = 0; i < nb; ++i) t += part[(b * nb + i) * NQ + threadIdx.x];
    tot[threadIdx.x] = t;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double wk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k] = (double)w[c * K + k];
    double m = 0.0, q = 0.0;
    int i = K;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      m += wk[k] * tot[k];
      q += wk[k] * wk[k] * tot[i++];
#pragma unroll
      for (int j = k + 1; j < K; ++j) q += 2.0 * wk[k] * wk[j] * tot[i++];
    }
    m /= (double)T0;
    const double var = fmax(q / (double)T0 - m * m, 0.0);
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = rstd * gamma[c];
    scsh[2 * (b * C + c)] = sc;
    scsh[2 * (b * C + c) + 1] = beta[c] - (float)m * sc;
  }
}

// recompute y, normalise, GELU; thread owns channel pair (2c, 2c+1) -> 4-B stores, 1 KB per wave row.
// VALU-bound (10 FMAs + affine + GELU per output): the channel pair is carried as a float2 so the
// FMAs, the affine and the GELU polynomial issue as packed v_pk_* f32 instructions.
typedef float f2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2_t gelu2(f2_t x) {  // gelu_f (common.h) on a channel pair
  const f2_t ax = {fabsf(x.x), fabsf(x.y)};
  const f2_t den = ax * 0.23164189f + 1.0f;
  const f2_t t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f2_t p = t * 0.5307027145f - 0.7265760135f;
  p = p * t + 0.7107068705f;
  p = p * t - 0.142248368f;
  p = p * t + 0.127414796f;
  const f2_t u = ax * (ax * -0.72134752044f);
  const f2_t e = {__builtin_amdgcn_exp2f(u.x), __builtin_amdgcn_exp2f(u.y)};
  const f2_t r = p * t * e;
  const f2_t mx = {fmaxf(x.x, 0.f), fmaxf(x.y, 0.f)};
  return mx - ax * r;
}

template <typename OT, int K>
__global__ void __launch_bounds__(256) conv0_apply_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ scsh, OT* __restrict__ out, long nsamp,
                                                          long T0, int C, int S) {
  extern __shared__ float xs[];
  const long b = blockIdx.y;
  const long t0 = (long)blockIdx.x * C0_FRAMES;
  const int nf = (int)min((long)C0_FRAMES, T0 - t0);
  const int span = (nf - 1) * S + K;
  for (int i = threadIdx.x; i < span; i += 256) xs[i] = x[b * nsamp + t0 * S + i];
  __syncthreads();
  for (int c = 2 * threadIdx.x; c < C; c += 512) {
    f2_t wk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) wk[k] = f2_t{w[c * K + k], w[(c + 1) * K + k]};
    const f2_t sc = {scsh[2 * (b * C + c)], scsh[2 * (b * C + c + 1)]};
    const f2_t sh = {scsh[2 * (b * C + c) + 1], scsh[2 * (b * C + c + 1) + 1]};
    OT* o = out + (b * T0 + t0) * C + c;
    for (int f = 0; f < nf; ++f) {
      f2_t y = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k < K; ++k) y += wk[k] * xs[f * S + k];
      f2_t gv;
      if constexpr (sizeof(OT) == 2) {  // bf16 output: the bf16-output GELU (common.h)
        const f2_t z = y * sc + sh;
        gv = f2_t{gelu_bf16out(z.x), gelu_bf16out(z.y)};
      } else {
        gv = gelu2(y * sc + sh);
      }
      if constexpr (sizeof(OT) == 2) {
        *(unsigned*)(o + (long)f * C) = pk_bf16(gv.x, gv.y);
      } else {
        o[(long)f * C] = gv.x;
        o[(long)f * C + 1] = gv.y;
      }
    }
  }
}

// bf16 output: the conv and the GroupNorm affine on the matrix cores. Per utterance b the affine folds into the
// weights, z = (sc w) . x + sh; v = sc w and sh are split into bf16 parts v = hi + lo (to ~2^-16 relative), and one
// v_mfma_f32_16x16x32_bf16 over K = 32 forms z = v_hi.x_hi + v_hi.x_lo + v_lo.x_hi + sh_hi + sh_lo for 16 channels
// x 16 frames (the dropped v_lo.x_lo term is ~2^-17 relative: f32-level accuracy, unlike a plain bf16 conv).
// Frame rows [x_hi(10) x_lo(10) x_hi(10) 1 1] are staged once per block in LDS (64 B per frame, one ds_read_b128
// per lane), channel rows [v_hi v_hi v_lo sh_hi sh_lo] stay in registers. Only GELU + convert remain on the VALU
// (~11 VALU instructions per output; the recompute kernel spent 5 more on the conv; VALU-bound either way,
// SQ_ACTIVE_INST_VALU ~70 % of the SIMD cycles). Wave = 64 channels as 4 MFMA tiles; row 4g + r of tile j is
// channel 32(j/2) + 8g + 4(j%2) + r, so lane (frame f, g) holds channels 8g..8g+7 and 32+8g..32+8g+7 of frame f.
constexpr int C0M_FRAMES = 512;  // frames per block: the per-block setup (weights, affine, LDS rows) amortised
__device__ __forceinline__ int c0m_part(int k) { return k >= 20 ? 2 : (k >= 10 ? 1 : 0); }

__global__ void __launch_bounds__(512) conv0_mfma_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ scsh, bf16_t* __restrict__ out,
                                                         long nsamp, long T0, int C, int S) {
  constexpr int K = 10;
  __shared__ __attribute__((aligned(16))) bf16_t xr[C0M_FRAMES * 32];
  const long b = blockIdx.y;
  const long t0 = (long)blockIdx.x * C0M_FRAMES;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int e = tid; e < C0M_FRAMES * 32; e += 512) {
    const int f = e >> 5, k = e & 31;
    float v = k >= 3 * K ? 1.f : 0.f;
    int part = 0;
    if (k < 3 * K && t0 + f < T0) {
      part = c0m_part(k);
      v = x[b * nsamp + (t0 + f) * S + (k - K * part)];
    }
    const bf16_t hi = f2bf(v);
    xr[e] = part == 1 ? f2bf(v - bf2f(hi)) : hi;
  }
  const int fr = lane & 15, g = lane >> 4;
  const int cb = blockIdx.z * 512 + wv * 64;
  bf16x8_t wa[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = cb + 32 * (j >> 1) + 8 * (fr >> 2) + 4 * (j & 1) + (fr & 3);
    const float sc = scsh[2 * (b * C + c)], sh = scsh[2 * (b * C + c) + 1];
    const bf16_t shh = f2bf(sh);
    bf16_t u[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = 8 * g + q;
      bf16_t r;
      if (k < 3 * K) {
        const int part = c0m_part(k);
        const float wk = sc * w[c * K + (k - K * part)];
        const bf16_t hi = f2bf(wk);
        r = part == 2 ? f2bf(wk - bf2f(hi)) : hi;
      } else {
        r = k == 3 * K ? shh : f2bf(sh - bf2f(shh));
      }
      u[q] = r;
    }
    wa[j] = __builtin_bit_cast(bf16x8_t, u);
  }
  __syncthreads();
  const f32x4_t zero = {0.f, 0.f, 0.f, 0.f};
  const bool hi8 = fr >= 8;
  const long tend = min(T0 - t0, (long)C0M_FRAMES);
  bf16_t* ob = out + (b * T0 + t0 + (fr & 7)) * C + cb + (hi8 ? 32 : 0) + 8 * g;
  for (int f0 = 0; f0 < tend; f0 += 16) {
    const bf16x8_t xb = *(const bf16x8_t*)(xr + (f0 + fr) * 32 + 8 * g);
    f32x4_t acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[j], xb, zero, 0, 0, 0);
    // acc[j][r] = channel 32(j/2) + 8g + 4(j%2) + r of frame f0 + fr
    unsigned pk[8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; r += 2) pk[2 * j + r / 2] = pk_bf16(gelu_bf16out(acc[j][r]), gelu_bf16out(acc[j][r + 1]));
    // whole 128-B lines per store: lanes f and f ^ 8 (DPP row_ror:8) trade a 16-B chunk so that the first store
    // writes frames 0..7 of the tile and the second frames 8..15, each frame's 64 channels by its 8 lanes
    uint4 a, c;
    {
      unsigned y[4], z[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[e] = hi8 ? pk[e] : pk[4 + e];
        z[e] = (unsigned)__builtin_amdgcn_mov_dpp((int)y[e], 0x128, 0xf, 0xf, false);
      }
      a = hi8 ? make_uint4(z[0], z[1], z[2], z[3]) : make_uint4(pk[0], pk[1], pk[2], pk[3]);
      c = hi8 ? make_uint4(pk[4], pk[5], pk[6], pk[7]) : make_uint4(z[0], z[1], z[2], z[3]);
    }
    const int fa = f0 + (fr & 7);
    bf16_t* o = ob + (long)f0 * C;
    if (fa < tend) *(uint4*)o = a;
    if (fa + 8 < tend) *(uint4*)(o + 8 * C) = c;
  }
}

// one thread per (token, head): 64-element slice in 16-B loads, W (8 x 64) broadcast from LDS
template <typename T>
__global__ void __launch_bounds__(256) wavlm_gate_kernel(const T* __restrict__ x, const float* __restrict__ W,
                                                         const float* __restrict__ bias, const float* __restrict__ cst,
                                                         float* __restrict__ gate, long B, long S, int H, long E) {
  __shared__ float ws[8 * 64];
  const int dh = (int)(E / H);
  for (int i = threadIdx.x; i < 8 * dh; i += 256) ws[i] = W[i];
  __syncthreads();
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // e = tok * H + h
  if (e >= B * S * H) return;
  const long tok = e / H;
  const int h = (int)(e % H);
  const long b = tok / S, s = tok % S;
  const T* xr = x + tok * E + (long)h * dh;
  float r[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) r[o] = bias[o];
  constexpr int EPC = 16 / sizeof(T);
  for (int d0 = 0; d0 < dh; d0 += EPC) {
    const uint4 u = *(const uint4*)(xr + d0);
    const T* v = (const T*)&u;
#pragma unroll
    for (int j = 0; j < EPC; ++j) {
      const float xv = ld<T>(v + j);
#pragma unroll
      for (int o = 0; o < 8; ++o) r[o] += ws[o * dh + d0 + j] * xv;
    }
  }
  const float ga = 1.f / (1.f + __expf(-(r[0] + r[1] + r[2] + r[3])));
  const float gb = 1.f / (1.f + __expf(-(r[4] + r[5] + r[6] + r[7])));
  gate[(b * H + h) * S + s] = ga * (gb * cst[h] - 1.f) + 2.f;
}

}  // namespace fddm

using namespace fddm;

// ws: zeroed f64 scratch of B*(K + K*K) + B*C (the GroupNorm affine is stored after the Gram block)
FDDM_API int fddm_conv0_gn_gelu(int out_dtype, const float* x, const float* w, const float* gamma, const float* beta,
                                double* ws, void* out, long B, long nsamp, long T0, int C, int K, int S, float eps,
                                void* hs) {
  if (B <= 0 || T0 <= 0) return 0;
  if (K > C0_MAXK || C % 2) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)hs;
  if (K != 10) return (int)hipErrorInvalidValue;  // WavLM conv layer 0 (kernel 10, stride 5)
  const int nb = (int)((T0 + C0_GRAM_FRAMES - 1) / C0_GRAM_FRAMES);
  hipLaunchKernelGGL(conv0_gram_kernel<10>, dim3((unsigned)nb, (unsigned)B), dim3(256), 0, s, x, ws, nsamp, T0, S);
  float* scsh = (float*)(ws + B * nb * c0_nq<10>());
  hipLaunchKernelGGL(conv0_gn_affine_kernel<10>, dim3((unsigned)B), dim3(512), 0, s, ws, nb, w, gamma, beta, scsh, T0, C,
                     eps);
  if (out_dtype == FDDM_BF16 && C % 512 == 0) {
    dim3 gm((unsigned)((T0 + C0M_FRAMES - 1) / C0M_FRAMES), (unsigned)B, (unsigned)(C / 512));
    hipLaunchKernelGGL(conv0_mfma_kernel, gm, dim3(512), 0, s, x, w, scsh, (bf16_t*)out, nsamp, T0, C, S);
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)((T0 + C0_FRAMES - 1) / C0_FRAMES), (unsigned)B);
  const size_t lds = ((C0_FRAMES - 1) * S + K) * sizeof(float);
  if (out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((conv0_apply_kernel<bf16_t, 10>), grid, dim3(256), lds, s, x, w, scsh, (bf16_t*)out, nsamp, T0,
                       C, S);
  else
    hipLaunchKernelGGL((conv0_apply_kernel<float, 10>), grid, dim3(256), lds, s, x, w, scsh, (float*)out, nsamp, T0, C,
                       S);
  return (int)hipGetLastError();
}

// gate out: [B*H][S] f32; x: [B*S][E] (T)
FDDM_API int fddm_wavlm_gate(int dtype, const void* x, const float* W, const float* bias, const float* cst, float* gate,
                             long B, long S, int H, long E, void* hs) {
  const long n = B * S * H;
  if (n <= 0) return 0;
  if (E / H > 64 || (E / H) % 8) return (int)hipErrorInvalidValue;
  dim3 g((unsigned)((n + 255) / 256));
  if (dtype == FDDM_BF16)
    hipLaunchKernelGGL((wavlm_gate_kernel<bf16_t>), g, dim3(256), 0, (hipStream_t)hs, (const bf16_t*)x, W, bias, cst, gate,
                       B, S, H, E);
  else
    hipLaunchKernelGGL((wavlm_gate_kernel<float>), g, dim3(256), 0, (hipStream_t)hs, (const float*)x, W, bias, cst, gate,
                       B, S, H, E);
  return (int)hipGetLastError();
}
