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

constexpr int C0_FRAMES = 64;  // frames per block

__global__ void __launch_bounds__(256) conv0_stats_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          double* __restrict__ sum, double* __restrict__ sq, long nsamp,
                                                          long T0, int C, int K, int S) {
  extern __shared__ float xs[];
  const long b = blockIdx.y;
  const long t0 = (long)blockIdx.x * C0_FRAMES;
  const int nf = (int)min((long)C0_FRAMES, T0 - t0);
  const int span = (nf - 1) * S + K;
  for (int i = threadIdx.x; i < span; i += 256) xs[i] = x[b * nsamp + t0 * S + i];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float wk[16];
    for (int k = 0; k < K; ++k) wk[k] = w[c * K + k];
    float s = 0.f, s2 = 0.f;
    for (int f = 0; f < nf; ++f) {
      float y = 0.f;
      for (int k = 0; k < K; ++k) y += wk[k] * xs[f * S + k];
      s += y;
      s2 += y * y;
    }
    atomicAdd(sum + b * C + c, (double)s);
    atomicAdd(sq + b * C + c, (double)s2);
  }
}

template <typename OT>
__global__ void __launch_bounds__(256) conv0_apply_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const double* __restrict__ sum, const double* __restrict__ sq,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          OT* __restrict__ out, long nsamp, long T0, int C, int K, int S,
                                                          float eps) {
  extern __shared__ float xs[];
  const long b = blockIdx.y;
  const long t0 = (long)blockIdx.x * C0_FRAMES;
  const int nf = (int)min((long)C0_FRAMES, T0 - t0);
  const int span = (nf - 1) * S + K;
  for (int i = threadIdx.x; i < span; i += 256) xs[i] = x[b * nsamp + t0 * S + i];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float wk[16];
    for (int k = 0; k < K; ++k) wk[k] = w[c * K + k];
    const double mean = sum[b * C + c] / (double)T0;
    const double var = fmax(sq[b * C + c] / (double)T0 - mean * mean, 0.0);
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = rstd * gamma[c];
    const float sh = beta[c] - (float)mean * sc;
    for (int f = 0; f < nf; ++f) {
      float y = 0.f;
      for (int k = 0; k < K; ++k) y += wk[k] * xs[f * S + k];
      st<OT>(out + (b * T0 + t0 + f) * C + c, gelu_f(y * sc + sh));
    }
  }
}

template <typename T>
__global__ void wavlm_gate_kernel(const T* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
                                  const float* __restrict__ cst, float* __restrict__ gate, long B, long S, int H, long E) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over B*S*H
  if (e >= B * S * H) return;
  const int h = (int)(e % H);
  const long bs = e / H;
  const long b = bs / S, s = bs % S;
  const int dh = (int)(E / H);
  const T* xr = x + bs * E + (long)h * dh;
  float r[8];
  for (int o = 0; o < 8; ++o) r[o] = bias[o];
  for (int d = 0; d < dh; ++d) {
    const float xv = ld<T>(xr + d);
    for (int o = 0; o < 8; ++o) r[o] += W[o * dh + d] * xv;
  }
  const float a = 1.f / (1.f + __expf(-(r[0] + r[1] + r[2] + r[3])));
  const float g = 1.f / (1.f + __expf(-(r[4] + r[5] + r[6] + r[7])));
  gate[(b * H + h) * S + s] = a * (g * cst[h] - 1.f) + 2.f;
}

}  // namespace fddm

using namespace fddm;

// sum/sq: [B][C] doubles, zeroed by the caller
FDDM_API int fddm_conv0_gn_gelu(int out_dtype, const float* x, const float* w, const float* gamma, const float* beta,
                                double* sum, double* sq, void* out, long B, long nsamp, long T0, int C, int K, int S,
                                float eps, void* hs) {
  if (B <= 0 || T0 <= 0) return 0;
  if (K > 16) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((T0 + C0_FRAMES - 1) / C0_FRAMES), (unsigned)B);
  const size_t lds = ((C0_FRAMES - 1) * S + K) * sizeof(float);
  hipStream_t s = (hipStream_t)hs;
  hipLaunchKernelGGL(conv0_stats_kernel, grid, dim3(256), lds, s, x, w, sum, sq, nsamp, T0, C, K, S);
  if (out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((conv0_apply_kernel<bf16_t>), grid, dim3(256), lds, s, x, w, sum, sq, gamma, beta, (bf16_t*)out,
                       nsamp, T0, C, K, S, eps);
  else
    hipLaunchKernelGGL((conv0_apply_kernel<float>), grid, dim3(256), lds, s, x, w, sum, sq, gamma, beta, (float*)out,
                       nsamp, T0, C, K, S, eps);
  return (int)hipGetLastError();
}

// gate out: [B*H][S] f32; x: [B*S][E] (T)
FDDM_API int fddm_wavlm_gate(int dtype, const void* x, const float* W, const float* bias, const float* cst, float* gate,
                             long B, long S, int H, long E, void* hs) {
  const long n = B * S * H;
  if (n <= 0) return 0;
  dim3 g((unsigned)((n + 255) / 256));
  if (dtype == FDDM_BF16)
    hipLaunchKernelGGL((wavlm_gate_kernel<bf16_t>), g, dim3(256), 0, (hipStream_t)hs, (const bf16_t*)x, W, bias, cst, gate,
                       B, S, H, E);
  else
    hipLaunchKernelGGL((wavlm_gate_kernel<float>), g, dim3(256), 0, (hipStream_t)hs, (const float*)x, W, bias, cst, gate,
                       B, S, H, E);
  return (int)hipGetLastError();
}
