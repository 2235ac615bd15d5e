// L_fd cross-modal feature decorrelation (losses/fddm_losses.py:18-58) — the non-GEMM parts.
// The [D x D] cross-correlation C = za~^T zb~ / (B*T) and its two backward products run on the MFMA
// GEMM (MC operands, no transposes); these kernels do the batch-dim standardisation and the loss.
#include "common.h"

namespace fddm {

// per column c of z [B][C] (C = T*D): mean / biased var over B, z~ = (z - mean)/sqrt(var + eps)
template <typename OT>
__global__ void lfd_std_fwd_kernel(const float* __restrict__ z, OT* __restrict__ zt, float* __restrict__ inv_std, long B,
                                   long C, float eps) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float m = 0.f;
  for (long b = 0; b < B; ++b) m += z[b * C + c];
  m /= (float)B;
  float v = 0.f;
  for (long b = 0; b < B; ++b) {
    const float t = z[b * C + c] - m;
    v += t * t;
  }
  v /= (float)B;
  const float is = 1.f / sqrtf(v + eps);
  inv_std[c] = is;
  for (long b = 0; b < B; ++b) st<OT>(zt + b * C + c, (z[b * C + c] - m) * is);
}

// dz = (dz~ - mean_b(dz~) - z~ * mean_b(dz~ * z~)) * inv_std
template <typename T>
__global__ void lfd_std_bwd_kernel(const float* __restrict__ dzt, const T* __restrict__ zt, const float* __restrict__ inv_std,
                                   float* __restrict__ dz, long B, long C) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float m1 = 0.f, m2 = 0.f;
  for (long b = 0; b < B; ++b) {
    const float g = dzt[b * C + c];
    m1 += g;
    m2 += g * ld<T>(zt + b * C + c);
  }
  m1 /= (float)B;
  m2 /= (float)B;
  const float is = inv_std[c];
  for (long b = 0; b < B; ++b) dz[b * C + c] = (dzt[b * C + c] - m1 - ld<T>(zt + b * C + c) * m2) * is;
}

// ---- data-parallel form: the batch statistics of the standardisation span every rank's rows.
// Each rank reduces its own rows per column; the caller all-reduces the partial sums between the passes.
// pass 1 (mean_sum == null): out[c] = sum_b z[b][c];  pass 2: out[c] = sum_b (z[b][c] - mean_sum[c]*inv_n)^2
__global__ void lfd_colstat_kernel(const float* __restrict__ z, float* __restrict__ out, const float* __restrict__ mean_sum,
                                   float inv_n, long B, long C) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float acc = 0.f;
  if (mean_sum == nullptr) {
    for (long b = 0; b < B; ++b) acc += z[b * C + c];
  } else {
    const float m = mean_sum[c] * inv_n;
    for (long b = 0; b < B; ++b) {
      const float t = z[b * C + c] - m;
      acc += t * t;
    }
  }
  out[c] = acc;
}

// z~ = (z - S1*inv_n) / sqrt(S2*inv_n + eps) from the global column sums S1 (sum z) and S2 (centred squares)
template <typename OT>
__global__ void lfd_std_apply_kernel(const float* __restrict__ z, OT* __restrict__ zt, float* __restrict__ inv_std,
                                     const float* __restrict__ s1, const float* __restrict__ s2, float inv_n, float eps,
                                     long B, long C) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float m = s1[c] * inv_n;
  const float is = 1.f / sqrtf(s2[c] * inv_n + eps);
  inv_std[c] = is;
  for (long b = 0; b < B; ++b) st<OT>(zt + b * C + c, (z[b * C + c] - m) * is);
}

// backward partial sums: out[c] = sum_b dz~, out[C + c] = sum_b dz~ * z~
template <typename T>
__global__ void lfd_bwd_colstat_kernel(const float* __restrict__ dzt, const T* __restrict__ zt, float* __restrict__ out,
                                       long B, long C) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float m1 = 0.f, m2 = 0.f;
  for (long b = 0; b < B; ++b) {
    const float g = dzt[b * C + c];
    m1 += g;
    m2 += g * ld<T>(zt + b * C + c);
  }
  out[c] = m1;
  out[C + c] = m2;
}

// dz = scale * (dz~ - S1*inv_n - z~ * S2*inv_n) * inv_std   (S1, S2: global sums of lfd_bwd_colstat)
template <typename T>
__global__ void lfd_std_bwd_apply_kernel(const float* __restrict__ dzt, const T* __restrict__ zt,
                                         const float* __restrict__ inv_std, const float* __restrict__ sums, float inv_n,
                                         float scale, float* __restrict__ dz, long B, long C) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float m1 = sums[c] * inv_n, m2 = sums[C + c] * inv_n;
  const float is = inv_std[c] * scale;
  for (long b = 0; b < B; ++b) dz[b * C + c] = (dzt[b * C + c] - m1 - ld<T>(zt + b * C + c) * m2) * is;
}

// loss = sum_j (1 - C_jj)^2 + lambda * sum_{j!=k} C_jk^2
//      = lambda * sum_{all} C^2 + sum_j [(1 - C_jj)^2 - lambda * C_jj^2]
// One 1024-thread workgroup: the all-element sum of squares with 16-B loads (16 in flight per thread at D = 256, no
// index arithmetic per element), the D diagonal terms by the first D threads, one block reduction. (Was one
// 256-thread workgroup with a 64-bit divide and modulo per element: 83 us at D = 256.)
__global__ void __launch_bounds__(1024) lfd_loss_kernel(const float* __restrict__ Cm, float* __restrict__ loss, int D,
                                                        float lam) {
  __shared__ float red[16];
  const int n = D * D;
  float sq = 0.f, dg = 0.f;
  int i0 = 0;
  if (!(((uintptr_t)Cm) & 15)) {
    const int n4 = n >> 2;
    const float4* c4 = (const float4*)Cm;
    float a0 = 0.f, a1 = 0.f;
    for (int j = threadIdx.x; j < n4; j += 1024) {
      const float4 v = c4[j];
      a0 += v.x * v.x + v.y * v.y;
      a1 += v.z * v.z + v.w * v.w;
    }
    sq = a0 + a1;
    i0 = n4 << 2;
  }
  for (int e = i0 + threadIdx.x; e < n; e += 1024) sq += Cm[e] * Cm[e];
  for (int j = threadIdx.x; j < D; j += 1024) {
    const float c = Cm[j * (D + 1)];
    dg += (1.f - c) * (1.f - c) - lam * c * c;
  }
  const float acc = block_sum(lam * sq + dg, red);
  if (threadIdx.x == 0) loss[0] = acc;
}

// dC = g * d loss / dC
template <typename OT>
__global__ void lfd_dloss_kernel(const float* __restrict__ Cm, const float* __restrict__ gscale, OT* __restrict__ dC, int D,
                                 float lam) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= D * D) return;
  const int j = e / D, k = e - j * D;
  const float c = Cm[e];
  const float g = gscale ? gscale[0] : 1.f;
  st<OT>(dC + e, g * ((j == k) ? -2.f * (1.f - c) : 2.f * lam * c));
}

}  // namespace fddm

using namespace fddm;

FDDM_API int fddm_lfd_std_fwd(int out_dtype, const float* z, void* zt, float* inv_std, long B, long C, float eps, void* hs) {
  if (C <= 0) return 0;
  dim3 g((unsigned)((C + 255) / 256));
  if (out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((lfd_std_fwd_kernel<bf16_t>), g, dim3(256), 0, (hipStream_t)hs, z, (bf16_t*)zt, inv_std, B, C, eps);
  else
    hipLaunchKernelGGL((lfd_std_fwd_kernel<float>), g, dim3(256), 0, (hipStream_t)hs, z, (float*)zt, inv_std, B, C, eps);
  return (int)hipGetLastError();
}

FDDM_API int fddm_lfd_std_bwd(int zt_dtype, const float* dzt, const void* zt, const float* inv_std, float* dz, long B,
                              long C, void* hs) {
  if (C <= 0) return 0;
  dim3 g((unsigned)((C + 255) / 256));
  if (zt_dtype == FDDM_BF16)
    hipLaunchKernelGGL((lfd_std_bwd_kernel<bf16_t>), g, dim3(256), 0, (hipStream_t)hs, dzt, (const bf16_t*)zt, inv_std, dz, B, C);
  else
    hipLaunchKernelGGL((lfd_std_bwd_kernel<float>), g, dim3(256), 0, (hipStream_t)hs, dzt, (const float*)zt, inv_std, dz, B, C);
  return (int)hipGetLastError();
}

FDDM_API int fddm_lfd_loss(const float* Cm, float* loss, long D, float lam, void* hs) {
  if (D <= 0 || D > 32768) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(lfd_loss_kernel, dim3(1), dim3(1024), 0, (hipStream_t)hs, Cm, loss, (int)D, lam);
  return (int)hipGetLastError();
}

FDDM_API int fddm_lfd_dloss(int out_dtype, const float* Cm, const float* gscale, void* dC, long D, float lam, void* hs) {
  if (D <= 0 || D > 32768) return (int)hipErrorInvalidValue;
  dim3 g((unsigned)((D * D + 255) / 256));
  if (out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((lfd_dloss_kernel<bf16_t>), g, dim3(256), 0, (hipStream_t)hs, Cm, gscale, (bf16_t*)dC, (int)D, lam);
  else
    hipLaunchKernelGGL((lfd_dloss_kernel<float>), g, dim3(256), 0, (hipStream_t)hs, Cm, gscale, (float*)dC, (int)D, lam);
  return (int)hipGetLastError();
}

FDDM_API int fddm_lfd_colstat(const float* z, float* out, const float* mean_sum, float inv_n, long B, long C, void* hs) {
  if (C <= 0) return 0;
  hipLaunchKernelGGL(lfd_colstat_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, (hipStream_t)hs, z, out,
                     mean_sum, inv_n, B, C);
  return (int)hipGetLastError();
}

FDDM_API int fddm_lfd_std_apply(int out_dtype, const float* z, void* zt, float* inv_std, const float* s1, const float* s2,
                                float inv_n, float eps, long B, long C, void* hs) {
  if (C <= 0) return 0;
  dim3 g((unsigned)((C + 255) / 256));
  if (out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((lfd_std_apply_kernel<bf16_t>), g, dim3(256), 0, (hipStream_t)hs, z, (bf16_t*)zt, inv_std, s1, s2,
                       inv_n, eps, B, C);
  else
    hipLaunchKernelGGL((lfd_std_apply_kernel<float>), g, dim3(256), 0, (hipStream_t)hs, z, (float*)zt, inv_std, s1, s2,
                       inv_n, eps, B, C);
  return (int)hipGetLastError();
}

FDDM_API int fddm_lfd_bwd_colstat(int zt_dtype, const float* dzt, const void* zt, float* out, long B, long C, void* hs) {
  if (C <= 0) return 0;
  dim3 g((unsigned)((C + 255) / 256));
  if (zt_dtype == FDDM_BF16)
    hipLaunchKernelGGL((lfd_bwd_colstat_kernel<bf16_t>), g, dim3(256), 0, (hipStream_t)hs, dzt, (const bf16_t*)zt, out, B, C);
  else
    hipLaunchKernelGGL((lfd_bwd_colstat_kernel<float>), g, dim3(256), 0, (hipStream_t)hs, dzt, (const float*)zt, out, B, C);
  return (int)hipGetLastError();
}

FDDM_API int fddm_lfd_std_bwd_apply(int zt_dtype, const float* dzt, const void* zt, const float* inv_std, const float* sums,
                                    float inv_n, float scale, float* dz, long B, long C, void* hs) {
  if (C <= 0) return 0;
  dim3 g((unsigned)((C + 255) / 256));
  if (zt_dtype == FDDM_BF16)
    hipLaunchKernelGGL((lfd_std_bwd_apply_kernel<bf16_t>), g, dim3(256), 0, (hipStream_t)hs, dzt, (const bf16_t*)zt, inv_std,
                       sums, inv_n, scale, dz, B, C);
  else
    hipLaunchKernelGGL((lfd_std_bwd_apply_kernel<float>), g, dim3(256), 0, (hipStream_t)hs, dzt, (const float*)zt, inv_std,
                       sums, inv_n, scale, dz, B, C);
  return (int)hipGetLastError();
}
