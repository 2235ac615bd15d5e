// Fused clip_grad_norm_(5.0) + AdamW over all trainable tensors in two launches (train.py:411-423):
//   1) sum of squares of every gradient (multi-tensor, chunked) -> one fp32 accumulator
//   2) per element: g' = s g * min(1, max_norm / (s sqrt(total) + 1e-6)), s = grad_scale (1/W under data
//      parallelism: the ranks' gradient all-reduce leaves SUMS, the 1/W average is folded in here);
//      p *= (1 - lr*wd); m = lerp(m, g', 1-b1); v = b2 v + (1-b2) g'^2;
//      p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)          (torch.optim.AdamW single-tensor form)
//      and optionally a bf16 copy of p for the next forward's MFMA operands.
//   3) per tensor: step += 1 (device-side step counters, torch's AdamW `state["step"]`).
// No host synchronisation: the clip coefficient and the bias corrections (from the device step counters, in
// double like torch's host arithmetic) are computed on the device. Non-finite guard: when the gradient sum of
// squares is inf/NaN the whole step is skipped — no parameter, moment or step-counter update — as
// GradScaler.step skips it on the reference's GPU path (train.py:401-413); `skipped` counts such steps.
// Tensors whose grad is None are simply not in the list (set_to_none semantics, train.py:400).
#include "common.h"

namespace fddm {

struct MTTable {
  const long* chunk_tensor;  // [nchunks]
  const long* chunk_start;   // [nchunks]
  const long* numel;         // [ntensors]
  float* const* p;
  const float* const* g;
  float* const* m;
  float* const* v;
  bf16_t* const* pbf;        // entries may be null
  float* const* step;        // [ntensors] device step counters (0-d fp32 tensors)
};

constexpr long MT_CHUNK = 65536;

__global__ void __launch_bounds__(1024) sumsq_kernel(MTTable t, float* total) {
  __shared__ float red[16];
  const long ci = blockIdx.x;
  const long ti = t.chunk_tensor[ci], s0 = t.chunk_start[ci];
  const long n = min(MT_CHUNK, t.numel[ti] - s0);
  const float* g = t.g[ti] + s0;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  long i = 0;
  if ((((uintptr_t)g) & 15) == 0) {  // 16-B loads, 4 independent accumulators
    const long n4 = n / 4;
    // 1024 threads, U iterations' loads issued before any accumulation: 32 KB in flight per block instead of 4 KB (the
    // 256-thread one-load loop was latency-bound: 158.7 MB in 55 us, 2.9 TB/s; tools/probe/sumsq.py)
    constexpr int U = 8;
    long j = threadIdx.x;
    for (; j + 1024 * (U - 1) < n4; j += 1024 * U) {
      float4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = ((const float4*)g)[j + 1024 * u];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[0] += x[u].x * x[u].x;
        acc[1] += x[u].y * x[u].y;
        acc[2] += x[u].z * x[u].z;
        acc[3] += x[u].w * x[u].w;
      }
    }
    for (; j < n4; j += 1024) {
      const float4 x = ((const float4*)g)[j];
      acc[0] += x.x * x.x;
      acc[1] += x.y * x.y;
      acc[2] += x.z * x.z;
      acc[3] += x.w * x.w;
    }
    i = n4 * 4;
  }
  for (long j = i + threadIdx.x; j < n; j += 1024) acc[0] += g[j] * g[j];
  float v = block_sum((acc[0] + acc[1]) + (acc[2] + acc[3]), red);
  if (threadIdx.x == 0) atomicAdd(total, v);
}

template <bool ZG>
__global__ void __launch_bounds__(256) adamw_kernel(MTTable t, const float* total, float gscale, float max_norm, float lr,
                                                    float lr_wd, float b1, float b2, float eps) {
  const long ci = blockIdx.x;
  const long ti = t.chunk_tensor[ci], s0 = t.chunk_start[ci];
  const long n = min(MT_CHUNK, t.numel[ti] - s0);
  float coef = gscale;
  if (total) {
    if (!isfinite(total[0])) {  // non-finite gradients: skip the step (GradScaler semantics)
      if constexpr (ZG) {       // ... but still leave the gradients zeroed for the next step
        float* gz = (float*)t.g[ti] + s0;
        for (long i = threadIdx.x; i < n; i += 256) gz[i] = 0.f;
      }
      return;
    }
    if (max_norm > 0.f) coef = gscale * fminf(max_norm / (gscale * sqrtf(total[0]) + 1e-6f), 1.f);
  }
  // bias corrections of this step (torch: step_size = lr / (1 - b1^step), bc2_sqrt = sqrt(1 - b2^step), in double)
  const double stp = (double)t.step[ti][0] + 1.0;
  const float ss = (float)((double)lr / (1.0 - pow((double)b1, stp)));
  const float bc2s = (float)sqrt(1.0 - pow((double)b2, stp));
  float* p = t.p[ti] + s0;
  float* g = (float*)t.g[ti] + s0;
  float* m = t.m[ti] + s0;
  float* v = t.v[ti] + s0;
  bf16_t* pb = t.pbf[ti] ? t.pbf[ti] + s0 : nullptr;
  auto upd = [&](float gg, float& pp, float& mm, float& vv) {
    gg *= coef;
    pp *= 1.f - lr_wd;
    mm += (1.f - b1) * (gg - mm);
    vv = vv * b2 + (1.f - b2) * gg * gg;
    pp -= ss * (mm / (sqrtf(vv) / bc2s + eps));
  };
  long i0 = 0;
  const bool vec = ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0 &&
                   (pb == nullptr || (((uintptr_t)pb) & 7) == 0);
  if (vec) {  // 4 elements per thread and iteration: 16-B loads/stores, 8-B bf16 copy
    const long n4 = n / 4;
    // a block owns a 64 K-element chunk (~2.5 blocks per CU for the decoder): 4 iterations' loads are issued
    // before any update so each thread keeps 16 loads in flight instead of 4
    constexpr int U = 4;
    long j0 = threadIdx.x;
    for (; j0 + 256 * (U - 1) < n4; j0 += 256 * U) {
      float4 gg[U], pp[U], mm[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long j = j0 + 256 * u;
        gg[u] = ((const float4*)g)[j];
        pp[u] = ((float4*)p)[j];
        mm[u] = ((float4*)m)[j];
        vv[u] = ((float4*)v)[j];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long j = j0 + 256 * u;
        if constexpr (ZG) ((float4*)g)[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        upd(gg[u].x, pp[u].x, mm[u].x, vv[u].x);
        upd(gg[u].y, pp[u].y, mm[u].y, vv[u].y);
        upd(gg[u].z, pp[u].z, mm[u].z, vv[u].z);
        upd(gg[u].w, pp[u].w, mm[u].w, vv[u].w);
        ((float4*)p)[j] = pp[u];
        ((float4*)m)[j] = mm[u];
        ((float4*)v)[j] = vv[u];
        if (pb) ((uint2*)pb)[j] = make_uint2(pk_bf16(pp[u].x, pp[u].y), pk_bf16(pp[u].z, pp[u].w));
      }
    }
    for (long j = j0; j < n4; j += 256) {
      const float4 gg = ((const float4*)g)[j];
      if constexpr (ZG) ((float4*)g)[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      float4 pp = ((float4*)p)[j], mm = ((float4*)m)[j], vv = ((float4*)v)[j];
      upd(gg.x, pp.x, mm.x, vv.x);
      upd(gg.y, pp.y, mm.y, vv.y);
      upd(gg.z, pp.z, mm.z, vv.z);
      upd(gg.w, pp.w, mm.w, vv.w);
      ((float4*)p)[j] = pp;
      ((float4*)m)[j] = mm;
      ((float4*)v)[j] = vv;
      if (pb) ((uint2*)pb)[j] = make_uint2(pk_bf16(pp.x, pp.y), pk_bf16(pp.z, pp.w));
    }
    i0 = n4 * 4;
  }
  for (long i = i0 + threadIdx.x; i < n; i += 256) {
    float pp = p[i], mm = m[i], vv = v[i];
    upd(g[i], pp, mm, vv);
    if constexpr (ZG) g[i] = 0.f;
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
    if (pb) pb[i] = f2bf(pp);
  }
}

// step counters advance after every chunk of the step has read them (separate launch); a skipped step leaves them
__global__ void __launch_bounds__(256) adamw_step_kernel(float* const* step, long ntensors, const float* total,
                                                         int* skipped) {
  const bool ok = total == nullptr || isfinite(total[0]);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < ntensors; i += (long)gridDim.x * blockDim.x)
    if (ok) step[i][0] += 1.f;
  if (!ok && skipped && blockIdx.x == 0 && threadIdx.x == 0) skipped[0] += 1;
}

}  // namespace fddm

using namespace fddm;

FDDM_API int fddm_grad_sumsq(const long* chunk_tensor, const long* chunk_start, const long* numel, const float* const* g,
                             long nchunks, float* total, void* hs) {
  if (nchunks <= 0) return 0;
  MTTable t{chunk_tensor, chunk_start, numel, nullptr, g, nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(sumsq_kernel, dim3((unsigned)nchunks), dim3(1024), 0, (hipStream_t)hs, t, total);
  return (int)hipGetLastError();
}

FDDM_API int fddm_adamw(const long* chunk_tensor, const long* chunk_start, const long* numel, float* const* p,
                        const float* const* g, float* const* m, float* const* v, bf16_t* const* pbf, float* const* step,
                        long ntensors, long nchunks, const float* total, float max_norm, float lr, float lr_wd, float b1,
                        float b2, float eps, int* skipped, int zero_g, float grad_scale, void* hs) {
  if (nchunks <= 0) return 0;
  MTTable t{chunk_tensor, chunk_start, numel, p, g, m, v, pbf, step};
  if (zero_g)
    hipLaunchKernelGGL(adamw_kernel<true>, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)hs, t, total, grad_scale,
                       max_norm, lr, lr_wd, b1, b2, eps);
  else
    hipLaunchKernelGGL(adamw_kernel<false>, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)hs, t, total, grad_scale,
                       max_norm, lr, lr_wd, b1, b2, eps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(adamw_step_kernel, dim3(1), dim3(256), 0, (hipStream_t)hs, step, ntensors, total, skipped);
  return (int)hipGetLastError();
}
