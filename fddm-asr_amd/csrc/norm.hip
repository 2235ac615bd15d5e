// Residual + dropout + LayerNorm (+ FiLM) fused forward / backward, one wave per row.
//
// forward:  s   = x + drop(y)                      (y optional; dropout = nn.Dropout before the add)
//           out = LN(s) * gamma + beta             (eps, biased variance: torch.nn.LayerNorm)
//           out = out * (1 + film_scale[b]) + film_shift[b]     (optional FiLM, models/denoise_decoder.py:87-89)
// Sites: DecoderBlock norm1/norm2(+FiLM)/norm3 (models/denoise_decoder.py:165-191), WavLM post-LN
// residual blocks and feature-projection/encoder LayerNorms (HF modeling_wavlm.py:102, 313-317, 405).
// backward: from dout (f32): ds (f32, the residual-branch gradient), dy = drop'(ds) in T for the
// producing GEMM, dgamma/dbeta and dfilm_scale/dfilm_shift accumulated with atomics (caller zeroes).
#include "common.h"

namespace fddm {

constexpr int LN_MAXPL = 16;  // d <= 1024

struct LnFwdArgs {
  const void* x; const void* y;
  const float *gamma, *beta, *fsc, *fsh;
  float* out_f32; void* out_t; float* save_s; float *mean, *rstd;
  long N, d, rows_per_batch;
  float eps;
  uint64_t seed, stream; unsigned thr16; float drop_scale;
};

template <typename XT, typename YT, typename OT>
__global__ void __launch_bounds__(256) ln_fwd_kernel(LnFwdArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.N) return;
  const long d = a.d;
  const XT* x = (const XT*)a.x + row * d;
  const YT* y = a.y ? (const YT*)a.y + row * d : nullptr;
  float v[LN_MAXPL];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXPL; ++i) {
    const long c = lane + 64L * i;
    float t = 0.f;
    if (c < d) {
      t = ld<XT>(x + c);
      if (y) {
        float yv = ld<YT>(y + c);
        if (a.thr16) yv = drop_keep(a.seed, a.stream, (uint64_t)(row * d + c), a.thr16) ? yv * a.drop_scale : 0.f;
        t += yv;
      }
    }
    v[i] = t;
    sum += t;
  }
  const float mean = wave_sum(sum) / (float)d;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXPL; ++i) {
    const long c = lane + 64L * i;
    if (c < d) {
      const float t = v[i] - mean;
      sq += t * t;
    }
  }
  const float var = wave_sum(sq) / (float)d;
  const float rstd = 1.f / sqrtf(var + a.eps);
  const long b = row / a.rows_per_batch;
#pragma unroll
  for (int i = 0; i < LN_MAXPL; ++i) {
    const long c = lane + 64L * i;
    if (c < d) {
      if (a.save_s) a.save_s[row * d + c] = v[i];
      float o = (v[i] - mean) * rstd * a.gamma[c] + a.beta[c];
      if (a.fsc) o = o * (1.f + a.fsc[b * d + c]) + a.fsh[b * d + c];
      if (a.out_f32) a.out_f32[row * d + c] = o;
      if (a.out_t) st<OT>((OT*)a.out_t + row * d + c, o);
    }
  }
  if (lane == 0) {
    if (a.mean) a.mean[row] = mean;
    if (a.rstd) a.rstd[row] = rstd;
  }
}

struct LnBwdArgs {
  const float* dout; const float* s; const float *mean, *rstd, *gamma, *beta, *fsc;
  float* dres; void* dy_t;
  float *dgamma, *dbeta, *dfsc, *dfsh;
  long N, d, rows_per_batch;
  uint64_t seed, stream; unsigned thr16; float drop_scale;
};

constexpr int LN_BWD_ROWS = 8;  // rows per wave

template <typename OT>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnBwdArgs a) {
  const int lane = threadIdx.x & 63;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * LN_BWD_ROWS;
  const long d = a.d;
  float dg[LN_MAXPL], db[LN_MAXPL], dsc[LN_MAXPL], dsh[LN_MAXPL];
#pragma unroll
  for (int i = 0; i < LN_MAXPL; ++i) dg[i] = db[i] = dsc[i] = dsh[i] = 0.f;
  long cur_b = -1;
  auto flush_film = [&]() {
    if (cur_b < 0 || !a.fsc) return;
#pragma unroll
    for (int i = 0; i < LN_MAXPL; ++i) {
      const long c = lane + 64L * i;
      if (c < d) {
        atomicAdd(a.dfsc + cur_b * d + c, dsc[i]);
        atomicAdd(a.dfsh + cur_b * d + c, dsh[i]);
      }
      dsc[i] = dsh[i] = 0.f;
    }
  };
  for (int r = 0; r < LN_BWD_ROWS; ++r) {
    const long row = row0 + r;
    if (row >= a.N) break;
    const long b = row / a.rows_per_batch;
    if (b != cur_b) {
      flush_film();
      cur_b = b;
    }
    const float mean = a.mean[row], rstd = a.rstd[row];
    float xh[LN_MAXPL], dxh[LN_MAXPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXPL; ++i) {
      const long c = lane + 64L * i;
      xh[i] = dxh[i] = 0.f;
      if (c < d) {
        const float x = (a.s[row * d + c] - mean) * rstd;
        float go = a.dout[row * d + c];
        if (a.fsc) {
          const float lo = x * a.gamma[c] + a.beta[c];
          dsc[i] += go * lo;
          dsh[i] += go;
          go *= 1.f + a.fsc[b * d + c];
        }
        dg[i] += go * x;
        db[i] += go;
        const float gx = go * a.gamma[c];
        xh[i] = x;
        dxh[i] = gx;
        s1 += gx;
        s2 += gx * x;
      }
    }
    s1 = wave_sum(s1) / (float)d;
    s2 = wave_sum(s2) / (float)d;
#pragma unroll
    for (int i = 0; i < LN_MAXPL; ++i) {
      const long c = lane + 64L * i;
      if (c < d) {
        const float ds = rstd * (dxh[i] - s1 - xh[i] * s2);
        if (a.dres) a.dres[row * d + c] = ds;
        if (a.dy_t) {
          float dy = ds;
          if (a.thr16) dy = drop_keep(a.seed, a.stream, (uint64_t)(row * d + c), a.thr16) ? dy * a.drop_scale : 0.f;
          st<OT>((OT*)a.dy_t + row * d + c, dy);
        }
      }
    }
  }
  flush_film();
#pragma unroll
  for (int i = 0; i < LN_MAXPL; ++i) {
    const long c = lane + 64L * i;
    if (c < d && a.dgamma) {
      atomicAdd(a.dgamma + c, dg[i]);
      atomicAdd(a.dbeta + c, db[i]);
    }
  }
}

}  // namespace fddm

using namespace fddm;

// x_dtype/y_dtype/out_dtype: FDDM_F32 / FDDM_BF16. y may be null. Outputs may be null.
FDDM_API int fddm_ln_fwd(int x_dtype, int y_dtype, int out_dtype, const void* x, const void* y, const float* gamma,
                         const float* beta, const float* film_scale, const float* film_shift, float* out_f32,
                         void* out_t, float* save_s, float* mean, float* rstd, long N, long d, long rows_per_batch,
                         float eps, float drop_p, unsigned long long seed, unsigned long long stream, void* hs) {
  if (N <= 0) return 0;
  if (d > 64 * LN_MAXPL) return (int)hipErrorInvalidValue;
  LnFwdArgs a{x, y, gamma, beta, film_scale, film_shift, out_f32, out_t, save_s, mean, rstd, N, d,
              rows_per_batch > 0 ? rows_per_batch : N, eps, seed, stream, 0u, 1.f};
  if (drop_p > 0.f) {
    a.thr16 = (unsigned)llrintf(drop_p * 65536.f);
    a.drop_scale = 1.f / (1.f - drop_p);
  }
  dim3 grid((unsigned)((N + 3) / 4));
  hipStream_t s = (hipStream_t)hs;
  if (x_dtype == FDDM_F32 && y_dtype == FDDM_BF16 && out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((ln_fwd_kernel<float, bf16_t, bf16_t>), grid, dim3(256), 0, s, a);
  else if (x_dtype == FDDM_F32 && y_dtype == FDDM_F32 && out_dtype == FDDM_F32)
    hipLaunchKernelGGL((ln_fwd_kernel<float, float, float>), grid, dim3(256), 0, s, a);
  else if (x_dtype == FDDM_BF16 && y_dtype == FDDM_BF16 && out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((ln_fwd_kernel<bf16_t, bf16_t, bf16_t>), grid, dim3(256), 0, s, a);
  else if (x_dtype == FDDM_F32 && y_dtype == FDDM_F32 && out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((ln_fwd_kernel<float, float, bf16_t>), grid, dim3(256), 0, s, a);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

FDDM_API int fddm_ln_bwd(int dy_dtype, const float* dout, const float* s, const float* mean, const float* rstd,
                         const float* gamma, const float* beta, const float* film_scale, float* dres, void* dy_t,
                         float* dgamma, float* dbeta, float* dfilm_scale, float* dfilm_shift, long N, long d,
                         long rows_per_batch, float drop_p, unsigned long long seed, unsigned long long stream,
                         void* hs) {
  if (N <= 0) return 0;
  if (d > 64 * LN_MAXPL) return (int)hipErrorInvalidValue;
  LnBwdArgs a{dout, s, mean, rstd, gamma, beta, film_scale, dres, dy_t, dgamma, dbeta, dfilm_scale, dfilm_shift,
              N, d, rows_per_batch > 0 ? rows_per_batch : N, seed, stream, 0u, 1.f};
  if (drop_p > 0.f) {
    a.thr16 = (unsigned)llrintf(drop_p * 65536.f);
    a.drop_scale = 1.f / (1.f - drop_p);
  }
  const long waves = (N + LN_BWD_ROWS - 1) / LN_BWD_ROWS;
  dim3 grid((unsigned)((waves + 3) / 4));
  hipStream_t st_ = (hipStream_t)hs;
  if (dy_dtype == FDDM_BF16)
    hipLaunchKernelGGL((ln_bwd_kernel<bf16_t>), grid, dim3(256), 0, st_, a);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<float>), grid, dim3(256), 0, st_, a);
  return (int)hipGetLastError();
}
