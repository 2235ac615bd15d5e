// Discrete-diffusion kernels:
//  * fddm_sample_q      — SchedulerAdapter.sample_q (train.py:180-188): closed-form two-valued
//                         inverse CDF over the q_sample distribution, counter-based RNG (bit-exact
//                         with oracle.sample_xt).
//  * fddm_kl_fwd/_bwd   — SchedulerAdapter.kl_term (train.py:190-255): per-token categorical KL
//                         q(x_{t-1}|x_t,x0) || p(x_{t-1}|x_t,softmax(z)) and its exact gradient,
//                         one workgroup per token, the V-row held in registers (one HBM read,
//                         one write). Closed form: SURVEY §8(a) "KL closed form".
//  * fddm_softmax_rows / fddm_softmax_bwd_rows — TextEmbedding (models/projection.py:41-47).
#include "common.h"
#include <type_traits>
#include <cstdlib>

namespace fddm {

__global__ void sample_q_kernel(const long* __restrict__ x0, const long* __restrict__ t,
                                const unsigned* __restrict__ thr, long* __restrict__ xt, long B, long L,
                                long K, uint64_t seed, uint64_t stream) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * L) return;
  const long b = e / L;
  const uint64_t h = mix64(seed, stream, (uint64_t)e);
  const unsigned r1 = (unsigned)(h >> 32), r2 = (unsigned)(h & 0xffffffffu);
  const long x = x0[e];
  const long tv = t[b];
  if (r1 < thr[tv - 1]) {
    xt[e] = x;
  } else {
    const long j = (long)(((uint64_t)r2 * (uint64_t)(K - 1)) >> 32);
    xt[e] = j + (j >= x ? 1 : 0);
  }
}

struct KlRow {
  float a_t, b_t, a_p, b_p, dq, inv_dq;
};

__device__ __forceinline__ KlRow kl_consts(const float* betas, long tv, long xt, long x0, float K) {
  KlRow c;
  const float bt = betas[tv - 1];
  const float bp = (tv == 1) ? 0.f : betas[tv - 2];
  c.a_t = 1.f - bt;
  c.b_t = bt / K;
  c.a_p = 1.f - bp;
  c.b_p = bp / K;
  c.dq = c.b_t + c.a_t * (x0 == xt ? 1.f : 0.f);
  c.inv_dq = 1.f / (c.dq + 1e-8f);
  return c;
}

// NPT = row elements held per thread (V <= 256 * NPT).
// Every index k other than x_t and x0 has M_k = b_t and Q_k = Qg = b_t b_p / dq, so the row pass evaluates that
// generic form for all k (one log per element forward; one rcp per element backward, kept in registers for the
// output pass) and the at most two special indices are corrected with scalar terms afterwards.
template <int NPT, bool BWD, typename OT>
__global__ void __launch_bounds__(256) kl_kernel(const float* __restrict__ logits, const long* __restrict__ xt_,
                                                 const long* __restrict__ x0_, const long* __restrict__ t_,
                                                 const float* __restrict__ betas, const float* __restrict__ w,
                                                 const float* __restrict__ gscale, float* __restrict__ kl_tok,
                                                 OT* __restrict__ dz, long L, long V) {
  __shared__ float red[8];
  const long row = blockIdx.x;
  const int tid = threadIdx.x;
  const float* z = logits + row * V;
  const long xt = xt_[row], x0 = x0_[row], tv = t_[row / L];
  const float eps = 1e-8f;
  const KlRow c = kl_consts(betas, tv, xt, x0, (float)V);

  float v[NPT];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const long k = tid + 256L * i;
    v[i] = k < V ? z[k] : -INFINITY;
    mx = fmaxf(mx, v[i]);
  }
  mx = block_max(mx, red);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    v[i] = __expf(v[i] - mx);  // exp(-inf) = 0 for padding lanes
    s += v[i];
  }
  s = block_sum(s, red);
  const float inv_s = 1.f / s;
  const float xhat_xt = __expf(z[xt] - mx) * inv_s;
  const float xhat_x0 = __expf(z[x0] - mx) * inv_s;
  const float dp = c.b_t + c.a_t * xhat_xt;
  const float inv_dp = 1.f / (dp + eps);
  const float Qg = c.b_t * c.b_p * c.inv_dq;
  // the exact per-index terms (P, Q, KL term, S1 term, g0 term) of index k with normalised probability xh
  auto special = [&](long k, float xh, float& P, float& Q, float& M) {
    M = c.b_t + (k == xt ? c.a_t : 0.f);
    Q = M * ((k == x0 ? c.a_p : 0.f) + c.b_p) * c.inv_dq;
    P = M * (c.a_p * xh + c.b_p) * inv_dp;
  };
  auto generic_P = [&](float xh) { return c.b_t * (c.a_p * xh + c.b_p) * inv_dp; };

  if (!BWD) {
    // KL = sum_k Q (log(Q+eps) - log(P+eps)): generic form for all k, then the special indices swapped in
    const float LQg = __logf(Qg + eps);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const long k = tid + 256L * i;
      if (k < V) acc += LQg - __logf(generic_P(v[i] * inv_s) + eps);
    }
    acc = block_sum(acc, red);
    if (tid == 0) {
      float kl = Qg * acc;
      const long ks[2] = {xt, x0};
      const float xs[2] = {xhat_xt, xhat_x0};
      for (int j = 0; j < (xt == x0 ? 1 : 2); ++j) {
        float P, Q, M;
        special(ks[j], xs[j], P, Q, M);
        kl += Q * (__logf(Q + eps) - __logf(P + eps)) - Qg * (LQg - __logf(generic_P(xs[j]) + eps));
      }
      kl_tok[row] = kl;
    }
    return;
  }
  // backward: S1 = sum Q P/(P+eps), G0 = sum -Q M a_p/(P+eps) inv_dp xh
  float r[NPT];
  float a1 = 0.f, a2 = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const long k = tid + 256L * i;
    const float xh = v[i] * inv_s;
    v[i] = xh;
    const float P = generic_P(xh);
    r[i] = 1.f / (P + eps);
    if (k < V) {
      a1 += P * r[i];
      a2 += xh * r[i];
    }
  }
  a1 = block_sum(a1, red);
  a2 = block_sum(a2, red);
  const float gc = -Qg * c.b_t * c.a_p * inv_dp;  // generic g0 factor: g0_k = gc * xh_k / (P_k + eps)
  float s1 = Qg * a1, g0s = gc * a2;
  {
    const long ks[2] = {xt, x0};
    const float xs[2] = {xhat_xt, xhat_x0};
    for (int j = 0; j < (xt == x0 ? 1 : 2); ++j) {
      float P, Q, M;
      special(ks[j], xs[j], P, Q, M);
      const float Pg = generic_P(xs[j]);
      s1 += Q * P / (P + eps) - Qg * Pg / (Pg + eps);
      g0s += -Q * M * c.a_p / (P + eps) * inv_dp * xs[j] - gc * xs[j] / (Pg + eps);
    }
  }
  const float gxt = c.a_t * s1 * inv_dp;
  const float G = g0s + xhat_xt * gxt;
  const float wr = w[row] * (gscale ? gscale[0] : 1.f);
  OT* out = dz + row * V;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const long k = tid + 256L * i;
    if (k < V) {
      const float xh = v[i];
      float g = gc * r[i];
      if (k == xt || k == x0) {
        float P, Q, M;
        special(k, xh, P, Q, M);
        g = -Q * M * c.a_p / (P + eps) * inv_dp + (k == xt ? gxt : 0.f);
      }
      st<OT>(out + k, wr * xh * (g - G));
    }
  }
}

// Lane partner of all-reduce step S (0..5) on the VALU instead of a ds_bpermute per step (__shfl_xor): quad_perm
// [1,0,3,2] and [2,3,0,1], then row_half_mirror (quad <-> quad within 8 lanes) and row_mirror (8 <-> 8 within 16),
// which pair whole groups once every lane of a group holds the same value, then v_permlane16_swap / 32_swap.
template <int S>
__device__ __forceinline__ float xpartner(float v) {
  const int u = __float_as_int(v);
  if constexpr (S == 0) return __int_as_float(__builtin_amdgcn_mov_dpp(u, 0xB1, 0xF, 0xF, false));
  else if constexpr (S == 1) return __int_as_float(__builtin_amdgcn_mov_dpp(u, 0x4E, 0xF, 0xF, false));
  else if constexpr (S == 2) return __int_as_float(__builtin_amdgcn_mov_dpp(u, 0x141, 0xF, 0xF, false));
  else if constexpr (S == 3) return __int_as_float(__builtin_amdgcn_mov_dpp(u, 0x140, 0xF, 0xF, false));
  else if constexpr (S == 4) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)u, (unsigned)u, false, false);
    return __uint_as_float((threadIdx.x & 16) ? r[0] : r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)u, (unsigned)u, false, false);
    return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
  }
}
template <int B, int E, typename F>
__device__ __forceinline__ void kl_static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    kl_static_for<B + 1, E>(f);
  }
}

// Vectorised variant for V % 4 == 0 (the train step: V = 8000): 16-B loads, 8-B (bf16) / 16-B (f32) stores, the
// row max and sum in one block reduction (per-thread max, exp relative to it, rescaled once the row max is
// known), and the two backward sums in one. NV = float4 chunks per thread (V <= 1024 * NV).
__device__ __forceinline__ float2 block_maxsum(float m, float s, float* red) {
  // combine (m, s) pairs: m = max, s = sum of exp(v - m)
  kl_static_for<0, 6>([&](auto sc) {
    constexpr int S = decltype(sc)::value;
    const float mo = xpartner<S>(m), so = xpartner<S>(s);
    const float mn = fmaxf(m, mo);
    s = (mn == -INFINITY) ? 0.f : s * __expf(m - mn) + so * __expf(mo - mn);
    m = mn;
  });
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) { red[2 * w] = m; red[2 * w + 1] = s; }
  __syncthreads();
  float M = -INFINITY;
  for (int i = 0; i < nw; ++i) M = fmaxf(M, red[2 * i]);
  float S = 0.f;
  for (int i = 0; i < nw; ++i) S += red[2 * i + 1] * __expf(red[2 * i] - M);
  return make_float2(M, S);
}
__device__ __forceinline__ float2 block_sum2(float a, float b, float* red) {
  kl_static_for<0, 6>([&](auto sc) {
    constexpr int S = decltype(sc)::value;
    a += xpartner<S>(a);
    b += xpartner<S>(b);
  });
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) { red[2 * w] = a; red[2 * w + 1] = b; }
  __syncthreads();
  float A = 0.f, Bs = 0.f;
  for (int i = 0; i < nw; ++i) { A += red[2 * i]; Bs += red[2 * i + 1]; }
  return make_float2(A, Bs);
}

template <typename OT> __device__ __forceinline__ void st4(OT* p, float a, float b, float c, float d);
template <> __device__ __forceinline__ void st4<float>(float* p, float a, float b, float c, float d) {
  *(float4*)p = make_float4(a, b, c, d);
}
template <> __device__ __forceinline__ void st4<bf16_t>(bf16_t* p, float a, float b, float c, float d) {
  uint2 u;
  u.x = pk_bf16(a, b);
  u.y = pk_bf16(c, d);
  *(uint2*)p = u;
}

template <int NV, bool BWD, typename OT, int NT>
__global__ void __launch_bounds__(NT) kl4_kernel(const float* __restrict__ logits, const long* __restrict__ xt_,
                                                  const long* __restrict__ x0_, const long* __restrict__ t_,
                                                  const float* __restrict__ betas, const float* __restrict__ w,
                                                  const float* __restrict__ gscale, float* __restrict__ kl_tok,
                                                  OT* __restrict__ dz, long L, long V) {
  __shared__ float red[2 * (NT / 64)];
  const long row = blockIdx.x;
  const int tid = threadIdx.x;
  const float* z = logits + row * V;
  const long V4 = V >> 2;
  const long xt = xt_[row], x0 = x0_[row], tv = t_[row / L];
  const float eps = 1e-8f;
  const KlRow c = kl_consts(betas, tv, xt, x0, (float)V);
  const float zxt = z[xt], zx0 = z[x0];

  float v[NV][4];
  float mt = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const long q = tid + (long)NT * i;
    float4 f = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    if (q < V4) f = *(const float4*)(z + 4 * q);
    v[i][0] = f.x; v[i][1] = f.y; v[i][2] = f.z; v[i][3] = f.w;
    mt = fmaxf(mt, fmaxf(fmaxf(f.x, f.y), fmaxf(f.z, f.w)));
  }
  float st_ = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[i][j] = (mt == -INFINITY) ? 0.f : __expf(v[i][j] - mt);
      st_ += v[i][j];
    }
  const float2 ms = block_maxsum(mt, st_, red);
  const float mx = ms.x, inv_s = 1.f / ms.y;
  const float resc = (mt == -INFINITY) ? 0.f : __expf(mt - mx) * inv_s;  // this thread's exps -> probabilities
  const float xhat_xt = __expf(zxt - mx) * inv_s;
  const float xhat_x0 = __expf(zx0 - mx) * inv_s;
  const float dp = c.b_t + c.a_t * xhat_xt;
  const float inv_dp = 1.f / (dp + eps);
  const float Qg = c.b_t * c.b_p * c.inv_dq;
  auto special = [&](long k, float xh, float& P, float& Q, float& M) {
    M = c.b_t + (k == xt ? c.a_t : 0.f);
    Q = M * ((k == x0 ? c.a_p : 0.f) + c.b_p) * c.inv_dq;
    P = M * (c.a_p * xh + c.b_p) * inv_dp;
  };
  // generic P = b_t (a_p xh + b_p) / dp as one FMA on xh
  const float pa = c.b_t * c.a_p * inv_dp, pb = c.b_t * c.b_p * inv_dp;
  const long ks[2] = {xt, x0};
  const float xs[2] = {xhat_xt, xhat_x0};
  const int nsp = (xt == x0) ? 1 : 2;

  if (!BWD) {
    const float LQg = __logf(Qg + eps);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (tid + (long)NT * i < V4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += LQg - __logf(fmaf(pa, v[i][j] * resc, pb) + eps);
      }
    }
    acc = block_sum(acc, red);
    if (tid == 0) {
      float kl = Qg * acc;
      for (int j = 0; j < nsp; ++j) {
        float P, Q, M;
        special(ks[j], xs[j], P, Q, M);
        kl += Q * (__logf(Q + eps) - __logf(P + eps)) - Qg * (LQg - __logf(fmaf(pa, xs[j], pb) + eps));
      }
      kl_tok[row] = kl;
    }
    return;
  }
  // 1/(P+eps) is recomputed in the output pass instead of held (keeps the kernel at <= 64 VGPRs)
  float a1 = 0.f, a2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const bool ok = tid + (long)NT * i < V4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = v[i][j] * resc;
      v[i][j] = xh;
      const float P = fmaf(pa, xh, pb);
      const float r = __builtin_amdgcn_rcpf(P + eps);
      if (ok) {
        a1 += P * r;
        a2 += xh * r;
      }
    }
  }
  const float2 aa = block_sum2(a1, a2, red);
  const float gc = -Qg * c.b_t * c.a_p * inv_dp;  // generic g0 factor: g0_k = gc * xh_k / (P_k + eps)
  float s1 = Qg * aa.x, g0s = gc * aa.y;
  for (int j = 0; j < nsp; ++j) {
    float P, Q, M;
    special(ks[j], xs[j], P, Q, M);
    const float Pg = fmaf(pa, xs[j], pb);
    s1 += Q * P / (P + eps) - Qg * Pg / (Pg + eps);
    g0s += -Q * M * c.a_p / (P + eps) * inv_dp * xs[j] - gc * xs[j] / (Pg + eps);
  }
  const float gxt = c.a_t * s1 * inv_dp;
  const float G = g0s + xhat_xt * gxt;
  const float wr = w[row] * (gscale ? gscale[0] : 1.f);
  OT* out = dz + row * V;
  const int qxt = (int)(xt >> 2), qx0 = (int)(x0 >> 2), iv4 = (int)V4;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int q = tid + NT * i;
    if (q < iv4) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = wr * v[i][j] * (gc * __builtin_amdgcn_rcpf(fmaf(pa, v[i][j], pb) + eps) - G);
      if (q == qxt || q == qx0) {  // the float4 holding x_t and/or x0: exact per-index terms
        for (int j = 0; j < 4; ++j) {
          const long k = 4L * q + j;
          if (k == xt || k == x0) {
            float P, Q, M;
            special(k, v[i][j], P, Q, M);
            const float g = -Q * M * c.a_p / (P + eps) * inv_dp + (k == xt ? gxt : 0.f);
            o[j] = wr * v[i][j] * (g - G);
          }
        }
      }
      st4<OT>(out + 4 * q, o[0], o[1], o[2], o[3]);
    }
  }
}

// Fused forward + gradient (the train step's KL): ONE read of the fp32 logits row yields kl_tok[row] and the
// row's logits gradient w[row] * d kl_tok / d z (w = d loss / d kl_tok of the masked mean, computed here from the
// utterance's mask row: mask / (count + 1e-8) / B, or 1 / (L B) without a mask — kl_reduce's weights). The
// upstream scalar is applied afterwards by fddm_scale_if, which returns without touching memory when it is 1
// (the train step: loss = kl + ...). 393 MB of HBM per step at V = 8000, B*L = 8192 (f32 in, bf16 out) instead of
// 262 + 393 MB for the separate forward and backward passes.
__device__ __forceinline__ float4 block_sum4(float a, float b, float c, float d, float* red) {
  kl_static_for<0, 6>([&](auto sc) {
    constexpr int S = decltype(sc)::value;
    a += xpartner<S>(a);
    b += xpartner<S>(b);
    c += xpartner<S>(c);
    d += xpartner<S>(d);
  });
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) { red[4 * w] = a; red[4 * w + 1] = b; red[4 * w + 2] = c; red[4 * w + 3] = d; }
  __syncthreads();
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = 0; i < nw; ++i) { r.x += red[4 * i]; r.y += red[4 * i + 1]; r.z += red[4 * i + 2]; r.w += red[4 * i + 3]; }
  return r;
}

#ifndef KL_WPE
#define KL_WPE 4  // waves per SIMD the fused KL targets: 128 VGPRs (1: 132 VGPRs, 3 waves, 97 us; 4: 86 us; 5 spills: 127 us)
#endif
template <int NV, typename OT, int NT>
__global__ void __launch_bounds__(NT, KL_WPE) kl4_fused_kernel(const float* __restrict__ logits, const long* __restrict__ xt_,
                                                        const long* __restrict__ x0_, const long* __restrict__ t_,
                                                        const float* __restrict__ betas,
                                                        const unsigned char* __restrict__ mask,
                                                        float* __restrict__ kl_tok, OT* __restrict__ dz, long L, long V,
                                                        long B) {
  __shared__ float red[2 * (NT / 64) + 4 * (NT / 64)];
  const long row = blockIdx.x;
  const int tid = threadIdx.x;
  const float* z = logits + row * V;
  const long V4 = V >> 2;
  const long xt = xt_[row], x0 = x0_[row], b = row / L, tv = t_[b];
  const float eps = 1e-8f;
  const KlRow c = kl_consts(betas, tv, xt, x0, (float)V);
  const float zxt = z[xt], zx0 = z[x0];

  float v[NV][4];
  float mt = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const long q = tid + (long)NT * i;
    float4 f = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    if (q < V4) f = *(const float4*)(z + 4 * q);
    v[i][0] = f.x; v[i][1] = f.y; v[i][2] = f.z; v[i][3] = f.w;
    mt = fmaxf(mt, fmaxf(fmaxf(f.x, f.y), fmaxf(f.z, f.w)));
  }
  // exp(v - mt) as one exp2 of an FMA; a thread whose elements are all padding (-inf) has mt = -inf: subtracting 0
  // instead gives its exps exactly 0 without a select per element
  constexpr float L2E = 1.4426950408889634f;
  const float mtl = (mt == -INFINITY) ? 0.f : mt * L2E;
  float st_ = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[i][j] = __builtin_amdgcn_exp2f(fmaf(v[i][j], L2E, -mtl));
      st_ += v[i][j];
    }
  const float2 ms = block_maxsum(mt, st_, red);
  const float mx = ms.x, inv_s = 1.f / ms.y;
  const float resc = (mt == -INFINITY) ? 0.f : __expf(mt - mx) * inv_s;
  const float xhat_xt = __expf(zxt - mx) * inv_s;
  const float xhat_x0 = __expf(zx0 - mx) * inv_s;
  const float dp = c.b_t + c.a_t * xhat_xt;
  const float inv_dp = 1.f / (dp + eps);
  const float Qg = c.b_t * c.b_p * c.inv_dq;
  const float LQg = __logf(Qg + eps);
  auto special = [&](long k, float xh, float& P, float& Q, float& M) {
    M = c.b_t + (k == xt ? c.a_t : 0.f);
    Q = M * ((k == x0 ? c.a_p : 0.f) + c.b_p) * c.inv_dq;
    P = M * (c.a_p * xh + c.b_p) * inv_dp;
  };
  const float pa = c.b_t * c.a_p * inv_dp, pb = c.b_t * c.b_p * inv_dp, pbe = pb + eps;
  const long ks[2] = {xt, x0};
  const float xs[2] = {xhat_xt, xhat_x0};
  const int nsp = (xt == x0) ? 1 : 2;

  // one row pass: the KL's generic log terms and the gradient's two sums; the mask count of this utterance rides
  // in the same block reduction. Per element one exp (above), one rcp (kept in registers for the output pass) and a
  // quarter of a log: sum_k log(P_k + eps) is taken as log of the product of each float4's four factors (each >= eps =
  // 1e-8, so a product >= 1e-32 stays a normal f32). sum_k P_k / (P_k + eps) = V - eps sum_k 1 / (P_k + eps): one
  // add per element instead of a subtract and an FMA. Chunks whose every lane is inside the row skip the validity
  // selects (a uniform branch per chunk).
  float acc = 0.f, sr = 0.f, a2 = 0.f, cnt = 0.f;
  float r[NV][4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float prod = 1.f, sri = 0.f, a2i = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = v[i][j] * resc;
      v[i][j] = xh;
      const float Pe = fmaf(pa, xh, pbe);
      r[i][j] = __builtin_amdgcn_rcpf(Pe);
      prod *= Pe;
      sri += r[i][j];
      a2i = fmaf(xh, r[i][j], a2i);
    }
    // prod >= eps^4 = 1e-32, a normal f32: the raw log2 instruction (no denormal scaling), times ln 2
    const float lt = fmaf(-0.6931471805599453f, __builtin_amdgcn_logf(prod), 4.f * LQg);
    if ((long)NT * (i + 1) <= V4) {  // uniform: every lane's float4 is in the row
      acc += lt;
      sr += sri;
      a2 += a2i;
    } else if (tid + (long)NT * i < V4) {
      acc += lt;
      sr += sri;
      a2 += a2i;
    }
  }
  if (mask)
    for (long l = tid; l < L; l += NT) cnt += mask[b * L + l] ? 1.f : 0.f;
  const float4 sums0 = block_sum4(acc, sr, a2, cnt, red + 2 * (NT / 64));
  const float4 sums = make_float4(sums0.x, (float)V - eps * sums0.y, sums0.z, sums0.w);
  if (tid == 0) {
    float kl = Qg * sums.x;
    for (int j = 0; j < nsp; ++j) {
      float P, Q, M;
      special(ks[j], xs[j], P, Q, M);
      kl += Q * (__logf(Q + eps) - __logf(P + eps)) - Qg * (LQg - __logf(fmaf(pa, xs[j], pb) + eps));
    }
    kl_tok[row] = kl;
  }
  const float gc = -Qg * c.b_t * c.a_p * inv_dp;
  float s1 = Qg * sums.y, g0s = gc * sums.z;
  for (int j = 0; j < nsp; ++j) {
    float P, Q, M;
    special(ks[j], xs[j], P, Q, M);
    const float Pg = fmaf(pa, xs[j], pb);
    s1 += Q * P / (P + eps) - Qg * Pg / (Pg + eps);
    g0s += -Q * M * c.a_p / (P + eps) * inv_dp * xs[j] - gc * xs[j] / (Pg + eps);
  }
  const float gxt = c.a_t * s1 * inv_dp;
  const float G = g0s + xhat_xt * gxt;
  const float wr = mask ? ((mask[row] ? 1.f : 0.f) / (sums.w + eps) / (float)B) : 1.f / ((float)L * (float)B);
  const float wgc = wr * gc, wG = wr * G;
  OT* out = dz + row * V;
  const int qxt = (int)(xt >> 2), qx0 = (int)(x0 >> 2), iv4 = (int)V4;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int q = tid + NT * i;
    if (q < iv4) {
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = v[i][j] * fmaf(wgc, r[i][j], -wG);
      if (q == qxt || q == qx0) {
        for (int j = 0; j < 4; ++j) {
          const long k = 4L * q + j;
          if (k == xt || k == x0) {
            float P, Q, M;
            special(k, v[i][j], P, Q, M);
            const float g = -Q * M * c.a_p / (P + eps) * inv_dp + (k == xt ? gxt : 0.f);
            o[j] = wr * v[i][j] * (g - G);
          }
        }
      }
      st4<OT>(out + 4 * q, o[0], o[1], o[2], o[3]);
    }
  }
}

// x *= g[0] unless g[0] == 1 (then no memory is touched): the upstream gradient of a fused forward+gradient pass
template <typename T>
__global__ void __launch_bounds__(256) scale_if_kernel(T* __restrict__ x, const float* __restrict__ g, long n) {
  const float s = g[0];
  if (s == 1.f) return;
  const long n8 = n / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    if constexpr (sizeof(T) == 2) {
      uint4 u = ((uint4*)x)[i];
      unsigned* w = (unsigned*)&u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = __uint_as_float(w[k] << 16) * s, hi = __uint_as_float(w[k] & 0xffff0000u) * s;
        w[k] = pk_bf16(lo, hi);
      }
      ((uint4*)x)[i] = u;
    } else {
      float4* p = (float4*)x + 2 * i;
      float4 a = p[0], c = p[1];
      a.x *= s; a.y *= s; a.z *= s; a.w *= s;
      c.x *= s; c.y *= s; c.z *= s; c.w *= s;
      p[0] = a;
      p[1] = c;
    }
  }
  for (long i = 8 * n8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    if constexpr (sizeof(T) == 2) {
      unsigned short* h = (unsigned short*)x;
      const float f = __uint_as_float(((unsigned)h[i]) << 16) * s;
      h[i] = (unsigned short)(pk_bf16(f, 0.f) & 0xffffu);
    } else {
      x[i] *= s;
    }
  }
}

// softmax over rows of length V (fp32 in) -> T out
template <int NPT, typename OT>
__global__ void __launch_bounds__(256) softmax_rows_kernel(const float* __restrict__ x, OT* __restrict__ y, long V) {
  __shared__ float red[8];
  const long row = blockIdx.x;
  const int tid = threadIdx.x;
  const float* z = x + row * V;
  float v[NPT];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const long k = tid + 256L * i;
    v[i] = k < V ? z[k] : -INFINITY;
    mx = fmaxf(mx, v[i]);
  }
  mx = block_max(mx, red);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    v[i] = __expf(v[i] - mx);
    s += v[i];
  }
  s = block_sum(s, red);
  const float inv = 1.f / s;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const long k = tid + 256L * i;
    if (k < V) st<OT>(y + row * V + k, v[i] * inv);
  }
}

// dz = y * (dy - sum(y*dy)); y, dy in T; dz written as T or accumulated into f32
template <int NPT, typename T, typename OT>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                          OT* __restrict__ dz, long V, int accumulate) {
  __shared__ float red[8];
  const long row = blockIdx.x;
  const int tid = threadIdx.x;
  float yv[NPT], dv[NPT];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const long k = tid + 256L * i;
    yv[i] = k < V ? ld<T>(y + row * V + k) : 0.f;
    dv[i] = k < V ? ld<T>(dy + row * V + k) : 0.f;
    s += yv[i] * dv[i];
  }
  s = block_sum(s, red);
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const long k = tid + 256L * i;
    if (k < V) {
      float r = yv[i] * (dv[i] - s);
      OT* o = dz + row * V + k;
      if (accumulate) r += ld<OT>(o);
      st<OT>(o, r);
    }
  }
}

// bf16 logits-gradient hand-over of the L_fd step (functions.TextEmbedFn / KLFn / HeadFn):
// out = bf16( y * (dy - sum(y*dy)) + add ), y = softmax rows (bf16), dy (bf16), add = the KL's gradient (bf16).
// 8 elements per 16-B load, NV loads per thread, one block per row (V % 8 == 0).
template <int NV>
__global__ void __launch_bounds__(256) softmax_bwd_add_kernel(const bf16_t* __restrict__ y, const bf16_t* __restrict__ dy,
                                                              const bf16_t* __restrict__ add, bf16_t* __restrict__ out,
                                                              long V) {
  __shared__ float red[8];
  const long row = blockIdx.x;
  const int tid = threadIdx.x;
  const long V8 = V >> 3;
  uint4 yv[NV], dv[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const long q = tid + 256L * i;
    yv[i] = make_uint4(0u, 0u, 0u, 0u);
    dv[i] = yv[i];
    if (q < V8) {
      yv[i] = ((const uint4*)(y + row * V))[q];
      dv[i] = ((const uint4*)(dy + row * V))[q];
    }
    const unsigned* a = (const unsigned*)&yv[i];
    const unsigned* b = (const unsigned*)&dv[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s = fmaf(__uint_as_float(a[k] << 16), __uint_as_float(b[k] << 16), s);
      s = fmaf(__uint_as_float(a[k] & 0xffff0000u), __uint_as_float(b[k] & 0xffff0000u), s);
    }
  }
  s = block_sum(s, red);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const long q = tid + 256L * i;
    if (q >= V8) continue;
    const uint4 ad = ((const uint4*)(add + row * V))[q];
    const unsigned* a = (const unsigned*)&yv[i];
    const unsigned* b = (const unsigned*)&dv[i];
    const unsigned* c = (const unsigned*)&ad;
    uint4 o;
    unsigned* ov = (unsigned*)&o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = __uint_as_float(a[k] << 16) * (__uint_as_float(b[k] << 16) - s) + __uint_as_float(c[k] << 16);
      const float hi = __uint_as_float(a[k] & 0xffff0000u) * (__uint_as_float(b[k] & 0xffff0000u) - s) +
                       __uint_as_float(c[k] & 0xffff0000u);
      ov[k] = pk_bf16(lo, hi);
    }
    ((uint4*)(out + row * V))[q] = o;
  }
}

// x += (g[0] - 1) * y (bf16), skipped without memory traffic when g[0] == 1: the KL's upstream scalar applied to
// its share of a hand-over buffer that already holds x = text part + KL part
__global__ void __launch_bounds__(256) axpy_if_kernel(bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
                                                      const float* __restrict__ g, long n8) {
  const float c = g[0] - 1.f;
  if (g[0] == 1.f) return;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    uint4 u = ((uint4*)x)[i];
    const uint4 v = ((const uint4*)y)[i];
    unsigned* a = (unsigned*)&u;
    const unsigned* b = (const unsigned*)&v;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = __uint_as_float(a[k] << 16) + c * __uint_as_float(b[k] << 16);
      const float hi = __uint_as_float(a[k] & 0xffff0000u) + c * __uint_as_float(b[k] & 0xffff0000u);
      a[k] = pk_bf16(lo, hi);
    }
    ((uint4*)x)[i] = u;
  }
}

}  // namespace fddm

using namespace fddm;

FDDM_API int fddm_sample_q(const long* x0, const long* t, const unsigned* thr, long* xt, long B, long L, long K,
                           unsigned long long seed, unsigned long long stream, void* hs) {
  const long n = B * L;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sample_q_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)hs, x0, t, thr,
                     xt, B, L, K, (uint64_t)seed, (uint64_t)stream);
  return (int)hipGetLastError();
}

// forward: 256 threads x 2*NV float4 (measured faster than 512 threads); backward: 512 threads x NV float4
#define KL4_DISPATCH(NV)                                                                                            \
  if (V <= 2048L * NV) {                                                                                           \
    if (!bwd) {                                                                                                    \
      hipLaunchKernelGGL((kl4_kernel<2 * NV, false, float, 256>), dim3((unsigned)N), dim3(256), 0, s, logits, xt, \
                         x0, t, betas, w, gscale, kl_tok, (float*)nullptr, L, V);                                  \
    } else if (dz_dtype == FDDM_BF16) {                                                                            \
      hipLaunchKernelGGL((kl4_kernel<NV, true, bf16_t, 512>), dim3((unsigned)N), dim3(512), 0, s, logits, xt, x0, t,   \
                         betas, w, gscale, kl_tok, (bf16_t*)dz, L, V);                                             \
    } else {                                                                                                       \
      hipLaunchKernelGGL((kl4_kernel<NV, true, float, 512>), dim3((unsigned)N), dim3(512), 0, s, logits, xt, x0, t,    \
                         betas, w, gscale, kl_tok, (float*)dz, L, V);                                              \
    }                                                                                                              \
    return (int)hipGetLastError();                                                                                 \
  }

#define KL_DISPATCH(NPT)                                                                                            \
  if (V <= 256L * NPT) {                                                                                           \
    if (!bwd) {                                                                                                    \
      hipLaunchKernelGGL((kl_kernel<NPT, false, float>), dim3((unsigned)N), dim3(256), 0, s, logits, xt, x0, t,   \
                         betas, w, gscale, kl_tok, (float*)nullptr, L, V);                                         \
    } else if (dz_dtype == FDDM_BF16) {                                                                            \
      hipLaunchKernelGGL((kl_kernel<NPT, true, bf16_t>), dim3((unsigned)N), dim3(256), 0, s, logits, xt, x0, t,   \
                         betas, w, gscale, kl_tok, (bf16_t*)dz, L, V);                                             \
    } else {                                                                                                       \
      hipLaunchKernelGGL((kl_kernel<NPT, true, float>), dim3((unsigned)N), dim3(256), 0, s, logits, xt, x0, t,    \
                         betas, w, gscale, kl_tok, (float*)dz, L, V);                                              \
    }                                                                                                              \
    return (int)hipGetLastError();                                                                                 \
  }

static int kl_launch(int bwd, const float* logits, const long* xt, const long* x0, const long* t, const float* betas,
                     const float* w, const float* gscale, float* kl_tok, void* dz, int dz_dtype, long N, long L,
                     long V, void* hs) {
  if (N <= 0) return 0;
  hipStream_t s = (hipStream_t)hs;
  if (V % 4 == 0 && !(((uintptr_t)logits) & 15) && !(((uintptr_t)dz) & 15)) {
    KL4_DISPATCH(1)
    KL4_DISPATCH(4)
    KL4_DISPATCH(8)
    KL4_DISPATCH(16)
  }
  KL_DISPATCH(4)
  KL_DISPATCH(16)
  KL_DISPATCH(32)
  KL_DISPATCH(64)
  return (int)hipErrorInvalidValue;
}

FDDM_API int fddm_kl_fwd(const float* logits, const long* xt, const long* x0, const long* t, const float* betas,
                         float* kl_tok, long N, long L, long V, void* hs) {
  return kl_launch(0, logits, xt, x0, t, betas, nullptr, nullptr, kl_tok, nullptr, FDDM_F32, N, L, V, hs);
}

FDDM_API int fddm_kl_bwd(const float* logits, const long* xt, const long* x0, const long* t, const float* betas,
                         const float* w, const float* gscale, void* dz, int dz_dtype, long N, long L, long V,
                         void* hs) {
  return kl_launch(1, logits, xt, x0, t, betas, w, gscale, nullptr, dz, dz_dtype, N, L, V, hs);
}

#define SM_DISPATCH(NPT)                                                                                 \
  if (V <= 256L * NPT) {                                                                                \
    if (out_dtype == FDDM_BF16)                                                                         \
      hipLaunchKernelGGL((softmax_rows_kernel<NPT, bf16_t>), dim3((unsigned)N), dim3(256), 0, s, x,   \
                         (bf16_t*)y, V);                                                                \
    else                                                                                                \
      hipLaunchKernelGGL((softmax_rows_kernel<NPT, float>), dim3((unsigned)N), dim3(256), 0, s, x,    \
                         (float*)y, V);                                                                 \
    return (int)hipGetLastError();                                                                      \
  }

FDDM_API int fddm_softmax_rows(const float* x, void* y, int out_dtype, long N, long V, void* hs) {
  if (N <= 0) return 0;
  hipStream_t s = (hipStream_t)hs;
  SM_DISPATCH(4)
  SM_DISPATCH(16)
  SM_DISPATCH(32)
  SM_DISPATCH(64)
  return (int)hipErrorInvalidValue;
}

#define SMB_DISPATCH(NPT)                                                                                        \
  if (V <= 256L * NPT) {                                                                                        \
    if (dtype == FDDM_BF16)                                                                                     \
      hipLaunchKernelGGL((softmax_bwd_kernel<NPT, bf16_t, float>), dim3((unsigned)N), dim3(256), 0, s,         \
                         (const bf16_t*)y, (const bf16_t*)dy, dz, V, accumulate);                               \
    else                                                                                                        \
      hipLaunchKernelGGL((softmax_bwd_kernel<NPT, float, float>), dim3((unsigned)N), dim3(256), 0, s,          \
                         (const float*)y, (const float*)dy, dz, V, accumulate);                                 \
    return (int)hipGetLastError();                                                                              \
  }

// dz (f32) = y*(dy - sum(y*dy)) [+ dz if accumulate]
FDDM_API int fddm_softmax_bwd_rows(const void* y, const void* dy, float* dz, int dtype, long N, long V, int accumulate,
                                   void* hs) {
  if (N <= 0) return 0;
  hipStream_t s = (hipStream_t)hs;
  SMB_DISPATCH(4)
  SMB_DISPATCH(16)
  SMB_DISPATCH(32)
  SMB_DISPATCH(64)
  return (int)hipErrorInvalidValue;
}

#define KLF_LAUNCH(NV, NT)                                                                                        \
  if (V <= 4L * NT * NV) {                                                                                       \
    if (dz_dtype == FDDM_BF16)                                                                                   \
      hipLaunchKernelGGL((kl4_fused_kernel<NV, bf16_t, NT>), dim3((unsigned)N), dim3(NT), 0, s, logits, xt, x0,  \
                         t, betas, mask, kl_tok, (bf16_t*)dz, L, V, N / L);                                      \
    else                                                                                                         \
      hipLaunchKernelGGL((kl4_fused_kernel<NV, float, NT>), dim3((unsigned)N), dim3(NT), 0, s, logits, xt, x0,   \
                         t, betas, mask, kl_tok, (float*)dz, L, V, N / L);                                       \
    return (int)hipGetLastError();                                                                               \
  }

// kl_tok[N] and dz[N][V] = w * d kl_tok / d logits in one pass (w: the masked-mean weights of fddm_kl_reduce)
FDDM_API int fddm_kl_fused(const float* logits, const long* xt, const long* x0, const long* t, const float* betas,
                           const unsigned char* mask, float* kl_tok, void* dz, int dz_dtype, long N, long L, long V,
                           void* hs) {
  if (N <= 0) return 0;
  if (L <= 0 || N % L || V % 4 || (((uintptr_t)logits) & 15) || (((uintptr_t)dz) & 15)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)hs;
  // 256-thread rows (measured against 128 / 1024, round 2); 512 threads for vocabularies beyond 16 x 4 x 256
  KLF_LAUNCH(2, 256)
#ifdef KL_PREFER512  // timing variant (tools/build_variant.sh): 512-thread rows from V > 2048
  KLF_LAUNCH(4, 512)
#endif
  KLF_LAUNCH(8, 256)
  KLF_LAUNCH(16, 256)
  KLF_LAUNCH(1, 512)
  KLF_LAUNCH(4, 512)
  KLF_LAUNCH(8, 512)
  KLF_LAUNCH(16, 512)
  return (int)hipErrorInvalidValue;
}

// x[n] *= g[0] on the device, skipped (no memory traffic) when g[0] == 1
FDDM_API int fddm_scale_if(void* x, int dtype, const float* g, long n, void* hs) {
  if (n <= 0) return 0;
  if (((uintptr_t)x) & 15) return (int)hipErrorInvalidValue;
  const long want = (n / 8 + 255) / 256 + 1;
  const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
  if (dtype == FDDM_BF16)
    hipLaunchKernelGGL(scale_if_kernel<bf16_t>, dim3(grid), dim3(256), 0, (hipStream_t)hs, (bf16_t*)x, g, n);
  else
    hipLaunchKernelGGL(scale_if_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)hs, (float*)x, g, n);
  return (int)hipGetLastError();
}

// out (bf16) = y * (dy - rowsum(y*dy)) + add: y, dy, add, out bf16 [N][V], V % 8 == 0 (out may alias add)
FDDM_API int fddm_softmax_bwd_add_bf16(const void* y, const void* dy, const void* add, void* out, long N, long V,
                                       void* hs) {
  if (N <= 0) return 0;
  if (V % 8 || ((((uintptr_t)y) | ((uintptr_t)dy) | ((uintptr_t)add) | ((uintptr_t)out)) & 15))
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)hs;
#define SMBA(NV)                                                                                            \
  if (V <= 2048L * NV) {                                                                                   \
    hipLaunchKernelGGL(softmax_bwd_add_kernel<NV>, dim3((unsigned)N), dim3(256), 0, s, (const bf16_t*)y,   \
                       (const bf16_t*)dy, (const bf16_t*)add, (bf16_t*)out, V);                           \
    return (int)hipGetLastError();                                                                        \
  }
  SMBA(1)
  SMBA(2)
  SMBA(4)
  SMBA(8)
  SMBA(16)
#undef SMBA
  return (int)hipErrorInvalidValue;
}

// x += (g[0] - 1) * y over n bf16 elements (n % 8 == 0); no memory traffic when g[0] == 1
FDDM_API int fddm_axpy_if_bf16(void* x, const void* y, const float* g, long n, void* hs) {
  if (n <= 0) return 0;
  if (n % 8 || ((((uintptr_t)x) | ((uintptr_t)y)) & 15)) return (int)hipErrorInvalidValue;
  const long want = (n / 8 + 255) / 256;
  const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
  hipLaunchKernelGGL(axpy_if_kernel, dim3(grid), dim3(256), 0, (hipStream_t)hs, (bf16_t*)x, (const bf16_t*)y, g, n / 8);
  return (int)hipGetLastError();
}
