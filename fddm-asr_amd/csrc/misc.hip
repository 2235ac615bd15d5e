// HBM-bound helper kernels of the train step: RoPE, token embedding, column sums, casts.
#include "common.h"
#include <algorithm>

namespace fddm {

// RoPE (models/denoise_decoder.py:42-53), applied to the full-width block input:
//   out[i]   = x[2i]*cos[p][2i] - x[2i+1]*sin[p][2i+1]
//   out[h+i] = x[2i]*sin[p][2i] + x[2i+1]*cos[p][2i+1]       (h = d/2, p = position)
// cos/sin tables [L][d] are the reference's emb.cos()/emb.sin() (computed once on the host).
// Vectorised (d % 8 == 0, N*d < 2^31): a thread owns i = 4q..4q+3 of one row — two float4 of x / cos / sin, 4
// outputs to each half; 32-bit index arithmetic (the 64-bit divisions of a scalar kernel cost more than its bytes).
template <typename OT>
__device__ __forceinline__ void st4v(OT* p, float a, float b, float c, float d_) {
  if constexpr (sizeof(OT) == 2) {
    uint2 u;
    u.x = pk_bf16(a, b);
    u.y = pk_bf16(c, d_);
    *(uint2*)p = u;
  } else {
    *(float4*)p = make_float4(a, b, c, d_);
  }
}
template <typename OT>
__global__ void __launch_bounds__(256) rope_fwd_kernel(const float* __restrict__ x, const float* __restrict__ cs,
                                                       const float* __restrict__ sn, OT* __restrict__ out, int N, int L,
                                                       int d) {
  const int h = d / 2, nq = h / 4;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * nq) return;
  const int r = e / nq, q = e - r * nq, p = r % L;
  const float* xr = x + (long)r * d + 8 * q;
  const float4 xa = *(const float4*)xr, xb = *(const float4*)(xr + 4);
  const float4 ca = *(const float4*)(cs + (long)p * d + 8 * q), cb = *(const float4*)(cs + (long)p * d + 8 * q + 4);
  const float4 sa = *(const float4*)(sn + (long)p * d + 8 * q), sb = *(const float4*)(sn + (long)p * d + 8 * q + 4);
  OT* o = out + (long)r * d;
  st4v<OT>(o + 4 * q, xa.x * ca.x - xa.y * sa.y, xa.z * ca.z - xa.w * sa.w, xb.x * cb.x - xb.y * sb.y,
           xb.z * cb.z - xb.w * sb.w);
  st4v<OT>(o + h + 4 * q, xa.x * sa.x + xa.y * ca.y, xa.z * sa.z + xa.w * ca.w, xb.x * sb.x + xb.y * cb.y,
           xb.z * sb.z + xb.w * cb.w);
}

// dx += RoPE^T(dy): a thread owns i = 4q..4q+3 of one row (dx elements 8q..8q+7)
__global__ void __launch_bounds__(256) rope_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ cs,
                                                       const float* __restrict__ sn, float* __restrict__ dx, int N,
                                                       int L, int d) {
  const int h = d / 2, nq = h / 4;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * nq) return;
  const int r = e / nq, q = e - r * nq, p = r % L;
  const float4 a = *(const float4*)(dy + (long)r * d + 4 * q), b = *(const float4*)(dy + (long)r * d + h + 4 * q);
  const float4 ca = *(const float4*)(cs + (long)p * d + 8 * q), cb = *(const float4*)(cs + (long)p * d + 8 * q + 4);
  const float4 sa = *(const float4*)(sn + (long)p * d + 8 * q), sb = *(const float4*)(sn + (long)p * d + 8 * q + 4);
  float* xr = dx + (long)r * d + 8 * q;
  float4 u = *(float4*)xr, v = *(float4*)(xr + 4);
  u.x += a.x * ca.x + b.x * sa.x;
  u.y += -a.x * sa.y + b.x * ca.y;
  u.z += a.y * ca.z + b.y * sa.z;
  u.w += -a.y * sa.w + b.y * ca.w;
  v.x += a.z * cb.x + b.z * sb.x;
  v.y += -a.z * sb.y + b.z * cb.y;
  v.z += a.w * cb.z + b.w * sb.z;
  v.w += -a.w * sb.w + b.w * cb.w;
  *(float4*)xr = u;
  *(float4*)(xr + 4) = v;
}

// x[r] = E[tok[r]] + tbias[r / L]   (models/denoise_decoder.py:254, 272-274): a thread owns 8 consecutive columns
template <typename OT>
__global__ void __launch_bounds__(256) embed_fwd_kernel(const long* __restrict__ tok, const float* __restrict__ E,
                                                        const float* __restrict__ tbias, float* __restrict__ out,
                                                        OT* __restrict__ out_t, int N, int L, int d) {
  const int nc = d / 8;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * nc) return;
  const int r = e / nc, c = 8 * (e - r * nc);
  const float* src = E + tok[r] * (long)d + c;
  float4 a = *(const float4*)src, b = *(const float4*)(src + 4);
  if (tbias) {
    const float* tb = tbias + (long)(r / L) * d + c;
    const float4 ta = *(const float4*)tb, tb4 = *(const float4*)(tb + 4);
    a.x += ta.x; a.y += ta.y; a.z += ta.z; a.w += ta.w;
    b.x += tb4.x; b.y += tb4.y; b.z += tb4.z; b.w += tb4.w;
  }
  const long o = (long)r * d + c;
  if (out) {
    *(float4*)(out + o) = a;
    *(float4*)(out + o + 4) = b;
  }
  if (out_t) {
    st4v<OT>(out_t + o, a.x, a.y, a.z, a.w);
    st4v<OT>(out_t + o + 4, b.x, b.y, b.z, b.w);
  }
}

// Scalar forms (any d, unaligned tensors): one element per thread.
template <typename OT>
__global__ void rope_fwd_scalar(const float* __restrict__ x, const float* __restrict__ cs, const float* __restrict__ sn,
                                OT* __restrict__ out, long N, long L, long d) {
  const long h = d / 2;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * h) return;
  const long r = e / h, i = e % h, p = r % L;
  const float x1 = x[r * d + 2 * i], x2 = x[r * d + 2 * i + 1];
  const float* C = cs + p * d;
  const float* S = sn + p * d;
  st<OT>(out + r * d + i, x1 * C[2 * i] - x2 * S[2 * i + 1]);
  st<OT>(out + r * d + h + i, x1 * S[2 * i] + x2 * C[2 * i + 1]);
}

// dx += RoPE^T(dy)
__global__ void rope_bwd_scalar(const float* __restrict__ dy, const float* __restrict__ cs, const float* __restrict__ sn,
                                float* __restrict__ dx, long N, long L, long d) {
  const long h = d / 2;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * h) return;
  const long r = e / h, i = e % h, p = r % L;
  const float a = dy[r * d + i], b = dy[r * d + h + i];
  const float* C = cs + p * d;
  const float* S = sn + p * d;
  dx[r * d + 2 * i] += a * C[2 * i] + b * S[2 * i];
  dx[r * d + 2 * i + 1] += -a * S[2 * i + 1] + b * C[2 * i + 1];
}

// x[r] = E[tok[r]] + tbias[r / L]   (models/denoise_decoder.py:254, 272-274)
template <typename OT>
__global__ void embed_fwd_scalar(const long* __restrict__ tok, const float* __restrict__ E,
                                 const float* __restrict__ tbias, float* __restrict__ out, OT* __restrict__ out_t, long N,
                                 long L, long d) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N * d) return;
  const long r = e / d, c = e % d;
  float v = E[tok[r] * d + c];
  if (tbias) v += tbias[(r / L) * d + c];
  if (out) out[e] = v;
  if (out_t) st<OT>(out_t + e, v);
}

// dE[tok[r]] += dx[r] (skip padding_idx rows), dtb[b] += sum_l dx[b,l]  — caller zeroes outputs.
// One block = EB_ROWS rows x d columns: the rows' token ids are wave-uniform scalar loads, each thread loads its
// columns of all EB_ROWS rows before the first atomic (one exposed load latency per block instead of one per row),
// then issues the row atomics (no return value) and one atomic per batch run for dtb. 8 rows per block: 1024
// blocks at the decoder's 8192 tokens (was 32 rows with a dependent load per row: 53 us at C2).
constexpr int EB_ROWS = 8;
__global__ void __launch_bounds__(256) embed_bwd_kernel(const long* __restrict__ tok, const float* __restrict__ dx,
                                                        float* __restrict__ dE, float* __restrict__ dtb, long N, long L,
                                                        long d, long pad_id) {
  const long r0 = (long)blockIdx.x * EB_ROWS;
  const int nr = (int)min((long)EB_ROWS, N - r0);
  long tk[EB_ROWS];
#pragma unroll
  for (int j = 0; j < EB_ROWS; ++j) tk[j] = j < nr ? tok[r0 + j] : pad_id;
  for (long c = threadIdx.x; c < d; c += blockDim.x) {
    float g[EB_ROWS];
#pragma unroll
    for (int j = 0; j < EB_ROWS; ++j) g[j] = dx[min(r0 + j, N - 1) * d + c];
    if (dE) {
#pragma unroll
      for (int j = 0; j < EB_ROWS; ++j)
        if (j < nr && tk[j] != pad_id) atomicAdd(dE + tk[j] * d + c, g[j]);
    }
    if (dtb) {
      long cur_b = r0 / L;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < EB_ROWS; ++j) {
        if (j < nr) {
          const long b = (r0 + j) / L;
          if (b != cur_b) {
            atomicAdd(dtb + cur_b * d + c, acc);
            acc = 0.f;
            cur_b = b;
          }
          acc += g[j];
        }
      }
      atomicAdd(dtb + cur_b * d + c, acc);
    }
  }
}

// out[n] += sum_m X[m][n]   (bias gradients): thread = 8 consecutive columns x a 64-row slab, one
// vector load per row, then 8 atomics (caller zeroes `out`)
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ X, float* __restrict__ out, long M, long N,
                                                     long ldx, long rows_per_block) {
  const long ncg = (N + 7) / 8;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long cg = tid % ncg, rc = tid / ncg;
  const long n0 = cg * 8;
  const long m0 = rc * rows_per_block;
  if (m0 >= M) return;
  const long m1 = min(M, m0 + rows_per_block);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (n0 + 8 <= N && ((ldx * sizeof(T)) % 16 == 0) && ((((uintptr_t)X) & 15) == 0)) {
#pragma unroll 4
    for (long m = m0; m < m1; ++m) {
      const T* p = X + m * ldx + n0;
      if constexpr (sizeof(T) == 2) {
        const uint4 u = *(const uint4*)p;
        const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[2 * i] += __uint_as_float(w[i] << 16);
          acc[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
        }
      } else {
        const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
      }
    }
  } else {
    for (long m = m0; m < m1; ++m)
      for (int i = 0; i < 8 && n0 + i < N; ++i) acc[i] += ld<T>(X + m * ldx + n0 + i);
  }
  for (int i = 0; i < 8 && n0 + i < N; ++i) atomicAdd(out + n0 + i, acc[i]);
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const float4 v = *(const float4*)(x + i);
    y[i] = f2bf(v.x); y[i + 1] = f2bf(v.y); y[i + 2] = f2bf(v.z); y[i + 3] = f2bf(v.w);
  } else {
    for (long j = i; j < n; ++j) y[j] = f2bf(x[j]);
  }
}

__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = bf2f(x[i]);
}

}  // namespace fddm

using namespace fddm;

static inline dim3 g1(long n, int bs = 256) { return dim3((unsigned)((n + bs - 1) / bs)); }

// the vectorised kernels: d % 8 == 0, 32-bit element indices, 16-B aligned tensors (null pointers allowed)
static bool vec_ok(long d, long N, std::initializer_list<const void*> ps) {
  if (d % 8 || N * d >= (1L << 31)) return false;
  for (const void* p : ps)
    if (((uintptr_t)p) & 15) return false;
  return true;
}

FDDM_API int fddm_rope_fwd(int out_dtype, const float* x, const float* cs, const float* sn, void* out, long N, long L,
                           long d, void* hs) {
  if (N <= 0) return 0;
  if (d % 2) return (int)hipErrorInvalidValue;
  const long n = N * (d / 2);
  if (vec_ok(d, N, {x, cs, sn, out})) {
    const long nv = N * (d / 8);
    if (out_dtype == FDDM_BF16)
      hipLaunchKernelGGL((rope_fwd_kernel<bf16_t>), g1(nv), dim3(256), 0, (hipStream_t)hs, x, cs, sn, (bf16_t*)out,
                         (int)N, (int)L, (int)d);
    else
      hipLaunchKernelGGL((rope_fwd_kernel<float>), g1(nv), dim3(256), 0, (hipStream_t)hs, x, cs, sn, (float*)out,
                         (int)N, (int)L, (int)d);
    return (int)hipGetLastError();
  }
  if (out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((rope_fwd_scalar<bf16_t>), g1(n), dim3(256), 0, (hipStream_t)hs, x, cs, sn, (bf16_t*)out, N, L, d);
  else
    hipLaunchKernelGGL((rope_fwd_scalar<float>), g1(n), dim3(256), 0, (hipStream_t)hs, x, cs, sn, (float*)out, N, L, d);
  return (int)hipGetLastError();
}

FDDM_API int fddm_rope_bwd(const float* dy, const float* cs, const float* sn, float* dx, long N, long L, long d,
                           void* hs) {
  if (N <= 0) return 0;
  const long n = N * (d / 2);
  if (vec_ok(d, N, {dy, cs, sn, dx}))
    hipLaunchKernelGGL(rope_bwd_kernel, g1(N * (d / 8)), dim3(256), 0, (hipStream_t)hs, dy, cs, sn, dx, (int)N, (int)L,
                       (int)d);
  else
    hipLaunchKernelGGL(rope_bwd_scalar, g1(n), dim3(256), 0, (hipStream_t)hs, dy, cs, sn, dx, N, L, d);
  return (int)hipGetLastError();
}

FDDM_API int fddm_embed_fwd(int out_dtype, const long* tok, const float* E, const float* tbias, float* out, void* out_t,
                            long N, long L, long d, void* hs) {
  if (N <= 0) return 0;
  if (vec_ok(d, N, {E, tbias, out, out_t})) {
    if (out_dtype == FDDM_BF16)
      hipLaunchKernelGGL((embed_fwd_kernel<bf16_t>), g1(N * (d / 8)), dim3(256), 0, (hipStream_t)hs, tok, E, tbias, out,
                         (bf16_t*)out_t, (int)N, (int)L, (int)d);
    else
      hipLaunchKernelGGL((embed_fwd_kernel<float>), g1(N * (d / 8)), dim3(256), 0, (hipStream_t)hs, tok, E, tbias, out,
                         (float*)out_t, (int)N, (int)L, (int)d);
    return (int)hipGetLastError();
  }
  if (out_dtype == FDDM_BF16)
    hipLaunchKernelGGL((embed_fwd_scalar<bf16_t>), g1(N * d), dim3(256), 0, (hipStream_t)hs, tok, E, tbias, out,
                       (bf16_t*)out_t, N, L, d);
  else
    hipLaunchKernelGGL((embed_fwd_scalar<float>), g1(N * d), dim3(256), 0, (hipStream_t)hs, tok, E, tbias, out,
                       (float*)out_t, N, L, d);
  return (int)hipGetLastError();
}

FDDM_API int fddm_embed_bwd(const long* tok, const float* dx, float* dE, float* dtb, long N, long L, long d, long pad_id,
                            void* hs) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)((N + EB_ROWS - 1) / EB_ROWS)), dim3(256), 0, (hipStream_t)hs, tok, dx, dE, dtb,
                     N, L, d, pad_id);
  return (int)hipGetLastError();
}

FDDM_API int fddm_colsum(int dtype, const void* X, float* out, long M, long N, long ldx, void* hs) {
  if (M <= 0 || N <= 0) return 0;
  const long ncg = (N + 7) / 8;
  long chunks = std::max(1L, std::min((M + 7) / 8, (65536 + ncg - 1) / ncg));
  const long rpb = (M + chunks - 1) / chunks;
  chunks = (M + rpb - 1) / rpb;
  dim3 grid((unsigned)((ncg * chunks + 255) / 256));
  if (dtype == FDDM_BF16)
    hipLaunchKernelGGL((colsum_kernel<bf16_t>), grid, dim3(256), 0, (hipStream_t)hs, (const bf16_t*)X, out, M, N, ldx, rpb);
  else
    hipLaunchKernelGGL((colsum_kernel<float>), grid, dim3(256), 0, (hipStream_t)hs, (const float*)X, out, M, N, ldx, rpb);
  return (int)hipGetLastError();
}

FDDM_API int fddm_cast(int src_dtype, int dst_dtype, const void* x, void* y, long n, void* hs) {
  if (n <= 0) return 0;
  if (src_dtype == FDDM_F32 && dst_dtype == FDDM_BF16)
    hipLaunchKernelGGL(cast_f32_bf16_kernel, g1((n + 3) / 4), dim3(256), 0, (hipStream_t)hs, (const float*)x,
                       (bf16_t*)y, n);
  else if (src_dtype == FDDM_BF16 && dst_dtype == FDDM_F32)
    hipLaunchKernelGGL(cast_bf16_f32_kernel, g1(n), dim3(256), 0, (hipStream_t)hs, (const bf16_t*)x, (float*)y, n);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

FDDM_API const char* fddm_error_string(int code) { return hipGetErrorString((hipError_t)code); }

FDDM_API int fddm_abi_version() { return 6; }  // 6: fddm_attn_bwd workspace 64 B*H*LqP floats (fused backward)

// HIP-graph replays of the train step (fddm_hip.graphs.StepGraphs): launches enqueued while `off` is set read their
// dropout seed as seed + *off (common.h eff_seed); null restores plain seeds. Returns the previous setting's state
// (0 = none was set, 1 = one was).
FDDM_API int fddm_set_seed_offset(const unsigned long long* off) {
  const int had = g_seed_off != nullptr;
  g_seed_off = (const uint64_t*)off;
  return had;
}
