// Small per-batch kernels of the decoder step (rows = the batch, B <= 64): the time-embedding MLP and the FiLM
// projections (models/denoise_decoder.py:74-119, 179-186, 272-274), the pooled acoustic condition (:185), and the
// KL term's masked batch reduction (train.py:247-253). Each is a handful of small launches on the main stream in
// place of ~40 framework launches (sinusoid ops, BLAS calls on 32-row operands, bias sums, concatenations,
// masked means). All arithmetic is fp32 (the reference's precision for these ops).
#include "common.h"
#include <cstdlib>

namespace fddm {
namespace small {

constexpr int MAXJ = 16;  // jobs per launch

// ------------------------------------------------------------------------------------------ pooled mean
// out[b][j] = mean_s x[b][s][j]. Block = one utterance x 64 columns: 8 column groups of 8 (bf16: one 16-B load per
// row; f32: two) x 32 row slices, each thread's loads independent (unrolled by 4); the 32 slice sums combine in LDS
// in a fixed order (deterministic). 8x the blocks of a 512-column block: at B 32, d 512 the 32 blocks of that layout
// kept 32 CUs busy for ~57 us beside the encoder, 256 blocks spread the 16 MB over the chip.
constexpr int RM_SL = 32;  // row slices per block
// 8 consecutive elements (bf16: one 16-B load, f32: two) as f32
template <typename T>
__device__ __forceinline__ void rm_ld8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const uint4 u = *(const uint4*)p;
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <typename T>
__global__ void __launch_bounds__(256) rows_mean_kernel(const T* __restrict__ x, float* __restrict__ out, long S,
                                                        long d) {
  __shared__ float part[RM_SL][64 + 4];
  const int cg = threadIdx.x & 7, sl = threadIdx.x >> 3;
  const long b = blockIdx.y, j0 = (long)blockIdx.x * 64 + cg * 8;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  if (j0 + 8 <= d && (d % 8) == 0) {
    const T* base = x + b * S * d + j0;
    long s = sl;
    for (; s + 3 * RM_SL < S; s += 4 * RM_SL) {
      float v[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) rm_ld8<T>(base + (s + RM_SL * q) * d, v[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[q][e];
    }
    for (; s < S; s += RM_SL) {
      float v[8];
      rm_ld8<T>(base + s * d, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  } else {
    for (int e = 0; e < 8; ++e)
      if (j0 + e < d)
        for (long s = sl; s < S; s += RM_SL) acc[e] += ld<T>(x + (b * S + s) * d + j0 + e);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[sl][cg * 8 + e] = acc[e];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
    const long j = (long)blockIdx.x * 64 + c;
    if (j < d) {
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < RM_SL; ++q) a += part[q][c];
      out[b * d + j] = a / (float)S;
    }
  }
}

// ------------------------------------------------------------------------------------------ time embedding
// emb[b] = [sin(t f), cos(t f)], f_k = exp(-k * ln(max_steps) / (half - 1)) (SinusoidalTimeEmbedding.forward,
// models/denoise_decoder.py:108-116: torch.linspace(log 1, log max_steps, half) * -1 then exp; odd d pads a 0)
__global__ void time_embed_kernel(const long* __restrict__ t, float* __restrict__ emb, long B, long d,
                                  float log_max) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * d) return;
  const long b = e / d, k = e % d, half = d / 2;
  float v = 0.f;
  if (k < 2 * half) {
    const long kk = k < half ? k : k - half;
    // torch.linspace(start, end, steps): start + i * step with step = (end - start) / (steps - 1)
    const float step = half > 1 ? log_max / (float)(half - 1) : 0.f;
    const float lin = (kk < half / 2) ? (float)kk * step : log_max - (float)(half - 1 - kk) * step;
    const float f = expf(-lin);
    const float a = (float)t[b] * f;
    v = k < half ? sinf(a) : cosf(a);
  }
  emb[e] = v;
}

// ------------------------------------------------------------------------------------------ linear family
// Job j: out_j[r][n] = act( sum_k in[r][k] * W_j(n, k) + b_j[n] ),  W_j(n, k) = W_j[n*ldw + k] (TW = 0) or
// W_j[k*ldw + n] (TW = 1, i.e. in @ W).  act 0: none; 1: out = pre, out2 = silu(pre); 2: out = acc * silu'(aux[r][n])
struct LinJobs {
  const float* W[MAXJ];
  const float* b[MAXJ];
  float* out[MAXJ];
  float* out2[MAXJ];
};

constexpr int LNC = 8;  // output columns per block

// Round 2: 1024 threads per block = 4 K-quarters x (32 rows x 8 columns); K in chunks of 512 staged in LDS (the
// decoder's conditioning Linears have K = d_model: one chunk), each thread a 128-long FMA chain over its quarter,
// the four partial sums added through LDS in a fixed order. A [32, 512] x [512, 512] Linear: 11.7 us with the
// round-1 256-thread block (512-long chains, four chunk rounds), the 12 FiLM projections 28 us (tools/cond_bench.py).
constexpr int LKC2 = 512, LKQ = LKC2 / 4;
template <bool TW>
__global__ void __launch_bounds__(1024) linear4_kernel(const float* __restrict__ in, long ldi, LinJobs J, long ldw,
                                                       long ldo, const float* __restrict__ aux, long R, long N, long K,
                                                       int act) {
  __shared__ float Is[32][LKC2 + 4];
  __shared__ float Ws[LNC][LKC2 + 4];
  const int tid = threadIdx.x, kq = tid >> 8, t8 = tid & 255, c = t8 & (LNC - 1), rr = t8 >> 3;
  const long n0 = (long)blockIdx.x * LNC, r0 = (long)blockIdx.z * 32;
  const int j = blockIdx.y;
  const float* W = J.W[j];
  float4 pin[4];
  float pw[4];
  auto fetch = [&](long k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 1024 * q;          // 4096 float4 slots = 32 rows x 128 float4
      const int ri = e >> 7, kq4 = e & 127;
      const long r = r0 + ri, k = k0 + 4 * kq4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < R) {
        const float* src = in + r * ldi + k;
        if (k + 3 < K && ((((uintptr_t)src) & 15) == 0)) {
          v = *(const float4*)src;
        } else {
          if (k < K) v.x = src[0];
          if (k + 1 < K) v.y = src[1];
          if (k + 2 < K) v.z = src[2];
          if (k + 3 < K) v.w = src[3];
        }
      }
      pin[q] = v;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 1024 * q;          // 4096 W elements = 8 columns x 512 k
      int cc, kk;
      if (TW) { kk = e >> 3; cc = e & 7; } else { cc = e >> 9; kk = e & 511; }
      const long n = n0 + cc, k = k0 + kk;
      pw[q] = (n < N && k < K) ? (TW ? W[k * ldw + n] : W[n * ldw + k]) : 0.f;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 1024 * q;
      *(float4*)&Is[e >> 7][4 * (e & 127)] = pin[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 1024 * q;
      if (TW) Ws[e & 7][e >> 3] = pw[q];
      else Ws[e >> 9][e & 511] = pw[q];
    }
  };
  float acc = 0.f;
  fetch(0);
  for (long k0 = 0; k0 < K; k0 += LKC2) {
    __syncthreads();
    stash();
    __syncthreads();
    if (k0 + LKC2 < K) fetch(k0 + LKC2);
#pragma unroll 8
    for (int kk = kq * LKQ; kk < (kq + 1) * LKQ; kk += 4) {
      const float4 a = *(const float4*)&Is[rr][kk];
      const float4 w = *(const float4*)&Ws[c][kk];
      acc = fmaf(a.x, w.x, acc);
      acc = fmaf(a.y, w.y, acc);
      acc = fmaf(a.z, w.z, acc);
      acc = fmaf(a.w, w.w, acc);
    }
  }
  __syncthreads();
  float* red = &Is[0][0];                    // [4][256] partial sums
  red[kq * 256 + t8] = acc;
  __syncthreads();
  if (kq != 0) return;
  acc = ((red[t8] + red[256 + t8]) + red[512 + t8]) + red[768 + t8];
  const long n = n0 + c, r = r0 + rr;
  if (n >= N || r >= R) return;
  const float bias = J.b[j] ? J.b[j][n] : 0.f;
  const float v = acc + bias;
  if (act == 1) {
    J.out[j][r * ldo + n] = v;
    J.out2[j][r * ldo + n] = v / (1.f + expf(-v));
  } else if (act == 2) {
    const float x = aux[r * ldo + n];
    const float sg = 1.f / (1.f + expf(-x));
    J.out[j][r * ldo + n] = acc * (sg * (1.f + x * (1.f - sg)));
  } else {
    J.out[j][r * ldo + n] = v;
  }
}

// Round 6: a 32 x 32 output tile (32 rows of one job's 32 columns) per 512-thread block; the 8 waves split K (64-wide
// chunks c = w, w + 8, ...), each lane keeps a 4 x 4 register tile (rows rg + 8 i, columns cg + 8 j), operands staged
// per wave in its own LDS (no barrier inside the K walk), the 8 partial tiles added in a fixed order (deterministic).
// Round 2's 32 x 8 tile re-read the whole [32, K] input per 8 columns (82 KB of LDS per block, one block per CU): the
// 12 FiLM projections took 28 us alone and 73 us beside the encoder; here each weight element is read once.
constexpr int LR_TC = 32, LR_KC = 64, LR_NW = 8, LR_LD = LR_KC + 4;  // tile columns, K chunk, waves, LDS row (floats)
constexpr int LR_WAVE_FLOATS = 2 * 32 * LR_LD;                       // input + weight chunk of one wave
constexpr size_t LR_LDS = (size_t)LR_NW * LR_WAVE_FLOATS * 4;         // 139 264 B (the partial tiles reuse it)
template <bool TW>
__global__ void __launch_bounds__(512) linrt_kernel(const float* __restrict__ in, long ldi, LinJobs J, long ldw,
                                                    long ldo, const float* __restrict__ aux, long R, long N, long K,
                                                    int act) {
  extern __shared__ __attribute__((aligned(16))) float lrs[];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, rg = lane >> 3, cg = lane & 7;
  const long n0 = (long)blockIdx.x * LR_TC, r0 = (long)blockIdx.z * 32;
  const int j = blockIdx.y;
  const float* W = J.W[j];
  float* Is = lrs + w * LR_WAVE_FLOATS;  // [32 rows][LR_LD]
  float* Ws = Is + 32 * LR_LD;           // [32 columns][LR_LD]
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) acc[i][jj] = 0.f;
  const long nch = (K + LR_KC - 1) / LR_KC;
  for (long c = w; c < nch; c += LR_NW) {
    const long k0 = c * LR_KC;
    // input chunk [32 rows][64 k]: 512 float4, 8 per lane (lane-consecutive k: coalesced rows)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = lane + 64 * q, ri = e >> 4, k4 = e & 15;
      const long r = r0 + ri, k = k0 + 4 * k4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < R) {
        const float* src = in + r * ldi + k;
        if (k + 3 < K && (((uintptr_t)src) & 15) == 0) {
          v = *(const float4*)src;
        } else {
          if (k < K) v.x = src[0];
          if (k + 1 < K) v.y = src[1];
          if (k + 2 < K) v.z = src[2];
          if (k + 3 < K) v.w = src[3];
        }
      }
      *(float4*)&Is[ri * LR_LD + 4 * k4] = v;
    }
    // weight chunk as [32 columns][64 k]
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = lane + 64 * q;
      if (!TW) {  // W[n][k]: rows of k, like the input
        const int ci = e >> 4, k4 = e & 15;
        const long n = n0 + ci, k = k0 + 4 * k4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n < N) {
          const float* src = W + n * ldw + k;
          if (k + 3 < K && (((uintptr_t)src) & 15) == 0) {
            v = *(const float4*)src;
          } else {
            if (k < K) v.x = src[0];
            if (k + 1 < K) v.y = src[1];
            if (k + 2 < K) v.z = src[2];
            if (k + 3 < K) v.w = src[3];
          }
        }
        *(float4*)&Ws[ci * LR_LD + 4 * k4] = v;
      } else {    // W[k][n] (in @ W): rows of n, transposed into the column-major chunk
        const int ki = e >> 3, n4 = e & 7;
        const long k = k0 + ki, n = n0 + 4 * n4;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        if (k < K) {
          const float* src = W + k * ldw + n;
          if (n + 3 < N && (((uintptr_t)src) & 15) == 0) {
            const float4 t = *(const float4*)src;
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (n + u < N) v[u] = src[u];
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) Ws[(4 * n4 + u) * LR_LD + ki] = v[u];
      }
    }
    // (one wave writes and reads its own chunk: LDS executes a wave's instructions in order)
#pragma unroll 4
    for (int kk = 0; kk < LR_KC; kk += 4) {
      float4 a[4], bw[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *(const float4*)&Is[(rg + 8 * i) * LR_LD + kk];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) bw[jj] = *(const float4*)&Ws[(cg + 8 * jj) * LR_LD + kk];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          acc[i][jj] = fmaf(a[i].x, bw[jj].x, acc[i][jj]);
          acc[i][jj] = fmaf(a[i].y, bw[jj].y, acc[i][jj]);
          acc[i][jj] = fmaf(a[i].z, bw[jj].z, acc[i][jj]);
          acc[i][jj] = fmaf(a[i].w, bw[jj].w, acc[i][jj]);
        }
    }
  }
  // the 8 waves' partial tiles, added in wave order
  __syncthreads();
  float* red = lrs;  // [8 waves][32 rows][32 columns]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) red[w * 1024 + (rg + 8 * i) * 32 + cg + 8 * jj] = acc[i][jj];
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int o = tid + 512 * h, ri = o >> 5, ci = o & 31;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < LR_NW; ++ww) v += red[ww * 1024 + o];
    const long n = n0 + ci, r = r0 + ri;
    if (n >= N || r >= R) continue;
    const float bias = J.b[j] ? J.b[j][n] : 0.f;
    const float pre = v + bias;
    if (act == 1) {
      J.out[j][r * ldo + n] = pre;
      J.out2[j][r * ldo + n] = pre / (1.f + expf(-pre));
    } else if (act == 2) {
      const float x = aux[r * ldo + n];
      const float sg = 1.f / (1.f + expf(-x));
      J.out[j][r * ldo + n] = v * (sg * (1.f + x * (1.f - sg)));
    } else {
      J.out[j][r * ldo + n] = pre;
    }
  }
}

// Job j: dW_j[n][k] += sum_r dy_j[r][n] * x_j[r][k];  db_j[n] += sum_r dy_j[r][n]   (accumulating: gradient slots)
struct DwJobs {
  const float* dy[MAXJ];
  const float* x[MAXJ];
  float* dW[MAXJ];
  float* db[MAXJ];
  long N[MAXJ], K[MAXJ], lddy[MAXJ], ldx[MAXJ];
};

// tile 32 (n) x 64 (k) per 256-thread block: thread (n = n0 + (tid >> 3), k = k0 + 8 (tid & 7) + 0..7), rows staged in
// chunks of 32; the dW rows are read-modified-written as two float4 per thread (round 2's 32 x 32 tile with one
// scalar per thread and row ran the FiLM weight gradients at ~1.3 TB/s of dW traffic)
__global__ void __launch_bounds__(256) dw_kernel(DwJobs J, long R) {
  __shared__ float Ds[32][33];
  __shared__ __attribute__((aligned(16))) float Xs[32][64 + 4];
  const int j = blockIdx.z;
  const long N = J.N[j], K = J.K[j];
  const long n0 = (long)blockIdx.y * 32, k0 = (long)blockIdx.x * 64;
  if (n0 >= N || k0 >= K) return;
  const int tid = threadIdx.x, ty = tid >> 3, tx = tid & 7;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float bacc = 0.f;
  const bool dob = J.db[j] && blockIdx.x == 0 && tx == 0;
  for (long rr0 = 0; rr0 < R; rr0 += 32) {
    for (int e = tid; e < 32 * 32; e += 256) {
      const int rr = e >> 5, cc = e & 31;
      const long r = rr0 + rr;
      Ds[rr][cc] = (r < R && n0 + cc < N) ? J.dy[j][r * J.lddy[j] + n0 + cc] : 0.f;
    }
    for (int e = tid; e < 32 * 64; e += 256) {
      const int rr = e >> 6, cc = e & 63;
      const long r = rr0 + rr;
      Xs[rr][cc] = (r < R && k0 + cc < K) ? J.x[j][r * J.ldx[j] + k0 + cc] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int rr = 0; rr < 32; ++rr) {
      const float dv = Ds[rr][ty];
      const float4 x0 = *(const float4*)&Xs[rr][8 * tx], x1 = *(const float4*)&Xs[rr][8 * tx + 4];
      acc[0] = fmaf(dv, x0.x, acc[0]);
      acc[1] = fmaf(dv, x0.y, acc[1]);
      acc[2] = fmaf(dv, x0.z, acc[2]);
      acc[3] = fmaf(dv, x0.w, acc[3]);
      acc[4] = fmaf(dv, x1.x, acc[4]);
      acc[5] = fmaf(dv, x1.y, acc[5]);
      acc[6] = fmaf(dv, x1.z, acc[6]);
      acc[7] = fmaf(dv, x1.w, acc[7]);
      if (dob) bacc += dv;
    }
    __syncthreads();
  }
  const long n = n0 + ty, k = k0 + 8 * tx;
  if (n < N && k < K) {
    float* dst = J.dW[j] + n * K + k;
    if (k + 7 < K && (((uintptr_t)dst) & 15) == 0) {
      float4 u = *(float4*)dst, v = *(float4*)(dst + 4);
      u.x += acc[0]; u.y += acc[1]; u.z += acc[2]; u.w += acc[3];
      v.x += acc[4]; v.y += acc[5]; v.z += acc[6]; v.w += acc[7];
      *(float4*)dst = u;
      *(float4*)(dst + 4) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (k + e < K) dst[e] += acc[e];
    }
  }
  if (dob && n < N) J.db[j][n] += bacc;
}

// ------------------------------------------------------------------------------------------ KL reduction
// SchedulerAdapter.kl_term's batch reduction (train.py:247-253): per[b] = sum_l m kl / (sum_l m + eps) (mask) or
// mean_l kl (no mask); loss = mean_b per[b]; w[b][l] = d loss / d kl[b][l] for the backward. One wave per
// utterance, fixed summation order (deterministic); one launch of 1024 threads.
__global__ void __launch_bounds__(1024) kl_reduce_kernel(const float* __restrict__ kl, const unsigned char* __restrict__ mask,
                                                         float* __restrict__ w, float* __restrict__ loss, long B,
                                                         long L) {
  __shared__ float per[1024];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float eps = 1e-8f;
  for (long b = wv; b < B; b += 16) {
    float s = 0.f, m = 0.f;
    for (long l = lane; l < L; l += 64) {
      const float mv = mask ? (mask[b * L + l] ? 1.f : 0.f) : 1.f;
      s += mv * kl[b * L + l];
      m += mv;
    }
    s = wave_sum(s);
    m = wave_sum(m);
    const float den = mask ? m + eps : (float)L;
    if (w)
      for (long l = lane; l < L; l += 64) {
        const float mv = mask ? (mask[b * L + l] ? 1.f : 0.f) : 1.f;
        w[b * L + l] = mask ? mv / den / (float)B : 1.f / ((float)L * (float)B);
      }
    if (lane == 0) per[b] = s / den;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float acc = 0.f;
    for (long b = 0; b < B; ++b) acc += per[b];
    loss[0] = acc / (float)B;
  }
}

}  // namespace small
}  // namespace fddm

using namespace fddm;
using namespace fddm::small;

FDDM_API int fddm_rows_mean(int dtype, const void* x, float* out, long B, long S, long d, void* hs) {
  if (B <= 0 || d <= 0) return 0;
  dim3 g((unsigned)((d + 63) / 64), (unsigned)B);  // 64 columns per block
  if (((uintptr_t)x) & 15) return (int)hipErrorInvalidValue;
  if (dtype == FDDM_BF16)
    hipLaunchKernelGGL(rows_mean_kernel<bf16_t>, g, dim3(256), 0, (hipStream_t)hs, (const bf16_t*)x, out, S, d);
  else
    hipLaunchKernelGGL(rows_mean_kernel<float>, g, dim3(256), 0, (hipStream_t)hs, (const float*)x, out, S, d);
  return (int)hipGetLastError();
}

FDDM_API int fddm_time_embed(const long* t, float* emb, long B, long d, float max_steps, void* hs) {
  if (B <= 0 || d <= 0) return 0;
  const long n = B * d;
  // the end point of torch.linspace(log 1, log max_steps, half): math.log in double, then the fp32 tensor value
  hipLaunchKernelGGL(time_embed_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)hs, t, emb, B, d,
                     (float)log((double)max_steps));
  return (int)hipGetLastError();
}

FDDM_API int fddm_small_linear(const float* in, long ldi, int njobs, const float* const* W, const float* const* bias,
                               float* const* out, float* const* out2, long ldw, long ldo, const float* aux, long R, long N,
                               long K, int act, int transpose_w, void* hs) {
  if (njobs <= 0 || njobs > MAXJ || R <= 0 || N <= 0) return njobs > MAXJ ? (int)hipErrorInvalidValue : 0;
  LinJobs J{};
  for (int j = 0; j < njobs; ++j) {
    J.W[j] = W[j];
    J.b[j] = bias ? bias[j] : nullptr;
    J.out[j] = out[j];
    J.out2[j] = out2 ? out2[j] : nullptr;
    if (act == 1 && !J.out2[j]) return (int)hipErrorInvalidValue;
  }
  if (act == 2 && !aux) return (int)hipErrorInvalidValue;
  // the register-tile kernel where its 32-column tiles make >= 128 blocks (the 12 FiLM projections: 192; 28 -> ~21 us
  // alone, 73 -> 22-37 us beside the encoder); narrower launches (the time MLP, the input gradients: 16-64 tiles)
  // keep round 2's 8-column blocks, whose 4 K-quarters give them 4-16x the waves (measured faster there in the step)
  const long rt_blocks = ((N + LR_TC - 1) / LR_TC) * njobs * ((R + 31) / 32);
  if (rt_blocks < 128) {
    dim3 g4((unsigned)((N + LNC - 1) / LNC), (unsigned)njobs, (unsigned)((R + 31) / 32));
    if (transpose_w)
      hipLaunchKernelGGL(linear4_kernel<true>, g4, dim3(1024), 0, (hipStream_t)hs, in, ldi, J, ldw, ldo, aux, R, N, K,
                         act);
    else
      hipLaunchKernelGGL(linear4_kernel<false>, g4, dim3(1024), 0, (hipStream_t)hs, in, ldi, J, ldw, ldo, aux, R, N, K,
                         act);
    return (int)hipGetLastError();
  }
  dim3 g((unsigned)((N + LR_TC - 1) / LR_TC), (unsigned)njobs, (unsigned)((R + 31) / 32));
  if (transpose_w)
    hipLaunchKernelGGL(linrt_kernel<true>, g, dim3(512), LR_LDS, (hipStream_t)hs, in, ldi, J, ldw, ldo, aux, R, N, K,
                       act);
  else
    hipLaunchKernelGGL(linrt_kernel<false>, g, dim3(512), LR_LDS, (hipStream_t)hs, in, ldi, J, ldw, ldo, aux, R, N, K,
                       act);
  return (int)hipGetLastError();
}

FDDM_API int fddm_small_dw(int njobs, const float* const* dy, const long* lddy, const float* const* x, const long* ldx,
                           float* const* dW, float* const* db, const long* N, const long* K, long R, void* hs) {
  if (njobs <= 0 || njobs > MAXJ || R <= 0) return njobs > MAXJ ? (int)hipErrorInvalidValue : 0;
  DwJobs J{};
  long nmax = 1, kmax = 1;
  for (int j = 0; j < njobs; ++j) {
    J.dy[j] = dy[j];
    J.x[j] = x[j];
    J.dW[j] = dW[j];
    J.db[j] = db ? db[j] : nullptr;
    J.N[j] = N[j];
    J.K[j] = K[j];
    J.lddy[j] = lddy[j];
    J.ldx[j] = ldx[j];
    nmax = N[j] > nmax ? N[j] : nmax;
    kmax = K[j] > kmax ? K[j] : kmax;
  }
  dim3 g((unsigned)((kmax + 63) / 64), (unsigned)((nmax + 31) / 32), (unsigned)njobs);
  hipLaunchKernelGGL(dw_kernel, g, dim3(256), 0, (hipStream_t)hs, J, R);
  return (int)hipGetLastError();
}

FDDM_API int fddm_kl_reduce(const float* kl_tok, const unsigned char* mask, float* w, float* loss, long B, long L,
                            void* hs) {
  if (B <= 0 || L <= 0) return 0;
  if (B > 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kl_reduce_kernel, dim3(1), dim3(1024), 0, (hipStream_t)hs, kl_tok, mask, w, loss, B, L);
  return (int)hipGetLastError();
}
