// Jumpy-sampler denoise step (sampler/jumpy_sampler.py:167-215 +
// fddm/sched/diffusion_scheduler.py:106-208 of the reference), fused into one pass per logits row.
//
// The reference materialises one-hot(x_t), softmax(logits) and the full [B,L,K] multi-step posterior
//   q(x_{t-Δ}=k | x_t, x̂0) ∝ (a_cum[k=x_t] + b_cum) · (a_tg x̂_k + b_tg Σx̂)
// and takes its argmax. Every k ≠ x_t shares the factor b_cum, so the argmax is x_t or the first
// argmax of x̂ over k ≠ x_t: one streaming pass finds the row max (→ x̂0 argmax, also the final
// decode), the best k ≠ x_t, and a second (L2-resident) pass the softmax normaliser. HBM traffic is one
// read of the logits row (4·V B) + 16 B of indices per token.
//
// Non-greedy decoding (posterior_mode "average", greedy=False) draws from the same posterior,
// tempered as the reference does (softmax(log(clamp(p, 1e-12)) / temperature)), by a Gumbel-max race
// on the build's counter RNG (mix64(seed, stream, row·V + k)).
#include "common.h"

namespace fddm {

enum { JUMP_FAST = 1, JUMP_SAMPLE = 2 };

struct JumpArgs {
  const float* z;  // logits rows, row stride ldz
  long ldz;
  const long* xt;     // [N]
  const float* coef;  // per batch element: exact {a_cum, b_cum, a_tg, b_tg}; fast {abar, 0, 0, 0}
  long* xnext;        // [N]  x_{t-Δ}
  long* x0hat;        // [N]  argmax x̂0 (optional)
  long N, L;
  int V;
  int mode;
  float inv_temp;
  unsigned long long seed, stream;
};

__device__ __forceinline__ void better(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

__global__ __launch_bounds__(256) void jump_kernel(JumpArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.N) return;
  const float* z = a.z + row * a.ldz;
  const int V = a.V;
  const int x = (int)min(max(a.xt[row], 0L), (long)V - 1);  // clamped: never read outside the row
  float m = -INFINITY, o = -INFINITY;
  int mi = 0x7fffffff, oi = 0x7fffffff;
  const bool vec = ((V & 3) == 0) && ((a.ldz & 3) == 0) && (((uintptr_t)a.z & 15) == 0);
  // pass 1: row max / first argmax, and the best k != x_t (each lane scans increasing k, so a strict
  // comparison keeps the first occurrence; ties across lanes go to the lower index)
  if (vec) {
    for (int c = lane * 4; c < V; c += 256) {
      const float4 v = *reinterpret_cast<const float4*>(z + c);
      const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = c + j;
        if (e[j] > m) { m = e[j]; mi = k; }
        if (k != x && e[j] > o) { o = e[j]; oi = k; }
      }
    }
  } else {
    for (int k = lane; k < V; k += 64) {
      const float e = z[k];
      if (e > m) { m = e; mi = k; }
      if (k != x && e > o) { o = e; oi = k; }
    }
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    better(m, mi, __shfl_xor(m, s, 64), __shfl_xor(mi, s, 64));
    better(o, oi, __shfl_xor(o, s, 64), __shfl_xor(oi, s, 64));
  }
  // pass 2: softmax normaliser
  float sum = 0.f;
  if (vec) {
    for (int c = lane * 4; c < V; c += 256) {
      const float4 v = *reinterpret_cast<const float4*>(z + c);
      sum += __expf(v.x - m) + __expf(v.y - m) + __expf(v.z - m) + __expf(v.w - m);
    }
  } else {
    for (int k = lane; k < V; k += 64) sum += __expf(z[k] - m);
  }
  sum = wave_sum(sum);
  const long b = row / a.L;
  const float* cf = a.coef + b * 4;
  const double inv_s = 1.0 / (double)sum;
  const double px = exp((double)z[x] - (double)m) * inv_s;   // x̂_{x_t}
  const double po = exp((double)o - (double)m) * inv_s;       // max_{k≠x_t} x̂_k
  long nx;
  if (!(a.mode & JUMP_SAMPLE)) {
    if (a.mode & JUMP_FAST) {
      nx = mi;  // argmax(ᾱ x̂ + (1-ᾱ)/K) = argmax x̂ for ᾱ > 0
    } else {
      const double ac = cf[0], bc = cf[1], atg = cf[2], btg = cf[3];
      const double sx = (ac + bc) * (atg * px + btg);
      const double so = bc * (atg * po + btg);
      nx = (sx > so || (sx == so && x < oi)) ? x : oi;
    }
  } else {
    // categorical draw over the normalised posterior P_k (Gumbel-max race)
    double Zn = 1.0, ac = 0, bc = 0, atg = 0, btg = 0, abar = cf[0];
    if (!(a.mode & JUMP_FAST)) {
      ac = cf[0]; bc = cf[1]; atg = cf[2]; btg = cf[3];
      // Σ_k A_k B_k with Σ x̂ = 1: b_cum (a_tg + V b_tg) + a_cum (a_tg x̂_{x_t} + b_tg)
      Zn = bc * (atg + (double)V * btg) + ac * (atg * px + btg);
    }
    float best = -INFINITY;
    int bi = 0x7fffffff;
    const float inv_sf = (float)inv_s;
    for (int k = lane; k < V; k += 64) {
      const float xh = __expf(z[k] - m) * inv_sf;
      float P;
      if (a.mode & JUMP_FAST) P = (float)abar * xh + (1.f - (float)abar) / (float)V;
      else P = (float)(((k == x ? ac : 0.0) + bc) * (atg * xh + btg) / Zn);
      const uint64_t h = mix64(a.seed, a.stream, (uint64_t)row * (uint64_t)V + (uint64_t)k);
      const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
      const float g = -__logf(-__logf(u));
      const float sc = __logf(fmaxf(P, 1e-12f)) * a.inv_temp + g;
      if (sc > best) { best = sc; bi = k; }
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) better(best, bi, __shfl_xor(best, s, 64), __shfl_xor(bi, s, 64));
    nx = bi;
  }
  if (lane == 0) {
    a.xnext[row] = nx;
    if (a.x0hat) a.x0hat[row] = mi;
  }
}

}  // namespace fddm

using namespace fddm;

FDDM_API int fddm_jump(const float* logits, long ldz, const long* xt, const float* coef, long* x_next, long* x0hat,
                       long N, long L, long V, int mode, float temperature, unsigned long long seed,
                       unsigned long long stream, void* hip_stream) {
  if (N <= 0) return 0;
  if (V <= 1 || V >= (1L << 30) || L <= 0 || ldz < V || temperature <= 0.f) return (int)hipErrorInvalidValue;
  JumpArgs a{logits, ldz, xt, coef, x_next, x0hat, N, L, (int)V, mode, 1.f / temperature, seed, stream};
  hipLaunchKernelGGL(jump_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, (hipStream_t)hip_stream, a);
  FDDM_LAUNCH_CHECK();
}
