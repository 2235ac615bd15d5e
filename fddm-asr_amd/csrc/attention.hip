// Flash-style multi-head attention for gfx950 (head_dim 64), forward + backward.
//
// Covers the three attention sites of the train step:
//  * decoder self-attention  (models/denoise_decoder.py:129,164 -> nn.MultiheadAttention):
//      key-padding mask (~x_mask), dropout p on the attention probabilities;
//  * decoder cross-attention (models/denoise_decoder.py:130,169-174): no mask, dropout p;
//  * WavLM gated relative-position attention (HF modeling_wavlm.py:152-200), forward only:
//      score += gate[b,h,q] * table[h][key - q + Lk - 1]  (bucketed rel-pos bias gathered from a
//      per-head table instead of the reference's materialised [B*H,S,S] bias).
//
// Structure ("swapped" products so a lane owns one query (fwd, dQ) or one key (dK/dV) end to end):
//   S^T = K Q^T  (16x16 MFMA tiles, C layout: lane l holds rows 4*(l>>4)+j, column l&15)
//   O^T = V^T P^T  — P^T is the lane's own softmax values (no LDS round trip); V^T fragments come
//                    from a [key][d] LDS image through ds_read_b64_tr_b16 (hardware transpose).
// Work split: 4 waves x 16 rows = 64 rows per workgroup; K/V (or Q/dO) tiles of 64 rows in LDS.
// T = bf16 (mfma_f32_16x16x32_bf16) or f32 (mfma_f32_16x16x4f32, exact fp32 parity mode).
#include "attn_common.h"

namespace fddm {
namespace attn {


template <typename T> struct Cfg;
template <> struct Cfg<bf16_t> { static constexpr int RB = 128, NSUB = 2, ECH = 8; };
template <> struct Cfg<float> { static constexpr int RB = 256, NSUB = 4, ECH = 4; };

__device__ __forceinline__ int hatt(int k) { return ((k >> 1) & 3) << 2; }

template <typename T>
__device__ __forceinline__ void mma(f32x4_t& c, const uint4& a, const uint4& b);
template <> __device__ __forceinline__ void mma<bf16_t>(f32x4_t& c, const uint4& a, const uint4& b) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
template <> __device__ __forceinline__ void mma<float>(f32x4_t& c, const uint4& a, const uint4& b) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
}

// Stage a 64-row x 64-col tile (rows row0.., `nvalid` valid) into LDS as a KC image (row reads)
// and/or an MC image (transposed reads).
template <typename T>
__device__ __forceinline__ void stage(unsigned char* kc, unsigned char* mc, const T* base, long stride, int row0,
                                      int nvalid) {
  constexpr int RB = Cfg<T>::RB, ECH = Cfg<T>::ECH, CPR = RB / 16;
  for (int idx = threadIdx.x; idx < 64 * CPR; idx += 256) {
    const int r = idx / CPR, c = idx % CPR;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < nvalid) v = *(const uint4*)(base + (long)(row0 + r) * stride + c * ECH);
    if (kc) *(uint4*)(kc + kc_off(RB, r, c)) = v;
    if (mc) {
      if constexpr (sizeof(T) == 2) *(uint4*)(mc + r * 128 + (((2 * c) ^ hatt(r)) << 3)) = v;
      else *(uint4*)(mc + r * 256 + c * 16) = v;
    }
  }
}

// lane's register fragments of its own row (16-B chunk sub*4+g of row `row`) from global
template <typename T>
__device__ __forceinline__ void row_frags(uint4 (&f)[Cfg<T>::NSUB], const T* base, long stride, long row, bool valid,
                                          int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int s = 0; s < Cfg<T>::NSUB; ++s)
    f[s] = valid ? *(const uint4*)(base + row * stride + (s * 4 + g) * Cfg<T>::ECH) : make_uint4(0, 0, 0, 0);
}

// acc[kb] = sum_sub  A(img rows kb*16..+15, KC) x B(lane fragment)
template <typename T>
__device__ __forceinline__ void rows_times_frag(f32x4_t (&acc)[4], const unsigned char* img, const uint4 (&f)[Cfg<T>::NSUB],
                                                int lane) {
  constexpr int RB = Cfg<T>::RB;
  const int g = lane >> 4, i = lane & 15;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    acc[kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < Cfg<T>::NSUB; ++s) {
      const uint4 a = *(const uint4*)(img + kc_off(RB, kb * 16 + i, s * 4 + g));
      mma<T>(acc[kb], a, f[s]);
    }
  }
}

__device__ __forceinline__ unsigned pk(float a, float b) { return pk_bf16(a, b); }

// out[db] += sum_rows  A(MC image transposed: [col d][row]) x B(lane-owned values v[kb][j] at row kb*16+4g+j)
template <typename T>
__device__ __forceinline__ void trans_times_vals(f32x4_t (&out)[4], const unsigned char* img, const float (&v)[4][4],
                                                 int lane) {
  const int g = lane >> 4, i = lane & 15;
  if constexpr (sizeof(T) == 2) {
    const int q = i >> 2, p = i & 3;
    typedef __attribute__((address_space(3))) s16x4_t* lp;
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      uint4 b;
      b.x = pk(v[2 * ss][0], v[2 * ss][1]);
      b.y = pk(v[2 * ss][2], v[2 * ss][3]);
      b.z = pk(v[2 * ss + 1][0], v[2 * ss + 1][1]);
      b.w = pk(v[2 * ss + 1][2], v[2 * ss + 1][3]);
      const int k1 = 32 * ss + 4 * g + q, k2 = k1 + 16;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int u = db * 4 + p;
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + k1 * 128 + ((u ^ hatt(k1)) << 3)));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + k2 * 128 + ((u ^ hatt(k2)) << 3)));
        const uint4 a = join_tr(lo, hi);
        mma<bf16_t>(out[db], a, b);
      }
    }
  } else {
    const float* f = (const float*)img;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        uint4 a, b;
        a.x = __float_as_uint(f[(kb * 16 + 4 * g + 0) * 64 + db * 16 + i]);
        a.y = __float_as_uint(f[(kb * 16 + 4 * g + 1) * 64 + db * 16 + i]);
        a.z = __float_as_uint(f[(kb * 16 + 4 * g + 2) * 64 + db * 16 + i]);
        a.w = __float_as_uint(f[(kb * 16 + 4 * g + 3) * 64 + db * 16 + i]);
        b = make_uint4(__float_as_uint(v[kb][0]), __float_as_uint(v[kb][1]), __float_as_uint(v[kb][2]),
                       __float_as_uint(v[kb][3]));
        mma<float>(out[db], a, b);
      }
    }
  }
}

// Diagnostic build only (-DATTN_STAMPS, tools/attn_stamps.py): s_memtime stamps of wave 0 of every workgroup at the
// phase boundaries of the v3 kernels (slot 0 entry, 1 loads issued, 2 data landed + barrier, 3.. after each key /
// query tile, 12 stores issued, 13 exit), s_memrealtime at entry / exit (slots 14, 15) for the clock. The stamps go
// to a buffer of their own; in the real build no stamp executes.
#ifdef ATTN_STAMPS
__device__ unsigned long long attn_stamps[8192 * 16];
#define ASTAMP(k)                                                                              \
  do {                                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    unsigned long long t_;                                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                  \
    __builtin_amdgcn_sched_barrier(0);                                                         \
    const int bl_ = blockIdx.x + blockIdx.y * gridDim.x;                                       \
    if (threadIdx.x == 0 && bl_ < 8192) attn_stamps[bl_ * 16 + (k)] = t_;                       \
  } while (0)
#define ARTIME(k)                                                                              \
  do {                                                                                         \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                            \
    __builtin_amdgcn_s_waitcnt(0xC07F);                                                        \
    const int bl_ = blockIdx.x + blockIdx.y * gridDim.x;                                       \
    if (threadIdx.x == 0 && bl_ < 8192) attn_stamps[bl_ * 16 + (k)] = t_;                       \
  } while (0)
#else
#define ASTAMP(k)
#define ARTIME(k)
#endif

// Attention-probability dropout: RNG contract v2 (oracle/fddm_oracle.py: attn_dropout_keep). Per (b, h) three
// tables of R = 4096 16-bit words, T_tau[j] = bits 16*(j&3).. of mix64(seed, stream, TAB0 + (bh*3 + tau)*1024 +
// (j>>2)); per query row r = bh*Lq + q three offsets o_tau = (mix64(seed, stream, OFF0 + r) >> 16*tau) & 0xFFC;
// the element (q, key) draws u = T_0[(o_0 + key) & 4095] ^ T_1[(o_1 + key) & 4095] ^ T_2[(o_2 + key) & 4095] and
// is kept iff u >= round(p * 65536). Within a row the 16-bit draws are distinct table entries (Lk <= 4096); two
// rows repeat each other's draws (shifted) only if all three offset differences coincide (2^-20 per pair). The
// forward kernel holds the three tables in LDS (24 KB, built once per workgroup): 3 ds_read_b64 + 2 64-bit XORs
// per 4 keys, instead of a 64-bit splitmix64 hash per 4 keys.
__device__ __forceinline__ uint64_t attn_offsets(const AttnArgs& a, int bh, int q) {
  return mix64(eff_seed(a.seed, a.seed_off), a.stream, ATTN_OFF0 + (uint64_t)bh * a.Lq + q);
}
// the 4 keep bits of keys k0..k0+3 (k0 % 4 == 0) of query q: generic form (4 hashes), for the kernels that do not
// stage the tables
__device__ __forceinline__ unsigned attn_keep4(const AttnArgs& a, int bh, int q, int k0) {
  const uint64_t off = attn_offsets(a, bh, q);
  uint64_t w = 0;
#pragma unroll
  for (int tau = 0; tau < 3; ++tau) {
    const unsigned j = ((unsigned)((off >> (16 * tau)) & 0xFFCu) + (unsigned)k0) & (ATTN_R - 1);
    w ^= mix64(eff_seed(a.seed, a.seed_off), a.stream, ATTN_TAB0 + ((uint64_t)bh * 3 + tau) * (ATTN_R / 4) + (j >> 2));
  }
  unsigned keep = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) keep |= (((unsigned)(w >> (16 * j)) & 0xFFFFu) >= a.thr16 ? 1u : 0u) << j;
  return keep;
}
__device__ __forceinline__ bool attn_keep(const AttnArgs& a, int bh, int q, int key) {
  return (attn_keep4(a, bh, q, key & ~3) >> (key & 3)) & 1u;
}

// ------------------------------------------------------------------------------------------- fwd
template <typename T>
__global__ void __launch_bounds__(256) fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int RB = Cfg<T>::RB;
  unsigned char* kimg = smem;
  unsigned char* vimg = smem + 64 * RB;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int q = bxi * 64 + w * 16 + i;
  const bool qv = q < a.Lq;
  const T* Qb = (const T*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const T* Kb = (const T*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const T* Vb = (const T*)a.V + (long)b * a.Lk * a.sv + h * DH;
  uint4 qf[Cfg<T>::NSUB];
  row_frags<T>(qf, Qb, a.sq, qv ? q : 0, qv, lane);
  const float gate = (a.gate && qv) ? a.gate[(long)bh * a.Lq + q] : 0.f;
  const float* tab = a.table ? a.table + (long)h * (2 * a.Lk - 1) + (a.Lk - 1) - q : nullptr;

  float m = -INFINITY, l = 0.f;
  f32x4_t o[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < a.Lk; k0 += 64) {
    const int nv = min(64, a.Lk - k0);
    __syncthreads();
    stage<T>(kimg, nullptr, Kb, a.sk, k0, nv);
    stage<T>(nullptr, vimg, Vb, a.sv, k0, nv);
    __syncthreads();
    f32x4_t s[4];
    rows_times_frag<T>(s, kimg, qf, lane);
    float p[4][4];
    float tmax = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = k0 + kb * 16 + 4 * g + j;
        float x = s[kb][j] * a.scale;
        if (tab && qv && key < a.Lk) x += gate * tab[key];
        if (!key_ok(a, b, key)) x = -INFINITY;
        p[kb][j] = x;
        tmax = fmaxf(tmax, x);
      }
    tmax = xmax16(tmax);
    tmax = xmax32(tmax);
    const float mn = fmaxf(m, tmax);
    const float alpha = (mn == -INFINITY) ? 1.f : __expf(m - mn);
    float ls = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float e = (mn == -INFINITY) ? 0.f : __expf(p[kb][j] - mn);
        ls += e;
        if (a.thr16) {
          const int key = k0 + kb * 16 + 4 * g + j;
          e = attn_keep(a, bh, q, key) ? e * a.drop_scale : 0.f;
        }
        p[kb][j] = e;
      }
    l = l * alpha + ls;
    m = mn;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] *= alpha;
    trans_times_vals<T>(o, vimg, p, lane);
  }
  l = xsum16(l);
  l = xsum32(l);
  if (!qv) return;
  const float inv = (l > 0.f) ? 1.f / l : NAN;  // fully masked row -> NaN like softmax(all -inf)
  T* Ob = (T*)a.Out + ((long)b * a.Lq + q) * a.so + h * DH;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int j = 0; j < 4; ++j) st<T>(Ob + d * 16 + 4 * g + j, o[d][j] * inv);
  if (a.lse && g == 0) a.lse[(long)bh * a.Lq + q] = (l > 0.f) ? m + __logf(l) : NAN;
}

// ------------------------------------------------------------------------------------ fwd (bf16)
// 128 queries per workgroup: each wave owns two 16-query groups, so every K fragment (LDS row read) and
// every V^T fragment (tr read) feeds two MFMAs. K/V tiles are double-buffered in LDS; the next tile's
// global loads are issued before this tile's MFMAs and written after them (one barrier per tile).
// The WavLM bias slice for the tile (191 table entries: key - q spans [k0-q0-127, k0+63-q0]) is staged
// with the tile instead of gathered from global memory per score.
// Template flags: DROP (dropout on P), MASK (key-padding mask and/or a ragged last tile: a 0/-inf bias row
// per tile in LDS), REL (WavLM gated relative-position bias).
#ifndef ATTN_FWD_WPS
#define ATTN_FWD_WPS 2  // waves per SIMD the register allocation targets (measured: 2 beats 1, 3-4 spill)
#endif
template <bool DROP, bool MASK, bool REL, int NG = 2>
__global__ void __launch_bounds__(256, ATTN_FWD_WPS) fwd2_kernel(AttnArgs a) {
  constexpr int RB = 128;
  __shared__ __attribute__((aligned(16))) unsigned char kbuf[2][64 * RB];
  __shared__ __attribute__((aligned(16))) unsigned char vbuf[2][64 * RB];
  __shared__ float tbuf[2][192];
  __shared__ __attribute__((aligned(16))) float mbuf[2][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int qbase = bxi * (64 * NG);
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  const float* tabh = REL ? a.table + (long)h * (2 * a.Lk - 1) : nullptr;
  int q[NG];
  bool qv[NG];
  uint4 qf[NG][2];
  float gate[NG];
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    q[gq] = qbase + w * (16 * NG) + gq * 16 + i;
    qv[gq] = q[gq] < a.Lq;
    row_frags<bf16_t>(qf[gq], Qb, a.sq, qv[gq] ? q[gq] : 0, qv[gq], lane);
    gate[gq] = (a.gate && qv[gq]) ? a.gate[(long)bh * a.Lq + q[gq]] : 0.f;
    if (REL && a.graw && qv[gq]) {
      // gate from the 8 pre-activations the Q|K|V projection appended (HF modeling_wavlm.py:177-186)
      const uint4 u = *(const uint4*)((const bf16_t*)a.graw + ((long)b * a.Lq + q[gq]) * a.sgr + h * 8);
      const float ra = bf2f((bf16_t)(u.x & 0xffff)) + bf2f((bf16_t)(u.x >> 16)) + bf2f((bf16_t)(u.y & 0xffff)) +
                       bf2f((bf16_t)(u.y >> 16));
      const float rb = bf2f((bf16_t)(u.z & 0xffff)) + bf2f((bf16_t)(u.z >> 16)) + bf2f((bf16_t)(u.w & 0xffff)) +
                       bf2f((bf16_t)(u.w >> 16));
      const float ga = 1.f / (1.f + __expf(-ra)), gb = 1.f / (1.f + __expf(-rb));
      gate[gq] = ga * (gb * a.gconst[h] - 1.f) + 2.f;
    }
  }
  // tile loader: 512 16-B chunks of K and of V per tile, 2 each per thread
  uint4 kr[2], vr[2];
  float tv = 0.f, mv = 0.f;
  auto load = [&](int k0) {
    const int nv = min(64, a.Lk - k0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + 256 * u, r = idx >> 3, c = idx & 7;
      kr[u] = vr[u] = make_uint4(0, 0, 0, 0);
      if (r < nv) {
        kr[u] = *(const uint4*)(Kb + (long)(k0 + r) * a.sk + c * 8);
        vr[u] = *(const uint4*)(Vb + (long)(k0 + r) * a.sv + c * 8);
      }
    }
    if (REL && tid < 191) {
      const long ti = (long)k0 - qbase - 127 + (a.Lk - 1) + tid;
      tv = (ti >= 0 && ti < 2L * a.Lk - 1) ? tabh[ti] : 0.f;
    }
    if (MASK && tid >= 192) {
      const int key = k0 + tid - 192;
      mv = key_ok(a, b, key) ? 0.f : -INFINITY;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + 256 * u, r = idx >> 3, c = idx & 7;
      *(uint4*)(kbuf[buf] + kc_off(RB, r, c)) = kr[u];
      *(uint4*)(vbuf[buf] + r * 128 + (((2 * c) ^ hatt(r)) << 3)) = vr[u];
    }
    if (REL && tid < 191) tbuf[buf][tid] = tv;
    if (MASK && tid >= 192) mbuf[buf][tid - 192] = mv;
  };

  const float sl2 = a.scale * 1.4426950408889634f;  // running max m is kept in log2 units
  float graw[NG];  // bias multiplier in raw score units (gate / scale), once per query instead of per tile
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) graw[gq] = REL ? gate[gq] / a.scale : 0.f;
  float m[NG], l[NG];
  f32x4_t o[NG][4];
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    m[gq] = -INFINITY;
    l[gq] = 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[gq][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  load(0);
  store(0);
  __syncthreads();
  const int ntiles = (a.Lk + 63) / 64;
  // lazy rescale (defer-max): a row's running max m moves only when a tile's max exceeds it by more than 8 in
  // log2 units, decided per wave; otherwise p = 2^(x*sl2 - m*sl2) <= 2^8 and O, l keep their scale (no alpha
  // exp, no O multiply on most tiles). The softmax result is unchanged; only rounding differs.
  const float th_raw = 8.f / sl2;
  auto tile = [&](const int t, auto mc) {
    constexpr bool MT = decltype(mc)::value;  // this tile adds the 0/-inf mask row
    const int cur = t & 1, k0 = t * 64;
    if (t + 1 < ntiles) load(k0 + 64);
    const unsigned char* kimg = kbuf[cur];
    const unsigned char* vimg = vbuf[cur];
    f32x4_t s[NG][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
      for (int gq = 0; gq < NG; ++gq) s[gq][kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const uint4 af = *(const uint4*)(kimg + kc_off(RB, kb * 16 + i, sub * 4 + g));
#pragma unroll
        for (int gq = 0; gq < NG; ++gq) mma<bf16_t>(s[gq][kb], af, qf[gq][sub]);
      }
    }
    // softmax. Scores stay in raw units x = s (+ (gate/scale)*bias) (+ the tile's 0/-inf mask row); the running
    // max m is in raw units and p = 2^(x*sl2 - m*sl2) is one FMA + v_exp_f32 per score. Score pairs are carried
    // as float2 so the bias FMA, the mask add, the exponent FMA and the row sum issue as packed v_pk_* f32
    // instructions. MASK kernels add the mask row on every tile (0 where keys are valid): a per-tile condition
    // compiled to an add plus a select per score on every tile. The dropout scale 1/(1-p) is applied to O once
    // at the end, not per kept probability.
    f32x2_t mrow[4][2];
    if constexpr (MT) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float4 mv4 = *(const float4*)(&mbuf[cur][kb * 16 + 4 * g]);
        mrow[kb][0] = f32x2_t{mv4.x, mv4.y};
        mrow[kb][1] = f32x2_t{mv4.z, mv4.w};
      }
    }
    float p[NG][4][4];
#pragma unroll
    for (int gq = 0; gq < NG; ++gq) {
      float tmax = -INFINITY;
      const int toff = 127 - (q[gq] - qbase);
      const f32x2_t gr2 = {graw[gq], graw[gq]};
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          f32x2_t x = {s[gq][kb][2 * jj], s[gq][kb][2 * jj + 1]};
          if constexpr (REL) {
            const int kl = kb * 16 + 4 * g + 2 * jj + toff;
            x = gr2 * f32x2_t{tbuf[cur][kl], tbuf[cur][kl + 1]} + x;
          }
          if constexpr (MT) x += mrow[kb][jj];
          p[gq][kb][2 * jj] = x.x;
          p[gq][kb][2 * jj + 1] = x.y;
        }
        tmax = fmaxf(tmax, fmaxf(fmaxf(p[gq][kb][0], p[gq][kb][1]), fmaxf(p[gq][kb][2], p[gq][kb][3])));
      }
      tmax = xmax16(tmax);
      tmax = xmax32(tmax);
      if (__any(tmax > m[gq] + th_raw)) {  // wave-uniform: rescale O and l to the new running max
        const float mn = fmaxf(m[gq], tmax);
        const float mref = (mn == -INFINITY) ? 0.f : mn;
        const float alpha = __builtin_amdgcn_exp2f((m[gq] - mref) * sl2);
        l[gq] *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[gq][d] *= alpha;
        m[gq] = mn;
      }
      const float mref = (m[gq] == -INFINITY) ? 0.f : m[gq];  // all-masked so far: exp2(-inf) = 0
      const float nbias = -mref * sl2;
      const f32x2_t sl2v = {sl2, sl2}, nb2 = {nbias, nbias};
      f32x2_t ls2 = {0.f, 0.f};
      uint64_t bits = 0;
      // dropout keep bits of the lane's 4 keys per block (generic contract form; fwd6 reads precomputed words)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        unsigned keep = 0xF;
        if constexpr (DROP) {
          keep = attn_keep4(a, bh, q[gq], k0 + kb * 16 + 4 * g);
          bits |= (uint64_t)keep << (kb * 16 + 4 * g);
        }
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const f32x2_t arg = f32x2_t{p[gq][kb][2 * jj], p[gq][kb][2 * jj + 1]} * sl2v + nb2;
          f32x2_t e = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
          ls2 += e;
          if constexpr (DROP) {
            e.x = ((keep >> (2 * jj)) & 1u) ? e.x : 0.f;
            e.y = ((keep >> (2 * jj + 1)) & 1u) ? e.y : 0.f;
          }
          p[gq][kb][2 * jj] = e.x;
          p[gq][kb][2 * jj + 1] = e.y;
        }
      }
      const float ls = ls2.x + ls2.y;
      if constexpr (DROP) {
        if (a.dbits) {  // the 4 lanes of a query hold disjoint key nibbles: OR them into the tile's 64-bit word
          unsigned lo = (unsigned)bits, hi = (unsigned)(bits >> 32);
          lo = xor16(lo);
          hi = xor16(hi);
          lo = xor32(lo);
          hi = xor32(hi);
          if (g == 0 && qv[gq]) a.dbits[((long)bh * ntiles + t) * a.Lq + q[gq]] = ((uint64_t)hi << 32) | lo;
        }
      }
      l[gq] += ls;
    }
    // O^T += V^T P^T for both query groups (one tr-read A fragment, two MFMAs)
    {
      const int qq = i >> 2, pp = i & 3;
      typedef __attribute__((address_space(3))) s16x4_t* lp;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        uint4 bq[NG];
#pragma unroll
        for (int gq = 0; gq < NG; ++gq) {
          bq[gq].x = pk(p[gq][2 * ss][0], p[gq][2 * ss][1]);
          bq[gq].y = pk(p[gq][2 * ss][2], p[gq][2 * ss][3]);
          bq[gq].z = pk(p[gq][2 * ss + 1][0], p[gq][2 * ss + 1][1]);
          bq[gq].w = pk(p[gq][2 * ss + 1][2], p[gq][2 * ss + 1][3]);
        }
        const int k1 = 32 * ss + 4 * g + qq, k2 = k1 + 16;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const int u = db * 4 + pp;
          const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(vimg + k1 * 128 + ((u ^ hatt(k1)) << 3)));
          const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(vimg + k2 * 128 + ((u ^ hatt(k2)) << 3)));
          const uint4 af = join_tr(lo, hi);
#pragma unroll
          for (int gq = 0; gq < NG; ++gq) mma<bf16_t>(o[gq][db], af, bq[gq]);
        }
      }
    }
    if (t + 1 < ntiles) {
      store(cur ^ 1);
      __syncthreads();
    }
  };
  // the mask row only where it can be non-zero: every tile with a key-padding mask, else only the ragged last one
  if (MASK && a.key_keep != nullptr) {
    for (int t = 0; t < ntiles; ++t) tile(t, std::integral_constant<bool, MASK>{});
  } else {
    for (int t = 0; t + 1 < ntiles; ++t) tile(t, std::false_type{});
    tile(ntiles - 1, std::integral_constant<bool, MASK>{});
  }
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    float lt = l[gq];
    lt = xsum16(lt);
    lt = xsum32(lt);
    if (!qv[gq]) continue;
    // fully masked row -> NaN like softmax(all -inf); the dropout scale of the kept probabilities goes here
    const float inv = (lt > 0.f) ? (DROP ? a.drop_scale : 1.f) / lt : NAN;
    bf16_t* Ob = (bf16_t*)a.Out + ((long)b * a.Lq + q[gq]) * a.so + h * DH;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint2 u2;
      u2.x = pk(o[gq][d][0] * inv, o[gq][d][1] * inv);
      u2.y = pk(o[gq][d][2] * inv, o[gq][d][3] * inv);
      *(uint2*)(Ob + d * 16 + 4 * g) = u2;
    }
    if (a.lse && g == 0)
      a.lse[(long)bh * a.Lq + q[gq]] = (lt > 0.f) ? (m[gq] * sl2 + __log2f(lt)) * 0.69314718055994531f : NAN;
  }
}

// ------------------------------------------------------------------------- fwd (bf16, WavLM, streamed ring)
// WavLM's gated relative-position attention (no dropout): fwd2's work split (4 waves x 2 query groups x 16 = 128
// queries per workgroup) and tile body, with the K / V tiles streamed through an NST-stage LDS ring by LDS-DMA
// (NST - 1 tiles in flight) instead of register staging (global loads, LDS writes and their address arithmetic per
// tile, and a __syncthreads fence that drained the next tile's loads); the smaller LDS footprint lets three
// workgroups share a CU (fwd2: two). The
// bias slice of the workgroup's query range and the key mask row are staged once (as fwd6). The DMA is
// inline asm (dma16_asm): hipcc does not track it, so it inserts no stream-draining wait before the tile's LDS
// reads; each tile waits for its own pieces with a counted vmcnt (every wave issues exactly 4 DMA instructions per
// tile — past the end the last tile is re-read into a free stage — and no other vector-memory instruction in the
// loop), then a barrier; the stage of tile t-1 is refilled after it. WavLM attention 56.5 -> 52 us at C2.
#ifndef FWD5_WPS
#define FWD5_WPS 2  // waves per SIMD the NG = 2 build's register allocation targets (timing variants: 3, 4)
#endif
template <bool MASK, int NST = 2, int NG = 2>
__global__ void __launch_bounds__(256, NG == 1 ? 4 : FWD5_WPS) fwd5_kernel(AttnArgs a) {
  constexpr int QW = 64 * NG, TB = 64 * 128, RB = 128;
  constexpr bool DROP = false, REL = true;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm5[];
  const int ntiles = (a.Lk + 63) / 64, LkP = ntiles * 64;
  unsigned char* kst = sm5;                      // [NST][64 rows][128 B] K, KC image
  unsigned char* vst = sm5 + NST * TB;           // [NST][64 rows][128 B] V, tr-read image
  float* mfull = (float*)(sm5 + 2 * NST * TB);   // [LkP] 0 / -inf
  float* tfull = mfull + LkP;                    // [LkP + QW] relative-bias slice
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int qbase = bxi * QW;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  // ---- ordinary loads first; hipcc waits for them before the stream starts (the asm below pins the registers)
  int q[NG];
  bool qv[NG];
  uint4 qf[NG][2];
  float gate[NG];
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    q[gq] = qbase + w * (16 * NG) + gq * 16 + i;
    qv[gq] = q[gq] < a.Lq;
    row_frags<bf16_t>(qf[gq], Qb, a.sq, qv[gq] ? q[gq] : 0, qv[gq], lane);
    gate[gq] = (a.gate && qv[gq]) ? a.gate[(long)bh * a.Lq + q[gq]] : 0.f;
    if (a.graw && qv[gq]) {
      // gate from the 8 pre-activations the Q|K|V projection appended (HF modeling_wavlm.py:177-186)
      const uint4 u = *(const uint4*)((const bf16_t*)a.graw + ((long)b * a.Lq + q[gq]) * a.sgr + h * 8);
      const float ra = bf2f((bf16_t)(u.x & 0xffff)) + bf2f((bf16_t)(u.x >> 16)) + bf2f((bf16_t)(u.y & 0xffff)) +
                       bf2f((bf16_t)(u.y >> 16));
      const float rb = bf2f((bf16_t)(u.z & 0xffff)) + bf2f((bf16_t)(u.z >> 16)) + bf2f((bf16_t)(u.w & 0xffff)) +
                       bf2f((bf16_t)(u.w >> 16));
      const float ga = 1.f / (1.f + __expf(-ra)), gb = 1.f / (1.f + __expf(-rb));
      gate[gq] = ga * (gb * a.gconst[h] - 1.f) + 2.f;
    }
  }
  if (a.gx) {
    // gate from the attention input x (HF modeling_wavlm.py:177-186 with the 4 + 4 pre-activations summed through
    // the folded weights): the 4 lanes of a query (groups g) each take 16 of the head's 64 inputs, then 2 lane swaps
    const float4* wa = (const float4*)(a.gw + 16 * g);
    const float4* wb = (const float4*)(a.gw + 64 + 16 * g);
#pragma unroll
    for (int gq = 0; gq < NG; ++gq) {
      float sa = 0.f, sb = 0.f;
      if (qv[gq]) {
        const bf16_t* xr = (const bf16_t*)a.gx + ((long)b * a.Lq + q[gq]) * a.sgx + h * DH + 16 * g;
        const uint4 x0 = *(const uint4*)xr, x1 = *(const uint4*)(xr + 8);
        const unsigned xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 A = wa[j], Bw = wb[j];
          const float e0 = __uint_as_float(xs[2 * j] << 16), e1 = __uint_as_float(xs[2 * j] & 0xFFFF0000u);
          const float e2 = __uint_as_float(xs[2 * j + 1] << 16), e3 = __uint_as_float(xs[2 * j + 1] & 0xFFFF0000u);
          sa = fmaf(e0, A.x, fmaf(e1, A.y, fmaf(e2, A.z, fmaf(e3, A.w, sa))));
          sb = fmaf(e0, Bw.x, fmaf(e1, Bw.y, fmaf(e2, Bw.z, fmaf(e3, Bw.w, sb))));
        }
      }
      sa = xsum32(xsum16(sa)) + a.gw[128];
      sb = xsum32(xsum16(sb)) + a.gw[129];
      if (qv[gq]) {
        const float ga = 1.f / (1.f + __expf(-sa)), gb = 1.f / (1.f + __expf(-sb));
        gate[gq] = ga * (gb * a.gconst[h] - 1.f) + 2.f;
      }
    }
  }
  for (int k = tid; k < LkP; k += 256) mfull[k] = (MASK && !key_ok(a, b, k)) ? -INFINITY : 0.f;
  {
    const float* tabh = a.table + (long)h * (2 * a.Lk - 1);
    const long off0 = (long)(a.Lk - 1) - (qbase + QW - 1);  // tfull[j] = table[h][off0 + j]
    for (int j = tid; j < LkP + QW; j += 256) {
      const long ti = off0 + j;
      tfull[j] = (ti >= 0 && ti < 2L * a.Lk - 1) ? tabh[ti] : 0.f;
    }
  }
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    pin16(qf[gq][0]);
    pin16(qf[gq][1]);
    asm volatile("" : "+v"(gate[gq]));
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  // ---- K / V stream: wave w fills rows 16w .. 16w+15 of a tile (2 K + 2 V instructions; XOR swizzles on the
  // per-lane source addresses)
  auto fill = [&](int tt, int st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int R = 16 * w + 8 * u;
      const int r = 64 * tt + R + (lane >> 3), pch = lane & 7;
      const int rr = min(r, a.Lk - 1);
      const int ck = pch ^ ((r >> 1) & 7), cv = pch ^ (((r >> 1) & 3) << 1);
      dma16_asm(Kb + (long)rr * a.sk + ck * 8, kst + st * TB + R * 128);
      dma16_asm(Vb + (long)rr * a.sv + cv * 8, vst + st * TB + R * 128);
    }
  };
#pragma unroll
  for (int u = 0; u < NST - 1; ++u) fill(min(u, ntiles - 1), u);

  const float sl2 = a.scale * 1.4426950408889634f;  // running max m is kept in log2 units
  float graw[NG];  // bias multiplier in raw score units (gate / scale)
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) graw[gq] = gate[gq] / a.scale;
  float m[NG], l[NG];
  f32x4_t o[NG][4];
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    m[gq] = -INFINITY;
    l[gq] = 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[gq][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  const float th_raw = 8.f / sl2;  // lazy rescale threshold, as in fwd2_kernel
  auto tile = [&](const int t, auto mc) {
    constexpr bool MT = decltype(mc)::value;  // this tile adds the 0/-inf mask row
    const int k0 = t * 64;
    const unsigned char* kimg = kst + (t % NST) * TB;
    const unsigned char* vimg = vst + (t % NST) * TB;
    f32x4_t s[NG][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
      for (int gq = 0; gq < NG; ++gq) s[gq][kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const uint4 af = *(const uint4*)(kimg + kc_off(RB, kb * 16 + i, sub * 4 + g));
#pragma unroll
        for (int gq = 0; gq < NG; ++gq) mma<bf16_t>(s[gq][kb], af, qf[gq][sub]);
      }
    }
    // softmax. Scores stay in raw units x = s (+ (gate/scale)*bias) (+ the tile's 0/-inf mask row); the running
    // max m is in raw units and p = 2^(x*sl2 - m*sl2) is one FMA + v_exp_f32 per score. Score pairs are carried
    // as float2 so the bias FMA, the mask add, the exponent FMA and the row sum issue as packed v_pk_* f32
    // instructions. MASK kernels add the mask row on every tile (0 where keys are valid): a per-tile condition
    // compiled to an add plus a select per score on every tile. The dropout scale 1/(1-p) is applied to O once
    // at the end, not per kept probability.
    f32x2_t mrow[4][2];
    if constexpr (MT) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float4 mv4 = *(const float4*)(&mfull[k0 + kb * 16 + 4 * g]);
        mrow[kb][0] = f32x2_t{mv4.x, mv4.y};
        mrow[kb][1] = f32x2_t{mv4.z, mv4.w};
      }
    }
    float p[NG][4][4];
#pragma unroll
    for (int gq = 0; gq < NG; ++gq) {
      float tmax = -INFINITY;
      const int toff = (QW - 1) - (q[gq] - qbase) + k0;
      const f32x2_t gr2 = {graw[gq], graw[gq]};
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          f32x2_t x = {s[gq][kb][2 * jj], s[gq][kb][2 * jj + 1]};
          if constexpr (REL) {
            const int kl = kb * 16 + 4 * g + 2 * jj + toff;
            x = gr2 * f32x2_t{tfull[kl], tfull[kl + 1]} + x;
          }
          if constexpr (MT) x += mrow[kb][jj];
          p[gq][kb][2 * jj] = x.x;
          p[gq][kb][2 * jj + 1] = x.y;
        }
        tmax = fmaxf(tmax, fmaxf(fmaxf(p[gq][kb][0], p[gq][kb][1]), fmaxf(p[gq][kb][2], p[gq][kb][3])));
      }
      tmax = xmax16(tmax);
      tmax = xmax32(tmax);
      if (__any(tmax > m[gq] + th_raw)) {  // wave-uniform: rescale O and l to the new running max
        const float mn = fmaxf(m[gq], tmax);
        const float mref = (mn == -INFINITY) ? 0.f : mn;
        const float alpha = __builtin_amdgcn_exp2f((m[gq] - mref) * sl2);
        l[gq] *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[gq][d] *= alpha;
        m[gq] = mn;
      }
      const float mref = (m[gq] == -INFINITY) ? 0.f : m[gq];  // all-masked so far: exp2(-inf) = 0
      const float nbias = -mref * sl2;
      const f32x2_t sl2v = {sl2, sl2}, nb2 = {nbias, nbias};
      f32x2_t ls2 = {0.f, 0.f};
      uint64_t bits = 0;
      // dropout keep bits of the lane's 4 keys per block (generic contract form; fwd6 reads precomputed words)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        unsigned keep = 0xF;
        if constexpr (DROP) {
          keep = attn_keep4(a, bh, q[gq], k0 + kb * 16 + 4 * g);
          bits |= (uint64_t)keep << (kb * 16 + 4 * g);
        }
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const f32x2_t arg = f32x2_t{p[gq][kb][2 * jj], p[gq][kb][2 * jj + 1]} * sl2v + nb2;
          f32x2_t e = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
          ls2 += e;
          if constexpr (DROP) {
            e.x = ((keep >> (2 * jj)) & 1u) ? e.x : 0.f;
            e.y = ((keep >> (2 * jj + 1)) & 1u) ? e.y : 0.f;
          }
          p[gq][kb][2 * jj] = e.x;
          p[gq][kb][2 * jj + 1] = e.y;
        }
      }
      const float ls = ls2.x + ls2.y;
      if constexpr (DROP) {
        if (a.dbits) {  // the 4 lanes of a query hold disjoint key nibbles: OR them into the tile's 64-bit word
          unsigned lo = (unsigned)bits, hi = (unsigned)(bits >> 32);
          lo = xor16(lo);
          hi = xor16(hi);
          lo = xor32(lo);
          hi = xor32(hi);
          if (g == 0 && qv[gq]) a.dbits[((long)bh * ntiles + t) * a.Lq + q[gq]] = ((uint64_t)hi << 32) | lo;
        }
      }
      l[gq] += ls;
    }
    // O^T += V^T P^T for both query groups (one tr-read A fragment, two MFMAs)
    {
      const int qq = i >> 2, pp = i & 3;
      typedef __attribute__((address_space(3))) s16x4_t* lp;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        uint4 bq[NG];
#pragma unroll
        for (int gq = 0; gq < NG; ++gq) {
          bq[gq].x = pk(p[gq][2 * ss][0], p[gq][2 * ss][1]);
          bq[gq].y = pk(p[gq][2 * ss][2], p[gq][2 * ss][3]);
          bq[gq].z = pk(p[gq][2 * ss + 1][0], p[gq][2 * ss + 1][1]);
          bq[gq].w = pk(p[gq][2 * ss + 1][2], p[gq][2 * ss + 1][3]);
        }
        const int k1 = 32 * ss + 4 * g + qq, k2 = k1 + 16;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const int u = db * 4 + pp;
          const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(vimg + k1 * 128 + ((u ^ hatt(k1)) << 3)));
          const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(vimg + k2 * 128 + ((u ^ hatt(k2)) << 3)));
          const uint4 af = join_tr(lo, hi);
#pragma unroll
          for (int gq = 0; gq < NG; ++gq) mma<bf16_t>(o[gq][db], af, bq[gq]);
        }
      }
    }
  };
  auto arrive = [&](int t) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NST - 2)) : "memory");  // own pieces of tile t landed
    __builtin_amdgcn_s_barrier();
    fill(min(t + NST - 1, ntiles - 1), (t + NST - 1) % NST);  // into the stage of tile t - 1
  };
  // the mask row only where it can be non-zero: every tile with a key-padding mask, else only the ragged last one
  if (MASK && a.key_keep != nullptr) {
    for (int t = 0; t < ntiles; ++t) {
      arrive(t);
      tile(t, std::integral_constant<bool, MASK>{});
    }
  } else {
    for (int t = 0; t + 1 < ntiles; ++t) {
      arrive(t);
      tile(t, std::false_type{});
    }
    arrive(ntiles - 1);
    tile(ntiles - 1, std::integral_constant<bool, MASK>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup retires
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    float lt = l[gq];
    lt = xsum16(lt);
    lt = xsum32(lt);
    if (!qv[gq]) continue;
    const float inv = (lt > 0.f) ? 1.f / lt : NAN;  // fully masked row -> NaN like softmax(all -inf)
    bf16_t* Ob = (bf16_t*)a.Out + ((long)b * a.Lq + q[gq]) * a.so + h * DH;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint2 u2;
      u2.x = pk(o[gq][d][0] * inv, o[gq][d][1] * inv);
      u2.y = pk(o[gq][d][2] * inv, o[gq][d][3] * inv);
      *(uint2*)(Ob + d * 16 + 4 * g) = u2;
    }
    if (a.lse && g == 0)
      a.lse[(long)bh * a.Lq + q[gq]] = (lt > 0.f) ? (m[gq] * sl2 + __log2f(lt)) * 0.69314718055994531f : NAN;
  }
}

// ------------------------------------------------------------------ dropout keep bits (contract v2, producer)
// The keep bits of one or more attention sites, written ahead of the attention forward (fwd6 reads them; the backward
// kernels read the same words): word ((bh * ntiles + t) * Lq + q) of site s, bit kk = keep(q, key 64 t + kk) under
// rng stream stream0 + s * stream_step. One workgroup per (b, h, site) builds that pair's three 4096-entry draw tables
// in LDS (one splitmix64 per 4 entries), then each thread owns queries and walks their key tiles (coalesced word
// stores per tile). Bit-identical to the words fwd6 records when it draws the bits from its own LDS tables (DM 2).
struct DbArgs {
  uint64_t* out;
  long site_words;  // words per site
  int BH, Lq, Lk;
  uint64_t seed, stream0, stream_step;
  unsigned thr16;
  const uint64_t* seed_off;  // graph-replay seed offset (common.h eff_seed) or null
};

__global__ void __launch_bounds__(256) dbits_kernel(DbArgs d) {
  __shared__ __attribute__((aligned(16))) uint64_t tab[3 * ATTN_R / 4];
  const int bh = blockIdx.x, site = blockIdx.y, tid = threadIdx.x;
  const uint64_t stream = d.stream0 + (uint64_t)site * d.stream_step;
  const uint64_t seed = eff_seed(d.seed, d.seed_off);
  for (int wi = tid; wi < 3 * ATTN_R / 4; wi += 256) {
    const int tau = wi / (ATTN_R / 4), jw = wi % (ATTN_R / 4);
    tab[wi] = mix64(seed, stream, ATTN_TAB0 + ((uint64_t)bh * 3 + tau) * (ATTN_R / 4) + jw);
  }
  __syncthreads();
  const int ntiles = (d.Lk + 63) / 64;
  uint64_t* out = d.out + (long)site * d.site_words + (long)bh * ntiles * d.Lq;
  const unsigned char* tb = (const unsigned char*)tab;
  for (int q = tid; q < d.Lq; q += 256) {
    const uint64_t off = mix64(seed, stream, ATTN_OFF0 + (uint64_t)bh * d.Lq + q);
    const unsigned o0 = (unsigned)(off & 0xFFCu), o1 = (unsigned)((off >> 16) & 0xFFCu),
                   o2 = (unsigned)((off >> 32) & 0xFFCu);
    for (int t = 0; t < ntiles; ++t) {
      uint64_t word = 0;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const unsigned kq = 64 * t + 4 * c;
        const uint64_t w = *(const uint64_t*)(tb + (((o0 + kq) & (ATTN_R - 1)) << 1)) ^
                           *(const uint64_t*)(tb + ATTN_R * 2 + (((o1 + kq) & (ATTN_R - 1)) << 1)) ^
                           *(const uint64_t*)(tb + ATTN_R * 4 + (((o2 + kq) & (ATTN_R - 1)) << 1));
        unsigned keep = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) keep |= (((unsigned)(w >> (16 * j)) & 0xFFFFu) >= d.thr16 ? 1u : 0u) << j;
        word |= (uint64_t)keep << (4 * c);
      }
      out[(long)t * d.Lq + q] = word;
    }
  }
}

// ---------------------------------------------------------------- fwd (bf16, decoder, streamed ring, v6)
// The decoder's self- and cross-attention forward (key-padding mask, dropout from precomputed keep bits): fwd5's
// streamed K / V ring (2 LDS stages filled by LDS-DMA one tile ahead, counted vmcnt + one barrier per tile) with
// the round-2 resident-K/V forward's tile body, and the dropout keep bits read from the words dbits_kernel wrote (staged in LDS for the
// workgroup's queries: one ds_read_b64 per tile and query instead of three table lookups, two XORs and four compares
// per 4 keys). 4 waves x NG query groups of 16 = 64 NG queries per workgroup and 34-38 KB of LDS at Lk <= 512, so
// three to four workgroups share a CU and one workgroup's K / V loads overlap another's MFMA / softmax work (the resident forward held
// the whole K / V range of a (b, h) in ~158 KB at Lk = 512: one workgroup per CU, 1.5 rounds of workgroups at C4).
// Key tiles whose 64 keys are all padding are skipped (neither loaded nor computed).
// MK: 0 no mask, 1 the ragged last tile only (Lk % 64 != 0, no key-padding mask), 2 key-padding mask on every tile.
// DM: 0 no dropout, 1 keep bits read from words dbits_kernel wrote, 2 keep bits drawn from the contract's three
// tables built in LDS and recorded in dbits for the backward.
template <int DM, int MK, int NG>
__global__ void __launch_bounds__(256, NG == 1 ? 4 : 2) fwd6_kernel(AttnArgs a) {
  constexpr bool MASK = MK != 0, DROP = DM != 0;
  constexpr int QW = 64 * NG, TB = 64 * 128, RB = 128, NST = 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm6[];
  const int ntiles = (a.Lk + 63) / 64, LkP = ntiles * 64;
  unsigned char* kst = sm6;                     // [NST][64 rows][128 B] K, KC image
  unsigned char* vst = sm6 + NST * TB;          // [NST][64 rows][128 B] V, tr-read image
  float* mfull = (float*)(sm6 + 2 * NST * TB);  // [LkP] 0 / -inf
  uint64_t* kbits = (uint64_t*)(mfull + LkP);   // DM 1: [ntiles][QW] keep words of the workgroup's queries
  unsigned char* dtab = (unsigned char*)(mfull + LkP);  // DM 2: [3][4096] u16 draw tables
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int qbase = bxi * QW;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  // ---- ordinary loads first (Q fragments, mask row, keep words); hipcc waits for them before the stream starts
  int q[NG];
  bool qv[NG];
  uint4 qf[NG][2];
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    q[gq] = qbase + w * (16 * NG) + gq * 16 + i;
    qv[gq] = q[gq] < a.Lq;
    row_frags<bf16_t>(qf[gq], Qb, a.sq, qv[gq] ? q[gq] : 0, qv[gq], lane);
  }
  for (int k = tid; k < LkP; k += 256) mfull[k] = (MASK && !key_ok(a, b, k)) ? -INFINITY : 0.f;
  if constexpr (DM == 1) {
    const uint64_t* src = a.dbits + (long)bh * ntiles * a.Lq;
    for (int e = tid; e < ntiles * QW; e += 256) {
      const int t = e / QW, qq = e - t * QW;
      kbits[e] = (qbase + qq < a.Lq) ? src[(long)t * a.Lq + qbase + qq] : 0ull;
    }
  }
  unsigned ooff[NG][3];  // DM 2: the rows' table offsets
  if constexpr (DM == 2) {
    for (int wi = tid; wi < 3 * ATTN_R / 4; wi += 256) {
      const int tau = wi / (ATTN_R / 4), jw = wi % (ATTN_R / 4);
      *(uint64_t*)(dtab + (size_t)wi * 8) =
          mix64(eff_seed(a.seed, a.seed_off), a.stream, ATTN_TAB0 + ((uint64_t)bh * 3 + tau) * (ATTN_R / 4) + jw);
    }
#pragma unroll
    for (int gq = 0; gq < NG; ++gq) {
      const uint64_t off = attn_offsets(a, bh, q[gq]);
#pragma unroll
      for (int tau = 0; tau < 3; ++tau) ooff[gq][tau] = (unsigned)((off >> (16 * tau)) & 0xFFCu);
    }
  }
  // active key tiles (wave-uniform): with a key-padding mask, tiles whose keys are all padding add exactly nothing
  unsigned tmask = ntiles >= 32 ? 0xFFFFFFFFu : ((1u << ntiles) - 1u);
  if (MK == 2) {
    tmask = 0;
    for (int t = 0; t < ntiles; ++t)
      if (__any(key_ok(a, b, 64 * t + lane))) tmask |= 1u << t;
  }
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    pin16(qf[gq][0]);
    pin16(qf[gq][1]);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // ---- K / V stream: wave w fills rows 16w .. 16w+15 of a tile (2 K + 2 V instructions; XOR swizzles on the
  // per-lane source addresses)
  auto fill = [&](int tt, int st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int R = 16 * w + 8 * u;
      const int r = 64 * tt + R + (lane >> 3), pch = lane & 7;
      const int rr = min(r, a.Lk - 1);
      const int ck = pch ^ ((r >> 1) & 7), cv = pch ^ (((r >> 1) & 3) << 1);
      dma16_asm(Kb + (long)rr * a.sk + ck * 8, kst + st * TB + R * 128);
      dma16_asm(Vb + (long)rr * a.sv + cv * 8, vst + st * TB + R * 128);
    }
  };
  unsigned rem = tmask;
  int tcur = rem ? __builtin_ctz(rem) : -1;
  if (tcur >= 0) fill(tcur, 0);

  const float sl2 = a.scale * 1.4426950408889634f;  // running max m is kept in raw units, p = 2^(x*sl2 - m*sl2)
  float m[NG], l[NG];
  f32x4_t o[NG][4];
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    m[gq] = -INFINITY;
    l[gq] = 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[gq][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  const float th_raw = 8.f / sl2;  // lazy rescale threshold (raw score units), as in fwd2_kernel
  auto tile = [&](const int t, const int st, auto mc) {
    constexpr bool MT = decltype(mc)::value;  // this tile adds the mask row
    const int k0 = t * 64;
    const unsigned char* kimg = kst + st * TB;
    const unsigned char* vimg = vst + st * TB;
    f32x4_t s[NG][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
      for (int gq = 0; gq < NG; ++gq) s[gq][kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const uint4 af = *(const uint4*)(kimg + kc_off(RB, kb * 16 + i, sub * 4 + g));
#pragma unroll
        for (int gq = 0; gq < NG; ++gq) mma<bf16_t>(s[gq][kb], af, qf[gq][sub]);
      }
    }
    f32x2_t mrow[4][2];
    if constexpr (MT) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float4 mv4 = *(const float4*)(&mfull[k0 + kb * 16 + 4 * g]);
        mrow[kb][0] = f32x2_t{mv4.x, mv4.y};
        mrow[kb][1] = f32x2_t{mv4.z, mv4.w};
      }
    }
    float p[NG][4][4];
#pragma unroll
    for (int gq = 0; gq < NG; ++gq) {
      uint64_t kw = 0;
      if constexpr (DM == 1) kw = kbits[t * QW + w * (16 * NG) + gq * 16 + i];
      if constexpr (DM == 2) {
        // 4 x 16-bit draws per 4 keys: one aligned 8-byte word from each table, XORed
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const int kq = k0 + kb * 16 + 4 * g;
          const uint64_t wd = *(const uint64_t*)(dtab + (((ooff[gq][0] + kq) & (ATTN_R - 1)) << 1)) ^
                              *(const uint64_t*)(dtab + ATTN_R * 2 + (((ooff[gq][1] + kq) & (ATTN_R - 1)) << 1)) ^
                              *(const uint64_t*)(dtab + ATTN_R * 4 + (((ooff[gq][2] + kq) & (ATTN_R - 1)) << 1));
          unsigned keep = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) keep |= (((unsigned)(wd >> (16 * j)) & 0xFFFFu) >= a.thr16 ? 1u : 0u) << j;
          kw |= (uint64_t)keep << (kb * 16 + 4 * g);
        }
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          f32x2_t x = {s[gq][kb][2 * jj], s[gq][kb][2 * jj + 1]};
          if constexpr (MT) x += mrow[kb][jj];
          p[gq][kb][2 * jj] = x.x;
          p[gq][kb][2 * jj + 1] = x.y;
        }
        tmax = fmaxf(tmax, fmaxf(fmaxf(p[gq][kb][0], p[gq][kb][1]), fmaxf(p[gq][kb][2], p[gq][kb][3])));
      }
      tmax = xmax16(tmax);
      tmax = xmax32(tmax);
      if (__any(tmax > m[gq] + th_raw)) {
        const float mn = fmaxf(m[gq], tmax);
        const float mref = (mn == -INFINITY) ? 0.f : mn;
        const float alpha = __builtin_amdgcn_exp2f((m[gq] - mref) * sl2);
        l[gq] *= alpha;
#pragma unroll
        for (int d = 0; d < 4; ++d) o[gq][d] *= alpha;
        m[gq] = mn;
      }
      const float mref = (m[gq] == -INFINITY) ? 0.f : m[gq];
      const float nbias = -mref * sl2;
      const f32x2_t sl2v = {sl2, sl2}, nb2 = {nbias, nbias};
      f32x2_t ls2 = {0.f, 0.f};
      const unsigned kwh[2] = {(unsigned)kw, (unsigned)(kw >> 32)};
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const f32x2_t arg = f32x2_t{p[gq][kb][2 * jj], p[gq][kb][2 * jj + 1]} * sl2v + nb2;
          f32x2_t e = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
          ls2 += e;
          if constexpr (DROP) {
            // keep bit of key kb*16 + 4g + 2jj (+1) as an all-ones / zero AND mask (v_bfe_i32)
            const unsigned hw = kwh[kb >> 1];
            const int pos = (kb & 1) * 16 + 4 * g + 2 * jj;
            const unsigned m0 = (unsigned)__builtin_amdgcn_sbfe((int)hw, pos, 1);
            const unsigned m1 = (unsigned)__builtin_amdgcn_sbfe((int)hw, pos + 1, 1);
            e.x = __uint_as_float(__float_as_uint(e.x) & m0);
            e.y = __uint_as_float(__float_as_uint(e.y) & m1);
          }
          p[gq][kb][2 * jj] = e.x;
          p[gq][kb][2 * jj + 1] = e.y;
        }
      }
      l[gq] += ls2.x + ls2.y;
      if constexpr (DM == 2) {
        if (a.dbits) {  // the 4 lanes of a query hold disjoint key nibbles: OR them into the tile's 64-bit word
          unsigned lo = (unsigned)kw, hi = (unsigned)(kw >> 32);
          lo = xor16(lo);
          hi = xor16(hi);
          lo = xor32(lo);
          hi = xor32(hi);
          if (g == 0 && qv[gq]) a.dbits[((long)bh * ntiles + t) * a.Lq + q[gq]] = ((uint64_t)hi << 32) | lo;
        }
      }
    }
    {
      const int qq = i >> 2, pp = i & 3;
      typedef __attribute__((address_space(3))) s16x4_t* lp;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        uint4 bq[NG];
#pragma unroll
        for (int gq = 0; gq < NG; ++gq) {
          bq[gq].x = pk(p[gq][2 * ss][0], p[gq][2 * ss][1]);
          bq[gq].y = pk(p[gq][2 * ss][2], p[gq][2 * ss][3]);
          bq[gq].z = pk(p[gq][2 * ss + 1][0], p[gq][2 * ss + 1][1]);
          bq[gq].w = pk(p[gq][2 * ss + 1][2], p[gq][2 * ss + 1][3]);
        }
        const int k1 = 32 * ss + 4 * g + qq, k2 = k1 + 16;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const int u = db * 4 + pp;
          const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(vimg + k1 * 128 + ((u ^ hatt(k1)) << 3)));
          const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(vimg + k2 * 128 + ((u ^ hatt(k2)) << 3)));
          const uint4 af = join_tr(lo, hi);
#pragma unroll
          for (int gq = 0; gq < NG; ++gq) mma<bf16_t>(o[gq][db], af, bq[gq]);
        }
      }
    }
  };
  // one active tile per iteration: wait for its pieces (the only DMA in flight), barrier (every wave's pieces landed
  // and every wave finished the previous tile, whose stage the next fill overwrites), fill the next active tile, run
  int st = 0;
  auto arrive = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    rem &= rem - 1;
    const int tnext = rem ? __builtin_ctz(rem) : -1;
    if (tnext >= 0) fill(tnext, st ^ 1);
    return tnext;
  };
  if constexpr (MK == 1) {  // every tile active; the mask row only on the ragged last one
    while (tcur >= 0 && tcur < ntiles - 1) {
      const int tnext = arrive();
      tile(tcur, st, std::false_type{});
      tcur = tnext;
      st ^= 1;
    }
    if (tcur >= 0) {
      arrive();
      tile(tcur, st, std::true_type{});
    }
  } else {
    while (tcur >= 0) {
      const int tnext = arrive();
      tile(tcur, st, std::integral_constant<bool, MK == 2>{});
      tcur = tnext;
      st ^= 1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup retires
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) {
    float lt = l[gq];
    lt = xsum16(lt);
    lt = xsum32(lt);
    if (!qv[gq]) continue;
    const float inv = (lt > 0.f) ? (DROP ? a.drop_scale : 1.f) / lt : NAN;
    bf16_t* Ob = (bf16_t*)a.Out + ((long)b * a.Lq + q[gq]) * a.so + h * DH;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint2 u2;
      u2.x = pk(o[gq][d][0] * inv, o[gq][d][1] * inv);
      u2.y = pk(o[gq][d][2] * inv, o[gq][d][3] * inv);
      *(uint2*)(Ob + d * 16 + 4 * g) = u2;
    }
    if (a.lse && g == 0)
      a.lse[(long)bh * a.Lq + q[gq]] = (lt > 0.f) ? (m[gq] * sl2 + __log2f(lt)) * 0.69314718055994531f : NAN;
  }
}

// ------------------------------------------------------------------------------------------- dQ
// query-owned: recompute S^T, dP^T = V dO^T; dS = P (dP - delta); dQ^T = K^T dS^T
template <typename T>
__global__ void __launch_bounds__(256) dq_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int RB = Cfg<T>::RB;
  unsigned char* kimg = smem;             // K rows (KC)
  unsigned char* ktimg = smem + 64 * RB;  // K transposed reads (MC)
  unsigned char* vimg = smem + 128 * RB;  // V rows (KC)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int q = bxi * 64 + w * 16 + i;
  const bool qv = q < a.Lq;
  const int qq = qv ? q : 0;
  const T* Qb = (const T*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const T* Ob = (const T*)a.O + (long)b * a.Lq * a.so + h * DH;
  const T* dOb = (const T*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const T* Kb = (const T*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const T* Vb = (const T*)a.V + (long)b * a.Lk * a.sv + h * DH;
  uint4 qf[Cfg<T>::NSUB], dof[Cfg<T>::NSUB], of[Cfg<T>::NSUB];
  row_frags<T>(qf, Qb, a.sq, qq, qv, lane);
  row_frags<T>(dof, dOb, a.sdo, qq, qv, lane);
  row_frags<T>(of, Ob, a.so, qq, qv, lane);
  // delta = rowsum(dO * O) over this lane's chunks, then across the 4 lane groups
  float delta = 0.f;
#pragma unroll
  for (int s = 0; s < Cfg<T>::NSUB; ++s) {
    const T* x = (const T*)&dof[s];
    const T* y = (const T*)&of[s];
#pragma unroll
    for (int e = 0; e < Cfg<T>::ECH; ++e) delta += ld<T>(x + e) * ld<T>(y + e);
  }
  delta = xsum16(delta);
  delta = xsum32(delta);
  if (qv && g == 0) a.delta[(long)bh * a.Lq + q] = delta;
  const float lse = qv ? a.lse[(long)bh * a.Lq + q] : 0.f;

  f32x4_t dq[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) dq[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < a.Lk; k0 += 64) {
    const int nv = min(64, a.Lk - k0);
    __syncthreads();
    stage<T>(kimg, ktimg, Kb, a.sk, k0, nv);
    stage<T>(vimg, nullptr, Vb, a.sv, k0, nv);
    __syncthreads();
    f32x4_t s[4], dp[4];
    rows_times_frag<T>(s, kimg, qf, lane);
    rows_times_frag<T>(dp, vimg, dof, lane);
    float ds[4][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = k0 + kb * 16 + 4 * g + j;
        float pr = 0.f;
        if (key_ok(a, b, key) && qv) pr = __expf(s[kb][j] * a.scale - lse);
        float dpv = dp[kb][j];
        if (a.thr16) dpv = attn_keep(a, bh, q, key) ? dpv * a.drop_scale : 0.f;
        ds[kb][j] = pr * (dpv - delta);
      }
    trans_times_vals<T>(dq, ktimg, ds, lane);
  }
  if (!qv) return;
  T* dQb = (T*)a.dQ + ((long)b * a.Lq + q) * a.sdq + h * DH;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int j = 0; j < 4; ++j) st<T>(dQb + d * 16 + 4 * g + j, dq[d][j] * a.scale);
}

// ------------------------------------------------------------------------------------------- dK dV
// key-owned: S = Q K^T (lane = key), dP = dO V^T, dV^T = dO^T P_drop, dK^T = Q^T dS
template <typename T>
__global__ void __launch_bounds__(256) dkv_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int RB = Cfg<T>::RB;
  unsigned char* qimg = smem;
  unsigned char* qtimg = smem + 64 * RB;
  unsigned char* doimg = smem + 128 * RB;
  unsigned char* dotimg = smem + 192 * RB;
  float* lse_s = (float*)(smem + 256 * RB);
  float* del_s = lse_s + 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int key = bxi * 64 + w * 16 + i;
  const bool kv = key < a.Lk;
  const bool kok = key_ok(a, b, kv ? key : 0) && kv;
  const T* Qb = (const T*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const T* dOb = (const T*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const T* Kb = (const T*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const T* Vb = (const T*)a.V + (long)b * a.Lk * a.sv + h * DH;
  uint4 kf[Cfg<T>::NSUB], vf[Cfg<T>::NSUB];
  row_frags<T>(kf, Kb, a.sk, kv ? key : 0, kv, lane);
  row_frags<T>(vf, Vb, a.sv, kv ? key : 0, kv, lane);

  f32x4_t dk[4], dv[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) dk[d] = dv[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int q0 = 0; q0 < a.Lq; q0 += 64) {
    const int nv = min(64, a.Lq - q0);
    __syncthreads();
    stage<T>(qimg, qtimg, Qb, a.sq, q0, nv);
    stage<T>(doimg, dotimg, dOb, a.sdo, q0, nv);
    if (threadIdx.x < 64) {
      const int qq = q0 + threadIdx.x;
      float lv = 0.f, dl = 0.f;
      if (qq < a.Lq) {
        lv = a.lse[(long)bh * a.Lq + qq];
        dl = a.delta[(long)bh * a.Lq + qq];
      }
      lse_s[threadIdx.x] = lv;
      del_s[threadIdx.x] = dl;
    }
    __syncthreads();
    f32x4_t s[4], dp[4];
    rows_times_frag<T>(s, qimg, kf, lane);    // S[q = qb*16+4g+j][key = lane]
    rows_times_frag<T>(dp, doimg, vf, lane);  // dP[q][key]
    float pd[4][4], ds[4][4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ql = qb * 16 + 4 * g + j;
        const int qq = q0 + ql;
        float pr = 0.f;
        if (kok && qq < a.Lq) pr = __expf(s[qb][j] * a.scale - lse_s[ql]);
        float keep = 1.f;
        if (a.thr16) keep = attn_keep(a, bh, qq, key) ? a.drop_scale : 0.f;
        pd[qb][j] = pr * keep;
        ds[qb][j] = pr * (dp[qb][j] * keep - del_s[ql]);
      }
    trans_times_vals<T>(dv, dotimg, pd, lane);
    trans_times_vals<T>(dk, qtimg, ds, lane);
  }
  if (!kv) return;
  T* dKb = (T*)a.dK + ((long)b * a.Lk + key) * a.sdk + h * DH;
  T* dVb = (T*)a.dV + ((long)b * a.Lk + key) * a.sdv + h * DH;
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      st<T>(dKb + d * 16 + 4 * g + j, dk[d][j] * a.scale);
      st<T>(dVb + d * 16 + 4 * g + j, dv[d][j]);
    }
}

// ------------------------------------------------------------------------------- bwd (bf16, v2)
// Shared pieces of the 2-group backward kernels: out[gq][db] += A^T(MC image [k][d]) x v[gq] with one tr-read
// A fragment feeding both groups.
__device__ __forceinline__ void trans_times_vals2(f32x4_t (&out)[2][4], const unsigned char* img,
                                                  const float (&v)[2][4][4], int lane) {
  const int g = lane >> 4, i = lane & 15, qq = i >> 2, pp = i & 3;
  typedef __attribute__((address_space(3))) s16x4_t* lp;
#pragma unroll
  for (int ss = 0; ss < 2; ++ss) {
    uint4 bq[2];
#pragma unroll
    for (int gq = 0; gq < 2; ++gq) {
      bq[gq].x = pk(v[gq][2 * ss][0], v[gq][2 * ss][1]);
      bq[gq].y = pk(v[gq][2 * ss][2], v[gq][2 * ss][3]);
      bq[gq].z = pk(v[gq][2 * ss + 1][0], v[gq][2 * ss + 1][1]);
      bq[gq].w = pk(v[gq][2 * ss + 1][2], v[gq][2 * ss + 1][3]);
    }
    const int k1 = 32 * ss + 4 * g + qq, k2 = k1 + 16;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const int u = db * 4 + pp;
      const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + k1 * 128 + ((u ^ hatt(k1)) << 3)));
      const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + k2 * 128 + ((u ^ hatt(k2)) << 3)));
      const uint4 af = join_tr(lo, hi);
      mma<bf16_t>(out[0][db], af, bq[0]);
      mma<bf16_t>(out[1][db], af, bq[1]);
    }
  }
}

// dQ, query-owned: 128 queries per workgroup (two 16-query groups per wave), K/V tiles double-buffered.
// S^T = K Q^T and dP^T = V dO^T share the LDS row reads across both groups; dS = P (dP' - delta);
// dQ^T += K^T dS^T from the K MC image. Writes delta = rowsum(dO*O) for the dK/dV kernel.
// DM: 0 no dropout, 1 rehash the keep bits, 2 read the forward's recorded bits
template <int DM, bool MASK>
__global__ void __launch_bounds__(256, 2) dq2_kernel(AttnArgs a) {
  constexpr bool DROP = DM != 0;
  constexpr int RB = 128;
  __shared__ __attribute__((aligned(16))) unsigned char kc[2][64 * RB];
  __shared__ __attribute__((aligned(16))) unsigned char kt[2][64 * RB];
  __shared__ __attribute__((aligned(16))) unsigned char vc[2][64 * RB];
  __shared__ __attribute__((aligned(16))) float mbuf[2][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int qbase = bxi * 128;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Ob = (const bf16_t*)a.O + (long)b * a.Lq * a.so + h * DH;
  const bf16_t* dOb = (const bf16_t*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  const float sl2 = a.scale * 1.4426950408889634f;
  int q[2];
  bool qv[2];
  uint4 qf[2][2], dof[2][2];
  float delta[2], lse2[2];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    q[gq] = qbase + w * 32 + gq * 16 + i;
    qv[gq] = q[gq] < a.Lq;
    const int qq = qv[gq] ? q[gq] : 0;
    row_frags<bf16_t>(qf[gq], Qb, a.sq, qq, qv[gq], lane);
    row_frags<bf16_t>(dof[gq], dOb, a.sdo, qq, qv[gq], lane);
    uint4 of[2];
    row_frags<bf16_t>(of, Ob, a.so, qq, qv[gq], lane);
    float dl = 0.f;
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      const bf16_t* x = (const bf16_t*)&dof[gq][sb];
      const bf16_t* y = (const bf16_t*)&of[sb];
#pragma unroll
      for (int e = 0; e < 8; ++e) dl += bf2f(x[e]) * bf2f(y[e]);
    }
    dl = xsum16(dl);
    dl = xsum32(dl);
    delta[gq] = dl;
    if (qv[gq] && g == 0) a.delta[(long)bh * a.Lq + q[gq]] = dl;
    lse2[gq] = qv[gq] ? a.lse[(long)bh * a.Lq + q[gq]] * 1.4426950408889634f : 0.f;
  }
  uint4 kr[2], vr[2];
  float mv = 0.f;
  auto load = [&](int k0) {
    const int nv = min(64, a.Lk - k0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + 256 * u, r = idx >> 3, c = idx & 7;
      kr[u] = vr[u] = make_uint4(0, 0, 0, 0);
      if (r < nv) {
        kr[u] = *(const uint4*)(Kb + (long)(k0 + r) * a.sk + c * 8);
        vr[u] = *(const uint4*)(Vb + (long)(k0 + r) * a.sv + c * 8);
      }
    }
    if (MASK && tid >= 192) mv = key_ok(a, b, k0 + tid - 192) ? 0.f : -INFINITY;  // added to the exponent
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + 256 * u, r = idx >> 3, c = idx & 7;
      *(uint4*)(kc[buf] + kc_off(RB, r, c)) = kr[u];
      *(uint4*)(kt[buf] + r * 128 + (((2 * c) ^ hatt(r)) << 3)) = kr[u];
      *(uint4*)(vc[buf] + kc_off(RB, r, c)) = vr[u];
    }
    if (MASK && tid >= 192) mbuf[buf][tid - 192] = mv;
  };
  f32x4_t dq[2][4];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq)
#pragma unroll
    for (int d = 0; d < 4; ++d) dq[gq][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  const int ntiles = (a.Lk + 63) / 64;
  auto tile = [&](const int t, auto mc) {
    constexpr bool MT = decltype(mc)::value;  // this tile adds the mask row (see fwd2_kernel)
    const int cur = t & 1, k0 = t * 64;
    if (t + 1 < ntiles) load(k0 + 64);
    f32x4_t s[2][4], dp[2][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[0][kb] = s[1][kb] = dp[0][kb] = dp[1][kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const uint4 ak = *(const uint4*)(kc[cur] + kc_off(RB, kb * 16 + i, sub * 4 + g));
        const uint4 av = *(const uint4*)(vc[cur] + kc_off(RB, kb * 16 + i, sub * 4 + g));
        mma<bf16_t>(s[0][kb], ak, qf[0][sub]);
        mma<bf16_t>(s[1][kb], ak, qf[1][sub]);
        mma<bf16_t>(dp[0][kb], av, dof[0][sub]);
        mma<bf16_t>(dp[1][kb], av, dof[1][sub]);
      }
    }
    float mrow[4][4];
    if constexpr (MT) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        const float4 m4 = *(const float4*)(&mbuf[cur][kb * 16 + 4 * g]);
        mrow[kb][0] = m4.x; mrow[kb][1] = m4.y; mrow[kb][2] = m4.z; mrow[kb][3] = m4.w;
      }
    }
    uint64_t wbits[2] = {0, 0};
    if constexpr (DM == 2) {
#pragma unroll
      for (int gq = 0; gq < 2; ++gq) wbits[gq] = qv[gq] ? a.dbits[((long)bh * ntiles + t) * a.Lq + q[gq]] : 0;
    }
    // dS = P (dP' - delta), P = 2^(s*sl2 - lse2 + mask) (the 0/-inf mask row in the exponent instead of a select),
    // dP' = dP & keep (sign-extended keep bit, v_bfe_i32) * 1/(1-p); score pairs as float2 (packed v_pk_* f32)
    float ds[2][4][4];
    const f32x2_t sl2v = {sl2, sl2}, dscv = {a.drop_scale, a.drop_scale};
#pragma unroll
    for (int gq = 0; gq < 2; ++gq)
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        unsigned keep = 0xF;
        if constexpr (DM == 2) keep = (unsigned)(wbits[gq] >> (kb * 16 + 4 * g)) & 0xFu;
        if constexpr (DM == 1) keep = attn_keep4(a, bh, q[gq], k0 + kb * 16 + 4 * g);
        const f32x2_t ndl = {-delta[gq], -delta[gq]};
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          f32x2_t off = {-lse2[gq], -lse2[gq]};
          if constexpr (MT) off += f32x2_t{mrow[kb][2 * jj], mrow[kb][2 * jj + 1]};
          const f32x2_t arg = f32x2_t{s[gq][kb][2 * jj], s[gq][kb][2 * jj + 1]} * sl2v + off;
          const f32x2_t pr = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
          f32x2_t dpv = {dp[gq][kb][2 * jj], dp[gq][kb][2 * jj + 1]};
          if constexpr (DROP) {
            dpv.x = __int_as_float(__float_as_int(dpv.x) & __builtin_amdgcn_sbfe((int)keep, 2 * jj, 1));
            dpv.y = __int_as_float(__float_as_int(dpv.y) & __builtin_amdgcn_sbfe((int)keep, 2 * jj + 1, 1));
            dpv = dpv * dscv + ndl;
          } else {
            dpv += ndl;
          }
          const f32x2_t d2 = pr * dpv;
          ds[gq][kb][2 * jj] = d2.x;
          ds[gq][kb][2 * jj + 1] = d2.y;
        }
      }
    trans_times_vals2(dq, kt[cur], ds, lane);
    if (t + 1 < ntiles) {
      store(cur ^ 1);
      __syncthreads();
    }
  };
  if (MASK && a.key_keep != nullptr) {
    unsigned tmask = 0;  // fully padded key tiles, skipped as in fwd6_kernel
    for (int t = 0; t < ntiles; ++t)
      if (__any(key_ok(a, b, 64 * t + lane))) tmask |= 1u << (t & 31);
    for (int t = 0; t < ntiles; ++t) {
      if (ntiles > 32 || ((tmask >> t) & 1u)) tile(t, std::integral_constant<bool, MASK>{});
      else if (t + 1 < ntiles) {  // keep the tile pipeline: the next tile's loads, stores and barrier
        if (t + 1 < ntiles) load((t + 1) * 64);
        store((t & 1) ^ 1);
        __syncthreads();
      }
    }
  } else {
    for (int t = 0; t + 1 < ntiles; ++t) tile(t, std::false_type{});
    tile(ntiles - 1, std::integral_constant<bool, MASK>{});
  }
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    if (!qv[gq]) continue;
    bf16_t* dQb = (bf16_t*)a.dQ + ((long)b * a.Lq + q[gq]) * a.sdq + h * DH;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint2 u2;
      u2.x = pk(dq[gq][d][0] * a.scale, dq[gq][d][1] * a.scale);
      u2.y = pk(dq[gq][d][2] * a.scale, dq[gq][d][3] * a.scale);
      *(uint2*)(dQb + d * 16 + 4 * g) = u2;
    }
  }
}

// One KC-layout image per operand serves both the row reads and the transposed ds_read_b64_tr_b16 reads: the
// 8-byte unit u of row k sits at kc_tr_off(k, u), through the same XOR swizzle as kc_off.
__device__ __forceinline__ int kc_tr_off(int k, int u) {  // 8-byte unit u of row k in a KC image
  return k * 128 + ((((u >> 1) ^ ((k >> 1) & 7)) << 4) | ((u & 1) << 3));
}

// dK, dV, key-owned: 128 keys per workgroup (two 16-key groups per wave), Q/dO tiles double-buffered
// (row images for S, dP and transposed images for dV^T += dO^T P', dK^T += Q^T dS).
template <int DM>
__global__ void __launch_bounds__(256, (DM == 1 ? 1 : 2)) dkv2_kernel(AttnArgs a) {
  constexpr bool DROP = DM != 0;
  constexpr int RB = 128;
  __shared__ __attribute__((aligned(16))) unsigned char qc[2][64 * RB];
  __shared__ __attribute__((aligned(16))) unsigned char qt[2][64 * RB];
  __shared__ __attribute__((aligned(16))) unsigned char oc[2][64 * RB];
  __shared__ __attribute__((aligned(16))) unsigned char ot[2][64 * RB];
  __shared__ float lse_s[2][64], del_s[2][64];
  __shared__ __attribute__((aligned(16))) uint64_t wb_s[2][2][64];  // [buf][key tile of the block][query]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int kbase = bxi * 128;
  const int ntk = (a.Lk + 63) / 64;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* dOb = (const bf16_t*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  const float sl2 = a.scale * 1.4426950408889634f;
  int key[2];
  bool kvld[2], kok[2];
  uint4 kf[2][2], vf[2][2];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    key[gq] = kbase + w * 32 + gq * 16 + i;
    kvld[gq] = key[gq] < a.Lk;
    kok[gq] = kvld[gq] && key_ok(a, b, key[gq]);
    row_frags<bf16_t>(kf[gq], Kb, a.sk, kvld[gq] ? key[gq] : 0, kvld[gq], lane);
    row_frags<bf16_t>(vf[gq], Vb, a.sv, kvld[gq] ? key[gq] : 0, kvld[gq], lane);
  }
  uint4 qr[2], orr[2];
  float lv = 0.f;
  uint64_t wv = 0;
  auto load = [&](int q0) {
    const int nv = min(64, a.Lq - q0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + 256 * u, r = idx >> 3, c = idx & 7;
      qr[u] = orr[u] = make_uint4(0, 0, 0, 0);
      if (r < nv) {
        qr[u] = *(const uint4*)(Qb + (long)(q0 + r) * a.sq + c * 8);
        orr[u] = *(const uint4*)(dOb + (long)(q0 + r) * a.sdo + c * 8);
      }
    }
    if (tid < 128) {
      const int qq = q0 + (tid & 63);
      lv = 0.f;
      if (qq < a.Lq) lv = tid < 64 ? a.lse[(long)bh * a.Lq + qq] * 1.4426950408889634f : a.delta[(long)bh * a.Lq + qq];
    }
    if (DM == 2 && tid >= 128) {
      const int qq = q0 + (tid & 63), kt = 2 * bxi + ((tid - 128) >> 6);
      wv = (qq < a.Lq && kt < ntk) ? a.dbits[((long)bh * ntk + kt) * a.Lq + qq] : 0;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = tid + 256 * u, r = idx >> 3, c = idx & 7;
      *(uint4*)(qc[buf] + kc_off(RB, r, c)) = qr[u];
      *(uint4*)(qt[buf] + r * 128 + (((2 * c) ^ hatt(r)) << 3)) = qr[u];
      *(uint4*)(oc[buf] + kc_off(RB, r, c)) = orr[u];
      *(uint4*)(ot[buf] + r * 128 + (((2 * c) ^ hatt(r)) << 3)) = orr[u];
    }
    if (tid < 64) lse_s[buf][tid] = lv;
    else if (tid < 128) del_s[buf][tid - 64] = lv;
    if (DM == 2 && tid >= 128) wb_s[buf][(tid - 128) >> 6][tid & 63] = wv;
  };
  f32x4_t dk[2][4], dv[2][4];
#pragma unroll
  for (int gq = 0; gq < 2; ++gq)
#pragma unroll
    for (int d = 0; d < 4; ++d) dk[gq][d] = dv[gq][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  // a block whose 128 keys are all padding: zero dK / dV (epilogue), no query loop
  const int ntiles = __syncthreads_or(kok[0] || kok[1]) ? (a.Lq + 63) / 64 : 0;
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1, q0 = t * 64;
    if (t + 1 < ntiles) load(q0 + 64);
    f32x4_t s[2][4], dp[2][4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      s[0][qb] = s[1][qb] = dp[0][qb] = dp[1][qb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const uint4 aq = *(const uint4*)(qc[cur] + kc_off(RB, qb * 16 + i, sub * 4 + g));
        const uint4 ao = *(const uint4*)(oc[cur] + kc_off(RB, qb * 16 + i, sub * 4 + g));
        mma<bf16_t>(s[0][qb], aq, kf[0][sub]);
        mma<bf16_t>(s[1][qb], aq, kf[1][sub]);
        mma<bf16_t>(dp[0][qb], ao, vf[0][sub]);
        mma<bf16_t>(dp[1][qb], ao, vf[1][sub]);
      }
    }
    // P = 2^(s*sl2 - lse2); P' = P & keep, dS = P (dP & keep * 1/(1-p) - delta) (the keep bit sign-extended by
    // v_bfe_i32; the 1/(1-p) of P' goes on dV once at the end). Query pairs as float2 (packed v_pk_* f32). The
    // lane owns one key: a masked key's P is not zeroed per score — its dK/dV column is written as zeros.
    float pd[2][4][4], ds[2][4][4];
    const int kbit = (w * 32 + i) & 63;  // key bit within its tile (groups gq add 16): the word half is w & 1
    const f32x2_t sl2v = {sl2, sl2}, dscv = {a.drop_scale, a.drop_scale};
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      const float4 l4 = *(const float4*)(&lse_s[cur][qb * 16 + 4 * g]);
      const float4 d4 = *(const float4*)(&del_s[cur][qb * 16 + 4 * g]);
      const f32x2_t nl[2] = {f32x2_t{-l4.x, -l4.y}, f32x2_t{-l4.z, -l4.w}};
      const f32x2_t nd[2] = {f32x2_t{-d4.x, -d4.y}, f32x2_t{-d4.z, -d4.w}};
      unsigned wq[4] = {0, 0, 0, 0};  // the 32-bit half of each query's keep word holding this wave's keys
      if constexpr (DM == 2) {
        const unsigned* src = (const unsigned*)&wb_s[cur][w >> 1][qb * 16 + 4 * g] + (w & 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) wq[j] = src[2 * j];
      }
#pragma unroll
      for (int gq = 0; gq < 2; ++gq) {
        const int kb5 = (kbit + 16 * gq) & 31;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const f32x2_t arg = f32x2_t{s[gq][qb][2 * jj], s[gq][qb][2 * jj + 1]} * sl2v + nl[jj];
          f32x2_t pr = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
          f32x2_t dpv = {dp[gq][qb][2 * jj], dp[gq][qb][2 * jj + 1]};
          f32x2_t pdv = pr;
          if constexpr (DROP) {
            int m0, m1;
            if constexpr (DM == 2) {
              m0 = __builtin_amdgcn_sbfe((int)wq[2 * jj], kb5, 1);
              m1 = __builtin_amdgcn_sbfe((int)wq[2 * jj + 1], kb5, 1);
            } else {
              const int qq = q0 + qb * 16 + 4 * g + 2 * jj;
              m0 = attn_keep(a, bh, qq, key[gq]) ? -1 : 0;
              m1 = attn_keep(a, bh, qq + 1, key[gq]) ? -1 : 0;
            }
            pdv.x = __int_as_float(__float_as_int(pr.x) & m0);
            pdv.y = __int_as_float(__float_as_int(pr.y) & m1);
            dpv.x = __int_as_float(__float_as_int(dpv.x) & m0);
            dpv.y = __int_as_float(__float_as_int(dpv.y) & m1);
            dpv = dpv * dscv + nd[jj];
          } else {
            dpv += nd[jj];
          }
          const f32x2_t d2 = pr * dpv;
          pd[gq][qb][2 * jj] = pdv.x;
          pd[gq][qb][2 * jj + 1] = pdv.y;
          ds[gq][qb][2 * jj] = d2.x;
          ds[gq][qb][2 * jj + 1] = d2.y;
        }
      }
    }
    trans_times_vals2(dv, ot[cur], pd, lane);
    trans_times_vals2(dk, qt[cur], ds, lane);
    if (t + 1 < ntiles) {
      store(cur ^ 1);
      __syncthreads();
    }
  }
#pragma unroll
  for (int gq = 0; gq < 2; ++gq) {
    if (!kvld[gq]) continue;
    bf16_t* dKb = (bf16_t*)a.dK + ((long)b * a.Lk + key[gq]) * a.sdk + h * DH;
    bf16_t* dVb = (bf16_t*)a.dV + ((long)b * a.Lk + key[gq]) * a.sdv + h * DH;
    // masked key: zero gradient (its P was never zeroed); dV carries the dropout scale of P'
    const float ksc = kok[gq] ? a.scale : 0.f, vsc = kok[gq] ? (DROP ? a.drop_scale : 1.f) : 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint2 uk, uv;
      uk.x = pk(kok[gq] ? dk[gq][d][0] * ksc : 0.f, kok[gq] ? dk[gq][d][1] * ksc : 0.f);
      uk.y = pk(kok[gq] ? dk[gq][d][2] * ksc : 0.f, kok[gq] ? dk[gq][d][3] * ksc : 0.f);
      uv.x = pk(kok[gq] ? dv[gq][d][0] * vsc : 0.f, kok[gq] ? dv[gq][d][1] * vsc : 0.f);
      uv.y = pk(kok[gq] ? dv[gq][d][2] * vsc : 0.f, kok[gq] ? dv[gq][d][3] * vsc : 0.f);
      *(uint2*)(dKb + d * 16 + 4 * g) = uk;
      *(uint2*)(dVb + d * 16 + 4 * g) = uv;
    }
  }
}

// --------------------------------------------------------------------- bwd (bf16, streamed ring, v4)
// the round-2 resident-operand kernels' (dq3 / dkv3) tile bodies (one KC image per operand serving the row reads and, through kc_tr_off, the transposed
// reads; 16 rows per wave) with the streamed operand pair in a 2-stage LDS ring filled by LDS-DMA one tile ahead
// (fwd6's scheme: inline-asm DMA, vmcnt(0) + one barrier per tile, no other vector-memory instruction in the loop)
// instead of resident in LDS: 4 waves x 16 rows = 64 rows per workgroup and 36-40 KB of LDS at L <= 512, so four
// workgroups share a CU (the resident v3 kernels need one 133-148 KB workgroup per CU at L = 512; the register-staged
// v2 kernels run two 2-group workgroups at 2 waves per SIMD). The side data (mask row, LSE / delta rows, the
// forward's keep words) is staged in LDS once. DM: 0 no dropout, 2 the recorded keep bits.
template <int DM, bool MASK>
__global__ void __launch_bounds__(256, 4) dq4_kernel(AttnArgs a) {
  static_assert(DM == 0 || DM == 2, "dq4: no-dropout or recorded keep bits");
  constexpr int QW = 64, TB = 64 * 128;
  extern __shared__ __attribute__((aligned(16))) unsigned char smq4[];
  const int ntiles = (a.Lk + 63) / 64, LkP = ntiles * 64;
  unsigned char* kst = smq4;                      // [2][64 rows][128 B] K, KC image
  unsigned char* vst = smq4 + 2 * TB;             // [2][64 rows][128 B] V, KC image
  float* mfull = (float*)(smq4 + 4 * TB);         // [LkP] 0 / -inf
  uint64_t* kw_s = (uint64_t*)(mfull + LkP);      // [ntiles][QW] keep words of the workgroup's queries (DM 2)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const int qbase = bxi * QW;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Ob = (const bf16_t*)a.O + (long)b * a.Lq * a.so + h * DH;
  const bf16_t* dOb = (const bf16_t*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  const float sl2 = a.scale * 1.4426950408889634f;
  const int q = qbase + w * 16 + i;
  const bool qv = q < a.Lq;
  const int qq0 = qv ? q : 0;
  uint4 qf[2], dof[2], of[2];
  row_frags<bf16_t>(qf, Qb, a.sq, qq0, qv, lane);
  row_frags<bf16_t>(dof, dOb, a.sdo, qq0, qv, lane);
  row_frags<bf16_t>(of, Ob, a.so, qq0, qv, lane);
  for (int k = tid; k < LkP; k += 256) mfull[k] = (MASK && !key_ok(a, b, k)) ? -INFINITY : 0.f;
  if constexpr (DM == 2) {
    const uint64_t* src = a.dbits + (long)bh * ntiles * a.Lq;
    for (int e = tid; e < ntiles * QW; e += 256) {
      const int t = e / QW, qq = e - t * QW;
      kw_s[e] = (qbase + qq < a.Lq) ? src[(long)t * a.Lq + qbase + qq] : 0ull;
    }
  }
  unsigned tmask = ntiles >= 32 ? 0xFFFFFFFFu : ((1u << ntiles) - 1u);
  if (MASK && a.key_keep != nullptr) {  // fully padded key tiles skipped (wave-uniform), as in fwd6_kernel
    tmask = 0;
    for (int t = 0; t < ntiles; ++t)
      if (__any(key_ok(a, b, 64 * t + lane))) tmask |= 1u << t;
  }
  float dl = 0.f;
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    const bf16_t* x = (const bf16_t*)&dof[sb];
    const bf16_t* y = (const bf16_t*)&of[sb];
#pragma unroll
    for (int e = 0; e < 8; ++e) dl += bf2f(x[e]) * bf2f(y[e]);
  }
  dl = xsum16(dl);
  dl = xsum32(dl);
  const float delta = dl;
  if (qv && g == 0) a.delta[(long)bh * a.Lq + q] = dl;
  const float lse2 = qv ? a.lse[(long)bh * a.Lq + q] * 1.4426950408889634f : 0.f;
  pin16(qf[0]);
  pin16(qf[1]);
  pin16(dof[0]);
  pin16(dof[1]);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  auto fill = [&](int tt, int st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int R = 16 * w + 8 * u;
      const int r = 64 * tt + R + (lane >> 3), pch = lane & 7;
      const int rr = min(r, a.Lk - 1);
      const int ck = pch ^ ((r >> 1) & 7);
      dma16_asm(Kb + (long)rr * a.sk + ck * 8, kst + st * TB + R * 128);
      dma16_asm(Vb + (long)rr * a.sv + ck * 8, vst + st * TB + R * 128);
    }
  };
  unsigned rem = tmask;
  int tcur = rem ? __builtin_ctz(rem) : -1;
  if (tcur >= 0) fill(tcur, 0);
  f32x4_t dq[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) dq[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const f32x2_t sl2v = {sl2, sl2}, dscv = {a.drop_scale, a.drop_scale}, ndl = {-delta, -delta};
  auto tile = [&](const int t, const int st, auto mc) {
    constexpr bool MT = decltype(mc)::value;
    const int k0 = t * 64;
    const unsigned char* kimg = kst + st * TB;
    const unsigned char* vimg = vst + st * TB;
    uint64_t wbits = 0;
    if constexpr (DM == 2) wbits = kw_s[t * QW + w * 16 + i];
    f32x4_t sc[4], dp[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      sc[kb] = dp[kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const uint4 ak = *(const uint4*)(kimg + kc_off(128, kb * 16 + i, sub * 4 + g));
        const uint4 av = *(const uint4*)(vimg + kc_off(128, kb * 16 + i, sub * 4 + g));
        mma<bf16_t>(sc[kb], ak, qf[sub]);
        mma<bf16_t>(dp[kb], av, dof[sub]);
      }
    }
    float ds[4][4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      unsigned keep = 0xF;
      if constexpr (DM == 2) keep = (unsigned)(wbits >> (kb * 16 + 4 * g)) & 0xFu;
      float4 m4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (MT) m4 = *(const float4*)(&mfull[k0 + kb * 16 + 4 * g]);
      const float mr[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        f32x2_t off = {-lse2, -lse2};
        if constexpr (MT) off += f32x2_t{mr[2 * jj], mr[2 * jj + 1]};
        const f32x2_t arg = f32x2_t{sc[kb][2 * jj], sc[kb][2 * jj + 1]} * sl2v + off;
        const f32x2_t pr = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
        f32x2_t dpv = {dp[kb][2 * jj], dp[kb][2 * jj + 1]};
        if constexpr (DM == 2) {
          dpv.x = __int_as_float(__float_as_int(dpv.x) & __builtin_amdgcn_sbfe((int)keep, 2 * jj, 1));
          dpv.y = __int_as_float(__float_as_int(dpv.y) & __builtin_amdgcn_sbfe((int)keep, 2 * jj + 1, 1));
          dpv = dpv * dscv + ndl;
        } else {
          dpv += ndl;
        }
        const f32x2_t d2 = pr * dpv;
        ds[kb][2 * jj] = d2.x;
        ds[kb][2 * jj + 1] = d2.y;
      }
    }
    const int qq = i >> 2, pp = i & 3;
    typedef __attribute__((address_space(3))) s16x4_t* lp;
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      uint4 bq;
      bq.x = pk(ds[2 * ss][0], ds[2 * ss][1]);
      bq.y = pk(ds[2 * ss][2], ds[2 * ss][3]);
      bq.z = pk(ds[2 * ss + 1][0], ds[2 * ss + 1][1]);
      bq.w = pk(ds[2 * ss + 1][2], ds[2 * ss + 1][3]);
      const int k1 = 32 * ss + 4 * g + qq, k2 = k1 + 16;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int u = db * 4 + pp;
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(kimg + kc_tr_off(k1, u)));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(kimg + kc_tr_off(k2, u)));
        mma<bf16_t>(dq[db], join_tr(lo, hi), bq);
      }
    }
  };
  int st = 0;
  auto arrive = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    rem &= rem - 1;
    const int tnext = rem ? __builtin_ctz(rem) : -1;
    if (tnext >= 0) fill(tnext, st ^ 1);
    return tnext;
  };
  const bool mask_all = MASK && a.key_keep != nullptr;
  if (!MASK || mask_all) {
    while (tcur >= 0) {
      const int tnext = arrive();
      tile(tcur, st, std::integral_constant<bool, MASK>{});
      tcur = tnext;
      st ^= 1;
    }
  } else {  // every tile active; the mask row only on the ragged last one
    while (tcur >= 0 && tcur < ntiles - 1) {
      const int tnext = arrive();
      tile(tcur, st, std::false_type{});
      tcur = tnext;
      st ^= 1;
    }
    if (tcur >= 0) {
      arrive();
      tile(tcur, st, std::true_type{});
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup retires
  if (qv) {
    bf16_t* dQb = (bf16_t*)a.dQ + ((long)b * a.Lq + q) * a.sdq + h * DH;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint2 u2;
      u2.x = pk(dq[d][0] * a.scale, dq[d][1] * a.scale);
      u2.y = pk(dq[d][2] * a.scale, dq[d][3] * a.scale);
      *(uint2*)(dQb + d * 16 + 4 * g) = u2;
    }
  }
}

// dK / dV, v4: key-owned, 4 waves x 16 keys = one 64-key tile per workgroup; the Q / dO query tiles streamed
// through the ring; the query rows' LSE / delta and the forward's keep words of this key tile staged in LDS.
template <int DM>
__global__ void __launch_bounds__(256, 4) dkv4_kernel(AttnArgs a) {
  static_assert(DM == 0 || DM == 2, "dkv4: no-dropout or recorded keep bits");
  constexpr bool DROP = DM != 0;
  constexpr int TB = 64 * 128;
  extern __shared__ __attribute__((aligned(16))) unsigned char smk4[];
  const int nq = (a.Lq + 63) / 64, LqP = nq * 64;
  const int ntk = (a.Lk + 63) / 64;
  unsigned char* qst = smk4;                       // [2][64 rows][128 B] Q, KC image
  unsigned char* ost = smk4 + 2 * TB;              // [2][64 rows][128 B] dO, KC image
  float* lse_s = (float*)(smk4 + 4 * TB);          // [LqP] lse * log2(e) (+inf past Lq: P = 0)
  float* del_s = lse_s + LqP;                      // [LqP] delta
  uint64_t* wb_s = (uint64_t*)(del_s + LqP);       // [LqP] keep words of this key tile (DM 2)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* dOb = (const bf16_t*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  for (int j = tid; j < 2 * LqP; j += 256) {
    const int qq = j < LqP ? j : j - LqP;
    float v = j < LqP ? INFINITY : 0.f;
    if (qq < a.Lq) v = j < LqP ? a.lse[(long)bh * a.Lq + qq] * 1.4426950408889634f : a.delta[(long)bh * a.Lq + qq];
    (j < LqP ? lse_s : del_s)[qq] = v;
  }
  if constexpr (DM == 2) {
    for (int qq = tid; qq < LqP; qq += 256)
      wb_s[qq] = (qq < a.Lq && bxi < ntk) ? a.dbits[((long)bh * ntk + bxi) * a.Lq + qq] : 0ull;
  }
  const float sl2 = a.scale * 1.4426950408889634f;
  const int key = bxi * 64 + w * 16 + i;
  const bool kvld = key < a.Lk;
  const bool kok = kvld && key_ok(a, b, key);
  uint4 kf[2], vf[2];
  row_frags<bf16_t>(kf, Kb, a.sk, kvld ? key : 0, kvld, lane);
  row_frags<bf16_t>(vf, Vb, a.sv, kvld ? key : 0, kvld, lane);
  pin16(kf[0]);
  pin16(kf[1]);
  pin16(vf[0]);
  pin16(vf[1]);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  // a workgroup whose 64 keys are all padding writes zeros (epilogue), no query loop
  const bool any_key = __syncthreads_or(kok);
  auto fill = [&](int tt, int st) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int R = 16 * w + 8 * u;
      const int r = 64 * tt + R + (lane >> 3), pch = lane & 7;
      const int rr = min(r, a.Lq - 1);
      const int ck = pch ^ ((r >> 1) & 7);
      dma16_asm(Qb + (long)rr * a.sq + ck * 8, qst + st * TB + R * 128);
      dma16_asm(dOb + (long)rr * a.sdo + ck * 8, ost + st * TB + R * 128);
    }
  };
  f32x4_t dk[4], dv[4];
#pragma unroll
  for (int d = 0; d < 4; ++d) dk[d] = dv[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int kbit = w * 16 + i;  // key bit within the 64-key tile
  const f32x2_t sl2v = {sl2, sl2}, dscv = {a.drop_scale, a.drop_scale};
  const int qq_ = i >> 2, pp = i & 3;
  typedef __attribute__((address_space(3))) s16x4_t* lp;
  const int nt = any_key ? nq : 0;
  if (nt > 0) fill(0, 0);
  for (int t = 0; t < nt; ++t) {
    const int st = t & 1, q0 = t * 64;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 1 < nt) fill(t + 1, st ^ 1);
    const unsigned char* qimg = qst + st * TB;
    const unsigned char* oimg = ost + st * TB;
    f32x4_t sc[4], dp[4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      sc[qb] = dp[qb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const uint4 aq = *(const uint4*)(qimg + kc_off(128, qb * 16 + i, sub * 4 + g));
        const uint4 ao = *(const uint4*)(oimg + kc_off(128, qb * 16 + i, sub * 4 + g));
        mma<bf16_t>(sc[qb], aq, kf[sub]);
        mma<bf16_t>(dp[qb], ao, vf[sub]);
      }
    }
    float pd[4][4], ds[4][4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      const float4 l4 = *(const float4*)(&lse_s[q0 + qb * 16 + 4 * g]);
      const float4 d4 = *(const float4*)(&del_s[q0 + qb * 16 + 4 * g]);
      const f32x2_t nl[2] = {f32x2_t{-l4.x, -l4.y}, f32x2_t{-l4.z, -l4.w}};
      const f32x2_t nd[2] = {f32x2_t{-d4.x, -d4.y}, f32x2_t{-d4.z, -d4.w}};
      unsigned wq[4] = {0, 0, 0, 0};  // the 32-bit half of each query's keep word holding this key's bit
      if constexpr (DM == 2) {
        const unsigned* src = (const unsigned*)&wb_s[q0 + qb * 16 + 4 * g] + (kbit >> 5);
#pragma unroll
        for (int j = 0; j < 4; ++j) wq[j] = src[2 * j];
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const f32x2_t arg = f32x2_t{sc[qb][2 * jj], sc[qb][2 * jj + 1]} * sl2v + nl[jj];
        const f32x2_t pr = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
        f32x2_t dpv = {dp[qb][2 * jj], dp[qb][2 * jj + 1]};
        f32x2_t pdv = pr;
        if constexpr (DROP) {
          const int m0 = __builtin_amdgcn_sbfe((int)wq[2 * jj], kbit & 31, 1);
          const int m1 = __builtin_amdgcn_sbfe((int)wq[2 * jj + 1], kbit & 31, 1);
          pdv.x = __int_as_float(__float_as_int(pr.x) & m0);
          pdv.y = __int_as_float(__float_as_int(pr.y) & m1);
          dpv.x = __int_as_float(__float_as_int(dpv.x) & m0);
          dpv.y = __int_as_float(__float_as_int(dpv.y) & m1);
          dpv = dpv * dscv + nd[jj];
        } else {
          dpv += nd[jj];
        }
        const f32x2_t d2 = pr * dpv;
        pd[qb][2 * jj] = pdv.x;
        pd[qb][2 * jj + 1] = pdv.y;
        ds[qb][2 * jj] = d2.x;
        ds[qb][2 * jj + 1] = d2.y;
      }
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      uint4 bp, bs;
      bp.x = pk(pd[2 * ss][0], pd[2 * ss][1]);
      bp.y = pk(pd[2 * ss][2], pd[2 * ss][3]);
      bp.z = pk(pd[2 * ss + 1][0], pd[2 * ss + 1][1]);
      bp.w = pk(pd[2 * ss + 1][2], pd[2 * ss + 1][3]);
      bs.x = pk(ds[2 * ss][0], ds[2 * ss][1]);
      bs.y = pk(ds[2 * ss][2], ds[2 * ss][3]);
      bs.z = pk(ds[2 * ss + 1][0], ds[2 * ss + 1][1]);
      bs.w = pk(ds[2 * ss + 1][2], ds[2 * ss + 1][3]);
      const int k1 = 32 * ss + 4 * g + qq_, k2 = k1 + 16;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int u = db * 4 + pp;
        const s16x4_t olo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(oimg + kc_tr_off(k1, u)));
        const s16x4_t ohi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(oimg + kc_tr_off(k2, u)));
        const s16x4_t qlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(qimg + kc_tr_off(k1, u)));
        const s16x4_t qhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(qimg + kc_tr_off(k2, u)));
        mma<bf16_t>(dv[db], join_tr(olo, ohi), bp);
        mma<bf16_t>(dk[db], join_tr(qlo, qhi), bs);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup retires
  if (kvld) {
    bf16_t* dKb = (bf16_t*)a.dK + ((long)b * a.Lk + key) * a.sdk + h * DH;
    bf16_t* dVb = (bf16_t*)a.dV + ((long)b * a.Lk + key) * a.sdv + h * DH;
    // masked key: zero gradient (its P was never zeroed); dV carries the dropout scale of P'
    const float ksc = kok ? a.scale : 0.f, vsc = kok ? (DROP ? a.drop_scale : 1.f) : 0.f;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint2 uk, uv;
      uk.x = pk(kok ? dk[d][0] * ksc : 0.f, kok ? dk[d][1] * ksc : 0.f);
      uk.y = pk(kok ? dk[d][2] * ksc : 0.f, kok ? dk[d][3] * ksc : 0.f);
      uv.x = pk(kok ? dv[d][0] * vsc : 0.f, kok ? dv[d][1] * vsc : 0.f);
      uv.y = pk(kok ? dv[d][2] * vsc : 0.f, kok ? dv[d][3] * vsc : 0.f);
      *(uint2*)(dKb + d * 16 + 4 * g) = uk;
      *(uint2*)(dVb + d * 16 + 4 * g) = uv;
    }
  }
}

// dQ, dK, dV of one (b, h) in ONE workgroup when Lq == Lk <= 256 (the decoder's self-attention; round 3): dq3 and
// dkv3 fused. The K, V, Q and dO rows are staged into four KC images once (LDS-DMA, 128 KB at L = 256) with the LSE
// rows, the forward's keep words and the key mask; delta = rowsum(dO * O) is formed in registers and shared through
// LDS. Phase 1 is dq3's query-owned loop (S^T = K Q^T, dP^T = V dO^T, dQ^T += K^T dS^T), phase 2 dkv3's key-owned
// loop on the same images (S = Q K^T, dP = dO V^T, dV^T += dO^T P', dK^T += Q^T dS). Against the two launches it
// saves the second kernel's load of Q / dO / K / V (the stamps put ~40 % of each kernel's cycles in its load phase)
// and one launch. DM: 0 no dropout, 2 the forward's recorded keep bits.
template <int DM, bool MASK>
__global__ void __launch_bounds__(1024, 1) bwd3s_kernel(AttnArgs a) {
  static_assert(DM == 0 || DM == 2, "bwd3s: no-dropout or recorded keep bits");
  constexpr bool DROP = DM != 0;
  constexpr int NW = 16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smb[];
  const int nt = (a.Lk + 63) / 64, LP = nt * 64;     // Lq == Lk
  unsigned char* kres = smb;                        // [LP][128 B] KC images of K, V, Q, dO
  unsigned char* vres = smb + LP * 128;
  unsigned char* qres = smb + 2 * LP * 128;
  unsigned char* ores = smb + 3 * LP * 128;
  float* mfull = (float*)(smb + 4 * LP * 128);      // [LP] key mask 0 / -inf
  float* lse_s = mfull + LP;                        // [LP] lse * log2(e), +inf past Lq
  float* del_s = lse_s + LP;                        // [LP] delta
  uint64_t* wb_s = (uint64_t*)(del_s + LP);         // [nt][LP] keep words (DM == 2)
  ARTIME(14);
  ASTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4,
            i = lane & 15;
  int bxi, bh;
  xcd_tile(bxi, bh);
  const int b = bh / a.H, h = bh % a.H;
  const bf16_t* Qb = (const bf16_t*)a.Q + (long)b * a.Lq * a.sq + h * DH;
  const bf16_t* Ob = (const bf16_t*)a.O + (long)b * a.Lq * a.so + h * DH;
  const bf16_t* dOb = (const bf16_t*)a.dO + (long)b * a.Lq * a.sdo + h * DH;
  const bf16_t* Kb = (const bf16_t*)a.K + (long)b * a.Lk * a.sk + h * DH;
  const bf16_t* Vb = (const bf16_t*)a.V + (long)b * a.Lk * a.sv + h * DH;
  // ---- ordinary loads first (one vmcnt(0) behind the LDS-DMA covers all of them)
  const int q = w * 16 + i;                        // phase 1: this lane's query; phase 2: this lane's key (same index)
  const bool qv = q < a.Lq;
  const int qq0 = qv ? q : 0;
  uint4 qf[2], dof[2], of[2];
  row_frags<bf16_t>(qf, Qb, a.sq, qq0, qv, lane);
  row_frags<bf16_t>(dof, dOb, a.sdo, qq0, qv, lane);
  row_frags<bf16_t>(of, Ob, a.so, qq0, qv, lane);
  bool kk_ok = true;
  float lraw = INFINITY;
  if (tid < LP) {
    kk_ok = !MASK || key_ok(a, b, tid);
    if (tid < a.Lq) lraw = a.lse[(long)bh * a.Lq + tid];
  }
  uint64_t wv = 0;
  if constexpr (DM == 2) {
    const int kt = tid / LP, q2 = tid % LP;          // nt * LP <= 1024 words, one per thread
    if (tid < nt * LP && q2 < a.Lq) wv = a.dbits[((long)bh * nt + kt) * a.Lq + q2];
  }
  // ---- LDS-DMA of the four images, tile order (waves 0-7: K and Q rows 8w.., waves 8-15: V and dO rows 8(w-8)..)
  {
    typedef __attribute__((address_space(1))) const void* gp_t;
    typedef __attribute__((address_space(3))) void* lp_t;
    for (int t = 0; t < nt; ++t) {
      const int R = 64 * t + 8 * (w & 7);
      const int r = R + (lane >> 3), pch = lane & 7;
      const int ck = pch ^ ((r >> 1) & 7);
      const int rk = min(r, a.Lk - 1), rq = min(r, a.Lq - 1);
      if (w < 8) {
        __builtin_amdgcn_global_load_lds((gp_t)(Kb + (long)rk * a.sk + ck * 8), (lp_t)(kres + R * 128), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gp_t)(Qb + (long)rq * a.sq + ck * 8), (lp_t)(qres + R * 128), 16, 0, 0);
      } else {
        __builtin_amdgcn_global_load_lds((gp_t)(Vb + (long)rk * a.sv + ck * 8), (lp_t)(vres + R * 128), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gp_t)(dOb + (long)rq * a.sdo + ck * 8), (lp_t)(ores + R * 128), 16, 0, 0);
      }
    }
  }
  const float sl2 = a.scale * 1.4426950408889634f;
  float dl = 0.f;
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    const bf16_t* x = (const bf16_t*)&dof[sb];
    const bf16_t* y = (const bf16_t*)&of[sb];
#pragma unroll
    for (int e = 0; e < 8; ++e) dl += bf2f(x[e]) * bf2f(y[e]);
  }
  dl = xsum16(dl);
  dl = xsum32(dl);
  const float delta = dl;
  const float lse2 = qv ? a.lse[(long)bh * a.Lq + q] * 1.4426950408889634f : 0.f;
  if (tid < LP) {
    mfull[tid] = kk_ok ? 0.f : -INFINITY;
    lse_s[tid] = lraw * 1.4426950408889634f;
  }
  if (g == 0 && q < LP) del_s[q] = qv ? delta : 0.f;
  if constexpr (DM == 2)
    if (tid < nt * LP) wb_s[tid] = wv;
  ASTAMP(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  ASTAMP(2);
  const f32x2_t sl2v = {sl2, sl2}, dscv = {a.drop_scale, a.drop_scale};
  typedef __attribute__((address_space(3))) s16x4_t* lp;
  // ================================================================ phase 1: dQ (query-owned, dq3's tile body)
  {
    f32x4_t dq[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) dq[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const f32x2_t ndl = {-delta, -delta};
    auto tile = [&](const int t, auto mc) {
      constexpr bool MT = decltype(mc)::value;
      const int k0 = t * 64;
      const unsigned char* kimg = kres + k0 * 128;
      const unsigned char* vimg = vres + k0 * 128;
      uint64_t wbits = 0;
      if constexpr (DM == 2) wbits = qv ? wb_s[t * LP + q] : 0;
      f32x4_t sc[4], dp[4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        sc[kb] = dp[kb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          const uint4 ak = *(const uint4*)(kimg + kc_off(128, kb * 16 + i, sub * 4 + g));
          const uint4 av = *(const uint4*)(vimg + kc_off(128, kb * 16 + i, sub * 4 + g));
          mma<bf16_t>(sc[kb], ak, qf[sub]);
          mma<bf16_t>(dp[kb], av, dof[sub]);
        }
      }
      float ds[4][4];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        unsigned keep = 0xF;
        if constexpr (DM == 2) keep = (unsigned)(wbits >> (kb * 16 + 4 * g)) & 0xFu;
        float4 m4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (MT) m4 = *(const float4*)(&mfull[k0 + kb * 16 + 4 * g]);
        const float mr[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          f32x2_t off = {-lse2, -lse2};
          if constexpr (MT) off += f32x2_t{mr[2 * jj], mr[2 * jj + 1]};
          const f32x2_t arg = f32x2_t{sc[kb][2 * jj], sc[kb][2 * jj + 1]} * sl2v + off;
          const f32x2_t pr = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
          f32x2_t dpv = {dp[kb][2 * jj], dp[kb][2 * jj + 1]};
          if constexpr (DM == 2) {
            dpv.x = __int_as_float(__float_as_int(dpv.x) & __builtin_amdgcn_sbfe((int)keep, 2 * jj, 1));
            dpv.y = __int_as_float(__float_as_int(dpv.y) & __builtin_amdgcn_sbfe((int)keep, 2 * jj + 1, 1));
            dpv = dpv * dscv + ndl;
          } else {
            dpv += ndl;
          }
          const f32x2_t d2 = pr * dpv;
          ds[kb][2 * jj] = d2.x;
          ds[kb][2 * jj + 1] = d2.y;
        }
      }
      const int qq = i >> 2, pp = i & 3;
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        uint4 bq;
        bq.x = pk(ds[2 * ss][0], ds[2 * ss][1]);
        bq.y = pk(ds[2 * ss][2], ds[2 * ss][3]);
        bq.z = pk(ds[2 * ss + 1][0], ds[2 * ss + 1][1]);
        bq.w = pk(ds[2 * ss + 1][2], ds[2 * ss + 1][3]);
        const int k1 = 32 * ss + 4 * g + qq, k2 = k1 + 16;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const int u = db * 4 + pp;
          const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(kimg + kc_tr_off(k1, u)));
          const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(kimg + kc_tr_off(k2, u)));
          mma<bf16_t>(dq[db], join_tr(lo, hi), bq);
        }
      }
      ASTAMP(3 + (t < 4 ? t : 4));
    };
    if (MASK && a.key_keep != nullptr) {
      for (int t = 0; t < nt; ++t)  // fully padded key tiles skipped (wave-uniform), as in fwd6_kernel
        if (__any(mfull[64 * t + lane] == 0.f)) tile(t, std::integral_constant<bool, MASK>{});
    } else {
      for (int t = 0; t + 1 < nt; ++t) tile(t, std::false_type{});
      tile(nt - 1, std::integral_constant<bool, MASK>{});
    }
    if (qv) {
      bf16_t* dQb = (bf16_t*)a.dQ + ((long)b * a.Lq + q) * a.sdq + h * DH;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint2 u2;
        u2.x = pk(dq[d][0] * a.scale, dq[d][1] * a.scale);
        u2.y = pk(dq[d][2] * a.scale, dq[d][3] * a.scale);
        *(uint2*)(dQb + d * 16 + 4 * g) = u2;
      }
    }
  }
  // ================================================================ phase 2: dK, dV (key-owned, dkv3's tile body)
  {
    const int key = q;
    const bool kvld = key < a.Lk;
    const bool kok = kvld && mfull[min(key, LP - 1)] == 0.f;
    uint4 kf[2], vf[2];
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {   // the key's own rows from the K / V images
      kf[sub] = *(const uint4*)(kres + kc_off(128, min(key, LP - 1), sub * 4 + g));
      vf[sub] = *(const uint4*)(vres + kc_off(128, min(key, LP - 1), sub * 4 + g));
    }
    f32x4_t dk[4], dv[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) dk[d] = dv[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int kbit = (w & 3) * 16 + i;     // key bit within its 64-key tile w >> 2
    const int kts = w >> 2;
    const int qq_ = i >> 2, pp = i & 3;
    if (__any(kok)) {
      for (int t = 0; t < nt; ++t) {
        const int q0 = t * 64;
        const unsigned char* qimg = qres + q0 * 128;
        const unsigned char* oimg = ores + q0 * 128;
        f32x4_t sc[4], dp[4];
#pragma unroll
        for (int qb = 0; qb < 4; ++qb) {
          sc[qb] = dp[qb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int sub = 0; sub < 2; ++sub) {
            const uint4 aq = *(const uint4*)(qimg + kc_off(128, qb * 16 + i, sub * 4 + g));
            const uint4 ao = *(const uint4*)(oimg + kc_off(128, qb * 16 + i, sub * 4 + g));
            mma<bf16_t>(sc[qb], aq, kf[sub]);
            mma<bf16_t>(dp[qb], ao, vf[sub]);
          }
        }
        float pd[4][4], ds[4][4];
#pragma unroll
        for (int qb = 0; qb < 4; ++qb) {
          const float4 l4 = *(const float4*)(&lse_s[q0 + qb * 16 + 4 * g]);
          const float4 d4 = *(const float4*)(&del_s[q0 + qb * 16 + 4 * g]);
          const f32x2_t nl[2] = {f32x2_t{-l4.x, -l4.y}, f32x2_t{-l4.z, -l4.w}};
          const f32x2_t nd[2] = {f32x2_t{-d4.x, -d4.y}, f32x2_t{-d4.z, -d4.w}};
          unsigned wq[4] = {0, 0, 0, 0};
          if constexpr (DM == 2) {
            const unsigned* src = (const unsigned*)&wb_s[kts * LP + q0 + qb * 16 + 4 * g] + (kbit >> 5);
#pragma unroll
            for (int j = 0; j < 4; ++j) wq[j] = src[2 * j];
          }
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const f32x2_t arg = f32x2_t{sc[qb][2 * jj], sc[qb][2 * jj + 1]} * sl2v + nl[jj];
            const f32x2_t pr = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
            f32x2_t dpv = {dp[qb][2 * jj], dp[qb][2 * jj + 1]};
            f32x2_t pdv = pr;
            if constexpr (DROP) {
              const int m0 = __builtin_amdgcn_sbfe((int)wq[2 * jj], kbit & 31, 1);
              const int m1 = __builtin_amdgcn_sbfe((int)wq[2 * jj + 1], kbit & 31, 1);
              pdv.x = __int_as_float(__float_as_int(pr.x) & m0);
              pdv.y = __int_as_float(__float_as_int(pr.y) & m1);
              dpv.x = __int_as_float(__float_as_int(dpv.x) & m0);
              dpv.y = __int_as_float(__float_as_int(dpv.y) & m1);
              dpv = dpv * dscv + nd[jj];
            } else {
              dpv += nd[jj];
            }
            const f32x2_t d2 = pr * dpv;
            pd[qb][2 * jj] = pdv.x;
            pd[qb][2 * jj + 1] = pdv.y;
            ds[qb][2 * jj] = d2.x;
            ds[qb][2 * jj + 1] = d2.y;
          }
        }
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          uint4 bp, bs;
          bp.x = pk(pd[2 * ss][0], pd[2 * ss][1]);
          bp.y = pk(pd[2 * ss][2], pd[2 * ss][3]);
          bp.z = pk(pd[2 * ss + 1][0], pd[2 * ss + 1][1]);
          bp.w = pk(pd[2 * ss + 1][2], pd[2 * ss + 1][3]);
          bs.x = pk(ds[2 * ss][0], ds[2 * ss][1]);
          bs.y = pk(ds[2 * ss][2], ds[2 * ss][3]);
          bs.z = pk(ds[2 * ss + 1][0], ds[2 * ss + 1][1]);
          bs.w = pk(ds[2 * ss + 1][2], ds[2 * ss + 1][3]);
          const int k1 = 32 * ss + 4 * g + qq_, k2 = k1 + 16;
#pragma unroll
          for (int db = 0; db < 4; ++db) {
            const int u = db * 4 + pp;
            const s16x4_t olo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(oimg + kc_tr_off(k1, u)));
            const s16x4_t ohi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(oimg + kc_tr_off(k2, u)));
            const s16x4_t qlo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(qimg + kc_tr_off(k1, u)));
            const s16x4_t qhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(qimg + kc_tr_off(k2, u)));
            mma<bf16_t>(dv[db], join_tr(olo, ohi), bp);
            mma<bf16_t>(dk[db], join_tr(qlo, qhi), bs);
          }
        }
        ASTAMP(7 + (t < 4 ? t : 4));
      }
    }
    if (kvld) {
      bf16_t* dKb = (bf16_t*)a.dK + ((long)b * a.Lk + key) * a.sdk + h * DH;
      bf16_t* dVb = (bf16_t*)a.dV + ((long)b * a.Lk + key) * a.sdv + h * DH;
      const float ksc = kok ? a.scale : 0.f, vsc = kok ? (DROP ? a.drop_scale : 1.f) : 0.f;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint2 uk, uv;
        uk.x = pk(kok ? dk[d][0] * ksc : 0.f, kok ? dk[d][1] * ksc : 0.f);
        uk.y = pk(kok ? dk[d][2] * ksc : 0.f, kok ? dk[d][3] * ksc : 0.f);
        uv.x = pk(kok ? dv[d][0] * vsc : 0.f, kok ? dv[d][1] * vsc : 0.f);
        uv.y = pk(kok ? dv[d][2] * vsc : 0.f, kok ? dv[d][3] * vsc : 0.f);
        *(uint2*)(dKb + d * 16 + 4 * g) = uk;
        *(uint2*)(dVb + d * 16 + 4 * g) = uv;
      }
    }
  }
  ASTAMP(12);
#ifdef ATTN_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  ASTAMP(13);
  ARTIME(15);
}

// Kernel choice per launch shape (bf16; the fp32 parity mode runs the generic kernels):
//  forward  WavLM gated rel-pos bias, Lk <= 1024: fwd7 with the bias (attn7.hip REL, round 6); longer, or under
//           fddm_attn_set_kernels(1 / 5): fwd5 (streamed ring, bias slice staged; gate from a precomputed row, from the
//           projection's extra columns, or from the attention input); decoder, Lk <= 1024: fwd8 (attn8.hip, two
//           32-query chains per wave on 32x32x16 MFMAs; keep bits from the producer); Lk > 1024: fwd2.
//  backward decoder, recorded bits or no dropout: Lq <= 256 and Lk <= 512: bwdf7 (attn7.hip, one fused launch per
//           (b, h), one pass per 256 keys); other Lk <= 1024: dq7 + dkv7; longer or rehashed:
//           dq2 + dkv2. Under fddm_attn_set_kernels(1) the round-4 kernels: bwd3s (Lq == Lk <= 256), dq4 + dkv4.
// fddm_attn_set_kernels (tests / tools only): 1 selects the round-4 16x16x32 kernels (fwd6 / dq4 / dkv4 / bwd3s)
// where the 32x32x16 family (attn7.hip) would run; 0 (default) the 32x32x16 family with the two-chain forward fwd8
// (attn8.hip); 2 the same without the fused backward (dq7 + dkv7 at every Lk); 3 the default with fwd7 as the forward;
// 4 fwd8 at every decoder shape; 5 the default with WavLM's biased attention on fwd5 instead of fwd7 (REL)
static int g_attn_v6 = 0;
#ifndef A7_FUSED_MAXLQ
#define A7_FUSED_MAXLQ 256  // fused backward up to this many queries, one or two key passes (more: one workgroup per
                            // (b, h) walks every 64-query tile, measured slower than dq7 + dkv7 at Lq 512)
#endif
static bool attn7_enabled() { return g_attn_v6 != 1; }
// compute units of the current device (cached; one process drives one GPU)
static long attn_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

template <typename T>
static int run(int which, AttnArgs& a, hipStream_t s) {
  constexpr int RB = Cfg<T>::RB;
  const bool drop = a.thr16 != 0, mask = a.key_keep != nullptr || (a.Lk % 64) != 0;
  if constexpr (sizeof(T) == 2) {
    if (which == 0) {
      const bool rel = a.table != nullptr && (a.gate != nullptr || a.graw != nullptr || a.gx != nullptr);
      const int LkP = (a.Lk + 63) / 64 * 64;
      if (rel) {
        if (drop) return (int)hipErrorInvalidValue;    // WavLM attention has no dropout in the frozen encoder
        // round 6: fwd7 with the bias (attn7.hip REL) where the keys fit its key-mask staging; fwd5 under the round-4
        // kernel selection (fddm_attn_set_kernels(1)) and for longer key ranges
        if (attn7_enabled() && a.Lk <= 1024 && g_attn_v6 != 5) return attn7_fwd(a, s);
        const size_t lds5 = (size_t)2 * 2 * 64 * 128 + (size_t)LkP * 4 + (size_t)(LkP + 128) * 4;
        dim3 grid5((a.Lq + 127) / 128, a.B * a.H);
        if (mask) hipLaunchKernelGGL((fwd5_kernel<true, 2, 2>), grid5, dim3(256), lds5, s, a);
        else hipLaunchKernelGGL((fwd5_kernel<false, 2, 2>), grid5, dim3(256), lds5, s, a);
        return (int)hipGetLastError();
      }
      if (a.Lk <= 1024) {
        const int ntiles = LkP / 64, qw = 128;
        const int dm = !drop ? 0 : (a.bits_ready && a.dbits) ? 1 : 2;
        if (attn7_enabled() && (dm != 2 || a.dbits)) {
          if (dm == 2) {  // the caller's buffer gets this site's keep masks (layout v3) first; fwd7 reads them
            const int e = attn7_drop_bits(a.dbits, 0, 1, a.B * a.H, a.Lq, a.Lk, a.seed, a.stream, 0, a.thr16,
                                          a.seed_off, s);
            if (e) return e;
          }
          // fwd8 (256 queries per workgroup, two chains per wave) unless its grid loads the busiest CU with more
          // queries than fwd7's (128 per workgroup) does: C2 (256 workgroups, one per CU) takes fwd8; C4 (B16 H12
          // Lq 512: 384 fwd8 workgroups -> 512 queries on half the CUs, vs 768 fwd7 workgroups -> 384 on every CU)
          // takes fwd7 (measured 24.5 vs 25.1-25.7 us)
          const long nh = (long)a.B * a.H, ncu = attn_cu_count();
          const long load8 = (nh * ((a.Lq + 255) / 256) + ncu - 1) / ncu * 256;
          const long load7 = (nh * ((a.Lq + 127) / 128) + ncu - 1) / ncu * 128;
          return (g_attn_v6 == 3 || (g_attn_v6 != 4 && load8 > load7)) ? attn7_fwd(a, s) : attn8_fwd(a, s);
        }
        const size_t lds = (size_t)2 * 2 * 64 * 128 + (size_t)LkP * 4 +
                           (dm == 1 ? (size_t)ntiles * qw * 8 : dm == 2 ? (size_t)3 * ATTN_R * 2 : 0);
        dim3 g6((a.Lq + qw - 1) / qw, a.B * a.H);
        const int mk = a.key_keep != nullptr ? 2 : (a.Lk % 64) != 0 ? 1 : 0;
#define FWD6(D, M) hipLaunchKernelGGL((fwd6_kernel<D, M, 2>), g6, dim3(256), lds, s, a)
#define FWD6M(D) do { if (mk == 2) FWD6(D, 2); else if (mk == 1) FWD6(D, 1); else FWD6(D, 0); } while (0)
        if (dm == 2) FWD6M(2);
        else if (dm == 1) FWD6M(1);
        else FWD6M(0);
#undef FWD6M
#undef FWD6
        return (int)hipGetLastError();
      }
      dim3 grid((a.Lq + 127) / 128, a.B * a.H);
#define FWD2(D, M) hipLaunchKernelGGL((fwd2_kernel<D, M, false>), grid, dim3(256), 0, s, a)
      if (drop) { if (mask) FWD2(true, true); else FWD2(true, false); }
      else { if (mask) FWD2(false, true); else FWD2(false, false); }
#undef FWD2
      return (int)hipGetLastError();
    }
    const int dm = drop ? (a.dbits ? 2 : 1) : 0;
    if (which == 1) {
      if (dm != 1 && a.Lk <= 1024) {
        const int ntiles = (a.Lk + 63) / 64;
        const size_t lds = (size_t)4 * 64 * 128 + (size_t)ntiles * 64 * 4 + (dm == 2 ? (size_t)ntiles * 64 * 8 : 0);
        dim3 g4((a.Lq + 63) / 64, a.B * a.H);
#define DQ4(D, M) hipLaunchKernelGGL((dq4_kernel<D, M>), g4, dim3(256), lds, s, a)
        if (dm == 2) { if (mask) DQ4(2, true); else DQ4(2, false); }
        else { if (mask) DQ4(0, true); else DQ4(0, false); }
#undef DQ4
        return (int)hipGetLastError();
      }
      dim3 grid((a.Lq + 127) / 128, a.B * a.H);
#define DQ2(D, M) hipLaunchKernelGGL((dq2_kernel<D, M>), grid, dim3(256), 0, s, a)
      if (dm == 2) { if (mask) DQ2(2, true); else DQ2(2, false); }
      else if (dm == 1) { if (mask) DQ2(1, true); else DQ2(1, false); }
      else { if (mask) DQ2(0, true); else DQ2(0, false); }
#undef DQ2
      return (int)hipGetLastError();
    }
    if (which == 2) {
      if (dm != 1 && a.Lq <= 1024) {
        const int LqP = (a.Lq + 63) / 64 * 64;
        const size_t lds = (size_t)4 * 64 * 128 + (size_t)LqP * 8 + (dm == 2 ? (size_t)LqP * 8 : 0);
        dim3 g4((a.Lk + 63) / 64, a.B * a.H);
        if (dm == 2) hipLaunchKernelGGL((dkv4_kernel<2>), g4, dim3(256), lds, s, a);
        else hipLaunchKernelGGL((dkv4_kernel<0>), g4, dim3(256), lds, s, a);
        return (int)hipGetLastError();
      }
      dim3 grid((a.Lk + 127) / 128, a.B * a.H);
      if (dm == 2) hipLaunchKernelGGL((dkv2_kernel<2>), grid, dim3(256), 0, s, a);
      else if (dm == 1) hipLaunchKernelGGL((dkv2_kernel<1>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((dkv2_kernel<0>), grid, dim3(256), 0, s, a);
      return (int)hipGetLastError();
    }
    if (which == 4) {  // the 32x32x16 family: the fused launch for Lq <= 256 and Lk <= 512 (one or two key passes),
                       // else dq7 (also writes dkv7's row terms), then dkv7
      if ((g_attn_v6 == 0 || g_attn_v6 >= 3) && a.Lk <= 512 && a.Lq <= A7_FUSED_MAXLQ) return attn7_bwdf(a, s);
      const int e = attn7_dq(a, s);
      return e ? e : attn7_dkv(a, s);
    }
    if (which == 3) {
      const int LP = (a.Lk + 63) / 64 * 64;
      const size_t lds = (size_t)LP * 512 + (size_t)LP * 12 + (drop ? (size_t)(LP / 64) * LP * 8 : 0);
      dim3 g3(1, a.B * a.H);
#define BW3(D, M) hipLaunchKernelGGL((bwd3s_kernel<D, M>), g3, dim3(1024), lds, s, a)
      if (drop) { if (mask) BW3(2, true); else BW3(2, false); }
      else { if (mask) BW3(0, true); else BW3(0, false); }
#undef BW3
      return (int)hipGetLastError();
    }
    return (int)hipErrorInvalidValue;
  } else {
    if (which == 0) {
      dim3 grid((a.Lq + 63) / 64, a.B * a.H);
      hipLaunchKernelGGL(fwd_kernel<T>, grid, dim3(256), 128 * RB, s, a);
    } else if (which == 1) {
      dim3 grid((a.Lq + 63) / 64, a.B * a.H);
      hipLaunchKernelGGL(dq_kernel<T>, grid, dim3(256), 192 * RB, s, a);
    } else if (which == 2) {
      dim3 grid((a.Lk + 63) / 64, a.B * a.H);
      hipLaunchKernelGGL(dkv_kernel<T>, grid, dim3(256), 256 * RB + 512, s, a);
    } else {
      return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
}

static bool aligned_ok(const void* p, long stride, int ech) {
  return p == nullptr || (((uintptr_t)p & 15) == 0 && stride % ech == 0);
}

}  // namespace attn
}  // namespace fddm

using namespace fddm;
using namespace fddm::attn;

static int attn_dispatch(int which, int dtype, AttnArgs& a, float drop_p, void* hs) {
  if (a.B <= 0 || a.H <= 0 || a.Lq <= 0 || a.Lk <= 0) return 0;
  const int ech = dtype == FDDM_BF16 ? 8 : 4;
  if (!aligned_ok(a.Q, a.sq, ech) || !aligned_ok(a.K, a.sk, ech) || !aligned_ok(a.V, a.sv, ech) ||
      !aligned_ok(a.O, a.so, ech) || !aligned_ok(a.dO, a.sdo, ech))
    return (int)hipErrorInvalidValue;
  a.thr16 = 0;
  a.drop_scale = 1.f;
  if (drop_p > 0.f) {
    a.thr16 = (unsigned)llrintf(drop_p * 65536.f);
    a.drop_scale = 1.f / (1.f - drop_p);
  }
  if (dtype == FDDM_BF16) return run<bf16_t>(which, a, (hipStream_t)hs);
  if (dtype == FDDM_F32) return run<float>(which, a, (hipStream_t)hs);
  return (int)hipErrorInvalidValue;
}

#ifdef ATTN_STAMPS
FDDM_API int fddm_attn_stamps(unsigned long long* host, long n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fddm::attn::attn_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}
FDDM_API int fddm_attn_stamps_clear() {
  static unsigned long long z[8192 * 16];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(fddm::attn::attn_stamps), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
#endif

FDDM_API int fddm_attn_set_kernels(int v6) {
  const int old = g_attn_v6;
  g_attn_v6 = (v6 >= 1 && v6 <= 5) ? v6 : 0;
  return old;
}

// Forward. Q/K/V/O: element (b, pos, h, d) at base + (b*L + pos)*stride + h*64 + d.
FDDM_API int fddm_attn_fwd(int dtype, const void* Q, long sq, const void* K, long sk, const void* V, long sv, void* O,
                           long so, float* lse, const unsigned char* key_keep, const float* gate, const float* table,
                           int B, int H, int Lq, int Lk, float scale, float drop_p, unsigned long long seed,
                           unsigned long long stream, unsigned long long* drop_bits, int drop_bits_ready, void* hs) {
  AttnArgs a{};
  a.dbits = (uint64_t*)drop_bits;
  a.bits_ready = drop_bits_ready;
  a.Q = Q; a.K = K; a.V = V; a.Out = O; a.lse = lse;
  a.sq = sq; a.sk = sk; a.sv = sv; a.so = so;
  a.key_keep = key_keep; a.gate = gate; a.table = table;
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk; a.scale = scale; a.seed = seed; a.stream = stream; a.seed_off = g_seed_off;
  return attn_dispatch(0, dtype, a, drop_p, hs);
}

// u64 words per site of the keep-bit buffer: room for either storage layout (the round-4 words [B*H][ntiles][Lq] or
// layout v3's lane masks, attn7.hip); fddm_attn_drop_bits writes the one the selected kernel family reads
FDDM_API long fddm_attn_drop_words(int B, int H, int Lq, int Lk) {
  const long v2 = (long)B * H * Lq * ((Lk + 63) / 64), v3 = attn7_drop_words(B, H, Lq, Lk);
  return v2 > v3 ? v2 : v3;
}

// floats of fddm_attn_bwd's delta_ws for this shape (the largest need: the two-pass fused launch's f32 dQ partials,
// 64 per query row; the 32x32x16 pair's [2][B*H][LqP] row terms plus the pre-scaled Q' [B*H][LqP][64] bf16 take 34,
// the round-4 kernels' [B*H][Lq] 1)
FDDM_API long fddm_attn_bwd_ws_floats(int B, int H, int Lq, int Lk) {
  (void)Lk;
  return 64L * B * H * ((Lq + 63) / 64 * 64);
}

// Dropout keep bits of nsites attention sites with the same shape, rng streams stream0 + s * stream_step (site s at
// out + s * site_words): the words fddm_attn_fwd(..., drop_bits_ready = 1) and fddm_attn_bwd read.
FDDM_API int fddm_attn_drop_bits(unsigned long long* out, long site_words, int nsites, int B, int H, int Lq, int Lk,
                                 float drop_p, unsigned long long seed, unsigned long long stream0,
                                 unsigned long long stream_step, void* hs) {
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0 || nsites <= 0) return 0;
  if (!out || drop_p <= 0.f || site_words < fddm_attn_drop_words(B, H, Lq, Lk)) return (int)hipErrorInvalidValue;
  // storage layout v3 (lane masks) where the 32x32x16 kernels read the bits (bf16, Lk <= 1024); the round-4 words
  // for the kernels that take longer key ranges (fwd2 draws its own, dq2 / dkv2 read these)
  if (attn7_enabled() && Lk <= 1024)
    return attn7_drop_bits((uint64_t*)out, site_words, nsites, B * H, Lq, Lk, seed, stream0, stream_step,
                           (unsigned)llrintf(drop_p * 65536.f), g_seed_off, (hipStream_t)hs);
  DbArgs d{(uint64_t*)out, site_words, B * H, Lq, Lk, seed, stream0, stream_step, (unsigned)llrintf(drop_p * 65536.f),
           g_seed_off};
  hipLaunchKernelGGL(dbits_kernel, dim3(B * H, nsites), dim3(256), 0, (hipStream_t)hs, d);
  return (int)hipGetLastError();
}

// WavLM forward with the gate computed in the kernel from 8 bf16 pre-activations per (token, head) that the Q|K|V
// projection appended as extra columns (graw, row stride sgr; gconst [H]): no separate gate pass over the input.
FDDM_API int fddm_attn_fwd_relgate(const void* Q, long sq, const void* K, long sk, const void* V, long sv, void* O,
                                   long so, const void* graw, long sgr, const float* gconst, const float* table, int B,
                                   int H, int Lq, int Lk, float scale, void* hs) {
  if (!graw || !gconst || !table || (((uintptr_t)graw) & 15) || sgr % 8) return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.Q = Q; a.K = K; a.V = V; a.Out = O;
  a.sq = sq; a.sk = sk; a.sv = sv; a.so = so;
  a.graw = graw; a.sgr = sgr; a.gconst = gconst; a.table = table;
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk; a.scale = scale;
  return attn_dispatch(0, FDDM_BF16, a, 0.f, hs);
}

// WavLM forward with the gate computed in the kernel from the attention input x itself (bf16 rows, stride sx; the
// head's 64 inputs against gw = [sum of gru_rel_pos_linear rows 0-3 | rows 4-7 | their bias sums], 130 floats): the
// Q|K|V projection needs no extra gate columns and no separate gate pass runs.
FDDM_API int fddm_attn_fwd_relgate_x(const void* Q, long sq, const void* K, long sk, const void* V, long sv, void* O,
                                     long so, const void* x, long sx, const float* gw, const float* gconst,
                                     const float* table, int B, int H, int Lq, int Lk, float scale, void* hs) {
  if (!x || !gw || !gconst || !table || (((uintptr_t)x) & 15) || (((uintptr_t)gw) & 15) || sx % 8)
    return (int)hipErrorInvalidValue;
  AttnArgs a{};
  a.Q = Q; a.K = K; a.V = V; a.Out = O;
  a.sq = sq; a.sk = sk; a.sv = sv; a.so = so;
  a.gx = x; a.sgx = sx; a.gw = gw; a.gconst = gconst; a.table = table;
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk; a.scale = scale;
  return attn_dispatch(0, FDDM_BF16, a, 0.f, hs);
}

// Backward: dQ (query-owned kernel) and dK/dV (key-owned kernel). lse from the forward.
FDDM_API int fddm_attn_bwd(int dtype, const void* Q, long sq, const void* K, long sk, const void* V, long sv,
                           const void* O, long so, const void* dO, long sdo, const float* lse, void* dQ, long sdq,
                           void* dK, long sdk, void* dV, long sdv, float* delta_ws, const unsigned char* key_keep,
                           int B, int H, int Lq, int Lk, float scale, float drop_p, unsigned long long seed,
                           unsigned long long stream, const unsigned long long* drop_bits, void* hs) {
  AttnArgs a{};
  a.dbits = (uint64_t*)drop_bits;
  a.delta = delta_ws;
  a.Q = Q; a.K = K; a.V = V; a.O = O; a.dO = dO; a.lse = (float*)lse;
  a.dQ = dQ; a.dK = dK; a.dV = dV;
  a.sq = sq; a.sk = sk; a.sv = sv; a.so = so; a.sdo = sdo; a.sdq = sdq; a.sdk = sdk; a.sdv = sdv;
  a.key_keep = key_keep;
  a.B = B; a.H = H; a.Lq = Lq; a.Lk = Lk; a.scale = scale; a.seed = seed; a.stream = stream; a.seed_off = g_seed_off;
  // bf16 with recorded or no dropout, Lk <= 1024: the 32x32x16 kernels (attn7.hip; delta_ws holds
  // fddm_attn_bwd_ws_floats = 64 * B*H*LqP floats)
  if (dtype == FDDM_BF16 && attn7_enabled() && Lk <= 1024 && (drop_p <= 0.f || drop_bits))
    return attn_dispatch(4, dtype, a, drop_p, hs);
  // self-attention shapes (Lq == Lk <= 256, bf16, no rehashed dropout): dQ, dK and dV in one fused launch
  if (dtype == FDDM_BF16 && Lq == Lk && Lk <= 256 && (drop_p <= 0.f || drop_bits))
    return attn_dispatch(3, dtype, a, drop_p, hs);
  int e = attn_dispatch(1, dtype, a, drop_p, hs);
  if (e) return e;
  return attn_dispatch(2, dtype, a, drop_p, hs);
}
