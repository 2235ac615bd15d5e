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
  const uint64_t* seed_off;  // graph-replay seed offset (common.h eff_seed) or null
  // optional RoPE of the output (the next decoder block's q = k input, misc.hip rope_fwd_kernel's formula):
  // rope_out[r][4q + j] = o[8q + 2j] cs[p][8q + 2j] - o[8q + 2j + 1] sn[p][8q + 2j + 1],
  // rope_out[r][d/2 + 4q + j] = o[8q + 2j] sn[p][8q + 2j] + o[8q + 2j + 1] cs[p][8q + 2j + 1], p = r % rope_L
  const float *rcos, *rsin; void* rope_out; long rope_L;
};

// 8 consecutive elements per lane per chunk (16-B bf16 / 32-B f32 accesses); d % 8 == 0
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
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
__device__ __forceinline__ void st8(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    uint4 u;
    u.x = pk_bf16(v[0], v[1]);
    u.y = pk_bf16(v[2], v[3]);
    u.z = pk_bf16(v[4], v[5]);
    u.w = pk_bf16(v[6], v[7]);
    *(uint4*)p = u;
  } else {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <typename OT>
__device__ __forceinline__ void st4v(OT* p, float a, float b, float c, float d_) {
  if constexpr (sizeof(OT) == 2) {
    *(uint2*)p = make_uint2(pk_bf16(a, b), pk_bf16(c, d_));
  } else {
    *(float4*)p = make_float4(a, b, c, d_);
  }
}

constexpr int LN_MAXCH = 2;  // chunks of 8 per lane: d <= 1024

// wave-wide sum in the VALU: DPP within rows of 16 lanes (quad swaps, half-row and row mirrors), then the
// gfx950 lane-swap instructions across rows — no LDS round trip (__shfl_xor is a ds_bpermute per step);
// every lane receives the total
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_v(float v) {
  v += dppf<0xB1>(v);   // quad_perm(1,0,3,2)
  v += dppf<0x4E>(v);   // quad_perm(2,3,0,1)
  v += dppf<0x141>(v);  // row_half_mirror
  v += dppf<0x140>(v);  // row_mirror
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// One wave per row. Every load of the row (x, y, gamma, beta, FiLM scale / shift) is issued before the first use,
// so a wave waits for one memory round trip, not three; the two row reductions run in the VALU (wave_sum_v).
// HY: residual branch y present, HF: FiLM present (compile-time: a load under a runtime branch gets its own wait)
// CH chunks of 8 per lane: 1 for d <= 512 (the decoder), 2 for d <= 1024 (WavLM 768)
template <typename XT, typename YT, typename OT, bool HY, bool HF, int CH, bool RP = false>
__global__ void __launch_bounds__(256) ln_fwd_kernel(LnFwdArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  if (row >= a.N) return;
  const long d = a.d, nch = d / 8;
  const XT* x = (const XT*)a.x + row * d;
  const YT* y = HY ? (const YT*)a.y + row * d : nullptr;
  const long b = HF ? row / a.rows_per_batch : 0;
  float v[CH][8], yv[CH][8], gm[CH][8], bt[CH][8], fs[CH][8], fh[CH][8], rc[CH][8], rs[CH][8];
  const long rp = RP ? row % a.rope_L : 0;
  // lanes past the row end load its last chunk again (no divergent branch around the loads: a load inside one
  // would be waited for at the branch join) and contribute zeros
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const long c0 = min(lane + 64L * i, nch - 1) * 8;
    ld8<XT>(x + c0, v[i]);
    if constexpr (HY) ld8<YT>(y + c0, yv[i]);
    ld8<float>(a.gamma + c0, gm[i]);
    ld8<float>(a.beta + c0, bt[i]);
    if constexpr (HF) {
      ld8<float>(a.fsc + b * d + c0, fs[i]);
      ld8<float>(a.fsh + b * d + c0, fh[i]);
    }
    if constexpr (RP) {
      ld8<float>(a.rcos + rp * d + c0, rc[i]);
      ld8<float>(a.rsin + rp * d + c0, rs[i]);
    }
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const long ch = lane + 64L * i;
    if (ch >= nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    } else {
      if constexpr (HY) {
        unsigned keep = 0xffu;  // d % 8 == 0: two hashes per 8 elements
        if (a.thr16) {
          const uint64_t e4 = (uint64_t)(row * d + ch * 8) >> 2;
          keep = drop_keep4(eff_seed(a.seed, a.seed_off), a.stream, e4, a.thr16) | (drop_keep4(eff_seed(a.seed, a.seed_off), a.stream, e4 + 1, a.thr16) << 4);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = yv[i][e];
          v[i][e] += a.thr16 ? ((keep >> e) & 1u ? t * a.drop_scale : 0.f) : t;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += v[i][e];
    }
  }
  const float mean = wave_sum_v(sum) / (float)d;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const long ch = lane + 64L * i;
    if (ch < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = v[i][e] - mean;
        sq += t * t;
      }
    }
  }
  const float var = wave_sum_v(sq) / (float)d;
  const float rstd = 1.f / sqrtf(var + a.eps);
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const long ch = lane + 64L * i;
    if (ch < nch) {
      const long c0 = ch * 8;
      if (a.save_s) st8<float>(a.save_s + row * d + c0, v[i]);
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * gm[i][e] + bt[i][e];
      if constexpr (HF) {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = o[e] * (1.f + fs[i][e]) + fh[i][e];
      }
      if (a.out_f32) st8<float>(a.out_f32 + row * d + c0, o);
      if (a.out_t) st8<OT>((OT*)a.out_t + row * d + c0, o);
      if constexpr (RP) {
        float lo[4], hi[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          lo[j] = o[2 * j] * rc[i][2 * j] - o[2 * j + 1] * rs[i][2 * j + 1];
          hi[j] = o[2 * j] * rs[i][2 * j] + o[2 * j + 1] * rc[i][2 * j + 1];
        }
        OT* ro = (OT*)a.rope_out + row * d;
        st4v<OT>(ro + 4 * ch, lo[0], lo[1], lo[2], lo[3]);
        st4v<OT>(ro + d / 2 + 4 * ch, hi[0], hi[1], hi[2], hi[3]);
      }
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
  float* part;  // fused pass: per-slab dgamma / dbeta / dFiLM sums [slab][4][d] (ln_fold_kernel) instead of atomics
  long N, d, rows_per_batch;
  uint64_t seed, stream; unsigned thr16; float drop_scale;
  const uint64_t* seed_off;  // graph-replay seed offset (common.h eff_seed) or null
};

// pass 1: one wave per row: ds (residual gradient) and the dropout-masked dy for the GEMM
template <typename OT>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnBwdArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.N) return;
  const long d = a.d;
  const long b = row / a.rows_per_batch;
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
      if (a.fsc) go *= 1.f + a.fsc[b * d + c];
      const float gx = go * a.gamma[c];
      xh[i] = x;
      dxh[i] = gx;
      s1 += gx;
      s2 += gx * x;
    }
  }
  s1 = wave_sum_v(s1) / (float)d;
  s2 = wave_sum_v(s2) / (float)d;
#pragma unroll
  for (int i = 0; i < LN_MAXPL; ++i) {
    const long c = lane + 64L * i;
    if (c < d) {
      const float ds = rstd * (dxh[i] - s1 - xh[i] * s2);
      if (a.dres) a.dres[row * d + c] = ds;
      if (a.dy_t) {
        float dy = ds;
        if (a.thr16) dy = drop_keep(eff_seed(a.seed, a.seed_off), a.stream, (uint64_t)(row * d + c), a.thr16) ? dy * a.drop_scale : 0.f;
        st<OT>((OT*)a.dy_t + row * d + c, dy);
      }
    }
  }
}

// Fused single pass: a workgroup takes a slab of LNB_ROWS rows (one FiLM batch), each wave its rows with 8
// consecutive columns per lane and chunk (32-B f32 / 16-B bf16 accesses), while every lane keeps per-column
// partial sums of the parameter gradients in registers; the 8 waves (4 rows each) combine them through LDS and
// the slab adds them with one atomic per column and quantity. CH = 8-column chunks per lane (d <= 512*CH).
// The device-scope atomics bound the kernel (every slab adds into the same d columns of dgamma/dbeta): at d 512,
// N 8192, 16-row slabs of 4 waves took 24.0 us, 8 waves 23.4, 32-row slabs 18.5, 64-row slabs 21.8 (occupancy).
#ifndef LN_BWD_ROWS
#define LN_BWD_ROWS 32
#endif
constexpr int LNB_ROWS = LN_BWD_ROWS;
constexpr int LN_FOLD_MAX = 4;  // jobs per fddm_ln_fold launch
// keep bits of the 8 dropout decisions of elements e0..e0+7 (e0 % 8 == 0): two hash words
__device__ __forceinline__ unsigned keep8(uint64_t seed, uint64_t stream, uint64_t e0, unsigned thr) {
  unsigned k = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint64_t w = mix64(seed, stream, (e0 >> 2) + h);
#pragma unroll
    for (int j = 0; j < 4; ++j) k |= ((((unsigned)(w >> (16 * j))) & 0xFFFFu) >= thr ? 1u : 0u) << (4 * h + j);
  }
  return k;
}
template <int CH, typename OT>
__global__ void __launch_bounds__(512) ln_bwd_fused_kernel(LnBwdArgs a) {
  __shared__ float red[4][4][512 * CH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long d = a.d, nch = d / 8;
  const long r0 = (long)blockIdx.x * LNB_ROWS;
  const long b = r0 / a.rows_per_batch;
  float pg[CH][8], pb[CH][8], psc[CH][8], psh[CH][8], gm[CH][8], bt[CH][8], fs[CH][8];
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const long ch = lane + 64L * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) pg[i][e] = pb[i][e] = psc[i][e] = psh[i][e] = gm[i][e] = bt[i][e] = fs[i][e] = 0.f;
    if (ch < nch) {
      ld8<float>(a.gamma + ch * 8, gm[i]);
      if (a.beta) ld8<float>(a.beta + ch * 8, bt[i]);
      if (a.fsc) ld8<float>(a.fsc + b * d + ch * 8, fs[i]);
    }
  }
#pragma unroll 2
  for (int rr = w; rr < LNB_ROWS; rr += 8) {
    const long row = r0 + rr;
    if (row >= a.N) break;
    const float mean = a.mean[row], rstd = a.rstd[row];
    float xh[CH][8], dxh[CH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const long ch = lane + 64L * i;
#pragma unroll
      for (int e = 0; e < 8; ++e) xh[i][e] = dxh[i][e] = 0.f;
      if (ch < nch) {
        float sv[8], go[8];
        ld8<float>(a.s + row * d + ch * 8, sv);
        ld8<float>(a.dout + row * d + ch * 8, go);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = (sv[e] - mean) * rstd;
          float g = go[e];
          if (a.fsc) {
            psc[i][e] += g * (x * gm[i][e] + bt[i][e]);
            psh[i][e] += g;
            g *= 1.f + fs[i][e];
          }
          pg[i][e] += g * x;
          pb[i][e] += g;
          const float gx = g * gm[i][e];
          xh[i][e] = x;
          dxh[i][e] = gx;
          s1 += gx;
          s2 += gx * x;
        }
      }
    }
    s1 = wave_sum_v(s1) / (float)d;
    s2 = wave_sum_v(s2) / (float)d;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const long ch = lane + 64L * i;
      if (ch < nch) {
        float ds[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) ds[e] = rstd * (dxh[i][e] - s1 - xh[i][e] * s2);
        if (a.dres) st8<float>(a.dres + row * d + ch * 8, ds);
        if (a.dy_t) {
          if (a.thr16) {
            const unsigned k = keep8(eff_seed(a.seed, a.seed_off), a.stream, (uint64_t)(row * d + ch * 8), a.thr16);
#pragma unroll
            for (int e = 0; e < 8; ++e) ds[e] = ((k >> e) & 1u) ? ds[e] * a.drop_scale : 0.f;
          }
          st8<OT>((OT*)a.dy_t + row * d + ch * 8, ds);
        }
      }
    }
  }
  // 8 waves, a 4-wave LDS image: waves 4-7 store, waves 0-3 add them to their own partials and store the sums
  if (w >= 4) {
#pragma unroll
    for (int i = 0; i < CH; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = (lane + 64 * i) * 8 + e;
        red[0][w - 4][c] = pg[i][e];
        red[1][w - 4][c] = pb[i][e];
        red[2][w - 4][c] = psc[i][e];
        red[3][w - 4][c] = psh[i][e];
      }
  }
  __syncthreads();
  if (w < 4) {
#pragma unroll
    for (int i = 0; i < CH; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = (lane + 64 * i) * 8 + e;
        pg[i][e] += red[0][w][c];
        pb[i][e] += red[1][w][c];
        psc[i][e] += red[2][w][c];
        psh[i][e] += red[3][w][c];
      }
  }
  __syncthreads();
  if (w < 4) {
#pragma unroll
    for (int i = 0; i < CH; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = (lane + 64 * i) * 8 + e;
        red[0][w][c] = pg[i][e];
        red[1][w][c] = pb[i][e];
        red[2][w][c] = psc[i][e];
        red[3][w][c] = psh[i][e];
      }
  }
  __syncthreads();
  for (long c = threadIdx.x; c < d; c += 512) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = red[q][0][c] + red[q][1][c] + red[q][2][c] + red[q][3][c];
    if (a.part) {
      float* pp = a.part + (long)blockIdx.x * 4 * d + c;
      pp[0] = v[0];
      pp[d] = v[1];
      if (a.fsc) {
        pp[2 * d] = v[2];
        pp[3 * d] = v[3];
      }
      continue;
    }
    if (a.dgamma) {
      atomicAdd(a.dgamma + c, v[0]);
      atomicAdd(a.dbeta + c, v[1]);
    }
    if (a.fsc) {
      atomicAdd(a.dfsc + b * d + c, v[2]);
      atomicAdd(a.dfsh + b * d + c, v[3]);
    }
  }
}

// pass 2: parameter gradients as column reductions over row slabs (no per-row atomics):
//   dgamma[c] += sum dout'*xhat, dbeta[c] += sum dout', dfilm_scale[b][c] += sum dout*lnout,
//   dfilm_shift[b][c] += sum dout   (dout' = dout * (1 + film_scale[b]))
constexpr int LNP_ROWS = 64;
__global__ void __launch_bounds__(256) ln_bwd_params_kernel(LnBwdArgs a) {
  const long d = a.d;
  const long c = (long)blockIdx.x * 256 + threadIdx.x;
  if (c >= d) return;
  const long r0 = (long)blockIdx.y * LNP_ROWS;
  const long r1 = min(a.N, r0 + LNP_ROWS);
  const float gm = a.gamma[c], bt = a.beta[c];
  float dg = 0.f, db = 0.f, dsc = 0.f, dsh = 0.f;
  long cur_b = r0 / a.rows_per_batch;
  for (long r = r0; r < r1; ++r) {
    const long b = r / a.rows_per_batch;
    if (a.fsc && b != cur_b) {
      atomicAdd(a.dfsc + cur_b * d + c, dsc);
      atomicAdd(a.dfsh + cur_b * d + c, dsh);
      dsc = dsh = 0.f;
      cur_b = b;
    }
    const float x = (a.s[r * d + c] - a.mean[r]) * a.rstd[r];
    float go = a.dout[r * d + c];
    if (a.fsc) {
      dsc += go * (x * gm + bt);
      dsh += go;
      go *= 1.f + a.fsc[b * d + c];
    }
    dg += go * x;
    db += go;
  }
  if (a.dgamma) {
    atomicAdd(a.dgamma + c, dg);
    atomicAdd(a.dbeta + c, db);
  }
  if (a.fsc) {
    atomicAdd(a.dfsc + cur_b * d + c, dsc);
    atomicAdd(a.dfsh + cur_b * d + c, dsh);
  }
}

// Slab sums -> parameter gradients (one job per blockIdx.y; 64 columns x 16 slab groups per workgroup, the groups'
// sums added in a fixed order: bit-reproducible, unlike the slab atomics). blockIdx.z 0: dgamma[c] / dbeta[c] += the
// sums of quantities 0 / 1 over all slabs; z = 1 + b: dfilm_scale[b][c] / dfilm_shift[b][c] += those of quantities
// 2 / 3 over FiLM batch b's slabs (spb consecutive slabs per batch).
struct LnFoldJob {
  const float* part;
  long nslab, d, spb;
  float *dgamma, *dbeta, *dfs, *dfh;
};
struct LnFold {
  LnFoldJob j[LN_FOLD_MAX];
};
__global__ void __launch_bounds__(1024) ln_fold_kernel(LnFold f) {
  __shared__ float red[2][16][64];
  const LnFoldJob& J = f.j[blockIdx.y];
  const int z = blockIdx.z;
  const bool film = z > 0;
  if (film && (J.dfs == nullptr || (long)(z - 1) * J.spb >= J.nslab)) return;  // workgroup-uniform
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long c = (long)blockIdx.x * 64 + cl;
  const long k0 = film ? (long)(z - 1) * J.spb : 0, k1 = film ? min(J.nslab, k0 + J.spb) : J.nslab;
  float s0 = 0.f, s1 = 0.f;
  if (c < J.d) {
    const float* p = J.part + (film ? 2 * J.d : 0) + c;
#pragma unroll 16
    for (long k = k0 + g; k < k1; k += 16) {
      s0 += p[k * 4 * J.d];
      s1 += p[k * 4 * J.d + J.d];
    }
  }
  red[0][g][cl] = s0;
  red[1][g][cl] = s1;
  __syncthreads();
  if (g < 2 && c < J.d) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[g][i][cl];
    float* dst = film ? (g == 0 ? J.dfs : J.dfh) + (long)(z - 1) * J.d : (g == 0 ? J.dgamma : J.dbeta);
    dst[c] += t;
  }
}

}  // namespace fddm

using namespace fddm;

// x_dtype/y_dtype/out_dtype: FDDM_F32 / FDDM_BF16. y may be null. Outputs may be null.
FDDM_API int fddm_ln_fwd(int x_dtype, int y_dtype, int out_dtype, const void* x, const void* y, const float* gamma,
                         const float* beta, const float* film_scale, const float* film_shift, float* out_f32,
                         void* out_t, float* save_s, float* mean, float* rstd, long N, long d, long rows_per_batch,
                         float eps, float drop_p, unsigned long long seed, unsigned long long stream,
                         const float* rope_cos, const float* rope_sin, void* rope_out, long rope_L, void* hs) {
  if (N <= 0) return 0;
  if (d > 64 * 8 * LN_MAXCH || d % 8) return (int)hipErrorInvalidValue;
  if (rope_out && (!rope_cos || !rope_sin || rope_L <= 0 || d % 16 ||
                   (((uintptr_t)rope_cos | (uintptr_t)rope_sin | (uintptr_t)rope_out) & 15)))
    return (int)hipErrorInvalidValue;
  if ((((uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)film_scale | (uintptr_t)film_shift | (uintptr_t)x |
        (uintptr_t)y) & 15))
    return (int)hipErrorInvalidValue;  // 16-B vector accesses
  LnFwdArgs a{x, y, gamma, beta, film_scale, film_shift, out_f32, out_t, save_s, mean, rstd, N, d,
              rows_per_batch > 0 ? rows_per_batch : N, eps, seed, stream, 0u, 1.f, g_seed_off, rope_cos, rope_sin,
              rope_out, rope_L};
  if (drop_p > 0.f) {
    a.thr16 = (unsigned)llrintf(drop_p * 65536.f);
    a.drop_scale = 1.f / (1.f - drop_p);
  }
  if ((film_scale == nullptr) != (film_shift == nullptr)) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((N + 3) / 4));
  hipStream_t s = (hipStream_t)hs;
  const bool hy = y != nullptr, hf = film_scale != nullptr;
  // one chunk of 8 per lane when d <= 512: the two-chunk form re-loaded every lane's last chunk (x, y, gamma, beta,
  // FiLM) for the decoder's d = 512 rows
  const bool ch1 = d <= 512;
  if (rope_out) {  // the decoder's LN3 (f32 residual + bf16 branch -> bf16) only
    if (!(x_dtype == FDDM_F32 && y_dtype == FDDM_BF16 && out_dtype == FDDM_BF16 && hy && !hf))
      return (int)hipErrorInvalidValue;
    if (ch1) hipLaunchKernelGGL((ln_fwd_kernel<float, bf16_t, bf16_t, true, false, 1, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((ln_fwd_kernel<float, bf16_t, bf16_t, true, false, 2, true>), grid, dim3(256), 0, s, a);
    return (int)hipGetLastError();
  }
#define LNF2(XT, YT, OT, C)                                                                                    \
  do {                                                                                                         \
    if (hy && hf) hipLaunchKernelGGL((ln_fwd_kernel<XT, YT, OT, true, true, C>), grid, dim3(256), 0, s, a);     \
    else if (hy) hipLaunchKernelGGL((ln_fwd_kernel<XT, YT, OT, true, false, C>), grid, dim3(256), 0, s, a);     \
    else if (hf) hipLaunchKernelGGL((ln_fwd_kernel<XT, YT, OT, false, true, C>), grid, dim3(256), 0, s, a);     \
    else hipLaunchKernelGGL((ln_fwd_kernel<XT, YT, OT, false, false, C>), grid, dim3(256), 0, s, a);            \
  } while (0)
#define LNF(XT, YT, OT)                \
  do {                                 \
    if (ch1) LNF2(XT, YT, OT, 1);      \
    else LNF2(XT, YT, OT, 2);          \
  } while (0)
  if (x_dtype == FDDM_F32 && y_dtype == FDDM_BF16 && out_dtype == FDDM_BF16)
    LNF(float, bf16_t, bf16_t);
  else if (x_dtype == FDDM_F32 && y_dtype == FDDM_F32 && out_dtype == FDDM_F32)
    LNF(float, float, float);
  else if (x_dtype == FDDM_BF16 && y_dtype == FDDM_BF16 && out_dtype == FDDM_BF16)
    LNF(bf16_t, bf16_t, bf16_t);
  else if (x_dtype == FDDM_F32 && y_dtype == FDDM_F32 && out_dtype == FDDM_BF16)
    LNF(float, float, bf16_t);
  else
    return (int)hipErrorInvalidValue;
#undef LNF
#undef LNF2
  return (int)hipGetLastError();
}

FDDM_API int fddm_ln_bwd(int dy_dtype, const float* dout, const float* s, const float* mean, const float* rstd,
                         const float* gamma, const float* beta, const float* film_scale, float* dres, void* dy_t,
                         float* dgamma, float* dbeta, float* dfilm_scale, float* dfilm_shift, long N, long d,
                         long rows_per_batch, float drop_p, unsigned long long seed, unsigned long long stream,
                         float* partials, void* hs) {
  if (N <= 0) return 0;
  if (d > 64 * LN_MAXPL) return (int)hipErrorInvalidValue;
  LnBwdArgs a{dout, s, mean, rstd, gamma, beta, film_scale, dres, dy_t, dgamma, dbeta, dfilm_scale, dfilm_shift,
              partials, N, d, rows_per_batch > 0 ? rows_per_batch : N, seed, stream, 0u, 1.f, g_seed_off};
  if (drop_p > 0.f) {
    a.thr16 = (unsigned)llrintf(drop_p * 65536.f);
    a.drop_scale = 1.f / (1.f - drop_p);
  }
  hipStream_t st_ = (hipStream_t)hs;
  // parameter gradients wanted and every row slab inside one FiLM batch: the fused single pass
  const bool vec_ok = d % 8 == 0 && d <= 1024 &&
                      !(((uintptr_t)dout | (uintptr_t)s | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)film_scale |
                         (uintptr_t)dres | (uintptr_t)dy_t) & 15);
  const bool fused = (dgamma || dfilm_scale) && (!film_scale || a.rows_per_batch % LNB_ROWS == 0) &&
                     (!dgamma || (beta && dbeta)) && vec_ok;
  if (partials && !dgamma) return (int)hipErrorInvalidValue;
  if (partials && !fused) {  // the two-pass form adds with atomics: the slabs the fold will read contribute zero
    a.part = nullptr;
    const hipError_t e = hipMemsetAsync(partials, 0, (size_t)((N + LNB_ROWS - 1) / LNB_ROWS) * 4 * d * sizeof(float), st_);
    if (e != hipSuccess) return (int)e;
  }
  if (fused) {
    dim3 fg((unsigned)((N + LNB_ROWS - 1) / LNB_ROWS));
    const bool small = d <= 512;
    if (dy_dtype == FDDM_BF16) {
      if (small) hipLaunchKernelGGL((ln_bwd_fused_kernel<1, bf16_t>), fg, dim3(512), 0, st_, a);
      else hipLaunchKernelGGL((ln_bwd_fused_kernel<2, bf16_t>), fg, dim3(512), 0, st_, a);
    } else {
      if (small) hipLaunchKernelGGL((ln_bwd_fused_kernel<1, float>), fg, dim3(512), 0, st_, a);
      else hipLaunchKernelGGL((ln_bwd_fused_kernel<2, float>), fg, dim3(512), 0, st_, a);
    }
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)((N + 3) / 4));
  if (dy_dtype == FDDM_BF16)
    hipLaunchKernelGGL((ln_bwd_kernel<bf16_t>), grid, dim3(256), 0, st_, a);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<float>), grid, dim3(256), 0, st_, a);
  if (dgamma || dfilm_scale) {
    dim3 pg((unsigned)((d + 255) / 256), (unsigned)((N + LNP_ROWS - 1) / LNP_ROWS));
    hipLaunchKernelGGL(ln_bwd_params_kernel, pg, dim3(256), 0, st_, a);
  }
  return (int)hipGetLastError();
}

FDDM_API int fddm_ln_bwd_slab_rows(void) { return LNB_ROWS; }

FDDM_API int fddm_ln_fold(int n, const float* const* partials, const long* nslab, const long* d, float* const* dgamma,
                          float* const* dbeta, float* const* dfilm_scale, float* const* dfilm_shift,
                          const long* slabs_per_batch, void* hs) {
  if (n <= 0) return 0;
  if (n > LN_FOLD_MAX) return (int)hipErrorInvalidValue;
  LnFold f{};
  long dmax = 0, zmax = 1;
  for (int i = 0; i < n; ++i) {
    if (!partials[i] || !dgamma[i] || !dbeta[i] || nslab[i] <= 0 || d[i] <= 0) return (int)hipErrorInvalidValue;
    float* fs = dfilm_scale ? dfilm_scale[i] : nullptr;
    float* fh = dfilm_shift ? dfilm_shift[i] : nullptr;
    const long spb = slabs_per_batch ? slabs_per_batch[i] : 0;
    if ((fs == nullptr) != (fh == nullptr) || (fs && spb <= 0)) return (int)hipErrorInvalidValue;
    f.j[i] = LnFoldJob{partials[i], nslab[i], d[i], spb, dgamma[i], dbeta[i], fs, fh};
    dmax = d[i] > dmax ? d[i] : dmax;
    if (fs && 1 + (nslab[i] + spb - 1) / spb > zmax) zmax = 1 + (nslab[i] + spb - 1) / spb;
  }
  hipLaunchKernelGGL(ln_fold_kernel, dim3((unsigned)((dmax + 63) / 64), (unsigned)n, (unsigned)zmax), dim3(1024), 0,
                     (hipStream_t)hs, f);
  return (int)hipGetLastError();
}
