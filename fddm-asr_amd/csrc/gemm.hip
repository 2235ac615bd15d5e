// MFMA GEMM for gfx950:  C[m][n] = alpha * sum_k A(m,k) * B(n,k)  (+ fused epilogue)
//
// Each operand is either K-contiguous ("KC": A stored [M][K], B stored [N][K]) or M/N-contiguous
// ("MC": A stored [K][M], B stored [K][N]). That covers every GEMM of the train step without
// materialised transposes:
//   forward  Y  = X  W^T : A=X  KC, B=W  KC        (also the WavLM conv feature extractor as an
//                                                 implicit GEMM: the A row of output frame t is the
//                                                 window x[s*t .. s*t+k) of a channels-last input,
//                                                 i.e. lda = s*C < K, overlapping rows)
//   backward dX = dY W   : A=dY KC, B=W  MC
//   backward dW = dY^T X : A=dY MC, B=X  MC
// A rows are batched for the conv case: A(m,k) at A + (m / Mi)*sAb + (m % Mi)*lda + k.
//
// Tile 128x128, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 tiles of 16x16.
// A K-step moves 128 bytes of the compute type per tile row (bf16: 64 k, 2 x mfma_f32_16x16x32_bf16;
// f32: 32 k, 8 x mfma_f32_16x16x4f32 — exact fp32, the parity mode).
// LDS images (16 KB per operand per stage, double-buffered):
//   KC: [128 rows][128 B], 16-B chunk c of row r at r*128 + ((c ^ ((r>>1)&7))<<4)  -> ds_read_b128
//   MC: [K-step rows][128 elems]; bf16 8-B unit u of row k at k*256 + ((u ^ h(k))<<3),
//       h(k) = ((k&3)<<2) | (((k>>3)&1)<<4) -> conflict-free ds_read_b64_tr_b16 (hardware transpose)
//       f32: plain rows of 512 B, scalar reads.
// Register-staged prefetch of step k+1 is issued before the MFMAs of step k (one barrier per step).
// A may be stored in f32 while the MFMA runs in bf16 (TA=float, T=bf16): converted while staging.
#include "gemm.h"
#include <algorithm>
#include <functional>
#include <vector>
#include <map>
#include <mutex>
#include <queue>
#include <algorithm>
#include <cstdlib>

namespace fddm {


constexpr int GBM = 128, GBN = 128;
constexpr int GTILE_BYTES = 16384;  // per operand per stage

__device__ __forceinline__ int hk(int k) { return ((k & 3) << 2) | (((k >> 3) & 1) << 4); }

template <typename T> struct Mma;
template <> struct Mma<bf16_t> {
  static constexpr int KSTEP = 64, ECH = 8;
  __device__ __forceinline__ static void mma(f32x4_t& c, const uint4& a, const uint4& b) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0,
                                                0, 0);
  }
};
template <> struct Mma<float> {
  static constexpr int KSTEP = 32, ECH = 4;
  __device__ __forceinline__ static void mma(f32x4_t& c, const uint4& a, const uint4& b) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
  }
};

__device__ __forceinline__ unsigned pack_bf2(float a, float b) { return pk_bf16(a, b); }

// load one 16-B chunk of compute type T (ECH elements) from storage type TS
template <typename T, typename TS>
__device__ __forceinline__ uint4 load_chunk(const TS* p) {
  if constexpr (sizeof(T) == sizeof(TS)) {
    return *(const uint4*)p;
  } else {  // TS = float, T = bf16: 8 floats -> 8 bf16
    const float4 a = *(const float4*)p;
    const float4 b = *(const float4*)(p + 4);
    return make_uint4(pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y), pack_bf2(b.z, b.w));
  }
}

// Operand stager/reader. ROWS = M (or N) extent of the tile = 128.
template <typename T, typename TS, bool KC, bool CONV = false>
struct Operand {
  static constexpr int KSTEP = Mma<T>::KSTEP, ECH = Mma<T>::ECH;
  static constexpr int CPR = KC ? 8 : (128 / ECH);  // chunks per LDS row
  const TS* src[4];
  bool ok[4];
  int lds_off[4];
  long ld, dim_ext, K;
  int kk[4];  // KC: chunk k offset (elements); MC: row k within the step
  long tpos[4];
  ConvGeo cg;
  uint4 r[4];

  // dim0: first row (m or n) of the tile; batched KC addressing via (Mi, sb)
  __device__ __forceinline__ void init(const TS* base, long ld_, long Mi, long sb, long dim0, long dim_ext_, long K_,
                                       ConvGeo geo = ConvGeo{1, 0, 0, 0}) {
    ld = ld_; dim_ext = dim_ext_; K = K_; cg = geo;
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      if (KC) {
        const int row = c >> 3, cc = c & 7;
        const long m = dim0 + row;
        ok[i] = m < dim_ext;
        const long mm = ok[i] ? m : 0;
        if (CONV) {
          src[i] = base + (mm / Mi) * sb;
          tpos[i] = (mm % Mi) * cg.cstride - cg.cpad;
        } else {
          src[i] = base + (mm / Mi) * sb + (mm % Mi) * ld + cc * ECH;
        }
        kk[i] = cc * ECH;
        lds_off[i] = swz_kc(row, cc);
      } else {
        const int k = c / CPR, mc = c % CPR;
        const long m = dim0 + (long)mc * ECH;
        ok[i] = m < dim_ext;  // dim_ext % ECH == 0 (checked on host)
        src[i] = base + (long)k * ld + (ok[i] ? m : 0);
        kk[i] = k;
        if constexpr (sizeof(T) == 2) lds_off[i] = k * 256 + (((2 * mc) ^ hk(k)) << 3);
        else lds_off[i] = k * 512 + mc * 16;
      }
    }
  }
  __device__ __forceinline__ void gload(long kt) {
    const long k0 = kt * KSTEP;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (KC && CONV) {
        const long k = k0 + kk[i];
        const long tap = k / cg.Cg, c = k - tap * cg.Cg;
        const long tm = tpos[i] + tap;
        const bool in = ok[i] && (k < K) && tm >= 0 && tm < cg.Tin;
        r[i] = in ? load_chunk<T, TS>(src[i] + tm * ld + c) : make_uint4(0, 0, 0, 0);
      } else if (KC) {
        const bool in = ok[i] && (k0 + kk[i] < K);
        r[i] = in ? load_chunk<T, TS>(src[i] + k0) : make_uint4(0, 0, 0, 0);
      } else {
        const bool in = ok[i] && (k0 + kk[i] < K);
        r[i] = in ? load_chunk<T, TS>(src[i] + k0 * ld) : make_uint4(0, 0, 0, 0);
      }
    }
  }
  __device__ __forceinline__ void lstore(unsigned char* s) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) *(uint4*)(s + lds_off[i]) = r[i];
  }
  // MC operand: the 4 chunks of a thread share the same 8 (bf16) / 4 (f32) consecutive m's
  __device__ __forceinline__ void accum_rows(float (&cs)[8]) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint4 u = r[i];
      if constexpr (sizeof(T) == 2) {
        const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          cs[2 * j] += __uint_as_float(w[j] << 16);
          cs[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
        }
      } else {
        cs[0] += __uint_as_float(u.x); cs[1] += __uint_as_float(u.y);
        cs[2] += __uint_as_float(u.z); cs[3] += __uint_as_float(u.w);
      }
    }
  }
  // fragment for the 16-row tile starting at rb, sub-step sub (0/1)
  __device__ __forceinline__ static uint4 frag(const unsigned char* s, int rb, int sub, int lane) {
    const int g = lane >> 4, i = lane & 15;
    if constexpr (KC) {
      return *(const uint4*)(s + swz_kc(rb + i, sub * 4 + g));
    } else if constexpr (sizeof(T) == 2) {
      const int q = i >> 2, p = i & 3;
      const int k = sub * 32 + 8 * g + q;
      const int u = (rb >> 2) + p;
      typedef __attribute__((address_space(3))) s16x4_t* lp;
      const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(s + k * 256 + ((u ^ hk(k)) << 3)));
      const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(s + (k + 4) * 256 + ((u ^ hk(k + 4)) << 3)));
      const uint4 o = join_tr(lo, hi);
      return o;
    } else {
      const int k = sub * 16 + 4 * g;
      const float* f = (const float*)s;
      uint4 o;
      o.x = __float_as_uint(f[(k + 0) * 128 + rb + i]);
      o.y = __float_as_uint(f[(k + 1) * 128 + rb + i]);
      o.z = __float_as_uint(f[(k + 2) * 128 + rb + i]);
      o.w = __float_as_uint(f[(k + 3) * 128 + rb + i]);
      return o;
    }
  }
};


// 8 consecutive outputs as one 16-B (bf16) or two 16-B (f32) accesses
__device__ __forceinline__ void st_vec8(bf16_t* p, const float (&v)[8]) {
  uint4 u;
  u.x = pk_bf16(v[0], v[1]);
  u.y = pk_bf16(v[2], v[3]);
  u.z = pk_bf16(v[4], v[5]);
  u.w = pk_bf16(v[6], v[7]);
  *(uint4*)p = u;
}
__device__ __forceinline__ void st_vec8(float* p, const float (&v)[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void ld_vec8(const bf16_t* p, float (&v)[8]) {
  const uint4 u = *(const uint4*)p;
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld_vec8(const float* p, float (&v)[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// one 128x128 output tile (bx, by) of K-slice / group bz out of nz
template <typename T, typename TA, bool AKC, bool BKC, int EPI, typename OT, bool CONV>
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, unsigned char* smem, long bx, long by, long bz, long nzs) {
  constexpr int KSTEP = Mma<T>::KSTEP;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const long m0 = by * GBM, n0 = bx * GBN;

  // bz: group index (implicit conv) or split-K slice (plain GEMM, f32 atomic epilogue)
  const long z = bz;
  Operand<T, TA, AKC, CONV> opa;
  Operand<T, T, BKC> opb;
  long kbeg = 0, klen = g.K;
  long zg = CONV ? z : 0;
  if (!CONV && nzs > 1) {
    kbeg = z * g.ksplit;
    klen = min(g.ksplit, g.K - kbeg);
  }
  const TA* Abase = (const TA*)g.A + zg * g.sAz + (AKC ? kbeg : kbeg * g.lda);
  const T* Bbase = (const T*)g.B + zg * g.sBz + (BKC ? kbeg : kbeg * g.ldb);
  opa.init(Abase, g.lda, g.Mi, g.sAb, m0, g.M, klen, g.geo);
  opb.init(Bbase, g.ldb, 1L << 62, 0, n0, g.N, klen);
  OT* Cz = (OT*)g.C + zg * g.sCz;
  const float* biasz = g.bias ? g.bias + zg * g.sbiasz : nullptr;
  if (!CONV && z > 0) biasz = nullptr;
  const bool atomic_out = !CONV && nzs > 1;

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const long nk = (klen + KSTEP - 1) / KSTEP;
  // fused bias gradient: only the first N-tile column of blocks sums its A rows (MC A, bf16/f32 A)
  const bool do_cs = !AKC && (sizeof(TA) == sizeof(T)) && g.colsum != nullptr && bx == 0;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  opa.gload(0);
  opb.gload(0);
  if constexpr (!AKC && sizeof(TA) == sizeof(T)) if (do_cs) opa.accum_rows(cs);
  opa.lstore(smem);
  opb.lstore(smem + GTILE_BYTES);
  __syncthreads();
  for (long kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) {
      opa.gload(kt + 1);
      opb.gload(kt + 1);
    }
    const unsigned char* sa = smem + buf * 2 * GTILE_BYTES;
    const unsigned char* sb = sa + GTILE_BYTES;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      uint4 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = Operand<T, TA, AKC, CONV>::frag(sa, wr * 64 + i * 16, sub, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = Operand<T, T, BKC>::frag(sb, wc * 64 + j * 16, sub, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) Mma<T>::mma(acc[i][j], af[i], bfr[j]);
    }
    if (kt + 1 < nk) {
      unsigned char* na = smem + (buf ^ 1) * 2 * GTILE_BYTES;
      if constexpr (!AKC && sizeof(TA) == sizeof(T)) if (do_cs) opa.accum_rows(cs);
      opa.lstore(na);
      opb.lstore(na + GTILE_BYTES);
    }
    __syncthreads();
  }
  if constexpr (!AKC && sizeof(TA) == sizeof(T)) {
    if (do_cs) {
      // reduce the 256/CPR threads that share each m in LDS (the K loop has retired every LDS read),
      // then one atomic per (block, m)
      constexpr int ECH = Mma<T>::ECH, CPR = 128 / ECH;
      float* red = (float*)smem;  // [256][ECH]
#pragma unroll
      for (int j = 0; j < ECH; ++j) red[tid * ECH + j] = cs[j];
      __syncthreads();
      if (tid < 128) {
        const int mc = tid / ECH, j = tid % ECH;
        float sacc = 0.f;
        for (int q = mc; q < 256; q += CPR) sacc += red[q * ECH + j];
        const long m = m0 + tid;
        if (m < g.M) atomicAdd(g.colsum + m, sacc);
      }
    }
  }

  // epilogue, staged through LDS so that global accesses run along rows: each wave parks its 64x64 f32
  // sub-tile (16 KB; column chunks XOR-swizzled by row group against bank conflicts), then
  //  * f32 accumulate (split-K atomics / +=): lane = column, one 256-B contiguous row per instruction;
  //  * other epilogues: 8 consecutive columns per lane (16-B bf16 / 2x16-B f32 accesses).
  __syncthreads();  // K loop / colsum reduction have retired every LDS read
  float* tile = (float*)smem + wid * 4096;
  {
    const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = i * 16 + 4 * fg + e, c = j * 16 + fr;
          tile[r * 64 + (c ^ (((r >> 2) & 3) << 4))] = acc[i][j][e];
        }
  }
  __syncthreads();
  const long mw = m0 + wr * 64, nw = n0 + wc * 64;
  if constexpr (EPI == EPI_ACC_F32) {
    const long n = nw + lane;
    const bool nok = n < g.N;
    const float bv = (biasz && nok) ? biasz[n] : 0.f;
    for (int r = 0; r < 64; ++r) {
      const long m = mw + r;
      if (m >= g.M) break;
      const float v = tile[r * 64 + (lane ^ (((r >> 2) & 3) << 4))] * g.alpha + bv;
      if (nok) {
        float* c = (float*)Cz + m * g.ldc + n;
        if (atomic_out) atomicAdd(c, v);
        else *c += v;
      }
    }
  } else {
    const int cq = lane & 7, rq = lane >> 3;  // 8 columns per lane, 8 rows per pass
    const long n = nw + cq * 8;
    const bool vec = ((g.N & 7) == 0) && ((g.ldc & 7) == 0) && ((((uintptr_t)Cz) | ((uintptr_t)g.C2)) & 15) == 0;
    float bv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) bv[t] = (biasz && n + t < g.N) ? biasz[n + t] : 0.f;
    for (int r0 = 0; r0 < 64; r0 += 8) {
      const int r = r0 + rq;
      const long m = mw + r;
      if (m >= g.M || n >= g.N) continue;
      const int sw = ((r >> 2) & 3) << 4;
      const float4 lo = *(const float4*)(tile + r * 64 + ((cq * 8) ^ sw));
      const float4 hi = *(const float4*)(tile + r * 64 + ((cq * 8 + 4) ^ sw));
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = v[t] * g.alpha + bv[t];
      OT* crow = Cz + m * g.ldc + n;
      if constexpr (EPI == EPI_GELU) {
        float a[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          a[t] = gelu_f(v[t]);
          if (g.thr16)
            a[t] = drop_keep(eff_seed(g.seed, g.seed_off), g.stream, (uint64_t)(m * g.N + n + t), g.thr16) ? a[t] * g.drop_scale : 0.f;
        }
        OT* c2 = (OT*)g.C2 + m * g.ldc + n;
        if (vec) {
          st_vec8(crow, v);   // pre-activation, saved for backward
          st_vec8(c2, a);
        } else {
          for (int t = 0; t < 8 && n + t < g.N; ++t) {
            st<OT>(crow + t, v[t]);
            st<OT>(c2 + t, a[t]);
          }
        }
      } else if constexpr (EPI == EPI_DGELU) {
        const OT* pre = (const OT*)g.C2 + m * g.ldc + n;
        float pv[8];
        if (vec) {
          ld_vec8(pre, pv);
        } else {
          for (int t = 0; t < 8; ++t) pv[t] = (n + t < g.N) ? ld<OT>(pre + t) : 0.f;
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          v[t] *= gelu_grad(pv[t]);
          if (g.thr16)
            v[t] = drop_keep(eff_seed(g.seed, g.seed_off), g.stream, (uint64_t)(m * g.N + n + t), g.thr16) ? v[t] * g.drop_scale : 0.f;
        }
        if (vec) st_vec8(crow, v);
        else for (int t = 0; t < 8 && n + t < g.N; ++t) st<OT>(crow + t, v[t]);
      } else {
        if constexpr (EPI == EPI_GELU_ONLY) {
#pragma unroll
          for (int t = 0; t < 8; ++t) v[t] = gelu_f(v[t]);
        }
        if (vec) st_vec8(crow, v);
        else for (int t = 0; t < 8 && n + t < g.N; ++t) st<OT>(crow + t, v[t]);
      }
    }
  }
}


template <typename T, typename TA, bool AKC, bool BKC, int EPI, typename OT, bool CONV>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  gemm_tile<T, TA, AKC, BKC, EPI, OT, CONV>(g, smem, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.z);
}

// Grouped launch of independent GEMMs of one layout/epilogue (the weight gradients of a decoder block):
// workgroups [start[p], start[p+1]) run problem p, tiles ordered (split, row, column).
constexpr int GROUP_MAX = 12;
struct GroupArgs {
  int np;
  int start[GROUP_MAX + 1];
  int tn[GROUP_MAX], tm[GROUP_MAX], nz[GROUP_MAX];
  GemmArgs g[GROUP_MAX];
};

template <typename T, typename TA, bool AKC, bool BKC, int EPI, typename OT>
__global__ void __launch_bounds__(256) gemm_grouped_kernel(GroupArgs ga) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  int p = 0;
  while (p + 1 < ga.np && b >= ga.start[p + 1]) ++p;
  const int local = b - ga.start[p], per = ga.tn[p] * ga.tm[p];
  const int bz = local / per, rem = local - bz * per;
  gemm_tile<T, TA, AKC, BKC, EPI, OT, false>(ga.g[p], smem, rem % ga.tn[p], rem / ga.tn[p], bz, ga.nz[p]);
}

// =====================================================================================================
// "big" bf16 NT GEMM for the large forward shapes (WavLM conv layers 1..6, encoder/decoder projections
// with >= 256 output tiles): 256x128 tile, 512 threads = 8 waves (4 x 2, 64x64 each), BK = 64,
// operands staged by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip) into a 3-deep LDS ring
// (3 x 48 KB), two K-steps in flight behind a counted vmcnt, one raw s_barrier per K-step,
// XCD-aware tile order (tiles that share an A panel run on one XCD and hit its L2).
// Preconditions (checked on the host): K % 64 == 0, no padded conv taps, 16-B aligned rows.
// =====================================================================================================
constexpr int BBM = 256, BBN = 128, BSTAGES = 3;
constexpr int BA_BYTES = BBM * 128, BB_BYTES = BBN * 128, BSTAGE_BYTES = BA_BYTES + BB_BYTES;

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// LDS fragment read issued as inline asm: hipcc's waitcnt pass would otherwise make every ds_read wait for
// ALL outstanding LDS-DMA (vmcnt(0)), serialising the ring. The caller waits lgkmcnt itself.
__device__ __forceinline__ u32x4_t ds_read128(const unsigned char* p) {
  const unsigned a = (unsigned)(size_t)(lptr_t)(void*)p;
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

template <int EPI, typename OT, bool CONV>
__global__ void __launch_bounds__(512) gemm_big_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (LDS-DMA base in M0)
  const int wr = wid >> 1, wc = wid & 1;
  // XCD-aware bijective remap of the linear block id (blocks b, b+8, ... share an XCD)
  const long nN = (g.N + BBN - 1) / BBN, nM = (g.M + BBM - 1) / BBM;
  const long nwg = nN * nM;
  const long orig = blockIdx.x;
  const long q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const long t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const long m0 = (t / nN) * BBM, n0 = (t % nN) * BBN;

  const bf16_t* A = (const bf16_t*)g.A;
  const bf16_t* B = (const bf16_t*)g.B;
  // LDS-DMA issue geometry: one wave instruction fills 1 KB = 8 rows x 128 B of an image; lane l lands at
  // byte 16*l, i.e. row (l >> 3), physical chunk (l & 7) which must hold logical chunk (l&7) ^ ((row>>1)&7).
  // A: 256 rows = 32 pieces -> 4 per wave; B: 128 rows = 16 pieces -> 2 per wave.
  const bf16_t* asrc[4];
  const bf16_t* bsrc[2];
  long atpos[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wid * 4 + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    long m = m0 + row;
    if (m >= g.M) m = g.M - 1;
    if (CONV) {
      asrc[i] = A + (m / g.Mi) * g.sAb + c * 8;
      atpos[i] = (m % g.Mi) * g.geo.cstride;
    } else {
      asrc[i] = A + m * g.lda + c * 8;
      atpos[i] = 0;
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wid * 2 + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    long n = n0 + row;
    if (n >= g.N) n = g.N - 1;
    bsrc[i] = B + n * g.ldb + c * 8;
  }
  // issue cursor (wave-uniform scalars): next K-step's element offset, conv (tap, channel) split
  int ik_tap = 0, ik_c = 0;
  long ik_k0 = 0;
  auto issue = [&](int stage) {
    unsigned char* sa = smem + stage * BSTAGE_BYTES;
    unsigned char* sb = sa + BA_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // implicit conv: the 64-wide K-step never crosses a tap (Cg % 64 == 0, host check)
      const bf16_t* src = CONV ? asrc[i] + (atpos[i] + ik_tap) * g.lda + ik_c : asrc[i] + ik_k0;
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(sa + (wid * 4 + i) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gptr_t)(bsrc[i] + ik_k0), (lptr_t)(sb + (wid * 2 + i) * 1024), 16, 0, 0);
    ik_k0 += 64;
    if (CONV) {
      ik_c += 64;
      if (ik_c == (int)g.geo.Cg) {
        ik_c = 0;
        ++ik_tap;
      }
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)(g.K / 64);
  issue(0);
  if (nk > 1) issue(1);
  int cur = 0, nxt = 2;  // ring slots of K-step kt and kt + 2
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed for this thread's DMAs (the next stage may stay in flight), then every wave's
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(nxt);
    const unsigned char* sa = smem + cur * BSTAGE_BYTES;
    cur = cur == BSTAGES - 1 ? 0 : cur + 1;
    nxt = nxt == BSTAGES - 1 ? 0 : nxt + 1;
    const unsigned char* sb = sa + BA_BYTES;
    const int fr = lane & 15, fg = lane >> 4;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      u32x4_t af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = ds_read128(sa + swz_kc(wr * 64 + i * 16 + fr, sub * 4 + fg));
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = ds_read128(sb + swz_kc(wc * 64 + j * 16 + fr, sub * 4 + fg));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[i]),
                                                              __builtin_bit_cast(bf16x8_t, bfr[j]), acc[i][j], 0, 0, 0);
    }
  }

  const int fr = lane & 15, fg = lane >> 4;
  float bvs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long n = n0 + wc * 64 + j * 16 + fr;
    bvs[j] = (g.bias && n < g.N) ? g.bias[n] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long n = n0 + wc * 64 + j * 16 + fr;
    if (n >= g.N) continue;
    const float bv = bvs[j];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long m = m0 + wr * 64 + i * 16 + 4 * fg + e;
        if (m >= g.M) continue;
        const float v = acc[i][j][e] * g.alpha + bv;
        OT* c = (OT*)g.C + m * g.ldc + n;
        if constexpr (EPI == EPI_STORE) {
          st<OT>(c, v);
        } else if constexpr (EPI == EPI_GELU) {
          st<OT>(c, v);
          float a = gelu_f(v);
          if (g.thr16) a = drop_keep(eff_seed(g.seed, g.seed_off), g.stream, (uint64_t)(m * g.N + n), g.thr16) ? a * g.drop_scale : 0.f;
          st<OT>((OT*)g.C2 + m * g.ldc + n, a);
        } else if constexpr (EPI == EPI_GELU_ONLY) {
          st<OT>(c, gelu_f(v));
        }
      }
    }
  }
}

template <int EPI, typename OT, bool CONV>
static int launch_big(const GemmArgs& g, hipStream_t s) {
  const long tiles = ((g.N + BBN - 1) / BBN) * ((g.M + BBM - 1) / BBM);
  hipLaunchKernelGGL((gemm_big_kernel<EPI, OT, CONV>), dim3((unsigned)tiles), dim3(512), BSTAGES * BSTAGE_BYTES, s, g);
  return (int)hipGetLastError();
}

static bool big_ok(const GemmArgs& g, bool conv) {
  if (g.K % 64) return false;
  const long tiles = ((g.N + BBN - 1) / BBN) * ((g.M + BBM - 1) / BBM);
  if (tiles < 240) return false;
  if (conv && (g.geo.cpad != 0 || g.geo.Cg % 64)) return false;
  return true;
}

template <typename T, typename TA, bool AKC, bool BKC, int EPI, typename OT, bool CONV = false>
static int launch(const GemmArgs& g, hipStream_t s, int nz) {
  dim3 grid((unsigned)((g.N + GBN - 1) / GBN), (unsigned)((g.M + GBM - 1) / GBM), (unsigned)nz);
  hipLaunchKernelGGL((gemm_kernel<T, TA, AKC, BKC, EPI, OT, CONV>), grid, dim3(256), 4 * GTILE_BYTES, s, g);
  return (int)hipGetLastError();
}

template <typename T, typename TA, bool AKC, bool BKC>
static int dispatch_epi(int epi, int out_dtype, const GemmArgs& g, hipStream_t s, int nz) {
  if (epi == EPI_STORE) {
    if (out_dtype == FDDM_F32) return launch<T, TA, AKC, BKC, EPI_STORE, float>(g, s, nz);
    if constexpr (sizeof(T) == 2) return launch<T, TA, AKC, BKC, EPI_STORE, bf16_t>(g, s, nz);
  } else if (epi == EPI_GELU) {
    return launch<T, TA, AKC, BKC, EPI_GELU, T>(g, s, nz);
  } else if (epi == EPI_ACC_F32) {
    return launch<T, TA, AKC, BKC, EPI_ACC_F32, float>(g, s, nz);
  } else if (epi == EPI_DGELU) {
    return launch<T, TA, AKC, BKC, EPI_DGELU, T>(g, s, nz);
  } else if (epi == EPI_GELU_ONLY) {
    return launch<T, TA, AKC, BKC, EPI_GELU_ONLY, T>(g, s, nz);
  }
  return (int)hipErrorInvalidValue;
}

template <typename T, typename TA>
static int dispatch_layout(int a_kc, int b_kc, int epi, int out_dtype, const GemmArgs& g, hipStream_t s, int nz) {
  if (a_kc && b_kc) return dispatch_epi<T, TA, true, true>(epi, out_dtype, g, s, nz);
  if (a_kc && !b_kc) return dispatch_epi<T, TA, true, false>(epi, out_dtype, g, s, nz);
  if (!a_kc && !b_kc) return dispatch_epi<T, TA, false, false>(epi, out_dtype, g, s, nz);
  return dispatch_epi<T, TA, false, true>(epi, out_dtype, g, s, nz);
}

// f32 [M][N] sub-matrix (row stride ldc) := 0 — the split-K pre-zero. A kernel on the launch stream, not
// hipMemset2DAsync: captured into a HIP graph, the memset node did not stay ordered before the accumulating
// GEMM on replays (the frozen encoder's graph, fddm_hip/graphs.py, read partially zeroed outputs).
__global__ void __launch_bounds__(256) zero2d_kernel(float* __restrict__ C, long ldc, long M, long N) {
  const long n4 = N / 4, per_row = n4 + (N & 3);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < M * per_row; i += (long)gridDim.x * 256) {
    const long m = i / per_row, j = i - m * per_row;
    float* row = C + m * ldc;
    if (j < n4 && !(((uintptr_t)row) & 15)) {
      *(float4*)(row + 4 * j) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else if (j < n4) {
      row[4 * j] = 0.f; row[4 * j + 1] = 0.f; row[4 * j + 2] = 0.f; row[4 * j + 3] = 0.f;
    } else {
      row[4 * n4 + (j - n4)] = 0.f;
    }
  }
}

static hipError_t zero2d(float* C, long ldc, long M, long N, hipStream_t s) {
  const long work = M * (N / 4 + (N & 3));
  if (work <= 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<long>((work + 255) / 256, 2048);
  hipLaunchKernelGGL(zero2d_kernel, dim3(grid), dim3(256), 0, s, C, ldc, M, N);
  return hipGetLastError();
}

}  // namespace fddm

using namespace fddm;

// Kernel-family override for tests and diagnostics (fddm_gemm_force_path; 0 = the automatic choice below):
// 1 "big" disables the 256x256 kernel, 2 "small" routes every GEMM through the register-staged 128x128 kernel,
// 3 "256" takes the 256x256 kernel wherever its preconditions hold, 4 "128" the 128x128 LDS-DMA ring kernel
static int g_gemm_path = 0;
static int gemm_path() { return g_gemm_path; }
static bool big_enabled() { return gemm_path() != 2 && gemm_path() != 4; }
static bool g256_enabled() { return gemm_path() == 0 || gemm_path() == 3; }
static bool g128_enabled() { return gemm_path() == 0 || gemm_path() == 4; }
// the persistent 256x256 kernel from a quarter round of tiles up: alone on the chip 64 tiles of 8192x512x512 lose
// to the 128x128 kernel, but beside the encoder's persistent GEMMs (half or a quarter of the CUs free) one round of
// 64 tiles beats two rounds of 256: the decoder's d-wide forward GEMMs (out-proj, cross Q / out, V, FF2) — C4
// (d 768: 96 tiles) 17.79-17.87 -> 17.36-17.37 ms/step, C2 (64 tiles) 9.89 -> 9.87 ms average of 6 alternating rounds
// (threshold 128 before; 32 measured neutral, round 3)
static bool prefer_256(long M, long N) { return gemm_path() == 3 || gemm256_tiles(M, N) >= 64; }
// split-K: aim at ~512 workgroups, at least 512 K elements per split
static long splitk_target() { return 512; }
static long splitk_mink() { return 512; }

FDDM_API int fddm_gemm_force_path(int path) {
  const int old = g_gemm_path;
  g_gemm_path = (path >= 0 && path <= 4) ? path : 0;
  return old;
}

// dx[M][N] += rope_bwd(dy[M][K] @ w[K][N]) — the decoder's self-attention input gradient through RoPE in one launch
// (gemm128 EPI_ROPE_ACC; replaces linear_dx into an f32 temporary + fddm_rope_bwd, ref models/denoise_decoder.py:
// 150-156 apply_rope backward). bf16 dy / w, f32 dx and tables [L][N]; N % 128 == 0.
FDDM_API int fddm_linear_dx_rope(const void* dy, long ldy, const void* w, long ldw, float* dx, long lddx, const float* cs,
                                 const float* sn, long M, long N, long K, long L, void* hip_stream) {
  if (M <= 0 || N <= 0) return 0;
  if (!g128_enabled() || K % 8 || ldy % 8 || ldw % 8 || ((uintptr_t)dy & 15) || ((uintptr_t)w & 15) || ((uintptr_t)dx & 15))
    return (int)hipErrorInvalidValue;
  GemmArgs g{dy, ldy, 1L << 62, 0, w, ldw, dx, lddx, nullptr, nullptr, 1.f, M, N, K, 0, 0, 0u, 1.f, ConvGeo{1, 0, 0, 0}, 0, 0, 0, 0, K,
             nullptr, g_seed_off, cs, sn, L};
  return gemm128_launch(g, true, false, EPI_ROPE_ACC, FDDM_F32, 1, (hipStream_t)hip_stream);
}

FDDM_API int fddm_gemm(int dtype, int a_dtype, int a_kc, int b_kc, int epi, int out_dtype, const void* A, long lda,
                       long Mi, long sAb, const void* B, long ldb, void* C, long ldc, void* C2, const float* bias,
                       float alpha, long M, long N, long K, unsigned long long seed, unsigned long long stream,
                       float drop_p, float* colsum, void* hip_stream) {
  if (M <= 0 || N <= 0) return 0;
  const int ech = dtype == FDDM_BF16 ? 8 : 4;
  // layout preconditions (16-B chunks never straddle a row end or the tile edge)
  if (a_kc ? (K % ech || lda % ech || sAb % ech) : (M % ech || lda % ech)) return (int)hipErrorInvalidValue;
  if (b_kc ? (K % ech || ldb % ech) : (N % ech || ldb % ech)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return (int)hipErrorInvalidValue;
  if (!C || ((epi == EPI_GELU || epi == EPI_DGELU) && !C2)) return (int)hipErrorInvalidValue;  // second output
  if (!a_kc && Mi > 0 && Mi != M) return (int)hipErrorInvalidValue;
  if (Mi <= 0) Mi = 1L << 62;
  GemmArgs g{A, lda, Mi, sAb, B, ldb, C, ldc, C2, bias, alpha, M, N, K, seed, stream, 0u, 1.f, ConvGeo{1, 0, 0, 0}, 0, 0, 0, 0, K, nullptr,
             g_seed_off};
  if (colsum) {
    if (a_kc || a_dtype != dtype) return (int)hipErrorInvalidValue;
    if (epi != EPI_ACC_F32) {  // colsum follows C: overwritten by STORE, accumulated by ACC
      hipError_t e = zero2d(colsum, M, 1, M, (hipStream_t)hip_stream);
      if (e != hipSuccess) return (int)e;
    }
    g.colsum = colsum;
  }
  if ((epi == EPI_GELU || epi == EPI_DGELU) && drop_p > 0.f) {
    g.thr16 = (unsigned)llrintf(drop_p * 65536.f);
    g.drop_scale = 1.f / (1.f - drop_p);
  }
  hipStream_t s = (hipStream_t)hip_stream;
  // bf16 operands: the 256x256 kernel for outputs of >= half a round of its tiles (NT only), else the 128x128
  // LDS-DMA ring kernel (NT, NN with W as stored, TN weight gradients)
  if (dtype == FDDM_BF16 && a_dtype == FDDM_BF16 && Mi >= M && g128_enabled() &&
      !(a_kc && b_kc && !colsum && g256_enabled() && gemm256_ok(g, epi, out_dtype, false) && prefer_256(M, N)) &&
      gemm128_ok(g, a_kc, b_kc, epi, out_dtype) && (!colsum || !a_kc)) {
    int nz128 = 1;
    const long t128 = gemm128_tiles(M, N);
    // split-K only for long reductions: a split slice adds its 128x128 tile with 64 KB of f32 atomics
    if (out_dtype == FDDM_F32 && (epi == EPI_STORE || epi == EPI_ACC_F32) && t128 < 192 && K >= 4096) {
      long want = (256 + t128 - 1) / t128;
      nz128 = (int)std::max(1L, std::min(want, K / 2048));
      if (nz128 > 1) {
        long ks = ((K + nz128 - 1) / nz128 + 63) / 64 * 64;
        nz128 = (int)((K + ks - 1) / ks);
        g.ksplit = ks;
        if (epi == EPI_STORE) {
          hipError_t e = zero2d((float*)C, ldc, M, N, s);
          if (e != hipSuccess) return (int)e;
          epi = EPI_ACC_F32;
        }
      }
    }
    return gemm128_launch(g, a_kc, b_kc, epi, out_dtype, nz128, s);
  }
  // split-K when the output has too few 128x128 tiles to fill 256 CUs (weight gradients, small N):
  // f32 output only, atomically accumulated; STORE becomes memset + accumulate.
  int nz = 1;
  const long tiles = ((M + GBM - 1) / GBM) * ((N + GBN - 1) / GBN);
  const int kstep = dtype == FDDM_BF16 ? 64 : 32;
  if (out_dtype == FDDM_F32 && (epi == EPI_STORE || epi == EPI_ACC_F32) && tiles < 512 && K >= 8 * kstep && Mi >= M) {
    // Split count: enough workgroups to cover the chip (splitk_target), but every split keeps at least
    // splitk_mink of K — each extra split costs M*N*4 B of float atomics (~1.3 TB/s chip-wide).
    long want = (splitk_target() + tiles - 1) / tiles;
    long maxs = K / std::max((long)kstep, splitk_mink());
    nz = (int)std::max(1L, std::min(want, std::min(maxs, 64L)));
    if (nz > 1) {
      long ks = (K + nz - 1) / nz;
      ks = (ks + kstep - 1) / kstep * kstep;
      nz = (int)((K + ks - 1) / ks);
      g.ksplit = ks;
      if (epi == EPI_STORE) {
        hipError_t e = zero2d((float*)C, ldc, M, N, s);
        if (e != hipSuccess) return (int)e;
        epi = EPI_ACC_F32;
      }
    }
  }
  if (dtype == FDDM_BF16 && a_dtype == FDDM_BF16 && a_kc && b_kc && nz == 1 && Mi >= M && !colsum &&
      g256_enabled() && gemm256_ok(g, epi, out_dtype, false) && prefer_256(M, N))
    return gemm256_launch(g, epi, out_dtype, false, s);
  if (dtype == FDDM_BF16 && a_dtype == FDDM_BF16 && a_kc && b_kc && nz == 1 && Mi >= M && !colsum &&
      out_dtype == FDDM_BF16 && big_ok(g, false) && big_enabled()) {
    if (epi == EPI_STORE) return launch_big<EPI_STORE, bf16_t, false>(g, s);
    if (epi == EPI_GELU) return launch_big<EPI_GELU, bf16_t, false>(g, s);
    if (epi == EPI_GELU_ONLY) return launch_big<EPI_GELU_ONLY, bf16_t, false>(g, s);
  }
  if (dtype == FDDM_BF16) {
    if (a_dtype == FDDM_BF16) return dispatch_layout<bf16_t, bf16_t>(a_kc, b_kc, epi, out_dtype, g, s, nz);
    if (a_dtype == FDDM_F32) return dispatch_layout<bf16_t, float>(a_kc, b_kc, epi, out_dtype, g, s, nz);
  } else if (dtype == FDDM_F32 && a_dtype == FDDM_F32) {
    return dispatch_layout<float, float>(a_kc, b_kc, epi, out_dtype, g, s, nz);
  }
  return (int)hipErrorInvalidValue;
}

// Implicit-GEMM 1-D convolution over a channels-last input x[b][time][lda] (KC A operand):
//   out[b*Tout + t][z*N + n] = act( sum_{tap,c} x[b][t*cstride - cpad + tap][z*Cg + c] * W[z][n][tap*Cg + c] + bias )
// for each group z < groups (gridDim.z). W is [groups][N][K = taps*Cg] (K-contiguous), out row stride ldc.
// epi: EPI_STORE or EPI_GELU_ONLY.  Sites: HF modeling_wavlm.py:675-693 (conv layers 1..6, groups=1) and
// 37-90 (positional grouped conv, groups=16, pad 64).
FDDM_API int fddm_conv1d_gemm(int dtype, int epi, const void* x, long lda, long sAb, long Tin, long Cg, long cstride,
                              long cpad, const void* W, void* out, long ldc, const float* bias, long Bn, long Tout,
                              long N, long K, int groups, void* hip_stream) {
  const int ech = dtype == FDDM_BF16 ? 8 : 4;
  if (Bn <= 0 || Tout <= 0) return 0;
  if (K % ech || Cg % ech || lda % ech || sAb % ech || ((uintptr_t)x & 15) || ((uintptr_t)W & 15))
    return (int)hipErrorInvalidValue;
  GemmArgs g{x, lda, Tout, sAb, W, K, out, ldc, nullptr, bias, 1.f, Bn * Tout, N, K, 0, 0, 0u, 1.f,
             ConvGeo{Cg, cstride, cpad, Tin}, Cg, N * K, N, N, K, nullptr};
  hipStream_t s = (hipStream_t)hip_stream;
  if (dtype == FDDM_BF16 && groups == 1 && g256_enabled() && gemm256_ok(g, epi, FDDM_BF16, true) &&
      prefer_256(g.M, N))
    return gemm256_launch(g, epi, FDDM_BF16, true, s);
  if (dtype == FDDM_BF16 && groups == 1 && big_ok(g, true) && big_enabled()) {
    if (epi == EPI_GELU_ONLY) return launch_big<EPI_GELU_ONLY, bf16_t, true>(g, s);
    return launch_big<EPI_STORE, bf16_t, true>(g, s);
  }
  if (dtype == FDDM_BF16) {
    if (epi == EPI_GELU_ONLY) return launch<bf16_t, bf16_t, true, true, EPI_GELU_ONLY, bf16_t, true>(g, s, groups);
    return launch<bf16_t, bf16_t, true, true, EPI_STORE, bf16_t, true>(g, s, groups);
  } else {
    if (epi == EPI_GELU_ONLY) return launch<float, float, true, true, EPI_GELU_ONLY, float, true>(g, s, groups);
    return launch<float, float, true, true, EPI_STORE, float, true>(g, s, groups);
  }
}

// Grouped weight-gradient GEMMs dW_p[M_p][N_p] += dY_p^T X_p (dY_p stored [K_p][M_p], X_p stored [K_p][N_p], both
// bf16 and M/N-contiguous), with the bias gradient db_p[m] += sum_k dY_p[k][m] fused (db_p may be null).
// One launch for up to 12 problems; a problem's K is split so that every workgroup reduces about
// `kchunk` tokens (f32 atomics between splits).
// Split choice for the 128x128 grouped launch: coordinate descent over each problem's split count
// (1, 2, 4, 8, 16) on the longest-processing-time schedule of all units over the CUs. Unit cost in K-tiles:
// its K-tiles + 6 (prologue / epilogue) + for split units the f32 atomics of its 128x128 tile (~20 K-tile
// times) or else a read-modify-write (2). Units run longest first (problem order on the host).
// The decision depends only on the shapes: cached per (tiles, K-tiles) signature.
static void g128_balance(int n, const long* tiles, const long* ktiles, int* nz, int ncu) {
  static std::mutex mu;
  static std::map<std::vector<long>, std::vector<int>> cache;
  std::vector<long> key(tiles, tiles + n);
  key.insert(key.end(), ktiles, ktiles + n);
  key.push_back(ncu);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) {
      std::copy(it->second.begin(), it->second.end(), nz);
      return;
    }
  }
  auto makespan = [&](const int* z) {
    std::vector<double> units;
    for (int p = 0; p < n; ++p)
      for (long u = 0; u < tiles[p] * z[p]; ++u)
        units.push_back((double)((ktiles[p] + z[p] - 1) / z[p]) + 6.0 + (z[p] > 1 ? 20.0 : 2.0));
    std::sort(units.begin(), units.end(), std::greater<double>());
    std::priority_queue<double, std::vector<double>, std::greater<double>> cu;
    for (int c = 0; c < ncu; ++c) cu.push(0.0);
    double mk = 0.0;
    for (double u : units) {
      const double t = cu.top() + u;
      cu.pop();
      cu.push(t);
      mk = std::max(mk, t);
    }
    return mk;
  };
  for (int p = 0; p < n; ++p) nz[p] = 1;
  double best = makespan(nz);
  for (int rnd = 0; rnd < 3; ++rnd) {
    bool changed = false;
    for (int p = 0; p < n; ++p)
      for (int c = 1; c <= 16; c *= 2) {
        if ((ktiles[p] + c - 1) / c < 8) break;
        const int old = nz[p];
        nz[p] = c;
        const double m = makespan(nz);
        if (m < best - 1e-9) {
          best = m;
          changed = true;
        } else {
          nz[p] = old;
        }
      }
    if (!changed) break;
  }
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = std::vector<int>(nz, nz + n);
}

static int g128_ncu() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  return ncu;
}

FDDM_API int fddm_gemm_dw_grouped(int n, const void* const* dy, const long* ldy, const void* const* x, const long* ldx,
                                  float* const* dw, const long* lddw, float* const* db, const long* M, const long* N,
                                  const long* K, long kchunk, void* hip_stream) {
  if (n <= 0) return 0;
  if (n > GROUP_MAX || n > G128_GROUP_MAX) return (int)hipErrorInvalidValue;
  bool g128 = g128_enabled() && kchunk <= 0;
  for (int p = 0; p < n && g128; ++p) {
    GemmArgs g{dy[p], ldy[p], 1L << 62, 0, x[p], ldx[p], dw[p], lddw[p], nullptr, nullptr, 1.f, M[p], N[p], K[p],
               0, 0, 0u, 1.f, ConvGeo{1, 0, 0, 0}, 0, 0, 0, 0, K[p], db[p]};
    g128 = gemm128_ok(g, false, false, EPI_ACC_F32, FDDM_F32);
  }
  if (g128) {
    // problems ordered by decreasing unit length, so the hardware's in-order dispatch approximates LPT
    long tiles[G128_GROUP_MAX], kt[G128_GROUP_MAX];
    int nz[G128_GROUP_MAX], ord[G128_GROUP_MAX];
    for (int p = 0; p < n; ++p) {
      tiles[p] = gemm128_tiles(M[p], N[p]);
      kt[p] = (K[p] + 63) / 64;
      ord[p] = p;
    }
    g128_balance(n, tiles, kt, nz, g128_ncu());
    std::sort(ord, ord + n, [&](int a, int b) { return (kt[a] + nz[a] - 1) / nz[a] > (kt[b] + nz[b] - 1) / nz[b]; });
    G128Group ga{};
    ga.np = n;
    int total = 0;
    for (int i = 0; i < n; ++i) {
      const int p = ord[i];
      GemmArgs g{dy[p], ldy[p], 1L << 62, 0, x[p], ldx[p], dw[p], lddw[p], nullptr, nullptr, 1.f, M[p], N[p], K[p],
                 0, 0, 0u, 1.f, ConvGeo{1, 0, 0, 0}, 0, 0, 0, 0, K[p], db[p]};
      if (nz[p] > 1) g.ksplit = ((K[p] + nz[p] - 1) / nz[p] + 63) / 64 * 64;
      ga.g[i] = g;
      ga.nz[i] = nz[p] > 1 ? (int)((K[p] + g.ksplit - 1) / g.ksplit) : 1;
      ga.tn[i] = (int)((N[p] + 127) / 128);
      ga.tm[i] = (int)((M[p] + 127) / 128);
      ga.start[i] = total;
      total += ga.tn[i] * ga.tm[i] * ga.nz[i];
    }
    ga.start[n] = total;
    return gemm128_grouped_dw(ga, total, (hipStream_t)hip_stream);
  }
  if (kchunk <= 0) kchunk = 8192;
  GroupArgs ga{};
  ga.np = n;
  int total = 0;
  for (int p = 0; p < n; ++p) {
    if (M[p] <= 0 || N[p] <= 0 || K[p] <= 0) return (int)hipErrorInvalidValue;
    if (M[p] % 8 || N[p] % 8 || ldy[p] % 8 || ldx[p] % 8) return (int)hipErrorInvalidValue;
    if ((((uintptr_t)dy[p]) | ((uintptr_t)x[p])) & 15) return (int)hipErrorInvalidValue;
    GemmArgs g{dy[p], ldy[p], 1L << 62, 0, x[p], ldx[p], dw[p], lddw[p], nullptr, nullptr, 1.f, M[p], N[p], K[p],
               0, 0, 0u, 1.f, ConvGeo{1, 0, 0, 0}, 0, 0, 0, 0, K[p], db[p]};
    long nz = kchunk > 0 ? (K[p] + kchunk / 2) / kchunk : 1;
    if (nz < 1) nz = 1;
    if (nz > 1) {
      long ks = (K[p] + nz - 1) / nz;
      ks = (ks + 63) / 64 * 64;
      nz = (K[p] + ks - 1) / ks;
      g.ksplit = ks;
    }
    ga.g[p] = g;
    ga.tn[p] = (int)((N[p] + GBN - 1) / GBN);
    ga.tm[p] = (int)((M[p] + GBM - 1) / GBM);
    ga.nz[p] = (int)nz;
    ga.start[p] = total;
    total += ga.tn[p] * ga.tm[p] * (int)nz;
  }
  ga.start[n] = total;
  hipLaunchKernelGGL((gemm_grouped_kernel<bf16_t, bf16_t, false, false, EPI_ACC_F32, float>), dim3(total), dim3(256),
                     4 * GTILE_BYTES, (hipStream_t)hip_stream, ga);
  return (int)hipGetLastError();
}
