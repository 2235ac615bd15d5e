// Helpers shared by the 32x32x16-MFMA decoder attention kernels (csrc/attn7.hip: fwd7 / dq7 / dkv7 / bwdf7 and the
// keep-bit producer; csrc/attn8.hip: the two-chain forward fwd8): MFMA wrapper, LDS-DMA pieces from SGPR bases,
// transposed LDS reads, the LDS image swizzles, the keep-bit storage layouts and the pre-scaled operand helpers.
#pragma once
#include <type_traits>

#include "attn_common.h"

namespace fddm {
namespace attn {

typedef __attribute__((ext_vector_type(16))) float f32x16_t;

// compile-time loop: f(integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ f32x16_t mfma32(const uint4& a, const uint4& b, const f32x16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// V image: 16-B chunk c of row r is stored at chunk c ^ vsw(r). A transposed read of a 32-lane half covers 4
// consecutive rows (4j .. 4j + 3) x 64 B; rows 4j and 4j + 2 share a 256-B bank window and land in opposite 64-B
// halves of it.
__device__ __forceinline__ int vsw(int r) { return (r & 2) << 1; }

// 4-B-per-lane LDS-DMA piece (256 B per wave-instruction into lds + 4 * lane)
__device__ __forceinline__ void dma4_asm(const void* src, const unsigned char* lds) {
  typedef __attribute__((address_space(3))) const void* lcp_t;
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lcp_t)(const void*)lds);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(la) : "memory", "m0");
}

// LDS-DMA piece from a wave-uniform 64-bit base (SGPRs) + a 32-bit per-lane byte offset: no 64-bit address math per
// lane and piece
__device__ __forceinline__ void dma16_sv(const void* sbase, unsigned voff, const unsigned char* lds) {
  typedef __attribute__((address_space(3))) const void* lcp_t;
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lcp_t)(const void*)lds);
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(la) : "memory", "m0");
}
__device__ __forceinline__ void dma4_sv(const void* sbase, unsigned voff, const unsigned char* lds) {
  typedef __attribute__((address_space(3))) const void* lcp_t;
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lcp_t)(const void*)lds);
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "s"(la) : "memory", "m0");
}

// the same with the LDS destination as a byte address (wave-uniform integer): no generic->LDS pointer conversion (and
// its null-pointer select) per piece
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  typedef __attribute__((address_space(3))) const void* lcp_t;
  return (unsigned)(size_t)(lcp_t)p;
}
__device__ __forceinline__ void dma16_so(const void* sbase, unsigned voff, unsigned la) {
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(la) : "memory", "m0");
}
__device__ __forceinline__ void dma4_so(const void* sbase, unsigned voff, unsigned la) {
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "s"(la) : "memory", "m0");
}

__device__ __forceinline__ s16x4_t tr_read(const unsigned char* p) {
  typedef __attribute__((address_space(3))) s16x4_t* lp;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(p));
}

constexpr int A7_TB = 64 * 128;  // one K or V tile in LDS: 64 rows x 128 B

// ------------------------------------------------------------------ dropout keep bits, storage layout v3 (lane masks)
// The keep decisions of RNG contract v2 (oracle attn_dropout_keep; attention.hip attn_keep4) stored so that one 64-bit
// word is the lane mask of one accumulator register of the 32x32x16 score MFMA with the query on the lane: for (b, h),
// 32-query group qg and 64-key tile t, slot j = 16 kb + r (kb = 32-key half, r = accumulator register), bit l =
// keep(query 32 qg + (l & 31), key 64 t + 32 kb + 8 (r >> 2) + 4 (l >> 5) + (r & 3)). Word index
// ((bh * nqg + qg) * ntiles + t) * 32 + j, nqg = ceil(Lq / 32). The forward and dQ kernels load a half-tile's 16
// words into SGPRs with scalar loads and drop a probability with one v_cndmask (inverse ballot); the dK / dV kernel
// (key on the lane) reads the one word of its key per 32-query half and extracts bits.
__device__ __forceinline__ long lm_word(int bh, int nqg, int ntiles, int qg, int t) {
  return (((long)bh * nqg + qg) * ntiles + t) * 32;
}
// The same bits per lane (the "per-lane dword" part of the site buffer, after the lane masks; layout v5): for (b, h, qg,
// t) 64 dwords, dword l = the 32 keep bits of lane l of the query-lane kernels. Register r of half kb (score pair
// p = 8 kb + (r >> 1), registers 2 p' and 2 p' + 1 of the half) sits at bit 15 - p (r even) or 31 - p (r odd): shifted
// left by p, the pair's two bits are bits 15 and 31, which one v_perm_b32 (selectors 8 / 9: the sign of byte 1 / 3)
// turns into the pair's 32-bit bf16 mask (fwd8). fwd7 and dq7 test single bits (bfe + and). The forward and dQ kernels
// stream one 256-B piece per wave and tile into LDS.
__host__ __device__ constexpr int lb_bit(int kb, int r) { return ((r & 1) ? 31 : 15) - (8 * kb + (r >> 1)); }
__device__ __forceinline__ long lb_dword(int bh, int nqg, int ntiles, int qg, int t) {
  return (((long)bh * nqg + qg) * ntiles + t) * 64;
}
// Images that serve both row reads (ds_read_b128, A = rows) and transposed reads (ds_read_b64_tr_b16, A = columns):
// chunk c of row r at c ^ dsw(r), dsw(r) = a ^ ((a & 1) << 2) with a = (r >> 1) & 7. A row-read lane group's 16 rows
// have distinct (r & 1, a), and a transposed read's rows 4j and 4j + 2 land 5 chunks apart (opposite 64-B halves).
__device__ __forceinline__ int dsw(int r) {
  const int a = (r >> 1) & 7;
  return a ^ ((a & 1) << 2);
}
// the register-resident operand of the backward's score MFMA (Q in dq7, K in dkv7) pre-scaled by sl2 = scale *
// log2(e) and rounded to bf16 once, so the product is the exponent in log2 units: 8 bf16 of one 16-B fragment
__device__ __forceinline__ uint4 scale_frag(const uint4& x, float c) {
  const u32x4v_t w = __builtin_bit_cast(u32x4v_t, x);
  u32x4v_t o;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    o[j] = pk_bf16(__uint_as_float(w[j] << 16) * c, __uint_as_float(w[j] & 0xFFFF0000u) * c);
  return __builtin_bit_cast(uint4, o);
}
// -x as a bf16 pair (hi, lo) with hi + lo = -x to ~2^-16 relative: the exact-constant fifth k-step of a score MFMA
__device__ __forceinline__ unsigned neg_split(float x) {
  const float hi = __uint_as_float(((unsigned)pk_bf16(-x, 0.f)) << 16);
  return pk_bf16(hi, -x - hi);
}

}  // namespace attn
}  // namespace fddm
