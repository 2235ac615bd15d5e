// Attention declarations shared by csrc/attention.hip (fwd2/5/6, dq/dkv 2/4, bwd3s, keep-bit producer) and
// csrc/attn7.hip (the 32x32x16-MFMA decoder kernels): launch arguments, XCD-aware block order, LDS image swizzle,
// lane-swap reductions and the inline-asm LDS-DMA helpers.
#pragma once
#include "common.h"

FDDM_API long fddm_attn_drop_words(int B, int H, int Lq, int Lk);

namespace fddm {
namespace attn {

// XCD-aware block order: the hardware deals workgroups round-robin over the 8 XCDs (linear id L -> XCD L % 8);
// remap so that each XCD receives a contiguous range of (bh, tile) work items — all tiles of one (batch, head) run
// on one XCD and read that head's K / V (or Q / dO) through one L2 instead of up to 8 (bijective for any grid size).
__device__ __forceinline__ void xcd_tile(int& bx, int& by) {
  const int nx = gridDim.x, n = nx * gridDim.y;
  const int L = blockIdx.x + blockIdx.y * nx;
  const int x = L & 7, j = L >> 3, q = n >> 3, r = n & 7;
  const int W = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
  by = W / nx;
  bx = W - by * nx;
}


constexpr int DH = 64;

__device__ __forceinline__ int kc_off(int RB, int r, int c) { return r * RB + ((c ^ ((r >> 1) & 7)) << 4); }

// cross-row reductions of the 16x16 C layout (lanes l, l^16, l^32, l^48 hold one query's keys) with the gfx950
// lane-swap instructions: v_permlane16_swap / v_permlane32_swap exchange a value between lanes l and l^16 (l^32) in
// the VALU, so r[0] and r[1] hold {own, partner} in some order — no LDS round trip (__shfl_xor's ds_bpermute)
__device__ __forceinline__ float xmax16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xsum16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ unsigned xor16(unsigned x) {
  const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return r[0] | r[1];
}
__device__ __forceinline__ unsigned xor32(unsigned x) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return r[0] | r[1];
}

// Attention-probability dropout, RNG contract v2 (oracle/fddm_oracle.py attn_dropout_keep): per (b, h) three tables of
// R = 4096 16-bit draws from splitmix64 at TAB0 + ..., per query row three offsets from splitmix64 at OFF0 + ...
constexpr int ATTN_R = 4096;
constexpr uint64_t ATTN_TAB0 = 1ull << 62, ATTN_OFF0 = 3ull << 62;

struct AttnArgs {
  const void *Q, *K, *V, *O, *dO;
  void *Out, *dQ, *dK, *dV;
  float* lse;
  float* delta;  // backward workspace, fddm_attn_bwd_ws_floats = 64 * B*H*LqP floats: the round-4 kernels' rowsum(dO*O)
                 // [B*H][Lq]; dq7's row terms [2][B*H][LqP] + pre-scaled Q' [B*H][LqP][64] bf16; bwdf7's f32 dQ partials
  uint64_t* dbits;  // dropout keep bits, fddm_attn_drop_words per site: layout v3 lane masks + v4 per-lane dwords
                    // (attn7.hip lm_word / lb_dword) for the 32x32x16 family, else round-4 words [B*H][ntiles][Lq]
  long sq, sk, sv, so, sdo, sdq, sdk, sdv;
  const unsigned char* key_keep;  // [B][Lk] or null
  const float* gate;              // [B*H][Lq] or null (WavLM)
  const float* table;             // [H][2*Lk-1]
  const void* graw;               // WavLM gate pre-activations (bf16) at graw + (b*Lq + q)*sgr + h*8 + o, or null
  long sgr;
  const float* gconst;            // [H] gru_rel_pos_const
  const void* gx;                 // WavLM gate from the attention input: x rows (bf16) at gx + (b*Lq + q)*sgx + h*64,
  long sgx;                       // folded weights gw = [sum of gru rows 0-3 (64) | rows 4-7 (64) | bias sums a, b]
  const float* gw;
  int B, H, Lq, Lk;
  float scale;
  uint64_t seed, stream;
  unsigned thr16;
  float drop_scale;
  int bits_ready;  // host side only: dbits already holds this site's keep bits (fddm_attn_drop_bits)
  const uint64_t* seed_off;  // graph-replay seed offset (common.h eff_seed) or null
};

__device__ __forceinline__ bool key_ok(const AttnArgs& a, int b, int key) {
  return key < a.Lk && (a.key_keep == nullptr || a.key_keep[(long)b * a.Lk + key]);
}

// inline-asm loads for the streamed kernels (hipcc does not track them; the kernels wait explicitly): a 1-KB
// LDS-DMA piece (16 B per lane into lds + 16 * lane; lds wave-uniform), and a register pin
typedef unsigned u32x4v_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void dma16_asm(const void* src, const unsigned char* lds) {
  typedef __attribute__((address_space(3))) const void* lcp_t;
  const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lcp_t)(const void*)lds);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(la) : "memory", "m0");
}
__device__ __forceinline__ void pin16(uint4& x) {
  u32x4v_t v = __builtin_bit_cast(u32x4v_t, x);
  asm volatile("" : "+v"(v));
  x = __builtin_bit_cast(uint4, v);
}

// csrc/attn7.hip: the 32x32x16-MFMA decoder forward (bf16, head_dim 64, Lk <= 1024, no dropout or keep bits already
// written by fddm_attn_drop_bits)
int attn7_fwd(AttnArgs& a, hipStream_t s);
// csrc/attn8.hip: the two-chain forward (same inputs, outputs and numerics contract as attn7_fwd)
int attn8_fwd(AttnArgs& a, hipStream_t s);
// the backward pair: dq7 (dQ; writes delta and -LSE log2(e) as [2][B*H][LqP] and the pre-scaled Q as
// [B*H][LqP][64] bf16 into a.delta) and dkv7 (dK, dV)
int attn7_dq(AttnArgs& a, hipStream_t s);
int attn7_dkv(AttnArgs& a, hipStream_t s);
// the fused backward for Lk <= 512 (dQ, dK, dV in one launch of one workgroup per (b, h), one pass per 256 keys;
// with two passes a.delta holds the f32 dQ partials, 64 floats per query row)
int attn7_bwdf(AttnArgs& a, hipStream_t s);
// the keep-bit producer of storage layout v3 (lane masks) and its words per site
int attn7_drop_bits(uint64_t* out, long site_words, int nsites, int BH, int Lq, int Lk, uint64_t seed,
                    uint64_t stream0, uint64_t stream_step, unsigned thr16, const uint64_t* seed_off, hipStream_t s);
long attn7_drop_words(int B, int H, int Lq, int Lk);

}  // namespace attn
}  // namespace fddm
