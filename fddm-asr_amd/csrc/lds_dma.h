// Device primitives shared by the LDS-DMA pipelined GEMM kernels (gemm256.hip, gemm128.hip).
#pragma once
#include "common.h"
#include <type_traits>

namespace fddm {
namespace ldsdma {

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));

template <int V> using IC = std::integral_constant<int, V>;

constexpr unsigned SRD_W3 = 0x00020000u;  // buffer resource word 3 (raw dword access) on gfx9xx

__device__ __forceinline__ unsigned lds_addr(const void* p) { return (unsigned)(size_t)(lptr_t)(void*)p; }

// LDS fragment reads as inline asm: hipcc's waitcnt pass would make a plain ds_read wait for every
// outstanding LDS-DMA (vmcnt(0)); the kernels wait lgkmcnt themselves before the MFMAs.
template <int OFF>
__device__ __forceinline__ u32x4_t ds_read128_at(unsigned a) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF) : "memory");
  return v;
}
// gfx950 transposed read: per 16-lane group, lane 4q+p addresses row q, columns 4p..4p+3 of a 4 x 16 block of
// 16-bit elements; lane i receives column i (row q in element q)
template <int OFF>
__device__ __forceinline__ u32x2_t ds_read_tr16_at(unsigned a) {
  u32x2_t v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF) : "memory");
  return v;
}

// leave at most N vector-memory instructions of this wave in flight (N is always a compile-time count)
template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 63 ? N : 63) : "memory");
}
__device__ __forceinline__ void lgkmcnt0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ i32x4_t make_srd(const void* base) {
  const unsigned long a = (unsigned long)base;
  return i32x4_t{(int)(unsigned)a, (int)(unsigned)(a >> 32), 0x7fffffff, (int)SRD_W3};
}

// raw workgroup barrier that does not drain outstanding LDS-DMA (a __syncthreads() fence would emit vmcnt(0))
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace ldsdma
}  // namespace fddm
