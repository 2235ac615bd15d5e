// Probe: verify MFMA fragment layouts and ds_read_b64_tr_b16 on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/libprobe.so tools/probe_mfma.hip
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

// A [16][32] row-major bf16 as ushort, B [32][16] row-major, C [16][16] f32
__global__ void k_bf16(const unsigned short* A, const unsigned short* B, float* C) {
  int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    unsigned short av = A[(l & 15) * 32 + 8 * (l >> 4) + j];
    unsigned short bv = B[(8 * (l >> 4) + j) * 16 + (l & 15)];
    a[j] = __builtin_bit_cast(__bf16, av);
    b[j] = __builtin_bit_cast(__bf16, bv);
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  for (int j = 0; j < 4; ++j) C[(4 * (l >> 4) + j) * 16 + (l & 15)] = c[j];
}

// A [16][4] f32, B [4][16], C [16][16]
__global__ void k_f32(const float* A, const float* B, float* C) {
  int l = threadIdx.x;
  float a = A[(l & 15) * 4 + (l >> 4)];
  float b = B[(l >> 4) * 16 + (l & 15)];
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  for (int j = 0; j < 4; ++j) C[(4 * (l >> 4) + j) * 16 + (l & 15)] = c[j];
}

// tr_b16: LDS tile [4][16] u16 (row-major). Lane 4q+p of each 16-lane group points at row q, cols 4p..4p+3.
// Output: out[l*4 + e]
__global__ void k_tr(const unsigned short* in, unsigned short* out) {
  __shared__ __attribute__((aligned(16))) unsigned short t[64 * 4];
  int l = threadIdx.x;
  for (int i = l; i < 256; i += 64) t[i] = in[i];
  __syncthreads();
  int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  // group g uses rows 4g..4g+3 of a [16][16] tile
  const unsigned short* addr = &t[(4 * g + q) * 16 + 4 * p];
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)addr);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = (unsigned short)v[e];
}

extern "C" int probe_bf16(const void* A, const void* B, void* C, void* stream) {
  hipLaunchKernelGGL(k_bf16, dim3(1), dim3(64), 0, (hipStream_t)stream, (const unsigned short*)A, (const unsigned short*)B, (float*)C);
  return (int)hipGetLastError();
}
extern "C" int probe_f32(const void* A, const void* B, void* C, void* stream) {
  hipLaunchKernelGGL(k_f32, dim3(1), dim3(64), 0, (hipStream_t)stream, (const float*)A, (const float*)B, (float*)C);
  return (int)hipGetLastError();
}
extern "C" int probe_tr(const void* in, void* out, void* stream) {
  hipLaunchKernelGGL(k_tr, dim3(1), dim3(64), 0, (hipStream_t)stream, (const unsigned short*)in, (unsigned short*)out);
  return (int)hipGetLastError();
}
