// Shared device helpers for the CDNA4 (gfx950) kernel library.
//
// Conventions used by every kernel in this directory:
//   * wave = 64 lanes; block sizes are multiples of 64.
//   * activations are bf16 or fp16 (template parameter T); accumulation is fp32.
//   * global loads/stores of activations are 16 B per lane (8 x 16-bit) wherever the
//     shape allows (guide: "Vectorize memory access - ALWAYS").
//   * no hipify / CUDA-compat headers: plain HIP + clang builtins.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace atta {

constexpr int kWave = 64;

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

// 16-byte packet of eight 16-bit values.
struct alignas(16) Pack8 {
  uint16_t v[8];
};
struct alignas(8) Pack4 {
  uint16_t v[4];
};

// ---- scalar conversions --------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float to_f32(uint16_t bits);
template <>
__device__ __forceinline__ float to_f32<__bf16>(uint16_t bits) {
  return __uint_as_float(static_cast<uint32_t>(bits) << 16);
}
template <>
__device__ __forceinline__ float to_f32<_Float16>(uint16_t bits) {
  return static_cast<float>(__builtin_bit_cast(_Float16, bits));
}

template <typename T>
__device__ __forceinline__ uint16_t from_f32(float f);
template <>
__device__ __forceinline__ uint16_t from_f32<__bf16>(float f) {
  // plain cast -> v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-preserving)
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
template <>
__device__ __forceinline__ uint16_t from_f32<_Float16>(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f));
}

// ---- wave / block reductions -----------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Sum over a whole block (blockDim.x multiple of 64, <= 1024).  `scratch` needs
// blockDim.x/64 floats of LDS.  Result is broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// 64-bit mix used by the sampler's counter-based RNG (splitmix64 finaliser).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace atta

#define ATTA_CHECK_LAUNCH() (void)hipGetLastError()
