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
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// fp8 (OCP e4m3fn on gfx950) -> 8 x 16-bit MFMA operand V (bf16x8 / f16x8): one
// v_cvt_scalef32_pk_{bf16,f16}_fp8 per byte pair (scale 1.0; exact - every e4m3 value is
// representable in bf16 and in f16), half the VALU of the f32 round trip
// (v_cvt_pk_f32_fp8 + v_cvt_pk_bf16_f32) the fp8 decode GEMVs used to spend per pair.
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
template <typename T>
__device__ __forceinline__ uint32_t fp8x2_cvt(uint32_t w, bool hi);
template <>
__device__ __forceinline__ uint32_t fp8x2_cvt<__bf16>(uint32_t w, bool hi) {
  return hi ? __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(
                                               static_cast<int>(w), 1.0f, true))
            : __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(
                                               static_cast<int>(w), 1.0f, false));
}
template <>
__device__ __forceinline__ uint32_t fp8x2_cvt<_Float16>(uint32_t w, bool hi) {
  return hi ? __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(
                                               static_cast<int>(w), 1.0f, true))
            : __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(
                                               static_cast<int>(w), 1.0f, false));
}
template <typename T, typename V>
__device__ __forceinline__ V fp8x8_cvt(uint32_t lo, uint32_t hi) {
  const u32x4 r = {fp8x2_cvt<T>(lo, false), fp8x2_cvt<T>(lo, true), fp8x2_cvt<T>(hi, false),
                   fp8x2_cvt<T>(hi, true)};
  return __builtin_bit_cast(V, r);
}

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

// ---- device-coherent hand-over between workgroups -------------------------------------
// MI355X has one L2 per XCD and the L2s are not coherent with each other, so data one
// workgroup hands to another inside a launch normally needs an agent-scope release/acquire
// pair - which on gfx950 writes back / invalidates the WHOLE L2 of the XCD (buffer_wbl2 sc1 /
// buffer_inv sc1): measured 2.5 us (ctx 1000) to 8 us (ctx 2000) per decode-attention
// launch.  Instead the handed-over data is stored and loaded with device scope (sc1 cache
// policy: written through / missed in the XCD L2) through buffer instructions, which needs
// no fence: a device-scope store is visible device-wide once its vmcnt ack is back, and a
// device-scope load never returns a stale L1/L2 line.  Byte offsets are 32-bit.
constexpr int kScDevice = 16;  // aux cache-policy bits: sc1 (scope = device)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dev_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ void dev_store16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kScDevice);
}
__device__ __forceinline__ u32x4 dev_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kScDevice);
}
__device__ __forceinline__ void dev_store4(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, kScDevice);
}
__device__ __forceinline__ float dev_load4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kScDevice));
}

// ---- IPC all-reduce buffer layout shared by allreduce.hip and the GEMV push epilogue ----
namespace arl {
constexpr int kMaxRanks = 8;
constexpr size_t kGenOffset = 2 * kMaxRanks * 32 * sizeof(uint32_t);  // uint32 generation, block 0
constexpr size_t kSlotOffset = 64 * 1024;                              // slots (parity, src)
constexpr size_t kPushOffset = 48 * 1024;  // uint64 tile counter of source q at + 64 q
}  // namespace arl

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
