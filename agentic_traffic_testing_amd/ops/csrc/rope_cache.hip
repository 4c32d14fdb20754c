// Fused rotary embedding + paged KV-cache write (SURVEY §2.4 K4 + K5).
//
// One workgroup per token.  Reads the packed QKV projection row once, applies
// neox-style (rotate-half) RoPE to q and k using a host-precomputed fp32 cos|sin table
// (llama3 frequency scaling is folded into that table on the host), writes rotated q to
// `q_out` and writes rotated k / raw v straight into the paged cache.
//
// Cache layouts (chosen for the MFMA attention kernels in attention.hip):
//   k_cache [num_blocks, n_kv_heads, block_size, head_dim]   (token rows contiguous)
//   v_cache [num_blocks, n_kv_heads, head_dim, block_size]   (transposed: a 16x16 V^T tile
//                                                             is the A operand of the PV MFMA)
// slot_mapping[t] (int32) = page * block_size + offset, or -1 to skip the cache write (padding).
#include "common.h"
#include "kernels.h"

namespace atta {

template <typename T>
__global__ __launch_bounds__(256) void rope_cache_kernel(
    uint16_t* __restrict__ q_out, uint16_t* __restrict__ k_cache, uint16_t* __restrict__ v_cache,
    const uint16_t* __restrict__ qkv, const int* __restrict__ positions,
    const int* __restrict__ slot_mapping, const float* __restrict__ cos_sin, int n_q_heads,
    int n_kv_heads, int head_dim, int block_size, int64_t qkv_stride, int64_t q_out_stride) {
  const int64_t t = blockIdx.x;
  const int64_t pos = positions[t];
  const int64_t slot = slot_mapping[t];
  const int half = head_dim >> 1;
  const int hv = half >> 3;      // 8-wide vectors per half head
  const int dv = head_dim >> 3;  // 8-wide vectors per full head
  const float* cs = cos_sin + pos * head_dim;
  const uint16_t* row = qkv + t * qkv_stride;
  const int nq = n_q_heads * hv;
  const int nk = n_kv_heads * hv;
  const int nv = n_kv_heads * dv;
  const int64_t page = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? static_cast<int>(slot % block_size) : 0;

  for (int task = threadIdx.x; task < nq + nk + nv; task += blockDim.x) {
    if (task < nq + nk) {
      const bool is_q = task < nq;
      const int local = is_q ? task : task - nq;
      const int h = local / hv;
      const int i0 = (local % hv) * 8;
      const uint16_t* src = row + (is_q ? h * head_dim : (n_q_heads + h) * head_dim);
      Pack8 a = *reinterpret_cast<const Pack8*>(src + i0);
      Pack8 b = *reinterpret_cast<const Pack8*>(src + i0 + half);
      Pack8 ra, rb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = cs[i0 + j];
        const float s = cs[half + i0 + j];
        const float x1 = to_f32<T>(a.v[j]);
        const float x2 = to_f32<T>(b.v[j]);
        ra.v[j] = from_f32<T>(x1 * c - x2 * s);
        rb.v[j] = from_f32<T>(x2 * c + x1 * s);
      }
      if (is_q) {
        uint16_t* dst = q_out + t * q_out_stride + h * head_dim;
        *reinterpret_cast<Pack8*>(dst + i0) = ra;
        *reinterpret_cast<Pack8*>(dst + i0 + half) = rb;
      } else if (slot >= 0) {
        uint16_t* dst =
            k_cache + ((page * n_kv_heads + h) * static_cast<int64_t>(block_size) + off) * head_dim;
        *reinterpret_cast<Pack8*>(dst + i0) = ra;
        *reinterpret_cast<Pack8*>(dst + i0 + half) = rb;
      }
    } else if (slot >= 0) {
      const int local = task - nq - nk;
      const int h = local / dv;
      const int d0 = (local % dv) * 8;
      Pack8 a = *reinterpret_cast<const Pack8*>(row + (n_q_heads + n_kv_heads + h) * head_dim + d0);
      uint16_t* dst = v_cache + ((page * n_kv_heads + h) * static_cast<int64_t>(head_dim) + d0) *
                                    block_size + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j * block_size] = a.v[j];
    }
  }
}

}  // namespace atta

using namespace atta;

int atta_rope_cache(void* q_out, void* k_cache, void* v_cache, const void* qkv,
                    const int* positions, const int* slot_mapping, const float* cos_sin,
                    int num_tokens, int n_q_heads, int n_kv_heads, int head_dim, int block_size,
                    int64_t qkv_stride, int64_t q_out_stride, int dtype, hipStream_t stream) {
  if (head_dim % 16 != 0) return -1;
  if (num_tokens == 0) return 0;
  dim3 grid(num_tokens), block(256);
  auto qo = static_cast<uint16_t*>(q_out);
  auto kc = static_cast<uint16_t*>(k_cache);
  auto vc = static_cast<uint16_t*>(v_cache);
  auto in = static_cast<const uint16_t*>(qkv);
  if (dtype == 0)
    rope_cache_kernel<__bf16><<<grid, block, 0, stream>>>(qo, kc, vc, in, positions, slot_mapping,
                                                          cos_sin, n_q_heads, n_kv_heads, head_dim,
                                                          block_size, qkv_stride, q_out_stride);
  else
    rope_cache_kernel<_Float16><<<grid, block, 0, stream>>>(
        qo, kc, vc, in, positions, slot_mapping, cos_sin, n_q_heads, n_kv_heads, head_dim,
        block_size, qkv_stride, q_out_stride);
  return static_cast<int>(hipGetLastError());
}
