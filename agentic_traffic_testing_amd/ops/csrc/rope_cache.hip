// Fused rotary embedding + paged KV-cache write (SURVEY §2.4 K4 + K5).
//
// One workgroup per token (decode-sized batches) or per 16-token tile (prefill, V staged
// through LDS for coalesced transposed stores).  Reads the packed QKV projection row once, applies
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

// 16-token tiles (prefill): one workgroup per (16 tokens, KV head) - the GQA group's q heads
// and the k head rotated as above, the head's V staged through LDS so the transposed V-cache
// stores are coalesced: lanes 16j..16j+15 write one dim's 16 consecutive token offsets (one
// 32-byte run when the tile's tokens fill one page) instead of the per-token kernel's 8
// single-element stores 32 B apart per lane.
constexpr int kRopeTile = 16;
template <typename T>
__global__ __launch_bounds__(256) void rope_cache_tile_kernel(
    uint16_t* __restrict__ q_out, uint16_t* __restrict__ k_cache, uint16_t* __restrict__ v_cache,
    const uint16_t* __restrict__ qkv, const int* __restrict__ positions,
    const int* __restrict__ slot_mapping, const float* __restrict__ cos_sin, int num_tokens,
    int n_q_heads, int n_kv_heads, int head_dim, int block_size, int64_t qkv_stride,
    int64_t q_out_stride) {
  extern __shared__ uint16_t vtile[];  // [kRopeTile][head_dim + 2]
  __shared__ int s_slot[kRopeTile];
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kRopeTile;
  const int hk = blockIdx.y;
  const int nt = min(kRopeTile, static_cast<int>(num_tokens - t0));
  const int G = n_q_heads / n_kv_heads;
  const int half = head_dim >> 1;
  const int hv = half >> 3;              // 8-wide vectors per half head
  const int per_tok = (G + 1) * hv;      // q heads of the group + the k head
  const int ldw = head_dim + 2;          // padded LDS row (16 rows on distinct banks)
  const int dv = head_dim >> 3;
  if (threadIdx.x < kRopeTile) s_slot[threadIdx.x] = threadIdx.x < nt ? slot_mapping[t0 + threadIdx.x] : -1;
  const int64_t vcol = static_cast<int64_t>(n_q_heads + n_kv_heads + hk) * head_dim;
  for (int e = threadIdx.x; e < nt * dv; e += blockDim.x) {
    const int i = e / dv, c = e - i * dv;
    const Pack8 a = *reinterpret_cast<const Pack8*>(qkv + (t0 + i) * qkv_stride + vcol + c * 8);
    uint16_t* d = vtile + i * ldw + c * 8;
#pragma unroll
    for (int j = 0; j < 8; j += 2)  // 4-byte LDS stores (the padded row is 4-byte aligned)
      *reinterpret_cast<uint32_t*>(d + j) = static_cast<uint32_t>(a.v[j]) |
                                            (static_cast<uint32_t>(a.v[j + 1]) << 16);
  }
  for (int task = threadIdx.x; task < nt * per_tok; task += blockDim.x) {
    const int i = task / per_tok, local = task - i * per_tok;
    const int64_t t = t0 + i;
    const int hh = local / hv;
    const int i0 = (local - hh * hv) * 8;
    const bool is_q = hh < G;
    const int slot = slot_mapping[t];
    if (!is_q && slot < 0) continue;
    const int head = is_q ? hk * G + hh : n_q_heads + hk;  // column block in the qkv row
    const float* cs = cos_sin + static_cast<int64_t>(positions[t]) * head_dim;
    const uint16_t* src = qkv + t * qkv_stride + static_cast<int64_t>(head) * head_dim;
    const Pack8 a = *reinterpret_cast<const Pack8*>(src + i0);
    const Pack8 b = *reinterpret_cast<const Pack8*>(src + i0 + half);
    Pack8 ra, rb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = cs[i0 + j];
      const float sn = cs[half + i0 + j];
      const float x1 = to_f32<T>(a.v[j]);
      const float x2 = to_f32<T>(b.v[j]);
      ra.v[j] = from_f32<T>(x1 * c - x2 * sn);
      rb.v[j] = from_f32<T>(x2 * c + x1 * sn);
    }
    uint16_t* dst = is_q ? q_out + t * q_out_stride + static_cast<int64_t>(head) * head_dim
                         : k_cache + ((static_cast<int64_t>(slot / block_size) * n_kv_heads + hk) *
                                          block_size + slot % block_size) * head_dim;
    *reinterpret_cast<Pack8*>(dst + i0) = ra;
    *reinterpret_cast<Pack8*>(dst + i0 + half) = rb;
  }
  __syncthreads();
  // transposed V writes: element f -> token f & 15, dim f >> 4
  for (int f = threadIdx.x; f < kRopeTile * head_dim; f += blockDim.x) {
    const int i = f & (kRopeTile - 1);
    const int d = f >> 4;
    const int slot = s_slot[i];
    if (slot < 0) continue;  // also tokens past the end (s_slot = -1)
    v_cache[((static_cast<int64_t>(slot / block_size) * n_kv_heads + hk) * head_dim + d) *
                block_size + slot % block_size] = vtile[i * ldw + d];
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
  auto qo = static_cast<uint16_t*>(q_out);
  auto kc = static_cast<uint16_t*>(k_cache);
  auto vc = static_cast<uint16_t*>(v_cache);
  auto in = static_cast<const uint16_t*>(qkv);
  const size_t lds = static_cast<size_t>(kRopeTile) * (head_dim + 2) * 2;
  if (num_tokens >= kRopeTile && n_q_heads % n_kv_heads == 0 && qkv_stride % 8 == 0) {
    dim3 g((num_tokens + kRopeTile - 1) / kRopeTile, n_kv_heads), b(256);
    if (dtype == 0)
      rope_cache_tile_kernel<__bf16><<<g, b, lds, stream>>>(
          qo, kc, vc, in, positions, slot_mapping, cos_sin, num_tokens, n_q_heads, n_kv_heads,
          head_dim, block_size, qkv_stride, q_out_stride);
    else
      rope_cache_tile_kernel<_Float16><<<g, b, lds, stream>>>(
          qo, kc, vc, in, positions, slot_mapping, cos_sin, num_tokens, n_q_heads, n_kv_heads,
          head_dim, block_size, qkv_stride, q_out_stride);
    return static_cast<int>(hipGetLastError());
  }
  dim3 grid(num_tokens), block(256);
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
