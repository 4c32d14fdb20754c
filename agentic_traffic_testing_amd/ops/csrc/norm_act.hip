// Normalisation and activation kernels.
//
//  * rms_norm            out = x * rsqrt(mean(x^2) + eps) * w
//  * fused_add_rms_norm  r = x + r (written back, rounded to T);  out = rmsnorm(r) * w
//  * silu_and_mul        out[:, i] = silu(x[:, i]) * x[:, I + i]   (gate | up packed)
//
// These replace the per-layer norm/activation work that vLLM runs for the reference
// (llm/serve_llm.py:527-531 -> engine.generate).  RMSNorm: one wave per row for hidden <= 8192
// (shuffle-only reduction), one 256-thread workgroup per row above that; 16-byte vector loads.
#include "common.h"
#include "kernels.h"

namespace atta {

constexpr int kNormThreads = 256;
constexpr int kNormMaxIters = 8;  // rows up to 256 * 8 * 8 = 16384 elements

template <typename T, bool kAdd>
__global__ __launch_bounds__(kNormThreads) void rms_norm_kernel(
    uint16_t* __restrict__ out, uint16_t* __restrict__ residual, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ w, int hidden, int64_t x_stride, int64_t out_stride,
    int64_t res_stride, float eps) {
  __shared__ float scratch[kNormThreads / kWave];
  const int64_t row = blockIdx.x;
  const int nvec = hidden >> 3;
  const Pack8* xin = reinterpret_cast<const Pack8*>(x + row * x_stride);
  Pack8* rrow = kAdd ? reinterpret_cast<Pack8*>(residual + row * res_stride) : nullptr;

  float vals[kNormMaxIters][8];
  float ss = 0.f;
#pragma unroll
  for (int it = 0; it < kNormMaxIters; ++it) {
    const int v = threadIdx.x + it * kNormThreads;
    if (v < nvec) {
      Pack8 a = xin[v];
      if constexpr (kAdd) {
        Pack8 r = rrow[v];
        Pack8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s.v[j] = from_f32<T>(to_f32<T>(a.v[j]) + to_f32<T>(r.v[j]));
          vals[it][j] = to_f32<T>(s.v[j]);
        }
        rrow[v] = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[it][j] = to_f32<T>(a.v[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += vals[it][j] * vals[it][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / static_cast<float>(hidden) + eps);
  const Pack8* wv = reinterpret_cast<const Pack8*>(w);
  Pack8* o = reinterpret_cast<Pack8*>(out + row * out_stride);
#pragma unroll
  for (int it = 0; it < kNormMaxIters; ++it) {
    const int v = threadIdx.x + it * kNormThreads;
    if (v < nvec) {
      Pack8 ww = wv[v];
      Pack8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // round the normalised value to T before the weight multiply (matches the
        // fp32-reference definition in ops/reference.py)
        const float n = to_f32<T>(from_f32<T>(vals[it][j] * inv));
        r.v[j] = from_f32<T>(n * to_f32<T>(ww.v[j]));
      }
      o[v] = r;
    }
  }
}

// Row-per-wave variant for hidden <= 8192 (every Llama geometry here): 4 rows per 256-thread
// workgroup, the row sum of squares is a wave shuffle (no LDS, no barrier), and the norm
// weight is loaded together with x (one memory round trip instead of two) - the prefill norm
// at 2.6k rows x 4096 ran at 2.6 TB/s as one 256-thread workgroup per row.  Same per-element
// arithmetic as rms_norm_kernel (only the fp32 summation order of the row sum differs).
// WPR > 1 (few rows: the burst / planning prefills, 73-382 rows) spreads a row over WPR waves
// so the launch has 4x the waves in flight; the partial sums of squares meet in LDS behind one
// barrier.  At 382 x 4096 the one-wave-per-row form ran 10.5 us (1.2 TB/s: 96 workgroups).
constexpr int kRowsPerWg = 4;
constexpr int kNormSmallRows = 1024;  // below: 4 waves per row
template <typename T, bool kAdd, int ITERS, int WPR = 1>
__global__ __launch_bounds__(256) void rms_norm_wave_kernel(
    uint16_t* __restrict__ out, uint16_t* __restrict__ residual, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ w, int rows, int hidden, int64_t x_stride, int64_t out_stride,
    int64_t res_stride, float eps) {
  constexpr int kRows = 4 / WPR;  // rows per 256-thread workgroup
  const int lane = threadIdx.x & (64 * WPR - 1);
  const int64_t row = static_cast<int64_t>(blockIdx.x) * kRows + threadIdx.x / (64 * WPR);
  if (WPR == 1 && row >= rows) return;  // wave-uniform; no block-level barrier below
  const bool live = row < rows;         // WPR > 1: every wave reaches the barrier
  const int nvec = live ? hidden >> 3 : 0;
  const Pack8* xin = reinterpret_cast<const Pack8*>(x + row * x_stride);
  Pack8* rrow = kAdd ? reinterpret_cast<Pack8*>(residual + row * res_stride) : nullptr;
  const Pack8* wv = reinterpret_cast<const Pack8*>(w);
  Pack8 xa[ITERS], wa[ITERS], ra[ITERS];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int v = lane + it * 64 * WPR;
    if (v < nvec) {
      xa[it] = xin[v];
      wa[it] = wv[v];
      if constexpr (kAdd) ra[it] = rrow[v];
    }
  }
  float vals[ITERS][8];
  float ss = 0.f;
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int v = lane + it * 64 * WPR;
    if (v < nvec) {
      if constexpr (kAdd) {
        Pack8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s.v[j] = from_f32<T>(to_f32<T>(xa[it].v[j]) + to_f32<T>(ra[it].v[j]));
          vals[it][j] = to_f32<T>(s.v[j]);
        }
        rrow[v] = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[it][j] = to_f32<T>(xa[it].v[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += vals[it][j] * vals[it][j];
    }
  }
  ss = wave_sum(ss);
  if constexpr (WPR > 1) {
    __shared__ float part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = ss;
    __syncthreads();
    const int w0 = (threadIdx.x >> 6) & ~(WPR - 1);
    ss = 0.f;
#pragma unroll
    for (int i = 0; i < WPR; ++i) ss += part[w0 + i];  // same order in every wave of the row
    if (!live) return;
  }
  const float inv = rsqrtf(ss / static_cast<float>(hidden) + eps);
  Pack8* o = reinterpret_cast<Pack8*>(out + row * out_stride);
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int v = lane + it * 64 * WPR;
    if (v < nvec) {
      Pack8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float n = to_f32<T>(from_f32<T>(vals[it][j] * inv));
        r.v[j] = from_f32<T>(n * to_f32<T>(wa[it].v[j]));
      }
      o[v] = r;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void silu_and_mul_kernel(uint16_t* __restrict__ out,
                                                           const uint16_t* __restrict__ x,
                                                           int inter, int64_t x_stride,
                                                           int64_t out_stride) {
  const int64_t row = blockIdx.y;
  const int nvec = inter >> 3;
  const Pack8* g = reinterpret_cast<const Pack8*>(x + row * x_stride);
  const Pack8* u = reinterpret_cast<const Pack8*>(x + row * x_stride + inter);
  Pack8* o = reinterpret_cast<Pack8*>(out + row * out_stride);
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += gridDim.x * blockDim.x) {
    Pack8 a = g[v], b = u[v], r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = to_f32<T>(a.v[j]);
      const float s = to_f32<T>(from_f32<T>(gf / (1.f + __expf(-gf))));
      r.v[j] = from_f32<T>(s * to_f32<T>(b.v[j]));
    }
    o[v] = r;
  }
}

// Token-embedding gather.  One workgroup per row, 16-byte copies.  Row r
// takes token ids[r], or prev[r] when *feed_prev != 0: an async-decode look-ahead step is
// enqueued before the host has read the previous step's samples, so it reads its input
// tokens straight from the sampler's device output (engine/llm_engine.py).
__global__ __launch_bounds__(256) void embed_kernel(uint16_t* __restrict__ out,
                                                    const uint16_t* __restrict__ table,
                                                    const int* __restrict__ ids,
                                                    const int64_t* __restrict__ prev,
                                                    const int* __restrict__ feed_prev, int hidden,
                                                    int64_t vocab, int64_t out_stride) {
  const int64_t row = blockIdx.x;
  int64_t tok = (feed_prev != nullptr && feed_prev[0] != 0) ? prev[row] : ids[row];
  tok = tok < 0 ? 0 : (tok >= vocab ? vocab - 1 : tok);
  const Pack8* src = reinterpret_cast<const Pack8*>(table + tok * hidden);
  Pack8* dst = reinterpret_cast<Pack8*>(out + row * out_stride);
  for (int v = threadIdx.x; v < (hidden >> 3); v += blockDim.x) dst[v] = src[v];
}

// HBM read-bandwidth probe (diagnostic: scripts/gpu/decode_sol.py): streams a buffer with
// 16-byte non-temporal loads, 8 in flight per lane, grid-stride - the load path of the
// decode GEMVs' pre-shuffled weight stream without their math.  The words are folded into a
// value stored only under a runtime-false test, so the loads stay live and nothing is written.
__global__ __launch_bounds__(256) void stream_read_kernel(const u32x4* __restrict__ x,
                                                          int64_t n16,
                                                          unsigned* __restrict__ sink) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  unsigned acc = 0u;
  int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  for (; i < n16; i += stride) {
    const u32x4 v = __builtin_nontemporal_load(x + i);
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  // runtime-false (n16 >= 0) but opaque to the compiler: every lane's loads stay live
  if (acc == 0x9e3779b9u && n16 < 0) sink[blockIdx.x] = acc;
}

}  // namespace atta

using namespace atta;

int atta_stream_read(const void* x, int64_t bytes, unsigned* sink, int blocks,
                     hipStream_t stream) {
  if (bytes % 16 != 0 || blocks < 1) return -1;
  if (bytes == 0) return 0;
  stream_read_kernel<<<blocks, 256, 0, stream>>>(static_cast<const u32x4*>(x), bytes / 16, sink);
  return static_cast<int>(hipGetLastError());
}

int atta_embed(void* out, const void* table, const int* ids, const int64_t* prev,
               const int* feed_prev, int rows, int hidden, int64_t vocab, int64_t out_stride,
               hipStream_t stream) {
  if (hidden % 8 != 0 || out_stride % 8 != 0) return -1;
  if (rows == 0) return 0;
  embed_kernel<<<rows, 256, 0, stream>>>(static_cast<uint16_t*>(out),
                                         static_cast<const uint16_t*>(table), ids, prev,
                                         feed_prev, hidden, vocab, out_stride);
  return static_cast<int>(hipGetLastError());
}

int atta_rms_norm(void* out, void* residual, const void* x, const void* w, int rows, int hidden,
                  int64_t x_stride, int64_t out_stride, int64_t res_stride, float eps, int dtype,
                  hipStream_t stream) {
  if (hidden % 8 != 0 || hidden > kNormThreads * kNormMaxIters * 8) return -1;
  if (rows == 0) return 0;
  dim3 grid(rows), block(kNormThreads);
  auto o = static_cast<uint16_t*>(out);
  auto r = static_cast<uint16_t*>(residual);
  auto xi = static_cast<const uint16_t*>(x);
  auto wi = static_cast<const uint16_t*>(w);
  const int iters = (hidden / 8 + 63) / 64;
  if (iters <= 16 && rows < kNormSmallRows) {
    // few rows: 4 waves per row, one row per workgroup
    const dim3 g2(rows), b2(256);
#define ATTA_RMSW(T_, ADD_, IT_)                                                                   \
  rms_norm_wave_kernel<T_, ADD_, IT_, 4><<<g2, b2, 0, stream>>>(o, r, xi, wi, rows, hidden, x_stride, \
                                                                out_stride, res_stride, eps)
#define ATTA_RMSW_IT(T_, ADD_)                 \
  if (iters <= 4) ATTA_RMSW(T_, ADD_, 1);      \
  else if (iters <= 8) ATTA_RMSW(T_, ADD_, 2); \
  else ATTA_RMSW(T_, ADD_, 4)
    if (dtype == 0) {
      if (r) { ATTA_RMSW_IT(__bf16, true); } else { ATTA_RMSW_IT(__bf16, false); }
    } else {
      if (r) { ATTA_RMSW_IT(_Float16, true); } else { ATTA_RMSW_IT(_Float16, false); }
    }
#undef ATTA_RMSW_IT
#undef ATTA_RMSW
    return static_cast<int>(hipGetLastError());
  }
  if (iters <= 16) {
    const dim3 g2((rows + kRowsPerWg - 1) / kRowsPerWg), b2(64 * kRowsPerWg);
#define ATTA_RMSW(T_, ADD_, IT_)                                                                \
  rms_norm_wave_kernel<T_, ADD_, IT_><<<g2, b2, 0, stream>>>(o, r, xi, wi, rows, hidden, x_stride, \
                                                             out_stride, res_stride, eps)
#define ATTA_RMSW_IT(T_, ADD_)                 \
  if (iters <= 2) ATTA_RMSW(T_, ADD_, 2);      \
  else if (iters <= 4) ATTA_RMSW(T_, ADD_, 4); \
  else if (iters <= 8) ATTA_RMSW(T_, ADD_, 8); \
  else ATTA_RMSW(T_, ADD_, 16)
    if (dtype == 0) {
      if (r) { ATTA_RMSW_IT(__bf16, true); } else { ATTA_RMSW_IT(__bf16, false); }
    } else {
      if (r) { ATTA_RMSW_IT(_Float16, true); } else { ATTA_RMSW_IT(_Float16, false); }
    }
#undef ATTA_RMSW_IT
#undef ATTA_RMSW
    return static_cast<int>(hipGetLastError());
  }
  if (dtype == 0) {
    if (r)
      rms_norm_kernel<__bf16, true><<<grid, block, 0, stream>>>(o, r, xi, wi, hidden, x_stride,
                                                                out_stride, res_stride, eps);
    else
      rms_norm_kernel<__bf16, false><<<grid, block, 0, stream>>>(o, r, xi, wi, hidden, x_stride,
                                                                 out_stride, res_stride, eps);
  } else {
    if (r)
      rms_norm_kernel<_Float16, true><<<grid, block, 0, stream>>>(o, r, xi, wi, hidden, x_stride,
                                                                  out_stride, res_stride, eps);
    else
      rms_norm_kernel<_Float16, false><<<grid, block, 0, stream>>>(
          o, r, xi, wi, hidden, x_stride, out_stride, res_stride, eps);
  }
  return static_cast<int>(hipGetLastError());
}

int atta_silu_and_mul(void* out, const void* x, int rows, int inter, int64_t x_stride,
                      int64_t out_stride, int dtype, hipStream_t stream) {
  if (inter % 8 != 0) return -1;
  if (rows == 0) return 0;
  const int nvec = inter / 8;
  int bx = (nvec + 255) / 256;
  dim3 grid(bx, rows), block(256);
  if (dtype == 0)
    silu_and_mul_kernel<__bf16><<<grid, block, 0, stream>>>(
        static_cast<uint16_t*>(out), static_cast<const uint16_t*>(x), inter, x_stride, out_stride);
  else
    silu_and_mul_kernel<_Float16><<<grid, block, 0, stream>>>(
        static_cast<uint16_t*>(out), static_cast<const uint16_t*>(x), inter, x_stride, out_stride);
  return static_cast<int>(hipGetLastError());
}
