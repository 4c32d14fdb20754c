// Single-pass token sampler.
//
// The reference samples with SamplingParams(temperature=0.2) inside vLLM
// (llm/serve_llm.py:379, 520-525).  Here sampling is one workgroup per sequence that
// streams its logits row once:
//   greedy (temperature <= 0):  argmax(logit)
//   otherwise:                   argmax(logit / T + Gumbel(u)),  u = hash(seed, step, idx)
// The Gumbel-max trick draws exactly from softmax(logit / T) without materialising the
// probabilities or a prefix sum.  The RNG is counter based (splitmix64 of seed, step and
// vocabulary index) so a request with a fixed seed replays bit-identically, including
// under hipGraph replay (seed / step live in device buffers, not kernel arguments).
#include "common.h"
#include "kernels.h"

namespace atta {

constexpr int kSampleThreads = 512;

__device__ __forceinline__ float gumbel(uint64_t seed, uint64_t step, uint32_t idx) {
  const uint64_t h = mix64(seed ^ mix64(step * 0x100000001B3ull + idx));
  // 24 random mantissa bits -> u in (0, 1)
  const float u = (static_cast<float>(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
  return -__logf(-__logf(u));
}

__device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
}

template <typename LT>
__device__ __forceinline__ float load_logit(const LT* row, int i);
template <>
__device__ __forceinline__ float load_logit<float>(const float* row, int i) {
  return row[i];
}
template <>
__device__ __forceinline__ float load_logit<uint16_t>(const uint16_t* row, int i) {
  return to_f32<__bf16>(row[i]);
}

template <typename LT>
__global__ __launch_bounds__(kSampleThreads) void sample_kernel(
    int64_t* __restrict__ out, const LT* __restrict__ logits, int vocab, int64_t stride,
    const float* __restrict__ temperature, const int64_t* __restrict__ seeds,
    const int64_t* __restrict__ steps) {
  __shared__ float sv[kSampleThreads / kWave];
  __shared__ int si[kSampleThreads / kWave];
  const int row = blockIdx.x;
  const LT* lr = logits + static_cast<int64_t>(row) * stride;
  const float t = temperature[row];
  const bool greedy = !(t > 1e-5f);
  const float inv_t = greedy ? 1.f : 1.f / t;
  const uint64_t seed = static_cast<uint64_t>(seeds[row]);
  const uint64_t step = static_cast<uint64_t>(steps[row]);

  float bv = -__builtin_huge_valf();
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < vocab; i += kSampleThreads) {
    float v = load_logit<LT>(lr, i);
    if (!greedy) v = v * inv_t + gumbel(seed, step, static_cast<uint32_t>(i));
    better(bv, bi, v, i);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, kWave);
    const int oi = __shfl_xor(bi, o, kWave);
    better(bv, bi, ov, oi);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sv[wid] = bv;
    si[wid] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = sv[0];
    int i = si[0];
    for (int w = 1; w < kSampleThreads / kWave; ++w) better(v, i, sv[w], si[w]);
    out[row] = (i == 0x7fffffff) ? 0 : i;
  }
}

// ---- top-k / top-p (nucleus) sampling ------------------------------------------------------
// Same draw as above restricted to the kept set: argmax over {i : x_i >= thr} of x_i + G_i,
// x = logit / T.  The thresholds are exact order statistics found by 4-pass radix selects
// over order-preserving uint32 keys of x (8 bits a pass, 256-bin LDS histograms, one wave
// walks the bins from the top):
//   top-k: thr_k = the k-th largest x (weights 1, target k)
//   top-p: among x >= thr_k, thr_p = the largest value whose mass sum_{x_j >= thr_p} e^(x_j - m)
//          reaches p * Z - the token crossing p is kept (the sort + cumsum definition, ties at
//          the threshold kept together).  Masses are 32.32 fixed point summed in uint64 LDS
//          atomics: integer sums, so the threshold (and the token) is deterministic.
// top_k <= 0 or >= vocab: off; top_p >= 1: off.  Both off -> the same token as sample_kernel.
// One 1024-thread workgroup per row; the row (<= 1 MB) is re-read per pass from L2.
constexpr int kTkThreads = 1024;

__device__ __forceinline__ uint32_t ordered_key(float v) {
  const uint32_t b = __float_as_uint(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// Wave 0: largest bin b with above + sum_{b' >= b} h[b'] >= target; returns b and the new
// 'above' (= above + sum_{b' > b} h[b']) through LDS.
__device__ __forceinline__ void pick_bin(const unsigned long long* h, unsigned long long above,
                                         unsigned long long target, int* bin_out,
                                         unsigned long long* above_out) {
  const int lane = threadIdx.x;  // called by wave 0 only
  // lane l owns bins 255 - 4l .. 252 - 4l (descending)
  unsigned long long v[4], local = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = h[255 - 4 * lane - j];
    local += v[j];
  }
  // exclusive prefix over lanes (descending bin order)
  unsigned long long incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long t = __shfl_up(incl, o, kWave);
    if (lane >= o) incl += t;
  }
  const unsigned long long excl = incl - local;
  const bool hit = above + incl >= target;
  const unsigned long long mask = __ballot(hit);
  const int first = mask ? __builtin_ctzll(mask) : 63;  // none: the lowest bins (cannot happen
  if (lane == first) {                                   // with target <= total)
    unsigned long long acc = above + excl;
    int b = 252 - 4 * lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (acc + v[j] >= target) {
        b = 255 - 4 * lane - j;
        break;
      }
      acc += v[j];
    }
    *bin_out = b;
    *above_out = acc;
  }
}

template <typename LT>
__global__ __launch_bounds__(kTkThreads) void sample_topkp_kernel(
    int64_t* __restrict__ out, const LT* __restrict__ logits, int vocab, int64_t stride,
    const float* __restrict__ temperature, const float* __restrict__ top_p,
    const int* __restrict__ top_k, const int64_t* __restrict__ seeds,
    const int64_t* __restrict__ steps) {
  __shared__ unsigned long long hist[256];
  __shared__ float sv[kTkThreads / kWave];
  __shared__ int si[kTkThreads / kWave];
  __shared__ int sel_bin;
  __shared__ unsigned long long sel_above, tot;
  const int row = blockIdx.x;
  const LT* lr = logits + static_cast<int64_t>(row) * stride;
  const float t = temperature[row];
  const bool greedy = !(t > 1e-5f);
  const float inv_t = greedy ? 1.f : 1.f / t;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t lo_key = 0;  // keep keys >= lo_key

  if (!greedy) {
    const int k = top_k[row];
    const float p = top_p[row];
    const bool use_k = k > 0 && k < vocab;
    const bool use_p = p < 1.f;
    // row max of x (kept by any top-k)
    float mx = -__builtin_huge_valf();
    if (use_p) {
      for (int i = threadIdx.x; i < vocab; i += kTkThreads)
        mx = fmaxf(mx, load_logit<LT>(lr, i) * inv_t);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, kWave));
      if (lane == 0) sv[wid] = mx;
      __syncthreads();
      mx = sv[0];
#pragma unroll
      for (int w = 1; w < kTkThreads / kWave; ++w) mx = fmaxf(mx, sv[w]);
      __syncthreads();
    }
    for (int pass = 0; pass < 2; ++pass) {
      const bool mass = pass == 1;
      if (mass ? !use_p : !use_k) continue;
      unsigned long long target;
      if (mass) {
        // Z over the kept set (fixed point), target = ceil(p Z)
        if (threadIdx.x == 0) tot = 0;
        __syncthreads();
        unsigned long long z = 0;
        for (int i = threadIdx.x; i < vocab; i += kTkThreads) {
          const float x = load_logit<LT>(lr, i) * inv_t;
          if (ordered_key(x) >= lo_key)
            z += static_cast<unsigned long long>(expf(x - mx) * 4294967296.f);
        }
        atomicAdd(&tot, z);
        __syncthreads();
        target = static_cast<unsigned long long>(ceil(static_cast<double>(p) *
                                                      static_cast<double>(tot)));
        if (target == 0) target = 1;
      } else {
        target = static_cast<unsigned long long>(k);
      }
      uint32_t prefix = 0, pmask = 0;
      unsigned long long above = 0;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += kTkThreads) hist[b] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < vocab; i += kTkThreads) {
          const float x = load_logit<LT>(lr, i) * inv_t;
          const uint32_t key = ordered_key(x);
          if ((key & pmask) == prefix && key >= lo_key) {
            const unsigned long long w =
                mass ? static_cast<unsigned long long>(expf(x - mx) * 4294967296.f) : 1ull;
            if (w) atomicAdd(&hist[(key >> shift) & 255u], w);
          }
        }
        __syncthreads();
        if (wid == 0) pick_bin(hist, above, target, &sel_bin, &sel_above);
        __syncthreads();
        prefix |= static_cast<uint32_t>(sel_bin) << shift;
        pmask |= 255u << shift;
        above = sel_above;
        __syncthreads();
      }
      lo_key = prefix > lo_key ? prefix : lo_key;
    }
  }

  const uint64_t seed = static_cast<uint64_t>(seeds[row]);
  const uint64_t step = static_cast<uint64_t>(steps[row]);
  float bv = -__builtin_huge_valf();
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < vocab; i += kTkThreads) {
    float v = load_logit<LT>(lr, i);
    if (!greedy) {
      v = v * inv_t;
      if (ordered_key(v) < lo_key) continue;
      v += gumbel(seed, step, static_cast<uint32_t>(i));
    }
    better(bv, bi, v, i);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, kWave);
    const int oi = __shfl_xor(bi, o, kWave);
    better(bv, bi, ov, oi);
  }
  if (lane == 0) {
    sv[wid] = bv;
    si[wid] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = sv[0];
    int i = si[0];
    for (int w = 1; w < kTkThreads / kWave; ++w) better(v, i, sv[w], si[w]);
    out[row] = (i == 0x7fffffff) ? 0 : i;
  }
}

}  // namespace atta

using namespace atta;

int atta_sample_topkp(int64_t* out, const void* logits, int rows, int vocab, int64_t stride,
                      int logits_is_fp32, const float* temperature, const float* top_p,
                      const int* top_k, const int64_t* seeds, const int64_t* steps,
                      hipStream_t stream) {
  if (rows == 0) return 0;
  if (logits_is_fp32)
    sample_topkp_kernel<float><<<rows, kTkThreads, 0, stream>>>(
        out, static_cast<const float*>(logits), vocab, stride, temperature, top_p, top_k, seeds,
        steps);
  else
    sample_topkp_kernel<uint16_t><<<rows, kTkThreads, 0, stream>>>(
        out, static_cast<const uint16_t*>(logits), vocab, stride, temperature, top_p, top_k,
        seeds, steps);
  return static_cast<int>(hipGetLastError());
}

int atta_sample(int64_t* out, const void* logits, int rows, int vocab, int64_t stride,
                int logits_is_fp32, const float* temperature, const int64_t* seeds,
                const int64_t* steps, hipStream_t stream) {
  if (rows == 0) return 0;
  if (logits_is_fp32)
    sample_kernel<float><<<rows, kSampleThreads, 0, stream>>>(
        out, static_cast<const float*>(logits), vocab, stride, temperature, seeds, steps);
  else
    sample_kernel<uint16_t><<<rows, kSampleThreads, 0, stream>>>(
        out, static_cast<const uint16_t*>(logits), vocab, stride, temperature, seeds, steps);
  return static_cast<int>(hipGetLastError());
}
