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

}  // namespace atta

using namespace atta;

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
