// One-shot intra-node all-reduce over IPC-mapped peer buffers.
//
// Decode-time TP all-reduces are tiny ([B, hidden] bf16: 8 KiB - 256 KiB) and latency-bound;
// a ring all-reduce pays 2(N-1) dependent hops.  Here every rank PUSHES its slice of the
// input straight into every peer's receive buffer over the point-to-point xGMI links (one hop,
// all 7 links busy at once), raises one flag per (peer, block), waits for the peers' flags in
// its own memory and sums the N copies locally.
//
// Buffer of one rank (hipExtMallocWithFlags(hipDeviceMallocUncached): peer stores land in
// memory and local loads bypass the non-coherent caches):
//   [flags   : 2 parities x kMaxRanks x kMaxBlocks uint32] written by peers
//   [counters: kMaxBlocks uint32 + 1 error word]             this rank's per-block generation
//   [data    : 2 parities x kMaxRanks x max_elems T]        slot (parity, src rank)
// Every launch uses the same fixed grid, so the per-block generation counters advance in
// lockstep and form one global generation g per call; call g uses parity g & 1 for ALL of its
// data (slices may differ between calls of different sizes).  Reusing a parity at g + 2 is
// safe without an end barrier: a rank starts call g + 2 only after its call g + 1 saw every
// peer's flags, and a peer raises call g + 1 flags only after its call g kernel - all of its
// reads of generation g - completed (stream order).
// The sum runs in rank order in fp32, so every rank produces bit-identical output.
// Graph-capturable: all state lives on the device, kernel arguments never change.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"
#include "kernels.h"

namespace atta {
namespace ar {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 32;
constexpr int kThreads = 512;
constexpr size_t kFlagBytes = 2 * kMaxRanks * kMaxBlocks * sizeof(uint32_t);
constexpr size_t kHeaderBytes = 64 * 1024;  // flags + counters, padded

struct Params {
  uint8_t* base[kMaxRanks];  // every rank's buffer base, mapped into this process
  int rank, world;
  int64_t max_elems;
};

__device__ __forceinline__ uint32_t* flag_ptr(uint8_t* base, int par, int src, int blk) {
  return reinterpret_cast<uint32_t*>(base) + (par * kMaxRanks + src) * kMaxBlocks + blk;
}

// 16-bit element storage; T (__bf16 / _Float16) selects the conversion only
__device__ __forceinline__ uint16_t* slot_ptr(uint8_t* base, int par, int src,
                                              int64_t max_elems) {
  return reinterpret_cast<uint16_t*>(base + kHeaderBytes) + (par * kMaxRanks + src) * max_elems;
}

// res != nullptr: y = bf16(bf16(sum) + res) - the row-parallel projection's residual-stream
// update fused into the reduction (the same two roundings as residual.add_(all_reduce(x)),
// without the extra launch and HBM pass); y may alias res.
template <typename T, int W>
__global__ void __launch_bounds__(kThreads) oneshot_kernel(Params p, const uint16_t* x,
                                                           uint16_t* y, const uint16_t* res,
                                                           int64_t n) {
  const int b = blockIdx.x;
  const int nb = gridDim.x;
  uint8_t* mine = p.base[p.rank];
  uint32_t* counters = reinterpret_cast<uint32_t*>(mine + kFlagBytes);
  __shared__ uint32_t gen_s;
  if (threadIdx.x == 0) gen_s = counters[b] + 1;
  __syncthreads();
  const uint32_t gen = gen_s;
  const int par = gen & 1;

  int64_t per = (n + nb - 1) / nb;
  per = (per + 7) & ~int64_t(7);
  const int64_t beg = b * per < n ? b * per : n;
  const int64_t end = beg + per < n ? beg + per : n;

  // 1) push my slice into slot (par, rank) of every rank's buffer (16-byte stores)
  using V = Pack8;
  for (int q = 0; q < W; ++q) {
    uint16_t* dst = slot_ptr(p.base[q], par, p.rank, p.max_elems);
    for (int64_t i = beg + 8 * threadIdx.x; i < end; i += 8 * kThreads) {
      if (i + 8 <= end) {
        *reinterpret_cast<V*>(dst + i) = *reinterpret_cast<const V*>(x + i);
      } else {
        for (int64_t j = i; j < end; ++j) dst[j] = x[j];
      }
    }
  }
  __threadfence_system();
  __syncthreads();
  // 2) one flag per (destination rank, block); 3) wait for every source's flag here
  if (threadIdx.x < W) {
    __hip_atomic_store(flag_ptr(p.base[threadIdx.x], par, p.rank, b), gen, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* f = flag_ptr(mine, par, threadIdx.x, b);
    // bounded wait (~2-4 s): a dead peer must not hang the GPU; the block then records the
    // failure in the error word and finishes (the result is garbage, the host checks it)
    uint32_t spins = 0;
    while (static_cast<int32_t>(__hip_atomic_load(f, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM) - gen) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 25)) {
        atomicOr(counters + kMaxBlocks, 1u << threadIdx.x);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope, once after the poll
  }
  __syncthreads();
  // 4) reduce the W slots in rank order (fp32) into y
  for (int64_t i = beg + 8 * threadIdx.x; i < end; i += 8 * kThreads) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const int cnt = i + 8 <= end ? 8 : static_cast<int>(end - i);
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint16_t* src = slot_ptr(mine, par, q, p.max_elems) + i;
      if (cnt == 8) {
        const V v = *reinterpret_cast<const V*>(src);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += to_f32<T>(v.v[j]);
      } else {
        for (int j = 0; j < cnt; ++j) acc[j] += to_f32<T>(src[j]);
      }
    }
    if (res != nullptr) {
      if (cnt == 8) {
        const V r = *reinterpret_cast<const V*>(res + i);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = to_f32<T>(from_f32<T>(acc[j])) + to_f32<T>(r.v[j]);
      } else {
        for (int j = 0; j < cnt; ++j) acc[j] = to_f32<T>(from_f32<T>(acc[j])) + to_f32<T>(res[i + j]);
      }
    }
    if (cnt == 8) {
      V o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.v[j] = from_f32<T>(acc[j]);
      *reinterpret_cast<V*>(y + i) = o;
    } else {
      for (int j = 0; j < cnt; ++j) y[i + j] = from_f32<T>(acc[j]);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) counters[b] = gen;
}

// ---- two-shot (reduce-scatter + all-gather) for prefill-sized messages ------------------
// Per rank, per call: (W-1)/W of the message leaves over xGMI twice instead of (W-1) whole
// copies (one-shot), so the link time stays flat in W - the bandwidth-optimal shape of a ring
// with 2 hops instead of 2(W-1).  Buffer of one rank (separate allocation, same uncached
// memory and generation scheme as the one-shot kernel):
//   [flags1 : 2 parities x kMaxRanks x k2Blocks]  phase-1 "my copy of your chunk landed"
//   [flags2 : 2 parities x kMaxRanks x k2Blocks]  phase-2 "my reduced chunk landed"
//   [counters: k2Blocks + 1 error word]
//   [slot1 : 2 parities x W x chunk_max]   peers' copies of MY chunk
//   [slot2 : 2 parities x W x chunk_max]   every rank's reduced chunk
// Block b owns sub-range b of every chunk; chunk c = ranks' elements [c*chunk, (c+1)*chunk).
// Reuse of parity g & 1 at call g + 2 is safe for the argument of the one-shot kernel: a
// rank enters call g + 2 only after its call g + 1 saw every peer's phase-1 flags, which
// peers raise only after their call g finished (stream order).
constexpr int k2Blocks = 64;
constexpr size_t k2FlagWords = 2 * kMaxRanks * k2Blocks;
constexpr size_t k2HeaderBytes = 64 * 1024;

struct Params2 {
  uint8_t* base[kMaxRanks];
  int rank, world;
  int64_t chunk_max;  // elements per (parity, src) slot
};

__device__ __forceinline__ uint32_t* flag2_ptr(uint8_t* base, int phase, int par, int src,
                                               int blk) {
  return reinterpret_cast<uint32_t*>(base) + phase * k2FlagWords +
         (par * kMaxRanks + src) * k2Blocks + blk;
}
template <int W>
__device__ __forceinline__ uint16_t* slot2_ptr(uint8_t* base, int region, int par, int src,
                                               int64_t chunk_max) {
  return reinterpret_cast<uint16_t*>(base + k2HeaderBytes) +
         ((region * 2 + par) * W + src) * chunk_max;
}

template <int W>
__device__ __forceinline__ void raise_and_wait(uint8_t* const* bases, uint8_t* mine, int phase,
                                               int par, int me, int b, uint32_t gen,
                                               uint32_t* errw) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < W) {
    __hip_atomic_store(flag2_ptr(bases[threadIdx.x], phase, par, me, b), gen, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* f = flag2_ptr(mine, phase, par, threadIdx.x, b);
    uint32_t spins = 0;  // bounded: a dead peer records itself in the error word
    while (static_cast<int32_t>(__hip_atomic_load(f, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM) - gen) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 25)) {
        atomicOr(errw, 1u << threadIdx.x);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

template <typename T, int W>
__global__ void __launch_bounds__(kThreads) twoshot_kernel(Params2 p, const uint16_t* x,
                                                           uint16_t* y, const uint16_t* res,
                                                           int64_t n) {
  using V = Pack8;
  const int b = blockIdx.x;
  const int me = p.rank;
  uint8_t* mine = p.base[me];
  uint32_t* counters = reinterpret_cast<uint32_t*>(mine) + 2 * k2FlagWords;
  __shared__ uint32_t gen_s;
  if (threadIdx.x == 0) gen_s = counters[b] + 1;
  __syncthreads();
  const uint32_t gen = gen_s;
  const int par = gen & 1;

  int64_t chunk = (n + W - 1) / W;
  chunk = (chunk + 7) & ~int64_t(7);
  int64_t sub = (chunk + k2Blocks - 1) / k2Blocks;
  sub = (sub + 7) & ~int64_t(7);
  const int64_t off = b * sub < chunk ? b * sub : chunk;   // within a chunk
  const int64_t len = off + sub < chunk ? sub : chunk - off;
  // elements [lo, hi) of chunk c that exist in the message
  auto span = [&](int c, int64_t& lo, int64_t& hi) {
    lo = c * chunk + off;
    hi = lo + len;
    if (hi > n) hi = n;
    if (lo > hi) lo = hi;
  };

  // 1) scatter: my copy of chunk q (sub-range b) -> rank q's slot1(par, me)
#pragma unroll
  for (int q = 0; q < W; ++q) {
    int64_t lo, hi;
    span(q, lo, hi);
    uint16_t* dst = slot2_ptr<W>(p.base[q], 0, par, me, p.chunk_max) + off - lo;
    for (int64_t i = lo + 8 * threadIdx.x; i < hi; i += 8 * kThreads) {
      if (i + 8 <= hi)
        *reinterpret_cast<V*>(dst + i) = *reinterpret_cast<const V*>(x + i);
      else
        for (int64_t j = i; j < hi; ++j) dst[j] = x[j];
    }
  }
  raise_and_wait<W>(p.base, mine, 0, par, me, b, gen, counters + k2Blocks);

  // 2) reduce my chunk in rank order (fp32) and push the result to every rank's slot2
  {
    int64_t lo, hi;
    span(me, lo, hi);
    for (int64_t i = lo + 8 * threadIdx.x; i < hi; i += 8 * kThreads) {
      const int cnt = i + 8 <= hi ? 8 : static_cast<int>(hi - i);
      const int64_t o = off + (i - lo);  // element index inside a slot
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const uint16_t* src = slot2_ptr<W>(mine, 0, par, q, p.chunk_max) + o;
        if (cnt == 8) {
          const V v = *reinterpret_cast<const V*>(src);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += to_f32<T>(v.v[j]);
        } else {
          for (int j = 0; j < cnt; ++j) acc[j] += to_f32<T>(src[j]);
        }
      }
      V r;
#pragma unroll
      for (int j = 0; j < 8; ++j) r.v[j] = from_f32<T>(acc[j]);
#pragma unroll
      for (int q = 0; q < W; ++q) {
        uint16_t* dst = slot2_ptr<W>(p.base[q], 1, par, me, p.chunk_max) + o;
        if (cnt == 8)
          *reinterpret_cast<V*>(dst) = r;
        else
          for (int j = 0; j < cnt; ++j) dst[j] = r.v[j];
      }
    }
  }
  raise_and_wait<W>(p.base, mine, 1, par, me, b, gen, counters + k2Blocks);

  // 3) gather every rank's reduced chunk (sub-range b) into y
#pragma unroll
  for (int q = 0; q < W; ++q) {
    int64_t lo, hi;
    span(q, lo, hi);
    const uint16_t* src = slot2_ptr<W>(mine, 1, par, q, p.chunk_max) + off - lo;
    for (int64_t i = lo + 8 * threadIdx.x; i < hi; i += 8 * kThreads) {
      if (res != nullptr) {  // residual-stream update fused (see oneshot_kernel)
        const int cnt = i + 8 <= hi ? 8 : static_cast<int>(hi - i);
        for (int j = 0; j < cnt; ++j)
          y[i + j] = from_f32<T>(to_f32<T>(src[i + j]) + to_f32<T>(res[i + j]));
      } else if (i + 8 <= hi) {
        *reinterpret_cast<V*>(y + i) = *reinterpret_cast<const V*>(src + i);
      } else {
        for (int64_t j = i; j < hi; ++j) y[j] = src[j];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) counters[b] = gen;
}

template <typename T>
static int launch2(const Params2& p, const void* x, void* y, const void* res, int64_t n,
                   hipStream_t st) {
  const uint16_t* xi = static_cast<const uint16_t*>(x);
  uint16_t* yo = static_cast<uint16_t*>(y);
  const uint16_t* ri = static_cast<const uint16_t*>(res);
  switch (p.world) {
    case 2: twoshot_kernel<T, 2><<<k2Blocks, kThreads, 0, st>>>(p, xi, yo, ri, n); break;
    case 4: twoshot_kernel<T, 4><<<k2Blocks, kThreads, 0, st>>>(p, xi, yo, ri, n); break;
    case 8: twoshot_kernel<T, 8><<<k2Blocks, kThreads, 0, st>>>(p, xi, yo, ri, n); break;
    default: return -1;
  }
  return static_cast<int>(hipGetLastError());
}

template <typename T>
static int launch(const Params& p, const void* x, void* y, const void* res, int64_t n,
                  int blocks, hipStream_t st) {
  const uint16_t* xi = static_cast<const uint16_t*>(x);
  uint16_t* yo = static_cast<uint16_t*>(y);
  const uint16_t* ri = static_cast<const uint16_t*>(res);
  switch (p.world) {
    case 2: oneshot_kernel<T, 2><<<blocks, kThreads, 0, st>>>(p, xi, yo, ri, n); break;
    case 4: oneshot_kernel<T, 4><<<blocks, kThreads, 0, st>>>(p, xi, yo, ri, n); break;
    case 8: oneshot_kernel<T, 8><<<blocks, kThreads, 0, st>>>(p, xi, yo, ri, n); break;
    default: return -1;
  }
  return static_cast<int>(hipGetLastError());
}


// ---- X1 / X2 with the push fused into the row-parallel GEMV (ar_push_reduce) ------------
// The one-shot kernel above reads the GEMV's output back from HBM, pushes it to the peers,
// fences and flags - a launch of its own between the GEMV and the next layer step.  With the
// push fused, the row-parallel o / down GEMV (skinny.h, EPI_PLAIN with SkinnyParams::push_*)
// writes every finished 16-column tile straight into slot (parity, my rank) of every peer's
// buffer, fences, and bumps that peer's 64-bit per-source tile counter; what is left here is
// the receive side: wait until every source's counter covers this call's tiles, then the
// rank-order fp32 sum (+ the residual add) of the W slots.  Same buffers, same per-block
// generation counters and parity as the one-shot kernel (the GEMV reads the generation from
// counter 0), so both kernels can be mixed on one buffer; the tile counters are monotonic
// (64-bit, never reset) and each block keeps the cumulative count it expects in the header.
constexpr size_t kPushRegion = 48 * 1024;  // per-source tile counters + per-block expectations
static_assert(kPushRegion > 8192 + 256 + 2 * kMaxRanks * 256 * 8, "push region overlaps keys");
static_assert(kPushRegion + 1024 + kMaxBlocks * 8 <= kHeaderBytes, "push region");
static_assert(arl::kPushOffset == kPushRegion && arl::kSlotOffset == kHeaderBytes &&
                  arl::kGenOffset == kFlagBytes && arl::kMaxRanks == kMaxRanks,
              "common.h arl layout");

__device__ __forceinline__ unsigned long long* push_ctr(uint8_t* base, int src) {
  return reinterpret_cast<unsigned long long*>(base + kPushRegion + src * 64);
}
__device__ __forceinline__ unsigned long long* push_exp(uint8_t* base, int blk) {
  return reinterpret_cast<unsigned long long*>(base + kPushRegion + 1024) + blk;
}

template <typename T, int W>
__global__ void __launch_bounds__(kThreads) push_reduce_kernel(Params p, uint16_t* y,
                                                               const uint16_t* res, int64_t n,
                                                               int ntiles) {
  const int b = blockIdx.x;
  const int nb = gridDim.x;
  uint8_t* mine = p.base[p.rank];
  uint32_t* counters = reinterpret_cast<uint32_t*>(mine + kFlagBytes);
  __shared__ uint32_t gen_s;
  __shared__ unsigned long long exp_s;
  if (threadIdx.x == 0) {
    gen_s = counters[b] + 1;
    exp_s = *push_exp(mine, b) + static_cast<unsigned long long>(ntiles);
  }
  __syncthreads();
  const uint32_t gen = gen_s;
  const unsigned long long want = exp_s;
  const int par = gen & 1;
  if (threadIdx.x < W) {
    const unsigned long long* c = push_ctr(mine, threadIdx.x);
    uint32_t spins = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 25)) {  // bounded: a dead peer must not hang the GPU
        atomicOr(counters + kMaxBlocks, 1u << threadIdx.x);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope, once after the poll
  }
  __syncthreads();
  int64_t per = (n + nb - 1) / nb;
  per = (per + 7) & ~int64_t(7);
  const int64_t beg = b * per < n ? b * per : n;
  const int64_t end = beg + per < n ? beg + per : n;
  using V = Pack8;
  for (int64_t i = beg + 8 * threadIdx.x; i < end; i += 8 * kThreads) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    const int cnt = i + 8 <= end ? 8 : static_cast<int>(end - i);
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const uint16_t* src = slot_ptr(mine, par, q, p.max_elems) + i;
      if (cnt == 8) {
        const V v = *reinterpret_cast<const V*>(src);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += to_f32<T>(v.v[j]);
      } else {
        for (int j = 0; j < cnt; ++j) acc[j] += to_f32<T>(src[j]);
      }
    }
    if (res != nullptr) {
      for (int j = 0; j < cnt; ++j) acc[j] = to_f32<T>(from_f32<T>(acc[j])) + to_f32<T>(res[i + j]);
    }
    if (cnt == 8) {
      V o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.v[j] = from_f32<T>(acc[j]);
      *reinterpret_cast<V*>(y + i) = o;
    } else {
      for (int j = 0; j < cnt; ++j) y[i + j] = from_f32<T>(acc[j]);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    counters[b] = gen;
    *push_exp(mine, b) = want;
  }
}

// ---- X4: int64 MAX of the vocab-parallel sampler keys (one tiny block) ------------------
// Each rank's LM-head shard reduces a decode row to one signed-orderable packed
// (score, -token) key; the MAX over ranks is the global Gumbel-max winner.  Same push /
// flag / rank-order protocol as the one-shot kernel, on a region of its own inside the
// one-shot buffer's header (its own flags, generation counter and 2 x kMaxRanks x kMaxKeys
// slots), so its single-block generations never interleave with the 32-block sum kernel's.
// Writes the reduced keys in place and, when tokens != nullptr, the decoded token ids - the
// step then ends on the device with no torch ops after the collective (graph-capturable).
constexpr int kMaxKeys = 256;
constexpr size_t kKeyRegion = 8192;  // byte offset of the max-kernel region in the header
__device__ __forceinline__ uint32_t* kflag_ptr(uint8_t* base, int par, int src) {
  return reinterpret_cast<uint32_t*>(base + kKeyRegion) + par * kMaxRanks + src;
}
__device__ __forceinline__ long long* kslot_ptr(uint8_t* base, int par, int src) {
  return reinterpret_cast<long long*>(base + kKeyRegion + 256) + (par * kMaxRanks + src) * kMaxKeys;
}
static_assert(kKeyRegion + 256 + 2 * kMaxRanks * kMaxKeys * 8 <= kHeaderBytes, "key region");

template <int W>
__global__ void __launch_bounds__(kMaxKeys) keymax_kernel(Params p, long long* keys,
                                                          int64_t* tokens, int n) {
  uint8_t* mine = p.base[p.rank];
  uint32_t* counter = reinterpret_cast<uint32_t*>(mine + kKeyRegion) + 2 * kMaxRanks;
  uint32_t* errw = reinterpret_cast<uint32_t*>(mine + kFlagBytes) + kMaxBlocks;
  __shared__ uint32_t gen_s;
  if (threadIdx.x == 0) gen_s = *counter + 1;
  __syncthreads();
  const uint32_t gen = gen_s;
  const int par = gen & 1;
  const int i = threadIdx.x;
  long long k = 0;
  if (i < n) {
    k = keys[i];
#pragma unroll
    for (int q = 0; q < W; ++q) kslot_ptr(p.base[q], par, p.rank)[i] = k;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < W) {
    __hip_atomic_store(kflag_ptr(p.base[threadIdx.x], par, p.rank), gen, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* f = kflag_ptr(mine, par, threadIdx.x);
    uint32_t spins = 0;  // bounded (~2-4 s): a dead peer sets its bit in the error word
    while (static_cast<int32_t>(__hip_atomic_load(f, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM) - gen) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 25)) {
        atomicOr(errw, 1u << threadIdx.x);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  if (i < n) {
    long long best = kslot_ptr(mine, par, 0)[i];
#pragma unroll
    for (int q = 1; q < W; ++q) {
      const long long o = kslot_ptr(mine, par, q)[i];
      best = o > best ? o : best;
    }
    keys[i] = best;
    if (tokens != nullptr)
      tokens[i] = static_cast<int64_t>(0xFFFFFFFFu - static_cast<unsigned>(best & 0xFFFFFFFFll));
  }
  __syncthreads();
  if (threadIdx.x == 0) *counter = gen;
}

}  // namespace ar
}  // namespace atta

using namespace atta;

size_t atta_ar_buffer_bytes(int64_t max_elems, int elem_bytes) {
  return ar::kHeaderBytes + 2 * ar::kMaxRanks * static_cast<size_t>(max_elems) * elem_bytes;
}

int atta_ar_alloc(void** ptr, size_t bytes) {
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return static_cast<int>(e);
  return static_cast<int>(hipMemset(*ptr, 0, bytes));
}

int atta_ar_free(void* ptr) { return static_cast<int>(hipFree(ptr)); }

int atta_ar_ipc_handle(void* ptr, void* handle_out) {
  return static_cast<int>(hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(handle_out), ptr));
}

int atta_ar_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return static_cast<int>(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
}

int atta_ar_ipc_close(void* ptr) { return static_cast<int>(hipIpcCloseMemHandle(ptr)); }

int atta_ar_handle_bytes() { return static_cast<int>(sizeof(hipIpcMemHandle_t)); }

// Byte offset of the error word (bit q set: timed out waiting for rank q).
int64_t atta_ar_error_offset() {
  return static_cast<int64_t>(ar::kFlagBytes + ar::kMaxBlocks * sizeof(uint32_t));
}

int atta_ar_run(void* const* bases, int rank, int world, int64_t max_elems, const void* x, void* y,
                const void* res, int64_t n, int dtype, hipStream_t stream) {
  if (world != 2 && world != 4 && world != 8) return -1;
  if (rank < 0 || rank >= world || n <= 0 || n > max_elems) return -1;
  ar::Params p{};
  for (int i = 0; i < world; ++i) p.base[i] = static_cast<uint8_t*>(bases[i]);
  p.rank = rank;
  p.world = world;
  p.max_elems = max_elems;
  // fixed grid (see the generation argument above); blocks past the data only signal
  return dtype == 0 ? ar::launch<__bf16>(p, x, y, res, n, ar::kMaxBlocks, stream)
                    : ar::launch<_Float16>(p, x, y, res, n, ar::kMaxBlocks, stream);
}

int atta_ar_keymax(void* const* bases, int rank, int world, long long* keys, int64_t* tokens,
                   int n, hipStream_t stream) {
  if (world != 2 && world != 4 && world != 8) return -1;
  if (rank < 0 || rank >= world || n <= 0 || n > ar::kMaxKeys) return -1;
  ar::Params p{};
  for (int i = 0; i < world; ++i) p.base[i] = static_cast<uint8_t*>(bases[i]);
  p.rank = rank;
  p.world = world;
  switch (world) {
    case 2: ar::keymax_kernel<2><<<1, ar::kMaxKeys, 0, stream>>>(p, keys, tokens, n); break;
    case 4: ar::keymax_kernel<4><<<1, ar::kMaxKeys, 0, stream>>>(p, keys, tokens, n); break;
    default: ar::keymax_kernel<8><<<1, ar::kMaxKeys, 0, stream>>>(p, keys, tokens, n); break;
  }
  return static_cast<int>(hipGetLastError());
}

// ---- two-shot entry points --------------------------------------------------------------
static int64_t chunk_max_of(int64_t max_elems, int world) {
  int64_t c = (max_elems + world - 1) / world;
  c = (c + 7) & ~int64_t(7);
  // + one sub-range of slack: the last block's sub-range may run past the chunk end
  return c + ((c / ar::k2Blocks + 8) & ~int64_t(7));
}

size_t atta_ar2_buffer_bytes(int64_t max_elems, int world, int elem_bytes) {
  return ar::k2HeaderBytes +
         4 * static_cast<size_t>(world) * chunk_max_of(max_elems, world) * elem_bytes;
}

int64_t atta_ar2_error_offset() {
  return static_cast<int64_t>((2 * ar::k2FlagWords + ar::k2Blocks) * sizeof(uint32_t));
}

int atta_ar2_run(void* const* bases, int rank, int world, int64_t max_elems, const void* x,
                 void* y, const void* res, int64_t n, int dtype, hipStream_t stream) {
  if (world != 2 && world != 4 && world != 8) return -1;
  if (rank < 0 || rank >= world || n <= 0 || n > max_elems) return -1;
  ar::Params2 p{};
  for (int i = 0; i < world; ++i) p.base[i] = static_cast<uint8_t*>(bases[i]);
  p.rank = rank;
  p.world = world;
  p.chunk_max = chunk_max_of(max_elems, world);
  return dtype == 0 ? ar::launch2<__bf16>(p, x, y, res, n, stream)
                    : ar::launch2<_Float16>(p, x, y, res, n, stream);
}

// Receive side of the GEMV-fused push (see push_reduce_kernel): y = sum over ranks of the
// pushed slots (+ res), n elements; ntiles = tiles each source's GEMV pushed for this call.
int atta_ar_push_reduce(void* const* bases, int rank, int world, int64_t max_elems, void* y,
                        const void* res, int64_t n, int ntiles, int dtype, hipStream_t stream) {
  if (world != 2 && world != 4 && world != 8) return -1;
  if (rank < 0 || rank >= world || n <= 0 || n > max_elems || ntiles <= 0) return -1;
  ar::Params p{};
  for (int i = 0; i < world; ++i) p.base[i] = static_cast<uint8_t*>(bases[i]);
  p.rank = rank;
  p.world = world;
  p.max_elems = max_elems;
  uint16_t* yo = static_cast<uint16_t*>(y);
  const uint16_t* ri = static_cast<const uint16_t*>(res);
#define ATTA_PR(T_)                                                                            \
  switch (world) {                                                                             \
    case 2: ar::push_reduce_kernel<T_, 2><<<ar::kMaxBlocks, ar::kThreads, 0, stream>>>(p, yo, ri, n, ntiles); break; \
    case 4: ar::push_reduce_kernel<T_, 4><<<ar::kMaxBlocks, ar::kThreads, 0, stream>>>(p, yo, ri, n, ntiles); break; \
    default: ar::push_reduce_kernel<T_, 8><<<ar::kMaxBlocks, ar::kThreads, 0, stream>>>(p, yo, ri, n, ntiles); break; \
  }
  if (dtype == 0) {
    ATTA_PR(__bf16)
  } else {
    ATTA_PR(_Float16)
  }
#undef ATTA_PR
  return static_cast<int>(hipGetLastError());
}

// Layout constants the GEMV's push epilogue needs (skinny.h): byte offsets of the generation
// counter 0, of the slots and of the per-source tile counters inside a rank's buffer.
int64_t atta_ar_push_layout(int what) {
  switch (what) {
    case 0: return static_cast<int64_t>(ar::kFlagBytes);   // uint32 generation counter 0
    case 1: return static_cast<int64_t>(ar::kHeaderBytes); // slot (par, src) base
    case 2: return static_cast<int64_t>(ar::kPushRegion);  // uint64 counter of source q at +64 q
    case 3: return ar::kMaxRanks;
    default: return -1;
  }
}
