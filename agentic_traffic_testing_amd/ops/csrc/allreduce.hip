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

template <typename T, int W>
__global__ void __launch_bounds__(kThreads) oneshot_kernel(Params p, const uint16_t* x,
                                                           uint16_t* y, int64_t n) {
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

template <typename T>
static int launch(const Params& p, const void* x, void* y, int64_t n, int blocks,
                  hipStream_t st) {
  const uint16_t* xi = static_cast<const uint16_t*>(x);
  uint16_t* yo = static_cast<uint16_t*>(y);
  switch (p.world) {
    case 2: oneshot_kernel<T, 2><<<blocks, kThreads, 0, st>>>(p, xi, yo, n); break;
    case 4: oneshot_kernel<T, 4><<<blocks, kThreads, 0, st>>>(p, xi, yo, n); break;
    case 8: oneshot_kernel<T, 8><<<blocks, kThreads, 0, st>>>(p, xi, yo, n); break;
    default: return -1;
  }
  return static_cast<int>(hipGetLastError());
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
                int64_t n, int dtype, hipStream_t stream) {
  if (world != 2 && world != 4 && world != 8) return -1;
  if (rank < 0 || rank >= world || n <= 0 || n > max_elems) return -1;
  ar::Params p{};
  for (int i = 0; i < world; ++i) p.base[i] = static_cast<uint8_t*>(bases[i]);
  p.rank = rank;
  p.world = world;
  p.max_elems = max_elems;
  // fixed grid (see the generation argument above); blocks past the data only signal
  return dtype == 0 ? ar::launch<__bf16>(p, x, y, n, ar::kMaxBlocks, stream)
                    : ar::launch<_Float16>(p, x, y, n, ar::kMaxBlocks, stream);
}
