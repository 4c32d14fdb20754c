// Infinity-Cache (MALL) prefetch: stream a byte range through the memory hierarchy so that a
// later kernel finds it in the 256 MiB die-level cache instead of HBM.
//
// Use: from a side stream while a latency-bound kernel (decode attention) leaves HBM idle,
// warm the weights of the next weight-streaming kernel.  `blocks` x 256 threads, each lane
// keeps `inflight` 16-byte loads outstanding, so the pressure this puts on HBM queues (and
// on the latency of the kernel it runs beside) is set by blocks * inflight.
#include "common.h"
#include "kernels.h"

namespace atta {
namespace pf {

template <int INFLIGHT>
__global__ __launch_bounds__(256) void prefetch_kernel(const u32x4* __restrict__ p, int64_t n16,
                                                       int64_t per_block) {
  const int64_t beg = static_cast<int64_t>(blockIdx.x) * per_block;
  const int64_t end = beg + per_block < n16 ? beg + per_block : n16;
  for (int64_t i = beg + threadIdx.x; i < end; i += 256 * INFLIGHT) {
    u32x4 v[INFLIGHT];
#pragma unroll
    for (int u = 0; u < INFLIGHT; ++u) {
      const int64_t j = i + 256 * u;
      v[u] = j < end ? p[j] : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < INFLIGHT; ++u) asm volatile("" ::"v"(v[u]));  // keep the loads
  }
}

}  // namespace pf
}  // namespace atta

using namespace atta;

int atta_prefetch(const void* ptr, int64_t bytes, int blocks, int inflight, hipStream_t stream) {
  if (bytes <= 0) return 0;
  if (blocks < 1 || blocks > 4096 || (reinterpret_cast<uintptr_t>(ptr) & 15)) return -1;
  const int64_t n16 = bytes / 16;
  const int64_t per = (n16 + blocks - 1) / blocks;
  const u32x4* p = static_cast<const u32x4*>(ptr);
  switch (inflight) {
    case 1: pf::prefetch_kernel<1><<<blocks, 256, 0, stream>>>(p, n16, per); break;
    case 2: pf::prefetch_kernel<2><<<blocks, 256, 0, stream>>>(p, n16, per); break;
    case 4: pf::prefetch_kernel<4><<<blocks, 256, 0, stream>>>(p, n16, per); break;
    case 8: pf::prefetch_kernel<8><<<blocks, 256, 0, stream>>>(p, n16, per); break;
    default: return -1;
  }
  return static_cast<int>(hipGetLastError());
}
