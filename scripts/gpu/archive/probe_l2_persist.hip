// Probe: does data a kernel brought into the XCD L2s survive the kernel boundary into the next
// dependent launch on the same stream?  (If it does, a decode GEMV could warm the NEXT GEMV's
// first weight stages into L2 during its own tail and take the ~2 us ramp of every launch off
// the critical path; r3_probe_mall.txt only tested whole-matrix warming through the MALL.)
//
// rd(buf): grid of G workgroups, workgroup b reads its contiguous 1/G slice (dispatch puts
// workgroup b on XCD b % 8 in every launch, so the same slices meet the same L2).  Timed: the
// second of two back-to-back launches, rd(A) after rd(A) (warm) vs rd(A) after rd(B) (cold),
// for total sizes from 4 to 64 MB (the 8 L2s hold 32 MB), default and nt loads.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_l2 scripts/gpu/probe_l2_persist.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) rd(const u32x4* __restrict__ p, int per_wg, u32x4* sink) {
  const u32x4* base = p + static_cast<size_t>(blockIdx.x) * per_wg;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int i = threadIdx.x; i < per_wg; i += 256) {
    const u32x4 v = NT ? __builtin_nontemporal_load(base + i) : base[i];
    acc ^= v;
  }
  if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) sink[blockIdx.x] = acc;  // keeps the loads
}

int main() {
  const int G = 1024;
  const size_t max_bytes = 64ull << 20;
  u32x4 *a, *b, *sink;
  CK(hipMalloc(&a, max_bytes));
  CK(hipMalloc(&b, max_bytes));
  CK(hipMalloc(&sink, G * sizeof(u32x4)));
  CK(hipMemset(a, 1, max_bytes));
  CK(hipMemset(b, 2, max_bytes));
  // flush buffer larger than MALL (256 MB)
  void* fl;
  const size_t fl_bytes = 512ull << 20;
  CK(hipMalloc(&fl, fl_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("# us for the 2nd of two back-to-back rd launches (median of 15), grid %d x 256\n", G);
  std::printf("%8s %4s | %9s %9s | %9s\n", "MB", "nt", "warm", "cold", "cold-warm");
  for (int mb : {4, 8, 16, 24, 32, 64}) {
    const int per_wg = static_cast<int>((static_cast<size_t>(mb) << 20) / 16 / G);
    for (int nt = 0; nt < 2; ++nt) {
      float med[2];
      for (int cold = 0; cold < 2; ++cold) {
        std::vector<float> ts;
        for (int r = 0; r < 15; ++r) {
          CK(hipMemsetAsync(fl, r, fl_bytes));  // evict L2 / MALL
          const u32x4* first = cold ? b : a;
          if (nt) rd<true><<<G, 256>>>(first, per_wg, sink);
          else rd<false><<<G, 256>>>(first, per_wg, sink);
          CK(hipEventRecord(e0));
          if (nt) rd<true><<<G, 256>>>(a, per_wg, sink);
          else rd<false><<<G, 256>>>(a, per_wg, sink);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0.f;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ts.push_back(ms * 1e3f);
        }
        std::sort(ts.begin(), ts.end());
        med[cold] = ts[ts.size() / 2];
      }
      std::printf("%8d %4d | %9.2f %9.2f | %9.2f\n", mb, nt, med[0], med[1], med[1] - med[0]);
    }
  }
  return 0;
}
