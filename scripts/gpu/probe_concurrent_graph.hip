// Probe: do two kernels on parallel branches of a captured hipGraph run CONCURRENTLY on
// MI355X, so a consumer kernel launched beside its producer can wait on a device flag
// instead of a launch boundary?  (Decode "early launch": a GEMV that streams its weights
// while the previous kernel is still running.)
//
// producer<<<P, 256>>>: every workgroup works ~T us, then adds 1 to a counter (agent scope).
// consumer<<<C, 512>>>: thread 0 of every workgroup polls the counter until it reaches P
// (bounded: 2 ms, then it gives up and records a timeout) and stamps when it saw it.
// Both orders of capture (consumer branch first / producer branch first), graph replays and
// eager two-stream launches; prints timeouts and the flag-seen -> last-producer-arrival gap.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/pcg scripts/gpu/probe_concurrent_graph.hip
//   timeout -k 10 60 /tmp/pcg
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void producer(int* ctr, unsigned long long* t_arrive, int work_ticks,
                         unsigned long long* t_start) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    t_start[blockIdx.x] = t0;
    while (wall_clock64() - t0 < static_cast<unsigned long long>(work_ticks)) __builtin_amdgcn_s_sleep(1);
    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    t_arrive[blockIdx.x] = wall_clock64();
  }
}

__global__ void consumer(int* ctr, int target, unsigned long long* t_seen, int* timeouts,
                         int* done, unsigned long long* t_start) {
  if (threadIdx.x == 0) {
    t_start[blockIdx.x] = wall_clock64();
    const unsigned long long t_end = wall_clock64() + 200000ull;  // 2 ms
    int to = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() > t_end) {
        to = 1;
        break;
      }
    }
    t_seen[blockIdx.x] = wall_clock64();
    if (to) atomicAdd(timeouts, 1);
    // last consumer re-arms the counter for the next replay
    if (atomicAdd(done, 1) == static_cast<int>(gridDim.x) - 1) {
      __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int main() {
  const int P = 200, C = 256, work = 500;  // 5 us of producer work at 100 MHz
  int *ctr, *timeouts, *done;
  unsigned long long *ta, *ts, *pst, *cst;
  CK(hipMalloc(&pst, P * 8));
  CK(hipMalloc(&cst, C * 8));
  CK(hipMalloc(&ctr, 4));
  CK(hipMalloc(&timeouts, 4));
  CK(hipMalloc(&done, 4));
  CK(hipMalloc(&ta, P * 8));
  CK(hipMalloc(&ts, C * 8));
  CK(hipMemset(ctr, 0, 4));
  CK(hipMemset(timeouts, 0, 4));
  CK(hipMemset(done, 0, 4));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  std::vector<unsigned long long> ha(P), hs(C), hps(P), hcs(C);

  auto report = [&](const char* name) -> int {
    int to = 0;
    CK(hipMemcpy(&to, timeouts, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ha.data(), ta, P * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs.data(), ts, C * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hps.data(), pst, P * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hcs.data(), cst, C * 8, hipMemcpyDeviceToHost));
    const unsigned long long last = *std::max_element(ha.begin(), ha.end());
    const unsigned long long p0 = *std::min_element(hps.begin(), hps.end());
    const unsigned long long c0 = *std::min_element(hcs.begin(), hcs.end());
    const unsigned long long c1 = *std::max_element(hcs.begin(), hcs.end());
    std::printf("  [last replay, us from producer start] consumer starts %+.2f .. %+.2f, last producer arrival %+.2f\n",
                (static_cast<double>(c0) - p0) / 100.0, (static_cast<double>(c1) - p0) / 100.0,
                (static_cast<double>(last) - p0) / 100.0);
    const unsigned long long smin = *std::min_element(hs.begin(), hs.end());
    const unsigned long long smax = *std::max_element(hs.begin(), hs.end());
    std::printf("%-34s timeouts %d | flag seen %+.2f .. %+.2f us after the last producer arrival\n",
                name, to, (static_cast<double>(smin) - last) / 100.0,
                (static_cast<double>(smax) - last) / 100.0);
    CK(hipMemset(timeouts, 0, 4));
    return 0;
  };

  // eager, two streams, consumer launched first
  for (int rep = 0; rep < 3; ++rep) {
    consumer<<<C, 512, 0, s0>>>(ctr, P, ts, timeouts, done, cst);
    producer<<<P, 256, 0, s1>>>(ctr, ta, work, pst);
    CK(hipDeviceSynchronize());
  }
  if (report("eager, consumer first")) return 1;

  for (int order = 0; order < 2; ++order) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(fork, s0));
    CK(hipStreamWaitEvent(s1, fork, 0));
    if (order == 0) {
      consumer<<<C, 512, 0, s0>>>(ctr, P, ts, timeouts, done, cst);
      producer<<<P, 256, 0, s1>>>(ctr, ta, work, pst);
    } else {
      producer<<<P, 256, 0, s1>>>(ctr, ta, work, pst);
      consumer<<<C, 512, 0, s0>>>(ctr, P, ts, timeouts, done, cst);
    }
    CK(hipEventRecord(join, s1));
    CK(hipStreamWaitEvent(s0, join, 0));
    CK(hipStreamEndCapture(s0, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 50; ++rep) CK(hipGraphLaunch(ge, s0));
    CK(hipStreamSynchronize(s0));
    if (report(order == 0 ? "graph x50, consumer branch first" : "graph x50, producer branch first"))
      return 1;
    // timing: replays back to back
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s0));
    for (int rep = 0; rep < 200; ++rep) CK(hipGraphLaunch(ge, s0));
    CK(hipEventRecord(e1, s0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("  %.2f us per replay (producer work %.1f us)\n", ms * 1000.f / 200.f, work / 100.0);
    if (report("  after timing replays")) return 1;
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
