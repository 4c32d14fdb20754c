// Prefill GEMM for CDNA4 (gfx950): C[M, N] = A[M, K] . W[N, K]^T, bf16 in, fp32 MFMA
// accumulate, with the epilogues the decoder layer needs fused in:
//   PLAIN   C = bf16(acc)
//   RESADD  C = bf16(res + acc)            (residual stream update, C may alias res)
//   SILU    C[:, j] = bf16(silu(acc_gate_j) * acc_up_j), W = [gate; up] ([2N, K]), so the
//           gate_up GEMM writes the MLP activation directly (no [M, 2I] intermediate).
// Replaces hipBLASLt for the prefill projections (reference hot
// path /root/reference/llm/serve_llm.py:527-531, where vLLM's GEMMs do this work).
//
// Design (MI355X-first, not a CUDA tiling):
//   * 256x256 output tile per workgroup, 512 threads = 8 waves as 2 (M) x 4 (N); each wave
//     owns 128 rows x 64 columns = 8 x 4 MFMA 16x16x32 bf16 accumulators (128 VGPRs).
//   * K advances 32 per PHASE.  A phase's operands (A: 256 rows x 32 k, W: 256 rows x 32 k,
//     16 KB each) live in one of FOUR LDS slots (4 x 32 KB = 128 KB, one __shared__ array, 1
//     workgroup per CU).  Slots are filled by LDS-DMA (global_load_lds_dwordx4) three phases
//     ahead: data for phase P is issued in phase P-3 and retired (counted vmcnt, never 0 in
//     the steady state) before the barrier of phase P-1, so ~2 phases of MFMA work cover the
//     HBM/L2 latency.  Wave group 0 (the 4 waves of rows 0-127) stages the A operand, group
//     1 stages W; each wave issues 4 DMAs per phase.
//   * LDS image: row r of a slot operand is 64 B (4 x 16-B chunks); chunk c of row r is
//     stored at chunk position c ^ ((r >> 2) & 3) - the 16 lanes of a ds_read_b128 that
//     read one chunk column of 16 rows then hit 16 distinct 16-B bank slots (conflict-free).
//     glds writes lane-linearly, so the swizzle is applied on the GLOBAL source address.
//   * Ping-pong: group 1 runs one s_barrier behind group 0 (two barriers per phase), so on
//     every SIMD (waves w and w+4) one wave issues its ds_reads / DMAs while the other runs
//     its 32 MFMAs.  Hazards: the DMA into slot (P+3)%4 = (P-1)%4 is issued after both
//     groups retired (lgkmcnt(0) before their barrier) every read of phase P-1; the reads
//     of phase P follow the barrier after the issuing waves' vmcnt retired phase P's DMAs.
//   * Operands are swapped in the MFMA (a = W fragment, b = A fragment) so each lane ends
//     up holding 4 CONSECUTIVE output columns of one row: 8-byte stores, and the SILU gate
//     and up values of a column sit in the same lane (W rows are gathered per tile so that
//     wave column fragments 0,1 are gate rows and 2,3 the matching up rows).
//   * Tiles are assigned XCD-aware: the 8 XCDs each get one contiguous range of tile ids
//     (bijective remap), ordered M-fastest, so the M tiles that share a W stripe run
//     together on one XCD and its L2 serves the stripe once.
#include "common.h"
#include "kernels.h"

namespace atta {
namespace {

constexpr int kThreads = 512;
constexpr int kRowBytes = 64;                 // 32 k x bf16 per operand row per phase
constexpr int kOpBytes = 256 * kRowBytes;     // 16 KB: one operand of one phase slot
constexpr int kSlotBytes = 2 * kOpBytes;      // A | W
constexpr int kSlots = 4;
constexpr int kLdsBytes = kSlots * kSlotBytes;  // 128 KB

enum { GEMM_PLAIN = 0, GEMM_RESADD = 1, GEMM_SILU = 2 };

struct GemmArgs {
  const uint16_t* a;
  const uint16_t* w;
  uint16_t* c;
  const uint16_t* res;
  int64_t lda, ldw, ldc, ldres;  // elements
  int M, N, K;                   // N = output columns (SILU: W has 2N rows)
  int mt, nt;                    // tile counts
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* glb_ptr_t;

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void wait_lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// retire every DMA except the newest `n` phases' (4 per phase per wave)
__device__ __forceinline__ void wait_dma(int keep_phases) {
  if (keep_phases >= 2)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (keep_phases == 1)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

template <int MODE>
__global__ void __launch_bounds__(kThreads, 1) prefill_gemm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char lds[kLdsBytes];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  // XCD-aware bijective tile remap (round-robin dispatch puts block b on XCD b % 8)
  const int nwg = p.mt * p.nt;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  const int tm = wg % p.mt, tn = wg / p.mt;

  // ---- staging addresses: this wave's 4 DMA rows per phase ------------------------------
  // DMA `it` of wave (wid & 3) in its group writes bytes [(it*256 + (wid&3)*64 + lane) * 16)
  // of the operand image: row r = it*64 + (wid&3)*16 + lane/4, stored chunk lane&3, which
  // holds global chunk (lane&3) ^ ((r>>2)&3).
  const char* src[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int r = it * 64 + (wid & 3) * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((r >> 2) & 3);
    int64_t row;
    if (wr == 0) {
      row = min(tm * 256 + r, p.M - 1);
      src[it] = reinterpret_cast<const char*>(p.a + row * p.lda) + chunk * 16;
    } else {
      if constexpr (MODE == GEMM_SILU) {
        const int c = r >> 6, f = (r >> 4) & 3;
        row = (f >= 2 ? p.N : 0) + tn * 128 + c * 32 + (f & 1) * 16 + (r & 15);
      } else {
        row = tn * 256 + r;
      }
      src[it] = reinterpret_cast<const char*>(p.w + row * p.ldw) + chunk * 16;
    }
  }
  const int dst_op = (wr ? kOpBytes : 0) + (wid & 3) * 1024;

  auto stage = [&](int ph) {
    const int slot = ph & 3;
    char* d = lds + slot * kSlotBytes + dst_op;
    const int64_t koff = static_cast<int64_t>(ph) * kRowBytes;
#pragma unroll
    for (int it = 0; it < 4; ++it)
      __builtin_amdgcn_global_load_lds((glb_ptr_t)(src[it] + koff), (lds_ptr_t)(d + it * 4096),
                                       16, 0, 0);
  };

  // ---- fragment read addresses ----------------------------------------------------------
  // lane reads row (lane & 15) of a 16-row fragment, global chunk lane >> 4, stored at
  // chunk (lane >> 4) ^ ((row >> 2) & 3); fragment bases are multiples of 16 rows.
  const int swz = (((lane >> 4) ^ ((lane >> 2) & 3)) << 4) + (lane & 15) * kRowBytes;
  const int a_rd = (wr * 128) * kRowBytes + swz;
  const int w_rd = kOpBytes + (wc * 64) * kRowBytes + swz;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int NP = p.K >> 5;
  // prologue: phases 0..2 in flight, 0 and 1 retired
  stage(0);
  if (NP > 1) stage(1);
  if (NP > 2) stage(2);
  wait_dma(NP > 2 ? 1 : 0);
  bar();
  if (wr == 1) bar();  // group 1 runs one barrier behind

  for (int ph = 0; ph < NP; ++ph) {
    const char* s = lds + (ph & 3) * kSlotBytes;
    bf16x8 xa[8], wb[4];
#pragma unroll
    for (int f = 0; f < 4; ++f)
      wb[f] = *reinterpret_cast<const bf16x8*>(s + w_rd + f * 16 * kRowBytes);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      xa[i] = *reinterpret_cast<const bf16x8*>(s + a_rd + i * 16 * kRowBytes);
    if (ph + 3 < NP) stage(ph + 3);
    wait_lgkm0();
    // keep in flight the phases issued beyond ph + 1 (data for ph + 1 retired)
    wait_dma(min(NP - 1, ph + 3) - (ph + 1));
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int f = 0; f < 4; ++f)
        acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[f], xa[i], acc[i][f], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
  }
  if (wr == 0) bar();  // balance the group-1 offset

  // ---- epilogue: lane holds rows m = i*16 + (lane&15), columns f*16 + (lane>>4)*4 + j ----
  const int m_base = tm * 256 + wr * 128 + (lane & 15);
  const int cq = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m_base + i * 16;
    if (m >= p.M) continue;
    uint16_t* crow = p.c + static_cast<int64_t>(m) * p.ldc;
    if constexpr (MODE == GEMM_SILU) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int n = tn * 128 + wc * 32 + f * 16 + cq;
        Pack4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o.v[j] = from_f32<__bf16>(silu(acc[i][f][j]) * acc[i][f + 2][j]);
        *reinterpret_cast<Pack4*>(crow + n) = o;
      }
    } else {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int n = tn * 256 + wc * 64 + f * 16 + cq;
        Pack4 o;
        if constexpr (MODE == GEMM_RESADD) {
          const Pack4 r = *reinterpret_cast<const Pack4*>(
              p.res + static_cast<int64_t>(m) * p.ldres + n);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            o.v[j] = from_f32<__bf16>(acc[i][f][j] + to_f32<__bf16>(r.v[j]));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o.v[j] = from_f32<__bf16>(acc[i][f][j]);
        }
        *reinterpret_cast<Pack4*>(crow + n) = o;
      }
    }
  }
}

}  // namespace
}  // namespace atta

using namespace atta;

// mode: 0 plain, 1 residual add (res may equal c), 2 silu(gate) * up with W = [gate; up]
int atta_prefill_gemm(void* c, const void* a, const void* w, const void* res, int M, int N,
                      int K, int64_t lda, int64_t ldw, int64_t ldc, int64_t ldres, int mode,
                      hipStream_t stream) {
  if (M <= 0 || K % 32 != 0 || K < 32) return -1;
  if (mode == GEMM_SILU ? (N % 128 != 0) : (N % 256 != 0)) return -1;
  if (mode == GEMM_RESADD && res == nullptr) return -1;
  // 16-byte DMA sources and 8-byte epilogue accesses
  if (lda % 8 != 0 || ldw % 8 != 0 || ldc % 4 != 0 || (mode == GEMM_RESADD && ldres % 4 != 0))
    return -1;
  GemmArgs p;
  p.a = static_cast<const uint16_t*>(a);
  p.w = static_cast<const uint16_t*>(w);
  p.c = static_cast<uint16_t*>(c);
  p.res = static_cast<const uint16_t*>(res);
  p.lda = lda;
  p.ldw = ldw;
  p.ldc = ldc;
  p.ldres = ldres;
  p.M = M;
  p.N = N;
  p.K = K;
  p.mt = (M + 255) / 256;
  p.nt = mode == GEMM_SILU ? N / 128 : N / 256;
  const dim3 grid(p.mt * p.nt), block(kThreads);
  switch (mode) {
    case GEMM_PLAIN:
      hipLaunchKernelGGL(prefill_gemm_kernel<GEMM_PLAIN>, grid, block, 0, stream, p);
      break;
    case GEMM_RESADD:
      hipLaunchKernelGGL(prefill_gemm_kernel<GEMM_RESADD>, grid, block, 0, stream, p);
      break;
    case GEMM_SILU:
      hipLaunchKernelGGL(prefill_gemm_kernel<GEMM_SILU>, grid, block, 0, stream, p);
      break;
    default:
      return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
