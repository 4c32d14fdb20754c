// Prefill GEMM for CDNA4 (gfx950): C[M, N] = A[M, K] . W[N, K]^T with fp32 MFMA accumulation
// and the epilogues the decoder layer needs fused in:
//   PLAIN   C = bf16(acc)
//   RESADD  C = bf16(res + acc)            (residual stream update, C may alias res)
//   SILU    C[:, j] = bf16(silu(acc_gate_j) * acc_up_j), W = [gate; up] ([2N, K]), so the
//           gate_up GEMM writes the MLP activation directly (no [M, 2I] intermediate).
// Two operand types:
//   bf16    A, W bf16; v_mfma_f32_16x16x32_bf16.
//   fp8     A, W OCP e4m3fn bytes with fp32 row scales (per token for A, per output channel
//           for W) applied in the epilogue; v_mfma_scale_f32_32x32x64_f8f6f4 with unit
//           block scales = twice the bf16 MFMA rate (MI355X_MICROARCH.md § Matrix cores).
// Replaces hipBLASLt for the prefill projections (reference hot
// path /root/reference/llm/serve_llm.py:527-531, where vLLM's GEMMs do this work).
//
// Design (MI355X-first, not a CUDA tiling):
//   * BM x 256 output tile per workgroup (BM = 256, 128 or 64: the tile height follows the
//     prompt burst - a 5-agent fan-out prefills ~380 rows, a planning call ~70 - so padding
//     rows stay few), 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns BM/2 rows x 64
//     columns (bf16: BM/32 x 4 MFMA 16x16 tiles; fp8: BM/64 x 2 MFMA 32x32 tiles).
//   * K advances 64 BYTES per row per PHASE (32 bf16 / 64 fp8 elements).  A phase's operands
//     (A: BM rows x 64 B, W: 256 rows x 64 B) live in one of FOUR LDS slots (one __shared__
//     array, 1 workgroup per CU).  Slots are filled by LDS-DMA (global_load_lds_dwordx4) three
//     phases ahead: data for phase P is issued in phase P-3 and retired (counted vmcnt, never 0
//     in the steady state) before the barrier of phase P-1.  A phase's BM/16 + 16 DMAs (1 KB =
//     16 rows x 64 B each) are dealt round-robin over the 8 waves: DMA g goes to wave g % 8
//     and lands at slot offset g * 1 KB.  Where a phase goes (BM 256, 4096^3, one round: 1.27
//     PF/s): staging alone 0.66 us, MFMA + ds_read alone 0.53 us, both 0.85 us
//     (profiles/r3_prefill_gemm_ablation.txt).
//   * LDS image: row r of a slot operand is 64 B (4 x 16-B chunks); chunk c of row r is
//     stored at chunk position c ^ swz(r).  A ds_read_b128 is serviced in the lane groups
//     {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32) (MI355X_MICROARCH.md §LDS); swz is chosen so
//     each group covers all 16 16-B bank slots of the 256-B bank row (conflict-free; the plain
//     image is 2-way):  bf16 (lane reads row l & 15, chunk l >> 4): swz = 2 ((r >> 3) & 1);
//     fp8 (lane reads row l & 31, chunks 2 (l >> 5) + {0, 1}): swz = g((r >> 2) & 7) with
//     g(q) = (q ^ (q >> 1)) & 3.  glds writes lane-linearly, so the swizzle is applied on the
//     GLOBAL source address.
//   * Ping-pong: group 1 runs one s_barrier behind group 0 (two barriers per phase), so on
//     every SIMD (waves w and w+4) one wave issues its ds_reads / DMAs while the other runs
//     its MFMAs.  Hazards: the DMA into slot (P+3)%4 = (P-1)%4 is issued after both groups
//     retired (lgkmcnt(0) before their barrier) every read of phase P-1; the reads of phase P
//     follow the barrier after the issuing waves' vmcnt retired phase P's DMAs.
//   * Operands are swapped in the MFMA (a = W fragment, b = A fragment) so each lane ends up
//     holding 4 CONSECUTIVE output columns of one row: 8-byte stores, and the SILU gate and
//     up values of a column sit in the same lane (W rows are gathered per tile so that each
//     wave's first column fragment(s) are gate rows and the others the matching up rows).
//   * Schedules: data-parallel rounds, Stream-K over persistent workgroups (XCD-aware worker
//     order) and split-K (co-resident K slices, parallel reduction) - chosen per call.
//   * Every cross-workgroup wait is bounded; a workgroup whose wait times out (a grid that is
//     not co-resident, e.g. another process holding CUs) recomputes its output rows over the
//     whole K range itself instead of reading partials nobody wrote, so the result stays
//     correct; the error word records it (bit 4) for the engine's health report.
#include <mutex>

#include "common.h"
#include "kernels.h"

namespace atta {
namespace {

constexpr int kThreads = 512;
constexpr int kRowBytes = 64;              // bytes of K per operand row per phase
constexpr int kWOpBytes = 256 * kRowBytes;  // 16 KB: the W operand of one phase slot
constexpr int kSlots = 4;
constexpr int kMaxSlabBytes = 256 * 256 * 4;  // one fp32 partial tile at BM = 256

enum { GEMM_PLAIN = 0, GEMM_RESADD = 1, GEMM_SILU = 2 };

struct GemmArgs {
  const void* a;
  const void* w;
  uint16_t* c;
  const uint16_t* res;
  const float* xs;               // fp8: A row scales [M]
  const float* wsc;              // fp8: W row scales [rows of W]
  int64_t lda, ldw, ldc, ldres;  // elements (bytes for fp8 operands)
  int M, N;                      // N = output columns (SILU: W has 2N rows)
  int mt, nt;                    // tile counts
  int np;                        // phases per tile (K bytes / 64)
  int units;                     // stream-K: phases per workgroup (last one may get fewer)
  int dp_tiles;                  // tiles [0, dp_tiles) run whole, round-robin over workgroups
  int gm;                        // tile order: groups of gm M-tiles, M fastest inside a group
  int splitk;                    // > 1: split-K schedule (below), workgroup b = tile b / S, split b % S
  float* ws;                     // partial tiles: one fp32 slab per workgroup
  int* flags;                    // stream-K "slab published" flags, per workgroup
  int* arrive;                   // split-K arrival / departure counters, 2 per tile
  unsigned* err;                 // bit 1 stream-K wait, 2 split-K wait timed out; 4 recomputed
  unsigned long long wait_ticks;  // bound of a cross-workgroup wait (100 MHz wall clock)
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* glb_ptr_t;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void wait_lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// retire every DMA of this wave except its newest `keep` phases' (D per phase per wave)
template <int D>
__device__ __forceinline__ void wait_dma_d(int keep) {
  if (keep >= 3)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * D) : "memory");
  else if (keep == 2)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * D) : "memory");
  else if (keep == 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(D) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// stored chunk position of chunk c of operand row r (see the header)
template <bool FP8>
__device__ __forceinline__ int swz(int r) {
  if constexpr (FP8) {
    const int q = (r >> 2) & 7;
    return (q ^ (q >> 1)) & 3;
  } else {
    return ((r >> 3) & 1) << 1;
  }
}

// Tile geometry of one BM
template <int BM, bool FP8>
struct Geo {
  static constexpr int kAOpBytes = BM * kRowBytes;
  static constexpr int kSlotBytes = kAOpBytes + kWOpBytes;
  static constexpr int kLdsBytes = kSlots * kSlotBytes;
  static constexpr int kDmas = BM / 16 + 16;     // 1-KB DMAs per phase
  static constexpr int kFragH = FP8 ? 32 : 16;   // rows per accumulator fragment
  static constexpr int MI = BM / 2 / kFragH;     // row fragments per wave
  static constexpr int kRegs = BM / 8;           // f32x4 accumulator groups per lane
  static constexpr int kSlabBytes = BM * 256 * 4;
};

// Accumulator set of one wave: BM/2 x 64 outputs, moved to / from the slabs as kRegs groups
// of 4 floats (get4 / add4 with compile-time k after unrolling: no register arrays are
// reinterpreted, which would push the accumulators to scratch).
template <bool FP8, int MI>
struct Acc;
template <int MI>
struct Acc<false, MI> {
  f32x4 v[MI][4];  // [m frag of 16][n frag of 16]; group k = i * 4 + f
  __device__ __forceinline__ f32x4 get4(int k) const { return v[k >> 2][k & 3]; }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int f = 0; f < 4; ++f) v[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
};
template <int MI>
struct Acc<true, MI> {
  f32x16 v[MI][2];  // [m frag of 32][n frag of 32]; group k = i * 8 + f * 4 + g
  __device__ __forceinline__ f32x4 get4(int k) const {
    const f32x16& a = v[k >> 3][(k >> 2) & 1];
    const int o = (k & 3) * 4;
    return f32x4{a[o], a[o + 1], a[o + 2], a[o + 3]};
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int e = 0; e < 16; ++e) v[i][f][e] = 0.f;
  }
};

// Split-K reduction unit of accumulator group k: the groups one epilogue step consumes
// together (SILU: a gate group and its up group), dealt to the S slices round-robin.
template <int MODE, bool FP8>
__device__ __forceinline__ int unit_of(int k) {
  if constexpr (MODE != GEMM_SILU) return k;
  if constexpr (FP8) return (k >> 3) * 4 + (k & 3);  // gate i*8+g, up i*8+4+g
  return (k >> 2) * 2 + (k & 1);                       // gate i*4+f, up i*4+f+2 (f < 2)
}

constexpr unsigned long long kWaitTicks = 2000000ull;  // 20 ms of the 100 MHz wall clock

// One workgroup = one worker.  Schedules (host-chosen):
//  * data-parallel rounds: tile vb + r * nwg runs whole;
//  * Stream-K: the remaining tiles x NP phases are cut into equal ranges of `units` phases; a
//    range covers the end of one tile, whole tiles and the start of another; segments run in
//    DESCENDING tile order, so a workgroup first publishes the partial start of its last tile
//    (fp32 slab, sc1 stores, flag) and finishes the tile it shares with lower-numbered
//    workgroups last; the finisher adds the contributors' partials in a fixed order
//    (deterministic, no atomics on the data);
//  * split-K (few whole tiles): every tile's K phases are cut into S equal slices on S
//    co-resident workgroups; each publishes the accumulator groups it does NOT reduce itself,
//    arrives on the tile's counter, waits for the other S - 1, then reduces ITS reduction
//    units over all S slices in slice order and runs the epilogue for them.
// ABL (A/B ablations of the bf16 main loop, measurement only): 1 no MFMA, 2 no LDS-DMA,
// 3 no ds_read - which side bounds a phase
template <int MODE, bool FP8, int BM, int ABL = 0>
__global__ void __launch_bounds__(kThreads, 1) prefill_gemm_kernel(GemmArgs p) {
  using G = Geo<BM, FP8>;
  constexpr int MI = G::MI;
  __shared__ __attribute__((aligned(1024))) char lds[G::kLdsBytes];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  constexpr int kEl = FP8 ? 1 : 2;  // operand element bytes
  // DMAs of this wave per phase: g = it * 8 + wid < kDmas
  constexpr int kDmaMax = (G::kDmas + 7) / 8;
  const int ndma = (G::kDmas - wid + 7) / 8;

  // XCD-aware bijective remap of the worker id (dispatch puts block b on XCD b % 8): the 32
  // workers of one XCD get consecutive unit ranges, i.e. neighbouring tiles sharing W stripes
  const int nwg = gridDim.x;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, rr = nwg & 7;
  const int vb = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  const int NP = p.np;
  const int T = p.mt * p.nt;
  const int n_dp = vb < p.dp_tiles ? (p.dp_tiles - vb + nwg - 1) / nwg : 0;
  const int64_t sk_total = static_cast<int64_t>(T - p.dp_tiles) * NP;
  const int64_t u0 = static_cast<int64_t>(vb) * p.units;
  const int64_t u1 = min(u0 + p.units, sk_total);
  const int S = p.splitk;
  const bool skp = S > 1;
  const int sk_t = skp ? b / S : 0, sk_s = skp ? b % S : 0;
  if (!skp && n_dp == 0 && u0 >= u1) return;

  // fragment read offsets (fragment bases are multiples of the fragment height)
  int a_rd, w_rd;
  {
    const int r = FP8 ? lane & 31 : lane & 15;
    const int c = FP8 ? 2 * (lane >> 5) : lane >> 4;
    const int o = r * kRowBytes + ((c ^ swz<FP8>(r)) << 4);
    a_rd = (wr * (BM / 2)) * kRowBytes + o;
    w_rd = G::kAOpBytes + (wc * 64) * kRowBytes + o;
  }
  auto wait_dma = [&](int keep) {
    if (ndma == kDmaMax)
      wait_dma_d<kDmaMax>(keep);
    else
      wait_dma_d<kDmaMax - 1>(keep);
  };

  Acc<FP8, MI> acc;
  int* lflag = reinterpret_cast<int*>(lds);  // scalar broadcasts, only outside the main loop
  const auto slab = dev_rsrc(p.ws);
  const int s_first = u0 < u1 ? static_cast<int>(u0 / NP) : 0;
  const int s_last = u0 < u1 ? static_cast<int>((u1 - 1) / NP) : -1;
  const int nseg = skp ? 1 : n_dp + (s_last - s_first + 1);
  for (int seg = 0; seg < nseg; ++seg) {
    int t, k0, k1;
    int64_t tu = 0;  // stream-K: first unit of tile t
    if (skp) {
      t = sk_t;
      k0 = sk_s * (NP / S);
      k1 = k0 + NP / S;
    } else if (seg < n_dp) {
      t = vb + seg * nwg;
      k0 = 0;
      k1 = NP;
    } else {
      const int st = s_last - (seg - n_dp);  // stream-K tiles in descending order
      tu = static_cast<int64_t>(st) * NP;
      k0 = static_cast<int>(max(u0, tu) - tu);
      k1 = static_cast<int>(min(u1, tu + NP) - tu);
      t = p.dp_tiles + st;
    }
    // grouped tile order: the 32 consecutive tiles of one XCD form a gm x (32 / gm) block,
    // so its concurrently running workgroups share A rows and W stripes through its L2
    const int gsz = p.gm * p.nt, grp = t / gsz, fm = grp * p.gm;
    const int gh = min(p.mt - fm, p.gm), rt = t - grp * gsz;
    const int tm = fm + rt % gh, tn = rt / gh;

    // ---- staging addresses of this tile: DMA g = it * 8 + wid writes slot bytes
    // [g KB + lane * 16): operand row r = (g or g - BM/16) * 16 + lane / 4, stored chunk
    // lane & 3, which holds global chunk (lane & 3) ^ swz(r).
    const char* src[kDmaMax];
#pragma unroll
    for (int it = 0; it < kDmaMax; ++it) {
      const int g = it * 8 + wid;
      const bool isa = g < BM / 16;
      const int r = (isa ? g : g - BM / 16) * 16 + (lane >> 2);
      const int chunk = (lane & 3) ^ swz<FP8>(r);
      int64_t row;
      if (isa) {
        row = min(tm * BM + r, p.M - 1);
        src[it] = static_cast<const char*>(p.a) + row * p.lda * kEl + chunk * 16;
      } else {
        if constexpr (MODE == GEMM_SILU) {
          // wave c's 64 columns: gate rows of outputs tn*128 + c*32 .. +31, then the up rows
          row = (((r >> 5) & 1) ? p.N : 0) + tn * 128 + (r >> 6) * 32 + (r & 31);
        } else {
          row = tn * 256 + r;
        }
        src[it] = static_cast<const char*>(p.w) + row * p.ldw * kEl + chunk * 16;
      }
    }
    auto stage = [&](int ph) {
      if constexpr (ABL == 2) return;
      char* d = lds + (ph % kSlots) * G::kSlotBytes + wid * 1024;
      const int64_t koff = static_cast<int64_t>(ph) * kRowBytes;
#pragma unroll
      for (int it = 0; it < kDmaMax; ++it)
        if (it < ndma)
          __builtin_amdgcn_global_load_lds((glb_ptr_t)(src[it] + koff),
                                           (lds_ptr_t)(d + it * 8192), 16, 0, 0);
    };

    bool full = false;      // recomputing the whole K range after a timed-out wait
    bool partial = false;   // stream-K: this segment only published a partial
    int c0 = 0, c1 = -1;    // stream-K contributors to add
    for (int pass = 0; pass < 2; ++pass) {
      acc.zero();
      // ---- main loop over phases [k0, k1): prologue puts 3 phases in flight, retires 1 ------
      const int n = k1 - k0;
      stage(k0);
      if (n > 1) stage(k0 + 1);
      if (n > 2) stage(k0 + 2);
      wait_dma(min(n, 3) - 1);
      bar();
      if (wr == 1) bar();  // group 1 runs one barrier behind
      for (int ph = k0; ph < k1; ++ph) {
        const char* s = lds + (ph % kSlots) * G::kSlotBytes;
        if constexpr (FP8) {
          i32x8 xa[MI], wb[2];
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            const u32x4 lo = *reinterpret_cast<const u32x4*>(s + w_rd + f * 32 * kRowBytes);
            const u32x4 hi = *reinterpret_cast<const u32x4*>(s + (w_rd ^ 16) + f * 32 * kRowBytes);
            wb[f] = __builtin_bit_cast(i32x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const u32x4 lo = *reinterpret_cast<const u32x4*>(s + a_rd + i * 32 * kRowBytes);
            const u32x4 hi = *reinterpret_cast<const u32x4*>(s + (a_rd ^ 16) + i * 32 * kRowBytes);
            xa[i] = __builtin_bit_cast(i32x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
          if (ph + 3 < k1) stage(ph + 3);
          wait_lgkm0();
          wait_dma(min(k1 - 1, ph + 3) - (ph + 1));
          bar();
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int f = 0; f < 2; ++f)
              acc.v[i][f] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                  wb[f], xa[i], acc.v[i][f], 0, 0, 0, 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
        } else {
          bf16x8 xa[MI], wb[4];
          if constexpr (ABL == 3) {
#pragma unroll
            for (int f = 0; f < 4; ++f) wb[f] = bf16x8{};
#pragma unroll
            for (int i = 0; i < MI; ++i) xa[i] = bf16x8{};
            asm volatile("" : "+v"(wb[0]), "+v"(xa[0]));
            // one real LDS read keeps the staging array allocated (DMA targets stay in range)
            asm volatile("" ::"v"(*reinterpret_cast<const int*>(s + a_rd)));
          } else {
#pragma unroll
            for (int f = 0; f < 4; ++f)
              wb[f] = *reinterpret_cast<const bf16x8*>(s + w_rd + f * 16 * kRowBytes);
#pragma unroll
            for (int i = 0; i < MI; ++i)
              xa[i] = *reinterpret_cast<const bf16x8*>(s + a_rd + i * 16 * kRowBytes);
          }
          if (ph + 3 < k1) stage(ph + 3);
          wait_lgkm0();
          // keep in flight the phases issued beyond ph + 1 (data for ph + 1 retired)
          wait_dma(min(k1 - 1, ph + 3) - (ph + 1));
          bar();
          __builtin_amdgcn_s_setprio(1);
          if constexpr (ABL == 1) {
#pragma unroll
            for (int i = 0; i < MI; ++i) asm volatile("" ::"v"(xa[i]));
#pragma unroll
            for (int f = 0; f < 4; ++f) asm volatile("" ::"v"(wb[f]));
          } else {
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
              for (int f = 0; f < 4; ++f)
                acc.v[i][f] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[f], xa[i], acc.v[i][f], 0, 0, 0);
          }
          __builtin_amdgcn_s_setprio(0);
        }
        bar();
      }
      if (wr == 0) bar();  // balance the group-1 offset: every wave has passed the same barriers
      if (full) break;     // recomputed over the whole K range: reduce from registers only

      bool timed_out = false;
      if (skp) {
        // ---- split-K: publish the groups other slices reduce (padding rows never read) ------
        const uint32_t base = static_cast<uint32_t>(b) * G::kSlabBytes;
#pragma unroll
        for (int k = 0; k < G::kRegs; ++k) {
          const int frag = FP8 ? (k >> 3) : (k >> 2);
          if (unit_of<MODE, FP8>(k) % S != sk_s &&
              tm * BM + wr * (BM / 2) + frag * G::kFragH < p.M)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(u32x4, acc.get4(k)), slab, static_cast<uint32_t>(tid * 16),
                base + static_cast<uint32_t>(k * kThreads * 16), kScDevice);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
          int* arr = p.arrive + 2 * t;
          __hip_atomic_fetch_add(arr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // bounded by wall clock: a grid that is not co-resident times out and recomputes
          const unsigned long long t_end = wall_clock64() + p.wait_ticks;
          int to = 0;
          while (__hip_atomic_load(arr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() > t_end) {
              to = 1;
              break;
            }
          }
          // depart; the last departure re-arms both counters for the next launch (every
          // slice has arrived before any departure can be the S-th)
          if (__hip_atomic_fetch_add(arr + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
              S - 1) {
            __hip_atomic_store(arr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(arr + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          lflag[0] = to;
        }
        __syncthreads();
        timed_out = lflag[0] != 0;
        __syncthreads();
      } else if (k1 < NP) {
        // ---- stream-K partial tile: publish to this worker's slab ---------------------------
        const uint32_t base = static_cast<uint32_t>(vb) * G::kSlabBytes;
#pragma unroll
        for (int k = 0; k < G::kRegs; ++k)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4, acc.get4(k)), slab, static_cast<uint32_t>(tid * 16),
              base + static_cast<uint32_t>(k * kThreads * 16), kScDevice);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // a finisher that gave up on this partial left -1: re-arm the flag for the next launch
        if (tid == 0 &&
            __hip_atomic_exchange(p.flags + vb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == -1)
          __hip_atomic_store(p.flags + vb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        partial = true;
      } else if (k0 > 0) {
        // ---- stream-K finisher: wait for the partials of the workers that computed phases
        // [0, k0); they are added group by group in the epilogue (adding them into the
        // accumulators here would make the register allocator copy whole accumulator tuples)
        c0 = static_cast<int>(tu / p.units);
        c1 = static_cast<int>((tu + k0 - 1) / p.units);
        if (tid == 0) {
          int to = 0;
          const unsigned long long t_end = wall_clock64() + p.wait_ticks;
          for (int cb = c0; cb <= c1; ++cb) {
            bool got = true;
            while (__hip_atomic_load(p.flags + cb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1) {
              __builtin_amdgcn_s_sleep(2);
              if (wall_clock64() > t_end) {
                got = false;
                break;
              }
            }
            if (got) {
              __hip_atomic_store(p.flags + cb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              // give up on it: mark the flag abandoned (-1) so the late contributor re-arms it;
              // if it published in the meantime, re-arm it here
              to = 1;
              if (__hip_atomic_exchange(p.flags + cb, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1)
                __hip_atomic_store(p.flags + cb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          lflag[0] = to;
        }
        __syncthreads();
        timed_out = lflag[0] != 0;
        __syncthreads();
      }
      if (!timed_out) break;
      if (tid == 0) atomicOr(p.err, (skp ? 2u : 1u) | 4u);
      full = true;  // recompute this tile over the whole K range, then reduce from registers
      k0 = 0;
      k1 = NP;
    }
    if (partial) continue;

    // accumulator group k (4 floats) plus the partials of the other slices / contributors
    auto part = [&](int k) {
      if (full) return acc.get4(k);
      if (skp) {  // the S slices of this tile in slice order, this workgroup's from registers
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int qq = 0; qq < S; ++qq)
          v += qq == sk_s ? acc.get4(k)
                          : __builtin_bit_cast(
                                f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           slab, static_cast<uint32_t>(tid * 16),
                                           static_cast<uint32_t>(t * S + qq) * G::kSlabBytes +
                                               static_cast<uint32_t>(k * kThreads * 16),
                                           kScDevice));
        return v;
      }
      f32x4 v = acc.get4(k);
      for (int cb = c0; cb <= c1; ++cb)
        v += __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       slab, static_cast<uint32_t>(tid * 16),
                       static_cast<uint32_t>(cb) * G::kSlabBytes + static_cast<uint32_t>(k * kThreads * 16),
                       kScDevice));
      return v;
    };
    // does this workgroup write the outputs of accumulator group k?
    auto mine = [&](int k) { return !skp || unit_of<MODE, FP8>(k) % S == sk_s; };

    // ---- epilogue ---------------------------------------------------------------------------
    if constexpr (FP8) {
      // lane holds rows m = i*32 + (lane&31), columns f*32 + 8 g + 4 (lane>>5) + j (reg 4g+j)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = tm * BM + wr * (BM / 2) + i * 32 + (lane & 31);
        if (tm * BM + wr * (BM / 2) + i * 32 >= p.M) continue;
        const float xsc = m < p.M ? p.xs[m] : 0.f;
        uint16_t* crow = p.c + static_cast<int64_t>(m) * p.ldc;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = 8 * g + 4 * (lane >> 5);
          if constexpr (MODE == GEMM_SILU) {
            if (!mine(i * 8 + g)) continue;
            const int nn = tn * 128 + wc * 32 + co;
            const f32x4 sg = *reinterpret_cast<const f32x4*>(p.wsc + nn);
            const f32x4 su = *reinterpret_cast<const f32x4*>(p.wsc + p.N + nn);
            const f32x4 ag = part(i * 8 + g), au = part(i * 8 + 4 + g);
            Pack4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              o.v[j] = from_f32<__bf16>(silu(ag[j] * xsc * sg[j]) * (au[j] * xsc * su[j]));
            if (m < p.M) *reinterpret_cast<Pack4*>(crow + nn) = o;
          } else {
#pragma unroll
            for (int f = 0; f < 2; ++f) {
              if (!mine(i * 8 + f * 4 + g)) continue;
              const int nn = tn * 256 + wc * 64 + f * 32 + co;
              const f32x4 sw = *reinterpret_cast<const f32x4*>(p.wsc + nn);
              const f32x4 av = part(i * 8 + f * 4 + g);
              if (m >= p.M) continue;
              Pack4 o;
              if constexpr (MODE == GEMM_RESADD) {
                const Pack4 r = *reinterpret_cast<const Pack4*>(
                    p.res + static_cast<int64_t>(m) * p.ldres + nn);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  o.v[j] = from_f32<__bf16>(av[j] * xsc * sw[j] + to_f32<__bf16>(r.v[j]));
              } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) o.v[j] = from_f32<__bf16>(av[j] * xsc * sw[j]);
              }
              *reinterpret_cast<Pack4*>(crow + nn) = o;
            }
          }
        }
      }
    } else {
      // lane holds rows m = i*16 + (lane&15), columns f*16 + (lane>>4)*4 + j
      const int cq = (lane >> 4) * 4;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = tm * BM + wr * (BM / 2) + i * 16 + (lane & 15);
        if (tm * BM + wr * (BM / 2) + i * 16 >= p.M) continue;
        uint16_t* crow = p.c + static_cast<int64_t>(m) * p.ldc;
        if constexpr (MODE == GEMM_SILU) {
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            if (!mine(i * 4 + f)) continue;
            const int nn = tn * 128 + wc * 32 + f * 16 + cq;
            const f32x4 ag = part(i * 4 + f), au = part(i * 4 + f + 2);
            if (m >= p.M) continue;
            Pack4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) o.v[j] = from_f32<__bf16>(silu(ag[j]) * au[j]);
            *reinterpret_cast<Pack4*>(crow + nn) = o;
          }
        } else {
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            if (!mine(i * 4 + f)) continue;
            const int nn = tn * 256 + wc * 64 + f * 16 + cq;
            const f32x4 av = part(i * 4 + f);
            if (m >= p.M) continue;
            Pack4 o;
            if constexpr (MODE == GEMM_RESADD) {
              const Pack4 r = *reinterpret_cast<const Pack4*>(
                  p.res + static_cast<int64_t>(m) * p.ldres + nn);
#pragma unroll
              for (int j = 0; j < 4; ++j)
                o.v[j] = from_f32<__bf16>(av[j] + to_f32<__bf16>(r.v[j]));
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) o.v[j] = from_f32<__bf16>(av[j]);
            }
            *reinterpret_cast<Pack4*>(crow + nn) = o;
          }
        }
      }
    }
  }
}

struct Workspace {
  float* ws = nullptr;
  int* flags = nullptr;
  int* arrive = nullptr;
  unsigned* err = nullptr;
  int cus = 0;
};

// per-device workspace (64 MB of slabs for 256 CUs), allocated on first use
Workspace* workspace(int dev) {
  static Workspace w[64];
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (dev < 0 || dev >= 64) return nullptr;
  Workspace& s = w[dev];
  if (s.ws == nullptr) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return nullptr;
    const int cus = prop.multiProcessorCount;
    float* ws = nullptr;
    int* flags = nullptr;
    const size_t nflags = static_cast<size_t>(3 * cus + 16);
    if (hipMalloc(&ws, static_cast<size_t>(cus) * kMaxSlabBytes) != hipSuccess) return nullptr;
    if (hipMalloc(&flags, nflags * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemset(flags, 0, nflags * sizeof(int)) != hipSuccess) return nullptr;
    if (hipDeviceSynchronize() != hipSuccess) return nullptr;
    s.ws = ws;
    s.flags = flags;
    s.arrive = flags + cus;
    s.err = reinterpret_cast<unsigned*>(flags + 3 * cus);
    s.cus = cus;
  }
  return &s;
}

int g_ablate = 0;

template <int MODE, bool FP8, int BM>
void launch_bm(dim3 grid, hipStream_t stream, const GemmArgs& p) {
  const dim3 block(kThreads);
  if (!FP8 && MODE == GEMM_PLAIN && g_ablate >= 1 && g_ablate <= 3) {
    if (g_ablate == 1)
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_PLAIN, false, BM, 1>), grid, block, 0, stream, p);
    else if (g_ablate == 2)
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_PLAIN, false, BM, 2>), grid, block, 0, stream, p);
    else
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_PLAIN, false, BM, 3>), grid, block, 0, stream, p);
    return;
  }
  hipLaunchKernelGGL((prefill_gemm_kernel<MODE, FP8, BM>), grid, block, 0, stream, p);
}

template <bool FP8>
hipError_t launch(int mode, int bm, dim3 grid, hipStream_t stream, const GemmArgs& p) {
#define ATTA_PG_BM(MODE)                                                   \
  do {                                                                     \
    if (bm == 256)                                                         \
      launch_bm<MODE, FP8, 256>(grid, stream, p);                          \
    else if (bm == 128)                                                    \
      launch_bm<MODE, FP8, 128>(grid, stream, p);                          \
    else                                                                   \
      launch_bm<MODE, FP8, 64>(grid, stream, p);                           \
  } while (0)
  switch (mode) {
    case GEMM_PLAIN:
      ATTA_PG_BM(GEMM_PLAIN);
      break;
    case GEMM_RESADD:
      ATTA_PG_BM(GEMM_RESADD);
      break;
    case GEMM_SILU:
      ATTA_PG_BM(GEMM_SILU);
      break;
    default:
      return hipErrorInvalidValue;
  }
#undef ATTA_PG_BM
  return hipGetLastError();
}

}  // namespace
}  // namespace atta

using namespace atta;

namespace {
int g_schedule = 0;  // 0 hybrid (data-parallel rounds + Stream-K remainder), 1 Stream-K, 2 DP,
                     // 3 split-K (co-resident K slices, parallel reduction) where it fits
int g_group_m = 4;   // M tiles per raster group
}  // namespace

// Process-wide defaults of the tile schedule (A/B knobs: scripts/gpu/bench_prefill_gemm.py);
// a call can override the schedule and the tile height for itself (atta_prefill_gemm).
// ablate 4 (tests only): every cross-workgroup wait gives up at once, which exercises the
// recompute fallback of a timed-out wait.
int atta_prefill_gemm_config(int schedule, int group_m, int ablate) {
  if (schedule < 0 || schedule > 3 || group_m < 1 || ablate < 0 || ablate > 4) return -1;
  g_schedule = schedule;
  g_group_m = group_m;
  g_ablate = ablate;
  return 0;
}

// Tile height for M rows when the caller leaves it to the library: the fewest padding rows,
// ties to the taller tile (more MFMA work per staged byte).
int atta_prefill_gemm_auto_bm(int M) {
  int best = 256;
  int64_t waste = (static_cast<int64_t>(M) + 255) / 256 * 256 - M;
  for (int bm : {128, 64}) {
    const int64_t w = (static_cast<int64_t>(M) + bm - 1) / bm * bm - M;
    // a smaller tile must save at least 1/8 of the rows to pay for its extra staging
    if (w + M / 8 < waste) {
      best = bm;
      waste = w;
    }
  }
  return best;
}

// mode: 0 plain, 1 residual add (res may equal c), 2 silu(gate) * up with W = [gate; up].
// fp8: a / w are e4m3fn bytes, xs [M] and wsc [rows of w] their fp32 row scales.
// schedule: -1 the configured default, else 0-3 as atta_prefill_gemm_config; bm: 0 auto, else
// 64 / 128 / 256 (the tile height).
int atta_prefill_gemm(void* c, const void* a, const void* w, const void* res, int M, int N,
                      int K, int64_t lda, int64_t ldw, int64_t ldc, int64_t ldres, int mode,
                      int fp8, const float* xs, const float* wsc, int schedule, int bm,
                      hipStream_t stream) {
  const int el = fp8 ? 1 : 2;
  if (M <= 0 || (K * el) % kRowBytes != 0 || K <= 0) return -1;
  if (mode == GEMM_SILU ? (N % 128 != 0) : (N % 256 != 0)) return -1;
  if (mode == GEMM_RESADD && res == nullptr) return -1;
  if (fp8 && (xs == nullptr || wsc == nullptr)) return -1;
  if (schedule < -1 || schedule > 3) return -1;
  if (bm == 0) bm = atta_prefill_gemm_auto_bm(M);
  if (bm != 64 && bm != 128 && bm != 256) return -1;
  if (schedule < 0) schedule = g_schedule;
  // 16-byte DMA sources and 8-byte epilogue accesses
  if ((lda * el) % 16 != 0 || (ldw * el) % 16 != 0 || ldc % 4 != 0 ||
      (mode == GEMM_RESADD && ldres % 4 != 0))
    return -1;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -2;
  Workspace* s = workspace(dev);
  if (s == nullptr) return -2;
  GemmArgs p;
  p.a = a;
  p.w = w;
  p.c = static_cast<uint16_t*>(c);
  p.res = static_cast<const uint16_t*>(res);
  p.xs = xs;
  p.wsc = wsc;
  p.lda = lda;
  p.ldw = ldw;
  p.ldc = ldc;
  p.ldres = ldres;
  p.M = M;
  p.N = N;
  p.mt = (M + bm - 1) / bm;
  p.nt = mode == GEMM_SILU ? N / 128 : N / 256;
  p.np = K * el / kRowBytes;
  const int T = p.mt * p.nt, cus = s->cus;
  p.gm = min(p.mt, g_group_m);
  // split-K: S = the largest power of two <= 16 with T * S workgroups co-resident (<= CUs,
  // one per CU), >= 4 K phases per slice and S <= the tile's reduction units (bm / 8
  // accumulator groups per lane, half of them for SiLU's gate / up pairs)
  p.splitk = 1;
  if (schedule == 3) {
    const int units = mode == GEMM_SILU ? bm / 16 : bm / 8;
    int S = 1;
    while (2 * S <= 16 && 2 * S <= units && T * 2 * S <= cus && p.np % (2 * S) == 0 &&
           p.np / (2 * S) >= 4)
      S *= 2;
    p.splitk = S;
  }
  // schedule (hybrid): whole rounds of `cus` tiles data-parallel (lock-step tiles share
  // operands in L2), the remainder Stream-K (every CU the same share of its phases); measured
  // on the 8B prefill shapes (profiles/r3_prefill_gemm_ab_*)
  if (p.splitk > 1)
    p.dp_tiles = T;  // unused by the split-K path
  else if (schedule == 1)
    p.dp_tiles = 0;  // all Stream-K
  else if (schedule == 2)
    p.dp_tiles = T;  // all data-parallel (last round partial)
  else if (T < 2 * cus)
    p.dp_tiles = 0;  // one or two partial rounds: Stream-K balances them (qkv / o / down)
  else if (T % cus >= (3 * cus) / 4)
    p.dp_tiles = T;  // a well-filled last round: whole tiles keep the L2 sharing (gate_up)
  else
    p.dp_tiles = (T / cus) * cus;
  const int64_t sk_total = static_cast<int64_t>(T - p.dp_tiles) * p.np;
  // Stream-K: an equal share per CU, never less than a quarter tile (bounds the partials a
  // finisher adds to ~4); slab offsets are 32-bit (cus * 256 KB < 4 GB)
  int workers = 0;
  p.units = 1;
  if (sk_total > 0) {
    workers = cus;
    const int64_t min_units = p.np >= 8 ? p.np / 4 : 1;
    if (sk_total / workers < min_units)
      workers = static_cast<int>(sk_total / min_units > 0 ? sk_total / min_units : 1);
    p.units = static_cast<int>((sk_total + workers - 1) / workers);
    workers = static_cast<int>((sk_total + p.units - 1) / p.units);
  }
  if (p.dp_tiles > 0) workers = max(workers, min(cus, p.dp_tiles));
  if (p.splitk > 1) workers = T * p.splitk;
  p.ws = s->ws;
  p.flags = s->flags;
  p.arrive = s->arrive;
  p.err = s->err;
  p.wait_ticks = g_ablate == 4 ? 0ull : kWaitTicks;
  const hipError_t e = fp8 ? launch<true>(mode, bm, dim3(workers), stream, p)
                           : launch<false>(mode, bm, dim3(workers), stream, p);
  return e == hipSuccess ? 0 : -2;
}

// nonzero once a cross-workgroup wait timed out (bit 1 stream-K, 2 split-K; bit 4: the
// workgroup recomputed its tile over the whole K range, so the results are still correct)
int atta_prefill_gemm_error() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -2;
  Workspace* s = workspace(dev);
  if (s == nullptr) return -2;
  unsigned e = 0;
  if (hipMemcpy(&e, s->err, sizeof(e), hipMemcpyDeviceToHost) != hipSuccess) return -2;
  return static_cast<int>(e);
}

// Enqueue a copy of the error word into `host` (4 bytes, pinned) on `stream`: the engine reads
// it after the step's own token sync, so the check costs no extra synchronisation.
// clear != 0: the word is zeroed behind the copy (stream order), so every read reports the
// timeouts since the previous read, not "ever" (ADVICE r4).
int atta_prefill_gemm_error_async(void* host, hipStream_t stream, int clear) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -2;
  Workspace* s = workspace(dev);
  if (s == nullptr) return -2;
  if (hipMemcpyAsync(host, s->err, sizeof(unsigned), hipMemcpyDeviceToHost, stream) !=
      hipSuccess)
    return -2;
  if (clear && hipMemsetAsync(s->err, 0, sizeof(unsigned), stream) != hipSuccess) return -2;
  return 0;
}

// Zero the error word (tests that force a timeout re-arm it in their finally block).
int atta_prefill_gemm_error_reset() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -2;
  Workspace* s = workspace(dev);
  if (s == nullptr) return 0;  // no workspace yet: nothing recorded
  return hipMemset(s->err, 0, sizeof(unsigned)) == hipSuccess ? 0 : -2;
}
