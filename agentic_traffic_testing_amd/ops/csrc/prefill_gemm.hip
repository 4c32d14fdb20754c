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
//   * 256x256 output tile per workgroup, 512 threads = 8 waves as 2 (M) x 4 (N); each wave
//     owns 128 rows x 64 columns = 128 fp32 accumulator VGPRs (bf16: 8 x 4 MFMA 16x16 tiles;
//     fp8: 4 x 2 MFMA 32x32 tiles).
//   * K advances 64 BYTES per row per PHASE (32 bf16 / 64 fp8 elements).  A phase's operands
//     (A: 256 rows x 64 B, W: 256 rows x 64 B, 16 KB each) live in one of FOUR LDS slots
//     (4 x 32 KB = 128 KB, one __shared__ array, 1 workgroup per CU).  Slots are filled by
//     LDS-DMA (global_load_lds_dwordx4) three phases ahead: data for phase P is issued in
//     phase P-3 and retired (counted vmcnt, never 0 in the steady state) before the barrier
//     of phase P-1 (2 phases, 64 KB per CU, in flight; a 5-slot ring with 3 in flight
//     measured no faster).  Wave group 0 (the 4 waves of rows 0-127) stages A, group 1
//     stages W; 4 DMAs per wave per phase.  Where a phase goes (4096^3, one round: 1.27
//     PF/s): staging alone 0.66 us, MFMA + ds_read alone 0.53 us, both 0.85 us
//     (profiles/r3_prefill_gemm_ablation.txt; full 128-B line DMAs would save ~12 % of the
//     staging side).
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
//   * Stream-K over persistent workgroups (below) with an XCD-aware worker order.
#include <mutex>

#include "common.h"
#include "kernels.h"

namespace atta {
namespace {

constexpr int kThreads = 512;
constexpr int kRowBytes = 64;                 // bytes of K per operand row per phase
constexpr int kOpBytes = 256 * kRowBytes;     // 16 KB: one operand of one phase slot
constexpr int kSlotBytes = 2 * kOpBytes;      // A | W
constexpr int kSlots = 4;
constexpr int kLdsBytes = kSlots * kSlotBytes;  // 128 KB
constexpr int kSlabBytes = 256 * 256 * 4;       // one fp32 partial tile

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
  float* ws;                     // stream-K partial tiles: one 256 KB fp32 slab per workgroup
  int* flags;                    // per-workgroup "slab published" flags (consumer resets)
  unsigned* err;                 // bounded-spin timeout report
};

constexpr int kSpinLimit = 1 << 26;

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

// retire every DMA except the newest `n` phases' (4 per phase per wave)
__device__ __forceinline__ void wait_dma(int keep_phases) {
  if (keep_phases >= 3)
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (keep_phases == 2)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (keep_phases == 1)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
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

// Accumulator set of one wave: 128 x 64 outputs, moved to / from the stream-K slabs as 32
// groups of 4 floats (get4 / add4 with compile-time k after unrolling: no register arrays
// are reinterpreted, which would push the accumulators to scratch).
template <bool FP8>
struct Acc;
template <>
struct Acc<false> {
  f32x4 v[8][4];  // [m frag of 16][n frag of 16]
  static constexpr int kRegs = 32;
  __device__ __forceinline__ f32x4 get4(int k) const { return v[k >> 2][k & 3]; }
  __device__ __forceinline__ void add4(int k, f32x4 x) { v[k >> 2][k & 3] += x; }
};
template <>
struct Acc<true> {
  f32x16 v[4][2];  // [m frag of 32][n frag of 32]
  static constexpr int kRegs = 32;
  __device__ __forceinline__ f32x4 get4(int k) const {
    const f32x16& a = v[k >> 3][(k >> 2) & 1];
    const int o = (k & 3) * 4;
    return f32x4{a[o], a[o + 1], a[o + 2], a[o + 3]};
  }
  __device__ __forceinline__ void add4(int k, f32x4 x) {
    f32x16& a = v[k >> 3][(k >> 2) & 1];
    const int o = (k & 3) * 4;
    a[o] += x[0];
    a[o + 1] += x[1];
    a[o + 2] += x[2];
    a[o + 3] += x[3];
  }
};

// One workgroup = one persistent worker of a Stream-K decomposition: the T tiles x NP phases
// of the GEMM are cut into gridDim.x equal ranges of `units` phases (gridDim.x = CU count),
// so every CU does the same MFMA work whatever T is (the 8B prefill shapes have 176-1232
// tiles: 0.7-4.8 waves of 256 CUs as whole tiles).  A range covers the end of one tile, whole
// tiles and the start of another; segments run in DESCENDING tile order, so a workgroup first
// computes the partial start of its last tile and publishes it (fp32 slab, sc1 stores, flag)
// before its own whole tiles, and finishes the tile it shares with lower-numbered workgroups
// last - by then their partials are long published.  The finisher of a tile adds the
// partials of the (lower-numbered, already dispatched) contributors in a fixed order:
// deterministic, no atomics on the data.
// ABL (A/B ablations of the bf16 main loop, measurement only): 1 no MFMA, 2 no LDS-DMA,
// 3 no ds_read - which side bounds a phase
template <int MODE, bool FP8, int ABL = 0>
__global__ void __launch_bounds__(kThreads, 1) prefill_gemm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char lds[kLdsBytes];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  constexpr int kEl = FP8 ? 1 : 2;  // operand element bytes

  // XCD-aware bijective remap of the worker id (dispatch puts block b on XCD b % 8): the 32
  // workers of one XCD get consecutive unit ranges, i.e. neighbouring tiles sharing W stripes
  const int nwg = gridDim.x;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, rr = nwg & 7;
  const int vb = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  const int NP = p.np;
  const int T = p.mt * p.nt;
  // data-parallel rounds first: tile vb + r * nwg; then this worker's stream-K unit range
  // over the remaining tiles
  const int n_dp = vb < p.dp_tiles ? (p.dp_tiles - vb + nwg - 1) / nwg : 0;
  const int64_t sk_total = static_cast<int64_t>(T - p.dp_tiles) * NP;
  const int64_t u0 = static_cast<int64_t>(vb) * p.units;
  const int64_t u1 = min(u0 + p.units, sk_total);
  // split-K schedule (small M: a few whole tiles, e.g. 2 x 16 at M 400 for down_proj): every
  // tile's K phases are cut into S equal slices on S co-resident workgroups (grid = T * S <=
  // CUs, one workgroup per CU).  Each publishes the accumulator groups it does NOT reduce
  // itself (fp32 slab, sc1 stores), arrives on the tile's counter, waits for the other S - 1,
  // then reduces ITS 1/S of the tile's row fragments over all S slices in slice order
  // (deterministic) and runs the epilogue for them: the reduction is spread over the S
  // workgroups instead of one finisher reading (S - 1) whole 256 KB slabs (Stream-K's fix-up).
  const int S = p.splitk;
  const bool skp = S > 1;
  const int sk_t = skp ? b / S : 0, sk_s = skp ? b % S : 0;
  if (!skp && n_dp == 0 && u0 >= u1) return;

  const int dst_op = (wr ? kOpBytes : 0) + (wid & 3) * 1024;
  // fragment read offsets (fragment bases are multiples of the fragment height)
  int a_rd, w_rd;
  if constexpr (FP8) {
    const int r = lane & 31, c = 2 * (lane >> 5);
    const int o = r * kRowBytes + ((c ^ swz<true>(r)) << 4);
    a_rd = (wr * 128) * kRowBytes + o;
    w_rd = kOpBytes + (wc * 64) * kRowBytes + o;
  } else {
    const int r = lane & 15, c = lane >> 4;
    const int o = r * kRowBytes + ((c ^ swz<false>(r)) << 4);
    a_rd = (wr * 128) * kRowBytes + o;
    w_rd = kOpBytes + (wc * 64) * kRowBytes + o;
  }

  Acc<FP8> acc;
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

    // ---- staging addresses of this tile: the wave's 4 DMA rows per phase ------------------
    // DMA `it` of wave (wid & 3) in its group writes bytes [(it*256 + (wid&3)*64 + lane) * 16)
    // of the operand image: row r = it*64 + (wid&3)*16 + lane/4, stored chunk lane&3, which
    // holds global chunk (lane&3) ^ swz(r).
    const char* src[4];
    const char* src2[4];  // ABL 4 probe: the tile's other 128 rows (clamped like src)
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      int r = it * 64 + (wid & 3) * 16 + (lane >> 2);
      int chunk = (lane & 3) ^ swz<FP8>(r);
      if constexpr (ABL == 4) {  // probe: 8 rows x full 128-B lines per DMA instruction
        r = it * 32 + (wid & 3) * 8 + (lane >> 3);
        chunk = lane & 7;
      }
      int64_t row;
      if (wr == 0) {
        row = min(tm * 256 + r, p.M - 1);
        src[it] = static_cast<const char*>(p.a) + row * p.lda * kEl + chunk * 16;
        src2[it] = static_cast<const char*>(p.a) +
                   static_cast<int64_t>(min(tm * 256 + 128 + r, p.M - 1)) * p.lda * kEl + chunk * 16;
      } else {
        if constexpr (MODE == GEMM_SILU) {
          // wave c's 64 columns: gate rows of outputs tn*128 + c*32 .. +31, then the up rows
          const int c = r >> 6;
          const int f = FP8 ? (r >> 5) & 1 : (r >> 5) & 1;
          const int rw = FP8 ? r & 31 : ((r >> 4) & 1) * 16 + (r & 15);
          row = (f ? p.N : 0) + tn * 128 + c * 32 + rw;
        } else {
          row = tn * 256 + r;
        }
        src[it] = static_cast<const char*>(p.w) + row * p.ldw * kEl + chunk * 16;
        src2[it] = src[it] + static_cast<int64_t>(128) * p.ldw * kEl;  // ABL 4 only (PLAIN)
      }
    }
    auto stage = [&](int ph) {
      if constexpr (ABL == 2) return;
      char* d = lds + (ph % kSlots) * kSlotBytes + dst_op;
      const int64_t koff = ABL == 4 ? static_cast<int64_t>(ph >> 1) * 128
                                    : static_cast<int64_t>(ph) * kRowBytes;
#pragma unroll
      for (int it = 0; it < 4; ++it)
        __builtin_amdgcn_global_load_lds((glb_ptr_t)(((ABL == 4 && (ph & 1)) ? src2[it] : src[it]) + koff),
                                         (lds_ptr_t)(d + it * 4096), 16, 0, 0);
    };

    if constexpr (FP8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc.v[i][f][e] = 0.f;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int f = 0; f < 4; ++f) acc.v[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // ---- main loop over phases [k0, k1): prologue puts 3 phases in flight, retires 1 -------
    const int n = k1 - k0;
    stage(k0);
    if (n > 1) stage(k0 + 1);
    if (n > 2) stage(k0 + 2);
    wait_dma(min(n, 3) - 1);
    bar();
    if (wr == 1) bar();  // group 1 runs one barrier behind
    for (int ph = k0; ph < k1; ++ph) {
      const char* s = lds + (ph % kSlots) * kSlotBytes;
      if constexpr (FP8) {
        i32x8 xa[4], wb[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const u32x4 lo = *reinterpret_cast<const u32x4*>(s + w_rd + f * 32 * kRowBytes);
          const u32x4 hi = *reinterpret_cast<const u32x4*>(s + (w_rd ^ 16) + f * 32 * kRowBytes);
          wb[f] = __builtin_bit_cast(i32x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
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
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int f = 0; f < 2; ++f)
            acc.v[i][f] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                wb[f], xa[i], acc.v[i][f], 0, 0, 0, 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      } else {
        bf16x8 xa[8], wb[4];
        if constexpr (ABL == 3) {
#pragma unroll
          for (int f = 0; f < 4; ++f) wb[f] = bf16x8{};
#pragma unroll
          for (int i = 0; i < 8; ++i) xa[i] = bf16x8{};
          asm volatile("" : "+v"(wb[0]), "+v"(xa[0]));
          // one real LDS read keeps the staging array allocated (DMA targets stay in range)
          asm volatile("" ::"v"(*reinterpret_cast<const int*>(s + a_rd)));
        } else {
#pragma unroll
          for (int f = 0; f < 4; ++f)
            wb[f] = *reinterpret_cast<const bf16x8*>(s + w_rd + f * 16 * kRowBytes);
#pragma unroll
          for (int i = 0; i < 8; ++i)
            xa[i] = *reinterpret_cast<const bf16x8*>(s + a_rd + i * 16 * kRowBytes);
        }
        if (ph + 3 < k1) stage(ph + 3);
        wait_lgkm0();
        // keep in flight the phases issued beyond ph + 1 (data for ph + 1 retired)
        wait_dma(min(k1 - 1, ph + 3) - (ph + 1));
        bar();
        __builtin_amdgcn_s_setprio(1);
        if constexpr (ABL == 1 || ABL == 4) {
#pragma unroll
          for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(xa[i]));
#pragma unroll
          for (int f = 0; f < 4; ++f) asm volatile("" ::"v"(wb[f]));
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i)
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

    // ---- partial tile: publish to this worker's slab ------------------------------------------
    const auto slab = dev_rsrc(p.ws);
    // row fragments this workgroup reduces and writes (split-K: its 1/S share)
    constexpr int kFrags = FP8 ? 4 : 8;
    const int i0 = skp ? sk_s * (kFrags / S) : 0;
    const int i1 = skp ? i0 + kFrags / S : kFrags;
    auto frag_of = [](int k) { return FP8 ? (k >> 3) : (k >> 2); };  // row fragment of group k
    if (skp) {
      const uint32_t base = static_cast<uint32_t>(b) * kSlabBytes;
#pragma unroll
      for (int k = 0; k < Acc<FP8>::kRegs; ++k)
        if ((frag_of(k) < i0 || frag_of(k) >= i1) &&
            tm * 256 + wr * 128 + frag_of(k) * (FP8 ? 32 : 16) < p.M)  // padding rows: never read
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(u32x4, acc.get4(k)), slab, static_cast<uint32_t>(tid * 16),
              base + static_cast<uint32_t>(k * kThreads * 16), kScDevice);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        int* ctr = p.flags + t;
        __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // bounded by wall clock (100 MHz): 20 ms, far past any real wait - a grid that is
        // not co-resident (another process's kernels holding CUs) reports instead of hanging
        const unsigned long long t_end = wall_clock64() + 2000000ull;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S) {
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() > t_end) {
            atomicOr(p.err, 2u);
            break;
          }
        }
        // depart; the last of the 2S adds re-arms the counter for the next launch
        if (__hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 2 * S - 1)
          __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
    }
    if (!skp && k1 < NP) {
      const uint32_t base = static_cast<uint32_t>(vb) * kSlabBytes;
#pragma unroll
      for (int k = 0; k < Acc<FP8>::kRegs; ++k)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, acc.get4(k)), slab, static_cast<uint32_t>(tid * 16),
            base + static_cast<uint32_t>(k * kThreads * 16), kScDevice);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(p.flags + vb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    // ---- finisher: wait for the partials of the workers that computed phases [0, k0); they
    // are added group by group in the epilogue (adding them into the accumulators here would
    // make the register allocator copy whole accumulator tuples and spill in the main loop)
    int c0 = 0, c1 = -1;
    if (!skp && k0 > 0) {
      c0 = static_cast<int>(tu / p.units);
      c1 = static_cast<int>((tu + k0 - 1) / p.units);
      if (tid == 0) {
        for (int cb = c0; cb <= c1; ++cb) {
          int spins = 0;
          while (__hip_atomic_load(p.flags + cb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > kSpinLimit) {
              atomicOr(p.err, 1u);
              break;
            }
          }
          __hip_atomic_store(p.flags + cb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      __syncthreads();
    }
    // accumulator group k (4 floats) plus the contributors' partials, in worker order
    auto part = [&](int k) {
      if (skp) {  // the S slices of this tile in slice order, this workgroup's from registers
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < S; ++q)
          v += q == sk_s ? acc.get4(k)
                         : __builtin_bit_cast(
                               f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                          slab, static_cast<uint32_t>(tid * 16),
                                          static_cast<uint32_t>(t * S + q) * kSlabBytes +
                                              static_cast<uint32_t>(k * kThreads * 16),
                                          kScDevice));
        return v;
      }
      f32x4 v = acc.get4(k);
      for (int cb = c0; cb <= c1; ++cb)
        v += __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       slab, static_cast<uint32_t>(tid * 16),
                       static_cast<uint32_t>(cb) * kSlabBytes + static_cast<uint32_t>(k * kThreads * 16),
                       kScDevice));
      return v;
    };

    // ---- epilogue ---------------------------------------------------------------------------
    if constexpr (FP8) {
      // lane holds rows m = i*32 + (lane&31), columns f*32 + 8 g + 4 (lane>>5) + j (reg 4g+j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = tm * 256 + wr * 128 + i * 32 + (lane & 31);
        if (i < i0 || i >= i1 || m >= p.M) continue;
        const float xsc = p.xs[m];
        uint16_t* crow = p.c + static_cast<int64_t>(m) * p.ldc;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = 8 * g + 4 * (lane >> 5);
          if constexpr (MODE == GEMM_SILU) {
            const int nn = tn * 128 + wc * 32 + co;
            const f32x4 sg = *reinterpret_cast<const f32x4*>(p.wsc + nn);
            const f32x4 su = *reinterpret_cast<const f32x4*>(p.wsc + p.N + nn);
            const f32x4 ag = part(i * 8 + g), au = part(i * 8 + 4 + g);
            Pack4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              o.v[j] = from_f32<__bf16>(silu(ag[j] * xsc * sg[j]) * (au[j] * xsc * su[j]));
            *reinterpret_cast<Pack4*>(crow + nn) = o;
          } else {
#pragma unroll
            for (int f = 0; f < 2; ++f) {
              const int nn = tn * 256 + wc * 64 + f * 32 + co;
              const f32x4 sw = *reinterpret_cast<const f32x4*>(p.wsc + nn);
              const f32x4 av = part(i * 8 + f * 4 + g);
              Pack4 o;
              if constexpr (MODE == GEMM_RESADD) {
                const Pack4 r = *reinterpret_cast<const Pack4*>(
                    p.res + static_cast<int64_t>(m) * p.ldres + nn);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  o.v[j] = from_f32<__bf16>(av[j] * xsc * sw[j] +
                                            to_f32<__bf16>(r.v[j]));
              } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  o.v[j] = from_f32<__bf16>(av[j] * xsc * sw[j]);
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
      for (int i = 0; i < 8; ++i) {
        const int m = tm * 256 + wr * 128 + i * 16 + (lane & 15);
        if (i < i0 || i >= i1 || m >= p.M) continue;
        uint16_t* crow = p.c + static_cast<int64_t>(m) * p.ldc;
        if constexpr (MODE == GEMM_SILU) {
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            const int nn = tn * 128 + wc * 32 + f * 16 + cq;
            const f32x4 ag = part(i * 4 + f), au = part(i * 4 + f + 2);
            Pack4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) o.v[j] = from_f32<__bf16>(silu(ag[j]) * au[j]);
            *reinterpret_cast<Pack4*>(crow + nn) = o;
          }
        } else {
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            const int nn = tn * 256 + wc * 64 + f * 16 + cq;
            const f32x4 av = part(i * 4 + f);
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
  unsigned* err = nullptr;
  int cus = 0;
};

// per-device stream-K workspace (64 MB of slabs for 256 CUs), allocated on first use
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
    if (hipMalloc(&ws, static_cast<size_t>(cus) * kSlabBytes) != hipSuccess) return nullptr;
    if (hipMalloc(&flags, static_cast<size_t>(cus + 1) * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemset(flags, 0, static_cast<size_t>(cus + 1) * sizeof(int)) != hipSuccess) return nullptr;
    if (hipDeviceSynchronize() != hipSuccess) return nullptr;
    s.ws = ws;
    s.flags = flags;
    s.err = reinterpret_cast<unsigned*>(flags + cus);
    s.cus = cus;
  }
  return &s;
}

int g_ablate = 0;

template <bool FP8>
hipError_t launch(int mode, dim3 grid, hipStream_t stream, const GemmArgs& p) {
  const dim3 block(kThreads);
  if (!FP8 && mode == GEMM_PLAIN && g_ablate >= 1 && g_ablate <= 4) {
    if (g_ablate == 4)
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_PLAIN, false, 4>), grid, block, 0, stream, p);
    else if (g_ablate == 1)
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_PLAIN, false, 1>), grid, block, 0, stream, p);
    else if (g_ablate == 2)
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_PLAIN, false, 2>), grid, block, 0, stream, p);
    else
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_PLAIN, false, 3>), grid, block, 0, stream, p);
    return hipGetLastError();
  }
  switch (mode) {
    case GEMM_PLAIN:
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_PLAIN, FP8>), grid, block, 0, stream, p);
      break;
    case GEMM_RESADD:
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_RESADD, FP8>), grid, block, 0, stream, p);
      break;
    case GEMM_SILU:
      hipLaunchKernelGGL((prefill_gemm_kernel<GEMM_SILU, FP8>), grid, block, 0, stream, p);
      break;
    default:
      return hipErrorInvalidValue;
  }
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

// A/B knobs of the tile schedule (scripts/gpu/bench_prefill_gemm.py --schedule)
int atta_prefill_gemm_config(int schedule, int group_m, int ablate) {
  if (schedule < 0 || schedule > 3 || group_m < 1 || ablate < 0 || ablate > 4) return -1;
  g_schedule = schedule;
  g_group_m = group_m;
  g_ablate = ablate;
  return 0;
}

// mode: 0 plain, 1 residual add (res may equal c), 2 silu(gate) * up with W = [gate; up].
// fp8: a / w are e4m3fn bytes, xs [M] and wsc [rows of w] their fp32 row scales.
int atta_prefill_gemm(void* c, const void* a, const void* w, const void* res, int M, int N,
                      int K, int64_t lda, int64_t ldw, int64_t ldc, int64_t ldres, int mode,
                      int fp8, const float* xs, const float* wsc, hipStream_t stream) {
  const int el = fp8 ? 1 : 2;
  if (M <= 0 || (K * el) % kRowBytes != 0 || K <= 0) return -1;
  if (mode == GEMM_SILU ? (N % 128 != 0) : (N % 256 != 0)) return -1;
  if (mode == GEMM_RESADD && res == nullptr) return -1;
  if (fp8 && (xs == nullptr || wsc == nullptr)) return -1;
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
  p.mt = (M + 255) / 256;
  p.nt = mode == GEMM_SILU ? N / 128 : N / 256;
  p.np = K * el / kRowBytes;
  const int T = p.mt * p.nt, cus = s->cus;
  p.gm = min(p.mt, g_group_m);
  // schedule (auto): whole rounds of `cus` tiles data-parallel (lock-step tiles share operands
  // in L2), the remainder Stream-K (every CU the same share of its phases); measured on the
  // 8B prefill shapes (profiles/r3_prefill_gemm_ab_*)
  // split-K: S = the largest power of two <= 8 (fp8: 4, its 32-row fragments) with T * S
  // workgroups co-resident (<= CUs, one per CU) and >= 8 K phases per slice
  p.splitk = 1;
  if (g_schedule == 3) {
    int S = 1;
    while (2 * S <= (fp8 ? 4 : 8) && T * 2 * S <= cus && p.np % (2 * S) == 0 &&
           p.np / (2 * S) >= 8)
      S *= 2;
    p.splitk = S;
  }
  if (p.splitk > 1)
    p.dp_tiles = T;  // unused by the split-K path
  else if (g_schedule == 1)
    p.dp_tiles = 0;  // all Stream-K
  else if (g_schedule == 2)
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
  p.err = s->err;
  const hipError_t e = fp8 ? launch<true>(mode, dim3(workers), stream, p)
                           : launch<false>(mode, dim3(workers), stream, p);
  return e == hipSuccess ? 0 : -2;
}

// nonzero once a stream-K finisher timed out waiting for a partial (results are then wrong)
int atta_prefill_gemm_error() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -2;
  Workspace* s = workspace(dev);
  if (s == nullptr) return -2;
  unsigned e = 0;
  if (hipMemcpy(&e, s->err, sizeof(e), hipMemcpyDeviceToHost) != hipSuccess) return -2;
  return static_cast<int>(e);
}
