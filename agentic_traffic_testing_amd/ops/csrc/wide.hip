// Wide small-M GEMM: 33 <= M <= 128 rows over pre-shuffled 16-bit weights, with the decode
// GEMVs' fused epilogues (skinny.h tile_epilogue: residual add, RMSNorm fold + RoPE + paged
// K/V write, SiLU-mul, LM-head sampler keys).  Serves the prefix-cached burst prefill (the
// headline's ~85-row burst, reference agents/agent_a/server.py:534-623) and decode batches of
// 33-128 sequences (reference llm/serve_llm.py:362-373 max_num_seqs), which the 16-row-tile
// GEMV (gemv.hip) serves badly: it re-reads every x row from L2 once per 16 weight rows in
// fragment-shaped 16 x 64-B pieces - at 32 rows gate_up streamed 2.9 TB/s
// (profiles/r4_skinny_mt_probe.txt).
//
// Decomposition.  A workgroup owns WAVES consecutive 16-column weight tiles (wave w: tile
// cb * WAVES + w) over one K slice (split-K S = gridDim.y, for the narrow projections so the
// grid covers the 256 CUs), and all M rows:
//   * x is staged ONCE per workgroup through LDS in 128-column chunks (M_pad x 256 B, full
//     128-B lines, plain 16-B loads into registers then ds_write_b128 into an XOR-swizzled
//     image - slot j of row r at slot j ^ (r & 15): every ds_read_b128 lane group of the
//     fragment reads is conflict-free) and read by all WAVES waves: x's L2 traffic is
//     M / (16 WAVES) of the weight bytes instead of M / 16;
//   * each wave streams its tile's pre-shuffled weights (one contiguous 1 KiB per 32-wide K
//     step) straight to VGPRs, two 4-step chunks ahead, non-temporal;
//   * per K step a wave applies its weight fragment (MFMA B operand) to all MT 16-row x
//     fragments (A operand, ds_read_b128) - the weights are read once for every row;
//   * the RMSNorm fold needs sum(x^2) per row: accumulated from the staged x registers;
//   * split-K: each slice publishes its fp32 accumulators and partial sums of squares with
//     device-scope (sc1) stores; the last arriving slice (arrival counter per column block)
//     sums them in slice order - bitwise deterministic - and runs the epilogue.
// One workgroup barrier per chunk.  Plain loads only (no LDS-DMA): mixing LDS-DMA with the
// register weight stream makes hipcc wait vmcnt(0) at every weight use (cdna_hip_programming
// §5, "Projection GEMM at M = 256" item 4(b)).
#include <cmath>

#include "common.h"
#include "kernels.h"
#include "skinny.h"

namespace atta {
namespace wide {

constexpr int kKC = 128;             // K columns per staged chunk (4 MFMA K steps)
constexpr int kRowB = kKC * 2;       // bytes of one staged x row
constexpr int kSlots = kRowB / 16;   // 16-B slots per staged row

template <typename T, int WAVES, int MT, int EPI>
__global__ __launch_bounds__(WAVES * 64) void wide_kernel(SkinnyParams p, int ntiles) {
  using MF = MfmaK32<T>;
  using frag8 = typename MF::frag8;
  constexpr int R = MT * 16;
  constexpr int NTHR = WAVES * 64;
  constexpr int PIECES = R * kSlots;
  constexpr int PPT = (PIECES + NTHR - 1) / NTHR;  // x pieces per thread per chunk
  constexpr int XBUF = R * kRowB;
  constexpr int REDB = WAVES * R * 17 * 4;
  constexpr int LDSB = 2 * XBUF > REDB ? 2 * XBUF : REDB;
  static_assert(NTHR % 16 == 0, "16 lanes per staged row");
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDSB];
  __shared__ float ssq[R];
  __shared__ float inv_rms[R];
  __shared__ int sk_last;

  // optional per-workgroup timeline (ops.set_gemv_trace, 100 MHz wall clock): [start, K loop
  // done, split-K partials published, end] at wg_trace[4 * (x + gridDim.x * y)]
  unsigned long long tr0 = 0, tr1 = 0, tr2 = 0;
  if (p.wg_trace != nullptr) tr0 = wall_clock64();
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int col = lane & 15;
  const int grp = lane >> 4;
  const int cb = blockIdx.x, ks = blockIdx.y, S = gridDim.y;
  const int tile = cb * WAVES + wid;
  const bool tvalid = tile < ntiles;
  const int nch = p.K / kKC;
  const int c0 = ks * nch / S, c1 = (ks + 1) * nch / S;
  const bool norm = p.eps > 0.f;

  // this wave's weight tile (idle waves of the last column block stream tile 0 and store
  // nothing: every wave takes part in the barriers)
  const uint16_t* wp = p.w + static_cast<int64_t>(tvalid ? tile : 0) * (p.K / 32) * 512 + lane * 8;
  // x pieces of this thread: piece q = tid + i * NTHR -> staged row q / 16, slot q % 16
  const uint16_t* xsrc[PPT];
  int xdst[PPT];
  bool xst[PPT], xss[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int q = tid + i * NTHR;
    const int row = q < PIECES ? q / kSlots : 0;
    const int slot = q % kSlots;
    xst[i] = q < PIECES;
    xss[i] = q < PIECES && row < p.M;
    // rows past M stage a copy of row M - 1 (finite; their accumulator rows are discarded)
    xsrc[i] = p.x + static_cast<int64_t>(min(row, p.M - 1)) * p.x_stride + slot * 8;
    xdst[i] = row * kRowB + ((slot ^ (row & 15)) << 4);
  }

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) ss[i] = 0.f;

  // weights: 3 register stages, chunk j in stage (j - c0) % 3 (two chunks in flight while one
  // computes); x: 2 register sets, chunk j loaded into set (j - c0) % 2 two chunks ahead and
  // written to LDS buffer (j - c0) % 2 one chunk ahead - every wait is for loads issued a full
  // chunk earlier (one chunk ahead exposed the whole load latency at each chunk: 2.2 TB/s)
  u32x4 w0[4], w1[4], w2[4], xa[PPT], xb[PPT];
  auto load_w = [&](u32x4 (&f)[4], int c) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
      f[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wp + (c * 4 + s) * 512));
  };
  auto load_x = [&](u32x4 (&xr)[PPT], int c) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) xr[i] = *reinterpret_cast<const u32x4*>(xsrc[i] + c * kKC);
  };
  auto store_x = [&](const u32x4 (&xr)[PPT], int buf) {
    unsigned char* b = lds + buf * XBUF;
#pragma unroll
    for (int i = 0; i < PPT; ++i)
      if (xst[i]) *reinterpret_cast<u32x4*>(b + xdst[i]) = xr[i];
    if (norm) {
#pragma unroll
      for (int i = 0; i < PPT; ++i)
        if (xss[i]) ss[i] = MF::sq8(__builtin_bit_cast(frag8, xr[i]), ss[i]);
    }
  };
  auto compute = [&](const u32x4 (&f)[4], int buf) {
    const unsigned char* b = lds + buf * XBUF + col * kRowB;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const frag8 wf = __builtin_bit_cast(frag8, f[s]);
      const int off = ((4 * s + grp) ^ col) << 4;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const frag8 xf = *reinterpret_cast<const frag8*>(b + t * 16 * kRowB + off);
        acc[t] = MF::mma(xf, wf, acc[t]);
      }
    }
  };
  // one chunk: issue chunk c + 2's loads, compute chunk c, stage chunk c + 1's x, barrier
  auto iter = [&](const u32x4 (&wcur)[4], u32x4 (&wnext)[4], const u32x4 (&xstage)[PPT],
                  u32x4 (&xload)[PPT], int c, int buf) {
    if (c + 2 < c1) {
      load_x(xload, c + 2);
      load_w(wnext, c + 2);
    }
    compute(wcur, buf);
    if (c + 1 < c1) store_x(xstage, buf ^ 1);
    __syncthreads();
  };

  if (c0 < c1) {
    load_x(xa, c0);
    load_w(w0, c0);
    if (c0 + 1 < c1) {
      load_x(xb, c0 + 1);
      load_w(w1, c0 + 1);
    }
    store_x(xa, 0);
  }
  __syncthreads();
  for (int c = c0; c < c1; c += 6) {
    iter(w0, w2, xb, xa, c, 0);
    if (c + 1 >= c1) break;
    iter(w1, w0, xa, xb, c + 1, 1);
    if (c + 2 >= c1) break;
    iter(w2, w1, xb, xa, c + 2, 0);
    if (c + 3 >= c1) break;
    iter(w0, w2, xa, xb, c + 3, 1);
    if (c + 4 >= c1) break;
    iter(w1, w0, xb, xa, c + 4, 0);
    if (c + 5 >= c1) break;
    iter(w2, w1, xa, xb, c + 5, 1);
  }

  if (p.wg_trace != nullptr) tr1 = tr2 = wall_clock64();
  // ---- row sums of squares: the 16 lanes staging one row are consecutive -------------------
  if (norm) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 1, kWave);
      v += __shfl_xor(v, 2, kWave);
      v += __shfl_xor(v, 4, kWave);
      v += __shfl_xor(v, 8, kWave);
      const int q = tid + i * NTHR;
      if ((tid & 15) == 0 && q < PIECES) ssq[q / kSlots] = v;
    }
  }
  __syncthreads();  // x buffers free from here on (the epilogue tiles reuse them)

  if (S > 1) {
    // ---- split-K hand-over: device-scope stores + arrival counter (common.h) -------------
    const auto rws = dev_rsrc(p.sk_ws);
    const uint32_t per_slice = static_cast<uint32_t>(WAVES * R * 16);
    const uint32_t ss_base = static_cast<uint32_t>(gridDim.x * S) * per_slice;
    const uint32_t mine = static_cast<uint32_t>(cb * S + ks) * per_slice +
                          static_cast<uint32_t>(wid * R * 16 + col * R + 4 * grp);
#pragma unroll
    for (int t = 0; t < MT; ++t)
      dev_store16(rws, (mine + 16 * t) * 4u, __builtin_bit_cast(u32x4, acc[t]));
    if (norm && tid < R)
      dev_store4(rws, (ss_base + static_cast<uint32_t>((cb * S + ks) * R + tid)) * 4u, ssq[tid]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores acknowledged
    __syncthreads();
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.sk_counters + cb, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      sk_last = (old == S - 1);
    }
    __syncthreads();
    if (p.wg_trace != nullptr) tr2 = wall_clock64();
    if (!sk_last) {  // block-uniform
      if (p.wg_trace != nullptr && tid == 0) {
        unsigned long long* t = p.wg_trace + 4 * (blockIdx.x + gridDim.x * blockIdx.y);
        t[0] = tr0;
        t[1] = tr1;
        t[2] = tr2;
        t[3] = tr2;
      }
      return;
    }
    const uint32_t first = static_cast<uint32_t>(cb * S) * per_slice +
                           static_cast<uint32_t>(wid * R * 16 + col * R + 4 * grp);
    f32x4 part[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < S; ++q) {  // slice order: deterministic sums
#pragma unroll
      for (int t = 0; t < MT; ++t)
        part[t] = __builtin_bit_cast(f32x4, dev_load16(rws, (first + q * per_slice + 16 * t) * 4u));
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] += part[t];
    }
    if (norm && tid < R) {
      float sum = 0.f;
      for (int q = 0; q < S; ++q)
        sum += dev_load4(rws, (ss_base + static_cast<uint32_t>((cb * S + q) * R + tid)) * 4u);
      ssq[tid] = sum;
    }
    if (tid == 0)
      __hip_atomic_store(p.sk_counters + cb, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (norm && tid < R) inv_rms[tid] = rsqrtf(ssq[tid] / static_cast<float>(p.K) + p.eps);
  float(*red)[17] = reinterpret_cast<float(*)[17]>(lds + wid * R * 17 * 4);
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[t * 16 + 4 * grp + i][col] = acc[t][i];
  __syncthreads();
  if (tvalid) tile_epilogue<T, EPI, MT>(p, tile, red, inv_rms, norm, lane, 64);
  if (p.wg_trace != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      unsigned long long* t = p.wg_trace + 4 * (blockIdx.x + gridDim.x * blockIdx.y);
      t[0] = tr0;
      t[1] = tr1;
      t[2] = tr2;
      t[3] = wall_clock64();
    }
  }
}

template <typename T, int WAVES, int MT>
static int launch_epi(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p, int ntiles) {
  const dim3 blk(WAVES * 64);
  switch (epi) {
    case EPI_PLAIN: wide_kernel<T, WAVES, MT, EPI_PLAIN><<<grid, blk, 0, st>>>(p, ntiles); return 0;
    case EPI_RESADD: wide_kernel<T, WAVES, MT, EPI_RESADD><<<grid, blk, 0, st>>>(p, ntiles); return 0;
    case EPI_QKVROPE: wide_kernel<T, WAVES, MT, EPI_QKVROPE><<<grid, blk, 0, st>>>(p, ntiles); return 0;
    case EPI_SILU: wide_kernel<T, WAVES, MT, EPI_SILU><<<grid, blk, 0, st>>>(p, ntiles); return 0;
    case EPI_SAMPLE: wide_kernel<T, WAVES, MT, EPI_SAMPLE><<<grid, blk, 0, st>>>(p, ntiles); return 0;
    default: return -1;
  }
}

template <typename T, int MT>
static int launch_w(int epi, int waves, dim3 grid, hipStream_t st, const SkinnyParams& p,
                    int ntiles) {
  switch (waves) {
    case 4: return launch_epi<T, 4, MT>(epi, grid, st, p, ntiles);
    case 6: return launch_epi<T, 6, MT>(epi, grid, st, p, ntiles);
    case 7: return launch_epi<T, 7, MT>(epi, grid, st, p, ntiles);
    case 8: return launch_epi<T, 8, MT>(epi, grid, st, p, ntiles);
    default: return -1;
  }
}

template <typename T>
static int launch_mt(int epi, int mt, int waves, dim3 grid, hipStream_t st,
                     const SkinnyParams& p, int ntiles) {
  switch (mt) {
    case 2: return launch_w<T, 2>(epi, waves, grid, st, p, ntiles);
    case 4: return launch_w<T, 4>(epi, waves, grid, st, p, ntiles);
    case 6: return launch_w<T, 6>(epi, waves, grid, st, p, ntiles);
    case 8: return launch_w<T, 8>(epi, waves, grid, st, p, ntiles);
    default: return -1;
  }
}

// Grid plan: per candidate wave count (tiles per workgroup) and K split S <= 8, a time
// estimate - rounds of the grid over the CUs x (a workgroup's weight bytes + x bytes / 3 at a
// per-CU streaming rate, plus ~1.5 us of ramp), plus the split-K hand-over (~1 us + 0.4 us
// per slice the last arriver reads back) - and the cheapest wins.  Slices keep >= 2 chunks
// of K.
static void plan(int ntiles, int K, int M, int& waves, int& ksplit) {
  constexpr double kCUs = 256.0, kBpus = 24e3;  // bytes per us per CU
  const int mpad = ((M + 15) / 16) * 16;
  const int nch = K / kKC;
  double best = 1e30;
  const int ws[4] = {4, 6, 7, 8};
  for (int wi = 0; wi < 4; ++wi) {
    const int w = ws[wi];
    const int ncb = (ntiles + w - 1) / w;
    for (int s = 1; s <= 8 && nch / s >= 2; ++s) {
      const double rounds = std::ceil(ncb * s / kCUs);
      const double kslice = static_cast<double>(K) / s;
      const double bytes = w * 16.0 * kslice * 2.0 + mpad * kslice * 2.0 / 3.0;
      const double idle = static_cast<double>(ncb * w - ntiles) / (ncb * w);  // empty waves
      const double t = rounds * (bytes / kBpus * (1.0 + 0.5 * idle) + 1.5) +
                       (s > 1 ? 1.0 + 0.4 * s : 0.0);
      if (t < best - 1e-9) {
        best = t;
        waves = w;
        ksplit = s;
      }
    }
  }
}

}  // namespace wide
}  // namespace atta

using namespace atta;

// Launch the wide kernel for a SkinnyParams already filled by a gemv.hip entry point (x, w
// pre-shuffled 16-bit, y / epilogue fields, eps, M, N, K).  ntiles: 16-column tiles (N / 16;
// SiLU: inter / 8).  waves / ksplit 0 = planned here.  Returns 0, -1 (unsupported shape) or
// -2 (split-K workspace missing / too small).
int atta_wide_launch(SkinnyParams& p, int epi, int ntiles, int waves, int ksplit, int dtype,
                     const float* sk_ws, int* sk_counters, int64_t ws_floats, int n_counters,
                     hipStream_t stream) {
  if (p.M < 1 || p.M > 128 || p.K % wide::kKC != 0 || !p.ps || p.wscale != nullptr) return -1;
  if (waves <= 0 || ksplit <= 0) wide::plan(ntiles, p.K, p.M, waves, ksplit);
  if (waves != 4 && waves != 6 && waves != 7 && waves != 8) return -1;
  if (ksplit < 1 || p.K / wide::kKC < ksplit) return -1;
  const int mt = p.M <= 32 ? 2 : p.M <= 64 ? 4 : p.M <= 96 ? 6 : 8;
  const int ncb = (ntiles + waves - 1) / waves;
  // a split whose slabs do not fit the workspace is halved until they do
  auto need = [&](int s) {
    return static_cast<int64_t>(ncb) * s * waves * mt * 16 * 16 +
           static_cast<int64_t>(ncb) * s * mt * 16;
  };
  while (ksplit > 1 && need(ksplit) > ws_floats) ksplit >>= 1;
  if (ksplit > 1) {
    if (sk_ws == nullptr || ncb > n_counters) return -2;
    p.sk_ws = const_cast<float*>(sk_ws);
    p.sk_counters = sk_counters;
  }
  p.ksplit = ksplit;
  const dim3 grid(ncb, ksplit);
  const int rc = dtype == 0 ? wide::launch_mt<__bf16>(epi, mt, waves, grid, stream, p, ntiles)
                            : wide::launch_mt<_Float16>(epi, mt, waves, grid, stream, p, ntiles);
  if (rc) return rc;
  return static_cast<int>(hipGetLastError());
}
