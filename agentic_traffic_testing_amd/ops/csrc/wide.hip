// Wide small-M GEMM launcher: plan, split-K reduce launch and the host entry point (the
// kernel itself: wide.h; one translation unit per 16-row block count: wide_mt<N>.hip).
#include <cstdlib>

#include "wide.h"

namespace atta {
namespace wide {

// Split-K combine + epilogue: one wave per (16-column tile, 64-row group), one ROW per lane -
// lane l sums row 64 g + l's 16 columns over the slices (four 16-B loads per slice, the whole
// row's slab reads of up to 4 slices in flight at once), sums of squares likewise, then runs
// the unsplit path's epi_apply on its row with all 64 lanes.  (One wave per 16-row group, a
// quarter row per lane and lanes 0-15 alone in the epilogue: 3x the waves, each with a quarter
// of the loads in flight - 5.5 us per reduce at 85 rows, profiles/r5_burst_breakdown.txt.)
template <typename T, int MT, int EPI, bool NORM>
__global__ __launch_bounds__(256) void wide_reduce_kernel(SkinnyParams p, int ntiles, int S,
                                                         int tpb) {
  constexpr int R = MT * 16;
  constexpr int NRG = (R + 63) / 64;  // 64-row groups per tile
  __shared__ float red_all[4][64][17];
  __shared__ float inv_all[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wid;
  const int tile = gw / NRG, rg = gw % NRG;
  if (tile >= ntiles) return;  // wave-uniform; no workgroup barrier below
  const int cb = tile / tpb;   // the main launch's column block (tiles per workgroup)
  const int r = rg * 64 + lane;
  const int rc = min(r, min(R, max(p.M, 1)) - 1);
  EpiIn<1> ein;
  epi_load<T, EPI, 1>(p, tile, rg * 64, 64, R, lane, ein);
  f32x4 sum[4] = {};
  float ss = 0.f;
  for (int k0 = 0; k0 < S; k0 += 4) {
    f32x4 part[4][4];
    float sp[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ks = min(k0 + u, S - 1);
      const int64_t at = ((static_cast<int64_t>(tile) * S + ks) * R + rc) * 16;
      if (p.sk_half) {  // bf16 slab: 16 values in two 16-B loads
        const u32x4* src = reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(p.sk_ws) + at);
        const u32x4 h0 = src[0], h1 = src[1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t w0 = (q < 2 ? h0 : h1)[(q & 1) * 2], w1 = (q < 2 ? h0 : h1)[(q & 1) * 2 + 1];
          part[u][q] = f32x4{__uint_as_float(w0 << 16), __uint_as_float(w0 & 0xffff0000u),
                             __uint_as_float(w1 << 16), __uint_as_float(w1 & 0xffff0000u)};
        }
      } else {
        const f32x4* src = reinterpret_cast<const f32x4*>(p.sk_ws + at);
#pragma unroll
        for (int q = 0; q < 4; ++q) part[u][q] = src[q];
      }
      if constexpr (NORM)
        sp[u] = p.sk_ws[static_cast<int64_t>(ntiles) * S * R * 16 +
                        (static_cast<int64_t>(cb) * S + ks) * R + rc];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool real = k0 + u < S;  // slice order: bitwise deterministic
#pragma unroll
      for (int q = 0; q < 4; ++q) sum[q] += real ? part[u][q] : f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (NORM) ss += real ? sp[u] : 0.f;
    }
  }
  float(*red)[17] = red_all[wid];
  float* inv_rms = inv_all[wid];
#pragma unroll
  for (int n = 0; n < 16; ++n) red[lane][n] = sum[n >> 2][n & 3];
  if (NORM) inv_rms[lane] = rsqrtf(ss / static_cast<float>(p.K) + p.eps);
  // each lane reads back only its own row: no cross-lane hand-over
  epi_apply<T, EPI, 1>(p, tile, red, inv_rms, rg * 64, NORM, ein);
}

template <typename T, int MT>
static int launch_reduce(int epi, const SkinnyParams& p, int ntiles, int S, int waves,
                         hipStream_t st) {
  constexpr int NRG = (MT * 16 + 63) / 64;
  const dim3 grid((ntiles * NRG + 3) / 4), blk(256);
  const bool norm = p.eps > 0.f;
  switch (epi) {
    case EPI_PLAIN: wide_reduce_kernel<T, MT, EPI_PLAIN, false><<<grid, blk, 0, st>>>(p, ntiles, S, waves); return 0;
    case EPI_RESADD: wide_reduce_kernel<T, MT, EPI_RESADD, false><<<grid, blk, 0, st>>>(p, ntiles, S, waves); return 0;
    case EPI_QKVROPE: wide_reduce_kernel<T, MT, EPI_QKVROPE, true><<<grid, blk, 0, st>>>(p, ntiles, S, waves); return 0;
    case EPI_SILU: wide_reduce_kernel<T, MT, EPI_SILU, true><<<grid, blk, 0, st>>>(p, ntiles, S, waves); return 0;
    case EPI_SAMPLE:
      if (norm) wide_reduce_kernel<T, MT, EPI_SAMPLE, true><<<grid, blk, 0, st>>>(p, ntiles, S, waves);
      else wide_reduce_kernel<T, MT, EPI_SAMPLE, false><<<grid, blk, 0, st>>>(p, ntiles, S, waves);
      return 0;
    default: return -1;
  }
}

template <typename T>
static int launch_reduce_mt(int epi, int mt, const SkinnyParams& p, int ntiles, int S,
                            int waves, hipStream_t st) {
  switch (mt) {
    case 2: return launch_reduce<T, 2>(epi, p, ntiles, S, waves, st);
    case 1: return launch_reduce<T, 1>(epi, p, ntiles, S, waves, st);
    case 3: return launch_reduce<T, 3>(epi, p, ntiles, S, waves, st);
    case 4: return launch_reduce<T, 4>(epi, p, ntiles, S, waves, st);
    case 5: return launch_reduce<T, 5>(epi, p, ntiles, S, waves, st);
    case 6: return launch_reduce<T, 6>(epi, p, ntiles, S, waves, st);
    case 7: return launch_reduce<T, 7>(epi, p, ntiles, S, waves, st);
    case 8: return launch_reduce<T, 8>(epi, p, ntiles, S, waves, st);
    default: return -1;
  }
}

#define ATTA_WIDE_MT_DECL(N)                                                                  \
  int launch_mt_##N(int epi, int waves, int tpw, dim3 grid, hipStream_t st,                    \
                    const SkinnyParams& p, int ntiles, int dtype);
ATTA_WIDE_MT_DECL(1)
ATTA_WIDE_MT_DECL(2)
ATTA_WIDE_MT_DECL(3)
ATTA_WIDE_MT_DECL(4)
ATTA_WIDE_MT_DECL(5)
ATTA_WIDE_MT_DECL(6)
ATTA_WIDE_MT_DECL(7)
ATTA_WIDE_MT_DECL(8)

int launch_mt_tu(int mt, int epi, int waves, int tpw, dim3 grid, hipStream_t st,
                 const SkinnyParams& p, int ntiles, int dtype) {
  switch (mt) {
    case 1: return launch_mt_1(epi, waves, tpw, grid, st, p, ntiles, dtype);
    case 2: return launch_mt_2(epi, waves, tpw, grid, st, p, ntiles, dtype);
    case 3: return launch_mt_3(epi, waves, tpw, grid, st, p, ntiles, dtype);
    case 4: return launch_mt_4(epi, waves, tpw, grid, st, p, ntiles, dtype);
    case 5: return launch_mt_5(epi, waves, tpw, grid, st, p, ntiles, dtype);
    case 6: return launch_mt_6(epi, waves, tpw, grid, st, p, ntiles, dtype);
    case 7: return launch_mt_7(epi, waves, tpw, grid, st, p, ntiles, dtype);
    case 8: return launch_mt_8(epi, waves, tpw, grid, st, p, ntiles, dtype);
    default: return -1;
  }
}

// Grid plan: per candidate (waves, tiles per wave) - T = waves x tpw tiles per workgroup - and
// K split S <= 8, a time estimate - rounds of the grid over the CUs x (a workgroup's weight
// bytes + x bytes / 6 at a per-CU streaming rate, plus ~1.5 us of ramp), plus for a split the
// reduce launch - and the cheapest wins.  Slices keep >= 2 chunks of K.
static double env_or(const char* name, double dflt) {
  const char* v = std::getenv(name);
  return v != nullptr ? std::atof(v) : dflt;
}

static void plan(int ntiles, int K, int M, bool norm, bool w8, int& waves, int& tpw,
                 int& ksplit) {
  constexpr double kCUs = 256.0, kBpus = 24e3;  // bytes per us per CU
  // cost-model knobs (env overrides for A/B runs; read once)
  static const double kXDiv = env_or("ATTA_WIDE_PLAN_XDIV", 6.0);
  static const double kRed = env_or("ATTA_WIDE_PLAN_RED_US", 1.0);
  // split-K slab bytes per us (written by the slices, read back by the reduce): 2e6 refit to
  // the round-6 graph-mode sweep of every (waves, split) plan of qkv / o / down at 50-105
  // rows (best-per-shape sum 374.6 us; the planner's picks 387.5 us at 5e6, 378.9 at 2e6:
  // down moves from 8 x 8 to 4 x 4).  The fp8-weight (W8) plans keep 5e6: at the 70B shapes
  // 2e6 chose fewer splits and the 76-row prefill went 21.4 -> 22.2 ms
  static const double kSlabBpus = env_or("ATTA_WIDE_PLAN_SLAB_BPUS", 2e6);
  // a wave count the 16-bit plans skip (A/B runs; 0 = none).  gate_up's 7 x 1 (256 workgroups)
  // loses to 8 x 1 in isolated back-to-back replays but wins in situ on the fan-out bench
  // (profiles/r6_gate_up_7v8_waves.txt), so nothing is skipped by default
  static const int kSkipW = static_cast<int>(env_or("ATTA_WIDE_PLAN_SKIP_WAVES", 0.0));
  const int mpad = ((M + 15) / 16) * 16;
  const int nch = K / kKC;
  double best = 1e30;
  const int ws[4] = {4, 6, 7, 8};
  for (int tp = 1; tp <= 1; ++tp) {  // tpw 2: measured slower, not built (wide.h launch_t)
    for (int wi = 0; wi < 4; ++wi) {
      const int w = ws[wi];
      if (!w8 && w == kSkipW) continue;
      if (norm && !norm_fits(w, (M + 15) / 16, tp)) continue;  // see launch_epi
      if (tp == 2 && !tpw2_built(w)) continue;
      const int tb = w * tp;
      const int ncb = (ntiles + tb - 1) / tb;
      for (int s = 1; s <= 8 && nch / s >= 2; ++s) {
        const double rounds = std::ceil(ncb * s / kCUs);
        const double kslice = static_cast<double>(K) / s;
        const double bytes = tb * 16.0 * kslice * (w8 ? 1.0 : 2.0) + mpad * kslice * 2.0 / kXDiv;
        const double idle = static_cast<double>(ncb * tb - ntiles) / (ncb * tb);  // empty tiles
        // split: a reduce launch (~1 us beyond the slabs it reads) reading every slice's slab;
        // x bytes at 1/6 and the 1 us fitted to the round-5 graph-mode sweep
        // (profiles/r5_wide_tiles_per_wave_negative.txt: 626 vs 640 us over 20 shapes)
        const double slab = static_cast<double>(ntiles) * s * mpad * 64.0;
        const double t = rounds * (bytes / kBpus * (1.0 + 0.5 * idle) + 1.5) +
                         (s > 1 ? kRed + slab / (w8 ? 5e6 : kSlabBpus) : 0.0);
        if (t < best - 1e-9) {
          best = t;
          waves = w;
          tpw = tp;
          ksplit = s;
        }
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
// split-K slab precision of the wide kernel (atta_set_splitk_half): 0 fp32, 1 bf16
static int g_sk_half = 0;
void atta_set_splitk_half(int on) { g_sk_half = on ? 1 : 0; }

int atta_wide_launch(SkinnyParams& p, int epi, int ntiles, int waves, int ksplit, int dtype,
                     const float* sk_ws, int* sk_counters, int64_t ws_floats, int n_counters,
                     hipStream_t stream) {
  if (p.M < 1 || p.M > 128 || p.K % wide::kKC != 0 || !p.ps) return -1;
  const bool w8 = p.wscale != nullptr;  // fp8 weights (the W8 builds)
  // waves 14 / 16 / 17 / 18 in an explicit plan = 4 / 6 / 7 / 8 waves x two tiles per wave
  // (measured slower and not built: such a plan returns -1 from the launcher)
  int tpw = 1;
  if (waves > 10) {
    tpw = 2;
    waves -= 10;
  }
  if (waves <= 0 || ksplit <= 0)
    wide::plan(ntiles, p.K, p.M, p.eps > 0.f, w8, waves, tpw, ksplit);
  if (waves != 4 && waves != 6 && waves != 7 && waves != 8) return -1;
  if (ksplit < 1 || p.K / wide::kKC < ksplit) return -1;
  // 16-row blocks: rows padded to the next 16 only (75 rows: 80, not 96)
  const int mt = (p.M + 15) / 16;
  const int tb = waves * tpw;
  const int ncb = (ntiles + tb - 1) / tb;
  // slices' row segments [tile][slice][row][16] + row sums of squares [cb][slice][row]; a
  // split whose slabs do not fit the workspace is halved until they do
  auto need = [&](int s) {
    return static_cast<int64_t>(ntiles) * s * mt * 16 * 16 +
           static_cast<int64_t>(ncb) * s * mt * 16;
  };
  while (ksplit > 1 && need(ksplit) > ws_floats) ksplit >>= 1;
  if (ksplit > 1) {
    if (sk_ws == nullptr) return -2;
    p.sk_ws = const_cast<float*>(sk_ws);
    p.sk_counters = sk_counters;
    p.sk_half = g_sk_half;
  }
  (void)n_counters;
  p.ksplit = ksplit;
  const dim3 grid(ncb, ksplit);
  int rc = wide::launch_mt_tu(mt, epi, waves, tpw, grid, stream, p, ntiles, dtype);
  if (rc) return rc;
  if (ksplit > 1) {
    p.wg_trace = nullptr;
    rc = dtype == 0 ? wide::launch_reduce_mt<__bf16>(epi, mt, p, ntiles, ksplit, tb, stream)
                    : wide::launch_reduce_mt<_Float16>(epi, mt, p, ntiles, ksplit, tb, stream);
    if (rc) return rc;
  }
  return static_cast<int>(hipGetLastError());
}
