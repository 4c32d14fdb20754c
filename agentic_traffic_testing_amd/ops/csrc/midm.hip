// Mid-M GEMM launcher: plan, split-K reduce launch and the host entry point (the kernel:
// midm.h; one translation unit per row-block height: midm_b<N>.hip).
#include <cmath>

#include "midm.h"

namespace atta {
namespace midm {

// Split-K combine + epilogue: one wave per (16-column tile, 64-row group), one ROW per lane
// (four 16-B loads per slice, up to 4 slices' loads in flight), summed in slice order -
// bitwise deterministic - then the unsplit path's epilogue on the lane's row (wide.hip's
// reduce, same layout).
template <typename T, int EPI>
__global__ __launch_bounds__(256) void midm_reduce_kernel(SkinnyParams p, int ntiles, int S, int R) {
  __shared__ float red_all[4][64][17];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nrg = (R + 63) / 64;
  const int gw = blockIdx.x * 4 + wid;
  const int tile = gw / nrg, rg = gw % nrg;
  if (tile >= ntiles) return;  // wave-uniform; no workgroup barrier below
  const int r = rg * 64 + lane;
  const int rc = min(r, max(p.M - 1, 0));
  wide::EpiIn<1> ein;
  wide::epi_load<T, EPI, 1>(p, tile, rg * 64, 64, R, lane, ein);
  f32x4 sum[4] = {};
  for (int k0 = 0; k0 < S; k0 += 4) {
    f32x4 part[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int s = min(k0 + u, S - 1);
      const f32x4* src =
          reinterpret_cast<const f32x4*>(p.sk_ws + ((static_cast<int64_t>(tile) * S + s) * R + rc) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) part[u][q] = src[q];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) sum[q] += (k0 + u < S) ? part[u][q] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float(*red)[17] = red_all[wid];
#pragma unroll
  for (int n = 0; n < 16; ++n) red[lane][n] = sum[n >> 2][n & 3];
  wide::epi_apply<T, EPI, 1>(p, tile, red, nullptr, rg * 64, false, ein);
}

template <typename T>
static int launch_reduce(int epi, const SkinnyParams& p, int ntiles, int S, int R,
                         hipStream_t st) {
  const dim3 grid((ntiles * ((R + 63) / 64) + 3) / 4), blk(256);
  switch (epi) {
    case EPI_PLAIN: midm_reduce_kernel<T, EPI_PLAIN><<<grid, blk, 0, st>>>(p, ntiles, S, R); return 0;
    case EPI_RESADD: midm_reduce_kernel<T, EPI_RESADD><<<grid, blk, 0, st>>>(p, ntiles, S, R); return 0;
    default: return -1;
  }
}

#define ATTA_MIDM_DECL(N)                                                                     \
  int launch_b_##N(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p, const Geo& g,   \
                   int dtype);
ATTA_MIDM_DECL(3)
ATTA_MIDM_DECL(4)
ATTA_MIDM_DECL(5)
ATTA_MIDM_DECL(6)
ATTA_MIDM_DECL(8)
ATTA_MIDM_DECL(10)
ATTA_MIDM_DECL(12)

constexpr int kBuilt[] = {3, 4, 5, 6, 8, 10, 12};

static int launch_tu(int bmt, int epi, dim3 grid, hipStream_t st, const SkinnyParams& p,
                     const Geo& g, int dtype) {
  switch (bmt) {
    case 3: return launch_b_3(epi, grid, st, p, g, dtype);
    case 4: return launch_b_4(epi, grid, st, p, g, dtype);
    case 5: return launch_b_5(epi, grid, st, p, g, dtype);
    case 6: return launch_b_6(epi, grid, st, p, g, dtype);
    case 8: return launch_b_8(epi, grid, st, p, g, dtype);
    case 10: return launch_b_10(epi, grid, st, p, g, dtype);
    case 12: return launch_b_12(epi, grid, st, p, g, dtype);
    default: return -1;
  }
}

// Cost model of one plan (us): rounds of the grid over the 256 CUs x a workgroup's time - the
// larger of its MFMA time and its operand bytes at a per-CU load rate - plus ramp; a split
// adds the slab stores and the reduce launch.  Constants fitted to the round-6 sweep of every
// (row block, split) plan at the 8B shapes, 188-475 rows (profiles/r6_midm_sweep.txt): a
// workgroup streams ~52 GB/s and keeps the MFMA pipe ~35 % busy; split-K costs ~6 us plus
// its slab traffic.
struct Cost {
  double mfma_eff = 0.35, cu_bps = 52e3, ramp = 2.0, red_fixed = 6.0, red_bps = 1.5e6;
};

static double plan_cost(const Cost& c, int M, int ntiles, int K, int bmt, int S, bool w8) {
  const int bm = 16 * bmt;
  const int nrb = (M + bm - 1) / bm;
  const int ncb = (ntiles + kTPB - 1) / kTPB;
  const double wgs = static_cast<double>(nrb) * ncb * S;
  const double rounds = std::ceil(wgs / 256.0);
  const double ks = static_cast<double>(K) / S;
  const double t_mfma = bm * 128.0 * ks / (2048.0 * c.mfma_eff) / 2400.0;
  const double t_load = (bm * 2.0 + 128.0 * (w8 ? 1.0 : 2.0)) * ks / c.cu_bps;
  double t = rounds * ((t_mfma > t_load ? t_mfma : t_load) + c.ramp);
  if (S > 1) {
    const int R = (M + 15) / 16 * 16;
    t += c.red_fixed + static_cast<double>(ntiles) * S * R * 64.0 / c.red_bps;
  }
  return t;
}

static void plan(int M, int ntiles, int K, bool can_split, bool norm, bool w8,
                 int64_t ws_floats, int& bmt, int& S) {
  static const Cost c;
  const int nch = K / kKC;
  const int R = (M + 15) / 16 * 16;
  double best = 1e30;
  bmt = 6;
  S = 1;
  for (int b : kBuilt) {
    if (norm && !norm_fits(b)) continue;
    for (int s = 1; s <= (can_split ? 8 : 1); ++s) {
      if (nch / s < 2) break;
      if (s > 1 && static_cast<int64_t>(ntiles) * s * R * 16 > ws_floats) break;
      const double t = plan_cost(c, M, ntiles, K, b, s, w8);
      if (t < best - 1e-9) {
        best = t;
        bmt = b;
        S = s;
      }
    }
  }
}

}  // namespace midm
}  // namespace atta

using namespace atta;

// the NEXT mid-M launch's plan (tuning sweeps); 0 = planned
static int g_midm_bmt = 0, g_midm_ksplit = 0;
void atta_set_midm_plan(int bmt, int ksplit) {
  g_midm_bmt = bmt;
  g_midm_ksplit = ksplit;
}


int atta_midm_plan(int M, int ntiles, int K, int epi, int64_t ws_floats, int* bmt, int* ksplit) {
  const bool can_split = epi == EPI_PLAIN || epi == EPI_RESADD;
  midm::plan(M, ntiles, K, can_split, !can_split, false, ws_floats, *bmt, *ksplit);
  return 0;
}

// Launch the mid-M kernel for a SkinnyParams filled by a gemv.hip entry point (x, w
// pre-shuffled 16-bit or fp8 with p.wscale, y / epilogue fields, eps, M, N, K).  ntiles: 16-column weight tiles
// (SiLU: inter / 8).  Returns 0, -1 (unsupported shape / plan) or -2 (split-K workspace).
int atta_midm_launch(SkinnyParams& p, int epi, int ntiles, int dtype, float* sk_ws,
                     int64_t ws_floats, hipStream_t stream) {
  if (p.M < 1 || p.K % midm::kKC != 0 || !p.ps) return -1;
  if (epi != EPI_PLAIN && epi != EPI_RESADD && epi != EPI_QKVROPE && epi != EPI_SILU) return -1;
  const bool can_split = epi == EPI_PLAIN || epi == EPI_RESADD;
  int bmt = g_midm_bmt, S = g_midm_ksplit;
  g_midm_bmt = g_midm_ksplit = 0;
  if (bmt <= 0 || S <= 0)
    midm::plan(p.M, ntiles, p.K, can_split, p.eps > 0.f, p.wscale != nullptr,
               sk_ws ? ws_floats : 0, bmt, S);
  if (S > 1 && !can_split) return -1;
  if (S < 1 || p.K / midm::kKC < S) return -1;
  // a split whose slabs do not fit the workspace is halved until they do (forced plans)
  const int64_t rpad = (p.M + 15) / 16 * 16;
  while (S > 1 && static_cast<int64_t>(ntiles) * S * rpad * 16 > (sk_ws ? ws_floats : 0)) S >>= 1;
  midm::Geo g;
  g.S = S;
  g.ntiles = ntiles;
  g.nrb = (p.M + 16 * bmt - 1) / (16 * bmt);
  g.ncb = (ntiles + midm::kTPB - 1) / midm::kTPB;
  g.R = (p.M + 15) / 16 * 16;
  if (S > 1) {
    if (sk_ws == nullptr) return -2;
    if (static_cast<int64_t>(ntiles) * S * g.R * 16 > ws_floats) return -2;
    p.sk_ws = sk_ws;
  }
  p.ksplit = S;
  const int64_t nwg = static_cast<int64_t>(g.nrb) * g.ncb * S;
  if (nwg > 0x7fffffff) return -1;
  const dim3 grid(static_cast<unsigned>(nwg));
  int rc = midm::launch_tu(bmt, epi, grid, stream, p, g, dtype);
  if (rc) return rc;
  if (S > 1) {
    rc = dtype == 0 ? midm::launch_reduce<__bf16>(epi, p, ntiles, S, g.R, stream)
                    : midm::launch_reduce<_Float16>(epi, p, ntiles, S, g.R, stream);
    if (rc) return rc;
  }
  return static_cast<int>(hipGetLastError());
}
