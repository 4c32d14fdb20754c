// Skinny (decode) GEMM on MFMA with fused prologue/epilogues.
//
//   acc[M, 16-col tile] = x[M, K] . W[rows(tile), K]^T          (M <= 32, W streamed once)
//
// Decode steps of the 8B model stream ~15 GB of weights per token while M (= sequences in
// the batch) is 1..16, so the layer GEMMs are pure HBM streams (guide: "GEMV / M <= 16
// decode weights: load straight to VGPRs, deep unroll, late vmcnt").  Structure:
//   * a workgroup owns one 16-column output tile; WAVES waves split K; each wave streams
//     its K slice of the tile's 16 weight rows with 16-byte loads, two register stages of
//     UNROLL loads each (software pipelined: the next stage is in flight while the current
//     one feeds the MFMAs);
//   * the 16 rows x 32 k chunk is the B operand of mfma_f32_16x16x32_bf16 (lane l: weight
//     row rows(tile, l&15), k = 8(l>>4)..+8); x rows are the A operand (lane l: row l&15,
//     L1/L2 resident; rows >= M are zeros);
//   * `rows(tile, c)` is an epilogue-defined row map, so the epilogue can see partner
//     columns without any weight permutation: RoPE pairs (d, d+64) and SwiGLU pairs
//     (gate_j, up_j) land in the same tile;
//   * RMSNorm fusion: with the norm weight folded into W on the host, the kernel only needs
//     sum(x^2) per row, accumulated from the x fragments it already loads for the MFMAs;
//     the epilogue scales by rsqrt(mean + eps);
//   * wave partials + row sums are reduced through LDS; epilogues:
//       PLAIN   y = acc                      RESADD  r += acc (residual stream, in place)
//       QKVROPE q/k rotated (RoPE) -> q buffer / paged K cache, v -> transposed V cache
//       SILU    out[:, j] = silu(gate_j) * up_j
//       SAMPLE  logits -> greedy / Gumbel-max key -> one partial max per (row, tile)
//               (sampler fused into the LM head; `sample_finalize` reduces a row's
//               partials to its token id with one workgroup per row)
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "skinny.h"

namespace atta {

template <typename T, int WAVES, int UNROLL, int MT, int EPI, bool NTL = false, bool PS = false,
          bool W8 = false>
__global__ __launch_bounds__(WAVES * 64) void skinny_kernel(SkinnyParams p) {
  unsigned long long t0 = 0;
  if (p.wg_trace != nullptr) t0 = wall_clock64();
  const int tile = blockIdx.x, ks = blockIdx.y;
  skinny_body<T, WAVES, UNROLL, MT, EPI, NTL, PS, W8>(p, tile, ks, p.ksplit);
  if (p.wg_trace != nullptr && ks == 0) {  // timeline probe (one entry per tile, bounded by
    // the tile count whatever the split): every thread's stores issued, then one stamp
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      p.wg_trace[2 * tile] = t0;
      p.wg_trace[2 * tile + 1] = wall_clock64();
    }
  }
}


// Weight-stream cache policy.  Non-temporal (nt) weight loads: every decode weight byte is
// read once per step by one CU, so keeping it out of the caches helps - but only with the
// pre-shuffled layout (one contiguous 1 KiB per wave instruction): there nt lifted the
// fan-out bench from 703 to 756 tok/s (profiles/bench_r1_v10_nt.log).  On the row-major
// layout (16 rows x 64 B per instruction) nt made every GEMV slower (gate_up 42 -> 48 us,
// profiles/bench_r1_ab_nt.log), so it stays off there.  ATTA_NT_WEIGHTS=0 disables it for
// A/B runs, =1 forces it on for row-major weights too.
static int nt_weights() {
  static const int mode = [] {
    const char* e = std::getenv("ATTA_NT_WEIGHTS");
    return e == nullptr ? -1 : (e[0] == '1' ? 1 : 0);  // -1 = default policy per layout
  }();
  return mode;
}

template <int WAVES, int UNROLL, int MT, int EPI>
static void launch_t(int dtype, dim3 grid, hipStream_t st, const SkinnyParams& p) {
  const int mode = nt_weights();
  const bool shuffled = p.ps || p.wscale != nullptr;
  const bool nt = shuffled ? mode != 0 : mode == 1;
  const dim3 blk(WAVES * 64);
#define ATTA_SK(T_, U_, NT_, PS_, W8_) \
  skinny_kernel<T_, WAVES, U_, MT, EPI, NT_, PS_, W8_><<<grid, blk, 0, st>>>(p)
  if (p.wscale != nullptr) {
    // fp8 weights (pre-shuffled by construction): a 16-byte lane load carries two K steps,
    // so the stage is twice as deep to keep the same bytes in flight per wave.  (Twice that
    // again - a wave's whole K slice in flight in its first two stages - measured slower in
    // situ: fp8 bench 986 vs 1022 tok/s, profiles/r2_ab_fp8_stage_depth.txt.)
    constexpr int U8 = UNROLL * 2;
    if (dtype == 0) {
      if (nt) ATTA_SK(__bf16, U8, true, true, true); else ATTA_SK(__bf16, U8, false, true, true);
    } else {
      if (nt) ATTA_SK(_Float16, U8, true, true, true); else ATTA_SK(_Float16, U8, false, true, true);
    }
    return;
  }
  if (dtype == 0) {
    if (p.ps && nt) ATTA_SK(__bf16, UNROLL, true, true, false);
    else if (p.ps) ATTA_SK(__bf16, UNROLL, false, true, false);
    else if (nt) ATTA_SK(__bf16, UNROLL, true, false, false);
    else ATTA_SK(__bf16, UNROLL, false, false, false);
  } else {
    if (p.ps && nt) ATTA_SK(_Float16, UNROLL, true, true, false);
    else if (p.ps) ATTA_SK(_Float16, UNROLL, false, true, false);
    else if (nt) ATTA_SK(_Float16, UNROLL, true, false, false);
    else ATTA_SK(_Float16, UNROLL, false, false, false);
  }
#undef ATTA_SK
}

template <int EPI>
static void launch_epi(int dtype, int mt, int waves, dim3 grid, hipStream_t st,
                       const SkinnyParams& p) {
  // (waves, unroll) picked from cold-cache on-device sweeps (profiles/r1_microbench_*):
  // row-major 16-bit weights: 8 x 2 for the small projections, 16 x 2 for the large ones;
  // pre-shuffled 16-bit weights: 8 waves stream best with 4-deep stages (o, down), 16 x 2
  // (gate_up, lm_head), 4 x 4 (qkv).  fp8 doubles the depth inside launch_t.
  const bool ps16 = p.ps && p.wscale == nullptr;
  if (waves == 16) {
    if (mt == 1) launch_t<16, 2, 1, EPI>(dtype, grid, st, p);
    else launch_t<16, 2, 2, EPI>(dtype, grid, st, p);
  } else if (waves == 8 && ps16) {
    if (mt == 1) launch_t<8, 4, 1, EPI>(dtype, grid, st, p);
    else launch_t<8, 4, 2, EPI>(dtype, grid, st, p);
  } else if (waves == 8) {
    if (mt == 1) launch_t<8, 2, 1, EPI>(dtype, grid, st, p);
    else launch_t<8, 2, 2, EPI>(dtype, grid, st, p);
  } else {
    if (mt == 1) launch_t<4, 4, 1, EPI>(dtype, grid, st, p);
    else launch_t<4, 4, 2, EPI>(dtype, grid, st, p);
  }
}

// Largest supported wave count <= requested that divides K into 32-wide MFMA steps.
// (fp8 weights stream 64-wide K-step pairs: granule 64, and 128 per wave at 4 waves.)
static int fit_waves(int waves, int K, bool fp8 = false) {
  if (waves != 4 && waves != 8 && waves != 16) waves = 8;
  const int gran = fp8 ? 64 : 32;
  while (waves > 4 && K % (gran * waves) != 0) waves >>= 1;
  return waves;
}

// One workgroup per row reduces the row's per-tile partial keys to the winning token.
// 1024 threads x 8 independent loads in flight cover the 8016 partials of a 128256 vocab
// in one memory round trip.
// KEY_OUT writes the row's packed key with the sign bit flipped (signed-int64 orderable) so
// TP ranks can combine their vocab shards with one int64 MAX all-reduce.
constexpr int kFinThreads = 1024;
template <bool KEY_OUT>
__global__ void __launch_bounds__(kFinThreads) sample_finalize_kernel(
    int64_t* out, const unsigned long long* keys, int n_tiles) {
  __shared__ unsigned long long red[kFinThreads / kWave];
  const int m = blockIdx.x;
  const unsigned long long* row = keys + static_cast<int64_t>(m) * n_tiles;
  unsigned long long best = 0ull;
  for (int base = 0; base < n_tiles; base += 8 * kFinThreads) {
    unsigned long long k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = base + j * kFinThreads + threadIdx.x;
      k[j] = i < n_tiles ? row[i] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) best = k[j] > best ? k[j] : best;
  }
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const unsigned long long other = __shfl_xor(best, o, kWave);
    best = other > best ? other : best;
  }
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = best;
  __syncthreads();
  if (threadIdx.x < kWave) {
    best = threadIdx.x < kFinThreads / kWave ? red[threadIdx.x] : 0ull;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const unsigned long long other = __shfl_xor(best, o, kWave);
      best = other > best ? other : best;
    }
    if (threadIdx.x == 0) {
      if constexpr (KEY_OUT)
        out[m] = static_cast<int64_t>(best ^ 0x8000000000000000ull);
      else
        out[m] = static_cast<int64_t>(0xFFFFFFFFu - static_cast<unsigned>(best & 0xFFFFFFFFull));
    }
  }
}
}  // namespace atta

using namespace atta;
// Timeline probe for the NEXT skinny launch only (nullptr: off); see SkinnyParams.wg_trace
static unsigned long long* g_gemv_trace = nullptr;
void atta_set_gemv_trace(void* trace) { g_gemv_trace = static_cast<unsigned long long*>(trace); }
static unsigned long long* take_trace() {
  unsigned long long* t = g_gemv_trace;
  g_gemv_trace = nullptr;
  return t;
}

// Rows past the 16-row-tile GEMV (33-128, pre-shuffled 16-bit weights) go to the wide
// small-M kernel (wide.hip); its (waves, split) plan is automatic unless overridden for the
// NEXT such launch by atta_set_wide_plan (tuning sweeps).
int atta_wide_launch(SkinnyParams& p, int epi, int ntiles, int waves, int ksplit, int dtype,
                     const float* sk_ws, int* sk_counters, int64_t ws_floats, int n_counters,
                     hipStream_t stream);
static int g_wide_waves = 0, g_wide_ksplit = 0;
void atta_set_wide_plan(int waves, int ksplit) {
  g_wide_waves = waves;
  g_wide_ksplit = ksplit;
}
static int wide(SkinnyParams& p, int epi, int ntiles, int dtype, hipStream_t stream);
// the wide kernel takes every call over 32 rows and, for pre-shuffled 16-bit weights, calls
// from g_wide_min_m rows (gate_up + SiLU: g_wide_min_m_silu).  At 17-32 rows the 16-row-tile
// GEMVs re-read x per weight tile in two row blocks (per layer 120-137 us vs 95-98 us wide);
// at 12-16 rows only gate_up gains (43.3 / 48.2 -> 39.3 / 39.1 us); at <= 8 rows (decode)
// the GEMVs win every projection (profiles/r5_wide_vs_skinny.txt)
static int g_wide_min_m = 17, g_wide_min_m_silu = 12;
void atta_set_wide_min_rows(int m, int m_silu) {
  g_wide_min_m = m < 1 ? 1 : m;
  g_wide_min_m_silu = m_silu < 1 ? 1 : m_silu;
}
void atta_get_wide_min_rows(int* m, int* m_silu) {
  *m = g_wide_min_m;
  *m_silu = g_wide_min_m_silu;
}
// pre-shuffled 16-bit calls of up to this many rows run the wide (<= 128) or mid-M kernels
constexpr int kMidmMaxM = 8192;
// rows one call may carry: row-major weights the 16-row-tile GEMV (<= 32); pre-shuffled
// 16-bit or fp8 weights also the wide (<= 128) and mid-M kernels
static int max_rows(int ps, const float* wscale) {
  (void)wscale;
  return !ps ? 32 : kMidmMaxM;
}
static bool use_wide(int M, int ps, const float* wscale, bool silu = false) {
  return M > 32 ||
         (ps && wscale == nullptr && M >= (silu ? g_wide_min_m_silu : g_wide_min_m));
}

static int skinny_checks(int M, int K, int waves) {
  if (M < 1 || M > 32) return -1;
  if (K % (32 * waves) != 0) return -1;
  return 0;
}

// Split-K workspace per device (ops.set_splitk_workspace): fp32 partial slots + one arrival
// counter per 16-column tile (zeroed once; the last arriver re-arms it).
struct SplitKWs {
  float* ws = nullptr;
  int* counters = nullptr;
  int64_t ws_floats = 0;
  int n_counters = 0;
};
static SplitKWs g_splitk[64];

int atta_set_splitk_ws(int device, float* ws, int* counters, int64_t ws_floats, int n_counters) {
  if (device < 0 || device >= 64) return -1;
  g_splitk[device] = SplitKWs{ws, counters, ws_floats, n_counters};
  return 0;
}

int atta_midm_launch(SkinnyParams& p, int epi, int ntiles, int dtype, float* sk_ws,
                     int64_t ws_floats, hipStream_t stream);
static int wide(SkinnyParams& p, int epi, int ntiles, int dtype, hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -2;
  const SplitKWs& w = g_splitk[dev];
  if (p.M > 128) {
    // past the wide kernel's 8 row blocks: the mid-M kernel (midm.hip, row-blocked grid)
    p.wg_trace = nullptr;
    return atta_midm_launch(p, epi, ntiles, dtype, w.ws, w.ws_floats, stream);
  }
  const int waves = g_wide_waves, ksplit = g_wide_ksplit;
  g_wide_waves = g_wide_ksplit = 0;
  p.wg_trace = take_trace();  // 4 stamps per workgroup here (wide.hip)
  return atta_wide_launch(p, epi, ntiles, waves, ksplit, dtype, w.ws, w.counters, w.ws_floats,
                          w.n_counters, stream);
}

// Resolve the split for one launch: waves fitted to the K slice (fp8: 64-wide granule), the
// split reduced until every wave's slice is whole; a split > 1 needs the device workspace.
// Returns 0 or -1 (unsupported), -2 (split requested but no / too small workspace).
static int setup_split(SkinnyParams& p, int& waves, int ksplit, int tiles, bool fp8) {
  const int gran = fp8 ? 64 : 32;
  if (ksplit < 1) ksplit = 1;
  while (ksplit > 1 && p.K % (ksplit * gran * 4) != 0) ksplit >>= 1;
  waves = fit_waves(waves, p.K / ksplit, fp8);
  if ((p.K / ksplit) % (gran * waves) != 0) return -1;
  p.ksplit = ksplit;
  if (ksplit == 1) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -2;
  const SplitKWs& w = g_splitk[dev];
  const int64_t slot = static_cast<int64_t>(p.M <= 16 ? 16 : 32) * 17;
  if (w.ws == nullptr || tiles > w.n_counters ||
      static_cast<int64_t>(tiles) * ksplit * slot > w.ws_floats)
    return -2;
  p.sk_ws = w.ws;
  p.sk_counters = w.counters;
  return 0;
}

int atta_skinny_gemm(void* y, const void* x, const void* w, const void* residual, int M, int N,
                     int K, int64_t x_stride, int64_t y_stride, int64_t res_stride, int waves,
                     int ksplit, const float* wscale, int dtype, hipStream_t stream) {
  const int ps = (dtype & kPreshuffled) ? 1 : 0;
  dtype &= ~kPreshuffled;
  if (M < 1 || M > max_rows(ps, wscale) || N % 16 != 0) return -1;
  SkinnyParams p{};
  p.ps = ps;
  p.wscale = wscale;
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.M = M;
  p.N = N;
  p.K = K;
  p.x_stride = x_stride;
  p.eps = 0.f;
  if (use_wide(M, ps, wscale)) {
    if (residual != nullptr && residual != y) return -1;
    p.y = static_cast<uint16_t*>(y);
    p.y_stride = residual != nullptr ? res_stride : y_stride;
    return wide(p, residual != nullptr ? EPI_RESADD : EPI_PLAIN, N / 16, dtype, stream);
  }
  if (const int rc = setup_split(p, waves, ksplit, N / 16, wscale != nullptr)) return rc;
  const int mt = M <= 16 ? 1 : 2;
  dim3 grid(N / 16, p.ksplit);
  p.wg_trace = take_trace();
  if (residual != nullptr) {
    // y := residual + x W^T, computed in place on the residual buffer when y == residual;
    // otherwise copy semantics are not supported (callers pass y == residual).
    if (residual != y) return -1;
    p.y = static_cast<uint16_t*>(y);
    p.y_stride = res_stride;
    launch_epi<EPI_RESADD>(dtype, mt, waves, grid, stream, p);
  } else {
    p.y = static_cast<uint16_t*>(y);
    p.y_stride = y_stride;
    launch_epi<EPI_PLAIN>(dtype, mt, waves, grid, stream, p);
  }
  return static_cast<int>(hipGetLastError());
}

// Row-parallel TP GEMV with the all-reduce push fused into its epilogue: x W^T of this rank's
// K shard goes straight into slot (parity, rank) of every rank's IPC buffer (bases[q]); the
// receive side is atta_ar_push_reduce (allreduce.hip), which also adds the residual.
int atta_skinny_gemm_push(const void* x, const void* w, int M, int N, int K, int64_t x_stride,
                          int waves, int ksplit, const float* wscale, int dtype,
                          void* const* bases, int rank, int world, int64_t max_elems,
                          hipStream_t stream) {
  const int ps = (dtype & kPreshuffled) ? 1 : 0;
  dtype &= ~kPreshuffled;
  if (M < 1 || M > 32 || N % 16 != 0) return -1;
  if ((world != 2 && world != 4 && world != 8) || rank < 0 || rank >= world ||
      static_cast<int64_t>(M) * N > max_elems)
    return -1;
  SkinnyParams p{};
  p.ps = ps;
  p.wscale = wscale;
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.M = M;
  p.N = N;
  p.K = K;
  p.x_stride = x_stride;
  p.eps = 0.f;
  for (int q = 0; q < world; ++q) p.push_base[q] = static_cast<uint8_t*>(bases[q]);
  p.push_world = world;
  p.push_rank = rank;
  p.push_max_elems = max_elems;
  if (const int rc = setup_split(p, waves, ksplit, N / 16, wscale != nullptr)) return rc;
  const int mt = M <= 16 ? 1 : 2;
  dim3 grid(N / 16, p.ksplit);
  p.wg_trace = take_trace();
  launch_epi<EPI_PLAIN>(dtype, mt, waves, grid, stream, p);
  return static_cast<int>(hipGetLastError());
}

int atta_fused_qkv_rope(void* q_out, void* k_cache, void* v_cache, const void* x, const void* w,
                        const int* positions, const int* slots, const float* cos_sin, int M,
                        int K, int64_t x_stride, int64_t q_stride, int n_q_heads, int n_kv_heads,
                        int block_size, float eps, int waves, int ksplit, const float* wscale,
                        int dtype, hipStream_t stream) {
  const int ps = (dtype & kPreshuffled) ? 1 : 0;
  dtype &= ~kPreshuffled;
  if (M < 1 || M > max_rows(ps, wscale)) return -1;
  int shift = 0;
  while ((1 << shift) < block_size) ++shift;
  if ((1 << shift) != block_size) return -1;
  SkinnyParams p{};
  p.ps = ps;
  p.wscale = wscale;
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.y = static_cast<uint16_t*>(q_out);
  p.x_stride = x_stride;
  p.y_stride = q_stride;
  p.M = M;
  p.K = K;
  p.N = (n_q_heads + 2 * n_kv_heads) * 128;
  p.eps = eps;
  p.k_cache = static_cast<uint16_t*>(k_cache);
  p.v_cache = static_cast<uint16_t*>(v_cache);
  p.positions = positions;
  p.slots = slots;
  p.cos_sin = cos_sin;
  p.n_q_heads = n_q_heads;
  p.n_kv_heads = n_kv_heads;
  p.bs_shift = shift;
  if (use_wide(M, ps, wscale)) return wide(p, EPI_QKVROPE, p.N / 16, dtype, stream);
  if (const int rc = setup_split(p, waves, ksplit, p.N / 16, wscale != nullptr)) return rc;
  dim3 grid(p.N / 16, p.ksplit);
  p.wg_trace = take_trace();
  launch_epi<EPI_QKVROPE>(dtype, M <= 16 ? 1 : 2, waves, grid, stream, p);
  return static_cast<int>(hipGetLastError());
}

int atta_fused_gate_up_silu(void* out, const void* x, const void* w, int M, int K, int inter,
                            int64_t x_stride, int64_t out_stride, float eps, int waves,
                            int ksplit, const float* wscale, int dtype, hipStream_t stream) {
  const int ps = (dtype & kPreshuffled) ? 1 : 0;
  dtype &= ~kPreshuffled;
  if (M < 1 || M > max_rows(ps, wscale) || inter % 8 != 0) return -1;
  SkinnyParams p{};
  p.ps = ps;
  p.wscale = wscale;
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.y = static_cast<uint16_t*>(out);
  p.x_stride = x_stride;
  p.y_stride = out_stride;
  p.M = M;
  p.K = K;
  p.N = 2 * inter;
  p.inter = inter;
  p.eps = eps;
  if (use_wide(M, ps, wscale, true)) return wide(p, EPI_SILU, inter / 8, dtype, stream);
  if (const int rc = setup_split(p, waves, ksplit, inter / 8, wscale != nullptr)) return rc;
  dim3 grid(inter / 8, p.ksplit);
  p.wg_trace = take_trace();
  launch_epi<EPI_SILU>(dtype, M <= 16 ? 1 : 2, waves, grid, stream, p);
  return static_cast<int>(hipGetLastError());
}

int atta_fused_lm_head_sample(int64_t* tokens, unsigned long long* keys, const void* x,
                              const void* w, int M, int N, int K, int64_t x_stride, float eps,
                              const float* temperature, const int64_t* seeds,
                              const int64_t* steps, int finalize, int vocab_offset,
                              int waves, const float* wscale, int dtype, hipStream_t stream) {
  const int ps = (dtype & kPreshuffled) ? 1 : 0;
  dtype &= ~kPreshuffled;
  waves = fit_waves(waves, K, wscale != nullptr);
  const bool wd = use_wide(M, ps, wscale) && ps && wscale == nullptr && M <= 128;
  if ((!wd && skinny_checks(M, K, waves)) || N % 16 != 0) return -1;
  SkinnyParams p{};
  p.ps = ps;
  p.wscale = wscale;
  if (wscale != nullptr && (K / waves) % 64 != 0) return -1;
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.x_stride = x_stride;
  p.M = M;
  p.N = N;
  p.K = K;
  p.eps = eps;
  p.keys = keys;
  p.key_stride = N / 16;
  p.vocab_offset = vocab_offset;
  p.ksplit = 1;
  p.temperature = temperature;
  p.seeds = seeds;
  p.steps = steps;
  if (wd) {
    if (const int rc = wide(p, EPI_SAMPLE, N / 16, dtype, stream)) return rc;
  } else {
    dim3 grid(N / 16);
    p.wg_trace = take_trace();
    launch_epi<EPI_SAMPLE>(dtype, M <= 16 ? 1 : 2, waves, grid, stream, p);
  }
  if (finalize == 1)
    sample_finalize_kernel<false><<<M, kFinThreads, 0, stream>>>(tokens, keys, N / 16);
  else if (finalize == 2)
    sample_finalize_kernel<true><<<M, kFinThreads, 0, stream>>>(tokens, keys, N / 16);
  return static_cast<int>(hipGetLastError());
}

// Tuning sweep entry: plain GEMM with a selectable (waves, unroll, load policy) variant.
int atta_skinny_variant(void* y, const void* x, const void* w, int M, int N, int K,
                        int variant, hipStream_t stream) {
  SkinnyParams p{};
  p.x = static_cast<const uint16_t*>(x);
  p.w = static_cast<const uint16_t*>(w);
  p.y = static_cast<uint16_t*>(y);
  p.x_stride = K;
  p.y_stride = N;
  p.M = M;
  p.N = N;
  p.K = K;
  p.ksplit = 1;
  if (M < 1 || M > 16 || N % 16) return -1;
  dim3 grid(N / 16);
  static const int waves_of[14] = {8, 8, 4, 4, 8, 16, 8, 16, 8, 16, 8, 16, 4, 4};
  if (variant < 0 || variant > 13 || K % (32 * waves_of[variant])) return -1;
  switch (variant) {
    case 0: skinny_kernel<__bf16, 8, 4, 1, EPI_PLAIN, true><<<grid, 512, 0, stream>>>(p); break;
    case 1: skinny_kernel<__bf16, 8, 8, 1, EPI_PLAIN, false><<<grid, 512, 0, stream>>>(p); break;
    case 2: skinny_kernel<__bf16, 4, 4, 1, EPI_PLAIN, false><<<grid, 256, 0, stream>>>(p); break;
    case 3: skinny_kernel<__bf16, 4, 8, 1, EPI_PLAIN, false><<<grid, 256, 0, stream>>>(p); break;
    case 4: skinny_kernel<__bf16, 8, 4, 1, EPI_PLAIN, false><<<grid, 512, 0, stream>>>(p); break;
    case 5: skinny_kernel<__bf16, 16, 4, 1, EPI_PLAIN, false><<<grid, 1024, 0, stream>>>(p); break;
    case 6: skinny_kernel<__bf16, 8, 2, 1, EPI_PLAIN, false><<<grid, 512, 0, stream>>>(p); break;
    case 7: skinny_kernel<__bf16, 16, 2, 1, EPI_PLAIN, false><<<grid, 1024, 0, stream>>>(p); break;
    // 8 / 9: pre-shuffled weights (w must come from ops.preshuffle)
    case 8: skinny_kernel<__bf16, 8, 2, 1, EPI_PLAIN, false, true><<<grid, 512, 0, stream>>>(p); break;
    case 9: skinny_kernel<__bf16, 16, 2, 1, EPI_PLAIN, false, true><<<grid, 1024, 0, stream>>>(p); break;
    case 10: skinny_kernel<__bf16, 8, 4, 1, EPI_PLAIN, false, true><<<grid, 512, 0, stream>>>(p); break;
    case 11: skinny_kernel<__bf16, 16, 4, 1, EPI_PLAIN, false, true><<<grid, 1024, 0, stream>>>(p); break;
    case 12: skinny_kernel<__bf16, 4, 4, 1, EPI_PLAIN, false, true><<<grid, 256, 0, stream>>>(p); break;
    case 13: skinny_kernel<__bf16, 4, 8, 1, EPI_PLAIN, false, true><<<grid, 256, 0, stream>>>(p); break;
    default: return -1;
  }
  return static_cast<int>(hipGetLastError());
}

int atta_sample_finalize(int64_t* tokens, const unsigned long long* keys, int M, int n_tiles,
                         hipStream_t stream) {
  if (M <= 0 || n_tiles <= 0) return 0;
  sample_finalize_kernel<false><<<M, kFinThreads, 0, stream>>>(tokens, keys, n_tiles);
  return static_cast<int>(hipGetLastError());
}
