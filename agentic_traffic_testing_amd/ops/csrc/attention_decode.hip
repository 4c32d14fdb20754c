// Decode paged attention: split-K over context partitions with an in-kernel combine
// (guide §5 "In-launch split-K reduction").
//
// grid = (seqs, kv_heads, max_partitions); a workgroup of WAVES waves owns one partition of
// WAVES * 16 * TPW tokens of one (sequence, KV head).  Decode attention at agent-workload
// sizes is LATENCY bound (a few MB of KV per layer), so the kernel minimises dependent
// memory round trips per wave:
//   1. Q fragment + the block-table entries of the wave's TPW tiles are loaded together;
//   2. the K/V fragments of ALL the wave's tiles are issued at once (no per-tile
//      block-table -> K/V dependency chain);
//   3. online softmax + PV over the tiles, one LDS merge of the WAVES partial states.
// The GQA group's G query heads are the MFMA columns (swapped QK^T, see attention.hip), so
// K/V are read once for all G heads.  Partitions past the sequence end exit immediately,
// so a hipGraph captured with the maximum partition count costs nothing for short contexts.
//
// Combine: with more than one partition each workgroup writes (O normalised, lse) fp32 to a
// workspace with device-scope stores and arrives on a per-(seq, kv-head) counter; the last
// arriver reads every partition back with device-scope loads, merges them and writes the
// bf16 output, then re-arms the counter (counters are zeroed once at allocation).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace atta {
namespace dec {

constexpr int kD = 128;
constexpr float kNegInf = -__builtin_huge_valf();

template <typename T>
struct Mf;
template <>
struct Mf<__bf16> {
  typedef bf16x8 frag8;
  __device__ static __forceinline__ f32x4 qk(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ f32x4 pv(i16x4 a, i16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  }
};
template <>
struct Mf<_Float16> {
  typedef f16x8 frag8;
  __device__ static __forceinline__ f32x4 qk(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ f32x4 pv(i16x4 a, i16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, a),
                                                 __builtin_bit_cast(f16x4, b), c, 0, 0, 0);
  }
};

struct DecParams {
  uint16_t* out;
  float* part_out;  // [S, Hkv, P, 16, D]
  float* part_lse;  // [S, Hkv, P, 16]
  int* counters;    // [S, Hkv]
  const uint16_t* q;
  const uint16_t* k_cache;
  const uint16_t* v_cache;
  const int* block_tables;
  const int* seq_kvlen;
  const int* seq_qstart;
  int64_t q_stride, out_stride;
  int bt_stride, n_kv_heads, bs_shift, part_tokens, max_parts;
  float scale_log2;
  // optional per-workgroup timeline (100 MHz wall clock): [start, past-wait, end, hw id]
  unsigned long long* wg_trace;
};

template <typename T>
struct TileFrags {
  typename Mf<T>::frag8 k[4];
  i16x4 v[8];
};

template <typename T, int G, int WAVES, int TPW>
__device__ __forceinline__ void decode_attention_body(const DecParams& p, const int s,
                                                      const int hk, const int part,
                                                      unsigned long long (&tr)[3]) {
  using frag8 = typename Mf<T>::frag8;
  __shared__ float lds_o[WAVES][G][kD + 4];
  __shared__ float lds_m[WAVES][G];
  __shared__ float lds_l[WAVES][G];
  __shared__ int lds_last;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int col = lane & 15;
  const int grp = lane >> 4;
  const int PT = WAVES * 16 * TPW;
  const int kv_begin = part * PT;
  // ---- round trip 1: sequence length, query row and the block-table entries of this wave's
  // tiles are independent loads - the entries are fetched unconditionally (index clamped to
  // the table row) and only used for tiles inside the sequence
  const int* bt = p.block_tables + static_cast<int64_t>(s) * p.bt_stride;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);  // wave-uniform -> scalar loads
  int kt[TPW], bte[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    kt[i] = kv_begin + (wid_u + i * WAVES) * 16;
    bte[i] = bt[min(kt[i] >> p.bs_shift, p.bt_stride - 1)];
  }
  int kvlen = p.seq_kvlen[s];
  int qrow = p.seq_qstart[s + 1] - 1;
  // one wait for all of them (keeps the compiler from chaining the loads behind branches)
  asm volatile("" : "+s"(kvlen), "+s"(qrow));
#pragma unroll
  for (int i = 0; i < TPW; ++i) asm volatile("" : "+s"(bte[i]));
  // timeline probe: clock reads only after the scalar loads above - an earlier one makes
  // them vector loads, which the scalar-operand asm cannot take
  tr[0] = wall_clock64();
  const int nparts = (kvlen + PT - 1) / PT;
  if (part >= nparts) return;  // block-uniform (also kvlen == 0 dummy sequences)
  const int kv_end = min(kvlen, kv_begin + PT);
  const int BS = 1 << p.bs_shift;
  const int64_t hs = static_cast<int64_t>(BS) * kD;
  int page[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) page[i] = kt[i] < kv_end ? bte[i] : 0;

  // ---- round trip 2: Q fragment (needs the query row) + K/V fragments of all tiles --------
  frag8 qf[4];
  {
    const bool ok = col < G;
    const uint16_t* qp = p.q + static_cast<int64_t>(qrow) * p.q_stride +
                         static_cast<int64_t>(hk * G + (ok ? col : 0)) * kD + 32 * grp;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      qf[kk] = ok ? *reinterpret_cast<const frag8*>(qp + 8 * kk) : frag8{};
  }

  TileFrags<T> f[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    if (kt[i] < kv_end) {
      const uint16_t* base = p.k_cache + (static_cast<int64_t>(page[i]) * p.n_kv_heads + hk) * hs;
      const uint16_t* kp = base + static_cast<int64_t>((kt[i] + col) & (BS - 1)) * kD + 32 * grp;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) f[i].k[kk] = *reinterpret_cast<const frag8*>(kp + 8 * kk);
      const uint16_t* vb = p.v_cache + (static_cast<int64_t>(page[i]) * p.n_kv_heads + hk) * hs;
      const uint16_t* vp = vb + static_cast<int64_t>(col) * BS + ((kt[i] + 4 * grp) & (BS - 1));
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
        f[i].v[dt] = *reinterpret_cast<const i16x4*>(vp + static_cast<int64_t>(16 * dt) * BS);
    }
  }

  // ---- compute --------------------------------------------------------------------------
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = kNegInf, l_run = 0.f;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    if (kt[i] >= kv_end) break;  // wave-uniform
    const TileFrags<T>& ft = f[i];
    const int kbase = kt[i];
    const int kend = kv_end;
    f32x4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) sacc = Mf<T>::qk(ft.k[kk], qf[kk], sacc);
    float sv[4], tmax = kNegInf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sv[j] = (kbase + 4 * grp + j < kend) ? sacc[j] * p.scale_log2 : kNegInf;
      tmax = fmaxf(tmax, sv[j]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, kWave));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, kWave));
    const float m_new = fmaxf(m_run, tmax);
    const float m_use = (m_new == kNegInf) ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    float psum = 0.f;
    i16x4 pf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float pv = exp2f(sv[j] - m_use);
      psum += pv;
      pf[j] = static_cast<short>(from_f32<T>(pv));
    }
    psum += __shfl_xor(psum, 16, kWave);
    psum += __shfl_xor(psum, 32, kWave);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    // keys past the sequence end (the tail slots of its last page) hold stale bytes of the
    // page's previous owner: P is 0 there, and V is zeroed too so a non-finite stale value
    // cannot make 0 * V a NaN (wave-uniform edge test: the last tile only)
    i16x4 vv[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) vv[dt] = ft.v[dt];
    if (kbase + 16 > kend) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (kbase + 4 * grp + j >= kend) {
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) vv[dt][j] = 0;
        }
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      o[dt] *= alpha;
      o[dt] = Mf<T>::pv(vv[dt], pf, o[dt]);
    }
  }
  tr[1] = wall_clock64();

  // ---- merge the WAVES partial states (only the G valid columns) ---------------------------
  if (col < G) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) lds_o[wid][col][16 * dt + 4 * grp + j] = o[dt][j];
    if (grp == 0) {
      lds_m[wid][col] = m_run;
      lds_l[wid][col] = l_run;
    }
  }
  __syncthreads();
  const bool merger = threadIdx.x < G * 16;
  const int c = threadIdx.x >> 4;          // column (query head in the group)
  const int d0 = (threadIdx.x & 15) * 8;   // dims d0..d0+7
  float r[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float mu = 0.f, L = 0.f;
  if (merger) {
    float mx = kNegInf;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) mx = fmaxf(mx, lds_m[w][c]);
    mu = (mx == kNegInf) ? 0.f : mx;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      const float fw = exp2f(lds_m[w][c] - mu);
      L += fw * lds_l[w][c];
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] += fw * lds_o[w][c][d0 + j];
    }
    const float invL = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] *= invL;
  }
  uint16_t* outp = p.out + static_cast<int64_t>(qrow) * p.out_stride +
                   static_cast<int64_t>(hk * G + c) * kD + d0;
  if (nparts == 1) {
    if (merger) {
      Pack8 o8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o8.v[j] = from_f32<T>(r[j]);
      *reinterpret_cast<Pack8*>(outp) = o8;
    }
    return;
  }

  // ---- publish this partition; the last arriver combines -----------------------------------
  // Partials travel with device-scope (sc1) buffer stores/loads (common.h "device-coherent
  // hand-over"): no agent-scope release/acquire, i.e. no whole-L2 writeback/invalidate per
  // workgroup - 12.6 -> 10.2 us at ctx 1000, 24.3 -> 16.0 us at ctx 2000 (B = 5,
  // profiles/r1_fused_attn_oproj_experiment.txt).
  const int64_t sh = static_cast<int64_t>(s) * p.n_kv_heads + hk;
  const auto rpo = dev_rsrc(p.part_out);
  const auto rpl = dev_rsrc(p.part_lse);
  if (merger) {
    const int64_t base = (sh * p.max_parts + part) * 16 + c;
    const uint32_t off = static_cast<uint32_t>((base * kD + d0) * 4);
    dev_store16(rpo, off, __builtin_bit_cast(u32x4, f32x4{r[0], r[1], r[2], r[3]}));
    dev_store16(rpo, off + 16, __builtin_bit_cast(u32x4, f32x4{r[4], r[5], r[6], r[7]}));
    if ((threadIdx.x & 15) == 0)
      dev_store4(rpl, static_cast<uint32_t>(base * 4), (L > 0.f) ? (mu + log2f(L)) : kNegInf);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // device-scope stores acknowledged
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(p.counters + sh, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    lds_last = (old == nparts - 1);
  }
  __syncthreads();
  tr[2] = wall_clock64();
  if (!lds_last) return;
  // merge in one round trip for <= 4 * NG partitions: the workgroup's threads form NG merge
  // groups of G * 16 (one thread per (head, 8 dims)); group g loads partitions g, g + NG, ...
  // (4 per round trip) and folds them into a running (max, weight sum, weighted sum); the
  // group states meet in LDS and group 0 folds them in group order (fixed order: the
  // output does not depend on timing or on the launch's partition grid).  Was: the 64
  // merger threads alone, 4 partitions per dependent round trip (12 partitions at 3k tokens
  // = 3 round trips).
  {
    constexpr int MG = G * 16;
    constexpr int NG_ALL = WAVES * 64 / MG;
    constexpr int NG = NG_ALL < 16 ? NG_ALL : 16;
    __shared__ float lds_mg[NG][10][MG];
    const int gidx = threadIdx.x / MG;
    const int lt = threadIdx.x % MG;
    const int mc = lt >> 4;
    const int md0 = (lt & 15) * 8;
    const int np = min(nparts, 64);
    float m_run = kNegInf, wsum = 0.f;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // partitions per round trip per thread: 8 when there are few merge groups (4-wave
    // workgroups: NG = 4 covers 32 partitions - a 4k context at 128-token partitions - in
    // one round trip), else 4
    constexpr int PPI = NG <= 4 ? 8 : 4;
    if (gidx < NG) {
      for (int u0 = 0; gidx + NG * u0 < np; u0 += PPI) {
        float lse[PPI];
        f32x4 pa[PPI], pb[PPI];
#pragma unroll
        for (int u = 0; u < PPI; ++u) {
          const int q = min(gidx + NG * (u0 + u), np - 1);
          const int64_t base = (sh * p.max_parts + q) * 16 + mc;
          const uint32_t off = static_cast<uint32_t>((base * kD + md0) * 4);
          lse[u] = dev_load4(rpl, static_cast<uint32_t>(base * 4));
          pa[u] = __builtin_bit_cast(f32x4, dev_load16(rpo, off));
          pb[u] = __builtin_bit_cast(f32x4, dev_load16(rpo, off + 16));
        }
#pragma unroll
        for (int u = 0; u < PPI; ++u) {
          if (gidx + NG * (u0 + u) >= np || lse[u] == kNegInf) continue;  // weight 0
          const float m_new = fmaxf(m_run, lse[u]);
          const float sc = exp2f(m_run - m_new);  // m_run == -inf -> 0
          const float w = exp2f(lse[u] - m_new);
          wsum = wsum * sc + w;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            acc[jj] = acc[jj] * sc + w * pa[u][jj];
            acc[4 + jj] = acc[4 + jj] * sc + w * pb[u][jj];
          }
          m_run = m_new;
        }
      }
      lds_mg[gidx][0][lt] = m_run;
      lds_mg[gidx][1][lt] = wsum;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) lds_mg[gidx][2 + jj][lt] = acc[jj];
    }
    __syncthreads();
    if (gidx == 0) {
      for (int g = 1; g < NG; ++g) {
        const float gm = lds_mg[g][0][lt];
        if (gm == kNegInf) continue;
        const float m_new = fmaxf(m_run, gm);
        const float sc = exp2f(m_run - m_new);
        const float w = exp2f(gm - m_new);
        wsum = wsum * sc + w * lds_mg[g][1][lt];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) acc[jj] = acc[jj] * sc + w * lds_mg[g][2 + jj][lt];
        m_run = m_new;
      }
      const float inv = wsum > 0.f ? 1.f / wsum : 0.f;
      Pack8 o8;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) o8.v[jj] = from_f32<T>(acc[jj] * inv);
      *reinterpret_cast<Pack8*>(p.out + static_cast<int64_t>(qrow) * p.out_stride +
                                static_cast<int64_t>(hk * G + mc) * kD + md0) = o8;
    }
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(p.counters + sh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T, int G, int WAVES, int TPW>
__global__ __launch_bounds__(WAVES * 64) void decode_attention_kernel(DecParams p) {
  unsigned long long tr[3] = {0, 0, 0};
  decode_attention_body<T, G, WAVES, TPW>(p, blockIdx.x, blockIdx.y, blockIdx.z, tr);
  // timeline probe (set_attention_trace): [past round trip 1, computed, published, end]
  if (p.wg_trace != nullptr && threadIdx.x == 0) {
    const int64_t b = blockIdx.x + static_cast<int64_t>(gridDim.x) *
                                       (blockIdx.y + static_cast<int64_t>(gridDim.y) * blockIdx.z);
    p.wg_trace[4 * b] = tr[0];
    p.wg_trace[4 * b + 1] = tr[1];
    p.wg_trace[4 * b + 2] = tr[2];
    p.wg_trace[4 * b + 3] = wall_clock64();
  }
}

template <typename T, int WAVES, int TPW>
static int launch_g(int G, dim3 grid, hipStream_t st, const DecParams& p) {
  switch (G) {
    case 1: decode_attention_kernel<T, 1, WAVES, TPW><<<grid, WAVES * 64, 0, st>>>(p); return 0;
    case 2: decode_attention_kernel<T, 2, WAVES, TPW><<<grid, WAVES * 64, 0, st>>>(p); return 0;
    case 3: decode_attention_kernel<T, 3, WAVES, TPW><<<grid, WAVES * 64, 0, st>>>(p); return 0;
    case 4: decode_attention_kernel<T, 4, WAVES, TPW><<<grid, WAVES * 64, 0, st>>>(p); return 0;
    case 8: decode_attention_kernel<T, 8, WAVES, TPW><<<grid, WAVES * 64, 0, st>>>(p); return 0;
    default: return -1;
  }
}

// part_tokens selects the workgroup shape: 64 = 4 waves x 1 tile, 128 = 8 waves x 1 tile (or
// 4 x 2, attn128_waves), 256 = 8 x 2, 512 = 16 x 2 (16 waves cap VGPRs at 128: more tiles per
// wave would spill).
// 128-token partitions (the decode batches <= 8 of the headline) run as 8 waves x 1 tile:
// half the serial QK / softmax / PV chain per wave and twice the waves in flight against
// 4 waves x 2 tiles - bench 767.9 / 769.2 vs 762.4 / 764.0 tok/s interleaved on one box
// (profiles/r5_attention_8wave.txt).  ATTA_ATTN128_WAVES=4 restores 4 x 2 (read once).
static int attn128_waves() {
  static const int w = [] {
    const char* v = std::getenv("ATTA_ATTN128_WAVES");
    return v != nullptr && std::atoi(v) == 4 ? 4 : 8;
  }();
  return w;
}

template <typename T>
static int launch(int G, int part_tokens, dim3 grid, hipStream_t st, const DecParams& p) {
  switch (part_tokens) {
    case 64: return launch_g<T, 4, 1>(G, grid, st, p);
    case 128:
      return attn128_waves() == 8 ? launch_g<T, 8, 1>(G, grid, st, p)
                                  : launch_g<T, 4, 2>(G, grid, st, p);
    case 256: return launch_g<T, 8, 2>(G, grid, st, p);
    case 512: return launch_g<T, 16, 2>(G, grid, st, p);
    default: return -1;
  }
}

}  // namespace dec
}  // namespace atta

using namespace atta;

static unsigned long long* g_attn_trace = nullptr;

// Timeline probe for the decode attention launches that follow (nullptr: off).
void atta_set_attention_trace(void* trace) {
  g_attn_trace = static_cast<unsigned long long*>(trace);
}

int atta_attention_decode_v2(void* out, float* part_out, float* part_lse, int* counters,
                             const void* q, const void* k_cache, const void* v_cache,
                             const int* block_tables, const int* seq_kvlen, const int* seq_qstart,
                             int num_seqs, int max_parts, int part_tokens, int n_q_heads,
                             int n_kv_heads, int head_dim, int block_size, int bt_stride,
                             int64_t q_stride, int64_t out_stride, float scale, int dtype,
                             hipStream_t stream) {
  const int G = n_q_heads / n_kv_heads;
  int shift = 0;
  while ((1 << shift) < block_size) ++shift;
  if (head_dim != 128 || (1 << shift) != block_size || block_size < 16) return -1;
  if (n_q_heads % n_kv_heads || G > 8 || ((G & (G - 1)) && G != 3)) return -1;
  if (max_parts < 1 || max_parts > 64) return -1;
  if (num_seqs == 0) return 0;
  dec::DecParams p{};
  p.out = static_cast<uint16_t*>(out);
  p.part_out = part_out;
  p.part_lse = part_lse;
  p.counters = counters;
  p.q = static_cast<const uint16_t*>(q);
  p.k_cache = static_cast<const uint16_t*>(k_cache);
  p.v_cache = static_cast<const uint16_t*>(v_cache);
  p.block_tables = block_tables;
  p.seq_kvlen = seq_kvlen;
  p.seq_qstart = seq_qstart;
  p.q_stride = q_stride;
  p.out_stride = out_stride;
  p.bt_stride = bt_stride;
  p.n_kv_heads = n_kv_heads;
  p.bs_shift = shift;
  p.part_tokens = part_tokens;
  p.max_parts = max_parts;
  p.scale_log2 = scale * 1.4426950408889634f;
  p.wg_trace = g_attn_trace;
  dim3 grid(num_seqs, n_kv_heads, max_parts);
  const int rc = dtype == 0 ? dec::launch<__bf16>(G, part_tokens, grid, stream, p)
                            : dec::launch<_Float16>(G, part_tokens, grid, stream, p);
  if (rc) return rc;
  return static_cast<int>(hipGetLastError());
}
