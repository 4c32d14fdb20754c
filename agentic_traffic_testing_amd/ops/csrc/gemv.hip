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

namespace atta {

enum Epi { EPI_PLAIN = 0, EPI_RESADD = 1, EPI_QKVROPE = 2, EPI_SILU = 3, EPI_SAMPLE = 4 };

template <typename T>
struct MfmaK32;
template <>
struct MfmaK32<__bf16> {
  typedef bf16x8 frag8;
  __device__ static __forceinline__ f32x4 mma(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ float sq8(frag8 a) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = static_cast<float>(a[j]);
      s += v * v;
    }
    return s;
  }
};
template <>
struct MfmaK32<_Float16> {
  typedef f16x8 frag8;
  __device__ static __forceinline__ f32x4 mma(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ float sq8(frag8 a) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = static_cast<float>(a[j]);
      s += v * v;
    }
    return s;
  }
};

template <typename T>
__device__ __forceinline__ typename MfmaK32<T>::frag8 fp8x8_to_frag(uint32_t lo, uint32_t hi) {
  return fp8x8_cvt<T, typename MfmaK32<T>::frag8>(lo, hi);
}

struct SkinnyParams {
  const uint16_t* x;
  const uint16_t* w;
  uint16_t* y;  // PLAIN / RESADD (in place) / SILU output / QKVROPE q output
  int64_t x_stride, y_stride;
  int M, N, K;
  float eps;  // > 0: fused RMSNorm (norm weight folded into W)
  // QKVROPE
  uint16_t* k_cache;
  uint16_t* v_cache;
  const int* positions;
  const int* slots;
  const float* cos_sin;
  int n_q_heads, n_kv_heads, bs_shift;
  // SILU
  int inter;
  // SAMPLE
  unsigned long long* keys;  // [M, key_stride] per-tile partial maxima
  int key_stride;
  int vocab_offset;          // first vocab id of this TP rank's LM-head shard
  int ps;                    // weights pre-shuffled into the MFMA lane order (see preshuffle)
  const float* wscale;       // fp8 weights: per-output-row dequant scale (original row index)
  const float* temperature;
  const int64_t* seeds;
  const int64_t* steps;
  // split-K (gridDim.y = ksplit slices of K per 16-column tile): each slice publishes its
  // fp32 partial tile (+ row sum-of-squares) to sk_ws; the tile's last arriving slice sums
  // them in slice order (bitwise deterministic) and runs the epilogue
  int ksplit;
  float* sk_ws;
  int* sk_counters;
};

__device__ __forceinline__ unsigned ordered_bits(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ float gumbel_noise(uint64_t seed, uint64_t step, uint32_t idx) {
  const uint64_t h = mix64(seed ^ mix64(step * 0x100000001B3ull + idx));
  const float u = (static_cast<float>(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
  return -__logf(-__logf(u));
}

template <int EPI>
__device__ __forceinline__ int tile_row(int tile, int c, const SkinnyParams& p) {
  if constexpr (EPI == EPI_QKVROPE) {
    // head-dim 128: tile = head * 8 + j covers dims {8j..8j+7} and {64+8j..64+8j+7}
    const int head = tile >> 3, j = tile & 7;
    return head * 128 + j * 8 + (c & 7) + ((c & 8) ? 64 : 0);
  } else if constexpr (EPI == EPI_SILU) {
    return (c < 8) ? (tile * 8 + c) : (p.inter + tile * 8 + c - 8);
  } else {
    return tile * 16 + c;
  }
}

// Weight layouts.  Row-major [N][K]: a wave's 16-byte-per-lane load touches 16 rows x 64 B
// (16 DRAM pages per instruction).  Pre-shuffled (PS): for every 16-row tile (rows already
// permuted by tile_row<EPI>) and every 32-wide K step, the 16 x 32 block is stored as the
// 1 KiB the 64 lanes read - lane l at byte 16*l holds row (l & 15), k 8*(l >> 4)..+7 - so
// each wave load instruction is one contiguous 1 KiB and a wave streams a contiguous
// range.  ops.preshuffle builds it once at weight-load time.
//
// W8 (fp8 weights, bf16/fp16 activations, weight-only quantisation): always pre-shuffled, in
// 16-row x 64-column blocks of 1 KiB - lane l's 16 bytes are its 8 k-values of two
// consecutive 32-wide K steps - converted to 16-bit MFMA operands in registers; the
// per-row scale multiplies the reduced accumulator.  Halves the weight stream.
template <typename T, int WAVES, int UNROLL, int MT, int EPI, bool NTL = false, bool PS = false,
          bool W8 = false>
__global__ __launch_bounds__(WAVES * 64) void skinny_kernel(SkinnyParams p) {
  static_assert(!W8 || (UNROLL % 2 == 0), "fp8 weights load K-step pairs");
  using MF = MfmaK32<T>;
  using frag8 = typename MF::frag8;
  constexpr int R = MT * 16;
  __shared__ float red[WAVES][R][17];
  __shared__ float ssq[WAVES][R];
  __shared__ float inv_rms[R];
  __shared__ int sk_last;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int col = lane & 15;
  const int grp = lane >> 4;
  const int tile = blockIdx.x;
  const int ks = blockIdx.y;  // split-K slice
  const int kslice = p.K / p.ksplit;
  const int kw = kslice / WAVES;
  const int kbeg = ks * kslice + wid * kw;
  const int wrow = tile_row<EPI>(tile, col, p);
  const uint16_t* wp =
      PS ? p.w + (static_cast<int64_t>(tile) * (p.K / 32) + kbeg / 32) * 512 + lane * 8
         : p.w + static_cast<int64_t>(wrow) * p.K + kbeg + 8 * grp;
  // element offset of K-offset k (a multiple of 32) from wp in either layout
  auto woff = [](int k) { return PS ? k * 16 : k; };
  const uint8_t* wp8 = reinterpret_cast<const uint8_t*>(p.w) +
                       (static_cast<int64_t>(tile) * (p.K / 64) + kbeg / 64) * 1024 + lane * 16;
  const uint16_t* xp[MT];
  bool xv[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + col;
    xv[t] = m < p.M;
    xp[t] = p.x + static_cast<int64_t>(xv[t] ? m : 0) * p.x_stride + kbeg + 8 * grp;
  }
  f32x4 acc[MT];
  float ss[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    ss[t] = 0.f;
  }
  const bool norm = p.eps > 0.f;

  constexpr int STEP = 32 * UNROLL;
  constexpr int NRAW = W8 ? UNROLL / 2 : UNROLL;  // 16-byte loads per lane per stage
  using Raw = u32x4;                                // 16 bytes
  const int nsteps = kw / STEP;
  auto load_w = [&](Raw (&f)[NRAW], int k) {
#pragma unroll
    for (int u = 0; u < NRAW; ++u) {
      const Raw* src = W8 ? reinterpret_cast<const Raw*>(wp8 + (k + 64 * u) * 16)
                          : reinterpret_cast<const Raw*>(wp + woff(k + 32 * u));
      if constexpr (NTL)
        f[u] = __builtin_nontemporal_load(src);
      else
        f[u] = *src;
    }
  };
  auto wfrag = [&](const Raw (&f)[NRAW], int u) -> frag8 {
    if constexpr (W8) {
      const Raw r = f[u >> 1];
      return (u & 1) ? fp8x8_to_frag<T>(r[2], r[3]) : fp8x8_to_frag<T>(r[0], r[1]);
    } else {
      return *reinterpret_cast<const frag8*>(&f[u]);
    }
  };
  auto compute = [&](const Raw (&f)[NRAW], int k) {
    frag8 wf[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) wf[u] = wfrag(f, u);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      frag8 xf[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
        xf[u] = xv[t] ? *reinterpret_cast<const frag8*>(xp[t] + k + 32 * u) : frag8{};
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        acc[t] = MF::mma(xf[u], wf[u], acc[t]);
        if (norm) ss[t] += MF::sq8(xf[u]);
      }
    }
  };
  if (nsteps > 0) {
    Raw wa[NRAW], wb[NRAW];
    load_w(wa, 0);
    int s = 0;
    for (; s + 2 <= nsteps; s += 2) {
      load_w(wb, (s + 1) * STEP);
      compute(wa, s * STEP);
      if (s + 2 < nsteps) load_w(wa, (s + 2) * STEP);
      compute(wb, (s + 1) * STEP);
    }
    if (s < nsteps) compute(wa, s * STEP);
  }
  if constexpr (W8) {
    for (int k = nsteps * STEP; k < kw; k += 64) {  // tail: one 64-wide K-step pair at a time
      const Raw r = *reinterpret_cast<const Raw*>(wp8 + k * 16);
      const frag8 w0 = fp8x8_to_frag<T>(r[0], r[1]);
      const frag8 w1 = fp8x8_to_frag<T>(r[2], r[3]);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const frag8 x0 = xv[t] ? *reinterpret_cast<const frag8*>(xp[t] + k) : frag8{};
        const frag8 x1 = xv[t] ? *reinterpret_cast<const frag8*>(xp[t] + k + 32) : frag8{};
        acc[t] = MF::mma(x0, w0, acc[t]);
        acc[t] = MF::mma(x1, w1, acc[t]);
        if (norm) ss[t] += MF::sq8(x0) + MF::sq8(x1);
      }
    }
  } else {
    for (int k = nsteps * STEP; k < kw; k += 32) {  // tail (K not a multiple of the stage)
      const frag8 wf = *reinterpret_cast<const frag8*>(wp + woff(k));
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const frag8 xf = xv[t] ? *reinterpret_cast<const frag8*>(xp[t] + k) : frag8{};
        acc[t] = MF::mma(xf, wf, acc[t]);
        if (norm) ss[t] += MF::sq8(xf);
      }
    }
  }

  // ---- cross-wave reduction ------------------------------------------------------------
#pragma unroll
  for (int t = 0; t < MT; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wid][t * 16 + 4 * grp + i][col] = acc[t][i];
    if (norm) {
      float v = ss[t];
      v += __shfl_xor(v, 16, kWave);
      v += __shfl_xor(v, 32, kWave);
      if (grp == 0) ssq[wid][t * 16 + col] = v;
    }
  }
  __syncthreads();
  // inv_rms[] holds the row sum of squares until the rsqrt below
  if (norm && threadIdx.x < R) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) s += ssq[q][threadIdx.x];
    inv_rms[threadIdx.x] = s;
  }
  // sum wave partials into red[0] (fp8 weights: times the row's dequant scale)
  for (int e = threadIdx.x; e < R * 16; e += WAVES * 64) {
    const int m = e >> 4, n = e & 15;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) s += red[q][m][n];
    if constexpr (W8) s *= p.wscale[tile_row<EPI>(tile, n, p)];
    red[0][m][n] = s;
  }
  __syncthreads();
  if (p.ksplit > 1) {
    // ---- split-K hand-over (device-scope sc1 stores/loads + arrival counter, no fences:
    // common.h "device-coherent hand-over"); slot = R*16 partial sums + R row sums of squares
    constexpr int kSlot = R * 16 + R;
    const auto rws = dev_rsrc(p.sk_ws);
    const uint32_t mine = static_cast<uint32_t>((tile * p.ksplit + ks) * kSlot) * 4u;
    for (int e = threadIdx.x; e < R * 16; e += WAVES * 64)
      if ((e >> 4) < p.M) dev_store4(rws, mine + e * 4, red[0][e >> 4][e & 15]);
    if (norm && threadIdx.x < R && threadIdx.x < p.M)
      dev_store4(rws, mine + (R * 16 + threadIdx.x) * 4, inv_rms[threadIdx.x]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores acknowledged
    __syncthreads();
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(p.sk_counters + tile, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      sk_last = (old == p.ksplit - 1);
    }
    __syncthreads();
    if (!sk_last) return;  // block-uniform
    const uint32_t first = static_cast<uint32_t>(tile * p.ksplit * kSlot) * 4u;
    for (int e = threadIdx.x; e < R * 16; e += WAVES * 64) {
      if ((e >> 4) >= p.M) continue;
      float s = 0.f;
      for (int q = 0; q < p.ksplit; ++q) s += dev_load4(rws, first + (q * kSlot + e) * 4);
      red[0][e >> 4][e & 15] = s;
    }
    if (norm && threadIdx.x < R && threadIdx.x < p.M) {
      float s = 0.f;
      for (int q = 0; q < p.ksplit; ++q)
        s += dev_load4(rws, first + (q * kSlot + R * 16 + threadIdx.x) * 4);
      inv_rms[threadIdx.x] = s;
    }
    if (threadIdx.x == 0)
      __hip_atomic_store(p.sk_counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
  }
  if (norm && threadIdx.x < R)
    inv_rms[threadIdx.x] = rsqrtf(inv_rms[threadIdx.x] / static_cast<float>(p.K) + p.eps);
  __syncthreads();

  // ---- epilogues -----------------------------------------------------------------------
  if constexpr (EPI == EPI_PLAIN || EPI == EPI_RESADD) {
    for (int e = threadIdx.x; e < R * 16; e += WAVES * 64) {
      const int m = e >> 4, n = e & 15;
      if (m >= p.M) continue;
      float v = red[0][m][n];
      if (norm) v *= inv_rms[m];
      uint16_t* dst = p.y + static_cast<int64_t>(m) * p.y_stride + tile * 16 + n;
      if constexpr (EPI == EPI_RESADD) v = to_f32<T>(from_f32<T>(v)) + to_f32<T>(*dst);
      *dst = from_f32<T>(v);
    }
  } else if constexpr (EPI == EPI_SILU) {
    for (int e = threadIdx.x; e < R * 8; e += WAVES * 64) {
      const int m = e >> 3, j = e & 7;
      if (m >= p.M) continue;
      const float sc = norm ? inv_rms[m] : 1.f;
      const float g = to_f32<T>(from_f32<T>(red[0][m][j] * sc));
      const float u = to_f32<T>(from_f32<T>(red[0][m][j + 8] * sc));
      const float si = to_f32<T>(from_f32<T>(g / (1.f + __expf(-g))));
      p.y[static_cast<int64_t>(m) * p.y_stride + tile * 8 + j] = from_f32<T>(si * u);
    }
  } else if constexpr (EPI == EPI_QKVROPE) {
    const int head = tile >> 3, jb = (tile & 7) * 8;
    const int nq = p.n_q_heads, nkv = p.n_kv_heads;
    const int BS = 1 << p.bs_shift;
    for (int e = threadIdx.x; e < R * 8; e += WAVES * 64) {
      const int m = e >> 3, c = e & 7;
      if (m >= p.M) continue;
      const float sc = norm ? inv_rms[m] : 1.f;
      // GEMM output rounded to T first (matches the unfused F.linear -> rope path)
      const float x1 = to_f32<T>(from_f32<T>(red[0][m][c] * sc));
      const float x2 = to_f32<T>(from_f32<T>(red[0][m][c + 8] * sc));
      const int d = jb + c;  // < 64
      const int slot = p.slots[m];
      if (head < nq + nkv) {
        const float* cs = p.cos_sin + static_cast<int64_t>(p.positions[m]) * 128;
        const float co = cs[d], si = cs[64 + d];
        const uint16_t o1 = from_f32<T>(x1 * co - x2 * si);
        const uint16_t o2 = from_f32<T>(x2 * co + x1 * si);
        if (head < nq) {
          uint16_t* q = p.y + static_cast<int64_t>(m) * p.y_stride + head * 128;
          q[d] = o1;
          q[d + 64] = o2;
        } else if (slot >= 0) {
          const int hk = head - nq;
          uint16_t* kc = p.k_cache + ((static_cast<int64_t>(slot >> p.bs_shift) * nkv + hk) * BS +
                                      (slot & (BS - 1))) * 128;
          kc[d] = o1;
          kc[d + 64] = o2;
        }
      } else if (slot >= 0) {
        const int hk = head - nq - nkv;
        uint16_t* vc = p.v_cache + (static_cast<int64_t>(slot >> p.bs_shift) * nkv + hk) * 128 * BS +
                       (slot & (BS - 1));
        vc[static_cast<int64_t>(d) * BS] = from_f32<T>(x1);
        vc[static_cast<int64_t>(d + 64) * BS] = from_f32<T>(x2);
      }
    }
  } else if constexpr (EPI == EPI_SAMPLE) {
    // one row per thread group of 16 columns: thread e handles (m, n) and reduces over n
    for (int e = threadIdx.x; e < R * 16; e += WAVES * 64) {
      const int m = e >> 4, n = e & 15;
      unsigned long long key = 0ull;
      if (m < p.M) {
        const float sc = norm ? inv_rms[m] : 1.f;
        float v = to_f32<T>(from_f32<T>(red[0][m][n] * sc));  // bf16 logits, as F.linear
        const float t = p.temperature[m];
        const int idx = p.vocab_offset + tile * 16 + n;  // global id: TP == TP1 noise
        if (t > 1e-5f)
          v = v / t + gumbel_noise(static_cast<uint64_t>(p.seeds[m]),
                                   static_cast<uint64_t>(p.steps[m]), static_cast<uint32_t>(idx));
        key = (static_cast<unsigned long long>(ordered_bits(v)) << 32) |
              static_cast<unsigned long long>(0xFFFFFFFFu - static_cast<unsigned>(idx));
      }
      // max over the 16 columns of this row: lanes e..e+15 are contiguous in a wave
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const unsigned long long other = __shfl_xor(key, o, kWave);
        key = other > key ? other : key;
      }
      // one plain store per (row, tile): no same-address atomics across the ~8k tiles
      if (n == 0 && m < p.M) p.keys[static_cast<int64_t>(m) * p.key_stride + tile] = key;
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
    // so the stage is twice as deep to keep the same bytes in flight per wave
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
  if (M < 1 || M > 32 || N % 16 != 0) return -1;
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
  if (const int rc = setup_split(p, waves, ksplit, N / 16, wscale != nullptr)) return rc;
  const int mt = M <= 16 ? 1 : 2;
  dim3 grid(N / 16, p.ksplit);
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

int atta_fused_qkv_rope(void* q_out, void* k_cache, void* v_cache, const void* x, const void* w,
                        const int* positions, const int* slots, const float* cos_sin, int M,
                        int K, int64_t x_stride, int64_t q_stride, int n_q_heads, int n_kv_heads,
                        int block_size, float eps, int waves, int ksplit, const float* wscale,
                        int dtype, hipStream_t stream) {
  const int ps = (dtype & kPreshuffled) ? 1 : 0;
  dtype &= ~kPreshuffled;
  if (M < 1 || M > 32) return -1;
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
  if (const int rc = setup_split(p, waves, ksplit, p.N / 16, wscale != nullptr)) return rc;
  dim3 grid(p.N / 16, p.ksplit);
  launch_epi<EPI_QKVROPE>(dtype, M <= 16 ? 1 : 2, waves, grid, stream, p);
  return static_cast<int>(hipGetLastError());
}

int atta_fused_gate_up_silu(void* out, const void* x, const void* w, int M, int K, int inter,
                            int64_t x_stride, int64_t out_stride, float eps, int waves,
                            int ksplit, const float* wscale, int dtype, hipStream_t stream) {
  const int ps = (dtype & kPreshuffled) ? 1 : 0;
  dtype &= ~kPreshuffled;
  if (M < 1 || M > 32 || inter % 8 != 0) return -1;
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
  if (const int rc = setup_split(p, waves, ksplit, inter / 8, wscale != nullptr)) return rc;
  dim3 grid(inter / 8, p.ksplit);
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
  if (skinny_checks(M, K, waves) || N % 16 != 0) return -1;
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
  dim3 grid(N / 16);
  launch_epi<EPI_SAMPLE>(dtype, M <= 16 ? 1 : 2, waves, grid, stream, p);
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
