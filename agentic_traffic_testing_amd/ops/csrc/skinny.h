// Skinny (decode) GEMM body of the GEMV kernels (gemv.hip: launchers and design notes),
// one 16-output-row tile per call - kept in a header so a persistent or fused launch can
// reuse it (the fused qkv + attention launch that did was measured slower and removed:
// profiles/r2_fused_qkv_attn_experiment.txt).
#pragma once

#include "common.h"

namespace atta {

enum Epi {
  EPI_PLAIN = 0,
  EPI_RESADD = 1,
  EPI_QKVROPE = 2,
  EPI_SILU = 3,
  EPI_SAMPLE = 4
};

template <typename T>
struct MfmaK32;
template <>
struct MfmaK32<__bf16> {
  typedef bf16x8 frag8;
  __device__ static __forceinline__ f32x4 mma(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  // sum of squares of the 8 activations (fused RMSNorm): bf16 -> f32 is a shift / mask,
  // the squares go through packed FMAs (v_pk_fma_f32, two per instruction).  (v_dot2c_f32_bf16
  // was measured 1.6 % high on this use - rounds its products - and is not used.)
  __device__ static __forceinline__ float sq8(frag8 a, float s) {
    const u32x4 w = __builtin_bit_cast(u32x4, a);
    f32x2_t acc = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2_t v = {__uint_as_float(w[j] << 16), __uint_as_float(w[j] & 0xffff0000u)};
      acc = __builtin_elementwise_fma(v, v, acc);
    }
    return s + (acc[0] + acc[1]);
  }
};
template <>
struct MfmaK32<_Float16> {
  typedef f16x8 frag8;
  __device__ static __forceinline__ f32x4 mma(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ float sq8(frag8 a, float s) {
    f32x2_t acc = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2_t v = {static_cast<float>(a[2 * j]), static_cast<float>(a[2 * j + 1])};
      acc = __builtin_elementwise_fma(v, v, acc);
    }
    return s + (acc[0] + acc[1]);
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
  // wide / mid-M split-K slabs in bf16 instead of fp32 (half the slab write + reduce read
  // traffic; each slice's partial rounded once before the fp32 slice-ordered sum)
  int sk_half;
  // optional per-workgroup timeline (ops.set_gemv_trace): [start, end] on the 100 MHz wall
  // clock per workgroup of the grid (gridDim.y == 1 launches only)
  unsigned long long* wg_trace;
  // TP row-parallel GEMV with the all-reduce push fused (allreduce.hip push_reduce_kernel):
  // push_world > 0 turns the PLAIN epilogue into "write this tile into slot (parity,
  // push_rank) of every rank's IPC buffer, fence, bump that rank's tile counter for this
  // source" - the [M, N] product never lands in local memory
  uint8_t* push_base[arl::kMaxRanks];
  int push_world, push_rank;
  int64_t push_max_elems;
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

// Epilogue of one 16-column output tile from its fp32 accumulator tile red[row][col] (rows
// < p.M are valid; inv_rms[row] = the fused RMSNorm scale when norm), run by `nthr` threads
// (tid = 0..nthr-1): the whole workgroup of the skinny GEMV, or one wave of the wide small-M
// GEMM (wide.hip).  Rows past p.M are skipped, so MTMAX only bounds the loops.
template <typename T, int EPI, int MTMAX = 8>
__device__ __forceinline__ void tile_epilogue(const SkinnyParams& p, const int tile,
                                              const float (*red)[17], const float* inv_rms,
                                              const bool norm, const int tid, const int nthr) {
  if constexpr (EPI == EPI_PLAIN || EPI == EPI_RESADD) {
    for (int e = tid; e < 16 * 16 * MTMAX; e += nthr) {
      const int m = e >> 4, n = e & 15;
      if (m >= p.M) continue;
      float v = red[m][n];
      if (norm) v *= inv_rms[m];
      uint16_t* dst = p.y + static_cast<int64_t>(m) * p.y_stride + tile * 16 + n;
      if constexpr (EPI == EPI_RESADD) v = to_f32<T>(from_f32<T>(v)) + to_f32<T>(*dst);
      *dst = from_f32<T>(v);
    }
  } else if constexpr (EPI == EPI_SILU) {
    for (int e = tid; e < 16 * 8 * MTMAX; e += nthr) {
      const int m = e >> 3, j = e & 7;
      if (m >= p.M) continue;
      const float sc = norm ? inv_rms[m] : 1.f;
      const float g = to_f32<T>(from_f32<T>(red[m][j] * sc));
      const float u = to_f32<T>(from_f32<T>(red[m][j + 8] * sc));
      const float si = to_f32<T>(from_f32<T>(g / (1.f + __expf(-g))));
      p.y[static_cast<int64_t>(m) * p.y_stride + tile * 8 + j] = from_f32<T>(si * u);
    }
  } else if constexpr (EPI == EPI_QKVROPE) {
    const int head = tile >> 3, jb = (tile & 7) * 8;
    const int nq = p.n_q_heads, nkv = p.n_kv_heads;
    const int BS = 1 << p.bs_shift;
    for (int e = tid; e < 16 * 8 * MTMAX; e += nthr) {
      const int m = e >> 3, c = e & 7;
      if (m >= p.M) continue;
      const float sc = norm ? inv_rms[m] : 1.f;
      // GEMM output rounded to T first (matches the unfused F.linear -> rope path)
      const float x1 = to_f32<T>(from_f32<T>(red[m][c] * sc));
      const float x2 = to_f32<T>(from_f32<T>(red[m][c + 8] * sc));
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
    for (int e = tid; e < 16 * 16 * MTMAX; e += nthr) {
      const int m = e >> 4, n = e & 15;
      unsigned long long key = 0ull;
      if (m < p.M) {
        const float sc = norm ? inv_rms[m] : 1.f;
        float v = to_f32<T>(from_f32<T>(red[m][n] * sc));  // bf16 logits, as F.linear
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
__device__ __forceinline__ void skinny_body(const SkinnyParams& p, const int tile, const int ks,
                                            const int ksplit) {
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
  const int kslice = p.K / ksplit;
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
        if (norm) ss[t] = MF::sq8(xf[u], ss[t]);
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
        if (norm) ss[t] = MF::sq8(x1, MF::sq8(x0, ss[t]));
      }
    }
  } else {
    for (int k = nsteps * STEP; k < kw; k += 32) {  // tail (K not a multiple of the stage)
      const frag8 wf = *reinterpret_cast<const frag8*>(wp + woff(k));
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const frag8 xf = xv[t] ? *reinterpret_cast<const frag8*>(xp[t] + k) : frag8{};
        acc[t] = MF::mma(xf, wf, acc[t]);
        if (norm) ss[t] = MF::sq8(xf, ss[t]);
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
  if (ksplit > 1) {
    // ---- split-K hand-over (device-scope sc1 stores/loads + arrival counter, no fences:
    // common.h "device-coherent hand-over"); slot = R*16 partial sums + R row sums of squares
    constexpr int kSlot = R * 16 + R;
    const auto rws = dev_rsrc(p.sk_ws);
    const uint32_t mine = static_cast<uint32_t>((tile * ksplit + ks) * kSlot) * 4u;
    for (int e = threadIdx.x; e < R * 16; e += WAVES * 64)
      if ((e >> 4) < p.M) dev_store4(rws, mine + e * 4, red[0][e >> 4][e & 15]);
    if (norm && threadIdx.x < R && threadIdx.x < p.M)
      dev_store4(rws, mine + (R * 16 + threadIdx.x) * 4, inv_rms[threadIdx.x]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores acknowledged
    __syncthreads();
    if (threadIdx.x == 0) {
      const int old = __hip_atomic_fetch_add(p.sk_counters + tile, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      sk_last = (old == ksplit - 1);
    }
    __syncthreads();
    if (!sk_last) return;  // block-uniform
    const uint32_t first = static_cast<uint32_t>(tile * ksplit * kSlot) * 4u;
    for (int e = threadIdx.x; e < R * 16; e += WAVES * 64) {
      if ((e >> 4) >= p.M) continue;
      float s = 0.f;
      for (int q = 0; q < ksplit; ++q) s += dev_load4(rws, first + (q * kSlot + e) * 4);
      red[0][e >> 4][e & 15] = s;
    }
    if (norm && threadIdx.x < R && threadIdx.x < p.M) {
      float s = 0.f;
      for (int q = 0; q < ksplit; ++q)
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
  if constexpr (EPI == EPI_PLAIN) {
    if (p.push_world > 0) {
      // generation of this call = the receive kernel's last completed generation + 1 (read
      // from this rank's own buffer; stream order makes the previous call's value final)
      const uint32_t gen = __hip_atomic_load(reinterpret_cast<const uint32_t*>(
                                                 p.push_base[p.push_rank] + arl::kGenOffset),
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
      const int par = gen & 1;
      for (int e = threadIdx.x; e < R * 16; e += WAVES * 64) {
        const int m = e >> 4, n = e & 15;
        if (m >= p.M) continue;
        float v = red[0][m][n];
        if (norm) v *= inv_rms[m];
        const uint16_t o = from_f32<T>(v);
        const int64_t off = (static_cast<int64_t>(par) * arl::kMaxRanks + p.push_rank) *
                                p.push_max_elems + static_cast<int64_t>(m) * p.N + tile * 16 + n;
        for (int q = 0; q < p.push_world; ++q)
          reinterpret_cast<uint16_t*>(p.push_base[q] + arl::kSlotOffset)[off] = o;
      }
      __threadfence_system();  // this tile's stores reach every peer before its counter bump
      __syncthreads();
      if (threadIdx.x < p.push_world)
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(
                                   p.push_base[threadIdx.x] + arl::kPushOffset + 64 * p.push_rank),
                               1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
  tile_epilogue<T, EPI, MT>(p, tile, red[0], inv_rms, norm, threadIdx.x, WAVES * 64);
}

}  // namespace atta
