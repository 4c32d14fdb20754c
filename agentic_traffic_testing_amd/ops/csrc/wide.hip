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
//   * split-K: each slice writes its fp32 row segments and partial sums of squares with
//     plain stores and exits; a second launch (wide_reduce_kernel, one wave per tile) sums
//     them in slice order - bitwise deterministic - and runs the epilogue.  (An in-launch
//     last-arriver combine read every slice of a column block from ONE workgroup: 5-17 us
//     at 85 rows against a 1.5 us launch boundary.)
// One workgroup barrier per chunk.  Plain loads only (no LDS-DMA): mixing LDS-DMA with the
// register weight stream makes hipcc wait vmcnt(0) at every weight use (cdna_hip_programming
// §5, "Projection GEMM at M = 256" item 4(b)).
#include <cmath>

#include "common.h"
#include "kernels.h"
#include "skinny.h"

namespace atta {
namespace wide {

#ifndef ATTA_WIDE_WSTAGES
#define ATTA_WIDE_WSTAGES 4
#endif
constexpr int kDeepW = ATTA_WIDE_WSTAGES;
constexpr int kKC = 128;             // K columns per staged chunk (4 MFMA K steps)
constexpr int kRowB = kKC * 2;       // bytes of one staged x row
constexpr int kSlots = kRowB / 16;   // 16-B slots per staged row

// Epilogue of one wave's 16-column tile, one accumulator ROW per lane (rows lane and lane + 64),
// in two phases: epi_load issues every global load the epilogue needs (residual segment,
// position / slot then cos-sin, sampler parameters) as early as the kernel can - before the
// split-K arrival counter, so they overlap the hand-over - and epi_apply computes and stores
// 16-B row vectors.  (The GEMV's element-per-thread tile_epilogue, run by one wave over up to
// 128 rows, paid one dependent load round trip per element: 24 per wave at 96 rows.)
template <int RPL_>
struct EpiIn {
  static constexpr int RPL = RPL_;  // rows per lane
  int rows[RPL];
  bool ok[RPL];
  u32x4 res[RPL][2];  // RESADD: the residual row segment (16 values)
  int slot[RPL];      // QKVROPE
  f32x4 cs[RPL][4];   // QKVROPE: cos d..d+7, sin d..d+7
  float temp[RPL];    // SAMPLE
  uint64_t seed[RPL], step[RPL];
};

// rows of this lane: row0 + lane + 64 j (j < RPL) for lanes < nl, rows < rmax and < p.M
template <typename T, int EPI, int RPL>
__device__ __forceinline__ void epi_load(const SkinnyParams& p, const int tile, const int row0,
                                         const int nl, const int rmax, const int lane,
                                         EpiIn<RPL>& in) {
#pragma unroll
  for (int j = 0; j < RPL; ++j) {
    in.rows[j] = row0 + lane + 64 * j;
    in.ok[j] = lane < nl && in.rows[j] < rmax && in.rows[j] < p.M;
  }
  if constexpr (EPI == EPI_RESADD) {
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      const u32x4* src = reinterpret_cast<const u32x4*>(
          p.y + static_cast<int64_t>(in.ok[j] ? in.rows[j] : 0) * p.y_stride + tile * 16);
      in.res[j][0] = src[0];
      in.res[j][1] = src[1];
    }
  } else if constexpr (EPI == EPI_QKVROPE) {
    const int head = tile >> 3, jb = (tile & 7) * 8;
    int pos[RPL];
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      const int m = in.ok[j] ? in.rows[j] : 0;
      pos[j] = p.positions[m];
      in.slot[j] = p.slots[m];
    }
    if (head < p.n_q_heads + p.n_kv_heads) {
#pragma unroll
      for (int j = 0; j < RPL; ++j) {
        const f32x4* c4 =
            reinterpret_cast<const f32x4*>(p.cos_sin + static_cast<int64_t>(pos[j]) * 128 + jb);
        in.cs[j][0] = c4[0];
        in.cs[j][1] = c4[1];
        in.cs[j][2] = c4[16];  // + 64 floats: the sin half
        in.cs[j][3] = c4[17];
      }
    }
  } else if constexpr (EPI == EPI_SAMPLE) {
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      const int m = in.ok[j] ? in.rows[j] : 0;
      in.temp[j] = p.temperature[m];
      in.seed[j] = static_cast<uint64_t>(p.seeds[m]);
      in.step[j] = static_cast<uint64_t>(p.steps[m]);
    }
  }
}

__device__ __forceinline__ u32x4 pack8(const uint16_t (&o)[8]) {
  return u32x4{o[0] | (uint32_t(o[1]) << 16), o[2] | (uint32_t(o[3]) << 16),
               o[4] | (uint32_t(o[5]) << 16), o[6] | (uint32_t(o[7]) << 16)};
}

// red[m - rbase][n] holds row m's 16 accumulators, inv_rms[m - rbase] its norm scale
template <typename T, int EPI, int RPL>
__device__ __forceinline__ void epi_apply(const SkinnyParams& p, const int tile,
                                          const float (*red)[17], const float* inv_rms,
                                          const int rbase, const bool norm,
                                          const EpiIn<RPL>& in) {
  if constexpr (EPI == EPI_PLAIN || EPI == EPI_RESADD) {
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      if (!in.ok[j]) continue;
      const int m = in.rows[j];
      const float sc = norm ? inv_rms[m - rbase] : 1.f;
      uint16_t o[2][8];
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        float v = red[m - rbase][n] * sc;
        if constexpr (EPI == EPI_RESADD) {
          const uint32_t w = in.res[j][n >> 3][(n >> 1) & 3];
          v = to_f32<T>(from_f32<T>(v)) + to_f32<T>(static_cast<uint16_t>((n & 1) ? w >> 16 : w));
        }
        o[n >> 3][n & 7] = from_f32<T>(v);
      }
      u32x4* dst = reinterpret_cast<u32x4*>(p.y + static_cast<int64_t>(m) * p.y_stride + tile * 16);
      dst[0] = pack8(o[0]);
      dst[1] = pack8(o[1]);
    }
  } else if constexpr (EPI == EPI_SILU) {
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      if (!in.ok[j]) continue;
      const int m = in.rows[j];
      const float sc = norm ? inv_rms[m - rbase] : 1.f;
      uint16_t o[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float g = to_f32<T>(from_f32<T>(red[m - rbase][c] * sc));
        const float u = to_f32<T>(from_f32<T>(red[m - rbase][c + 8] * sc));
        const float si = to_f32<T>(from_f32<T>(g / (1.f + __expf(-g))));
        o[c] = from_f32<T>(si * u);
      }
      *reinterpret_cast<u32x4*>(p.y + static_cast<int64_t>(m) * p.y_stride + tile * 8) = pack8(o);
    }
  } else if constexpr (EPI == EPI_QKVROPE) {
    const int head = tile >> 3, jb = (tile & 7) * 8;
    const int nq = p.n_q_heads, nkv = p.n_kv_heads;
    const int BS = 1 << p.bs_shift;
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      if (!in.ok[j]) continue;
      const int m = in.rows[j];
      const float sc = norm ? inv_rms[m - rbase] : 1.f;
      uint16_t o1[8], o2[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        // GEMM output rounded to T first (matches the unfused F.linear -> rope path)
        const float x1 = to_f32<T>(from_f32<T>(red[m - rbase][c] * sc));
        const float x2 = to_f32<T>(from_f32<T>(red[m - rbase][c + 8] * sc));
        if (head < nq + nkv) {
          const float co = in.cs[j][c >> 2][c & 3], si = in.cs[j][2 + (c >> 2)][c & 3];
          o1[c] = from_f32<T>(x1 * co - x2 * si);
          o2[c] = from_f32<T>(x2 * co + x1 * si);
        } else {
          o1[c] = from_f32<T>(x1);
          o2[c] = from_f32<T>(x2);
        }
      }
      const int sl = in.slot[j];
      if (head < nq) {
        uint16_t* q = p.y + static_cast<int64_t>(m) * p.y_stride + head * 128 + jb;
        *reinterpret_cast<u32x4*>(q) = pack8(o1);
        *reinterpret_cast<u32x4*>(q + 64) = pack8(o2);
      } else if (sl >= 0 && head < nq + nkv) {
        uint16_t* kc = p.k_cache + ((static_cast<int64_t>(sl >> p.bs_shift) * nkv + (head - nq)) * BS +
                                    (sl & (BS - 1))) * 128 + jb;
        *reinterpret_cast<u32x4*>(kc) = pack8(o1);
        *reinterpret_cast<u32x4*>(kc + 64) = pack8(o2);
      } else if (sl >= 0) {
        uint16_t* vc = p.v_cache + (static_cast<int64_t>(sl >> p.bs_shift) * nkv + (head - nq - nkv)) *
                                       128 * BS + (sl & (BS - 1));
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          vc[static_cast<int64_t>(jb + c) * BS] = o1[c];
          vc[static_cast<int64_t>(jb + c + 64) * BS] = o2[c];
        }
      }
    }
  } else if constexpr (EPI == EPI_SAMPLE) {
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      if (!in.ok[j]) continue;
      const int m = in.rows[j];
      const float sc = norm ? inv_rms[m - rbase] : 1.f;
      unsigned long long best = 0ull;
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        float v = to_f32<T>(from_f32<T>(red[m - rbase][n] * sc));  // bf16 logits, as F.linear
        const int idx = p.vocab_offset + tile * 16 + n;    // global id: TP == TP1 noise
        if (in.temp[j] > 1e-5f)
          v = v / in.temp[j] + gumbel_noise(in.seed[j], in.step[j], static_cast<uint32_t>(idx));
        const unsigned long long key =
            (static_cast<unsigned long long>(ordered_bits(v)) << 32) |
            static_cast<unsigned long long>(0xFFFFFFFFu - static_cast<unsigned>(idx));
        best = key > best ? key : best;
      }
      p.keys[static_cast<int64_t>(m) * p.key_stride + tile] = best;
    }
  }
}

template <typename T, int WAVES, int MT, int EPI, bool NORM>
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
  constexpr bool norm = NORM;  // p.eps > 0: fused RMSNorm (compile-time: no branches in the loop)
  constexpr int kWStages = kDeepW;  // weight register stages (chunks of weights in flight + 1)

  // this wave's weight tile (idle waves of the last column block stream tile 0 and store
  // nothing: every wave takes part in the barriers)
  const uint16_t* wp = p.w + static_cast<int64_t>(tvalid ? tile : 0) * (p.K / 32) * 512 + lane * 8;
  // x pieces of this thread: piece q = tid + i * NTHR -> staged row q / 16, slot q % 16
  int xsrc[PPT];  // element offsets from p.x (32-bit: x is < 4 MB here)
  int xdst[PPT];
  bool xst[PPT], xss[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int q = tid + i * NTHR;
    const int row = q < PIECES ? q / kSlots : 0;
    const int slot = q % kSlots;
    xst[i] = q < PIECES;  // only the last piece can be out of range (PIECES % NTHR != 0)
    xss[i] = q < PIECES && row < p.M;
    // rows past M stage a copy of row M - 1 (finite; their accumulator rows are discarded)
    xsrc[i] = min(row, p.M - 1) * static_cast<int>(p.x_stride) + slot * 8;
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
  u32x4 w0[4], w1[4], w2[4], w3[4], xa[PPT], xb[PPT];
  auto load_w = [&](u32x4 (&f)[4], int c) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
      f[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wp + (c * 4 + s) * 512));
  };
  auto load_x = [&](u32x4 (&xr)[PPT], int c) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) xr[i] = *reinterpret_cast<const u32x4*>(p.x + xsrc[i] + c * kKC);
  };
  // no data-dependent control flow around the staging: branches between the loads and their
  // uses made hipcc's waitcnt pass fall back to near-vmcnt(0) waits at every block join
  auto store_x = [&](const u32x4 (&xr)[PPT], int buf, bool real) {
    unsigned char* b = lds + buf * XBUF;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      if (PIECES % NTHR == 0 || i + 1 < PPT || xst[i])
        *reinterpret_cast<u32x4*>(b + xdst[i]) = xr[i];
    }
    if constexpr (norm) {
#pragma unroll
      for (int i = 0; i < PPT; ++i) {
        // rows past M (and an out-of-range last piece) add 0: the select keeps it branch-free
        const float v = MF::sq8(__builtin_bit_cast(frag8, xr[i]), 0.f);
        ss[i] += (xss[i] && real) ? v : 0.f;
      }
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
  // one chunk: issue chunk c + 2's loads, compute chunk c, stage chunk c + 1's x, barrier.
  // Past the slice end the loads re-read the slice's last chunk and the staging writes the
  // idle buffer (never computed): unconditional, so the loop body has no branches.
  const int clast = c1 - 1;
  auto iter = [&](const u32x4 (&wcur)[4], u32x4 (&wnext)[4], const u32x4 (&xstage)[PPT],
                  u32x4 (&xload)[PPT], int c, int buf) {
    load_x(xload, min(c + 2, clast));
    load_w(wnext, min(c + kWStages - 1, clast));
    compute(wcur, buf);
    store_x(xstage, buf ^ 1, c + 1 < c1);  // past the end: a re-staged chunk, no squares
    // LDS hand-over only: ds_writes retired, then a bare s_barrier - __syncthreads()' fence
    // semantics made hipcc drain the weight / x loads in flight (vmcnt(0)) at the period's
    // loop header
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  if (c0 < c1) {
    load_x(xa, c0);
    load_w(w0, c0);
    load_x(xb, min(c0 + 1, clast));
    load_w(w1, min(c0 + 1, clast));
    if constexpr (kWStages == 4) load_w(w2, min(c0 + 2, clast));
    store_x(xa, 0, true);
  }
  __syncthreads();
  int c = c0;
  if constexpr (kWStages == 4) {
    // whole 4-chunk periods (4 weight stages x 2 x sets: three chunks of weights in flight
    // while one computes), then the <= 3 remaining chunks
    for (; c + 4 <= c1; c += 4) {
      iter(w0, w3, xb, xa, c, 0);
      iter(w1, w0, xa, xb, c + 1, 1);
      iter(w2, w1, xb, xa, c + 2, 0);
      iter(w3, w2, xa, xb, c + 3, 1);
    }
    if (c < c1) {
      iter(w0, w3, xb, xa, c, 0);
      if (c + 1 < c1) {
        iter(w1, w0, xa, xb, c + 1, 1);
        if (c + 2 < c1) iter(w2, w1, xb, xa, c + 2, 0);
      }
    }
    c = c1;
  }
  // whole 6-chunk periods (3 weight stages x 2 x sets) with no exits inside the loop body, then
  // the <= 5 remaining chunks
  for (; c + 6 <= c1; c += 6) {
    iter(w0, w2, xb, xa, c, 0);
    iter(w1, w0, xa, xb, c + 1, 1);
    iter(w2, w1, xb, xa, c + 2, 0);
    iter(w0, w2, xa, xb, c + 3, 1);
    iter(w1, w0, xb, xa, c + 4, 0);
    iter(w2, w1, xa, xb, c + 5, 1);
  }
  if (c < c1) {
    iter(w0, w2, xb, xa, c, 0);
    if (c + 1 < c1) {
      iter(w1, w0, xa, xb, c + 1, 1);
      if (c + 2 < c1) {
        iter(w2, w1, xb, xa, c + 2, 0);
        if (c + 3 < c1) {
          iter(w0, w2, xa, xb, c + 3, 1);
          if (c + 4 < c1) iter(w1, w0, xb, xa, c + 4, 0);
        }
      }
    }
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
  float(*red)[17] = reinterpret_cast<float(*)[17]>(lds + wid * R * 17 * 4);
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[t * 16 + 4 * grp + i][col] = acc[t][i];
  if (S > 1) {
    // ---- split-K: publish this slice's rows (plain stores: the reduce launch that follows
    // in stream order combines them - no in-launch hand-over, no last-arriver serial read of
    // every slice's slab: 5-17 us at 85 rows, profiles/r5_wide_gemm.txt) ------------------
    __syncthreads();
    if (tvalid) {
#pragma unroll
      for (int j = 0; j < (R > 64 ? 2 : 1); ++j) {
        const int row = lane + 64 * j;
        if (row < R && row < p.M) {
          float* dst = p.sk_ws + ((static_cast<int64_t>(tile) * S + ks) * R + row) * 16;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            reinterpret_cast<f32x4*>(dst)[q] =
                f32x4{red[row][4 * q], red[row][4 * q + 1], red[row][4 * q + 2], red[row][4 * q + 3]};
        }
      }
    }
    if (norm && tid < R && tid < p.M)
      p.sk_ws[static_cast<int64_t>(ntiles) * S * R * 16 + (static_cast<int64_t>(cb) * S + ks) * R + tid] =
          ssq[tid];
    if (p.wg_trace != nullptr) {
      if (tid == 0) {
        unsigned long long* t = p.wg_trace + 4 * (blockIdx.x + gridDim.x * blockIdx.y);
        t[0] = tr0;
        t[1] = tr1;
        t[2] = wall_clock64();
        t[3] = t[2];
      }
    }
    return;
  }
  // the epilogue's global inputs
  EpiIn<(R > 64 ? 2 : 1)> ein;
  epi_load<T, EPI, (R > 64 ? 2 : 1)>(p, tvalid ? tile : 0, 0, 64, R, lane, ein);
  if (norm && tid < R) inv_rms[tid] = rsqrtf(ssq[tid] / static_cast<float>(p.K) + p.eps);
  __syncthreads();
  if (tvalid) epi_apply<T, EPI, (R > 64 ? 2 : 1)>(p, tile, red, inv_rms, 0, norm, ein);
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

// Split-K combine + epilogue: one wave per (16-column tile, 16-row group); lane l loads
// columns 4 (l >> 4) .. +3 of row (l & 15) from every slice (16 B each, all issued together:
// one round trip for S <= 8), sums them in slice order - bitwise deterministic - with the row
// sums of squares, and lanes 0-15 run the unsplit path's epi_apply on their row.  (One wave
// per tile over all rows left most CUs idle: 10 us.)
template <typename T, int MT, int EPI, bool NORM>
__global__ __launch_bounds__(256) void wide_reduce_kernel(SkinnyParams p, int ntiles, int S,
                                                         int waves) {
  constexpr int R = MT * 16;
  __shared__ float red_all[4][16][17];
  __shared__ float inv_all[4][16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int gw = blockIdx.x * 4 + wid;
  const int tile = gw / MT, rg = gw % MT;
  if (tile >= ntiles) return;  // wave-uniform; no workgroup barrier below
  const int cb = tile / waves;
  const int r = rg * 16 + (lane & 15), qd = lane >> 4;
  const int rc = min(r, max(p.M - 1, 0));
  EpiIn<1> ein;
  epi_load<T, EPI, 1>(p, tile, rg * 16, 16, R, lane, ein);
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;
  for (int k0 = 0; k0 < S; k0 += 8) {
    f32x4 part[8];
    float sp[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int ks = min(k0 + u, S - 1);
      part[u] = reinterpret_cast<const f32x4*>(
          p.sk_ws + ((static_cast<int64_t>(tile) * S + ks) * R + rc) * 16)[qd];
      if constexpr (NORM)
        sp[u] = p.sk_ws[static_cast<int64_t>(ntiles) * S * R * 16 +
                        (static_cast<int64_t>(cb) * S + ks) * R + rc];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool real = k0 + u < S;
      sum += real ? part[u] : f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (NORM) ss += real ? sp[u] : 0.f;
    }
  }
  float(*red)[17] = red_all[wid];
  float* inv_rms = inv_all[wid];
#pragma unroll
  for (int e = 0; e < 4; ++e) red[lane & 15][4 * qd + e] = sum[e];
  if (NORM && qd == 0) inv_rms[lane & 15] = rsqrtf(ss / static_cast<float>(p.K) + p.eps);
  __builtin_amdgcn_wave_barrier();  // rows were written by 4 lanes each: in-wave hand-over
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  epi_apply<T, EPI, 1>(p, tile, red, inv_rms, rg * 16, NORM, ein);
}

template <typename T, int MT>
static int launch_reduce(int epi, const SkinnyParams& p, int ntiles, int S, int waves,
                         hipStream_t st) {
  const dim3 grid((ntiles * MT + 3) / 4), blk(256);
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

constexpr bool norm_fits(int waves, int mt) {
  return !((mt == 8 && (waves == 6 || waves == 7)) || (mt == 7 && waves == 6));
}

// RMSNorm fold per epilogue as the engine uses them: never for the plain / residual
// projections (x is already the attention / SiLU output), always for qkv and gate_up (eps > 0),
// either way for the LM-head sampler (decode: final norm fused; prefill rows: already normed)
template <typename T, int WAVES, int MT>
static int launch_epi(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p, int ntiles) {
  const dim3 blk(WAVES * 64);
  const bool norm = p.eps > 0.f;
  // 6 / 7 waves at 128 rows and 6 waves at 112 rows with the norm fold spill past 256 VGPRs
  // (the plan avoids them)
  constexpr bool kNormOk = norm_fits(WAVES, MT);
  if constexpr (!kNormOk) {
    if (norm) return -1;
  }
  switch (epi) {
    case EPI_PLAIN:
      if (norm) return -1;
      wide_kernel<T, WAVES, MT, EPI_PLAIN, false><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_RESADD:
      if (norm) return -1;
      wide_kernel<T, WAVES, MT, EPI_RESADD, false><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_QKVROPE:
      if (!norm) return -1;
      if constexpr (kNormOk) wide_kernel<T, WAVES, MT, EPI_QKVROPE, true><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_SILU:
      if (!norm) return -1;
      if constexpr (kNormOk) wide_kernel<T, WAVES, MT, EPI_SILU, true><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_SAMPLE:
      if (norm) {
        if constexpr (kNormOk) wide_kernel<T, WAVES, MT, EPI_SAMPLE, true><<<grid, blk, 0, st>>>(p, ntiles);
      } else {
        wide_kernel<T, WAVES, MT, EPI_SAMPLE, false><<<grid, blk, 0, st>>>(p, ntiles);
      }
      return 0;
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
    case 1: return launch_w<T, 1>(epi, waves, grid, st, p, ntiles);
    case 3: return launch_w<T, 3>(epi, waves, grid, st, p, ntiles);
    case 4: return launch_w<T, 4>(epi, waves, grid, st, p, ntiles);
    case 5: return launch_w<T, 5>(epi, waves, grid, st, p, ntiles);
    case 6: return launch_w<T, 6>(epi, waves, grid, st, p, ntiles);
    case 7: return launch_w<T, 7>(epi, waves, grid, st, p, ntiles);
    case 8: return launch_w<T, 8>(epi, waves, grid, st, p, ntiles);
    default: return -1;
  }
}

// Grid plan: per candidate wave count (tiles per workgroup) and K split S <= 8, a time
// estimate - rounds of the grid over the CUs x (a workgroup's weight bytes + x bytes / 3 at a
// per-CU streaming rate, plus ~1.5 us of ramp), plus for a split the reduce launch - and the
// cheapest wins.  Slices keep >= 2 chunks of K.
static void plan(int ntiles, int K, int M, bool norm, int& waves, int& ksplit) {
  constexpr double kCUs = 256.0, kBpus = 24e3;  // bytes per us per CU
  const int mpad = ((M + 15) / 16) * 16;
  const int nch = K / kKC;
  double best = 1e30;
  const int ws[4] = {4, 6, 7, 8};
  for (int wi = 0; wi < 4; ++wi) {
    const int w = ws[wi];
    if (norm && !norm_fits(w, (M + 15) / 16)) continue;  // see launch_epi
    const int ncb = (ntiles + w - 1) / w;
    for (int s = 1; s <= 8 && nch / s >= 2; ++s) {
      const double rounds = std::ceil(ncb * s / kCUs);
      const double kslice = static_cast<double>(K) / s;
      const double bytes = w * 16.0 * kslice * 2.0 + mpad * kslice * 2.0 / 3.0;
      const double idle = static_cast<double>(ncb * w - ntiles) / (ncb * w);  // empty waves
      // split: a reduce launch (~2 us incl. its boundary) reading every slice's slab
      const double slab = static_cast<double>(ntiles) * s * mpad * 64.0;
      const double t = rounds * (bytes / kBpus * (1.0 + 0.5 * idle) + 1.5) +
                       (s > 1 ? 2.0 + slab / 5e6 : 0.0);
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
  if (waves <= 0 || ksplit <= 0) wide::plan(ntiles, p.K, p.M, p.eps > 0.f, waves, ksplit);
  if (waves != 4 && waves != 6 && waves != 7 && waves != 8) return -1;
  if (ksplit < 1 || p.K / wide::kKC < ksplit) return -1;
  // 16-row blocks: rows padded to the next 16 only (75 rows: 80, not 96)
  const int mt = (p.M + 15) / 16;
  const int ncb = (ntiles + waves - 1) / waves;
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
  }
  (void)n_counters;
  p.ksplit = ksplit;
  const dim3 grid(ncb, ksplit);
  int rc = dtype == 0 ? wide::launch_mt<__bf16>(epi, mt, waves, grid, stream, p, ntiles)
                      : wide::launch_mt<_Float16>(epi, mt, waves, grid, stream, p, ntiles);
  if (rc) return rc;
  if (ksplit > 1) {
    p.wg_trace = nullptr;
    rc = dtype == 0 ? wide::launch_reduce_mt<__bf16>(epi, mt, p, ntiles, ksplit, waves, stream)
                    : wide::launch_reduce_mt<_Float16>(epi, mt, p, ntiles, ksplit, waves, stream);
    if (rc) return rc;
  }
  return static_cast<int>(hipGetLastError());
}
