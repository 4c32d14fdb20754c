// Wide small-M GEMM: 1 <= M <= 128 rows (routed from 17 rows, gate_up + SiLU from 12:
// gemv.hip use_wide) over pre-shuffled 16-bit weights, with the decode GEMVs' fused epilogues
// (residual add, RMSNorm fold + RoPE + paged K/V write, SiLU-mul, LM-head sampler keys).
// Serves the prefix-cached burst and planning prefills (the headline's 50-105-row bursts,
// reference agents/agent_a/server.py:534-623) and decode batches of 17-128 sequences
// (reference llm/serve_llm.py:362-373 max_num_seqs), which the 16-row-tile GEMV (gemv.hip)
// serves badly: it re-reads every x row from L2 once per 16 weight rows in fragment-shaped
// 16 x 64-B pieces - at 32 rows gate_up streamed 2.9 TB/s (profiles/r4_skinny_mt_probe.txt).
//
// Decomposition.  A workgroup owns WAVES x TPW consecutive 16-column weight tiles (wave w:
// tiles cb * WAVES * TPW + w * TPW + j; only TPW = 1 is built: two tiles per wave measured
// slower) over one K slice (split-K S = gridDim.y, for the narrow projections so the grid
// covers the 256 CUs), and all M rows in MT = ceil(M / 16) 16-row blocks:
//   * x is staged ONCE per workgroup through LDS in 128-column chunks (M_pad x 256 B, full
//     128-B lines, plain 16-B loads into registers then ds_write_b128 into an XOR-swizzled
//     image - slot j of row r at slot j ^ (r & 15): every ds_read_b128 lane group of the
//     fragment reads is conflict-free) and read by all waves: x's L2 traffic is
//     M / (16 WAVES) of the weight bytes instead of M / 16;
//   * each wave streams its tile's pre-shuffled weights (one contiguous 1 KiB per 32-wide K
//     step) straight to VGPRs, three 4-step chunks ahead (4 register stages), non-temporal;
//   * per K step a wave applies its weight fragment (MFMA B operand) to all MT 16-row x
//     fragments (A operand, ds_read_b128) - the weights are read once for every row;
//   * the RMSNorm fold needs sum(x^2) per row: accumulated from the staged x registers;
//   * split-K: each slice writes its fp32 row segments and partial sums of squares with
//     plain stores and exits; a second launch (wide.hip wide_reduce_kernel, one wave per
//     (tile, 16-row group)) sums them in slice order - bitwise deterministic - and runs the
//     epilogue.  (In-launch hand-overs measured slower: one last arriver reading every slice
//     5-17 us at 85 rows; every slice reducing 1/S after a counter wait 7-17 us.)
// One workgroup barrier per chunk.  Plain loads only (no LDS-DMA): mixing LDS-DMA with the
// register weight stream makes hipcc wait vmcnt(0) at every weight use (cdna_hip_programming
// §5, "Projection GEMM at M = 256" item 4(b)).  Compiled one 16-row block count per
// translation unit (wide_mt<N>.hip) so the build runs them in parallel.
#pragma once
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

// W8: fp8 (e4m3fn) weights in the skinny GEMV's 16-row x 64-K blocks of 1 KiB (skinny.h), two
// 16-byte loads per tile per chunk instead of four, converted to 16-bit MFMA operands in
// registers (v_cvt_scalef32_pk_*_fp8) and the per-row dequant scale applied to the finished
// accumulators: weight-only quantisation, the activations stay 16-bit (no per-token quant pass)
template <typename T, int WAVES, int MT, int EPI, bool NORM, int TPW, bool W8 = false>
__global__ __launch_bounds__(WAVES * 64) void wide_kernel(SkinnyParams p, int ntiles) {
  using MF = MfmaK32<T>;
  using frag8 = typename MF::frag8;
  constexpr int R = MT * 16;
  constexpr int NTHR = WAVES * 64;
  constexpr int TPB = WAVES * TPW;  // tiles per workgroup (TPW consecutive tiles per wave)
  constexpr int PIECES = R * kSlots;
  constexpr int PPT = (PIECES + NTHR - 1) / NTHR;  // x pieces per thread per chunk
  constexpr int XBUF = R * kRowB;
  constexpr int REDB = TPB * R * 17 * 4;
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
  const int tile0 = cb * TPB + wid * TPW;  // this wave's first tile
  const int nch = p.K / kKC;
  const int c0 = ks * nch / S, c1 = (ks + 1) * nch / S;
  constexpr bool norm = NORM;  // p.eps > 0: fused RMSNorm (compile-time: no branches in the loop)
  // weight register stages (chunks of weights in flight + 1): 4 x one tile, 3 x two tiles
  constexpr int kWStages = TPW == 1 ? kDeepW : 3;
  constexpr int NW = W8 ? 2 : 4;  // 16-B weight loads per tile per chunk
  constexpr int NWF = TPW * NW;   // weight registers (u32x4) per chunk per wave

  // this wave's weight tiles (idle tiles of the last column block stream tile 0 and store
  // nothing: every wave takes part in the barriers)
  // (byte pointers: a tile's pre-shuffled weights are K / 32 (16-bit) or K / 64 (fp8) 1 KiB
  // blocks, chunk c's are blocks c * NW .. c * NW + NW - 1)
  const unsigned char* wp[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
    wp[j] = reinterpret_cast<const unsigned char*>(p.w) +
            static_cast<int64_t>(tile0 + j < ntiles ? tile0 + j : 0) * (p.K / (W8 ? 64 : 32)) * 1024 +
            lane * 16;
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

  f32x4 acc[TPW][MT];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) ss[i] = 0.f;

  // weights: 3 register stages, chunk j in stage (j - c0) % 3 (two chunks in flight while one
  // computes); x: 2 register sets, chunk j loaded into set (j - c0) % 2 two chunks ahead and
  // written to LDS buffer (j - c0) % 2 one chunk ahead - every wait is for loads issued a full
  // chunk earlier (one chunk ahead exposed the whole load latency at each chunk: 2.2 TB/s)
  u32x4 w0[NWF], w1[NWF], w2[NWF], w3[NWF], xa[PPT], xb[PPT];
  auto load_w = [&](u32x4 (&f)[NWF], int c) {
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int s = 0; s < NW; ++s)
        f[j * NW + s] =
            __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wp[j] + (c * NW + s) * 1024));
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
  // each x fragment read from LDS feeds the MFMAs of all TPW tiles of the wave
  // per K step: the MT fragment reads first, then the MT MFMAs (hipcc otherwise pairs each
  // read with its MFMA behind an lgkmcnt wait, and the wave idles on LDS latency)
  auto compute = [&](const u32x4 (&f)[NWF], int buf) {
    const unsigned char* b = lds + buf * XBUF + col * kRowB;
    // weight fragment of tile j, K step s (fp8: converted up front, outside the MFMA groups)
    frag8 wf[TPW][4];
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if constexpr (W8) {
          const u32x4 r = f[j * 2 + (s >> 1)];
          wf[j][s] = (s & 1) ? fp8x8_to_frag<T>(r[2], r[3]) : fp8x8_to_frag<T>(r[0], r[1]);
        } else {
          wf[j][s] = __builtin_bit_cast(frag8, f[j * 4 + s]);
        }
      }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int off = ((4 * s + grp) ^ col) << 4;
      frag8 xf[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) xf[t] = *reinterpret_cast<const frag8*>(b + t * 16 * kRowB + off);
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int j = 0; j < TPW; ++j)
          acc[j][t] = MF::mma(xf[t], wf[j][s], acc[j][t]);
      __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);        // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, MT * TPW, 0);  // MFMA
    }
  };
  // one chunk: issue chunk c + 2's loads, compute chunk c, stage chunk c + 1's x, barrier.
  // Past the slice end the loads re-read the slice's last chunk and the staging writes the
  // idle buffer (never computed): unconditional, so the loop body has no branches.
  const int clast = c1 - 1;
  auto iter = [&](const u32x4 (&wcur)[NWF], u32x4 (&wnext)[NWF], const u32x4 (&xstage)[PPT],
                  u32x4 (&xload)[PPT], int c, int buf) {
    load_x(xload, min(c + 2, clast));
    load_w(wnext, min(c + kWStages - 1, clast));
    // the prefetches stay at the chunk head and the LDS writes after the MFMAs (hipcc sank
    // the loads below the MFMAs, one chunk less of lead on the weight stream)
    __builtin_amdgcn_sched_barrier(0);
    compute(wcur, buf);
    __builtin_amdgcn_sched_barrier(0);
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
  if constexpr (W8) {
    // dequant: lane column col of tile j is weight row tile_row(tile, col) (split-K slices
    // publish scaled partials - the sum is linear)
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const float sc = p.wscale[tile_row<EPI>(tile0 + j < ntiles ? tile0 + j : 0, col, p)];
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][t][i] *= sc;
    }
  }
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
  // tile j of this wave: accumulator image at red area wid * TPW + j
  auto red_of = [&](int j) {
    return reinterpret_cast<float(*)[17]>(lds + (wid * TPW + j) * R * 17 * 4);
  };
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    float(*red)[17] = red_of(j);
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[t * 16 + 4 * grp + i][col] = acc[j][t][i];
  }
  if (S > 1) {
    // ---- split-K: publish this slice's rows (plain stores: the reduce launch that follows
    // in stream order combines them - no in-launch hand-over, no last-arriver serial read of
    // every slice's slab: 5-17 us at 85 rows, profiles/r5_wide_gemm.txt) ------------------
    __syncthreads();
#pragma unroll
    for (int jt = 0; jt < TPW; ++jt) {
      const int tile = tile0 + jt;
      if (tile >= ntiles) continue;  // wave-uniform
      float(*red)[17] = red_of(jt);
#pragma unroll
      for (int j = 0; j < (R > 64 ? 2 : 1); ++j) {
        const int row = lane + 64 * j;
        if (row < R && row < p.M) {
          const int64_t at = ((static_cast<int64_t>(tile) * S + ks) * R + row) * 16;
          if (p.sk_half) {
            uint16_t o[2][8];
#pragma unroll
            for (int n = 0; n < 16; ++n) o[n >> 3][n & 7] = from_f32<__bf16>(red[row][n]);
            u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<uint16_t*>(p.sk_ws) + at);
            dst[0] = pack8(o[0]);
            dst[1] = pack8(o[1]);
          } else {
            float* dst = p.sk_ws + at;
#pragma unroll
            for (int q = 0; q < 4; ++q)
              reinterpret_cast<f32x4*>(dst)[q] =
                  f32x4{red[row][4 * q], red[row][4 * q + 1], red[row][4 * q + 2], red[row][4 * q + 3]};
          }
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
  EpiIn<(R > 64 ? 2 : 1)> ein[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
    epi_load<T, EPI, (R > 64 ? 2 : 1)>(p, tile0 + j < ntiles ? tile0 + j : 0, 0, 64, R, lane,
                                       ein[j]);
  if (norm && tid < R) inv_rms[tid] = rsqrtf(ssq[tid] / static_cast<float>(p.K) + p.eps);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TPW; ++j)
    if (tile0 + j < ntiles)
      epi_apply<T, EPI, (R > 64 ? 2 : 1)>(p, tile0 + j, red_of(j), inv_rms, 0, norm, ein[j]);
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

// builds that fit 256 VGPRs with the RMSNorm fold (the others spill; the plan avoids them)
constexpr bool norm_fits(int waves, int mt, int tpw = 1) {
  if (tpw == 2) return mt <= 5 || (mt == 6 && (waves == 4 || waves == 8));
  return !((mt == 8 && (waves == 6 || waves == 7)) || (mt == 7 && waves == 6));
}
// two tiles per wave are built for 4 and 8 waves (8 / 16 tiles per workgroup)
constexpr bool tpw2_built(int waves) { return waves == 4 || waves == 8; }

// RMSNorm fold per epilogue as the engine uses them: never for the plain / residual
// projections (x is already the attention / SiLU output), always for qkv and gate_up (eps > 0),
// either way for the LM-head sampler (decode: final norm fused; prefill rows: already normed)
template <typename T, int WAVES, int MT, int TPW>
inline int launch_epi_w8(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p, int ntiles) {
  const dim3 blk(WAVES * 64);
  const bool norm = p.eps > 0.f;
  switch (epi) {
    case EPI_PLAIN:
      if (norm) return -1;
      wide_kernel<T, WAVES, MT, EPI_PLAIN, false, TPW, true><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_RESADD:
      if (norm) return -1;
      wide_kernel<T, WAVES, MT, EPI_RESADD, false, TPW, true><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_QKVROPE:
      if (!norm) return -1;
      wide_kernel<T, WAVES, MT, EPI_QKVROPE, true, TPW, true><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_SILU:
      if (!norm) return -1;
      wide_kernel<T, WAVES, MT, EPI_SILU, true, TPW, true><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    default: return -1;  // the LM head stays 16-bit
  }
}

// (the non-norm fp8 epilogues of the builds whose norm fold spills)
template <typename T, int WAVES, int MT, int TPW>
inline int launch_epi_w8_plain(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p,
                               int ntiles) {
  const dim3 blk(WAVES * 64);
  if (p.eps > 0.f) return -1;
  switch (epi) {
    case EPI_PLAIN:
      wide_kernel<T, WAVES, MT, EPI_PLAIN, false, TPW, true><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_RESADD:
      wide_kernel<T, WAVES, MT, EPI_RESADD, false, TPW, true><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    default: return -1;
  }
}

template <typename T, int WAVES, int MT, int TPW>
inline int launch_epi(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p, int ntiles) {
  const dim3 blk(WAVES * 64);
  const bool norm = p.eps > 0.f;
  constexpr bool kNormOk = norm_fits(WAVES, MT, TPW);
  if (p.wscale != nullptr) {
    // fp8 weights (every wave count: 7 waves tile the 70B gate_up's 3584 SiLU tiles into
    // exactly two rounds of 256 workgroups)
    if constexpr (TPW == 1) {
      if (norm && !kNormOk) return -1;
      if constexpr (kNormOk) return launch_epi_w8<T, WAVES, MT, TPW>(epi, grid, st, p, ntiles);
      return launch_epi_w8_plain<T, WAVES, MT, TPW>(epi, grid, st, p, ntiles);
    }
    return -1;
  }
  if constexpr (!kNormOk) {
    if (norm) return -1;
  }
  switch (epi) {
    case EPI_PLAIN:
      if (norm) return -1;
      wide_kernel<T, WAVES, MT, EPI_PLAIN, false, TPW><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_RESADD:
      if (norm) return -1;
      wide_kernel<T, WAVES, MT, EPI_RESADD, false, TPW><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_QKVROPE:
      if (!norm) return -1;
      if constexpr (kNormOk) wide_kernel<T, WAVES, MT, EPI_QKVROPE, true, TPW><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_SILU:
      if (!norm) return -1;
      if constexpr (kNormOk) wide_kernel<T, WAVES, MT, EPI_SILU, true, TPW><<<grid, blk, 0, st>>>(p, ntiles);
      return 0;
    case EPI_SAMPLE:
      if (norm) {
        if constexpr (kNormOk) wide_kernel<T, WAVES, MT, EPI_SAMPLE, true, TPW><<<grid, blk, 0, st>>>(p, ntiles);
      } else {
        wide_kernel<T, WAVES, MT, EPI_SAMPLE, false, TPW><<<grid, blk, 0, st>>>(p, ntiles);
      }
      return 0;
    default: return -1;
  }
}

template <typename T, int MT, int TPW>
inline int launch_w(int epi, int waves, dim3 grid, hipStream_t st, const SkinnyParams& p,
                    int ntiles) {
  switch (waves) {
    case 4: return launch_epi<T, 4, MT, TPW>(epi, grid, st, p, ntiles);
    case 8: return launch_epi<T, 8, MT, TPW>(epi, grid, st, p, ntiles);
    default: break;
  }
  if constexpr (TPW == 1) {
    switch (waves) {
      case 6: return launch_epi<T, 6, MT, 1>(epi, grid, st, p, ntiles);
      case 7: return launch_epi<T, 7, MT, 1>(epi, grid, st, p, ntiles);
      default: break;
    }
  }
  return -1;
}

// tpw == 2 (two 16-column tiles per wave sharing each x fragment read) measured 5-15 % slower
// at every shape (profiles/r5_wide_tiles_per_wave_negative.txt) and is not built
template <typename T, int MT>
inline int launch_t(int epi, int waves, int tpw, dim3 grid, hipStream_t st,
                    const SkinnyParams& p, int ntiles) {
  return tpw == 1 ? launch_w<T, MT, 1>(epi, waves, grid, st, p, ntiles) : -1;
}


// per-row-block translation units (wide_mt<N>.hip): the 16-row block count is compiled one
// per file so the build runs them in parallel
int launch_mt_tu(int mt, int epi, int waves, int tpw, dim3 grid, hipStream_t st,
                 const SkinnyParams& p, int ntiles, int dtype);
#define ATTA_WIDE_MT_TU(N)                                                                    \
  int launch_mt_##N(int epi, int waves, int tpw, dim3 grid, hipStream_t st,                    \
                    const SkinnyParams& p, int ntiles, int dtype) {                            \
    return dtype == 0 ? launch_t<__bf16, N>(epi, waves, tpw, grid, st, p, ntiles)              \
                      : launch_t<_Float16, N>(epi, waves, tpw, grid, st, p, ntiles);           \
  }

}  // namespace wide
}  // namespace atta
