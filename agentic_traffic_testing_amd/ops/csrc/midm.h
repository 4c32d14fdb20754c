// Mid-M GEMM: 129 - ~1k rows (the uncached burst / planning prefills of the 5-agent fan-out,
// reference agents/agent_a/server.py:534-623, and their TTFT, llm/serve_llm.py:547-559) over
// the PRE-SHUFFLED 16-bit weights the decode path already keeps, with the same fused epilogues
// as the decode GEMVs / wide kernel (RMSNorm fold + RoPE + paged K/V write, SiLU-mul, residual
// add).  Replaces the library GEMMs whose 256 x 256 tiles left 48 of 256 CUs busy at 382 rows
// (qkv 35.9 us = 0.53 PF/s, profiles/r4_prefill_gemm_tiles_sweep.txt).
//
// Decomposition (one 512-thread workgroup per CU):
//   * output tile BM x 128: BM = 16 BMT rows (a ROW BLOCK of the step, 48-192, host-planned so
//     the grid is ~256 workgroups) x 8 16-column weight tiles;
//   * 8 waves = 4 column waves x 2 K groups: wave w owns tiles 2 (w & 3), +1 and, of every
//     128-column K chunk, the two 32-wide MFMA K steps 2 (w >> 2), +1 (the K groups are summed
//     once, through LDS, at the end) - two waves per SIMD for latency hiding, and every x
//     fragment a wave reads from LDS feeds 2 MFMAs (one per tile: LDS reads at half the MFMA
//     issue rate, ds_read_b128 at 4 LDS cycles per 16-cycle MFMA pair);
//   * weights: each wave streams its own tiles' pre-shuffled 1 KiB fragments straight to
//     VGPRs, 3 chunks ahead (4 register stages), default cache policy - the nrb row-block
//     workgroups of a column block re-read the same bytes, and the XCD-aware block order below
//     puts them on one XCD so the re-reads hit its L2 (nt would evict them: cdna_hip_programming
//     nt-weights row, "never on slices every CU re-reads");
//   * x: staged once per workgroup through LDS in 128-column chunks into the XOR-swizzled
//     image of the wide kernel (slot j of row r at j ^ (r & 15): conflict-free ds_read_b128),
//     double-buffered, loaded two chunks ahead; one barrier per chunk;
//   * XCD-aware bijective block order (cdna_hip_programming §5 "XCD swizzle must be
//     bijective"): logical id L = the blocks of one XCD (b % 8) numbered consecutively, row
//     block fastest - the workgroups sharing a weight column block run on one XCD;
//   * split-K (S = K slices, o / down at 4096 columns: 32 column blocks only): slices publish
//     fp32 row segments [tile][slice][row][16] with plain stores and exit; midm_reduce (next
//     launch, stream order) sums them in slice order - bitwise deterministic - and runs the
//     epilogue.
// RMSNorm fold (qkv, gate_up: eps > 0): sum(x^2) per row accumulated from the staged x
// registers over the whole K (never split).  Plain loads only: no LDS-DMA beside the register
// weight stream (wide.h header, the vmcnt(0) trap).
#pragma once
#include "wide.h"

namespace atta {
namespace midm {

constexpr int kKC = 128;            // K columns per staged chunk (4 MFMA K steps)
constexpr int kRowB = kKC * 2;      // bytes of one staged x row
constexpr int kSlots = kRowB / 16;  // 16-B slots per staged row
constexpr int kThr = 512;           // 8 waves
constexpr int kNTW = 2;             // 16-column tiles per wave
constexpr int kTPB = 4 * kNTW;      // tiles per workgroup (4 column waves)
// weight register stages: 4 (3 chunks in flight) up to 128-row blocks; 3 above, where four
// stages push the 2-waves-per-SIMD budget (256 VGPRs) into spills
constexpr int wstages(int bmt) { return bmt <= 8 ? 4 : 3; }

struct Geo {
  int nrb, ncb, S;  // row blocks, column blocks, K slices (grid = nrb * ncb * S)
  int ntiles;       // 16-column weight tiles (SiLU: inter / 8)
  int R;            // rows of the split-K slab layout (M padded to 16)
};

// W8: fp8 (e4m3fn) weights in the 16-row x 64-K blocks of the skinny GEMV (skinny.h) - a
// wave's two K steps of a chunk (2 kg, 2 kg + 1) are exactly one such block, one 16-B load
// per tile per chunk - converted to 16-bit MFMA operands in registers, the per-row scale on
// the finished accumulators (weight-only quantisation, as wide.h)
template <typename T, int BMT, int EPI, bool NORM, int XD, bool W8 = false>
__global__ __launch_bounds__(kThr) void midm_kernel(SkinnyParams p, Geo g) {
  using MF = MfmaK32<T>;
  using frag8 = typename MF::frag8;
  constexpr int BM = BMT * 16;
  constexpr int PIECES = BM * kSlots;
  constexpr int PPT = (PIECES + kThr - 1) / kThr;  // x pieces per thread per chunk
  constexpr int XBUF = BM * kRowB;
  constexpr int REDB = kTPB * BM * 17 * 4;
  // XD (deep x pipeline, built for <= 128-row blocks): three x register sets loaded three
  // chunks ahead into three LDS buffers, three weight stages - the LDS write of a chunk waits
  // for loads issued two chunks earlier (qkv at 382 rows 38.7 -> 36.1 us); larger blocks keep
  // two x sets / buffers (three buffers of 192 rows cost them their LDS headroom)
  constexpr int NXB = XD == 1 ? 3 : 2;
  constexpr int LDSB = NXB * XBUF > REDB ? NXB * XBUF : REDB;
  constexpr int NW = W8 ? 1 : 2;  // 16-B weight loads per tile per chunk
  constexpr int NWF = kNTW * NW;  // weight registers (u32x4) per chunk per wave
  constexpr int RPL = (BM + 63) / 64;
  constexpr int kWStages = XD == 1 ? 3 : wstages(BMT);
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDSB];
  __shared__ float ssq[BM];
  __shared__ float inv_rms[BM];

  // ---- block -> (column block, K slice, row block), XCD-aware and bijective -------------
  const int nwg = gridDim.x;
  const int b = blockIdx.x, xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int rb = L % g.nrb;
  const int ks = (L / g.nrb) % g.S;
  const int cb = L / (g.nrb * g.S);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int cg = wid & 3, kg = wid >> 2;
  const int col = lane & 15, grp = lane >> 4;
  const int row0 = rb * BM;
  const int tile0 = cb * kTPB + cg * kNTW;  // this wave's first weight tile
  const int nch = p.K / kKC;
  const int c0 = ks * nch / g.S, c1 = (ks + 1) * nch / g.S;

  // weight bytes of tile j: 16-bit, K step (c, s) at wp[j] + (4 c + s) * 1 KiB (this wave's
  // steps 2 kg + s); fp8, chunk c at wp[j] + 2 c * 1 KiB (the block of steps 2 kg, 2 kg + 1)
  const unsigned char* wp[kNTW];
#pragma unroll
  for (int j = 0; j < kNTW; ++j)
    wp[j] = reinterpret_cast<const unsigned char*>(p.w) +
            static_cast<int64_t>(tile0 + j < g.ntiles ? tile0 + j : 0) * (p.K / (W8 ? 64 : 32)) * 1024 +
            (W8 ? kg : 2 * kg) * 1024 + lane * 16;
  // x pieces of this thread: piece q = tid + i * kThr -> staged row q / 16, slot q % 16
  int xsrc[PPT];
  int xdst[PPT];
  bool xst[PPT], xss[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int q = tid + i * kThr;
    const int row = q < PIECES ? q / kSlots : 0;
    const int slot = q % kSlots;
    xst[i] = q < PIECES;
    xss[i] = q < PIECES && row0 + row < p.M;
    // rows past M stage a copy of row M - 1 (finite; their accumulator rows are discarded)
    xsrc[i] = min(row0 + row, p.M - 1) * static_cast<int>(p.x_stride) + slot * 8;
    xdst[i] = row * kRowB + ((slot ^ (row & 15)) << 4);
  }

  f32x4 acc[kNTW][BMT];
#pragma unroll
  for (int j = 0; j < kNTW; ++j)
#pragma unroll
    for (int t = 0; t < BMT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) ss[i] = 0.f;

  u32x4 w0[NWF], w1[NWF], w2[NWF], w3[NWF], xa[PPT], xb[PPT], xc[PPT];
  auto load_w = [&](u32x4 (&f)[NWF], int c) {
#pragma unroll
    for (int j = 0; j < kNTW; ++j)
#pragma unroll
      for (int s = 0; s < NW; ++s)
        f[j * NW + s] = *reinterpret_cast<const u32x4*>(wp[j] + (c * (W8 ? 2 : 4) + s) * 1024);
  };
  // MFMA B operand of tile j, K step s (fp8: converted here, ahead of the MFMA groups)
  auto wfrag = [&](const u32x4 (&f)[NWF], int j, int s) -> frag8 {
    if constexpr (W8)
      return s ? fp8x8_to_frag<T>(f[j][2], f[j][3]) : fp8x8_to_frag<T>(f[j][0], f[j][1]);
    else
      return __builtin_bit_cast(frag8, f[j * 2 + s]);
  };
  auto load_x = [&](u32x4 (&xr)[PPT], int c) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) xr[i] = *reinterpret_cast<const u32x4*>(p.x + xsrc[i] + c * kKC);
  };
  auto store_x = [&](const u32x4 (&xr)[PPT], int buf, bool real) {
    unsigned char* bb = lds + buf * XBUF;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      if (PIECES % kThr == 0 || i + 1 < PPT || xst[i])
        *reinterpret_cast<u32x4*>(bb + xdst[i]) = xr[i];
    }
    if constexpr (NORM) {
#pragma unroll
      for (int i = 0; i < PPT; ++i) {
        const float v = MF::sq8(__builtin_bit_cast(frag8, xr[i]), 0.f);
        ss[i] += (xss[i] && real) ? v : 0.f;
      }
    }
  };
  // this wave's two K steps of the chunk in `buf`: each x fragment feeds both tiles' MFMAs.
  // Every fragment read of the chunk is issued before the first MFMA (up to 8 row blocks:
  // the register budget): waiting on each ds_read right before its two MFMAs left the
  // waves idle on LDS latency between MFMA pairs (one barrier per chunk, two waves per SIMD)
  auto compute = [&](const u32x4 (&f)[NWF], int buf) {
    const unsigned char* bb = lds + buf * XBUF + col * kRowB;
    frag8 wf[kNTW][2];
#pragma unroll
    for (int j = 0; j < kNTW; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) wf[j][s] = wfrag(f, j, s);
    if constexpr (BMT <= 8) {
      frag8 xf[2][BMT];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int off = (((2 * kg + s) * 4 + grp) ^ col) << 4;
#pragma unroll
        for (int t = 0; t < BMT; ++t)
          xf[s][t] = *reinterpret_cast<const frag8*>(bb + t * 16 * kRowB + off);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < BMT; ++t)
#pragma unroll
          for (int j = 0; j < kNTW; ++j)
            acc[j][t] = MF::mma(xf[s][t], wf[j][s], acc[j][t]);
      // pin the order (hipcc otherwise sinks each read next to its MFMA pair): all reads,
      // then the MFMAs, with counted lgkmcnt waits between them
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * BMT, 0);          // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * BMT * kNTW, 0);   // MFMA
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int off = (((2 * kg + s) * 4 + grp) ^ col) << 4;
#pragma unroll
        for (int t = 0; t < BMT; ++t) {
          const frag8 xf = *reinterpret_cast<const frag8*>(bb + t * 16 * kRowB + off);
#pragma unroll
          for (int j = 0; j < kNTW; ++j)
            acc[j][t] = MF::mma(xf, wf[j][s], acc[j][t]);
        }
      }
    }
  };
  const int clast = c1 - 1;
  auto iter = [&](const u32x4 (&wcur)[NWF], u32x4 (&wnext)[NWF], const u32x4 (&xstage)[PPT],
                  u32x4 (&xload)[PPT], int c, int buf) {
    load_x(xload, min(c + 2, clast));
    load_w(wnext, min(c + kWStages - 1, clast));
    // keep the prefetches at the top of the chunk: left alone, hipcc sinks them below the
    // MFMAs and the stores, so the x loads led their LDS write by under a chunk and the
    // kernel ran latency-bound (48 GB/s per CU at 382 rows)
    __builtin_amdgcn_sched_barrier(0);
    compute(wcur, buf);
    // and the LDS writes of the next chunk after the MFMAs (their wait on the x loads must
    // not stall the chunk's MFMAs)
    __builtin_amdgcn_sched_barrier(0);
    store_x(xstage, buf ^ 1, c + 1 < c1);
    // LDS hand-over only (wide.h: a bare s_barrier keeps the register loads in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  if constexpr (XD == 1) {
    // chunk c (r = c - c0): weights in stage r % 3, x in register set r % 3, LDS buffer r % 3
    auto iter3 = [&](const u32x4 (&wcur)[NWF], u32x4 (&wnext)[NWF], const u32x4 (&xw)[PPT],
                     u32x4 (&xl)[PPT], int c, int buf) {
      load_x(xl, min(c + 3, clast));
      load_w(wnext, min(c + 2, clast));
      __builtin_amdgcn_sched_barrier(0);
      compute(wcur, buf);
      __builtin_amdgcn_sched_barrier(0);
      store_x(xw, buf == 2 ? 0 : buf + 1, c + 1 < c1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    if (c0 < c1) {
      load_x(xa, c0);
      load_w(w0, c0);
      load_x(xb, min(c0 + 1, clast));
      load_w(w1, min(c0 + 1, clast));
      load_x(xc, min(c0 + 2, clast));
      store_x(xa, 0, true);
    }
    __syncthreads();
    int c = c0;
    for (; c + 3 <= c1; c += 3) {
      iter3(w0, w2, xb, xa, c, 0);
      iter3(w1, w0, xc, xb, c + 1, 1);
      iter3(w2, w1, xa, xc, c + 2, 2);
    }
    if (c < c1) {
      iter3(w0, w2, xb, xa, c, 0);
      if (c + 1 < c1) iter3(w1, w0, xc, xb, c + 1, 1);
    }
  } else {
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
      // whole 4-chunk periods (4 weight stages x 2 x sets), then the <= 3 remaining chunks
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
    } else {
      // whole 6-chunk periods (3 weight stages x 2 x sets), then the <= 5 remaining chunks
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
    }
  }

  if constexpr (W8) {
    // dequant: lane column col of tile j is weight row tile_row(tile, col)
#pragma unroll
    for (int j = 0; j < kNTW; ++j) {
      const float sc = p.wscale[tile_row<EPI>(tile0 + j < g.ntiles ? tile0 + j : 0, col, p)];
#pragma unroll
      for (int t = 0; t < BMT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][t][i] *= sc;
    }
  }
  // ---- row sums of squares (the 16 lanes staging one row are consecutive) ---------------
  if constexpr (NORM) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 1, kWave);
      v += __shfl_xor(v, 2, kWave);
      v += __shfl_xor(v, 4, kWave);
      v += __shfl_xor(v, 8, kWave);
      const int q = tid + i * kThr;
      if ((tid & 15) == 0 && q < PIECES) ssq[q / kSlots] = v;
    }
  }
  __syncthreads();  // x buffers free: the accumulator images reuse them
  // ---- K groups: group 1 stores its partial tile images, group 0 adds its own ------------
  auto red_of = [&](int tl) { return reinterpret_cast<float(*)[17]>(lds + tl * BM * 17 * 4); };
  if (kg == 1) {
#pragma unroll
    for (int j = 0; j < kNTW; ++j) {
      float(*red)[17] = red_of(cg * kNTW + j);
#pragma unroll
      for (int t = 0; t < BMT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[t * 16 + 4 * grp + i][col] = acc[j][t][i];
    }
  }
  __syncthreads();
  if (kg == 0) {
#pragma unroll
    for (int j = 0; j < kNTW; ++j) {
      float(*red)[17] = red_of(cg * kNTW + j);
#pragma unroll
      for (int t = 0; t < BMT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float& e = red[t * 16 + 4 * grp + i][col];
          e = e + acc[j][t][i];
        }
    }
  }
  __syncthreads();
  // ---- one 16-column tile per wave from here on -----------------------------------------
  const int tile = cb * kTPB + wid;
  if (g.S > 1) {
    // split-K: publish this slice's rows of the tile (plain stores; midm_reduce combines)
    if (tile < g.ntiles) {
      float(*red)[17] = red_of(wid);
#pragma unroll
      for (int j = 0; j < RPL; ++j) {
        const int r = lane + 64 * j;
        if (r < BM && row0 + r < p.M) {
          float* dst = p.sk_ws + ((static_cast<int64_t>(tile) * g.S + ks) * g.R + row0 + r) * 16;
#pragma unroll
          for (int qd = 0; qd < 4; ++qd)
            reinterpret_cast<f32x4*>(dst)[qd] =
                f32x4{red[r][4 * qd], red[r][4 * qd + 1], red[r][4 * qd + 2], red[r][4 * qd + 3]};
        }
      }
    }
    return;
  }
  wide::EpiIn<RPL> ein;
  wide::epi_load<T, EPI, RPL>(p, tile < g.ntiles ? tile : 0, row0, 64, row0 + BM, lane, ein);
  if (NORM && tid < BM) inv_rms[tid] = rsqrtf(ssq[tid] / static_cast<float>(p.K) + p.eps);
  __syncthreads();
  if (tile < g.ntiles)
    wide::epi_apply<T, EPI, RPL>(p, tile, red_of(wid), inv_rms, row0, NORM, ein);
}

// the RMSNorm-folded builds (qkv, gate_up) fit 2 waves per SIMD up to 128-row blocks; larger
// ones spill 30-124 VGPRs and are not built (the plan skips them)
constexpr bool norm_fits(int bmt) { return bmt <= 8; }

// launch one (BMT) instantiation; -1 = epilogue / norm combination not built
template <typename T, int BMT, int XD, bool W8>
inline int launch_bmt_w(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p, const Geo& g) {
  const dim3 blk(kThr);
  const bool norm = p.eps > 0.f;
  if constexpr (!norm_fits(BMT)) {
    if (norm) return -1;
  }
  switch (epi) {
    case EPI_PLAIN:
      if (norm) return -1;
      midm_kernel<T, BMT, EPI_PLAIN, false, XD, W8><<<grid, blk, 0, st>>>(p, g);
      return 0;
    case EPI_RESADD:
      if (norm) return -1;
      midm_kernel<T, BMT, EPI_RESADD, false, XD, W8><<<grid, blk, 0, st>>>(p, g);
      return 0;
    case EPI_QKVROPE:
      if (!norm || g.S > 1) return -1;
      if constexpr (norm_fits(BMT)) midm_kernel<T, BMT, EPI_QKVROPE, true, XD, W8><<<grid, blk, 0, st>>>(p, g);
      return 0;
    case EPI_SILU:
      if (!norm || g.S > 1) return -1;
      if constexpr (norm_fits(BMT)) midm_kernel<T, BMT, EPI_SILU, true, XD, W8><<<grid, blk, 0, st>>>(p, g);
      return 0;
    default: return -1;
  }
}

template <typename T, int BMT, int XD>
inline int launch_bmt(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p, const Geo& g) {
  return p.wscale != nullptr ? launch_bmt_w<T, BMT, XD, true>(epi, grid, st, p, g)
                             : launch_bmt_w<T, BMT, XD, false>(epi, grid, st, p, g);
}

// per-BMT translation units (midm_b<N>.hip), built in parallel
#define ATTA_MIDM_TU(N)                                                                       \
  int launch_b_##N(int epi, dim3 grid, hipStream_t st, const SkinnyParams& p, const Geo& g,   \
                   int dtype) {                                                               \
    constexpr int xd = N <= 8 ? 1 : 0;                                                        \
    return dtype == 0 ? launch_bmt<__bf16, N, xd>(epi, grid, st, p, g)                        \
                      : launch_bmt<_Float16, N, xd>(epi, grid, st, p, g);                     \
  }

}  // namespace midm
}  // namespace atta
