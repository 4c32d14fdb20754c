// Prefill flash attention over the paged KV cache, LDS-staged K/V tiles on 32x32x16 MFMA
// (replaces the attention vLLM runs under engine.generate(), reference
// llm/serve_llm.py:527-531).  Varlen batches, causal with a context offset (chunked prefill
// and prefix-cache hits: query token i of a sequence sits at position kvlen - qlen + i),
// GQA G = Hq / Hkv in {1, 2, 3, 4, 8}, head_dim 128, bf16 / fp16 (G = 3: Llama-3.2-3B, 24 q /
// 8 kv heads; a wave's last 32 mod 3 = 2 columns idle).
//
// Work decomposition: grid tiles x Hkv (1-D, KV head fastest).  A workgroup = 4 waves owns 128 "columns" = the G
// query heads of one KV head x 128 / G consecutive query tokens of one sequence; wave w owns
// columns 32w..32w+31 (column c: token c / G, head c % G).  Every K/V tile is staged ONCE in
// LDS per workgroup and read by all 128 columns (G x the reuse of a per-head kernel).
//
// Per 32-key block, per wave (cdna_hip_programming.md §3 "swapped QK^T"):
//   S^T[32 keys x 32 cols] = K[32 x 128] . Q^T[128 x 32]       8 x mfma_f32_32x32x16
//     A = K rows from LDS (16 B reads, rows padded to 272 B: conflict-free), B = Q (registers);
//     the accumulator has the column on the lane, so the online-softmax row statistics are
//     lane-local over 16 registers plus one xor-32 exchange;
//   O^T[128 x 32] += V^T[128 x 32 keys] . P^T[32 keys x 32]    8 x mfma_f32_32x32x16
//     B = P^T straight from the S^T accumulator registers (pairs packed to 16 bit; the k order
//     inside a step is permuted, and the V^T A-operand reads follow the same permutation),
//     A = V^T rows from LDS (one 16 B read per fragment from a key-permuted, padded image).
// 64-key blocks (two 32-key sub-tiles).  O^T is rescaled only when a running max grew by more
// than 2^8 (defer-max).
// Pipelining: the next block's K/V are loaded global -> registers while the current block
// computes, then written to the other LDS buffer; one workgroup barrier per block.  The
// sequence's block-table slice is staged in LDS once so K/V addresses need no dependent
// global load inside the loop.  Causal masking touches only the diagonal blocks.
#include "common.h"
#include "kernels.h"

namespace atta {
namespace fp {

constexpr int kD = 128;
constexpr int kNS = 2;                   // 32-key sub-tiles per block
constexpr int kKB = 32 * kNS;            // keys per block
constexpr int kKStride = kD + 8;         // K tile row: 272 B (16 B reads conflict-free)
// V^T tile row: 144 B (16-B aligned rows; 36-dword stride: the PV operand's ds_read_b128 and
// the staging ds_write_b64 pairs are bank-conflict-free).  Inside every 16-key group the keys
// are stored permuted - key 8 a + 4 h + b at column 8 h + 4 a + b - so the 8 keys one lane
// needs for a PV fragment (keys 4 h .. 4 h + 3 and 8 + 4 h .. 8 + 4 h + 3, the order of the P^T
// registers) are one contiguous 16 B read: one ds_read_b128 (4 LDS cycles) instead of a
// ds_read2_b64 (8).
constexpr int kVStride = kKB + 8;
constexpr int kKTile = kKB * kKStride;   // elements
constexpr int kVTile = kD * kVStride;
constexpr int kBtLds = 2048;             // block-table entries staged in LDS
constexpr float kNegInf = -__builtin_huge_valf();
constexpr float kRescale = 8.f;  // defer-max threshold (log2 units)

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

template <typename T>
struct Mf32;
template <>
struct Mf32<__bf16> {
  typedef bf16x8 frag;
  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct Mf32<_Float16> {
  typedef f16x8 frag;
  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

struct FlashParams {
  uint16_t* out;            // [n_q_tokens, Hq, D] rows of out_stride
  const uint16_t* q;        // [n_q_tokens, Hq, D] rows of q_stride
  const uint16_t* k_cache;  // [nb, Hkv, BS, D]
  const uint16_t* v_cache;  // [nb, Hkv, D, BS]
  const int* block_tables;  // [S, bt_stride]
  const int* seq_kvlen;
  const int* seq_qstart;
  const int* tile_seq;
  const int* tile_qoff;
  int num_tiles;
  int64_t q_stride, out_stride;
  int bt_stride, n_kv_heads, bs_shift;
  float scale_log2;
  // split-KV (few tiles over long cached prefixes: the cached burst / planning steps): up to
  // nsplit workgroups per (tile, KV head) each walk a contiguous range of key blocks and
  // publish (O, m, l) partials; the last to arrive merges them (device-scope hand-over)
  int nsplit;
  int split_blocks;  // key blocks per split at least (atta_set_flash_split_blocks)
  float* part;    // [tile, Hkv, nsplit] slots of kPartBytes
  int* counters;  // [tile * Hkv], zero between launches (the last arriver re-arms)
};
// one split's partial: 128 columns x 128 fp32 O values, then 128 (m, l) pairs
constexpr uint32_t kPartOBytes = 128 * kD * 4;
constexpr uint32_t kPartBytes = kPartOBytes + 128 * 8;
constexpr int kMaxSplit = 8;
constexpr int kSplitBlocks = 8;  // 512 keys: the default of split_blocks

// two floats -> one packed 16-bit pair.  bf16: a single v_cvt_pk_bf16_f32 (RNE); element-wise
// conversion compiled to 2 converts + shift + or per pair, 64 VALU per block per wave.
template <typename T>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return static_cast<uint32_t>(from_f32<T>(a)) | (static_cast<uint32_t>(from_f32<T>(b)) << 16);
}
template <>
__device__ __forceinline__ uint32_t pack2<__bf16>(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{a, b}), bf16x2_t));
}

// lane l <-> lane l ^ 32 exchange: one ds_bpermute with the byte index hoisted out of the loop
// (__shfl_xor recomputed it per call: 7 VALU).  Not v_permlane32_swap: with both operands the
// same value the compiler folded its two results into one (sum -> 2 * r0), a wrong softmax sum.
__device__ __forceinline__ float xor32(float v, int idx4) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(idx4, __builtin_bit_cast(int, v)));
}

// NW = 4: every wave stages 16 keys of both K and V; NW = 8 (two workgroup halves): waves
// 0-3 stage K, waves 4-7 stage V, so each staged K/V block serves 256 columns and a wave issues
// half the staging instructions.
template <typename T, int G, int NW>
__global__ __launch_bounds__(NW * 64, 8 / NW) void flash_prefill_kernel(FlashParams p) {
  using MF = Mf32<T>;
  using frag = typename MF::frag;
  constexpr int kTokPerWave = 32 / G;
  constexpr int kTokPerWg = NW * kTokPerWave;
  __shared__ __attribute__((aligned(16))) uint16_t lds_k[2][kKTile];
  __shared__ __attribute__((aligned(16))) uint16_t lds_v[2][kVTile];
  __shared__ int lds_bt[kBtLds];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> SGPR
  const int r = lane & 31;   // column within the wave / row within a 32-row operand
  const int h = lane >> 5;   // lane half
  const int x32 = (lane ^ 32) << 2;  // ds_bpermute byte index of the partner lane
  // 1-D grid, KV head fastest: blocks are dealt round-robin over the 8 XCDs, so with 8 KV
  // heads every tile of head hk runs on one XCD and the head's K/V (re-read by all its
  // tiles) stays in that XCD's L2 instead of being pulled into all eight (placement is a
  // speed choice only, never correctness).  Heaviest (latest-token) tiles first: tiles are
  // emitted in token order per sequence.
  const int bid = static_cast<int>(blockIdx.x);
  const int hk = bid % p.n_kv_heads;
  const int rest = bid / p.n_kv_heads;
  const int sp = rest % p.nsplit;  // key-range split of this workgroup
  const int tile = p.num_tiles - 1 - rest / p.nsplit;
  const int s = p.tile_seq[tile];
  const int qoff = p.tile_qoff[tile];
  const int kvlen = p.seq_kvlen[s];  // >= wg_end: every key this workgroup reads is below it
  const int qstart = p.seq_qstart[s];
  const int qlen = p.seq_qstart[s + 1] - qstart;
  const int ctx0 = kvlen - qlen;
  const int BS = 1 << p.bs_shift;
  const int* bt = p.block_tables + static_cast<int64_t>(s) * p.bt_stride;

  // this lane's column
  const int c_tok = qoff + wid * kTokPerWave + r / G;
  const int c_head = hk * G + r % G;
  // (G = 3: columns 30, 31 of a wave would spill into the next wave's tokens)
  const bool c_valid = r < kTokPerWave * G && c_tok < qlen;
  const int c_end = c_valid ? ctx0 + c_tok + 1 : 0;  // keys [0, c_end) are visible
  // workgroup key range: up to the last valid token's causal limit
  const int wg_last_tok = min(qoff + kTokPerWg, qlen) - 1;
  const int wg_end = ctx0 + wg_last_tok + 1;
  const int nblocks = (wg_end + kKB - 1) / kKB;
  // wave key range (wave-uniform): blocks at or past it only need the wave at the barrier
  const int w_last_tok = min(qoff + (wid + 1) * kTokPerWave, qlen) - 1;
  const int w_end = w_last_tok >= qoff + wid * kTokPerWave ? ctx0 + w_last_tok + 1 : 0;
  const int w_first = qoff + wid * kTokPerWave;  // first token: fully visible below ctx0+w_first+1
  // this tile's splits: >= kSplitBlocks key blocks each (a split pays a publish + merge chain
  // of ~2 us: at the cached burst's ~10 blocks per tile it measured a wash), workgroups past
  // them exit before any barrier
  const int ns = max(1, min(p.nsplit, nblocks / p.split_blocks));
  if (sp >= ns) return;
  const int kb0 = sp * nblocks / ns, kb1 = (sp + 1) * nblocks / ns;

  // ---- block table slice -> LDS -------------------------------------------------------
  const int npages = min((wg_end + BS - 1) >> p.bs_shift, kBtLds);
  for (int i = tid; i < npages; i += NW * 64) lds_bt[i] = bt[i];

  // ---- Q (B operand): Q[col r][16 st + 8 h .. +8], 8 k-steps over D ----------------------
  frag qf[8];
  {
    const uint16_t* qp = p.q + static_cast<int64_t>(qstart + (c_valid ? c_tok : 0)) * p.q_stride +
                         static_cast<int64_t>(c_head) * kD + 8 * h;
#pragma unroll
    for (int st = 0; st < 8; ++st)
      qf[st] = c_valid ? *reinterpret_cast<const frag*>(qp + 16 * st) : frag{};
  }
  __syncthreads();  // lds_bt ready

  // ---- global -> register staging of one K/V block --------------------------------------
  // Wave w stages keys 16 w .. 16 w + 15 of the block for BOTH tensors: with BS >= 16 those
  // keys sit in one page, so the page lookup is wave-uniform (one LDS read + readfirstlane,
  // a scalar base) and every lane offset is a loop constant - the per-lane 64-bit address
  // arithmetic of 8 independent lookups was ~70 VALU per block and wave.
  //   K: lane l, chunk u -> key row 16 w + 4 u + (l >> 4), dims 8 (l & 15): each
  //      instruction reads 4 contiguous 256 B rows (1 KiB);
  //   V: lane l, chunk u -> d-row 32 u + (l >> 1), keys 16 w + 8 (l & 1) .. + 7: each
  //      instruction reads 32 d-rows x 16 keys (1 KiB contiguous at BS = 16).
  constexpr int kChunks = kKB * 16 / 256;   // per thread, per tensor
  static_assert(kKB == 64 && kChunks == 4, "wave w stages keys 16 w .. 16 w + 15");
  const int pshift = p.bs_shift + 7;        // log2(BS * kD) elements per (page, head)
  const int last_page = npages - 1;
  // staging key group of this wave (16 keys) and which tensors it stages
  const int sg = NW == 8 ? (wid & 3) : wid;
  constexpr bool kBoth = NW == 4;
  const bool stage_k = kBoth || wid < 4;
  const bool stage_v = kBoth || wid >= 4;
  const int w_keyoff = (16 * sg) & (BS - 1);                // group's first key in its page
  const int k_lane = (lane >> 4) * kD + 8 * (lane & 15) + w_keyoff * kD;
  const int v_lane = (lane >> 1) * BS + 8 * (lane & 1) + w_keyoff;
  const int k_lds = (16 * sg + (lane >> 4)) * kKStride + 8 * (lane & 15);
  const int v_lds = (lane >> 1) * kVStride + 16 * sg + 4 * (lane & 1);  // permuted: see kVStride
  // LDS only (the launcher rejects bt_stride > kBtLds): a select between the LDS copy and the
  // global table compiled to FLAT loads, whose vmcnt wait put a dependent global round trip
  // in front of every block's K/V loads.  Keys past the workgroup's range (>= wg_end) read a
  // clamped page or the unused tail slots of the last page - stale bytes of whatever sequence
  // held that page before.  Their scores are masked (P = 0), and their V^T columns are zeroed
  // at staging (store_block), so a non-finite stale value cannot turn 0 * V into NaN
  // (no invariant on the cache contents is needed).
  u32x4 kr[kBoth ? kChunks : 1], vr[kChunks];  // NW = 8: one register set (vr) per wave
  auto load_block = [&](int kb) {
    const int pi = min((kb * kKB + 16 * sg) >> p.bs_shift, last_page);
    const int pg = __builtin_amdgcn_readfirstlane(lds_bt[pi]);
    const uint64_t off = static_cast<uint64_t>(static_cast<uint32_t>(pg * p.n_kv_heads + hk)) << pshift;
    const uint16_t* kb_ = p.k_cache + off;
    const uint16_t* vb_ = p.v_cache + off;
    if constexpr (kBoth) {
#pragma unroll
      for (int u = 0; u < kChunks; ++u)
        kr[u] = *reinterpret_cast<const u32x4*>(kb_ + k_lane + u * 4 * kD);
#pragma unroll
      for (int u = 0; u < kChunks; ++u)
        vr[u] = *reinterpret_cast<const u32x4*>(vb_ + v_lane + u * 32 * BS);
    } else {
      // wave-uniform choice of tensor; the same registers carry K rows or V rows
#pragma unroll
      for (int u = 0; u < kChunks; ++u)
        vr[u] = stage_k ? *reinterpret_cast<const u32x4*>(kb_ + k_lane + u * 4 * kD)
                        : *reinterpret_cast<const u32x4*>(vb_ + v_lane + u * 32 * BS);
    }
  };
  auto store_block = [&](int buf, int kb) {
    if (stage_k) {
#pragma unroll
      for (int u = 0; u < kChunks; ++u)
        *reinterpret_cast<u32x4*>(&lds_k[buf][k_lds + u * 4 * kKStride]) =
            kBoth ? kr[kBoth ? u : 0] : vr[u];
    }
    if (!stage_v) return;
    // this lane's 8 V keys: kb * kKB + 16 sg + 8 (lane & 1) + j; only the last block can
    // reach past wg_end (uniform per workgroup except at that edge)
    const int vkey = kb * kKB + 16 * sg + 8 * (lane & 1);
    if (vkey + 8 > wg_end) {
#pragma unroll
      for (int u = 0; u < kChunks; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned lo = vkey + 2 * j < wg_end ? 0x0000ffffu : 0u;
          const unsigned hi = vkey + 2 * j + 1 < wg_end ? 0xffff0000u : 0u;
          vr[u][j] &= (lo | hi);
        }
    }
#pragma unroll
    for (int u = 0; u < kChunks; ++u) {
      // keys 8 g .. 8 g + 3 -> columns 4 g .., keys 8 g + 4 .. 8 g + 7 -> columns 8 + 4 g ..
      uint16_t* dst = &lds_v[buf][v_lds + u * 32 * kVStride];
      reinterpret_cast<u32x2*>(dst)[0] = u32x2{vr[u][0], vr[u][1]};
      reinterpret_cast<u32x2*>(dst + 8)[0] = u32x2{vr[u][2], vr[u][3]};
    }
  };

  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
  float m_run = kNegInf, l_run = 0.f;

  if (kb0 < kb1) {
    load_block(kb0);
    store_block(0, kb0);
  }
  __syncthreads();

  for (int kb = kb0; kb < kb1; ++kb) {
    const int buf = (kb - kb0) & 1;
    const bool more = kb + 1 < kb1;
    const int k0 = kb * kKB;
    bool issued = false;
    if (k0 < w_end) {  // wave-uniform: the wave has visible keys in this block
      const uint16_t* kl = lds_k[buf];
      const uint16_t* vl = lds_v[buf];
      // S^T = K . Q^T, one 32x32 accumulator per 32-key sub-tile
      f32x16 sacc[kNS];
#pragma unroll
      for (int t = 0; t < kNS; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[t][i] = 0.f;
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const frag kf =
              *reinterpret_cast<const frag*>(kl + (32 * t + r) * kKStride + 16 * st + 8 * h);
          sacc[t] = MF::mma(kf, qf[st], sacc[t]);
        }
      }
      // next block's K/V -> registers, issued after QK^T (guide §5.5 T14): in flight during
      // softmax + PV.  Issued at the top of the loop instead, the first QK^T MFMA (whose
      // accumulator the compiler had overlapped with the loads' address registers) waited
      // vmcnt(0) for them: every block paid the whole load latency.
      if (more) load_block(kb + 1);
      issued = true;
      // mask: only blocks crossing the diagonal of the wave's first token (wave-uniform
      // branch); element (t, i) holds key k0 + 4 h + 32 t + (i & 3) + 8 (i >> 2), a compile-
      // time offset from the lane's base, so a compare with one per-lane limit suffices
      if (k0 + kKB > ctx0 + w_first + 1) {
        const int lim = c_end - k0 - 4 * h;
#pragma unroll
        for (int t = 0; t < kNS; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (32 * t + (i & 3) + 8 * (i >> 2) >= lim) sacc[t][i] = kNegInf;
      }
      // running max on the raw scores (scale > 0), softmax in the log2 domain with the scale
      // folded into one fma per element: p = 2^(s * scale_log2 - m)
      float tmax = kNegInf;
#pragma unroll
      for (int t = 0; t < kNS; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, sacc[t][i]);
      tmax = fmaxf(tmax, xor32(tmax, x32));
      // defer-max (guide §5.5 T13): the running max m_run moves only when some column's max
      // grew by more than kRescale (log2 units), so P = 2^(s - m_run) stays <= 2^kRescale;
      // O and l are rescaled only then - with the max nearly settled after the first block,
      // the 32 packed multiplies of the rescale were paid on most blocks.  O, l and P of a
      // block always use the same m_run, so the result is exact up to rounding.
      const float m_cand = fmaxf(m_run, tmax * p.scale_log2);
      const bool grow = m_cand > m_run + kRescale;  // m_run == -inf: any finite m_cand
      if (__any(grow)) {
        const float m_new = grow ? m_cand : m_run;
        const float alpha = __builtin_amdgcn_exp2f(m_run - ((m_new == kNegInf) ? 0.f : m_new));
        l_run *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
        m_run = m_new;
      }
      const float m_use = (m_run == kNegInf) ? 0.f : m_run;
      // exponent arguments and the row sum on packed f32 pairs (v_pk_fma_f32 / v_pk_add_f32)
      typedef float f32x2_t __attribute__((ext_vector_type(2)));
      const f32x2_t sc2 = {p.scale_log2, p.scale_log2};
      const f32x2_t nm2 = {-m_use, -m_use};
      f32x2_t ps2 = {0.f, 0.f};
#pragma unroll
      for (int t = 0; t < kNS; ++t)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f32x2_t a = __builtin_elementwise_fma(f32x2_t{sacc[t][i], sacc[t][i + 1]}, sc2, nm2);
          const f32x2_t e = {__builtin_amdgcn_exp2f(a[0]), __builtin_amdgcn_exp2f(a[1])};
          sacc[t][i] = e[0];
          sacc[t][i + 1] = e[1];
          ps2 += e;
        }
      float psum = ps2[0] + ps2[1];
      psum += xor32(psum, x32);
      l_run += psum;
      // P^T fragments per 16-key step: registers 8s..8s+7 of the sub-tile packed pairwise;
      // O^T += V^T . P^T (A element j of half h = key 16 s + 8 (j >> 2) + 4 h + (j & 3))
#pragma unroll
      for (int t = 0; t < kNS; ++t) {
        frag pf[2];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          u32x4 w;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            w[j] = pack2<T>(sacc[t][8 * st + 2 * j], sacc[t][8 * st + 2 * j + 1]);
          pf[st] = __builtin_bit_cast(frag, w);
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const uint16_t* vrow = vl + (32 * dt + r) * kVStride + 32 * t + 8 * h;
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const frag vf = *reinterpret_cast<const frag*>(vrow + 16 * st);
            o[dt] = MF::mma(vf, pf[st], o[dt]);
          }
        }
      }
    }
    if (more && !issued) load_block(kb + 1);  // waves with no visible key in this block
    if (more) store_block(buf ^ 1, kb + 1);
    __syncthreads();
  }

  if (ns > 1) {
    // ---- split-KV hand-over: publish (O, m, l) with device-scope stores, count arrivals; the
    // last workgroup of the tile merges every split's partial into its own registers
    __shared__ int fl_last;
    const auto rw = dev_rsrc(p.part);
    const int pair = tile * p.n_kv_heads + hk;
    const uint32_t base = static_cast<uint32_t>(pair * p.nsplit) * kPartBytes;
    const int col = wid * 32 + r;
    // lane (col r, half h): O^T element (dt, i) is d = 32 dt + 8 (i >> 2) + 4 h + (i & 3)
    if (c_valid) {
      const uint32_t mine = base + static_cast<uint32_t>(sp) * kPartBytes;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          dev_store16(rw, mine + (col * kD + 32 * dt + 8 * g + 4 * h) * 4,
                      u32x4{__float_as_uint(o[dt][4 * g]), __float_as_uint(o[dt][4 * g + 1]),
                            __float_as_uint(o[dt][4 * g + 2]), __float_as_uint(o[dt][4 * g + 3])});
      if (h == 0) {
        dev_store4(rw, mine + kPartOBytes + col * 8, m_run);
        dev_store4(rw, mine + kPartOBytes + col * 8 + 4, l_run);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores acknowledged
    __syncthreads();
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(p.counters + pair, 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      fl_last = old == ns - 1;
    }
    __syncthreads();
    if (!fl_last) return;  // block-uniform
    if (tid == 0)
      __hip_atomic_store(p.counters + pair, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c_valid) {
      float mq[kMaxSplit], lq[kMaxSplit];  // fully unrolled: registers, not scratch
      float M = m_run;
#pragma unroll
      for (int q = 0; q < kMaxSplit; ++q) {
        mq[q] = kNegInf;
        lq[q] = 0.f;
        if (q >= ns || q == sp) continue;
        const uint32_t at = base + static_cast<uint32_t>(q) * kPartBytes + kPartOBytes + col * 8;
        mq[q] = dev_load4(rw, at);
        lq[q] = dev_load4(rw, at + 4);
        M = fmaxf(M, mq[q]);
      }
      // every split's O and l are relative to its own running max (log2 units)
      const float Mu = M == kNegInf ? 0.f : M;
      const float wself = __builtin_amdgcn_exp2f(m_run - Mu);
      l_run *= wself;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= wself;
#pragma unroll
      for (int q = 0; q < kMaxSplit; ++q) {
        if (q >= ns || q == sp) continue;
        const float wq = __builtin_amdgcn_exp2f(mq[q] - Mu);
        l_run += wq * lq[q];
        const uint32_t at = base + static_cast<uint32_t>(q) * kPartBytes;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const u32x4 v = dev_load16(rw, at + (col * kD + 32 * dt + 8 * g + 4 * h) * 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) o[dt][4 * g + j] += wq * __uint_as_float(v[j]);
          }
      }
    }
  }

  // ---- epilogue: O = O^T / l, lane (col r, half h) holds d = 32 dt + (i & 3) + 8 (i >> 2) + 4 h
  if (c_valid) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    uint16_t* op = p.out + static_cast<int64_t>(qstart + c_tok) * p.out_stride +
                   static_cast<int64_t>(c_head) * kD + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u32x2 w;
        w[0] = pack2<T>(o[dt][4 * g + 0] * inv, o[dt][4 * g + 1] * inv);
        w[1] = pack2<T>(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
        *reinterpret_cast<u32x2*>(op + 32 * dt + 8 * g) = w;
      }
  }
}

template <typename T, int NW>
static int launch_nw(int G, dim3 grid, hipStream_t st, const FlashParams& p) {
  switch (G) {
    case 1: flash_prefill_kernel<T, 1, NW><<<grid, NW * 64, 0, st>>>(p); return 0;
    case 2: flash_prefill_kernel<T, 2, NW><<<grid, NW * 64, 0, st>>>(p); return 0;
    case 3: flash_prefill_kernel<T, 3, NW><<<grid, NW * 64, 0, st>>>(p); return 0;
    case 4: flash_prefill_kernel<T, 4, NW><<<grid, NW * 64, 0, st>>>(p); return 0;
    case 8: flash_prefill_kernel<T, 8, NW><<<grid, NW * 64, 0, st>>>(p); return 0;
    default: return -1;
  }
}

// waves per workgroup (4 or 8); the host's tiles must hold NW * (32 / G) tokens
// (ops.prefill_tile_tokens reads the same setting)
static int g_flash_waves = 4;

template <typename T>
static int launch(int G, dim3 grid, hipStream_t st, const FlashParams& p) {
  return g_flash_waves == 8 ? launch_nw<T, 8>(G, grid, st, p) : launch_nw<T, 4>(G, grid, st, p);
}

}  // namespace fp
}  // namespace atta

using namespace atta;

void atta_set_flash_waves(int nw) { fp::g_flash_waves = nw == 8 ? 8 : 4; }
static int g_split_blocks = fp::kSplitBlocks;
void atta_set_flash_split_blocks(int nb) { g_split_blocks = nb < 1 ? 1 : nb; }

int atta_flash_prefill(void* out, const void* q, const void* k_cache, const void* v_cache,
                       const int* block_tables, const int* seq_kvlen, const int* seq_qstart,
                       const int* tile_seq, const int* tile_qoff, int num_tiles, int n_q_heads,
                       int n_kv_heads, int head_dim, int block_size, int bt_stride,
                       int64_t q_stride, int64_t out_stride, float scale, int nsplit,
                       float* part, int* counters, int dtype, hipStream_t stream) {
  const int G = n_q_heads / n_kv_heads;
  int shift = 0;
  while ((1 << shift) < block_size) ++shift;
  if (head_dim != fp::kD || (1 << shift) != block_size || block_size < 16) return -1;
  if (n_q_heads % n_kv_heads || G > 8 || ((G & (G - 1)) && G != 3)) return -1;
  // 16-byte row loads of q / stores of out need 8-element aligned row strides
  if (q_stride % 8 || out_stride % 4) return -1;
  if (bt_stride > fp::kBtLds) return -1;  // the block-table row is staged whole in LDS
  if (num_tiles == 0) return 0;
  fp::FlashParams prm{};
  prm.out = static_cast<uint16_t*>(out);
  prm.q = static_cast<const uint16_t*>(q);
  prm.k_cache = static_cast<const uint16_t*>(k_cache);
  prm.v_cache = static_cast<const uint16_t*>(v_cache);
  prm.block_tables = block_tables;
  prm.seq_kvlen = seq_kvlen;
  prm.seq_qstart = seq_qstart;
  prm.tile_seq = tile_seq;
  prm.tile_qoff = tile_qoff;
  prm.num_tiles = num_tiles;
  prm.q_stride = q_stride;
  prm.out_stride = out_stride;
  prm.bt_stride = bt_stride;
  prm.n_kv_heads = n_kv_heads;
  prm.bs_shift = shift;
  prm.scale_log2 = scale * 1.4426950408889634f;
  if (nsplit < 1 || nsplit > fp::kMaxSplit) return -1;
  if (nsplit > 1 && (part == nullptr || counters == nullptr)) return -2;
  // 32-bit byte offsets of the device-scope partial stores
  if (static_cast<int64_t>(num_tiles) * n_kv_heads * nsplit * fp::kPartBytes > 0x7FFFFFFF) return -1;
  prm.nsplit = nsplit;
  prm.split_blocks = g_split_blocks;
  prm.part = part;
  prm.counters = counters;
  dim3 grid(num_tiles * n_kv_heads * nsplit);
  const int rc = dtype == 0 ? fp::launch<__bf16>(G, grid, stream, prm)
                            : fp::launch<_Float16>(G, grid, stream, prm);
  if (rc) return rc;
  return static_cast<int>(hipGetLastError());
}
