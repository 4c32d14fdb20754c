// Paged attention on MFMA for prefill (varlen, causal, chunked, prefix-cached) and decode
// (SURVEY §2.4 K6 + K7).  Replaces the attention vLLM runs under engine.generate()
// (reference llm/serve_llm.py:527-531).  head_dim is fixed at 128 (all Llama-3 shapes).
//
// Formulation ("swapped" QK^T, cdna_hip_programming.md §3 / T12):
//   S^T[16 tok x 16 col] = K[16 tok x 128] . Q^T[128 x 16 col]      4 x mfma_f32_16x16x32
//   O^T[16 d x 16 col]  += V^T[16 d x 16 tok] . P^T[16 tok x 16 col] 8 x mfma_f32_16x16x16 (1k)
// A "column" is one (query token, query head) pair that shares the KV head of the
// workgroup (GQA group G = Hq/Hkv; a wave holds 16/G tokens x G heads).  With the column
// on the lane, online-softmax row statistics are lane-local except for one xor-16/32
// shuffle, and the S^T accumulator registers ARE the B operand of the PV MFMA (lane l
// holds rows 4(l>>4)+i of column l&15 in both layouts) - no LDS round trip for P.
//
// K rows are read straight from the paged cache with 16-byte loads (each lane reads 64
// contiguous bytes of one token row); V is cached transposed ([.., D, block]) so each
// lane's A fragment of V^T is one 8-byte load.
//
// Two modes:
//   kSplitKV = false (prefill): grid (tiles, Hkv); 4 waves own 4 disjoint column sets.
//   kSplitKV = true  (decode) : grid (seqs, Hkv, partitions); the 4 waves share one column
//       set (the G heads of one token) and split the partition's KV tiles round-robin; the
//       4 partial (m, l, O) are merged through LDS.  With >1 partition the merged result is
//       written as fp32 (O, lse) and `attn_combine_kernel` reduces partitions.
#include "common.h"
#include "kernels.h"

namespace atta {

constexpr int kD = 128;
constexpr float kNegInf = -__builtin_huge_valf();

template <typename T>
struct Mfma;
template <>
struct Mfma<__bf16> {
  typedef bf16x8 frag8;
  __device__ static __forceinline__ f32x4 qk(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ f32x4 pv(i16x4 a, i16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  }
};
template <>
struct Mfma<_Float16> {
  typedef f16x8 frag8;
  __device__ static __forceinline__ f32x4 qk(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ f32x4 pv(i16x4 a, i16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, a),
                                                 __builtin_bit_cast(f16x4, b), c, 0, 0, 0);
  }
};

struct AttnParams {
  uint16_t* out;            // [n_q_tokens, Hq, D]
  float* part_out;          // [S, Hkv, P, 16, D]
  float* part_lse;          // [S, Hkv, P, 16]
  const uint16_t* q;        // [n_q_tokens, Hq, D] rows of q_stride elements
  const uint16_t* k_cache;  // [nb, Hkv, BS, D]
  const uint16_t* v_cache;  // [nb, Hkv, D, BS]
  const int* block_tables;  // [S, bt_stride]
  const int* seq_kvlen;     // [S]
  const int* seq_qstart;    // [S+1]
  const int* tile_seq;      // prefill: [tiles]
  const int* tile_qoff;     // prefill: [tiles]
  int64_t q_stride;
  int64_t out_stride;
  int bt_stride;
  int n_q_heads;
  int n_kv_heads;
  int bs_shift;  // log2(block_size)
  int part_tokens;
  int num_parts;
  float scale_log2;
};

template <typename T, int G, bool kSplitKV>
__global__ __launch_bounds__(256) void paged_attention_kernel(AttnParams p) {
  using M = Mfma<T>;
  using frag8 = typename M::frag8;
  constexpr int kTokPerWave = 16 / G;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int col = lane & 15;
  const int grp = lane >> 4;  // 0..3
  const int hk = blockIdx.y;
  const int BS = 1 << p.bs_shift;

  int s, qoff, kv_begin, kv_end;
  if constexpr (kSplitKV) {
    s = blockIdx.x;
    qoff = 0;
    const int kvlen = p.seq_kvlen[s];
    kv_begin = blockIdx.z * p.part_tokens;
    kv_end = min(kvlen, kv_begin + p.part_tokens);
  } else {
    s = p.tile_seq[blockIdx.x];
    qoff = p.tile_qoff[blockIdx.x] + wid * kTokPerWave;
    kv_begin = 0;
    kv_end = 0;  // set per column below
  }
  const int kvlen = p.seq_kvlen[s];
  const int qstart = p.seq_qstart[s];
  const int qlen = p.seq_qstart[s + 1] - qstart;
  const int ctx0 = kvlen - qlen;  // position of the first query token
  if (qlen <= 0) return;          // block-uniform: nothing to compute for this sequence

  // ---- this lane's column: (token, head) --------------------------------------------
  const int c_tok = kSplitKV ? (qlen - 1) : (qoff + col / G);
  const bool c_valid = (col < G * kTokPerWave) && (c_tok < qlen) && (kSplitKV ? col < G : true);
  const int c_head = hk * G + (col % G);
  const int c_pos = ctx0 + c_tok;  // causal limit (inclusive)
  int c_end = kSplitKV ? kv_end : (c_valid ? c_pos + 1 : 0);

  if constexpr (!kSplitKV) {
    // wave-uniform loop bound = max over the wave's columns
    int e = c_end;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) e = max(e, __shfl_xor(e, o, kWave));
    kv_end = e;
  }

  // ---- load Q fragment (B operand): Q[col][dims 32*grp + 8*kk + j] -------------------
  frag8 qf[4];
  {
    const uint16_t* qp = p.q + static_cast<int64_t>(qstart + c_tok) * p.q_stride +
                         static_cast<int64_t>(c_head) * kD + 32 * grp;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (c_valid) {
        qf[kk] = *reinterpret_cast<const frag8*>(qp + 8 * kk);
      } else {
        qf[kk] = frag8{};
      }
    }
  }

  f32x4 o_acc[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o_acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = kNegInf;  // running max (log2 domain) for column `col`
  float l_run = 0.f;

  const int* bt = p.block_tables + static_cast<int64_t>(s) * p.bt_stride;
  const int64_t kv_head_stride = static_cast<int64_t>(BS) * kD;  // elements per (page, head)
  const int tile_step = kSplitKV ? 64 : 16;
  int kt = kv_begin + (kSplitKV ? wid * 16 : 0);

  for (; kt < kv_end; kt += tile_step) {
    // -- K fragment: token kt + col, dims 32*grp .. +32
    const int tk = kt + col;
    const int pg_k = tk < kvlen ? bt[tk >> p.bs_shift] : 0;
    const uint16_t* kp = p.k_cache +
                         (static_cast<int64_t>(pg_k) * p.n_kv_heads + hk) * kv_head_stride +
                         static_cast<int64_t>(tk & (BS - 1)) * kD + 32 * grp;
    frag8 kf[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) kf[kk] = *reinterpret_cast<const frag8*>(kp + 8 * kk);

    // -- V^T fragments: dims 16*dt + col, tokens kt + 4*grp .. +3
    const int tv = kt + 4 * grp;
    const int pg_v = tv < kvlen ? bt[tv >> p.bs_shift] : 0;
    const uint16_t* vp = p.v_cache +
                         (static_cast<int64_t>(pg_v) * p.n_kv_heads + hk) * kv_head_stride +
                         static_cast<int64_t>(col) * BS + (tv & (BS - 1));
    i16x4 vf[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      vf[dt] = *reinterpret_cast<const i16x4*>(vp + static_cast<int64_t>(16 * dt) * BS);

    f32x4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) sacc = M::qk(kf[kk], qf[kk], sacc);

    // -- mask + online softmax for column `col` (rows = tokens kt + 4*grp + i)
    float sv[4];
    float tmax = kNegInf;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int tt = kt + 4 * grp + i;
      const bool ok = tt < c_end;
      sv[i] = ok ? sacc[i] * p.scale_log2 : kNegInf;
      tmax = fmaxf(tmax, sv[i]);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, kWave));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, kWave));
    const float m_new = fmaxf(m_run, tmax);
    const float m_use = (m_new == kNegInf) ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    float psum = 0.f;
    float pv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pv[i] = exp2f(sv[i] - m_use);
      psum += pv[i];
    }
    psum += __shfl_xor(psum, 16, kWave);
    psum += __shfl_xor(psum, 32, kWave);
    l_run = l_run * alpha + psum;
    m_run = m_new;

    i16x4 pf;
#pragma unroll
    for (int i = 0; i < 4; ++i) pf[i] = static_cast<short>(from_f32<T>(pv[i]));
    // V of keys past the sequence end (stale tail slots of the last page) is zeroed: P = 0
    // there, and 0 * V must not become NaN on a non-finite stale value
    if (tv + 4 > kvlen) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (tv + i >= kvlen) {
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) vf[dt][i] = 0;
        }
    }

#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      o_acc[dt] *= alpha;
      o_acc[dt] = M::pv(vf[dt], pf, o_acc[dt]);
    }
  }

  if constexpr (kSplitKV) {
    // ---- merge the 4 waves' partial states through LDS --------------------------------
    __shared__ float lds_o[4][16][kD + 4];
    __shared__ float lds_m[4][16];
    __shared__ float lds_l[4][16];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) lds_o[wid][col][16 * dt + 4 * grp + i] = o_acc[dt][i];
    if (grp == 0) {
      lds_m[wid][col] = m_run;
      lds_l[wid][col] = l_run;
    }
    __syncthreads();
    // 256 threads: thread -> column c = tid / 16, dims (tid % 16) * 8 .. +8
    const int c = threadIdx.x >> 4;
    const int d0 = (threadIdx.x & 15) * 8;
    float mw[4], mx = kNegInf;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      mw[w] = lds_m[w][c];
      mx = fmaxf(mx, mw[w]);
    }
    const float mu = (mx == kNegInf) ? 0.f : mx;
    float L = 0.f, f[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      f[w] = exp2f(mw[w] - mu);
      L += f[w] * lds_l[w][c];
    }
    const float invL = L > 0.f ? 1.f / L : 0.f;
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) a += f[w] * lds_o[w][c][d0 + j];
      r[j] = a * invL;
    }
    if (c < G) {
      const int head = hk * G + c;
      if (p.num_parts > 1) {
        const int64_t base = ((static_cast<int64_t>(s) * p.n_kv_heads + hk) * p.num_parts +
                              blockIdx.z) * 16 + c;
        float* po = p.part_out + base * kD + d0;
#pragma unroll
        for (int j = 0; j < 8; ++j) po[j] = r[j];
        if ((threadIdx.x & 15) == 0)
          p.part_lse[base] = (L > 0.f) ? (mu + log2f(L)) : kNegInf;
      } else {
        Pack8 o8;
#pragma unroll
        for (int j = 0; j < 8; ++j) o8.v[j] = from_f32<T>(r[j]);
        *reinterpret_cast<Pack8*>(p.out + static_cast<int64_t>(qstart + qlen - 1) * p.out_stride +
                                  static_cast<int64_t>(head) * kD + d0) = o8;
      }
    }
  } else {
    if (c_valid) {
      const float invL = l_run > 0.f ? 1.f / l_run : 0.f;
      uint16_t* op = p.out + static_cast<int64_t>(qstart + c_tok) * p.out_stride +
                     static_cast<int64_t>(c_head) * kD;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        Pack4 o4;
#pragma unroll
        for (int i = 0; i < 4; ++i) o4.v[i] = from_f32<T>(o_acc[dt][i] * invL);
        *reinterpret_cast<Pack4*>(op + 16 * dt + 4 * grp) = o4;
      }
    }
  }
}

// Reduce decode partitions: out[s, head, :] = sum_p w_p O_p, w_p = 2^(lse_p - lse*) / sum.
template <typename T>
__global__ __launch_bounds__(128) void attn_combine_kernel(AttnParams p, int G) {
  const int s = blockIdx.x;
  const int head = blockIdx.y;
  const int hk = head / G;
  const int c = head % G;
  const int d = threadIdx.x;
  const int64_t base = ((static_cast<int64_t>(s) * p.n_kv_heads + hk) * p.num_parts) * 16 + c;
  float mx = kNegInf;
  for (int q = 0; q < p.num_parts; ++q) mx = fmaxf(mx, p.part_lse[base + q * 16]);
  float acc = 0.f, wsum = 0.f;
  if (mx != kNegInf) {
    for (int q = 0; q < p.num_parts; ++q) {
      const float l = p.part_lse[base + q * 16];
      if (l == kNegInf) continue;
      const float w = exp2f(l - mx);
      wsum += w;
      acc += w * p.part_out[(base + q * 16) * kD + d];
    }
  }
  const int qrow = p.seq_qstart[s + 1] - 1;
  p.out[static_cast<int64_t>(qrow) * p.out_stride + static_cast<int64_t>(head) * kD + d] =
      from_f32<T>(wsum > 0.f ? acc / wsum : 0.f);
}

template <typename T, bool kSplit>
static void launch_attn(const AttnParams& prm, int G, dim3 grid, hipStream_t stream) {
  switch (G) {
    case 1: paged_attention_kernel<T, 1, kSplit><<<grid, 256, 0, stream>>>(prm); break;
    case 2: paged_attention_kernel<T, 2, kSplit><<<grid, 256, 0, stream>>>(prm); break;
    case 3: paged_attention_kernel<T, 3, kSplit><<<grid, 256, 0, stream>>>(prm); break;
    case 4: paged_attention_kernel<T, 4, kSplit><<<grid, 256, 0, stream>>>(prm); break;
    case 8: paged_attention_kernel<T, 8, kSplit><<<grid, 256, 0, stream>>>(prm); break;
    default: break;
  }
}

}  // namespace atta

using namespace atta;

static int bs_to_shift(int bs) {
  int s = 0;
  while ((1 << s) < bs) ++s;
  return ((1 << s) == bs && bs >= 16) ? s : -1;
}

int atta_attention_prefill(void* out, const void* q, const void* k_cache, const void* v_cache,
                           const int* block_tables, const int* seq_kvlen, const int* seq_qstart,
                           const int* tile_seq, const int* tile_qoff, int num_tiles,
                           int n_q_heads, int n_kv_heads, int head_dim, int block_size,
                           int bt_stride, int64_t q_stride, int64_t out_stride, float scale,
                           int dtype, hipStream_t stream) {
  const int G = n_q_heads / n_kv_heads;
  const int shift = bs_to_shift(block_size);
  if (head_dim != kD || shift < 0 || n_q_heads % n_kv_heads != 0 || ((G & (G - 1)) && G != 3) || G > 8)
    return -1;
  if (num_tiles == 0) return 0;
  AttnParams prm{};
  prm.out = static_cast<uint16_t*>(out);
  prm.q = static_cast<const uint16_t*>(q);
  prm.k_cache = static_cast<const uint16_t*>(k_cache);
  prm.v_cache = static_cast<const uint16_t*>(v_cache);
  prm.block_tables = block_tables;
  prm.seq_kvlen = seq_kvlen;
  prm.seq_qstart = seq_qstart;
  prm.tile_seq = tile_seq;
  prm.tile_qoff = tile_qoff;
  prm.q_stride = q_stride;
  prm.out_stride = out_stride;
  prm.bt_stride = bt_stride;
  prm.n_q_heads = n_q_heads;
  prm.n_kv_heads = n_kv_heads;
  prm.bs_shift = shift;
  prm.num_parts = 1;
  prm.scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(num_tiles, n_kv_heads);
  if (dtype == 0)
    launch_attn<__bf16, false>(prm, G, grid, stream);
  else
    launch_attn<_Float16, false>(prm, G, grid, stream);
  return static_cast<int>(hipGetLastError());
}

int atta_attention_decode(void* out, float* part_out, float* part_lse, const void* q,
                          const void* k_cache, const void* v_cache, const int* block_tables,
                          const int* seq_kvlen, const int* seq_qstart, int num_seqs,
                          int num_parts, int part_tokens, int n_q_heads, int n_kv_heads,
                          int head_dim, int block_size, int bt_stride, int64_t q_stride,
                          int64_t out_stride, float scale, int dtype, hipStream_t stream) {
  const int G = n_q_heads / n_kv_heads;
  const int shift = bs_to_shift(block_size);
  if (head_dim != kD || shift < 0 || n_q_heads % n_kv_heads != 0 || ((G & (G - 1)) && G != 3) || G > 8)
    return -1;
  if (part_tokens % 64 != 0 || num_parts < 1) return -1;
  if (num_seqs == 0) return 0;
  AttnParams prm{};
  prm.out = static_cast<uint16_t*>(out);
  prm.part_out = part_out;
  prm.part_lse = part_lse;
  prm.q = static_cast<const uint16_t*>(q);
  prm.k_cache = static_cast<const uint16_t*>(k_cache);
  prm.v_cache = static_cast<const uint16_t*>(v_cache);
  prm.block_tables = block_tables;
  prm.seq_kvlen = seq_kvlen;
  prm.seq_qstart = seq_qstart;
  prm.q_stride = q_stride;
  prm.out_stride = out_stride;
  prm.bt_stride = bt_stride;
  prm.n_q_heads = n_q_heads;
  prm.n_kv_heads = n_kv_heads;
  prm.bs_shift = shift;
  prm.part_tokens = part_tokens;
  prm.num_parts = num_parts;
  prm.scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(num_seqs, n_kv_heads, num_parts);
  if (dtype == 0)
    launch_attn<__bf16, true>(prm, G, grid, stream);
  else
    launch_attn<_Float16, true>(prm, G, grid, stream);
  if (num_parts > 1) {
    dim3 g2(num_seqs, n_q_heads);
    if (dtype == 0)
      attn_combine_kernel<__bf16><<<g2, 128, 0, stream>>>(prm, G);
    else
      attn_combine_kernel<_Float16><<<g2, 128, 0, stream>>>(prm, G);
  }
  return static_cast<int>(hipGetLastError());
}
