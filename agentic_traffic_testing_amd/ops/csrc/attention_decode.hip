// Decode paged attention v2: split-K over context partitions with an in-kernel combine
// (guide §5 "In-launch split-K reduction").
//
// grid = (seqs, kv_heads, max_partitions), 4 waves per workgroup.  One workgroup handles
// `part_tokens` tokens of one (sequence, KV head); its 4 waves take every 4th 16-token tile
// and keep the next tile's K/V fragments in flight while computing the current one
// (register double buffer).  The GQA group's G query heads are the MFMA columns (same
// swapped-QK^T formulation as attention.hip).  Partitions past the sequence end exit at
// once, so a hipGraph captured with the maximum partition count costs nothing extra for
// short contexts.
//
// Combine: every partition writes (O normalised, lse) fp32 to a workspace, then arrives on
// a per-(seq, kv-head) counter with an agent-scope release; the last arriver acquires,
// merges all partitions and writes the bf16 output, then re-arms the counter (counters are
// zeroed once at allocation).  A context that fits one partition skips the workspace.
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
};

template <typename T>
struct TileFrags {
  typename Mf<T>::frag8 k[4];
  i16x4 v[8];
};

template <typename T>
__device__ __forceinline__ void load_tile(TileFrags<T>& f, const DecParams& p, const int* bt,
                                          int kt, int kvlen, int hk, int col, int grp) {
  using frag8 = typename Mf<T>::frag8;
  const int BS = 1 << p.bs_shift;
  const int64_t hs = static_cast<int64_t>(BS) * kD;
  const int tk = kt + col;
  const int pk = tk < kvlen ? bt[tk >> p.bs_shift] : 0;
  const uint16_t* kp = p.k_cache + (static_cast<int64_t>(pk) * p.n_kv_heads + hk) * hs +
                       static_cast<int64_t>(tk & (BS - 1)) * kD + 32 * grp;
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) f.k[kk] = *reinterpret_cast<const frag8*>(kp + 8 * kk);
  const int tv = kt + 4 * grp;
  const int pv = tv < kvlen ? bt[tv >> p.bs_shift] : 0;
  const uint16_t* vp = p.v_cache + (static_cast<int64_t>(pv) * p.n_kv_heads + hk) * hs +
                       static_cast<int64_t>(col) * BS + (tv & (BS - 1));
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
    f.v[dt] = *reinterpret_cast<const i16x4*>(vp + static_cast<int64_t>(16 * dt) * BS);
}

template <typename T>
__device__ __forceinline__ void compute_tile(const TileFrags<T>& f,
                                             const typename Mf<T>::frag8 (&qf)[4], int kt,
                                             int kv_end, int grp, float scale_log2, float& m_run,
                                             float& l_run, f32x4 (&o)[8]) {
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) s = Mf<T>::qk(f.k[kk], qf[kk], s);
  float sv[4], tmax = kNegInf;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sv[i] = (kt + 4 * grp + i < kv_end) ? s[i] * scale_log2 : kNegInf;
    tmax = fmaxf(tmax, sv[i]);
  }
  tmax = fmaxf(tmax, __shfl_xor(tmax, 16, kWave));
  tmax = fmaxf(tmax, __shfl_xor(tmax, 32, kWave));
  const float m_new = fmaxf(m_run, tmax);
  const float m_use = (m_new == kNegInf) ? 0.f : m_new;
  const float alpha = exp2f(m_run - m_use);
  float psum = 0.f;
  i16x4 pf;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float pv = exp2f(sv[i] - m_use);
    psum += pv;
    pf[i] = static_cast<short>(from_f32<T>(pv));
  }
  psum += __shfl_xor(psum, 16, kWave);
  psum += __shfl_xor(psum, 32, kWave);
  l_run = l_run * alpha + psum;
  m_run = m_new;
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) {
    o[dt] *= alpha;
    o[dt] = Mf<T>::pv(f.v[dt], pf, o[dt]);
  }
}

template <typename T, int G>
__global__ __launch_bounds__(256) void decode_attention_kernel(DecParams p) {
  using frag8 = typename Mf<T>::frag8;
  __shared__ float lds_o[4][16][kD + 4];
  __shared__ float lds_m[4][16];
  __shared__ float lds_l[4][16];
  __shared__ int lds_last;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int col = lane & 15;
  const int grp = lane >> 4;
  const int s = blockIdx.x;
  const int hk = blockIdx.y;
  const int part = blockIdx.z;
  const int kvlen = p.seq_kvlen[s];
  const int nparts = (kvlen + p.part_tokens - 1) / p.part_tokens;
  if (part >= nparts) return;  // block-uniform; also covers kvlen == 0 dummy sequences
  const int kv_begin = part * p.part_tokens;
  const int kv_end = min(kvlen, kv_begin + p.part_tokens);
  const int qrow = p.seq_qstart[s + 1] - 1;

  // Q fragment: column = GQA head (col < G), dims 32*grp + 8*kk + j
  frag8 qf[4];
  {
    const bool ok = col < G;
    const uint16_t* qp = p.q + static_cast<int64_t>(qrow) * p.q_stride +
                         static_cast<int64_t>(hk * G + (ok ? col : 0)) * kD + 32 * grp;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
      qf[kk] = ok ? *reinterpret_cast<const frag8*>(qp + 8 * kk) : frag8{};
  }
  f32x4 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = kNegInf, l_run = 0.f;
  const int* bt = p.block_tables + static_cast<int64_t>(s) * p.bt_stride;

  int kt = kv_begin + wid * 16;
  if (kt < kv_end) {
    TileFrags<T> fa, fb;
    load_tile<T>(fa, p, bt, kt, kvlen, hk, col, grp);
    while (true) {
      const int kn = kt + 64;
      if (kn < kv_end) load_tile<T>(fb, p, bt, kn, kvlen, hk, col, grp);
      compute_tile<T>(fa, qf, kt, kv_end, grp, p.scale_log2, m_run, l_run, o);
      if (kn >= kv_end) break;
      const int kn2 = kn + 64;
      if (kn2 < kv_end) load_tile<T>(fa, p, bt, kn2, kvlen, hk, col, grp);
      compute_tile<T>(fb, qf, kn, kv_end, grp, p.scale_log2, m_run, l_run, o);
      if (kn2 >= kv_end) break;
      kt = kn2;
    }
  }

  // ---- merge the 4 waves -----------------------------------------------------------------
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) lds_o[wid][col][16 * dt + 4 * grp + i] = o[dt][i];
  if (grp == 0) {
    lds_m[wid][col] = m_run;
    lds_l[wid][col] = l_run;
  }
  __syncthreads();
  const int c = threadIdx.x >> 4;         // column 0..15
  const int d0 = (threadIdx.x & 15) * 8;  // dims d0..d0+7
  float mw[4], mx = kNegInf;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    mw[w] = lds_m[w][c];
    mx = fmaxf(mx, mw[w]);
  }
  const float mu = (mx == kNegInf) ? 0.f : mx;
  float L = 0.f, fw[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    fw[w] = exp2f(mw[w] - mu);
    L += fw[w] * lds_l[w][c];
  }
  const float invL = L > 0.f ? 1.f / L : 0.f;
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) a += fw[w] * lds_o[w][c][d0 + j];
    r[j] = a * invL;
  }
  uint16_t* outp = p.out + static_cast<int64_t>(qrow) * p.out_stride +
                   static_cast<int64_t>(hk * G + c) * kD + d0;
  if (nparts == 1) {
    if (c < G) {
      Pack8 o8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o8.v[j] = from_f32<T>(r[j]);
      *reinterpret_cast<Pack8*>(outp) = o8;
    }
    return;
  }

  // ---- publish this partition, last arriver combines ----------------------------------------
  const int64_t sh = static_cast<int64_t>(s) * p.n_kv_heads + hk;
  if (c < G) {
    const int64_t base = (sh * p.max_parts + part) * 16 + c;
    float* po = p.part_out + base * kD + d0;
    *reinterpret_cast<float4*>(po) = make_float4(r[0], r[1], r[2], r[3]);
    *reinterpret_cast<float4*>(po + 4) = make_float4(r[4], r[5], r[6], r[7]);
    if ((threadIdx.x & 15) == 0) p.part_lse[base] = (L > 0.f) ? (mu + log2f(L)) : kNegInf;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(p.counters + sh, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    const int last = (old == nparts - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_last = last;
  }
  __syncthreads();
  if (!lds_last) return;
  if (c < G) {
    float lmax = kNegInf;
    for (int q = 0; q < nparts; ++q)
      lmax = fmaxf(lmax, p.part_lse[(sh * p.max_parts + q) * 16 + c]);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float wsum = 0.f;
    if (lmax != kNegInf) {
      for (int q = 0; q < nparts; ++q) {
        const int64_t base = (sh * p.max_parts + q) * 16 + c;
        const float l = p.part_lse[base];
        if (l == kNegInf) continue;
        const float w = exp2f(l - lmax);
        wsum += w;
        const float4 a = *reinterpret_cast<const float4*>(p.part_out + base * kD + d0);
        const float4 b = *reinterpret_cast<const float4*>(p.part_out + base * kD + d0 + 4);
        acc[0] += w * a.x; acc[1] += w * a.y; acc[2] += w * a.z; acc[3] += w * a.w;
        acc[4] += w * b.x; acc[5] += w * b.y; acc[6] += w * b.z; acc[7] += w * b.w;
      }
    }
    const float inv = wsum > 0.f ? 1.f / wsum : 0.f;
    Pack8 o8;
#pragma unroll
    for (int j = 0; j < 8; ++j) o8.v[j] = from_f32<T>(acc[j] * inv);
    *reinterpret_cast<Pack8*>(outp) = o8;
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(p.counters + sh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T>
static void launch(int G, dim3 grid, hipStream_t st, const DecParams& p) {
  switch (G) {
    case 1: decode_attention_kernel<T, 1><<<grid, 256, 0, st>>>(p); break;
    case 2: decode_attention_kernel<T, 2><<<grid, 256, 0, st>>>(p); break;
    case 4: decode_attention_kernel<T, 4><<<grid, 256, 0, st>>>(p); break;
    case 8: decode_attention_kernel<T, 8><<<grid, 256, 0, st>>>(p); break;
    case 16: decode_attention_kernel<T, 16><<<grid, 256, 0, st>>>(p); break;
    default: break;
  }
}

}  // namespace dec
}  // namespace atta

using namespace atta;

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
  if (n_q_heads % n_kv_heads || G > 16 || (G & (G - 1))) return -1;
  if (part_tokens % 64 != 0 || max_parts < 1) return -1;
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
  dim3 grid(num_seqs, n_kv_heads, max_parts);
  if (dtype == 0)
    dec::launch<__bf16>(G, grid, stream, p);
  else
    dec::launch<_Float16>(G, grid, stream, p);
  return static_cast<int>(hipGetLastError());
}
