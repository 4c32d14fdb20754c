// Skinny (decode) GEMM on MFMA: y[M, N] = x[M, K] . W[N, K]^T  (+ residual), M <= 64.
//
// Decode steps of the 8B model stream ~15 GB of weights per token while M (= sequences in
// the batch) is 1..16, so the layer GEMMs are pure HBM streams.  Design (guide: "GEMV /
// M <= 16 decode weights: load straight to VGPRs, deep unroll, late vmcnt"):
//   * one workgroup owns 16 output features (16 weight rows); its WAVES waves split K, each
//     streams its K slice of the 16 rows with 16-byte loads (UNROLL loads in flight/wave);
//   * the 16 rows x 32 k chunk a wave loads is exactly the B operand of
//     mfma_f32_16x16x32_bf16 (lane l: row n0 + (l&15), k = 8(l>>4)..+8), the x chunk is the A
//     operand (lane l: x row l&15) - x is tiny and L1/L2 resident, rows >= M are zeros;
//     MT 16-row tiles of x reuse each weight fragment (M up to 16*MT);
//   * partial 16x16 tiles of the waves are summed through LDS; the epilogue optionally
//     adds a residual row block (o_proj / down_proj -> residual stream).
// grid = N / 16 workgroups (256 for N = 4096, 1792 for the gate_up projection).
#include "common.h"
#include "kernels.h"

namespace atta {

template <typename T>
struct MfmaK32;
template <>
struct MfmaK32<__bf16> {
  typedef bf16x8 frag8;
  __device__ static __forceinline__ f32x4 mma(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct MfmaK32<_Float16> {
  typedef f16x8 frag8;
  __device__ static __forceinline__ f32x4 mma(frag8 a, frag8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

template <typename T, int WAVES, int UNROLL, int MT>
__global__ __launch_bounds__(WAVES * 64) void skinny_gemm_kernel(
    uint16_t* __restrict__ y, const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
    const uint16_t* __restrict__ res, int M, int N, int K, int64_t x_stride, int64_t y_stride,
    int64_t res_stride) {
  using frag8 = typename MfmaK32<T>::frag8;
  __shared__ float red[WAVES][MT][16][17];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int col = lane & 15;
  const int grp = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int kw = K / WAVES;  // K % (32 * WAVES) == 0 checked on the host
  const int kbeg = wid * kw;
  const uint16_t* wp = w + static_cast<int64_t>(n0 + col) * K + kbeg + 8 * grp;
  const uint16_t* xp[MT];
  bool xv[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + col;
    xv[t] = m < M;
    xp[t] = x + static_cast<int64_t>(xv[t] ? m : 0) * x_stride + kbeg + 8 * grp;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  int k = 0;
  constexpr int STEP = 32 * UNROLL;
  for (; k + STEP <= kw; k += STEP) {
    frag8 wf[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      wf[u] = __builtin_nontemporal_load(reinterpret_cast<const frag8*>(wp + k + 32 * u));
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      frag8 xf[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u)
        xf[u] = xv[t] ? *reinterpret_cast<const frag8*>(xp[t] + k + 32 * u) : frag8{};
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) acc[t] = MfmaK32<T>::mma(xf[u], wf[u], acc[t]);
    }
  }
  for (; k < kw; k += 32) {
    frag8 wf = __builtin_nontemporal_load(reinterpret_cast<const frag8*>(wp + k));
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      frag8 xf = xv[t] ? *reinterpret_cast<const frag8*>(xp[t] + k) : frag8{};
      acc[t] = MfmaK32<T>::mma(xf, wf, acc[t]);
    }
  }

  // C layout: row m = 4*grp + i, col n = lane & 15
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wid][t][4 * grp + i][col] = acc[t][i];
  __syncthreads();
  for (int e = threadIdx.x; e < MT * 256; e += WAVES * 64) {
    const int t = e >> 8;
    const int m = (e >> 4) & 15;
    const int n = e & 15;
    const int row = t * 16 + m;
    if (row >= M) continue;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) s += red[q][t][m][n];
    if (res != nullptr) {
      // round the GEMM result first (matches F.linear followed by a bf16 add)
      s = to_f32<T>(from_f32<T>(s)) + to_f32<T>(res[static_cast<int64_t>(row) * res_stride + n0 + n]);
    }
    y[static_cast<int64_t>(row) * y_stride + n0 + n] = from_f32<T>(s);
  }
}

template <typename T, int WAVES, int UNROLL>
static void launch_skinny(int mt, dim3 grid, hipStream_t st, uint16_t* y, const uint16_t* x,
                          const uint16_t* w, const uint16_t* res, int M, int N, int K,
                          int64_t xs, int64_t ys, int64_t rs) {
  switch (mt) {
    case 1:
      skinny_gemm_kernel<T, WAVES, UNROLL, 1><<<grid, WAVES * 64, 0, st>>>(y, x, w, res, M, N, K,
                                                                          xs, ys, rs);
      break;
    case 2:
      skinny_gemm_kernel<T, WAVES, UNROLL, 2><<<grid, WAVES * 64, 0, st>>>(y, x, w, res, M, N, K,
                                                                          xs, ys, rs);
      break;
    default:
      skinny_gemm_kernel<T, WAVES, UNROLL, 4><<<grid, WAVES * 64, 0, st>>>(y, x, w, res, M, N, K,
                                                                          xs, ys, rs);
      break;
  }
}

}  // namespace atta

using namespace atta;

int atta_skinny_gemm(void* y, const void* x, const void* w, const void* residual, int M, int N,
                     int K, int64_t x_stride, int64_t y_stride, int64_t res_stride, int waves,
                     int dtype, hipStream_t stream) {
  if (M < 1 || M > 64 || N % 16 != 0) return -1;
  if (waves != 4 && waves != 8) waves = 4;
  if (K % (32 * waves) != 0) return -1;
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  dim3 grid(N / 16);
  auto yo = static_cast<uint16_t*>(y);
  auto xi = static_cast<const uint16_t*>(x);
  auto wi = static_cast<const uint16_t*>(w);
  auto ri = static_cast<const uint16_t*>(residual);
  if (dtype == 0) {
    if (waves == 8)
      launch_skinny<__bf16, 8, 8>(mt, grid, stream, yo, xi, wi, ri, M, N, K, x_stride, y_stride,
                                  res_stride);
    else
      launch_skinny<__bf16, 4, 8>(mt, grid, stream, yo, xi, wi, ri, M, N, K, x_stride, y_stride,
                                  res_stride);
  } else {
    if (waves == 8)
      launch_skinny<_Float16, 8, 8>(mt, grid, stream, yo, xi, wi, ri, M, N, K, x_stride, y_stride,
                                    res_stride);
    else
      launch_skinny<_Float16, 4, 8>(mt, grid, stream, yo, xi, wi, ri, M, N, K, x_stride, y_stride,
                                    res_stride);
  }
  return static_cast<int>(hipGetLastError());
}
