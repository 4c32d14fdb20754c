// Per-token (row-wise) OCP e4m3fn activation quantisation fused into the producing
// elementwise op.  The fp8 prefill path runs every projection as one
// hipBLASLt fp8 GEMM with row-wise scales on both operands (torch._scaled_mm: fp8 MFMA,
// y = (s_x[m] s_w[n]) sum_k q_x[m,k] q_w[n,k], bf16 out), so the activations have to arrive
// as (fp8 row, fp32 row scale) - these kernels produce them in the pass that computes them:
//
//   MODE_NORM : q, s <- quant(rmsnorm(x) * w)            (input / post-attention norms)
//   MODE_SILU : q, s <- quant(silu(gate) * up)           (gate | up packed, width 2I)
//   MODE_PLAIN: q, s <- quant(x)                          (attention output -> o_proj)
//   MODE_ADDNORM: r <- r + x (residual stream, rounded to T, written back);
//                 q, s <- quant(rmsnorm(r) * w)          (GEMM output + residual + norm)
//
// One workgroup per row.  Rows up to 4096 8-wide vectors (every Llama width here) keep their
// values in registers between the block reduction and the quantisation (one HBM read,
// quant_rows_reg_kernel); wider rows take two passes over the (L2-resident) row: pass 1 gathers
// sum(x^2) (norm) and the row amax of the unscaled values, pass 2 recomputes each value,
// divides by s = amax / 448 and converts pairs with v_cvt_pk_fp8_f32 (values pre-clamped to
// +-448, the e4m3fn finite range).  Rows of zeros get s = 1 (all-zero codes).
#include "common.h"
#include "kernels.h"

namespace atta {
namespace q8 {

constexpr int kThreads = 256;
constexpr float kFp8Max = 448.f;
enum Mode { MODE_NORM = 0, MODE_SILU = 1, MODE_PLAIN = 2, MODE_ADDNORM = 3 };

template <typename T, int MODE>
__device__ __forceinline__ void load8(float (&v)[8], const uint16_t* x, const uint16_t* w,
                                      int inter, int idx) {
  const Pack8 a = *reinterpret_cast<const Pack8*>(x + 8 * idx);
  if constexpr (MODE == MODE_SILU) {
    const Pack8 b = *reinterpret_cast<const Pack8*>(x + inter + 8 * idx);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = to_f32<T>(a.v[j]);
      // silu rounded to T first: the same value the bf16 silu_and_mul kernel produces
      const float sg = to_f32<T>(from_f32<T>(g / (1.f + __expf(-g))));
      v[j] = sg * to_f32<T>(b.v[j]);
    }
  } else if constexpr (MODE == MODE_NORM || MODE == MODE_ADDNORM) {
    const Pack8 ww = *reinterpret_cast<const Pack8*>(w + 8 * idx);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = to_f32<T>(a.v[j]) * to_f32<T>(ww.v[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = to_f32<T>(a.v[j]);
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(kThreads) void quant_rows_kernel(
    uint8_t* __restrict__ q, float* __restrict__ scale, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ w, int width, int64_t x_stride, int64_t q_stride, float eps,
    uint16_t* __restrict__ residual, int64_t res_stride) {
  __shared__ float red[2][kThreads / kWave];
  const int64_t row = blockIdx.x;
  const uint16_t* xr = x + row * x_stride;
  const int nvec = width >> 3;
  if constexpr (MODE == MODE_ADDNORM) {
    // r <- r + x; every later read of this row is of r (each thread re-reads only the
    // chunks it wrote itself: program order, no barrier needed)
    uint16_t* rr = residual + row * res_stride;
    for (int i = threadIdx.x; i < nvec; i += kThreads) {
      const Pack8 a = *reinterpret_cast<const Pack8*>(xr + 8 * i);
      Pack8 b = *reinterpret_cast<const Pack8*>(rr + 8 * i);
#pragma unroll
      for (int j = 0; j < 8; ++j) b.v[j] = from_f32<T>(to_f32<T>(a.v[j]) + to_f32<T>(b.v[j]));
      *reinterpret_cast<Pack8*>(rr + 8 * i) = b;
    }
    xr = rr;
  }
  float ss = 0.f, amax = 0.f;
  for (int i = threadIdx.x; i < nvec; i += kThreads) {
    float v[8];
    if constexpr (MODE == MODE_NORM || MODE == MODE_ADDNORM) {
      const Pack8 a = *reinterpret_cast<const Pack8*>(xr + 8 * i);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = to_f32<T>(a.v[j]);
        ss += f * f;
      }
    }
    load8<T, MODE>(v, xr, w, width, i);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
  }
  // block reduction of (ss, amax)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ss += __shfl_xor(ss, o, kWave);
    amax = fmaxf(amax, __shfl_xor(amax, o, kWave));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = ss;
    red[1][wid] = amax;
  }
  __syncthreads();
  ss = 0.f;
  amax = 0.f;
#pragma unroll
  for (int k = 0; k < kThreads / kWave; ++k) {
    ss += red[0][k];
    amax = fmaxf(amax, red[1][k]);
  }
  const float inv_rms = (MODE == MODE_NORM || MODE == MODE_ADDNORM)
                            ? rsqrtf(ss / static_cast<float>(width) + eps)
                            : 1.f;
  amax *= inv_rms;
  const float s = amax > 0.f ? amax / kFp8Max : 1.f;
  const float rs = inv_rms / s;
  if (threadIdx.x == 0) scale[row] = s;
  uint8_t* qr = q + row * q_stride;
  for (int i = threadIdx.x; i < nvec; i += kThreads) {
    float v[8];
    load8<T, MODE>(v, xr, w, width, i);
    float c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fminf(fmaxf(v[j] * rs, -kFp8Max), kFp8Max);
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
    *reinterpret_cast<uint2*>(qr + 8 * i) =
        make_uint2(static_cast<uint32_t>(lo), static_cast<uint32_t>(hi));
  }
}

// Register-resident variant (rows that fit THREADS x NPT 8-wide vectors): the row is read
// from HBM once - each thread keeps its unscaled values (and, for the norms, the RMS
// sum) in registers across the block reduction, so pass 2 neither re-reads the row nor
// recomputes SiLU.  Prefill 2.6k rows: SiLU-mul 14336 and residual-add + norm 4096 were
// ~3 TB/s as two passes over L2.  Same per-element arithmetic as quant_rows_kernel.
template <typename T, int MODE, int THREADS, int NPT>
__global__ __launch_bounds__(THREADS) void quant_rows_reg_kernel(
    uint8_t* __restrict__ q, float* __restrict__ scale, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ w, int width, int64_t x_stride, int64_t q_stride, float eps,
    uint16_t* __restrict__ residual, int64_t res_stride) {
  __shared__ float red[2][THREADS / kWave];
  const int64_t row = blockIdx.x;
  const uint16_t* xr = x + row * x_stride;
  const int nvec = width >> 3;
  float v[NPT][8];
  float ss = 0.f, amax = 0.f;
#pragma unroll
  for (int it = 0; it < NPT; ++it) {
    const int i = threadIdx.x + it * THREADS;
    if (i < nvec) {
      if constexpr (MODE == MODE_ADDNORM || MODE == MODE_NORM) {
        Pack8 a = *reinterpret_cast<const Pack8*>(xr + 8 * i);
        const Pack8 ww = *reinterpret_cast<const Pack8*>(w + 8 * i);
        if constexpr (MODE == MODE_ADDNORM) {
          uint16_t* rr = residual + row * res_stride;
          const Pack8 b = *reinterpret_cast<const Pack8*>(rr + 8 * i);
#pragma unroll
          for (int j = 0; j < 8; ++j) a.v[j] = from_f32<T>(to_f32<T>(a.v[j]) + to_f32<T>(b.v[j]));
          *reinterpret_cast<Pack8*>(rr + 8 * i) = a;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = to_f32<T>(a.v[j]);
          ss += f * f;
          v[it][j] = f * to_f32<T>(ww.v[j]);
        }
      } else {
        load8<T, MODE>(v[it], xr, w, width, i);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[it][j]));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ss += __shfl_xor(ss, o, kWave);
    amax = fmaxf(amax, __shfl_xor(amax, o, kWave));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wid] = ss;
    red[1][wid] = amax;
  }
  __syncthreads();
  ss = 0.f;
  amax = 0.f;
#pragma unroll
  for (int k = 0; k < THREADS / kWave; ++k) {
    ss += red[0][k];
    amax = fmaxf(amax, red[1][k]);
  }
  const float inv_rms = (MODE == MODE_NORM || MODE == MODE_ADDNORM)
                            ? rsqrtf(ss / static_cast<float>(width) + eps)
                            : 1.f;
  amax *= inv_rms;
  const float s = amax > 0.f ? amax / kFp8Max : 1.f;
  const float rs = inv_rms / s;
  if (threadIdx.x == 0) scale[row] = s;
  uint8_t* qr = q + row * q_stride;
#pragma unroll
  for (int it = 0; it < NPT; ++it) {
    const int i = threadIdx.x + it * THREADS;
    if (i < nvec) {
      float c[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) c[j] = fminf(fmaxf(v[it][j] * rs, -kFp8Max), kFp8Max);
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], lo, true);
      int hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], hi, true);
      *reinterpret_cast<uint2*>(qr + 8 * i) =
          make_uint2(static_cast<uint32_t>(lo), static_cast<uint32_t>(hi));
    }
  }
}

template <typename T, int MODE>
static bool launch_reg(uint8_t* q, float* scale, const uint16_t* x, const uint16_t* w, int rows,
                       int width, int64_t x_stride, int64_t q_stride, float eps, uint16_t* res,
                       int64_t res_stride, hipStream_t st) {
  const int nvec = width / 8;
  const dim3 grid(rows);
#define ATTA_QREG(TH_, NPT_)                                                              \
  quant_rows_reg_kernel<T, MODE, TH_, NPT_><<<grid, TH_, 0, st>>>(q, scale, x, w, width,    \
                                                                   x_stride, q_stride, eps, \
                                                                   res, res_stride)
  if (nvec <= 256 * 2) ATTA_QREG(256, 2);
  else if (nvec <= 256 * 4) ATTA_QREG(256, 4);
  else if (nvec <= 1024 * 2) ATTA_QREG(1024, 2);
  else if (nvec <= 1024 * 4) ATTA_QREG(1024, 4);
  else return false;
#undef ATTA_QREG
  return true;
}

template <typename T>
static int launch(int mode, uint8_t* q, float* scale, const uint16_t* x, const uint16_t* w,
                  int rows, int width, int64_t x_stride, int64_t q_stride, float eps,
                  uint16_t* res, int64_t res_stride, hipStream_t st) {
  const dim3 grid(rows), blk(kThreads);
  switch (mode) {
    case MODE_NORM:
      if (launch_reg<T, MODE_NORM>(q, scale, x, w, rows, width, x_stride, q_stride, eps, res,
                                   res_stride, st))
        return 0;
      break;
    case MODE_SILU:
      if (launch_reg<T, MODE_SILU>(q, scale, x, w, rows, width, x_stride, q_stride, eps, res,
                                   res_stride, st))
        return 0;
      break;
    case MODE_PLAIN:
      if (launch_reg<T, MODE_PLAIN>(q, scale, x, w, rows, width, x_stride, q_stride, eps, res,
                                    res_stride, st))
        return 0;
      break;
    case MODE_ADDNORM:
      if (launch_reg<T, MODE_ADDNORM>(q, scale, x, w, rows, width, x_stride, q_stride, eps, res,
                                      res_stride, st))
        return 0;
      break;
    default:
      return -1;
  }
  switch (mode) {
    case MODE_NORM:
      quant_rows_kernel<T, MODE_NORM><<<grid, blk, 0, st>>>(q, scale, x, w, width, x_stride,
                                                            q_stride, eps, res, res_stride);
      return 0;
    case MODE_SILU:
      quant_rows_kernel<T, MODE_SILU><<<grid, blk, 0, st>>>(q, scale, x, w, width, x_stride,
                                                            q_stride, eps, res, res_stride);
      return 0;
    case MODE_PLAIN:
      quant_rows_kernel<T, MODE_PLAIN><<<grid, blk, 0, st>>>(q, scale, x, w, width, x_stride,
                                                             q_stride, eps, res, res_stride);
      return 0;
    case MODE_ADDNORM:
      quant_rows_kernel<T, MODE_ADDNORM><<<grid, blk, 0, st>>>(q, scale, x, w, width, x_stride,
                                                               q_stride, eps, res, res_stride);
      return 0;
    default:
      return -1;
  }
}

}  // namespace q8
}  // namespace atta

using namespace atta;

int atta_quant_rows_fp8(void* q, float* scale, const void* x, const void* w, int rows, int width,
                        int64_t x_stride, int64_t q_stride, int mode, float eps, void* residual,
                        int64_t res_stride, int dtype, hipStream_t stream) {
  if (width % 8 != 0 || x_stride % 8 != 0 || q_stride % 8 != 0) return -1;
  if ((mode == q8::MODE_NORM || mode == q8::MODE_ADDNORM) && w == nullptr) return -1;
  if (mode == q8::MODE_ADDNORM && (residual == nullptr || res_stride % 8 != 0)) return -1;
  auto ro = static_cast<uint16_t*>(residual);
  if (rows == 0) return 0;
  auto qo = static_cast<uint8_t*>(q);
  auto xi = static_cast<const uint16_t*>(x);
  auto wi = static_cast<const uint16_t*>(w);
  const int rc = dtype == 0
                     ? q8::launch<__bf16>(mode, qo, scale, xi, wi, rows, width, x_stride, q_stride, eps, ro, res_stride, stream)
                     : q8::launch<_Float16>(mode, qo, scale, xi, wi, rows, width, x_stride, q_stride, eps, ro, res_stride, stream);
  if (rc) return rc;
  return static_cast<int>(hipGetLastError());
}
