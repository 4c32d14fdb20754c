// Torch operator registration for the CDNA4 kernel library (namespace `atta`).
//
// Each op validates shapes/dtypes on the host, then calls the raw-pointer launcher on
// the current HIP stream, so ops are safe inside torch.cuda.graph capture (no
// allocation, no sync).  Ops only accept device tensors: CPU execution of the same math
// lives in ops/reference.py and is selected by the Python wrappers by tensor device,
// never as a silent fallback for a GPU tensor.
#include <string>
#include <vector>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dtype_code(const at::Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return 0;
  if (t.scalar_type() == at::kHalf) return 1;
  TORCH_CHECK(false, "atta: expected bf16/fp16 tensor, got ", t.scalar_type());
}

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "atta::", what, " launch failed (rc=", rc, ")");
}

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "atta: ", name, " must be a GPU tensor");
}

void rms_norm(at::Tensor out, const at::Tensor& x, const at::Tensor& w, double eps) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && out.stride(1) == 1, "rms_norm: 2-D rows");
  const at::DeviceGuard g(x.device());
  check_rc(atta_rms_norm(out.data_ptr(), nullptr, x.data_ptr(), w.data_ptr(), x.size(0),
                         x.size(1), x.stride(0), out.stride(0), 0, static_cast<float>(eps),
                         dtype_code(x), cur_stream()),
           "rms_norm");
}

void fused_add_rms_norm(at::Tensor out, at::Tensor residual, const at::Tensor& x,
                        const at::Tensor& w, double eps) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && residual.stride(1) == 1 && out.stride(1) == 1,
              "fused_add_rms_norm: 2-D rows");
  TORCH_CHECK(residual.sizes() == x.sizes(), "fused_add_rms_norm: residual shape");
  const at::DeviceGuard g(x.device());
  check_rc(atta_rms_norm(out.data_ptr(), residual.data_ptr(), x.data_ptr(), w.data_ptr(),
                         x.size(0), x.size(1), x.stride(0), out.stride(0), residual.stride(0),
                         static_cast<float>(eps), dtype_code(x), cur_stream()),
           "fused_add_rms_norm");
}

void silu_and_mul(at::Tensor out, const at::Tensor& x) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 2 == 0 && x.stride(1) == 1, "silu_and_mul: x");
  TORCH_CHECK(out.size(1) * 2 == x.size(1) && out.size(0) == x.size(0), "silu_and_mul: out");
  const at::DeviceGuard g(x.device());
  check_rc(atta_silu_and_mul(out.data_ptr(), x.data_ptr(), x.size(0), out.size(1), x.stride(0),
                             out.stride(0), dtype_code(x), cur_stream()),
           "silu_and_mul");
}

// prev (int64) is read only while *feed_prev != 0, i.e. for async-decode look-ahead steps
// (decode batches, rows <= the sampler output buffer); prefill steps leave the flag 0.
void stream_read(const at::Tensor& x, at::Tensor sink) {
  TORCH_CHECK(x.is_cuda() && sink.is_cuda() && x.is_contiguous() && sink.scalar_type() == at::kInt,
              "stream_read: CUDA tensors, int32 sink");
  const int64_t bytes = x.numel() * x.element_size();
  TORCH_CHECK(bytes % 16 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "stream_read: 16-byte aligned, whole 16-byte words");
  const at::DeviceGuard g(x.device());
  check_rc(atta_stream_read(x.data_ptr(), bytes, reinterpret_cast<unsigned*>(sink.data_ptr()),
                            static_cast<int>(sink.numel()), cur_stream()),
           "stream_read");
}

void embed(at::Tensor out, const at::Tensor& table, const at::Tensor& ids,
           const c10::optional<at::Tensor>& prev, const c10::optional<at::Tensor>& feed_prev) {
  check_dev(table, "table");
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous(), "embed: table [V, H] contiguous");
  TORCH_CHECK(out.dim() == 2 && out.size(1) == table.size(1) && out.stride(1) == 1,
              "embed: out [T, H]");
  TORCH_CHECK(ids.scalar_type() == at::kInt && ids.is_contiguous() && ids.numel() >= out.size(0),
              "embed: ids int32 [T]");
  TORCH_CHECK(out.scalar_type() == table.scalar_type(), "embed: dtype");
  check_dev(ids, "ids");
  check_dev(out, "out");
  TORCH_CHECK(ids.device() == table.device() && out.device() == table.device(),
              "embed: tensors on different devices");
  // the kernel moves rows with 16-byte loads/stores
  TORCH_CHECK(reinterpret_cast<uintptr_t>(table.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 &&
                  (table.size(1) * table.element_size()) % 16 == 0 &&
                  (out.stride(0) * out.element_size()) % 16 == 0,
              "embed: table/out rows must be 16-byte aligned");
  const int64_t* pv = nullptr;
  const int* fp = nullptr;
  if (feed_prev.has_value()) {
    TORCH_CHECK(prev.has_value() && prev->scalar_type() == at::kLong && prev->is_contiguous(),
                "embed: prev int64");
    check_dev(*prev, "prev");
    check_dev(*feed_prev, "feed_prev");
    TORCH_CHECK(prev->numel() >= out.size(0), "embed: prev shorter than the output rows");
    TORCH_CHECK(feed_prev->scalar_type() == at::kInt && feed_prev->numel() >= 1, "embed: flag");
    pv = prev->data_ptr<int64_t>();
    fp = feed_prev->data_ptr<int>();
  }
  dtype_code(table);
  const at::DeviceGuard g(table.device());
  check_rc(atta_embed(out.data_ptr(), table.data_ptr(), ids.data_ptr<int>(), pv, fp, out.size(0),
                      table.size(1), table.size(0), out.stride(0), cur_stream()),
           "embed");
}

void rope_cache(at::Tensor q_out, at::Tensor k_cache, at::Tensor v_cache, const at::Tensor& qkv,
                const at::Tensor& positions, const at::Tensor& slot_mapping,
                const at::Tensor& cos_sin, int64_t n_q_heads, int64_t n_kv_heads,
                int64_t head_dim) {
  check_dev(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "rope_cache: qkv 2-D");
  TORCH_CHECK(qkv.size(1) >= (n_q_heads + 2 * n_kv_heads) * head_dim, "rope_cache: qkv width");
  TORCH_CHECK(positions.scalar_type() == at::kInt && slot_mapping.scalar_type() == at::kInt,
              "rope_cache: positions/slot_mapping int32");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == head_dim,
              "rope_cache: cos_sin [max_pos, head_dim] fp32");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == n_kv_heads && k_cache.size(3) == head_dim,
              "rope_cache: k_cache [nb, Hkv, BS, D]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(2) == head_dim, "rope_cache: v_cache [nb,Hkv,D,BS]");
  const int64_t q_out_stride = q_out.dim() == 3 ? q_out.stride(0) : q_out.stride(0);
  const at::DeviceGuard g(qkv.device());
  check_rc(atta_rope_cache(q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                           qkv.data_ptr(), positions.data_ptr<int>(),
                           slot_mapping.data_ptr<int>(), cos_sin.data_ptr<float>(),
                           qkv.size(0), n_q_heads, n_kv_heads, head_dim, k_cache.size(2),
                           qkv.stride(0), q_out_stride, dtype_code(qkv), cur_stream()),
           "rope_cache");
}

void attention_prefill(at::Tensor out, const at::Tensor& q, const at::Tensor& k_cache,
                       const at::Tensor& v_cache, const at::Tensor& block_tables,
                       const at::Tensor& seq_kvlen, const at::Tensor& seq_qstart,
                       const at::Tensor& tile_seq, const at::Tensor& tile_qoff, int64_t n_q_heads,
                       int64_t n_kv_heads, double scale) {
  check_dev(q, "q");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && seq_kvlen.scalar_type() == at::kInt &&
                  seq_qstart.scalar_type() == at::kInt && tile_seq.scalar_type() == at::kInt &&
                  tile_qoff.scalar_type() == at::kInt,
              "attention_prefill: metadata must be int32");
  TORCH_CHECK(q.stride(-1) == 1 && out.stride(-1) == 1, "attention_prefill: last dim contiguous");
  const at::DeviceGuard g(q.device());
  check_rc(atta_attention_prefill(
               out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
               block_tables.data_ptr<int>(), seq_kvlen.data_ptr<int>(), seq_qstart.data_ptr<int>(),
               tile_seq.data_ptr<int>(), tile_qoff.data_ptr<int>(), tile_seq.size(0), n_q_heads,
               n_kv_heads, k_cache.size(3), k_cache.size(2), block_tables.stride(0), q.stride(0),
               out.stride(0), static_cast<float>(scale), dtype_code(q), cur_stream()),
           "attention_prefill");
}

// LDS-staged flash prefill (flash_prefill.hip); tiles must hold 128 / G query tokens.
void flash_prefill(at::Tensor out, const at::Tensor& q, const at::Tensor& k_cache,
                   const at::Tensor& v_cache, const at::Tensor& block_tables,
                   const at::Tensor& seq_kvlen, const at::Tensor& seq_qstart,
                   const at::Tensor& tile_seq, const at::Tensor& tile_qoff, int64_t n_q_heads,
                   int64_t n_kv_heads, double scale, int64_t nsplit,
                   const c10::optional<at::Tensor>& part,
                   const c10::optional<at::Tensor>& counters) {
  check_dev(q, "q");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && seq_kvlen.scalar_type() == at::kInt &&
                  seq_qstart.scalar_type() == at::kInt && tile_seq.scalar_type() == at::kInt &&
                  tile_qoff.scalar_type() == at::kInt,
              "flash_prefill: metadata must be int32");
  float* part_p = nullptr;
  int* counters_p = nullptr;
  if (nsplit > 1) {
    TORCH_CHECK(part.has_value() && counters.has_value() &&
                    part->scalar_type() == at::kFloat && counters->scalar_type() == at::kInt &&
                    part->is_cuda() && counters->is_cuda() &&
                    part->numel() * 4 >= tile_seq.size(0) * n_kv_heads * nsplit * 66560 &&
                    counters->numel() >= tile_seq.size(0) * n_kv_heads,
                "flash_prefill: split-KV needs fp32 partials [tiles * Hkv * nsplit * 16640] and "
                "zeroed int32 counters [tiles * Hkv]");
    part_p = part->data_ptr<float>();
    counters_p = counters->data_ptr<int>();
  }
  TORCH_CHECK(q.stride(-1) == 1 && out.stride(-1) == 1, "flash_prefill: last dim contiguous");
  TORCH_CHECK(q.scalar_type() == out.scalar_type() && k_cache.scalar_type() == q.scalar_type() &&
                  v_cache.scalar_type() == q.scalar_type(),
              "flash_prefill: dtypes");
  TORCH_CHECK(k_cache.dim() == 4 && v_cache.dim() == 4 && k_cache.size(1) == n_kv_heads &&
                  k_cache.size(3) == 128 && v_cache.size(2) == 128 &&
                  v_cache.size(3) == k_cache.size(2),
              "flash_prefill: caches [nb, Hkv, BS, 128] / [nb, Hkv, 128, BS]");
  TORCH_CHECK(tile_qoff.numel() >= tile_seq.numel(), "flash_prefill: tile arrays");
  const at::DeviceGuard g(q.device());
  check_rc(atta_flash_prefill(
               out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
               block_tables.data_ptr<int>(), seq_kvlen.data_ptr<int>(), seq_qstart.data_ptr<int>(),
               tile_seq.data_ptr<int>(), tile_qoff.data_ptr<int>(), tile_seq.size(0), n_q_heads,
               n_kv_heads, k_cache.size(3), k_cache.size(2), block_tables.stride(0), q.stride(0),
               out.stride(0), static_cast<float>(scale), static_cast<int>(nsplit), part_p,
               counters_p, dtype_code(q), cur_stream()),
           "flash_prefill");
}

void attention_decode(at::Tensor out, at::Tensor part_out, at::Tensor part_lse,
                      const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                      const at::Tensor& block_tables, const at::Tensor& seq_kvlen,
                      const at::Tensor& seq_qstart, int64_t num_seqs, int64_t num_parts,
                      int64_t part_tokens, int64_t n_q_heads, int64_t n_kv_heads, double scale) {
  check_dev(q, "q");
  if (num_seqs < 0) num_seqs = seq_kvlen.size(0);
  TORCH_CHECK(num_seqs <= seq_kvlen.size(0), "attention_decode: num_seqs");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && seq_kvlen.scalar_type() == at::kInt &&
                  seq_qstart.scalar_type() == at::kInt,
              "attention_decode: metadata must be int32");
  if (num_parts > 1) {
    TORCH_CHECK(part_out.numel() >= num_seqs * n_kv_heads * num_parts * 16 * 128 &&
                    part_lse.numel() >= num_seqs * n_kv_heads * num_parts * 16,
                "attention_decode: partition workspace too small");
  }
  const at::DeviceGuard g(q.device());
  check_rc(atta_attention_decode(
               out.data_ptr(), part_out.data_ptr<float>(), part_lse.data_ptr<float>(),
               q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr<int>(),
               seq_kvlen.data_ptr<int>(), seq_qstart.data_ptr<int>(), num_seqs, num_parts,
               part_tokens, n_q_heads, n_kv_heads, k_cache.size(3), k_cache.size(2),
               block_tables.stride(0), q.stride(0), out.stride(0), static_cast<float>(scale),
               dtype_code(q), cur_stream()),
           "attention_decode");
}

void sample(at::Tensor out, const at::Tensor& logits, const at::Tensor& temperature,
            const at::Tensor& seeds, const at::Tensor& steps) {
  check_dev(logits, "logits");
  TORCH_CHECK(out.scalar_type() == at::kLong && seeds.scalar_type() == at::kLong &&
                  steps.scalar_type() == at::kLong && temperature.scalar_type() == at::kFloat,
              "sample: dtypes");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "sample: logits 2-D");
  const bool is_f32 = logits.scalar_type() == at::kFloat;
  TORCH_CHECK(is_f32 || logits.scalar_type() == at::kBFloat16, "sample: logits fp32/bf16");
  const at::DeviceGuard g(logits.device());
  check_rc(atta_sample(out.data_ptr<int64_t>(), logits.data_ptr(), logits.size(0),
                       logits.size(1), logits.stride(0), is_f32 ? 1 : 0,
                       temperature.data_ptr<float>(), seeds.data_ptr<int64_t>(),
                       steps.data_ptr<int64_t>(), cur_stream()),
           "sample");
}

void sample_topkp(at::Tensor out, const at::Tensor& logits, const at::Tensor& temperature,
                  const at::Tensor& top_p, const at::Tensor& top_k, const at::Tensor& seeds,
                  const at::Tensor& steps) {
  check_dev(logits, "logits");
  TORCH_CHECK(out.scalar_type() == at::kLong && seeds.scalar_type() == at::kLong &&
                  steps.scalar_type() == at::kLong && temperature.scalar_type() == at::kFloat &&
                  top_p.scalar_type() == at::kFloat && top_k.scalar_type() == at::kInt,
              "sample_topkp: dtypes");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "sample_topkp: logits 2-D");
  const int64_t rows = logits.size(0);
  TORCH_CHECK(out.numel() >= rows && temperature.numel() >= rows && top_p.numel() >= rows &&
                  top_k.numel() >= rows && seeds.numel() >= rows && steps.numel() >= rows,
              "sample_topkp: per-row arrays");
  const bool is_f32 = logits.scalar_type() == at::kFloat;
  TORCH_CHECK(is_f32 || logits.scalar_type() == at::kBFloat16, "sample_topkp: logits fp32/bf16");
  const at::DeviceGuard g(logits.device());
  check_rc(atta_sample_topkp(out.data_ptr<int64_t>(), logits.data_ptr(), rows, logits.size(1),
                             logits.stride(0), is_f32 ? 1 : 0, temperature.data_ptr<float>(),
                             top_p.data_ptr<float>(), top_k.data_ptr<int>(),
                             seeds.data_ptr<int64_t>(), steps.data_ptr<int64_t>(), cur_stream()),
           "sample_topkp");
}

// fp8 weight-only quantisation: w is uint8 (OCP e4m3fn bytes, pre-shuffled in 16 x 64 blocks)
// and w_scale the fp32 per-row dequant scale; returns the scale pointer (nullptr: 16-bit w).
const float* fp8_scale(const at::Tensor& w, const c10::optional<at::Tensor>& w_scale,
                       const char* what) {
  if (!w_scale.has_value() || !w_scale->defined()) {
    TORCH_CHECK(w.scalar_type() != at::kByte, what, ": uint8 (fp8) weights need w_scale");
    return nullptr;
  }
  TORCH_CHECK(w.scalar_type() == at::kByte, what, ": w_scale given but weights are not fp8 bytes");
  TORCH_CHECK(w_scale->scalar_type() == at::kFloat && w_scale->is_contiguous() &&
                  w_scale->numel() == w.size(0) && w_scale->is_cuda(),
              what, ": w_scale must be fp32 [N] on the GPU");
  TORCH_CHECK(w.size(1) % 64 == 0, what, ": fp8 weights need K % 64 == 0");
  return w_scale->data_ptr<float>();
}

// dtype code for the skinny GEMV entry points; bit 8 flags pre-shuffled weights (kPreshuffled)
int skinny_dtype(const at::Tensor& x, bool preshuffled) {
  return dtype_code(x) | (preshuffled ? kPreshuffled : 0);
}

void skinny_gemm(at::Tensor y, const at::Tensor& x, const at::Tensor& w,
                 const c10::optional<at::Tensor>& residual, int64_t waves, bool preshuffled,
                 const c10::optional<at::Tensor>& w_scale, int64_t ksplit) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2, "skinny_gemm: 2-D operands");
  TORCH_CHECK(x.stride(1) == 1 && y.stride(1) == 1 && w.is_contiguous(), "skinny_gemm: layout");
  TORCH_CHECK(x.size(1) == w.size(1) && y.size(0) == x.size(0) && y.size(1) == w.size(0),
              "skinny_gemm: shapes");
  TORCH_CHECK((x.scalar_type() == w.scalar_type() || w.scalar_type() == at::kByte) &&
                  y.scalar_type() == x.scalar_type(),
              "skinny_gemm: dtypes");
  const float* ws = fp8_scale(w, w_scale, "skinny_gemm");
  const void* r = nullptr;
  int64_t rs = 0;
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->sizes() == y.sizes() && residual->stride(1) == 1, "skinny_gemm: residual");
    r = residual->data_ptr();
    rs = residual->stride(0);
  }
  const at::DeviceGuard g(x.device());
  check_rc(atta_skinny_gemm(y.data_ptr(), x.data_ptr(), w.data_ptr(), r, x.size(0), w.size(0),
                            w.size(1), x.stride(0), y.stride(0), rs, waves, ksplit, ws,
                            skinny_dtype(x, preshuffled), cur_stream()),
           "skinny_gemm");
}

// c = a . w^T (mode 0), c = res + a . w^T (mode 1, res may alias c), c = silu(a . gate^T) *
// (a . up^T) with w = [gate; up] (mode 2): the hand-written CDNA4 prefill GEMM.  bf16 a / w, or
// uint8 (e4m3fn) a / w with fp32 row scales xs [M, 1] / ws [rows of w].
void prefill_gemm(at::Tensor c, const at::Tensor& a, const at::Tensor& w,
                  const c10::optional<at::Tensor>& residual, int64_t mode,
                  const c10::optional<at::Tensor>& xs, const c10::optional<at::Tensor>& ws,
                  int64_t schedule, int64_t bm) {
  check_dev(a, "a");
  TORCH_CHECK(a.dim() == 2 && w.dim() == 2 && c.dim() == 2, "prefill_gemm: 2-D operands");
  TORCH_CHECK(schedule >= -1 && schedule <= 3 && (bm == 0 || bm == 64 || bm == 128 || bm == 256),
              "prefill_gemm: schedule -1..3, bm 0 / 64 / 128 / 256");
  const bool fp8 = a.scalar_type() == at::kByte;
  TORCH_CHECK(c.scalar_type() == at::kBFloat16 && w.scalar_type() == a.scalar_type() &&
                  (fp8 || a.scalar_type() == at::kBFloat16),
              "prefill_gemm: bf16 or fp8 (uint8) operands, bf16 output");
  TORCH_CHECK(a.stride(1) == 1 && w.stride(1) == 1 && c.stride(1) == 1, "prefill_gemm: layout");
  const int64_t n = mode == 2 ? w.size(0) / 2 : w.size(0);
  TORCH_CHECK(a.size(1) == w.size(1) && c.size(0) == a.size(0) && c.size(1) == n &&
                  (mode != 2 || w.size(0) % 2 == 0),
              "prefill_gemm: shapes");
  const float* xsp = nullptr;
  const float* wsp = nullptr;
  if (fp8) {
    TORCH_CHECK(xs.has_value() && ws.has_value() && xs->scalar_type() == at::kFloat &&
                    ws->scalar_type() == at::kFloat && xs->is_contiguous() &&
                    ws->is_contiguous() && xs->numel() == a.size(0) && ws->numel() == w.size(0),
                "prefill_gemm: fp8 needs fp32 row scales xs [M] and ws [rows of w]");
    xsp = xs->data_ptr<float>();
    wsp = ws->data_ptr<float>();
  }
  const void* r = nullptr;
  int64_t rs = 0;
  if (mode == 1) {
    TORCH_CHECK(residual.has_value() && residual->defined() && residual->sizes() == c.sizes() &&
                    residual->stride(1) == 1 && residual->scalar_type() == at::kBFloat16,
                "prefill_gemm: residual");
    r = residual->data_ptr();
    rs = residual->stride(0);
  }
  const at::DeviceGuard g(a.device());
  check_rc(atta_prefill_gemm(c.data_ptr(), a.data_ptr(), w.data_ptr(), r, a.size(0), n, a.size(1),
                             a.stride(0), w.stride(0), c.stride(0), rs, mode, fp8 ? 1 : 0, xsp,
                             wsp, static_cast<int>(schedule), static_cast<int>(bm), cur_stream()),
           "prefill_gemm");
}

int64_t prefill_gemm_error() { return atta_prefill_gemm_error(); }
void prefill_gemm_error_to(at::Tensor host, bool clear) {
  TORCH_CHECK(host.device().is_cpu() && host.is_pinned() && host.scalar_type() == at::kInt &&
                  host.numel() >= 1,
              "prefill_gemm_error_to: a pinned int32 host tensor");
  check_rc(atta_prefill_gemm_error_async(host.data_ptr(), cur_stream(), clear ? 1 : 0),
           "prefill_gemm_error_to");
}
void set_wide_plan(int64_t waves, int64_t ksplit) {
  atta_set_wide_plan(static_cast<int>(waves), static_cast<int>(ksplit));
}
void set_flash_waves(int64_t nw) { atta_set_flash_waves(static_cast<int>(nw)); }
std::vector<int64_t> get_wide_min_rows() {
  int m = 0, ms = 0;
  atta_get_wide_min_rows(&m, &ms);
  return {m, ms};
}
void set_splitk_half(int64_t on) { atta_set_splitk_half(static_cast<int>(on)); }
void set_flash_split_blocks(int64_t nb) { atta_set_flash_split_blocks(static_cast<int>(nb)); }
void set_midm_plan(int64_t bmt, int64_t ksplit) {
  atta_set_midm_plan(static_cast<int>(bmt), static_cast<int>(ksplit));
}
std::vector<int64_t> midm_plan(int64_t M, int64_t ntiles, int64_t K, int64_t epi,
                               int64_t ws_floats) {
  int bmt = 0, ks = 0;
  atta_midm_plan(static_cast<int>(M), static_cast<int>(ntiles), static_cast<int>(K),
                 static_cast<int>(epi), ws_floats, &bmt, &ks);
  return {bmt, ks};
}
void set_wide_min_rows(int64_t m, int64_t m_silu) {
  atta_set_wide_min_rows(static_cast<int>(m), static_cast<int>(m_silu));
}
void prefill_gemm_error_reset() {
  check_rc(atta_prefill_gemm_error_reset(), "prefill_gemm_error_reset");
}
int64_t prefill_gemm_auto_bm(int64_t m) { return atta_prefill_gemm_auto_bm(static_cast<int>(m)); }
void prefill_gemm_config(int64_t schedule, int64_t group_m, int64_t ablate) {
  check_rc(atta_prefill_gemm_config(static_cast<int>(schedule), static_cast<int>(group_m),
                                    static_cast<int>(ablate)),
           "prefill_gemm_config");
}

void check_skinny(const at::Tensor& x, const at::Tensor& w, const char* what) {
  TORCH_CHECK(w.size(0) % 16 == 0 && w.size(1) % 32 == 0, what, ": weight tile shape");
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.is_contiguous(), what,
              ": layout");
  TORCH_CHECK(x.size(1) == w.size(1) &&
                  (x.scalar_type() == w.scalar_type() || w.scalar_type() == at::kByte),
              what, ": shapes / dtypes");
}

void fused_qkv_rope(at::Tensor q_out, at::Tensor k_cache, at::Tensor v_cache, const at::Tensor& x,
                    const at::Tensor& w, const at::Tensor& positions, const at::Tensor& slots,
                    const at::Tensor& cos_sin, int64_t n_q_heads, int64_t n_kv_heads, double eps,
                    int64_t waves, bool preshuffled, const c10::optional<at::Tensor>& w_scale,
                    int64_t ksplit) {
  check_skinny(x, w, "fused_qkv_rope");
  const float* ws = fp8_scale(w, w_scale, "fused_qkv_rope");
  TORCH_CHECK(w.size(0) == (n_q_heads + 2 * n_kv_heads) * 128, "fused_qkv_rope: w rows");
  TORCH_CHECK(positions.scalar_type() == at::kInt && slots.scalar_type() == at::kInt,
              "fused_qkv_rope: int32 positions/slots");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == 128, "fused_qkv_rope: cos_sin");
  TORCH_CHECK(q_out.stride(-1) == 1, "fused_qkv_rope: q_out layout");
  TORCH_CHECK(k_cache.size(1) == n_kv_heads && k_cache.size(3) == 128, "fused_qkv_rope: k_cache");
  const at::DeviceGuard g(x.device());
  check_rc(atta_fused_qkv_rope(q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                               x.data_ptr(), w.data_ptr(), positions.data_ptr<int>(),
                               slots.data_ptr<int>(), cos_sin.data_ptr<float>(), x.size(0),
                               x.size(1), x.stride(0), q_out.stride(0), n_q_heads, n_kv_heads,
                               k_cache.size(2), static_cast<float>(eps), waves, ksplit, ws,
                               skinny_dtype(x, preshuffled), cur_stream()),
           "fused_qkv_rope");
}

void fused_gate_up_silu(at::Tensor out, const at::Tensor& x, const at::Tensor& w, double eps,
                        int64_t waves, bool preshuffled,
                        const c10::optional<at::Tensor>& w_scale, int64_t ksplit) {
  check_skinny(x, w, "fused_gate_up_silu");
  const float* ws = fp8_scale(w, w_scale, "fused_gate_up_silu");
  TORCH_CHECK(w.size(0) == 2 * out.size(1) && out.size(0) == x.size(0) && out.stride(1) == 1,
              "fused_gate_up_silu: out");
  const at::DeviceGuard g(x.device());
  check_rc(atta_fused_gate_up_silu(out.data_ptr(), x.data_ptr(), w.data_ptr(), x.size(0),
                                   x.size(1), out.size(1), x.stride(0), out.stride(0),
                                   static_cast<float>(eps), waves, ksplit, ws,
                                   skinny_dtype(x, preshuffled), cur_stream()),
           "fused_gate_up_silu");
}

void fused_lm_head_sample(at::Tensor tokens, at::Tensor keys, const at::Tensor& x,
                          const at::Tensor& w, double eps, const at::Tensor& temperature,
                          const at::Tensor& seeds, const at::Tensor& steps, int64_t finalize,
                          int64_t vocab_offset, int64_t waves, bool preshuffled,
                          const c10::optional<at::Tensor>& w_scale) {
  TORCH_CHECK(finalize >= 0 && finalize <= 2, "fused_lm_head_sample: finalize mode 0/1/2");
  check_skinny(x, w, "fused_lm_head_sample");
  const float* ws = fp8_scale(w, w_scale, "fused_lm_head_sample");
  TORCH_CHECK(tokens.scalar_type() == at::kLong && keys.scalar_type() == at::kLong &&
                  seeds.scalar_type() == at::kLong && steps.scalar_type() == at::kLong &&
                  temperature.scalar_type() == at::kFloat,
              "fused_lm_head_sample: dtypes");
  TORCH_CHECK(keys.numel() >= x.size(0) * (w.size(0) / 16) && tokens.numel() >= x.size(0),
              "fused_lm_head_sample: keys needs M * (vocab / 16) entries");
  const at::DeviceGuard g(x.device());
  check_rc(atta_fused_lm_head_sample(
               tokens.data_ptr<int64_t>(),
               reinterpret_cast<unsigned long long*>(keys.data_ptr<int64_t>()), x.data_ptr(),
               w.data_ptr(), x.size(0), w.size(0), x.size(1), x.stride(0), static_cast<float>(eps),
               temperature.data_ptr<float>(), seeds.data_ptr<int64_t>(), steps.data_ptr<int64_t>(),
               static_cast<int>(finalize), static_cast<int>(vocab_offset), waves, ws,
               skinny_dtype(x, preshuffled), cur_stream()),
           "fused_lm_head_sample");
}

// Row-wise fp8 activation quantisation fused into norm / SiLU-mul / plain rows.
void quant_rows_fp8(at::Tensor q, at::Tensor scale, const at::Tensor& x,
                    const c10::optional<at::Tensor>& w, int64_t mode, double eps,
                    const c10::optional<at::Tensor>& residual) {
  check_dev(x, "x");
  check_dev(q, "q");
  TORCH_CHECK(mode >= 0 && mode <= 3,
              "quant_rows_fp8: mode 0 (norm) / 1 (silu) / 2 (plain) / 3 (add + norm)");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && q.dim() == 2 && q.stride(1) == 1 &&
                  q.scalar_type() == at::kByte,
              "quant_rows_fp8: 2-D rows, uint8 q");
  const int64_t width = q.size(1);
  TORCH_CHECK(q.size(0) == x.size(0) && x.size(1) == (mode == 1 ? 2 * width : width),
              "quant_rows_fp8: shapes");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.is_contiguous() &&
                  scale.numel() >= x.size(0) && scale.is_cuda(),
              "quant_rows_fp8: fp32 scale [rows]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(q.data_ptr()) % 8 == 0,
              "quant_rows_fp8: 16-byte aligned x rows, 8-byte aligned q rows");
  void* rp = nullptr;
  int64_t rs = 0;
  if (mode == 3) {
    TORCH_CHECK(residual.has_value() && residual->sizes() == x.sizes() &&
                    residual->stride(1) == 1 && residual->scalar_type() == x.scalar_type() &&
                    residual->is_cuda() &&
                    reinterpret_cast<uintptr_t>(residual->data_ptr()) % 16 == 0,
                "quant_rows_fp8: mode 3 needs a residual shaped like x");
    rp = residual->data_ptr();
    rs = residual->stride(0);
  }
  const void* wp = nullptr;
  if (mode == 0 || mode == 3) {
    TORCH_CHECK(w.has_value() && w->numel() == width && w->scalar_type() == x.scalar_type() &&
                    w->is_cuda() && w->is_contiguous(),
                "quant_rows_fp8: norm weight [width]");
    wp = w->data_ptr();
  }
  const at::DeviceGuard g(x.device());
  check_rc(atta_quant_rows_fp8(q.data_ptr(), scale.data_ptr<float>(), x.data_ptr(), wp,
                               x.size(0), width, x.stride(0), q.stride(0), mode,
                               static_cast<float>(eps), rp, rs, dtype_code(x), cur_stream()),
           "quant_rows_fp8");
}

// Registers the split-K workspace of the skinny GEMVs on ws's device.  The tensors must
// outlive every launch (and captured graph) that uses a split > 1; counters start zeroed.
void set_splitk_workspace(const at::Tensor& ws, const at::Tensor& counters) {
  check_dev(ws, "ws");
  check_dev(counters, "counters");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() &&
                  counters.scalar_type() == at::kInt && counters.is_contiguous() &&
                  ws.device() == counters.device(),
              "set_splitk_workspace: fp32 ws + int32 counters on one device");
  TORCH_CHECK(ws.numel() < (int64_t(1) << 29), "set_splitk_workspace: ws must stay under 2 GiB");
  check_rc(atta_set_splitk_ws(ws.device().index(), ws.data_ptr<float>(), counters.data_ptr<int>(),
                              ws.numel(), static_cast<int>(counters.numel())),
           "set_splitk_workspace");
}

void sample_finalize(at::Tensor tokens, const at::Tensor& keys, int64_t n_tiles) {
  check_dev(keys, "keys");
  TORCH_CHECK(n_tiles > 0 && keys.numel() >= tokens.numel() * n_tiles, "sample_finalize: sizes");
  const at::DeviceGuard g(keys.device());
  check_rc(atta_sample_finalize(tokens.data_ptr<int64_t>(),
                                reinterpret_cast<const unsigned long long*>(keys.data_ptr<int64_t>()),
                                tokens.numel(), n_tiles, cur_stream()),
           "sample_finalize");
}

void attention_decode_v2(at::Tensor out, at::Tensor part_out, at::Tensor part_lse,
                         at::Tensor counters, const at::Tensor& q, const at::Tensor& k_cache,
                         const at::Tensor& v_cache, const at::Tensor& block_tables,
                         const at::Tensor& seq_kvlen, const at::Tensor& seq_qstart,
                         int64_t num_seqs, int64_t max_parts, int64_t part_tokens,
                         int64_t n_q_heads, int64_t n_kv_heads, double scale) {
  check_dev(q, "q");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && seq_kvlen.scalar_type() == at::kInt &&
                  seq_qstart.scalar_type() == at::kInt && counters.scalar_type() == at::kInt,
              "attention_decode_v2: int32 metadata");
  if (num_seqs < 0) num_seqs = seq_kvlen.size(0);
  TORCH_CHECK(num_seqs <= seq_kvlen.size(0), "attention_decode_v2: num_seqs");
  TORCH_CHECK(part_out.numel() >= num_seqs * n_kv_heads * max_parts * 16 * 128 &&
                  part_lse.numel() >= num_seqs * n_kv_heads * max_parts * 16 &&
                  counters.numel() >= num_seqs * n_kv_heads,
              "attention_decode_v2: workspace too small");
  const at::DeviceGuard g(q.device());
  check_rc(atta_attention_decode_v2(
               out.data_ptr(), part_out.data_ptr<float>(), part_lse.data_ptr<float>(),
               counters.data_ptr<int>(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
               block_tables.data_ptr<int>(), seq_kvlen.data_ptr<int>(), seq_qstart.data_ptr<int>(),
               num_seqs, max_parts, part_tokens, n_q_heads, n_kv_heads, k_cache.size(3),
               k_cache.size(2), block_tables.stride(0), q.stride(0), out.stride(0),
               static_cast<float>(scale), dtype_code(q), cur_stream()),
           "attention_decode_v2");
}

void set_gemv_trace(const c10::optional<at::Tensor>& trace) {
  if (trace.has_value() && trace->defined()) {
    TORCH_CHECK(trace->is_cuda() && trace->scalar_type() == at::kLong,
                "set_gemv_trace: int64 cuda tensor");
    atta_set_gemv_trace(trace->data_ptr());
  } else {
    atta_set_gemv_trace(nullptr);
  }
}

void set_attention_trace(const c10::optional<at::Tensor>& trace) {
  if (trace.has_value()) {
    TORCH_CHECK(trace->scalar_type() == at::kLong && trace->is_contiguous() && trace->is_cuda(),
                "set_attention_trace: int64 cuda tensor");
    atta_set_attention_trace(trace->data_ptr());
  } else {
    atta_set_attention_trace(nullptr);
  }
}

void skinny_variant(at::Tensor y, const at::Tensor& x, const at::Tensor& w, int64_t variant) {
  check_skinny(x, w, "skinny_variant");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.scalar_type() == at::kBFloat16,
              "skinny_variant: contiguous bf16");
  const at::DeviceGuard g(x.device());
  check_rc(atta_skinny_variant(y.data_ptr(), x.data_ptr(), w.data_ptr(), x.size(0), w.size(0),
                               w.size(1), static_cast<int>(variant), cur_stream()),
           "skinny_variant");
}

// ---- one-shot IPC all-reduce -------------------------------------------------------------
// Buffers are raw device allocations (uncached, IPC-exportable) addressed by int64 pointers;
// the Python side (parallel/custom_allreduce.py) owns their lifetime.
int64_t ar_buffer_bytes(int64_t max_elems, int64_t elem_bytes) {
  return static_cast<int64_t>(atta_ar_buffer_bytes(max_elems, static_cast<int>(elem_bytes)));
}

int64_t ar_alloc(int64_t bytes, int64_t device) {
  hipSetDevice(static_cast<int>(device));
  void* p = nullptr;
  check_rc(atta_ar_alloc(&p, static_cast<size_t>(bytes)), "ar_alloc");
  return reinterpret_cast<int64_t>(p);
}

void ar_free(int64_t ptr) { check_rc(atta_ar_free(reinterpret_cast<void*>(ptr)), "ar_free"); }

at::Tensor ar_handle(int64_t ptr) {
  at::Tensor h = at::zeros({atta_ar_handle_bytes()}, at::TensorOptions().dtype(at::kByte));
  check_rc(atta_ar_ipc_handle(reinterpret_cast<void*>(ptr), h.data_ptr()), "ar_handle");
  return h;
}

int64_t ar_open(const at::Tensor& handle) {
  TORCH_CHECK(!handle.is_cuda() && handle.scalar_type() == at::kByte &&
                  handle.numel() == atta_ar_handle_bytes(), "ar_open: CPU uint8 IPC handle");
  void* p = nullptr;
  check_rc(atta_ar_ipc_open(handle.contiguous().data_ptr(), &p), "ar_open");
  return reinterpret_cast<int64_t>(p);
}

int64_t ar_error(int64_t ptr) {
  uint32_t word = 0;
  check_rc(static_cast<int>(hipMemcpy(&word, reinterpret_cast<uint8_t*>(ptr) + atta_ar_error_offset(),
                                      sizeof(word), hipMemcpyDeviceToHost)),
           "ar_error");
  return word;
}

void ar_close(int64_t ptr) {
  check_rc(atta_ar_ipc_close(reinterpret_cast<void*>(ptr)), "ar_close");
}

const void* res_ptr(const c10::optional<at::Tensor>& res, const at::Tensor& x, const char* what) {
  if (!res.has_value()) return nullptr;
  TORCH_CHECK(res->is_contiguous() && res->numel() == x.numel() &&
                  res->scalar_type() == x.scalar_type() && res->device() == x.device(),
              what, ": residual layout");
  return res->data_ptr();
}

void ar_run(const at::Tensor& x, at::Tensor y, at::IntArrayRef bases, int64_t rank,
            int64_t max_elems, const c10::optional<at::Tensor>& residual) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel() &&
                  x.scalar_type() == y.scalar_type(), "ar_run: layout");
  TORCH_CHECK(bases.size() >= 2 && bases.size() <= 8, "ar_run: 2..8 ranks");
  void* b[8] = {};
  for (size_t i = 0; i < bases.size(); ++i) b[i] = reinterpret_cast<void*>(bases[i]);
  const at::DeviceGuard g(x.device());
  check_rc(atta_ar_run(b, static_cast<int>(rank), static_cast<int>(bases.size()), max_elems,
                       x.data_ptr(), y.data_ptr(), res_ptr(residual, x, "ar_run"), x.numel(),
                       dtype_code(x), cur_stream()),
           "ar_run");
}

// Row-parallel TP GEMV with the all-reduce push fused (X1 / X2): x @ w^T of this rank's K
// shard goes straight into every rank's IPC receive slot; ar_push_reduce finishes the sum.
void skinny_gemm_push(const at::Tensor& x, const at::Tensor& w, int64_t n_out, int64_t waves,
                      bool preshuffled, const c10::optional<at::Tensor>& w_scale, int64_t ksplit,
                      at::IntArrayRef bases, int64_t rank, int64_t max_elems) {
  check_dev(x, "x");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.is_contiguous(),
              "skinny_gemm_push: layout");
  TORCH_CHECK(x.size(1) == w.size(1) && w.size(0) == n_out &&
                  (x.scalar_type() == w.scalar_type() || w.scalar_type() == at::kByte),
              "skinny_gemm_push: shapes / dtypes");
  TORCH_CHECK(bases.size() >= 2 && bases.size() <= 8, "skinny_gemm_push: 2..8 ranks");
  const float* ws = fp8_scale(w, w_scale, "skinny_gemm_push");
  void* b[8] = {};
  for (size_t i = 0; i < bases.size(); ++i) b[i] = reinterpret_cast<void*>(bases[i]);
  const at::DeviceGuard g(x.device());
  check_rc(atta_skinny_gemm_push(x.data_ptr(), w.data_ptr(), x.size(0), w.size(0), w.size(1),
                                 x.stride(0), waves, ksplit, ws, skinny_dtype(x, preshuffled),
                                 b, static_cast<int>(rank), static_cast<int>(bases.size()),
                                 max_elems, cur_stream()),
           "skinny_gemm_push");
}

// Receive side: y (+)= sum over ranks of the pushed [rows, n] products (rank order, fp32);
// with residual: y = residual + sum (y may alias residual).  ntiles = tiles each source pushed.
void ar_push_reduce(at::Tensor y, const c10::optional<at::Tensor>& residual,
                    at::IntArrayRef bases, int64_t rank, int64_t max_elems, int64_t ntiles) {
  check_dev(y, "y");
  TORCH_CHECK(y.is_contiguous(), "ar_push_reduce: layout");
  TORCH_CHECK(bases.size() >= 2 && bases.size() <= 8, "ar_push_reduce: 2..8 ranks");
  void* b[8] = {};
  for (size_t i = 0; i < bases.size(); ++i) b[i] = reinterpret_cast<void*>(bases[i]);
  const at::DeviceGuard g(y.device());
  check_rc(atta_ar_push_reduce(b, static_cast<int>(rank), static_cast<int>(bases.size()),
                               max_elems, y.data_ptr(), res_ptr(residual, y, "ar_push_reduce"),
                               y.numel(), static_cast<int>(ntiles), dtype_code(y), cur_stream()),
           "ar_push_reduce");
}

void ar_keymax(at::Tensor keys, const c10::optional<at::Tensor>& tokens, at::IntArrayRef bases,
               int64_t rank) {
  check_dev(keys, "keys");
  TORCH_CHECK(keys.is_contiguous() && keys.scalar_type() == at::kLong && keys.numel() > 0 &&
                  keys.numel() <= 256, "ar_keymax: <= 256 contiguous int64 keys");
  TORCH_CHECK(bases.size() >= 2 && bases.size() <= 8, "ar_keymax: 2..8 ranks");
  int64_t* tok = nullptr;
  if (tokens.has_value()) {
    TORCH_CHECK(tokens->is_contiguous() && tokens->scalar_type() == at::kLong &&
                    tokens->numel() >= keys.numel() && tokens->device() == keys.device(),
                "ar_keymax: tokens");
    tok = tokens->data_ptr<int64_t>();
  }
  void* b[8] = {};
  for (size_t i = 0; i < bases.size(); ++i) b[i] = reinterpret_cast<void*>(bases[i]);
  const at::DeviceGuard g(keys.device());
  check_rc(atta_ar_keymax(b, static_cast<int>(rank), static_cast<int>(bases.size()),
                          reinterpret_cast<long long*>(keys.data_ptr<int64_t>()), tok,
                          static_cast<int>(keys.numel()), cur_stream()),
           "ar_keymax");
}

int64_t ar2_buffer_bytes(int64_t max_elems, int64_t world, int64_t elem_bytes) {
  return static_cast<int64_t>(
      atta_ar2_buffer_bytes(max_elems, static_cast<int>(world), static_cast<int>(elem_bytes)));
}

int64_t ar2_error(int64_t ptr) {
  uint32_t word = 0;
  check_rc(static_cast<int>(hipMemcpy(&word, reinterpret_cast<uint8_t*>(ptr) + atta_ar2_error_offset(),
                                      sizeof(word), hipMemcpyDeviceToHost)),
           "ar2_error");
  return word;
}

void ar2_run(const at::Tensor& x, at::Tensor y, at::IntArrayRef bases, int64_t rank,
             int64_t max_elems, const c10::optional<at::Tensor>& residual) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel() &&
                  x.scalar_type() == y.scalar_type(), "ar2_run: layout");
  TORCH_CHECK(bases.size() >= 2 && bases.size() <= 8, "ar2_run: 2..8 ranks");
  void* b[8] = {};
  for (size_t i = 0; i < bases.size(); ++i) b[i] = reinterpret_cast<void*>(bases[i]);
  const at::DeviceGuard g(x.device());
  check_rc(atta_ar2_run(b, static_cast<int>(rank), static_cast<int>(bases.size()), max_elems,
                        x.data_ptr(), y.data_ptr(), res_ptr(residual, x, "ar2_run"), x.numel(),
                        dtype_code(x), cur_stream()),
           "ar2_run");
}

// ---- persistent decode step ----------------------------------------------------------------
// Node list of a captured hipGraph (torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()):
// "kernel:<name> grid=x,y,z block=x" / "memcpy" / "memset" / "host" / ... in graph order -
// evidence of what a captured decode step contains (scripts/gpu/graph_nodes.py).
std::vector<std::string> graph_nodes(int64_t graph) {
  auto g = reinterpret_cast<hipGraph_t>(graph);
  size_t n = 0;
  check_rc(static_cast<int>(hipGraphGetNodes(g, nullptr, &n)), "hipGraphGetNodes");
  std::vector<hipGraphNode_t> nodes(n);
  check_rc(static_cast<int>(hipGraphGetNodes(g, nodes.data(), &n)), "hipGraphGetNodes");
  std::vector<std::string> out;
  for (auto node : nodes) {
    hipGraphNodeType t;
    check_rc(static_cast<int>(hipGraphNodeGetType(node, &t)), "hipGraphNodeGetType");
    switch (t) {
      case hipGraphNodeTypeKernel: {
        hipKernelNodeParams kp{};
        std::string name = "?";
        if (hipGraphKernelNodeGetParams(node, &kp) == hipSuccess && kp.func != nullptr) {
          const char* nm = hipKernelNameRefByPtr(kp.func, nullptr);
          if (nm == nullptr) nm = hipKernelNameRef(reinterpret_cast<hipFunction_t>(kp.func));
          if (nm != nullptr) name = nm;
        }
        out.push_back("kernel:" + name + " grid=" + std::to_string(kp.gridDim.x) + "," +
                      std::to_string(kp.gridDim.y) + "," + std::to_string(kp.gridDim.z) +
                      " block=" + std::to_string(kp.blockDim.x));
        break;
      }
      case hipGraphNodeTypeMemcpy: out.push_back("memcpy"); break;
      case hipGraphNodeTypeMemset: out.push_back("memset"); break;
      case hipGraphNodeTypeHost: out.push_back("host"); break;
      case hipGraphNodeTypeEmpty: out.push_back("empty"); break;
      case hipGraphNodeTypeWaitEvent: out.push_back("wait_event"); break;
      case hipGraphNodeTypeEventRecord: out.push_back("event_record"); break;
      default: out.push_back("other:" + std::to_string(static_cast<int>(t))); break;
    }
  }
  return out;
}

}  // namespace

TORCH_LIBRARY(atta, m) {
  m.def("graph_nodes(int graph) -> str[]", &graph_nodes);
  m.def("ar_buffer_bytes(int max_elems, int elem_bytes) -> int", &ar_buffer_bytes);
  m.def("skinny_gemm_push(Tensor x, Tensor w, int n_out, int waves, bool preshuffled, "
        "Tensor? w_scale, int ksplit, int[] bases, int rank, int max_elems) -> ()");
  m.def("ar_push_reduce(Tensor(a!) y, Tensor? residual, int[] bases, int rank, int max_elems, "
        "int ntiles) -> ()");
  m.def("ar_alloc(int bytes, int device) -> int", &ar_alloc);
  m.def("set_attention_trace(Tensor? trace) -> ()", &set_attention_trace);
  m.def("set_gemv_trace(Tensor? trace) -> ()", &set_gemv_trace);
  m.def("ar_free(int ptr) -> ()", &ar_free);
  m.def("ar_handle(int ptr) -> Tensor", &ar_handle);
  m.def("ar_open(Tensor handle) -> int", &ar_open);
  m.def("ar_close(int ptr) -> ()", &ar_close);
  m.def("ar_error(int ptr) -> int", &ar_error);
  m.def("ar_run(Tensor x, Tensor(a!) y, int[] bases, int rank, int max_elems, "
        "Tensor? residual=None) -> ()");
  m.def("ar_keymax(Tensor(a!) keys, Tensor(b!)? tokens, int[] bases, int rank) -> ()");
  m.def("ar2_buffer_bytes(int max_elems, int world, int elem_bytes) -> int", &ar2_buffer_bytes);
  m.def("ar2_error(int ptr) -> int", &ar2_error);
  m.def("ar2_run(Tensor x, Tensor(a!) y, int[] bases, int rank, int max_elems, "
        "Tensor? residual=None) -> ()");
  m.def("skinny_variant(Tensor(a!) y, Tensor x, Tensor w, int variant) -> ()");
  m.def(
      "attention_decode_v2(Tensor(a!) out, Tensor(b!) part_out, Tensor(c!) part_lse, "
      "Tensor(d!) counters, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
      "Tensor seq_kvlen, Tensor seq_qstart, int num_seqs, int max_parts, int part_tokens, "
      "int n_q_heads, int n_kv_heads, float scale) -> ()");
  m.def(
      "fused_qkv_rope(Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor x, "
      "Tensor w, Tensor positions, Tensor slots, Tensor cos_sin, int n_q_heads, int n_kv_heads, "
      "float eps, int waves, bool preshuffled=False, Tensor? w_scale=None, int ksplit=1) -> ()");
  m.def("fused_gate_up_silu(Tensor(a!) out, Tensor x, Tensor w, float eps, int waves, "
        "bool preshuffled=False, Tensor? w_scale=None, int ksplit=1) -> ()");
  m.def("set_splitk_workspace(Tensor ws, Tensor counters) -> ()");
  m.def("quant_rows_fp8(Tensor(a!) q, Tensor(b!) scale, Tensor x, Tensor? w, int mode, "
        "float eps, Tensor(c!)? residual=None) -> ()");
  m.def(
      "fused_lm_head_sample(Tensor(a!) tokens, Tensor(b!) keys, Tensor x, Tensor w, float eps, "
      "Tensor temperature, Tensor seeds, Tensor steps, int finalize, int vocab_offset, "
      "int waves, bool preshuffled=False, Tensor? w_scale=None) -> ()");
  m.def("sample_finalize(Tensor(a!) tokens, Tensor keys, int n_tiles) -> ()");
  m.def("skinny_gemm(Tensor(a!) y, Tensor x, Tensor w, Tensor? residual, int waves, "
        "bool preshuffled=False, Tensor? w_scale=None, int ksplit=1) -> ()");
  m.def("prefill_gemm(Tensor(a!) c, Tensor a, Tensor w, Tensor? residual, int mode, Tensor? xs=None, Tensor? ws=None, int schedule=-1, int bm=0) -> ()");
  m.def("prefill_gemm_auto_bm(int m) -> int", &prefill_gemm_auto_bm);
  m.def("prefill_gemm_error() -> int", &prefill_gemm_error);
  m.def("prefill_gemm_error_to(Tensor(a!) host, bool clear) -> ()", &prefill_gemm_error_to);
  m.def("prefill_gemm_error_reset() -> ()", &prefill_gemm_error_reset);
  m.def("set_wide_plan(int waves, int ksplit) -> ()", &set_wide_plan);
  m.def("set_wide_min_rows(int m, int m_silu) -> ()", &set_wide_min_rows);
  m.def("get_wide_min_rows() -> int[]", &get_wide_min_rows);
  m.def("set_midm_plan(int bmt, int ksplit) -> ()", &set_midm_plan);
  m.def("set_splitk_half(int on) -> ()", &set_splitk_half);
  m.def("set_flash_split_blocks(int nb) -> ()", &set_flash_split_blocks);
  m.def("midm_plan(int M, int ntiles, int K, int epi, int ws_floats) -> int[]", &midm_plan);
  m.def("set_flash_waves(int nw) -> ()", &set_flash_waves);
  m.def("prefill_gemm_config(int schedule, int group_m, int ablate=0) -> ()", &prefill_gemm_config);
  m.def("rms_norm(Tensor(a!) out, Tensor x, Tensor w, float eps) -> ()");
  m.def("fused_add_rms_norm(Tensor(a!) out, Tensor(b!) residual, Tensor x, Tensor w, float eps) -> ()");
  m.def("silu_and_mul(Tensor(a!) out, Tensor x) -> ()");
  m.def("embed(Tensor(a!) out, Tensor table, Tensor ids, Tensor? prev, Tensor? feed_prev) -> ()");
  m.def("stream_read(Tensor x, Tensor(a!) sink) -> ()");
  m.def(
      "rope_cache(Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor qkv, "
      "Tensor positions, Tensor slot_mapping, Tensor cos_sin, int n_q_heads, int n_kv_heads, "
      "int head_dim) -> ()");
  m.def(
      "attention_prefill(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, "
      "Tensor block_tables, Tensor seq_kvlen, Tensor seq_qstart, Tensor tile_seq, "
      "Tensor tile_qoff, int n_q_heads, int n_kv_heads, float scale) -> ()");
  m.def(
      "flash_prefill(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, "
      "Tensor block_tables, Tensor seq_kvlen, Tensor seq_qstart, Tensor tile_seq, "
      "Tensor tile_qoff, int n_q_heads, int n_kv_heads, float scale, int nsplit=1, "
      "Tensor(b!)? part=None, Tensor(c!)? counters=None) -> ()");
  m.def(
      "attention_decode(Tensor(a!) out, Tensor(b!) part_out, Tensor(c!) part_lse, Tensor q, "
      "Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor seq_kvlen, "
      "Tensor seq_qstart, int num_seqs, int num_parts, int part_tokens, int n_q_heads, int n_kv_heads, "
      "float scale) -> ()");
  m.def("sample(Tensor(a!) out, Tensor logits, Tensor temperature, Tensor seeds, Tensor steps) -> ()");
  m.def("sample_topkp(Tensor(a!) out, Tensor logits, Tensor temperature, Tensor top_p, "
        "Tensor top_k, Tensor seeds, Tensor steps) -> ()");
}

TORCH_LIBRARY_IMPL(atta, CUDA, m) {
  m.impl("ar_run", &ar_run);
  m.impl("skinny_gemm_push", &skinny_gemm_push);
  m.impl("ar_push_reduce", &ar_push_reduce);
  m.impl("ar2_run", &ar2_run);
  m.impl("ar_keymax", &ar_keymax);
  m.impl("rms_norm", &rms_norm);
  m.impl("fused_add_rms_norm", &fused_add_rms_norm);
  m.impl("silu_and_mul", &silu_and_mul);
  m.impl("embed", &embed);
  m.impl("stream_read", &stream_read);
  m.impl("rope_cache", &rope_cache);
  m.impl("attention_prefill", &attention_prefill);
  m.impl("flash_prefill", &flash_prefill);
  m.impl("attention_decode", &attention_decode);
  m.impl("sample", &sample);
  m.impl("sample_topkp", &sample_topkp);
  m.impl("skinny_gemm", &skinny_gemm);
  m.impl("prefill_gemm", &prefill_gemm);
  m.impl("fused_qkv_rope", &fused_qkv_rope);
  m.impl("fused_gate_up_silu", &fused_gate_up_silu);
  m.impl("fused_lm_head_sample", &fused_lm_head_sample);
  m.impl("sample_finalize", &sample_finalize);
  m.impl("set_splitk_workspace", &set_splitk_workspace);
  m.impl("quant_rows_fp8", &quant_rows_fp8);
  m.impl("attention_decode_v2", &attention_decode_v2);
  m.impl("skinny_variant", &skinny_variant);
}
