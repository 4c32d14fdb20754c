// Host-side launcher declarations for the CDNA4 kernel library.  Every launcher takes raw
// device pointers plus the HIP stream to launch on (graph-capture safe: no allocation, no
// synchronisation) and returns 0 on success, -1 for an unsupported shape, or a hipError_t.
// dtype: 0 = bf16, 1 = fp16.
#pragma once

// OR-ed into the dtype code of the skinny GEMV entry points: weights are pre-shuffled
// into the MFMA lane order (ops.preshuffle).
constexpr int kPreshuffled = 256;
#include <hip/hip_runtime.h>
#include <stdint.h>

int atta_rms_norm(void* out, void* residual, const void* x, const void* w, int rows, int hidden,
                  int64_t x_stride, int64_t out_stride, int64_t res_stride, float eps, int dtype,
                  hipStream_t stream);

int atta_silu_and_mul(void* out, const void* x, int rows, int inter, int64_t x_stride,
                      int64_t out_stride, int dtype, hipStream_t stream);
int atta_stream_read(const void* x, int64_t bytes, unsigned* sink, int blocks,
                     hipStream_t stream);
int atta_embed(void* out, const void* table, const int* ids, const int64_t* prev,
               const int* feed_prev, int rows, int hidden, int64_t vocab, int64_t out_stride,
               hipStream_t stream);

int atta_rope_cache(void* q_out, void* k_cache, void* v_cache, const void* qkv,
                    const int* positions, const int* slot_mapping, const float* cos_sin,
                    int num_tokens, int n_q_heads, int n_kv_heads, int head_dim, int block_size,
                    int64_t qkv_stride, int64_t q_out_stride, int dtype, hipStream_t stream);

int atta_attention_prefill(void* out, const void* q, const void* k_cache, const void* v_cache,
                           const int* block_tables, const int* seq_kvlen, const int* seq_qstart,
                           const int* tile_seq, const int* tile_qoff, int num_tiles,
                           int n_q_heads, int n_kv_heads, int head_dim, int block_size,
                           int bt_stride, int64_t q_stride, int64_t out_stride, float scale,
                           int dtype, hipStream_t stream);

// LDS-staged flash attention for prefill (flash_prefill.hip): tiles of 128 / G query tokens.
int atta_flash_prefill(void* out, const void* q, const void* k_cache, const void* v_cache,
                       const int* block_tables, const int* seq_kvlen, const int* seq_qstart,
                       const int* tile_seq, const int* tile_qoff, int num_tiles, int n_q_heads,
                       int n_kv_heads, int head_dim, int block_size, int bt_stride,
                       int64_t q_stride, int64_t out_stride, float scale, int nsplit,
                       float* part, int* counters, int dtype, hipStream_t stream);

int atta_attention_decode(void* out, float* part_out, float* part_lse, const void* q,
                          const void* k_cache, const void* v_cache, const int* block_tables,
                          const int* seq_kvlen, const int* seq_qstart, int num_seqs,
                          int num_parts, int part_tokens, int n_q_heads, int n_kv_heads,
                          int head_dim, int block_size, int bt_stride, int64_t q_stride,
                          int64_t out_stride, float scale, int dtype, hipStream_t stream);

int atta_sample(int64_t* out, const void* logits, int rows, int vocab, int64_t stride,
                int logits_is_fp32, const float* temperature, const int64_t* seeds,
                const int64_t* steps, hipStream_t stream);

// top-k / top-p sampling (exact radix-select thresholds, same Gumbel draw as atta_sample)
int atta_sample_topkp(int64_t* out, const void* logits, int rows, int vocab, int64_t stride,
                      int logits_is_fp32, const float* temperature, const float* top_p,
                      const int* top_k, const int64_t* seeds, const int64_t* steps,
                      hipStream_t stream);

int atta_skinny_gemm_push(const void* x, const void* w, int M, int N, int K, int64_t x_stride,
                          int waves, int ksplit, const float* wscale, int dtype,
                          void* const* bases, int rank, int world, int64_t max_elems,
                          hipStream_t stream);
int atta_ar_push_reduce(void* const* bases, int rank, int world, int64_t max_elems, void* y,
                        const void* res, int64_t n, int ntiles, int dtype, hipStream_t stream);
int64_t atta_ar_push_layout(int what);
int atta_skinny_gemm(void* y, const void* x, const void* w, const void* residual, int M, int N,
                     int K, int64_t x_stride, int64_t y_stride, int64_t res_stride, int waves,
                     int ksplit, const float* wscale, int dtype, hipStream_t stream);

int atta_fused_qkv_rope(void* q_out, void* k_cache, void* v_cache, const void* x, const void* w,
                        const int* positions, const int* slots, const float* cos_sin, int M,
                        int K, int64_t x_stride, int64_t q_stride, int n_q_heads, int n_kv_heads,
                        int block_size, float eps, int waves, int ksplit, const float* wscale,
                        int dtype, hipStream_t stream);

int atta_fused_gate_up_silu(void* out, const void* x, const void* w, int M, int K, int inter,
                            int64_t x_stride, int64_t out_stride, float eps, int waves,
                            int ksplit, const float* wscale, int dtype, hipStream_t stream);

// Split-K workspace of `device` for the skinny GEMVs (fp32 slots + per-tile counters, zeroed).
int atta_set_splitk_ws(int device, float* ws, int* counters, int64_t ws_floats, int n_counters);

int atta_fused_lm_head_sample(int64_t* tokens, unsigned long long* keys, const void* x,
                              const void* w, int M, int N, int K, int64_t x_stride, float eps,
                              const float* temperature, const int64_t* seeds,
                              const int64_t* steps, int finalize, int vocab_offset,
                              int waves, const float* wscale, int dtype, hipStream_t stream);

int atta_sample_finalize(int64_t* tokens, const unsigned long long* keys, int M, int n_tiles,
                         hipStream_t stream);

// per-workgroup timeline of later decode attention launches (int64 [4 x grid]; nullptr off)
void atta_set_attention_trace(void* trace);
void atta_set_gemv_trace(void* trace);

int atta_attention_decode_v2(void* out, float* part_out, float* part_lse, int* counters,
                             const void* q, const void* k_cache, const void* v_cache,
                             const int* block_tables, const int* seq_kvlen, const int* seq_qstart,
                             int num_seqs, int max_parts, int part_tokens, int n_q_heads,
                             int n_kv_heads, int head_dim, int block_size, int bt_stride,
                             int64_t q_stride, int64_t out_stride, float scale, int dtype,
                             hipStream_t stream);

int atta_skinny_variant(void* y, const void* x, const void* w, int M, int N, int K,
                        int variant, hipStream_t stream);

// Row-wise e4m3fn activation quantisation (quant_fp8.hip): mode 0 = rmsnorm(x) * w,
// 1 = silu(gate) * up (x rows hold gate | up, width = I), 2 = x, 3 = residual += x then
// rmsnorm(residual) * w.  q [rows, width] uint8, scale [rows] fp32 (value = fp8 * scale).
int atta_quant_rows_fp8(void* q, float* scale, const void* x, const void* w, int rows, int width,
                        int64_t x_stride, int64_t q_stride, int mode, float eps, void* residual,
                        int64_t res_stride, int dtype, hipStream_t stream);

// ---- one-shot IPC all-reduce (allreduce.hip) ---------------------------------------------
size_t atta_ar_buffer_bytes(int64_t max_elems, int elem_bytes);
int atta_ar_alloc(void** ptr, size_t bytes);
int atta_ar_free(void* ptr);
int atta_ar_handle_bytes();
int64_t atta_ar_error_offset();
int atta_ar_ipc_handle(void* ptr, void* handle_out);
int atta_ar_ipc_open(const void* handle, void** ptr);
int atta_ar_ipc_close(void* ptr);
// res != nullptr: y = res + sum (residual-stream update fused; y may alias res)
int atta_ar_run(void* const* bases, int rank, int world, int64_t max_elems, const void* x,
                void* y, const void* res, int64_t n, int dtype, hipStream_t stream);
// X4: in-place int64 MAX of n <= 256 sampler keys (+ decoded token ids when tokens != null)
int atta_ar_keymax(void* const* bases, int rank, int world, long long* keys, int64_t* tokens,
                   int n, hipStream_t stream);

// ---- two-shot IPC all-reduce (allreduce.hip): reduce-scatter + all-gather ----------------
size_t atta_ar2_buffer_bytes(int64_t max_elems, int world, int elem_bytes);
int64_t atta_ar2_error_offset();
int atta_ar2_run(void* const* bases, int rank, int world, int64_t max_elems, const void* x,
                 void* y, const void* res, int64_t n, int dtype, hipStream_t stream);


// Prefill GEMM (prefill_gemm.hip): c[M, N] = a[M, K] . w[N, K]^T; mode 0 plain, 1 c = res +
// a.w^T (res may alias c), 2 c = silu(a.gate^T) * (a.up^T) with w = [gate; up].  fp8: a / w are
// e4m3fn bytes with fp32 row scales xs [M] / wsc [rows of w]; else bf16.  schedule -1 = the
// configured default (atta_prefill_gemm_config), else 0-3; bm 0 = auto, else 64 / 128 / 256.
int atta_prefill_gemm(void* c, const void* a, const void* w, const void* res, int M, int N,
                      int K, int64_t lda, int64_t ldw, int64_t ldc, int64_t ldres, int mode,
                      int fp8, const float* xs, const float* wsc, int schedule, int bm,
                      hipStream_t stream);
int atta_prefill_gemm_auto_bm(int M);
int atta_prefill_gemm_error();
int atta_prefill_gemm_error_async(void* host, hipStream_t stream, int clear);
int atta_prefill_gemm_error_reset();
void atta_set_wide_plan(int waves, int ksplit);
void atta_set_wide_min_rows(int m, int m_silu);
void atta_get_wide_min_rows(int* m, int* m_silu);
// mid-M GEMM (midm.hip): the next launch's plan (row-block height bmt x 16, K slices; 0 =
// planned) and the plan the library would pick for a shape
void atta_set_midm_plan(int bmt, int ksplit);
void atta_set_splitk_half(int on);
void atta_set_flash_split_blocks(int nb);
int atta_midm_plan(int M, int ntiles, int K, int epi, int64_t ws_floats, int* bmt, int* ksplit);
void atta_set_flash_waves(int nw);
int atta_prefill_gemm_config(int schedule, int group_m, int ablate);
