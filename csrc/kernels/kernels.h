// Host-side launcher declarations for every HIP kernel in csrc/kernels.
// Launchers return 0 on success, a hipError_t (>0) on a launch failure, or a
// negative code for an unsupported shape. They never allocate or synchronise,
// so callers may capture them into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace oamd {
typedef uint16_t bf16_t;

// ---- explanation-model ops ----
int rmsnorm(const bf16_t* x, bf16_t* residual, const bf16_t* w, bf16_t* y, int rows, int hidden,
            int64_t x_stride, int64_t r_stride, int64_t y_stride, float eps, const float* xp, int S,
            hipStream_t stream);
int silu_mul(const bf16_t* gu, bf16_t* out, int64_t rows, int inter, int block, int64_t in_stride,
             int64_t out_stride, hipStream_t stream);
// Decode-step bookkeeping (norm_act.hip): cache slots + sampler positions of the step's tokens,
// then the state advance after sampling (B <= 1024 rows, one workgroup each).
int decode_slots(const int* bt, const int64_t* pos, const int* ctx, int64_t* slots, int64_t* spos, int B,
                 int max_pages, int page_size, hipStream_t stream);
int decode_advance(const int64_t* tok, int64_t* ids, int64_t* hist, int64_t* pos, int* ctx, int64_t* step, int B,
                   int ms, hipStream_t stream);
int embedding(const int64_t* ids, const bf16_t* table, bf16_t* out, int tokens, int hidden,
              int64_t vocab, hipStream_t stream);
int rope_kv(const bf16_t* qkv, int64_t qkv_stride, const int64_t* pos, const float* cos_t,
            const float* sin_t, int tokens, int Hq, int Hkv, int head_dim, bf16_t* q_out,
            bf16_t* k_out, bf16_t* v_out, void* k_cache, void* v_cache, const int64_t* slots,
            int page_size, int64_t max_pos, const float* xp, int S, const bf16_t* bias,
            bool fp8_cache, float k_scale, float v_scale, hipStream_t stream);  // cache: bf16 or e4m3fn
// Y[M,N] = X[M,K] W[N,K]^T for decode buckets (M a multiple of the BM-row tile, BM in {64,128,256}); S-way split-K
// (S | 8) with fp32 slabs P[S][M][N] reduced into Y; BN in {64, 128} columns per tile.
int gemm_decode(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, int BN,
                int BM, bool silu_gu, bool w_tiled, int stages, hipStream_t stream);

// Compute-bound 256x256-tile GEMM (prefill projections, lm_head; gemm_tile.hip): Y[M, N] = X[M,K] W[N,K]^T
// (+ bias[N]) for any M >= 1, N % 16 == 0, K % 64 == 0; silu_gu: fused SwiGLU over the 64-row interleaved
// gate|up weight (N % 128 == 0), Y [M, N/2]. ldy = Y's row stride in elements.
// S > 1: S-way split-K into fp32 slabs P[S][M][N], then reduced into Y (SwiGLU applied when silu_gu);
// Y == nullptr leaves the slabs to the consumer (rmsnorm / rope_kv sum them).
int gemm_tile(const bf16_t* X, const bf16_t* W, bf16_t* Y, const bf16_t* bias, int M, int N, int K, int ldy,
              bool silu_gu, int variant, int S, float* P, hipStream_t stream);
// Decode-bucket GEMM on the ping-pong schedule (gemm_pp.hip): Y[M,N] = X[M,K] W[N,K]^T, bm-row tiles
// (128 / 256), 128-column tiles (N % 128 == 0), S-way split-K slabs P (S > 1; reduced into Y unless Y is
// nullptr); silu_gu: fused SwiGLU (S == 1), Y [M, N/2]; nt: non-temporal weight loads.
// ws / flags (both given): the stream-K form for bm 256, S 1, nt (gemm_pp.hip SK): ws >= (N / 128) x 32768
// floats, flags >= N / 128 ints, zero (left zero). gemm_pp_sk_grid: its block count, 0 = plain launch.
int gemm_pp(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, int bm, bool silu_gu,
            bool nt, hipStream_t stream, bool one_seg = false, float* ws = nullptr, int* flags = nullptr);
int gemm_pp_sk_grid(int tiles, int steps);
// 256-row decode GEMM with register-streamed activations (gemm_xr.hip): Xt = X [256, K] in the tiled
// layout [16][K/32][64][8]; N % 128 == 0, K % (64 S) == 0; epi 0 = fp32 slabs P[S][256][N], 1 = bf16 Y,
// 2 = SwiGLU (interleaved gate|up, S == 1) Y [256, N/2], 3 = the same written tiled.
int gemm_xr(const bf16_t* Xt, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, int epi,
            hipStream_t stream);
// x [rows, K] row-major -> the tiled layout gemm_xr reads (rows % 16 == 0, K % 32 == 0).
int tile_rows(const bf16_t* x, bf16_t* xt, int rows, int K, hipStream_t stream);
// Y[M, N] = bf16(sum_s P[s][M][N]) (fp32 split-K slabs).
int splitk_reduce(const float* P, bf16_t* Y, int64_t MN, int S, hipStream_t stream);
// Skinny-M decode GEMM (M <= 32, gemm_skinny.hip): N % 16 == 0, K % (128 S) == 0; S-way split-K slabs P
// reduced into Y (Y == nullptr: left for the consumer); silu_gu: fused SwiGLU over the 64-row
// interleaved gate|up weight, Y [M, N/2].
int gemm_skinny(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, bool silu_gu,
                hipStream_t stream);

// FP8 e4m3fn W8A8: Y = (X8 . W8^T) * sx[m] * sw[n]; any M (BM-row tiles), S | 8 split-K.
int gemm_fp8(const uint8_t* X, const uint8_t* W, const float* sx, const float* sw, bf16_t* Y, float* P, int M,
             int N, int K, int S, int BN, int BM, hipStream_t stream);
// Per-row dynamic quantization to e4m3fn: sx[m] = max|x[m]| / 448.
int quantize_fp8_rows(const bf16_t* x, uint8_t* q, float* sx, int M, int K, int64_t ld, hipStream_t stream);
// Fused SwiGLU + per-row e4m3fn quantization of the 64-feature-interleaved gate|up rows [M, 2 inter]
// (inter % 64 == 0, <= 16384): q [M, inter], sx [M].
// gu == nullptr: the gate|up rows are the S fp32 split-K slabs P [S, M, 2 inter] (summed, bf16-rounded).
int silu_quantize_fp8(const bf16_t* gu, const float* P, int S, uint8_t* q, float* sx, int M, int inter, int64_t ld,
                      hipStream_t stream);

// Pattern-event scoring + per-doc ranking / summary (N5), see score.hip.
int score_events(const int64_t* keys, const int* hit_doc, const int* doc_ptr, int n_hits, int n_docs,
                 const int* prim_ptr, const int* prim_pat, const int* ev_ptr, const int* ev_doc_ptr,
                 const int* sec_ptr, const int* sec_matcher, const double* sec_w, const int* sec_win,
                 const double* conf, const int* severity, int num_matchers, double significance, double* ev_score,
                 int* ev_pat, int* ev_line, int* order, int* summary, hipStream_t stream);

// The decode step's RoPE + KV-cache write folded into decode attention (rope_kv's decode
// work): q is rotated from the QKV projection inside every workgroup, and the workgroup
// holding a sequence's last token writes that token's rotated K and its V into the cache.
// Row b of the projection is bf16(sum of S fp32 split-K slabs [S][rows][ncol] (+ bias)) or
// a bf16 row (+ bias), ncol = (Hq + 2 Hkv) * 128 -- the numerics of rope_kv.
struct DecRope {
  const float* xp;          // split-K slabs, or nullptr
  const bf16_t* row;        // bf16 rows [rows][row_stride] when xp == nullptr
  int64_t row_stride;
  int S;                    // slab count (xp)
  int64_t slab;             // elements per slab = rows * ncol
  const bf16_t* bias;       // [(Hq + 2 Hkv) * 128] or nullptr
  const int64_t* pos;       // [rows] positions of the decode tokens
  const float* cos_t;       // [max_pos][64]
  const float* sin_t;
  int64_t max_pos;
  const int64_t* slots;     // [rows] cache slot of the decode token (< 0: none)
  float k_inv, v_inv;       // fp8 cache: 1 / k_scale, 1 / v_scale
};

// k_cache / v_cache: bf16, or (fp8) OCP e4m3fn bytes holding x / k_scale, x / v_scale
// rope != nullptr: q is unused; see DecRope
int attn_decode(const bf16_t* q, const void* k_cache, const void* v_cache, bool fp8, float k_scale, float v_scale,
                const int* block_tables, const int* seq_lens, bf16_t* out, float* o_part, float* ml_part, int B,
                int Hq, int Hkv, int head_dim, int page_size, int max_pages, int num_splits, float scale, int variant,
                hipStream_t stream, uint8_t* q8 = nullptr, float* sx = nullptr, const DecRope* rope = nullptr);
// (q8, sx non-null: the output rows are also emitted as per-token e4m3fn [B, Hq*128] + fp32 scales,
// == quantize_fp8_rows(out); `out` then holds valid bf16 only for rows of a single split.)
// Causal prefill attention; the work list holds one item per attn_prefill_block_q(Hq, Hkv, variant)
// query rows of a sequence. variant 1 = per-query-head kernel (64 rows), 2 = GQA-grouped 16-row
// waves, 3 = GQA-grouped swapped-operand 32x32 MFMA waves (2 and 3 need Hq / Hkv in {1, 2, 4, 8}).
int attn_prefill_block_q(int Hq, int Hkv, int variant);
int attn_prefill(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, const int* cu_seqlens,
                 const int* work_seq, const int* work_q0, int num_work, int Hq, int Hkv, int head_dim,
                 float scale, int variant, hipStream_t stream,
                 const bf16_t* pk = nullptr, const bf16_t* pv = nullptr, const int* seq_pfx = nullptr);
int sample_tokens(const void* logits, bool logits_bf16, int64_t stride, int rows, int vocab,
                  const float* temperature, const int64_t* seeds, const int64_t* positions,
                  int64_t* out_tokens, int64_t col_offset, float* out_val, hipStream_t stream);

// One-shot all-reduce over peer-mapped fine-grained buffers (allreduce.hip).
size_t car_buffer_bytes(size_t cap_bytes, int world);
int car_alloc(size_t cap_bytes, int world, void** base, void* handle_out /* 64 B hipIpcMemHandle_t */);
int car_open(const void* handle, void** ptr);
int car_close(void* ptr);
int car_free(void* base);
int car_host_flag(uint32_t** host, uint32_t** dev);   // host-mapped error word (read without a device sync)
void car_free_host_flag(uint32_t* host);
int car_error(const uint32_t* host);
int car_reset(void* base, size_t bytes, uint32_t* host);
// Fused one-shot all-reduce + residual add + RMSNorm (bf16 rows of `hidden`, hidden % 8 == 0, <= 16384):
// residual += bf16(sum over ranks of in); y = rmsnorm(residual) * w. Exactly one of `in` (bf16 rows) and
// `slabs` (S fp32 split-K slabs [S, rows, hidden], summed then bf16-rounded) is non-null; q8/sx non-null
// also emit per-row e4m3fn of y (== quantize_fp8_rows(y)).
// all-reduce protocols (allreduce.hip): one-shot / two-shot (reduce-scatter + all-gather)
// with sc0 sc1 hand-offs, and the original system-fence one-shot (A/B)
constexpr int kCarOneShot = 0, kCarTwoShot = 1, kCarOneShotFence = 2, kCarLL = 3;
int car_all_reduce_rmsnorm(const void* in, const float* slabs, int S, bf16_t* residual, const bf16_t* w, bf16_t* y,
                           uint8_t* q8, float* sx, int rows, int hidden, float eps, int rank, int world,
                           void* const* bases, size_t cap_bytes, int blocks, uint32_t* herr_dev, double timeout_s,
                           int proto, hipStream_t stream);
int car_all_reduce(const void* in, void* out, int64_t bytes, bool bf16, int rank, int world, void* const* bases,
                   size_t cap_bytes, int blocks, uint32_t* herr_dev, double timeout_s, int proto,
                   hipStream_t stream);

}  // namespace oamd
