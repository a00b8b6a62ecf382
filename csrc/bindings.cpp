// Python bindings for the gfx950 kernels (operator_amd._C).
//
// Every binding validates dtype / device / contiguity / shape on the host
// BEFORE launching, so a hand-written kernel never runs with operands whose
// shapes differ from what its grid assumes. Kernels are launched on PyTorch's
// current HIP stream, so they are captured by torch.cuda.CUDAGraph (hipGraph).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels/kernels.h"
#include "kernels/scan.h"

namespace {

using oamd::bf16_t;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " has wrong dtype ", (t).scalar_type())
#define CHECK_BF16(t) CHECK_DT(t, at::kBFloat16)
#define ROWMAJOR_VEC(t) \
  TORCH_CHECK((t).dim() == 2 && (t).stride(1) == 1 && (t).stride(0) % 8 == 0, #t " must be [rows, cols] row-major with 16-B aligned rows")
#define RC(call)                                                           \
  do {                                                                     \
    int rc__ = (call);                                                     \
    TORCH_CHECK(rc__ == 0, "kernel launch failed: " #call " rc=", rc__);   \
  } while (0)

template <typename T>
T* ptr(const at::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
template <typename T>
T* optr(const c10::optional<at::Tensor>& t) { return t.has_value() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr; }

void rmsnorm(const at::Tensor& x, const c10::optional<at::Tensor>& residual, const at::Tensor& w,
             at::Tensor& y, double eps, const c10::optional<at::Tensor>& partial, int64_t splits, bool tiled_out) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(y); ROWMAJOR_VEC(x); ROWMAJOR_VEC(y);
  CHECK_CONTIG(w);
  const int64_t rows = x.size(0), hidden = x.size(1);
  const float* xp = nullptr;
  if (partial.has_value()) {  // x = bf16(sum of `splits` fp32 [rows, hidden] slabs); x only gives the shape
    CHECK_DT(*partial, at::kFloat); CHECK_CONTIG(*partial);
    TORCH_CHECK(splits >= 1 && partial->numel() >= splits * rows * hidden, "rmsnorm: partial slabs too small");
    xp = partial->data_ptr<float>();
  }
  TORCH_CHECK(hidden % 8 == 0 && hidden <= 256 * 8 * 8, "hidden must be a multiple of 8 and <= 16384");
  TORCH_CHECK(w.numel() == hidden && y.size(0) == rows && y.size(1) == hidden, "rmsnorm shape mismatch");
  int64_t rstride = 0;
  if (residual.has_value()) {
    CHECK_BF16(*residual); ROWMAJOR_VEC(*residual);
    TORCH_CHECK(residual->size(0) == rows && residual->size(1) == hidden, "residual shape mismatch");
    rstride = residual->stride(0);
  }
  // tiled_out: y (contiguous, [rows, hidden] elements) receives the gemm_xr activation layout
  TORCH_CHECK(!tiled_out || (rows % 16 == 0 && hidden % 64 == 0 && y.is_contiguous()),
              "rmsnorm: tiled output needs rows % 16 == 0, hidden % 64 == 0 and a contiguous y");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  RC(oamd::rmsnorm(ptr<bf16_t>(x), optr<bf16_t>(residual), ptr<bf16_t>(w), ptr<bf16_t>(y), (int)rows,
                   (int)hidden, x.stride(0), rstride, tiled_out ? -1 : y.stride(0), (float)eps, xp, (int)splits,
                   cur_stream()));
}

// gemm_xr (csrc/kernels/gemm_xr.hip): the 256-row decode GEMM with register-streamed activations.
// xt: the activations [256, K] in the tiled layout (rmsnorm(tiled_out=True) / tile_rows / the SwiGLU
// epilogue with epi 3); epi 0 = fp32 split-K slabs into p, 1 = bf16 y [256, N], 2 = SwiGLU y [256, N/2],
// 3 = SwiGLU y [256, N/2] written tiled.
void gemm_xr(const at::Tensor& xt, const at::Tensor& w, const c10::optional<at::Tensor>& y_opt,
             const c10::optional<at::Tensor>& p, int64_t splits, int64_t epi) {
  CHECK_DEV(xt); CHECK_BF16(xt); CHECK_BF16(w); CHECK_CONTIG(xt); CHECK_CONTIG(w);
  TORCH_CHECK(xt.dim() == 2 && w.dim() == 2 && w.size(1) == xt.size(1), "gemm_xr: xt [256,K], w [N,K]");
  const int64_t M = xt.size(0), K = xt.size(1), N = w.size(0);
  TORCH_CHECK(M == 256 && N % 128 == 0 && K % 64 == 0, "gemm_xr: M == 256, N % 128 == 0, K % 64 == 0");
  TORCH_CHECK(splits >= 1 && splits <= 16 && K % (64 * splits) == 0, "gemm_xr: K % (64 * splits) == 0");
  TORCH_CHECK((epi >= 0 && epi <= 3) || (epi >= 10 && epi <= 12), "gemm_xr: epi in 0..3 (10..12: timing ablations)");
  TORCH_CHECK(epi == 0 || epi >= 10 || splits == 1, "gemm_xr: bf16 / SwiGLU outputs need splits == 1");
  bf16_t* yp = nullptr;
  float* pp = nullptr;
  if (epi == 0 || epi >= 10) {
    TORCH_CHECK(p.has_value(), "gemm_xr: slabs need p");
    CHECK_DT(*p, at::kFloat); CHECK_CONTIG(*p);
    TORCH_CHECK(p->numel() >= splits * M * N, "gemm_xr: p too small");
    pp = p->data_ptr<float>();
  } else {
    TORCH_CHECK(y_opt.has_value() && splits == 1, "gemm_xr: y needed (one K slice)");
    CHECK_BF16(*y_opt); CHECK_CONTIG(*y_opt);
    TORCH_CHECK(y_opt->numel() == M * (epi == 1 ? N : N / 2), "gemm_xr: y size");
    yp = ptr<bf16_t>(*y_opt);
  }
  TORCH_CHECK(N * K < (1LL << 40), "gemm too large");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(xt.device());
  RC(oamd::gemm_xr(ptr<bf16_t>(xt), ptr<bf16_t>(w), yp, pp, (int)M, (int)N, (int)K, (int)splits, (int)epi,
                   cur_stream()));
}

void tile_rows(const at::Tensor& x, at::Tensor& xt) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(xt); CHECK_CONTIG(x); CHECK_CONTIG(xt);
  TORCH_CHECK(x.dim() == 2 && x.numel() == xt.numel() && x.size(0) % 16 == 0 && x.size(1) % 64 == 0,
              "tile_rows: x [rows % 16, K % 64], xt of the same size");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  RC(oamd::tile_rows(ptr<bf16_t>(x), ptr<bf16_t>(xt), (int)x.size(0), (int)x.size(1), cur_stream()));
}

void silu_mul(const at::Tensor& gu, at::Tensor& out, int64_t block) {
  CHECK_DEV(gu); CHECK_BF16(gu); CHECK_BF16(out); ROWMAJOR_VEC(gu); ROWMAJOR_VEC(out);
  const int64_t rows = gu.size(0), inter = out.size(1);
  TORCH_CHECK(gu.size(1) == 2 * inter && out.size(0) == rows && inter % 8 == 0, "silu_mul shape mismatch");
  if (block == 0) block = inter;
  TORCH_CHECK(block % 8 == 0 && inter % block == 0, "silu_mul: interleave block must divide inter, % 8");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  RC(oamd::silu_mul(ptr<bf16_t>(gu), ptr<bf16_t>(out), rows, (int)inter, (int)block, gu.stride(0), out.stride(0),
                    cur_stream()));
}

void embedding(const at::Tensor& ids, const at::Tensor& table, at::Tensor& out) {
  CHECK_DEV(ids); CHECK_DT(ids, at::kLong); CHECK_BF16(table); CHECK_BF16(out);
  CHECK_CONTIG(ids); CHECK_CONTIG(table); CHECK_CONTIG(out);
  TORCH_CHECK(table.dim() == 2 && table.size(1) % 8 == 0, "table must be [vocab, hidden%8==0]");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == ids.numel() && out.size(1) == table.size(1), "embedding out shape");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(ids.device());
  RC(oamd::embedding(ptr<int64_t>(ids), ptr<bf16_t>(table), ptr<bf16_t>(out), (int)ids.numel(),
                     (int)table.size(1), table.size(0), cur_stream()));
}

void decode_slots(const at::Tensor& bt, const at::Tensor& pos, const at::Tensor& ctx, at::Tensor& slots,
                  at::Tensor& spos, int64_t page_size) {
  CHECK_DEV(bt); CHECK_DT(bt, at::kInt); CHECK_CONTIG(bt); CHECK_DT(pos, at::kLong); CHECK_CONTIG(pos);
  CHECK_DT(ctx, at::kInt); CHECK_CONTIG(ctx); CHECK_DT(slots, at::kLong); CHECK_CONTIG(slots);
  CHECK_DT(spos, at::kLong); CHECK_CONTIG(spos);
  const int64_t B = pos.numel();
  TORCH_CHECK(bt.dim() == 2 && bt.size(0) == B && ctx.numel() == B && slots.numel() == B && spos.numel() == B &&
                  B <= 1024 && page_size > 0,
              "decode_slots: bt [B, max_pages], pos/ctx/slots/spos [B], B <= 1024");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(pos.device());
  RC(oamd::decode_slots(ptr<int>(bt), ptr<int64_t>(pos), ptr<int>(ctx), ptr<int64_t>(slots), ptr<int64_t>(spos),
                        (int)B, (int)bt.size(1), (int)page_size, cur_stream()));
}

void decode_advance(const at::Tensor& tok, at::Tensor& ids, at::Tensor& hist, at::Tensor& pos, at::Tensor& ctx,
                    at::Tensor& step) {
  CHECK_DEV(tok); CHECK_DT(tok, at::kLong); CHECK_CONTIG(tok); CHECK_DT(ids, at::kLong); CHECK_CONTIG(ids);
  CHECK_DT(hist, at::kLong); CHECK_CONTIG(hist); CHECK_DT(pos, at::kLong); CHECK_CONTIG(pos);
  CHECK_DT(ctx, at::kInt); CHECK_CONTIG(ctx); CHECK_DT(step, at::kLong);
  const int64_t B = ids.numel();
  TORCH_CHECK(tok.numel() == B && pos.numel() == B && ctx.numel() == B && hist.dim() == 2 && hist.size(0) == B &&
                  step.numel() == 1 && B <= 1024,
              "decode_advance: tok/ids/pos/ctx [B], hist [B, ms], step [1], B <= 1024");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(ids.device());
  RC(oamd::decode_advance(ptr<int64_t>(tok), ptr<int64_t>(ids), ptr<int64_t>(hist), ptr<int64_t>(pos),
                          ptr<int>(ctx), ptr<int64_t>(step), (int)B, (int)hist.size(1), cur_stream()));
}

static bool kv_is_fp8(const at::Tensor& t) {
  return t.scalar_type() == at::kFloat8_e4m3fn || t.scalar_type() == at::kByte;
}

void rope_kv(const at::Tensor& qkv, const at::Tensor& pos, const at::Tensor& cos_t, const at::Tensor& sin_t,
             int64_t Hq, int64_t Hkv, at::Tensor& q_out, const c10::optional<at::Tensor>& k_out,
             const c10::optional<at::Tensor>& v_out, const c10::optional<at::Tensor>& k_cache,
             const c10::optional<at::Tensor>& v_cache, const c10::optional<at::Tensor>& slots,
             const c10::optional<at::Tensor>& partial, int64_t splits, const c10::optional<at::Tensor>& bias,
             double k_scale, double v_scale) {
  CHECK_DT(pos, at::kLong); CHECK_CONTIG(pos); CHECK_DEV(pos);
  CHECK_DT(cos_t, at::kFloat); CHECK_DT(sin_t, at::kFloat); CHECK_CONTIG(cos_t); CHECK_CONTIG(sin_t);
  const int64_t T = pos.numel();
  const int64_t D = cos_t.size(1) * 2;
  TORCH_CHECK(D == 128, "only head_dim 128 is supported");
  const float* xp = nullptr;
  const bf16_t* qp = nullptr;
  int64_t qstride = 0;
  if (partial.has_value()) {  // qkv = bf16(sum of `splits` fp32 [T, (Hq+2Hkv)D] slabs); qkv unused
    CHECK_DT(*partial, at::kFloat); CHECK_CONTIG(*partial);
    TORCH_CHECK(splits >= 1 && partial->numel() >= splits * T * (Hq + 2 * Hkv) * D, "rope_kv: slabs too small");
    xp = partial->data_ptr<float>();
  } else {
    CHECK_DEV(qkv); CHECK_BF16(qkv); ROWMAJOR_VEC(qkv);
    TORCH_CHECK(qkv.size(0) == T && qkv.size(1) == (Hq + 2 * Hkv) * D, "qkv must be [T, (Hq+2Hkv)*D]");
    qp = ptr<bf16_t>(qkv);
    qstride = qkv.stride(0);
  }
  TORCH_CHECK(pos.numel() == T && sin_t.sizes() == cos_t.sizes(), "pos/cos/sin shape");
  CHECK_BF16(q_out); CHECK_CONTIG(q_out);
  TORCH_CHECK(q_out.numel() == T * Hq * D, "q_out shape");
  if (k_out.has_value()) { CHECK_BF16(*k_out); CHECK_CONTIG(*k_out); TORCH_CHECK(k_out->numel() == T * Hkv * D, "k_out shape"); }
  if (v_out.has_value()) { CHECK_BF16(*v_out); CHECK_CONTIG(*v_out); TORCH_CHECK(v_out->numel() == T * Hkv * D, "v_out shape"); }
  int page = 1;
  if (k_cache.has_value()) {
    TORCH_CHECK(v_cache.has_value() && slots.has_value(), "k_cache needs v_cache and slots");
    TORCH_CHECK(kv_is_fp8(*k_cache) ? kv_is_fp8(*v_cache)
                                    : (k_cache->scalar_type() == at::kBFloat16 &&
                                       v_cache->scalar_type() == at::kBFloat16),
                "KV cache must be bf16 or float8_e4m3fn (both K and V)");
    CHECK_DEV(*k_cache); CHECK_CONTIG(*k_cache); CHECK_CONTIG(*v_cache);
    CHECK_DT(*slots, at::kLong); CHECK_CONTIG(*slots);
    TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == Hkv && k_cache->size(3) == D &&
                    k_cache->sizes() == v_cache->sizes(), "cache must be [pages, Hkv, page, D]");
    TORCH_CHECK(slots->numel() == T, "slots shape");
    page = (int)k_cache->size(2);
  }
  if (bias.has_value()) {
    CHECK_BF16(*bias); CHECK_CONTIG(*bias); CHECK_DEV(*bias);
    TORCH_CHECK(bias->numel() == (Hq + 2 * Hkv) * D, "rope_kv: bias must be [(Hq + 2 Hkv) * D]");
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(pos.device());
  const bool fp8 = k_cache.has_value() && kv_is_fp8(*k_cache);
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "KV scales must be positive");
  RC(oamd::rope_kv(qp, qstride, ptr<int64_t>(pos), ptr<float>(cos_t), ptr<float>(sin_t),
                   (int)T, (int)Hq, (int)Hkv, (int)D, ptr<bf16_t>(q_out), optr<bf16_t>(k_out), optr<bf16_t>(v_out),
                   k_cache.has_value() ? k_cache->data_ptr() : nullptr,
                   v_cache.has_value() ? v_cache->data_ptr() : nullptr, optr<int64_t>(slots), page, cos_t.size(0),
                   xp, (int)splits, optr<bf16_t>(bias), fp8, (float)k_scale, (float)v_scale, cur_stream()));
}

void gemm_decode(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& y_opt,
                 const c10::optional<at::Tensor>& p,
                 int64_t splits, int64_t bn, int64_t bm, bool silu_gu, bool w_tiled, int64_t stages) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2, "x [M,K], w [N,K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  bf16_t* yp = nullptr;
  if (y_opt.has_value()) {
    const at::Tensor& y = *y_opt;
    CHECK_BF16(y); CHECK_CONTIG(y);
    TORCH_CHECK(y.dim() == 2 && y.size(0) == M && y.size(1) == (silu_gu ? N / 2 : N), "gemm shapes");
    yp = ptr<bf16_t>(y);
  } else {
    TORCH_CHECK(splits > 1 && !silu_gu, "y may be omitted only for split-K slabs summed by the consumer");
  }
  TORCH_CHECK(w.size(1) == K, "gemm shapes (a tiled w keeps its logical [N, K] shape)");
  TORCH_CHECK(!silu_gu || (bn == 128 && splits == 1), "fused SwiGLU needs bn = 128, splits = 1");
  if (bm == 0) bm = std::min<int64_t>(M, 256);
  TORCH_CHECK((bm == 64 || bm == 128 || bm == 256) && M % bm == 0, "gemm_decode: M % bm, bm in {64,128,256}");
  TORCH_CHECK((bn == 64 || bn == 128) && N % bn == 0, "gemm_decode: N % bn, bn in {64, 128}");
  TORCH_CHECK(splits >= 1 && splits <= 16 && K % 64 == 0 && K / 64 >= splits, "gemm_decode: bad split count");
  float* pp = nullptr;
  if (splits > 1) {
    TORCH_CHECK(p.has_value(), "split-K needs a partial buffer");
    CHECK_DT(*p, at::kFloat); CHECK_CONTIG(*p);
    TORCH_CHECK(p->numel() >= splits * M * N, "partial buffer too small");
    pp = p->data_ptr<float>();
  }
  TORCH_CHECK(K < (1LL << 31) / 64 && M * K < (1LL << 31) && N * K < (1LL << 40), "gemm too large");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  RC(oamd::gemm_decode(ptr<bf16_t>(x), ptr<bf16_t>(w), yp, pp, (int)M, (int)N, (int)K, (int)splits,
                       (int)bn, (int)bm, silu_gu, w_tiled, (int)stages, cur_stream()));
}

void gemm_tile(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& y_opt,
               const c10::optional<at::Tensor>& bias, bool silu_gu, int64_t variant, int64_t splits,
               const c10::optional<at::Tensor>& partial) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2, "x [M,K], w [N,K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemm_tile: w [N, K] must match x [M, K]");
  TORCH_CHECK(M >= 1 && K >= 64 && K % 64 == 0 && N % 16 == 0, "gemm_tile: K % 64 == 0, N % 16 == 0");
  TORCH_CHECK(splits >= 1 && splits <= 64 && K % (64 * splits) == 0, "gemm_tile: K % (64 * splits) == 0");
  bf16_t* yp = nullptr;
  int64_t ldy = silu_gu ? N / 2 : N;
  if (y_opt.has_value()) {
    const at::Tensor& y = *y_opt;
    CHECK_BF16(y);
    TORCH_CHECK(y.dim() == 2 && y.size(0) == M && y.size(1) == (silu_gu ? N / 2 : N) && y.stride(1) == 1 &&
                    y.stride(0) % 4 == 0,
                "gemm_tile: y [M, N] (N/2 with silu_gu), unit column stride, 8-B aligned rows");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(y.data_ptr()) % 8 == 0, "gemm_tile: y must be 8-B aligned");
    TORCH_CHECK(splits == 1 || silu_gu || y.stride(0) == N, "gemm_tile: split-K reduce needs a contiguous y");
    yp = ptr<bf16_t>(y);
    ldy = y.stride(0);
  } else {
    TORCH_CHECK(splits > 1 && !silu_gu, "y may be omitted only for split-K slabs summed by the consumer");
  }
  TORCH_CHECK(!silu_gu || (N % 128 == 0 && !bias.has_value()), "gemm_tile: SwiGLU needs N % 128, no bias");
  TORCH_CHECK(splits == 1 || !bias.has_value(), "gemm_tile: no bias with split-K");
  if (bias.has_value()) {
    CHECK_BF16(*bias); CHECK_CONTIG(*bias);
    TORCH_CHECK(bias->numel() == N, "gemm_tile: bias [N]");
  }
  float* pp = nullptr;
  if (splits > 1) {
    TORCH_CHECK(partial.has_value(), "gemm_tile: split-K needs a partial buffer");
    CHECK_DT(*partial, at::kFloat); CHECK_CONTIG(*partial);
    TORCH_CHECK(partial->numel() >= splits * M * N, "gemm_tile: partial buffer too small");
    pp = partial->data_ptr<float>();
  }
  TORCH_CHECK(M * K < (1LL << 40) && N * K < (1LL << 40) && M < (1LL << 31) && N < (1LL << 31), "gemm too large");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  RC(oamd::gemm_tile(ptr<bf16_t>(x), ptr<bf16_t>(w), yp, optr<bf16_t>(bias), (int)M, (int)N, (int)K, (int)ldy,
                     silu_gu, (int)variant, (int)splits, pp, cur_stream()));
}

void gemm_pp(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& y_opt,
             const c10::optional<at::Tensor>& p, int64_t splits, int64_t bm, bool silu_gu, bool nt, bool one_seg,
             const c10::optional<at::Tensor>& sk_ws, const c10::optional<at::Tensor>& sk_flags) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && w.size(1) == x.size(1), "x [M,K], w [N,K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && N % 128 == 0, "gemm_pp: N % 128 == 0");
  TORCH_CHECK(bm == 128 || bm == 256, "gemm_pp: bm in {128, 256}");
  TORCH_CHECK(splits >= 1 && splits <= 32 && K % (64 * splits) == 0, "gemm_pp: K % (64 * splits) == 0");
  TORCH_CHECK(!silu_gu || splits == 1, "gemm_pp: fused SwiGLU needs splits == 1");
  bf16_t* yp = nullptr;
  if (y_opt.has_value()) {
    CHECK_BF16(*y_opt); CHECK_CONTIG(*y_opt);
    TORCH_CHECK(y_opt->dim() == 2 && y_opt->size(0) == M && y_opt->size(1) == (silu_gu ? N / 2 : N), "gemm_pp: y");
    yp = ptr<bf16_t>(*y_opt);
  } else {
    TORCH_CHECK(splits > 1 && !silu_gu, "y may be omitted only for split-K slabs summed by the consumer");
  }
  float* pp = nullptr;
  if (splits > 1) {
    TORCH_CHECK(p.has_value(), "split-K needs a partial buffer");
    CHECK_DT(*p, at::kFloat); CHECK_CONTIG(*p);
    TORCH_CHECK(p->numel() >= splits * M * N, "partial buffer too small");
    pp = p->data_ptr<float>();
  }
  TORCH_CHECK(M * K < (1LL << 40) && N * K < (1LL << 40), "gemm too large");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  float* wsp = nullptr;
  int* flp = nullptr;
  if (sk_ws.has_value() || sk_flags.has_value()) {   // stream-K workspace: fp32 partials + zeroed int flags
    TORCH_CHECK(sk_ws.has_value() && sk_flags.has_value(), "gemm_pp: stream-K needs sk_ws and sk_flags");
    CHECK_DEV(*sk_ws); CHECK_DEV(*sk_flags); CHECK_CONTIG(*sk_ws); CHECK_CONTIG(*sk_flags);
    CHECK_DT(*sk_ws, at::kFloat); CHECK_DT(*sk_flags, at::kInt);
    TORCH_CHECK(sk_ws->numel() >= (N / 128) * 32768 && sk_flags->numel() >= N / 128, "gemm_pp: stream-K workspace too small");
    wsp = sk_ws->data_ptr<float>();
    flp = sk_flags->data_ptr<int>();
  }
  RC(oamd::gemm_pp(ptr<bf16_t>(x), ptr<bf16_t>(w), yp, pp, (int)M, (int)N, (int)K, (int)splits, (int)bm, silu_gu, nt,
                   cur_stream(), one_seg, wsp, flp));
}

void gemm_skinny(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& y_opt,
                 const c10::optional<at::Tensor>& p, int64_t splits, bool silu_gu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && w.size(1) == x.size(1), "x [M,K], w [N,K]");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 32, "gemm_skinny: M must be 1..32");
  TORCH_CHECK(N % (silu_gu ? 128 : 16) == 0, "gemm_skinny: N % 16 (128 for the fused SwiGLU)");
  TORCH_CHECK(splits >= 1 && splits <= 8 && K % (128 * splits) == 0, "gemm_skinny: K % (128 * splits)");
  TORCH_CHECK(!silu_gu || splits == 1, "fused SwiGLU needs splits = 1");
  bf16_t* yp = nullptr;
  if (y_opt.has_value()) {
    CHECK_BF16(*y_opt); CHECK_CONTIG(*y_opt);
    TORCH_CHECK(y_opt->dim() == 2 && y_opt->size(0) == M && y_opt->size(1) == (silu_gu ? N / 2 : N), "gemm shapes");
    yp = ptr<bf16_t>(*y_opt);
  } else {
    TORCH_CHECK(splits > 1 && !silu_gu, "y may be omitted only for split-K slabs summed by the consumer");
  }
  float* pp = nullptr;
  if (splits > 1) {
    TORCH_CHECK(p.has_value(), "split-K needs a partial buffer");
    CHECK_DT(*p, at::kFloat); CHECK_CONTIG(*p);
    TORCH_CHECK(p->numel() >= splits * M * N, "partial buffer too small");
    TORCH_CHECK((M * N) % 4 == 0 || yp == nullptr, "split-K reduce needs M * N % 4 == 0");
    pp = p->data_ptr<float>();
  }
  TORCH_CHECK(N * K < (1LL << 40) && M * K < (1LL << 31), "gemm too large");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  RC(oamd::gemm_skinny(ptr<bf16_t>(x), ptr<bf16_t>(w), yp, pp, (int)M, (int)N, (int)K, (int)splits, silu_gu,
                       cur_stream()));
}

void quantize_fp8(const at::Tensor& x, at::Tensor& q, at::Tensor& sx) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(q); CHECK_CONTIG(sx); CHECK_DT(sx, at::kFloat);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be [M, K] row-major");
  TORCH_CHECK(q.scalar_type() == at::kByte || q.scalar_type() == at::kFloat8_e4m3fn, "q must be uint8 / e4m3fn");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(q.numel() == M * K && sx.numel() == M && K % 8 == 0, "quantize_fp8 shapes");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  RC(oamd::quantize_fp8_rows(ptr<bf16_t>(x), static_cast<uint8_t*>(q.data_ptr()), ptr<float>(sx), (int)M, (int)K,
                             x.stride(0), cur_stream()));
}

// gu: bf16 [M, 2I] gate|up rows, or (slabs given) a shape carrier [M, 2I] whose values are the
// S fp32 split-K slabs [S, M, 2I] of the producing GEMM.
void silu_quantize_fp8(const at::Tensor& gu, at::Tensor& q, at::Tensor& sx, const c10::optional<at::Tensor>& slabs,
                       int64_t splits) {
  CHECK_DEV(gu); CHECK_CONTIG(q); CHECK_CONTIG(sx); CHECK_DT(sx, at::kFloat);
  TORCH_CHECK(gu.dim() == 2 && gu.stride(1) == 1, "gu must be [M, 2I] row-major");
  TORCH_CHECK(q.scalar_type() == at::kByte || q.scalar_type() == at::kFloat8_e4m3fn, "q must be uint8 / e4m3fn");
  const int64_t M = gu.size(0), I = gu.size(1) / 2;
  TORCH_CHECK(gu.size(1) % 128 == 0 && I <= 16384, "silu_quantize_fp8: 2I % 128 == 0, I <= 16384");
  TORCH_CHECK(q.numel() == M * I && sx.numel() == M, "silu_quantize_fp8 shapes");
  const float* pp = nullptr;
  if (slabs.has_value()) {
    CHECK_DT(*slabs, at::kFloat); CHECK_CONTIG(*slabs);
    TORCH_CHECK(splits >= 1 && slabs->numel() >= splits * M * 2 * I, "slabs: fp32 [splits, M, 2I]");
    pp = slabs->data_ptr<float>();
  } else {
    CHECK_BF16(gu);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  RC(oamd::silu_quantize_fp8(pp != nullptr ? nullptr : ptr<bf16_t>(gu), pp, (int)splits,
                             static_cast<uint8_t*>(q.data_ptr()), ptr<float>(sx), (int)M, (int)I,
                             pp != nullptr ? 2 * I : gu.stride(0), cur_stream()));
}

void gemm_fp8(const at::Tensor& x8, const at::Tensor& w8, const at::Tensor& sx, const at::Tensor& sw, at::Tensor& y,
              const c10::optional<at::Tensor>& p, int64_t splits, int64_t bn, int64_t bm, bool reduce) {
  CHECK_DEV(x8); CHECK_CONTIG(x8); CHECK_CONTIG(w8); CHECK_CONTIG(sx); CHECK_CONTIG(sw); CHECK_BF16(y);
  CHECK_CONTIG(y); CHECK_DT(sx, at::kFloat); CHECK_DT(sw, at::kFloat);
  for (auto* t : {&x8, &w8})
    TORCH_CHECK(t->scalar_type() == at::kByte || t->scalar_type() == at::kFloat8_e4m3fn, "fp8 operands");
  TORCH_CHECK(x8.dim() == 2 && w8.dim() == 2, "x8 [M,K], w8 [N,K]");
  const int64_t M = x8.size(0), K = x8.size(1), N = w8.size(0);
  TORCH_CHECK(w8.size(1) == K && y.size(0) == M && y.size(1) == N && sx.numel() == M && sw.numel() == N,
              "gemm_fp8 shapes");
  TORCH_CHECK((bn == 64 || bn == 128) && N % bn == 0, "gemm_fp8: N % bn");
  TORCH_CHECK(bm == 64 || bm == 128 || bm == 256, "gemm_fp8: bm in {64,128,256}");
  TORCH_CHECK(splits >= 1 && splits <= 16 && K % 128 == 0 && K / 128 >= splits, "gemm_fp8: K % 128, 1 <= splits <= min(16, K / 128)");
  float* pp = nullptr;
  if (splits > 1) {
    TORCH_CHECK(p.has_value() && p->scalar_type() == at::kFloat && p->numel() >= splits * M * N,
                "split-K needs an fp32 partial buffer");
    pp = p->data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x8.device());
  RC(oamd::gemm_fp8(static_cast<const uint8_t*>(x8.data_ptr()), static_cast<const uint8_t*>(w8.data_ptr()),
                    ptr<float>(sx), ptr<float>(sw), (reduce || splits == 1) ? ptr<bf16_t>(y) : nullptr, pp, (int)M, (int)N, (int)K, (int)splits, (int)bn,
                    (int)bm, cur_stream()));
}

void score_events(const at::Tensor& keys, const at::Tensor& hit_doc, const at::Tensor& doc_ptr,
                  const at::Tensor& prim_ptr, const at::Tensor& prim_pat, const at::Tensor& ev_ptr,
                  const at::Tensor& ev_doc_ptr, const at::Tensor& sec_ptr, const at::Tensor& sec_matcher,
                  const at::Tensor& sec_w, const at::Tensor& sec_win, const at::Tensor& conf,
                  const at::Tensor& severity, double significance, at::Tensor& ev_score, at::Tensor& ev_pat,
                  at::Tensor& ev_line, at::Tensor& order, at::Tensor& summary) {
  CHECK_DEV(keys); CHECK_DT(keys, at::kLong); CHECK_CONTIG(keys);
  for (auto* t : {&hit_doc, &doc_ptr, &prim_ptr, &prim_pat, &ev_ptr, &ev_doc_ptr, &sec_ptr, &sec_matcher, &sec_win,
                  &severity}) {
    CHECK_DT(*t, at::kInt); CHECK_CONTIG(*t); CHECK_DEV(*t);
  }
  for (auto* t : {&sec_w, &conf}) { CHECK_DT(*t, at::kDouble); CHECK_CONTIG(*t); }
  CHECK_DT(ev_score, at::kDouble); CHECK_DT(ev_pat, at::kInt); CHECK_DT(ev_line, at::kInt); CHECK_DT(order, at::kInt);
  CHECK_DT(summary, at::kInt);
  const int64_t n_hits = keys.numel(), n_docs = doc_ptr.numel() - 1;
  const int64_t n_pat = conf.numel(), n_m = prim_ptr.numel() - 1;
  TORCH_CHECK(hit_doc.numel() == n_hits && ev_ptr.numel() == n_hits + 1 && ev_doc_ptr.numel() == n_docs + 1,
              "score_events: hit index shapes");
  TORCH_CHECK(sec_ptr.numel() == n_pat + 1 && severity.numel() == n_pat && sec_matcher.numel() == sec_w.numel() &&
                  sec_w.numel() == sec_win.numel(), "score_events: pattern table shapes");
  TORCH_CHECK(summary.numel() >= 3 * n_docs, "summary [docs, 3]");
  const int64_t n_ev = ev_score.numel();
  TORCH_CHECK(ev_pat.numel() == n_ev && ev_line.numel() == n_ev && order.numel() == n_ev, "event buffer shapes");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(keys.device());
  RC(oamd::score_events(ptr<int64_t>(keys), ptr<int>(hit_doc), ptr<int>(doc_ptr), (int)n_hits, (int)n_docs,
                        ptr<int>(prim_ptr), ptr<int>(prim_pat), ptr<int>(ev_ptr), ptr<int>(ev_doc_ptr),
                        ptr<int>(sec_ptr), ptr<int>(sec_matcher), ptr<double>(sec_w), ptr<int>(sec_win),
                        ptr<double>(conf), ptr<int>(severity), (int)n_m, significance, ptr<double>(ev_score),
                        ptr<int>(ev_pat), ptr<int>(ev_line), ptr<int>(order), ptr<int>(summary), cur_stream()));
}

void attn_decode(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                 const at::Tensor& block_tables, const at::Tensor& seq_lens, at::Tensor& out,
                 at::Tensor& o_part, at::Tensor& ml_part, int64_t num_splits, double scale, int64_t variant,
                 double k_scale, double v_scale, const c10::optional<at::Tensor>& q8,
                 const c10::optional<at::Tensor>& sx, const c10::optional<at::Tensor>& rope_x, int64_t rope_splits,
                 const c10::optional<at::Tensor>& pos, const c10::optional<at::Tensor>& cos_t,
                 const c10::optional<at::Tensor>& sin_t, const c10::optional<at::Tensor>& slots,
                 const c10::optional<at::Tensor>& bias) {
  CHECK_DEV(q); CHECK_BF16(q); CHECK_CONTIG(q); CHECK_BF16(out); CHECK_CONTIG(out);
  const bool fp8 = kv_is_fp8(k_cache);
  TORCH_CHECK(fp8 ? kv_is_fp8(v_cache) : (k_cache.scalar_type() == at::kBFloat16 &&
                                          v_cache.scalar_type() == at::kBFloat16),
              "KV cache must be bf16 or float8_e4m3fn (both K and V)");
  CHECK_DEV(k_cache); CHECK_DEV(v_cache); CHECK_CONTIG(k_cache); CHECK_CONTIG(v_cache);
  CHECK_DT(block_tables, at::kInt); CHECK_CONTIG(block_tables); CHECK_DT(seq_lens, at::kInt); CHECK_CONTIG(seq_lens);
  CHECK_DT(o_part, at::kFloat); CHECK_DT(ml_part, at::kFloat); CHECK_CONTIG(o_part); CHECK_CONTIG(ml_part);
  TORCH_CHECK(q.dim() == 3, "q must be [B, Hq, D]");
  const int64_t B = q.size(0), Hq = q.size(1), D = q.size(2);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.sizes() == v_cache.sizes() && k_cache.size(3) == D, "cache shape");
  const int64_t Hkv = k_cache.size(1), page = k_cache.size(2);
  TORCH_CHECK(D == 128 && Hq % Hkv == 0, "head_dim must be 128 and Hq % Hkv == 0");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) == B && seq_lens.numel() == B, "tables shape");
  TORCH_CHECK(out.numel() == B * Hq * D, "out shape");
  TORCH_CHECK(num_splits >= 1, "num_splits >= 1");
  TORCH_CHECK(block_tables.size(1) <= 1024, "at most 1024 pages per sequence");
  TORCH_CHECK(num_splits == 1 ||
                  (o_part.numel() >= B * Hq * num_splits * D && ml_part.numel() >= B * Hq * num_splits * 2),
              "partial buffers too small");
  TORCH_CHECK(B * num_splits < (1LL << 31), "grid too large");
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "KV scales must be positive");
  TORCH_CHECK(q8.has_value() == sx.has_value(), "q8 and sx together");
  uint8_t* q8p = nullptr;
  float* sxp = nullptr;
  if (q8.has_value()) {
    CHECK_CONTIG(*q8); CHECK_CONTIG(*sx); CHECK_DT(*sx, at::kFloat);
    TORCH_CHECK((q8->scalar_type() == at::kByte || q8->scalar_type() == at::kFloat8_e4m3fn) &&
                    q8->numel() == B * Hq * D && sx->numel() == B && Hq * D <= 8192,
                "q8 e4m3fn [B, Hq*D], sx fp32 [B], Hq*D <= 8192");
    q8p = static_cast<uint8_t*>(q8->data_ptr());
    sxp = sx->data_ptr<float>();
  }
  // rope_x: the decode step's RoPE + KV write folded in (q unused, a shape carrier): the QKV
  // projection as `rope_splits` fp32 split-K slabs [S, B, (Hq+2Hkv)D] or bf16 rows [B, (Hq+2Hkv)D]
  oamd::DecRope rp{};
  const oamd::DecRope* rpp = nullptr;
  if (rope_x.has_value()) {
    TORCH_CHECK(pos.has_value() && cos_t.has_value() && sin_t.has_value() && slots.has_value(),
                "fused RoPE needs pos, cos, sin and slots");
    const int64_t ncol = (Hq + 2 * Hkv) * D;
    CHECK_DEV(*rope_x); CHECK_CONTIG(*rope_x);
    if (rope_x->scalar_type() == at::kFloat) {
      TORCH_CHECK(rope_splits >= 1 && rope_x->numel() >= rope_splits * B * ncol, "fused RoPE: slabs too small");
      rp.xp = rope_x->data_ptr<float>();
      rp.S = (int)rope_splits;
      rp.slab = B * ncol;
    } else {
      CHECK_BF16(*rope_x);
      TORCH_CHECK(rope_x->dim() == 2 && rope_x->size(0) == B && rope_x->size(1) == ncol, "fused RoPE: qkv [B, ncol]");
      rp.row = ptr<bf16_t>(*rope_x);
      rp.row_stride = rope_x->stride(0);
      rp.S = 1;
    }
    CHECK_DT(*pos, at::kLong); CHECK_CONTIG(*pos); CHECK_DT(*slots, at::kLong); CHECK_CONTIG(*slots);
    TORCH_CHECK(pos->numel() == B && slots->numel() == B, "fused RoPE: pos / slots [B]");
    CHECK_DT(*cos_t, at::kFloat); CHECK_DT(*sin_t, at::kFloat); CHECK_CONTIG(*cos_t); CHECK_CONTIG(*sin_t);
    TORCH_CHECK(cos_t->dim() == 2 && cos_t->size(1) == D / 2 && sin_t->sizes() == cos_t->sizes(), "cos/sin [max_pos, 64]");
    if (bias.has_value()) {
      CHECK_BF16(*bias); CHECK_CONTIG(*bias);
      TORCH_CHECK(bias->numel() == ncol, "fused RoPE: bias [(Hq+2Hkv)D]");
      rp.bias = ptr<bf16_t>(*bias);
    }
    rp.pos = pos->data_ptr<int64_t>();
    rp.slots = slots->data_ptr<int64_t>();
    rp.cos_t = cos_t->data_ptr<float>();
    rp.sin_t = sin_t->data_ptr<float>();
    rp.max_pos = cos_t->size(0);
    rp.k_inv = (float)(1.0 / k_scale);
    rp.v_inv = (float)(1.0 / v_scale);
    rpp = &rp;
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  RC(oamd::attn_decode(ptr<bf16_t>(q), k_cache.data_ptr(), v_cache.data_ptr(), fp8, (float)k_scale, (float)v_scale,
                       ptr<int>(block_tables), ptr<int>(seq_lens), ptr<bf16_t>(out), ptr<float>(o_part),
                       ptr<float>(ml_part), (int)B, (int)Hq, (int)Hkv, (int)D, (int)page, (int)block_tables.size(1),
                       (int)num_splits, (float)scale, (int)variant, cur_stream(), q8p, sxp, rpp));
}

// pk / pv / seq_pfx: a shared prompt prefix (kernels.h attn_prefill, variant 3): seq_pfx[s] prefix
// keys (at most pk.size(0)) precede sequence s's own keys.
void attn_prefill(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& o,
                  const at::Tensor& cu_seqlens, const at::Tensor& work_seq, const at::Tensor& work_q0,
                  double scale, int64_t variant, const c10::optional<at::Tensor>& pk,
                  const c10::optional<at::Tensor>& pv, const c10::optional<at::Tensor>& seq_pfx) {
  CHECK_DEV(q); for (auto* t : {&q, &k, &v}) { CHECK_BF16(*t); CHECK_CONTIG(*t); }
  CHECK_BF16(o); CHECK_CONTIG(o);
  for (auto* t : {&cu_seqlens, &work_seq, &work_q0}) { CHECK_DT(*t, at::kInt); CHECK_CONTIG(*t); }
  TORCH_CHECK(q.dim() == 3 && k.dim() == 3 && v.sizes() == k.sizes() && o.sizes() == q.sizes(), "qkvo shapes");
  TORCH_CHECK(q.size(0) == k.size(0) && q.size(2) == 128 && k.size(2) == 128, "T / head_dim mismatch");
  TORCH_CHECK(q.size(1) % k.size(1) == 0, "Hq % Hkv");
  TORCH_CHECK(work_seq.numel() == work_q0.numel(), "work list shape");
  const bf16_t *pkp = nullptr, *pvp = nullptr;
  const int* pfx = nullptr;
  if (seq_pfx.has_value()) {
    TORCH_CHECK(pk.has_value() && pv.has_value() && (variant == 3 || variant == 4), "a prefix needs pk, pv and variant 3 / 4");
    for (const auto* t : {&*pk, &*pv}) { CHECK_DEV(*t); CHECK_BF16(*t); CHECK_CONTIG(*t); }
    TORCH_CHECK(pk->dim() == 3 && pv->sizes() == pk->sizes() && pk->size(1) == k.size(1) && pk->size(2) == 128,
                "pk / pv [prefix, Hkv, 128]");
    CHECK_DEV(*seq_pfx); CHECK_DT(*seq_pfx, at::kInt); CHECK_CONTIG(*seq_pfx);
    TORCH_CHECK(seq_pfx->numel() >= cu_seqlens.numel() - 1, "seq_pfx: one prefix length per sequence");
    pkp = ptr<bf16_t>(*pk);
    pvp = ptr<bf16_t>(*pv);
    pfx = ptr<int>(*seq_pfx);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  RC(oamd::attn_prefill(ptr<bf16_t>(q), ptr<bf16_t>(k), ptr<bf16_t>(v), ptr<bf16_t>(o), ptr<int>(cu_seqlens),
                        ptr<int>(work_seq), ptr<int>(work_q0), (int)work_seq.numel(), (int)q.size(1),
                        (int)k.size(1), 128, (float)scale, (int)variant, cur_stream(), pkp, pvp, pfx));
}

void sample(const at::Tensor& logits, const at::Tensor& temperature, const at::Tensor& seeds,
            const at::Tensor& positions, at::Tensor& out, int64_t col_offset,
            const c10::optional<at::Tensor>& out_val) {
  CHECK_DEV(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [rows, vocab] row-major");
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16, "logits dtype");
  const int64_t rows = logits.size(0);
  CHECK_DT(temperature, at::kFloat); CHECK_DT(seeds, at::kLong); CHECK_DT(positions, at::kLong); CHECK_DT(out, at::kLong);
  TORCH_CHECK(temperature.numel() == rows && seeds.numel() == rows && positions.numel() == rows && out.numel() == rows,
              "sampler per-row tensor shape");
  if (out_val.has_value()) {
    CHECK_DT(*out_val, at::kFloat);
    TORCH_CHECK(out_val->numel() == rows, "out_val shape");
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  RC(oamd::sample_tokens(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, logits.stride(0), (int)rows,
                         (int)logits.size(1), ptr<float>(temperature), ptr<int64_t>(seeds), ptr<int64_t>(positions),
                         ptr<int64_t>(out), col_offset, optr<float>(out_val), cur_stream()));
}

}  // namespace

// Launch an instantiated hipGraph `count` times back to back on `stream` with the
// GIL released (decode windows: one call per window instead of one Python
// replay per step, so host threads contending for the GIL cannot stall the feed).
void graph_launch(int64_t exec, int64_t count, int64_t stream) {
  TORCH_CHECK(exec != 0 && count >= 0, "graph_launch: bad graph / count");
  hipError_t err = hipSuccess;
  {
    pybind11::gil_scoped_release nogil;
    for (int64_t i = 0; i < count && err == hipSuccess; ++i)
      err = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(exec), reinterpret_cast<hipStream_t>(stream));
  }
  TORCH_CHECK(err == hipSuccess, "hipGraphLaunch failed: ", hipGetErrorString(err));
}

void register_scan_bindings(pybind11::module_& m);
void register_comm_bindings(pybind11::module_& m);

PYBIND11_MODULE(_C, m) {
  m.doc() = "operator_amd gfx950 kernels";
  m.def("rmsnorm", &rmsnorm, "RMSNorm with optional fused residual add (and split-K slab sum)", pybind11::arg("x"),
        pybind11::arg("residual"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("eps"),
        pybind11::arg("partial") = pybind11::none(), pybind11::arg("splits") = 1, pybind11::arg("tiled_out") = false);
  m.def("gemm_xr", &gemm_xr, pybind11::arg("xt"), pybind11::arg("w"), pybind11::arg("y") = pybind11::none(),
        pybind11::arg("p") = pybind11::none(), pybind11::arg("splits") = 1, pybind11::arg("epi") = 1);
  m.def("tile_rows", &tile_rows, pybind11::arg("x"), pybind11::arg("xt"));
  m.def("silu_mul", &silu_mul, pybind11::arg("gu"), pybind11::arg("out"), pybind11::arg("block") = 0);
  m.def("embedding", &embedding);
  m.def("rope_kv", &rope_kv, pybind11::arg("qkv"), pybind11::arg("pos"), pybind11::arg("cos"),
        pybind11::arg("sin"), pybind11::arg("Hq"), pybind11::arg("Hkv"), pybind11::arg("q_out"),
        pybind11::arg("k_out"), pybind11::arg("v_out"), pybind11::arg("k_cache"), pybind11::arg("v_cache"),
        pybind11::arg("slots"), pybind11::arg("partial") = pybind11::none(), pybind11::arg("splits") = 1,
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("k_scale") = 1.0, pybind11::arg("v_scale") = 1.0);
  m.def("attn_decode", &attn_decode, pybind11::arg("q"), pybind11::arg("k_cache"), pybind11::arg("v_cache"),
        pybind11::arg("block_tables"), pybind11::arg("seq_lens"), pybind11::arg("out"), pybind11::arg("o_part"),
        pybind11::arg("ml_part"), pybind11::arg("num_splits"), pybind11::arg("scale"), pybind11::arg("variant") = 0,
        pybind11::arg("k_scale") = 1.0, pybind11::arg("v_scale") = 1.0, pybind11::arg("q8") = pybind11::none(),
        pybind11::arg("sx") = pybind11::none(), pybind11::arg("rope_x") = pybind11::none(),
        pybind11::arg("rope_splits") = 1, pybind11::arg("pos") = pybind11::none(), pybind11::arg("cos") = pybind11::none(),
        pybind11::arg("sin") = pybind11::none(), pybind11::arg("slots") = pybind11::none(),
        pybind11::arg("bias") = pybind11::none());
  m.def("decode_slots", &decode_slots);
  m.def("decode_advance", &decode_advance);
  m.def("quantize_fp8", &quantize_fp8);
  m.def("silu_quantize_fp8", &silu_quantize_fp8, pybind11::arg("gu"), pybind11::arg("q"), pybind11::arg("sx"),
        pybind11::arg("slabs") = pybind11::none(), pybind11::arg("splits") = 1);
  m.def("score_events", &score_events);
  m.def("gemm_fp8", &gemm_fp8, pybind11::arg("x8"), pybind11::arg("w8"), pybind11::arg("sx"), pybind11::arg("sw"),
        pybind11::arg("y"), pybind11::arg("p") = pybind11::none(), pybind11::arg("splits") = 1,
        pybind11::arg("bn") = 64, pybind11::arg("bm") = 64, pybind11::arg("reduce") = true);
  m.def("gemm_decode", &gemm_decode, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"),
        pybind11::arg("p") = pybind11::none(), pybind11::arg("splits") = 1, pybind11::arg("bn") = 64,
        pybind11::arg("bm") = 0, pybind11::arg("silu_gu") = false, pybind11::arg("w_tiled") = false,
        pybind11::arg("stages") = 3);
  m.def("gemm_tile", &gemm_tile, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"),
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("silu_gu") = false, pybind11::arg("variant") = 0,
        pybind11::arg("splits") = 1, pybind11::arg("partial") = pybind11::none());
  m.def("gemm_pp", &gemm_pp, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"),
        pybind11::arg("p") = pybind11::none(), pybind11::arg("splits") = 1, pybind11::arg("bm") = 256,
        pybind11::arg("silu_gu") = false, pybind11::arg("nt") = true, pybind11::arg("one_seg") = false,
        pybind11::arg("sk_ws") = pybind11::none(), pybind11::arg("sk_flags") = pybind11::none());
  m.def("gemm_pp_sk_grid", &oamd::gemm_pp_sk_grid, pybind11::arg("tiles"), pybind11::arg("steps"));
  m.def("gemm_skinny", &gemm_skinny, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"),
        pybind11::arg("p") = pybind11::none(), pybind11::arg("splits") = 1, pybind11::arg("silu_gu") = false);
  m.def("attn_prefill", &attn_prefill, pybind11::arg("q"), pybind11::arg("k"), pybind11::arg("v"),
        pybind11::arg("o"), pybind11::arg("cu_seqlens"), pybind11::arg("work_seq"), pybind11::arg("work_q0"),
        pybind11::arg("scale"), pybind11::arg("block_q") = 64, pybind11::arg("pk") = pybind11::none(),
        pybind11::arg("pv") = pybind11::none(), pybind11::arg("seq_pfx") = pybind11::none());
  m.def("attn_prefill_block_q", &oamd::attn_prefill_block_q);
  m.def("sample", &sample, pybind11::arg("logits"), pybind11::arg("temperature"), pybind11::arg("seeds"),
        pybind11::arg("positions"), pybind11::arg("out"), pybind11::arg("col_offset") = 0,
        pybind11::arg("out_val") = pybind11::none());
  m.def("graph_launch", &graph_launch, pybind11::arg("graph_exec"), pybind11::arg("count"), pybind11::arg("stream"));
  register_scan_bindings(m);
  register_comm_bindings(m);
  m.attr("ARCH") = "gfx950";
}
