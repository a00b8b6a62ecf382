// RMSNorm (+ fused residual add), SiLU-and-mul, embedding gather.
//
// These are the memory-bound elementwise/normalisation ops of the explanation
// model. All bf16 traffic is 16 B per lane.
#include "common.h"
#include "kernels.h"

namespace oamd {

// One 256-thread block per row. Each thread owns up to MAXV vectors of 8 bf16
// kept in registers between the reduction and the scaling pass, so the row is
// read from HBM exactly once (x, and residual when fused).
// With `xp` set, x is not read: the row is the bf16 rounding of the sum of S
// fp32 split-K slabs xp[s * slab + row * hidden + c] written by gemm_decode —
// the GEMM's reduction pass is folded into this kernel (same numerics: the
// projection output is rounded to bf16 once, then added to the residual).
// SC = compile-time slab count (0: runtime S) so the S slab loads of a vector are
// all issued before the first add (a runtime-trip-count loop waits for each load
// in turn: S dependent L2/HBM round trips per vector).
template <int NT, int MAXV, int SC>
__global__ void __launch_bounds__(NT) rmsnorm_kernel(
    const bf16_t* __restrict__ x, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int hidden,
    int64_t x_stride, int64_t r_stride, int64_t y_stride, float eps,
    const float* __restrict__ xp, int S_rt, int64_t slab) {
  const int S = SC > 0 ? SC : S_rt;
  __shared__ float scratch[NT / 64];
  const int row = blockIdx.x;
  const int nvec = hidden >> 3;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + row * x_stride);
  u16x8* rr = residual ? reinterpret_cast<u16x8*>(residual + row * r_stride) : nullptr;
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      u16x8 a;
      if (xp) {
        const float* pr = xp + (int64_t)row * hidden + vi * 8;
        f32x4 lo = *reinterpret_cast<const f32x4*>(pr), hi = *reinterpret_cast<const f32x4*>(pr + 4);
        if constexpr (SC > 0) {
          f32x4 pl[SC > 1 ? SC - 1 : 1], ph[SC > 1 ? SC - 1 : 1];
#pragma unroll
          for (int sp = 1; sp < SC; ++sp) {
            pl[sp - 1] = *reinterpret_cast<const f32x4*>(pr + sp * slab);
            ph[sp - 1] = *reinterpret_cast<const f32x4*>(pr + sp * slab + 4);
          }
#pragma unroll
          for (int sp = 1; sp < SC; ++sp) {
            lo += pl[sp - 1];
            hi += ph[sp - 1];
          }
        } else {
          for (int sp = 1; sp < S; ++sp) {
            lo += *reinterpret_cast<const f32x4*>(pr + sp * slab);
            hi += *reinterpret_cast<const f32x4*>(pr + sp * slab + 4);
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = f2bf(lo[j]);
          a[4 + j] = f2bf(hi[j]);
        }
      } else {
        a = xr[vi];
      }
      if (rr) {
        u16x8 b = rr[vi];
        u16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // residual stream is bf16: round the sum before normalising it
          s[j] = f2bf(bf2f(a[j]) + bf2f(b[j]));
        }
        rr[vi] = s;
        a = s;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = bf2f(a[j]);
        ss += v[i][j] * v[i][j];
      }
    }
  }
  // the weight vectors are requested before the block reduction, so their round trip
  // overlaps the barrier instead of following it
  const u16x8* wr = reinterpret_cast<const u16x8*>(w);
  u16x8 wpre[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) wpre[i] = wr[vi];
  }
  const float tot = block_sum<NT>(ss, scratch);
  const float rs = rsqrtf(tot / static_cast<float>(hidden) + eps);
  // y_stride < 0: y is written in the fragment-major tiled layout that gemm_xr reads its
  // activations from (common.h xr_tiled_off; one block per row, rows % 16 == 0)
  const bool tiled = y_stride < 0;
  u16x8* yr = reinterpret_cast<u16x8*>(y + (tiled ? 0 : row * y_stride));
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = threadIdx.x + i * NT;
    if (vi < nvec) {
      const u16x8 wv = wpre[i];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // HF semantics: normalised value is rounded to bf16, then scaled by w
        o[j] = f2bf(bf2f(f2bf(v[i][j] * rs)) * bf2f(wv[j]));
      }
      if (tiled) {
        *reinterpret_cast<u16x8*>(y + xr_tiled_off(row, vi * 8, gridDim.x)) = o;
      } else {
        yr[vi] = o;
      }
    }
  }
}

int rmsnorm(const bf16_t* x, bf16_t* residual, const bf16_t* w, bf16_t* y,
            int rows, int hidden, int64_t x_stride, int64_t r_stride,
            int64_t y_stride, float eps, const float* xp, int S, hipStream_t stream) {
  if (rows == 0) return 0;
  constexpr int NT = 256;
  const int nvec = hidden / 8;
  const int64_t slab = (int64_t)rows * hidden;
  const int sc = xp == nullptr ? 1 : S;
  // split-K slab sums of rows up to 4096 wide: 512 threads, one vector each, so a row's
  // slab loads all leave in one round (OAMD_RMS_WIDE=0: 256 threads x 2 vectors)
  static const bool wide = [] { const char* e = getenv("OAMD_RMS_WIDE"); return !(e && e[0] == '0'); }();
  if (wide && xp != nullptr && sc > 1 && nvec > NT && nvec <= 2 * NT) {
    switch (sc) {
      case 2: rmsnorm_kernel<2 * NT, 1, 2><<<rows, 2 * NT, 0, stream>>>(x, residual, w, y, hidden, x_stride, r_stride, y_stride, eps, xp, S, slab); break;
      case 4: rmsnorm_kernel<2 * NT, 1, 4><<<rows, 2 * NT, 0, stream>>>(x, residual, w, y, hidden, x_stride, r_stride, y_stride, eps, xp, S, slab); break;
      case 8: rmsnorm_kernel<2 * NT, 1, 8><<<rows, 2 * NT, 0, stream>>>(x, residual, w, y, hidden, x_stride, r_stride, y_stride, eps, xp, S, slab); break;
      default: rmsnorm_kernel<2 * NT, 1, 0><<<rows, 2 * NT, 0, stream>>>(x, residual, w, y, hidden, x_stride, r_stride, y_stride, eps, xp, S, slab); break;
    }
    OAMD_LAUNCH_CHECK();
    return 0;
  }
#define OAMD_RMS(MV, SCC) \
  rmsnorm_kernel<NT, MV, SCC><<<rows, NT, 0, stream>>>(x, residual, w, y, hidden, x_stride, r_stride, y_stride, eps, xp, S, slab)
#define OAMD_RMS_S(MV)                  \
  switch (sc) {                         \
    case 1: OAMD_RMS(MV, 1); break;     \
    case 2: OAMD_RMS(MV, 2); break;     \
    case 4: OAMD_RMS(MV, 4); break;     \
    case 8: OAMD_RMS(MV, 8); break;     \
    default: OAMD_RMS(MV, 0); break;    \
  }
  if (nvec <= NT * 2) {
    OAMD_RMS_S(2)
  } else if (nvec <= NT * 4) {
    OAMD_RMS_S(4)
  } else {
    OAMD_RMS_S(8)
  }
#undef OAMD_RMS_S
#undef OAMD_RMS
  OAMD_LAUNCH_CHECK();
  return 0;
}

// out[m, i] = silu(gate) * up; grid-stride over 8-element vectors. gate|up
// columns are interleaved in blocks of `block` features (block == inter: the
// plain [gate | up] concatenation): gate of feature i at (i / block) * 2 * block
// + i % block, up `block` columns later.
__global__ void silu_mul_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ out,
                                int64_t rows, int inter, int block, int64_t in_stride, int64_t out_stride) {
  const int vpr = inter >> 3;
  const int64_t total = rows * vpr;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = idx / vpr;
    const int c = static_cast<int>(idx - m * vpr) << 3;
    const int gc = (c / block) * 2 * block + c % block;
    const u16x8 g = *reinterpret_cast<const u16x8*>(gu + m * in_stride + gc);
    const u16x8 u = *reinterpret_cast<const u16x8*>(gu + m * in_stride + gc + block);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]);
      // HF: act(gate) rounded to bf16, then multiplied by up in bf16
      const float s = bf2f(f2bf(gf / (1.f + __expf(-gf))));
      o[j] = f2bf(s * bf2f(u[j]));
    }
    *reinterpret_cast<u16x8*>(out + m * out_stride + c) = o;
  }
}

int silu_mul(const bf16_t* gu, bf16_t* out, int64_t rows, int inter, int block,
             int64_t in_stride, int64_t out_stride, hipStream_t stream) {
  if (rows == 0) return 0;
  if (block <= 0 || block % 8 != 0 || inter % block != 0) return -1;
  const int64_t total = rows * (inter / 8);
  const int nt = 256;
  int64_t blocks = (total + nt - 1) / nt;
  if (blocks > 256 * 16) blocks = 256 * 16;
  silu_mul_kernel<<<static_cast<int>(blocks), nt, 0, stream>>>(gu, out, rows, inter, block, in_stride,
                                                               out_stride);
  OAMD_LAUNCH_CHECK();
  return 0;
}

// Row gather: out[t, :] = table[ids[t], :]. One block per token, 16 B per lane.
__global__ void embedding_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ table,
                                 bf16_t* __restrict__ out, int hidden, int64_t vocab) {
  const int t = blockIdx.x;
  int64_t id = ids[t];
  if (id < 0 || id >= vocab) id = 0;  // out-of-range ids are clamped, never read OOB
  const u16x8* src = reinterpret_cast<const u16x8*>(table + id * hidden);
  u16x8* dst = reinterpret_cast<u16x8*>(out + (int64_t)t * hidden);
  for (int i = threadIdx.x; i < (hidden >> 3); i += blockDim.x) dst[i] = src[i];
}

int embedding(const int64_t* ids, const bf16_t* table, bf16_t* out, int tokens,
              int hidden, int64_t vocab, hipStream_t stream) {
  if (tokens == 0) return 0;
  embedding_kernel<<<tokens, 256, 0, stream>>>(ids, table, out, hidden, vocab);
  OAMD_LAUNCH_CHECK();
  return 0;
}

// Decode-step bookkeeping of a hipGraph-captured step (engine/llm.py _DecodeGraph), one
// thread per batch row instead of ~15 one-op torch kernels:
//   decode_slots:   slot = page(bt[row], pos / P) * P + pos % P for live rows (ctx > 0), else -1;
//                   spos = pos + 1 (the sampler's stream position)
//   decode_advance: ids = tok; hist[row, step % ms] = tok; live rows pos += 1, ctx += 1; then
//                   (one thread) step += 1
__global__ void decode_slots_kernel(const int* __restrict__ bt, const int64_t* __restrict__ pos,
                                    const int* __restrict__ ctx, int64_t* __restrict__ slots,
                                    int64_t* __restrict__ spos, int B, int max_pages, int page_size) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  const int64_t p = pos[r];
  int64_t pg = p / page_size;
  pg = pg < max_pages - 1 ? pg : max_pages - 1;
  slots[r] = ctx[r] > 0 ? (int64_t)bt[(int64_t)r * max_pages + pg] * page_size + p % page_size : -1;
  spos[r] = p + 1;
}

__global__ void decode_advance_kernel(const int64_t* __restrict__ tok, int64_t* __restrict__ ids,
                                      int64_t* __restrict__ hist, int64_t* __restrict__ pos, int* __restrict__ ctx,
                                      int64_t* __restrict__ step, int B, int ms) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < B) {
    const int64_t t = tok[r];
    ids[r] = t;
    hist[(int64_t)r * ms + (int)(step[0] % ms)] = t;
    if (ctx[r] > 0) {
      pos[r] += 1;
      ctx[r] += 1;
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // every block read step[0] before block 0's thread 0 bumps it: one block covers all rows
    step[0] += 1;
  }
}

int decode_slots(const int* bt, const int64_t* pos, const int* ctx, int64_t* slots, int64_t* spos, int B,
                 int max_pages, int page_size, hipStream_t stream) {
  if (B <= 0) return 0;
  if (B > 1024) return -1;
  decode_slots_kernel<<<1, 1024, 0, stream>>>(bt, pos, ctx, slots, spos, B, max_pages, page_size);
  OAMD_LAUNCH_CHECK();
  return 0;
}

int decode_advance(const int64_t* tok, int64_t* ids, int64_t* hist, int64_t* pos, int* ctx, int64_t* step, int B,
                   int ms, hipStream_t stream) {
  if (B <= 0) return 0;
  if (B > 1024) return -1;   // one block: every row reads step before it is bumped
  decode_advance_kernel<<<1, 1024, 0, stream>>>(tok, ids, hist, pos, ctx, step, B, ms);
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
