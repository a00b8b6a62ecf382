// Decode-shape GEMM: Y[M, N] = X[M, K] . W[N, K]^T, bf16 in, fp32 accumulate
// (SURVEY.md §2.4 N7 — the explanation model's projections at decode batch).
//
// At decode the activations are small (M = bucket size, 64..256 rows) and the
// weights are streamed once per step, so the kernel is designed around the
// two streams rather than around a square tile:
//   * W (HBM, read once) and X (L2-resident, re-read by every column tile) are
//     both staged through LDS by LDS-DMA (global_load_lds_dwordx4) in full
//     128-B lines — no VGPR round trip, no fragment-shaped global loads
//     (cdna_hip_programming.md §5 "Projection GEMM at M = 256", item 3);
//   * a 3-deep LDS ring with a counted vmcnt + raw s_barrier keeps two stages
//     of both operands in flight across every barrier (never a vmcnt(0) drain
//     inside the k-loop);
//   * the LDS image is XOR-swizzled on the SOURCE address (the DMA writes LDS
//     lane-linearly), slot = chunk ^ ((row >> 1) & 7), which makes every
//     ds_read_b128 fragment read conflict-free;
//   * 8 waves (4 x 2), two per SIMD; the tile is BM = M rows x 64 columns; K is split S ways when N / 64
//     column tiles alone cannot fill 256 CUs. Split-K partials are fp32 slabs
//     [S][M][N] summed by gemm_splitk_reduce (or by a consumer kernel). With
//     S | 8 the blocks of one K-slice share an XCD (block id % 8), so each
//     XCD's L2 holds only its slice of X; other S (<= 16) cut K into slices
//     that differ by at most one 64-column step.
// MFMA v_mfma_f32_16x16x32_bf16; fragment maps as in attn_decode.hip.
#include "common.h"
#include "kernels.h"

namespace oamd {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kBK = 64;     // K per stage: one 128-B line per row
constexpr int kStages = 3;  // default LDS ring depth (2: two blocks per CU for the smaller tiles; 4 / 5 / 6:
                            // three / four / five stages in flight for tiles with BM + BN <= 320 / 256 /
                            // 192 rows, 160 KB of LDS at most)

// 8 waves (2 per SIMD: one wave's LDS-read latency hides under the other's
// MFMAs) laid out 4 (M) x 2 (N).
constexpr int kWaves = 8;

// BN = 128 halves the LDS fragment traffic per MFMA (64 x 64 wave tiles at
// M = 256: 0.5 KB of ds_read per MFMA vs 0.75 KB at BN = 64, where the LDS
// port, not the MFMA, sets the pace); BN = 64 gives twice the column tiles for
// the narrow projections.
template <int BM, int BN, int NS = kStages>
struct GemmCfg {
  static constexpr int WM = 4;                           // waves along M
  static constexpr int WN = kWaves / WM;                 // waves along N
  static constexpr int FM = BM / WM / 16;                // 16-row fragments per wave
  static constexpr int FN = BN / WN / 16;                // 16-col fragments per wave
  static constexpr int ROWS = BM + BN;                   // rows of one stage (A then B)
  static constexpr int STAGE_BYTES = ROWS * kBK * 2;     // bf16
  static constexpr int GL = ROWS / 8 / kWaves;           // LDS-DMA instructions per wave per stage
  static constexpr int LDS_BYTES = NS * STAGE_BYTES;
  static_assert(ROWS % (8 * kWaves) == 0, "stage rows must split evenly over the waves");
};

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Epilogues: plain bf16 store, fp32 split-K slab, or the fused SwiGLU of the
// gate|up projection (weights interleaved in 64-row blocks: tile columns
// [0,64) = gate, [64,128) = up of the same 64 features; output [M, N/2]).
enum { kEpiStore = 0, kEpiPartial = 1, kEpiSiluGU = 2 };

template <int BM, int BN, int EPI, int NS = kStages>
__global__ void __launch_bounds__(kWaves * 64, NS == 2 ? 2 : 1) gemm_tn_kernel(const bf16_t* __restrict__ X,
                                                                 const bf16_t* __restrict__ W, bf16_t* __restrict__ Y,
                                                                 float* __restrict__ P, int M, int N, int K, int S,
                                                                 int w_tiled) {
  using C = GemmCfg<BM, BN, NS>;
  __shared__ __attribute__((aligned(1024))) char lds[C::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kz = blockIdx.x % S, nt = blockIdx.x / S;
  const int n0 = nt * BN;
  const int m0 = blockIdx.y * BM;  // row tile (M may be split into BM-row tiles)
  X += (int64_t)m0 * K;
  // K-slice kz = K-steps [kz * TK / S, (kz + 1) * TK / S): slices differ by at most one step
  // when S does not divide TK (S = 5 puts 240 workgroups of the 48-tile qkv on 256 CUs)
  const int TK = K / kBK;
  const int t0 = kz * TK / S;
  const int kbase = t0 * kBK;
  const int T = (kz + 1) * TK / S - t0;

  // ---- LDS-DMA issue of one stage: instruction q covers rows 8q..8q+7 of the
  // stage (A rows [0, BM), then B rows [BM, BM + BN)); lane l -> row 8q + l/8,
  // LDS slot l%8, global chunk swz(row, slot).
  const int lrow = lane >> 3, lslot = lane & 7;
  auto issue_one = [&](int t, int buf, int i) {
    const int k0 = kbase + t * kBK;
    char* sbase = lds + buf * C::STAGE_BYTES;
    {
      const int q = w + kWaves * i;
      const int row = 8 * q + lrow;
      const int chunk = swz(row, lslot);
      const int wn_ = n0 + row - BM;
      // tiled W ([N/64][K/64][64][64]): each 8-row x 128-B piece of a stage is one
      // contiguous 1 KB of HBM instead of 8 separate 128-B row segments
      const bf16_t* wsrc = (w_tiled & 1) ? W + ((int64_t)(wn_ >> 6) * (K >> 6) + (k0 >> 6)) * 4096 + (wn_ & 63) * 64 + chunk * 8
                                   : W + (int64_t)wn_ * K + k0 + chunk * 8;
      const bf16_t* src = (row < BM) ? X + (int64_t)row * K + k0 + chunk * 8 : wsrc;
      if ((w_tiled & 2) && row >= BM)   // wave-uniform (8-row pieces): weights stream non-temporal
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sbase + q * 1024), 16, 0, 2);
      else
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(sbase + q * 1024), 16, 0, 0);
    }
  };
  auto issue = [&](int t, int buf) {
#pragma unroll
    for (int i = 0; i < C::GL; ++i) issue_one(t, buf, i);
  };

  const int wm = w / C::WN, wn = w % C::WN;
  const int l15 = lane & 15, lg = lane >> 4;
  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One stage of MFMAs; the LDS-DMA pieces of stage `tn` are spread between them
  // (piece g after MFMA ((g+1) * TOT) / (GL+1)) so the issue cost of the DMA
  // overlaps MFMA execution instead of stalling both waves of a SIMD after the
  // barrier.
  constexpr int TOT = (kBK / 32) * C::FM * C::FN;
  auto compute = [&](int buf, int tn, bool do_issue) {
    const char* sbase = lds + buf * C::STAGE_BYTES;
#pragma unroll
    for (int s = 0; s < kBK / 32; ++s) {
      const int chunk = 4 * s + lg;
      u16x8 a[C::FM], b[C::FN];
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const int row = wm * (BM / C::WM) + 16 * i + l15;
        a[i] = *reinterpret_cast<const u16x8*>(sbase + row * 128 + (swz(row, chunk) << 4));
      }
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int row = BM + wn * (BN / C::WN) + 16 * j + l15;
        b[j] = *reinterpret_cast<const u16x8*>(sbase + row * 128 + (swz(row, chunk) << 4));
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a[i]),
                                                              __builtin_bit_cast(bf16x8_t, b[j]), acc[i][j], 0, 0, 0);
          const int idx = (s * C::FM + i) * C::FN + j + 1;
#pragma unroll
          for (int g = 0; g < C::GL; ++g)
            if (idx == ((g + 1) * TOT) / (C::GL + 1) && do_issue) issue_one(tn, tn % NS, g);
        }
    }
  };

  // prologue: stages 0 .. NS-2 in flight; iteration t issues stage t + NS - 1
  // into the buffer compute(t - 1) just released (fenced by the barrier)
  issue(0, 0);
#pragma unroll
  for (int st = 1; st < NS - 1; ++st)
    if (T > st) issue(st, st);
  for (int t = 0; t < T; ++t) {
    // stages issued so far: min(T, t + NS - 1); leave all but stage t in flight
    const int rem = min(T - 1 - t, NS - 2);   // stages younger than t in flight
    if (NS >= 6 && rem >= 4) wait_vmcnt<4 * C::GL>();
    else if (NS >= 5 && rem >= 3) wait_vmcnt<3 * C::GL>();
    else if (NS >= 4 && rem >= 2) wait_vmcnt<2 * C::GL>();
    else if (NS >= 3 && rem >= 1) wait_vmcnt<C::GL>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    compute(t % NS, t + NS - 1, t + NS - 1 < T);
  }

  if constexpr (EPI == kEpiSiluGU) {
    // Stage the tile through LDS (the ring is idle now) so each thread sees a
    // feature's gate and up values: HF numerics, act(bf16(g)) rounded to bf16,
    // times bf16(u), rounded.
    static_assert(BN == 128, "fused SwiGLU needs gate and up halves in one tile");
    constexpr int LD = BN + 4;  // fp32 row stride (+4: spreads the column writes over banks)
    static_assert(BM * LD * 4 <= C::LDS_BYTES, "C tile must fit the LDS ring");
    float* ct = reinterpret_cast<float*>(lds);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int col = wn * (BN / C::WN) + 16 * j + l15;
#pragma unroll
        for (int r = 0; r < 4; ++r) ct[(wm * (BM / C::WM) + 16 * i + 4 * lg + r) * LD + col] = acc[i][j][r];
      }
    __syncthreads();
    const int NO = N / 2;  // output features
    for (int v = tid; v < BM * 8; v += kWaves * 64) {
      const int row = v >> 3, f0 = (v & 7) * 8;
      const float* cr = ct + row * LD;
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = bf2f(f2bf(cr[f0 + e]));
        const float u = bf2f(f2bf(cr[64 + f0 + e]));
        const float sg = bf2f(f2bf(g / (1.f + __expf(-g))));
        o[e] = f2bf(sg * u);
      }
      *reinterpret_cast<u16x8*>(Y + (int64_t)(m0 + row) * NO + nt * 64 + f0) = o;
    }
  } else {
    // ---- C lane l -> row 4*lg + r, col l15 of each fragment ----
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int col = n0 + wn * (BN / C::WN) + 16 * j + l15;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * (BM / C::WM) + 16 * i + 4 * lg + r;
          if constexpr (EPI == kEpiPartial) P[((int64_t)kz * M + m0 + row) * N + col] = acc[i][j][r];
          else Y[(int64_t)(m0 + row) * N + col] = f2bf(acc[i][j][r]);
        }
      }
  }
}

// Y[m, n] = bf16(sum_s P[s, m, n]); 4 columns per thread.
__global__ void gemm_splitk_reduce_kernel(const float* __restrict__ P, bf16_t* __restrict__ Y, int64_t MN, int S) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= MN) return;
  f32x4 a = *reinterpret_cast<const f32x4*>(P + i);
  for (int s = 1; s < S; ++s) a += *reinterpret_cast<const f32x4*>(P + s * MN + i);
  uint2 o;
  o.x = pack_bf2(a[0], a[1]);
  o.y = pack_bf2(a[2], a[3]);
  *reinterpret_cast<uint2*>(Y + i) = o;
}

int splitk_reduce(const float* P, bf16_t* Y, int64_t MN, int S, hipStream_t stream) {
  if (MN % 4 != 0 || S < 1) return -1;
  const int64_t threads = MN / 4;
  gemm_splitk_reduce_kernel<<<(threads + 255) / 256, 256, 0, stream>>>(P, Y, MN, S);
  OAMD_LAUNCH_CHECK();
  return 0;
}

int gemm_decode(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, int BN,
                int BM, bool silu_gu, bool w_tiled_b, int stages, hipStream_t stream) {
  // bit 0: tiled W layout; bit 1: W streams with the non-temporal policy (OAMD_BF16_WNT)
  static const int wnt = [] { const char* e = getenv("OAMD_BF16_WNT"); return e && e[0] == '0' ? 0 : 2; }();
  const int w_tiled = (w_tiled_b ? 1 : 0) | wnt;
  if (w_tiled_b && (N % 64 != 0 || K % 64 != 0)) return -6;
  if ((BM != 64 && BM != 128 && BM != 256) || M % BM != 0) return -1;
  if (silu_gu) {  // fused SwiGLU: one K slice, 128-column tiles of 64 gate + 64 up rows
    if (BN != 128 || S != 1 || N % 128 != 0 || K % kBK != 0) return -5;
    const dim3 grid(N / 128, M / BM);
    switch (BM) {
      case 64:
        if (stages == 2) gemm_tn_kernel<64, 128, kEpiSiluGU, 2><<<grid, kWaves * 64, 0, stream>>>(X, W, Y, P, M, N, K, 1, w_tiled);
        else if (stages == 4) gemm_tn_kernel<64, 128, kEpiSiluGU, 4><<<grid, kWaves * 64, 0, stream>>>(X, W, Y, P, M, N, K, 1, w_tiled);
        else gemm_tn_kernel<64, 128, kEpiSiluGU><<<grid, kWaves * 64, 0, stream>>>(X, W, Y, P, M, N, K, 1, w_tiled);
        break;
      case 128:
        if (stages == 4) gemm_tn_kernel<128, 128, kEpiSiluGU, 4><<<grid, kWaves * 64, 0, stream>>>(X, W, Y, P, M, N, K, 1, w_tiled);
        else gemm_tn_kernel<128, 128, kEpiSiluGU><<<grid, kWaves * 64, 0, stream>>>(X, W, Y, P, M, N, K, 1, w_tiled);
        break;
      default: gemm_tn_kernel<256, 128, kEpiSiluGU><<<grid, kWaves * 64, 0, stream>>>(X, W, Y, P, M, N, K, 1, w_tiled); break;
    }
    OAMD_LAUNCH_CHECK();
    return 0;
  }
  if ((BN != 64 && BN != 128) || N % BN != 0) return -2;
  if (S < 1 || S > 16 || K % kBK != 0 || K / kBK < S) return -3;
  if (S > 1 && P == nullptr) return -4;
  const dim3 grid((N / BN) * S, M / BM);
#define OAMD_GEMM3(BM, BNN, NSS)                                                                               \
  if (S > 1) gemm_tn_kernel<BM, BNN, kEpiPartial, NSS><<<grid, kWaves * 64, 0, stream>>>(X, W, Y, P, M, N, K, S,   \
                                                                                       w_tiled);              \
  else gemm_tn_kernel<BM, BNN, kEpiStore, NSS><<<grid, kWaves * 64, 0, stream>>>(X, W, Y, P, M, N, K, S, w_tiled)
#define OAMD_GEMM2(BM, BNN)                                   \
  if (stages == 2 && BM <= 128) {                              \
    OAMD_GEMM3(BM, BNN, 2);                                    \
  } else if (stages == 4 && BM + BNN <= 320) {                 \
    OAMD_GEMM3(BM, BNN, (BM + BNN <= 320 ? 4 : 3));            \
  } else if (stages == 5 && BM + BNN <= 256) {                 \
    OAMD_GEMM3(BM, BNN, (BM + BNN <= 256 ? 5 : 3));            \
  } else if (stages == 6 && BM + BNN <= 192) {                 \
    OAMD_GEMM3(BM, BNN, (BM + BNN <= 192 ? 6 : 3));            \
  } else {                                                     \
    OAMD_GEMM3(BM, BNN, 3);                                    \
  }
#define OAMD_GEMM(BM) \
  if (BN == 64) { OAMD_GEMM2(BM, 64); } else { OAMD_GEMM2(BM, 128); }
  switch (BM) {
    case 64: OAMD_GEMM(64); break;
    case 128: OAMD_GEMM(128); break;
    default: OAMD_GEMM(256); break;
  }
#undef OAMD_GEMM
#undef OAMD_GEMM2
#undef OAMD_GEMM3
  OAMD_LAUNCH_CHECK();
  if (S > 1 && Y != nullptr) {  // Y == nullptr: the consumer sums the slabs (rmsnorm)
    const int64_t MN = (int64_t)M * N;
    const int64_t threads = MN / 4;
    gemm_splitk_reduce_kernel<<<(threads + 255) / 256, 256, 0, stream>>>(P, Y, MN, S);
    OAMD_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace oamd
