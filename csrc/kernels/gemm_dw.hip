// Decode GEMM with a deep, decoupled weight stream (the M = 256 decode bucket):
//   Y[M, N] = X[M, K] . W[N, K]^T,  M <= 256, bf16 in, fp32 accumulate
// (SURVEY.md §2.4 N7 "Decode uses skinny-M split-K with nt weight streaming"; replaces
// the external LLM behind J/service/AIInterfaceRestClient.java:37-39).
//
// At M = 256 a projection is balanced between the MFMA pipe and HBM (256 FLOP per weight
// byte: at a CU's share of HBM, ~25-33 GB/s, the MFMAs must be ~75 % busy just to keep
// pace), so the weight stream needs ~2 us of loads in flight per CU while the
// activations (2 MB, L2-resident) only need one step. With one wave doing both, the
// in-order vmcnt makes the deep weight loads as "due" as the shallow activation loads
// issued after them (waiting for X(t+1) retires every older W(t+2..)). Here the two
// streams are issued by DIFFERENT waves, so each counter covers one stream:
//   * 8 waves (2 per SIMD). Group 0 (waves 0-3) LDS-DMAs the weight tile of K-step
//     t + WD while computing step t (WD = 4: 64 KiB of weights in flight per CU at
//     BN = 128); group 1 (waves 4-7) LDS-DMAs the activation tile of step t + 1.
//     Each group waits only for its own stream (counted vmcnt), then one raw
//     s_barrier per K-step publishes both;
//   * the tile is ALL M rows (one row tile: every weight byte is read once) x BN
//     columns, BK = 64; weight ring WD + 1 slots, activation ring 2 slots, all LDS
//     in one array; rows are 128-B lines stored lane-linearly by the DMA with the
//     chunk ^ ((row >> 1) & 7) swizzle applied to the SOURCE and the read
//     (conflict-free ds_read_b128);
//   * weights stream with the non-temporal policy (read once per launch, by one CU:
//     MI355X_MICROARCH.md "nt-weights"), activations with the default policy;
//   * waves 4 (M) x 2 (N); operands swapped in the MFMA (A = weight fragment) so a lane
//     holds 4 consecutive features of one token: 8-B bf16 stores, 16-B fp32 split-K slab
//     stores, and the fused SwiGLU of the 64-row interleaved gate|up weight in
//     registers (wave wn owns gate rows wn*32.. and the matching up rows 64 + wn*32..);
//   * split-K over blockIdx: block b -> K-slice b % S, column tile b / S; with S | 8 the
//     blocks of one K-slice share an XCD (speed only), so each L2 holds its slice of X.
#include "common.h"
#include "kernels.h"

namespace oamd {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kBK = 64;
constexpr int kRows = 256;              // M tile (all decode rows)
constexpr int kXSlot = kRows * 128;     // 32 KiB per activation stage

enum { kStore = 0, kPartial = 1, kSilu = 2 };

template <int N>
__device__ __forceinline__ void vmw() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint2 pack4(f32x4 v) { return make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])); }

// wait until at most n * G of this wave's vector-memory ops are outstanding (n < 8)
template <int G>
__device__ __forceinline__ void vmw_n(int n) {
  switch (n) {
    case 0: vmw<0>(); break;
    case 1: vmw<G>(); break;
    case 2: vmw<2 * G>(); break;
    case 3: vmw<3 * G>(); break;
    case 4: vmw<4 * G>(); break;
    case 5: vmw<5 * G>(); break;
    case 6: vmw<6 * G>(); break;
    default: vmw<7 * G>(); break;
  }
}

}  // namespace

template <int BN, int EPI, int WD>
__global__ void __launch_bounds__(512) gemm_dw_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                      bf16_t* __restrict__ Y, float* __restrict__ P, int M, int N,
                                                      int K, int S) {
  constexpr int NW = WD + 1;                       // weight ring slots
  constexpr int WSLOT = BN * 128;                  // bytes per weight stage
  constexpr int GW = BN / 8 / 4;                   // weight DMA instructions per group-0 wave per stage
  constexpr int GX = kRows / 8 / 4;                // activation DMA instructions per group-1 wave per stage
  constexpr int WF = BN / 2 / 16;                  // weight (feature) fragments per wave
  __shared__ __attribute__((aligned(1024))) char lds[2 * kXSlot + NW * WSLOT];
  char* const xs_lds = lds;
  char* const ws_lds = lds + 2 * kXSlot;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2;                            // 0: weight loader, 1: activation loader
  const int wm = w & 3, wn = w >> 2;               // compute position: 64-row quarter, column half
  const int kz = blockIdx.x % S, nt = blockIdx.x / S;
  const int n0 = nt * BN;
  const int Kc = K / S;
  const int T = Kc / kBK;
  const int64_t kbase = (int64_t)kz * Kc;

  // DMA sources: instruction q of a stage covers rows 8q .. 8q+7 (lane l -> row 8q + l/8,
  // LDS slot l%8, global chunk slot ^ ((row >> 1) & 7)); group-g wave (w & 3) issues
  // q = (w & 3) + 4i
  const int lrow = lane >> 3, lslot = lane & 7;
  const int wl = w & 3;
  const bf16_t* src[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 8 * (wl + 4 * i) + lrow;
    const int chunk = lslot ^ ((row >> 1) & 7);
    if (g == 0) src[i] = W + (int64_t)(n0 + min(row, BN - 1)) * K + kbase + chunk * 8;
    else src[i] = X + (int64_t)min(row, M - 1) * K + kbase + chunk * 8;
  }
  auto issue_w = [&](int kt) {   // group 0
    char* dst = ws_lds + (kt % NW) * WSLOT;
#pragma unroll
    for (int i = 0; i < GW; ++i)
      __builtin_amdgcn_global_load_lds(src[i] + kt * kBK,
                                       (__attribute__((address_space(3))) void*)(dst + (wl + 4 * i) * 1024), 16, 0,
                                       2);   // nt: streamed once
  };
  auto issue_x = [&](int kt) {   // group 1
    char* dst = xs_lds + (kt & 1) * kXSlot;
#pragma unroll
    for (int i = 0; i < GX; ++i)
      __builtin_amdgcn_global_load_lds(src[i] + kt * kBK,
                                       (__attribute__((address_space(3))) void*)(dst + (wl + 4 * i) * 1024), 16, 0,
                                       0);
  };

  // fragment read offsets (row & 15 == lane & 15 for every fragment: the swizzle term is
  // per lane); k-substep s reads chunks 4s + lq
  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int c0 = (lq ^ sw) << 4, c1 = ((4 + lq) ^ sw) << 4;
  const int xrow = (wm * 64 + l15) * 128;
  // weight fragment j: rows (j / 2) * 64 + wn * 32 + (j % 2) * 16 at BN = 128 (gate|up
  // interleave: j < 2 gate, j >= 2 up); at BN = 64, rows wn * 32 + j * 16
  auto wrow = [&](int j) {
    const int r = (BN == 128) ? (j >> 1) * 64 + wn * 32 + (j & 1) * 16 : wn * 32 + j * 16;
    return (r + l15) * 128;
  };

  f32x4 acc[4][WF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: weights of steps 0 .. WD-1, activations of step 0
  if (g == 0) {
    for (int t = 0; t < WD; ++t)
      if (t < T) issue_w(t);
    vmw_n<GW>(min(WD, T) - 1);   // step 0's weights landed
  } else {
    issue_x(0);
    vmw<0>();
  }
  __builtin_amdgcn_s_barrier();

  for (int t = 0; t < T; ++t) {
    if (g == 0) {
      if (t + WD < T) issue_w(t + WD);
    } else if (t + 1 < T) {
      issue_x(t + 1);
    }
    const char* xb = xs_lds + (t & 1) * kXSlot;
    const char* wb = ws_lds + (t % NW) * WSLOT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = s ? c1 : c0;
      u16x8 xf[4], wf[WF];
#pragma unroll
      for (int j = 0; j < WF; ++j) wf[j] = *reinterpret_cast<const u16x8*>(wb + wrow(j) + c);
#pragma unroll
      for (int i = 0; i < 4; ++i) xf[i] = *reinterpret_cast<const u16x8*>(xb + xrow + i * 2048 + c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < WF; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[j]),
                                                              __builtin_bit_cast(bf16x8_t, xf[i]), acc[i][j], 0, 0, 0);
    }
    // own stream's next stage landed; own fragment reads done (the slot refilled next
    // step was read this step)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (g == 0) vmw_n<GW>(min(WD - 1, T - 2 - t) < 0 ? 0 : min(WD - 1, T - 2 - t));
    else vmw<0>();
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: lane holds features 4*lq .. 4*lq+3 of token l15 per (token block i, fragment j)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int tok = wm * 64 + i * 16 + l15;
    if (tok >= M) continue;
    if constexpr (EPI == kSilu) {
      // fragments j = 0, 1: gate rows wn*32 + 16j; j = 2, 3: the matching up rows
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = (n0 >> 1) + wn * 32 + j * 16 + 4 * lq;
        const f32x4 gt = acc[i][j], up = acc[i][j + 2];
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gg = bf2f(f2bf(gt[r]));
          const float uu = bf2f(f2bf(up[r]));
          o[r] = bf2f(f2bf(gg / (1.f + __expf(-gg)))) * uu;
        }
        *reinterpret_cast<uint2*>(Y + (int64_t)tok * (N >> 1) + col) = pack4(o);
      }
    } else {
#pragma unroll
      for (int j = 0; j < WF; ++j) {
        const int col = n0 + ((BN == 128) ? (j >> 1) * 64 + wn * 32 + (j & 1) * 16 : wn * 32 + j * 16) + 4 * lq;
        if constexpr (EPI == kPartial)
          *reinterpret_cast<f32x4*>(P + ((int64_t)kz * M + tok) * N + col) = acc[i][j];
        else
          *reinterpret_cast<uint2*>(Y + (int64_t)tok * N + col) = pack4(acc[i][j]);
      }
    }
  }
}

int gemm_dw(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, int BN, bool silu_gu,
            hipStream_t stream) {
  if (M < 1 || M > kRows || (BN != 64 && BN != 128) || N % BN != 0) return -1;
  if (S < 1 || S > 32 || K % (kBK * S) != 0) return -2;
  if (silu_gu && (S != 1 || BN != 128)) return -3;
  if (S > 1 && P == nullptr) return -4;
  if (S == 1 && Y == nullptr) return -5;
  const dim3 grid((N / BN) * S);
  const int epi = silu_gu ? kSilu : (S > 1 ? kPartial : kStore);
#define OAMD_DW(B, E) gemm_dw_kernel<B, E, 4><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K, S)
  if (BN == 128) {
    if (epi == kSilu) OAMD_DW(128, kSilu);
    else if (epi == kPartial) OAMD_DW(128, kPartial);
    else OAMD_DW(128, kStore);
  } else {
    if (epi == kPartial) OAMD_DW(64, kPartial);
    else OAMD_DW(64, kStore);
  }
#undef OAMD_DW
  OAMD_LAUNCH_CHECK();
  if (S > 1 && Y != nullptr) return splitk_reduce(P, Y, (int64_t)M * N, S, stream);
  return 0;
}

}  // namespace oamd
