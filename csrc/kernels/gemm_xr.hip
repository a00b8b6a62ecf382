// Decode GEMM for the 256-row bucket with the activations streamed through REGISTERS
// ("xr"): Y[256, N] = X[256, K] . W[N, K]^T, bf16 in, fp32 accumulate
// (SURVEY.md §2.4 N7 decode GEMMs; replaces the external LLM behind
// J/service/AIInterfaceRestClient.java:37-39).
//
// Why: at M = 256 the decode GEMMs are bound by what one CU can keep in flight, not by the
// MFMA (round 5: gemm_pp's gate|up spends 55 of its 71 us loading operands; a CU ingests
// ~ its bytes in flight / ~2.1 us, profiles/decode_gemm_ingest_gate_up.jsonl). Every
// workgroup of a column tile needs ALL 256 activation rows, so X is 2/3 of what a CU
// ingests, and with both operands staged through LDS the 160 KiB of LDS caps what is in
// flight at ~96 KiB. Here
//   * the workgroup is 4 waves, one per SIMD, each owning 64 TOKENS x the BN = 128 features
//     of the column tile (128 accumulators); a wave needs only its own 64 activation rows,
//     so X never touches LDS: it arrives global -> VGPR in a 4-slot register ring, three
//     K-steps ahead, as whole 1 KiB MFMA B-fragments -- X is read in the fragment-major
//     "tiled" layout [K/64][M/16][2][64 lanes][8] that its producer writes (rmsnorm with a
//     tiled output, or this kernel's own SwiGLU epilogue for the down projection): each
//     wave-load is one contiguous KiB (no fragment-shaped row gathers) and one K-step of all
//     256 rows is one contiguous 32 KiB (every workgroup reads the same step at about the
//     same time: spread over the L2 channels, not strided onto a few);
//   * the whole LDS is a weight ring: NS = 8 stages of 128 rows x 64 k (16 KiB, LDS-DMA,
//     non-temporal), issued 8 steps ahead;
//   * both streams are counted by hand (the X loads are inline asm so hipcc's waitcnt pass,
//     which cannot count LDS-DMA, never drains the queue): one vmcnt + one barrier per K-step.
// In flight per CU: ~120 KiB of weights + ~80 KiB of activations (vs 96 KiB for gemm_pp).
// Epilogues: fp32 split-K slabs [S][256][N] (summed by rmsnorm / rope_kv), bf16 rows, or the
// fused SwiGLU of the 64-row interleaved gate|up weight written row-major or TILED (the down
// projection's X).
#include "common.h"
#include "kernels.h"

namespace oamd {

namespace {

constexpr int kXrBK = 64;       // K per step
constexpr int kXrBN = 128;      // features per workgroup
constexpr int kXrNS = 8;        // weight-ring stages (16 KiB each)
constexpr int kXrR = 4;         // activation register-ring slots
constexpr int kXrPX = 3;        // activation prefetch distance (steps)
constexpr int kXrStage = kXrBN * kXrBK * 2;

enum { kXrPartial = 0, kXrStore = 1, kXrSilu = 2, kXrSiluTiled = 3 };

template <int N>
__device__ __forceinline__ void xr_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// one 1 KiB MFMA B-fragment of the tiled activations: lane l loads its 16 B at
// base + voff (the block's byte offset + 16 l); hipcc does not see this load
__device__ __forceinline__ void xr_load(u16x8& dst, const void* base, uint32_t voff) {
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(dst) : "v"(voff), "s"(base) : "memory");
}

__device__ __forceinline__ void xr_mfma(f32x4& acc, const u16x8& a, const u16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

}  // namespace

// grid: (N / 128) * S blocks, block = n-tile * S + k-slice; 256 threads
// ABL (ablation arms for timing only, wrong results): bit 0 = no activation loads past the
// prologue, bit 1 = no weight loads past the prologue
template <int EPI, int ABL = 0>
__global__ void __launch_bounds__(256) gemm_xr_kernel(const bf16_t* __restrict__ Xt, const bf16_t* __restrict__ W,
                                                      bf16_t* __restrict__ Y, float* __restrict__ P, int N, int K,
                                                      int S) {
  constexpr int M = 256;
  __shared__ __attribute__((aligned(1024))) char lds[kXrNS * kXrStage];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kz = blockIdx.x % S, nt = blockIdx.x / S;
  const int n0 = nt * kXrBN;
  const int Kc = K / S, kbase = kz * Kc;
  const int T = Kc / kXrBK;

  // ---- weight pieces: piece q (0..15) = tile rows 8q .. 8q+7; wave w issues q = w + 4i;
  // lane l -> row 8q + l/8, LDS slot l % 8, source chunk slot ^ ((row >> 1) & 7)
  const int lrow = lane >> 3, lslot = lane & 7;
  const bf16_t* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 8 * (w + 4 * i) + lrow;
    wsrc[i] = W + (int64_t)(n0 + row) * K + kbase + ((lslot ^ ((row >> 1) & 7)) * 8);
  }
  auto issue_w = [&](int t, int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds(wsrc[i] + t * kXrBK,
                                       (__attribute__((address_space(3))) void*)(lds + buf * kXrStage +
                                                                                 (w + 4 * i) * 1024),
                                       16, 0, 2);
  };
  // ---- activation fragments of this wave: token block b (0..3) = rows 64 w + 16 b .. +15;
  // step t = 64-k block kbase / 64 + t: 32 KiB at (kbase / 64 + t) * 32 KiB, fragment
  // (token block, k-half kb) at ((16 b' + ...) * 2 + kb) KiB
  const char* xbase = reinterpret_cast<const char*>(Xt) + (int64_t)(kbase / kXrBK) * 32768;
  uint32_t xoff[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) xoff[b] = (uint32_t)(((4 * w + b) * 2) * 1024 + lane * 16);
  u16x8 xr[kXrR][4][2];
  auto issue_x = [&](int t, u16x8 (&slot)[4][2]) {
    const char* base = xbase + (int64_t)t * 32768;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      xr_load(slot[b][0], base, xoff[b]);
      xr_load(slot[b][1], base + 1024, xoff[b]);
    }
  };
  // ---- weight fragments: W fragment j = tile rows 16 j + l15, k-half h chunk 4h + lane/16
  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;

  f32x4 acc[4][8];
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[b][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+a"(acc[b][j]));
    }
  asm volatile("s_nop 4");

  // Issue order (what every vmcnt below counts): prologue X(0), W(0), X(1), W(1), X(2), W(2),
  // W(3) .. W(NS-1) -- the first step's operands first, so its wait is not behind the whole
  // weight prefill (in-order vmcnt: the round-6 first cut issued W(0..7) first and its first
  // MFMA waited for 128 KiB per CU); then in the middle of step s: X(s + PX) into ring slot
  // (s + PX) % R (last read by step s - 1) and W(s + NS) into LDS buffer s % NS (released by
  // the barrier just passed), each only if < T.
  // Step t: k-half 0 MFMAs (+ reads of k-half 1's weight fragments) | wait for X(t+1) and
  // W(t+1), barrier | issue | k-half 1 MFMAs (+ reads of step t+1's k-half-0 fragments).
  static_assert(kXrPX == 3 && kXrNS == 8, "the wait counts below are written for PX = 3, NS = 8");
#pragma unroll
  for (int s = 0; s < kXrPX; ++s) {
    if (s < T) issue_x(s, xr[s]);
    if (s < T) issue_w(s, s);
  }
#pragma unroll
  for (int s = kXrPX; s < kXrNS; ++s)
    if (s < T) issue_w(s, s);
  auto wcount = [&](int lo, int hi) {   // prologue weight stages lo .. hi-1 that exist (4 loads each)
    int n = 0;
    for (int s = lo; s < hi; ++s) n += s < T ? 4 : 0;
    return n;
  };
  // vm ops issued after the later of X(t+1), W(t+1) by the time step t - 1 has issued
  // (t = -1: before step 0, which needs X(0), W(0)); steady state 16
  auto after = [&](int t) -> int {
    const int u = t + 1;
    if (u <= 2) {   // W(u) follows X(u) in the prologue
      int n = (u + 1 <= 2 && u + 1 < T ? 8 + 4 : 0) + (u + 2 <= 2 && u + 2 < T ? 8 + 4 : 0) + wcount(3, kXrNS);
      for (int s = 0; s < t; ++s) n += (s + kXrPX < T ? 8 : 0) + (s + kXrNS < T ? 4 : 0);
      return n;
    }
    const int s0 = u - kXrPX;   // the step that issued X(u); W(u) left earlier
    int n = s0 + kXrNS < T ? 4 : 0;
    for (int s = s0 + 1; s < t; ++s) n += (s + kXrPX < T ? 8 : 0) + (s + kXrNS < T ? 4 : 0);
    return n;
  };
  auto wait_n = [&](int n) {
    if (n >= 44) xr_vmcnt<44>();
    else if (n >= 40) xr_vmcnt<40>();
    else if (n >= 32) xr_vmcnt<32>();
    else if (n >= 28) xr_vmcnt<28>();
    else if (n >= 24) xr_vmcnt<24>();
    else if (n >= 20) xr_vmcnt<20>();
    else if (n >= 16) xr_vmcnt<16>();
    else if (n >= 12) xr_vmcnt<12>();
    else if (n >= 8) xr_vmcnt<8>();
    else if (n >= 4) xr_vmcnt<4>();
    else xr_vmcnt<0>();
  };
  const int wo0 = l15 * 128 + ((lq ^ sw) << 4), wo1 = l15 * 128 + (((4 + lq) ^ sw) << 4);
  u16x8 wf0[8], wf1[8];
  auto rdw = [&](u16x8 (&wf)[8], int buf, int off, int j) {
    wf[j] = *reinterpret_cast<const u16x8*>(lds + buf * kXrStage + off + j * 2048);
  };
  wait_n(after(-1));
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < 8; ++j) rdw(wf0, 0, wo0, j);

  auto step = [&](int t, u16x8 (&xs)[4][2], u16x8 (&xn)[4][2], bool steady) {
    const int buf = t % kXrNS;
    // k-half 0: MFMA row j (4 token blocks) after the read of k-half 1's fragment j
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      rdw(wf1, buf, wo1, j);
#pragma unroll
      for (int b = 0; b < 4; ++b) xr_mfma(acc[b][j], wf0[j], xs[b][0]);
    }
    if (steady) xr_vmcnt<16>();   // X(t+1) (and, older, W(t+1)) landed for this wave
    else wait_n(after(t));   // steps 0 .. t-1 have issued
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this step's reads of buffer `buf` are done
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (!(ABL & 1) && (steady || t + kXrPX < T)) issue_x(t + kXrPX, xn);
    if (!(ABL & 2) && (steady || t + kXrNS < T)) issue_w(t + kXrNS, buf);
    const bool more = steady || t + 1 < T;
    const int nbuf = (t + 1) % kXrNS;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (more) rdw(wf0, nbuf, wo0, j);
#pragma unroll
      for (int b = 0; b < 4; ++b) xr_mfma(acc[b][j], wf1[j], xs[b][1]);
    }
  };
  // ring slot of X(t) = t % 4; X(t + 3) goes to slot (t + 3) % 4 = (t - 1) % 4. A steady step
  // (t >= 2, t + NS < T) issues both streams and finds 16 loads after X(t+1). Steps 0, 1, then
  // steady chunks of 4, then a fully unrolled tail (a run-time ring-slot choice makes hipcc
  // merge the slots with register copies -- reads of registers whose asm loads are in flight)
  int t = 0;
  if (0 < T) step(0, xr[0], xr[3], false);
  if (1 < T) step(1, xr[1], xr[0], false);
  for (t = 2; t + 3 + kXrNS < T; t += 4) {
    step(t, xr[2], xr[1], true);
    step(t + 1, xr[3], xr[2], true);
    step(t + 2, xr[0], xr[3], true);
    step(t + 3, xr[1], xr[0], true);
  }
  // t = 2 (mod 4), at most 11 steps left
  if (t < T) step(t, xr[2], xr[1], false);
  if (t + 1 < T) step(t + 1, xr[3], xr[2], false);
  if (t + 2 < T) step(t + 2, xr[0], xr[3], false);
  if (t + 3 < T) step(t + 3, xr[1], xr[0], false);
  if (t + 4 < T) step(t + 4, xr[2], xr[1], false);
  if (t + 5 < T) step(t + 5, xr[3], xr[2], false);
  if (t + 6 < T) step(t + 6, xr[0], xr[3], false);
  if (t + 7 < T) step(t + 7, xr[1], xr[0], false);
  if (t + 8 < T) step(t + 8, xr[2], xr[1], false);
  if (t + 9 < T) step(t + 9, xr[3], xr[2], false);
  if (t + 10 < T) step(t + 10, xr[0], xr[3], false);
  xr_vmcnt<0>();
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");

  // ---- epilogue: lane holds features 16 j + 4 lq .. +3 of token 64 w + 16 b + l15
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int tok = 64 * w + 16 * b + l15;
    if constexpr (EPI == kXrSilu || EPI == kXrSiluTiled) {
      const int NO = N / 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // j: gate rows, j + 4: the same features' up rows
        const f32x4 gt = acc[b][j], up = acc[b][j + 4];
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gg = bf2f(f2bf(gt[r]));
          const float uu = bf2f(f2bf(up[r]));
          o[r] = bf2f(f2bf(gg / (1.f + __expf(-gg)))) * uu;
        }
        const int of = nt * 64 + 16 * j + 4 * lq;   // output feature
        const uint2 v = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
        if constexpr (EPI == kXrSiluTiled) {
          *reinterpret_cast<uint2*>(Y + xr_tiled_off(tok, of, M)) = v;
        } else {
          *reinterpret_cast<uint2*>(Y + (int64_t)tok * NO + of) = v;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = n0 + 16 * j + 4 * lq;
        if constexpr (EPI == kXrPartial)
          *reinterpret_cast<f32x4*>(P + ((int64_t)kz * M + tok) * N + col) = acc[b][j];
        else
          *reinterpret_cast<uint2*>(Y + (int64_t)tok * N + col) =
              make_uint2(pack_bf2(acc[b][j][0], acc[b][j][1]), pack_bf2(acc[b][j][2], acc[b][j][3]));
      }
    }
  }
}

// x [rows, K] row-major -> the fragment-major tiled layout [K/64][rows/16][2][64][8]
__global__ void tile_rows_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xt, int rows, int K) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // one 16-B vector each
  if (i >= (int64_t)rows * (K / 8)) return;
  const int r = (int)(i / (K / 8)), c = (int)(i % (K / 8)) * 8;
  *reinterpret_cast<u16x8*>(xt + xr_tiled_off(r, c, rows)) = *reinterpret_cast<const u16x8*>(x + (int64_t)r * K + c);
}

int tile_rows(const bf16_t* x, bf16_t* xt, int rows, int K, hipStream_t stream) {
  if (rows % 16 != 0 || K % 64 != 0) return -1;
  const int64_t n = (int64_t)rows * (K / 8);
  tile_rows_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(x, xt, rows, K);
  OAMD_LAUNCH_CHECK();
  return 0;
}

int gemm_xr(const bf16_t* Xt, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, int epi,
            hipStream_t stream) {
  if (M != 256 || N % kXrBN != 0 || S < 1 || K % (kXrBK * S) != 0 || K % 32 != 0) return -1;
  if ((epi == kXrPartial || epi >= 10) != (P != nullptr) || (epi != kXrPartial && epi < 10 && Y == nullptr)) return -2;
  if ((epi == kXrSilu || epi == kXrSiluTiled) && S != 1) return -3;
  if (epi == kXrSiluTiled && (N / 2) % 64 != 0) return -4;
  const int grid = (N / kXrBN) * S;
  switch (epi) {
    case kXrPartial: gemm_xr_kernel<kXrPartial><<<grid, 256, 0, stream>>>(Xt, W, Y, P, N, K, S); break;
    case 10: gemm_xr_kernel<kXrPartial, 1><<<grid, 256, 0, stream>>>(Xt, W, Y, P, N, K, S); break;   // ablations
    case 11: gemm_xr_kernel<kXrPartial, 2><<<grid, 256, 0, stream>>>(Xt, W, Y, P, N, K, S); break;
    case 12: gemm_xr_kernel<kXrPartial, 3><<<grid, 256, 0, stream>>>(Xt, W, Y, P, N, K, S); break;
    case kXrStore: gemm_xr_kernel<kXrStore><<<grid, 256, 0, stream>>>(Xt, W, Y, P, N, K, S); break;
    case kXrSilu: gemm_xr_kernel<kXrSilu><<<grid, 256, 0, stream>>>(Xt, W, Y, P, N, K, S); break;
    case kXrSiluTiled: gemm_xr_kernel<kXrSiluTiled><<<grid, 256, 0, stream>>>(Xt, W, Y, P, N, K, S); break;
    default: return -5;
  }
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
