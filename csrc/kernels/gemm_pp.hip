// Decode-bucket GEMM on the ping-pong schedule of gemm_tile.hip:
//   Y[M, N] = X[M, K] . W[N, K]^T, M <= 256 (decode batch), bf16 in, fp32 accumulate
// (SURVEY.md §2.4 N7 "Decode uses skinny-M split-K with nt weight streaming";
// replaces the external LLM behind J/service/AIInterfaceRestClient.java:37-39).
//
// Round 2's gemm_decode waits for a stage, barriers all 8 waves and then reads
// fragments and runs MFMAs in lock-step, once per k-step: rocprofv3 put 38 % of
// its wave-cycles in s_waitcnt (profiles/gemm_decode_m256_stalls_pmc.txt). Here:
//   * tile = BM (128 x XH) tokens x 128 features, 8 waves in two groups running
//     one barrier segment apart (waves 4-7 behind): on every SIMD one wave reads
//     LDS fragments / issues DMA while its partner runs 16 MFMAs (16x16x32 bf16);
//   * a K-tile (BK = 64) = XH phases, one per 128-token half; every phase reads its
//     X fragments, the first also the W fragments, and issues one 16 KiB region of
//     the K-tile TWO ahead (3 LDS buffers x (XH + 1) regions): the weight rows come
//     from HBM, so they get ~2 K-tiles of latency; vmcnt is counted, never drained;
//   * weights stream with the non-temporal policy when NT (one CU reads each weight
//     byte once: MI355X_MICROARCH.md "nt-weights"); X (L2-resident) default policy;
//   * operands swapped in the MFMA (A = W) so each lane holds 4 consecutive
//     features of one token: 8-B bf16 stores, 16-B fp32 split-K slab stores, and the
//     fused SwiGLU of the 64-row interleaved gate|up weight (wave wc owns gate rows
//     wc*16.. and up rows 64 + wc*16.. of the 128-row tile) in registers;
//   * split-K: blockIdx.y = K slice, fp32 slabs P[S][M][N] summed by the consumer
//     (rmsnorm / rope_kv) or gemm_splitk_reduce.
// LDS image: lane-linear LDS-DMA rows of 128 B with the chunk ^ ((row >> 1) & 7)
// swizzle applied on the source and the read (conflict-free ds_read_b128).
#include "common.h"
#include "kernels.h"

namespace oamd {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kBK = 64;
constexpr int kRegion = 16384;   // 128 rows x 128 B
constexpr int kNBuf = 3;

enum { kStore = 0, kPartial = 1, kSilu = 2 };

template <int N>
__device__ __forceinline__ void vmw() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void seg() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ uint2 pack4(f32x4 v) { return make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])); }

}  // namespace

// XH: 128-token halves per tile (1 or 2). Regions per buffer: [X half 0][W][X half 1].
// SCHED (XH == 2):
//   0: ping-pong, two barrier segments per K-tile (one per X half);
//   1 (ONE): ping-pong, the K-tile in ONE barrier segment per wave group (both X halves'
//      32 MFMAs behind one pair of barriers, all three regions of tile t+2 issued together);
//   2 (LOCKSTEP): no wave groups: per K-tile every wave waits for tile t, ONE barrier,
//      issues tile t+2's three regions, then reads its 20 fragments and runs 32 MFMAs.
//      Measured on the gate|up shape with the kernel's loop in isolation
//      (tools/microbench/ingest.hip, profiles/decode_gemm_ingest_gate_up.jsonl): loads
//      alone 55.1 us, MFMA alone 44.9 us, both 60.6 us -- against 72 us for schedule 0:
//      with 2 waves per SIMD the MFMA of one wave covers the other's fragment reads
//      without the second barrier set of the ping-pong.
template <int XH, int EPI, bool NT, int SCHED = 0>
__global__ void __launch_bounds__(512) gemm_pp_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                      bf16_t* __restrict__ Y, float* __restrict__ P, int M, int N,
                                                      int K) {
  constexpr int NR = XH + 1;               // regions per K-tile
  constexpr int BUF = NR * kRegion;
  constexpr int GL = 2;                    // DMA instructions per wave per region
  __shared__ __attribute__((aligned(1024))) char lds[kNBuf * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, wc = w & 3;
  const int n0 = blockIdx.x * 128;
  const int m0 = blockIdx.z * (128 * XH);
  const int S = gridDim.y, kz = blockIdx.y;
  const int Kc = K / S;
  const int T = Kc / kBK;

  // region r: 0 = X rows 0-127, 1 = W rows 0-127, 2 = X rows 128-255 (XH == 2)
  const int lrow = lane >> 3, lslot = lane & 7;
  // [NR][GL] in fixed size: with a template-dependent array type, passing its
  // elements to the LDS-DMA builtin makes the host pass of hipcc (ROCm 7.2) silently
  // drop the kernel's launch stub (undefined symbol at load time)
  const bf16_t* src[3][2];
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      const int row = 8 * (w + 8 * i) + lrow;
      const int chunk = lslot ^ ((row >> 1) & 7);
      const int64_t koff = (int64_t)kz * Kc + chunk * 8;
      if (r == 1) src[r][i] = W + (int64_t)(n0 + row) * K + koff;
      else src[r][i] = X + (int64_t)min(m0 + (r == 2 ? 128 : 0) + row, M - 1) * K + koff;
    }
  auto issue = [&](int r, int buf, int kt) {
    char* dst = lds + buf * BUF + r * kRegion;
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      if (NT && r == 1)
        __builtin_amdgcn_global_load_lds(src[r][i] + kt * kBK,
                                         (__attribute__((address_space(3))) void*)(dst + (w + 8 * i) * 1024), 16, 0, 2);
      else
        __builtin_amdgcn_global_load_lds(src[r][i] + kt * kBK,
                                         (__attribute__((address_space(3))) void*)(dst + (w + 8 * i) * 1024), 16, 0, 0);
    }
  };

  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int xo0 = (g * 64 + l15) * 128 + ((lq ^ sw) << 4);
  const int xo1 = (g * 64 + l15) * 128 + (((4 + lq) ^ sw) << 4);
  const int wo0 = (wc * 16 + l15) * 128 + ((lq ^ sw) << 4);
  const int wo1 = (wc * 16 + l15) * 128 + (((4 + lq) ^ sw) << 4);

  f32x4 acc[XH][4][2];
#pragma unroll
  for (int h = 0; h < XH; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[h][b][0] = acc[h][b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 xf[4][2], xf2[4][2], wf[2][2];
  auto read_x = [&](const char* reg) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      xf[b][0] = *reinterpret_cast<const u16x8*>(reg + xo0 + b * 2048);
      xf[b][1] = *reinterpret_cast<const u16x8*>(reg + xo1 + b * 2048);
    }
  };
  auto read_x2 = [&](const char* reg) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      xf2[b][0] = *reinterpret_cast<const u16x8*>(reg + xo0 + b * 2048);
      xf2[b][1] = *reinterpret_cast<const u16x8*>(reg + xo1 + b * 2048);
    }
  };
  auto read_w = [&](const char* reg) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      wf[e][0] = *reinterpret_cast<const u16x8*>(reg + wo0 + e * 8192);
      wf[e][1] = *reinterpret_cast<const u16x8*>(reg + wo1 + e * 8192);
    }
  };
  auto mfma_q = [&](f32x4 (&a)[4][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          a[b][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[e][s]),
                                                            __builtin_bit_cast(bf16x8_t, xf[b][s]), a[b][e], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_q2 = [&](f32x4 (&a0)[4][2], f32x4 (&a1)[4][2]) {   // both X halves, one cluster
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          a0[b][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[e][s]),
                                                             __builtin_bit_cast(bf16x8_t, xf[b][s]), a0[b][e], 0, 0, 0);
          a1[b][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[e][s]),
                                                             __builtin_bit_cast(bf16x8_t, xf2[b][s]), a1[b][e], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  constexpr bool ONE = SCHED == 1;
  if constexpr (SCHED == 2) {
    static_assert(XH == 2, "lock-step schedule: 256-token tiles");
#pragma unroll
    for (int r = 0; r < NR; ++r) issue(r, 0, 0);
    if (T > 1) {
#pragma unroll
      for (int r = 0; r < NR; ++r) issue(r, 1, 1);
    }
    for (int t = 0; t < T; ++t) {
      // tile t landed (tile t+1 may stay in flight); every wave's reads of tile t-1 were
      // retired before its MFMAs, so after the barrier buffer (t+2) % 3 is free
      if (t + 1 < T) vmw<GL * NR>(); else vmw<0>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < T) {
#pragma unroll
        for (int r = 0; r < NR; ++r) issue(r, (t + 2) % kNBuf, t + 2);
      }
      const char* cur = lds + (t % kNBuf) * BUF;
      read_x(cur);
      read_w(cur + kRegion);
      read_x2(cur + 2 * kRegion);
      mfma_q2(acc[0], acc[XH - 1]);
    }
  } else {
  // prologue: K-tiles 0 and 1 in flight; tile 0's first phase regions (X0, W) retired
#pragma unroll
  for (int r = 0; r < NR; ++r) issue(r, 0, 0);
  if (T > 1) {
#pragma unroll
    for (int r = 0; r < NR; ++r) issue(r, 1, 1);
    if constexpr (XH == 2 && !ONE) vmw<GL * 4>(); else vmw<GL * NR>();   // leave X1(0) [XH 2] + tile 1 in flight
  } else {
    if constexpr (XH == 2 && !ONE) vmw<GL>(); else vmw<0>();
  }
  seg();
  if (g == 1) seg();   // ping-pong: waves 4-7 one segment behind

  // steady state, per K-tile t (buffer t % 3): phase h issues region(s) of tile t+2
  // into buffer (t+2) % 3 — the buffer tile t-1 used, free since the barrier that
  // ended tile t-1 (every wave had waited for its reads of it).
  // Wait counts (regions in issue order, GL instructions each): before phase 1 of
  // tile t+1 the wave must have X0/W of t+1 — everything but [X1(t+1)], tile t+2.
  for (int t = 0; t < T; ++t) {
    const char* cur = lds + (t % kNBuf) * BUF;
    const int nb = (t + 2) % kNBuf;
    const bool m2 = t + 2 < T;
    const bool m1 = t + 1 < T;
    if constexpr (XH == 2 && !ONE) {
      // phase 1 (X0, W): issue X0 and W of tile t+2
      read_x(cur);
      read_w(cur + kRegion);
      if (m2) { issue(0, nb, t + 2); issue(1, nb, t + 2); }
      // X1(t) must be retired before phase 2 reads it: in flight after it are
      // [tile t+1: 3 regions] and what this phase issued
      if (g == 1) { if (m2) vmw<GL * 5>(); else if (m1) vmw<GL * 3>(); else vmw<0>(); }
      seg();
      mfma_q(acc[0]);
      if (g == 0) { if (m2) vmw<GL * 5>(); else if (m1) vmw<GL * 3>(); else vmw<0>(); }
      seg();
      // phase 2 (X1, W from registers): issue X1 of tile t+2; retire X0/W of tile t+1
      read_x(cur + 2 * kRegion);
      if (m2) issue(2, nb, t + 2);
      if (g == 1) { if (m2) vmw<GL * 4>(); else if (m1) vmw<GL * 1>(); }
      seg();
      mfma_q(acc[1]);
      if (g == 0) { if (m2) vmw<GL * 4>(); else if (m1) vmw<GL * 1>(); }
      seg();
    } else {
      // one phase (X0, W): issue both regions of tile t+2; retire tile t+1 first.
      // Buffer (t+2) % 3 held tile t-1, whose LAST reader is the partner group one
      // segment behind: waves 0-3 may overwrite it only after their MFMA segment
      // (by then waves 4-7 have waited for their reads of tile t-1), waves 4-7 in
      // their read segment already.
      read_x(cur);
      read_w(cur + kRegion);
      if constexpr (XH == 2) read_x2(cur + 2 * kRegion);
      if (m2 && g == 1) {
#pragma unroll
        for (int r = 0; r < NR; ++r) issue(r, nb, t + 2);
      }
      if (g == 1) { if (m2) vmw<GL * NR>(); else vmw<0>(); }
      seg();
      if constexpr (XH == 2) mfma_q2(acc[0], acc[XH - 1]); else mfma_q(acc[0]);
      if (m2 && g == 0) {
#pragma unroll
        for (int r = 0; r < NR; ++r) issue(r, nb, t + 2);
      }
      if (g == 0) { if (m2) vmw<GL * NR>(); else vmw<0>(); }
      seg();
    }
  }
  if (g == 0) seg();
  }

#pragma unroll
  for (int h = 0; h < XH; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int tok = m0 + h * 128 + g * 64 + b * 16 + l15;
      if (tok >= M) continue;
      if constexpr (EPI == kSilu) {
        const int col = (n0 >> 1) + wc * 16 + 4 * lq;
        const f32x4 gt = acc[h][b][0], up = acc[h][b][1];
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gg = bf2f(f2bf(gt[r]));
          const float uu = bf2f(f2bf(up[r]));
          o[r] = bf2f(f2bf(gg / (1.f + __expf(-gg)))) * uu;
        }
        *reinterpret_cast<uint2*>(Y + (int64_t)tok * (N >> 1) + col) = pack4(o);
      } else {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int col = n0 + e * 64 + wc * 16 + 4 * lq;
          if constexpr (EPI == kPartial)
            *reinterpret_cast<f32x4*>(P + ((int64_t)kz * M + tok) * N + col) = acc[h][b][e];
          else
            *reinterpret_cast<uint2*>(Y + (int64_t)tok * N + col) = pack4(acc[h][b][e]);
        }
      }
    }
}

// Wave-specialised loaders (sched 3..5): the same 256-token x 128-feature tile, fragments,
// MFMAs and epilogues as the lock-step schedule, but the two operand streams are issued by
// different waves: waves 0-3 stream the weight rows (HBM, ~1.3 us under load) through an
// NW-deep ring (NW-1 K-tiles issued ahead), waves 4-7 the activation rows (L2-resident)
// through an NX-deep ring. s_waitcnt vmcnt is in issue order per wave, so with both
// streams in one wave (sched 2) every wait for the next X tile also waits for the weight
// tiles issued before it, and the weight prefetch can never run deeper than X's; split
// over waves, each stream is waited for on its own. Measured in isolation
// (tools/microbench/ingest.hip, gate|up shape): loads of both operands from one wave
// 55.1 us against 41.3 us for the weights alone and 17.7 us for X alone.
template <int EPI, int NW, int NX>
__global__ void __launch_bounds__(512) gemm_ws_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                      bf16_t* __restrict__ Y, float* __restrict__ P, int M, int N,
                                                      int K) {
  constexpr int WBUF = kRegion, XBUF = 2 * kRegion;
  static_assert(NW * WBUF + NX * XBUF <= 163840, "LDS");
  __shared__ __attribute__((aligned(1024))) char lds[NW * WBUF + NX * XBUF];
  char* wl = lds;
  char* xl = lds + NW * WBUF;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool wwave = w < 4;
  const int wi = w & 3;
  const int g = w >> 2, wc = w & 3;
  const int n0 = blockIdx.x * 128;
  const int m0 = blockIdx.z * 256;
  const int S = gridDim.y, kz = blockIdx.y;
  const int Kc = K / S;
  const int T = Kc / kBK;
  const int lrow = lane >> 3, lslot = lane & 7;
  // piece q (0..3) of a 128-row region for loader wave wi: rows 8 (wi + 4 q) + lrow
  const bf16_t* src[2][4];   // W: src[0][q]; X: src[r][q] for region r
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = 8 * (wi + 4 * q) + lrow;
    const int64_t koff = (int64_t)kz * Kc + (lslot ^ ((row >> 1) & 7)) * 8;
    if (wwave) {
      src[0][q] = W + (int64_t)(n0 + row) * K + koff;
      src[1][q] = src[0][q];
    } else {
#pragma unroll
      for (int r = 0; r < 2; ++r) src[r][q] = X + (int64_t)min(m0 + r * 128 + row, M - 1) * K + koff;
    }
  }
  auto issue_w = [&](int kt) {
    char* dst = wl + (kt % NW) * WBUF;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(src[0][q] + kt * kBK,
                                       (__attribute__((address_space(3))) void*)(dst + (wi + 4 * q) * 1024), 16, 0, 2);
  };
  auto issue_x = [&](int kt) {
    char* dst = xl + (kt % NX) * XBUF;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds(src[r][q] + kt * kBK,
                                         (__attribute__((address_space(3))) void*)(dst + r * kRegion + (wi + 4 * q) * 1024),
                                         16, 0, 0);
  };
  auto wait_n = [&](int n) {   // n outstanding pieces of this wave's stream (compile-time cases)
    switch (n) {
      case 0: vmw<0>(); break;
      case 4: vmw<4>(); break;
      case 8: vmw<8>(); break;
      case 12: vmw<12>(); break;
      case 16: vmw<16>(); break;
      case 20: vmw<20>(); break;
      default: vmw<0>(); break;
    }
  };

  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int xo0 = (g * 64 + l15) * 128 + ((lq ^ sw) << 4);
  const int xo1 = (g * 64 + l15) * 128 + (((4 + lq) ^ sw) << 4);
  const int wo0 = (wc * 16 + l15) * 128 + ((lq ^ sw) << 4);
  const int wo1 = (wc * 16 + l15) * 128 + (((4 + lq) ^ sw) << 4);
  f32x4 acc[2][4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[h][b][0] = acc[h][b][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (wwave) {
    for (int p = 0; p < NW - 1 && p < T; ++p) issue_w(p);
  } else {
    for (int p = 0; p < NX - 1 && p < T; ++p) issue_x(p);
  }
  for (int t = 0; t < T; ++t) {
    // this wave's stream: tile t landed, the later ones stay in flight
    if (wwave) wait_n(4 * min(NW - 2, T - 1 - t));
    else wait_n(8 * min(NX - 2, T - 1 - t));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // slot (t - 1) of each ring was read (and its reads retired) before this barrier
    if (wwave) {
      if (t + NW - 1 < T) issue_w(t + NW - 1);
    } else {
      if (t + NX - 1 < T) issue_x(t + NX - 1);
    }
    const char* xc = xl + (t % NX) * XBUF;
    const char* wcur = wl + (t % NW) * WBUF;
    u16x8 xf[2][4][2], wf[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        xf[h][b][0] = *reinterpret_cast<const u16x8*>(xc + h * kRegion + xo0 + b * 2048);
        xf[h][b][1] = *reinterpret_cast<const u16x8*>(xc + h * kRegion + xo1 + b * 2048);
      }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      wf[e][0] = *reinterpret_cast<const u16x8*>(wcur + wo0 + e * 8192);
      wf[e][1] = *reinterpret_cast<const u16x8*>(wcur + wo1 + e * 8192);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int e = 0; e < 2; ++e)
            acc[h][b][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[e][s]),
                                                                   __builtin_bit_cast(bf16x8_t, xf[h][b][s]),
                                                                   acc[h][b][e], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }

#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int tok = m0 + h * 128 + g * 64 + b * 16 + l15;
      if (tok >= M) continue;
      if constexpr (EPI == kSilu) {
        const int col = (n0 >> 1) + wc * 16 + 4 * lq;
        const f32x4 gt = acc[h][b][0], up = acc[h][b][1];
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gg = bf2f(f2bf(gt[r]));
          const float uu = bf2f(f2bf(up[r]));
          o[r] = bf2f(f2bf(gg / (1.f + __expf(-gg)))) * uu;
        }
        *reinterpret_cast<uint2*>(Y + (int64_t)tok * (N >> 1) + col) = pack4(o);
      } else {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int col = n0 + e * 64 + wc * 16 + 4 * lq;
          if constexpr (EPI == kPartial)
            *reinterpret_cast<f32x4*>(P + ((int64_t)kz * M + tok) * N + col) = acc[h][b][e];
          else
            *reinterpret_cast<uint2*>(Y + (int64_t)tok * N + col) = pack4(acc[h][b][e]);
        }
      }
    }
}

// gemm_ws with the fragment reads software-pipelined (sched 6, 7): the 20 fragments of K-tile
// t+1 are read from LDS while the 32 MFMAs of tile t run from registers (X fragments refilled
// in place right after the two MFMAs that use them, W fragments double-buffered with the loop
// unrolled by two so both sets are named statically). With reads and MFMAs in separate
// phases (gemm_ws) the two waves of a SIMD both read after every barrier and then both
// compute; here the matrix pipe starts right after the barrier. Each ring slot is refilled
// one K-tile earlier than in gemm_ws (its tile is in registers by then), so the prefetch
// distance in K-tiles is unchanged.
// SPEC = false: every wave issues its share of all three regions (the lock-step loaders,
// one 48 KiB ring of NW K-tiles laid out [X0][W][X1] as gemm_pp); true: gemm_ws's split
// loaders (W ring NW deep, X ring NX deep).
template <int EPI, int NW, int NX, bool SPEC = true>
__global__ void __launch_bounds__(512) gemm_wsp_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                       bf16_t* __restrict__ Y, float* __restrict__ P, int M, int N,
                                                       int K) {
  constexpr int WBUF = kRegion, XBUF = 2 * kRegion;
  constexpr int LDSB = SPEC ? NW * WBUF + NX * XBUF : NW * 3 * kRegion;
  static_assert(LDSB <= 163840, "LDS");
  static_assert(NW >= 3 && (NX >= 2 || !SPEC), "ring depths");
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];
  char* wl = lds;
  char* xl = lds + NW * WBUF;
  // slot bases: W region and the two X regions of K-tile kt
  auto wslot = [&](int kt) -> char* { return SPEC ? wl + (kt % NW) * WBUF : lds + (kt % NW) * 3 * kRegion + kRegion; };
  auto xslot = [&](int kt, int h) -> char* {
    return SPEC ? xl + (kt % NX) * XBUF + h * kRegion : lds + (kt % NW) * 3 * kRegion + h * 2 * kRegion;
  };
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool wwave = w < 4;
  const int wi = w & 3;
  const int g = w >> 2, wc = w & 3;
  const int n0 = blockIdx.x * 128;
  const int m0 = blockIdx.z * 256;
  const int S = gridDim.y, kz = blockIdx.y;
  const int Kc = K / S;
  const int T = Kc / kBK;
  const int lrow = lane >> 3, lslot = lane & 7;
  // SPEC: piece q (0..3) of a 128-row region for loader wave wi = rows 8 (wi + 4 q) + lrow;
  // !SPEC: pieces i = 0, 1 of each region for wave w = rows 8 (w + 8 i) + lrow (src[region][i])
  const bf16_t* src[3][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = SPEC ? 8 * (wi + 4 * q) + lrow : 8 * (w + 8 * (q & 1)) + lrow;
    const int64_t koff = (int64_t)kz * Kc + (lslot ^ ((row >> 1) & 7)) * 8;
    if (!SPEC) {
      src[0][q] = X + (int64_t)min(m0 + row, M - 1) * K + koff;
      src[1][q] = W + (int64_t)(n0 + row) * K + koff;
      src[2][q] = X + (int64_t)min(m0 + 128 + row, M - 1) * K + koff;
    } else if (wwave) {
      src[0][q] = W + (int64_t)(n0 + row) * K + koff;
      src[1][q] = src[2][q] = src[0][q];
    } else {
#pragma unroll
      for (int r = 0; r < 2; ++r) src[r][q] = X + (int64_t)min(m0 + r * 128 + row, M - 1) * K + koff;
      src[2][q] = src[1][q];
    }
  }
  auto issue_w = [&](int kt) {
    char* dst = wslot(kt);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(src[0][q] + kt * kBK,
                                       (__attribute__((address_space(3))) void*)(dst + (wi + 4 * q) * 1024), 16, 0, 2);
  };
  auto issue_x = [&](int kt) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      char* dst = xslot(kt, r);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds(src[r][q] + kt * kBK,
                                         (__attribute__((address_space(3))) void*)(dst + (wi + 4 * q) * 1024), 16, 0, 0);
    }
  };
  auto issue_all = [&](int kt) {   // !SPEC: X0, W, X1 pieces of this wave, the gemm_pp order
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      char* dst = r == 1 ? wslot(kt) : xslot(kt, r >> 1);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (r == 1)
          __builtin_amdgcn_global_load_lds(src[1][i] + kt * kBK,
                                           (__attribute__((address_space(3))) void*)(dst + (w + 8 * i) * 1024), 16, 0, 2);
        else
          __builtin_amdgcn_global_load_lds(src[r][i] + kt * kBK,
                                           (__attribute__((address_space(3))) void*)(dst + (w + 8 * i) * 1024), 16, 0, 0);
      }
    }
  };
  auto wait_n = [&](int n) {
    switch (n) {
      case 0: vmw<0>(); break;
      case 4: vmw<4>(); break;
      case 8: vmw<8>(); break;
      case 12: vmw<12>(); break;
      case 16: vmw<16>(); break;
      case 20: vmw<20>(); break;
      case 6: vmw<6>(); break;
      default: vmw<0>(); break;
    }
  };
  // this wave's stream: every tile up to `kt` landed (tiles issued so far: < issued)
  auto wait_tile = [&](int kt, int issued_w, int issued_x) {
    if (!SPEC) wait_n(6 * max(0, min(issued_w, T) - 1 - kt));
    else if (wwave) wait_n(4 * max(0, min(issued_w, T) - 1 - kt));
    else wait_n(8 * max(0, min(issued_x, T) - 1 - kt));
  };

  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int xo0 = (g * 64 + l15) * 128 + ((lq ^ sw) << 4);
  const int xo1 = (g * 64 + l15) * 128 + (((4 + lq) ^ sw) << 4);
  const int wo0 = (wc * 16 + l15) * 128 + ((lq ^ sw) << 4);
  const int wo1 = (wc * 16 + l15) * 128 + (((4 + lq) ^ sw) << 4);
  f32x4 acc[2][4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[h][b][0] = acc[h][b][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments: X single-buffered and refilled in place (x[h][b][s] of tile t+1 is read as soon
  // as the two MFMAs of tile t that use it have issued), W double-buffered (every MFMA of a
  // tile uses one of its four W fragments)
  u16x8 xf[2][4][2], wa[2][2], wb[2][2];
  auto xaddr = [&](int kt, int h, int b, int s2) { return xslot(kt, h) + (s2 ? xo1 : xo0) + b * 2048; };
  auto read_w = [&](int kt, u16x8 (&wf)[2][2]) {
    const char* wcur = wslot(kt);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      wf[e][0] = *reinterpret_cast<const u16x8*>(wcur + wo0 + e * 8192);
      wf[e][1] = *reinterpret_cast<const u16x8*>(wcur + wo1 + e * 8192);
    }
  };
  // one K-tile: MFMAs from (xf, wc), the next tile's fragments read into (xf, wn) in between
  auto step = [&](int kt, u16x8 (&wc_)[2][2], u16x8 (&wn)[2][2]) {
    // tile kt + 1 landed (every wave); the slot of tile kt (in registers) is free
    if (kt + 1 < T) wait_tile(kt + 1, kt + NW, kt + NX);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (!SPEC) {
      if (kt + NW < T) issue_all(kt + NW);
    } else if (wwave) {
      if (kt + NW < T) issue_w(kt + NW);
    } else {
      if (kt + NX < T) issue_x(kt + NX);
    }
    // the next tile's reads are unconditional (the last step re-reads its own tile): a
    // runtime guard per read makes hipcc branch around each one
    const int kn = min(kt + 1, T - 1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
#pragma unroll
          for (int e = 0; e < 2; ++e)
            acc[h][b][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wc_[e][s2]),
                                                                   __builtin_bit_cast(bf16x8_t, xf[h][b][s2]),
                                                                   acc[h][b][e], 0, 0, 0);
          xf[h][b][s2] = *reinterpret_cast<const u16x8*>(xaddr(kn, h, b, s2));
        }
      // W of the next tile half-way: the first MFMAs of a step wait only for older reads
      if (s2 == 0) read_w(kn, wn);
    }
    // pin the interleave (hipcc otherwise runs 16 MFMAs, then bunches the reads): MFMA / DS_READ
    // groups in program order -- 8 x (2, 1) for the first k-substep's X refills, then the 4 W
    // reads one per MFMA, then the second substep's 8 X refills behind their MFMA pairs
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  if (!SPEC) {
    for (int p = 0; p < NW && p < T; ++p) issue_all(p);
  } else if (wwave) {
    for (int p = 0; p < NW && p < T; ++p) issue_w(p);
  } else {
    for (int p = 0; p < NX && p < T; ++p) issue_x(p);
  }
  wait_tile(0, NW, NX);
  __builtin_amdgcn_s_barrier();
  read_w(0, wa);
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) xf[h][b][s2] = *reinterpret_cast<const u16x8*>(xaddr(0, h, b, s2));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  int t = 0;
  for (; t + 1 < T; t += 2) {
    step(t, wa, wb);
    step(t + 1, wb, wa);
  }
  if (t < T) step(t, wa, wb);

#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int tok = m0 + h * 128 + g * 64 + b * 16 + l15;
      if (tok >= M) continue;
      if constexpr (EPI == kSilu) {
        const int col = (n0 >> 1) + wc * 16 + 4 * lq;
        const f32x4 gt = acc[h][b][0], up = acc[h][b][1];
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gg = bf2f(f2bf(gt[r]));
          const float uu = bf2f(f2bf(up[r]));
          o[r] = bf2f(f2bf(gg / (1.f + __expf(-gg)))) * uu;
        }
        *reinterpret_cast<uint2*>(Y + (int64_t)tok * (N >> 1) + col) = pack4(o);
      } else {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int col = n0 + e * 64 + wc * 16 + 4 * lq;
          if constexpr (EPI == kPartial)
            *reinterpret_cast<f32x4*>(P + ((int64_t)kz * M + tok) * N + col) = acc[h][b][e];
          else
            *reinterpret_cast<uint2*>(Y + (int64_t)tok * N + col) = pack4(acc[h][b][e]);
        }
      }
    }
}

int gemm_pp(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, int bm, bool silu_gu,
            bool nt, hipStream_t stream, int sched) {
  if (M < 1 || N % 128 != 0 || S < 1 || S > 32 || K % (kBK * S) != 0) return -1;
  if (bm != 128 && bm != 256) return -2;
  if (sched < 0 || sched > 8 || (sched > 0 && bm != 256)) return -6;
  if (silu_gu && S != 1) return -3;
  if (S > 1 && P == nullptr) return -4;
  if (S == 1 && Y == nullptr) return -5;
  const dim3 grid(N / 128, S, (M + bm - 1) / bm);
  const int epi = silu_gu ? kSilu : (S > 1 ? kPartial : kStore);
#define OAMD_PP(XH, E, NTB) gemm_pp_kernel<XH, E, NTB><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K)
#define OAMD_PP_E(XH, NTB)                  \
  if (epi == kSilu) OAMD_PP(XH, kSilu, NTB); \
  else if (epi == kPartial) OAMD_PP(XH, kPartial, NTB); \
  else OAMD_PP(XH, kStore, NTB)
#define OAMD_PP1(E, SC) gemm_pp_kernel<2, E, true, SC><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K)
  if (sched == 1) {   // one barrier segment per K-tile (nt weights)
    if (epi == kSilu) OAMD_PP1(kSilu, 1);
    else if (epi == kPartial) OAMD_PP1(kPartial, 1);
    else OAMD_PP1(kStore, 1);
  } else if (sched >= 6) {   // pipelined fragment reads: split loaders (4, 2), (4, 3); 8: lock-step loaders
#define OAMD_WSP(E)                                                                                \
  if (sched == 6) gemm_wsp_kernel<E, 4, 2><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K);         \
  else if (sched == 7) gemm_wsp_kernel<E, 4, 3><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K);    \
  else gemm_wsp_kernel<E, 3, 3, false><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K);
    if (epi == kSilu) { OAMD_WSP(kSilu) }
    else if (epi == kPartial) { OAMD_WSP(kPartial) }
    else { OAMD_WSP(kStore) }
#undef OAMD_WSP
  } else if (sched >= 3) {   // wave-specialised loaders: (W ring, X ring) = (4, 2), (6, 2), (4, 3)
#define OAMD_WS(E)                                                                                 \
  if (sched == 3) gemm_ws_kernel<E, 4, 2><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K);          \
  else if (sched == 4) gemm_ws_kernel<E, 6, 2><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K);     \
  else gemm_ws_kernel<E, 4, 3><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K);
    if (epi == kSilu) { OAMD_WS(kSilu) }
    else if (epi == kPartial) { OAMD_WS(kPartial) }
    else { OAMD_WS(kStore) }
#undef OAMD_WS
  } else if (sched == 2) {   // lock-step (nt weights)
    if (epi == kSilu) OAMD_PP1(kSilu, 2);
    else if (epi == kPartial) OAMD_PP1(kPartial, 2);
    else OAMD_PP1(kStore, 2);
  } else if (bm == 256) {
    if (nt) { OAMD_PP_E(2, true); } else { OAMD_PP_E(2, false); }
  } else {
    if (nt) { OAMD_PP_E(1, true); } else { OAMD_PP_E(1, false); }
  }
#undef OAMD_PP1
#undef OAMD_PP_E
#undef OAMD_PP
  OAMD_LAUNCH_CHECK();
  if (S > 1 && Y != nullptr) return splitk_reduce(P, Y, (int64_t)M * N, S, stream);
  return 0;
}

}  // namespace oamd
