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
//
// SK (stream-K, 256-row tiles, one K slice; an A/B arm, not the default): the 224 column
// tiles of the 8B gate|up projection leave 32 of 256 CUs idle, so grid = one block per CU,
// each running 7/8 of a tile's K-steps with ONE continuous LDS-DMA stream across its tile
// boundary; a cut tile's first block stores an fp32 partial that its second block adds before
// the epilogue. Measured SLOWER than the per-tile launch (profiles/gemm_pp_stream_k_r6.jsonl):
// even with the hand-off removed, 256 blocks x 7/8 of a tile take 75 us against 73 for 224
// blocks x 1 tile, so the M = 256 GEMM is not bound per CU; the hand-off adds 12 us more.
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
// ONE (XH == 2): the K-tile in ONE barrier segment per wave group (both X halves' 32
// MFMAs behind one pair of barriers, all three regions of tile t+2 issued together) —
// the XH == 1 schedule with a second X fragment set, half the barriers of two phases.
template <int XH, int EPI, bool NT, bool ONE = false, bool SK = false>
__global__ void __launch_bounds__(512) gemm_pp_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                      bf16_t* __restrict__ Y, float* __restrict__ P, int M, int N,
                                                      int K, float* __restrict__ ws, int* __restrict__ flags) {
  constexpr int NR = XH + 1;               // regions per K-tile
  constexpr int BUF = NR * kRegion;
  constexpr int GL = 2;                    // DMA instructions per wave per region
  static_assert(!SK || (XH == 2 && !ONE), "stream-K runs the two-phase 256-row schedule");
  __shared__ __attribute__((aligned(1024))) char lds[kNBuf * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, wc = w & 3;
  const int m0 = SK ? 0 : blockIdx.z * (128 * XH);
  const int S = SK ? 1 : gridDim.y, kz = SK ? 0 : blockIdx.y;
  const int Kc = K / S;
  const int TT = Kc / kBK;                 // K-steps per tile
  // SK: logical block lb (XCD-grouped: the blocks one XCD runs -- block ids = x mod 8 -- hold
  // consecutive ranges, so both blocks of a cut tile normally share an L2) owns the K-steps
  // [F0, F0 + T) of the flattened (tile, k) stream. It runs them as segment A = the piece of
  // the LAST tile it touches (from k = 0), then segment B = the piece of the first one (to the
  // tile's end): at local step j every block reads K-step j or j + TT - T, so all blocks walk X
  // in step and its panel stays in L2 (tile-major order scattered them over 8 phases, 85 vs
  // 73 us with no hand-off at all).
  int T = TT, tA = 0, kA = 0, nA = TT, tB = 0, kB = 0;
  if constexpr (SK) {
    const int G = gridDim.x;
    const int lb = (G % 8 == 0) ? (int)(blockIdx.x % 8) * (G / 8) + (int)blockIdx.x / 8 : (int)blockIdx.x;
    const int64_t Ft = (int64_t)(N / 128) * TT;
    const int F0 = (int)((int64_t)lb * Ft / G), F1 = (int)((int64_t)(lb + 1) * Ft / G);
    T = F1 - F0;
    const int tf = F0 / TT, tl = (F1 - 1) / TT;   // host: at most two tiles, never strictly inside one
    if (tf == tl) {
      tA = tf; kA = F0 - tf * TT; nA = T;
    } else {
      tA = tl; kA = 0; nA = F1 - tl * TT; tB = tf; kB = F0 - tf * TT;
    }
  }
  const int n0 = SK ? 0 : blockIdx.x * 128;   // SK: per K-step (tile * 128 rows of W)

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
  // element offset of local K-step j in region r's source (SK: segment A, then B)
  auto step_off = [&](int r, int j) -> int64_t {
    if constexpr (SK) {
      const bool a = j < nA;
      const int tile = a ? tA : tB, k = a ? kA + j : kB + j - nA;
      return (int64_t)k * kBK + (r == 1 ? (int64_t)tile * 128 * K : 0);
    } else {
      return (int64_t)j * kBK;
    }
  };
  auto issue = [&](int r, int buf, int kt) {
    char* dst = lds + buf * BUF + r * kRegion;
    const int64_t off = step_off(r, kt);
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      if (NT && r == 1)
        __builtin_amdgcn_global_load_lds(src[r][i] + off,
                                         (__attribute__((address_space(3))) void*)(dst + (w + 8 * i) * 1024), 16, 0, 2);
      else
        __builtin_amdgcn_global_load_lds(src[r][i] + off,
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

  // bf16 / SwiGLU / slab stores of the accumulators for the tile at column n0t
  auto epilogue = [&](int n0t) {
#pragma unroll
    for (int h = 0; h < XH; ++h)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int tok = m0 + h * 128 + g * 64 + b * 16 + l15;
        if (tok >= M) continue;
        if constexpr (EPI == kSilu) {
          const int col = (n0t >> 1) + wc * 16 + 4 * lq;
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
            const int col = n0t + e * 64 + wc * 16 + 4 * lq;
            if constexpr (EPI == kPartial)
              *reinterpret_cast<f32x4*>(P + ((int64_t)kz * M + tok) * N + col) = acc[h][b][e];
            else
              *reinterpret_cast<uint2*>(Y + (int64_t)tok * N + col) = pack4(acc[h][b][e]);
          }
        }
      }
  };
  // SK partial of a cut tile: slot (h, b, e) of thread tid, lane-linear (both blocks of the
  // tile map threads to accumulators identically)
  auto ws_at = [&](int tile, int h, int b, int e) {
    return reinterpret_cast<f32x4*>(ws) + ((int64_t)tile * (XH * 8) + (h * 4 + b) * 2 + e) * 512 + tid;
  };
  auto zero_acc = [&]() {
#pragma unroll
    for (int h = 0; h < XH; ++h)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[h][b][0] = acc[h][b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  int part_tile = -1, fin_tile = -1;   // SK: the cut tile this block starts (partial) / ends (finishes)
  // SK, after local K-step t (every wave has run its MFMAs of it; no barrier in here)
  auto seg_end = [&](int t) {
    if constexpr (SK) {
      int tile, k0, n;
      if (t == nA - 1) { tile = tA; k0 = kA; n = nA; }
      else if (t == T - 1) { tile = tB; k0 = kB; n = T - nA; }
      else return;
      if (k0 == 0 && n == TT) {
        epilogue(tile * 128);
        zero_acc();
      } else if (k0 == 0) {   // the tile's start: its partial, for the block running its end (lb + 1)
#pragma unroll
        for (int h = 0; h < XH; ++h)
#pragma unroll
          for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int e = 0; e < 2; ++e) *ws_at(tile, h, b, e) = acc[h][b][e];
        zero_acc();
        part_tile = tile;
      } else {
        fin_tile = tile;   // the tile's end = the block's last K-step: finished after the stream
      }
    }
  };

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
      seg_end(t);
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

  if constexpr (SK) {
    // Hand-off: every wave's partial stores have reached L2 at its vmcnt(0); after the barrier one
    // thread writes the XCD's L2 back (agent-scope fence: the reader may sit on another XCD) and
    // raises the flag with the writer's XCC id. The reader invalidates its own L2 only when that
    // id differs from its own (never, with the XCD-grouped order): an invalidate per block under
    // the blocks still streaming cost them their X panel (profiles/gemm_pp_stream_k_r6.jsonl).
    const int xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15;   // HW_REG_XCC_ID
    if (part_tile >= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (part_tile >= 0 && tid == 0) {
      __threadfence();
      __hip_atomic_store(flags + part_tile, 1 + xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (fin_tile >= 0) {
      if (tid == 0) {
        // bounded: the block holding the tile's start raises the flag right after its last
        // K-step, before it waits for anything
        int n = 0, f = 0;
        while ((f = __hip_atomic_load(flags + fin_tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0 && ++n < (1 << 22))
          __builtin_amdgcn_s_sleep(2);
        if (f != 1 + xcc) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      __syncthreads();
      f32x4 pt[XH][4][2];
#pragma unroll
      for (int h = 0; h < XH; ++h)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int e = 0; e < 2; ++e) pt[h][b][e] = __builtin_nontemporal_load(ws_at(fin_tile, h, b, e));
#pragma unroll
      for (int h = 0; h < XH; ++h)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int e = 0; e < 2; ++e) acc[h][b][e] += pt[h][b][e];
      epilogue(fin_tile * 128);
      if (tid == 0) __hip_atomic_store(flags + fin_tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {
    epilogue(n0);
  }
}

static int pp_device_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// Stream-K grid for `tiles` column tiles of `steps` K-steps: one block per CU when that is
// more blocks than tiles, every block at least 2 K-steps, and no block strictly inside one
// tile (a tile is cut at most once, so it has at most one partial); else 0 (plain launch)
int gemm_pp_sk_grid(int tiles, int steps) {
  const int64_t Ft = (int64_t)tiles * steps;
  const int G = pp_device_cus();
  if (G <= tiles || Ft < 2LL * G) return 0;
  for (int b = 0; b < G; ++b) {
    const int64_t f0 = (int64_t)b * Ft / G, f1 = (int64_t)(b + 1) * Ft / G;
    if (f0 % steps != 0 && f1 < (f0 / steps + 1) * steps) return 0;   // strictly inside a tile
    if ((f1 - 1) / steps > f0 / steps + 1) return 0;                    // three tiles
  }
  return G;
}

int gemm_pp(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* P, int M, int N, int K, int S, int bm, bool silu_gu,
            bool nt, hipStream_t stream, bool one_seg, float* ws, int* flags) {
  if (M < 1 || N % 128 != 0 || S < 1 || S > 32 || K % (kBK * S) != 0) return -1;
  if (bm != 128 && bm != 256) return -2;
  if (silu_gu && S != 1) return -3;
  if (S > 1 && P == nullptr) return -4;
  if (S == 1 && Y == nullptr) return -5;
  const dim3 grid(N / 128, S, (M + bm - 1) / bm);
  const int epi = silu_gu ? kSilu : (S > 1 ? kPartial : kStore);
  // stream-K: 256-row tile (M <= 256), one K slice, workspace ((N / 128) x 128 KiB fp32) and
  // zeroed flags (N / 128 ints; the kernel leaves them zero) given
  const int skg = (ws != nullptr && flags != nullptr && bm == 256 && M <= 256 && S == 1 && !one_seg && nt)
                      ? gemm_pp_sk_grid(N / 128, K / kBK) : 0;
  if (skg > 0) {
    if (epi == kSilu)
      gemm_pp_kernel<2, kSilu, true, false, true><<<skg, 512, 0, stream>>>(X, W, Y, P, M, N, K, ws, flags);
    else
      gemm_pp_kernel<2, kStore, true, false, true><<<skg, 512, 0, stream>>>(X, W, Y, P, M, N, K, ws, flags);
    OAMD_LAUNCH_CHECK();
    return 0;
  }
#define OAMD_PP(XH, E, NTB) gemm_pp_kernel<XH, E, NTB><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K, nullptr, nullptr)
#define OAMD_PP_E(XH, NTB)                  \
  if (epi == kSilu) OAMD_PP(XH, kSilu, NTB); \
  else if (epi == kPartial) OAMD_PP(XH, kPartial, NTB); \
  else OAMD_PP(XH, kStore, NTB)
#define OAMD_PP1(E) gemm_pp_kernel<2, E, true, true><<<grid, 512, 0, stream>>>(X, W, Y, P, M, N, K, nullptr, nullptr)
  if (bm == 256 && one_seg) {   // one barrier segment per K-tile (nt weights)
    if (epi == kSilu) OAMD_PP1(kSilu);
    else if (epi == kPartial) OAMD_PP1(kPartial);
    else OAMD_PP1(kStore);
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
