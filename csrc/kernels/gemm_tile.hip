// Compute-bound GEMM for prefill projections and the lm_head:
//   Y[M, N] = X[M, K] . W[N, K]^T     bf16 in, fp32 accumulate, bf16 out
// (SURVEY.md §2.4 N7 "prefill is compute-bound tiles (256² 8-phase template)";
// replaces the external LLM behind J/service/AIInterfaceRestClient.java:37-39).
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template", T1-T5):
//   * one 256 x 256 output tile per 512-thread workgroup (8 waves, 2 per SIMD),
//     BK = 64, both operands staged global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4) into two 64 KiB buffers; every tile is split
//     into four 16 KiB regions (X rows 0-127, W rows 0-127, W rows 128-255,
//     X rows 128-255) that are loaded, waited for and recycled one at a time;
//   * the K-tile is computed in four phases, one per (X half, W half) quadrant,
//     16 MFMA v_mfma_f32_16x16x32_bf16 per wave each; a phase issues one region
//     of the NEXT K-tile, so 1.5 tiles stay in flight with only 2 buffers and
//     the LDS-DMA never drains inside the loop (counted vmcnt, raw s_barrier);
//   * ping-pong: waves 4-7 run one barrier segment behind waves 0-3, so on
//     every SIMD one wave issues its LDS fragment reads + DMA while the other
//     runs its MFMA cluster (s_setprio 1 around it, T5);
//   * the LDS image is lane-linear (DMA) with the st_16x32-style XOR swizzle
//     applied to the global SOURCE chunk and the read address (rule 21):
//     slot = chunk ^ ((row >> 1) & 7), conflict-free for ds_read_b128;
//   * operands swapped in the MFMA (A = W fragment, B = X fragment) so each
//     lane's accumulator holds 4 consecutive OUTPUT FEATURES of one token:
//     8-byte stores, and a fused SwiGLU epilogue in registers when the gate|up
//     weight is interleaved in 64-row blocks (wave wc owns gate rows
//     wc*16..+16 and the matching up rows 64 + wc*16..+16 of every 128 rows);
//   * XCD-aware, grouped tile order (T1 bijective remap, then GROUP_M m-tiles
//     per n-tile) so the 32 tiles an XCD runs at once share X/W panels in L2.
// M and N tails are handled by clamped loads and masked stores; K % 64 == 0.
#include "common.h"
#include "kernels.h"

namespace oamd {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kT = 256;          // tile rows / cols
constexpr int kBK = 64;          // K per tile step (one 128-B line per row)
constexpr int kRegion = 16384;   // 128 rows x 128 B
constexpr int kBuf = 4 * kRegion;
constexpr int kGroupM = 8;

enum { kEpiStore = 0, kEpiBias = 1, kEpiSilu = 2, kEpiPartial = 3 };   // partial: fp32 split-K slab

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void seg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ uint2 pack4(f32x4 v) {
  return make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
}

}  // namespace

// PH2: the K-tile in TWO barrier segments per wave group instead of four — segment A
// computes quadrants (X0, W0) and (X0, W1) (32 MFMAs) and issues X0 / W0 / W1 of the next
// K-tile (all three were last read in segment A of the previous tile), segment B computes
// (X1, W0) and (X1, W1) from the W fragments still in registers and issues X1. Half the
// barriers per K-tile; every region still has a whole K-tile of DMA flight.
template <int EPI, bool PH2 = false>
__global__ void __launch_bounds__(512) gemm_tile256_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ W,
                                                           bf16_t* __restrict__ Y, const bf16_t* __restrict__ bias,
                                                           int M, int N, int K, int ldy, float* __restrict__ P) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 2, wc = w & 3;

  // ---- tile order: XCD-contiguous chunks, GROUP_M-row groups inside them
  const int mt = (M + kT - 1) / kT, nt = (N + kT - 1) / kT;
  const int nwg = mt * nt;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int gsz = kGroupM * nt;
  const int first_m = (lid / gsz) * kGroupM;
  const int gm = min(mt - first_m, kGroupM);
  const int tm = first_m + (lid % gsz) % gm;
  const int tn = (lid % gsz) / gm;
  const int m0 = tm * kT, n0 = tn * kT;

  // ---- LDS-DMA sources: region r (issue order 0 = X rows 0-127, 1 = W rows 0-127,
  // 2 = W rows 128-255, 3 = X rows 128-255); wave w issues instructions q = w, w + 8
  // of each region, lane l -> region row 8q + l/8, LDS slot l%8, global chunk swz
  const int lrow = lane >> 3, lslot = lane & 7;
  const bf16_t* src[4][2];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 8 * (w + 8 * i) + lrow;
      const int chunk = lslot ^ ((row >> 1) & 7);
      const bool isx = (r == 0 || r == 3);
      const int half = (r == 2 || r == 3) ? 128 : 0;
      const int64_t grow = isx ? min(m0 + half + row, M - 1) : min(n0 + half + row, N - 1);
      src[r][i] = (isx ? X : W) + grow * K + chunk * 8 + (int64_t)blockIdx.y * (K / gridDim.y);
    }
  auto issue = [&](int r, int buf, int kt) {
    char* dst = lds + buf * kBuf + r * kRegion;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds(src[r][i] + kt * kBK, (__attribute__((address_space(3))) void*)(dst + (w + 8 * i) * 1024),
                                       16, 0, 0);
  };

  // ---- fragment read offsets (bytes within a region); row & 15 == lane & 15 for
  // every fragment, so the swizzle term depends on the lane only
  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int xo0 = (g * 64 + l15) * 128 + ((lq ^ sw) << 4);         // k-substep 0
  const int xo1 = (g * 64 + l15) * 128 + (((4 + lq) ^ sw) << 4);   // k-substep 1
  const int wo0 = (wc * 16 + l15) * 128 + ((lq ^ sw) << 4);
  const int wo1 = (wc * 16 + l15) * 128 + (((4 + lq) ^ sw) << 4);

  f32x4 acc[2][2][4][2];   // [X half][W half][token block][feature block (gate, up)]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int e = 0; e < 2; ++e) acc[h][f][b][e] = f32x4{0.f, 0.f, 0.f, 0.f};

  u16x8 xf[4][2], wf0[2][2], wf1[2][2];
  auto read_x = [&](const char* reg) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      xf[b][0] = *reinterpret_cast<const u16x8*>(reg + xo0 + b * 2048);
      xf[b][1] = *reinterpret_cast<const u16x8*>(reg + xo1 + b * 2048);
    }
  };
  auto read_w = [&](const char* reg, u16x8 (&wf)[2][2]) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      wf[e][0] = *reinterpret_cast<const u16x8*>(reg + wo0 + e * 8192);
      wf[e][1] = *reinterpret_cast<const u16x8*>(reg + wo1 + e * 8192);
    }
  };
  auto mfma_q = [&](f32x4 (&a)[4][2], u16x8 (&wf)[2][2]) {
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

  const int T = K / gridDim.y / kBK;   // K-tiles of this block's split-K slice (blockIdx.y)
  if constexpr (PH2) {
    // prologue: all four regions of K-tile 0; X0, W0 and W1 retired before the first reads
#pragma unroll
    for (int r = 0; r < 4; ++r) issue(r, 0, 0);
    vm_wait<2>();
    seg_barrier();
    if (g == 1) seg_barrier();   // ping-pong: waves 4-7 one segment behind
    for (int t = 0; t < T; ++t) {
      const char* cur = lds + (t & 1) * kBuf;
      const int nb = (t + 1) & 1;
      const bool more = t + 1 < T;
      // -- segment A: (X0, W0), (X0, W1); issue X0, W0, W1 of tile t+1; retire X1 of tile t
      read_x(cur + 0 * kRegion);
      read_w(cur + 1 * kRegion, wf0);
      read_w(cur + 2 * kRegion, wf1);
      if (more) {
        issue(0, nb, t + 1);
        issue(1, nb, t + 1);
        issue(2, nb, t + 1);
      }
      if (g == 1) { if (more) vm_wait<6>(); else vm_wait<0>(); }
      seg_barrier();
      mfma_q(acc[0][0], wf0);
      mfma_q(acc[0][1], wf1);
      if (g == 0) { if (more) vm_wait<6>(); else vm_wait<0>(); }
      seg_barrier();
      // -- segment B: (X1, W0), (X1, W1); issue X1 of tile t+1; retire X0 / W0 / W1 of t+1
      read_x(cur + 3 * kRegion);
      if (more) issue(3, nb, t + 1);
      if (g == 1 && more) vm_wait<2>();
      seg_barrier();
      mfma_q(acc[1][0], wf0);
      mfma_q(acc[1][1], wf1);
      if (g == 0 && more) vm_wait<2>();
      seg_barrier();
    }
  } else {
  // prologue: all four regions of K-tile 0; X0 and W0 retired before the first reads
#pragma unroll
  for (int r = 0; r < 4; ++r) issue(r, 0, 0);
  vm_wait<4>();
  seg_barrier();
  if (g == 1) seg_barrier();   // ping-pong: waves 4-7 one segment behind

  for (int t = 0; t < T; ++t) {
    const char* cur = lds + (t & 1) * kBuf;
    const int nb = (t + 1) & 1;
    const bool more = t + 1 < T;
    // -- phase 1: quadrant (X0, W0); issue X0 of tile t+1
    read_x(cur + 0 * kRegion);
    read_w(cur + 1 * kRegion, wf0);
    if (more) issue(0, nb, t + 1);
    if (g == 1) { if (more) vm_wait<4>(); else vm_wait<2>(); }
    seg_barrier();
    mfma_q(acc[0][0], wf0);
    if (g == 0) { if (more) vm_wait<4>(); else vm_wait<2>(); }
    seg_barrier();
    // -- phase 2: quadrant (X0, W1); issue W0 of tile t+1
    read_w(cur + 2 * kRegion, wf1);
    if (more) issue(1, nb, t + 1);
    if (g == 1) { if (more) vm_wait<4>(); else vm_wait<0>(); }
    seg_barrier();
    mfma_q(acc[0][1], wf1);
    if (g == 0) { if (more) vm_wait<4>(); else vm_wait<0>(); }
    seg_barrier();
    // -- phase 3: quadrant (X1, W0); issue W1 of tile t+1
    read_x(cur + 3 * kRegion);
    if (more) issue(2, nb, t + 1);
    seg_barrier();
    mfma_q(acc[1][0], wf0);
    seg_barrier();
    // -- phase 4: quadrant (X1, W1) from registers; issue X1 of tile t+1 and retire
    // X0 / W0 of tile t+1 before phase 1 reads them
    if (more) issue(3, nb, t + 1);
    if (g == 1 && more) vm_wait<4>();
    seg_barrier();
    mfma_q(acc[1][1], wf1);
    if (g == 0 && more) vm_wait<4>();
    seg_barrier();
  }
  }
  if (g == 0) seg_barrier();   // pairs with the waves 4-7 stagger barrier

  // ---- epilogue: lane holds features 4*lq .. 4*lq+3 of token l15 per fragment
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int tok = m0 + h * 128 + g * 64 + b * 16 + l15;
      if (tok >= M) continue;
      bf16_t* yrow = Y + (int64_t)tok * ldy;
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        if constexpr (EPI == kEpiPartial) {   // fp32 slab [blockIdx.y][M][N], 16-B stores
          float* prow = P + ((int64_t)blockIdx.y * M + tok) * N;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int col = n0 + f * 128 + e * 64 + wc * 16 + 4 * lq;
            if (col < N) *reinterpret_cast<f32x4*>(prow + col) = acc[h][f][b][e];
          }
        } else if constexpr (EPI == kEpiSilu) {
          // interleaved gate|up: 128-row block f = 64 gate rows then their 64 up rows
          const int col = (n0 >> 1) + f * 64 + wc * 16 + 4 * lq;
          if (2 * col >= N) continue;
          const f32x4 gt = acc[h][f][b][0], up = acc[h][f][b][1];
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gg = bf2f(f2bf(gt[r]));
            const float uu = bf2f(f2bf(up[r]));
            const float sg = bf2f(f2bf(gg / (1.f + __expf(-gg))));
            o[r] = sg * uu;
          }
          *reinterpret_cast<uint2*>(yrow + col) = pack4(o);
        } else {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int col = n0 + f * 128 + e * 64 + wc * 16 + 4 * lq;
            if (col >= N) continue;
            f32x4 v = acc[h][f][b][e];
            if constexpr (EPI == kEpiBias) {
              const uint2 bb = *reinterpret_cast<const uint2*>(bias + col);
              v[0] += __uint_as_float(bb.x << 16);
              v[1] += __uint_as_float(bb.x & 0xffff0000u);
              v[2] += __uint_as_float(bb.y << 16);
              v[3] += __uint_as_float(bb.y & 0xffff0000u);
            }
            *reinterpret_cast<uint2*>(yrow + col) = pack4(v);
          }
        }
      }
    }
}

// Variant 1 ("ring-4"): four waves (one per SIMD), each owning a 128 x 128 output block
// (64 accumulator fragments = 256 AGPRs, 0.25 KB of LDS fragment reads per MFMA), and a
// 4-deep ring of BK = 32 stages (32 KiB each: 128 KiB of LDS) so two stages are always
// in flight behind the one being computed and the one being read: the counted
// vmcnt(8) at the end of a step leaves the youngest stage's DMA outstanding, never 0
// inside the loop (round 3's 2-buffer BK = 64 version waited 15 % of its wave-cycles on
// a vmcnt(0) per K-tile, profiles/gemm_tile_pmc_vs_hipblaslt.txt).
//   * LDS image: a stage is 32 pieces of 1 KiB (16 rows x 64 B; pieces 0-15 X rows,
//     16-31 W rows). Inside a piece, row r's four 16-B k-chunks c sit at slots
//     4r + (c ^ f(r >> 2)), f = {0, 3, 2, 1}: the DMA (lane-linear: lane l writes slot l)
//     reads each row's 64 B with four consecutive lanes (coalesced), and a fragment is ONE
//     ds_read_b128 per lane (lane l: row l & 15, chunk l >> 4) whose four 16-lane groups
//     each hit 16 distinct bank slots — conflict-free by the choice of f.
//   * per step and wave: 64 MFMAs (v_mfma_f32_16x16x32_bf16, accumulator tied in an AGPR
//     by inline asm: the builtin makes hipcc shuffle 256 accumulators through
//     v_accvgpr copies), the 16 fragment reads of the NEXT stage (register double
//     buffer) and 8 LDS-DMA pieces of the stage three ahead, spread one row of 8 MFMAs
//     apart; one raw s_barrier per step.
// Stage t lives in buffer t % 4; step t reads stage t+1 and refills buffer (t+3) % 4,
// whose stage t-1 every wave finished reading before the barrier that ended step t-1.
__device__ __forceinline__ void mfma_tied(f32x4& acc, const u16x8& a, const u16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// DM: how the stages are loaded — 0: global_load_lds (flat address per lane), 1: buffer_load
// ... lds (SGPR descriptor, 32-bit lane offset, K step in soffset), 6: register staging
// (global_load_dwordx4 into one of two register sets in step t, ds_write_b128 of that set
// into the LDS image in step t+1, same image as the DMA). Timing experiments only
// (wrong results): 2 no loads inside the loop; 3 every piece read from 1 KiB of contiguous
// memory; 4 the 8 pieces issued back to back after the first MFMA row; 5 W pieces only
template <int EPI, int DM = 0>
__global__ void __launch_bounds__(256) gemm_tile256_r4_kernel(const bf16_t* __restrict__ X,
                                                              const bf16_t* __restrict__ W, bf16_t* __restrict__ Y,
                                                              const bf16_t* __restrict__ bias, int M, int N, int K,
                                                              int ldy) {
  constexpr int kBK4 = 32, kNS = 4, kStage = 32768, kWOff = 16384;
  __shared__ __attribute__((aligned(1024))) char lds[kNS * kStage];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;

  const int mt = (M + kT - 1) / kT, nt = (N + kT - 1) / kT;
  const int nwg = mt * nt;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int gsz = kGroupM * nt;
  const int first_m = (lid / gsz) * kGroupM;
  const int gm = min(mt - first_m, kGroupM);
  const int tm = first_m + (lid % gsz) % gm;
  const int tn = (lid % gsz) / gm;
  const int m0 = tm * kT, n0 = tn * kT;

  // DMA: wave w issues pieces w + 4i (i < 4: X rows 16(w + 4i).., i >= 4: W rows
  // 16(w + 4(i - 4))..); lane l -> row l >> 2, chunk (l & 3) ^ f(l >> 4). 32-bit byte offsets
  // (the launcher guarantees M*K*2 and N*K*2 < 4 GiB): scalar base + vector offset loads.
  const int r15 = lane >> 2, ck = (lane & 3) ^ ((4 - (lane >> 4)) & 3);
  uint32_t xs[4], ws[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xs[i] = ((uint32_t)min(m0 + 16 * (w + 4 * i) + r15, M - 1) * (uint32_t)K + ck * 8) * 2u;
    ws[i] = ((uint32_t)min(n0 + 16 * (w + 4 * i) + r15, N - 1) * (uint32_t)K + ck * 8) * 2u;
  }
  const char* Xb = reinterpret_cast<const char*>(X);
  const char* Wb = reinterpret_cast<const char*>(W);
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((uint32_t)M * (uint32_t)K * 2u), 0x00020000);
  const auto wr = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((uint32_t)N * (uint32_t)K * 2u), 0x00020000);
  auto dma = [&](int kt, int buf, int q) {   // piece q (0..7) of this wave for K-step kt, into buffer buf
    char* dst = lds + buf * kStage + w * 1024;
    const uint32_t k2 = (uint32_t)kt * (kBK4 * 2);
    if constexpr (DM == 1) {
      if (q < 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(dst + q * 4096), 16,
                                                 (int)xs[q], (int)k2, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void*)(dst + kWOff + (q - 4) * 4096),
                                                 16, (int)ws[q - 4], (int)k2, 0, 0);
    } else if constexpr (DM == 3) {
      const char* base = (q < 4 ? Xb : Wb) + (uint32_t)(w * 8 + q) * 1024u + (uint32_t)lane * 16u + k2 * 64u;
      __builtin_amdgcn_global_load_lds(base, (__attribute__((address_space(3))) void*)(dst + (q < 4 ? q * 4096 : kWOff + (q - 4) * 4096)),
                                       16, 0, 0);
    } else {
      if (q < 4)
        __builtin_amdgcn_global_load_lds(Xb + xs[q] + k2, (__attribute__((address_space(3))) void*)(dst + q * 4096),
                                         16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds(Wb + ws[q - 4] + k2,
                                         (__attribute__((address_space(3))) void*)(dst + kWOff + (q - 4) * 4096), 16, 0,
                                         0);
    }
  };

  // fragment reads: X fragment i = piece wm*8 + i; W fragment j = the rows of feature
  // block j = f*4 + type*2 + jj (128-row half f, gate/up 64-row type, wave's 32 rows)
  const int l16 = 16 * (4 * (lane & 15) + ((lane >> 4) ^ ((4 - ((lane & 15) >> 2)) & 3)));
  auto rd1 = [&](int kt, u16x8 (&xf)[8], u16x8 (&wf)[8], int q) {
    constexpr int kOrd[16] = {8, 9, 0, 10, 11, 1, 12, 13, 2, 14, 15, 3, 4, 5, 6, 7};   // >= 8: W fragment
    const char* buf = lds + (kt & (kNS - 1)) * kStage + l16;
    const int o = kOrd[q];
    if (o >= 8) {
      const int j = o - 8;
      const int piece = (j >> 2) * 8 + ((j >> 1) & 1) * 4 + wn * 2 + (j & 1);
      wf[j] = *reinterpret_cast<const u16x8*>(buf + kWOff + piece * 1024);
    } else {
      xf[o] = *reinterpret_cast<const u16x8*>(buf + (wm * 8 + o) * 1024);
    }
  };

  // register staging (DM 6): piece q of stage kt -> set[q]; set -> this wave's LDS slot
  auto gload = [&](int kt, u32x4 (&st)[8], int q) {
    const uint32_t k2 = (uint32_t)kt * (kBK4 * 2);
    st[q] = q < 4 ? __builtin_amdgcn_raw_buffer_load_b128(xr, (int)xs[q], (int)k2, 0)
                  : __builtin_amdgcn_raw_buffer_load_b128(wr, (int)ws[q - 4], (int)k2, 0);
  };
  auto lwrite = [&](int buf, const u32x4 (&st)[8], int q) {
    char* dst = lds + buf * kStage + w * 1024 + (q < 4 ? q * 4096 : kWOff + (q - 4) * 4096) + lane * 16;
    *reinterpret_cast<u32x4*>(dst) = st[q];
  };

  f32x4 acc[8][8];   // [token block][feature block]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 xa[8], wa[8], xb[8], wb[8];
  u32x4 sa[8], sb[8];
  // one K-step: 64 MFMAs; after each 8-MFMA row, two fragment reads of step kt+1 and one
  // DMA piece of step kt+3. Branch-free: past the last step the reads fetch a buffer no
  // one uses and the DMA re-loads step T-1 into buffer (kt+3) % 4, whose stage (kt-1) is
  // consumed and which no later step reads; the loop's exit drains those DMAs.
  // DM 6: the row's global load of stage kt+3 goes to set `ld`, and the row writes piece i
  // of set `wr` (stage kt+2, loaded in step kt-1) into buffer (kt+2) % 4 (stage kt-2's,
  // whose fragments were read in step kt-3); the barrier ending step kt publishes it for
  // the fragment reads of step kt+1.
  const int T = K / kBK4;   // even (K % 64 == 0)
  auto step = [&](u16x8 (&xf)[8], u16x8 (&wf)[8], u16x8 (&nx)[8], u16x8 (&nw)[8], int kt, u32x4 (&ld)[8],
                  u32x4 (&wr)[8]) {
    const int ks = min(kt + 3, T - 1), kb = (kt + 3) & (kNS - 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma_tied(acc[i][j], wf[j], xf[i]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (DM == 6) {
        gload(ks, ld, i);
        lwrite((kt + 2) & (kNS - 1), wr, i);
      } else if constexpr (DM == 7) {   // timing: loads only (the set kept live, never written)
        gload(ks, ld, i);
        asm volatile("" ::"v"(wr[i]));
      } else if constexpr (DM == 8) {   // timing: LDS writes only (of registers never loaded)
        asm volatile("" : "+v"(wr[i]));
        lwrite((kt + 2) & (kNS - 1), wr, i);
      } else if constexpr (DM == 4) {
        if (i == 0)
#pragma unroll
          for (int q = 0; q < 8; ++q) dma(ks, kb, q);
      } else if constexpr (DM == 5) {
        if (i >= 4) dma(ks, kb, i);
      } else if constexpr (DM != 2) {
        dma(ks, kb, i);
      }
      rd1(kt + 1, nx, nw, 2 * i);
      rd1(kt + 1, nx, nw, 2 * i + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // zero-initialised accumulators are read as SrcC by asm MFMAs, whose hazards hipcc
  // does not pad: pin the writes above an explicit nop
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_nop 4");

  if constexpr (DM >= 6) {   // stages 0, 1 into LDS; stage 2 in set B (written by step 0)
#pragma unroll
    for (int q = 0; q < 8; ++q) gload(0, sa, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) gload(min(1, T - 1), sb, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) lwrite(0, sa, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) lwrite(1, sb, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) gload(min(2, T - 1), sb, q);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(0, 0, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(min(1, T - 1), 1, q);
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(min(2, T - 1), 2, q);
    vm_wait<8>();   // stages 0 and 1 landed (this wave's pieces); stage 2 in flight
  }
  seg_barrier();
#pragma unroll
  for (int q = 0; q < 16; ++q) rd1(0, xa, wa, q);
  // one loop, no peeled copy: a second code path makes hipcc move accumulators with
  // v_accvgpr_write right before an asm MFMA reads them (an unpadded hazard)
  for (int t = 0; t < T; t += 2) {
    // step t: regs A hold stage t; read stage t+1 into B; DMA stage t+3
    step(xa, wa, xb, wb, t, sa, sb);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (DM < 6) vm_wait<8>();   // stage t+2 landed (this wave's pieces); stage t+3 in flight
    seg_barrier();
    // step t+1: regs B hold stage t+1; read stage t+2 into A; DMA stage t+4
    step(xb, wb, xa, wa, t + 1, sb, sa);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (DM < 6) vm_wait<8>();
    seg_barrier();
  }
  vm_wait<0>();   // the tail's dummy DMAs must land before the workgroup's LDS is released
  // the accumulators were written by asm MFMAs the hazard recognizer cannot see:
  // cover the MFMA-write -> accvgpr-read latency before the epilogue reads them
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");

  const int l15 = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int tok = m0 + wm * 128 + i * 16 + l15;
    if (tok >= M) continue;
    bf16_t* yrow = Y + (int64_t)tok * ldy;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (EPI == kEpiSilu) {
          const int col = (n0 >> 1) + f * 64 + wn * 32 + j * 16 + 4 * lq;
          if (2 * col >= N) continue;
          const f32x4 gt = acc[i][f * 4 + j], up = acc[i][f * 4 + 2 + j];
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gg = bf2f(f2bf(gt[r]));
            const float uu = bf2f(f2bf(up[r]));
            const float sg = bf2f(f2bf(gg / (1.f + __expf(-gg))));
            o[r] = sg * uu;
          }
          *reinterpret_cast<uint2*>(yrow + col) = pack4(o);
        } else {
#pragma unroll
          for (int ty = 0; ty < 2; ++ty) {
            const int col = n0 + f * 128 + ty * 64 + wn * 32 + j * 16 + 4 * lq;
            if (col >= N) continue;
            f32x4 v = acc[i][f * 4 + ty * 2 + j];
            if constexpr (EPI == kEpiBias) {
              const uint2 bb = *reinterpret_cast<const uint2*>(bias + col);
              v[0] += __uint_as_float(bb.x << 16);
              v[1] += __uint_as_float(bb.x & 0xffff0000u);
              v[2] += __uint_as_float(bb.y << 16);
              v[3] += __uint_as_float(bb.y & 0xffff0000u);
            }
            *reinterpret_cast<uint2*>(yrow + col) = pack4(v);
          }
        }
      }
  }
}

// Variant 9 ("region ring"): four waves (one per SIMD, 128 x 128 outputs each, 256 tied
// AGPR accumulators) with BK = 64 K-tiles loaded in full 128-B row segments: measured on
// the ring-4 kernel, an LDS-DMA instruction of 16 rows x 64 B costs about twice what one of
// 8 rows x 128 B does (the memory pipeline's request count, not the bytes: M 16384, N 4096,
// K 14336: 1.25 PF/s with 64-B segments, 1.57 with 1-KiB contiguous pieces, 1.80 with no
// loads at all; tools/gemm_tile_variants.py). A 64-deep tile is 64 KiB, so the ring is cut
// into 16 KiB regions (X rows 0-127, X 128-255, W 0-127, W 128-255 of a tile): 10 regions
// (160 KiB) = 2.5 tiles. Region i = 4 * tile + r lives in slot i % 10; while tile t is
// computed the waves issue regions 4t+6 .. 4t+9 (tile t+1's second half, tile t+2's first)
// into tile t-1's slots, and the counted vmcnt(8) at the end of tile t leaves exactly the
// two youngest regions in flight. One raw barrier per tile. LDS image: 128-B rows with the
// chunk ^ ((row >> 1) & 7) swizzle on the DMA source and the read (conflict-free b128).
template <int EPI>
__global__ void __launch_bounds__(256) gemm_tile256_q4_kernel(const bf16_t* __restrict__ X,
                                                              const bf16_t* __restrict__ W, bf16_t* __restrict__ Y,
                                                              const bf16_t* __restrict__ bias, int M, int N, int K,
                                                              int ldy) {
  constexpr int kSlots = 10;
  __shared__ __attribute__((aligned(1024))) char lds[kSlots * kRegion];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;

  const int mt = (M + kT - 1) / kT, nt = (N + kT - 1) / kT;
  const int nwg = mt * nt;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int gsz = kGroupM * nt;
  const int first_m = (lid / gsz) * kGroupM;
  const int gm = min(mt - first_m, kGroupM);
  const int tm = first_m + (lid % gsz) % gm;
  const int tn = (lid % gsz) / gm;
  const int m0 = tm * kT, n0 = tn * kT;

  // DMA: region r (0: X rows 0-127, 1: X 128-255, 2: W 0-127, 3: W 128-255), piece q (0..3)
  // of wave w = region rows 8 (w + 4q) .. +7; lane l -> row + l/8, LDS slot l%8, source
  // chunk slot ^ ((row >> 1) & 7). 32-bit byte offsets (the launcher checks the extents).
  const int lrow = lane >> 3, lslot = lane & 7;
  uint32_t so[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 8 * (w + 4 * q) + lrow;
      const int chunk = lslot ^ ((row >> 1) & 7);
      const int g = (r < 2) ? min(m0 + 128 * r + row, M - 1) : min(n0 + 128 * (r - 2) + row, N - 1);
      so[r][q] = ((uint32_t)g * (uint32_t)K + chunk * 8) * 2u;
    }
  const char* Xb = reinterpret_cast<const char*>(X);
  const char* Wb = reinterpret_cast<const char*>(W);
  const int T = K / kBK;
  // region i (tile i / 4, part i % 4); past the last tile it re-loads tile T-1 (its slot is
  // free and never read again), so every tile issues the same number of DMAs
  auto dma = [&](int i, int q) {
    const int r = i & 3;
    const int kt = min(i >> 2, T - 1);
    char* dst = lds + (i % kSlots) * kRegion + (w + 4 * q) * 1024;
    const char* src = (r < 2 ? Xb : Wb) + so[r][q] + (uint32_t)kt * (kBK * 2);
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  };

  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int c0 = (lq ^ sw) << 4, c1 = ((4 + lq) ^ sw) << 4;
  // fragment rows: X fragment i = rows 16 i + l15 of region wm; W fragment j (f = j / 4,
  // type = (j / 2) % 2, jj = j % 2) = rows type*64 + wn*32 + jj*16 + l15 of region 2 + f
  auto rd1 = [&](int t, int c, u16x8 (&xf)[8], u16x8 (&wf)[8], int q) {
    constexpr int kOrd[16] = {8, 9, 0, 10, 11, 1, 12, 13, 2, 14, 15, 3, 4, 5, 6, 7};   // >= 8: W fragment
    const int o = kOrd[q];
    if (o >= 8) {
      const int j = o - 8;
      const char* reg = lds + ((4 * t + 2 + (j >> 2)) % kSlots) * kRegion;
      wf[j] = *reinterpret_cast<const u16x8*>(reg + (((j >> 1) & 1) * 64 + wn * 32 + (j & 1) * 16 + l15) * 128 + c);
    } else {
      const char* reg = lds + ((4 * t + wm) % kSlots) * kRegion;
      xf[o] = *reinterpret_cast<const u16x8*>(reg + (16 * o + l15) * 128 + c);
    }
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 xa[8], wa[8], xb[8], wb[8];
  // one k-substep of tile t: 64 MFMAs; after each 8-MFMA row two fragment reads of the next
  // substep (from tile tn, chunk cn) and, in the first substep, one DMA piece of regions
  // 4t+6 .. 4t+9 (2 per row: the 16 pieces of the four regions over the 8 rows)
  auto mm = [&](u16x8 (&xf)[8], u16x8 (&wf)[8], int tn, int cn, u16x8 (&nx)[8], u16x8 (&nw)[8], int t,
                bool first) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma_tied(acc[i][j], wf[j], xf[i]);
      __builtin_amdgcn_sched_barrier(0);
      if (first) {
        dma(4 * t + 6 + (i >> 1), (2 * i) & 3);
        dma(4 * t + 6 + (i >> 1), (2 * i + 1) & 3);
      }
      rd1(tn, cn, nx, nw, 2 * i);
      rd1(tn, cn, nx, nw, 2 * i + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_nop 4");

  // prologue: regions 0 .. 5 (tile 0, tile 1's first half); tile 0 landed, 2 regions in flight
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) dma(i, q);
  vm_wait<8>();
  seg_barrier();
#pragma unroll
  for (int q = 0; q < 16; ++q) rd1(0, c0, xa, wa, q);
  // one loop, no peeled copy (a second code path makes hipcc move accumulators with
  // v_accvgpr_write right before an asm MFMA reads them)
  for (int t = 0; t < T; ++t) {
    // substep 0 of tile t (regs A), reading substep 1 of tile t; issues regions 4t+6 .. 4t+9
    mm(xa, wa, t, c1, xb, wb, t, true);
    // substep 1 of tile t (regs B), reading substep 0 of tile t+1 (landed: see below)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    vm_wait<8>();      // tile t+1 landed (this wave's pieces); regions 4t+8, 4t+9 in flight
    seg_barrier();     // ... every wave's pieces; tile t-1's reads long done
    mm(xb, wb, t + 1, c0, xa, wa, t, false);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    seg_barrier();     // every wave done reading tile t: its slots are refilled next tile
  }
  vm_wait<0>();        // the tail's re-loads land before the workgroup's LDS is released
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");

#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int tok = m0 + wm * 128 + i * 16 + l15;
    if (tok >= M) continue;
    bf16_t* yrow = Y + (int64_t)tok * ldy;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (EPI == kEpiSilu) {
          const int col = (n0 >> 1) + f * 64 + wn * 32 + j * 16 + 4 * lq;
          if (2 * col >= N) continue;
          const f32x4 gt = acc[i][f * 4 + j], up = acc[i][f * 4 + 2 + j];
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gg = bf2f(f2bf(gt[r]));
            const float uu = bf2f(f2bf(up[r]));
            const float sg = bf2f(f2bf(gg / (1.f + __expf(-gg))));
            o[r] = sg * uu;
          }
          *reinterpret_cast<uint2*>(yrow + col) = pack4(o);
        } else {
#pragma unroll
          for (int ty = 0; ty < 2; ++ty) {
            const int col = n0 + f * 128 + ty * 64 + wn * 32 + j * 16 + 4 * lq;
            if (col >= N) continue;
            f32x4 v = acc[i][f * 4 + ty * 2 + j];
            if constexpr (EPI == kEpiBias) {
              const uint2 bb = *reinterpret_cast<const uint2*>(bias + col);
              v[0] += __uint_as_float(bb.x << 16);
              v[1] += __uint_as_float(bb.x & 0xffff0000u);
              v[2] += __uint_as_float(bb.y << 16);
              v[3] += __uint_as_float(bb.y & 0xffff0000u);
            }
            *reinterpret_cast<uint2*>(yrow + col) = pack4(v);
          }
        }
      }
  }
}

// Variant 13 ("two buffers, four phases"): four waves (one per SIMD, 128 x 128 outputs
// each, 256 tied AGPR accumulators), BK = 64 tiles in two 64 KiB LDS buffers filled by
// LDS-DMA pieces of 8 rows x 128 B (buffer_load ... lds: per-lane 32-bit row offsets fixed
// for the kernel, the K step in soffset) — half the memory requests of 16 x 64-B pieces
// (profiles/gemm_tile_pmc_l2_r4.txt: TCC_HIT 2.2e8 vs 9.9e7, TA_BUSY 2.5x). Tile t (buffer
// t & 1) runs in four 32-MFMA phases:
//   1. k-half 0 from registers A; read k-half 1 (registers B) — the tile's last reads;
//      lgkmcnt(0) + barrier: every wave is done with buffer t & 1
//   2. k-half 0 cont.; 8 X pieces of tile t+2 into buffer t & 1;
//      vmcnt(16) + barrier: tile t+1's X pieces (issued in phase 2 of tile t-1) landed
//   3. k-half 1 from registers B; 8 W pieces of tile t+2; read X of tile t+1, k-half 0;
//      vmcnt(16) + barrier: tile t+1's W pieces landed
//   4. k-half 1 cont.; read W of tile t+1, k-half 0 (registers A)
// so every piece has a whole tile (128 MFMAs per wave) to land, a buffer is refilled only
// after the barrier that follows its last read, and each staged piece is read one phase
// after the wait + barrier that retire it. DMAs and fragment reads sit between MFMAs (one
// per two). LDS image: 128-B rows, chunk slot = chunk ^ ((row >> 1) & 7) on the DMA
// source and the read (conflict-free ds_read_b128, as variant 9).
template <int EPI, int AUX = 0>
__global__ void __launch_bounds__(256) gemm_tile256_h4_kernel(const bf16_t* __restrict__ X,
                                                              const bf16_t* __restrict__ W, bf16_t* __restrict__ Y,
                                                              const bf16_t* __restrict__ bias, int M, int N, int K,
                                                              int ldy) {
  constexpr int kHalf = 32768;       // one operand of a tile: 256 rows x 128 B
  constexpr int kTile = 2 * kHalf;   // X then W
  __shared__ __attribute__((aligned(1024))) char lds[2 * kTile];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;

  const int mt = (M + kT - 1) / kT, nt = (N + kT - 1) / kT;
  const int nwg = mt * nt;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int gsz = kGroupM * nt;
  const int first_m = (lid / gsz) * kGroupM;
  const int gm = min(mt - first_m, kGroupM);
  const int tm = first_m + (lid % gsz) % gm;
  const int tn = (lid % gsz) / gm;
  const int m0 = tm * kT, n0 = tn * kT;

  // DMA piece q (0..7) of an operand for wave w = rows 8 (w + 4q) .. +7; lane l -> row + l/8,
  // LDS slot l % 8, source chunk slot ^ ((row >> 1) & 7). 32-bit byte offsets (launcher checks)
  const int lrow = lane >> 3, lslot = lane & 7;
  uint32_t xo[8], wo[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int row = 8 * (w + 4 * q) + lrow;
    const int chunk = lslot ^ ((row >> 1) & 7);
    xo[q] = ((uint32_t)min(m0 + row, M - 1) * (uint32_t)K + chunk * 8) * 2u;
    wo[q] = ((uint32_t)min(n0 + row, N - 1) * (uint32_t)K + chunk * 8) * 2u;
  }
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((uint32_t)M * (uint32_t)K * 2u), 0x00020000);
  const auto wr = __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((uint32_t)N * (uint32_t)K * 2u), 0x00020000);
  const int T = K / kBK;
  auto dma_x = [&](int kt, int buf, int q) {
    char* dst = lds + buf * kTile + (w + 4 * q) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)dst, 16, (int)xo[q],
                                             min(kt, T - 1) * (kBK * 2), 0, AUX);
  };
  auto dma_w = [&](int kt, int buf, int q) {
    char* dst = lds + buf * kTile + kHalf + (w + 4 * q) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (__attribute__((address_space(3))) void*)dst, 16, (int)wo[q],
                                             min(kt, T - 1) * (kBK * 2), 0, AUX);
  };

  // fragments: X fragment i = rows wm*128 + 16 i + l15; W fragment j (f = j / 4, type =
  // (j / 2) % 2, jj = j % 2) = rows f*128 + type*64 + wn*32 + jj*16 + l15; k-half h reads
  // chunk 4h + lane/16 of the row, at its swizzled slot
  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int c0 = (lq ^ sw) << 4, c1 = ((4 + lq) ^ sw) << 4;
  const int xrow = (wm * 128 + l15) * 128, wrow = (wn * 32 + l15) * 128;
  auto rdx = [&](int buf, int c, u16x8 (&xf)[8], int i) {
    xf[i] = *reinterpret_cast<const u16x8*>(lds + buf * kTile + xrow + i * 2048 + c);
  };
  auto rdw = [&](int buf, int c, u16x8 (&wf)[8], int j) {
    const int r = (j >> 2) * 128 + ((j >> 1) & 1) * 64 + (j & 1) * 16;
    wf[j] = *reinterpret_cast<const u16x8*>(lds + buf * kTile + kHalf + wrow + r * 128 + c);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 xa[8], wa[8], xb[8], wb[8];
  // one MFMA row (token block i: 8 MFMAs) with up to four other instructions, one after
  // every second MFMA (op(k), k = 0..3)
  auto row = [&](const u16x8 (&xf)[8], const u16x8 (&wf)[8], int i, auto op) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mfma_tied(acc[i][j], wf[j], xf[i]);
      if (j & 1) {
        __builtin_amdgcn_sched_barrier(0);
        op(j >> 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_nop 4");

  // prologue: tiles 0 and 1 (buffers 0, 1); tile 0 landed; k-half 0 of tile 0 into A
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_x(0, 0, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_w(0, 0, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_x(1, 1, q);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_w(1, 1, q);
  vm_wait<16>();
  seg_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) rdx(0, c0, xa, i);
#pragma unroll
  for (int j = 0; j < 8; ++j) rdw(0, c0, wa, j);

  // one loop, no peeled copy (a second code path makes hipcc move accumulators with
  // v_accvgpr_write right before an asm MFMA reads them)
  for (int t = 0; t < T; ++t) {
    const int b = t & 1, nb = b ^ 1;
    // phase 1: rows 0-3 of k-half 0; read k-half 1 of tile t (X 8, W 8)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      row(xa, wa, i, [&](int k) {
        if (k < 2) rdx(b, c1, xb, 2 * i + k);
        else rdw(b, c1, wb, 2 * i + k - 2);
      });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    seg_barrier();
    // phase 2: rows 4-7 of k-half 0; X pieces of tile t+2 into buffer b
#pragma unroll
    for (int i = 4; i < 8; ++i)
      row(xa, wa, i, [&](int k) {
        if (!(k & 1)) dma_x(t + 2, b, 2 * (i - 4) + (k >> 1));
      });
    vm_wait<16>();   // tile t+1's X pieces (this wave's)
    seg_barrier();   // ... every wave's
    // phase 3: rows 0-3 of k-half 1; W pieces of tile t+2; X of tile t+1, k-half 0
#pragma unroll
    for (int i = 0; i < 4; ++i)
      row(xb, wb, i, [&](int k) {
        if (!(k & 1)) dma_w(t + 2, b, 2 * i + (k >> 1));
        else rdx(nb, c0, xa, 2 * i + (k >> 1));
      });
    vm_wait<16>();   // tile t+1's W pieces
    seg_barrier();
    // phase 4: rows 4-7 of k-half 1; W of tile t+1, k-half 0
#pragma unroll
    for (int i = 4; i < 8; ++i)
      row(xb, wb, i, [&](int k) {
        if (!(k & 1)) rdw(nb, c0, wa, 2 * (i - 4) + (k >> 1));
      });
  }
  vm_wait<0>();   // the tail's clamped re-loads land before the workgroup's LDS is released
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");

#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int tok = m0 + wm * 128 + i * 16 + l15;
    if (tok >= M) continue;
    bf16_t* yrow = Y + (int64_t)tok * ldy;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (EPI == kEpiSilu) {
          const int col = (n0 >> 1) + f * 64 + wn * 32 + j * 16 + 4 * lq;
          if (2 * col >= N) continue;
          const f32x4 gt = acc[i][f * 4 + j], up = acc[i][f * 4 + 2 + j];
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float gg = bf2f(f2bf(gt[r]));
            const float uu = bf2f(f2bf(up[r]));
            const float sg = bf2f(f2bf(gg / (1.f + __expf(-gg))));
            o[r] = sg * uu;
          }
          *reinterpret_cast<uint2*>(yrow + col) = pack4(o);
        } else {
#pragma unroll
          for (int ty = 0; ty < 2; ++ty) {
            const int col = n0 + f * 128 + ty * 64 + wn * 32 + j * 16 + 4 * lq;
            if (col >= N) continue;
            f32x4 v = acc[i][f * 4 + ty * 2 + j];
            if constexpr (EPI == kEpiBias) {
              const uint2 bb = *reinterpret_cast<const uint2*>(bias + col);
              v[0] += __uint_as_float(bb.x << 16);
              v[1] += __uint_as_float(bb.x & 0xffff0000u);
              v[2] += __uint_as_float(bb.y << 16);
              v[3] += __uint_as_float(bb.y & 0xffff0000u);
            }
            *reinterpret_cast<uint2*>(yrow + col) = pack4(v);
          }
        }
      }
  }
}

// y[m, f] = SwiGLU of the split-K sums of the interleaved gate|up slabs (64-feature
// blocks): g = bf16(sum_s P[s][m][128 b + j]), u = bf16(sum_s P[s][m][128 b + 64 + j]),
// y = bf16(bf16(silu(g)) * u) — the numerics of the fused epilogue. 4 features per thread.
__global__ void splitk_silu_reduce_kernel(const float* __restrict__ P, bf16_t* __restrict__ Y, int M, int N, int S,
                                          int ldy) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int NO = N / 2;
  if (i >= (int64_t)M * NO) return;
  const int m = (int)(i / NO), f = (int)(i % NO);
  const int col = (f >> 6) * 128 + (f & 63);
  const int64_t MN = (int64_t)M * N;
  const float* pr = P + (int64_t)m * N + col;
  f32x4 g = *reinterpret_cast<const f32x4*>(pr), u = *reinterpret_cast<const f32x4*>(pr + 64);
  for (int s = 1; s < S; ++s) {
    g += *reinterpret_cast<const f32x4*>(pr + s * MN);
    u += *reinterpret_cast<const f32x4*>(pr + s * MN + 64);
  }
  f32x4 o;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float gg = bf2f(f2bf(g[r]));
    const float uu = bf2f(f2bf(u[r]));
    o[r] = bf2f(f2bf(gg / (1.f + __expf(-gg)))) * uu;
  }
  *reinterpret_cast<uint2*>(Y + (int64_t)m * ldy + f) = pack4(o);
}

int gemm_tile(const bf16_t* X, const bf16_t* W, bf16_t* Y, const bf16_t* bias, int M, int N, int K, int ldy,
              bool silu_gu, int variant, int S, float* P, hipStream_t stream) {
  if (M < 1 || N < 16 || N % 16 != 0 || K < kBK || K % kBK != 0) return -1;
  if (silu_gu && (N % 128 != 0 || bias != nullptr)) return -2;
  if (Y != nullptr && ldy < (silu_gu ? N / 2 : N)) return -3;
  if (S < 1 || S > 64 || K % (kBK * S) != 0 || (S > 1 && (P == nullptr || bias != nullptr))) return -5;
  if (Y == nullptr && (S == 1 || silu_gu)) return -6;
  const int nwg = ((M + kT - 1) / kT) * ((N + kT - 1) / kT);
  if (S > 1) {   // fp32 slabs, then (unless the consumer sums them) one reduce pass
    gemm_tile256_kernel<kEpiPartial><<<dim3(nwg, S), 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, P);
    OAMD_LAUNCH_CHECK();
    if (Y == nullptr) return 0;
    if (silu_gu) {
      const int64_t threads = (int64_t)M * (N / 2) / 4;
      splitk_silu_reduce_kernel<<<(threads + 255) / 256, 256, 0, stream>>>(P, Y, M, N, S, ldy);
      OAMD_LAUNCH_CHECK();
      return 0;
    }
    if (ldy != N) return -7;
    return splitk_reduce(P, Y, (int64_t)M * N, S, stream);
  }
  const bool off32 = (int64_t)M * K * 2 < (1LL << 32) && (int64_t)N * K * 2 < (1LL << 32);
  if (variant == 1 && off32) {   // 4-wave, 4-stage BK = 32 ring (32-bit source offsets)
    if (silu_gu) gemm_tile256_r4_kernel<kEpiSilu><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (bias) gemm_tile256_r4_kernel<kEpiBias><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_r4_kernel<kEpiStore><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if (variant == 9 && off32) {   // 4-wave, BK = 64 region ring
    if (silu_gu) gemm_tile256_q4_kernel<kEpiSilu><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (bias) gemm_tile256_q4_kernel<kEpiBias><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_q4_kernel<kEpiStore><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if (variant == 13 && off32) {   // 4-wave, two 64 KiB buffers, four phases per K-tile
    if (silu_gu) gemm_tile256_h4_kernel<kEpiSilu><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (bias) gemm_tile256_h4_kernel<kEpiBias><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_h4_kernel<kEpiStore><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if (variant >= 14 && variant <= 16 && off32 && !silu_gu && !bias) {   // variant 13, DMA cache policy
    if (variant == 14) gemm_tile256_h4_kernel<kEpiStore, 16><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (variant == 15) gemm_tile256_h4_kernel<kEpiStore, 2><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_h4_kernel<kEpiStore, 18><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if (variant == 10 && off32) {   // 4-wave ring, register-staged loads
    if (silu_gu) gemm_tile256_r4_kernel<kEpiSilu, 6><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (bias) gemm_tile256_r4_kernel<kEpiBias, 6><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_r4_kernel<kEpiStore, 6><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if ((variant == 11 || variant == 12) && off32 && !silu_gu && !bias) {   // register-staging timing splits
    if (variant == 11) gemm_tile256_r4_kernel<kEpiStore, 7><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_r4_kernel<kEpiStore, 8><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if (variant >= 4 && variant <= 8 && off32 && !silu_gu && !bias) {   // ring-4 load experiments
    if (variant == 4) gemm_tile256_r4_kernel<kEpiStore, 1><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (variant == 5) gemm_tile256_r4_kernel<kEpiStore, 2><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (variant == 6) gemm_tile256_r4_kernel<kEpiStore, 3><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (variant == 7) gemm_tile256_r4_kernel<kEpiStore, 4><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_r4_kernel<kEpiStore, 5><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if (variant == 2 || (variant == 0 && M > 256)) {
    // 8-wave ping-pong, two barrier segments per K-tile: 1.8-2.7 % over four segments on
    // the prefill shapes (M = 32k, profiles/gemm_tile_ph2_vs_ph4.jsonl); the lm_head at
    // M <= 256 keeps four (weight-streaming bound there, 1 % the other way)
    if (silu_gu) gemm_tile256_kernel<kEpiSilu, true><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
    else if (bias) gemm_tile256_kernel<kEpiBias, true><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
    else gemm_tile256_kernel<kEpiStore, true><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
  } else {   // 8-wave ping-pong, four segments per K-tile (variant 3, or 0 at M <= 256)
    if (silu_gu) gemm_tile256_kernel<kEpiSilu><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
    else if (bias) gemm_tile256_kernel<kEpiBias><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
    else gemm_tile256_kernel<kEpiStore><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
  }
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
