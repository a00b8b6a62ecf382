// Compute-bound GEMM for prefill projections and the lm_head:
//   Y[M, N] = X[M, K] . W[N, K]^T     bf16 in, fp32 accumulate, bf16 out
// (SURVEY.md §2.4 N7 "prefill is compute-bound tiles (256² 8-phase template)";
// replaces the external LLM behind J/service/AIInterfaceRestClient.java:37-39).
//
// Two schedules of one 256 x 256 output tile per workgroup, BK = 64, both operands staged
// global -> LDS by LDS-DMA into two 64 KiB buffers (128-B rows; the st_16x32-style XOR
// swizzle slot = chunk ^ ((row >> 1) & 7) applied to the global SOURCE chunk and to the read
// address, rule 21: conflict-free ds_read_b128), v_mfma_f32_16x16x32_bf16 with operands
// swapped (A = W fragment, B = X fragment) so each lane's accumulator holds 4 consecutive
// OUTPUT FEATURES of one token: 8-byte stores, and a fused SwiGLU epilogue in registers when
// the gate|up weight is interleaved in 64-row blocks. XCD-aware, grouped tile order (T1
// bijective remap, then GROUP_M m-tiles per n-tile) so the 32 tiles an XCD runs at once
// share X/W panels in L2.
//   * h4 (default, gemm_tile256_h4_kernel below): 4 waves, one per SIMD, 128 x 128 outputs
//     each in 256 tied AGPRs; four 32-MFMA phases per K-tile with the next tile's DMA and
//     fragment reads between the MFMAs and 3 barriers (details at the kernel);
//   * ping-pong (gemm_tile256_kernel, variants 2 / 3 and the split-K slabs): 8 waves, two
//     per SIMD; every tile split into four 16 KiB regions (X rows 0-127, W rows 0-127, W rows
//     128-255, X rows 128-255) loaded, waited for and recycled one at a time; the K-tile in
//     four (or two, PH2) phases, one per (X half, W half) quadrant; waves 4-7 run one
//     barrier segment behind waves 0-3 so on every SIMD one wave issues its LDS reads + DMA
//     while the other runs its MFMA cluster (s_setprio 1 around it, T5).
// Round 4 measured and deleted three other 4-wave schedules (a 4-stage BK = 32 ring with
// LDS-DMA or register staging, a BK = 64 region ring): 16 x 64-B DMA pieces cost twice the
// memory requests of 8 x 128-B ones and register-staged loads cost as much as LDS-DMA
// (profiles/gemm_tile_pmc_l2_r4.txt, gemm_tile_variants_r4*.jsonl).
// M and N tails are handled by clamped loads and masked stores; K % 64 == 0.
#include "common.h"
#include "kernels.h"

namespace oamd {

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

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

// 16x16x32 bf16 MFMA with the accumulator tied in AGPRs by inline asm: the builtin makes
// hipcc shuffle 256 accumulators through v_accvgpr copies.
__device__ __forceinline__ void mfma_tied(f32x4& acc, const u16x8& a, const u16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// Variant 1, the default ("h4": two buffers, four phases): four waves (one per SIMD, 128 x 128 outputs
// each, 256 tied AGPR accumulators), BK = 64 tiles in two 64 KiB LDS buffers filled by
// LDS-DMA pieces of 8 rows x 128 B (buffer_load ... lds: per-lane 32-bit row offsets fixed
// for the kernel, the K step in soffset) — half the memory requests of 16 x 64-B pieces
// (profiles/gemm_tile_pmc_l2_r4.txt: TCC_HIT 2.2e8 vs 9.9e7, TA_BUSY 2.5x). Tile t (buffer
// t & 1) runs in four 32-MFMA phases:
//   1. k-half 0 from registers A; read k-half 1 (registers B) — the tile's last reads;
//      lgkmcnt(0) + barrier: every wave is done with buffer t & 1
//   2. k-half 0 cont.; 8 W pieces of tile t+2 into buffer t & 1;
//      vmcnt(16) + barrier: tile t+1's W pieces (issued in phase 2 of tile t-1) landed
//   3. k-half 1 from registers B; 8 X pieces of tile t+2; read W of tile t+1, k-half 0;
//      vmcnt(16) + barrier: tile t+1's X pieces landed
//   4. k-half 1 cont.; read X of tile t+1, k-half 0 (registers A) — X last: every MFMA row
//      of the next phase 1 needs all 8 W fragments but only its own X fragment
// so every piece has a whole tile (128 MFMAs per wave) to land, a buffer is refilled only
// after the barrier that follows its last read, and each staged piece is read one phase
// after the wait + barrier that retire it. DMAs and fragment reads sit between MFMAs (one
// per two). LDS image: 128-B rows, chunk slot = chunk ^ ((row >> 1) & 7) on the DMA
// source and the read (conflict-free ds_read_b128). The DMAs carry the sc1
// cache policy (AUX 16: 1-3 % over the default on down / qkv; nt costs 4-20 %,
// profiles/gemm_tile_variants_r4_c.jsonl).
// COLS: the MFMA groups run over W fragments (A operand fixed for 8 MFMAs, as hipBLASLt's
// MT256x256x64 loop does) instead of X fragments; every group then needs all 8 X fragments,
// so the X pieces / fragments of the next tile come first (phases 2-3) and W last.
template <int EPI, int AUX = 16, bool COLS = false>
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
      if constexpr (COLS) mfma_tied(acc[j][i], wf[i], xf[j]);
      else mfma_tied(acc[i][j], wf[j], xf[i]);
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
  for (int tt = 0; tt < 2; ++tt) {   // per tile in the order the loop issues them
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if constexpr (COLS) dma_x(tt, tt, q);
      else dma_w(tt, tt, q);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if constexpr (COLS) dma_w(tt, tt, q);
      else dma_x(tt, tt, q);
    }
  }
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
    // phase 2: rows 4-7 of k-half 0; W pieces of tile t+2 into buffer b
#pragma unroll
    for (int i = 4; i < 8; ++i)
      row(xa, wa, i, [&](int k) {
        if (!(k & 1)) {
          if constexpr (COLS) dma_x(t + 2, b, 2 * (i - 4) + (k >> 1));
          else dma_w(t + 2, b, 2 * (i - 4) + (k >> 1));
        }
      });
    vm_wait<16>();   // tile t+1's W pieces (this wave's)
    seg_barrier();   // ... every wave's
    // phase 3: rows 0-3 of k-half 1; X pieces of tile t+2; W of tile t+1, k-half 0
#pragma unroll
    for (int i = 0; i < 4; ++i)
      row(xb, wb, i, [&](int k) {
        if constexpr (COLS) {
          if (!(k & 1)) dma_w(t + 2, b, 2 * i + (k >> 1));
          else rdx(nb, c0, xa, 2 * i + (k >> 1));
        } else {
          if (!(k & 1)) dma_x(t + 2, b, 2 * i + (k >> 1));
          else rdw(nb, c0, wa, 2 * i + (k >> 1));
        }
      });
    vm_wait<16>();   // tile t+1's X pieces
    seg_barrier();
    // phase 4: rows 4-7 of k-half 1; X of tile t+1, k-half 0
#pragma unroll
    for (int i = 4; i < 8; ++i)
      row(xb, wb, i, [&](int k) {
        if (!(k & 1)) {
          if constexpr (COLS) rdw(nb, c0, wa, 2 * (i - 4) + (k >> 1));
          else rdx(nb, c0, xa, 2 * (i - 4) + (k >> 1));
        }
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

// Variant 5, the persistent "p5" schedule (round 6): the h4 tile (4 waves, 128 x 128 outputs
// per wave in 256 tied AGPRs, BK = 64, two 64 KiB LDS buffers filled by 8-row x 128-B LDS-DMA
// pieces with a source-side chunk swizzle), but
//   * ONE workgroup per CU (grid = min(tiles, CUs)) walking its tiles in rounds: in round r
//     block b takes linear tile r * G + xcd_remap(b, G), and the linear tile goes through the
//     GROUP_M = 8 order, so the 32 tiles an XCD holds at once share X / W panels in its L2;
//   * the LDS-DMA stream is continuous ACROSS tiles: K-step g issues the pieces of step g + 2
//     of the block's flattened (tile, k) stream, so the last two steps of a tile already load
//     the next tile's steps 0 and 1, whose first fragments are in registers when the previous
//     tile's epilogue stores go out (no per-tile prologue fill, no workgroup relaunch);
//   * two barriers and one counted vmcnt per K-step (the h4 loop had three and two):
//       segment A: k-half 0 (64 MFMAs); the 16 fragment reads of k-half 1 ride on its first
//         16 MFMAs; after 40 MFMAs lgkmcnt(0) + barrier (every wave is done with this buffer)
//         and the 8 W pieces of step g + 2 go into it between the last 24;
//       segment B: k-half 1 (64 MFMAs); the 8 X pieces of step g + 2 ride on its first 40;
//         then vmcnt(16) + barrier (step g + 1 landed for every wave) and its k-half-0
//         fragment reads ride on the last 24 MFMAs;
//   * 16-B output stores: the two W fragments of a 32-feature block take interleaved feature
//     rows (fragment jj, row m -> feature 8 (m / 4) + 4 jj + m % 4), so the lane holding
//     accumulator rows 4q .. 4q+3 of both has features 8q .. 8q+7 -- one dwordx4 store per
//     fragment pair, half the store instructions of the 8-B form: a tile's 128 KiB epilogue
//     is bound by store ISSUE (cdna guide T21), and at the prefill shapes it was ~10 % of the
//     kernel (K sweep, profiles/gemm_tile_p5_vs_hipblaslt_r6.jsonl). The chunk swizzle
//     slot ^ (bit1(row) << 1 | bit3(row) << 2) keeps both fragment-read patterns conflict-free;
//   * per-tile buffer resources (base = the tile's first row, num_records = its rows x K x 2):
//     rows past M / N read as zeros, no clamps, no 32-bit limit on the operand size.
// DEEP: which operand streams through THREE LDS buffers (its pieces issued 3 K-steps ahead, two steps
// of flight) -- 0: neither (2 + 2 buffers, 128 KiB), 1: X (narrow N: the X panels come from HBM,
// W stays in the Infinity Cache), 2: W (wide N: the W panels come from HBM); 160 KiB of LDS.
// OPT (A/B arms): bit 0 = s_setprio 1 over the MFMA streams; bit 1 = MFMA groups over W fragments
// (srcA fixed for 8 MFMAs, as hipBLASLt's MT256x256x64 loop issues them)
template <int EPI, int DEEP = 0, int OPT = 0>
__global__ void __launch_bounds__(256) gemm_tile256_p5_kernel(const bf16_t* __restrict__ X,
                                                              const bf16_t* __restrict__ W, bf16_t* __restrict__ Y,
                                                              const bf16_t* __restrict__ bias, int M, int N, int K,
                                                              int ldy, int group_m) {
  constexpr int AUX = 16;
  constexpr int kHalf = 32768;   // one operand of a K-step: 256 rows x 128 B
  __shared__ __attribute__((aligned(1024))) char lds[DEEP ? 5 * kHalf : 4 * kHalf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int mt = (M + kT - 1) / kT, nt = (N + kT - 1) / kT;
  const int ntiles = mt * nt;
  const int G = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G);
  const int T = K / kBK;
  const int gsz = group_m * nt;
  // linear tile of round r -> (m0, n0); false past the last tile
  auto tile_rc = [&](int r, int& m0, int& n0) -> bool {
    const int lid = r * G + slot;
    if (lid >= ntiles) return false;
    const int first_m = (lid / gsz) * group_m;
    const int gm = min(mt - first_m, group_m);
    m0 = (first_m + (lid % gsz) % gm) * kT;
    n0 = ((lid % gsz) / gm) * kT;
    return true;
  };
  // LDS byte offsets of an operand's buffer for K-step (parity p2 = g & 1, p3 = g % 3)
  auto xoff = [&](int p2, int p3) -> int {
    if constexpr (DEEP == 0) return p2 * 2 * kHalf;
    else if constexpr (DEEP == 1) return 2 * kHalf + p3 * kHalf;
    else return p2 * kHalf;
  };
  auto woff = [&](int p2, int p3) -> int {
    if constexpr (DEEP == 0) return p2 * 2 * kHalf + kHalf;
    else if constexpr (DEEP == 2) return 2 * kHalf + p3 * kHalf;
    else return p2 * kHalf;
  };
  auto swz = [](int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); };

  // DMA piece q (0..7) of an operand for wave w = tile rows 8 (w + 4q) .. +7; lane l -> row + l/8,
  // LDS slot l % 8, source chunk slot ^ swz(row). Same offsets for X and W (both K wide).
  const int lrow = lane >> 3, lslot = lane & 7;
  uint32_t vo[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int row = 8 * (w + 4 * q) + lrow;
    vo[q] = ((uint32_t)row * (uint32_t)K + (uint32_t)((lslot ^ swz(row)) * 8)) * 2u;
  }

  // issue cursors: the (tile, k) step whose pieces go out next, per operand. A tile's operand is a
  // buffer resource: base = its first row, num_records = its rows x K x 2 (rows past M / N read as
  // zeros); the resource is rebuilt from (base, bytes) at each use
  struct Cur { int r, kt; const bf16_t* p; int n; };
  Cur cx{0, 0, nullptr, 0}, cw{0, 0, nullptr, 0};
  {
    int m0 = 0, n0 = 0;
    if (!tile_rc(0, m0, n0)) return;   // grid <= tiles: never taken
    cx.p = X + (int64_t)m0 * K;
    cx.n = (int)((uint32_t)min(M - m0, kT) * (uint32_t)K * 2u);
    cw.p = W + (int64_t)n0 * K;
    cw.n = (int)((uint32_t)min(N - n0, kT) * (uint32_t)K * 2u);
  }
  auto advance = [&](Cur& c, bool isx) {
    if (++c.kt == T) {
      int m0n = 0, n0n = 0;
      if (tile_rc(c.r + 1, m0n, n0n)) {
        ++c.r;
        c.kt = 0;
        const int row0 = isx ? m0n : n0n;
        c.p = (isx ? X : W) + (int64_t)row0 * K;
        c.n = (int)((uint32_t)min((isx ? M : N) - row0, kT) * (uint32_t)K * 2u);
      } else {
        c.kt = T - 1;   // past the block's last tile: harmless re-loads of its last step
      }
    }
  };
  // (scalar parameters: hipcc's host pass silently drops the kernel's launch stub when the
  // buffer-resource builtin reads struct members -- an undefined symbol at load time)
  auto dma_ = [&](const bf16_t* cp, int cn, int ckt, int off, int q) {
    char* dst = lds + off + (w + 4 * q) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc((void*)cp, (short)0, cn, 0x00020000),
                                             (__attribute__((address_space(3))) void*)dst, 16, (int)vo[q],
                                             ckt * (kBK * 2), 0, AUX);
  };
  auto dma = [&](const Cur& c, int off, int q) { dma_(c.p, c.n, c.kt, off, q); };

  // fragments: X fragment i = tile rows wm*128 + 16 i + l15; W fragment j (f = j / 4, type =
  // (j / 2) % 2, jj = j % 2) = rows f*128 + type*64 + wn*32 + 8 (l15 / 4) + 4 jj + l15 % 4; k-half h
  // reads chunk 4h + lane/16 of the row at its swizzled slot (swz depends on the lane only)
  const int l15 = lane & 15, lq = lane >> 4;
  const int xs = swz(l15), wr = 8 * (l15 >> 2) + (l15 & 3), ws = swz(wr);
  const int xo0 = (wm * 128 + l15) * 128 + ((lq ^ xs) << 4), xo1 = (wm * 128 + l15) * 128 + (((4 + lq) ^ xs) << 4);
  const int wo0 = (wn * 32 + wr) * 128 + ((lq ^ ws) << 4), wo1 = (wn * 32 + wr) * 128 + (((4 + lq) ^ ws) << 4);
  auto rdx = [&](int off, int h, u16x8 (&xf)[8], int i) {
    xf[i] = *reinterpret_cast<const u16x8*>(lds + off + (h ? xo1 : xo0) + i * 2048);
  };
  auto rdw = [&](int off, int h, u16x8 (&wf)[8], int j) {
    const int r = (j >> 2) * 128 + ((j >> 1) & 1) * 64 + (j & 1) * 4;
    wf[j] = *reinterpret_cast<const u16x8*>(lds + off + (h ? wo1 : wo0) + r * 128);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  asm volatile("s_nop 4");
  u16x8 xa[8], wa[8], xb[8], wb[8];
  constexpr bool kCols = (OPT & 2) != 0;
  // one MFMA row: 8 MFMAs sharing fragment `u` of the per-row set (X fragment i = u, or with
  // kCols W fragment j = u), op(v) after MFMA v
  auto row = [&](const u16x8 (&xf)[8], const u16x8 (&wf)[8], int u, auto op) {
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      if constexpr (kCols) mfma_tied(acc[v][u], wf[u], xf[v]);
      else mfma_tied(acc[u][v], wf[v], xf[u]);
      __builtin_amdgcn_sched_barrier(0);
      op(v);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // fragment reads in row order: the set every row needs (W, or X with kCols) first
  auto rd_all = [&](int ox, int ow, int h, u16x8 (&xf)[8], u16x8 (&wf)[8], int v) {
    if constexpr (kCols) rdx(ox, h, xf, v);
    else rdw(ow, h, wf, v);
  };
  auto rd_row = [&](int ox, int ow, int h, u16x8 (&xf)[8], u16x8 (&wf)[8], int u) {
    if constexpr (kCols) rdw(ow, h, wf, u);
    else rdx(ox, h, xf, u);
  };
  auto none = [](int) {};

  // prologue. DEEP == 0: steps 0 and 1 of both operands (W, X per step). DEEP != 0: shallow 0,
  // deep 0, shallow 1, deep 1, deep 2 -- the order the loop keeps (shallow g+2, deep g+3 per step),
  // so "step g+1 landed" is always "all but the 16 / 24 youngest pieces"
  if constexpr (DEEP == 0) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int q = 0; q < 8; ++q) dma(cw, woff(st, 0), q);
#pragma unroll
      for (int q = 0; q < 8; ++q) dma(cx, xoff(st, 0), q);
      advance(cx, true);
      advance(cw, false);
    }
    vm_wait<16>();
  } else {
    Cur& cs = DEEP == 1 ? cw : cx;   // shallow operand
    Cur& cd = DEEP == 1 ? cx : cw;   // deep operand
    auto soff = [&](int st) { return DEEP == 1 ? woff(st & 1, st % 3) : xoff(st & 1, st % 3); };
    auto doff = [&](int st) { return DEEP == 1 ? xoff(st & 1, st % 3) : woff(st & 1, st % 3); };
#pragma unroll
    for (int st = 0; st < 2; ++st) {
#pragma unroll
      for (int q = 0; q < 8; ++q) dma(cs, soff(st), q);
      advance(cs, DEEP == 2);
#pragma unroll
      for (int q = 0; q < 8; ++q) dma(cd, doff(st), q);
      advance(cd, DEEP == 1);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(cd, doff(2), q);
    advance(cd, DEEP == 1);
    vm_wait<24>();
  }
  seg_barrier();
#pragma unroll
  for (int v = 0; v < 8; ++v) rd_all(xoff(0, 0), woff(0, 0), 0, xa, wa, v);
#pragma unroll
  for (int u = 0; u < 8; ++u) rd_row(xoff(0, 0), woff(0, 0), 0, xa, wa, u);

  int g = 0, p3 = 0;   // flattened step counter (buffer parity) and g % 3
  int m0 = 0, n0 = 0;
  for (int r = 0; tile_rc(r, m0, n0); ++r) {
    for (int t = 0; t < T; ++t, ++g) {
      const int p2 = g & 1, n2 = p2 ^ 1, n3 = p3 == 2 ? 0 : p3 + 1;
      const int ox = xoff(p2, p3), ow = woff(p2, p3);          // this step's buffers
      const int nox = xoff(n2, n3), now_ = woff(n2, n3);       // step g + 1's
      // ---- segment A: k-half 0 from A; k-half 1 reads (row 0, row 1); this step's buffers released
      if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(1);
      asm volatile("s_waitcnt lgkmcnt(7)" ::: "memory");   // the 8 shared + row 0's fragment
      __builtin_amdgcn_sched_barrier(0);
      row(xa, wa, 0, [&](int v) { rd_all(ox, ow, 1, xb, wb, v); });
      asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory");  // + row 1's
      __builtin_amdgcn_sched_barrier(0);
      row(xa, wa, 1, [&](int v) { rd_row(ox, ow, 1, xb, wb, v); });
      asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");  // every k-half-0 read of the step
      __builtin_amdgcn_sched_barrier(0);
      row(xa, wa, 2, none);
      row(xa, wa, 3, none);
      row(xa, wa, 4, none);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(0);
      seg_barrier();   // every wave is done reading this step's buffers
      if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(1);
      // DEEP == 0: W of step g+2 here, X of step g+2 in segment B (both into this step's buffers);
      // DEEP != 0: the shallow operand of step g+2 here, the deep one of step g+3 in segment B
#pragma unroll
      for (int i = 5; i < 8; ++i)
        row(xa, wa, i, [&](int j) {
          const int m = (i - 5) * 8 + j;
          if (m % 3 == 0) {
            if constexpr (DEEP == 1) dma(cw, ow, m / 3);
            else if constexpr (DEEP == 2) dma(cx, ox, m / 3);
            else dma(cw, ow, m / 3);
          }
        });
      // ---- segment B: k-half 1 from B; then step g + 1 lands
#pragma unroll
      for (int i = 0; i < 5; ++i)
        row(xb, wb, i, [&](int j) {
          const int m = i * 8 + j;
          if (m % 5 == 0) {
            if constexpr (DEEP == 1) dma(cx, ox, m / 5);
            else if constexpr (DEEP == 2) dma(cw, ow, m / 5);
            else dma(cx, ox, m / 5);
          }
        });
      advance(cx, true);
      advance(cw, false);
      if constexpr (DEEP == 0) vm_wait<16>();   // this wave's pieces of step g + 1
      else vm_wait<24>();
      if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(0);
      seg_barrier();   // ... every wave's
      if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 5; i < 8; ++i)
        row(xb, wb, i, [&](int j) {
          const int m = (i - 5) * 8 + j;   // 16 reads on 24 MFMAs: the shared 8, then the per-row 8
          if (m % 3 != 2) {
            const int k = m - m / 3;
            if (k < 8) rd_all(nox, now_, 0, xa, wa, k);
            else rd_row(nox, now_, 0, xa, wa, k - 8);
          }
        });
      p3 = n3;
    }
    if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(0);

    // ---- epilogue of the tile (the next tile's step 0 is in registers / flight); lane holds
    // features 8 lq .. 8 lq + 7 of each 32-feature block (fragments jj = 0, 1) of token l15
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    f32x4 bv[2][2][2];   // bias of this lane's features per (f, type, jj): independent of the token block
    if constexpr (EPI == kEpiBias) {
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int ty = 0; ty < 2; ++ty) {
          const int col = min(n0 + f * 128 + ty * 64 + wn * 32 + 8 * lq, N - 8);
          const uint4 bb = *reinterpret_cast<const uint4*>(bias + col);
          bv[f][ty][0] = f32x4{__uint_as_float(bb.x << 16), __uint_as_float(bb.x & 0xffff0000u),
                               __uint_as_float(bb.y << 16), __uint_as_float(bb.y & 0xffff0000u)};
          bv[f][ty][1] = f32x4{__uint_as_float(bb.z << 16), __uint_as_float(bb.z & 0xffff0000u),
                               __uint_as_float(bb.w << 16), __uint_as_float(bb.w & 0xffff0000u)};
        }
    }
    auto store8 = [&](bf16_t* yrow, int col, bool ok, f32x4 v0, f32x4 v1) {
      if (ok)
        *reinterpret_cast<uint4*>(yrow + col) =
            make_uint4(pack_bf2(v0[0], v0[1]), pack_bf2(v0[2], v0[3]), pack_bf2(v1[0], v1[1]), pack_bf2(v1[2], v1[3]));
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int tok = m0 + wm * 128 + i * 16 + l15;
      bf16_t* yrow = Y + (int64_t)tok * ldy;
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        if constexpr (EPI == kEpiSilu) {
          f32x4 o[2];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const f32x4 gt = acc[i][f * 4 + jj], up = acc[i][f * 4 + 2 + jj];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
              const float gg = bf2f(f2bf(gt[rr]));
              const float uu = bf2f(f2bf(up[rr]));
              const float sg = bf2f(f2bf(gg / (1.f + __expf(-gg))));
              o[jj][rr] = sg * uu;
            }
          }
          const int col = (n0 >> 1) + f * 64 + wn * 32 + 8 * lq;
          store8(yrow, col, tok < M && 2 * col < N, o[0], o[1]);
        } else {
#pragma unroll
          for (int ty = 0; ty < 2; ++ty) {
            f32x4 v0 = acc[i][f * 4 + ty * 2], v1 = acc[i][f * 4 + ty * 2 + 1];
            if constexpr (EPI == kEpiBias) {
              v0 += bv[f][ty][0];
              v1 += bv[f][ty][1];
            }
            const int col = n0 + f * 128 + ty * 64 + wn * 32 + 8 * lq;
            store8(yrow, col, tok < M && col < N, v0, v1);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+a"(acc[i][j]));
      }
    asm volatile("s_nop 4");
  }
  vm_wait<0>();   // the trailing re-loads land before the workgroup's LDS is released
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

template <int DEEP>
static void launch_p5(const bf16_t* X, const bf16_t* W, bf16_t* Y, const bf16_t* bias, int M, int N, int K, int ldy,
                      bool silu_gu, int grid, hipStream_t stream, int gm = kGroupM) {
  if (silu_gu) gemm_tile256_p5_kernel<kEpiSilu, DEEP><<<grid, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, gm);
  else if (bias) gemm_tile256_p5_kernel<kEpiBias, DEEP><<<grid, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, gm);
  else gemm_tile256_p5_kernel<kEpiStore, DEEP><<<grid, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, gm);
}

// compute units of the current device (persistent grids), cached per device
static int device_cus() {
  static int cus[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
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
  const bool st16 = ldy % 8 == 0 && reinterpret_cast<uintptr_t>(Y) % 16 == 0;   // p5's 16-B stores
  // persistent p5 (variant 5; the default past 256 rows): one workgroup per CU; wide N (>= 16384:
  // gate|up, the W panels stream from HBM) gives W a third LDS buffer -- a 2-step prefetch
  // (M = 32k, N = 28672: 5786 -> 5366 us; at N = 4096 / 6144 the 2-buffer form is faster,
  // profiles/gemm_tile_p5_vs_hipblaslt_r6.jsonl)
  if ((variant == 5 || (variant == 0 && M > kT)) && K >= 2 * kBK && st16) {
    const int grid = min(nwg, device_cus());
    // GROUP_M 4 for the narrow projections (M = 32k, N = 6144: 1106 vs 1145 us at GROUP_M 8; N = 4096
    // equal; 16 / 32 slower: profiles/gemm_tile_p5_vs_hipblaslt_r6.jsonl)
    if (N >= 16384) launch_p5<2>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 4);   // GROUP_M 4: -1.1 / -1.4 % at M = 12k / 32k
    else launch_p5<0>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 4);
  } else if (variant >= 6 && variant <= 14 && K >= 2 * kBK && st16) {   // p5 A/B arms (timing, same numerics)
    const int grid = min(nwg, device_cus());
    if (variant == 6) launch_p5<0>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 4);         // GROUP_M 4
    else if (variant == 7) launch_p5<0>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 16);   // GROUP_M 16
    else if (variant == 8) launch_p5<2>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream);       // W third buffer
    else if (variant == 10) launch_p5<2>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 4);   // W third, GROUP_M 4
    else if (variant == 11) launch_p5<2>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 16);  // W third, GROUP_M 16
    else if (variant == 12) launch_p5<2>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 2);   // W third, GROUP_M 2
    else if (variant == 13) launch_p5<1>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 4);   // X third, GROUP_M 4
    else if (variant == 14) launch_p5<0>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 2);   // GROUP_M 2
    else launch_p5<0>(X, W, Y, bias, M, N, K, ldy, silu_gu, grid, stream, 32);                      // GROUP_M 32
  } else if ((variant == 0 || variant == 1) && off32) {   // 4-wave, two 64 KiB buffers, four phases per K-tile
    if (silu_gu) gemm_tile256_h4_kernel<kEpiSilu><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (bias) gemm_tile256_h4_kernel<kEpiBias><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_h4_kernel<kEpiStore><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if (variant == 4 && off32) {   // h4 with W-fragment MFMA groups (timing)
    if (silu_gu) gemm_tile256_h4_kernel<kEpiSilu, 16, true><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else if (bias) gemm_tile256_h4_kernel<kEpiBias, 16, true><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
    else gemm_tile256_h4_kernel<kEpiStore, 16, true><<<nwg, 256, 0, stream>>>(X, W, Y, bias, M, N, K, ldy);
  } else if (variant == 2 || (variant == 0 && M > 256)) {
    // 8-wave ping-pong, two barrier segments per K-tile (the round-3 default; 2-8 % behind
    // variant 1 on the prefill shapes, profiles/gemm_tile_h4_vs_ph2_m32k.jsonl); also the
    // fallback for operands past 32-bit offsets
    if (silu_gu) gemm_tile256_kernel<kEpiSilu, true><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
    else if (bias) gemm_tile256_kernel<kEpiBias, true><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
    else gemm_tile256_kernel<kEpiStore, true><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
  } else {   // 8-wave ping-pong, four segments per K-tile (variant 3, or 0 at M <= 256 past 32-bit offsets)
    if (silu_gu) gemm_tile256_kernel<kEpiSilu><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
    else if (bias) gemm_tile256_kernel<kEpiBias><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
    else gemm_tile256_kernel<kEpiStore><<<nwg, 512, 0, stream>>>(X, W, Y, bias, M, N, K, ldy, nullptr);
  }
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
