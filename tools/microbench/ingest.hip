// Per-CU ingest ceilings of the M = 256 decode GEMM (gate|up shape: X [256, 4096] bf16,
// L2-resident; W [28672, 4096] bf16 streamed cold from HBM). Not production code: a
// diagnostic that times the pieces of gemm_pp's K-loop in isolation on one MI355X --
// LDS-DMA of the X and/or W regions only (no MFMA), MFMA on LDS only (no loads), and both
// -- so the decode GEMM's limiter can be read off directly.
//   hipcc --offload-arch=gfx950 -O3 -o ingest ingest.hip && ./ingest
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kRegion = 16384;  // 128 rows x 64 k bf16

template <int N>
__device__ __forceinline__ void vmw() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// NX X regions (128 token rows each) + NW W regions (128 weight rows each) per K-tile,
// NBUF K-tiles of LDS ring; LOADS / MFMA switch the two halves of the work on and off.
template <int NBUF, int NX, int NW, bool LOADS, bool MFMA, bool NT>
__global__ void __launch_bounds__(512) ingest_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                     int K, float* __restrict__ sink) {
  constexpr int NR = NX + NW;
  constexpr int BUF = NR * kRegion;
  __shared__ __attribute__((aligned(1024))) char lds[NBUF * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = blockIdx.x * 128 * (NW > 0 ? NW : 1);
  const int T = K / 64;
  const int lrow = lane >> 3, lslot = lane & 7;
  const uint16_t* src[4][2];   // fixed size: a template-sized array here drops the launch stub (hipcc 7.2)
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 8 * (w + 8 * i) + lrow;
      const int chunk = lslot ^ ((row >> 1) & 7);
      if (r < NX) src[r][i] = X + (int64_t)(r * 128 + row) * K + chunk * 8;
      else src[r][i] = W + (int64_t)(n0 + (r - NX) * 128 + row) * K + chunk * 8;
    }
  auto issue = [&](int buf, int kt) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      char* dst = lds + buf * BUF + r * kRegion;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (NT && r >= NX)
          __builtin_amdgcn_global_load_lds(src[r][i] + kt * 64, (__attribute__((address_space(3))) void*)(dst + (w + 8 * i) * 1024), 16, 0, 2);
        else
          __builtin_amdgcn_global_load_lds(src[r][i] + kt * 64, (__attribute__((address_space(3))) void*)(dst + (w + 8 * i) * 1024), 16, 0, 0);
      }
    }
  };
  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int g = w >> 2, wc = w & 3;
  f32x4 acc[NX > 0 ? NX : 1][4][2];
#pragma unroll
  for (int h = 0; h < (NX > 0 ? NX : 1); ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[h][b][0] = acc[h][b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const char* cur) {
    u16x8 xf[NX > 0 ? NX : 1][4][2], wf[2][2];
#pragma unroll
    for (int h = 0; h < (NX > 0 ? NX : 1); ++h)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          xf[h][b][s] = *reinterpret_cast<const u16x8*>(cur + h * kRegion + (g * 64 + b * 16 + l15) * 128 +
                                                       (((4 * s + lq) ^ sw) << 4));
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        wf[e][s] = *reinterpret_cast<const u16x8*>(cur + NX * kRegion + (e * 64 + wc * 16 + l15) * 128 +
                                                  (((4 * s + lq) ^ sw) << 4));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int h = 0; h < (NX > 0 ? NX : 1); ++h)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int e = 0; e < 2; ++e)
            acc[h][b][e] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[e][s]),
                                                                   __builtin_bit_cast(bf16x8_t, xf[h][b][s]),
                                                                   acc[h][b][e], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  if (LOADS) {
#pragma unroll
    for (int p = 0; p < NBUF - 1; ++p)
      if (p < T) issue(p, p);
  }
  for (int t = 0; t < T; ++t) {
    if (LOADS) {
      if (t + NBUF - 2 < T) vmw<(NBUF - 2) * NR * 2>(); else vmw<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (LOADS && t + NBUF - 1 < T) issue((t + NBUF - 1) % NBUF, t + NBUF - 1);
    if (MFMA) compute(lds + (t % NBUF) * BUF);
  }
  float s = 0.f;
#pragma unroll
  for (int h = 0; h < (NX > 0 ? NX : 1); ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) s += acc[h][b][0][0] + acc[h][b][1][3];
  if (!MFMA) s = reinterpret_cast<const float*>(lds)[tid];
  sink[blockIdx.x * 512 + tid] = s;
}

__device__ __forceinline__ void vm_wait_n(int n) {
  switch (n) {
    case 0: vmw<0>(); break;
    case 4: vmw<4>(); break;
    case 8: vmw<8>(); break;
    case 12: vmw<12>(); break;
    case 16: vmw<16>(); break;
    case 24: vmw<24>(); break;
    default: vmw<0>(); break;
  }
}

// Wave-specialised loaders: waves 0-3 stream W (one 16 KiB region per K-tile, NW-deep
// ring: NW-1 tiles issued ahead), waves 4-7 stream X (two 16 KiB regions per K-tile,
// NX-deep ring). vmcnt is in order per wave, so a W wave never waits for X loads issued
// after its W loads and vice versa: the W prefetch depth is independent of X's.
template <int NW, int NX, bool LOADS, bool MFMA>
__global__ void __launch_bounds__(512) spec_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                   int K, float* __restrict__ sink) {
  constexpr int WBUF = kRegion, XBUF = 2 * kRegion;
  __shared__ __attribute__((aligned(1024))) char lds[NW * WBUF + NX * XBUF];
  char* wl = lds;
  char* xl = lds + NW * WBUF;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool wwave = w < 4;
  const int wi = w & 3;
  const int n0 = blockIdx.x * 128;
  const int T = K / 64;
  const int lrow = lane >> 3, lslot = lane & 7;
  // W wave wi: pieces q = 0..3 -> rows 8 (wi + 4 q) + lrow; X wave: region r, pieces q = 0..3
  const uint16_t* wsrc[4];
  const uint16_t* xsrc[2][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = 8 * (wi + 4 * q) + lrow;
    const int chunk = lslot ^ ((row >> 1) & 7);
    wsrc[q] = W + (int64_t)(n0 + row) * K + chunk * 8;
#pragma unroll
    for (int r = 0; r < 2; ++r) xsrc[r][q] = X + (int64_t)(r * 128 + row) * K + chunk * 8;
  }
  auto issue_w = [&](int kt) {
    char* dst = wl + (kt % NW) * WBUF;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(wsrc[q] + kt * 64, (__attribute__((address_space(3))) void*)(dst + (wi + 4 * q) * 1024), 16, 0, 2);
  };
  auto issue_x = [&](int kt) {
    char* dst = xl + (kt % NX) * XBUF;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds(xsrc[r][q] + kt * 64,
                                         (__attribute__((address_space(3))) void*)(dst + r * kRegion + (wi + 4 * q) * 1024), 16, 0, 0);
  };
  const int l15 = lane & 15, lq = lane >> 4, sw = (l15 >> 1) & 7;
  const int g = w >> 2, wc = w & 3;
  f32x4 acc[2][4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[h][b][0] = acc[h][b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const char* xc, const char* wc_) {
    u16x8 xf[2][4][2], wf[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          xf[h][b][s] = *reinterpret_cast<const u16x8*>(xc + h * kRegion + (g * 64 + b * 16 + l15) * 128 + (((4 * s + lq) ^ sw) << 4));
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        wf[e][s] = *reinterpret_cast<const u16x8*>(wc_ + (e * 64 + wc * 16 + l15) * 128 + (((4 * s + lq) ^ sw) << 4));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
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
    __builtin_amdgcn_sched_barrier(0);
  };
  if (LOADS) {
    if (wwave) {
      for (int p = 0; p < NW - 1 && p < T; ++p) issue_w(p);
    } else {
      for (int p = 0; p < NX - 1 && p < T; ++p) issue_x(p);
    }
  }
  for (int t = 0; t < T; ++t) {
    if (LOADS) {
      if (wwave) vm_wait_n(4 * min(NW - 2, T - 1 - t));
      else vm_wait_n(8 * min(NX - 2, T - 1 - t));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (LOADS) {
      if (wwave) {
        if (t + NW - 1 < T) issue_w(t + NW - 1);
      } else {
        if (t + NX - 1 < T) issue_x(t + NX - 1);
      }
    }
    if (MFMA) compute(xl + (t % NX) * XBUF, wl + (t % NW) * WBUF);
  }
  float s = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int b = 0; b < 4; ++b) s += acc[h][b][0][0] + acc[h][b][1][3];
  if (!MFMA) s = reinterpret_cast<const float*>(lds)[tid];
  sink[blockIdx.x * 512 + tid] = s;
}

template <int NW, int NX, bool LOADS, bool MFMA>
int run_spec(const char* name, int grid, const uint16_t* X, const std::vector<uint16_t*>& Ws, int K, float* sink) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto launch = [&](int i) { spec_kernel<NW, NX, LOADS, MFMA><<<grid, 512>>>(X, Ws[i % Ws.size()], K, sink); };
  for (int i = 0; i < 6; ++i) launch(i);
  CK(hipDeviceSynchronize());
  const int iters = 30;
  std::vector<float> ts;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch(i);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms * 1000.f / iters);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[2];
  const double bytes_per_wg = 3.0 * kRegion * (K / 64);
  printf("{\"variant\": \"%s\", \"grid\": %d, \"w_ring\": %d, \"x_ring\": %d, \"loads\": %d, \"mfma\": %d, \"us\": %.2f, "
         "\"ingest_gb_s_per_cu\": %.1f, \"w_tb_s\": %.2f}\n",
         name, grid, NW, NX, (int)LOADS, (int)MFMA, us, LOADS ? bytes_per_wg / us / 1e3 : 0.0,
         LOADS ? (double)grid * kRegion * (K / 64) / us / 1e6 : 0.0);
  fflush(stdout);
  return 0;
}

template <int NBUF, int NX, int NW, bool LOADS, bool MFMA, bool NT>
int run(const char* name, int grid, const uint16_t* X, const std::vector<uint16_t*>& Ws, int K, float* sink) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto launch = [&](int i) {
    ingest_kernel<NBUF, NX, NW, LOADS, MFMA, NT><<<grid, 512>>>(X, Ws[i % Ws.size()], K, sink);
  };
  for (int i = 0; i < 6; ++i) launch(i);
  CK(hipDeviceSynchronize());
  const int iters = 30;
  std::vector<float> ts;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch(i);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms * 1000.f / iters);
  }
  std::sort(ts.begin(), ts.end());
  const double us = ts[2];
  const double bytes_per_wg = (double)(NX + NW) * kRegion * (K / 64);
  printf("{\"variant\": \"%s\", \"grid\": %d, \"nbuf\": %d, \"x_regions\": %d, \"w_regions\": %d, \"loads\": %d, "
         "\"mfma\": %d, \"nt\": %d, \"us\": %.2f, \"ingest_gb_s_per_cu\": %.1f, \"w_tb_s\": %.2f}\n",
         name, grid, NBUF, NX, NW, (int)LOADS, (int)MFMA, (int)NT, us, LOADS ? bytes_per_wg / us / 1e3 : 0.0,
         LOADS && NW ? (double)grid * NW * kRegion * (K / 64) / us / 1e6 : 0.0);
  fflush(stdout);
  return 0;
}

// uniform-ish random bf16 in [-1, 1) from a hash (constant operands inflate MFMA clocks:
// cdna_hip_programming.md §5.4 rule 25)
__global__ void fill_random(uint16_t* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    const float f = ((h & 0xffffff) / 16777216.f * 2.f - 1.f) * scale;
    p[i] = (uint16_t)(__float_as_uint(f) >> 16);
  }
}

int main() {
  const int K = 4096, N = 28672, M = 256;
  uint16_t* X;
  CK(hipMalloc(&X, (size_t)M * K * 2));
  fill_random<<<1024, 256>>>(X, (size_t)M * K, 1u, 1.f);
  std::vector<uint16_t*> Ws(3);
  for (auto& w : Ws) {
    CK(hipMalloc(&w, (size_t)N * K * 2));
    fill_random<<<4096, 256>>>(w, (size_t)N * K, 7u, 0.05f);
  }
  float* sink;
  CK(hipMalloc(&sink, 512 * 512 * 4));
  // the gate|up tile of gemm_pp (2 X regions + 1 W region per K-tile, 3-deep ring), 224 workgroups
  run<3, 2, 1, true, false, true>("loads_x2w1", 224, X, Ws, K, sink);
  run<3, 0, 1, true, false, true>("loads_w1", 224, X, Ws, K, sink);
  run<3, 2, 0, true, false, true>("loads_x2", 224, X, Ws, K, sink);
  run<3, 2, 1, false, true, true>("mfma_only", 224, X, Ws, K, sink);
  run<3, 2, 1, true, true, true>("loads_x2w1+mfma", 224, X, Ws, K, sink);

  // wave-specialised loaders (waves 0-3 W, 4-7 X), independent ring depths
  run_spec<3, 2, true, false>("spec_w3x2_loads", 224, X, Ws, K, sink);
  run_spec<4, 2, true, false>("spec_w4x2_loads", 224, X, Ws, K, sink);
  run_spec<6, 2, true, false>("spec_w6x2_loads", 224, X, Ws, K, sink);
  run_spec<4, 3, true, false>("spec_w4x3_loads", 224, X, Ws, K, sink);
  run_spec<4, 2, true, true>("spec_w4x2_loads+mfma", 224, X, Ws, K, sink);
  run_spec<6, 2, true, true>("spec_w6x2_loads+mfma", 224, X, Ws, K, sink);
  run_spec<4, 3, true, true>("spec_w4x3_loads+mfma", 224, X, Ws, K, sink);
  return 0;
}
