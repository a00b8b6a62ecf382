// Paged KV streaming probe (decides the decode-attention load path, csrc/kernels/attn_decode.hip):
// how fast can the flagship's decode KV (B = 256 sequences x 8 kv heads, ~1.15k tokens, 64-token
// pages, bf16 [pages][Hkv][64][128] K and V, shuffled page table) be read, with the same work
// split as the kernel (workgroup = one (sequence, kv-head) item, 4 waves, wave w reads tokens
// 16w..16w+15 of every 64-token page = 4 KB of K + 4 KB of V) and a minimal consumer (XOR of
// every dword, so no load is dead)?
//   mode 0  register loads (nontemporal), double-buffered        = today's kernel
//   mode 1  LDS-DMA (global_load_lds, nt), per-wave ring of S slots of 8 KB, counted vmcnt
//   mode 2  mode 0, persistent: grid = CUs x 3, each wave streams its workgroup's items back to
//           back (no per-item prologue / launch tail)
// Build: hipcc -O3 --offload-arch=gfx950 -o kv_stream tools/probe/kv_stream.hip
// Run:   ./kv_stream   (prints one JSON line per mode: us per pass, TB/s of KV bytes)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kHkv = 8, kPage = 64, kD = 128;
constexpr int kPageHeadBytes = kPage * kD * 2;  // 16 KB of K (or V) per page and kv head

__device__ __forceinline__ u32x4 ldnt(const char* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// ---- mode 0: register loads, one item per workgroup --------------------------------------
__global__ void __launch_bounds__(256, 3) stream_reg(const char* __restrict__ kc, const char* __restrict__ vc,
                                                     const int* __restrict__ bt, const int* __restrict__ lens,
                                                     int max_pages, unsigned* __restrict__ out, int head_major = 0,
                                                     int work = 0) {
  const int B = gridDim.x / kHkv;
  const int item = blockIdx.x;
  const int b = head_major ? item % B : item / kHkv, h = head_major ? item / B : item % kHkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = lens[b] / kPage;
  const int64_t hoff = (int64_t)h * kPageHeadBytes + w * 4096 + lane * 16;
  const int64_t pstride = (int64_t)kHkv * kPageHeadBytes;
  u32x4 a[8], c[8];
  unsigned acc = 0;
  auto load = [&](u32x4 (&r)[8], int ch) {
    const int64_t base = (int64_t)bt[b * max_pages + ch] * pstride + hoff;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = ldnt(kc + base + j * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) r[4 + j] = ldnt(vc + base + j * 1024);
  };
  float f = (float)lane;
  auto use = [&](const u32x4 (&r)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= r[j][0] ^ r[j][1] ^ r[j][2] ^ r[j][3];
    // synthetic per-chunk compute: a dependent chain of `work` exp/fma pairs (the
    // attention consume is a dependent MFMA -> softmax -> P.V chain of this kind)
    f += (float)(acc & 1u);
    for (int k = 0; k < work; ++k) f = __expf(f * 0.999f) * 0.5f;
  };
  load(a, 0);
  for (int ch = 0; ch < nch; ch += 2) {
    load(c, min(ch + 1, nch - 1));
    use(a);
    load(a, min(ch + 2, nch - 1));
    if (ch + 1 < nch) use(c);
  }
  if (acc == 0x12345678u || f == 1.2345f) out[item] = acc;
}

// ---- mode 1: LDS-DMA into a per-wave ring of S 8-KB slots ---------------------------------
template <int S>
__global__ void __launch_bounds__(256) stream_lds(const char* __restrict__ kc, const char* __restrict__ vc,
                                                  const int* __restrict__ bt, const int* __restrict__ lens,
                                                  int max_pages, unsigned* __restrict__ out) {
  __shared__ __attribute__((aligned(1024))) char ring[4][S][8192];
  const int item = blockIdx.x, b = item / kHkv, h = item % kHkv;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = lens[b] / kPage;
  const int64_t hoff = (int64_t)h * kPageHeadBytes + w * 4096 + lane * 16;
  const int64_t pstride = (int64_t)kHkv * kPageHeadBytes;
  unsigned acc = 0;
  auto issue = [&](int ch) {   // always 8 instructions (past the end: re-issue the last page)
    const int64_t base = (int64_t)bt[b * max_pages + min(ch, nch - 1)] * pstride + hoff;
    char* dst = ring[w][ch % S];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(kc + base + j * 1024, (__attribute__((address_space(3))) void*)(dst + j * 1024),
                                       16, 0, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(vc + base + j * 1024,
                                       (__attribute__((address_space(3))) void*)(dst + 4096 + j * 1024), 16, 0, 2);
  };
#pragma unroll
  for (int s = 0; s < S; ++s) issue(s);
  for (int ch = 0; ch < nch; ++ch) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (S - 1)) : "memory");   // chunk ch landed
    const char* src = ring[w][ch % S];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(src + j * 1024 + lane * 16);
      acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // slot read before it is refilled
    issue(ch + S);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x12345678u) out[item] = acc;
}

// ---- mode 1b: LDS-DMA ring with the consumer's compute after the refill ---------------------
// per chunk: wait for the slot, copy it to registers (ds_read), refill the slot with chunk
// c + S (DMA in flight during the compute), then a `work`-long dependent compute chain
template <int S, int OCC>
__global__ void __launch_bounds__(256, OCC) stream_lds_compute(const char* __restrict__ kc,
                                                               const char* __restrict__ vc,
                                                               const int* __restrict__ bt,
                                                               const int* __restrict__ lens, int max_pages,
                                                               unsigned* __restrict__ out, int work) {
  __shared__ __attribute__((aligned(1024))) char ring[4][S][8192];
  const int item = blockIdx.x, b = item / kHkv, h = item % kHkv;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nch = lens[b] / kPage;
  const int64_t hoff = (int64_t)h * kPageHeadBytes + w * 4096 + lane * 16;
  const int64_t pstride = (int64_t)kHkv * kPageHeadBytes;
  unsigned acc = 0;
  float f = (float)lane;
  auto issue = [&](int ch) {
    const int64_t base = (int64_t)bt[b * max_pages + min(ch, nch - 1)] * pstride + hoff;
    char* dst = ring[w][ch % S];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(kc + base + j * 1024, (__attribute__((address_space(3))) void*)(dst + j * 1024),
                                       16, 0, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(vc + base + j * 1024,
                                       (__attribute__((address_space(3))) void*)(dst + 4096 + j * 1024), 16, 0, 2);
  };
#pragma unroll
  for (int s = 0; s < S; ++s) issue(s);
  for (int ch = 0; ch < nch; ++ch) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (S - 1)) : "memory");
    const char* src = ring[w][ch % S];
    u32x4 r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = *reinterpret_cast<const u32x4*>(src + j * 1024 + lane * 16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    issue(ch + S);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= r[j][0] ^ r[j][1] ^ r[j][2] ^ r[j][3];
    f += (float)(acc & 1u);
    for (int k = 0; k < work; ++k) f = __expf(f * 0.999f) * 0.5f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x12345678u || f == 1.2345f) out[item] = acc;
}

// ---- mode 2: persistent register streaming ------------------------------------------------
__global__ void __launch_bounds__(256, 3) stream_persist(const char* __restrict__ kc, const char* __restrict__ vc,
                                                         const int* __restrict__ bt, const int* __restrict__ lens,
                                                         int max_pages, int n_items, unsigned* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t pstride = (int64_t)kHkv * kPageHeadBytes;
  // flattened stream of (item, chunk) for this workgroup: items blockIdx.x + k * gridDim.x
  int it = blockIdx.x;
  if (it >= n_items) return;
  int ch = 0, nch = lens[it / kHkv] / kPage;
  auto adv = [&](int& i, int& c, int& n) -> bool {   // next position; false at the end
    if (++c < n) return true;
    i += gridDim.x;
    if (i >= n_items) return false;
    c = 0;
    n = lens[i / kHkv] / kPage;
    return true;
  };
  auto load = [&](u32x4 (&r)[8], int i, int c) {
    const int bb = i / kHkv, hh = i % kHkv;
    const int64_t base = (int64_t)bt[bb * max_pages + c] * pstride + (int64_t)hh * kPageHeadBytes + w * 4096 + lane * 16;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = ldnt(kc + base + j * 1024);
#pragma unroll
    for (int j = 0; j < 4; ++j) r[4 + j] = ldnt(vc + base + j * 1024);
  };
  unsigned acc = 0;
  auto use = [&](const u32x4 (&r)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= r[j][0] ^ r[j][1] ^ r[j][2] ^ r[j][3];
  };
  u32x4 a[8], c[8];
  int li = it, lc = ch, ln = nch;   // load position (one chunk ahead)
  load(a, li, lc);
  bool more = adv(li, lc, ln);
  while (true) {
    if (more) load(c, li, lc);
    use(a);
    if (!more) break;
    more = adv(li, lc, ln);
    if (more) load(a, li, lc);
    use(c);
    if (!more) break;
    more = adv(li, lc, ln);
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  const int B = 256, n_items = B * kHkv;
  std::mt19937 rng(0);
  std::vector<int> lens(B);
  int64_t tokens = 0;
  int max_pages = 0;
  for (int b = 0; b < B; ++b) {
    lens[b] = (15 + (int)(rng() % 7)) * kPage;   // 960..1344 tokens (~1.15k mean, +-15 %)
    tokens += lens[b];
    max_pages = std::max(max_pages, lens[b] / kPage);
  }
  const int total_pages = B * max_pages + 8;
  std::vector<int> perm(total_pages);
  for (int i = 0; i < total_pages; ++i) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<int> bt(B * max_pages);
  for (int i = 0; i < B * max_pages; ++i) bt[i] = perm[i];
  const size_t cache_bytes = (size_t)total_pages * kHkv * kPageHeadBytes;
  char *kc, *vc;
  int *dbt, *dlens;
  unsigned* out;
  CK(hipMalloc(&kc, cache_bytes));
  CK(hipMalloc(&vc, cache_bytes));
  CK(hipMemset(kc, 1, cache_bytes));
  CK(hipMemset(vc, 2, cache_bytes));
  CK(hipMalloc(&dbt, bt.size() * 4));
  CK(hipMalloc(&dlens, B * 4));
  CK(hipMalloc(&out, n_items * 4));
  CK(hipMemcpy(dbt, bt.data(), bt.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlens, lens.data(), B * 4, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double bytes = (double)tokens * kHkv * kD * 2 * 2;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int n = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < n; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / n;
    printf("{\"mode\": \"%s\", \"B\": %d, \"mean_ctx\": %.0f, \"us\": %.1f, \"TBps\": %.3f}\n", name, B,
           (double)tokens / B, us, bytes / us / 1e6);
    fflush(stdout);
  };
  timeit("reg_per_item", [&] { stream_reg<<<n_items, 256>>>(kc, vc, dbt, dlens, max_pages, out); });
  timeit("reg_per_item_head_major", [&] { stream_reg<<<n_items, 256>>>(kc, vc, dbt, dlens, max_pages, out, 1); });
  for (int work : {16, 64, 256}) {
    char name[64];
    snprintf(name, sizeof(name), "reg_per_item_compute%d", work);
    timeit(name, [&] { stream_reg<<<n_items, 256>>>(kc, vc, dbt, dlens, max_pages, out, 0, work); });
  }
  for (int work : {0, 64, 128}) {
    char name[64];
    snprintf(name, sizeof(name), "lds_dma_ring2_occ2_compute%d", work);
    timeit(name, [&] { stream_lds_compute<2, 2><<<n_items, 256>>>(kc, vc, dbt, dlens, max_pages, out, work); });
    snprintf(name, sizeof(name), "lds_dma_ring3_occ1_compute%d", work);
    timeit(name, [&] { stream_lds_compute<3, 1><<<n_items, 256>>>(kc, vc, dbt, dlens, max_pages, out, work); });
  }
  timeit("lds_dma_ring2", [&] { stream_lds<2><<<n_items, 256>>>(kc, vc, dbt, dlens, max_pages, out); });
  timeit("lds_dma_ring3", [&] { stream_lds<3><<<n_items, 256>>>(kc, vc, dbt, dlens, max_pages, out); });
  timeit("lds_dma_ring4", [&] { stream_lds<4><<<n_items, 256>>>(kc, vc, dbt, dlens, max_pages, out); });
  for (int occ : {2, 3}) {
    const int grid = std::min(n_items, cus * occ);
    char name[64];
    snprintf(name, sizeof(name), "reg_persistent_x%d", occ);
    timeit(name, [&] { stream_persist<<<grid, 256>>>(kc, vc, dbt, dlens, max_pages, n_items, out); });
  }
  CK(hipDeviceSynchronize());
  return 0;
}
