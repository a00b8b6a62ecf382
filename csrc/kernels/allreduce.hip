// One-shot and two-shot all-reduce over peer-mapped HBM.
//
// Tensor-parallel decode all-reduces are small (M x hidden x 2 B: 16 KB per
// token at 70B) and latency-bound; a ring all-reduce over xGMI takes 2 (n - 1)
// dependent link hops. Two protocols, both one kernel, no host per call:
//
//  * ONE-SHOT: every rank PUSHES its whole input into a per-source slot of every
//    peer's receive buffer (one hop over the direct point-to-point link to each
//    peer; the 7 links of an MI355X run in parallel), raises a per-block flag in
//    each peer, waits for the flags of all peers and reduces the n slots from its
//    OWN HBM. Out of each rank: (n - 1) x S bytes. For small messages.
//  * TWO-SHOT (reduce-scatter + all-gather over the same buffers): each block's
//    range is cut into n pieces, piece q owned by rank q. A rank pushes piece q of
//    its input into rank q's slot, waits, reduces ITS piece (the same fp32 sum in
//    rank order as one-shot, so results are bit-identical), pushes the reduced piece
//    into every rank's gather buffer, waits, and reads the whole range back. Out of
//    each rank: 2 (n - 1) / n x S bytes -- at the 70B B=256 decode all-reduce (4 MB,
//    world 8) 7 MB instead of one-shot's 28 MB. For large messages; the crossover
//    is a config key (parallel/custom_ar.py), unmeasured until an 8-GPU node exists.
//
// Memory: each rank owns one fine-grained (uncached) allocation, exported with
// hipIpcGetMemHandle and opened by every peer:
//   [0, 2 KB)        flags[kMaxBlocks][kMaxRanks]     u32 (one-shot; two-shot scatter phase)
//   [2 KB, 4 KB)     gflags[kMaxBlocks][kMaxRanks]    u32 (two-shot gather phase)
//   [8 KB, 8 KB+256) rounds[kMaxBlocks]               u32, this rank's per-block call counter
//   [12 KB]          err                              u32, set when a wait times out
//   [64 KB, ...)     recv[2][world][cap]              parity-double-buffered slots
//   then             gather[2][cap]                   two-shot reduced pieces
// Hand-off (system scope: the producer is another device). Every slot and flag
// access is a system-coherent (sc0 sc1) buffer access, which bypasses the GPU
// caches whatever the page's cache type, so no cache maintenance is needed:
// data stores -> each storing wave's s_waitcnt vmcnt(0) (the stores are complete
// at the destination) -> block barrier -> sc0 sc1 flag store; the consumer polls
// its flag with sc0 sc1 loads, barriers, and reads the slots with sc0 sc1 loads.
// The previous protocol (__threadfence_system + release / acquire at system
// scope: an L2 write-back and invalidate per block and call, ~15.7 us per fused
// call even at world 1 in the TP=8 simulation) is kept as the "fence" protocol
// (OAMD_CAR_PROTOCOL=fence) for A/B.
// Round numbers are per block and kept on the device, so a call is a pure kernel
// launch (capturable into a hipGraph) and ranks never exchange host state per
// call. Every call of either kind advances every block's round by one. Parity
// buffers make slot reuse safe: a peer can be at most one round ahead (it needs
// this rank's flag of round r+1 to finish r+1, raised only after this rank
// finished reading round r; the two-shot gather buffer likewise, through the
// scatter flags of round r+1). Every wait is bounded (wall clock, ~2 s by
// default): a missing peer sets `err` and the kernel drains instead of spinning
// forever. A timed-out block never leaves a partial sum behind: it writes NaN over
// its output slice, and the error is STICKY -- every later call sees `err` at
// entry, poisons its whole output and touches no peer -- because after a timeout
// the per-block round counters of the ranks no longer agree. The error is
// mirrored into a host-mapped word, so the engine polls it after each decode
// window with a plain host read (no device sync) and fails the TP replica; the
// pool respawns it with fresh buffers.
#include <cstring>

#include "common.h"
#include "kernels.h"

namespace oamd {

namespace car {
constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 64;
constexpr int kThreads = 512;
constexpr size_t kFlagsOff = 0;
constexpr size_t kGFlagsOff = 2 << 10;
constexpr size_t kRoundsOff = 8 << 10;
constexpr size_t kErrOff = 12 << 10;
constexpr size_t kDataOff = 64 << 10;
constexpr uint64_t kDefaultTimeoutTicks = 200000000ull;  // wall_clock64 runs at 100 MHz: 2 s
}  // namespace car

struct CarPeers {
  char* base[car::kMaxRanks];
};

namespace car {
constexpr int kSys = 17;   // buffer-op cache policy sc0 | sc1: system coherent, bypasses every GPU cache
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(char* base) {
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int64_t off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, r, (int)off, 0, kSys);
}
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t r, int64_t off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kSys);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
// byte offsets inside a rank's buffer
__device__ __forceinline__ int64_t slot_off(int par, int W, int src, int64_t capvec, int64_t v) {
  return (int64_t)kDataOff + (((int64_t)par * W + src) * capvec + v) * 16;
}
__device__ __forceinline__ int64_t gather_off(int par, int W, int64_t capvec, int64_t v) {
  return (int64_t)kDataOff + ((2 * (int64_t)W + par) * capvec + v) * 16;
}

// Raise this block's flag (value `round`) in every rank for phase `flags_off`, after
// every store the block made: LIGHT = each wave waits for its own sc0 sc1 stores to
// complete, then the barrier, then an sc0 sc1 flag store; otherwise the system-scope
// fence + release store of the original protocol.
template <int W, bool LIGHT>
__device__ __forceinline__ void publish(const CarPeers& peers, size_t flags_off, int b, int rank, uint32_t round,
                                        int tid) {
  if (LIGHT) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    __threadfence_system();
    __syncthreads();
  }
  if (tid < W) {
    uint32_t* f = reinterpret_cast<uint32_t*>(peers.base[tid] + flags_off) + b * kMaxRanks + rank;
    if (LIGHT) __hip_atomic_store(f, round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_store(f, round, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Wait (bounded) until every rank raised this block's flag of phase `flags_off` to
// `round`; ends with a block barrier. Sets *s_err on a timeout.
template <int W, bool LIGHT>
__device__ __forceinline__ void wait_all(char* mine, size_t flags_off, int b, uint32_t round, uint64_t timeout_ticks,
                                         int tid, uint32_t* s_err) {
  if (tid < W) {
    uint32_t* f = reinterpret_cast<uint32_t*>(mine + flags_off) + b * kMaxRanks + tid;
    const uint64_t t0 = (uint64_t)wall_clock64();
    while ((LIGHT ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                  : __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) < round) {
      __builtin_amdgcn_s_sleep(2);
      if ((uint64_t)wall_clock64() - t0 > timeout_ticks) {
        *s_err = 1;
        break;
      }
    }
  }
  __syncthreads();
}
}  // namespace car

__device__ __forceinline__ void acc8(float* a, uint4 v, bool is_bf16) {
  if (is_bf16) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[2 * i] += __uint_as_float(w[i] << 16);
      a[2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    a[0] += __uint_as_float(v.x);
    a[1] += __uint_as_float(v.y);
    a[2] += __uint_as_float(v.z);
    a[3] += __uint_as_float(v.w);
  }
}

__device__ __forceinline__ uint4 pack8(const float* a, bool is_bf16) {
  if (is_bf16)
    return make_uint4(pack_bf2(a[0], a[1]), pack_bf2(a[2], a[3]), pack_bf2(a[4], a[5]), pack_bf2(a[6], a[7]));
  return make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]), __float_as_uint(a[3]));
}

// NaN over out[v0, v1): a failed call must never look like a valid sum.
template <bool BF16>
__device__ __forceinline__ void poison(uint4* __restrict__ out, int64_t v0, int64_t v1, int tid) {
  const uint32_t nan = BF16 ? 0x7FC07FC0u : 0x7FC00000u;
  for (int64_t v = v0 + tid; v < v1; v += car::kThreads) out[v] = make_uint4(nan, nan, nan, nan);
}

// The sum over the W receive slots of vector v, fp32 in rank order (both protocols).
template <int W>
__device__ __forceinline__ void sum_slots(float* a, __amdgpu_buffer_rsrc_t rm, int par, int64_t capvec, int64_t v,
                                          bool is_bf16) {
  uint4 x[W];
#pragma unroll
  for (int p = 0; p < W; ++p) x[p] = car::ld16(rm, car::slot_off(par, W, p, capvec, v));
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.f;
#pragma unroll
  for (int p = 0; p < W; ++p) acc8(a, x[p], is_bf16);
}

// LL (flag-in-data) one-shot: a 16-B vector travels as two 16-B packets
// {d0, round, d1, round}, {d2, round, d3, round}, so a consumer that sees the round in
// both flag words of a packet has its data -- no store-completion wait, barrier, flag
// store and flag poll between the push and the reduce (each 8-B half is written whole;
// a torn packet shows a stale flag and is re-read). Packets 2v, 2v+1 of a slot hold
// vector v, so a slot holds half as many vectors as with the flag protocol. Slots
// alternate parity per round as before, so a stale packet carries round - 2.
__device__ __forceinline__ void ll_st(__amdgpu_buffer_rsrc_t r, int par, int W, int src, int64_t capvec, int64_t v,
                                      uint4 x, uint32_t round) {
  car::st16(r, car::slot_off(par, W, src, capvec, 2 * v), make_uint4(x.x, round, x.y, round));
  car::st16(r, car::slot_off(par, W, src, capvec, 2 * v + 1), make_uint4(x.z, round, x.w, round));
}
// Vector v of slot `src`, polled until both packets carry `round` (bounded: *err set and
// whatever was read returned when the wall clock passes `deadline`).
__device__ __forceinline__ uint4 ll_ld(__amdgpu_buffer_rsrc_t rm, int par, int W, int src, int64_t capvec, int64_t v,
                                       uint32_t round, uint64_t deadline, uint32_t* err) {
  uint4 a = car::ld16(rm, car::slot_off(par, W, src, capvec, 2 * v));
  uint4 b = car::ld16(rm, car::slot_off(par, W, src, capvec, 2 * v + 1));
  while ((a.y != round) | (a.w != round) | (b.y != round) | (b.w != round)) {
    if ((uint64_t)wall_clock64() > deadline) {
      *err = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    a = car::ld16(rm, car::slot_off(par, W, src, capvec, 2 * v));
    b = car::ld16(rm, car::slot_off(par, W, src, capvec, 2 * v + 1));
  }
  return make_uint4(a.x, a.z, b.x, b.z);
}
template <int W>
__device__ __forceinline__ void ll_sum_slots(float* a, __amdgpu_buffer_rsrc_t rm, int par, int64_t capvec, int64_t v,
                                             bool is_bf16, uint32_t round, uint64_t deadline, uint32_t* err) {
  uint4 x[W];
#pragma unroll
  for (int p = 0; p < W; ++p) x[p] = ll_ld(rm, par, W, p, capvec, v, round, deadline, err);
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.f;
#pragma unroll
  for (int p = 0; p < W; ++p) acc8(a, x[p], is_bf16);
}

// Call prologue shared by every kernel: this block's round, and whether an earlier
// call left the sticky error.
struct CarCall {
  uint32_t round;
  int par;
  bool failed;
};
__device__ __forceinline__ CarCall car_begin(char* mine, int b, int tid, uint32_t* s_round, uint32_t* s_err) {
  uint32_t* rounds = reinterpret_cast<uint32_t*>(mine + car::kRoundsOff);
  uint32_t* err = reinterpret_cast<uint32_t*>(mine + car::kErrOff);
  if (tid == 0) {
    *s_round = rounds[b] + 1;
    *s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  return CarCall{*s_round, static_cast<int>(*s_round & 1), *s_err != 0};
}
__device__ __forceinline__ void car_fail(char* mine, int b, int tid, uint32_t round, uint32_t* herr) {
  if (tid == 0) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(mine + car::kErrOff), 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    if (herr != nullptr) __hip_atomic_store(herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    reinterpret_cast<uint32_t*>(mine + car::kRoundsOff)[b] = round;
  }
}
__device__ __forceinline__ void car_end(char* mine, int b, int tid, uint32_t round) {
  if (tid == 0) reinterpret_cast<uint32_t*>(mine + car::kRoundsOff)[b] = round;
}

// Plain all-reduce, one 16-B vector = 8 bf16 or 4 fp32 elements. TWO: two-shot; LL:
// one-shot with the flags in the data packets.
template <int W, bool BF16, bool TWO, bool LIGHT, bool LL = false>
__global__ void __launch_bounds__(car::kThreads) allreduce_kernel(const uint4* __restrict__ in,
                                                                  uint4* __restrict__ out, int64_t nvec,
                                                                  int64_t capvec, int rank, CarPeers peers,
                                                                  uint32_t* herr, uint64_t timeout_ticks) {
  __shared__ uint32_t s_round;
  __shared__ uint32_t s_err;
  const int b = blockIdx.x, tid = threadIdx.x;
  char* mine = peers.base[rank];
  const CarCall c = car_begin(mine, b, tid, &s_round, &s_err);
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = min(nvec, per * b), v1 = min(nvec, v0 + per);
  if (c.failed) {   // sticky: an earlier call timed out, the ranks are out of step
    poison<BF16>(out, v0, v1, tid);
    return;
  }
  __amdgpu_buffer_rsrc_t rs[W];
#pragma unroll
  for (int p = 0; p < W; ++p) rs[p] = car::rsrc(peers.base[p]);
  const __amdgpu_buffer_rsrc_t rm = car::rsrc(mine);
  const int64_t pq = (v1 - v0 + W - 1) / W;   // two-shot piece per owner
  if constexpr (LL) {
    const uint64_t deadline = (uint64_t)wall_clock64() + timeout_ticks;
#pragma unroll
    for (int p = 0; p < W; ++p)
      for (int64_t v = v0 + tid; v < v1; v += car::kThreads) ll_st(rs[p], c.par, W, rank, capvec, v, in[v], c.round);
    for (int64_t v = v0 + tid; v < v1; v += car::kThreads) {
      float a[8];
      ll_sum_slots<W>(a, rm, c.par, capvec, v, BF16, c.round, deadline, &s_err);
      out[v] = pack8(a, BF16);
    }
    __syncthreads();
    if (s_err) {
      car_fail(mine, b, tid, c.round, herr);
      poison<BF16>(out, v0, v1, tid);
      return;
    }
    car_end(mine, b, tid, c.round);
    return;
  }
  // ---- push: one-shot: the whole range into slot [par][rank] of every rank;
  //      two-shot: piece q into rank q's slot [par][rank]
#pragma unroll
  for (int p = 0; p < W; ++p) {
    const int64_t a = TWO ? min(v1, v0 + p * pq) : v0, e = TWO ? min(v1, a + pq) : v1;
    for (int64_t v = a + tid; v < e; v += car::kThreads) car::st16(rs[p], car::slot_off(c.par, W, rank, capvec, v), in[v]);
  }
  car::publish<W, LIGHT>(peers, car::kFlagsOff, b, rank, c.round, tid);
  car::wait_all<W, LIGHT>(mine, car::kFlagsOff, b, c.round, timeout_ticks, tid, &s_err);
  if (s_err) {
    car_fail(mine, b, tid, c.round, herr);
    poison<BF16>(out, v0, v1, tid);
    return;
  }
  if constexpr (!TWO) {
    for (int64_t v = v0 + tid; v < v1; v += car::kThreads) {
      float a[8];
      sum_slots<W>(a, rm, c.par, capvec, v, BF16);
      out[v] = pack8(a, BF16);
    }
  } else {
    // reduce this rank's piece, hand it to every rank's gather buffer
    const int64_t a0 = min(v1, v0 + rank * pq), e0 = min(v1, a0 + pq);
    for (int64_t v = a0 + tid; v < e0; v += car::kThreads) {
      float a[8];
      sum_slots<W>(a, rm, c.par, capvec, v, BF16);
      const uint4 o = pack8(a, BF16);
#pragma unroll
      for (int p = 0; p < W; ++p) car::st16(rs[p], car::gather_off(c.par, W, capvec, v), o);
    }
    car::publish<W, LIGHT>(peers, car::kGFlagsOff, b, rank, c.round, tid);
    car::wait_all<W, LIGHT>(mine, car::kGFlagsOff, b, c.round, timeout_ticks, tid, &s_err);
    if (s_err) {
      car_fail(mine, b, tid, c.round, herr);
      poison<BF16>(out, v0, v1, tid);
      return;
    }
    for (int64_t v = v0 + tid; v < v1; v += car::kThreads) out[v] = car::ld16(rm, car::gather_off(c.par, W, capvec, v));
  }
  car_end(mine, b, tid, c.round);
}

// Fused TP block epilogue: h = h + bf16(sum over ranks of in); y = RMSNorm(h) * w.
// Row-partitioned (block b owns rows [r0, r1)), so after the all-reduce each block
// holds whole rows and normalises them in place: the all-reduce's output never
// round-trips through HBM before the norm, and one launch replaces two (SURVEY.md
// §7.4 item 6: the fusion that makes TP=8 pay). TWO: the block's rows go through the
// two-shot protocol (reduce-scatter of pieces, all-gather of their sums) instead of
// one-shot; the sums are bit-identical.
// Numerics are those of all-reduce + rmsnorm_kernel: the sum is rounded to bf16,
// the residual add is rounded to bf16, the normalised value is rounded before w.
// SLABS: the input is S fp32 split-K slabs [S, rows, hidden] of the producing GEMM,
// summed in slab order and rounded to bf16 on the way into the peers' receive slots
// (bit-identical to splitk_reduce_fp32 + the bf16 path, one kernel fewer).
// Q8: also emit the normalised rows as per-row e4m3fn (q8, sx) for the next fp8 GEMM,
// bit-identical to quantize_fp8(y) — the activation quantization kernel disappears.
template <int W, int MAXV, bool SLABS, bool Q8, bool TWO, bool LIGHT, bool LL = false>
__global__ void __launch_bounds__(car::kThreads) ar_rmsnorm_kernel(
    const uint4* __restrict__ in, const float* __restrict__ slabs, int S, bf16_t* __restrict__ residual,
    const bf16_t* __restrict__ w, bf16_t* __restrict__ y, uint8_t* __restrict__ q8, float* __restrict__ sx,
    int rows, int hidden, float eps, int64_t capvec, int rank, CarPeers peers, uint32_t* herr,
    uint64_t timeout_ticks) {
  __shared__ uint32_t s_round;
  __shared__ uint32_t s_err;
  __shared__ float scratch[car::kThreads / 64];
  __shared__ float mscratch[car::kThreads / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  char* mine = peers.base[rank];
  const CarCall c = car_begin(mine, b, tid, &s_round, &s_err);
  const int nvr = hidden >> 3;
  const int per = (rows + gridDim.x - 1) / gridDim.x;
  const int r0 = min(rows, per * b), r1 = min(rows, r0 + per);
  const int64_t v0 = (int64_t)r0 * nvr, v1 = (int64_t)r1 * nvr;
  uint4* y4 = reinterpret_cast<uint4*>(y);
  auto fail_out = [&]() {
    poison<true>(y4, v0, v1, tid);
    if constexpr (Q8)
      for (int r = r0 + tid; r < r1; r += car::kThreads) sx[r] = __builtin_nanf("");
  };
  if (c.failed) {
    fail_out();
    return;
  }
  __amdgpu_buffer_rsrc_t rs[W];
#pragma unroll
  for (int p = 0; p < W; ++p) rs[p] = car::rsrc(peers.base[p]);
  const __amdgpu_buffer_rsrc_t rm = car::rsrc(mine);
  const int64_t MN = (int64_t)rows * hidden;
  auto load_x = [&](int64_t v) -> uint4 {
    if constexpr (SLABS) {
      const float* pv = slabs + v * 8;
      f32x4 a0 = *reinterpret_cast<const f32x4*>(pv), a1 = *reinterpret_cast<const f32x4*>(pv + 4);
      if (S == 2) {   // the usual decode split: both slabs' loads in flight together
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(pv + MN), b1 = *reinterpret_cast<const f32x4*>(pv + MN + 4);
        a0 += b0;
        a1 += b1;
      } else if (S == 4) {
        f32x4 bb[3][2];
#pragma unroll
        for (int s = 1; s < 4; ++s) {
          bb[s - 1][0] = *reinterpret_cast<const f32x4*>(pv + s * MN);
          bb[s - 1][1] = *reinterpret_cast<const f32x4*>(pv + s * MN + 4);
        }
#pragma unroll
        for (int s = 0; s < 3; ++s) {   // slab order
          a0 += bb[s][0];
          a1 += bb[s][1];
        }
      } else {
        for (int s = 1; s < S; ++s) {
          a0 += *reinterpret_cast<const f32x4*>(pv + s * MN);
          a1 += *reinterpret_cast<const f32x4*>(pv + s * MN + 4);
        }
      }
      return make_uint4(pack_bf2(a0[0], a0[1]), pack_bf2(a0[2], a0[3]), pack_bf2(a1[0], a1[1]),
                        pack_bf2(a1[2], a1[3]));
    } else {
      return in[v];
    }
  };
  const int64_t pq = (v1 - v0 + W - 1) / W;
  const uint64_t deadline = (uint64_t)wall_clock64() + timeout_ticks;   // LL polls
  if constexpr (LL) {
    for (int64_t v = v0 + tid; v < v1; v += car::kThreads) {
      const uint4 x = load_x(v);
#pragma unroll
      for (int p = 0; p < W; ++p) ll_st(rs[p], c.par, W, rank, capvec, v, x, c.round);
    }
  } else {
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const int64_t a = TWO ? min(v1, v0 + p * pq) : v0, e = TWO ? min(v1, a + pq) : v1;
      for (int64_t v = a + tid; v < e; v += car::kThreads) car::st16(rs[p], car::slot_off(c.par, W, rank, capvec, v), load_x(v));
    }
  }
  // the first row's residual and weight vectors, loaded while the hand-off is in flight
  // (they do not depend on it): one memory round trip off the critical path
  const u16x8* w8 = reinterpret_cast<const u16x8*>(w);
  u16x8 h_pre[MAXV], w_pre[MAXV];
  if (r0 < r1) {
    const u16x8* hr0 = reinterpret_cast<const u16x8*>(residual + (int64_t)r0 * hidden);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int vi = tid + i * car::kThreads;
      if (vi < nvr) {
        h_pre[i] = hr0[vi];
        w_pre[i] = w8[vi];
      }
    }
  }
  if constexpr (!LL) {
    car::publish<W, LIGHT>(peers, car::kFlagsOff, b, rank, c.round, tid);
    car::wait_all<W, LIGHT>(mine, car::kFlagsOff, b, c.round, timeout_ticks, tid, &s_err);
    if (s_err) {
      car_fail(mine, b, tid, c.round, herr);
      fail_out();
      return;
    }
  }
  if constexpr (TWO) {
    const int64_t a0 = min(v1, v0 + rank * pq), e0 = min(v1, a0 + pq);
    for (int64_t v = a0 + tid; v < e0; v += car::kThreads) {
      float a[8];
      sum_slots<W>(a, rm, c.par, capvec, v, true);
      const uint4 o = pack8(a, true);
#pragma unroll
      for (int p = 0; p < W; ++p) car::st16(rs[p], car::gather_off(c.par, W, capvec, v), o);
    }
    car::publish<W, LIGHT>(peers, car::kGFlagsOff, b, rank, c.round, tid);
    car::wait_all<W, LIGHT>(mine, car::kGFlagsOff, b, c.round, timeout_ticks, tid, &s_err);
    if (s_err) {
      car_fail(mine, b, tid, c.round, herr);
      fail_out();
      return;
    }
  }
  for (int r = r0; r < r1; ++r) {
    u16x8* hr = reinterpret_cast<u16x8*>(residual + (int64_t)r * hidden);
    u16x8* yr = reinterpret_cast<u16x8*>(y + (int64_t)r * hidden);
    float v[MAXV][8];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int vi = tid + i * car::kThreads;
      if (vi < nvr) {
        const int64_t g = (int64_t)r * nvr + vi;
        float a[8];
        if constexpr (TWO) {   // the gathered bf16 sums
          const uint4 x = car::ld16(rm, car::gather_off(c.par, W, capvec, g));
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] = 0.f;
          acc8(a, x, true);
        } else {
          if constexpr (LL)
            ll_sum_slots<W>(a, rm, c.par, capvec, g, true, c.round, deadline, &s_err);
          else
            sum_slots<W>(a, rm, c.par, capvec, g, true);
#pragma unroll
          for (int j = 0; j < 8; ++j) a[j] = bf2f(f2bf(a[j]));
        }
        const u16x8 hv = r == r0 ? h_pre[i] : hr[vi];
        u16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] = f2bf(a[j] + bf2f(hv[j]));
          v[i][j] = bf2f(s[j]);
          ss += v[i][j] * v[i][j];
        }
        if constexpr (!LL) hr[vi] = s;
      }
    }
    const float tot = block_sum<car::kThreads>(ss, scratch);
    if constexpr (LL) {
      // a peer that never arrived: nothing of this row reaches the residual (the
      // block's barrier in block_sum orders every lane's s_err write before this read)
      if (s_err) {
        car_fail(mine, b, tid, c.round, herr);
        fail_out();
        return;
      }
#pragma unroll
      for (int i = 0; i < MAXV; ++i) {
        const int vi = tid + i * car::kThreads;
        if (vi < nvr) {
          u16x8 s;
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] = f2bf(v[i][j]);
          hr[vi] = s;
        }
      }
    }
    const float rs_ = rsqrtf(tot / static_cast<float>(hidden) + eps);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int vi = tid + i * car::kThreads;
      if (vi < nvr) {
        const u16x8 wv = w_pre[i];   // the same weight vector for every row
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(f2bf(v[i][j] * rs_)) * bf2f(wv[j]));
        yr[vi] = o;
        if constexpr (Q8) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] = bf2f(o[j]);
        }
      }
    }
    if constexpr (Q8) {
      float am = 0.f;
#pragma unroll
      for (int i = 0; i < MAXV; ++i)
        if (tid + i * car::kThreads < nvr)
#pragma unroll
          for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v[i][j]));
      am = wave_max(am);
      if ((tid & 63) == 0) mscratch[tid >> 6] = am;
      __syncthreads();
      am = 0.f;
#pragma unroll
      for (int k = 0; k < car::kThreads / 64; ++k) am = fmaxf(am, mscratch[k]);
      __syncthreads();   // mscratch is reused by the next row
      const float sc = am > 0.f ? am / 448.f : 1.f;
      const float inv = 1.f / sc;
      if (tid == 0) sx[r] = sc;
      uint8_t* qr = q8 + (int64_t)r * hidden;
#pragma unroll
      for (int i = 0; i < MAXV; ++i) {
        const int vi = tid + i * car::kThreads;
        if (vi < nvr) {
          int lo = 0, hi = 0;
          lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][0] * inv, v[i][1] * inv, lo, false);
          lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][2] * inv, v[i][3] * inv, lo, true);
          hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][4] * inv, v[i][5] * inv, hi, false);
          hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][6] * inv, v[i][7] * inv, hi, true);
          *reinterpret_cast<uint2*>(qr + vi * 8) = make_uint2(static_cast<uint32_t>(lo), static_cast<uint32_t>(hi));
        }
      }
    }
  }
  car_end(mine, b, tid, c.round);
}

// ------------------------------------------------------------------ host side

// receive slots [2][world][cap] + the two-shot gather buffer [2][cap]
size_t car_buffer_bytes(size_t cap_bytes, int world) { return car::kDataOff + 2 * ((size_t)world + 1) * cap_bytes; }

int car_alloc(size_t cap_bytes, int world, void** base, void* handle_out) {
  if (world < 1 || world > car::kMaxRanks || cap_bytes % 16 != 0) return -1;
  const size_t bytes = car_buffer_bytes(cap_bytes, world);
  hipError_t e = hipExtMallocWithFlags(base, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*base, 0, car::kDataOff);
  if (e != hipSuccess) return (int)e;
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, *base);
  if (e != hipSuccess) return (int)e;
  std::memcpy(handle_out, &h, sizeof(h));
  return 0;
}

int car_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

int car_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

int car_free(void* base) { return (int)hipFree(base); }

int car_host_flag(uint32_t** host, uint32_t** dev) {
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(host), 4, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  **host = 0;
  return (int)hipHostGetDevicePointer(reinterpret_cast<void**>(dev), *host, 0);
}

void car_free_host_flag(uint32_t* host) {
  if (host != nullptr) (void)hipHostFree(host);
}

int car_error(const uint32_t* host) { return (int)__atomic_load_n(host, __ATOMIC_ACQUIRE); }

int car_reset(void* base, size_t bytes, uint32_t* host) {
  // flags, rounds and err back to zero; only meaningful when EVERY rank resets
  // between two barriers with no call in flight (a collective restart). The data slots
  // too: rounds restart at 1, and an LL packet left from before must not carry a live round.
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemset(base, 0, bytes > car::kDataOff ? bytes : car::kDataOff);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (host != nullptr) __atomic_store_n(host, 0u, __ATOMIC_RELEASE);
  return (int)e;
}

// proto: kCarOneShot / kCarTwoShot (sc0 sc1 hand-off) or kCarOneShotFence (the original
// system-scope fence protocol, for A/B). A two-shot call at world 1 runs one-shot.
int car_all_reduce(const void* in, void* out, int64_t bytes, bool bf16, int rank, int world, void* const* bases,
                   size_t cap_bytes, int blocks, uint32_t* herr_dev, double timeout_s, int proto,
                   hipStream_t stream) {
  if (world < 1 || world > car::kMaxRanks || rank < 0 || rank >= world) return -1;
  if (bytes % 16 != 0 || (size_t)bytes > cap_bytes || cap_bytes % 16 != 0) return -2;
  if (blocks < 1 || blocks > car::kMaxBlocks) return -3;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) return -4;
  if (proto < kCarOneShot || proto > kCarLL) return -6;
  if (world == 1 && proto == kCarTwoShot) proto = kCarOneShot;
  if (proto == kCarLL && (size_t)bytes * 2 > cap_bytes) return -7;   // LL packets: twice the bytes
  CarPeers peers{};
  for (int p = 0; p < world; ++p) peers.base[p] = static_cast<char*>(bases[p]);
  const int64_t nvec = bytes / 16, capvec = cap_bytes / 16;
  const uint4* i4 = static_cast<const uint4*>(in);
  uint4* o4 = static_cast<uint4*>(out);
  const uint64_t ticks = timeout_s > 0 ? (uint64_t)(timeout_s * 1e8) : car::kDefaultTimeoutTicks;
#define OAMD_CARP(W, B, T, L, LLP) \
  allreduce_kernel<W, B, T, L, LLP><<<blocks, car::kThreads, 0, stream>>>(i4, o4, nvec, capvec, rank, peers, herr_dev, ticks)
#define OAMD_CARD(W, B)                                    \
  if (proto == kCarTwoShot) OAMD_CARP(W, B, (W > 1), true, false); \
  else if (proto == kCarOneShot) OAMD_CARP(W, B, false, true, false); \
  else if (proto == kCarLL) OAMD_CARP(W, B, false, true, true); \
  else OAMD_CARP(W, B, false, false, false);
#define OAMD_CAR(W)                 \
  case W:                           \
    if (bf16) { OAMD_CARD(W, true) } \
    else { OAMD_CARD(W, false) }     \
    break;
  switch (world) {
    OAMD_CAR(1)
    OAMD_CAR(2)
    OAMD_CAR(3)
    OAMD_CAR(4)
    OAMD_CAR(5)
    OAMD_CAR(6)
    OAMD_CAR(7)
    OAMD_CAR(8)
    default: return -1;
  }
#undef OAMD_CAR
#undef OAMD_CARD
#undef OAMD_CARP
  OAMD_LAUNCH_CHECK();
  return 0;
}

int car_all_reduce_rmsnorm(const void* in, const float* slabs, int S, bf16_t* residual, const bf16_t* w, bf16_t* y,
                           uint8_t* q8, float* sx, int rows, int hidden, float eps, int rank, int world,
                           void* const* bases, size_t cap_bytes, int blocks, uint32_t* herr_dev, double timeout_s,
                           int proto, hipStream_t stream) {
  if ((slabs == nullptr) == (in == nullptr) || (slabs != nullptr && S < 1)) return -5;
  if ((q8 == nullptr) != (sx == nullptr)) return -5;
  if (world < 1 || world > car::kMaxRanks || rank < 0 || rank >= world) return -1;
  if (rows < 1 || hidden < 8 || hidden % 8 != 0 || hidden > car::kThreads * 8 * 4) return -2;
  if ((size_t)rows * hidden * 2 > cap_bytes || cap_bytes % 16 != 0) return -2;
  if (blocks < 1 || blocks > car::kMaxBlocks) return -3;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(slabs) | reinterpret_cast<uintptr_t>(residual) |
       reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(q8)) & 15)
    return -4;
  if (proto < kCarOneShot || proto > kCarLL) return -6;
  if (world == 1 && proto == kCarTwoShot) proto = kCarOneShot;
  if (proto == kCarLL && (size_t)rows * hidden * 2 * 2 > cap_bytes) return -7;   // LL packets: twice the bytes
  CarPeers peers{};
  for (int p = 0; p < world; ++p) peers.base[p] = static_cast<char*>(bases[p]);
  const int64_t capvec = cap_bytes / 16;
  const uint4* i4 = static_cast<const uint4*>(in);
  const uint64_t ticks = timeout_s > 0 ? (uint64_t)(timeout_s * 1e8) : car::kDefaultTimeoutTicks;
  const bool big = hidden > car::kThreads * 8 * 2;
  const int mode = (slabs != nullptr ? 1 : 0) | (q8 != nullptr ? 2 : 0);
#define OAMD_CARK(W, MV, SL, Q, T, L, LLP)                                                                     \
  ar_rmsnorm_kernel<W, MV, SL, Q, T, L, LLP><<<blocks, car::kThreads, 0, stream>>>(                            \
      i4, slabs, S, residual, w, y, q8, sx, rows, hidden, eps, capvec, rank, peers, herr_dev, ticks)
#define OAMD_CARP(W, MV, SL, Q)                                                                                \
  if (proto == kCarTwoShot) OAMD_CARK(W, MV, SL, Q, (W > 1), true, false);                                     \
  else if (proto == kCarOneShot) OAMD_CARK(W, MV, SL, Q, false, true, false);                                  \
  else if (proto == kCarLL) OAMD_CARK(W, MV, SL, Q, false, true, true);                                        \
  else OAMD_CARK(W, MV, SL, Q, false, false, false);
#define OAMD_CARM(W, MV)                                                                                       \
  switch (mode) {                                                                                              \
    case 0: { OAMD_CARP(W, MV, false, false) } break;                                                          \
    case 1: { OAMD_CARP(W, MV, true, false) } break;                                                           \
    case 2: { OAMD_CARP(W, MV, false, true) } break;                                                           \
    default: { OAMD_CARP(W, MV, true, true) } break;                                                           \
  }
#define OAMD_CARN(W)                                                                                           \
  case W:                                                                                                      \
    if (big) {                                                                                                 \
      OAMD_CARM(W, 4)                                                                                          \
    } else {                                                                                                   \
      OAMD_CARM(W, 2)                                                                                          \
    }                                                                                                          \
    break;
  switch (world) {
    OAMD_CARN(1)
    OAMD_CARN(2)
    OAMD_CARN(3)
    OAMD_CARN(4)
    OAMD_CARN(5)
    OAMD_CARN(6)
    OAMD_CARN(7)
    OAMD_CARN(8)
    default: return -1;
  }
#undef OAMD_CARM
#undef OAMD_CARK
#undef OAMD_CARP
#undef OAMD_CARN
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
