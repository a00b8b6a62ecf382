// Causal flash attention for prefill, variable-length packed sequences, GQA,
// on MFMA. Four variants share the work-list contract
// (attn_prefill_block_q): v1 per-query-head (below), v2 GQA-grouped 16-row waves
// with a software-pipelined K/V tile, v3 GQA-grouped swapped-operand 32x32 MFMA
// waves (S^T = K Q^T, P stays in registers as the next MFMA's B operand) in 8-wave
// workgroups, v4 the same waves in 4-wave workgroups (two per CU; GQA groups <= 4).
//
// v1 work item = (64-row query block of one sequence, query head). 4 waves; each
// wave owns 16 query rows. Per 64-key tile:
//   S = Q K^T      16 x v_mfma_f32_16x16x32_bf16 per wave (Q in registers)
//   online softmax in the C-fragment layout (row max/sum over 16 lanes)
//   O += P V       16 x MFMA per wave, P bounced through a per-wave LDS image
// K is staged row-major and V transposed ([d][key]) in LDS, both XOR-swizzled
// on 16-B chunks so every ds_read_b128 of a 16-lane group hits 16 distinct
// bank slots (cdna_hip_programming.md §5.5 T2).
// Fragment maps for 16x16x32 bf16 (cdna_hip_programming.md §3):
//   A: lane l -> A[l&15][8(l>>4)+j]   B: lane l -> B[8(l>>4)+j][l&15]
//   C: col = l&15, row = 4(l>>4)+i
#include "common.h"
#include "kernels.h"

namespace oamd {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8_t as_bf8(u16x8 v) { return __builtin_bit_cast(bf16x8_t, v); }

__global__ void __launch_bounds__(256) attn_prefill_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, const int* __restrict__ cu_seqlens, const int* __restrict__ work_seq,
    const int* __restrict__ work_q0, int Hq, int Hkv, float scale_log2) {
  constexpr int D = 128, BQ = 64, BK = 64;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BK * D];       // [key][d], 256-B rows
  __shared__ __attribute__((aligned(16))) bf16_t Vt[D * BK];       // [d][key], 128-B rows
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][16 * BK];   // per wave [row][key]

  const int wi = blockIdx.x, hq = blockIdx.y;
  const int kvh = hq / (Hq / Hkv);
  const int seq = work_seq[wi];
  if (seq < 0) return;  // padding item of a graph-captured prefill (fixed grid)
  const int s0 = cu_seqlens[seq];
  const int slen = cu_seqlens[seq + 1] - s0;
  const int q0 = work_q0[wi];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l15 = lane & 15, lhi = lane >> 4;

  // Q fragments (A operand) for this wave's 16 rows, 4 k-steps over D = 128
  u16x8 qa[4];
  {
    const int row = q0 + w * 16 + l15;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (row < slen)
        qa[s] = *reinterpret_cast<const u16x8*>(q + ((int64_t)(s0 + row) * Hq + hq) * D + 32 * s + 8 * lhi);
      else
        qa[s] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }

  f32x4 oacc[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) oacc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { mrow[i] = -INFINITY; lrow[i] = 0.f; }

  const int kend = min(slen, q0 + BQ);  // causal: keys < last row of the block + 1
  const int ntiles = (kend + BK - 1) / BK;
  char* ks_b = reinterpret_cast<char*>(Ks);
  char* vt_b = reinterpret_cast<char*>(Vt);
  char* ps_b = reinterpret_cast<char*>(Ps[w]);

  for (int kt = 0; kt < ntiles; ++kt) {
    const int kb = kt * BK;
    __syncthreads();
    // ---- stage K (row-major, swizzled) and V (transposed, swizzled) ----
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = tid + r * 256;
      const int key = c >> 4, ch = c & 15;
      u16x8 kv = u16x8{0, 0, 0, 0, 0, 0, 0, 0}, vv = kv;
      if (kb + key < slen) {
        const int64_t off = ((int64_t)(s0 + kb + key) * Hkv + kvh) * D + ch * 8;
        kv = *reinterpret_cast<const u16x8*>(k + off);
        vv = *reinterpret_cast<const u16x8*>(v + off);
      }
      *reinterpret_cast<u16x8*>(ks_b + key * 256 + ((ch ^ (key & 15)) << 4)) = kv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = ch * 8 + j;
        const int pc = (key >> 3) ^ ((d >> 1) & 7);
        *reinterpret_cast<bf16_t*>(vt_b + d * 128 + (pc << 4) + ((key & 7) << 1)) = vv[j];
      }
    }
    __syncthreads();

    // ---- S = Q K^T ----
    f32x4 sacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      sacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int key = 16 * n + l15;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ch = 4 * s + lhi;
        const u16x8 kb8 = *reinterpret_cast<const u16x8*>(ks_b + key * 256 + ((ch ^ (key & 15)) << 4));
        sacc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(qa[s]), as_bf8(kb8), sacc[n], 0, 0, 0);
      }
    }

    // ---- online softmax (rows 4*lhi+i, key col l15 + 16n) ----
    const bool diag = (kb + BK > q0 + w * 16);  // some key may exceed some row of this wave
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qrow = q0 + w * 16 + 4 * lhi + i;
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int key = kb + 16 * n + l15;
        float sv = sacc[n][i] * scale_log2;
        if (key >= slen || (diag && key > qrow)) sv = -INFINITY;
        sacc[n][i] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, kWave));
      const float mnew = fmaxf(mrow[i], mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      alpha[i] = exp2f(mrow[i] - msafe);
      float rs = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float p = exp2f(sacc[n][i] - msafe);
        sacc[n][i] = p;
        rs += p;
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) rs += __shfl_xor(rs, o2, kWave);
      lrow[i] = lrow[i] * alpha[i] + rs;
      mrow[i] = mnew;
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) oacc[m][i] *= alpha[i];

    // ---- P -> LDS (bf16), re-read as A fragments ----
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lhi + i, key = 16 * n + l15;
        const int pc = (key >> 3) ^ ((r >> 1) & 7);
        *reinterpret_cast<bf16_t*>(ps_b + r * 128 + (pc << 4) + ((key & 7) << 1)) = f2bf(sacc[n][i]);
      }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    u16x8 pa[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 4 * s + lhi;
      pa[s] = *reinterpret_cast<const u16x8*>(ps_b + l15 * 128 + ((ch ^ ((l15 >> 1) & 7)) << 4));
    }
    // ---- O += P V ----
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int d = 16 * m + l15;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = 4 * s + lhi;
        const u16x8 vb = *reinterpret_cast<const u16x8*>(vt_b + d * 128 + ((ch ^ ((d >> 1) & 7)) << 4));
        oacc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(pa[s]), as_bf8(vb), oacc[m], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }

  // ---- epilogue ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = q0 + w * 16 + 4 * lhi + i;
    if (row < slen) {
      const float inv = lrow[i] > 0.f ? 1.f / lrow[i] : 0.f;
      bf16_t* dst = o + ((int64_t)(s0 + row) * Hq + hq) * D;
#pragma unroll
      for (int m = 0; m < 8; ++m) dst[16 * m + l15] = f2bf(oacc[m][i] * inv);
    }
  }
}

// ---------------------------------------------------------------------------
// v2: GQA-grouped, software-pipelined. A block is (16 x RG query rows, one KV
// head) with 8 waves: wave w computes query head kvh * G + (w % G) for rows
// 16 (w / G) .. +16 (G = Hq / Hkv in {1, 2, 4, 8}, RG = 8 / G), so every staged
// K/V tile feeds all G query heads that share it (v1 staged it once per query
// head). The next tile's K/V is loaded into registers while the current tile's
// MFMAs run and is written to LDS after the barrier, so global-load latency
// hides behind compute instead of being paid once per tile.
template <int G>
__global__ void __launch_bounds__(512) attn_prefill_gqa_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, const int* __restrict__ cu_seqlens, const int* __restrict__ work_seq,
    const int* __restrict__ work_q0, int Hq, int Hkv, float scale_log2) {
  constexpr int D = 128, BK = 64, RG = 8 / G, BQ = 16 * RG;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BK * D];       // [key][d], 256-B rows
  __shared__ __attribute__((aligned(16))) bf16_t Vt[D * BK];       // [d][key], 128-B rows
  __shared__ __attribute__((aligned(16))) bf16_t Ps[8][16 * BK];   // per wave [row][key]

  const int wi = blockIdx.x, kvh = blockIdx.y;
  const int seq = work_seq[wi];
  if (seq < 0) return;  // padding item of a graph-captured prefill (fixed grid)
  const int s0 = cu_seqlens[seq];
  const int slen = cu_seqlens[seq + 1] - s0;
  const int q0 = work_q0[wi];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l15 = lane & 15, lhi = lane >> 4;
  const int hq = kvh * G + (w % G);
  const int rbase = q0 + 16 * (w / G);  // this wave's first query row

  u16x8 qa[4];
  {
    const int row = rbase + l15;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (row < slen)
        qa[s] = *reinterpret_cast<const u16x8*>(q + ((int64_t)(s0 + row) * Hq + hq) * D + 32 * s + 8 * lhi);
      else
        qa[s] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  f32x4 oacc[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) oacc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4], lrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { mrow[i] = -INFINITY; lrow[i] = 0.f; }

  const int kend = min(slen, q0 + BQ);
  const int ntiles = (kend + BK - 1) / BK;
  // rows of this wave that exist at all: a wave past the sequence end only stages
  const bool active = rbase < slen;
  const int wend = min(slen, rbase + 16);  // keys this wave can see: < wend
  char* ks_b = reinterpret_cast<char*>(Ks);
  char* vt_b = reinterpret_cast<char*>(Vt);
  char* ps_b = reinterpret_cast<char*>(Ps[w]);

  // K/V chunk c = tid + 512 r (r < 2): key c >> 4, 16-B chunk c & 15 of the 256-B row
  u16x8 kr[2], vr[2];
  auto load_tile = [&](int kb) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + r * 512;
      const int key = c >> 4, ch = c & 15;
      kr[r] = vr[r] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (kb + key < slen) {
        const int64_t off = ((int64_t)(s0 + kb + key) * Hkv + kvh) * D + ch * 8;
        kr[r] = *reinterpret_cast<const u16x8*>(k + off);
        vr[r] = *reinterpret_cast<const u16x8*>(v + off);
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = tid + r * 512;
      const int key = c >> 4, ch = c & 15;
      *reinterpret_cast<u16x8*>(ks_b + key * 256 + ((ch ^ (key & 15)) << 4)) = kr[r];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = ch * 8 + j;
        const int pc = (key >> 3) ^ ((d >> 1) & 7);
        *reinterpret_cast<bf16_t*>(vt_b + d * 128 + (pc << 4) + ((key & 7) << 1)) = vr[r][j];
      }
    }
  };

  load_tile(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    const int kb = kt * BK;
    __syncthreads();  // previous tile fully consumed
    store_tile();
    __syncthreads();
    if (kt + 1 < ntiles) load_tile(kb + BK);  // in flight during this tile's MFMAs
    if (!active || kb >= wend) continue;      // no visible key in this tile for this wave

    f32x4 sacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      sacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int key = 16 * n + l15;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ch = 4 * s + lhi;
        const u16x8 kb8 = *reinterpret_cast<const u16x8*>(ks_b + key * 256 + ((ch ^ (key & 15)) << 4));
        sacc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(qa[s]), as_bf8(kb8), sacc[n], 0, 0, 0);
      }
    }
    const bool diag = (kb + BK > rbase);
    float alpha[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qrow = rbase + 4 * lhi + i;
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int key = kb + 16 * n + l15;
        float sv = sacc[n][i] * scale_log2;
        if (key >= slen || (diag && key > qrow)) sv = -INFINITY;
        sacc[n][i] = sv;
        mx = fmaxf(mx, sv);
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o2, kWave));
      const float mnew = fmaxf(mrow[i], mx);
      const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
      alpha[i] = exp2f(mrow[i] - msafe);
      float rs = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float p = exp2f(sacc[n][i] - msafe);
        sacc[n][i] = p;
        rs += p;
      }
#pragma unroll
      for (int o2 = 8; o2 > 0; o2 >>= 1) rs += __shfl_xor(rs, o2, kWave);
      lrow[i] = lrow[i] * alpha[i] + rs;
      mrow[i] = mnew;
    }
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) oacc[m][i] *= alpha[i];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * lhi + i, key = 16 * n + l15;
        const int pc = (key >> 3) ^ ((r >> 1) & 7);
        *reinterpret_cast<bf16_t*>(ps_b + r * 128 + (pc << 4) + ((key & 7) << 1)) = f2bf(sacc[n][i]);
      }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    u16x8 pa[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = 4 * s + lhi;
      pa[s] = *reinterpret_cast<const u16x8*>(ps_b + l15 * 128 + ((ch ^ ((l15 >> 1) & 7)) << 4));
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int d = 16 * m + l15;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = 4 * s + lhi;
        const u16x8 vb = *reinterpret_cast<const u16x8*>(vt_b + d * 128 + ((ch ^ ((d >> 1) & 7)) << 4));
        oacc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(pa[s]), as_bf8(vb), oacc[m], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (!active) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = rbase + 4 * lhi + i;
    if (row < slen) {
      const float inv = lrow[i] > 0.f ? 1.f / lrow[i] : 0.f;
      bf16_t* dst = o + ((int64_t)(s0 + row) * Hq + hq) * D;
#pragma unroll
      for (int m = 0; m < 8; ++m) dst[16 * m + l15] = f2bf(oacc[m][i] * inv);
    }
  }
}

// ---------------------------------------------------------------------------
// v3: swapped-operand 32x32 MFMA kernel (cdna_hip_programming.md §3
// "accumulator tile as the next MFMA's operand", §5.5 T10/T12). Block = (32 x RG
// query rows, one KV head), 8 waves; wave w computes query head kvh * G + (w % G)
// for 32 rows starting 32 (w / G). Per 64-key tile:
//   S^T = K Q^T   v_mfma_f32_32x32x16_bf16, A = K rows from LDS, B = Q^T held in
//                 registers; the result has the query row on the lane and the keys
//                 in the 16 accumulator registers, so the softmax row max/sum is
//                 lane-local (one lane^32 exchange per tile for the max, none for
//                 the sum, which stays a per-lane partial until the epilogue)
//   O^T += V^T P^T  the S^T accumulator converted to bf16 IS the B operand (no LDS
//                 bounce for P); V^T comes from the row-major V tile with
//                 ds_read_b64_tr_b16 (hardware transpose)
// A 32-row wave reads each staged K/V byte from LDS once per 32 rows instead of
// once per 16 (v2), halving LDS read traffic per MFMA, and both tiles are staged
// with plain 16-B row writes (v2 scattered V with 2-B transposing writes).
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

// K tile image: rows padded to 272 B (kRowK), chunk ch of row r at 272 r + 16 ch -> the
// ds_read_b128 of 16 consecutive rows at one chunk hits 16 distinct bank groups, and a
// lane's reads of one tile are its row base plus compile-time offsets (no per-read
// address arithmetic, unlike an XOR swizzle).
constexpr int kRowK = 272;
__device__ __forceinline__ int k_img(int r, int ch) { return kRowK * r + 16 * ch; }
// V tile image (§5.5 T10 image (b)): conflict-free for the 32x32x16 transposed reads.
__device__ __forceinline__ int v_img(int r, int ch) { return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

__device__ __forceinline__ s16x4 ds_read_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// Shared prompt prefix (seq_pfx != nullptr): sequence seq's keys are seq_pfx[seq] prefix
// keys (rows of pk / pv [prefix, Hkv, D], the cached K/V of a prompt prefix many requests
// share) followed by its own slen keys; its query rows are its own tokens, at positions
// seq_pfx[seq] + row. Prefix keys are visible to every row; a last, partial prefix tile is
// masked past the prefix length.
// Schedule: the next tile's K/V loads are issued after this tile's S MFMAs (they are in
// flight during softmax + P.V instead of holding registers across the S MFMAs), and the
// rescale is deferred — a row keeps its running max until a tile raises it by more than 8
// (log2 units, so P <= 256 in fp32 / bf16), skipping the O / l rescale otherwise. Measured
// against the plain schedule on MI355X (profiles/prefill_attn_v3_schedule_variants.jsonl):
// 16x1024 0.290 vs 0.326 ms, 4x4096 0.857 vs 0.963 ms; the late loads alone, and two LDS
// tile buffers with one barrier per tile (with or without the deferred rescale), were
// slower than this pair and were removed.
// NW: waves per workgroup. 8 (one work item = 8 waves of (head, 32-row block)) holds a CU
// alone at 239 VGPRs (2 waves per SIMD), so every barrier of its K/V tile loop idles the
// CU; NW = 4 (G <= 4) halves the work item and puts two workgroups on each CU.
template <int G, int NW = 8>
__global__ void __launch_bounds__(NW * 64, 2) attn_prefill_mfma32_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, const int* __restrict__ cu_seqlens, const int* __restrict__ work_seq,
    const int* __restrict__ work_q0, int Hq, int Hkv, float scale_log2, const bf16_t* __restrict__ pk,
    const bf16_t* __restrict__ pv, const int* __restrict__ seq_pfx) {
  constexpr int D = 128, BK = 64, RG = NW / G, BQ = 32 * RG;
  constexpr int NT = NW * 64, NC = BK * 16 / NT;   // threads; 16-B K (and V) chunks each stages per tile
  static_assert(RG >= 1, "a workgroup needs a row block per head");
  __shared__ __attribute__((aligned(16))) char Ks[BK * kRowK];
  __shared__ __attribute__((aligned(16))) char Vs[BK * 256];

  const int wi = blockIdx.x, kvh = blockIdx.y;
  const int seq = work_seq[wi];
  if (seq < 0) return;  // padding item of a graph-captured prefill (fixed grid)
  const int s0 = cu_seqlens[seq];
  const int slen = cu_seqlens[seq + 1] - s0;
  const int q0 = work_q0[wi];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int hq = kvh * G + (w % G);
  const int rbase = q0 + 32 * (w / G);  // this wave's first query row
  const int qrow = rbase + r32;          // this lane's query row (C column)
  // G = 3, 5, 6, 7: only G x RG of the NW waves have a (head, row block); the rest
  // stage K/V tiles with the others and compute nothing
  const bool wave_used = w < G * RG;

  // Q^T as the B operand: k-step s covers d = 16s .. 16s+15; lane holds d = 16s + 8h + j
  u16x8 qb[8];
#pragma unroll
  for (int s = 0; s < 8; ++s)
    qb[s] = qrow < slen ? *reinterpret_cast<const u16x8*>(q + ((int64_t)(s0 + qrow) * Hq + hq) * D + 16 * s + 8 * h)
                        : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  f32x16 oacc[4];
#pragma unroll
  for (int dd = 0; dd < 4; ++dd)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[dd][i] = 0.f;
  float mrow = -INFINITY, lpart = 0.f;

  const int kend = min(slen, q0 + BQ);
  const int pl = seq_pfx != nullptr ? seq_pfx[seq] : 0;   // shared-prefix keys first
  const int npt = (pl + BK - 1) / BK;
  const int ntiles = npt + (kend + BK - 1) / BK;
  const bool active = wave_used && rbase < slen;
  const int wend = min(slen, rbase + 32);  // own keys this wave can see: < wend

  // transposed-read addressing: 16-lane group g reads rows r0 + q (q = i >> 2) at
  // columns d0 + 4p .. +3 (p = i & 3), d0 = 32 dd + 16 (g & 1); lane i gets column d0 + i
  const int gi = lane & 15, g = lane >> 4;
  const int trq = gi >> 2, trp = gi & 3;

  u16x8 kr[NC], vr[NC];
  auto load_tile = [&](int kt) {   // key tile kt: a prefix tile (kt < npt) or own tile kt - npt
#pragma unroll
    for (int r = 0; r < NC; ++r) {
      const int c = tid + r * NT;
      const int key = c >> 4, ch = c & 15;
      kr[r] = vr[r] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (kt < npt) {
        if (kt * BK + key < pl) {
          const int64_t off = ((int64_t)(kt * BK + key) * Hkv + kvh) * D + ch * 8;
          kr[r] = *reinterpret_cast<const u16x8*>(pk + off);
          vr[r] = *reinterpret_cast<const u16x8*>(pv + off);
        }
      } else if ((kt - npt) * BK + key < slen) {
        const int64_t off = ((int64_t)(s0 + (kt - npt) * BK + key) * Hkv + kvh) * D + ch * 8;
        kr[r] = *reinterpret_cast<const u16x8*>(k + off);
        vr[r] = *reinterpret_cast<const u16x8*>(v + off);
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int r = 0; r < NC; ++r) {
      const int c = tid + r * NT;
      const int key = c >> 4, ch = c & 15;
      *reinterpret_cast<u16x8*>(Ks + k_img(key, ch)) = kr[r];
      *reinterpret_cast<u16x8*>(Vs + v_img(key, ch)) = vr[r];
    }
  };

  load_tile(0);
  for (int kt = 0; kt < ntiles; ++kt) {
    const int kb = (kt - npt) * BK;   // own-key coordinates (negative: a prefix tile)
    const char* Kc = Ks;
    const char* Vc = Vs;
    __syncthreads();  // previous tile fully consumed
    store_tile();
    __syncthreads();
    if (!active || kb >= wend) {   // wave-uniform: no visible key for this wave
      if (kt + 1 < ntiles) load_tile(kt + 1);
      continue;
    }

    // ---- S^T = K Q^T (two 32-key blocks) ----
    f32x16 sacc[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[b][i] = 0.f;
      const int key = 32 * b + r32;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const u16x8 ka = *reinterpret_cast<const u16x8*>(Kc + k_img(key, 2 * s + h));
        sacc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf8(ka), as_bf8(qb[s]), sacc[b], 0, 0, 0);
      }
    }
    if (kt + 1 < ntiles) load_tile(kt + 1);   // in flight during softmax + P.V
    // ---- online softmax: register i of block b is key kb + 32b + (i&3) + 8(i>>2) + 4h ----
    const bool ptile = kb < 0;
    const int pend = pl - kt * BK;   // prefix tile: its keys below pend are prefix keys
    const bool mask = ptile ? (pend < BK) : ((kb + BK > rbase + 1) || (kb + BK > slen));
    float mx = -INFINITY;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float sv = sacc[b][i] * scale_log2;
        if (mask) {
          const int j = 32 * b + (i & 3) + 8 * (i >> 2) + 4 * h;   // key within the tile
          if (ptile ? (j >= pend) : (kb + j > qrow || kb + j >= slen)) sv = -INFINITY;
        }
        sacc[b][i] = sv;
        mx = fmaxf(mx, sv);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
    float mnew = fmaxf(mrow, mx);
    const bool rescale = mrow == -INFINITY || mnew > mrow + 8.f;   // deferred rescale
    if (!rescale) mnew = mrow;
    const float msafe = (mnew == -INFINITY) ? 0.f : mnew;
    const float alpha = rescale ? exp2f(mrow - msafe) : 1.f;
    mrow = mnew;
    float rs = 0.f;
    u16x8 pb[2][2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f32x8 p;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          p[j] = exp2f(sacc[b][8 * s + j] - msafe);
          rs += p[j];
        }
        pb[b][s] = __builtin_bit_cast(u16x8, __builtin_convertvector(p, bf16x8_t));
      }
    lpart = lpart * alpha + rs;
    if (rescale) {
#pragma unroll
      for (int dd = 0; dd < 4; ++dd)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dd][i] *= alpha;
    }

    // ---- O^T += V^T P^T: B element j of half h is key 32b + 16s + 8(j>>2) + 4h + (j&3) ----
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r0 = 32 * b + 16 * s + 4 * h + trq;
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
          const int d = 32 * dd + 16 * (g & 1) + 4 * trp;
          const s16x4 lo = ds_read_tr16(Vc + v_img(r0, d >> 3) + 8 * ((d >> 2) & 1));
          const s16x4 hi = ds_read_tr16(Vc + v_img(r0 + 8, d >> 3) + 8 * ((d >> 2) & 1));
          const s16x8 va = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          oacc[dd] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, va),
                                                            as_bf8(pb[b][s]), oacc[dd], 0, 0, 0);
        }
      }
  }
  if (!active) return;
  const float lsum = lpart + __shfl_xor(lpart, 32, kWave);
  if (qrow >= slen) return;
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  bf16_t* dst = o + ((int64_t)(s0 + qrow) * Hq + hq) * D;
  // O^T register i of d-block dd is d = 32 dd + (i&3) + 8(i>>2) + 4h: 4 contiguous d per 8-B store
#pragma unroll
  for (int dd = 0; dd < 4; ++dd)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      u16x4 st;
#pragma unroll
      for (int e = 0; e < 4; ++e) st[e] = f2bf(oacc[dd][4 * c + e] * inv);
      *reinterpret_cast<u16x4*>(dst + 32 * dd + 8 * c + 4 * h) = st;
    }
}

// Query rows per work item of each variant: 1 = per-query-head (64 rows, any G),
// 2 = GQA-grouped 16-row waves (G = Hq / Hkv in {1, 2, 4, 8}), 3 = GQA-grouped
// swapped 32x32 (32-row waves, any G <= 8: 8 / G row blocks per item); else -1.
int attn_prefill_block_q(int Hq, int Hkv, int variant) {
  if (variant == 1) return 64;
  if (Hkv <= 0 || Hq % Hkv != 0) return -1;
  const int G = Hq / Hkv;
  if (variant == 2 && (G == 1 || G == 2 || G == 4 || G == 8)) return 16 * (8 / G);
  if (variant == 3 && G >= 1 && G <= 8) return 32 * (8 / G);
  if (variant == 4 && G >= 1 && G <= 4) return 32 * (4 / G);   // v3 in 4-wave workgroups
  return -1;
}

int attn_prefill(const bf16_t* q, const bf16_t* k, const bf16_t* v, bf16_t* o, const int* cu_seqlens,
                 const int* work_seq, const int* work_q0, int num_work, int Hq, int Hkv, int head_dim,
                 float scale, int variant, hipStream_t stream, const bf16_t* pk, const bf16_t* pv,
                 const int* seq_pfx) {
  if (num_work == 0) return 0;
  if (head_dim != 128) return -1;
  if (Hq % Hkv != 0) return -3;
  if (attn_prefill_block_q(Hq, Hkv, variant) < 0) return -4;
  if (seq_pfx != nullptr && (variant < 3 || pk == nullptr || pv == nullptr)) return -5;   // v3 / v4 only
  const float sl2 = scale * 1.4426950408889634f;
  const int G = Hq / Hkv;
  if (variant == 1) {
    dim3 grid(num_work, Hq);
    attn_prefill_kernel<<<grid, 256, 0, stream>>>(q, k, v, o, cu_seqlens, work_seq, work_q0, Hq, Hkv, sl2);
  } else {
    dim3 grid(num_work, Hkv);
#define OAMD_PF(KERN, GG) KERN<GG><<<grid, 512, 0, stream>>>(q, k, v, o, cu_seqlens, work_seq, work_q0, Hq, Hkv, sl2)
#define OAMD_PF3(GG)                                                                                          \
  attn_prefill_mfma32_kernel<GG><<<grid, 512, 0, stream>>>(q, k, v, o, cu_seqlens, work_seq, work_q0, Hq, Hkv, sl2, \
                                                           pk, pv, seq_pfx)
#define OAMD_PF4(GG)                                                                                          \
  attn_prefill_mfma32_kernel<GG, 4><<<grid, 256, 0, stream>>>(q, k, v, o, cu_seqlens, work_seq, work_q0, Hq, Hkv,  \
                                                              sl2, pk, pv, seq_pfx)
#define OAMD_PF_G(KERN)            \
  switch (G) {                     \
    case 1: OAMD_PF(KERN, 1); break; \
    case 2: OAMD_PF(KERN, 2); break; \
    case 4: OAMD_PF(KERN, 4); break; \
    default: OAMD_PF(KERN, 8); break; \
  }
    if (variant == 2) {
      OAMD_PF_G(attn_prefill_gqa_kernel)
    } else if (variant == 4) {
      switch (G) {
        case 1: OAMD_PF4(1); break;
        case 2: OAMD_PF4(2); break;
        case 3: OAMD_PF4(3); break;
        default: OAMD_PF4(4); break;
      }
    } else {
      switch (G) {  // groups of Llama-3.2-3B (3), Qwen2.5-32B (5), Qwen2.5-7B (7)
        case 1: OAMD_PF3(1); break;
        case 2: OAMD_PF3(2); break;
        case 3: OAMD_PF3(3); break;
        case 4: OAMD_PF3(4); break;
        case 5: OAMD_PF3(5); break;
        case 6: OAMD_PF3(6); break;
        case 7: OAMD_PF3(7); break;
        default: OAMD_PF3(8); break;
      }
    }
#undef OAMD_PF4
#undef OAMD_PF3
#undef OAMD_PF_G
#undef OAMD_PF
  }
  OAMD_LAUNCH_CHECK();
  return 0;
}

}  // namespace oamd
