// Fused vocab projection + softmax cross-entropy for the MLM head (SURVEY K-12/K-13).
//
// Reference: TextOutputAdapter linear (perceiver/adapter.py:146-149) followed by
// rearrange + nn.CrossEntropyLoss(ignore_index=-100) (perceiver/lightning.py:223-226), which
// materialises (B, V, L) fp32 logits (20.5 MB/sample at L=512) plus a contiguous copy.
// Here logits exist only as MFMA accumulator tiles:
//   fwd  : per (64-row tile, vocab split): transposed logit tiles (W·Hᵀ: one row per lane),
//          running per-lane (max, sum-exp2) online logsumexp, label logit picked in passing;
//          a combine kernel merges splits → per-row loss and LSE.
//   bwd-a: dH  = (softmax − onehot)·g · W   (rows × vocab split, fp32 atomics into dH)
//   bwd-b: dW  = (softmax − onehot)ᵀ·g · H, db = Σ rows   (vocab chunk × row split, fp32 atomics)
// Streamed operands (W chunks, H tiles) are register-prefetched one tile ahead.
// Only the ~15 % masked positions are ever passed in (rows compacted on device).
#include <cstdlib>

#include "common.h"

namespace pio {

constexpr int HB = 64;  // rows per tile
constexpr int VB = 64;  // vocab entries per tile

// Transposed logits tile (vocab on the accumulator rows, the query row on the lane):
// wave w covers vocab [v0 + 32(w & 1), +32) × rows [m0 + 32(w >> 1), +32) of a 64 × 64 tile;
// lane l holds row 32(w >> 1) + (l & 31) and the 16 vocab entries 32(w & 1) + acc_row(i, l >> 5).
// With every value of a lane belonging to ONE row, the softmax statistics need no cross-lane
// work inside the vocab loop: one max over 16 registers, one rescale exp per tile, and one
// v_exp_f32 per logit (log2 domain) — ≈4 VALU instructions per logit instead of ≈20.
// A = W chunk [v][c], B = H tile [r][c] (both k-contiguous).
constexpr float kL2E = 1.4426950408889634f;
constexpr float kLN2 = 0.6931471805599453f;
template <int C>
__device__ __forceinline__ f32x16 logits_tile_t(const uint16_t* sH, const uint16_t* sW, int ld) {
  const int w = wave_id();
  f32x16 acc = f32x16{};
#pragma unroll
  for (int k0 = 0; k0 < C; k0 += 16) acc = mfma32(frag_kc(sW, ld, 32 * (w & 1), k0), frag_kc(sH, ld, 32 * (w >> 1), k0), acc);
  return acc;
}
// the 16 per-register values of a 64-entry LDS vector (vocab-indexed) for this lane:
// register i <-> entry 32(w & 1) + 4h + (i & 3) + 8(i >> 2): four 16-byte reads
__device__ __forceinline__ void vocab_regs(const float* sv, float (&out)[16]) {
  const float* p = sv + 32 * (wave_id() & 1) + 4 * (lane_id() >> 5);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 v = *reinterpret_cast<const float4*>(p + 8 * q);
    out[4 * q] = v.x; out[4 * q + 1] = v.y; out[4 * q + 2] = v.z; out[4 * q + 3] = v.w;
  }
}
// register of this lane holding entry j of the wave's 32-entry vocab block, or -1
__device__ __forceinline__ int vocab_reg(int j) {
  if (j < 0 || j >= 32 || ((j >> 2) & 1) != (lane_id() >> 5)) return -1;
  return (j & 3) + 4 * (j >> 3);
}
// Row r of the head input is H[idx[r]] (idx == nullptr: H[r]) of the fp32 decoder output: the
// compaction gather and the bf16 cast happen on load, no gathered copy is ever written.
template <int C>
__device__ __forceinline__ bf16x8 hrow8(const float* __restrict__ H, const int64_t* __restrict__ idx, int r, int c) {
  const long long row = idx ? idx[r] : (long long)r;
  const float4 a = *reinterpret_cast<const float4*>(H + row * C + c);
  const float4 b = *reinterpret_cast<const float4*>(H + row * C + c + 4);
  bf16x8 v;
  v[0] = (short)f2bf(a.x); v[1] = (short)f2bf(a.y); v[2] = (short)f2bf(a.z); v[3] = (short)f2bf(a.w);
  v[4] = (short)f2bf(b.x); v[5] = (short)f2bf(b.y); v[6] = (short)f2bf(b.z); v[7] = (short)f2bf(b.w);
  return v;
}

// rows [r0, r0+64) of H (gathered) → LDS bf16 [64][ld]
template <int C>
__device__ __forceinline__ void stage_hrows(uint16_t* s, int ld, const float* H, const int64_t* idx, int r0, int R) {
  constexpr int CH = C / 8;
  for (int e = threadIdx.x; e < 64 * CH; e += blockDim.x) {
    const int rr = e / CH, c = (e % CH) * 8;
    bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + rr < R) v = hrow8<C>(H, idx, r0 + rr, c);
    *reinterpret_cast<bf16x8*>(s + rr * ld + c) = v;
  }
}

// rows [r0, r0+64) × C of a bf16 row-major matrix → LDS
template <int C>
__device__ __forceinline__ void stage_rows(uint16_t* s, int ld, const uint16_t* g, int r0, int R) {
  constexpr int CH = C / 8;
  for (int e = threadIdx.x; e < 64 * CH; e += blockDim.x) {
    const int rr = e / CH, c = (e % CH) * 8;
    bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + rr < R) v = *reinterpret_cast<const bf16x8*>(g + (long long)(r0 + rr) * C + c);
    *reinterpret_cast<bf16x8*>(s + rr * ld + c) = v;
  }
}

// register-staged variant: rows [r0, r0+64) × C of a bf16 row-major matrix → NI = C/32
// 16-byte chunks per thread (issued early, written to LDS after the next barrier)
template <int C>
__device__ __forceinline__ void fetch_rows(bf16x8 (&v)[C / 32], const uint16_t* g, int r0, int R) {
  constexpr int CH = C / 8;
#pragma unroll
  for (int i = 0; i < C / 32; ++i) {
    const int e = threadIdx.x + 256 * i, rr = e / CH, c = (e % CH) * 8;
    v[i] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + rr < R) v[i] = *reinterpret_cast<const bf16x8*>(g + (long long)(r0 + rr) * C + c);
  }
}
template <int C>
__device__ __forceinline__ void store_rows(const bf16x8 (&v)[C / 32], uint16_t* s, int ld) {
  constexpr int CH = C / 8;
#pragma unroll
  for (int i = 0; i < C / 32; ++i) {
    const int e = threadIdx.x + 256 * i, rr = e / CH, c = (e % CH) * 8;
    *reinterpret_cast<bf16x8*>(s + rr * ld + c) = v[i];
  }
}

template <int C>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ Hm, const int64_t* __restrict__ hidx,
                                                     const int64_t* __restrict__ labels,
                                                     const uint16_t* __restrict__ W, const float* __restrict__ bias,
                                                     int M, int V, int chunks_per_split, float* __restrict__ part_ms,
                                                     float* __restrict__ picked, uint16_t* __restrict__ hs_out,
                                                     float* __restrict__ zero_out, long long zero_n4) {
  constexpr int LD = C + 8;
  __shared__ __attribute__((aligned(16))) uint16_t sH[HB * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[VB * LD];
  __shared__ __attribute__((aligned(16))) float sB[VB];  // bias * log2e of the chunk (-inf past V)
  __shared__ float sMS[2][64][2];
  const int w = wave_id(), l = lane_id();
  const int m0 = blockIdx.x * HB, split = blockIdx.y;
  const int nchunks = (V + VB - 1) / VB;
  const int c_begin = split * chunks_per_split, c_end = min(nchunks, c_begin + chunks_per_split);
  stage_hrows<C>(sH, LD, Hm, hidx, m0, M);
  if (split == 0 && hs_out != nullptr) {  // the compact bf16 rows for the backward kernels
    lds_sync();
    constexpr int CH = C / 8;
    for (int e = threadIdx.x; e < 64 * CH; e += blockDim.x) {
      const int rr = e / CH, c = (e % CH) * 8;
      if (m0 + rr < M)
        *reinterpret_cast<bf16x8*>(hs_out + (long long)(m0 + rr) * C + c) = *reinterpret_cast<const bf16x8*>(sH + rr * LD + c);
    }
  }
  const int rl = 32 * (w >> 1) + (l & 31), gr = m0 + rl;
  const int lab = gr < M ? (int)labels[gr] : -100;
#if PIO_CHECKS
  if (split == 0 && (w & 1) == 0 && (lab >= V || (lab < 0 && lab != -100))) pio_flag(kErrLabel);
#endif
  float m = -1e30f, s = 0.f;  // log2-domain running max / sum of 2^(t - m) over this lane's logits
  bf16x8 wr[C / 32];
  float bnext = 0.f;
  auto fetch = [&](int c) {
    fetch_rows<C>(wr, W, c * VB, V);
    const int v = c * VB + threadIdx.x;
    if (threadIdx.x < VB) bnext = v < V ? bias[v] * kL2E : -__builtin_inff();
  };
  if (c_begin < c_end) fetch(c_begin);
  for (int c = c_begin; c < c_end; ++c) {
    const int v0 = c * VB;
    lds_sync();
    store_rows<C>(wr, sW, LD);
    if (threadIdx.x < VB) sB[threadIdx.x] = bnext;
    lds_sync();
    if (c + 1 < c_end) fetch(c + 1);
    const f32x16 acc = logits_tile_t<C>(sH, sW, LD);
    float t[16];
    vocab_regs(sB, t);
    float mt = -__builtin_inff();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      t[i] = fmaf(acc[i], kL2E, t[i]);
      mt = fmaxf(mt, t[i]);
    }
    const float mn = fmaxf(m, mt);
    float acc_s = s * fast_exp2(m - mn);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc_s += fast_exp2(t[i] - mn);
    s = acc_s;
    m = mn;
    const int ri = vocab_reg(lab - v0 - 32 * (w & 1));
    if (ri >= 0) {  // this lane holds the label's logit (stored in natural units)
      float pv = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) pv = i == ri ? t[i] : pv;
      picked[gr] = pv * kLN2;
    }
  }
  // merge the two lanes of each row (l, l ^ 32), then the two waves sharing the rows
  float ma, mb, sa, sb;
  xor32_pair(m, ma, mb);
  xor32_pair(s, sa, sb);
  const float mm = fmaxf(ma, mb);
  const float ss = sa * fast_exp2(ma - mm) + sb * fast_exp2(mb - mm);
  if (l < 32) {
    sMS[w & 1][rl][0] = mm;
    sMS[w & 1][rl][1] = ss;
  }
  lds_sync();
  if (threadIdx.x < 64) {
    const int rr = threadIdx.x, g = m0 + rr;
    if (g < M) {
      const float m1 = sMS[0][rr][0], m2 = sMS[1][rr][0];
      const float mx = fmaxf(m1, m2);
      const float sx = sMS[0][rr][1] * fast_exp2(m1 - mx) + sMS[1][rr][1] * fast_exp2(m2 - mx);
      part_ms[((long long)split * M + g) * 2] = mx * kLN2;  // natural-log units for the combine
      part_ms[((long long)split * M + g) * 2 + 1] = sx;
    }
  }
  // the backward's atomically accumulated dH rows are cleared here (no separate fill launch)
  if (zero_out != nullptr) {
    const long long nwg = (long long)gridDim.x * gridDim.y, wg = (long long)split * gridDim.x + blockIdx.x;
    const long long per = (zero_n4 + nwg - 1) / nwg, z1 = min(zero_n4, (wg + 1) * per);
    for (long long i = wg * per + threadIdx.x; i < z1; i += blockDim.x)
      reinterpret_cast<float4*>(zero_out)[i] = float4{0.f, 0.f, 0.f, 0.f};
  }
}

// per-row lse (kept for backward) and loss = lse − picked (0 for ignored rows), kCombineQ threads
// per row (splits q, q + kCombineQ, … merged online, then across the group in LDS); the mean loss
// Σ rows / max(count, 1) is finalised in-kernel: each workgroup stores its partial sum, and the
// last one to take a ticket adds the partials in a fixed order (deterministic) and resets the
// ticket.  (picked[r] is written by the forward for every row with a label, so it needs no zero
// fill.)
constexpr int kCombineRows = 64, kCombineQ = 16;
__global__ __launch_bounds__(kCombineRows * kCombineQ) void ce_combine_kernel(
    const float* __restrict__ part_ms, const float* __restrict__ picked, const int64_t* __restrict__ labels, int M,
    int nsplit, float* __restrict__ lse, float* __restrict__ count, float* __restrict__ loss,
    float* __restrict__ blk, unsigned* __restrict__ ticket, int count_labels) {
  __shared__ float sM[kCombineQ][kCombineRows], sS[kCombineQ][kCombineRows], red[32];
  __shared__ int last;
  const int rr = threadIdx.x % kCombineRows, q = threadIdx.x / kCombineRows;
  const int r = blockIdx.x * kCombineRows + rr;
  float mx = -1e30f, sx = 0.f;
  if (r < M) {
    for (int s = q; s < nsplit; s += kCombineQ) {
      const float m = part_ms[((long long)s * M + r) * 2], e = part_ms[((long long)s * M + r) * 2 + 1];
      const float mn = fmaxf(mx, m);
      sx = sx * __expf(mx - mn) + e * __expf(m - mn);
      mx = mn;
    }
  }
  sM[q][rr] = mx;
  sS[q][rr] = sx;
  __syncthreads();
  float lr = 0.f, nr = 0.f;
  if (q == 0 && r < M) {
    float mm = sM[0][rr];
#pragma unroll
    for (int k = 1; k < kCombineQ; ++k) mm = fmaxf(mm, sM[k][rr]);
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < kCombineQ; ++k) ss += sS[k][rr] * __expf(sM[k][rr] - mm);
    const float L = mm + __logf(ss);
    lse[r] = L;
    const bool has = labels[r] >= 0;
    lr = has ? L - picked[r] : 0.f;
    nr = has ? 1.f : 0.f;
  }
  lr = wave_sum(lr);  // rows of q == 0 live in wave 0
  if (count_labels) nr = wave_sum(nr);
  // partials published write-through (sc1 agent-scope stores) and read back with sc1 loads by the
  // last arriver: no release / acquire fences (an L2 write-back per workgroup otherwise)
  if (threadIdx.x == 0) {
    __hip_atomic_store(reinterpret_cast<unsigned*>(blk + blockIdx.x), __float_as_uint(lr), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (count_labels)
      __hip_atomic_store(reinterpret_cast<unsigned*>(blk + gridDim.x + blockIdx.x), __float_as_uint(nr), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  float t = 0.f, n = 0.f;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) {
    t += __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(blk + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (count_labels)
      n += __uint_as_float(
          __hip_atomic_load(reinterpret_cast<unsigned*>(blk + gridDim.x + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  t = wave_sum(t);
  n = wave_sum(n);
  if (lane_id() == 0) { red[wave_id()] = t; red[16 + wave_id()] = n; }  // 16 waves
  __syncthreads();
  if (threadIdx.x == 0) {
    float tt = 0.f, nn = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { tt += red[k]; nn += red[16 + k]; }
    // count_labels: the denominator is the number of rows with a label (written for the backward)
    if (count_labels) count[0] = nn;
    loss[0] = tt / fmaxf(count_labels ? nn : count[0], 1.f);
    *ticket = 0u;
  }
}

// dl = (softmax - onehot) * g for the 16 logits of this lane's row (transposed tile):
// d_i = 2^(acc_i * log2e + b_i - lse * log2e) * g, minus g at the label's entry.  g = 0 for
// ignored rows (label -100: unselected positions and compaction padding).
__device__ __forceinline__ void dl_regs(const f32x16& acc, const float (&b)[16], float lse_l2, float g, int lab_reg,
                                        float (&d)[16]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) d[i] = fast_exp2(fmaf(acc[i], kL2E, b[i] - lse_l2)) * g;
  if (lab_reg >= 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] -= i == lab_reg ? g : 0.f;
  }
}

// ---- register-operand variants (default): the dl tile never goes through LDS -------------
// The logits tile's accumulator is used directly as an MFMA operand (pack_acc: the 16 values of
// a lane in the accumulator's permuted row order, matched by a frag_ks_perm read of the other
// operand), so a chunk costs two workgroup barriers instead of three and no dl store / reload.
// Each wave owns a (32-row, 32-vocab) quarter of the 64 × 64 tile; the two waves that share an
// output block add their partials once, through LDS, at the end.
__device__ __forceinline__ bf16x8 pack_regs(const float (&d)[16], int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(d[8 * s + j]);
  return r;
}
// owner wave parity of output tile t when two waves hold partials of it
template <int NT>
__device__ __forceinline__ int tile_owner(int t) { return NT == 1 ? 0 : (t & 1); }

// bwd-a: dH[r][c] += Σ_v dl[r][v] W[v][c]; wave w: rows 32(w >> 1) + [0, 32), vocab 32(w & 1) + [0, 32)
// of each chunk (the transposed logits tile: a lane holds one row), partial over its vocab half
template <int C>
__global__ __launch_bounds__(256) void ce_bwd_dh_reg_kernel(const uint16_t* __restrict__ Hm,
                                                            const int64_t* __restrict__ labels,
                                                            const uint16_t* __restrict__ W, const float* __restrict__ bias,
                                                            const float* __restrict__ lse, const float* __restrict__ gout,
                                                            const float* __restrict__ count, int M, int V,
                                                            int chunks_per_split, float* __restrict__ dH,
                                                            const int64_t* __restrict__ rowmap, long long dh_rows) {
  constexpr int LD = C + 8, NT = C / 32;
  __shared__ __attribute__((aligned(16))) uint16_t sH[HB * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[VB * LD];
  __shared__ __attribute__((aligned(16))) float sB[VB];
  __shared__ __attribute__((aligned(16))) float sX[2][NT][16 * 64];
  __shared__ long long sDst[HB];  // dH row of each tile row (-1: ignored row)
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int m0 = blockIdx.x * HB, split = blockIdx.y;
  const int nchunks = (V + VB - 1) / VB;
  const int c_begin = split * chunks_per_split, c_end = min(nchunks, c_begin + chunks_per_split);
  stage_rows<C>(sH, LD, Hm, m0, M);
  if (threadIdx.x < HB) {
    const int gr = m0 + threadIdx.x;
    const long long r = (gr < M && labels[gr] >= 0) ? (rowmap ? rowmap[gr] : gr) : -1;
    sDst[threadIdx.x] = r < dh_rows ? r : -1;  // a row outside dH is dropped, never written
  }
  const int rl = 32 * (w >> 1) + (l & 31), gr = m0 + rl;
  const int lab = gr < M ? (int)labels[gr] : -100;
  const float lse_l2 = gr < M ? lse[gr] * kL2E : 0.f;
  const float g = lab >= 0 ? gout[0] / fmaxf(count[0], 1.f) : 0.f;  // d(mean loss) / d(row loss)
  f32x16 acc_o[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc_o[t] = f32x16{};
  bf16x8 wr[C / 32];
  float bnext = 0.f;
  auto fetch = [&](int c) {
    fetch_rows<C>(wr, W, c * VB, V);
    const int v = c * VB + threadIdx.x;
    if (threadIdx.x < VB) bnext = v < V ? bias[v] * kL2E : -__builtin_inff();
  };
  if (c_begin < c_end) fetch(c_begin);
  for (int c = c_begin; c < c_end; ++c) {
    const int v0 = c * VB;
    lds_sync();
    store_rows<C>(wr, sW, LD);
    if (threadIdx.x < VB) sB[threadIdx.x] = bnext;
    lds_sync();
    if (c + 1 < c_end) fetch(c + 1);
    const f32x16 acc = logits_tile_t<C>(sH, sW, LD);
    float b[16], d[16];
    vocab_regs(sB, b);
    dl_regs(acc, b, lse_l2, g, vocab_reg(lab - v0 - 32 * (w & 1)), d);
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 pa = pack_regs(d, ss);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc_o[t] = mfma32(pa, frag_ks_perm(sW, LD, 32 * t, 32 * (w & 1) + 16 * ss), acc_o[t]);
    }
  }
  // the two vocab halves of each row block: the non-owner hands its partial over
#pragma unroll
  for (int t = 0; t < NT; ++t)
    if ((w & 1) != tile_owner<NT>(t)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sX[w >> 1][t][i * 64 + l] = acc_o[t][i];
    }
  lds_sync();  // also publishes sDst (no in-loop barrier has run for an empty split)
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if ((w & 1) != tile_owner<NT>(t)) continue;
    const int r0 = 32 * (w >> 1), n0 = 32 * t;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      // dH row: the compacted row's source position (rowmap) or the row itself; ignored rows
      // (label -100, incl. compaction padding) carry no gradient
      const long long dst = sDst[r0 + acc_row(i, hh)];
      if (dst >= 0) atomicAdd(dH + dst * C + n0 + (l & 31), acc_o[t][i] + sX[w >> 1][t][i * 64 + l]);
    }
  }
}

// bwd-b: dW[v][c] += Σ_r dl[r][v] H[r][c], db[v] += Σ_r dl[r][v]; grid (vocab chunk, row split).
// The logits tile is NOT transposed here (a lane holds one vocab entry), so dl feeds the dW
// product as its A operand directly; wave w: rows 32(w >> 1), vocab 32(w & 1), partial over its
// row half.  H tiles (+ their LSE / labels) are register-prefetched one tile ahead.
template <int C>
__global__ __launch_bounds__(256) void ce_bwd_dw_reg_kernel(const uint16_t* __restrict__ Hm,
                                                            const int64_t* __restrict__ labels,
                                                            const uint16_t* __restrict__ W, const float* __restrict__ bias,
                                                            const float* __restrict__ lse, const float* __restrict__ gout,
                                                            const float* __restrict__ count, int M, int V,
                                                            int tiles_per_split, float* __restrict__ dW,
                                                            float* __restrict__ db, float* __restrict__ slab) {
  constexpr int LD = C + 8, NT = C / 32;
  __shared__ __attribute__((aligned(16))) uint16_t sH[HB * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[VB * LD];
  __shared__ __attribute__((aligned(16))) float sLse[HB];
  __shared__ __attribute__((aligned(16))) float sG[HB];    // row-loss gradient (0: ignored row)
  __shared__ __attribute__((aligned(16))) int sLab[HB];
  __shared__ __attribute__((aligned(16))) float sX[2][NT][16 * 64];
  __shared__ float sBs[2][64];
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int v0 = blockIdx.x * VB;
  const int mt_begin = blockIdx.y * tiles_per_split;
  const int mt_end = min((M + HB - 1) / HB, mt_begin + tiles_per_split);
  const float gs = gout[0] / fmaxf(count[0], 1.f);
  stage_rows<C>(sW, LD, W, v0, V);
  const int vl = 32 * (w & 1) + (l & 31), vg = v0 + vl;  // this lane's vocab entry
  const float bl2 = vg < V ? bias[vg] * kL2E : -__builtin_inff();
  const int r0 = 32 * (w >> 1);
  f32x16 acc_o[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc_o[t] = f32x16{};
  float bsum = 0.f;
  bf16x8 hr[C / 32];
  float aux = 0.f;  // threads [0,64): LSE * log2e of row tid, [64,128): label of row tid-64
  auto fetch = [&](int mt) {
    fetch_rows<C>(hr, Hm, mt * HB, M);
    const int t = threadIdx.x & 63, gr = mt * HB + t;
    if (threadIdx.x < 64) aux = gr < M ? lse[gr] * kL2E : 0.f;
    else if (threadIdx.x < 128) aux = __int_as_float(gr < M ? (int)labels[gr] : -100);
  };
  if (mt_begin < mt_end) fetch(mt_begin);
  for (int mt = mt_begin; mt < mt_end; ++mt) {
    lds_sync();
    store_rows<C>(hr, sH, LD);
    if (threadIdx.x < 64) {
      sLse[threadIdx.x] = aux;
    } else if (threadIdx.x < 128) {
      const int lb = __float_as_int(aux);
      sLab[threadIdx.x - 64] = lb;
      sG[threadIdx.x - 64] = lb >= 0 ? gs : 0.f;
    }
    lds_sync();
    if (mt + 1 < mt_end) fetch(mt + 1);
    f32x16 acc = f32x16{};
#pragma unroll
    for (int k0 = 0; k0 < C; k0 += 16) acc = mfma32(frag_kc(sH, LD, r0, k0), frag_kc(sW, LD, 32 * (w & 1), k0), acc);
    float d[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // rows r0 + 4hh + 8q + (0..3): four consecutive LDS entries
      const int rr = r0 + 4 * hh + 8 * q;
      const float4 ls = *reinterpret_cast<const float4*>(sLse + rr);
      const float4 gg = *reinterpret_cast<const float4*>(sG + rr);
      const int4 lb = *reinterpret_cast<const int4*>(sLab + rr);
      const float lsv[4] = {ls.x, ls.y, ls.z, ls.w}, ggv[4] = {gg.x, gg.y, gg.z, gg.w};
      const int lbv[4] = {lb.x, lb.y, lb.z, lb.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * q + j;
        const float p = fast_exp2(fmaf(acc[i], kL2E, bl2 - lsv[j])) * ggv[j];
        d[i] = lbv[j] == vg ? p - ggv[j] : p;
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) bsum += d[i];
    // dW (vocab 32(w & 1) + [0, 32) × C) += dlᵀ · H over this wave's 32 rows
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 pa = pack_regs(d, ss);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc_o[t] = mfma32(pa, frag_ks_perm(sH, LD, 32 * t, r0 + 16 * ss), acc_o[t]);
    }
  }
  // bias: the lane's vocab entry summed over its 16 rows, then the other lane half, then the
  // other row-half wave
  bsum = xor32_sum(bsum);
  if (l < 32) sBs[w >> 1][vl] = bsum;
#pragma unroll
  for (int t = 0; t < NT; ++t)
    if ((w >> 1) != tile_owner<NT>(t)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sX[w & 1][t][i * 64 + l] = acc_o[t][i];
    }
  lds_sync();
  // partials: atomics into dW / db, or (slab) plain stores into row blockIdx.y of a
  // (row splits, V·C + V₄) slab that a SlabJob later sums into dW | db (common.h)
  float* dWp = dW;
  float* dbp = db;
  if (slab) {
    dWp = slab + (long long)blockIdx.y * ((long long)V * C + ((V + 3) & ~3));
    dbp = dWp + (long long)V * C;
  }
  if (threadIdx.x < 64 && v0 + threadIdx.x < V) {
    const float v = sBs[0][threadIdx.x] + sBs[1][threadIdx.x];
    if (slab) dbp[v0 + threadIdx.x] = v;
    else atomicAdd(dbp + v0 + threadIdx.x, v);
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if ((w >> 1) != tile_owner<NT>(t)) continue;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int vv = v0 + 32 * (w & 1) + acc_row(i, hh);
      float* p = dWp + (long long)vv * C + 32 * t + (l & 31);
      const float x = acc_o[t][i] + sX[w & 1][t][i * 64 + l];
      if (vv < V) {
        if (slab) *p = x;
        else atomicAdd(p, x);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// selected-position bookkeeping for the MLM loss (replaces ~15 small framework kernels)
//   rows  : per sequence b, slots [0, cap): positions of labels != -100 in order (unused
//           slots → slot mod L, label −100), count[b]
//   global: the valid slots of all sequences compacted into gcap rows for the vocab GEMMs
//           (unused → slot 0 with label −100), total = Σ count (the mean's denominator)
// ------------------------------------------------------------------------------------
// select_rows: workgroup b compacts sequence b.  select_global, workgroup (b, 0): finds sequence
// b's offset in the global rows from all the per-sequence counts (each workgroup scans them
// itself: no grid-wide hand-off) and writes its valid slots; workgroup (0, 0) also writes the
// totals, the last one the unused tail.  Every workgroup (b, y) also copies the output-query rows
// q[b, j] = P[idx_b[b, j]] of its kSelSlots slots (the gather of the decoder's query array,
// spread over the whole grid).
constexpr int kSelThreads = 1024;
constexpr int kSelSlots = 128;  // query-gather slots per select_global workgroup
__global__ __launch_bounds__(kSelThreads) void select_rows_kernel(const int64_t* __restrict__ labels, int L, int cap,
                                                                  int64_t* __restrict__ idx_b, int64_t* __restrict__ lab_b,
                                                                  int* __restrict__ count) {
  __shared__ int sW[kSelThreads / 64], sOff;
  const int b = blockIdx.x, w = wave_id(), l = lane_id(), nw = blockDim.x >> 6;
  if (threadIdx.x == 0) sOff = 0;
  lds_sync();
  for (int c0 = 0; c0 < L; c0 += blockDim.x) {
    const int i = c0 + threadIdx.x;
    const int64_t lab = i < L ? labels[(long long)b * L + i] : -100;
    const bool sel = lab != -100;
    const uint64_t m = __ballot(sel);
    const int pre = __popcll(m & ((1ull << l) - 1ull));
    if (l == 0) sW[w] = __popcll(m);
    lds_sync();
    int woff = 0, tot = 0;
    for (int k = 0; k < nw; ++k) {
      woff += k < w ? sW[k] : 0;
      tot += sW[k];
    }
    const int pos = sOff + woff + pre;
    if (sel && pos < cap) {
      idx_b[(long long)b * cap + pos] = i;
      lab_b[(long long)b * cap + pos] = lab;
    }
    lds_sync();
    if (threadIdx.x == 0) sOff += tot;
    lds_sync();
  }
  const int cnt = sOff;
  for (int j = (cnt < cap ? cnt : cap) + threadIdx.x; j < cap; j += blockDim.x) {
    idx_b[(long long)b * cap + j] = j % L;
    lab_b[(long long)b * cap + j] = -100;
  }
  if (threadIdx.x == 0) count[b] = cnt;
}

__device__ __forceinline__ int wave_isum(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

__global__ __launch_bounds__(256) void select_global_kernel(const int* __restrict__ count, int B, int cap,
                                                            const int64_t* __restrict__ lab_b, int gcap,
                                                            int64_t* __restrict__ gidx, int64_t* __restrict__ glab,
                                                            float* __restrict__ total, bool* __restrict__ overflow,
                                                            bool* __restrict__ sticky, const int64_t* __restrict__ idx_b,
                                                            const float* __restrict__ P, int C, float* __restrict__ q) {
  __shared__ int sRed[4][4];
  __shared__ long long sI[kSelSlots];
  const int b = blockIdx.x, w = wave_id(), l = lane_id();
  if (q != nullptr) {  // slots [kSelSlots·y, +kSelSlots) of sequence b: q[b, j] = P[idx_b[b, j]]
    const int C4 = C >> 2, j0 = blockIdx.y * kSelSlots, nj = min(cap - j0, kSelSlots);
    const float4* P4 = reinterpret_cast<const float4*>(P);
    float4* q4 = reinterpret_cast<float4*>(q) + ((long long)b * cap + j0) * C4;
    for (int j = threadIdx.x; j < nj; j += blockDim.x) sI[j] = idx_b[(long long)b * cap + j0 + j];
    __syncthreads();
    for (int e0 = 0; e0 < nj * C4; e0 += 8 * 256) {  // eight independent row loads in flight per thread
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 256 + threadIdx.x;
        if (e < nj * C4) {
          const int j = e / C4;
          v[u] = P4[sI[j] * C4 + (e - j * C4)];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 256 + threadIdx.x;
        if (e < nj * C4) q4[e] = v[u];
      }
    }
  }
  if (blockIdx.y != 0) return;
  int pre = 0, used = 0, all = 0, ovf = 0;
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    const int c = count[i], n = c < cap ? c : cap;
    pre += i < b ? n : 0;
    used += n;
    all += c;
    ovf += c > cap ? 1 : 0;
  }
  pre = wave_isum(pre); used = wave_isum(used); all = wave_isum(all); ovf = wave_isum(ovf);
  if (l == 0) { sRed[0][w] = pre; sRed[1][w] = used; sRed[2][w] = all; sRed[3][w] = ovf; }
  __syncthreads();
  pre = sRed[0][0] + sRed[0][1] + sRed[0][2] + sRed[0][3];
  used = sRed[1][0] + sRed[1][1] + sRed[1][2] + sRed[1][3];
  const int c = count[b], n = c < cap ? c : cap;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const int g = pre + j;
    if (g < gcap) {
      const long long s = (long long)b * cap + j;
      gidx[g] = s;
      glab[g] = lab_b[s];
    }
  }
  if (b == B - 1)
    for (int g = (used < gcap ? used : gcap) + threadIdx.x; g < gcap; g += blockDim.x) {
      gidx[g] = 0;
      glab[g] = -100;
    }
  if (b == 0 && threadIdx.x == 0) {
    const bool o = (sRed[3][0] + sRed[3][1] + sRed[3][2] + sRed[3][3]) > 0 || used > gcap;
    total[0] = (float)(sRed[2][0] + sRed[2][1] + sRed[2][2] + sRed[2][3]);
    overflow[0] = o;
    if (sticky != nullptr && o) sticky[0] = true;  // the persistent per-device flag (never cleared here)
  }
}

void mlm_select_launch(const int64_t* labels, int B, int L, int cap, int gcap, int64_t* idx_b, int64_t* lab_b,
                       int* count, int64_t* gidx, int64_t* glab, float* total, bool* overflow, bool* sticky,
                       const float* P, int C, float* q, hipStream_t st) {
  hipLaunchKernelGGL(select_rows_kernel, dim3(B), dim3(kSelThreads), 0, st, labels, L, cap, idx_b, lab_b, count);
  const int gy = q ? (cap + kSelSlots - 1) / kSelSlots : 1;
  hipLaunchKernelGGL(select_global_kernel, dim3(B, gy), dim3(256), 0, st, count, B, cap, lab_b, gcap, gidx, glab, total,
                     overflow, sticky, idx_b, P, C, q);
}

// vocab splits so that a launch has ≈ target workgroups (several per CU hide the W-chunk latency);
// rounded so that every split owns at least one chunk (ceil(nchunks / ceil(nchunks / s)) splits)
static int pick_split(int M, int nchunks, int target) {
  const int mt = (M + HB - 1) / HB;
  int s = (target + mt - 1) / mt;
  s = s < 1 ? 1 : (s > nchunks ? nchunks : s);
  const int cps = (nchunks + s - 1) / s;
  return (nchunks + cps - 1) / cps;
}

int ce_combine_blocks(int M);

// workgroup targets of the three CE launches (the C = 32 / 128 heads; C = 64 runs ce_head.hip)
static int ce_target(const char*, int dflt) { return dflt; }

// tickets: one zeroed counter (the combine kernel's)
void ce_fwd_launch(int C, const float* Hm, const int64_t* hidx, const int64_t* labels, const uint16_t* W,
                   const float* bias, int M, int V, float* part_ms, float* picked, float* lse, float* count,
                   float* loss, float* blk, unsigned* tickets, uint16_t* hs_out, int nsplit, float* zero_out,
                   long long zero_n, int count_labels, hipStream_t st) {
  const int nchunks = (V + VB - 1) / VB;
  const int cps = (nchunks + nsplit - 1) / nsplit;
  dim3 grid((M + HB - 1) / HB, nsplit);
#define CEF(CC)                                                                                                 \
  hipLaunchKernelGGL(ce_fwd_kernel<CC>, grid, dim3(256), 0, st, Hm, hidx, labels, W, bias, M, V, cps, part_ms, picked, \
                     hs_out, zero_out, zero_n / 4)
  if (C == 64) { CEF(64); }
  else if (C == 128) { CEF(128); }
  else if (C == 32) { CEF(32); }
#undef CEF
  hipLaunchKernelGGL(ce_combine_kernel, dim3(ce_combine_blocks(M)), dim3(kCombineRows * kCombineQ), 0, st, part_ms, picked,
                     labels, M, nsplit,
                     lse, count, loss, blk, tickets, count_labels);
}

int ce_combine_blocks(int M) { return (M + kCombineRows - 1) / kCombineRows; }

int ce_num_splits(int M, int V) { return pick_split(M, (V + VB - 1) / VB, ce_target("PIO_CE_FWD_WGS", 2048)); }

// row splits of the dW kernel (≈ 4 workgroups per CU): the slab height in slab mode
int ce_dw_splits(int M, int V) {
  const int nchunks = (V + VB - 1) / VB, mtiles = (M + HB - 1) / HB;
  int rsplit = (ce_target("PIO_CE_DW_WGS", 1024) + nchunks - 1) / nchunks;
  rsplit = rsplit < 1 ? 1 : (rsplit > mtiles ? mtiles : rsplit);
  const int tps = (mtiles + rsplit - 1) / rsplit;
  return (mtiles + tps - 1) / tps;
}

void ce_bwd_launch(int C, const uint16_t* Hm, const int64_t* labels, const uint16_t* W,
                   const float* bias, const float* lse, const float* gout, const float* count, int M, int V, float* dH, long long dh_rows, const int64_t* rowmap, float* dW,
                   float* db, int accumulate, float* slab, int det, hipStream_t st) {
  const int nchunks = (V + VB - 1) / VB;
  // dH partials are added atomically: few splits; deterministic mode: one (a single writer per
  // dH element — every compacted row maps to its own source position)
  const int nsplit = det ? 1 : pick_split(M, nchunks, ce_target("PIO_CE_DH_WGS", 1024));
  const int cps = (nchunks + nsplit - 1) / nsplit;
  // dW: (vocab chunk × row split) workgroups, ≈ 4 per CU; dW / db partials added atomically
  // or stored into the slab
  const int mtiles = (M + HB - 1) / HB;
  const int rsplit = ce_dw_splits(M, V);
  const int tps = (mtiles + rsplit - 1) / rsplit;
  if (!accumulate) {
    (void)hipMemsetAsync(dW, 0, sizeof(float) * (size_t)V * C, st);
    (void)hipMemsetAsync(db, 0, sizeof(float) * (size_t)V, st);
  }
  dim3 ga((M + HB - 1) / HB, nsplit), gb(nchunks, rsplit);
#define CEB(CC)                                                                                                 \
  hipLaunchKernelGGL(ce_bwd_dh_reg_kernel<CC>, ga, dim3(256), 0, st, Hm, labels, W, bias, lse, gout, count, M, V,   \
                     cps, dH, rowmap, dh_rows);                                                                    \
  hipLaunchKernelGGL(ce_bwd_dw_reg_kernel<CC>, gb, dim3(256), 0, st, Hm, labels, W, bias, lse, gout, count, M, V,   \
                     tps, dW, db, slab)
  if (C == 64) { CEB(64); }
  else if (C == 128) { CEB(128); }
  else if (C == 32) { CEB(32); }
#undef CEB
}

}  // namespace pio

namespace pio {
unsigned check_errors_mlm_head(bool reset) { return pio_read_errors(reset); }
}  // namespace pio

