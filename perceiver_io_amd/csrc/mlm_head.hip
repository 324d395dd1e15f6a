// Fused vocab projection + softmax cross-entropy for the MLM head (SURVEY K-12/K-13).
//
// Reference: TextOutputAdapter linear (perceiver/adapter.py:146-149) followed by
// rearrange + nn.CrossEntropyLoss(ignore_index=-100) (perceiver/lightning.py:223-226), which
// materialises (B, V, L) fp32 logits (20.5 MB/sample at L=512) plus a contiguous copy.
// Here logits exist only as MFMA accumulator tiles:
//   fwd  : per (64-row tile, vocab split): logits = H·Wᵀ + b tile by tile, running
//          per-lane (max, sum-exp) with a deferred-rescale online logsumexp, label logit
//          picked in passing; a combine kernel merges splits → per-row loss and LSE.
//   bwd-a: dH  = (softmax − onehot)·g · W   (rows × vocab split, fp32 atomics into dH)
//   bwd-b: dW  = (softmax − onehot)ᵀ·g · H, db = Σ rows   (vocab chunk × row split, fp32 atomics)
// Streamed operands (W chunks, H tiles) are register-prefetched one tile ahead.
// Only the ~15 % masked positions are ever passed in (rows compacted on device).
#include "common.h"

namespace pio {

constexpr int HB = 64;  // rows per tile
constexpr int VB = 64;  // vocab entries per tile

// logits tile for rows [m0, m0+64) × vocab [v0, v0+64): 4 sub-tiles, one per wave
// A = H tile [r][c] (k-contiguous), B = W chunk [v][c] (k-contiguous)
template <int C>
__device__ __forceinline__ f32x16 logits_tile(const uint16_t* sH, const uint16_t* sW, int ld) {
  const int w = wave_id();
  f32x16 acc = f32x16{};
#pragma unroll
  for (int k0 = 0; k0 < C; k0 += 16) acc = mfma32(frag_kc(sH, ld, 32 * (w >> 1), k0), frag_kc(sW, ld, 32 * (w & 1), k0), acc);
  return acc;
}

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
__global__ __launch_bounds__(256) void ce_fwd_kernel(const uint16_t* __restrict__ Hm, const int64_t* __restrict__ labels,
                                                     const uint16_t* __restrict__ W, const float* __restrict__ bias,
                                                     int M, int V, int chunks_per_split, float* __restrict__ part_ms,
                                                     float* __restrict__ picked) {
  constexpr int LD = C + 8;
  __shared__ __attribute__((aligned(16))) uint16_t sH[HB * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[VB * LD];
  __shared__ float sMS[2][64][2];
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int m0 = blockIdx.x * HB, split = blockIdx.y;
  const int nchunks = (V + VB - 1) / VB;
  const int c_begin = split * chunks_per_split, c_end = min(nchunks, c_begin + chunks_per_split);
  stage_rows<C>(sH, LD, Hm, m0, M);
  int lab[16];
  float m[16], s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int gr = m0 + 32 * (w >> 1) + acc_row(i, hh);
    lab[i] = gr < M ? (int)labels[gr] : -100;
    m[i] = -1e30f;
    s[i] = 0.f;
  }
  bf16x8 wr[C / 32];
  if (c_begin < c_end) fetch_rows<C>(wr, W, c_begin * VB, V);
  for (int c = c_begin; c < c_end; ++c) {
    const int v0 = c * VB;
    __syncthreads();
    store_rows<C>(wr, sW, LD);
    __syncthreads();
    if (c + 1 < c_end) fetch_rows<C>(wr, W, v0 + VB, V);
    const int col = v0 + 32 * (w & 1) + (l & 31);
    const bool valid = col < V;
    const float bv = valid ? bias[col] : 0.f;
    const f32x16 acc = logits_tile<C>(sH, sW, LD);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (valid) {
        const float v = acc[i] + bv;
        if (v > m[i]) { s[i] *= __expf(m[i] - v); m[i] = v; }
        s[i] += __expf(v - m[i]);
        if (col == lab[i]) picked[m0 + 32 * (w >> 1) + acc_row(i, hh)] = v;
      }
    }
  }
  // combine over the 32 lanes of each half (same rows), then the two waves sharing rows
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float mm = half_max(m[i]);
    const float ss = half_sum(s[i] * __expf(m[i] - mm));
    if ((l & 31) == 0) {
      const int rr = 32 * (w >> 1) + acc_row(i, hh);
      sMS[w & 1][rr][0] = mm;
      sMS[w & 1][rr][1] = ss;
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int rr = threadIdx.x, gr = m0 + rr;
    if (gr < M) {
      const float m1 = sMS[0][rr][0], m2 = sMS[1][rr][0];
      const float mm = fmaxf(m1, m2);
      const float ss = sMS[0][rr][1] * __expf(m1 - mm) + sMS[1][rr][1] * __expf(m2 - mm);
      part_ms[((long long)split * M + gr) * 2] = mm;
      part_ms[((long long)split * M + gr) * 2 + 1] = ss;
    }
  }
}

// per-row loss = lse − picked (0 for ignored rows); lse kept for backward
__global__ void ce_combine_kernel(const float* __restrict__ part_ms, const float* __restrict__ picked,
                                  const int64_t* __restrict__ labels, int M, int nsplit, float* __restrict__ loss_rows,
                                  float* __restrict__ lse) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= M) return;
  float mm = -1e30f;
  for (int s = 0; s < nsplit; ++s) mm = fmaxf(mm, part_ms[((long long)s * M + r) * 2]);
  float ss = 0.f;
  for (int s = 0; s < nsplit; ++s) ss += part_ms[((long long)s * M + r) * 2 + 1] * __expf(part_ms[((long long)s * M + r) * 2] - mm);
  const float L = mm + __logf(ss);
  lse[r] = L;
  loss_rows[r] = labels[r] >= 0 ? L - picked[r] : 0.f;
}

// dlogit for one accumulator element
__device__ __forceinline__ float dlogit(float v, float lse, int col, int lab, float g) {
  return lab < 0 ? 0.f : (__expf(v - lse) - (col == lab ? 1.f : 0.f)) * g;
}

// bwd-a: dH[r][c] += Σ_v dl[r][v] W[v][c]  over this split's vocab chunks (fp32 atomics)
template <int C>
__global__ __launch_bounds__(256) void ce_bwd_dh_kernel(const uint16_t* __restrict__ Hm,
                                                        const int64_t* __restrict__ labels,
                                                        const uint16_t* __restrict__ W, const float* __restrict__ bias,
                                                        const float* __restrict__ lse, const float* __restrict__ gscale,
                                                        int M, int V, int chunks_per_split, float* __restrict__ dH,
                                                        const int64_t* __restrict__ rowmap) {
  constexpr int LD = C + 8, LDL = VB + 8, NT = C / 32;
  __shared__ __attribute__((aligned(16))) uint16_t sH[HB * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[VB * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sL[HB * LDL];
  __shared__ long long sDst[HB];  // dH row of each tile row (−1: ignored row)
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int m0 = blockIdx.x * HB, split = blockIdx.y;
  const int nchunks = (V + VB - 1) / VB;
  const int c_begin = split * chunks_per_split, c_end = min(nchunks, c_begin + chunks_per_split);
  const float g = gscale[0];
  stage_rows<C>(sH, LD, Hm, m0, M);
  if (threadIdx.x < HB) {
    const int gr = m0 + threadIdx.x;
    sDst[threadIdx.x] = (gr < M && labels[gr] >= 0) ? (rowmap ? rowmap[gr] : gr) : -1;
  }
  int lab[16];
  float ls[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int gr = m0 + 32 * (w >> 1) + acc_row(i, hh);
    lab[i] = gr < M ? (int)labels[gr] : -100;
    ls[i] = gr < M ? lse[gr] : 0.f;
  }
  // output dH tile 64 × C: sub-tiles (2 × NT), wave w owns tiles w, w+4
  constexpr int MAXT = (2 * NT + 3) / 4;
  f32x16 acc_o[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc_o[t] = f32x16{};
  bf16x8 wr[C / 32];
  if (c_begin < c_end) fetch_rows<C>(wr, W, c_begin * VB, V);
  for (int c = c_begin; c < c_end; ++c) {
    const int v0 = c * VB;
    __syncthreads();
    store_rows<C>(wr, sW, LD);
    __syncthreads();
    if (c + 1 < c_end) fetch_rows<C>(wr, W, v0 + VB, V);
    const int coll = 32 * (w & 1) + (l & 31);
    const int col = v0 + coll;
    const bool valid = col < V;
    const float bv = valid ? bias[col] : 0.f;
    const f32x16 acc = logits_tile<C>(sH, sW, LD);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float d = valid ? dlogit(acc[i] + bv, ls[i], col, lab[i], g) : 0.f;
      sL[(32 * (w >> 1) + acc_row(i, hh)) * LDL + coll] = f2bf(d);
    }
    __syncthreads();
    // dH += dl (64 × 64 vocab) · Wchunk (64 vocab × C): A k-contiguous, B = W[v][c] k-strided
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      const int tg = w + 4 * t;
      if (tg < 2 * NT) {
        const int r0 = 32 * (tg / NT), n0 = 32 * (tg % NT);
#pragma unroll
        for (int k0 = 0; k0 < VB; k0 += 16) acc_o[t] = mfma32(frag_kc(sL, LDL, r0, k0), frag_ks(sW, LD, n0, k0), acc_o[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int tg = w + 4 * t;
    if (tg < 2 * NT) {
      const int r0 = 32 * (tg / NT), n0 = 32 * (tg % NT);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        // dH row: the compacted row's source position (rowmap) or the row itself; ignored rows
        // (label −100, incl. compaction padding) carry no gradient
        const long long dst = sDst[r0 + acc_row(i, hh)];
        if (dst >= 0) atomicAdd(dH + dst * C + n0 + (l & 31), acc_o[t][i]);
      }
    }
  }
}

// bwd-b: dW[v][c] += Σ_r dl[r][v] H[r][c], db[v] += Σ_r dl[r][v]; grid (vocab chunk, row split),
// H tiles (+ their LSE / labels) register-prefetched one tile ahead, partials added atomically
template <int C>
__global__ __launch_bounds__(256) void ce_bwd_dw_kernel(const uint16_t* __restrict__ Hm,
                                                        const int64_t* __restrict__ labels,
                                                        const uint16_t* __restrict__ W, const float* __restrict__ bias,
                                                        const float* __restrict__ lse, const float* __restrict__ gscale,
                                                        int M, int V, int tiles_per_split, float* __restrict__ dW,
                                                        float* __restrict__ db) {
  constexpr int LD = C + 8, LDL = VB + 8, NT = C / 32;
  __shared__ __attribute__((aligned(16))) uint16_t sH[HB * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[VB * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sL[HB * LDL];
  __shared__ float sLse[HB];
  __shared__ int sLab[HB];
  __shared__ float sB[2][64];
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int v0 = blockIdx.x * VB;
  const int mt_begin = blockIdx.y * tiles_per_split;
  const int mt_end = min((M + HB - 1) / HB, mt_begin + tiles_per_split);
  const float g = gscale[0];
  stage_rows<C>(sW, LD, W, v0, V);
  const int coll = 32 * (w & 1) + (l & 31);
  const int col = v0 + coll;
  const bool valid = col < V;
  const float bv = valid ? bias[col] : 0.f;
  constexpr int MAXT = (2 * NT + 3) / 4;
  f32x16 acc_o[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc_o[t] = f32x16{};
  float bsum = 0.f;
  bf16x8 hr[C / 32];
  float aux = 0.f;  // threads [0,64): LSE of row tid, [64,128): label of row tid-64
  auto fetch = [&](int mt) {
    fetch_rows<C>(hr, Hm, mt * HB, M);
    const int t = threadIdx.x & 63, gr = mt * HB + t;
    if (threadIdx.x < 64) aux = gr < M ? lse[gr] : 0.f;
    else if (threadIdx.x < 128) aux = __int_as_float(gr < M ? (int)labels[gr] : -100);
  };
  if (mt_begin < mt_end) fetch(mt_begin);
  for (int mt = mt_begin; mt < mt_end; ++mt) {
    const int m0 = mt * HB;
    __syncthreads();
    store_rows<C>(hr, sH, LD);
    if (threadIdx.x < 64) sLse[threadIdx.x] = aux;
    else if (threadIdx.x < 128) sLab[threadIdx.x - 64] = __float_as_int(aux);
    __syncthreads();
    if (mt + 1 < mt_end) fetch(mt + 1);
    const f32x16 acc = logits_tile<C>(sH, sW, LD);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int rr = 32 * (w >> 1) + acc_row(i, hh);
      float d = 0.f;
      if (m0 + rr < M && valid) d = dlogit(acc[i] + bv, sLse[rr], col, sLab[rr], g);
      bsum += d;
      sL[rr * LDL + coll] = f2bf(d);
    }
    __syncthreads();
    // dW chunk (64 vocab × C) += dlᵀ · H : A = dl stored [r][v] (k=r strided), B = H [r][c] (k strided)
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      const int tg = w + 4 * t;
      if (tg < 2 * NT) {
        const int r0 = 32 * (tg / NT), n0 = 32 * (tg % NT);
#pragma unroll
        for (int k0 = 0; k0 < HB; k0 += 16) acc_o[t] = mfma32(frag_ks(sL, LDL, r0, k0), frag_ks(sH, LD, n0, k0), acc_o[t]);
      }
    }
  }
  // bias: reduce bsum over the two lane halves and the two waves sharing a column set
  bsum = xor32_sum(bsum);
  if (hh == 0) sB[w >> 1][coll] = bsum;
  __syncthreads();
  if (threadIdx.x < 64 && v0 + threadIdx.x < V) atomicAdd(db + v0 + threadIdx.x, sB[0][threadIdx.x] + sB[1][threadIdx.x]);
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int tg = w + 4 * t;
    if (tg < 2 * NT) {
      const int r0 = 32 * (tg / NT), n0 = 32 * (tg % NT);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int vv = v0 + r0 + acc_row(i, hh);
        if (vv < V) atomicAdd(dW + (long long)vv * C + n0 + (l & 31), acc_o[t][i]);
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
__global__ void select_rows_kernel(const int64_t* __restrict__ labels, int L, int cap, int64_t* __restrict__ idx_b,
                                   int64_t* __restrict__ lab_b, int* __restrict__ count) {
  __shared__ int sW[4], sOff;
  const int b = blockIdx.x, w = wave_id(), l = lane_id();
  if (threadIdx.x == 0) sOff = 0;
  __syncthreads();
  for (int c0 = 0; c0 < L; c0 += 256) {
    const int i = c0 + threadIdx.x;
    const int64_t lab = i < L ? labels[(long long)b * L + i] : -100;
    const bool sel = lab != -100;
    const uint64_t m = __ballot(sel);
    const int pre = __popcll(m & ((1ull << l) - 1ull));
    if (l == 0) sW[w] = __popcll(m);
    __syncthreads();
    int woff = 0;
    for (int k = 0; k < w; ++k) woff += sW[k];
    const int pos = sOff + woff + pre;
    if (sel && pos < cap) {
      idx_b[(long long)b * cap + pos] = i;
      lab_b[(long long)b * cap + pos] = lab;
    }
    __syncthreads();
    if (threadIdx.x == 0) sOff += sW[0] + sW[1] + sW[2] + sW[3];
    __syncthreads();
  }
  const int cnt = sOff;
  for (int j = (cnt < cap ? cnt : cap) + threadIdx.x; j < cap; j += blockDim.x) {
    idx_b[(long long)b * cap + j] = j % L;
    lab_b[(long long)b * cap + j] = -100;
  }
  if (threadIdx.x == 0) count[b] = cnt;
}

__global__ void select_global_kernel(const int* __restrict__ count, int B, int cap, const int64_t* __restrict__ lab_b,
                                     int gcap, int64_t* __restrict__ gidx, int64_t* __restrict__ glab,
                                     float* __restrict__ total, bool* __restrict__ overflow) {
  extern __shared__ int sOffs[];  // [B + 1] exclusive prefix of min(count, cap)
  if (threadIdx.x == 0) {
    int acc = 0, all = 0;
    bool ovf = false;
    for (int b = 0; b < B; ++b) {
      const int n = count[b] < cap ? count[b] : cap;
      ovf |= count[b] > cap;
      sOffs[b] = acc;
      acc += n;
      all += count[b];
    }
    sOffs[B] = acc;
    total[0] = (float)all;
    overflow[0] = ovf || acc > gcap;
  }
  __syncthreads();
  const int used = sOffs[B] < gcap ? sOffs[B] : gcap;
  for (long long s = threadIdx.x; s < (long long)B * cap; s += blockDim.x) {
    const int b = (int)(s / cap), j = (int)(s - (long long)b * cap);
    const int n = sOffs[b + 1] - sOffs[b];
    const int g = sOffs[b] + j;
    if (j < n && g < gcap) {
      gidx[g] = s;
      glab[g] = lab_b[s];
    }
  }
  for (int g = used + threadIdx.x; g < gcap; g += blockDim.x) {
    gidx[g] = 0;
    glab[g] = -100;
  }
}

void mlm_select_launch(const int64_t* labels, int B, int L, int cap, int gcap, int64_t* idx_b, int64_t* lab_b,
                       int* count, int64_t* gidx, int64_t* glab, float* total, bool* overflow, hipStream_t st) {
  hipLaunchKernelGGL(select_rows_kernel, dim3(B), dim3(256), 0, st, labels, L, cap, idx_b, lab_b, count);
  hipLaunchKernelGGL(select_global_kernel, dim3(1), dim3(1024), (B + 1) * sizeof(int), st, count, B, cap, lab_b, gcap,
                     gidx, glab, total, overflow);
}

// vocab splits so that a launch has ≈ target workgroups (several per CU hide the W-chunk latency)
static int pick_split(int M, int nchunks, int target) {
  const int mt = (M + HB - 1) / HB;
  int s = (target + mt - 1) / mt;
  s = s < 1 ? 1 : s;
  return s > nchunks ? nchunks : s;
}

void ce_fwd_launch(int C, const uint16_t* Hm, const int64_t* labels, const uint16_t* W, const float* bias, int M,
                   int V, float* part_ms, float* picked, float* loss_rows, float* lse, int nsplit, hipStream_t st) {
  const int nchunks = (V + VB - 1) / VB;
  const int cps = (nchunks + nsplit - 1) / nsplit;
  dim3 grid((M + HB - 1) / HB, nsplit);
  if (C == 64) hipLaunchKernelGGL(ce_fwd_kernel<64>, grid, dim3(256), 0, st, Hm, labels, W, bias, M, V, cps, part_ms, picked);
  else if (C == 128) hipLaunchKernelGGL(ce_fwd_kernel<128>, grid, dim3(256), 0, st, Hm, labels, W, bias, M, V, cps, part_ms, picked);
  else if (C == 32) hipLaunchKernelGGL(ce_fwd_kernel<32>, grid, dim3(256), 0, st, Hm, labels, W, bias, M, V, cps, part_ms, picked);
  hipLaunchKernelGGL(ce_combine_kernel, dim3((M + 255) / 256), dim3(256), 0, st, part_ms, picked, labels, M, nsplit,
                     loss_rows, lse);
}

int ce_num_splits(int M, int V) { return pick_split(M, (V + VB - 1) / VB, 2048); }

void ce_bwd_launch(int C, const uint16_t* Hm, const int64_t* labels, const uint16_t* W, const float* bias,
                   const float* lse, const float* gscale, int M, int V, float* dH, const int64_t* rowmap, float* dW,
                   float* db, int accumulate, hipStream_t st) {
  const int nchunks = (V + VB - 1) / VB;
  const int nsplit = pick_split(M, nchunks, 512);  // dH partials are added atomically: few splits
  const int cps = (nchunks + nsplit - 1) / nsplit;
  // dW: (vocab chunk × row split) workgroups, ≈ 4 per CU; dW / db partials added atomically
  const int mtiles = (M + HB - 1) / HB;
  int rsplit = (1024 + nchunks - 1) / nchunks;
  rsplit = rsplit < 1 ? 1 : (rsplit > mtiles ? mtiles : rsplit);
  const int tps = (mtiles + rsplit - 1) / rsplit;
  rsplit = (mtiles + tps - 1) / tps;
  if (!accumulate) {
    (void)hipMemsetAsync(dW, 0, sizeof(float) * (size_t)V * C, st);
    (void)hipMemsetAsync(db, 0, sizeof(float) * (size_t)V, st);
  }
  dim3 ga((M + HB - 1) / HB, nsplit), gb(nchunks, rsplit);
#define CEB(CC)                                                                                                  \
  hipLaunchKernelGGL(ce_bwd_dh_kernel<CC>, ga, dim3(256), 0, st, Hm, labels, W, bias, lse, gscale, M, V, cps, dH, rowmap); \
  hipLaunchKernelGGL(ce_bwd_dw_kernel<CC>, gb, dim3(256), 0, st, Hm, labels, W, bias, lse, gscale, M, V, tps, dW, db)
  if (C == 64) { CEB(64); }
  else if (C == 128) { CEB(128); }
  else if (C == 32) { CEB(32); }
#undef CEB
}

}  // namespace pio
