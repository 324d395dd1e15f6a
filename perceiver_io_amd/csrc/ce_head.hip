// Vocab projection + softmax cross-entropy head, two streaming passes (C = 64; SURVEY K-12/K-13).
//
// Reference: TextOutputAdapter linear (perceiver/adapter.py:146-149) + CrossEntropyLoss over the
// (B, V, L) logits with ignore_index -100 (perceiver/lightning.py:223-226).  Only the ~15 %
// selected rows are passed in (compacted on device).  Logits exist only as MFMA tiles.
//
//   pass 1 (forward)  rows × vocab split: transposed logit tiles Sᵀ = W·Hᵀ (vocab on the
//                     accumulator rows, one query row per lane) with an online log-sum-exp, AND
//                     the softmax-weighted vocab sum Σ_v p[r, v]·W[v] — a flash-attention forward
//                     whose keys and values are both W — so the hidden-state gradient needs no
//                     further pass over the vocabulary: dH[r] = g·(Σ_v p[r, v]·W[v] − W[label]).
//   pass 1 tail       the last split workgroup of each row block (arrival ticket) merges the
//                     splits' (max, sum) into the rows' lse and the block's loss partial; the last
//                     row block (second ticket) finalises the mean loss — no combine launch.
//   pass 2 (backward) vocab × row split: logit tiles S = H·Wᵀ (vocab on the lane), p, dW += g·pᵀ·H
//                     and db += g·Σ p, the one-hot terms dW[label] −= g·H[r], db[label] −= g of
//                     each tile's few rows whose label the wave holds (a ballot scan per tile;
//                     a classifier-sized vocabulary subtracts it per logit in the tile instead),
//                     partials stored into a slab row (or added); in appended workgroups the dH
//                     rows g·u[r] with u[r] = Σ_v p·W − W[label] merged from pass 1's per-split
//                     partials, scattered to their source positions.
// Per-logit VALU work is what bounds both passes (MFMA busy ≈ 13 % in round 4): the logit
// accumulators start at the bias (the MFMAs add it); the exp2 arguments and the sums are packed
// fp32 pairs (v_pk_fma_f32, v_pk_add_f32); pass 1 tests a tile's Σ p against 2^kRescale instead of
// forming its max (the max only on the rare rescale branch) and takes the label's logit from one
// dot product in split 0 instead of a per-tile label test; pass 2 keeps g and the one-hot term out
// of its tiles (a per-tile ballot over the rows' labels instead).
//
// LDS images ([rows][64] bf16, 128 B per row, no padding) are XOR-swizzled on their 16-byte
// slots with sw(v) = v₁·4 + v₂·2 + v₃ (bits of the row index): a k-contiguous ds_read_b128
// fragment (16 rows of a lane group, one slot each) and a transposed ds_read_b64_tr_b16
// fragment (4 consecutive rows × 4 slots per 32 lanes) both land on distinct banks.
// Stats are kept in the log2 domain; the online rescale of the running sum and the W-weighted
// accumulator is lazy: only when a tile's Σ p exceeds 2^kRescale (a logit ≳ kRescale above the
// reference max; 2^8 headroom, far inside fp32 / bf16 range), a wave-uniform branch taken a
// handful of times per row.
// The cross-workgroup hand-offs below rely on the write-through (sc1) store / L1-bypassing load
// behaviour measured on gfx950 (MI355X_MICROARCH.md, inter-workgroup visibility): no other target.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "this translation unit's sc1 hand-off protocol is validated on gfx950 (MI355X) only"
#endif
#include <algorithm>

#include "common.h"

namespace pio {

namespace ce2 {

constexpr int C = 64;            // head width (the C = 64 specialisation)
constexpr int RB = 128;          // pass 1: rows per workgroup (4 waves × 32)
constexpr int VC = 64;           // pass 1: vocab entries per staged chunk
constexpr int VB2 = 128;         // pass 2: vocab entries per workgroup (4 waves × 32)
constexpr int HT = 64;           // pass 2: rows per staged H tile
constexpr float kL2E = 1.4426950408889634f;
constexpr float kLN2 = 0.6931471805599453f;
constexpr float kRescale = 8.f;  // lazy-rescale threshold (log2 units)
constexpr float kRescaleSum = 256.f;  // 2^kRescale: a tile's Σ p above it takes the rescale branch
constexpr int kCeMaxSplitsFwd = 16;  // ce2_num_splits caps the vocab splits of pass 1 here
// pass 2 at a vocabulary this small (a classifier head: most tile rows' labels fall inside every
// wave's 32 vocab entries) takes the one-hot term inside the tile, d = p − [label = v] (one
// compare per logit), instead of the per-hit ballot scan, which would serialise on every row
constexpr int kOneHotInTileMaxV = 256;
constexpr int kDhRowsPerWg = 32;  // pass 2's appended dH workgroups: rows each (2 passes of 16)
typedef float f2v __attribute__((ext_vector_type(2)));  // packed fp32 (v_pk_fma_f32 / v_pk_add_f32)

// p = 2^(t·log2e − m) for the 16 logits of a tile (natural units) in packed pairs; returns Σ p
__device__ __forceinline__ float exp_tile(const f32x16& t, float m, f32x16& p) {
  const f2v k2 = {kL2E, kL2E}, nm = {-m, -m};
  f2v sum = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 16; i += 2) {
    const f2v x = {t[i], t[i + 1]};
    const f2v y = __builtin_elementwise_fma(x, k2, nm);
    p[i] = __builtin_amdgcn_exp2f(y.x);
    p[i + 1] = __builtin_amdgcn_exp2f(y.y);
    sum += f2v{p[i], p[i + 1]};
  }
  return sum.x + sum.y;
}

// element offset of (row v, 16-byte slot s) in a swizzled [rows][64] bf16 image
__device__ __forceinline__ int swz(int v, int s) {
  const int sw = ((v >> 1) & 1) << 2 | ((v >> 2) & 1) << 1 | ((v >> 3) & 1);
  return v * C + 8 * (s ^ sw);
}
// k-contiguous 32x32x16 operand: row i0 + (l & 31), k = 16·ks + 8·(l >> 5) .. + 7
__device__ __forceinline__ bf16x8 img_kc(const uint16_t* img, int i0, int ks) {
  const int l = lane_id();
  return *reinterpret_cast<const bf16x8*>(img + swz(i0 + (l & 31), 2 * ks + (l >> 5)));
}
// transposed operand with the permuted k order of an accumulator used as the other operand
// (frag_ks_perm of common.h on a swizzled image): image rows = k (k0 + …), columns = i (i0 + …)
__device__ __forceinline__ bf16x8 img_ks_perm(const uint16_t* img, int i0, int k0) {
  const int l = lane_id();
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int row = k0 + 4 * (g >> 1) + q, col = i0 + 16 * (g & 1) + 4 * p;
  const uint16_t* a = img + swz(row, col >> 3) + (col & 7);
  const uint16_t* b = img + swz(row + 8, col >> 3) + (col & 7);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(a));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(b));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

}  // namespace ce2

// ---- pass 1 ---------------------------------------------------------------------------
// grid (⌈M / 128⌉, splits); wave w: rows m0 + 32w + (l & 31).  Per split: part_ml[split][row] =
// (max, sum) in log2 units, part_acc[split][row][c] = Σ_v 2^(t_v − max)·W[v][c] over the split's
// vocabulary; picked[row] = the label's logit (natural units, written by the split holding it);
// split 0 also writes the compact bf16 rows hs for pass 2.
__global__ __launch_bounds__(256) void ce2_fwd_kernel(const float* __restrict__ Hm, const int64_t* __restrict__ hidx,
                                                      const int64_t* __restrict__ labels, const uint16_t* __restrict__ W,
                                                      const float* __restrict__ bias, int M, int V, int chunks_per_split,
                                                      float2* __restrict__ part_ml, float* __restrict__ part_acc,
                                                      float* __restrict__ picked, uint16_t* __restrict__ hs_out,
                                                      float* __restrict__ lse, float* __restrict__ count, int count_labels,
                                                      float* __restrict__ loss, float* __restrict__ blk,
                                                      unsigned* __restrict__ rb_ticket, unsigned* __restrict__ ticket,
                                                      float* __restrict__ zero_out, long long zero_n4) {
  using namespace ce2;
  __shared__ __attribute__((aligned(16))) uint16_t sW[2][VC * C];
  __shared__ __attribute__((aligned(16))) float sB[2][VC];  // bias (−inf past V): the logit accumulators' initial value
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int m0 = blockIdx.x * RB, split = blockIdx.y;
  const int nchunks = (V + VC - 1) / VC;
  const int c_begin = split * chunks_per_split, c_end = min(nchunks, c_begin + chunks_per_split);
  const int gr = m0 + 32 * w + (l & 31);
  const bool rin = gr < M;
  // this lane's half row (c = 16s + 8hh .. + 7, s < 4) as the B operand of Sᵀ = W·Hᵀ, gathered
  // from the fp32 decoder output and cast on load
  bf16x8 hb[4];
  {
    const long long src = hidx ? hidx[rin ? gr : 0] : (long long)(rin ? gr : 0);
    const float* hp = Hm + src * C + 8 * hh;
    float4 a[4], b[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      a[s] = *reinterpret_cast<const float4*>(rin ? hp + 16 * s : kZero32B);
      b[s] = *reinterpret_cast<const float4*>(rin ? hp + 16 * s + 4 : kZero32B);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      hb[s][0] = (short)f2bf(a[s].x); hb[s][1] = (short)f2bf(a[s].y); hb[s][2] = (short)f2bf(a[s].z);
      hb[s][3] = (short)f2bf(a[s].w); hb[s][4] = (short)f2bf(b[s].x); hb[s][5] = (short)f2bf(b[s].y);
      hb[s][6] = (short)f2bf(b[s].z); hb[s][7] = (short)f2bf(b[s].w);
    }
    if (split == 0 && hs_out != nullptr && rin)
#pragma unroll
      for (int s = 0; s < 4; ++s) *reinterpret_cast<bf16x8*>(hs_out + (long long)gr * C + 16 * s + 8 * hh) = hb[s];
  }
  const int lab = rin ? (int)labels[gr] : -100;
#if PIO_CHECKS
  if (split == 0 && hh == 0 && (lab >= V || (lab < 0 && lab != -100))) pio_flag(kErrLabel);
#endif
  // the label's logit (natural units) by split 0: the row's bf16 operand · W[label] + bias, the
  // products the logit tiles form (fp32 sums in another order) — no per-tile label test
  if (split == 0 && rin && lab >= 0 && lab < V) {
    float d = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const bf16x8 wl = *reinterpret_cast<const bf16x8*>(W + (long long)lab * C + 16 * s2 + 8 * hh);
#pragma unroll
      for (int j = 0; j < 8; ++j) d = fmaf(bf2f((uint16_t)hb[s2][j]), bf2f((uint16_t)wl[j]), d);
    }
    d += __shfl_xor(d, 32);
    if (hh == 0)
      __hip_atomic_store(reinterpret_cast<unsigned*>(picked + gr), __float_as_uint(d + bias[lab]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  // chunk staging: 64 vocab rows × 8 slots = 512 16-byte pieces, two per thread (+ the bias)
  bf16x8 wr[2];
  float bnext = 0.f;
  auto fetch = [&](int c) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = threadIdx.x + 256 * i, v = c * VC + (e >> 3);
      wr[i] = *reinterpret_cast<const bf16x8*>(v < V ? W + (long long)v * C + 8 * (e & 7)
                                                     : reinterpret_cast<const uint16_t*>(kZero32B));
    }
    const int v = c * VC + (threadIdx.x & (VC - 1));
    const float bv = bias[v < V ? v : 0];  // unconditional load (address select)
    bnext = v < V ? bv : -__builtin_inff();
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = threadIdx.x + 256 * i;
      *reinterpret_cast<bf16x8*>(&sW[buf][swz(e >> 3, e & 7)]) = wr[i];
    }
    if (threadIdx.x < VC) sB[buf][threadIdx.x] = bnext;
  };
  float m_ref = -__builtin_inff(), l_run = 0.f;
  f32x16 acc[2] = {f32x16{}, f32x16{}};  // Σ p·W, transposed: [c = 32ct + acc_row][row = lane]
  if (c_begin < c_end) {
    fetch(c_begin);
    stage(0);
  }
  lds_sync();
  for (int c = c_begin; c < c_end; ++c) {
    const int buf = (c - c_begin) & 1;
    if (c + 1 < c_end) fetch(c + 1);  // in flight under this chunk's MFMAs
    const uint16_t* img = sW[buf];
#pragma unroll
    for (int vb = 0; vb < 2; ++vb) {  // two 32-vocab blocks per chunk
      // register i: vocab 32vb + acc_row(i, hh) of the chunk; the accumulator starts at the bias,
      // so the MFMAs add it (no per-logit VALU add) and the logit stays in natural units until
      // the exp2 argument (one fma)
      f32x16 st;
      {
        const float* bp = sB[buf] + 32 * vb + 4 * hh;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 bb = *reinterpret_cast<const float4*>(bp + 8 * q);
          st[4 * q] = bb.x; st[4 * q + 1] = bb.y; st[4 * q + 2] = bb.z; st[4 * q + 3] = bb.w;
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) st = mfma32(ce2::img_kc(img, 32 * vb, s), hb[s], st);
      // p against the running reference max; a tile whose sum leaves [0, 2^kRescale] (a logit
      // more than ~kRescale above the reference, or the first tile: m_ref = −inf → inf) takes
      // the rare wave-uniform branch: new reference = the row max, lazy rescale, p again
      f32x16 p;
      float ps = exp_tile(st, m_ref, p);
      if (__ballot(!(ps <= ce2::kRescaleSum))) {
        float mx = st[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) mx = fmaxf(mx, st[i]);
        mx = xor32_max(mx) * kL2E;  // both halves of the row share its reference max (log2 units)
        const float mn = fmaxf(m_ref, mx);
        const float alpha = fast_exp2(m_ref - mn);  // 0 on the first block
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) { acc[0][i] *= alpha; acc[1][i] *= alpha; }
        m_ref = mn;
        ps = exp_tile(st, m_ref, p);
      }
      l_run += ps;
      // Σ p·W: accᵀ[c][row] += Wᵀ[c][v]·Pᵀ[v][row] (the logits accumulator as the B operand)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 pb = pack_acc(p, ss);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct] = mfma32(ce2::img_ks_perm(img, 32 * ct, 32 * vb + 16 * ss), pb, acc[ct]);
      }
    }
    if (c + 1 < c_end) stage(buf ^ 1);
    lds_sync();
  }
  const float ls = xor32_sum(l_run);
  // (max, sum) and the picked logit are read back inside this launch by the row block's last
  // split: stored write-through (sc1, agent-scope relaxed atomic stores), so no release fence is
  // needed; the Σ p·W partials are read by the next launch only (plain stores)
  if (rin) {
    if (hh == 0)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(part_ml + (long long)split * M + gr),
                         (unsigned long long)__float_as_uint(m_ref) | ((unsigned long long)__float_as_uint(ls) << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float* pa = part_acc + ((long long)split * M + gr) * C;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int q = 0; q < 4; ++q)  // registers 4q .. 4q+3 = c 32ct + 8q + 4hh + 0..3
        *reinterpret_cast<float4*>(pa + 32 * ct + 8 * q + 4 * hh) =
            make_float4(acc[ct][4 * q], acc[ct][4 * q + 1], acc[ct][4 * q + 2], acc[ct][4 * q + 3]);
  }
  // a slice of the backward's dH accumulator cleared on the way (no fill launch)
  if (zero_out != nullptr) {
    const long long nwg = (long long)gridDim.x * gridDim.y, wg = (long long)blockIdx.y * gridDim.x + blockIdx.x;
    const long long per = (zero_n4 + nwg - 1) / nwg, z1 = min(zero_n4, (wg + 1) * per);
    for (long long i = wg * per + threadIdx.x; i < z1; i += blockDim.x)
      reinterpret_cast<float4*>(zero_out)[i] = float4{0.f, 0.f, 0.f, 0.f};
  }
  // ---- arrival ticket of the row block: every wave drains its stores, one lane counts ----
  // Hand-off form (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md § visibility, the
  // write-through table's first row): every handed-off word is stored sc1 (agent-scope relaxed
  // atomic stores) and drained by its storing wave (vmcnt(0)) before the barrier behind which
  // one lane adds to ONE unsharded counter; only the workgroup whose add returned last reads,
  // and only with sc1 loads (L1 bypass), after that add returned (its other waves after a
  // barrier).  No release/acquire fence is needed in this form (each costs ≈1.7 µs).  The
  // ticket words assume one ce_fwd in flight per device (every launch is on the step's stream).
  __shared__ unsigned last;
  __shared__ float red[2][4];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(rb_ticket + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.y - 1;
  __syncthreads();
  if (!last) return;
  // the last split merges the splits' (max, sum) of the block's rows (sc1 loads of the sc1 stores)
  float lr = 0.f, nr = 0.f;
  if (threadIdx.x < RB) {
    const int r = m0 + threadIdx.x;
    if (r < M) {
      float2 ml[kCeMaxSplitsFwd];
#pragma unroll
      for (int s = 0; s < kCeMaxSplitsFwd; ++s) {  // every split's load in flight (address selects)
        const unsigned long long x = __hip_atomic_load(
            reinterpret_cast<unsigned long long*>(part_ml + (long long)(s < (int)gridDim.y ? s : 0) * M + r),
            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ml[s] = make_float2(__uint_as_float((unsigned)x), __uint_as_float((unsigned)(x >> 32)));
      }
      float mx = -__builtin_inff();
#pragma unroll
      for (int s = 0; s < kCeMaxSplitsFwd; ++s) mx = s < (int)gridDim.y ? fmaxf(mx, ml[s].x) : mx;
      float L = 0.f;
#pragma unroll
      for (int s = 0; s < kCeMaxSplitsFwd; ++s) L += s < (int)gridDim.y ? ml[s].y * fast_exp2(ml[s].x - mx) : 0.f;
      const float L2 = (mx + __log2f(L)) * kLN2;
      lse[r] = L2;  // read by the next launch
      const int lab = (int)labels[r];
      const float pk_r = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(picked + r), __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
      lr = lab >= 0 ? L2 - pk_r : 0.f;
      nr = lab >= 0 ? 1.f : 0.f;
    }
  }
  lr = wave_sum(lr);
  nr = wave_sum(nr);
  if (lane_id() == 0) { red[0][wave_id()] = lr; red[1][wave_id()] = nr; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float bl = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    const float bn = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    __hip_atomic_store(reinterpret_cast<unsigned*>(blk + blockIdx.x), __float_as_uint(bl), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned*>(blk + gridDim.x + blockIdx.x), __float_as_uint(bn), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    rb_ticket[blockIdx.x] = 0u;  // re-armed for the next call (graph replays)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  // ---- the last row block: the mean loss over all row blocks, fixed order ----
  float t = 0.f, n = 0.f;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) {
    t += __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(blk + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    n += __uint_as_float(
        __hip_atomic_load(reinterpret_cast<unsigned*>(blk + gridDim.x + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
  t = wave_sum(t);
  n = wave_sum(n);
  __syncthreads();
  if (lane_id() == 0) { red[0][wave_id()] = t; red[1][wave_id()] = n; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tt = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    const float nn = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    if (count_labels) count[0] = nn;
    loss[0] = tt / fmaxf(count_labels ? nn : count[0], 1.f);
    *ticket = 0u;
  }
}

// ---- pass 2 ---------------------------------------------------------------------------
// grid (⌈V / 128⌉, rsplit + 1).  y < rsplit: wave w owns vocab v0 = 128·x + 32w + (l & 31) (its
// 32 rows of W as the B operand of S = H·Wᵀ, in registers) and streams the rows of split y in
// 64-row tiles (bf16 H, lse, labels) through LDS; dl = (2^(t − lse) − [label = v])·g;
// dW[v] += dlᵀ·H, db[v] += Σ dl; partials stored into slab row y (or added atomically).
// y = rsplit: dH[rowmap[r]] (+)= g·u[r] for the rows of slice x (appended workgroups).
template <bool SMALLV>  // SMALLV: V ≤ kOneHotInTileMaxV, the one-hot term inside the tile
__global__ __launch_bounds__(256) void ce2_bwd_kernel(const uint16_t* __restrict__ Hs, const int64_t* __restrict__ labels,
                                                      const uint16_t* __restrict__ W, const float* __restrict__ bias,
                                                      const float* __restrict__ lse, const float* __restrict__ part_acc,
                                                      const float2* __restrict__ part_ml, int nsplit,
                                                      const float* __restrict__ gout, const float* __restrict__ count,
                                                      int M, int V, int rsplit, int tiles_per_split,
                                                      float* __restrict__ dW, float* __restrict__ db,
                                                      float* __restrict__ slab, float* __restrict__ dH,
                                                      const int64_t* __restrict__ rowmap, long long dh_rows) {
  using namespace ce2;
  __shared__ __attribute__((aligned(16))) uint16_t sH[2][HT * C];
  __shared__ __attribute__((aligned(16))) float sL[2][HT];  // lse·log2e; +inf for a row without a label
  __shared__ __attribute__((aligned(16))) int sLab[2][HT];     // the rows' labels (−1: none)
  static_assert(HT == 64, "one tile row per lane in the one-hot scan");
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const float g = gout[0] / fmaxf(count[0], 1.f);
  if ((int)blockIdx.y >= rsplit) {
    // dH rows: u[r] = Σ_v p·W − W[label] merged from pass 1's split partials (a row per 16
    // threads, 4 channels each), then dH[rowmap[r]] += g·u[r]; the appended rows y ≥ rsplit of the
    // grid, ≈ kDhRowsPerWg rows per workgroup
    const int nb = (int)gridDim.x * ((int)gridDim.y - rsplit), bid = ((int)blockIdx.y - rsplit) * (int)gridDim.x + (int)blockIdx.x;
    const int per = (M + nb - 1) / nb, r0 = bid * per, r1 = min(M, r0 + per);
    const int cq = threadIdx.x & 15;
    for (int r = r0 + (int)(threadIdx.x >> 4); r < r1; r += 16) {
      const int lab = (int)labels[r];
      if (lab < 0 || lab >= V) continue;
      const long long dst = rowmap ? rowmap[r] : (long long)r;
      if (dst < 0 || dst >= dh_rows) continue;
      float2 ml[kCeMaxSplitsFwd];
      float4 v[kCeMaxSplitsFwd];
#pragma unroll
      for (int s = 0; s < kCeMaxSplitsFwd; ++s) {  // every split's loads in flight (address selects)
        const int ss = s < nsplit ? s : 0;
        ml[s] = part_ml[(long long)ss * M + r];
        v[s] = *reinterpret_cast<const float4*>(part_acc + ((long long)ss * M + r) * C + 4 * cq);
      }
      float mx = -__builtin_inff();
#pragma unroll
      for (int s = 0; s < kCeMaxSplitsFwd; ++s) mx = s < nsplit ? fmaxf(mx, ml[s].x) : mx;
      float L = 0.f;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int s = 0; s < kCeMaxSplitsFwd; ++s) {
        const float f = s < nsplit ? fast_exp2(ml[s].x - mx) : 0.f;
        L = fmaf(ml[s].y, f, L);
        a.x = fmaf(v[s].x, f, a.x); a.y = fmaf(v[s].y, f, a.y); a.z = fmaf(v[s].z, f, a.z); a.w = fmaf(v[s].w, f, a.w);
      }
      const float inv = g / L;
      const uint2 wv = *reinterpret_cast<const uint2*>(W + (long long)lab * C + 4 * cq);
      float4* d = reinterpret_cast<float4*>(dH + dst * C) + cq;
      float4 o = *d;
      o.x += fmaf(a.x, inv, -g * bf2f((uint16_t)(wv.x & 0xFFFF)));
      o.y += fmaf(a.y, inv, -g * bf2f((uint16_t)(wv.x >> 16)));
      o.z += fmaf(a.z, inv, -g * bf2f((uint16_t)(wv.y & 0xFFFF)));
      o.w += fmaf(a.w, inv, -g * bf2f((uint16_t)(wv.y >> 16)));
      *d = o;
    }
    return;
  }
  const int vl = 32 * w + (l & 31), vg = blockIdx.x * VB2 + vl;
  const bool vin = vg < V;
  // this lane's vocab row as the B operand (k = c = 16s + 8hh .. + 7)
  bf16x8 wb[4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
    wb[s] = *reinterpret_cast<const bf16x8*>(vin ? W + (long long)vg * C + 16 * s + 8 * hh
                                                 : reinterpret_cast<const uint16_t*>(kZero32B));
  const float bnat = vin ? bias[vg] : 0.f;  // the logit accumulators' initial value
  const int ntiles = (M + HT - 1) / HT;
  const int t_begin = blockIdx.y * tiles_per_split, t_end = min(ntiles, t_begin + tiles_per_split);
  bf16x8 hr[2];
  float aux = 0.f;
  int labn = -1;
  auto fetch = [&](int t) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = threadIdx.x + 256 * i, r = t * HT + (e >> 3);
      hr[i] = *reinterpret_cast<const bf16x8*>(r < M ? Hs + (long long)r * C + 8 * (e & 7)
                                                     : reinterpret_cast<const uint16_t*>(kZero32B));
    }
    const int r = t * HT + (threadIdx.x & (HT - 1));
    if (threadIdx.x < HT) {  // a row without a label (capacity padding, r ≥ M): p = 2^−inf = 0
      const int lb = r < M ? (int)labels[r] : -1;
      const bool lv = lb >= 0;
      aux = lv ? lse[r] * kL2E : __builtin_inff();
      labn = lv ? lb : -1;
    }
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = threadIdx.x + 256 * i;
      *reinterpret_cast<bf16x8*>(&sH[buf][swz(e >> 3, e & 7)]) = hr[i];
    }
    if (threadIdx.x < HT) {
      sL[buf][threadIdx.x] = aux;
      sLab[buf][threadIdx.x] = labn;
    }
  };
  f32x16 acc[2] = {f32x16{}, f32x16{}};  // dW: [v = acc_row][c = 32ct + lane]
  float bsum = 0.f;
  if (t_begin < t_end) {
    fetch(t_begin);
    stage(0);
  }
  lds_sync();
  for (int t = t_begin; t < t_end; ++t) {
    const int buf = (t - t_begin) & 1;
    if (t + 1 < t_end) fetch(t + 1);
    const uint16_t* img = sH[buf];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {  // two 32-row blocks per tile
      f32x16 st;
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = bnat;
#pragma unroll
      for (int s = 0; s < 4; ++s) st = mfma32(ce2::img_kc(img, 32 * rb, s), wb[s], st);
      // register i: row 32rb + acc_row(i, hh) of the tile; lane: vocab vg.  d = p (the softmax;
      // the gradient scale g and the one-hot term are applied outside the tile loop: g on the
      // sums, −g·H[r] at the label by the appended row workgroups)
      f32x16 d;
      f2v bs2 = {0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 ls = *reinterpret_cast<const float4*>(&sL[buf][32 * rb + 8 * q + 4 * hh]);
        const f2v k2 = {kL2E, kL2E};
        const f2v y0 = __builtin_elementwise_fma(f2v{st[4 * q], st[4 * q + 1]}, k2, f2v{-ls.x, -ls.y});
        const f2v y1 = __builtin_elementwise_fma(f2v{st[4 * q + 2], st[4 * q + 3]}, k2, f2v{-ls.z, -ls.w});
        d[4 * q] = fast_exp2(y0.x);
        d[4 * q + 1] = fast_exp2(y0.y);
        d[4 * q + 2] = fast_exp2(y1.x);
        d[4 * q + 3] = fast_exp2(y1.y);
        if constexpr (SMALLV) {  // the one-hot term in the tile (rows 32rb + 8q + 4hh + 0..3)
          const int4 lb = *reinterpret_cast<const int4*>(&sLab[buf][32 * rb + 8 * q + 4 * hh]);
          d[4 * q] -= lb.x == vg ? 1.f : 0.f;
          d[4 * q + 1] -= lb.y == vg ? 1.f : 0.f;
          d[4 * q + 2] -= lb.z == vg ? 1.f : 0.f;
          d[4 * q + 3] -= lb.w == vg ? 1.f : 0.f;
        }
        bs2 += f2v{d[4 * q], d[4 * q + 1]} + f2v{d[4 * q + 2], d[4 * q + 3]};
      }
      bsum += bs2.x + bs2.y;
      // dW[v][c] += Σ_r dl[r][v]·H[r][c]: the dl accumulator as the A operand (Xᵀ·B)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 pa = pack_acc(d, ss);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct] = mfma32(pa, ce2::img_ks_perm(img, 32 * ct, 32 * rb + 16 * ss), acc[ct]);
      }
    }
    // the one-hot term of the tile's rows whose label is one of this wave's 32 vocab entries (on
    // average 64·32/V of them per tile: a ballot, rarely a hit): dW[label] −= H[r], db[label] −= 1
    // (g applied at the store), so the slab / accumulators hold the whole vocab gradient
    if constexpr (!SMALLV) {
      const int v0w = blockIdx.x * VB2 + 32 * w;
      const int lb = sLab[buf][l];  // lane l: row l of the tile
      unsigned long long hits = __ballot(lb >= v0w && lb < v0w + 32);
      while (hits) {
        const int r = __builtin_ctzll(hits);
        hits &= hits - 1;
        const int j = sLab[buf][r] - v0w;  // wave-uniform
        const int it = (j & 3) + 4 * (j >> 3), ht = (j >> 2) & 1;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const int c = 32 * ct + (l & 31);
          const float hv = bf2f(img[ce2::swz(r, c >> 3) + (c & 7)]);
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (i == it && hh == ht) acc[ct][i] -= hv;
        }
        if (hh == 0 && (l & 31) == j) bsum -= 1.f;
      }
    }
    if (t + 1 < t_end) stage(buf ^ 1);
    lds_sync();
  }
  bsum = xor32_sum(bsum) * g;
  float* dWp = dW;
  float* dbp = db;
  if (slab) {
    dWp = slab + (long long)blockIdx.y * ((long long)V * C + ((V + 3) & ~3));
    dbp = dWp + (long long)V * C;
  }
  if (hh == 0 && vin) {
    if (slab) dbp[vg] = bsum;
    else atomicAdd(dbp + vg, bsum);
  }
  // accumulator: col = lane & 31 = c (within tile ct), row = acc_row(i, hh) = vocab within the wave's 32
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int vv = blockIdx.x * VB2 + 32 * w + acc_row(i, hh);
      if (vv < V) {
        float* p = dWp + (long long)vv * C + 32 * ct + (l & 31);
        if (slab) *p = acc[ct][i] * g;
        else atomicAdd(p, acc[ct][i] * g);
      }
    }
}

// ---- host side --------------------------------------------------------------------------
int ce2_num_splits(int M, int V) {
  // ≈ 2 workgroups per CU over (row blocks × vocab splits); every split ≥ 4 chunks
  const int rb = (M + ce2::RB - 1) / ce2::RB, nchunks = (V + ce2::VC - 1) / ce2::VC;
  int s = (512 + rb - 1) / rb;
  s = s < 1 ? 1 : s;
  const int cap = (nchunks + 3) / 4;
  s = s > cap ? cap : s;
  s = s > ce2::kCeMaxSplitsFwd ? ce2::kCeMaxSplitsFwd : s;
  const int cps = (nchunks + s - 1) / s;
  return (nchunks + cps - 1) / cps;
}
int ce2_bwd_splits(int M, int V) {
  // row splits of pass 2: ≈ 512 workgroups, every split ≥ 4 tiles (the slab height)
  const int vb = (V + ce2::VB2 - 1) / ce2::VB2, nt = (M + ce2::HT - 1) / ce2::HT;
  int s = (512 + vb - 1) / vb;
  const int cap = (nt + 3) / 4;
  s = s > cap ? cap : s;
  s = s < 1 ? 1 : s;
  const int tps = (nt + s - 1) / s;
  return (nt + tps - 1) / tps;
}
int ce2_row_blocks(int M) { return (M + ce2::RB - 1) / ce2::RB; }

void ce2_fwd_launch(const float* Hm, const int64_t* hidx, const int64_t* labels, const uint16_t* W, const float* bias,
                    int M, int V, int nsplit, float2* part_ml, float* part_acc, float* picked, uint16_t* hs_out,
                    float* lse, float* count, int count_labels, float* loss, float* blk, unsigned* rb_ticket,
                    unsigned* ticket, float* zero_out, long long zero_n, hipStream_t st) {
  const int nchunks = (V + ce2::VC - 1) / ce2::VC;
  const int cps = (nchunks + nsplit - 1) / nsplit;
  hipLaunchKernelGGL(ce2_fwd_kernel, dim3(ce2_row_blocks(M), nsplit), dim3(256), 0, st, Hm, hidx, labels, W, bias, M, V,
                     cps, part_ml, part_acc, picked, hs_out, lse, count, count_labels, loss, blk, rb_ticket, ticket,
                     zero_out, zero_n / 4);
}

void ce2_bwd_launch(const uint16_t* Hs, const int64_t* labels, const uint16_t* W, const float* bias, const float* lse,
                    const float* part_acc, const float2* part_ml, int nsplit, const float* gout, const float* count,
                    int M, int V, float* dW, float* db, float* slab, int accumulate, float* dH, long long dh_rows,
                    const int64_t* rowmap, hipStream_t st) {
  const int rsplit = ce2_bwd_splits(M, V);
  const int nt = (M + ce2::HT - 1) / ce2::HT;
  const int tps = (nt + rsplit - 1) / rsplit;
  if (!accumulate && slab == nullptr) {
    (void)hipMemsetAsync(dW, 0, sizeof(float) * (size_t)V * ce2::C, st);
    (void)hipMemsetAsync(db, 0, sizeof(float) * (size_t)V, st);
  }
  const int vb = (V + ce2::VB2 - 1) / ce2::VB2;
  // appended dH grid rows: one row (vb workgroups) at a wide vocabulary — more cost the MLM head
  // 3 µs (31.7 → 34.9 µs, r6) — and ≈ kDhRowsPerWg rows per workgroup at a classifier's few blocks
  const int ndh = (M + ce2::kDhRowsPerWg - 1) / ce2::kDhRowsPerWg;
  const int ndy = vb >= 16 ? 1 : std::max(1, (ndh + vb - 1) / vb);
  if (V <= ce2::kOneHotInTileMaxV)
    hipLaunchKernelGGL(ce2_bwd_kernel<true>, dim3(vb, rsplit + ndy), dim3(256), 0, st, Hs, labels, W, bias, lse, part_acc,
                       part_ml, nsplit, gout, count, M, V, rsplit, tps, dW, db, slab, dH, rowmap, dh_rows);
  else
    hipLaunchKernelGGL(ce2_bwd_kernel<false>, dim3(vb, rsplit + ndy), dim3(256), 0, st, Hs, labels, W, bias, lse, part_acc,
                       part_ml, nsplit, gout, count, M, V, rsplit, tps, dW, db, slab, dH, rowmap, dh_rows);
}

unsigned check_errors_ce_head(bool reset) { return pio_read_errors(reset); }

}  // namespace pio
