// Chain-layout (CL) kernels: the fused self-attention layer forward and the layer-boundary
// backward as register-resident row chains on v_mfma_f32_16x16x32_bf16 (see the CL banner
// below).  Compiled with -mllvm -amdgpu-mfma-vgpr-form=1 (csrc/build.py): MFMA results stay in
// VGPRs, so the softmax and LayerNorm VALU work reads them directly instead of copying every
// accumulator out of (and back into) AGPRs (≈1,300 v_accvgpr moves per wave in the attention
// phase otherwise).
#include "common.h"

namespace pio {

// ------------------------------------------------------------------------------------
// Chain layout (CL): register-resident row chains with v_mfma_f32_16x16x32_bf16.
// Wave w of a 64-row tile owns rows 16w + (l & 15); lane group g = l >> 4 holds channels
// 16·mt + 4g + i (i < 4) of every 16-channel block mt — exactly the accumulator layout of a
// TRANSPOSED product Yᵀ = W·Xᵀ (col = lane & 15 = row, acc row = 4g + i = channel).  Such an
// accumulator feeds the next transposed product as its B operand with no lane movement: the
// k order of step t is permuted to channel 32t + 16(j >> 2) + 4g + (j & 3) for element j, and
// the weight (A operand) is staged into LDS with its columns permuted the same way, so every
// A fragment is one ds_read_b128.  A row's reductions (LayerNorm, per-head sums) are 16 local
// values + two lane swaps (l ^ 16, l ^ 32).  So a whole post-attention block — out-projection,
// residual, LN2, W1, GELU, W2, residual, LN1 + the next projection — runs per wave, from
// registers, with no LDS round trip of an activation and no workgroup barrier.
// ------------------------------------------------------------------------------------
// B fragment of k-step t from a CL activation (permuted k order)
template <int NM>
__device__ __forceinline__ bf16x8 cl_bfrag(const float (&v)[NM][4], int t) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(v[2 * t + (j >> 2)][j & 3]);
  return r;
}
// A fragment (m-tile mt, k-step t) of a weight image in LDS ([rows][ld], permuted or natural)
__device__ __forceinline__ bf16x8 cl_afrag(const uint16_t* sW, int ld, int mt, int t) {
  const int l = lane_id();
  return *reinterpret_cast<const bf16x8*>(sW + (16 * mt + (l & 15)) * ld + 32 * t + 8 * (l >> 4));
}
// Y^T (NMO m-tiles) = W·X^T over K = 32·KT channels; acc in CL
template <int NMO, int KT>
__device__ __forceinline__ void cl_gemm(const uint16_t* sW, int ld, const bf16x8 (&b)[KT], f32x4 (&acc)[NMO]) {
#pragma unroll
  for (int mt = 0; mt < NMO; ++mt) {
    acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < KT; ++t) acc[mt] = mfma16(cl_afrag(sW, ld, mt, t), b[t], acc[mt]);
  }
}
// one 16-byte chunk (row r, source columns c0 .. c0 + 7 of a 64-wide bf16 row) of a weight into
// its LDS image: natural, or columns permuted to the CL k order (two 8-byte pieces)
__device__ __forceinline__ void cl_wstore(uint16_t* sW, int ld, int r, int c0, const bf16x8& v, bool perm) {
  if (!perm) {
    *reinterpret_cast<bf16x8*>(sW + r * ld + c0) = v;
    return;
  }
  const int t = c0 >> 5, s = (c0 >> 4) & 1, gp = (c0 >> 2) & 3;  // gp even
  bf16x4 lo, hi;
  lo[0] = v[0]; lo[1] = v[1]; lo[2] = v[2]; lo[3] = v[3];
  hi[0] = v[4]; hi[1] = v[5]; hi[2] = v[6]; hi[3] = v[7];
  *reinterpret_cast<bf16x4*>(sW + r * ld + 32 * t + 8 * gp + 4 * s) = lo;
  *reinterpret_cast<bf16x4*>(sW + r * ld + 32 * t + 8 * (gp + 1) + 4 * s) = hi;
}
// row sums over the 64 channels of a CL row (all four lane groups get the total)
template <int NM>
__device__ __forceinline__ float cl_rowsum(const float (&v)[NM][4]) {
  float s = 0.f;
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) s += v[mt][i];
  return xor32_sum(xor16_sum(s));
}
// LayerNorm of CL rows in place (affine from LDS vectors, 16-byte broadcast reads)
template <int NM>
__device__ __forceinline__ void cl_layernorm(float (&v)[NM][4], const float* sg, const float* sb, float eps,
                                             float& mean, float& rstd) {
  constexpr int C = 16 * NM;
  const int g = lane_id() >> 4;
  mean = cl_rowsum<NM>(v) / C;
  float d[NM][4];
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) { d[mt][i] = v[mt][i] - mean; d[mt][i] *= d[mt][i]; }
  rstd = rsqrtf(cl_rowsum<NM>(d) / C + eps);
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    const float4 gg = *reinterpret_cast<const float4*>(sg + 16 * mt + 4 * g);
    const float4 bb = *reinterpret_cast<const float4*>(sb + 16 * mt + 4 * g);
    v[mt][0] = (v[mt][0] - mean) * rstd * gg.x + bb.x;
    v[mt][1] = (v[mt][1] - mean) * rstd * gg.y + bb.y;
    v[mt][2] = (v[mt][2] - mean) * rstd * gg.z + bb.z;
    v[mt][3] = (v[mt][3] - mean) * rstd * gg.w + bb.w;
  }
}
// CL residual dropout (same element hash as drop_rows: index row·C + channel)
template <int NM>
__device__ __forceinline__ void cl_drop(float (&v)[NM][4], const DropCfg& d, uint32_t sub, int gr) {
  if (d.thresh == 0u) return;
  constexpr int C = 16 * NM;
  const uint32_t key = drop_key(d.seed, d.site, sub);
  const int g = lane_id() >> 4;
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t idx = (uint32_t)gr * (uint32_t)C + (uint32_t)(16 * mt + 4 * g + i);
      v[mt][i] = keep_elem(key, 0u, idx, d.thresh) ? v[mt][i] * d.scale : 0.f;
    }
}
template <int NM>
__device__ __forceinline__ void cl_store_f32(float* __restrict__ Y, int ld, int gr, const float (&v)[NM][4]) {
  const int g = lane_id() >> 4;
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
    *reinterpret_cast<float4*>(Y + (long long)gr * ld + 16 * mt + 4 * g) = make_float4(v[mt][0], v[mt][1], v[mt][2], v[mt][3]);
}
template <int NM>
__device__ __forceinline__ void cl_store_bf16(uint16_t* __restrict__ Y, int ld, int gr, const float (&v)[NM][4]) {
  const int g = lane_id() >> 4;
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    uint2 pk;
    pk.x = pack2(v[mt][0], v[mt][1]);
    pk.y = pack2(v[mt][2], v[mt][3]);
    *reinterpret_cast<uint2*>(Y + (long long)gr * ld + 16 * mt + 4 * g) = pk;
  }
}
template <int NM>
__device__ __forceinline__ void cl_load_f32(float (&v)[NM][4], const float* __restrict__ X, int ld, int gr) {
  const int g = lane_id() >> 4;
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    const float4 a = *reinterpret_cast<const float4*>(X + (long long)gr * ld + 16 * mt + 4 * g);
    v[mt][0] = a.x; v[mt][1] = a.y; v[mt][2] = a.z; v[mt][3] = a.w;
  }
}
// acc (CL) + bias vector from LDS
template <int NM>
__device__ __forceinline__ void cl_bias(float (&v)[NM][4], const f32x4 (&acc)[NM], const float* sb) {
  const int g = lane_id() >> 4;
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    const float4 bb = *reinterpret_cast<const float4*>(sb + 16 * mt + 4 * g);
    v[mt][0] = acc[mt][0] + bb.x; v[mt][1] = acc[mt][1] + bb.y; v[mt][2] = acc[mt][2] + bb.z; v[mt][3] = acc[mt][3] + bb.w;
  }
}

// Fused latent self-attention layer forward, chain variant (same operands and results as
// sa_layer_fwd_kernel; all operands 16-byte aligned, host-checked).  Phase 0 issues every load
// and stages V, the four weight matrices (W1, W2, Wq permuted; Wo natural: its B operand, the
// attention output, is read from LDS in natural order) and the bias / LN vectors into LDS; the
// attention (wave = head) leaves O in LDS; after ONE barrier each wave runs the post-attention
// chain of its 16 rows from registers.
template <bool NEXT, int NQ>
__global__ __launch_bounds__(256) void sa_layer_fwd_chain_kernel(
    const uint16_t* __restrict__ QKV, int N, float scale_log2, uint16_t* __restrict__ Oout, float* __restrict__ LSE,
    const float* __restrict__ X, const uint16_t* __restrict__ Wo, const float* __restrict__ bo,
    const float* __restrict__ g2, const float* __restrict__ be2, float eps, const uint16_t* __restrict__ W1,
    const float* __restrict__ b1, const uint16_t* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ Z,
    float* __restrict__ Ysave, float* __restrict__ mean2, float* __restrict__ rstd2, uint16_t* __restrict__ Usave, int R,
    const float* __restrict__ lnw, const float* __restrict__ lnb, const uint16_t* __restrict__ Wq,
    const float* __restrict__ bq, uint16_t* __restrict__ QKVn, float* __restrict__ mean1, float* __restrict__ rstd1,
    DropCfg dr) {
  constexpr int C = 64, H = 4, D = 16, LD = C + 8, LDV = C + 8, C3 = 3 * C, MAXKT = 8, NM = 4;
  constexpr int nq = NQ * C, NWR = 3 * C + (NEXT ? nq : 0);  // weight rows staged: Wo, W1, W2 (+ Wq)
  constexpr int NWC = NWR * 8 / 256;                          // 16-byte weight chunks per thread
  __shared__ __attribute__((aligned(16))) uint16_t sV[256 * LDV + 64];  // V rows of the batch element (+ overrun)
  __shared__ __attribute__((aligned(16))) uint16_t sO[64 * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[NWR * LD];        // Wo | W1 | W2 | Wq
  __shared__ __attribute__((aligned(16))) float sVec[7 * C + (NEXT ? nq : 0)];  // bo b1 b2 γ2 β2 γ1 β1 | bq
  const int w = wave_id(), l = lane_id(), hh = l >> 5, r = l & 31;
  const int m0 = blockIdx.x * 64;
  const int b = m0 / N;
  const long long rb = (long long)b * N;
  const int nkt = N / 32;
  const int h = w;
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(kZero32B);

  // ---- phase 0: every load issued, branch-free (address selects) ----
  PIO_TS(0);
  bf16x8 kf[MAXKT], qf[2], vr[8], wr[NWC];
#pragma unroll
  for (int kt = 0; kt < MAXKT; ++kt)
    kf[kt] = *reinterpret_cast<const bf16x8*>(kt < nkt ? QKV + (rb + 32 * kt + r) * C3 + C + h * D + 8 * hh : zp);
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
    qf[qb] = *reinterpret_cast<const bf16x8*>(QKV + (long long)(m0 + 32 * qb + r) * C3 + h * D + 8 * hh);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = threadIdx.x + 256 * i, key = c >> 3, col = (c & 7) * 8;
    vr[i] = *reinterpret_cast<const bf16x8*>(key < N ? QKV + (rb + key) * C3 + 2 * C + col : zp);
  }
#pragma unroll
  for (int i = 0; i < NWC; ++i) {
    const int c = threadIdx.x + 256 * i, row = c >> 3, col = (c & 7) * 8;
    const uint16_t* src = row < C ? Wo + row * C : row < 2 * C ? W1 + (row - C) * C
                        : row < 3 * C ? W2 + (row - 2 * C) * C : Wq + (row - 3 * C) * C;
    wr[i] = *reinterpret_cast<const bf16x8*>(src + col);
  }
  const int gr = m0 + 16 * w + (l & 15);  // this lane's chain row
  float xr[NM][4];
  cl_load_f32<NM>(xr, X, C, gr);
  // bias / LN vectors: unconditional loads (address selects), predicated LDS stores
  PIO_TS(1);
  float pv[8];
  {
    const int k = threadIdx.x & (C - 1);
    pv[0] = bo[k]; pv[1] = b1[k]; pv[2] = b2[k]; pv[3] = g2[k]; pv[4] = be2[k];
    if constexpr (NEXT) {
      pv[5] = lnw[k]; pv[6] = lnb[k];
      pv[7] = bq[threadIdx.x < nq ? threadIdx.x : 0];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = threadIdx.x + 256 * i, key = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<bf16x8*>(sV + key * LDV + col) = vr[i];
  }
  if (threadIdx.x < C) {
    const int k = threadIdx.x;
    sVec[k] = pv[0]; sVec[C + k] = pv[1]; sVec[2 * C + k] = pv[2]; sVec[3 * C + k] = pv[3]; sVec[4 * C + k] = pv[4];
    if constexpr (NEXT) { sVec[5 * C + k] = pv[5]; sVec[6 * C + k] = pv[6]; }
  }
  if constexpr (NEXT)
    if ((int)threadIdx.x < nq) sVec[7 * C + threadIdx.x] = pv[7];
#pragma unroll
  for (int i = 0; i < NWC; ++i) {
    const int c = threadIdx.x + 256 * i, row = c >> 3, col = (c & 7) * 8;
    cl_wstore(sW, LD, row, col, wr[i], row >= C);  // Wo natural, the rest permuted
  }
  PIO_TS(2);
  lds_sync();
  PIO_TS(3);

  // ---- attention: wave h, two 32-query blocks; keys in chunks of 128 with an online softmax, so
  // one chunk's 64 scores per lane live at a time (all 256 keys at once kept 128 accumulators
  // live, which the allocator moved to AGPRs: ≈1,300 accvgpr copies per wave) ----
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    float m_run = -INFINITY, l_run = 0.f;
    f32x16 o = f32x16{};
#pragma unroll
    for (int ch = 0; ch < MAXKT / 4; ++ch) {
      if (4 * ch < nkt) {  // wave-uniform
        f32x16 sc[4];
        float mt = -INFINITY;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int kt = 4 * ch + k;
          sc[k] = f32x16{};
          if (kt < nkt) {
            sc[k] = mfma32(kf[kt], qf[qb], sc[k]);
#pragma unroll
            for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sc[k][i]);
          }
        }
        const float m_new = fmaxf(m_run, xor32_max(mt) * scale_log2);
        const float alpha = fast_exp2(m_run - m_new);  // 0 on the first chunk
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] *= alpha;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (4 * ch + k < nkt) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              sc[k][i] = fast_exp2(fmaf(sc[k][i], scale_log2, -m_new));
              l_run += sc[k][i];
            }
          }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int kt = 4 * ch + k;
          if (kt < nkt) {
#pragma unroll
            for (int ss = 0; ss < 2; ++ss)
              o = mfma32(frag_ks_perm(sV, LDV, h * D, 32 * kt + 16 * ss), pack_acc(sc[k], ss), o);
          }
        }
        m_run = m_new;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    const float ls = xor32_sum(l_run);
    const float inv = 1.f / ls;
    const int row = 32 * qb + r;
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
      uint2 pk;
      pk.x = pack2(o[4 * gg] * inv, o[4 * gg + 1] * inv);
      pk.y = pack2(o[4 * gg + 2] * inv, o[4 * gg + 3] * inv);
      *reinterpret_cast<uint2*>(sO + row * LD + h * D + 8 * gg + 4 * hh) = pk;
    }
    if (hh == 0) LSE[(long long)(m0 + row) * H + h] = m_run + __log2f(ls);
  }
  PIO_TS(4);
  lds_sync();
  PIO_TS(5);
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // the O tile for the backward
    const int c = threadIdx.x + 256 * i, row = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<bf16x8*>(Oout + (long long)(m0 + row) * C + col) =
        *reinterpret_cast<const bf16x8*>(sO + row * LD + col);
  }

  // ---- the post-attention chain of this wave's 16 rows ----
  const int g = l >> 4, lr = 16 * w + (l & 15);
  const uint16_t *sWo = sW, *sW1 = sW + C * LD, *sW2 = sW + 2 * C * LD, *sWq = sW + 3 * C * LD;
  f32x4 acc[NM];
  {
    bf16x8 bo_[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) bo_[t] = *reinterpret_cast<const bf16x8*>(sO + lr * LD + 32 * t + 8 * g);
    cl_gemm<NM, 2>(sWo, LD, bo_, acc);
  }
  PIO_TS(6);
  float y[NM][4], t0[NM][4];
  cl_bias<NM>(t0, acc, sVec);
  cl_drop<NM>(t0, dr, 0u, gr);
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) y[mt][i] = xr[mt][i] + t0[mt][i];
  cl_store_f32<NM>(Ysave, C, gr, y);
  float mu, rs;
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[mt][i] = y[mt][i];
  cl_layernorm<NM>(t0, sVec + 3 * C, sVec + 4 * C, eps, mu, rs);
  if (g == 0) { mean2[gr] = mu; rstd2[gr] = rs; }
  PIO_TS(7);
  {
    bf16x8 bb[2] = {cl_bfrag<NM>(t0, 0), cl_bfrag<NM>(t0, 1)};
    cl_gemm<NM, 2>(sW1, LD, bb, acc);
  }
  cl_bias<NM>(t0, acc, sVec + C);
  cl_store_bf16<NM>(Usave, C, gr, t0);
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[mt][i] = gelu_f(t0[mt][i]);
  {
    bf16x8 bb[2] = {cl_bfrag<NM>(t0, 0), cl_bfrag<NM>(t0, 1)};
    cl_gemm<NM, 2>(sW2, LD, bb, acc);
  }
  cl_bias<NM>(t0, acc, sVec + 2 * C);
  cl_drop<NM>(t0, dr, 1u, gr);
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[mt][i] += y[mt][i];
  cl_store_f32<NM>(Z, C, gr, t0);
  PIO_TS(8);
  if constexpr (NEXT) {
    cl_layernorm<NM>(t0, sVec + 5 * C, sVec + 6 * C, eps, mu, rs);
    if (g == 0) { mean1[gr] = mu; rstd1[gr] = rs; }
    bf16x8 bb[2] = {cl_bfrag<NM>(t0, 0), cl_bfrag<NM>(t0, 1)};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {  // 64 output channels at a time
      f32x4 aq[NM];
      cl_gemm<NM, 2>(sWq + q * C * LD, LD, bb, aq);
      float v[NM][4];
      cl_bias<NM>(v, aq, sVec + 7 * C + q * C);
      cl_store_bf16<NM>(QKVn + q * C, nq, gr, v);
    }
  }
  PIO_TS(9);
}

// ------------------------------------------------------------------------------------
// Self-attention layer boundary backward, chain variant (C = 64, H = 4; same operands and
// results as ln_linear_post_attn_bwd_kernel, all 16-byte aligned).  One 64-row tile per
// workgroup, wave w owns rows 16w..16w+15 in the chain layout (CL, see sa_layer_fwd_chain):
//   A  dXn1ᵀ = Wqᵀ·Gᵀ (G = dQKV of layer l+1, natural k order; Wqᵀ fragments by transposed LDS
//      reads of the natural Wq image), LN1 backward + dres → dZ of layer l, in registers;
//   B  the post-attention backward of layer l from registers: dHᵀ = W2ᵀ·dZmᵀ, dU = dH∘GELU'(U),
//      dXn2ᵀ = W1ᵀ·dUᵀ, LN2 backward → dY, dOᵀ = Woᵀ·dYmᵀ, delta = per-head rowsum(dO∘O);
//      (Wᵀ fragments: transposed reads of the natural W images in the CL k order);
//   C  every parameter gradient of the tile from bf16 LDS images of the operands (written
//      row-major along the way; the only two workgroup barriers of the chain precede this
//      phase and the overlay of Wq): each weight gradient is Tᵀ·A over the 64 rows
//      (16x16x32, both operands by transposed reads), its bias the same product with an
//      all-ones B operand, the LayerNorm γ gradients the diagonal of dXnᵀ·x̂.  The affine of a
//      LayerNorm-ed operand is applied in the epilogue (dW = γ∘(Gᵀ·x̂) + β⊗db), so only x̂ is
//      staged.  Partials go to this tile's slab row (plain stores).
// ------------------------------------------------------------------------------------
// the same in the CL k order of k-step t (element j ↔ k = 32t + 16(j >> 2) + 4g + (j & 3))
__device__ __forceinline__ bf16x8 frag16_tr_cl(const uint16_t* lds, int ld, int i0, int t) {
  const int l = lane_id(), g = l >> 4, i = l & 15;
  const uint16_t* base = lds + (32 * t + 4 * g + (i >> 2)) * ld + i0 + 4 * (i & 3);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + 16 * ld));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// dXᵀ (4 m-tiles over C = 64 input channels) = Wᵀ·dYᵀ for a CL gradient dY (2 k-steps)
__device__ __forceinline__ void cl_gemm_t(const uint16_t* sW, int ld, const bf16x8 (&b)[2], f32x4 (&acc)[4]) {
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[mt] = mfma16(frag16_tr_cl(sW, ld, 16 * mt, t), b[t], acc[mt]);
  }
}
// CL rows → a row-major bf16 LDS image [64][ld] (this wave's 16 rows)
template <int NM>
__device__ __forceinline__ void cl_tile_store(uint16_t* sT, int ld, const float (&v)[NM][4]) {
  const int l = lane_id(), row = 16 * wave_id() + (l & 15), g = l >> 4;
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    uint2 pk;
    pk.x = pack2(v[mt][0], v[mt][1]);
    pk.y = pack2(v[mt][2], v[mt][3]);
    *reinterpret_cast<uint2*>(sT + row * ld + 16 * mt + 4 * g) = pk;
  }
}
__device__ __forceinline__ bf16x8 ones_frag() {
  const short o = (short)0x3F80;  // bf16 1.0
  return bf16x8{o, o, o, o, o, o, o, o};
}
// slab partial of one 16-row block (m-tile mt) of a 64-column weight gradient
//   dW[m][n] = Σ_r A[r][m]·B[r][n]  (A, B bf16 row-major LDS images over the 64 rows)
// and its bias db[m] = Σ_r A[r][m]; with an LN affine (γ, β over n): dW = γ[n]·dW + β[n]·db[m]
__device__ __forceinline__ void cl_wgrad_block(const uint16_t* sA, int lda, int mt, const uint16_t* sB, int ldb,
                                               const float* gam, const float* bet, float* __restrict__ dW,
                                               float* __restrict__ db) {
  const int l = lane_id(), g = l >> 4, c = l & 15;
  f32x4 acc[5];
#pragma unroll
  for (int n = 0; n < 5; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const bf16x8 a = frag16_tr(sA, lda, 16 * mt, 32 * t);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma16(a, frag16_tr(sB, ldb, 16 * nt, 32 * t), acc[nt]);
    acc[4] = mfma16(a, ones_frag(), acc[4]);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = 16 * nt + c;
    const float gn = gam ? gam[n] : 1.f, bn = bet ? bet[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 16 * mt + 4 * g + i;
      dW[m * 64 + n] = acc[nt][i] * gn + acc[4][i] * bn;
    }
  }
  if (c == 0)
#pragma unroll
    for (int i = 0; i < 4; ++i) db[16 * mt + 4 * g + i] = acc[4][i];
}
// LayerNorm parameter gradients of channel block mt: dγ = diag(dXnᵀ·x̂), dβ = Σ_r dXn
__device__ __forceinline__ void cl_ln_grads(const uint16_t* sD, const uint16_t* sXh, int ld, int mt,
                                            float* __restrict__ dg, float* __restrict__ dbt) {
  const int l = lane_id(), g = l >> 4, c = l & 15;
  f32x4 dia = f32x4{0.f, 0.f, 0.f, 0.f}, sum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const bf16x8 a = frag16_tr(sD, ld, 16 * mt, 32 * t);
    dia = mfma16(a, frag16_tr(sXh, ld, 16 * mt, 32 * t), dia);
    sum = mfma16(a, ones_frag(), sum);
  }
  const int i = c - 4 * g;  // acc row 4g + i is channel column c on the diagonal
  if (i >= 0 && i < 4) dg[16 * mt + c] = i == 0 ? dia[0] : i == 1 ? dia[1] : i == 2 ? dia[2] : dia[3];
  if (c == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) dbt[16 * mt + 4 * g + k] = sum[k];
}

template <int NQ>
constexpr int lpb_chain_smem() {
  // W images (Wo W1 W2) | LL images (G, x̂1, dXn1) | Wq image, overlaid by the 7 PA images | vectors
  return 2 * (3 * 64 * 72) + 2 * (64 * (NQ * 64 + 8) + 2 * 64 * 72) +
         2 * (NQ * 64 * 72 > 7 * 64 * 72 ? NQ * 64 * 72 : 7 * 64 * 72) + 4 * 4 * 64;
}

// TG: the element type of G (float, or uint16_t = bf16 straight from the attention backward's
// bf16 outputs: the kernel consumes G only as bf16 MFMA operands, so both give identical results)
template <int NQ, typename TG>
__global__ __launch_bounds__(256) void ln_linear_post_attn_bwd_chain_kernel(
    const TG* __restrict__ G, const uint16_t* __restrict__ Wq, const float* __restrict__ X,
    const float* __restrict__ mean1, const float* __restrict__ rstd1, const float* __restrict__ lnw,
    const float* __restrict__ lnb, const float* __restrict__ dres, float* __restrict__ dlnw, float* __restrict__ dlnb,
    float* __restrict__ dWq, float* __restrict__ dbq, const float* __restrict__ Ysave, const float* __restrict__ mean2,
    const float* __restrict__ rstd2, const uint16_t* __restrict__ U, const uint16_t* __restrict__ O,
    const uint16_t* __restrict__ Wo, const uint16_t* __restrict__ W1, const uint16_t* __restrict__ W2,
    const float* __restrict__ g2, const float* __restrict__ be2, float* __restrict__ dY, uint16_t* __restrict__ dO,
    float* __restrict__ delta, PostAttnGrads gr_out, int R, SlabJob job, DropCfg dr) {
  constexpr int C = 64, LD = 72, NM = 4, nq = NQ * C, LDG = nq + 8, KT = nq / 32;
  constexpr int NWC = (3 * C + nq) * 8 / 256;  // 16-byte weight chunks per thread
  __shared__ __attribute__((aligned(16))) unsigned char smem[lpb_chain_smem<NQ>()];
  uint16_t* sWo = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sW1 = sWo + C * LD;
  uint16_t* sW2 = sW1 + C * LD;
  uint16_t* sG = sW2 + C * LD;         // [64][LDG]  G (bf16)
  uint16_t* sX1 = sG + 64 * LDG;       // [64][LD]   x̂ of LN1
  uint16_t* sD1 = sX1 + 64 * LD;       // [64][LD]   dXn1
  uint16_t* sWq = sD1 + 64 * LD;       // [nq][LD]   Wq (phase A), then the PA images:
  uint16_t* sZm = sWq;                 //   dZ∘m₁
  uint16_t* sGu = sZm + 64 * LD;       //   GELU(U)
  uint16_t* sDu = sGu + 64 * LD;       //   dU
  uint16_t* sYh = sDu + 64 * LD;       //   ŷ of LN2
  uint16_t* sD2 = sYh + 64 * LD;       //   dXn2
  uint16_t* sYm = sD2 + 64 * LD;       //   dY∘m₀
  uint16_t* sOt = sYm + 64 * LD;       //   O
  float* sVec = reinterpret_cast<float*>(smem + lpb_chain_smem<NQ>() - 4 * 4 * 64);  // γ1 β1 γ2 β2
  zero_span_block(job);
  if ((int)blockIdx.x >= (R + 63) / 64) {  // appended workgroups: the previous kernel's slab job
    slab_reduce_block(job, blockIdx.x - (R + 63) / 64, reinterpret_cast<float4*>(smem));
    return;
  }
  const int w = wave_id(), l = lane_id(), g = l >> 4;
  const int gr = blockIdx.x * 64 + 16 * w + (l & 15);

  // ---- phase 0: every load in flight ----
  PIO_TS(0);
  bf16x8 wr[NWC];
#pragma unroll
  for (int i = 0; i < NWC; ++i) {
    const int c = threadIdx.x + 256 * i, row = c >> 3, col = (c & 7) * 8;
    const uint16_t* src = row < C ? Wo + row * C : row < 2 * C ? W1 + (row - C) * C
                        : row < 3 * C ? W2 + (row - 2 * C) * C : Wq + (row - 3 * C) * C;
    wr[i] = *reinterpret_cast<const bf16x8*>(src + col);
  }
  constexpr bool GBF = sizeof(TG) == 2;
  float4 gv[GBF ? 1 : KT][2];
  bf16x8 gvb[GBF ? KT : 1];
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const TG* p = G + (long long)gr * nq + 32 * t + 8 * g;
    if constexpr (GBF) {
      gvb[t] = *reinterpret_cast<const bf16x8*>(p);
    } else {
      gv[t][0] = *reinterpret_cast<const float4*>(p);
      gv[t][1] = *reinterpret_cast<const float4*>(p + 4);
    }
  }
  float xv[NM][4], dv[NM][4], yv[NM][4];
  cl_load_f32<NM>(xv, X, C, gr);
  cl_load_f32<NM>(dv, dres, C, gr);
  cl_load_f32<NM>(yv, Ysave, C, gr);
  uint2 ub[NM], obv[NM];
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    ub[mt] = *reinterpret_cast<const uint2*>(U + (long long)gr * C + 16 * mt + 4 * g);
    obv[mt] = *reinterpret_cast<const uint2*>(O + (long long)gr * C + 16 * mt + 4 * g);
  }
  const float mu1 = mean1[gr], rs1 = rstd1[gr], mu2 = mean2[gr], rs2 = rstd2[gr];
  PIO_TS(1);
  float pv[4];
  {
    const int k = threadIdx.x & (C - 1);
    pv[0] = lnw[k]; pv[1] = lnb[k]; pv[2] = g2[k]; pv[3] = be2[k];
  }
#pragma unroll
  for (int i = 0; i < NWC; ++i) {
    const int c = threadIdx.x + 256 * i, row = c >> 3, col = (c & 7) * 8;
    uint16_t* dst = row < 3 * C ? sWo + row * LD : sWq + (row - 3 * C) * LD;
    *reinterpret_cast<bf16x8*>(dst + col) = wr[i];
  }
  if (threadIdx.x < C) {
    const int k = threadIdx.x;
    sVec[k] = pv[0]; sVec[C + k] = pv[1]; sVec[2 * C + k] = pv[2]; sVec[3 * C + k] = pv[3];
  }
  PIO_TS(2);
  lds_sync();
  PIO_TS(3);

  // ---- A: LN1 + QKV backward of layer l+1 → dZ of layer l ----
  f32x4 acc[NM];
  {
    bf16x8 gb[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if constexpr (GBF) {
        gb[t] = gvb[t];
      } else {
        const float4 a = gv[t][0], b = gv[t][1];
        gb[t][0] = (short)f2bf(a.x); gb[t][1] = (short)f2bf(a.y); gb[t][2] = (short)f2bf(a.z); gb[t][3] = (short)f2bf(a.w);
        gb[t][4] = (short)f2bf(b.x); gb[t][5] = (short)f2bf(b.y); gb[t][6] = (short)f2bf(b.z); gb[t][7] = (short)f2bf(b.w);
      }
      *reinterpret_cast<bf16x8*>(sG + (16 * w + (l & 15)) * LDG + 32 * t + 8 * g) = gb[t];
    }
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) {
      acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KT; ++t) acc[mt] = mfma16(frag16_tr(sWq, LD, 16 * mt, 32 * t), gb[t], acc[mt]);
    }
  }
  PIO_TS(4);
  float dz[NM][4], t0[NM][4];
  {
    float gg[NM][4];
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) {
      const float4 ga = *reinterpret_cast<const float4*>(sVec + 16 * mt + 4 * g);
      const float gw[4] = {ga.x, ga.y, ga.z, ga.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xv[mt][i] = (xv[mt][i] - mu1) * rs1;  // x̂
        t0[mt][i] = acc[mt][i];               // dXn1
        gg[mt][i] = acc[mt][i] * gw[i];
        dz[mt][i] = gg[mt][i] * xv[mt][i];
      }
    }
    const float s1 = cl_rowsum<NM>(gg) / C, s2 = cl_rowsum<NM>(dz) / C;
#pragma unroll
    for (int mt = 0; mt < NM; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) dz[mt][i] = rs1 * (gg[mt][i] - s1 - xv[mt][i] * s2) + dv[mt][i];
  }
  cl_tile_store<NM>(sX1, LD, xv);
  cl_tile_store<NM>(sD1, LD, t0);
  PIO_TS(5);
  lds_sync();  // every wave is done with the Wq image: the PA images overlay it
  PIO_TS(6);

  // ---- B: post-attention backward of layer l ----
  float gp[NM][4];
#pragma unroll
  for (int mt = 0; mt < NM; ++mt) {
    const float u4[4] = {bf2f((uint16_t)(ub[mt].x & 0xFFFF)), bf2f((uint16_t)(ub[mt].x >> 16)),
                         bf2f((uint16_t)(ub[mt].y & 0xFFFF)), bf2f((uint16_t)(ub[mt].y >> 16))};
#pragma unroll
    for (int i = 0; i < 4; ++i) gelu_pair(u4[i], t0[mt][i], gp[mt][i]);
  }
  cl_tile_store<NM>(sGu, LD, t0);
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[mt][i] = dz[mt][i];
  cl_drop<NM>(t0, dr, 1u, gr);  // dZ∘m₁: the MLP output layer's gradient
  cl_tile_store<NM>(sZm, LD, t0);
  {
    bf16x8 bb[2] = {cl_bfrag<NM>(t0, 0), cl_bfrag<NM>(t0, 1)};
    cl_gemm_t(sW2, LD, bb, acc);  // dH
  }
  PIO_TS(7);
#pragma unroll
  for (int mt = 0; mt < NM; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) t0[mt][i] = acc[mt][i] * gp[mt][i];  // dU
  cl_tile_store<NM>(sDu, LD, t0);
  {
    bf16x8 bb[2] = {cl_bfrag<NM>(t0, 0), cl_bfrag<NM>(t0, 1)};
    cl_gemm_t(sW1, LD, bb, acc);  // dXn2
  }
  {
    float gg[NM][4];
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) {
      const float4 ga = *reinterpret_cast<const float4*>(sVec + 2 * C + 16 * mt + 4 * g);
      const float gw[4] = {ga.x, ga.y, ga.z, ga.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        yv[mt][i] = (yv[mt][i] - mu2) * rs2;  // ŷ
        t0[mt][i] = acc[mt][i];               // dXn2
        gg[mt][i] = acc[mt][i] * gw[i];
        gp[mt][i] = gg[mt][i] * yv[mt][i];
      }
    }
    const float s1 = cl_rowsum<NM>(gg) / C, s2 = cl_rowsum<NM>(gp) / C;
#pragma unroll
    for (int mt = 0; mt < NM; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) dz[mt][i] += rs2 * (gg[mt][i] - s1 - yv[mt][i] * s2);  // dY
  }
  PIO_TS(8);
  cl_tile_store<NM>(sYh, LD, yv);
  cl_tile_store<NM>(sD2, LD, t0);
  cl_store_f32<NM>(dY, C, gr, dz);
  cl_drop<NM>(dz, dr, 0u, gr);  // dY∘m₀: the out-projection's gradient
  cl_tile_store<NM>(sYm, LD, dz);
  {
    bf16x8 bb[2] = {cl_bfrag<NM>(dz, 0), cl_bfrag<NM>(dz, 1)};
    cl_gemm_t(sWo, LD, bb, acc);  // dO
  }
  {
    float ov[NM][4], dd[NM];
#pragma unroll
    for (int mt = 0; mt < NM; ++mt) {
      ov[mt][0] = bf2f((uint16_t)(obv[mt].x & 0xFFFF)); ov[mt][1] = bf2f((uint16_t)(obv[mt].x >> 16));
      ov[mt][2] = bf2f((uint16_t)(obv[mt].y & 0xFFFF)); ov[mt][3] = bf2f((uint16_t)(obv[mt].y >> 16));
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        t0[mt][i] = bf2f(f2bf(acc[mt][i]));  // dO as the attention backward sees it
        s += t0[mt][i] * ov[mt][i];
      }
      dd[mt] = xor32_sum(xor16_sum(s));  // head mt = channels 16mt .. 16mt + 15
    }
    cl_store_bf16<NM>(dO, C, gr, t0);
    if (g == 0) *reinterpret_cast<float4*>(delta + (long long)gr * 4) = make_float4(dd[0], dd[1], dd[2], dd[3]);
    cl_tile_store<NM>(sOt, LD, ov);
  }
  PIO_TS(9);
  lds_sync();
  PIO_TS(10);

  // ---- C: parameter gradients of the tile → slab row blockIdx.x ----
  const int vrs = gr_out.vrs;
  const long long so = (long long)blockIdx.x * vrs;
  const float *gam1 = sVec, *bet1 = sVec + C, *gam2 = sVec + 2 * C, *bet2 = sVec + 3 * C;
  auto sp = [&](float* p) { return p + so; };  // this tile's slab row
  cl_wgrad_block(sZm, LD, w, sGu, LD, nullptr, nullptr, sp(gr_out.dW2), sp(gr_out.db2));
  cl_wgrad_block(sDu, LD, w, sYh, LD, gam2, bet2, sp(gr_out.dW1), sp(gr_out.db1));
  cl_wgrad_block(sYm, LD, w, sOt, LD, nullptr, nullptr, sp(gr_out.dWo), sp(gr_out.dbo));
  cl_ln_grads(sD2, sYh, LD, w, sp(gr_out.dg2), sp(gr_out.dbe2));
  PIO_TS(11);
#pragma unroll
  for (int q = 0; q < NQ; ++q)  // 16-row blocks w, w + 4, w + 8 of dWq (nq rows)
    cl_wgrad_block(sG, LDG, w + 4 * q, sX1, LD, gam1, bet1, sp(dWq), sp(dbq));
  cl_ln_grads(sD1, sX1, LD, w, sp(dlnw), sp(dlnb));
  PIO_TS(12);
}

// ---- launchers (called by rowgemm.hip's launchers once the operands qualify: C = 64, H = 4,
// every pointer 16-byte aligned, R % 64 == 0) ----
bool sa_layer_fwd_chain_launch(const uint16_t* QKV, int N, float scale_log2, uint16_t* O, float* LSE, const float* X,
                               const uint16_t* Wo, const float* bo, const float* g2, const float* be2, float eps,
                               const uint16_t* W1, const float* b1, const uint16_t* W2, const float* b2, float* Z,
                               float* Ysave, float* mean2, float* rstd2, uint16_t* Usave, int R, const float* lnw,
                               const float* lnb, const uint16_t* Wq, const float* bq, uint16_t* QKVn, float* mean1,
                               float* rstd1, const DropCfg& dr, int nq, hipStream_t st) {
  const bool next = Wq != nullptr;
  if (next && nq != 64 && nq != 128 && nq != 192) return false;
  dim3 grid(R / 64);
#define SAC(NX, NQ)                                                                                                   \
  hipLaunchKernelGGL((sa_layer_fwd_chain_kernel<NX, NQ>), grid, dim3(256), 0, st, QKV, N, scale_log2, O, LSE, X, Wo, bo, \
                     g2, be2, eps, W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, lnw, lnb, Wq, bq, QKVn, mean1,      \
                     rstd1, dr)
  if (!next) SAC(false, 3);
  else if (nq == 64) SAC(true, 1);
  else if (nq == 128) SAC(true, 2);
  else SAC(true, 3);
#undef SAC
  return true;
}

bool ln_linear_post_attn_bwd_chain_launch(const void* G, bool g_bf16, const uint16_t* Wq, const float* X, const float* mean1,
                                          const float* rstd1, const float* lnw, const float* lnb, const float* dres,
                                          float* dlnw, float* dlnb, float* dWq, float* dbq, const float* Ysave,
                                          const float* mean2, const float* rstd2, const uint16_t* U, const uint16_t* O,
                                          const uint16_t* Wo, const uint16_t* W1, const uint16_t* W2, const float* g2,
                                          const float* be2, float* dY, uint16_t* dO, float* delta,
                                          const PostAttnGrads& grads, int R, const SlabJob& job, const DropCfg& dr,
                                          int nq, hipStream_t st) {
  if (nq != 192 && nq != 64) return false;
  dim3 grid((R + 63) / 64 + (job.slab ? job.nblk : 0));
#define LPC(NQ, TG)                                                                                                    \
  hipLaunchKernelGGL((ln_linear_post_attn_bwd_chain_kernel<NQ, TG>), grid, dim3(256), 0, st, static_cast<const TG*>(G), \
                     Wq, X, mean1, rstd1, lnw, lnb, dres, dlnw, dlnb, dWq, dbq, Ysave, mean2, rstd2, U, O, Wo, W1, W2, g2,  \
                     be2, dY, dO, delta, grads, R, job, dr)
  if (g_bf16) {
    if (nq != 192) return false;  // bf16 G only from the self-attention backward (nq = 3C)
    LPC(3, uint16_t);
  } else if (nq == 192) {
    LPC(3, float);
  } else {
    LPC(1, float);
  }
#undef LPC
  return true;
}

}  // namespace pio
