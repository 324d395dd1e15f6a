// Chain-layout (CL) kernels: the fused self-attention layer forward and the layer-boundary
// backward as register-resident row chains on v_mfma_f32_16x16x32_bf16 (see the CL banner
// below).  Compiled with -mllvm -amdgpu-mfma-vgpr-form=1 (csrc/build.py): MFMA results stay in
// VGPRs, so the softmax and LayerNorm VALU work reads them directly instead of copying every
// accumulator out of (and back into) AGPRs (≈1,300 v_accvgpr moves per wave in the attention
// phase otherwise).  The CL / CL2 helpers live in chain_cl.h (shared with persist.hip).
#include <stdlib.h>

#include <algorithm>

#include "chain_cl.h"

namespace pio {


// The fused latent self-attention layer forward on 8 waves (same operands and results as
// sa_layer_fwd_chain_kernel).  Attention: wave w = (head w & 3, 32-query block w >> 2).  The
// post-attention chain: the paired CL2 layout above (5 pair exchanges: LN2, W1, W2, LN1, Wq).
// MAXKT: 32-key tiles of the K / V operand (8: N ≤ 256, 16: N ≤ 512 — the long-context MLM's
// 512 latents; every K fragment is loaded in phase 0, the V rows of the batch element live in LDS).
template <bool NEXT, int NQ, int MAXKT, bool ADROP>
__global__ __launch_bounds__(512) void sa_layer_fwd_chain8_kernel(
    const uint16_t* __restrict__ QKV, int N, float scale_log2, uint16_t* __restrict__ Oout, float* __restrict__ LSE,
    const float* __restrict__ X, const uint16_t* __restrict__ Wo, const float* __restrict__ bo,
    const float* __restrict__ g2, const float* __restrict__ be2, float eps, const uint16_t* __restrict__ W1,
    const float* __restrict__ b1, const uint16_t* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ Z,
    float* __restrict__ Ysave, float* __restrict__ mean2, float* __restrict__ rstd2, uint16_t* __restrict__ Usave, int R,
    const float* __restrict__ lnw, const float* __restrict__ lnb, const uint16_t* __restrict__ Wq,
    const float* __restrict__ bq, uint16_t* __restrict__ QKVn, float* __restrict__ mean1, float* __restrict__ rstd1,
    DropCfg dr) {
  constexpr int C = 64, H = 4, D = 16, LD = C + 8, LDV = C + 8, C3 = 3 * C, NT = 512;
  constexpr int NVI = MAXKT * 32 * 8 / NT;  // 16-byte V chunks per thread
  static_assert(MAXKT % 4 == 0 && MAXKT * 32 * 8 % NT == 0, "key tiles");
  constexpr int nq = NQ * C, NWR = 3 * C + (NEXT ? nq : 0);  // weight rows staged: Wo, W1, W2 (+ Wq)
  constexpr int NWC = NWR * 8 / NT;                           // 16-byte weight chunks per thread
  static_assert(NWR * 8 % NT == 0, "weight staging");
  __shared__ __attribute__((aligned(16))) uint16_t sV[MAXKT * 32 * LDV + 64];  // V rows of the batch element (+ overrun)
  __shared__ __attribute__((aligned(16))) uint16_t sO[64 * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[NWR * LD];        // Wo | W1 | W2 | Wq
  __shared__ __attribute__((aligned(16))) float sVec[7 * C + (NEXT ? nq : 0)];  // bo b1 b2 γ2 β2 γ1 β1 | bq
  __shared__ __attribute__((aligned(16))) bf16x8 sX[2][8 * 64];           // pair fragment slots
  __shared__ __attribute__((aligned(16))) float2 sR[2][8 * 16];           // pair LN slots
  __shared__ __attribute__((aligned(16))) uint16_t sOnes[16 * 16];          // bf16 ones (P·V denominator rows)
  // the body is instantiated once per wave half (hf = qb = w >> 2, compile-time inside)
  PIO_WG_BEGIN();
  auto body = [&](auto hfc) {
  constexpr int hf = decltype(hfc)::value, qb = hf;
  const int w = wave_id(), l = lane_id(), hh = l >> 5, r = l & 31;
  // consecutive tiles (the tiles of one batch element, which all read its K / V) on one XCD, so
  // the K / V rows come through that XCD's L2 once instead of once per tile
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * 64;
  const int b = m0 / N;
  const long long rb = (long long)b * N;
  const int nkt = N / 32;
  const int h = w & 3;  // attention role: head h, query block qb; chain role: rows of pair w & 3, channel half hf
  const uint16_t* zp = reinterpret_cast<const uint16_t*>(kZero32B);

  // ---- phase 0: every load issued, branch-free (address selects) ----
  PIO_TS(0);
  bf16x8 kf[MAXKT], qf, vr[NVI], wr[NWC];
#pragma unroll
  for (int kt = 0; kt < MAXKT; ++kt)
    kf[kt] = *reinterpret_cast<const bf16x8*>(kt < nkt ? QKV + (rb + 32 * kt + r) * C3 + C + h * D + 8 * hh : zp);
  qf = *reinterpret_cast<const bf16x8*>(QKV + (long long)(m0 + 32 * qb + r) * C3 + h * D + 8 * hh);
#pragma unroll
  for (int i = 0; i < NVI; ++i) {
    const int c = threadIdx.x + NT * i, key = c >> 3, col = (c & 7) * 8;
    vr[i] = *reinterpret_cast<const bf16x8*>(key < N ? QKV + (rb + key) * C3 + 2 * C + col : zp);
  }
#pragma unroll
  for (int i = 0; i < NWC; ++i) {
    const int c = threadIdx.x + NT * i, row = c >> 3, col = (c & 7) * 8;
    const uint16_t* src = row < C ? Wo + row * C : row < 2 * C ? W1 + (row - C) * C
                        : row < 3 * C ? W2 + (row - 2 * C) * C : Wq + (row - 3 * C) * C;
    wr[i] = *reinterpret_cast<const bf16x8*>(src + col);
  }
  const int g = l >> 4;
  const int gr = m0 + 16 * (w & 3) + (l & 15);  // this lane's chain row
  float xr[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float4 a = *reinterpret_cast<const float4*>(X + (long long)gr * C + 16 * (2 * hf + i) + 4 * g);
    xr[i][0] = a.x; xr[i][1] = a.y; xr[i][2] = a.z; xr[i][3] = a.w;
  }
  PIO_TS(1);
  float pv = 0.f;
  {
    // vector slots: [0, 7C) = bo b1 b2 γ2 β2 γ1 β1, [7C, 7C + nq) = bq (address selects)
    const int k = threadIdx.x;
    const int vi = k >> 6, kk = k & 63;
    const float* src = vi == 0 ? bo : vi == 1 ? b1 : vi == 2 ? b2 : vi == 3 ? g2 : vi == 4 ? be2
                     : vi == 5 ? (NEXT ? lnw : bo) : vi == 6 ? (NEXT ? lnb : bo) : bo;
    pv = src[kk];  // unconditional (threads past 7C read bo and store nothing)
  }
  float pq = 0.f;
  if constexpr (NEXT) pq = bq[(int)threadIdx.x < nq ? threadIdx.x : 0];
#pragma unroll
  for (int i = 0; i < NVI; ++i) {
    const int c = threadIdx.x + NT * i, key = c >> 3, col = (c & 7) * 8;
    *reinterpret_cast<bf16x8*>(sV + key * LDV + col) = vr[i];
  }
  if ((int)threadIdx.x < 7 * C) sVec[threadIdx.x] = pv;
  if (threadIdx.x < 128) reinterpret_cast<uint32_t*>(sOnes)[threadIdx.x] = 0x3F803F80u;
  if constexpr (NEXT)
    if ((int)threadIdx.x < nq) sVec[7 * C + threadIdx.x] = pq;
#pragma unroll
  for (int i = 0; i < NWC; ++i) {
    const int c = threadIdx.x + NT * i, row = c >> 3, col = (c & 7) * 8;
    cl_wstore(sW, LD, row, col, wr[i], row >= C);  // Wo natural, the rest permuted
  }
  PIO_TS(2);
  lds_sync();
  PIO_TS(3);

  // ---- attention: head h, query block qb; keys in chunks of 128 with an online softmax.  The
  // P·V product's A operand (Vᵀ, 32 rows) has only 16 rows of this head (D = 16): rows 16..31
  // are ones, so accumulator rows 16..31 (registers 8..15) collect the softmax denominator
  // Σ_k P[k][q] — no per-element VALU sum (and the denominator of exactly the bf16 P that
  // weights V) ----
  {
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
            sc[k] = mfma32(kf[kt], qf, sc[k]);
#pragma unroll
            for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sc[k][i]);
          }
        }
        const float m_new = fmaxf(m_run, xor32_max(mt) * scale_log2);
        const float alpha = fast_exp2(m_run - m_new);  // 0 on the first chunk
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] *= alpha;
        if constexpr (ADROP) l_run *= alpha;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (4 * ch + k < nkt) {
#pragma unroll
            for (int i = 0; i < 16; ++i) sc[k][i] = fast_exp2(fmaf(sc[k][i], scale_log2, -m_new));
            if constexpr (ADROP) {
              // attention-probability dropout (reference model.py:66-71, nn.MultiheadAttention's
              // dropout): the softmax denominator sums the kept AND the dropped probabilities, the
              // P·V product sees P∘mask/(1−p); masks as attn_bwd regenerates them (stream b·H + h,
              // element q·N + key of the sample)
              const uint32_t dkey = drop_key(dr.seed, dr.site, 2u);
              // element index (row)·N + 32(4ch + k) + 4hh + acc_row(i, 0) (keep_elem_m)
              uint32_t cm0 = ((uint32_t)(m0 - rb + 32 * qb + r) * (uint32_t)N + (uint32_t)(32 * (4 * ch + k) + 4 * hh)) * kHashM1;
              asm volatile("" : "+v"(cm0));
              const uint32_t hs = hash3_seed(dkey, (uint32_t)(b * H + h));
#pragma unroll
              for (int i = 0; i < 16; ++i) {
                l_run += sc[k][i];
                sc[k][i] = keep_elem_m(hs, cm0 + (uint32_t)acc_row(i, 0) * kHashM1, dr.thresh) ? sc[k][i] * dr.scale : 0.f;
              }
            }
          }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int kt = 4 * ch + k;
          if (kt < nkt) {
#pragma unroll
            for (int ss = 0; ss < 2; ++ss)
              o = mfma32(frag_ks_perm_ones(sV, LDV, h * D, 32 * kt + 16 * ss, sOnes), pack_acc(sc[k], ss), o);
          }
        }
        m_run = m_new;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // row 16 (a ones row): Σ_k P[k][q] of this lane's query; with dropout the explicit sum of the
    // undropped probabilities (the ones rows summed the dropped ones)
    const float ls = ADROP ? xor32_sum(l_run) : o[8];
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
  {  // the O tile for the backward: one 16-byte chunk per thread
    const int row = threadIdx.x >> 3, col = (threadIdx.x & 7) * 8;
    *reinterpret_cast<bf16x8*>(Oout + (long long)(m0 + row) * C + col) = *reinterpret_cast<const bf16x8*>(sO + row * LD + col);
  }

  // ---- the post-attention chain: pair w & 3, channel half hf ----
  const int lr = 16 * (w & 3) + (l & 15);
  const uint16_t *sWo = sW, *sW1 = sW + C * LD, *sW2 = sW + 2 * C * LD, *sWq = sW + 3 * C * LD;
  f32x4 acc[2];
  {
    bf16x8 bo_[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) bo_[t] = *reinterpret_cast<const bf16x8*>(sO + lr * LD + 32 * t + 8 * g);
    cl2_gemm(sWo, LD, hf, bo_, acc);
  }
  PIO_TS(6);
  float y[2][4], t0[2][4];
  cl2_bias(t0, acc, sVec, hf);
  cl2_drop(t0, dr, 0u, gr, hf);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { y[i][j] = xr[i][j] + t0[i][j]; t0[i][j] = y[i][j]; }
  cl2_store_f32(Ysave, C, gr, hf, y);
  float mu, rs;
  cl2_layernorm(t0, sR[0], hf, sVec + 3 * C, sVec + 4 * C, eps, mu, rs);
  if (g == 0 && hf == 0) { mean2[gr] = mu; rstd2[gr] = rs; }
  PIO_TS(7);
  {
    bf16x8 bb[2];
    cl2_swap_frag(sX[0], cl2_frag(t0), hf, bb);
    cl2_gemm(sW1, LD, hf, bb, acc);
  }
  cl2_bias(t0, acc, sVec + C, hf);
  cl2_store_bf16(Usave, C, gr, hf, t0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) t0[i][j] = gelu_f(t0[i][j]);
  {
    bf16x8 bb[2];
    cl2_swap_frag(sX[1], cl2_frag(t0), hf, bb);
    cl2_gemm(sW2, LD, hf, bb, acc);
  }
  cl2_bias(t0, acc, sVec + 2 * C, hf);
  cl2_drop(t0, dr, 1u, gr, hf);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) t0[i][j] += y[i][j];
  cl2_store_f32(Z, C, gr, hf, t0);
  PIO_TS(8);
  if constexpr (NEXT) {
    cl2_layernorm(t0, sR[1], hf, sVec + 5 * C, sVec + 6 * C, eps, mu, rs);
    if (g == 0 && hf == 0) { mean1[gr] = mu; rstd1[gr] = rs; }
    bf16x8 bb[2];
    cl2_swap_frag(sX[0], cl2_frag(t0), hf, bb);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {  // 64 output channels at a time, this wave's half of them
      f32x4 aq[2];
      cl2_gemm(sWq + q * C * LD, LD, hf, bb, aq);
      float v[2][4];
      cl2_bias(v, aq, sVec + 7 * C + q * C, hf);
      cl2_store_bf16(QKVn + q * C, nq, gr, hf, v);
    }
  }
  PIO_TS(9);
  };
  if (wave_id() >> 2) body(std::integral_constant<int, 1>{});
  else body(std::integral_constant<int, 0>{});
  PIO_WG_END();
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

// ATT (N = 64 latents per sample, one sample per tile): phase D appends the attention backward
// of layer l itself — Q / K / V of layer l and its LSE are loaded in phase 0, dO and δ come
// from phase B's registers — and the kernel stores dQKV of layer l (bf16) instead of dO / δ:
// the separate attention-backward launch of the layer disappears.  Wave w = (head w & 3, keys
// 32(w >> 2) .. + 31); per 32-query tile: S = Q·Kᵀ, dP = dO·Vᵀ, dS = P∘(dP − δ) (+ the
// attention-probability dropout of the forward, same hash stream as attn_bwd), dV += Pᵀ·dO,
// dK += dSᵀ·Q; the dS slabs of both key halves meet in LDS for dQ = dS·K; the dQKV tile leaves
// through LDS as 16-byte rows.
struct ChainAttn {
  const uint16_t* qkv;  // layer l's packed Q | K | V rows (R, 3C) bf16
  const float* lse;     // (R, H) log2-domain softmax statistics of the forward
  uint16_t* dqkv;       // (R, 3C) bf16 out
  float scale, scale_log2;
};

template <int NQ, typename TG, bool ATT>
__global__ __launch_bounds__(512) void ln_linear_post_attn_bwd_chain8_kernel(
    const TG* __restrict__ G, const uint16_t* __restrict__ Wq, const float* __restrict__ X,
    const float* __restrict__ mean1, const float* __restrict__ rstd1, const float* __restrict__ lnw,
    const float* __restrict__ lnb, const float* __restrict__ dres, float* __restrict__ dlnw, float* __restrict__ dlnb,
    float* __restrict__ dWq, float* __restrict__ dbq, const float* __restrict__ Ysave, const float* __restrict__ mean2,
    const float* __restrict__ rstd2, const uint16_t* __restrict__ U, const uint16_t* __restrict__ O,
    const uint16_t* __restrict__ Wo, const uint16_t* __restrict__ W1, const uint16_t* __restrict__ W2,
    const float* __restrict__ g2, const float* __restrict__ be2, float* __restrict__ dY, uint16_t* __restrict__ dO,
    float* __restrict__ delta, PostAttnGrads gr_out, int R, SlabJob job, DropCfg dr, ChainAttn at) {
  constexpr int C = 64, LD = 64, nq = NQ * C, LDG = nq, KT = nq / 32, NT = 512;  // swizzled images (swz8)
  constexpr int NWC = (3 * C + nq) * 8 / NT;  // 16-byte weight chunks per thread
  static_assert((3 * C + nq) * 8 % NT == 0 && KT % 2 == 0, "staging split");
  __shared__ __attribute__((aligned(16))) unsigned char smem[lpb_chain8_smem<NQ>()];
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
  float2* sR = reinterpret_cast<float2*>(smem + lpb_chain_smem<NQ>());              // 2 pair-sum slots
  PIO_WG_BEGIN();
  zero_span_block(job);
  if ((int)blockIdx.x >= (R + 63) / 64) {  // appended workgroups: the previous kernel's slab job
    slab_reduce_block(job, blockIdx.x - (R + 63) / 64, reinterpret_cast<float4*>(smem));
    PIO_WG_END();
    return;
  }
  // the body is instantiated once per channel half (hf = w >> 2, a compile-time constant inside):
  // every channel offset folds into the instructions instead of living in scalar registers
  auto body = [&](auto hfc) {
  constexpr int hf = decltype(hfc)::value;
  const int w = wave_id(), l = lane_id(), g = l >> 4;
  const int lr = 16 * (w & 3) + (l & 15);
  // the tiles of one batch element on one XCD, the same tile → XCD map as the attention backward
  // (xcd_block3) and the layer forward (xcd_remap): the dO / dY rows this kernel stores are read
  // back by the next kernels through the same L2, and so is the dQKV it loads
  const int tile = xcd_remap(blockIdx.x, (R + 63) / 64);
  const int gr = tile * 64 + lr;

  // ---- phase 0: every load in flight; G: this wave's half of the k-steps (t ≡ hf mod 2) ----
  PIO_TS(0);
  bf16x8 wr[NWC];
#pragma unroll
  for (int i = 0; i < NWC; ++i) {
    const int c = threadIdx.x + NT * i, row = c >> 3, col = (c & 7) * 8;
    const uint16_t* src = row < C ? Wo + row * C : row < 2 * C ? W1 + (row - C) * C
                        : row < 3 * C ? W2 + (row - 2 * C) * C : Wq + (row - 3 * C) * C;
    wr[i] = *reinterpret_cast<const bf16x8*>(src + col);
  }
  constexpr bool GBF = sizeof(TG) == 2;
  constexpr int KH = KT / 2;
  float4 gv[GBF ? 1 : KH][2];
  bf16x8 gvb[GBF ? KH : 1];
#pragma unroll
  for (int u = 0; u < KH; ++u) {
    const int t = 2 * u + hf;
    const TG* p = G + (long long)gr * nq + 32 * t + 8 * g;
    if constexpr (GBF) {
      gvb[u] = *reinterpret_cast<const bf16x8*>(p);
    } else {
      gv[u][0] = *reinterpret_cast<const float4*>(p);
      gv[u][1] = *reinterpret_cast<const float4*>(p + 4);
    }
  }
  float xv[2][4], dv[2][4], yv[2][4];
  uint2 ub[2], obv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = 16 * (2 * hf + i) + 4 * g;
    const float4 a = *reinterpret_cast<const float4*>(X + (long long)gr * C + c);
    const float4 d = *reinterpret_cast<const float4*>(dres + (long long)gr * C + c);
    const float4 y = *reinterpret_cast<const float4*>(Ysave + (long long)gr * C + c);
    xv[i][0] = a.x; xv[i][1] = a.y; xv[i][2] = a.z; xv[i][3] = a.w;
    dv[i][0] = d.x; dv[i][1] = d.y; dv[i][2] = d.z; dv[i][3] = d.w;
    yv[i][0] = y.x; yv[i][1] = y.y; yv[i][2] = y.z; yv[i][3] = y.w;
    ub[i] = *reinterpret_cast<const uint2*>(U + (long long)gr * C + c);
    obv[i] = *reinterpret_cast<const uint2*>(O + (long long)gr * C + c);
  }
  const float mu1 = mean1[gr], rs1 = rstd1[gr], mu2 = mean2[gr], rs2 = rstd2[gr];
  // phase D operands (ATT): this wave's K / V fragments (head w & 3, key 32hf + (l & 31)), one
  // 16-byte chunk of the Q and K rows per thread, one LSE value per thread < 256
  bf16x8 akf, avf, aq, ak;
  float alse = 0.f;
  if constexpr (ATT) {
    const long long kr = (long long)(tile * 64 + 32 * hf + (l & 31)) * (3 * C) + (w & 3) * 16 + 8 * (l >> 5);
    akf = *reinterpret_cast<const bf16x8*>(at.qkv + kr + C);
    avf = *reinterpret_cast<const bf16x8*>(at.qkv + kr + 2 * C);
    const long long qr = (long long)(tile * 64 + (threadIdx.x >> 3)) * (3 * C) + (threadIdx.x & 7) * 8;
    aq = *reinterpret_cast<const bf16x8*>(at.qkv + qr);
    ak = *reinterpret_cast<const bf16x8*>(at.qkv + qr + C);
    alse = at.lse[(long long)tile * 256 + (threadIdx.x & 255)];
  }
  PIO_TS(1);
  float pv;
  {
    const int k = threadIdx.x & (C - 1), vi = (threadIdx.x >> 6) & 3;
    pv = (vi == 0 ? lnw : vi == 1 ? lnb : vi == 2 ? g2 : be2)[k];
  }
#pragma unroll
  for (int i = 0; i < NWC; ++i) {
    const int c = threadIdx.x + NT * i, row = c >> 3, col = (c & 7) * 8;
    uint16_t* dst = row < 3 * C ? sWo + swzi(row, LD, col) : sWq + swzi(row - 3 * C, LD, col);
    *reinterpret_cast<bf16x8*>(dst) = wr[i];
  }
  if (threadIdx.x < 4 * C) sVec[threadIdx.x] = pv;
  bf16x8 gb[KT];
#pragma unroll
  for (int u = 0; u < KH; ++u) {
    const int t = 2 * u + hf;
    if constexpr (GBF) {
      gb[t] = gvb[u];
    } else {
      const float4 a = gv[u][0], b = gv[u][1];
      gb[t][0] = (short)f2bf(a.x); gb[t][1] = (short)f2bf(a.y); gb[t][2] = (short)f2bf(a.z); gb[t][3] = (short)f2bf(a.w);
      gb[t][4] = (short)f2bf(b.x); gb[t][5] = (short)f2bf(b.y); gb[t][6] = (short)f2bf(b.z); gb[t][7] = (short)f2bf(b.w);
    }
    *reinterpret_cast<bf16x8*>(sG + swzi(lr, LDG, 32 * t + 8 * g)) = gb[t];
  }
  PIO_TS(2);
  lds_sync();
  PIO_TS(3);
#pragma unroll
  for (int u = 0; u < KH; ++u) {  // the partner's k-steps of G, from the image
    const int t = 2 * u + 1 - hf;
    gb[t] = *reinterpret_cast<const bf16x8*>(sG + swzi(lr, LDG, 32 * t + 8 * g));
  }

  // ---- A: LN1 + QKV backward of layer l+1 → dZ of layer l (this wave's channels) ----
  f32x4 acc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < KT; ++t) acc[i] = mfma16(frag16_tr_sw(sWq, LD, 16 * (2 * hf + i), 32 * t), gb[t], acc[i]);
  }
  PIO_TS(4);
  float dz[2][4], t0[2][4];
  {
    float gg[2][4], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float4 ga = *reinterpret_cast<const float4*>(sVec + 16 * (2 * hf + i) + 4 * g);
      const float gw[4] = {ga.x, ga.y, ga.z, ga.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xv[i][j] = (xv[i][j] - mu1) * rs1;  // x̂
        t0[i][j] = acc[i][j];               // dXn1
        gg[i][j] = acc[i][j] * gw[j];
        s1 += gg[i][j];
        s2 += gg[i][j] * xv[i][j];
      }
    }
    // also the barrier after which no wave reads the Wq image any more (the PA images overlay it)
    cl2_pair_sums(s1, s2, sR, s1, s2);
    s1 *= 1.f / C;
    s2 *= 1.f / C;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) dz[i][j] = rs1 * (gg[i][j] - s1 - xv[i][j] * s2) + dv[i][j];
  }
  cl2_tile_store(sX1, LD, lr, hf, xv);
  cl2_tile_store(sD1, LD, lr, hf, t0);
  PIO_TS(5);

  // ---- B: post-attention backward of layer l ----
  float gp[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float u4[4] = {bf2f((uint16_t)(ub[i].x & 0xFFFF)), bf2f((uint16_t)(ub[i].x >> 16)),
                         bf2f((uint16_t)(ub[i].y & 0xFFFF)), bf2f((uint16_t)(ub[i].y >> 16))};
#pragma unroll
    for (int j = 0; j < 4; ++j) gelu_pair(u4[j], t0[i][j], gp[i][j]);
  }
  cl2_tile_store(sGu, LD, lr, hf, t0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) t0[i][j] = dz[i][j];
  cl2_drop(t0, dr, 1u, gr, hf);  // dZ∘m₁: the MLP output layer's gradient
  cl2_tile_store(sZm, LD, lr, hf, t0);
  {
    bf16x8 bb[2];
    bb[hf] = cl2_frag(t0);
    lds_sync();
    bb[1 - hf] = cl2_img_frag(sZm, LD, lr, 1 - hf);
    cl2_gemm_t(sW2, LD, hf, bb, acc);  // dH
  }
  PIO_TS(6);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) t0[i][j] = acc[i][j] * gp[i][j];  // dU
  cl2_tile_store(sDu, LD, lr, hf, t0);
  {
    bf16x8 bb[2];
    bb[hf] = cl2_frag(t0);
    lds_sync();
    bb[1 - hf] = cl2_img_frag(sDu, LD, lr, 1 - hf);
    cl2_gemm_t(sW1, LD, hf, bb, acc);  // dXn2
  }
  PIO_TS(7);
  {
    float gg[2][4], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float4 ga = *reinterpret_cast<const float4*>(sVec + 2 * C + 16 * (2 * hf + i) + 4 * g);
      const float gw[4] = {ga.x, ga.y, ga.z, ga.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        yv[i][j] = (yv[i][j] - mu2) * rs2;  // ŷ
        t0[i][j] = acc[i][j];               // dXn2
        gg[i][j] = acc[i][j] * gw[j];
        s1 += gg[i][j];
        s2 += gg[i][j] * yv[i][j];
      }
    }
    cl2_pair_sums(s1, s2, sR + 8 * 16, s1, s2);
    s1 *= 1.f / C;
    s2 *= 1.f / C;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) dz[i][j] += rs2 * (gg[i][j] - s1 - yv[i][j] * s2);  // dY
  }
  cl2_tile_store(sYh, LD, lr, hf, yv);
  cl2_tile_store(sD2, LD, lr, hf, t0);
  cl2_store_f32(dY, C, gr, hf, dz);
  cl2_drop(dz, dr, 0u, gr, hf);  // dY∘m₀: the out-projection's gradient
  cl2_tile_store(sYm, LD, lr, hf, dz);
  {
    bf16x8 bb[2];
    bb[hf] = cl2_frag(dz);
    lds_sync();
    bb[1 - hf] = cl2_img_frag(sYm, LD, lr, 1 - hf);
    cl2_gemm_t(sWo, LD, hf, bb, acc);  // dO
  }
  PIO_TS(8);
  float dd[2];
  {
    float ov[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ov[i][0] = bf2f((uint16_t)(obv[i].x & 0xFFFF)); ov[i][1] = bf2f((uint16_t)(obv[i].x >> 16));
      ov[i][2] = bf2f((uint16_t)(obv[i].y & 0xFFFF)); ov[i][3] = bf2f((uint16_t)(obv[i].y >> 16));
      float sacc = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t0[i][j] = bf2f(f2bf(acc[i][j]));  // dO as the attention backward sees it
        sacc += t0[i][j] * ov[i][j];
      }
      dd[i] = xor32_sum(xor16_sum(sacc));  // head 2hf + i = channels 16(2hf + i) .. + 15
    }
    if constexpr (!ATT) {  // ATT: phase D consumes dO / δ from these registers
      cl2_store_bf16(dO, C, gr, hf, t0);
      if (g == 0) *reinterpret_cast<float2*>(delta + (long long)gr * 4 + 2 * hf) = make_float2(dd[0], dd[1]);
    }
    cl2_tile_store(sOt, LD, lr, hf, ov);
  }
  PIO_TS(9);
  lds_sync();
  PIO_TS(10);

  // ---- C: parameter gradients of the tile → its slab row, 16-row blocks over 8 waves ----
  const int vrs = gr_out.vrs;
  const long long so = (long long)tile * vrs;
  const float *gam1 = sVec, *bet1 = sVec + C, *gam2 = sVec + 2 * C, *bet2 = sVec + 3 * C;
  const int p4 = w & 3;
  auto sp = [&](float* p) { return p + so; };  // this tile's slab row
  if constexpr (hf == 0) {
    cl_wgrad_block(sZm, LD, p4, sGu, LD, nullptr, nullptr, sp(gr_out.dW2), sp(gr_out.db2));
    cl_wgrad_block(sYm, LD, p4, sOt, LD, nullptr, nullptr, sp(gr_out.dWo), sp(gr_out.dbo));
    cl_wgrad_block(sG, LDG, p4, sX1, LD, gam1, bet1, sp(dWq), sp(dbq));  // dWq rows 16p4 ..
    cl_ln_grads(sD2, sYh, LD, p4, sp(gr_out.dg2), sp(gr_out.dbe2));
  } else {
    cl_wgrad_block(sDu, LD, p4, sYh, LD, gam2, bet2, sp(gr_out.dW1), sp(gr_out.db1));
#pragma unroll
    for (int q = 1; q < NQ; ++q)  // dWq 16-row blocks p4 + 4q
      cl_wgrad_block(sG, LDG, p4 + 4 * q, sX1, LD, gam1, bet1, sp(dWq), sp(dbq));
    cl_ln_grads(sD1, sX1, LD, p4, sp(dlnw), sp(dlnb));
  }
  PIO_TS(11);
  if constexpr (ATT) {
    // ---- D: attention backward of layer l (N = 64: the tile is the sample) ----
    constexpr int LDA = 40, LDS_ = 40;  // [row][d] tiles, d 16..31 zero; dS slabs [key][q]
    uint16_t* sm16 = reinterpret_cast<uint16_t*>(smem);
    uint16_t* sQa = sm16;                      // [4][64][LDA]  Q
    uint16_t* sdOa = sQa + 4 * 64 * LDA;       // [4][64][LDA]  dO
    uint16_t* sKa = sdOa + 4 * 64 * LDA;       // [4][64][LDA]  K
    uint16_t* sdSa = sKa + 4 * 64 * LDA;       // [4 heads][2 query tiles][64 keys][LDS_]
    float* sLa = reinterpret_cast<float*>(sdSa + 4 * 2 * 64 * LDS_);  // [4][64] LSE
    float* sDa = sLa + 4 * 64;                 // [4][64] δ
    uint16_t* sOut = sm16;                     // [64][3C] dQKV tile (over Q / dO, after they are consumed)
    static_assert((4 * 3 * 64 * LDA + 4 * 2 * 64 * LDS_) * 2 + 2 * 4 * 64 * 4 <= lpb_chain8_smem<NQ>(), "phase D LDS");
    static_assert(64 * 3 * C * 2 <= 2 * 4 * 64 * LDA * 2, "dQKV tile over the Q / dO tiles");
    lds_sync();  // phase C's reads of the images are done
    {
      const int row = threadIdx.x >> 3, cc = (threadIdx.x & 7) * 8, hq = cc >> 4, d0 = cc & 15;
      *reinterpret_cast<bf16x8*>(sQa + (hq * 64 + row) * LDA + d0) = aq;
      *reinterpret_cast<bf16x8*>(sKa + (hq * 64 + row) * LDA + d0) = ak;
      if (threadIdx.x < 256) {
        const int zh = threadIdx.x >> 6, zr = threadIdx.x & 63;
        const bf16x8 z8 = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        *reinterpret_cast<bf16x8*>(sQa + (zh * 64 + zr) * LDA + 16) = z8;
        *reinterpret_cast<bf16x8*>(sQa + (zh * 64 + zr) * LDA + 24) = z8;
        *reinterpret_cast<bf16x8*>(sdOa + (zh * 64 + zr) * LDA + 16) = z8;
        *reinterpret_cast<bf16x8*>(sdOa + (zh * 64 + zr) * LDA + 24) = z8;
        sLa[(threadIdx.x & 3) * 64 + (threadIdx.x >> 2)] = alse;
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {  // dO of row lr, head 2hf + i, dims 4g .. 4g + 3
        uint2 pk;
        pk.x = pack2(t0[i][0], t0[i][1]);
        pk.y = pack2(t0[i][2], t0[i][3]);
        *reinterpret_cast<uint2*>(sdOa + ((2 * hf + i) * 64 + lr) * LDA + 4 * g) = pk;
        if (g == 0) sDa[(2 * hf + i) * 64 + lr] = dd[i];
      }
    }
    lds_sync();
    const int ah = w & 3, hh = l >> 5, r = l & 31;
    const int b = tile;  // the sample (N = 64 rows)
    const uint16_t* tQh = sQa + ah * 64 * LDA;
    const uint16_t* tdOh = sdOa + ah * 64 * LDA;
    const uint32_t dkey = dr.thresh ? drop_key(dr.seed, dr.site, 2u) : 0u;
    const int key = 32 * hf + r;  // this lane's key (S / dP column)
    f32x16 dKa = f32x16{}, dVa = f32x16{};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint16_t* tQ = tQh + 32 * j * LDA;
      const uint16_t* tdO = tdOh + 32 * j * LDA;
      const f32x16 S = mfma32(frag_kc(tQ, LDA, 0, 0), akf, f32x16{});
      const f32x16 dP = mfma32(frag_kc(tdO, LDA, 0, 0), avf, f32x16{});
      f32x4 lrow[4], drow[4];
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        lrow[gg] = *reinterpret_cast<const f32x4*>(sLa + ah * 64 + 32 * j + 8 * gg + 4 * hh);
        drow[gg] = *reinterpret_cast<const f32x4*>(sDa + ah * 64 + 32 * j + 8 * gg + 4 * hh);
      }
      f32x16 P, dS;
      if (!dr.thresh) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fast_exp2(S[i] * at.scale_log2 - lrow[i >> 2][i & 3]);
          P[i] = p;
          dS[i] = p * (dP[i] - drow[i >> 2][i & 3]);
        }
      } else {
        // element index (32j + 4hh)·64 + key + acc_row(i, 0)·64 (keep_elem_m)
        uint32_t cm0 = ((uint32_t)(32 * j + 4 * hh) * 64u + (uint32_t)key) * kHashM1;
        asm volatile("" : "+v"(cm0));
        const uint32_t hs = hash3_seed(dkey, (uint32_t)(b * 4 + ah));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fast_exp2(S[i] * at.scale_log2 - lrow[i >> 2][i & 3]);
          const bool keep = keep_elem_m(hs, cm0 + (uint32_t)acc_row(i, 0) * 64u * kHashM1, dr.thresh);
          P[i] = keep ? p * dr.scale : 0.f;
          dS[i] = p * ((keep ? dP[i] * dr.scale : 0.f) - drow[i >> 2][i & 3]);
        }
      }
      bf16x8 sa[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        sa[ss] = pack_acc(dS, ss);
        dVa = mfma32(pack_acc(P, ss), frag_ks_perm(tdO, LDA, 0, 16 * ss), dVa);
        dKa = mfma32(sa[ss], frag_ks_perm(tQ, LDA, 0, 16 * ss), dKa);
      }
      uint16_t* slab = sdSa + ((ah * 2 + j) * 64 + 32 * hf) * LDS_;
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const bf16x8& v = sa[gg >> 1];
        const int o = 4 * (gg & 1);
        const bf16x4 q4 = {v[o], v[o + 1], v[o + 2], v[o + 3]};
        *reinterpret_cast<bf16x4*>(slab + r * LDS_ + 8 * gg + 4 * hh) = q4;
      }
    }
    lds_sync();  // both key halves' dS slabs are in; Q / dO are consumed (sOut may overwrite them)
    // dK (scaled) / dV rows: key 32hf + acc_row(i, hh), dim r (< 16)
    if (r < 16) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kk = 32 * hf + acc_row(i, hh);
        sOut[kk * (3 * C) + C + ah * 16 + r] = f2bf(dKa[i] * at.scale);
        sOut[kk * (3 * C) + 2 * C + ah * 16 + r] = f2bf(dVa[i]);
      }
    }
    {  // dQ of query tile hf (both 16-row halves): Σ over the 64 keys of dS[key][q]·K[key][d]
      const uint16_t* tS = sdSa + (ah * 2 + hf) * 64 * LDS_;
      const uint16_t* tK = sKa + ah * 64 * LDA;
      const int gq = l >> 4;
#pragma unroll
      for (int mh = 0; mh < 2; ++mh) {
        f32x4 a0 = mfma16(frag16_tr(tS, LDS_, 16 * mh, 0), frag16_tr(tK, LDA, 0, 0), f32x4{0.f, 0.f, 0.f, 0.f});
        f32x4 a1 = mfma16(frag16_tr(tS, LDS_, 16 * mh, 32), frag16_tr(tK, LDA, 0, 32), f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qq = 32 * hf + 16 * mh + 4 * gq + i;
          sOut[qq * (3 * C) + ah * 16 + (l & 15)] = f2bf((a0[i] + a1[i]) * at.scale);
        }
      }
    }
    lds_sync();
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // the dQKV tile: 64 rows × 24 16-byte chunks
      const int c = threadIdx.x + NT * k, row = c / 24, col = (c % 24) * 8;
      *reinterpret_cast<bf16x8*>(at.dqkv + (long long)(tile * 64 + row) * (3 * C) + col) =
          *reinterpret_cast<const bf16x8*>(sOut + row * (3 * C) + col);
    }
  }
  };
  if (wave_id() >> 2) body(std::integral_constant<int, 1>{});
  else body(std::integral_constant<int, 0>{});
  PIO_WG_END();
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
  if (N > 512) return false;
  dim3 grid(R / 64);
#define SAC(NX, NQ, KT)                                                                                                  \
  if (dr.thresh)                                                                                                         \
    hipLaunchKernelGGL((sa_layer_fwd_chain8_kernel<NX, NQ, KT, true>), grid, dim3(512), 0, st, QKV, N, scale_log2, O, LSE, \
                       X, Wo, bo, g2, be2, eps, W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, lnw, lnb, Wq, bq, QKVn,  \
                       mean1, rstd1, dr);                                                                                \
  else                                                                                                                   \
    hipLaunchKernelGGL((sa_layer_fwd_chain8_kernel<NX, NQ, KT, false>), grid, dim3(512), 0, st, QKV, N, scale_log2, O,    \
                       LSE, X, Wo, bo, g2, be2, eps, W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, lnw, lnb, Wq, bq,  \
                       QKVn, mean1, rstd1, dr)
#define SAK(KT)              \
  if (!next) {               \
    SAC(false, 3, KT);       \
  } else if (nq == 64) {     \
    SAC(true, 1, KT);        \
  } else if (nq == 128) {    \
    SAC(true, 2, KT);        \
  } else {                   \
    SAC(true, 3, KT);        \
  }
  if (N <= 256) {
    SAK(8)
  } else {
    SAK(16)
  }
#undef SAK
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
                                          int nq, const uint16_t* att_qkv, const float* att_lse, uint16_t* att_out,
                                          float att_scale, hipStream_t st) {
  if (nq != 192 && nq != 64) return false;
  // phase D (att): layer l is a self-attention layer in both forms — NQ = 3 (layer l+1 a
  // self-attention layer too) and NQ = 1 (layer l+1 the next cross-attention layer's query path)
  const bool att = att_out != nullptr;
  dim3 grid((R + 63) / 64 + (job.slab ? job.nblk : 0));
  const ChainAttn at{att_qkv, att_lse, att_out, att_scale, att_scale * 1.4426950408889634f};
#define LPC(NQ, TG, A)                                                                                                   \
  hipLaunchKernelGGL((ln_linear_post_attn_bwd_chain8_kernel<NQ, TG, A>), grid, dim3(512), 0, st, static_cast<const TG*>(G), \
                     Wq, X, mean1, rstd1, lnw, lnb, dres, dlnw, dlnb, dWq, dbq, Ysave, mean2, rstd2, U, O, Wo, W1, W2,       \
                     g2, be2, dY, dO, delta, grads, R, job, dr, at)
  if (g_bf16) {
    if (nq != 192) return false;  // bf16 G only from the self-attention backward (nq = 3C)
    if (att) LPC(3, uint16_t, true);
    else LPC(3, uint16_t, false);
  } else if (nq == 192) {
    if (att) LPC(3, float, true);
    else LPC(3, float, false);
  } else if (att) {
    LPC(1, float, true);
  } else {
    LPC(1, float, false);
  }
#undef LPC
  return true;
}

}  // namespace pio
