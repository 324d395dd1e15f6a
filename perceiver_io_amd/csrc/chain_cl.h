// Chain-layout (CL / CL2) register-row helpers shared by the per-layer chain kernels
// (chain.hip) and the persistent self-attention block kernels (persist.hip).
#pragma once
#include <type_traits>

#include "common.h"

namespace pio {

// ------------------------------------------------------------------------------------
// Chain layout (CL): register-resident row chains with v_mfma_f32_16x16x32_bf16.
// A row lives on lane (l & 15) of a wave; lane group g = l >> 4 holds channels
// 16·mt + 4g + i (i < 4) of every 16-channel block (m-tile) mt — exactly the accumulator layout
// of a TRANSPOSED product Yᵀ = W·Xᵀ (col = lane & 15 = row, acc row = 4g + i = channel).  Such
// an accumulator feeds the next transposed product as its B operand with no lane movement: the
// k order of step t is permuted to channel 32t + 16(j >> 2) + 4g + (j & 3) for element j, and
// the weight (A operand) is staged into LDS with its columns permuted the same way, so every A
// fragment is one ds_read_b128.  A row's reductions (LayerNorm, per-head sums) are local values
// + two lane swaps (l ^ 16, l ^ 32).  So a whole post-attention block — out-projection,
// residual, LN2, W1, GELU, W2, residual, LN1 + the next projection — runs from registers with no
// LDS round trip of an activation except the pair hand-offs of CL2 below.
// ------------------------------------------------------------------------------------
// A fragment (m-tile mt, k-step t) of a weight image in LDS ([rows][ld], permuted or natural)
__device__ __forceinline__ bf16x8 cl_afrag(const uint16_t* sW, int ld, int mt, int t) {
  const int l = lane_id();
  return *reinterpret_cast<const bf16x8*>(sW + (16 * mt + (l & 15)) * ld + 32 * t + 8 * (l >> 4));
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

// frag_ks_perm (common.h) whose A rows 16..31 read a ones image instead (sOnes: 16 × 16 bf16 1.0):
// the lanes that supply those rows address the ones block, so no select follows the read
__device__ __forceinline__ bf16x8 frag_ks_perm_ones(const uint16_t* lds, int ld, int i0, int k0, const uint16_t* sOnes) {
  const int l = lane_id();
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const uint16_t* base = (g & 1) ? sOnes + (4 * (g >> 1) + q) * 16 + 4 * p
                                 : lds + (k0 + 4 * (g >> 1) + q) * ld + i0 + 4 * p;
  const int hs = (g & 1) ? 8 * 16 : 8 * ld;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + hs));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// ------------------------------------------------------------------------------------
// Paired chain layout (CL2): 8 waves per 64-row tile, two waves per 16-row chain.  Wave w owns
// rows 16·(w & 3) + (l & 15) and the channel half hf = w >> 2, i.e. m-tiles 2hf, 2hf + 1 of the
// CL layout (channels 32hf + 16i + 4g + j).  Every product Yᵀ = W·Xᵀ over K = 64 splits over the
// pair by OUTPUT channels: a wave computes its two m-tiles over both k-steps.  The B fragment of
// k-step t is built from m-tiles 2t, 2t + 1, i.e. exactly the activations wave hf = t holds, so
// each wave packs its own fragment and takes its partner's (w ^ 4) through a 1 KB LDS slot —
// one barrier per product.  Row reductions (LayerNorm) combine the pair's two 32-channel
// partial (mean, M2) by Chan's formula through an 8-byte-per-row slot: one barrier per LN.
// Half the MFMA / VALU work per wave, and two waves per SIMD to hide each other's latency.
// ------------------------------------------------------------------------------------
// own k-step fragment (local m-tiles 0, 1 = global 2hf, 2hf + 1), CL k order
__device__ __forceinline__ bf16x8 cl2_frag(const float (&v)[2][4]) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(v[j >> 2][j & 3]);
  return r;
}
// pair exchange of a bf16x8 fragment through slot sx (8 waves × 64 lanes × 16 B): b[hf] = own,
// b[1 - hf] = the partner's
__device__ __forceinline__ void cl2_swap_frag(bf16x8* sx, const bf16x8& own, int hf, bf16x8 (&b)[2]) {
  const int w = wave_id(), l = lane_id();
  sx[w * 64 + l] = own;
  lds_sync();
  const bf16x8 o = sx[(w ^ 4) * 64 + l];
  b[0] = hf ? o : own;
  b[1] = hf ? own : o;
}
// Yᵀ (this wave's two m-tiles) = W·Xᵀ over K = 64 (two k-steps)
__device__ __forceinline__ void cl2_gemm(const uint16_t* sW, int ld, int hf, const bf16x8 (&b)[2], f32x4 (&acc)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[i] = mfma16(cl_afrag(sW, ld, 2 * hf + i, t), b[t], acc[i]);
  }
}
// LayerNorm over the pair's 64 channels (in place on this wave's 32); sr: 8 waves × 16 rows float2
__device__ __forceinline__ void cl2_layernorm(float (&v)[2][4], float2* sr, int hf, const float* sg, const float* sb,
                                              float eps, float& mean, float& rstd) {
  const int w = wave_id(), l = lane_id(), g = l >> 4;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[i][j];
  const float ma = xor32_sum(xor16_sum(s)) * (1.f / 32.f);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { const float d = v[i][j] - ma; q = fmaf(d, d, q); }
  const float m2a = xor32_sum(xor16_sum(q));
  if (g == 0) sr[w * 16 + (l & 15)] = make_float2(ma, m2a);
  lds_sync();
  const float2 o = sr[(w ^ 4) * 16 + (l & 15)];
  const float dm = ma - o.x;
  mean = 0.5f * (ma + o.x);
  rstd = rsqrtf((m2a + o.y + 16.f * dm * dm) * (1.f / 64.f) + eps);  // Chan: M2 = M2a + M2b + δ²·32·32/64
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = 16 * (2 * hf + i) + 4 * g;
    const float4 gg = *reinterpret_cast<const float4*>(sg + c);
    const float4 bb = *reinterpret_cast<const float4*>(sb + c);
    v[i][0] = (v[i][0] - mean) * rstd * gg.x + bb.x;
    v[i][1] = (v[i][1] - mean) * rstd * gg.y + bb.y;
    v[i][2] = (v[i][2] - mean) * rstd * gg.z + bb.z;
    v[i][3] = (v[i][3] - mean) * rstd * gg.w + bb.w;
  }
}
// acc + bias (own channels)
__device__ __forceinline__ void cl2_bias(float (&v)[2][4], const f32x4 (&acc)[2], const float* sb, int hf) {
  const int g = lane_id() >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float4 bb = *reinterpret_cast<const float4*>(sb + 16 * (2 * hf + i) + 4 * g);
    v[i][0] = acc[i][0] + bb.x; v[i][1] = acc[i][1] + bb.y; v[i][2] = acc[i][2] + bb.z; v[i][3] = acc[i][3] + bb.w;
  }
}
__device__ __forceinline__ void cl2_drop(float (&v)[2][4], const DropCfg& d, uint32_t sub, int gr, int hf) {
  if (d.thresh == 0u) return;
  const uint32_t key = drop_key(d.seed, d.site, sub);
  const int g = lane_id() >> 4;
  // element index gr·64 + 32hf + 4g + (16i + j): base product once (keep_elem_m)
  uint32_t cm0 = ((uint32_t)gr * 64u + (uint32_t)(32 * hf + 4 * g)) * kHashM1;
  asm volatile("" : "+v"(cm0));
  const uint32_t hs = hash3_seed(key, 0u);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      v[i][j] = keep_elem_m(hs, cm0 + (uint32_t)(16 * i + j) * kHashM1, d.thresh) ? v[i][j] * d.scale : 0.f;
}
__device__ __forceinline__ void cl2_store_f32(float* __restrict__ Y, int ld, int gr, int hf, const float (&v)[2][4]) {
  const int g = lane_id() >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
    *reinterpret_cast<float4*>(Y + (long long)gr * ld + 16 * (2 * hf + i) + 4 * g) =
        make_float4(v[i][0], v[i][1], v[i][2], v[i][3]);
}
__device__ __forceinline__ void cl2_store_bf16(uint16_t* __restrict__ Y, int ld, int gr, int hf, const float (&v)[2][4]) {
  const int g = lane_id() >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint2 pk;
    pk.x = pack2(v[i][0], v[i][1]);
    pk.y = pack2(v[i][2], v[i][3]);
    *reinterpret_cast<uint2*>(Y + (long long)gr * ld + 16 * (2 * hf + i) + 4 * g) = pk;
  }
}

// The boundary kernel's LDS images are unpadded ([rows][64·k] bf16, 128-byte multiples) with
// the column bits 3..5 of row r XOR-ed with 8·ψ(r), ψ(r) = r₃ | r₁·2 | (r₂ ⊕ r₃)·4 (rₖ = bit k
// of r).  Every access of the kernel — 16-byte row chunks (weights, G), 8-byte row pieces
// (cl2_tile_store / cl2_img_frag) and the transposed ds_read_b64_tr_b16 fragments (frag16_tr_sw,
// frag16_tr_cl: 8 rows × 32 bytes per 32 lanes) — then touches 64 distinct banks per lane group
// (a padded 72-column layout conflicts 2-way on the transposed reads).
__device__ __forceinline__ int swz8(int r) {
  return 8 * (((r >> 3) & 1) | (((r >> 1) & 1) << 1) | ((((r >> 2) ^ (r >> 3)) & 1) << 2));
}
// element (r, c) of a swizzled image; c may be any column of a 4-aligned (8-byte) piece
__device__ __forceinline__ int swzi(int r, int ld, int c) { return r * ld + (c ^ swz8(r)); }
// frag16_tr (common.h) on a swizzled image
__device__ __forceinline__ bf16x8 frag16_tr_sw(const uint16_t* lds, int ld, int i0, int k0) {
  const int l = lane_id(), g = l >> 4, i = l & 15;
  const int r = k0 + 8 * g + (i >> 2), c = i0 + 4 * (i & 3);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds + swzi(r, ld, c)));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds + swzi(r + 4, ld, c)));
  bf16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return v;
}
// the same in the CL k order of k-step t (element j ↔ k = 32t + 16(j >> 2) + 4g + (j & 3)), swizzled
__device__ __forceinline__ bf16x8 frag16_tr_cl(const uint16_t* lds, int ld, int i0, int t) {
  const int l = lane_id(), g = l >> 4, i = l & 15;
  const int rr = 32 * t + 4 * g + (i >> 2), c = i0 + 4 * (i & 3);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds + swzi(rr, ld, c)));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds + swzi(rr + 16, ld, c)));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
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
    const bf16x8 a = frag16_tr_sw(sA, lda, 16 * mt, 32 * t);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma16(a, frag16_tr_sw(sB, ldb, 16 * nt, 32 * t), acc[nt]);
    acc[4] = mfma16(a, ones_frag(), acc[4]);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int n = 16 * nt + c;
    const float gn = gam ? gam[n] : 1.f, bn = bet ? bet[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) dW[(16 * mt + 4 * g + i) * 64 + n] = acc[nt][i] * gn + acc[4][i] * bn;
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
    const bf16x8 a = frag16_tr_sw(sD, ld, 16 * mt, 32 * t);
    dia = mfma16(a, frag16_tr_sw(sXh, ld, 16 * mt, 32 * t), dia);
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
  // (swizzled, unpadded rows: swz8 / swzi)
  return 2 * (3 * 64 * 64) + 2 * (64 * (NQ * 64) + 2 * 64 * 64) +
         2 * (NQ * 64 * 64 > 7 * 64 * 64 ? NQ * 64 * 64 : 7 * 64 * 64) + 4 * 4 * 64;
}

// ------------------------------------------------------------------------------------
// The layer-boundary backward on 8 waves (same operands and results as
// ln_linear_post_attn_bwd_chain_kernel), paired chain layout CL2: wave w owns rows
// 16(w & 3) + (l & 15), channel half hf = w >> 2.  The transposed products dXᵀ = Wᵀ·dYᵀ split
// over the pair by output channels; each wave's k-step fragment of dY comes from its own
// registers, the partner's from the bf16 row-major image of dY that phase C needs anyway
// (written by the partner, one barrier).  LayerNorm backward sums: one float2 exchange each.
// Phase C splits the parameter-gradient blocks over all 8 waves.
// ------------------------------------------------------------------------------------
// CL k-order fragment of k-step t of row lr from a row-major bf16 image [64][ld]
__device__ __forceinline__ bf16x8 cl2_img_frag(const uint16_t* sT, int ld, int lr, int t) {
  const int g = lane_id() >> 4;
  const bf16x4 lo = *reinterpret_cast<const bf16x4*>(sT + swzi(lr, ld, 32 * t + 4 * g));
  const bf16x4 hi = *reinterpret_cast<const bf16x4*>(sT + swzi(lr, ld, 32 * t + 16 + 4 * g));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// this wave's channels of its rows → a row-major bf16 image
__device__ __forceinline__ void cl2_tile_store(uint16_t* sT, int ld, int lr, int hf, const float (&v)[2][4]) {
  const int g = lane_id() >> 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint2 pk;
    pk.x = pack2(v[i][0], v[i][1]);
    pk.y = pack2(v[i][2], v[i][3]);
    *reinterpret_cast<uint2*>(sT + swzi(lr, ld, 16 * (2 * hf + i) + 4 * g)) = pk;
  }
}
// dXᵀ (this wave's two m-tiles of the 64 input channels) = Wᵀ·dYᵀ over 2 k-steps
__device__ __forceinline__ void cl2_gemm_t(const uint16_t* sW, int ld, int hf, const bf16x8 (&b)[2], f32x4 (&acc)[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[i] = mfma16(frag16_tr_cl(sW, ld, 16 * (2 * hf + i), t), b[t], acc[i]);
  }
}
// pair totals of two per-row partial sums (each over this wave's 32 channels)
__device__ __forceinline__ void cl2_pair_sums(float a, float b, float2* sr, float& ta, float& tb) {
  const int w = wave_id(), l = lane_id();
  a = xor32_sum(xor16_sum(a));
  b = xor32_sum(xor16_sum(b));
  if ((l >> 4) == 0) sr[w * 16 + (l & 15)] = make_float2(a, b);
  lds_sync();
  const float2 o = sr[(w ^ 4) * 16 + (l & 15)];
  ta = a + o.x;
  tb = b + o.y;
}

template <int NQ>
constexpr int lpb_chain8_smem() { return lpb_chain_smem<NQ>() + 2 * 8 * 16 * 8; }

}  // namespace pio
