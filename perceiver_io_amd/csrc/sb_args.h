// Argument blocks of the per-sample latent-block kernels (sample_block.hip), shared by the kernel
// translation unit and the host binding (binding.cpp).  Plain C++ (stdint only).
#pragma once
#include <stdint.h>

namespace pio {

constexpr int kSBMaxLayers = 4;  // self-attention layers per block (the image configs run 3)

// one self-attention layer (reference model.py:36-44: x → LN1 → MHA → +x → LN2 → MLP → +) of a
// C ∈ {64, 128}, H = 4 block over N = 32 latents: weights, then the forward's saved rows (every one
// an operand of the backward or of the weight-gradient GEMMs)
struct SBLayer {
  const uint16_t *Wqkv, *Wo, *W1, *W2;         // bf16 [3C][C], [C][C] ×3 (nn.Linear layout)
  const float *bqkv, *g1, *be1, *bo, *g2, *be2, *b1, *b2;
  uint16_t *LN1X, *QKV, *O, *LN2Y, *U, *GU;    // bf16 rows: LN1(x), packed QKV, attention out, LN2(y), W1 out, GELU
  float *Y, *Z, *mean1, *rstd1, *mean2, *rstd2;  // fp32: residual after attention, layer output, LN stats
};
// post (has_post): the LayerNorm + query projection of the cross-attention layer after the block
// (its query path, model.py:48-74 q = LN_q(z)·Wqᵀ + bq over the block output z).  Forward epilogue:
// Q (bf16 rows), the LN statistics and LN_q(z) (bf16 rows, the dWq operand).  Backward prologue:
// the block's output gradient is dres + LN_q backward of dQ·Wq (dQ fp32 rows in), with the dQ rows
// (bf16, the dWq operand) and the LN_q affine partials (slab) out.
struct SBQPath {
  int N;               // outputs: C (a query projection) or 2C (a decoder's packed K | V projection)
  const uint16_t* Wq;  // bf16 [N][C]
  const float *bq, *g, *b;
  uint16_t *Q, *LNX;   // forward: bf16 rows out
  float *mean, *rstd;  // forward: LN statistics out (backward: in)
  const float* dQ;     // backward: fp32 rows in
  const float* dres;   // backward: the other gradient of z (fp32 rows in; nullptr: none)
  uint16_t* dQb;       // backward: bf16 rows out
  float *dg, *db;      // backward: LN_q affine partials (slab row base)
};
// pre (has_pre): the post-attention half of the cross-attention layer in front of the block
// (model.py:36-44 applied to the cross layer's attention output): z0 = y + MLP(LN2(y)),
// y = Wo·O + bo + x_q.  Its Wo / W1 / W2 / bo / γ2 / β2 / b1 / b2 and saved LN2Y / U / GU / Y /
// mean2 / rstd2 are those of an SBLayer; its Z is the block input (X0, written by the forward).
struct SBFwdArgs {
  SBLayer ly[kSBMaxLayers];
  SBLayer pre;
  const float* X0;        // block input rows (B·32, C) fp32 (pre: written, = pre.Z)
  const uint16_t* preO;   // pre: the cross attention's output rows (B·32, C) bf16
  const float* preX;      // pre: the residual rows x_q, (B·32, C) or (32, C) broadcast
  int preX_bs;            // pre: rows between two samples' residual rows (32, or 0: broadcast)
  int has_pre;
  SBQPath post;
  int has_post;
  int L, B;
  float scale_log2, eps;
};
// backward: the gradient rows the weight-gradient GEMMs need (bf16) and the sample's LayerNorm
// affine gradient partials (fp32 slab rows: row b = sample b, stride ln_rs floats in SBBwdArgs;
// every element stored once, summed over the samples by a slab reduction — per-sample atomics
// on the same 4·C addresses serialise at the L2)
struct SBGrad {
  uint16_t *dQKV, *dY, *dU, *dZ;
  float *dg1, *dbe1, *dg2, *dbe2;
};
// pre (has_pre): the cross layer's post-attention backward after the block's: dX is then the
// gradient of x_q's residual path (= dY of the pre stage); preDO / preDelta receive the cross
// attention's dO (bf16) and δ = per-head rowsum(dO∘O) (fp32 (B·32, 4)); pgr its gradient rows and
// LayerNorm partials (dg2 / dbe2 only).  zero_p / zero_n4: an fp32 buffer cleared on the way (the
// cross attention backward's atomic accumulators), one slice per workgroup.
struct SBBwdArgs {
  SBLayer ly[kSBMaxLayers];
  SBGrad gr[kSBMaxLayers];
  SBLayer pre;
  SBGrad pgr;
  const float* X0;   // the block input (layer 0's LN1 input)
  const float* dZ;   // gradient of the block output (B·32, C) fp32
  float* dX;         // gradient of the block input (B·32, C) fp32 (written)
  uint16_t* preDO;
  float* preDelta;
  float* zero_p;
  long long zero_n4;
  int has_pre;
  SBQPath post;        // has_post: dZ is then unused (dres + the query path's LN backward)
  int has_post;
  int L, B;
  int ln_rs;         // row stride of the LayerNorm partial slab (floats)
  float scale_log2, eps;
};
// grouped weight-gradient GEMMs: dW[n][k] += Σ_rows G[r][n] · A[r][k], db[n] += Σ_rows G[r][n]
// (A is C wide: every self-attention weight's input); one job per weight
constexpr int kSBMaxJobs = 4 * kSBMaxLayers + 3;  // + the pre stage's Wo, W1, W2
struct SBWgradJob {
  const uint16_t* G;  // bf16 [R][N]
  const uint16_t* A;  // bf16 [R][C]
  float* dW;          // fp32 [N][C] (added to)
  float* db;          // fp32 [N] (added to)
  int N;              // C or 3C (a multiple of 64)
  int tile0;          // first 64-column tile index of this job in the grid
};
struct SBWgradArgs {
  SBWgradJob job[kSBMaxJobs];
  int njobs, R, rows_per_split;
};

}  // namespace pio
