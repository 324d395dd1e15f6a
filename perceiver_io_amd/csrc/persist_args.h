// Argument blocks of the persistent self-attention block kernels (persist.hip), shared by the
// kernel translation unit and the host binding (binding.cpp) so the two cannot drift.  Include
// after DropCfg / PostAttnGrads / SlabJob are declared (common.h on the device side, the mirrors
// at the top of binding.cpp on the host side).
#pragma once
#include <stdint.h>

namespace pio {

constexpr int kPersistMaxLayers = 8;

// ---- forward: one launch runs every layer of a C = 64, H = 4 latent self-attention block ----
// Layer i reads its packed QKV (layer 0: qkv0, produced before the launch; layer i > 0: the
// previous layer's QKVn, produced inside the launch) and writes the tensors the backward saves.
struct SAFwdLayer {
  const uint16_t *Wo, *W1, *W2;
  const uint16_t* Wq;                     // the next LN1 + projection (nullptr: none)
  const float *bo, *g2, *be2, *b1, *b2;
  const float *lnw, *lnb, *bq;            // the next LN1 affine and projection bias
  uint16_t *O, *U, *QKVn;                 // attention output, MLP pre-activation, next projection
  float *LSE, *Z, *Y, *mean2, *rstd2, *mean1n, *rstd1n;
  int nq;                                 // rows of Wq: 0, 64 / 128 (a query / K-V projection), 192 (QKV)
  int pad_;
};
struct SABlockFwdArgs {
  SAFwdLayer ly[kPersistMaxLayers];
  const uint16_t* QKV0;                   // layer 0's packed QKV (R, 3C) bf16
  const float* X0;                        // the block input rows (R, C) fp32
  unsigned* sync;                         // [0] tile ticket, [1] finished workgroups, [4 + b] per-sample
                                          // counters: zero at launch, reset by the last workgroup
  int L, N, R, pad_;
  float scale_log2, eps;
  DropCfg dr;                             // residual dropout; site = layer index
};

}  // namespace pio
