// Kernel argument structs of attention_pe.hip, shared verbatim by the HIP translation unit and
// the host binding (binding.cpp, compiled by g++): one definition, no hand-kept mirror.
#pragma once
#include <stdint.h>

namespace pio {

struct PeBwdArgs {
  const uint16_t* q; long long q_bs; int q_rs;  // (1 | B, Nq, ≥ C) bf16; head h = cols [32h, 32h + 32)
  const uint16_t* kv; int kv_rs;                 // (B·M, ≥ 2C) bf16: K = cols [0, C), V = [C, 2C)
  const uint16_t* dO;                            // (B, Nq, C) bf16 contiguous
  const float* lse;                              // (B, Nq, H), log2 units
  const float* delta;                            // (B, Nq, H) = rowsum(dO∘O)
  const float* mean; const float* rstd;          // (B·M) LayerNorm row statistics of the K/V input (not IMPL)
  // implicit K/V (IMPL): generated per batch element from P' (M, 2C) bf16, the PE row sums and the
  // generation table (see pe_kv_elem); kv / mean / rstd unused
  const uint16_t* P; const float* pes; const float* pesq; const float* wt;
  float inv_k, eps;
  const float* pix;                              // (B·M, nc) pixel channels
  float* dq;                                     // (Nq, C) Σ over the batch (q_bs = 0) or (B, Nq, C); zeroed
  float* D;                                      // (M, 2C)
  float* part;                                   // (gridDim.x · gridDim.z, (2 + nc) · 2C)
  int B, H, Nq, M, C, nc, bper;
  float scale, scale_log2;
  int accumulate;  // add onto D / part (a later application of the weight-shared layer)
  int d_atomic;    // batch split over several workgroups: D by atomics
  long long dq_kbs;  // deterministic mode: dq slice per key block (plain stores, summed by the caller)
  // persistent mode (nbg > 0): nslots workgroups over (key block, head, batch group) items, nbg
  // batch groups per pair; leading partial runs write D to Dside (nslots, 256, 64) and record
  // their pair in side_pair (nslots); part has nkb + nslots rows (the extra rows zeroed when
  // not accumulating)
  int nbg, nslots;
  float* Dside;
  int* side_pair;
};

struct PeFwdArgs {
  const uint16_t* q; long long q_bs; int q_rs;  // (1 | B, Nq, ≥ C) bf16
  const uint16_t* P;                            // (M, 2C) bf16 P' = K | V columns
  const float* pix;                             // (B·M, nc)
  const float* pes; const float* pesq;          // (M) Σe, Σe² of the PE row
  const float* wt;                              // (PE_NWT, 2C)
  float* Opart; float* MLpart;                  // [split][b][q][h][32], [split][b][q][h][2]
  int B, H, Nq, M, C, nc, nsplit, chunks;       // chunks: 32-key chunks per split
  float scale_log2, inv_k, eps;
};

}  // namespace pio
