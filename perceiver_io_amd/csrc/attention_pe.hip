// Cross-attention backward fused with the factored K/V-projection reductions (image encoder,
// SURVEY K-03/K-06/K-07a; reference perceiver/model.py:185-187 applies the weight-shared
// layer_n to the same [pixels ‖ Fourier PE] input num_layers-1 times).
//
// The encoder cross-attention has few latent queries (Nq ≤ 32, the learned latent array,
// identical for every sample) and B·M keys (M = 50,176 pixels at 224×224).  Its dK/dV are only
// ever consumed by the factored projection backward (pe_proj.hip), which needs nothing but
// row-weighted sums of dY = [dK | dV]:
//     D[m,o] = Σ_b dY[b,m,o]·rσ[b,m]          (→ the PE part of dW through one GEMM)
//     S_o = Σ dY,  e_o = Σ dY·μ·rσ,  G[c,o] = Σ dY·x̂_c   (pixel channels c < nc)
// and, for the first cross layer (whose queries are the batch-broadcast latent array), dQ only as
// the sum over the batch.  So this kernel
// never writes dK/dV (an fp32 (B·M, 2C) tensor: 1.6 GB at B = 32): it folds them into D (fp32
// FMAs) and into the column sums (one MFMA per 16 keys: Σ_key W[key][seg]·dY[key][d] with the
// weights W = [1 | μ·rσ | x̂_c] as the A operand and dY straight from the accumulator, k-order
// permuted to the accumulator's row order), and the weight-shared layer's later applications
// accumulate into the same D / partials.  Broadcast queries (QB = false): dQ is accumulated over
// the whole batch in registers and reduced over the waves once per workgroup; per-sample queries
// (QB = true, the weight-shared layer_n): each element's wave partials are summed after a second
// LDS barrier and added to dq[b] with fp32 atomics.
//
// Grid (key block, head, batch group).  A workgroup owns KB = 32·NW keys of one head and loops
// over its batch group; per batch element each wave forms S = Q·Kᵀ and dP = dO·Vᵀ for its 32 keys
// (v_mfma_f32_32x32x16_bf16, key on the lane), dV_b = Pᵀ·dO, dK_b = dSᵀ·Q, its dQ share from its
// dS slab, and the folds above.  Software pipeline, one LDS-only barrier per element:
//   iteration b:  write the element-(b+1) inputs loaded last iteration (dO tile, LSE / delta, key
//                 statistics, each wave's own 32 K/V rows) into LDS buffer (b+1)&1  ·  issue the
//                 global loads of element b+2 (registers; nothing reads them before the next
//                 iteration)  ·  compute element b from LDS buffer b&1  ·  barrier.
// The barrier waits for LDS traffic only (lgkmcnt), never for the global loads in flight
// (__syncthreads' workgroup fence would drain them).  Each (key block, head) owns its D columns:
// no atomics on D unless the batch is split over several workgroups (small images).
#include "common.h"

namespace pio {

struct PeBwdArgs {
  const uint16_t* q; long long q_bs; int q_rs;  // (1 | B, Nq, ≥ C) bf16; head h = cols [32h, 32h + 32)
  const uint16_t* kv; int kv_rs;                 // (B·M, ≥ 2C) bf16: K = cols [0, C), V = [C, 2C)
  const uint16_t* dO;                            // (B, Nq, C) bf16 contiguous
  const float* lse;                              // (B, Nq, H), log2 units
  const float* delta;                            // (B, Nq, H) = rowsum(dO∘O)
  const float* mean; const float* rstd;          // (B·M) LayerNorm row statistics of the K/V input
  const float* pix;                              // (B·M, nc) pixel channels
  float* dq;                                     // (Nq, C) Σ over the batch (q_bs = 0) or (B, Nq, C); zeroed
  float* D;                                      // (M, 2C)
  float* part;                                   // (gridDim.x · gridDim.z, (2 + nc) · 2C)
  int B, H, Nq, M, C, nc, bper;
  float scale, scale_log2;
  int accumulate;  // add onto D / part (a later application of the weight-shared layer)
  int d_atomic;    // batch split over several workgroups: D by atomics
  long long dq_kbs;  // deterministic mode: dq slice per key block (plain stores, summed by the caller)
};

constexpr int PD = 32;          // head dim
constexpr int PLD = PD + 8;     // LDS row stride (bf16) of the Q / dO / dS tiles
constexpr int PMAXC = 4;        // pixel channels
constexpr int PNSEG = 8;        // weight rows of the column-sum MFMA: 1, μ·rσ, x̂_c (≤ 6 used)

template <int NW, bool QB>
__global__ __launch_bounds__(64 * NW) void attn_bwd_pe_kernel(PeBwdArgs a) {
  constexpr int KB = 32 * NW, NTH = 64 * NW;
  constexpr int KVLD = 2 * PD + 8;  // K|V row stride of the per-wave K/V tile
  constexpr int WLD = KB + 8;       // row stride (bf16) of the weight rows
  static_assert(KB == 256, "threads < 256 stage the block's key statistics");
  __shared__ __attribute__((aligned(16))) uint16_t sQb[QB ? 2 : 1][32 * PLD];
  __shared__ __attribute__((aligned(16))) float sDQb[QB ? NW : 1][QB ? 32 * 36 : 1];  // per wave: dQ_b [d][q]
  __shared__ __attribute__((aligned(16))) uint16_t sdO[2][32 * PLD];
  __shared__ __attribute__((aligned(16))) float sL[2][32], sDl[2][32];
  __shared__ __attribute__((aligned(16))) float sRs[2][KB];                 // rσ per key
  __shared__ __attribute__((aligned(16))) uint16_t sW[2][PNSEG * WLD];      // [seg][key] bf16 weights
  __shared__ __attribute__((aligned(16))) uint16_t sKV[2][NW][32 * KVLD];   // per wave: [key][K | V]
  __shared__ __attribute__((aligned(16))) uint16_t sS[NW][32 * PLD];        // per wave: dS slab [key][q]
  // epilogue aliases over the K/V tiles: dQ partials [w][q][d], column sums [w][2][seg][d]
  float(*sDQ)[32 * 33] = reinterpret_cast<float(*)[32 * 33]>(&sKV[0][0][0]);
  float(*sCS)[2][PNSEG][32] = reinterpret_cast<float(*)[2][PNSEG][32]>(&sKV[1][0][0]);

  const int w = wave_id(), l = lane_id(), r = l & 31, hh = l >> 5;
  const int kb = blockIdx.x, h = blockIdx.y, bg = blockIdx.z;
  const int kbase = kb * KB;
  const int key = kbase + 32 * w + r;  // this lane's key (S / dP column)
  const bool kval = key < a.M;
  const int b0 = bg * a.bper, b1 = min(a.B, b0 + a.bper);
  const int C = a.C, O = 2 * C, nc = a.nc;

  // ---- register staging of one batch element.  fetch() only ISSUES loads — unconditional, with
  // clamped addresses (a branch around a load, or arithmetic on a loaded value, makes hipcc wait
  // for every outstanding load at that point); stage() masks, transforms and writes LDS one
  // iteration later.
  bf16x8 kv8[4];   // this lane's 4 chunks of its wave's 32 K|V rows: rows (l >> 3) + 8j, 8 columns
  bf16x8 qd;       // a 16-byte chunk of the Q (threads < 128, QB) / dO (threads 128..255) tile
  float ld = 0.f;  // LSE / delta (threads 256..319)
  float smu = 0.f, srs = 0.f, spx[PMAXC];  // raw statistics + pixels of key kbase + threadIdx.x
  const int qrow = min((int)(threadIdx.x & 127) >> 2, a.Nq - 1), qcol = (threadIdx.x & 3) * 8;
  const int lrow_i = min((int)(threadIdx.x & 31), a.Nq - 1);
  const int skey = min(kbase + (int)(threadIdx.x % KB), a.M - 1);
  const int kvcol = (l & 7) * 8;  // 0..56: K columns 0..31, V columns 32..63
  const int kvsrc = kvcol < PD ? h * PD + kvcol : C + h * PD + kvcol - PD;
  auto fetch = [&](int b) {
    const long long rb = (long long)b * a.M;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = min(kbase + 32 * w + (l >> 3) + 8 * j, a.M - 1);
      kv8[j] = *reinterpret_cast<const bf16x8*>(a.kv + (rb + row) * a.kv_rs + kvsrc);
    }
    if (threadIdx.x < 256) {
      if (QB && threadIdx.x < 128)
        qd = *reinterpret_cast<const bf16x8*>(a.q + (long long)b * a.q_bs + (long long)qrow * a.q_rs + h * PD + qcol);
      else
        qd = *reinterpret_cast<const bf16x8*>(a.dO + ((long long)b * a.Nq + qrow) * C + h * PD + qcol);
      const long long rr = rb + skey;
      smu = a.mean[rr];
      srs = a.rstd[rr];
#pragma unroll
      for (int c = 0; c < PMAXC; ++c) spx[c] = a.pix[rr * nc + min(c, nc - 1)];
    } else if (threadIdx.x < 320) {
      const long long idx = ((long long)b * a.Nq + lrow_i) * a.H + h;
      ld = threadIdx.x >= 288 ? a.delta[idx] : a.lse[idx];
    }
  };
  auto stage = [&](int buf) {
    uint16_t* t = sKV[buf][w];
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<bf16x8*>(t + ((l >> 3) + 8 * j) * KVLD + kvcol) = kv8[j];
    if (threadIdx.x < 256) {
      if (QB || threadIdx.x >= 128) {
        const int c = threadIdx.x & 127;
        bf16x8 v = qd;
        if ((c >> 2) >= a.Nq) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        *reinterpret_cast<bf16x8*>((threadIdx.x >= 128 ? sdO[buf] : sQb[QB ? buf : 0]) + (c >> 2) * PLD + (c & 3) * 8) = v;
      }
      const int k = threadIdx.x;
      const bool ok = kbase + k < a.M;
      sRs[buf][k] = ok ? srs : 0.f;
      uint16_t* wcol = sW[buf] + k;
      wcol[0] = f2bf(ok ? 1.f : 0.f);
      wcol[WLD] = f2bf(ok ? smu * srs : 0.f);
#pragma unroll
      for (int c = 0; c < PMAXC; ++c) wcol[(2 + c) * WLD] = f2bf((ok && c < nc) ? (spx[c] - smu) * srs : 0.f);
#pragma unroll
      for (int c = 2 + PMAXC; c < PNSEG; ++c) wcol[c * WLD] = 0;
    } else if (threadIdx.x < 320) {
      const int i = threadIdx.x - 256, row = i & 31;
      const bool ok = row < a.Nq;
      if (i < 32) sL[buf][row] = ok ? ld : INFINITY;
      else sDl[buf][row] = ok ? ld : 0.f;
    }
  };
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x16 accD[2];   // D for this wave's 32 keys × 32 columns of head h: [0] K part, [1] V part
  f32x16 accX[2];   // column sums: rows = weight segment, columns = d; [0] K part, [1] V part
  f32x16 accQ;      // dQ Σ over the batch: rows = query, columns = d (this wave's keys)
  accD[0] = accD[1] = accX[0] = accX[1] = accQ = f32x16{};

  // the (batch-broadcast) query tile, once
  if (!QB && threadIdx.x < 128) {
    const int c = threadIdx.x;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(a.q + (long long)qrow * a.q_rs + h * PD + qcol);
    if ((c >> 2) >= a.Nq) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    *reinterpret_cast<bf16x8*>(sQb[0] + (c >> 2) * PLD + (c & 3) * 8) = v;
  }
  if (b0 < b1) {
    fetch(b0);
    stage(b0 & 1);
    if (b0 + 1 < b1) fetch(b0 + 1);
  }
  lds_barrier();

  for (int b = b0; b < b1; ++b) {
    const int cur = b & 1;
    // (1) element b+1 → LDS (its loads were issued one iteration ago), loads of b+2
    if (b + 1 < b1) {
      stage(cur ^ 1);
      if (b + 2 < b1) fetch(b + 2);
    }
    // (2) element b.  S = Q·Kᵀ, dP = dO·Vᵀ (rows: queries, lane: key); K/V operand fragments
    // B[k = d][col = key] straight from this wave's LDS rows
    const uint16_t* tdO = sdO[cur];
    const uint16_t* sQ = sQb[QB ? cur : 0];
    const uint16_t* tKV = sKV[cur][w];
    f32x16 S = f32x16{}, dP = f32x16{};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(tKV + r * KVLD + 16 * s + 8 * hh);
      const bf16x8 vf = *reinterpret_cast<const bf16x8*>(tKV + r * KVLD + PD + 16 * s + 8 * hh);
      S = mfma32(frag_kc(sQ, PLD, 0, 16 * s), kf, S);
      dP = mfma32(frag_kc(tdO, PLD, 0, 16 * s), vf, dP);
    }
    f32x4 lrow[4], drow[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      lrow[g] = *reinterpret_cast<const f32x4*>(&sL[cur][8 * g + 4 * hh]);
      drow[g] = *reinterpret_cast<const f32x4*>(&sDl[cur][8 * g + 4 * hh]);
    }
    f32x16 P, dS;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p = fast_exp2(kval ? S[i] * a.scale_log2 - lrow[i >> 2][i & 3] : -INFINITY);
      P[i] = p;
      dS[i] = p * (dP[i] - drow[i >> 2][i & 3]);
    }
    // dV_b = Pᵀ·dO, dK_b = dSᵀ·Q (rows: this wave's keys, lane: head-dim column; dK unscaled)
    f32x16 dV = f32x16{}, dK = f32x16{};
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      dV = mfma32(pack_acc(P, ss), frag_ks_perm(tdO, PLD, 0, 16 * ss), dV);
      dK = mfma32(pack_acc(dS, ss), frag_ks_perm(sQ, PLD, 0, 16 * ss), dK);
    }
    // dS slab [key][q] (wave-private) for the dQ share
    uint16_t* tS = sS[w];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 pk;
      pk.x = pack2(dS[4 * g], dS[4 * g + 1]);
      pk.y = pack2(dS[4 * g + 2], dS[4 * g + 3]);
      *reinterpret_cast<uint2*>(&tS[r * PLD + 8 * g + 4 * hh]) = pk;
    }
    // D += dY·rσ: accumulator row i ↔ key 32w + acc_row(i, hh); 4 consecutive rows per float4
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 rs4 = *reinterpret_cast<const f32x4*>(&sRs[cur][32 * w + 8 * g + 4 * hh]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        accD[0][4 * g + e] += dK[4 * g + e] * rs4[e];
        accD[1][4 * g + e] += dV[4 * g + e] * rs4[e];
      }
    }
    // column sums Σ_key W[seg][key]·dY[key][d]: A[row = seg][k] with k in the accumulator's row
    // order — for step s lane half hh supplies keys 16s + 4hh + 0..3 and 16s + 8 + 4hh + 0..3
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint16_t* wr = sW[cur] + (r & (PNSEG - 1)) * WLD + 32 * w + 16 * s + 4 * hh;
      const bf16x4 lo = *reinterpret_cast<const bf16x4*>(wr);
      const bf16x4 hi = *reinterpret_cast<const bf16x4*>(wr + 8);
      bf16x8 wa;
      const bool real = r < PNSEG;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wa[j] = real ? lo[j] : (short)0;
        wa[4 + j] = real ? hi[j] : (short)0;
      }
      accX[0] = mfma32(wa, pack_acc(dK, s), accX[0]);
      accX[1] = mfma32(wa, pack_acc(dV, s), accX[1]);
    }
    // this wave's dQ share Σ_key dS[key][q]·K[key][d] from its own slab and K rows (a wave reads
    // back its own LDS writes in order), summed over the batch in registers
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if constexpr (QB) {
      f32x16 dq = f32x16{};
      dq = mfma32(frag_ks(tS, PLD, 0, 0), frag_ks(tKV, KVLD, 0, 0), dq);
      dq = mfma32(frag_ks(tS, PLD, 0, 16), frag_ks(tKV, KVLD, 0, 16), dq);
      // partial [d][q]: registers 4g..4g+3 are 4 consecutive queries → one 16-byte store
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(&sDQb[w][r * 36 + 8 * g + 4 * hh]) =
            f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
      lds_barrier();
      // Σ over the waves: thread t → d = t >> 3, queries 4·(t & 7) .. +3
      if (threadIdx.x < 256) {
        const int dd = threadIdx.x >> 3, q0 = 4 * (threadIdx.x & 7);
        f32x4 v = *reinterpret_cast<const f32x4*>(&sDQb[0][dd * 36 + q0]);
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) v += *reinterpret_cast<const f32x4*>(&sDQb[ww][dd * 36 + q0]);
        float* dst = a.dq + (long long)kb * a.dq_kbs + ((long long)b * a.Nq) * C + h * PD + dd;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (q0 + e < a.Nq) {
            if (a.dq_kbs) dst[(long long)(q0 + e) * C] = v[e] * a.scale;
            else atomicAdd(dst + (long long)(q0 + e) * C, v[e] * a.scale);
          }
        }
      }
    } else {
      accQ = mfma32(frag_ks(tS, PLD, 0, 0), frag_ks(tKV, KVLD, 0, 0), accQ);
      accQ = mfma32(frag_ks(tS, PLD, 0, 16), frag_ks(tKV, KVLD, 0, 16), accQ);
    }
    lds_barrier();
  }

  // ---- D rows of this wave's keys (K part columns 32h + r, V part C + 32h + r)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = kbase + 32 * w + acc_row(i, hh);
    if (m < a.M) {
      float* dk = a.D + (long long)m * O + h * PD + r;
      float* dv = dk + C;
      const float vk = accD[0][i] * a.scale, vv = accD[1][i];
      if (a.d_atomic) {
        atomicAdd(dk, vk);
        atomicAdd(dv, vv);
      } else if (a.accumulate) {
        *dk += vk;
        *dv += vv;
      } else {
        *dk = vk;
        *dv = vv;
      }
    }
  }
  // ---- dQ and column sums: per-wave partials through LDS (aliases of the consumed K/V tiles)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = acc_row(i, hh);
    if (!QB) sDQ[w][row * 33 + r] = accQ[i];
    if (row < PNSEG) {
      sCS[w][0][row][r] = accX[0][i];
      sCS[w][1][row][r] = accX[1][i];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < (QB ? 0 : 32 * PD); e += NTH) {
    const int qq = e >> 5, dd = e & 31;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += sDQ[ww][qq * 33 + dd];
    if (qq < a.Nq) {
      float* dst = a.dq + (long long)kb * a.dq_kbs + (long long)qq * C + h * PD + dd;
      if (a.dq_kbs) *dst = v * a.scale;
      else atomicAdd(dst, v * a.scale);
    }
  }
  const long long prow = (long long)blockIdx.x * gridDim.z + blockIdx.z;
  const int nseg = 2 + nc;
  for (int e = threadIdx.x; e < 2 * nseg * 32; e += NTH) {
    const int p = e / (nseg * 32), rem = e % (nseg * 32), seg = rem / 32, j = rem % 32;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += sCS[ww][p][seg][j];
    if (p == 0) v *= a.scale;
    float* dst = a.part + prow * (long long)(nseg * O) + (long long)seg * O + p * C + h * PD + j;
    *dst = a.accumulate ? *dst + v : v;
  }
}

void attn_bwd_pe_launch(const PeBwdArgs& a0, int nkb, int bsplit, hipStream_t st) {
  PeBwdArgs a = a0;
  a.bper = (a.B + bsplit - 1) / bsplit;
  a.d_atomic = bsplit > 1 ? 1 : 0;
  constexpr int NW = 8;
  if (a.q_bs == 0)
    hipLaunchKernelGGL((attn_bwd_pe_kernel<NW, false>), dim3(nkb, a.H, bsplit), dim3(64 * NW), 0, st, a);
  else
    hipLaunchKernelGGL((attn_bwd_pe_kernel<NW, true>), dim3(nkb, a.H, bsplit), dim3(64 * NW), 0, st, a);
}

}  // namespace pio
