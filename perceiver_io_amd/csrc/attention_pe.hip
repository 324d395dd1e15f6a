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
#include <stdlib.h>

#include <algorithm>

#include <type_traits>

#include "common.h"
#include "pe_args.h"

namespace pio {

// PeBwdArgs: pe_args.h (shared with the host binding)

constexpr int PD = 32;          // head dim
constexpr int PLD = PD + 8;     // LDS row stride (bf16) of the Q / dO / dS tiles
constexpr int PMAXC = 4;        // pixel channels
constexpr int PNSEG = 8;        // weight rows of the column-sum MFMA: 1, μ·rσ, x̂_c (≤ 6 used)


// ---- implicit K/V (SURVEY K-03/K-05: the encoder's K/V are never materialised) -------------
// K/V row m of sample b, column o (K: o < C, V: C ≤ o < 2C), from the factored projection:
//     y = rσ·P'[m, o] + Σ_c x̂_c·wpg[c, o] + μrσ·(Σ_c wpg[c, o] − gw[o]) + bw[o]
// with P' = (E⊙γ_e)·W_eᵀ the batch-independent PE part (bf16, one GEMM per step), x̂_c =
// (p_c − μ)·rσ the normalised pixel channels and the per-column table rows
// wt = {wpg_0..wpg_3, Σwpg − gw, bw} (pe_weight_prep_kernel).  Neither direction forms these rows:
// both factor the products over P' plus a per-sample augmentation (attn_fwd_pe_fact_kernel,
// attn_bwd_pe_fact_kernel); ops/emulation.py pe_kv materialises them for the reference.
constexpr int PE_NWT = 6;

// ------------------------------------------------------------------------------------
// Encoder cross-attention forward over implicit K/V (head dim 32, Nq ≤ 32, no mask, no
// dropout), factored: the K/V tiles are never formed.  With K/V row m of sample b written as (pe_kv_elem)
//     y[m, o] = rσ_m·(P'[m, o] + Σ_c (p_c − μ)_m·wt[c][o] + μ_m·wt[4][o]) + wt[5][o],
// the scores and the output of one head factor into products with the BATCH-INDEPENDENT P':
//     S[q, m]  = rσ_m·(P'_K[m]·Q[q] + Σ_c (p_c − μ)_m·β_c[q] + μ_m·γ[q]) + cq[q]
//                (β_c = Q·wt[c], γ = Q·wt[4], cq = Q·wt[5] over the head's K columns; cq is a
//                per-query constant: softmax-invariant, added to the LSE only)
//     O[q]·l   = Σ_m p̃·P'_V[m] + Σ_c A_c·wt_V[c] + A_μ·wt_V[4] + l·wt_V[5],   p̃ = p·rσ_m,
//                A_c = Σ_m p̃·(p_c − μ)_m, A_μ = Σ_m p̃·μ_m, l = Σ_m p̃ / rσ_m.
// So Sᵀ = [P'_K | p − μ | μ]·[Q | β | γ]ᵀ is one 32×32×(32 + 16) MFMA product whose 16-wide
// augmentation carries the per-sample terms, rσ_m·scale and log2 rσ_m (→ p̃ straight out of
// the exponential) are folded into the score's one FMA, and the P̃ᵀ product runs against the
// shared P'_V tile plus a per-sample augmentation tile [p − μ | μ | 1/rσ] whose row NC + 1 is
// the softmax denominator l.  Per key and sample: no K/V row is formed; per score element one FMA (scale, rσ and log2 rσ), the max
// and the exponential; the accumulators are rescaled only when a lazy softmax offset moves.  The P' chunk (32 keys × the
// head's 64 K|V columns) is staged ONCE per workgroup in LDS (one 16-byte load per thread,
// double-buffered, one barrier per chunk) and serves 4·NS samples: wave w owns samples
// 4·NS·bg + NS·w + [0, NS).
// ------------------------------------------------------------------------------------
template <int NC, int NS>
__global__ __launch_bounds__(256, 2) void attn_fwd_pe_fact_kernel(PeFwdArgs a) {
  constexpr int LDT = PD + 8;       // augmentation tile row stride (bf16)
  constexpr int LKV = 2 * PD + 8;   // P' chunk row stride: K columns [0, 32), V columns [32, 64)
  static_assert(NC + 4 <= 8, "augmentation rows live in accumulator registers 0..3 of both halves; "
                            "score slots NC + 1..NC + 3 carry the folded softmax offset");
  __shared__ __attribute__((aligned(16))) uint16_t sKV[2][32 * LKV];
  __shared__ __attribute__((aligned(16))) uint16_t sA[4][NS][32 * LDT];  // [key][aug row], rows ≥ NC + 2 zero
  __shared__ __attribute__((aligned(16))) float sCL[4][NS][2][32];       // [key]: rσ·scale_log2, log2 rσ
  __shared__ __attribute__((aligned(16))) float sWt[PE_NWT][64];         // head h's table: K | V columns
  const int w = wave_id(), l = lane_id(), r = l & 31, hh = l >> 5;
  const Blk3 blk = xcd_block3();  // x: batch group (fastest), y: split, z: head
  const int split = blk.y, h = blk.z;
  const int C = a.C, M = a.M;
  for (int t = threadIdx.x; t < 64 * PE_NWT; t += 256) {
    const int j = t >> 6, c = t & 63;
    sWt[j][c] = a.wt[(long long)j * 2 * C + (c < PD ? h * PD + c : C + h * PD + c - PD)];
  }
  for (int t = threadIdx.x; t < 4 * NS * 32 * LDT / 8; t += 256)
    reinterpret_cast<bf16x8*>(&sA[0][0][0])[t] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  const int kbeg = split * a.chunks * 32;
  const int kend = min(M, kbeg + a.chunks * 32);
  const int bw0 = (blk.x * 4 + w) * NS;  // this wave's first sample (waves past B idle but keep barriers)
  __syncthreads();

  // queries (lane = query, clamped) and their augmentation β / γ / cq per sample
  const int qi = r, qc = min(qi, a.Nq - 1);
  bf16x8 qa[NS][3];
  float cq[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int b = min(bw0 + s, a.B - 1);
    const uint16_t* qp = a.q + (long long)b * a.q_bs + (long long)qc * a.q_rs + h * PD + 8 * hh;
    qa[s][0] = *reinterpret_cast<const bf16x8*>(qp);
    qa[s][1] = *reinterpret_cast<const bf16x8*>(qp + 16);
    float part[NC + 2];
#pragma unroll
    for (int j = 0; j < NC + 2; ++j) part[j] = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float qv = bf2f(qa[s][t][e]);
        const int d = 16 * t + 8 * hh + e;
#pragma unroll
        for (int j = 0; j < NC + 2; ++j) part[j] = fmaf(qv, sWt[j < NC ? j : j + 4 - NC][d], part[j]);
      }
    bf16x8 au = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < NC + 2; ++j) part[j] = xor32_sum(part[j]);
#pragma unroll
    for (int j = 0; j < NC + 1; ++j) au[j] = (short)f2bf(part[j]);  // β_0..β_{NC-1}, γ
    qa[s][2] = hh == 0 ? au : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    cq[s] = part[NC + 1];
  }

  // per-chunk staging registers: one 16-byte piece of the P' chunk per thread (row tid >> 3,
  // columns 8·(tid & 7): K for < 32), the lane's key statistics inputs per sample
  const int srow = threadIdx.x >> 3, scol = 8 * (threadIdx.x & 7);
  const long long prs = 2LL * C;
  const uint16_t* pp = a.P + (long long)(min(kbeg, M) + srow) * prs + (scol < PD ? h * PD + scol : C + h * PD + scol - PD);
  bf16x8 pst;
  float spe = 0.f, spq = 0.f, spx[NS][NC];
  auto fetch = [&](int k0) {  // loads only (rows past M are the zero pad rows of P')
    pst = *reinterpret_cast<const bf16x8*>(pp);
    pp += 32 * prs;
    const int key = min(k0 + r, M - 1);
    spe = a.pes[key];
    spq = a.pesq[key];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int b = min(bw0 + s, a.B - 1);
      const float* px = a.pix + ((long long)b * M + key) * NC;
#pragma unroll
      for (int c = 0; c < NC; ++c) spx[s][c] = px[c];
    }
  };

  f32x16 om[NS], oa[NS];
  float m_run[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    om[s] = f32x16{};
    oa[s] = f32x16{};
    m_run[s] = 0.f;  // folded into the score MFMA (qa[s][2] slots NC + 1..NC + 3), set by chunk 0
  }
  const float sl2 = a.scale_log2, isl2 = 1.f / sl2;
  auto set_offset = [&](int s) {  // −m_run[s] → the query augmentation's offset slots
    const float nm = -m_run[s];
    const uint16_t mh = f2bf(nm);
    if (hh == 0) {
      qa[s][2][NC + 1] = (short)mh;
      qa[s][2][NC + 2] = (short)f2bf(nm - bf2f(mh));
      qa[s][2][NC + 3] = (short)mh;
    }
  };
  const int nch = kend > kbeg ? (kend - kbeg + 31) / 32 : 0;  // an empty split (kbeg ≥ M) has none
  auto chunk = [&](int ci, auto masked_t) {
    constexpr bool masked = decltype(masked_t)::value;
    const int k0 = kbeg + 32 * ci;
    uint16_t* kv = sKV[ci & 1];
    *reinterpret_cast<bf16x8*>(kv + srow * LKV + scol) = pst;
    bf16x8 ka[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {  // key k0 + r of sample s: statistics → tables + A augmentation
      float sm = spe, sq = spq;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        sm += spx[s][c];
        sq = fmaf(spx[s][c], spx[s][c], sq);
      }
      const float mu = sm * a.inv_k;
      const float var = fmaxf(sq * a.inv_k - mu * mu, 0.f) + a.eps;
      const float rs = rsqrtf(var);
      bf16x8 au = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < NC; ++c) au[c] = (short)f2bf(spx[s][c] - mu);
      au[NC] = (short)f2bf(mu);
      if (hh == 0) {
        sCL[w][s][0][r] = rs * sl2;
        sCL[w][s][1][r] = -0.5f * __log2f(var);  // log2 rσ
        bf16x8 vrow = au;
        vrow[NC + 1] = (short)f2bf(var * rs);    // 1/rσ: row NC + 1 of P̃ᵀ·A = the denominator l
        *reinterpret_cast<bf16x8*>(&sA[w][s][r * LDT]) = vrow;
      }
      // score slots NC + 1..NC + 3: 1 / (rσ·scale_log2) as bf16 hi, hi, lo against the queries'
      // −m_run as hi, lo, hi — the MFMA subtracts the softmax offset (to ~2^-16 relative)
      const float icv = var * rs * isl2;
      const uint16_t ih = f2bf(icv);
      au[NC + 1] = (short)ih;
      au[NC + 2] = (short)ih;
      au[NC + 3] = (short)f2bf(icv - bf2f(ih));
      ka[s] = hh == 0 ? au : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    __syncthreads();  // the chunk and the tables are in LDS; buffer (ci + 1) & 1 is free
    if (ci + 1 < nch) fetch(k0 + 32);
    if (bw0 >= a.B) return;
    const bf16x8 pk0 = frag_kc(kv, LKV, 0, 0), pk1 = frag_kc(kv, LKV, 0, 16);
    f32x16 sc[NS];  // every sample's scores first: their MFMAs overlap the softmax VALU below
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      sc[s] = mfma32(pk0, qa[s][0], f32x16{});
      sc[s] = mfma32(pk1, qa[s][1], sc[s]);
      sc[s] = mfma32(ka[s], qa[s][2], sc[s]);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float mt = -INFINITY;
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // keys 8g + 4hh + (0..3) of the chunk: registers 4g..4g+3
        const float4 cf = *reinterpret_cast<const float4*>(&sCL[w][s][0][8 * g + 4 * hh]);
        const float4 lf = *reinterpret_cast<const float4*>(&sCL[w][s][1][8 * g + 4 * hh]);
        const float cv[4] = {cf.x, cf.y, cf.z, cf.w}, lv[4] = {lf.x, lf.y, lf.z, lf.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          float t = fmaf(sc[s][i], cv[e], lv[e]);
          if constexpr (masked) t = k0 + acc_row(i, hh) < kend ? t : -INFINITY;
          sc[s][i] = t;
          mt = fmaxf(mt, t);
        }
      }
      mt = xor32_max(mt);
      // the scores come out of the MFMA relative to the lazy offset m_run (no per-element
      // subtraction).  The offset moves only when a score exceeds it by more than 2^8 (p̃ ≤ 2^8 is
      // exact in fp32 and in range for bf16) or on the split's first chunk, so the accumulators
      // are rescaled on a handful of chunks, not on nearly every one (a new maximum among 32
      // queries is the rule for the first ~50 chunks)
      const bool mv = ci == 0 || mt > 8.f;
      if (__ballot(mv)) {
        const float dm = mv ? mt : 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[s][i] -= dm;
        if (ci > 0) {  // chunk 0: nothing accumulated yet (and exp2(−dm) may overflow)
          const float alpha = fast_exp2(-dm);
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            om[s][i] *= alpha;
            oa[s][i] *= alpha;
          }
        }
        m_run[s] += dm;
        set_offset(s);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[s][i] = fast_exp2(sc[s][i]);
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 pb = pack_acc(sc[s], ss);
        om[s] = mfma32(frag_ks_perm(kv + PD, LKV, 0, 16 * ss), pb, om[s]);
        oa[s] = mfma32(frag_ks_perm(&sA[w][s][0], LDT, 0, 16 * ss), pb, oa[s]);
      }
    }
  };
  if (nch > 0) fetch(kbeg);
  const int nfull = kend > kbeg ? (kend - kbeg) / 32 : 0;
  for (int ci = 0; ci < nfull; ++ci) chunk(ci, std::false_type{});
  if (nfull < nch) chunk(nfull, std::true_type{});  // the last chunk of a split ending mid-chunk
  if (bw0 >= a.B) return;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int b = bw0 + s;
    if (b >= a.B) break;
    // augmentation rows R < 8 of query r: R < 4 in registers R of the lower half, 4..7 in the upper
    float aug[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float own = oa[s][i], oth = __shfl_xor(own, 32);
      aug[hh == 0 ? i : i + 4] = own;
      aug[hh == 0 ? i + 4 : i] = oth;
    }
    const float lsum = aug[NC + 1];
    if (qi >= a.Nq) continue;
    const long long row = (((long long)split * a.B + b) * a.Nq + qi) * a.H + h;
    float* op = a.Opart + row * PD;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float ov[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g + e, d = PD + acc_row(i, hh);  // V column of the head
        float y = fmaf(aug[NC], sWt[4][d], fmaf(lsum, sWt[5][d], om[s][i]));
#pragma unroll
        for (int c = 0; c < NC; ++c) y = fmaf(aug[c], sWt[c][d], y);
        ov[e] = y;
      }
      *reinterpret_cast<float4*>(op + 8 * g + 4 * hh) = make_float4(ov[0], ov[1], ov[2], ov[3]);
    }
    if (hh == 0) {
      a.MLpart[row * 2] = (nch > 0 ? m_run[s] : -1e30f) + cq[s] * sl2;  // an empty split: l = 0
      a.MLpart[row * 2 + 1] = lsum;
    }
  }
}

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
  // per wave: [key][K | V] — double-buffered staging of the loaded rows
  __shared__ __attribute__((aligned(16))) uint16_t sKV[2][NW][32 * KVLD];
  __shared__ __attribute__((aligned(16))) uint16_t sS[NW][32 * PLD];        // per wave: dS slab [key][q]
  // epilogue aliases over the consumed tiles: dQ partials [w][q][d], column sums [w][2][seg][d]
  float(*sDQ)[32 * 33] = reinterpret_cast<float(*)[32 * 33]>(&sKV[0][0][0]);
  float(*sCS)[2][PNSEG][32] =
      reinterpret_cast<float(*)[2][PNSEG][32]>(&sKV[1][0][0]);
  static_assert(sizeof(float) * NW * 32 * 33 <= sizeof(uint16_t) * NW * 32 * KVLD, "dQ partial alias");
  static_assert(sizeof(float) * NW * 2 * PNSEG * 32 <= sizeof(uint16_t) * NW * 32 * PLD, "column-sum alias");

  const int w = wave_id(), l = lane_id(), r = l & 31, hh = l >> 5;
  const int C = a.C, O = 2 * C, nc = a.nc;

  // one run = one (key block, head) over a contiguous batch range [b0, b1).  Grid mode: the run
  // of this workgroup's (key block, head, batch group).  Persistent mode (a.nbg > 0): workgroup
  // g owns items [g·T/G, (g+1)·T/G) of the T = pairs × nbg (key block, head, batch group) items,
  // pair-major, and sweeps them as runs of consecutive items of one pair — the same work per
  // workgroup to within one item, instead of grid rounds that leave most CUs idle in the last
  // one.  A pair is shared by at most two workgroups; its first contributor (the run holding
  // batch group 0) writes D as in grid mode, the other one (a workgroup's leading partial run)
  // writes its D slice to its side slot (added into D by attn_pe_side_add_kernel) and its column
  // sums to partial row nkb + g.
  const int nkb = (a.M + KB - 1) / KB;
  long long it = 0, it_end = 0;
  if (a.nbg > 0 && !a.accumulate) {  // this workgroup's slot row of the partials, before any run writes it
    float* prow0 = a.part + (long long)(nkb + blockIdx.x) * ((2 + nc) * O);
    for (int e = threadIdx.x; e < (2 + nc) * O; e += NTH) prow0[e] = 0.f;
  }
  if (a.nbg > 0) {
    const long long T = (long long)nkb * a.H * a.nbg;
    it = T * blockIdx.x / gridDim.x;
    it_end = T * (blockIdx.x + 1) / gridDim.x;
    if (threadIdx.x == 0) a.side_pair[blockIdx.x] = (it % a.nbg) != 0 ? (int)(it / a.nbg) : -1;
  }
  for (bool first_run = true;; first_run = false) {
  int kb, h, b0, b1, side = -1;
  long long prow;
  if (a.nbg > 0) {
    if (it >= it_end) break;
    if (!first_run) __syncthreads();  // the previous run's epilogue LDS traffic is done
    const int pair = (int)(it / a.nbg), bgs = (int)(it % a.nbg);
    const int bge = (int)min((long long)a.nbg, bgs + (it_end - it));
    kb = pair / a.H;
    h = pair % a.H;
    b0 = bgs * a.bper;
    b1 = min(a.B, bge * a.bper);
    if (bgs > 0) side = blockIdx.x;
    prow = bgs > 0 ? nkb + blockIdx.x : kb;
    it += bge - bgs;
  } else {
    if (!first_run) break;
    kb = blockIdx.x;
    h = blockIdx.y;
    b0 = blockIdx.z * a.bper;
    b1 = min(a.B, b0 + a.bper);
    prow = (long long)blockIdx.x * gridDim.z + blockIdx.z;
  }
  const int kbase = kb * KB;
  const int key = kbase + 32 * w + r;  // this lane's key (S / dP column)
  const bool kval = key < a.M;

  // ---- register staging of one batch element.  fetch() only ISSUES loads — unconditional, with
  // clamped addresses (a branch around a load, or arithmetic on a loaded value, makes hipcc wait
  // for every outstanding load at that point); stage() masks, transforms and writes LDS one
  // iteration later.
  bf16x8 kv8[4];  // this lane's 4 chunks of its wave's 32 K|V rows: rows (l >> 3) + 8j, 8 columns
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
    {
      uint16_t* t = sKV[buf][w];
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<bf16x8*>(t + ((l >> 3) + 8 * j) * KVLD + kvcol) = kv8[j];
    }
    if (threadIdx.x < 256) {
      if (QB || threadIdx.x >= 128) {
        const int c = threadIdx.x & 127;
        bf16x8 v = qd;
        if ((c >> 2) >= a.Nq) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        *reinterpret_cast<bf16x8*>((threadIdx.x >= 128 ? sdO[buf] : sQb[QB ? buf : 0]) + (c >> 2) * PLD + (c & 3) * 8) = v;
      }
      const int k = threadIdx.x;
      const bool ok = kbase + k < a.M;
      float st[2 + PMAXC];  // rσ, μrσ, x̂_c
      st[0] = srs;
      st[1] = smu * srs;
#pragma unroll
      for (int c = 0; c < PMAXC; ++c) st[2 + c] = c < nc ? (spx[c] - smu) * srs : 0.f;
      sRs[buf][k] = ok ? st[0] : 0.f;
      uint16_t* wcol = sW[buf] + k;
      wcol[0] = f2bf(ok ? 1.f : 0.f);
      wcol[WLD] = f2bf(ok ? st[1] : 0.f);
#pragma unroll
      for (int c = 0; c < PMAXC; ++c) wcol[(2 + c) * WLD] = f2bf((ok && c < nc) ? st[2 + c] : 0.f);
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
      if (side >= 0) {  // the slot holds this application's contribution only (added after the kernel)
        float* sd = a.Dside + ((long long)side * KB + m - kbase) * 64 + r;
        sd[0] = vk;
        sd[PD] = vv;
      } else if (a.d_atomic) {
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
  }  // runs
}

// ------------------------------------------------------------------------------------
// Encoder cross-attention backward over implicit K/V, factored like attn_fwd_pe_fact_kernel: no
// K/V tile is ever formed.  With K/V row m of sample b written as
//     y[m, o] = rσ_m·(P'[m, o] + Σ_j a_j[m]·T_j[o]) + wt5[o],   a = [p_c − μ (c < NC) | μ | 1/rσ],
//     T = [wt_c | wt4 | wt5]   (the 1/rσ row of a carries the bias row wt5)
// the products of one (sample, 32-key slice, head) are
//     S   = rσ·(Q·P'_Kᵀ + β·aᵀ) + cq             β = Q·T_K (NC + 1 columns), cq = Q·wt5_K
//     dP  = rσ·(dO·P'_Vᵀ + ω·aᵀ) + d5            ω = dO·T_V,                 d5 = dO·wt5_V
//     P̃ = P·rσ, dS̃ = dS·rσ = P̃·(dP − δ)        (rσ of the lane's key)
//     dQ  = dS̃·P'_K + (dS̃·a)·T_K
//     dK̃, dṼ = dS̃ᵀ·Q, P̃ᵀ·dO = rσ·dK, rσ·dV      → D += dK̃ | dṼ;  column sums Σ_key a_j·dỸ
// (Σ W·dY with W = rσ·a = [x̂_c | μrσ | 1], the [1 | μrσ | x̂_c] segments of attn_bwd_pe_kernel).
// β / ω / cq / d5 are formed ONCE per sample by the staging threads (8 threads per query row,
// 4 dims each, DPP sums over the 8) and land in LDS as ready bf16 operand rows; cq / d5 are folded
// into the per-query exponent offset cq·scale·log2e − LSE and the dS offset d5 − δ in fp32, so the
// only bf16-rounded per-sample terms are the ones the forward rounds the same way.  Every lane forms
// the statistics of its own key (pixels prefetched one sample ahead, PE row sums in registers) and
// writes its row of a (wave-private LDS: the transposed products read it); the batch-invariant
// P' fragments of S / dP and the dQ table operand stay in registers for the whole run.  Per
// 32-key slice and sample: 19 MFMAs and one workgroup barrier (per-sample queries: the wave
// partials of dQ_b are double-buffered and summed during sample b + 1).  Same
// run structure, outputs and partial-row layout as attn_bwd_pe_kernel.
// ------------------------------------------------------------------------------------
template <int NC, bool QB>
__global__ __launch_bounds__(512) void attn_bwd_pe_fact_kernel(PeBwdArgs a) {
  constexpr int NW = 8, KB = 256, NTH = 512;
  constexpr int PPL = 2 * PD + 8;  // P' tile row stride (bf16): K columns [0, 32), V [32, 64)
  constexpr int NA = NC + 2;       // rows of a: p_c − μ, μ, 1/rσ
  static_assert(NA <= 6, "a fits the first 8 slots of one operand half");
  __shared__ __attribute__((aligned(16))) uint16_t sQ[QB ? 2 : 1][32 * PLD];
  __shared__ __attribute__((aligned(16))) uint16_t sdO[2][32 * PLD];
  // per query: the augmentation operand row [β_c | γ] / [ω_c | ω_4] (slots 0..7: lane half 0;
  // slots 8..15 stay zero: lane half 1)
  __shared__ __attribute__((aligned(16))) uint16_t sAq[QB ? 2 : 1][32 * 16];
  __shared__ __attribute__((aligned(16))) uint16_t sAo[2][32 * 16];
  __shared__ __attribute__((aligned(16))) float sL[2][32], sDl[2][32];  // cq·sl2 − LSE, d5 − δ
  __shared__ __attribute__((aligned(16))) float sWt[PE_NWT][64];        // head h's table: K | V columns
  __shared__ __attribute__((aligned(16))) uint16_t sP[NW][32 * PPL];    // run setup: the wave's P' rows
  __shared__ __attribute__((aligned(16))) uint16_t sS[NW][32 * PLD];    // dS̃ slab [key][q]
  __shared__ __attribute__((aligned(16))) uint16_t sA[NW][33 * 16];     // [key][j]: a (j < NA), 0 (j 8..15)
  // per-sample queries: per wave dQ_b [d][q], double-buffered (sample b's partials are summed
  // during sample b + 1: one workgroup barrier per sample)
  __shared__ __attribute__((aligned(16))) float sDQb[QB ? 2 : 1][QB ? NW : 1][QB ? 32 * 36 : 1];
  // epilogue aliases over the consumed tiles: dQ partials [w][q][d], column sums [w][2][seg][d]
  float(*sDQ)[32 * 33] = reinterpret_cast<float(*)[32 * 33]>(&sP[0][0]);
  float(*sCS)[2][PNSEG][32] = reinterpret_cast<float(*)[2][PNSEG][32]>(&sS[0][0]);
  static_assert(sizeof(float) * NW * 32 * 33 <= sizeof(uint16_t) * NW * 32 * PPL, "dQ partial alias");
  static_assert(sizeof(float) * NW * 2 * PNSEG * 32 <= sizeof(uint16_t) * NW * 32 * PLD, "column-sum alias");

  const int w = wave_id(), l = lane_id(), r = l & 31, hh = l >> 5;
  const int C = a.C, O = 2 * C;
  const float sl2 = a.scale_log2;
  const bf16x8 z8 = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};

  // zero slots that are never rewritten: operand-row halves 8..15, a's slots 8..15
  for (int t = threadIdx.x; t < (QB ? 2 : 1) * 32; t += NTH) *reinterpret_cast<bf16x8*>(&sAq[t >> 5][(t & 31) * 16 + 8]) = z8;
  for (int t = threadIdx.x; t < 2 * 32; t += NTH) *reinterpret_cast<bf16x8*>(&sAo[t >> 5][(t & 31) * 16 + 8]) = z8;
  for (int t = threadIdx.x; t < NW * 33; t += NTH) *reinterpret_cast<bf16x8*>(&sA[t / 33][(t % 33) * 16 + 8]) = z8;

  // run bookkeeping: identical to attn_bwd_pe_kernel
  const int nkb = (a.M + KB - 1) / KB;
  long long it = 0, it_end = 0;
  if (a.nbg > 0 && !a.accumulate) {
    float* prow0 = a.part + (long long)(nkb + blockIdx.x) * ((2 + NC) * O);
    for (int e = threadIdx.x; e < (2 + NC) * O; e += NTH) prow0[e] = 0.f;
  }
  if (a.nbg > 0) {
    const long long T = (long long)nkb * a.H * a.nbg;
    it = T * blockIdx.x / gridDim.x;
    it_end = T * (blockIdx.x + 1) / gridDim.x;
    if (threadIdx.x == 0) a.side_pair[blockIdx.x] = (it % a.nbg) != 0 ? (int)(it / a.nbg) : -1;
  }
  // staging roles (per sample): thread t → tensor t >> 8 (0: Q, 1: dO), query row (t >> 3) & 31,
  // dims 4·(t & 7) .. +3; the row's first thread also loads the row's LSE / δ
  const int st_ten = threadIdx.x >> 8, st_row = (threadIdx.x >> 3) & 31, st_c = 4 * (threadIdx.x & 7);
  const bool st_lead = (threadIdx.x & 7) == 0;
  const int st_rowc = min(st_row, a.Nq - 1);
  const bool st_ok = st_row < a.Nq;

  for (bool first_run = true;; first_run = false) {
    int kb, h, b0, b1, side = -1;
    long long prow;
    if (a.nbg > 0) {
      if (it >= it_end) break;
      if (!first_run) __syncthreads();  // the previous run's epilogue LDS traffic is done
      const int pair = (int)(it / a.nbg), bgs = (int)(it % a.nbg);
      const int bge = (int)min((long long)a.nbg, bgs + (it_end - it));
      kb = pair / a.H;
      h = pair % a.H;
      b0 = bgs * a.bper;
      b1 = min(a.B, bge * a.bper);
      if (bgs > 0) side = blockIdx.x;
      prow = bgs > 0 ? nkb + blockIdx.x : kb;
      it += bge - bgs;
    } else {
      if (!first_run) break;
      kb = blockIdx.x;
      h = blockIdx.y;
      b0 = blockIdx.z * a.bper;
      b1 = min(a.B, b0 + a.bper);
      prow = (long long)blockIdx.x * gridDim.z + blockIdx.z;
    }
    const int kbase = kb * KB;
    const int key = kbase + 32 * w + r;  // this lane's key (S / dP column)
    const bool kval = key < a.M;
    const int keyc = min(key, a.M - 1);
    const bool masked = kbase + KB > a.M;  // uniform: the run's last key block is partial

    // ---- run setup: table columns of head h, the wave's P' rows, the lane's PE row sums
    for (int t = threadIdx.x; t < 64 * PE_NWT; t += NTH) {
      const int j = t >> 6, c = t & 63;
      sWt[j][c] = a.wt[(long long)j * O + (c < PD ? h * PD + c : C + h * PD + c - PD)];
    }
    const uint16_t* prp = a.P + (long long)keyc * O + h * PD;
    bf16x8 pk[2], pv[2];  // S / dP B operands: P'_K / P'_V [key r][d = 16s + 8hh .. +7]
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      pk[s] = *reinterpret_cast<const bf16x8*>(prp + 16 * s + 8 * hh);
      pv[s] = *reinterpret_cast<const bf16x8*>(prp + C + 16 * s + 8 * hh);
      *reinterpret_cast<bf16x8*>(&sP[w][r * PPL + 16 * s + 8 * hh]) = pk[s];
    }
    const float pes = a.pes[keyc], pesq = a.pesq[keyc];
    __syncthreads();  // sWt, sP
    // dQ B operands: P'_K [k = key 16s + 8hh + j][n = d = r], and the table operand of the dQ
    // augmentation: slot t of half hh ↔ row j = 4hh + (t & 3) + 8(t >> 2) of Gᵀ (pack_acc order)
    bf16x8 tq;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int j = 4 * hh + (t & 3) + 8 * (t >> 2);
      const int row = j < NC ? j : (j == NC ? 4 : 5);
      tq[t] = (short)f2bf(j < NA ? sWt[row][r] : 0.f);
    }
    // table values of this staging thread's 4 dims (K table for Q rows, V table for dO rows)
    // rows [wt_c | wt4 | wt5] → NA dot products per staged row
    float cq_keep = 0.f;  // broadcast queries: this row's Q·wt5_K (staging leaders of tensor 0)

    // dot products of one staged 4-dim piece with the table rows, summed over the row's 8
    // threads; the leader writes the operand row (slots 0..NC) and returns the wt5 product
    auto stage_aug = [&](const bf16x4& v, uint16_t* arow) -> float {
      float part[NA];
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int trow = j < NC ? j : (j == NC ? 4 : 5);
        const f32x4 tw = *reinterpret_cast<const f32x4*>(&sWt[trow][32 * st_ten + st_c]);
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) s = fmaf(bf2f(v[e]), tw[e], s);
        s += dpp<0xB1>(s);
        s += dpp<0x4E>(s);
        s += dpp<0x141>(s);  // row_half_mirror: lanes 0-7 ↔ 7-0 (sums the two quads of 8)
        part[j] = s;
      }
      if (st_lead) {
        bf16x8 au = z8;
#pragma unroll
        for (int j = 0; j < NC + 1; ++j) au[j] = (short)f2bf(part[j]);
        *reinterpret_cast<bf16x8*>(arow) = au;
      }
      return part[NA - 1];
    };

    // ---- per-sample register staging: fetch() only issues loads (clamped addresses)
    bf16x4 st_v = bf16x4{0, 0, 0, 0};
    float st_ld = 0.f;
    float px[NC];  // the current sample's pixels of this lane's key; refilled with the next
                   // sample's once consumed (no second register set: no loop-carried copy of a
                   // load still in flight, whose wait would drain every memory operation)
    // per-thread sample-0 addresses + wave-uniform per-sample strides (scalar multiplies)
    const int wten = __builtin_amdgcn_readfirstlane(st_ten);
    const uint16_t* st_src = wten == 0 ? a.q + (long long)st_rowc * a.q_rs + h * PD + st_c
                                       : a.dO + (long long)st_rowc * C + h * PD + st_c;
    const long long st_bs = wten == 0 ? a.q_bs : (long long)a.Nq * C;
    const float* ld_src = (wten == 0 ? a.lse : a.delta) + (long long)st_rowc * a.H + h;
    const long long ld_bs = (long long)a.Nq * a.H;
    const float* px_src = a.pix + (long long)keyc * NC;
    const long long px_bs = (long long)a.M * NC;
    auto fetch = [&](int b) {
      if (QB || wten == 1) st_v = *reinterpret_cast<const bf16x4*>(st_src + b * st_bs);
      if (st_lead) st_ld = ld_src[b * ld_bs];
    };
    auto fetch_px = [&](int b, float (&dst)[NC]) {
      const float* pp = px_src + b * px_bs;
#pragma unroll
      for (int c = 0; c < NC; ++c) dst[c] = pp[c];
    };
    auto stage = [&](int buf) {
      float cst;
      if (QB || wten == 1) {
        const bf16x4 v = st_ok ? st_v : bf16x4{0, 0, 0, 0};
        uint16_t* tile = wten == 0 ? sQ[QB ? buf : 0] : sdO[buf];
        *reinterpret_cast<bf16x4*>(tile + st_row * PLD + st_c) = v;
        cst = stage_aug(v, wten == 0 ? &sAq[QB ? buf : 0][st_row * 16] : &sAo[buf][st_row * 16]);
      } else {
        cst = cq_keep;
      }
      if (st_lead) {
        if (wten == 0) sL[buf][st_row] = st_ok ? fmaf(cst, sl2, -st_ld) : -INFINITY;
        else sDl[buf][st_row] = st_ok ? cst - st_ld : 0.f;
      }
    };
    auto lds_barrier = [] {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };

    // broadcast queries: the Q tile, its augmentation row and cq once per run
    if (!QB && st_ten == 0) {
      const bf16x4 v = st_ok ? *reinterpret_cast<const bf16x4*>(a.q + (long long)st_rowc * a.q_rs + h * PD + st_c)
                             : bf16x4{0, 0, 0, 0};
      *reinterpret_cast<bf16x4*>(&sQ[0][st_row * PLD + st_c]) = v;
      cq_keep = stage_aug(v, &sAq[0][st_row * 16]);
    }

    f32x16 accD[2];  // D for this wave's 32 keys × 32 columns of head h: [0] K part, [1] V part
    f32x16 accX[2];  // column sums: rows = segment j of W, columns = d; [0] K part, [1] V part
    f32x16 accQ;     // dQ Σ over the batch (broadcast queries): rows = query, columns = d
    accD[0] = accD[1] = accX[0] = accX[1] = accQ = f32x16{};

    // sample order b0 .. b1 - 1 (a workgroup-staggered start was measured: no change,
    // profiles/r5_ab/README.md)
    const int nb = b1 - b0;
    auto perm = [&](int j) { return b0 + j; };
    if (nb > 0) {
      fetch(perm(0));
      fetch_px(perm(0), px);
      stage(0);
      if (nb > 1) {
        fetch(perm(1));
      }
    }
    lds_barrier();

    // Σ over the waves of sample bb's dQ partials (threads < 256: d = t >> 3, queries 4·(t & 7) .. +3)
    auto dq_reduce = [&](int jj) {  // jj: position in the sample order
      if (threadIdx.x >= 256) return;
      const int bb = perm(jj);
      const int dd = threadIdx.x >> 3, q0 = 4 * (threadIdx.x & 7);
      const float(*src)[32 * 36] = reinterpret_cast<const float(*)[32 * 36]>(&sDQb[QB ? (jj & 1) : 0][0][0]);
      f32x4 v = *reinterpret_cast<const f32x4*>(&src[0][dd * 36 + q0]);
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) v += *reinterpret_cast<const f32x4*>(&src[ww][dd * 36 + q0]);
      float* dst = a.dq + (long long)kb * a.dq_kbs + ((long long)bb * a.Nq) * C + h * PD + dd;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (q0 + e < a.Nq) {
          if (a.dq_kbs) dst[(long long)(q0 + e) * C] = v[e] * a.scale;
          else atomicAdd(dst + (long long)(q0 + e) * C, v[e] * a.scale);
        }
      }
    };

    auto body = [&](int jb, auto masked_t) {  // jb: position in the sample order
      constexpr bool MK = decltype(masked_t)::value;
      const int cur = jb & 1;
      // (0) statistics of key `key` for sample b → a, W, rσ rows (wave-private) and the key-side
      // augmentation operand of S / dP
      float sm = pes, sq = pesq;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        sm += px[c];
        sq = fmaf(px[c], px[c], sq);
      }
      const float mu = sm * a.inv_k;
      const float var = fmaxf(sq * a.inv_k - mu * mu, 0.f) + a.eps;
      const float rs = rsqrtf(var);
      float av[NA];
#pragma unroll
      for (int c = 0; c < NC; ++c) av[c] = px[c] - mu;
      av[NC] = mu;
      av[NC + 1] = var * rs;  // 1/rσ
      if constexpr (MK) {
        if (!kval) {
#pragma unroll
          for (int j = 0; j < NA; ++j) av[j] = 0.f;
        }
      }
      bf16x8 kaug = z8, row = z8;
#pragma unroll
      for (int j = 0; j < NA; ++j) row[j] = (short)f2bf(av[j]);
      if (hh == 0) {
#pragma unroll
        for (int j = 0; j < NC + 1; ++j) kaug[j] = row[j];
        *reinterpret_cast<bf16x8*>(&sA[w][r * 16]) = row;
      }
      // this lane's pixels are consumed: the next sample's
      if (jb + 1 < nb) fetch_px(perm(jb + 1), px);
      // (1) the next sample → LDS (its loads were issued one iteration ago), loads of the one after
      if (jb + 1 < nb) {
        stage(cur ^ 1);
        if (jb + 2 < nb) fetch(perm(jb + 2));
      }
      if constexpr (QB) {
        if (jb > 0) dq_reduce(jb - 1);  // written last iteration, before its barrier
      }
      // (2) S and dP: rows = queries, lane = key
      const uint16_t* tQ = sQ[QB ? cur : 0];
      const uint16_t* tdO = sdO[cur];
      const bf16x8 qaug = *reinterpret_cast<const bf16x8*>(&sAq[QB ? cur : 0][r * 16 + 8 * hh]);
      const bf16x8 oaug = *reinterpret_cast<const bf16x8*>(&sAo[cur][r * 16 + 8 * hh]);
      f32x16 S = mfma32(qaug, kaug, f32x16{}), dP = mfma32(oaug, kaug, f32x16{});
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        S = mfma32(frag_kc(tQ, PLD, 0, 16 * s), pk[s], S);
        dP = mfma32(frag_kc(tdO, PLD, 0, 16 * s), pv[s], dP);
      }
      // P̃ = P·rσ and dS̃ = dS·rσ (rσ of the lane's key): dṼ = P̃ᵀ·dO = rσ·dV and dK̃ = dS̃ᵀ·Q =
      // rσ·dK are exactly the D increments, and the column sums Σ W·dY = Σ a·dỸ
      const float cl = rs * sl2;
      f32x16 P, dS;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lr = *reinterpret_cast<const f32x4*>(&sL[cur][8 * g + 4 * hh]);
        const f32x4 dr = *reinterpret_cast<const f32x4*>(&sDl[cur][8 * g + 4 * hh]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = 4 * g + e;
          float p = fast_exp2(fmaf(S[i], cl, lr[e])) * rs;
          if constexpr (MK) p = kval ? p : 0.f;
          P[i] = p;
          dS[i] = p * fmaf(dP[i], rs, dr[e]);
        }
      }
      // dṼ_b = P̃ᵀ·dO, dK̃_b = dS̃ᵀ·Q (rows: this wave's keys, lane: head-dim column; dK̃ unscaled)
      f32x16 dV = f32x16{}, dK = f32x16{};
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        dV = mfma32(pack_acc(P, ss), frag_ks_perm(tdO, PLD, 0, 16 * ss), dV);
        dK = mfma32(pack_acc(dS, ss), frag_ks_perm(tQ, PLD, 0, 16 * ss), dK);
      }
      // dS̃ slab [key][q] (wave-private) for the dQ products
      uint16_t* tS = sS[w];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 pkd;
        pkd.x = pack2(dS[4 * g], dS[4 * g + 1]);
        pkd.y = pack2(dS[4 * g + 2], dS[4 * g + 3]);
        *reinterpret_cast<uint2*>(&tS[r * PLD + 8 * g + 4 * hh]) = pkd;
      }
      accD[0] += dK;
      accD[1] += dV;
      // column sums Σ_key a[j][key]·dỸ[key][d]: A = a (k order permuted to the accumulator's rows)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 wa = frag_ks_perm(&sA[w][0], 16, 0, 16 * s);
        accX[0] = mfma32(wa, pack_acc(dK, s), accX[0]);
        accX[1] = mfma32(wa, pack_acc(dV, s), accX[1]);
      }
      // dQ_b = dS̃·P'_K + (dS̃·a)·T_K from the wave's own slab and a rows
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      bf16x8 ts[2];
      f32x16 G = f32x16{};  // Gᵀ: rows = j, columns = q
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        ts[s] = frag_ks(tS, PLD, 0, 16 * s);
        G = mfma32(frag_ks(&sA[w][0], 16, 0, 16 * s), ts[s], G);
      }
      if constexpr (QB) {
        f32x16 dq = mfma32(ts[0], frag_ks(&sP[w][0], PPL, 0, 0), f32x16{});
        dq = mfma32(ts[1], frag_ks(&sP[w][0], PPL, 0, 16), dq);
        dq = mfma32(pack_acc(G, 0), tq, dq);
        // partial [d][q]: registers 4g..4g+3 are 4 consecutive queries → one 16-byte store
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(&sDQb[cur][w][r * 36 + 8 * g + 4 * hh]) =
              f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
      } else {
        accQ = mfma32(ts[0], frag_ks(&sP[w][0], PPL, 0, 0), accQ);
        accQ = mfma32(ts[1], frag_ks(&sP[w][0], PPL, 0, 16), accQ);
        accQ = mfma32(pack_acc(G, 0), tq, accQ);
      }
      lds_barrier();
    };
    if (masked) {  // two loops: one register assignment each (no copies at a merged loop head)
      for (int jb = 0; jb < nb; ++jb) body(jb, std::true_type{});
    } else {
      for (int jb = 0; jb < nb; ++jb) body(jb, std::false_type{});
    }
    if constexpr (QB) {
      if (nb > 0) dq_reduce(nb - 1);  // the last sample's partials (after its barrier)
    }

    // ---- D rows of this wave's keys (K part columns 32h + r, V part C + 32h + r)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = kbase + 32 * w + acc_row(i, hh);
      if (m < a.M) {
        float* dk = a.D + (long long)m * O + h * PD + r;
        float* dv = dk + C;
        const float vk = accD[0][i] * a.scale, vv = accD[1][i];
        if (side >= 0) {
          float* sd = a.Dside + ((long long)side * KB + m - kbase) * 64 + r;
          sd[0] = vk;
          sd[PD] = vv;
        } else if (a.d_atomic) {
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
    // ---- dQ and column sums: per-wave partials through LDS (aliases of the consumed tiles)
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
    // partial segments in attn_bwd_pe_kernel's order: 0 ↔ Σ dY (W row NC + 1 = 1),
    // 1 ↔ Σ dY·μrσ (W row NC), 2 + c ↔ Σ dY·x̂_c (W row c)
    constexpr int nseg = 2 + NC;
    for (int e = threadIdx.x; e < 2 * nseg * 32; e += NTH) {
      const int p = e / (nseg * 32), rem = e % (nseg * 32), seg = rem / 32, j = rem % 32;
      const int wrow = seg == 0 ? NC + 1 : (seg == 1 ? NC : seg - 2);
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) v += sCS[ww][p][wrow][j];
      if (p == 0) v *= a.scale;
      float* dst = a.part + prow * (long long)(nseg * O) + (long long)seg * O + p * C + h * PD + j;
      *dst = a.accumulate ? *dst + v : v;
    }
  }  // runs
}

// D[pair rows] += Dside[slot] for every slot holding a leading partial run (persistent mode)
__global__ __launch_bounds__(256) void attn_pe_side_add_kernel(const float* __restrict__ Dside,
                                                               const int* __restrict__ side_pair, float* __restrict__ D,
                                                               int M, int H, int C) {
  const int pair = side_pair[blockIdx.x];
  if (pair < 0) return;
  const int kb = pair / H, h = pair % H;
  const float4* src = reinterpret_cast<const float4*>(Dside + (long long)blockIdx.x * 256 * 64);
  // 16 float4 per thread in two batches of 8 (all loads of a batch in flight before the adds)
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    float4 s[8], d[8];
    float* dp[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e4 = threadIdx.x + 256 * (8 * half + i), k = e4 >> 4, c = (e4 & 15) * 4, m = kb * 256 + k;
      dp[i] = m < M ? D + (long long)m * 2 * C + (c < PD ? h * PD + c : C + h * PD + c - PD) : nullptr;
      s[i] = src[e4];
      if (dp[i]) d[i] = *reinterpret_cast<const float4*>(dp[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (dp[i])
        *reinterpret_cast<float4*>(dp[i]) = make_float4(d[i].x + s[i].x, d[i].y + s[i].y, d[i].z + s[i].z, d[i].w + s[i].w);
  }
}

void attn_bwd_pe_launch(const PeBwdArgs& a0, int nkb, int bsplit, hipStream_t st) {
  PeBwdArgs a = a0;
  constexpr int NW = 8;
  dim3 grid(nkb, a.H, bsplit);
  if (a.nbg > 0) {  // persistent: a.nslots workgroups, batch groups of bper
    a.bper = (a.B + a.nbg - 1) / a.nbg;
    a.d_atomic = 0;
    grid = dim3((unsigned)a.nslots, 1, 1);
  } else {
    a.bper = (a.B + bsplit - 1) / bsplit;
    a.d_atomic = bsplit > 1 ? 1 : 0;
  }
  if (a.P) {  // implicit K/V: the factored kernel
#define PIO_PEBF(NC_)                                                                                      \
  if (a.q_bs == 0) hipLaunchKernelGGL((attn_bwd_pe_fact_kernel<NC_, false>), grid, dim3(64 * NW), 0, st, a); \
  else hipLaunchKernelGGL((attn_bwd_pe_fact_kernel<NC_, true>), grid, dim3(64 * NW), 0, st, a)
    switch (a.nc) {
      case 1: PIO_PEBF(1); break;
      case 2: PIO_PEBF(2); break;
      case 3: PIO_PEBF(3); break;
      default: PIO_PEBF(4); break;
    }
#undef PIO_PEBF
  } else {
    if (a.q_bs == 0) hipLaunchKernelGGL((attn_bwd_pe_kernel<NW, false>), grid, dim3(64 * NW), 0, st, a);
    else hipLaunchKernelGGL((attn_bwd_pe_kernel<NW, true>), grid, dim3(64 * NW), 0, st, a);
  }
  if (a.nbg > 0)
    hipLaunchKernelGGL(attn_pe_side_add_kernel, dim3((unsigned)a.nslots), dim3(256), 0, st, a.Dside, a.side_pair, a.D, a.M,
                       a.H, a.C);
}

// key splits of one launch: about one round of workgroups (2 per CU) of the factored kernel.  (A
// floor of 6 key chunks per split ran MNIST's forward 22.5 → 19.5 µs but moved the 4-sample
// 28×28 classifier test's decoder query-LN gradient — an ill-conditioned tensor — past its
// bf16 floor: not kept, profiles/r6_ab/README.md)
int attn_fwd_pe_auto_splits(int B, int H, int ncu) {
  constexpr int ns = 2;  // samples per wave (3 measured equal, 4 spills at 2 waves / SIMD)
  const int bg = (B + 4 * ns - 1) / (4 * ns);
  return std::max(1, 2 * ncu / (bg * H));
}

// splits × 32-key chunks covering M keys; grid (batch groups, splits, heads), 4 waves each
void attn_fwd_pe_launch(const PeFwdArgs& a0, hipStream_t st) {
  PeFwdArgs a = a0;
  const int nch = (a.M + 31) / 32;
  a.chunks = (nch + a.nsplit - 1) / a.nsplit;
  constexpr int ns = 2;
  const dim3 grid((unsigned)((a.B + 4 * ns - 1) / (4 * ns)), (unsigned)a.nsplit, (unsigned)a.H);
#define PIO_PEFF(NC_) hipLaunchKernelGGL((attn_fwd_pe_fact_kernel<NC_, ns>), grid, dim3(256), 0, st, a)
  switch (a.nc) {
    case 1: PIO_PEFF(1); break;
    case 2: PIO_PEFF(2); break;
    case 3: PIO_PEFF(3); break;
    default: PIO_PEFF(4); break;
  }
#undef PIO_PEFF
}

}  // namespace pio
