// Flash-style multi-head attention for the Perceiver's asymmetric shapes (CDNA4 / gfx950).
//
// Replaces nn.MultiheadAttention's unfused core (reference perceiver/model.py:59-74,
// SURVEY K-07/K-08): QK^T → key-padding mask → softmax → dropout → PV, never
// materialising P.  One kernel family serves all three Perceiver attentions:
//   * encoder cross-attention: few latent queries × many inputs (split-KV over the grid)
//   * latent self-attention:   N × N, N ≤ 512
//   * decoder cross-attention: many output queries × few latents (q batch-stride 0
//     lets the batch-independent output-query projection be computed once)
//
// Layouts (element strides, bf16): X[b, n, h*D + j] at X + b*bstride + n*rstride + h*D + j,
// so Q/K/V can be column slices of packed projection outputs.  O is (B, Nq, H*D) bf16,
// LSE / delta are (B, Nq, H) fp32 in log2 units (scores are pre-multiplied by
// scale*log2(e) so every exponential is a native v_exp_f32 = exp2).
//
// Forward, per wave: 32 queries.  S^T = K·Q^T (v_mfma_f32_32x32x16_bf16: keys on the
// accumulator rows, the query on the lane) so the softmax max/sum over keys is
// in-register + one lane^32 exchange, and P^T feeds O^T += V^T·P^T straight from the
// accumulator registers (no LDS round trip for P).  V^T fragments come from the LDS V
// tile with ds_read_b64_tr_b16 (hardware transpose).
//
// Backward, per workgroup: 128 keys (32 per wave), sweeping every query tile:
//   S = Q·K^T, dP = dO·V^T (query rows in registers, key on the lane),
//   dV += P^T·dO and dK += dS^T·Q from the accumulators (transpose reads of the LDS Q/dO
//   tiles), dQ via one LDS transpose of dS, summed over the waves in LDS; a single key block
//   (Nk ≤ 256 for d ≤ 32) stores dQ outright, several add with fp32 atomics.
// Both directions stage the next K/V (forward) or Q/dO (backward) tile in registers while
// the current tile's MFMAs run, so global latency is paid once per kernel, not per tile.
// Fully-masked query rows produce O = 0 and zero gradients (defect D10 defined).
#include "common.h"

namespace pio {

constexpr int KT = 64;  // keys per forward tile

struct AttnArgs {
  const uint16_t* q; long long q_bs; int q_rs;
  const uint16_t* k; long long k_bs; int k_rs;
  const uint16_t* v; long long v_bs; int v_rs;
  const uint8_t* kmask;  // (B, Nk), nonzero = padding key; may be null
  int B, H, Nq, Nk;
  float scale_log2;      // softmax scale * log2(e)
  float scale;           // softmax scale (backward)
  uint32_t drop_thresh;  // dropout probability * 2^32 (0 = off)
  float drop_scale;      // 1 / (1 - p)
  const int64_t* seedp;  // device seed of the call (common.h DropCfg); read only when drop_thresh
  uint32_t site;
};

// ------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------
template <int D, int NWV>
__global__ __launch_bounds__(64 * NWV) void attn_fwd_kernel(AttnArgs a, uint16_t* __restrict__ O,
                                                            float* __restrict__ LSE, float* __restrict__ Opart,
                                                            float* __restrict__ MLpart, int nsplit,
                                                            int tiles_per_split) {
  constexpr int LDK = D + 8;                 // K tile [key][d], 16-B padded rows
  constexpr int LDV = (D < 32 ? 32 : D) + 8;  // V tile [key][d]; D=16 zero-padded to 32 columns
  constexpr int NT = (D < 32) ? 1 : D / 32;   // O^T tiles of 32 rows (head-dim)
  constexpr int KS = D / 16;                  // k-steps for QK^T
  constexpr int CH = D / 8;                   // 16-byte chunks per K/V row
  constexpr int NTH = 64 * NWV;
  // keys are staged in rounds of NST 64-key tiles (≤ 4 16-byte chunks per thread per tensor),
  // the next round register-prefetched while this round's tiles are processed
  constexpr int NST0 = 4 * NTH / (KT * CH);
  constexpr int NST = NST0 >= 4 ? 4 : (NST0 >= 1 ? NST0 : 1);
  constexpr int NI = (NST * KT * CH + NTH - 1) / NTH;
  constexpr bool PF = NI <= 4;
  __shared__ __attribute__((aligned(16))) uint16_t sK[NST * KT * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t sV[NST * KT * LDV + 64];

  const int w = wave_id(), l = lane_id(), r = l & 31, hh = l >> 5;
  const Blk3 blk = xcd_block3();  // the heads / q-blocks / splits of one batch element share an L2
  const int h = blk.y;
  const int b = blk.z / nsplit, split = blk.z % nsplit;
  const int q0 = (blk.x * NWV + w) * 32;
  const int qi = q0 + r;
  const uint32_t dkey = a.drop_thresh ? drop_key(a.seedp, a.site, 2u) : 0u;
  const int qc = qi < a.Nq ? qi : a.Nq - 1;

  // this wave's Q^T operand fragments (B operand: B[k=d][col=query])
  bf16x8 qf[KS];
  {
    const uint16_t* qp = a.q + (long long)b * a.q_bs + (long long)qc * a.q_rs + h * D + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qp + 16 * s);
  }

  // D = 16: head-dim columns 16..31 of the V tiles (O^T rows 16..31) are padding.  Without
  // dropout they hold ones, so those O^T rows accumulate the softmax denominator Σ_k P (no
  // per-element VALU sum); with dropout zeros (the denominator is over the undropped P)
  const bool ones_den = D < 32 && !a.drop_thresh;
  if (D < 32) {
    const short pv = ones_den ? (short)0x3F80 : (short)0;  // bf16 1.0 / 0
    const bf16x8 pad8 = {pv, pv, pv, pv, pv, pv, pv, pv};
    for (int i = threadIdx.x; i < NST * KT; i += NTH)
      *reinterpret_cast<bf16x8*>(sV + i * LDV + 16) = pad8, *reinterpret_cast<bf16x8*>(sV + i * LDV + 24) = pad8;
  }

  f32x16 o[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) o[t] = f32x16{};
  float m_run = -1e30f, l_run = 0.f;

  const int ntiles = (a.Nk + KT - 1) / KT;
  const int t_begin = split * tiles_per_split;
  const int t_end = min(ntiles, t_begin + tiles_per_split);
  const int k_end = min(a.Nk, t_end * KT);  // keys of this split
  const uint16_t* kb = a.k + (long long)b * a.k_bs + h * D;
  const uint16_t* vb = a.v + (long long)b * a.v_bs + h * D;

  // staging: items c = tid + NTH·i of the round's NST·KT × CH 16-byte chunks
  bf16x8 kreg[PF ? NI : 1], vreg[PF ? NI : 1];
  bool pad_next[NST];
  // branch-free fetches (see kZero32B): out-of-range keys read zeros, the mask byte of a
  // key outside the split / without a mask reads a zero byte and is then overridden
  const unsigned char* zb = reinterpret_cast<const unsigned char*>(kZero32B);
  const unsigned char* kmb = a.kmask ? a.kmask + (long long)b * a.Nk : nullptr;
  auto fetch_pad = [&](int key0) {
    if (kmb == nullptr) {  // wave-uniform: no mask, no loads
#pragma unroll
      for (int j = 0; j < NST; ++j) pad_next[j] = key0 + j * KT + l >= k_end;
      return;
    }
#pragma unroll
    for (int j = 0; j < NST; ++j) {
      const int key = key0 + j * KT + l;
      const bool in = key < k_end;
      const unsigned char mv = *(in ? kmb + key : zb);  // unconditional load (address select)
      pad_next[j] = (mv != 0) | !in;                      // bitwise: no short-circuit branch
    }
  };
  auto fetch = [&](int key0) {
#pragma unroll
    for (int i = 0; i < (PF ? NI : 1); ++i) {
      const int c = threadIdx.x + NTH * i, key = key0 + c / CH, col = (c % CH) * 8;
      const bool ok = c < NST * KT * CH && key < k_end;
      const uint16_t* kp = ok ? kb + (long long)key * a.k_rs + col : reinterpret_cast<const uint16_t*>(kZero32B);
      const uint16_t* vp = ok ? vb + (long long)key * a.v_rs + col : reinterpret_cast<const uint16_t*>(kZero32B);
      kreg[i] = *reinterpret_cast<const bf16x8*>(kp);
      vreg[i] = *reinterpret_cast<const bf16x8*>(vp);
    }
    fetch_pad(key0);
  };
  // unconditional prefetches (rows past the split read zeros): a load inside a branch makes the
  // compiler drain every outstanding load (vmcnt(0)) before it, serialising the prologue
  if constexpr (PF) fetch(t_begin * KT);

  for (int t0 = t_begin; t0 < t_end; t0 += NST) {
    const int rkey0 = t0 * KT;
    lds_sync();
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int c = threadIdx.x + NTH * i, kr = c / CH, col = (c % CH) * 8;
        if (c < NST * KT * CH) {
          *reinterpret_cast<bf16x8*>(sK + kr * LDK + col) = kreg[i];
          *reinterpret_cast<bf16x8*>(sV + kr * LDV + col) = vreg[i];
        }
      }
    } else {
      for (int c = threadIdx.x; c < NST * KT * CH; c += NTH) {
        const int kr = c / CH, col = (c % CH) * 8, key = rkey0 + kr;
        bf16x8 kv = bf16x8{0, 0, 0, 0, 0, 0, 0, 0}, vv = kv;
        if (key < k_end) {
          kv = *reinterpret_cast<const bf16x8*>(kb + (long long)key * a.k_rs + col);
          vv = *reinterpret_cast<const bf16x8*>(vb + (long long)key * a.v_rs + col);
        }
        *reinterpret_cast<bf16x8*>(sK + kr * LDK + col) = kv;
        *reinterpret_cast<bf16x8*>(sV + kr * LDV + col) = vv;
      }
      fetch_pad(rkey0);
    }
    // key-padding bits per tile of the round (bit i = key is padding or outside the split)
    uint64_t padbits[NST];
#pragma unroll
    for (int j = 0; j < NST; ++j) padbits[j] = __ballot(pad_next[j]);
    lds_sync();
    if constexpr (PF) fetch((t0 + NST) * KT);  // past the last round: zeros, never used

#pragma unroll
    for (int j = 0; j < NST; ++j) {
      if (t0 + j >= t_end) break;
      const int key0 = (t0 + j) * KT;
      const uint16_t* tK = sK + j * KT * LDK;
      const uint16_t* tV = sV + j * KT * LDV;
      f32x16 s[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        s[kh] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[kh] = mfma32(frag_kc(tK, LDK, 32 * kh, 16 * ks), qf[ks], s[kh]);
      }
      // mask (only tiles that hold padding keys) and tile max on the RAW scores (the scale is
      // positive), then one fma + exp2 per score: p = 2^(s·scale·log2e − m)
      float mt = -INFINITY;
      if (padbits[j] == 0ull) {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 16; ++i) mt = fmaxf(mt, s[kh][i]);
      } else {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          // bits of this lane-half's 16 accumulator rows: row = 32kh + (i&3) + 8(i>>2) + 4hh
          const uint32_t word = (uint32_t)(padbits[j] >> (32 * kh)) >> (4 * hh);
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float v = ((word >> ((i & 3) + 8 * (i >> 2))) & 1u) ? -INFINITY : s[kh][i];
            s[kh][i] = v;
            mt = fmaxf(mt, v);
          }
        }
      }
      mt = xor32_max(mt);
      const float m_new = fmaxf(m_run, mt * a.scale_log2);
      const float alpha = fast_exp2(m_run - m_new);
      m_run = m_new;
      float ls = 0.f;
      if (ones_den) {  // wave-uniform; the denominator comes out of the P·V product
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 16; ++i) s[kh][i] = fast_exp2(fmaf(s[kh][i], a.scale_log2, -m_new));
      } else {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            s[kh][i] = fast_exp2(fmaf(s[kh][i], a.scale_log2, -m_new));
            ls += s[kh][i];
          }
      }
      if (a.drop_thresh) {  // uniform: the element loop above stays branch-free
        // element index qi·Nk + key0 + 4hh + (32kh + acc_row(i, 0)): base product once (keep_elem_m)
        uint32_t cm0 = ((uint32_t)qi * (uint32_t)a.Nk + (uint32_t)(key0 + 4 * hh)) * kHashM1;
        asm volatile("" : "+v"(cm0));
        const uint32_t hs = hash3_seed(dkey, (uint32_t)(b * a.H + h));
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const uint32_t cm = cm0 + (uint32_t)(32 * kh + acc_row(i, 0)) * kHashM1;
            s[kh][i] = keep_elem_m(hs, cm, a.drop_thresh) ? s[kh][i] * a.drop_scale : 0.f;
          }
      }
      l_run = l_run * alpha + ls;
#pragma unroll
      for (int t2 = 0; t2 < NT; ++t2)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[t2][i] *= alpha;
      // O^T += V^T · P^T
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const bf16x8 pb = pack_acc(s[kh], ss);
#pragma unroll
          for (int t2 = 0; t2 < NT; ++t2)
            o[t2] = mfma32(frag_ks_perm(tV, LDV, 32 * t2, 32 * kh + 16 * ss), pb, o[t2]);
        }
    }
  }

  // O^T row 16 (a ones row when ones_den) = Σ_k P of this lane's query, complete in every lane
  const float l_tot = ones_den ? o[0][8] : xor32_sum(l_run);
  if (qi >= a.Nq) return;
  const int HD = a.H * D;
  if (nsplit == 1) {
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    uint16_t* op = O + ((long long)b * a.Nq + qi) * HD + h * D;
#pragma unroll
    for (int t2 = 0; t2 < NT; ++t2)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * t2 + 8 * g + 4 * hh;
        if (dd < D) {
          uint2 pk;
          pk.x = pack2(o[t2][4 * g] * inv, o[t2][4 * g + 1] * inv);
          pk.y = pack2(o[t2][4 * g + 2] * inv, o[t2][4 * g + 3] * inv);
          *reinterpret_cast<uint2*>(op + dd) = pk;
        }
      }
    if (hh == 0) LSE[((long long)b * a.Nq + qi) * a.H + h] = l_tot > 0.f ? m_run + __log2f(l_tot) : INFINITY;
  } else {
    // unnormalised partials: Opart[split][b][q][h][D], MLpart[split][b][q][h][2]
    const long long row = (((long long)split * a.B + b) * a.Nq + qi) * a.H + h;
    float* op = Opart + row * D;
#pragma unroll
    for (int t2 = 0; t2 < NT; ++t2)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * t2 + 8 * g + 4 * hh;
        if (dd < D)
          *reinterpret_cast<float4*>(op + dd) = make_float4(o[t2][4 * g], o[t2][4 * g + 1], o[t2][4 * g + 2], o[t2][4 * g + 3]);
      }
    if (hh == 0) {
      MLpart[row * 2] = m_run;
      MLpart[row * 2 + 1] = l_tot;
    }
  }
}

// combine split-KV partials: one thread per (b, q, h, d).  One online pass over the splits, four
// at a time with their twelve loads independent (a two-pass loop of dependent loads is latency
// bound: 21 µs for 32 splits at the ImageNet encoder shape)
__global__ void attn_combine_kernel(const float* __restrict__ Opart, const float* __restrict__ MLpart,
                                    uint16_t* __restrict__ O, float* __restrict__ LSE, int nsplit, int rows, int D) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)rows * D) return;
  const long long row = idx / D;
  const int d = idx % D;
  const long long sstride = (long long)rows;
  float M = -1e30f, L = 0.f, acc = 0.f;
  int s = 0;
  for (; s + 4 <= nsplit; s += 4) {
    float m[4], l[4], o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long r = (s + j) * sstride + row;
      m[j] = MLpart[r * 2];
      l[j] = MLpart[r * 2 + 1];
      o[j] = Opart[r * D + d];
    }
    const float mx = fmaxf(fmaxf(M, fmaxf(m[0], m[1])), fmaxf(m[2], m[3]));
    const float sc = exp2f(M - mx);
    L *= sc;
    acc *= sc;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float w = exp2f(m[j] - mx);
      L = fmaf(l[j], w, L);
      acc = fmaf(o[j], w, acc);
    }
    M = mx;
  }
  for (; s < nsplit; ++s) {
    const long long r = s * sstride + row;
    const float m = MLpart[r * 2];
    const float mx = fmaxf(M, m);
    const float sc = exp2f(M - mx), w = exp2f(m - mx);
    L = fmaf(MLpart[r * 2 + 1], w, L * sc);
    acc = fmaf(Opart[r * D + d], w, acc * sc);
    M = mx;
  }
  O[row * D + d] = f2bf(L > 0.f ? acc / L : 0.f);  // rows ordered (b, q, h) → O[(b*Nq+q)*HD + h*D + d]
  if (d == 0) LSE[row] = L > 0.f ? M + __log2f(L) : INFINITY;
}

// ------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------
// delta[b, q, h] = sum_d dO * O (fp32), and zero dQ accumulator rows
__global__ void attn_bwd_prep_kernel(const uint16_t* __restrict__ dO, const uint16_t* __restrict__ O,
                                     float* __restrict__ delta, float* __restrict__ dq, int rows, int H, int D,
                                     int dq_rs) {
  const int row = blockIdx.x * (blockDim.x >> 6) + wave_id();
  if (row >= rows) return;
  const int l = lane_id();
  const int HD = H * D;
  for (int h = 0; h < H; ++h) {
    float acc = 0.f;
    for (int d = l; d < D; d += 64) acc += bf2f(dO[(long long)row * HD + h * D + d]) * bf2f(O[(long long)row * HD + h * D + d]);
    acc = wave_sum(acc);
    if (l == 0) delta[(long long)row * H + h] = acc;
  }
  if (dq)
    for (int j = l; j < HD; j += 64) dq[(long long)row * dq_rs + j] = 0.f;
}

// QR > 0 fixes the query tiles per round (QR = 1 for ≤ 32 queries, 2 for ≤ 64: a quarter / half
// of the LDS, so several workgroups share a CU on the few-query / many-key cross-attention)
// OBF: dQ / dK / dV stored as bf16 (the pointers are uint16_t views; every element written once:
// a single key block, no query split, no accumulation — host-checked), for a consumer that reads
// them as bf16 MFMA operands anyway (the chain-layout layer-boundary backward)
// KM = false: no key padding mask and every key of the grid's blocks exists (Nk a multiple of the
// block's keys): no per-element masking select in the softmax
// DRP = false: no attention-probability dropout compiled in (host-checked), for the register
// budget of the slab-carrying variant (≤ 128 VGPRs: two 8-wave workgroups per CU)
template <int D, int NW, int QR = 0, bool OBF = false, bool KM = true, bool DRP = true>
__global__ __launch_bounds__(64 * NW, (QR == 2 && !DRP) ? 4 : 1) void attn_bwd_kernel(AttnArgs a, const uint16_t* __restrict__ dO,
                                                           const float* __restrict__ LSE,
                                                           const float* __restrict__ delta, float* __restrict__ dq,
                                                           long long dq_bs, int dq_rs, float* __restrict__ dk,
                                                           long long dk_bs, int dk_rs, float* __restrict__ dv,
                                                           long long dv_bs, int dv_rs, int dq_atomic, int kv_acc,
                                                           long long dq_kbs, int nqs, int q_tiles_per_split,
                                                           SlabJob job) {
  constexpr int LD = (D < 32 ? 32 : D) + 8;  // Q / dO / K tiles [row][d] (D=16 zero-padded to 32 cols)
  constexpr int NT = (D < 32) ? 1 : D / 32;
  constexpr int KS = D / 16;
  constexpr int LDS_ = 40;                   // dS tiles [key][q] (32 q + pad)
  constexpr int KB = 32 * NW;                // keys per workgroup
  constexpr int NTH = 64 * NW, CH = D / 8;
  // queries in rounds of NQS 32-query tiles (≤ 4 16-byte chunks of Q + dO per thread), the
  // next round register-prefetched.  Every wave writes its dS slab of each tile into LDS;
  // after one barrier wave j (< NQS) forms tile j's dQ over all KB keys of the block with
  // MFMAs (no cross-wave reduction, no atomics inside the block).
  // (the generic dQ step below gives one query tile per wave: at most NW tiles per round)
  constexpr int NQS0 = 4 * NTH / (64 * CH);
  constexpr int NQS1 = NQS0 >= 4 ? 4 : (NQS0 >= 1 ? NQS0 : 1);
  constexpr int NQS = QR > 0 ? QR : (NQS1 < NW ? NQS1 : NW);
  static_assert(NQS <= NW || (D == 16 && NW == 8), "one dQ query tile per wave");
  constexpr int NI = (NQS * 64 * CH + NTH - 1) / NTH;
  __shared__ __attribute__((aligned(16))) uint16_t sQ[NQS * 32 * LD + 64];
  __shared__ __attribute__((aligned(16))) uint16_t sdO[NQS * 32 * LD + 64];
  __shared__ __attribute__((aligned(16))) uint16_t sK[KB * LD + 64];
  __shared__ __attribute__((aligned(16))) uint16_t sdS[NQS * KB * LDS_];
  __shared__ __attribute__((aligned(16))) float sL[NQS * 32];
  __shared__ __attribute__((aligned(16))) float sDl[NQS * 32];

  PIO_WG_BEGIN();
  if ((int)blockIdx.z >= a.B) {  // z-slices past the batch: the previous kernel's slab job
    const int jb = ((blockIdx.z - a.B) * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (jb < job.nblk) slab_reduce_block(job, jb, reinterpret_cast<float4*>(sdS));
    PIO_WG_END();
    return;
  }
  PIO_TS(0);
  const int w = wave_id(), l = lane_id(), r = l & 31, hh = l >> 5;
  const Blk3 blk = xcd_block3(a.B);  // the heads / key blocks of one batch element share an L2
  const int h = blk.y, b = blk.z;
  // blk.x = key block × nqs + query split: many-query / few-key shapes (a decoder's pixel or
  // token queries over a few dozen latents) split the query range across workgroups, whose
  // dK / dV partials are added atomically (the host zeroes dK / dV first unless accumulating)
  const int kblk = blk.x / nqs, qsplit = blk.x - kblk * nqs;
  const int kbase = kblk * KB;
  dq += (long long)kblk * dq_kbs;  // deterministic mode: one dQ partial slice per key block
  const int key = kbase + 32 * w + r;  // this lane's key (column of S / dP)
  const int kc = key < a.Nk ? key : a.Nk - 1;
  const uint32_t dkey = DRP && a.drop_thresh ? drop_key(a.seedp, a.site, 2u) : 0u;
  const bool kin = key < a.Nk;
  bool kpad = false;
  if constexpr (KM) {
    const unsigned char* kmp = (a.kmask && kin) ? a.kmask + (long long)b * a.Nk + key
                                                : reinterpret_cast<const unsigned char*>(kZero32B);
    const unsigned char kmv = *kmp;  // unconditional load (address select)
    kpad = (kmv != 0) | !kin;
  }

  const int HD = a.H * D;
  // 16-byte output rows possible (fp32 dQ / dK / dV views 16-byte aligned)
  const bool vec_out = ((((uintptr_t)dq | (uintptr_t)dk | (uintptr_t)dv) & 15) == 0) &&
                       (((dq_bs | dk_bs | dv_bs) & 3) == 0) && (((dq_rs | dk_rs | dv_rs) & 3) == 0);
  const uint16_t* kbp = a.k + (long long)b * a.k_bs + h * D;
  const uint16_t* vbp = a.v + (long long)b * a.v_bs + h * D;
  const uint16_t* qbp = a.q + (long long)b * a.q_bs + h * D;
  const uint16_t* dobp = dO + (long long)b * a.Nq * HD + h * D;
  const int nqt_all = (a.Nq + 31) / 32;
  const int qt_begin = qsplit * q_tiles_per_split;
  const int nqt = min(nqt_all, qt_begin + q_tiles_per_split);  // end of this split's query tiles

  // round staging: chunk c < NQS·32·CH is Q, the next NQS·32·CH are dO; threads [0, NQS·32)
  // carry the round's LSE, [NQS·32, NQS·64) its delta
  bf16x8 qreg[NI];
  float lreg = 0.f;
  bool lq_out = false;
  // branch-free fetches (see kZero32B): out-of-range rows read zeros; the LSE of a query past
  // Nq is forced to +inf after the (unconditional) load
  auto fetch = [&](int qt0) {
    const int q00 = qt0 * 32;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int c = threadIdx.x + NTH * i, isdo = c >= NQS * 32 * CH, cc = isdo ? c - NQS * 32 * CH : c;
      const int qq = q00 + cc / CH, col = (cc % CH) * 8;
      const bool ok = c < NQS * 64 * CH && qq < a.Nq;
      const uint16_t* p = !ok ? reinterpret_cast<const uint16_t*>(kZero32B)
                              : (isdo ? dobp + (long long)qq * HD + col : qbp + (long long)qq * a.q_rs + col);
      qreg[i] = *reinterpret_cast<const bf16x8*>(p);
    }
    {
      const int t = threadIdx.x < NQS * 64 ? threadIdx.x : 0;
      const int isd = t >= NQS * 32, qq = q00 + (isd ? t - NQS * 32 : t);
      const long long idx = ((long long)b * a.Nq + qq) * a.H + h;
      const bool ok = qq < a.Nq;
      lreg = *(!ok ? kZero32B : (isd ? delta + idx : LSE + idx));
      lq_out = !ok && !isd;  // LSE of a missing query: +inf (set when the value is stored)
    }
  };
  // every prologue load is issued before the first wait: this wave's K^T / V^T operand
  // fragments (B[k=d][col=key]; the K ones also fill the block's LDS K tile for dQ), the
  // first query round
  bf16x8 kf[KS], vf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(kbp + (long long)kc * a.k_rs + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const bf16x8*>(vbp + (long long)kc * a.v_rs + 16 * s + 8 * hh);
  }
  fetch(qt_begin);  // unconditional (see the forward): out-of-range query rows read zeros
  if (D < 32) {  // zero the padded head-dim columns 16..31
    for (int i = threadIdx.x; i < KB; i += NTH) {
      *reinterpret_cast<bf16x8*>(sK + i * LD + 16) = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      *reinterpret_cast<bf16x8*>(sK + i * LD + 24) = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    for (int i = threadIdx.x; i < NQS * 32; i += NTH) {
      *reinterpret_cast<bf16x8*>(sQ + i * LD + 16) = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      *reinterpret_cast<bf16x8*>(sQ + i * LD + 24) = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      *reinterpret_cast<bf16x8*>(sdO + i * LD + 16) = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      *reinterpret_cast<bf16x8*>(sdO + i * LD + 24) = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  // the block's K tile (for dQ) from this wave's own K fragments: no second global read of K
  // (keys past Nk hold the clamped last key — finite, and their dS is zero)
#pragma unroll
  for (int s2 = 0; s2 < KS; ++s2)
    *reinterpret_cast<bf16x8*>(sK + (32 * w + r) * LD + 16 * s2 + 8 * hh) = kf[s2];
  f32x16 dK[NT], dV[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) dK[t] = dV[t] = f32x16{};
  PIO_TS(1);

  for (int qt0 = qt_begin; qt0 < nqt; qt0 += NQS) {
    lds_sync();  // the previous round's tiles and dS slabs are consumed
    if (qt0 == qt_begin) PIO_TS(30);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int c = threadIdx.x + NTH * i, isdo = c >= NQS * 32 * CH, cc = isdo ? c - NQS * 32 * CH : c;
      if (c < NQS * 64 * CH) *reinterpret_cast<bf16x8*>((isdo ? sdO : sQ) + (cc / CH) * LD + (cc % CH) * 8) = qreg[i];
    }
    if (qt0 == qt_begin) PIO_TS(31);
    if (threadIdx.x < NQS * 32) sL[threadIdx.x] = lq_out ? INFINITY : lreg;
    else if (threadIdx.x < NQS * 64) sDl[threadIdx.x - NQS * 32] = lreg;
    if (qt0 == qt_begin) PIO_TS(32);
    lds_sync();
    PIO_TS(2 + 4 * ((qt0 - qt_begin) / NQS));
    fetch(qt0 + NQS);  // past the last round: zeros, never used

#pragma unroll
    for (int j = 0; j < NQS; ++j) {
      if (qt0 + j >= nqt) break;
      const int q0 = (qt0 + j) * 32;
      const uint16_t* tQ = sQ + j * 32 * LD;
      const uint16_t* tdO = sdO + j * 32 * LD;
      // S = Q K^T and dP = dO V^T  (rows: queries; lane: key)
      f32x16 S = f32x16{}, dP = f32x16{};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        S = mfma32(frag_kc(tQ, LD, 0, 16 * s), kf[s], S);
        dP = mfma32(frag_kc(tdO, LD, 0, 16 * s), vf[s], dP);
      }
      // LSE / delta of this lane's accumulator rows (registers 4g..4g+3 = tile rows
      // 8g + 4hh + 0..3): 8 vector LDS reads, then a branch-free element loop (a per-element
      // condition around an LDS read serialises the loop on LDS latency)
      f32x16 P, dS;
      if constexpr (!DRP) {  // register budget: the delta rows are read once P is formed
        f32x4 lr[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) lr[g] = *reinterpret_cast<const f32x4*>(sL + j * 32 + 8 * g + 4 * hh);
#pragma unroll
        for (int i = 0; i < 16; ++i) P[i] = fast_exp2(kpad ? -INFINITY : S[i] * a.scale_log2 - lr[i >> 2][i & 3]);
        asm volatile("" ::: "memory");
        f32x4 dr[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) dr[g] = *reinterpret_cast<const f32x4*>(sDl + j * 32 + 8 * g + 4 * hh);
#pragma unroll
        for (int i = 0; i < 16; ++i) dS[i] = P[i] * (dP[i] - dr[i >> 2][i & 3]);
      }
      f32x4 lrow[4], drow[4];
      if constexpr (DRP) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          lrow[g] = *reinterpret_cast<const f32x4*>(sL + j * 32 + 8 * g + 4 * hh);
          drow[g] = *reinterpret_cast<const f32x4*>(sDl + j * 32 + 8 * g + 4 * hh);
        }
      }
      if (!DRP) {
      } else if (!a.drop_thresh) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fast_exp2(kpad ? -INFINITY : S[i] * a.scale_log2 - lrow[i >> 2][i & 3]);
          P[i] = p;
          dS[i] = p * (dP[i] - drow[i >> 2][i & 3]);
        }
      } else {
        // Nk made opaque inside the dropout branch: the per-element index products cannot be
        // hoisted into the prologue of the dropout-free path
        uint32_t nk = (uint32_t)a.Nk;
        asm volatile("" : "+s"(nk));
        // element index (q0 + 4hh)·Nk + key + acc_row(i, 0)·Nk: base product once, the offsets'
        // products wave-uniform (keep_elem_m)
        uint32_t cm0 = ((uint32_t)(q0 + 4 * hh) * nk + (uint32_t)key) * kHashM1;
        asm volatile("" : "+v"(cm0));
        const uint32_t nkm = nk * kHashM1;
        const uint32_t hs = hash3_seed(dkey, (uint32_t)(b * a.H + h));
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fast_exp2(kpad ? -INFINITY : S[i] * a.scale_log2 - lrow[i >> 2][i & 3]);
          const bool keep = keep_elem_m(hs, cm0 + (uint32_t)acc_row(i, 0) * nkm, a.drop_thresh);
          P[i] = keep ? p * a.drop_scale : 0.f;
          dS[i] = p * ((keep ? dP[i] * a.drop_scale : 0.f) - drow[i >> 2][i & 3]);
        }
      }
      // dV += P^T dO ; dK += dS^T Q   (accumulator as A operand: X^T · B)
      bf16x8 sa[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const bf16x8 pa = pack_acc(P, ss);
        sa[ss] = pack_acc(dS, ss);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          dV[t] = mfma32(pa, frag_ks_perm(tdO, LD, 32 * t, 16 * ss), dV[t]);
          dK[t] = mfma32(sa[ss], frag_ks_perm(tQ, LD, 32 * t, 16 * ss), dK[t]);
        }
      }
      // dS slab of (this wave's 32 keys) × (tile j's 32 queries) as [key][q]: the packed dS
      // halves above (registers 4g .. 4g + 3 = queries 8g + 4hh .. + 3)
      uint16_t* slab = sdS + (j * KB + 32 * w) * LDS_;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const bf16x8& v = sa[g >> 1];
        const int o = 4 * (g & 1);
        const bf16x4 q4 = {v[o], v[o + 1], v[o + 2], v[o + 3]};
        *reinterpret_cast<bf16x4*>(slab + r * LDS_ + 8 * g + 4 * hh) = q4;
      }
    }
    PIO_TS(3 + 4 * ((qt0 - qt_begin) / NQS));
    lds_sync();
    PIO_TS(4 + 4 * ((qt0 - qt_begin) / NQS));
    // dQ of tile j = w: Σ over the block's keys of dS[key][q] · K[key][d]
    if constexpr (D == 16 && NW == 8 && (NQS == 4 || NQS == 2)) {
      // head width 16: a wave takes 16 queries (tile w % NQS, half w / NQS) × the 16 head dims
      // with 16x16x32 MFMAs over the KB keys — none of the 32x32 tile's padding columns (the
      // 32x32x16 form below computes 32 dims of which 16 are real); NQS = 4 leaves no wave idle
      const int j = w % NQS, mh = w / NQS, g = l >> 4;
      if (mh < 2 && qt0 + j < nqt) {
        const uint16_t* tS = sdS + j * KB * LDS_;
        f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k0 = 0; k0 < KB; k0 += 64) {
          a0 = mfma16(frag16_tr(tS, LDS_, 16 * mh, k0), frag16_tr(sK, LD, 0, k0), a0);
          a1 = mfma16(frag16_tr(tS, LDS_, 16 * mh, k0 + 32), frag16_tr(sK, LD, 0, k0 + 32), a1);
        }
        // accumulator: col = l & 15 = head dim, row = 4g + i = query within the 16
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qq = (qt0 + j) * 32 + 16 * mh + 4 * g + i;
          if (qq < a.Nq) {
            const long long di = (long long)b * dq_bs + (long long)qq * dq_rs + h * D + (l & 15);
            const float v = (a0[i] + a1[i]) * a.scale;
            if constexpr (OBF) reinterpret_cast<uint16_t*>(dq)[di] = f2bf(v);
            else if (dq_atomic) atomicAdd(dq + di, v);
            else dq[di] = v;
          }
        }
      }
    } else if (w < NQS && qt0 + w < nqt) {
      const uint16_t* tS = sdS + w * KB * LDS_;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        // all KB keys (slab rows / K rows past the block's keys are zero): unrolled, two
        // independent accumulation chains
        f32x16 dq_acc = f32x16{}, dq_acc2 = f32x16{};
#pragma unroll
        for (int k0 = 0; k0 < KB; k0 += 32) {
          dq_acc = mfma32(frag_ks(tS, LDS_, 0, k0), frag_ks(sK, LD, 32 * t, k0), dq_acc);
          dq_acc2 = mfma32(frag_ks(tS, LDS_, 0, k0 + 16), frag_ks(sK, LD, 32 * t, k0 + 16), dq_acc2);
        }
        dq_acc += dq_acc2;
        // accumulator: col = lane&31 = d, row = acc_row = query within the tile
        if (dq_atomic || !vec_out || D > 32) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int dd = 32 * t + r, qq = (qt0 + w) * 32 + acc_row(i, hh);
            if (dd < D && qq < a.Nq) {
              float* dst = dq + (long long)b * dq_bs + (long long)qq * dq_rs + h * D + dd;
              const float v = dq_acc[i] * a.scale;
              if (dq_atomic) atomicAdd(dst, v);
              else *dst = v;
            }
          }
        } else {
          // single key block: transpose through this wave's own (consumed) dS slab, then
          // 16-byte row stores
          float* sE = reinterpret_cast<float*>(sdS + w * KB * LDS_);
          constexpr int LDE = D + 4;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (r < D) sE[acc_row(i, hh) * LDE + r] = dq_acc[i] * a.scale;
          constexpr int CPR = D / 4;
#pragma unroll
          for (int c = l; c < 32 * CPR; c += 64) {
            const int qq = (qt0 + w) * 32 + c / CPR, col = (c % CPR) * 4;
            if (qq < a.Nq)
              *reinterpret_cast<float4*>(dq + (long long)b * dq_bs + (long long)qq * dq_rs + h * D + col) =
                  *reinterpret_cast<const float4*>(sE + (c / CPR) * LDE + col);
          }
        }
      }
    }
    PIO_TS(5 + 4 * ((qt0 - qt_begin) / NQS));
  }
  PIO_TS(40);
  // write dK (scaled) and dV: rows = keys (registers), lane = head-dim column
  // accumulator: col = lane&31 = d, row = acc_row(reg) = key within the wave's 32
  // (needs the dS slabs to hold both [KB][D + 4] fp32 tiles: not in the QR = 1 variant)
  if constexpr (D <= 32 && 2 * KB * (D + 4) * 4 <= NQS * KB * LDS_ * 2) {
    if (vec_out && nqs == 1) {  // transpose through LDS (the dS slabs are consumed), 16-byte row stores
      constexpr int LDE = D + 4, CPR = D / 4;
      float* sE = reinterpret_cast<float*>(sdS);  // [dK | dV][KB keys][LDE]
      lds_sync();
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (r < D) {
          const int kl = 32 * w + acc_row(i, hh);
          sE[kl * LDE + r] = dK[0][i] * a.scale;
          sE[(KB + kl) * LDE + r] = dV[0][i];
        }
      lds_sync();
#pragma unroll
      for (int c = threadIdx.x; c < 2 * KB * CPR; c += NTH) {
        const int isv = c >= KB * CPR, cc = isv ? c - KB * CPR : c;
        const int kl = cc / CPR, col = (cc % CPR) * 4, kk = kbase + kl;
        if (kk < a.Nk) {
          float4 v = *reinterpret_cast<const float4*>(sE + ((isv ? KB : 0) + kl) * LDE + col);
          const long long di = (isv ? (long long)b * dv_bs + (long long)kk * dv_rs
                                    : (long long)b * dk_bs + (long long)kk * dk_rs) + h * D + col;
          if constexpr (OBF) {
            uint2 pk;
            pk.x = pack2(v.x, v.y);
            pk.y = pack2(v.z, v.w);
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(isv ? dv : dk) + di) = pk;
            continue;
          }
          float* dst = (isv ? dv : dk) + di;
          if (kv_acc) {
            const float4 o = *reinterpret_cast<const float4*>(dst);
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *reinterpret_cast<float4*>(dst) = v;
        }
      }
      PIO_TS(41);
      PIO_WG_END();
      return;
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kk = kbase + 32 * w + acc_row(i, hh);
      const int dd = 32 * t + r;
      if (kk < a.Nk && dd < D) {
        // kv_acc: add onto earlier contributions (K/V shared by several applications, K-06)
        if constexpr (OBF) {
          reinterpret_cast<uint16_t*>(dk)[(long long)b * dk_bs + (long long)kk * dk_rs + h * D + dd] =
              f2bf(dK[t][i] * a.scale);
          reinterpret_cast<uint16_t*>(dv)[(long long)b * dv_bs + (long long)kk * dv_rs + h * D + dd] = f2bf(dV[t][i]);
          continue;
        }
        float* pk = dk + (long long)b * dk_bs + (long long)kk * dk_rs + h * D + dd;
        float* pv = dv + (long long)b * dv_bs + (long long)kk * dv_rs + h * D + dd;
        if (nqs > 1) {
          atomicAdd(pk, dK[t][i] * a.scale);
          atomicAdd(pv, dV[t][i]);
        } else {
          *pk = kv_acc ? *pk + dK[t][i] * a.scale : dK[t][i] * a.scale;
          *pv = kv_acc ? *pv + dV[t][i] : dV[t][i];
        }
      }
    }
  PIO_TS(41);
  PIO_WG_END();
}

// host ABI check (binding.cpp mirrors these structs)
int abi_struct_size(int which) {
  switch (which) {
    case 0: return (int)sizeof(DropCfg);
    case 1: return (int)sizeof(PostAttnGrads);
    case 2: return (int)sizeof(SlabJob);
    case 3: return (int)sizeof(AttnArgs);
    default: return -1;
  }
}

// zero rows of a strided fp32 (B, N, W) view (dQ accumulator when several key blocks add into it)
__global__ void zero_rows_kernel(float* __restrict__ p, long long bs, int rs, int N, int W, long long total) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long row = i / W;
    const int c = (int)(i - row * W);
    const long long bb = row / N;
    p[bb * bs + (row - bb * N) * rs + c] = 0.f;
  }
}

// ------------------------------------------------------------------------------------
// few-key decode attention backward (an image classifier's decoder: one query per sample over
// the 32 latents, head width 128): one wave per (sample, head), lane = key, VALU dot products —
// the MFMA kernels above spend most of such a call staging 32×32 tiles for one useful row
// (9.2 vs 17.6 µs at the ImageNet / MNIST decoders; the forward analogue was slower than the MFMA
// forward, 11.7 vs 10 µs, and is not built: profiles/r5_ab/README.md)
// ------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(64) void attn_decode_bwd_kernel(AttnArgs a, const uint16_t* __restrict__ dO,
                                                             const float* __restrict__ LSE,
                                                             const float* __restrict__ delta, float* __restrict__ dq,
                                                             long long dq_bs, int dq_rs, float* __restrict__ dk,
                                                             long long dk_bs, int dk_rs, float* __restrict__ dv,
                                                             long long dv_bs, int dv_rs, int kv_acc) {
  constexpr int DL = D / 64;
  __shared__ __attribute__((aligned(16))) float sq[D], sdo[D];
  const int l = threadIdx.x, h = blockIdx.y, b = blockIdx.x;
  const uint16_t* qp = a.q + (long long)b * a.q_bs + h * D;
  const uint16_t* dop = dO + (long long)b * a.H * D + h * D;
  float qv[DL], dov[DL];
#pragma unroll
  for (int i = 0; i < DL; ++i) {
    qv[i] = bf2f(qp[l + 64 * i]);
    dov[i] = bf2f(dop[l + 64 * i]);
    sq[l + 64 * i] = qv[i];
    sdo[l + 64 * i] = dov[i];
  }
  __syncthreads();
  const bool kv = l < a.Nk;
  const int key = kv ? l : 0;
  const uint16_t* kp = a.k + (long long)b * a.k_bs + (long long)key * a.k_rs + h * D;
  const uint16_t* vp = a.v + (long long)b * a.v_bs + (long long)key * a.v_rs + h * D;
  float s = 0.f, dp = 0.f;
#pragma unroll
  for (int c = 0; c < D / 8; ++c) {
    const bf16x8 k8 = *reinterpret_cast<const bf16x8*>(kp + 8 * c);
    const bf16x8 v8 = *reinterpret_cast<const bf16x8*>(vp + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s = fmaf(sq[8 * c + e], bf2f(k8[e]), s);
      dp = fmaf(sdo[8 * c + e], bf2f(v8[e]), dp);
    }
  }
  const long long row = (long long)b * a.H + h;
  const float p = kv ? exp2f(fmaf(s, a.scale_log2, -LSE[row])) : 0.f;
  const float ds = p * (dp - delta[row]);
  float dqa[DL];
#pragma unroll
  for (int i = 0; i < DL; ++i) dqa[i] = 0.f;
  const uint16_t* kb = a.k + (long long)b * a.k_bs + h * D + l;
  float* dkb = dk + (long long)b * dk_bs + h * D + l;
  float* dvb = dv + (long long)b * dv_bs + h * D + l;
#pragma unroll 4
  for (int j = 0; j < a.Nk; ++j) {
    const float dsj = __shfl(ds, j), pj = __shfl(p, j);
#pragma unroll
    for (int i = 0; i < DL; ++i) {
      dqa[i] = fmaf(dsj, bf2f(kb[(long long)j * a.k_rs + 64 * i]), dqa[i]);
      float* dkp = dkb + (long long)j * dk_rs + 64 * i;
      float* dvp = dvb + (long long)j * dv_rs + 64 * i;
      const float gk = a.scale * dsj * qv[i], gv = pj * dov[i];
      *dkp = kv_acc ? *dkp + gk : gk;
      *dvp = kv_acc ? *dvp + gv : gv;
    }
  }
  float* dqp = dq + (long long)b * dq_bs + h * D + l;
#pragma unroll
  for (int i = 0; i < DL; ++i) dqp[64 * i] = a.scale * dqa[i];
  (void)dq_rs;
}

// the decode backward's shape: head width 128, one query, ≤ 64 keys, no key mask, no dropout
static bool decode_bwd_ok(const AttnArgs& a, int D) {
  return D == 128 && a.Nq == 1 && a.Nk >= 1 && a.Nk <= 64 && a.kmask == nullptr && a.drop_thresh == 0;
}

// ------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------
template <int D, int NWV>
static void fwd_launch_t(const AttnArgs& a, uint16_t* O, float* LSE, float* Opart, float* MLpart, int nsplit,
                         hipStream_t st) {
  const int ntiles = (a.Nk + KT - 1) / KT;
  const int tps = (ntiles + nsplit - 1) / nsplit;
  dim3 grid((a.Nq + 32 * NWV - 1) / (32 * NWV), a.H, a.B * nsplit);
  hipLaunchKernelGGL((attn_fwd_kernel<D, NWV>), grid, dim3(64 * NWV), 0, st, a, O, LSE, Opart, MLpart, nsplit, tps);
}

template <int D>
static void fwd_dispatch(const AttnArgs& a, uint16_t* O, float* LSE, float* Opart, float* MLpart, int nsplit,
                         hipStream_t st) {
  if (a.Nq <= 32) fwd_launch_t<D, 1>(a, O, LSE, Opart, MLpart, nsplit, st);
  else if (a.Nq <= 64) fwd_launch_t<D, 2>(a, O, LSE, Opart, MLpart, nsplit, st);
  else fwd_launch_t<D, 4>(a, O, LSE, Opart, MLpart, nsplit, st);
}

void attn_fwd_launch(const AttnArgs& a, int D, uint16_t* O, float* LSE, float* Opart, float* MLpart, int nsplit,
                     hipStream_t st) {
  switch (D) {
    case 16: fwd_dispatch<16>(a, O, LSE, Opart, MLpart, nsplit, st); break;
    case 32: fwd_dispatch<32>(a, O, LSE, Opart, MLpart, nsplit, st); break;
    case 64: fwd_dispatch<64>(a, O, LSE, Opart, MLpart, nsplit, st); break;
    case 128: fwd_dispatch<128>(a, O, LSE, Opart, MLpart, nsplit, st); break;
    default: break;
  }
  if (nsplit > 1) {
    const long long rows = (long long)a.B * a.Nq * a.H;
    const long long n = rows * D;
    hipLaunchKernelGGL(attn_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, Opart, MLpart, O, LSE,
                       nsplit, (int)rows, D);
  }
}

void attn_combine_launch(const float* Opart, const float* MLpart, uint16_t* O, float* LSE, int nsplit, long long rows,
                         int D, hipStream_t st) {
  const long long n = rows * D;
  hipLaunchKernelGGL(attn_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, Opart, MLpart, O, LSE, nsplit,
                     (int)rows, D);
}


// query splits of the backward grid when key blocks × heads × batch leave the GPU idle (≥ 4
// query tiles each; no empty split)
static int bwd_query_splits(int nkb, int H, int B, int Nq, int qsplit_ok) {
  const int nqt = (Nq + 31) / 32, base = nkb * H * B;
  int nqs = 1;
  if (qsplit_ok && base < 256 && nqt >= 8) {
    nqs = (512 + base - 1) / base;
    const int cap = (nqt + 3) / 4;
    nqs = nqs < cap ? nqs : cap;
  }
  const int tps = (nqt + nqs - 1) / nqs;
  return (nqt + tps - 1) / tps;
}

// which accumulators a (non-deterministic, non-accumulating) backward launch clears itself:
// bit 0 dQ (several key blocks add into it), bit 1 dK / dV (query splits add into them) — a
// caller that clears them on the way (a SlabJob zero span of the previous kernel) passes the
// same bits back as dq_zeroed
int attn_bwd_zero_plan(int B, int H, int Nq, int Nk, int D) {
  const int nw = D <= 32 ? 8 : 4;
  const int nkb = (Nk + 32 * nw - 1) / (32 * nw);
  return (nkb > 1 ? 1 : 0) | (bwd_query_splits(nkb, H, B, Nq, 1) > 1 ? 2 : 0);
}

template <int D, int NW>
static void bwd_launch_t(const AttnArgs& a, const uint16_t* dO, const float* LSE, float* delta, float* dq,
                         long long dq_bs, int dq_rs, float* dk, long long dk_bs, int dk_rs, float* dv, long long dv_bs,
                         int dv_rs, int kv_acc, long long dq_kbs, int qsplit_ok, int dq_zeroed, hipStream_t st) {
  const int nkb = (a.Nk + 32 * NW - 1) / (32 * NW);
  const int nqt = (a.Nq + 31) / 32;
  const int nqs = bwd_query_splits(nkb, a.H, a.B, a.Nq, qsplit_ok);
  const int tps = (nqt + nqs - 1) / nqs;
  if (nqs > 1 && !kv_acc && !(dq_zeroed & 2)) {  // the splits add into dK / dV (bit 1: cleared by the caller)
    const long long total = (long long)a.B * a.Nk * a.H * D;
    const unsigned zb = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(zero_rows_kernel, dim3(zb), dim3(256), 0, st, dk, dk_bs, dk_rs, a.Nk, a.H * D, total);
    hipLaunchKernelGGL(zero_rows_kernel, dim3(zb), dim3(256), 0, st, dv, dv_bs, dv_rs, a.Nk, a.H * D, total);
  }
  // several key blocks add into dQ (fp32 atomics), unless each stores its own partial slice
  // (deterministic mode: dq_kbs > 0, summed by the caller)
  const int atomic = nkb > 1 && dq_kbs == 0;
  if (atomic && !(dq_zeroed & 1)) {
    const long long total = (long long)a.B * a.Nq * a.H * D;
    hipLaunchKernelGGL(zero_rows_kernel, dim3((unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096)), dim3(256), 0,
                       st, dq, dq_bs, dq_rs, a.Nq, a.H * D, total);
  }
  dim3 grid(nkb * nqs, a.H, a.B);
  constexpr bool small_lds = true;
  // head width 16, no dropout, a grid wider than the chip: the two-query-tile variant at ≤ 128
  // VGPRs runs two 8-wave workgroups per CU (1.342 → 1.327 ms on the headline step, r5)
  const bool wide = D == 16 && NW == 8 && !a.drop_thresh && a.Nq > 64 &&
                    (long long)grid.x * grid.y * grid.z > 256;
  if (wide) {
    if (a.kmask == nullptr && a.Nk % (32 * NW) == 0)
      hipLaunchKernelGGL((attn_bwd_kernel<D, NW, 2, false, false, false>), grid, dim3(64 * NW), 0, st, a, dO, LSE, delta,
                         dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, atomic, kv_acc, dq_kbs, nqs, tps, SlabJob{});
    else
      hipLaunchKernelGGL((attn_bwd_kernel<D, NW, 2, false, true, false>), grid, dim3(64 * NW), 0, st, a, dO, LSE, delta,
                         dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, atomic, kv_acc, dq_kbs, nqs, tps, SlabJob{});
    return;
  }
  // ≤ 64 queries (few-query cross-attention): the small-LDS variants let several workgroups
  // share a CU
  if (a.Nq <= 32 && small_lds)
    hipLaunchKernelGGL((attn_bwd_kernel<D, NW, 1>), grid, dim3(64 * NW), 0, st, a, dO, LSE, delta, dq, dq_bs, dq_rs,
                       dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, atomic, kv_acc, dq_kbs, nqs, tps, SlabJob{});
  else if (a.Nq <= 64 && small_lds)
    hipLaunchKernelGGL((attn_bwd_kernel<D, NW, 2>), grid, dim3(64 * NW), 0, st, a, dO, LSE, delta, dq, dq_bs, dq_rs,
                       dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, atomic, kv_acc, dq_kbs, nqs, tps, SlabJob{});
  else if (a.kmask == nullptr && a.Nk % (32 * NW) == 0)
    hipLaunchKernelGGL((attn_bwd_kernel<D, NW, 0, false, false>), grid, dim3(64 * NW), 0, st, a, dO, LSE, delta, dq,
                       dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, atomic, kv_acc, dq_kbs, nqs, tps, SlabJob{});
  else
    hipLaunchKernelGGL((attn_bwd_kernel<D, NW>), grid, dim3(64 * NW), 0, st, a, dO, LSE, delta, dq, dq_bs, dq_rs, dk,
                       dk_bs, dk_rs, dv, dv_bs, dv_rs, atomic, kv_acc, dq_kbs, nqs, tps, SlabJob{});
}

void slab_reduce_launch(const SlabJob& job, hipStream_t st);  // elementwise.hip

// key blocks of the backward grid (dQ partial slices in deterministic mode)
int attn_bwd_key_blocks(int Nk, int D) {
  const int nw = D <= 32 ? 8 : 4;
  return (Nk + 32 * nw - 1) / (32 * nw);
}

void attn_bwd_launch(const AttnArgs& a, int D, const uint16_t* O, const uint16_t* dO, const float* LSE, float* delta,
                     float* dq, long long dq_bs, int dq_rs, float* dk, long long dk_bs, int dk_rs, float* dv,
                     long long dv_bs, int dv_rs, bool compute_delta, bool kv_acc, long long dq_kbs, int qsplit_ok,
                     int dq_zeroed, hipStream_t st) {
  // delta = rowsum(dO∘O) is normally produced by the post-attention backward kernel;
  // compute it here otherwise.  dQ needs no zero fill from the caller.
  const int rows = a.B * a.Nq;
  if (compute_delta)
    hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, dO, O, delta, (float*)nullptr,
                       rows, a.H, D, dq_rs);
  if (decode_bwd_ok(a, D)) {  // one query: its dK / dV rows are its own (no sum over queries)
    const dim3 grid((unsigned)a.B, (unsigned)a.H);
    hipLaunchKernelGGL((attn_decode_bwd_kernel<128>), grid, dim3(64), 0, st, a, dO, LSE, delta, dq, dq_bs, dq_rs, dk,
                       dk_bs, dk_rs, dv, dv_bs, dv_rs, (int)kv_acc);
    return;
  }
  switch (D) {  // waves per workgroup: 8 for d ≤ 32, 4 above (keys per block = 32 × waves)
    case 16:  // ≤ 64 keys (the 64-latent self-attention of the text classifiers / MLM-64): 2 waves, not 6 idle of 8
      if (a.Nk <= 64) bwd_launch_t<16, 2>(a, dO, LSE, delta, dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, kv_acc, dq_kbs, qsplit_ok, dq_zeroed, st);
      else bwd_launch_t<16, 8>(a, dO, LSE, delta, dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, kv_acc, dq_kbs, qsplit_ok, dq_zeroed, st);
      break;
    case 32:  // ≤ 64 keys (the image configs' 32-latent self-attention): 2 waves, not 6 idle of 8
      if (a.Nk <= 64) bwd_launch_t<32, 2>(a, dO, LSE, delta, dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, kv_acc, dq_kbs, qsplit_ok, dq_zeroed, st);
      else bwd_launch_t<32, 8>(a, dO, LSE, delta, dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, kv_acc, dq_kbs, qsplit_ok, dq_zeroed, st);
      break;
    case 64: bwd_launch_t<64, 4>(a, dO, LSE, delta, dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, kv_acc, dq_kbs, qsplit_ok, dq_zeroed, st); break;
    case 128: bwd_launch_t<128, 4>(a, dO, LSE, delta, dq, dq_bs, dq_rs, dk, dk_bs, dk_rs, dv, dv_bs, dv_rs, kv_acc, dq_kbs, qsplit_ok, dq_zeroed, st); break;
    default: break;
  }
}

// bf16 dQ / dK / dV (attn_bwd_kernel OBF): head width 16, one key block (Nk ≤ 256), no query
// split, more than 64 queries (the full-LDS variant), nothing to accumulate onto; false (nothing
// launched) when the shape does not qualify
bool attn_bwd_bf16_ok(const AttnArgs& a, int D) {
  return D == 16 && a.Nk <= 32 * 8 && a.Nq > 64 && bwd_query_splits(1, a.H, a.B, a.Nq, 1) == 1;
}
// job: the previous kernel's slab reduction in z-slices appended past the batch.  Carrying one,
// the two-query-tile variant runs (≈ 70 KB of LDS: two workgroups per CU), so the reduction
// shares the CUs with the attention tiles instead of queueing behind a one-per-CU carrier's tiles.
bool attn_bwd_bf16_launch(const AttnArgs& a, int D, const uint16_t* dO, const float* LSE, const float* delta,
                          uint16_t* dq, long long dq_bs, int dq_rs, uint16_t* dk, long long dk_bs, int dk_rs,
                          uint16_t* dv, long long dv_bs, int dv_rs, const SlabJob& job, hipStream_t st) {
  if (!attn_bwd_bf16_ok(a, D)) return false;
  const int nqt = (a.Nq + 31) / 32;
  const bool carry = job.slab != nullptr && job.nblk > 0 && a.kmask == nullptr && a.Nk == 256 && !a.drop_thresh;
  dim3 grid(1, a.H, a.B + (carry ? (job.nblk + a.H - 1) / a.H : 0));
#define BF16L(QR_, KM_, J_)                                                                                         \
  hipLaunchKernelGGL((attn_bwd_kernel<16, 8, QR_, true, KM_, QR_ == 0>), grid, dim3(512), 0, st, a, dO, LSE, delta,           \
                     reinterpret_cast<float*>(dq), dq_bs, dq_rs, reinterpret_cast<float*>(dk), dk_bs, dk_rs,         \
                     reinterpret_cast<float*>(dv), dv_bs, dv_rs, 0, 0, 0LL, 1, nqt, J_)
  if (carry) BF16L(2, false, job);
  else if (a.kmask == nullptr && a.Nk == 256) BF16L(0, false, SlabJob{});
  else BF16L(0, true, SlabJob{});
#undef BF16L
  if (job.slab != nullptr && !carry) slab_reduce_launch(job, st);
  return true;
}

}  // namespace pio
