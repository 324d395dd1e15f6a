// Factored LayerNorm + K/V projection over [pixels ‖ Fourier PE] (SURVEY K-03/K-05/K-06).
//
// The image adapter's input row is x = [p ‖ e_m]: nc (≤ 4) pixel channels of sample b and the
// batch-independent position encoding e_m of pixel m (reference adapter.py:99-109 concatenates
// them; model.py:89-99 then applies kv_norm and the K/V in-projection).  With
// x̂ = (x − μ)·rσ, LN(x) = x̂⊙γ + β and y = W·LN(x) + b:
//
//     y_o = rσ·( P'[m,o] + Σ_c p_c·W[o,c]γ_c ) − μ·rσ·(Wγ)_o + (Wβ + b)_o,
//     P' = (E ⊙ γ_e)·W_eᵀ            (one (M × Kin) · (Kin × O) GEMM per step, not per sample)
//
// and μ, rσ follow from Σe_m, Σe_m² (per pixel, batch-independent) plus the nc pixel values.
// So the per-sample work is a bandwidth-bound epilogue (read P' from L2/MALL, write bf16 K/V)
// instead of a (B·M × Kin × O) GEMM.  The backward is the mirror image: one streaming pass
// over dY produces
//     D[m,o] = Σ_b dY·rσ,  S_o = Σ dY,  e_o = Σ dY·μ·rσ,  Gp[c,o] = Σ dY·x̂_c  (pixel channels)
// and the weight / LayerNorm gradients follow from small GEMMs on the host side
// (ops/fused.py: _pe_proj_bwd).  No atomics: per-block partials are summed afterwards.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace pio {

// one wave per pixel m: P'[m] (≤ 512 outputs) is read once into registers and reused for the
// B rows r = b·M + m of that pixel (a row-per-wave mapping would re-read it B times)
__global__ __launch_bounds__(256) void pe_proj_fwd_kernel(
    const float* __restrict__ pix, int nc, const float* __restrict__ P, const float* __restrict__ pes,
    const float* __restrict__ pesq, const float* __restrict__ wpg, const float* __restrict__ gw,
    const float* __restrict__ bw, int B, int bchunk, int M, int O, float inv_k, float eps,
    uint16_t* __restrict__ y, float* __restrict__ mean, float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int b0 = blockIdx.y * bchunk, b1 = b0 + bchunk < B ? b0 + bchunk : B;  // this block's batch slice
  const int nw = (gridDim.x * blockDim.x) >> 6;
  const int O4 = O >> 2;
  float4 wc[4][2], g[2], bb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int o4 = lane + 64 * j;
    const bool ok = o4 < O4;
    g[j] = ok ? reinterpret_cast<const float4*>(gw)[o4] : make_float4(0.f, 0.f, 0.f, 0.f);
    bb[j] = ok ? reinterpret_cast<const float4*>(bw)[o4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int c = 0; c < 4; ++c)
      wc[c][j] = (ok && c < nc) ? reinterpret_cast<const float4*>(wpg + (long long)c * O)[o4]
                                : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int m = ((int)(blockIdx.x * blockDim.x + threadIdx.x)) >> 6; m < M; m += nw) {
    float4 pm[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o4 = lane + 64 * j;
      pm[j] = o4 < O4 ? reinterpret_cast<const float4*>(P + (long long)m * O)[o4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // row statistics lane-parallel (lane i ↔ sample b0 + i, bchunk ≤ 64), then broadcast with
    // cross-lane reads inside the loop: no dependent global load per output row
    float my_mu = 0.f, my_rs = 0.f, my_px[4] = {0.f, 0.f, 0.f, 0.f};
    if (b0 + lane < b1) {
      const long long r = (long long)(b0 + lane) * M + m;
      float s = pes[m], sq = pesq[m];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < nc) {
          const float v = pix[r * nc + c];
          my_px[c] = v;
          s += v;
          sq += v * v;
        }
      }
      my_mu = s * inv_k;
      my_rs = rsqrtf(fmaxf(sq * inv_k - my_mu * my_mu, 0.f) + eps);
      mean[r] = my_mu;
      rstd[r] = my_rs;
    }
#pragma unroll 4
    for (int b = b0; b < b1; ++b) {
      const long long r = (long long)b * M + m;
      const float mu = __shfl(my_mu, b - b0), rs = __shfl(my_rs, b - b0);
      float px[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) px[c] = __shfl(my_px[c], b - b0);
      const float mrs = mu * rs;
      uint2* yr = reinterpret_cast<uint2*>(y + r * O);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int o4 = lane + 64 * j;
        if (o4 < O4) {
          float4 a = pm[j];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            a.x += px[c] * wc[c][j].x; a.y += px[c] * wc[c][j].y; a.z += px[c] * wc[c][j].z; a.w += px[c] * wc[c][j].w;
          }
          yr[o4] = make_uint2(pack2(a.x * rs - mrs * g[j].x + bb[j].x, a.y * rs - mrs * g[j].y + bb[j].y),
                              pack2(a.z * rs - mrs * g[j].z + bb[j].z, a.w * rs - mrs * g[j].w + bb[j].w));
        }
      }
    }
  }
}

// one wave per pixel m (all B samples of it); lane owns outputs 4·(lane + 64j) .. +3, j < 2
__global__ __launch_bounds__(256) void pe_proj_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ pix, int nc, const float* __restrict__ mean,
    const float* __restrict__ rstd, int B, int M, int O, float* __restrict__ D, float* __restrict__ part) {
  extern __shared__ float red[];  // (4 waves) × (2 + nc)·O
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int O4 = O >> 2;
  const int W = (2 + nc) * O;
  float4 S[2], E[2], G[4][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    S[j] = E[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int c = 0; c < 4; ++c) G[c][j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int m = blockIdx.x * 4 + wid; m < M; m += gridDim.x * 4) {
    float4 d[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    for (int bb = 0; bb < B; bb += 64) {
      // per-row factors lane-parallel (lane i ↔ sample bb + i), broadcast in the loop
      float my_rs = 0.f, my_mrs = 0.f, my_xh[4] = {0.f, 0.f, 0.f, 0.f};
      if (bb + lane < B) {
        const long long r = (long long)(bb + lane) * M + m;
        my_rs = rstd[r];
        const float mu = mean[r];
        my_mrs = mu * my_rs;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c < nc) my_xh[c] = (pix[r * nc + c] - mu) * my_rs;
      }
      const int be = B - bb < 64 ? B - bb : 64;
#pragma unroll 4
      for (int i = 0; i < be; ++i) {
        const long long r = (long long)(bb + i) * M + m;
        const float rs = __shfl(my_rs, i), mrs = __shfl(my_mrs, i);
        float xh[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) xh[c] = __shfl(my_xh[c], i);
        const float4* dyr = reinterpret_cast<const float4*>(dy + r * O);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int o4 = lane + 64 * j;
          if (o4 < O4) {
            const float4 v = dyr[o4];
            d[j].x += v.x * rs; d[j].y += v.y * rs; d[j].z += v.z * rs; d[j].w += v.w * rs;
            S[j].x += v.x; S[j].y += v.y; S[j].z += v.z; S[j].w += v.w;
            E[j].x += v.x * mrs; E[j].y += v.y * mrs; E[j].z += v.z * mrs; E[j].w += v.w * mrs;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              G[c][j].x += v.x * xh[c]; G[c][j].y += v.y * xh[c]; G[c][j].z += v.z * xh[c]; G[c][j].w += v.w * xh[c];
            }
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o4 = lane + 64 * j;
      if (o4 < O4) reinterpret_cast<float4*>(D + (long long)m * O)[o4] = d[j];
    }
  }
  float* mine = red + wid * W;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int o4 = lane + 64 * j;
    if (o4 < O4) {
      reinterpret_cast<float4*>(mine)[o4] = S[j];
      reinterpret_cast<float4*>(mine + O)[o4] = E[j];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < nc) reinterpret_cast<float4*>(mine + (2 + c) * O)[o4] = G[c][j];
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < W; k += blockDim.x)
    part[(long long)blockIdx.x * W + k] = red[k] + red[W + k] + red[2 * W + k] + red[3 * W + k];
}

// ------------------------------------------------------------------------------------
// The per-step PE GEMM P'[m, o] = Σ_k Ebf[m, k]·Wg[o, k] (replaces a library GEMM plus the
// per-step pad / scale / cast kernels around it).  Ebf is the bf16 PE table, zero outside the
// PE columns [nc, kin) and padded to Kp (a multiple of 32): a constant cached across steps.
// Wg = (W ⊙ γ) with the same column layout is built each step by pe_weight_prep_kernel, which
// also emits the per-sample epilogue vectors wpg, gw, bw.
// Tiles: 128 × 128 outputs per workgroup (2 × 2 waves of 64 × 64, v_mfma_f32_32x32x16_bf16),
// K in 32-wide chunks staged through double-buffered LDS (k-contiguous rows), the next chunk
// register-prefetched while the current one is multiplied.  fp32 output (pe_proj_fwd input).
// ------------------------------------------------------------------------------------
constexpr int GT = 128, GKC = 32, GLD = GKC + 8;

template <bool BF16OUT>
__global__ __launch_bounds__(256) void pe_gemm_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ Bw,
                                                      void* __restrict__ Cv, int M, int N, int K, int Mst) {
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][GT * GLD];
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][GT * GLD];
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.x * GT, n0 = blockIdx.y * GT;
  // chunk staging: 128 rows × 32 k = 512 16-byte pieces per operand, 2 per thread
  bf16x8 ra[2], rb[2];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = threadIdx.x + 256 * i, row = c >> 2, kk = k0 + (c & 3) * 8;
      const int gm = m0 + row;
      const uint16_t* pa = gm < M ? A + (long long)gm * K + kk : reinterpret_cast<const uint16_t*>(kZero32B);
      ra[i] = *reinterpret_cast<const bf16x8*>(pa);
      rb[i] = *reinterpret_cast<const bf16x8*>(Bw + (long long)(n0 + row) * K + kk);
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = threadIdx.x + 256 * i, row = c >> 2, kk = (c & 3) * 8;
      *reinterpret_cast<bf16x8*>(&sA[buf][row * GLD + kk]) = ra[i];
      *reinterpret_cast<bf16x8*>(&sB[buf][row * GLD + kk]) = rb[i];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  const int nk = K / GKC;
  fetch(0);
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    stash(buf);  // the other buffer is still being read by the previous chunk's MFMAs: double buffer
    lds_sync();
    if (kc + 1 < nk) fetch((kc + 1) * GKC);
#pragma unroll
    for (int ks = 0; ks < GKC; ks += 16) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        fa[i] = frag_kc(sA[buf], GLD, 64 * wm + 32 * i, ks);
        fb[i] = frag_kc(sB[buf], GLD, 64 * wn + 32 * i, ks);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
    }
  }
  // accumulator: col = lane & 31 (n), row = acc_row (m)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 64 * wn + 32 * j + (l & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * i + acc_row(r, hh);
        if (m < Mst) {  // rows [M, Mst): A rows read as zeros → the zero pad rows of C
          if constexpr (BF16OUT) reinterpret_cast<uint16_t*>(Cv)[(long long)m * N + n] = f2bf(acc[i][j][r]);
          else reinterpret_cast<float*>(Cv)[(long long)m * N + n] = acc[i][j][r];
        }
      }
    }
}

// one workgroup per output row o of the factored projection (O ≤ 65535 rows, blockDim 256):
//   Wg[o, k] = W[o, k]·γ[k] for k in [nc, kin), 0 elsewhere (k < Kp), bf16
//   wpg[c, o] = W[o, c]·γ[c] (c < nc), gw[o] = Σ_k W[o, k]γ[k], bw[o] = Σ_k W[o, k]β[k] + bias[o]
// and (wt non-null) the implicit-K/V generation table of attention_pe.hip, wt (PE_NWT, O):
//   rows c < 4: wpg[c, o] (0 for c ≥ nc),  row 4: Σ_c wpg[c, o] − gw[o],  row 5: bw[o]
// W2 (optional): rows [O1, O) come from W2 (the V projection weight of a separate K / V pair)
__global__ __launch_bounds__(256) void pe_weight_prep_kernel(const float* __restrict__ W, const float* __restrict__ W2,
                                                             int O1, const float* __restrict__ g,
                                                             const float* __restrict__ b, const float* __restrict__ bias,
                                                             int O, int nc, int kin, int Kp, uint16_t* __restrict__ Wg,
                                                             float* __restrict__ wpg, float* __restrict__ gw,
                                                             float* __restrict__ bw, float* __restrict__ wt) {
  __shared__ float red[2][4];
  const int o = blockIdx.x;
  const float* Wr = W2 != nullptr && o >= O1 ? W2 + (long long)(o - O1) * kin : W + (long long)o * kin;
  float sg = 0.f, sb = 0.f;
  for (int k = threadIdx.x; k < Kp; k += blockDim.x) {
    float wgk = 0.f;
    if (k < kin) {
      const float wv = Wr[k];
      wgk = wv * g[k];
      sg += wgk;
      sb += wv * b[k];
      if (k < nc) wpg[(long long)k * O + o] = wgk;
    }
    Wg[(long long)o * Kp + k] = f2bf(k >= nc && k < kin ? wgk : 0.f);
  }
  sg = wave_sum(sg);
  sb = wave_sum(sb);
  if (lane_id() == 0) { red[0][wave_id()] = sg; red[1][wave_id()] = sb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float gsum = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    const float bsum = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]) + bias[o];
    gw[o] = gsum;
    bw[o] = bsum;
    if (wt) {
      float ps = 0.f;
      for (int c = 0; c < 4; ++c) {
        const float v = c < nc ? Wr[c] * g[c] : 0.f;  // = wpg[c, o]
        wt[(long long)c * O + o] = v;
        ps += v;
      }
      wt[4LL * O + o] = ps - gsum;
      wt[5LL * O + o] = bsum;
    }
  }
}

// ------------------------------------------------------------------------------------
// Backward of the factored projection's weights (replaces a split-K library GEMM, its batch
// sum and ~20 small framework kernels per call):
//   A  pe_gemm_tn : slab[s] = Ebf[rows of split s]ᵀ · bf16(D[rows of split s])   (Kp × O fp32)
//   B  pe_grad_reduce : Graw = Σ_s slab[s],  tot = Σ_blocks part  (= [S | e | Gp])
//   C  pe_grad_finalize : per input column k,  G[o] = Gp[k][o] (pixel k < nc) or Graw[k][o] − e[o],
//      dW[o][k] += G·γ_k + S_o·β_k,  dγ_k += Σ_o W[o][k]·G[o],  dβ_k += Σ_o W[o][k]·S_o,  db += S
// W / dW are split in two row blocks (the separate K and V projection weights, rows [0, Ch) and
// [Ch, O)).  Every gradient element has exactly one writer: deterministic.
// ------------------------------------------------------------------------------------
// LDS row stride (bf16) of the transposed-read tiles: ≡ 32 (mod 128), i.e. 16 (mod 64) dwords, so the
// 8-byte pieces of ds_read_b64_tr_b16 (4 rows × 4 pieces per 16-lane group, two groups 16 columns
// apart per pass) land on 64 distinct banks
__host__ __device__ constexpr int tn_ld(int x) { return x + ((32 - x) % 128 + 128) % 128; }

// grid (row splits, column groups): workgroup (s, c) accumulates output columns [c·on, c·on + on)
// over rows [s·rps, (s+1)·rps) in 32-row chunks — two chunks of loads in flight (two register
// sets, the loop unrolled by two), double-buffered LDS, one barrier per chunk — and stores its
// (Kp × on) partial into slab[s].  MAXT: output 32 × 32 tiles per wave (⌈(Kp/32)·(on/32) / 4⌉),
// NE / ND: 16-byte E pieces / float4 D pieces per thread and chunk (⌈Kp / 64⌉, ⌈on / 32⌉).
template <int MAXT, int NE, int ND>
__global__ __launch_bounds__(256) void pe_gemm_tn_kernel(const uint16_t* __restrict__ E, const float* __restrict__ D,
                                                         float* __restrict__ slab, int M, int Kp, int O, int on,
                                                         int rows_per_split) {
  extern __shared__ __attribute__((aligned(16))) uint16_t tsm[];
  const int LDE = tn_ld(Kp), LDD = tn_ld(on);
  uint16_t* sE[2] = {tsm, tsm + 32 * LDE};
  uint16_t* sD[2] = {tsm + 64 * LDE, tsm + 64 * LDE + 32 * LDD};
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int r_begin = blockIdx.x * rows_per_split, r_end = min(M, r_begin + rows_per_split);
  const int c0 = blockIdx.y * on;
  const int ntj = on / 32, ntiles = (Kp / 32) * ntj;
  const int ce = Kp / 8, cd = on / 4;  // 16-byte pieces per E row, float4 per D row slice
  struct Regs {
    bf16x8 e[NE];
    float4 d[ND];
  } ra, rb;
  // branch-free: rows past the split (or the matrix) read zeros, so a prefetch past the last
  // chunk is harmless and every fetch is straight-line code (see kZero32B)
  auto fetch = [&](Regs& R, int r0) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / ce, col = (c % ce) * 8;
      const bool ok = (c < 32 * ce) & (r0 + row < r_end);
      const uint16_t* p = ok ? E + (long long)(r0 + row) * Kp + col : reinterpret_cast<const uint16_t*>(kZero32B);
      R.e[i] = *reinterpret_cast<const bf16x8*>(p);
    }
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / cd, col = (c % cd) * 4;
      const bool ok = (c < 32 * cd) & (r0 + row < r_end);
      const float* p = ok ? D + (long long)(r0 + row) * O + c0 + col : kZero32B;
      R.d[i] = *reinterpret_cast<const float4*>(p);
    }
  };
  auto stash = [&](const Regs& R, int buf) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / ce, col = (c % ce) * 8;
      if (c < 32 * ce) *reinterpret_cast<bf16x8*>(sE[buf] + row * LDE + col) = R.e[i];
    }
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int c = threadIdx.x + 256 * i, row = c / cd, col = (c % cd) * 4;
      if (c < 32 * cd) {
        uint2 pk;
        pk.x = pack2(R.d[i].x, R.d[i].y);
        pk.y = pack2(R.d[i].z, R.d[i].w);
        *reinterpret_cast<uint2*>(sD[buf] + row * LDD + col) = pk;
      }
    }
  };
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  auto compute = [&](int buf) {
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      const int tile = w + 4 * t;
      if (tile < ntiles) {  // wave-uniform
        const int ti = tile / ntj, tj = tile % ntj;
#pragma unroll
        for (int ks = 0; ks < 32; ks += 16)
          acc[t] = mfma32(frag_ks(sE[buf], LDE, 32 * ti, ks), frag_ks(sD[buf], LDD, 32 * tj, ks), acc[t]);
      }
    }
  };
  fetch(ra, r_begin);
  fetch(rb, r_begin + 32);
  for (int r0 = r_begin; r0 < r_end; r0 += 64) {
    stash(ra, 0);
    lds_sync();
    fetch(ra, r0 + 64);
    compute(0);
    stash(rb, 1);
    lds_sync();
    fetch(rb, r0 + 96);
    compute(1);  // an odd last chunk: zero rows
  }
  // accumulator: col = lane & 31 → o, row = acc_row → k
  float* out = slab + (long long)blockIdx.x * Kp * O + c0;
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int tile = w + 4 * t;
    if (tile < ntiles) {
      const int ti = tile / ntj, tj = tile % ntj;
#pragma unroll
      for (int i = 0; i < 16; ++i) out[(long long)(32 * ti + acc_row(i, hh)) * O + 32 * tj + (l & 31)] = acc[t][i];
    }
  }
}

// Graw = Σ_s slab[s] (Kp·O floats) and tot = Σ_b part[b] ((2 + nc)·O floats) in one launch: a
// block sums 64 float4 columns with 4 row groups (loads 8 deep), fixed combination order
__global__ __launch_bounds__(256) void pe_grad_reduce_kernel(const float* __restrict__ slab, int S, long long KO4,
                                                             const float* __restrict__ part, int nblk, long long W4,
                                                             float* __restrict__ Graw, float* __restrict__ tot) {
  __shared__ float4 red[4][64];
  const int l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long long c = (long long)blockIdx.x * 64 + l;  // float4 column of [slab | part]
  const bool second = c >= KO4;
  const long long cc = second ? c - KO4 : c;
  const long long stride = second ? W4 : KO4;
  const int rows = second ? nblk : S;
  const float4* src = reinterpret_cast<const float4*>(second ? part : slab) + cc;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < KO4 + W4) {
#pragma unroll 8
    for (int r = g; r < rows; r += 4) {
      const float4 v = src[(long long)r * stride];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[g][l] = acc;
  __syncthreads();
  if (g == 0 && c < KO4 + W4) {
    float4 r = red[0][l];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 v = red[k][l];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    reinterpret_cast<float4*>(second ? tot : Graw)[cc] = r;
  }
}

struct PeGradTargets {
  float *dWa, *dWb, *db, *dg, *dbeta;  // dW rows [0, Ch) / [Ch, O) (kin columns each); any may be null
};

// one block per input column k (< kin), threads over the outputs o
__global__ __launch_bounds__(256) void pe_grad_finalize_kernel(const float* __restrict__ Graw, const float* __restrict__ tot,
                                                               const float* __restrict__ Wa, const float* __restrict__ Wb,
                                                               const float* __restrict__ g, const float* __restrict__ b,
                                                               int O, int Ch, int kin, int nc, PeGradTargets t) {
  __shared__ float red[2][4];
  const int k = blockIdx.x;
  float sg = 0.f, sb = 0.f;
  for (int o = threadIdx.x; o < O; o += blockDim.x) {
    const float S = tot[o];
    const float G = k < nc ? tot[(long long)(2 + k) * O + o] : Graw[(long long)k * O + o] - tot[O + o];
    const bool lo = o < Ch;
    const int oo = lo ? o : o - Ch;
    const float wv = (lo ? Wa : Wb)[(long long)oo * kin + k];
    sg += wv * G;
    sb += wv * S;
    float* dW = lo ? t.dWa : t.dWb;
    if (dW) dW[(long long)oo * kin + k] += G * g[k] + S * b[k];
    if (k == 0 && t.db) t.db[o] += S;
  }
  sg = wave_sum(sg);
  sb = wave_sum(sb);
  if (lane_id() == 0) { red[0][wave_id()] = sg; red[1][wave_id()] = sb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (t.dg) t.dg[k] += (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    if (t.dbeta) t.dbeta[k] += (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

int pe_grad_splits(int M) {
  const int s = (M + 383) / 384;  // ≈ 384 rows (12 chunks) per workgroup, ≤ 128 slab rows
  return s < 1 ? 1 : (s > 128 ? 128 : s);
}

void pe_grads_launch(const uint16_t* E, const float* D, int M, int Kp, int O, const float* part, int nblk, float* slab,
                     float* Graw, float* tot, const float* Wa, const float* Wb, const float* g, const float* b, int Ch,
                     int kin, int nc, PeGradTargets t, hipStream_t st) {
  const int S0 = pe_grad_splits(M);
  const int rps = ((M + S0 - 1) / S0 + 31) / 32 * 32;
  const int S = (M + rps - 1) / rps;
  const int on = O % 128 == 0 ? 128 : O;  // output columns per workgroup
  const size_t lds = (size_t)2 * 32 * (tn_ld(Kp) + tn_ld(on)) * sizeof(uint16_t);
  const int tiles = (Kp / 32) * (on / 32), ne = (Kp + 63) / 64, nd = (on + 31) / 32;
  const dim3 grid((unsigned)S, (unsigned)(O / on));
#define TNL(MT, NE_, ND_)                                                                                      \
  {                                                                                                          \
    static bool attr = false;                                                                                \
    if (!attr) {                                                                                             \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(pe_gemm_tn_kernel<MT, NE_, ND_>),              \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                     \
      attr = true;                                                                                           \
    }                                                                                                        \
    hipLaunchKernelGGL((pe_gemm_tn_kernel<MT, NE_, ND_>), grid, dim3(256), lds, st, E, D, slab, M, Kp, O, on, rps); \
  }
  if (tiles <= 20 && ne <= 3 && nd <= 4) TNL(5, 3, 4)  // the ImageNet shape: Kp = 160, 128 columns
  else TNL(9, 6, 8)
#undef TNL
  const long long KO4 = (long long)Kp * O / 4, W4 = (long long)(2 + nc) * O / 4;
  hipLaunchKernelGGL(pe_grad_reduce_kernel, dim3((unsigned)((KO4 + W4 + 63) / 64)), dim3(256), 0, st, slab, S, KO4, part,
                     nblk, W4, Graw, tot);
  hipLaunchKernelGGL(pe_grad_finalize_kernel, dim3((unsigned)kin), dim3(256), 0, st, Graw, tot, Wa, Wb, g, b, O, Ch, kin,
                     nc, t);
}

// C has Mst ≥ M rows; rows past M are written as zeros by the same launch
void pe_gemm_launch(const uint16_t* A, const uint16_t* Bw, void* C, bool bf16_out, int M, int N, int K, int Mst,
                    hipStream_t st) {
  const dim3 grid((unsigned)((Mst + GT - 1) / GT), (unsigned)(N / GT));
  if (bf16_out) hipLaunchKernelGGL(pe_gemm_kernel<true>, grid, dim3(256), 0, st, A, Bw, C, M, N, K, Mst);
  else hipLaunchKernelGGL(pe_gemm_kernel<false>, grid, dim3(256), 0, st, A, Bw, C, M, N, K, Mst);
}
void pe_weight_prep_launch(const float* W, const float* W2, int O1, const float* g, const float* b, const float* bias,
                           int O, int nc, int kin, int Kp, uint16_t* Wg, float* wpg, float* gw, float* bw, float* wt,
                           hipStream_t st) {
  hipLaunchKernelGGL(pe_weight_prep_kernel, dim3((unsigned)O), dim3(256), 0, st, W, W2, O1, g, b, bias, O, nc, kin, Kp, Wg,
                     wpg, gw, bw, wt);
}

void pe_proj_fwd_launch(const float* pix, int nc, const float* P, const float* pes, const float* pesq,
                        const float* wpg, const float* gw, const float* bw, long long R, int M, int O, int kin,
                        float eps, uint16_t* y, float* mean, float* rstd, hipStream_t st) {
  // one wave per pixel looping over a batch slice; small images split the batch over
  // blockIdx.y so the grid still holds ≥ 16k waves
  const int B = (int)(R / M);
  int splits = (16384 + M - 1) / M;
  splits = splits < 1 ? 1 : (splits > B ? B : splits);
  if ((B + splits - 1) / splits > 64) splits = (B + 63) / 64;  // a batch slice fits one wave's lanes
  const int bchunk = (B + splits - 1) / splits;
  const dim3 grid((unsigned)((M + 3) / 4), (unsigned)((B + bchunk - 1) / bchunk));
  hipLaunchKernelGGL(pe_proj_fwd_kernel, grid, dim3(256), 0, st, pix, nc, P, pes, pesq, wpg, gw, bw, B, bchunk, M, O,
                     1.f / (float)kin, eps, y, mean, rstd);
}

int pe_proj_bwd_blocks(int M) {
  int blocks = (M + 3) / 4;
  return blocks > 8192 ? 8192 : blocks;
}

void pe_proj_bwd_launch(const float* dy, const float* pix, int nc, const float* mean, const float* rstd, int B, int M,
                        int O, float* D, float* part, hipStream_t st) {
  const size_t lds = (size_t)4 * (2 + nc) * O * sizeof(float);
  hipLaunchKernelGGL(pe_proj_bwd_kernel, dim3((unsigned)pe_proj_bwd_blocks(M)), dim3(256), lds, st, dy, pix, nc, mean,
                     rstd, B, M, O, D, part);
}

}  // namespace pio
