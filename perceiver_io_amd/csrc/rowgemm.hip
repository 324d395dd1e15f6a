// Row-local fused GEMM kernels for the Perceiver's narrow layers (C = 64..133 channels).
//
// With C ≤ 133 every projection in the model is a skinny GEMM (K-dim 64–160) whose cost is
// moving activations, not MFMA time, so these kernels fuse everything
// that is row-local around the attention core:
//   ln_linear_fwd   : LayerNorm prologue (fp32 stats) → X·Wᵀ + b (+GELU) (+residual)
//                     (reference mlp/q_norm/kv_norm/norm + MHA in-proj, model.py:20-26,89-99,108-116)
//   post_attn_fwd   : out-proj + bias + residual → LN2 → W1 + b1 → GELU → W2 + b2 + residual,
//                     one kernel per 64-row tile, intermediates in LDS (Residual(attn) →
//                     Residual(mlp), model.py:29-56)
//   post_attn_bwd   : the reverse chain for one 64-row tile: dZ → dH → dU (GELU') → LN2 bwd →
//                     dY → dO (+ softmax delta = rowsum(dO∘O) for the attention backward), with
//                     the Wo/W1/W2/bias/LN2 parameter gradients computed from the resident tiles
//   ln_linear_bwd   : dX = LN_bwd(G·W) (+ residual grad) plus dW = Gᵀ·LN(X), db, dγ, dβ
//   wgrad           : standalone dW = Σ_rows Gᵀ·A', db = Σ_rows G, A' recomputed on load
// Parameter gradients are accumulated with fp32 atomics straight into the caller's gradient
// tensors (views of the flat gradient buffer): no partial slabs, no reduction launches.
// All GEMMs are v_mfma_f32_32x32x16_bf16 on LDS tiles (common.h operand helpers); a 64-row
// tile spans four waves, each owning whole 32×32 output sub-tiles.
#include "common.h"

namespace pio {

__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ float ldf(const uint16_t* p) { return bf2f(*p); }
__device__ __forceinline__ void stf(float* p, float v) { *p = v; }
__device__ __forceinline__ void stf(uint16_t* p, float v) { *p = f2bf(v); }

// C (+)= A·B over K on LDS tiles; sub-tile tg = w + 4t of a (BM/32)×(BN/32) grid.
// A_KC: A stored [m][k] (else [k][m]); B_KC: B stored [n][k] (else [k][n]).
template <int MAXT, bool A_KC, bool B_KC>
__device__ __forceinline__ void tile_gemm(const uint16_t* sA, int lda, const uint16_t* sB, int ldb, int BM, int BN,
                                          int K, f32x16 (&acc)[MAXT]) {
  const int w = wave_id();
  const int ntn = BN / 32, nt = (BM / 32) * ntn;
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int tg = w + 4 * t;
    if (tg < nt) {  // wave-uniform
      const int m0 = 32 * (tg / ntn), n0 = 32 * (tg % ntn);
      for (int k0 = 0; k0 < K; k0 += 16) {
        const bf16x8 a = A_KC ? frag_kc(sA, lda, m0, k0) : frag_ks(sA, lda, m0, k0);
        const bf16x8 b = B_KC ? frag_kc(sB, ldb, n0, k0) : frag_ks(sB, ldb, n0, k0);
        acc[t] = mfma32(a, b, acc[t]);
      }
    }
  }
}

// visit every element of this wave's accumulator sub-tiles: f(t, m, n, reg)
template <int MAXT, typename F>
__device__ __forceinline__ void for_acc(int BM, int BN, F&& f) {
  const int w = wave_id(), l = lane_id(), hh = l >> 5;
  const int ntn = BN / 32, nt = (BM / 32) * ntn;
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int tg = w + 4 * t;
    if (tg < nt) {
      const int m0 = 32 * (tg / ntn), n0 = 32 * (tg % ntn);
#pragma unroll
      for (int i = 0; i < 16; ++i) f(t, m0 + acc_row(i, hh), n0 + (l & 31), i);
    }
  }
}

// stage rows [r0, r0+rows) × cols [c0, c0+cols) of a row-major matrix into an LDS bf16
// tile [rows][ld] (zero outside the matrix).
__device__ __forceinline__ bf16x8 load8(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ bf16x8 load8(const float* p) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  bf16x8 r;
  r[0] = (short)f2bf(a.x); r[1] = (short)f2bf(a.y); r[2] = (short)f2bf(a.z); r[3] = (short)f2bf(a.w);
  r[4] = (short)f2bf(b.x); r[5] = (short)f2bf(b.y); r[6] = (short)f2bf(b.z); r[7] = (short)f2bf(b.w);
  return r;
}

template <typename T>
__device__ __forceinline__ void stage(uint16_t* s, int ld, const T* g, long long g_rs, int r0, int R, int c0, int Cmax,
                                      int rows, int cols) {
  // 16-byte path (8 elements per access) when the layout allows it, scalar otherwise
  if ((cols & 7) == 0 && (ld & 7) == 0 && (g_rs & 7) == 0 && (c0 & 7) == 0 &&
      (reinterpret_cast<uintptr_t>(g) & 15) == 0) {
    const int cpr = cols >> 3;
    for (int e = threadIdx.x; e < rows * cpr; e += blockDim.x) {
      const int rr = e / cpr, cc = (e % cpr) * 8;
      const int gr = r0 + rr, gc = c0 + cc;
      bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (gr < R) {
        const T* p = g + (long long)gr * g_rs + gc;
        if (gc + 8 <= Cmax) {
          v = load8(p);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = gc + j < Cmax ? (short)f2bf(ldf(p + j)) : (short)0;
        }
      }
      *reinterpret_cast<bf16x8*>(s + rr * ld + cc) = v;
    }
    return;
  }
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
    const int rr = e / cols, cc = e % cols;
    const int gr = r0 + rr, gc = c0 + cc;
    float v = 0.f;
    if (gr < R && gc < Cmax) v = ldf(g + (long long)gr * g_rs + gc);
    s[rr * ld + cc] = f2bf(v);
  }
}

// fp32 gradient targets of the post-attention block (views of the flat gradient buffer)
struct PostAttnGrads {
  float *dWo, *dbo, *dg2, *dbe2, *dW1, *db1, *dW2, *db2;
};

__host__ __device__ __forceinline__ int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ------------------------------------------------------------------------------------
// LayerNorm(+)Linear forward
// ------------------------------------------------------------------------------------
template <typename TIn, typename TOut>
__global__ __launch_bounds__(256) void ln_linear_fwd_kernel(const TIn* __restrict__ X, int x_rs, int R, int Kin,
                                                            const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                            float eps, const uint16_t* __restrict__ W,
                                                            const float* __restrict__ bias, int N, int act,
                                                            const float* __restrict__ res, int res_rs,
                                                            TOut* __restrict__ Y, int y_rs, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int KP = round_up(Kin, 16), ld = KP + 8;
  uint16_t* sA = smem;
  uint16_t* sB = smem + 64 * ld;
  const int m0 = blockIdx.x * 64;
  const int w = wave_id(), l = lane_id();

  // LN prologue once per 64-row tile (one wave per row, x row cached in registers), then all
  // N columns of the output are produced 64 at a time against the resident normalised tile
  float gw[4], gb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = l + 64 * j;
    gw[j] = (lnw && k < Kin) ? lnw[k] : 1.f;
    gb[j] = (lnw && k < Kin) ? lnb[k] : 0.f;
  }
  for (int rr = w; rr < 64; rr += 4) {
    const int gr = m0 + rr;
    float xv[4] = {0.f, 0.f, 0.f, 0.f};
    if (gr < R) {
      const TIn* xr = X + (long long)gr * x_rs;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (l + 64 * j < Kin) xv[j] = ldf(xr + l + 64 * j);
      if (lnw) {
        const float mean = wave_sum(xv[0] + xv[1] + xv[2] + xv[3]) / Kin;
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (l + 64 * j < Kin) v += (xv[j] - mean) * (xv[j] - mean);
        const float rstd = rsqrtf(wave_sum(v) / Kin + eps);
        if (l == 0 && mean_out) { mean_out[gr] = mean; rstd_out[gr] = rstd; }
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[j] = (xv[j] - mean) * rstd * gw[j] + gb[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = l + 64 * j;
      if (k < KP) sA[rr * ld + k] = (gr < R && k < Kin) ? f2bf(xv[j]) : (uint16_t)0;
    }
  }
  for (int n0 = 0; n0 < N; n0 += 64) {
    stage(sB, ld, W, Kin, n0, N, 0, Kin, 64, KP);
    __syncthreads();
    f32x16 acc[1] = {f32x16{}};
    tile_gemm<1, true, true>(sA, ld, sB, ld, 64, 64, KP, acc);
    for_acc<1>(64, 64, [&](int t, int m, int n, int i) {
      const int gr = m0 + m, gc = n0 + n;
      if (gr < R && gc < N) {
        float v = acc[t][i] + (bias ? bias[gc] : 0.f);
        if (act == 1) v = gelu_f(v);
        if (res) v += res[(long long)gr * res_rs + gc];
        stf(Y + (long long)gr * y_rs + gc, v);
      }
    });
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
// post-attention block forward: Z = Y + W2·gelu(W1·LN2(Y) + b1) + b2, Y = X + Wo·O + bo
// ------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(256) void post_attn_fwd_kernel(
    const uint16_t* __restrict__ O, const float* __restrict__ X, const uint16_t* __restrict__ Wo,
    const float* __restrict__ bo, const float* __restrict__ g2, const float* __restrict__ be2, float eps,
    const uint16_t* __restrict__ W1, const float* __restrict__ b1, const uint16_t* __restrict__ W2,
    const float* __restrict__ b2, float* __restrict__ Z, float* __restrict__ Ysave, float* __restrict__ mean2,
    float* __restrict__ rstd2, uint16_t* __restrict__ Usave, int R) {
  constexpr int LD = C + 8, LDF = C + 4, MAXT = (2 * C / 32 + 3) / 4;
  __shared__ __attribute__((aligned(16))) uint16_t sA[64 * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[C * LD];
  __shared__ __attribute__((aligned(16))) float sY[64 * LDF];
  const int m0 = blockIdx.x * 64;
  const int w = wave_id(), l = lane_id();

  stage(sA, LD, O, C, m0, R, 0, C, 64, C);
  stage(sW, LD, Wo, C, 0, C, 0, C, C, C);
  __syncthreads();
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, true>(sA, LD, sW, LD, 64, C, C, acc);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) {
    const int gr = m0 + m;
    float y = 0.f;
    if (gr < R) {
      y = X[(long long)gr * C + n] + acc[t][i] + bo[n];
      Ysave[(long long)gr * C + n] = y;
    }
    sY[m * LDF + n] = y;
  });
  __syncthreads();
  // LN2 (one wave per row) → sA ; W1 → sW
  for (int rr = w; rr < 64; rr += 4) {
    float s = 0.f;
    for (int k = l; k < C; k += 64) s += sY[rr * LDF + k];
    const float mean = wave_sum(s) / C;
    float v = 0.f;
    for (int k = l; k < C; k += 64) { const float d = sY[rr * LDF + k] - mean; v += d * d; }
    const float rstd = rsqrtf(wave_sum(v) / C + eps);
    const int gr = m0 + rr;
    if (l == 0 && gr < R) { mean2[gr] = mean; rstd2[gr] = rstd; }
    for (int k = l; k < C; k += 64) sA[rr * LD + k] = f2bf((sY[rr * LDF + k] - mean) * rstd * g2[k] + be2[k]);
  }
  stage(sW, LD, W1, C, 0, C, 0, C, C, C);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, true>(sA, LD, sW, LD, 64, C, C, acc);
  __syncthreads();  // everyone done reading sA / sW
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) {
    const int gr = m0 + m;
    const float u = acc[t][i] + b1[n];
    if (gr < R) Usave[(long long)gr * C + n] = f2bf(u);
    sA[m * LD + n] = f2bf(gelu_f(u));
  });
  stage(sW, LD, W2, C, 0, C, 0, C, C, C);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, true>(sA, LD, sW, LD, 64, C, C, acc);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) {
    const int gr = m0 + m;
    if (gr < R) Z[(long long)gr * C + n] = sY[m * LDF + n] + acc[t][i] + b2[n];
  });
}

// ------------------------------------------------------------------------------------
// activation tile staging with the forward transform re-applied on load:
// mode 0 plain, 1 LayerNorm (row stats + affine), 2 GELU.  Rows ≥ R and cols ≥ Kin are zero.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void xform8(float (&v)[8], int amode, int gr, int k, const float* mean, const float* rstd,
                                       const float* lnw, const float* lnb) {
  if (amode == 1) {
    const float mu = mean[gr], rs = rstd[gr];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (v[j] - mu) * rs * lnw[k + j] + lnb[k + j];
  } else if (amode == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_f(v[j]);
  }
}

template <typename T>
__device__ __forceinline__ void stage_act(uint16_t* s, int ld, const T* A, long long a_rs, int r0, int R, int Kin,
                                          int cols, int amode, const float* mean, const float* rstd,
                                          const float* lnw, const float* lnb) {
  if ((Kin & 7) == 0 && (a_rs & 7) == 0 && (cols & 7) == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0) {
    const int cpr = cols >> 3;
    for (int e = threadIdx.x; e < 64 * cpr; e += blockDim.x) {
      const int rr = e / cpr, k = (e % cpr) * 8;
      const int gr = r0 + rr;
      bf16x8 o = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (gr < R && k < Kin) {
        const T* p = A + (long long)gr * a_rs + k;
        float v[8];
        if constexpr (sizeof(T) == 2) {
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = bf2f(b[j]);
        } else {
          const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        }
        xform8(v, amode, gr, k, mean, rstd, lnw, lnb);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(v[j]);
      }
      *reinterpret_cast<bf16x8*>(s + rr * ld + k) = o;
    }
    return;
  }
  for (int e = threadIdx.x; e < 64 * cols; e += blockDim.x) {
    const int rr = e / cols, k = e % cols;
    const int gr = r0 + rr;
    float v = 0.f;
    if (gr < R && k < Kin) {
      v = ldf(A + (long long)gr * a_rs + k);
      if (amode == 1) v = (v - mean[gr]) * rstd[gr] * lnw[k] + lnb[k];
      else if (amode == 2) v = gelu_f(v);
    }
    s[rr * ld + k] = f2bf(v);
  }
}

// weight-gradient partial of one 64-row tile, flushed with atomics into the fp32 gradient:
// dW[n][k] += Σ_r sG[r][n] · sX[r][k]  (both tiles row-major [r][·] in LDS → k-strided
// operands).  Each wave instruction adds two 128-byte row segments: the full-rate atomic shape.
template <int MAXW>
__device__ __forceinline__ void wgrad_tile(const uint16_t* sG, int ldg, const uint16_t* sX, int ldx, int NG, int KX,
                                           int Nvalid, int Kvalid, float* __restrict__ dW, int dw_rs) {
  f32x16 acc[MAXW];
#pragma unroll
  for (int t = 0; t < MAXW; ++t) acc[t] = f32x16{};
  tile_gemm<MAXW, false, false>(sG, ldg, sX, ldx, NG, KX, 64, acc);
  for_acc<MAXW>(NG, KX, [&](int t, int m, int n, int i) {
    if (m < Nvalid && n < Kvalid) atomicAdd(dW + (long long)m * dw_rs + n, acc[t][i]);
  });
}

// ------------------------------------------------------------------------------------
// post-attention block backward, one 64-row tile, weight gradients included:
//   dH = dZ·W2, dW2 += dZᵀ·GELU(U), db2 += Σ dZ
//   dU = dH∘GELU'(U), dXn2 = dU·W1, dW1 += dUᵀ·LN2(Y), db1 += Σ dU
//   dY = dZ + LN2_bwd(dXn2), dγ2/dβ2 partials
//   dO = dY·Wo, dWo += dYᵀ·O, dbo += Σ dY, delta = rowsum_head(dO∘O)
// The gradient tile (sG) and its matching activation tile (sX) sit side by side in LDS, so
// each weight gradient is one extra MFMA pass over tiles that are already resident.
// ------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(256) void post_attn_bwd_kernel(
    const float* __restrict__ dZ, const float* __restrict__ Ysave, const float* __restrict__ mean2,
    const float* __restrict__ rstd2, const uint16_t* __restrict__ U, const uint16_t* __restrict__ O,
    const uint16_t* __restrict__ Wo, const uint16_t* __restrict__ W1, const uint16_t* __restrict__ W2,
    const float* __restrict__ g2, const float* __restrict__ be2, float* __restrict__ dY, uint16_t* __restrict__ dO,
    float* __restrict__ delta, int H, PostAttnGrads gr_out, int R) {
  constexpr int LD = C + 8, LDF = C + 4, MAXT = (2 * C / 32 + 3) / 4, MAXW = ((C / 32) * (C / 32) + 3) / 4;
  constexpr int NJ = (C + 63) / 64, GRP = 256 / C, RPG = 64 / GRP;
  __shared__ __attribute__((aligned(16))) uint16_t sG[64 * LD];  // dZ → dU → dY
  __shared__ __attribute__((aligned(16))) uint16_t sX[64 * LD];  // GELU(U) → LN2(Y) → O
  __shared__ __attribute__((aligned(16))) uint16_t sW[C * LD];   // W2 → W1 → Wo
  __shared__ __attribute__((aligned(16))) float sF[64 * LDF];
  __shared__ float sPart[4][4][C];  // per-wave column partials: dγ2, dβ2, Σ dY, Σ dZ
  const int m0 = blockIdx.x * 64;
  const int w = wave_id(), l = lane_id();

  // ---- MLP output layer
  stage(sG, LD, dZ, C, m0, R, 0, C, 64, C);
  stage_act(sX, LD, U, C, m0, R, C, C, 2, nullptr, nullptr, nullptr, nullptr);
  stage(sW, LD, W2, C, 0, C, 0, C, C, C);
  __syncthreads();
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, false>(sG, LD, sW, LD, 64, C, C, acc);  // dH
  wgrad_tile<MAXW>(sG, LD, sX, LD, C, C, C, C, gr_out.dW2, C);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) {
    const int gr = m0 + m;
    sF[m * LDF + n] = gr < R ? acc[t][i] * gelu_grad(bf2f(U[(long long)gr * C + n])) : 0.f;
  });
  __syncthreads();
  // ---- MLP hidden layer: db1 column sums (fp32), dU → bf16 tile, LN2(Y) tile, W1
  {
    const int c = threadIdx.x % C, g = threadIdx.x / C;
    float s = 0.f;
#pragma unroll 4
    for (int r = g * RPG; r < (g + 1) * RPG; ++r) s += sF[r * LDF + c];
    atomicAdd(gr_out.db1 + c, s);
  }
  for (int e = threadIdx.x; e < 64 * C / 4; e += blockDim.x) {
    const int r = e / (C / 4), c = (e % (C / 4)) * 4;
    const float4 v = *reinterpret_cast<const float4*>(sF + r * LDF + c);
    *reinterpret_cast<uint32_t*>(sG + r * LD + c) = pack2(v.x, v.y);
    *reinterpret_cast<uint32_t*>(sG + r * LD + c + 2) = pack2(v.z, v.w);
  }
  stage_act(sX, LD, Ysave, C, m0, R, C, C, 1, mean2, rstd2, g2, be2);
  stage(sW, LD, W1, C, 0, C, 0, C, C, C);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, false>(sG, LD, sW, LD, 64, C, C, acc);  // dXn2 = dU · W1
  wgrad_tile<MAXW>(sG, LD, sX, LD, C, C, C, C, gr_out.dW1, C);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) { sF[m * LDF + n] = acc[t][i]; });
  __syncthreads();
  // ---- LN2 backward → dY = dZ + LN_bwd ; column partials
  float pg[NJ], pb[NJ], py[NJ], pz[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) pg[j] = pb[j] = py[j] = pz[j] = 0.f;
  for (int rr = w; rr < 64; rr += 4) {
    const int gr = m0 + rr;
    if (gr >= R) {
      for (int k = l; k < C; k += 64) sG[rr * LD + k] = 0;
      continue;
    }
    const float mean = mean2[gr], rstd = rstd2[gr];
    float xh[NJ], dxn[NJ], dz[NJ];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = l + 64 * j;
      xh[j] = dxn[j] = dz[j] = 0.f;
      if (k < C) {
        xh[j] = (Ysave[(long long)gr * C + k] - mean) * rstd;
        dxn[j] = sF[rr * LDF + k];
        dz[j] = dZ[(long long)gr * C + k];
        const float g = dxn[j] * g2[k];
        s1 += g;
        s2 += g * xh[j];
      }
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int k = l + 64 * j;
      if (k < C) {
        const float d = dz[j] + rstd * (dxn[j] * g2[k] - s1 - xh[j] * s2);
        dY[(long long)gr * C + k] = d;
        sG[rr * LD + k] = f2bf(d);
        pg[j] += dxn[j] * xh[j];
        pb[j] += dxn[j];
        py[j] += d;
        pz[j] += dz[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int k = l + 64 * j;
    if (k < C) { sPart[0][w][k] = pg[j]; sPart[1][w][k] = pb[j]; sPart[2][w][k] = py[j]; sPart[3][w][k] = pz[j]; }
  }
  // ---- out-projection
  stage(sX, LD, O, C, m0, R, 0, C, 64, C);
  stage(sW, LD, Wo, C, 0, C, 0, C, C, C);
  __syncthreads();
  for (int e = threadIdx.x; e < 4 * C; e += blockDim.x) {
    const int q = e / C, k = e % C;
    float* dst = q == 0 ? gr_out.dg2 : q == 1 ? gr_out.dbe2 : q == 2 ? gr_out.dbo : gr_out.db2;
    atomicAdd(dst + k, sPart[q][0][k] + sPart[q][1][k] + sPart[q][2][k] + sPart[q][3][k]);
  }
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, false>(sG, LD, sW, LD, 64, C, C, acc);  // dO = dY · Wo
  wgrad_tile<MAXW>(sG, LD, sX, LD, C, C, C, C, gr_out.dWo, C);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) {
    const int gr = m0 + m;
    const uint16_t d = f2bf(acc[t][i]);
    sF[m * LDF + n] = bf2f(d);
    if (gr < R) dO[(long long)gr * C + n] = d;
  });
  __syncthreads();
  // delta[r, h] = Σ_d dO·O over the head's columns (bf16 values, as the attention sees them)
  const int D = C / H;
  for (int e = threadIdx.x; e < 64 * H; e += blockDim.x) {
    const int rr = e / H, h = e % H;
    const int gr = m0 + rr;
    if (gr < R) {
      float s = 0.f;
      for (int d = 0; d < D; ++d) s += sF[rr * LDF + h * D + d] * bf2f(sX[rr * LD + h * D + d]);
      delta[(long long)gr * H + h] = s;
    }
  }
}

// ------------------------------------------------------------------------------------
// LayerNorm(+)Linear backward, one 64-row tile:
//   dXn = G·W (N streamed in 64-column chunks), dW += Gᵀ·LN(X), db += Σ G (per chunk, atomics)
//   dX = LN_bwd(dXn) (+ dres), dγ/dβ partials (atomics)
// ------------------------------------------------------------------------------------
template <typename TG, typename TX>
__global__ __launch_bounds__(256) void ln_linear_bwd_kernel(
    const TG* __restrict__ G, int g_rs, int N, const uint16_t* __restrict__ W, int Kin, const TX* __restrict__ X,
    int x_rs, const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ lnw,
    const float* __restrict__ lnb, const float* __restrict__ dres, int dres_rs, float* __restrict__ dX, int dx_rs,
    float* __restrict__ dlnw, float* __restrict__ dlnb, float* __restrict__ dW, float* __restrict__ db, int R) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int KP = round_up(Kin, 32), ld = KP + 8, ldg = 64 + 8, ldF = KP + 4;
  uint16_t* sG = smem;                 // [64 rows][64 n]
  uint16_t* sW = sG + 64 * ldg;        // [64 n][KP]
  uint16_t* sXn = sW + 64 * ld;        // [64 rows][KP]  LN(X), the forward GEMM's A operand
  float* sF = reinterpret_cast<float*>(sXn + 64 * ld);  // [64][KP] fp32
  float* sPart = sF + 64 * ldF;        // [2][4][KP]
  const int m0 = blockIdx.x * 64;
  const int w = wave_id(), l = lane_id();
  constexpr int MAXT = 3;  // (64/32)*(KP/32) ≤ 10 sub-tiles (KP ≤ 160)
  if (dW) stage_act(sXn, ld, X, x_rs, m0, R, Kin, KP, lnw ? 1 : 0, mean, rstd, lnw, lnb);
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  for (int nc = 0; nc < N; nc += 64) {
    __syncthreads();
    stage(sG, ldg, G, g_rs, m0, R, nc, N, 64, 64);
    stage(sW, ld, W, Kin, nc, N, 0, Kin, 64, KP);
    __syncthreads();
    tile_gemm<MAXT, true, false>(sG, ldg, sW, ld, 64, KP, 64, acc);
    if (dW) {
      wgrad_tile<MAXT>(sG, ldg, sXn, ld, 64, KP, N - nc, Kin, dW + (long long)nc * Kin, Kin);
      if (db) {  // fp32 column sums of this G chunk: 4 row-quarters per column
        const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
        if (nc + c < N) {
          float s = 0.f;
#pragma unroll 4
          for (int r = m0 + 16 * q; r < min(R, m0 + 16 * q + 16); ++r) s += ldf(G + (long long)r * g_rs + nc + c);
          atomicAdd(db + nc + c, s);
        }
      }
    }
  }
  for_acc<MAXT>(64, KP, [&](int t, int m, int n, int i) { sF[m * ldF + n] = acc[t][i]; });
  __syncthreads();
  const int NJ = (KP + 63) / 64;
  float pg[3] = {0.f, 0.f, 0.f}, pb[3] = {0.f, 0.f, 0.f};
  float gw[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) gw[j] = (lnw && l + 64 * j < Kin) ? lnw[l + 64 * j] : 0.f;
  for (int rr = w; rr < 64; rr += 4) {
    const int gr = m0 + rr;
    if (gr >= R) continue;
    if (lnw) {
      const float mu = mean[gr], rs = rstd[gr];
      float xh[3], dxn[3];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int k = l + 64 * j;
        xh[j] = dxn[j] = 0.f;
        if (j < NJ && k < Kin) {
          xh[j] = (ldf(X + (long long)gr * x_rs + k) - mu) * rs;
          dxn[j] = sF[rr * ldF + k];
          const float g = dxn[j] * gw[j];
          s1 += g;
          s2 += g * xh[j];
        }
      }
      s1 = wave_sum(s1) / Kin;
      s2 = wave_sum(s2) / Kin;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int k = l + 64 * j;
        if (j < NJ && k < Kin) {
          pg[j] += dxn[j] * xh[j];
          pb[j] += dxn[j];
          if (dX) {
            float d = rs * (dxn[j] * gw[j] - s1 - xh[j] * s2);
            if (dres) d += dres[(long long)gr * dres_rs + k];
            dX[(long long)gr * dx_rs + k] = d;
          }
        }
      }
    } else if (dX) {
      for (int k = l; k < Kin; k += 64) {
        float d = sF[rr * ldF + k];
        if (dres) d += dres[(long long)gr * dres_rs + k];
        dX[(long long)gr * dx_rs + k] = d;
      }
    }
  }
  if (lnw && dlnw) {
    for (int j = 0; j < NJ; ++j) {
      const int k = l + 64 * j;
      if (k < Kin) { sPart[(0 * 4 + w) * KP + k] = pg[j]; sPart[(1 * 4 + w) * KP + k] = pb[j]; }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < Kin; k += blockDim.x) {
      float a = 0.f, b = 0.f;
      for (int ww = 0; ww < 4; ++ww) { a += sPart[ww * KP + k]; b += sPart[(4 + ww) * KP + k]; }
      atomicAdd(dlnw + k, a);
      atomicAdd(dlnb + k, b);
    }
  }
}

// ------------------------------------------------------------------------------------
// standalone weight gradient (for projections without a fused backward producer):
// dW[n][k] += Σ_rows G[r][n] · A'[r][k], db[n] += Σ_rows G[r][n], A' = A | LN(A) | GELU(A)
// grid (N/64, row splits); partials flushed with atomics
// ------------------------------------------------------------------------------------
template <typename TG, typename TA>
__global__ __launch_bounds__(256) void wgrad_kernel(const TG* __restrict__ G, int g_rs, int N, const TA* __restrict__ A,
                                                    int a_rs, int Kin, int amode, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, const float* __restrict__ lnw,
                                                    const float* __restrict__ lnb, int R, int rows_per_split,
                                                    float* __restrict__ dW, float* __restrict__ db) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int KP = round_up(Kin, 32), lda = KP + 8, ldg = 64 + 8;
  uint16_t* sG = smem;           // [64 rows][64 n]
  uint16_t* sA = sG + 64 * ldg;  // [64 rows][KP]
  const int n0 = blockIdx.x * 64, s = blockIdx.y;
  const int r_begin = s * rows_per_split, r_end = min(R, r_begin + rows_per_split);
  constexpr int MAXT = 3;
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  float bsum = 0.f;  // thread n = threadIdx.x (< 64)
  for (int r0 = r_begin; r0 < r_end; r0 += 64) {
    __syncthreads();
    stage(sG, ldg, G, g_rs, r0, r_end, n0, N, 64, 64);
    stage_act(sA, lda, A, a_rs, r0, r_end, Kin, KP, amode, mean, rstd, lnw, lnb);
    __syncthreads();
    if (threadIdx.x < 64 && n0 + threadIdx.x < N)
      for (int rr = r0; rr < min(r_end, r0 + 64); ++rr) bsum += ldf(G + (long long)rr * g_rs + n0 + threadIdx.x);
    tile_gemm<MAXT, false, false>(sG, ldg, sA, lda, 64, KP, 64, acc);
  }
  for_acc<MAXT>(64, KP, [&](int t, int m, int n, int i) {
    const int gn = n0 + m;
    if (gn < N && n < Kin) atomicAdd(dW + (long long)gn * Kin + n, acc[t][i]);
  });
  if (db && threadIdx.x < 64 && n0 + threadIdx.x < N) atomicAdd(db + n0 + threadIdx.x, bsum);
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
// kernels whose dynamic LDS can exceed 64 KiB: raise the per-function limit once (gfx950: 160 KiB/CU)
static void set_smem_once(const void* fn) {
  static const void* done[8] = {nullptr};
  for (auto& d : done) {
    if (d == fn) return;
    if (d == nullptr) {
      (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      d = fn;
      return;
    }
  }
}

void ln_linear_fwd_launch(const void* X, bool x_bf16, int x_rs, int R, int Kin, const float* lnw, const float* lnb,
                          float eps, const uint16_t* W, const float* bias, int N, int act, const float* res,
                          int res_rs, void* Y, bool y_bf16, int y_rs, float* mean, float* rstd, hipStream_t st) {
  const int KP = round_up(Kin, 16);
  const size_t smem = 2 * 64 * (KP + 8) * sizeof(uint16_t);
  dim3 grid((R + 63) / 64);
#define LNL(TI, TO)                                                                                         \
  hipLaunchKernelGGL((ln_linear_fwd_kernel<TI, TO>), grid, dim3(256), smem, st, (const TI*)X, x_rs, R, Kin, \
                     lnw, lnb, eps, W, bias, N, act, res, res_rs, (TO*)Y, y_rs, mean, rstd)
  if (x_bf16 && y_bf16) LNL(uint16_t, uint16_t);
  else if (x_bf16) LNL(uint16_t, float);
  else if (y_bf16) LNL(float, uint16_t);
  else LNL(float, float);
#undef LNL
}

void post_attn_fwd_launch(int C, const uint16_t* O, const float* X, const uint16_t* Wo, const float* bo,
                          const float* g2, const float* be2, float eps, const uint16_t* W1, const float* b1,
                          const uint16_t* W2, const float* b2, float* Z, float* Ysave, float* mean2, float* rstd2,
                          uint16_t* Usave, int R, hipStream_t st) {
  dim3 grid((R + 63) / 64);
  if (C == 64)
    hipLaunchKernelGGL(post_attn_fwd_kernel<64>, grid, dim3(256), 0, st, O, X, Wo, bo, g2, be2, eps, W1, b1, W2, b2,
                       Z, Ysave, mean2, rstd2, Usave, R);
  else if (C == 128)
    hipLaunchKernelGGL(post_attn_fwd_kernel<128>, grid, dim3(256), 0, st, O, X, Wo, bo, g2, be2, eps, W1, b1, W2,
                       b2, Z, Ysave, mean2, rstd2, Usave, R);
  else if (C == 32)
    hipLaunchKernelGGL(post_attn_fwd_kernel<32>, grid, dim3(256), 0, st, O, X, Wo, bo, g2, be2, eps, W1, b1, W2, b2,
                       Z, Ysave, mean2, rstd2, Usave, R);
}

void post_attn_bwd_launch(int C, const float* dZ, const float* Ysave, const float* mean2, const float* rstd2,
                          const uint16_t* U, const uint16_t* O, const uint16_t* Wo, const uint16_t* W1,
                          const uint16_t* W2, const float* g2, const float* be2, float* dY, uint16_t* dO,
                          float* delta, int H, const PostAttnGrads& grads, int R, hipStream_t st) {
  dim3 grid((R + 63) / 64);
#define PAB(CC)                                                                                                  \
  hipLaunchKernelGGL(post_attn_bwd_kernel<CC>, grid, dim3(256), 0, st, dZ, Ysave, mean2, rstd2, U, O, Wo, W1, W2, \
                     g2, be2, dY, dO, delta, H, grads, R)
  if (C == 64) PAB(64);
  else if (C == 128) PAB(128);
  else if (C == 32) PAB(32);
#undef PAB
}

void ln_linear_bwd_launch(const void* G, bool g_bf16, int g_rs, int N, const uint16_t* W, int Kin, const void* X,
                          bool x_bf16, int x_rs, const float* mean, const float* rstd, const float* lnw,
                          const float* lnb, const float* dres, int dres_rs, float* dX, int dx_rs, float* dlnw,
                          float* dlnb, float* dW, float* db, int R, hipStream_t st) {
  const int KP = round_up(Kin, 32);
  const size_t smem = 64 * (64 + 8) * 2 + 2 * 64 * (KP + 8) * 2 + 64 * (KP + 4) * 4 + 2 * 4 * KP * 4;
  dim3 grid((R + 63) / 64);
#define LDG(TG, TX)                                                                                              \
  do {                                                                                                           \
    set_smem_once((const void*)ln_linear_bwd_kernel<TG, TX>);                                                    \
    hipLaunchKernelGGL((ln_linear_bwd_kernel<TG, TX>), grid, dim3(256), smem, st, (const TG*)G, g_rs, N, W, Kin, \
                       (const TX*)X, x_rs, mean, rstd, lnw, lnb, dres, dres_rs, dX, dx_rs, dlnw, dlnb, dW, db, R); \
  } while (0)
  if (g_bf16 && x_bf16) LDG(uint16_t, uint16_t);
  else if (g_bf16) LDG(uint16_t, float);
  else if (x_bf16) LDG(float, uint16_t);
  else LDG(float, float);
#undef LDG
}

void wgrad_launch(const void* G, bool g_bf16, int g_rs, int N, const void* A, bool a_bf16, int a_rs, int Kin,
                  int amode, const float* mean, const float* rstd, const float* lnw, const float* lnb, int R,
                  int rows_per_wg, float* dW, float* db, hipStream_t st) {
  const int KP = round_up(Kin, 32);
  const size_t smem = (64 * (64 + 8) + 64 * (KP + 8)) * 2;
  const int rps = round_up(rows_per_wg > 0 ? rows_per_wg : 256, 64);
  dim3 grid((N + 63) / 64, (R + rps - 1) / rps);
#define WG(TG, TA)                                                                                                 \
  hipLaunchKernelGGL((wgrad_kernel<TG, TA>), grid, dim3(256), smem, st, (const TG*)G, g_rs, N, (const TA*)A, a_rs, \
                     Kin, amode, mean, rstd, lnw, lnb, R, rps, dW, db)
  if (g_bf16 && a_bf16) WG(uint16_t, uint16_t);
  else if (g_bf16) WG(uint16_t, float);
  else if (a_bf16) WG(float, uint16_t);
  else WG(float, float);
#undef WG
}

}  // namespace pio
