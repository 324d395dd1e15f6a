// Fused per-pixel classification head + class-weighted cross-entropy (SURVEY K-17).
//
// Reference: the LArTPC decoder output (B, H·W, C) → ClassificationOutputAdapter linear
// (C → K) → F.cross_entropy(weight = class weights, background 0) (run.py:105-112, 234-241),
// plus the per-class accuracies logged every step (run.py:190-206).  PyTorch runs that as a
// K = 3-column library GEMM (a pathological N for MFMA tiles), softmax, nll_loss and half a dozen
// reductions.  Here one pass reads each row once:
//   fwd: logits (16 lanes per row, C/16 channels per lane, DPP row sums), log-sum-exp, weighted
//        CE, argmax; per-block partial sums [Σw·ce, Σw, n(lab>0), hit(lab>0), (n_k, hit_k)…]
//   bwd: logits again, coef_k = w_lab · g/Σw · (softmax_k − [k = lab]),
//        dH = coefᵀ·W (written once), dW = Σ coef ⊗ h, db = Σ coef (per-block partials)
// Two one-block finalize kernels sum the partials in a fixed order (deterministic; no
// atomics): the loss / accuracies, and dW / db added into the parameter gradients.
#include "common.h"

namespace pio {

__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x124>(v);  // row_ror:4
  v += dpp<0x128>(v);  // row_ror:8
  return v;
}

constexpr int PH_ROWS = 16;  // rows per block iteration: 4 waves × 4 rows (16 lanes per row)

template <int CPL>
__device__ __forceinline__ void load_row(const float* p, float (&h)[CPL]) {
  if constexpr (CPL % 4 == 0) {
#pragma unroll
    for (int j = 0; j < CPL; j += 4) {
      const float4 v = *reinterpret_cast<const float4*>(p + j);
      h[j] = v.x; h[j + 1] = v.y; h[j + 2] = v.z; h[j + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < CPL; j += 2) {
      const float2 v = *reinterpret_cast<const float2*>(p + j);
      h[j] = v.x; h[j + 1] = v.y;
    }
  }
}

template <int C, int K>
__device__ __forceinline__ void row_logits(const float (&h)[C / 16], const float (&wk)[K][C / 16], const float (&bk)[K],
                                           float (&z)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < C / 16; ++j) s = fmaf(h[j], wk[k][j], s);
    z[k] = row16_sum(s) + bk[k];
  }
}

template <int C, int K>
__global__ __launch_bounds__(256) void pixel_ce_fwd_kernel(const float* __restrict__ H, const float* __restrict__ W,
                                                           const float* __restrict__ bias,
                                                           const int64_t* __restrict__ labels,
                                                           const float* __restrict__ wts, long long R,
                                                           float* __restrict__ part) {
  constexpr int CPL = C / 16, NS = 4 + 2 * K;
  const int l = lane_id(), w = wave_id(), sub = l & 15, grp = l >> 4;
  float wk[K][CPL], bk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    load_row<CPL>(W + k * C + sub * CPL, wk[k]);
    bk[k] = bias[k];
  }
  float acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) acc[s] = 0.f;
  for (long long r = (long long)blockIdx.x * PH_ROWS + w * 4 + grp; r < R; r += (long long)gridDim.x * PH_ROWS) {
    float h[CPL], z[K];
    load_row<CPL>(H + r * C + sub * CPL, h);
    const long long lab64 = labels[r];
    row_logits<C, K>(h, wk, bk, z);
    const int lab = (lab64 >= 0 && lab64 < K) ? (int)lab64 : -1;
    float m = z[0];
    int pred = 0;
#pragma unroll
    for (int k = 1; k < K; ++k) {
      pred = z[k] > m ? k : pred;
      m = fmaxf(m, z[k]);
    }
    float se = 0.f, zl = 0.f, wl = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      se += __expf(z[k] - m);
      zl = k == lab ? z[k] : zl;
    }
    if (lab >= 0) wl = wts[lab];
    if (sub == 0 && lab >= 0) {
      const float ce = m + __logf(se) - zl;
      const float hit = pred == lab ? 1.f : 0.f;
      acc[0] += wl * ce;
      acc[1] += wl;
      if (lab > 0) {
        acc[2] += 1.f;
        acc[3] += hit;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        acc[4 + 2 * k] += k == lab ? 1.f : 0.f;
        acc[5 + 2 * k] += k == lab ? hit : 0.f;
      }
    }
  }
  __shared__ float sred[4][NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const float v = wave_sum(acc[s]);
    if (l == 0) sred[w][s] = v;
  }
  __syncthreads();
  if (threadIdx.x < NS)
    part[(long long)blockIdx.x * NS + threadIdx.x] =
        sred[0][threadIdx.x] + sred[1][threadIdx.x] + sred[2][threadIdx.x] + sred[3][threadIdx.x];
}

template <int C, int K>
__global__ __launch_bounds__(256) void pixel_ce_bwd_kernel(const float* __restrict__ H, const float* __restrict__ W,
                                                           const float* __restrict__ bias,
                                                           const int64_t* __restrict__ labels,
                                                           const float* __restrict__ wts,
                                                           const float* __restrict__ gout,
                                                           const float* __restrict__ stats, long long R,
                                                           float* __restrict__ dH, float* __restrict__ part) {
  constexpr int CPL = C / 16, NP = K * C + K;
  const int l = lane_id(), w = wave_id(), sub = l & 15, grp = l >> 4;
  float wk[K][CPL], bk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    load_row<CPL>(W + k * C + sub * CPL, wk[k]);
    bk[k] = bias[k];
  }
  const float gs = gout[0] / stats[1];  // d(Σw·ce / Σw): the loss gradient over Σw
  float gw[K][CPL], gb[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    gb[k] = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j) gw[k][j] = 0.f;
  }
  for (long long r = (long long)blockIdx.x * PH_ROWS + w * 4 + grp; r < R; r += (long long)gridDim.x * PH_ROWS) {
    float h[CPL], z[K];
    load_row<CPL>(H + r * C + sub * CPL, h);
    const long long lab64 = labels[r];
    row_logits<C, K>(h, wk, bk, z);
    const int lab = (lab64 >= 0 && lab64 < K) ? (int)lab64 : -1;
    float m = z[0];
#pragma unroll
    for (int k = 1; k < K; ++k) m = fmaxf(m, z[k]);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      z[k] = __expf(z[k] - m);
      se += z[k];
    }
    const float scale = lab >= 0 ? wts[lab] * gs / se : 0.f;
    const float g1 = lab >= 0 ? wts[lab] * gs : 0.f;
    float coef[K];
#pragma unroll
    for (int k = 0; k < K; ++k) coef[k] = z[k] * scale - (k == lab ? g1 : 0.f);
    float dh[CPL];
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) s = fmaf(coef[k], wk[k][j], s);
      dh[j] = s;
    }
    float* dp = dH + r * C + sub * CPL;
    if constexpr (CPL % 4 == 0) {
#pragma unroll
      for (int j = 0; j < CPL; j += 4) *reinterpret_cast<float4*>(dp + j) = make_float4(dh[j], dh[j + 1], dh[j + 2], dh[j + 3]);
    } else {
#pragma unroll
      for (int j = 0; j < CPL; j += 2) *reinterpret_cast<float2*>(dp + j) = make_float2(dh[j], dh[j + 1]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
      for (int j = 0; j < CPL; ++j) gw[k][j] = fmaf(coef[k], h[j], gw[k][j]);
      gb[k] += sub == 0 ? coef[k] : 0.f;
    }
  }
  // the 4 row groups of a wave hold the same channels (lanes l, l ^ 16, l ^ 32, l ^ 48)
  __shared__ float sred[4][NP];
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const float v = xor32_sum(xor16_sum(gw[k][j]));
      if (grp == 0) sred[w][k * C + sub * CPL + j] = v;
    }
    const float vb = wave_sum(gb[k]);
    if (l == 0) sred[w][K * C + k] = vb;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NP; i += blockDim.x)
    part[(long long)blockIdx.x * NP + i] = sred[0][i] + sred[1][i] + sred[2][i] + sred[3][i];
}

// stats = [column sums of the partials (NS) | acc(lab > 0), acc_1 … acc_{K-1}], loss = Σw·ce / Σw.
// One block of NS waves: wave s sums column s.
__global__ void pixel_ce_finalize_kernel(const float* __restrict__ part, int nblk, int NS, int K,
                                         float* __restrict__ stats, float* __restrict__ loss) {
  const int w = wave_id(), l = lane_id();
  float s = 0.f;
  for (int i = l; i < nblk; i += 64) s += part[(long long)i * NS + w];
  s = wave_sum(s);
  __shared__ float tot[16];
  if (l == 0) tot[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int j = 0; j < NS; ++j) stats[j] = tot[j];
    loss[0] = tot[0] / tot[1];
    stats[NS] = tot[2] > 0.f ? tot[3] / tot[2] : 0.f;
    for (int k = 1; k < K; ++k) stats[NS + k] = tot[4 + 2 * k] > 0.f ? tot[5 + 2 * k] / tot[4 + 2 * k] : 0.f;
  }
}

// dW (K·C) and db (K) += column sums of the (nblk, K·C + K) partials; 64 columns × 16 row
// phases per block, two independent chains per thread, a fixed-order LDS tree at the end
__global__ __launch_bounds__(1024) void pixel_ce_wgrad_kernel(const float* __restrict__ part, int nblk, int NP, int KC,
                                                              float* __restrict__ dW, float* __restrict__ db) {
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6, col = blockIdx.x * 64 + c;
  float s0 = 0.f, s1 = 0.f;
  if (col < NP) {
    int i = ph;
    for (; i + 16 < nblk; i += 32) {
      s0 += part[(long long)i * NP + col];
      s1 += part[(long long)(i + 16) * NP + col];
    }
    if (i < nblk) s0 += part[(long long)i * NP + col];
  }
  __shared__ float red[16][64];
  red[ph][c] = s0 + s1;
  __syncthreads();
  for (int h = 8; h > 0; h >>= 1) {
    if (ph < h) red[ph][c] += red[ph + h][c];
    __syncthreads();
  }
  if (ph == 0 && col < NP) {
    if (col < KC) dW[col] += red[0][c];
    else db[col - KC] += red[0][c];
  }
}

int pixel_ce_blocks(long long R) {
  long long b = (R + PH_ROWS - 1) / PH_ROWS;
  if (b > 512) b = 512;
  return b < 1 ? 1 : (int)b;
}

#define PH_DISPATCH(KERNEL, ...)                                                            \
  do {                                                                                      \
    const dim3 g(pixel_ce_blocks(R)), t(256);                                               \
    if (C == 32 && K == 2) hipLaunchKernelGGL((KERNEL<32, 2>), g, t, 0, st, __VA_ARGS__);   \
    else if (C == 32 && K == 3) hipLaunchKernelGGL((KERNEL<32, 3>), g, t, 0, st, __VA_ARGS__); \
    else if (C == 32 && K == 4) hipLaunchKernelGGL((KERNEL<32, 4>), g, t, 0, st, __VA_ARGS__); \
    else if (C == 64 && K == 2) hipLaunchKernelGGL((KERNEL<64, 2>), g, t, 0, st, __VA_ARGS__); \
    else if (C == 64 && K == 3) hipLaunchKernelGGL((KERNEL<64, 3>), g, t, 0, st, __VA_ARGS__); \
    else if (C == 64 && K == 4) hipLaunchKernelGGL((KERNEL<64, 4>), g, t, 0, st, __VA_ARGS__); \
    else if (C == 128 && K == 2) hipLaunchKernelGGL((KERNEL<128, 2>), g, t, 0, st, __VA_ARGS__); \
    else if (C == 128 && K == 3) hipLaunchKernelGGL((KERNEL<128, 3>), g, t, 0, st, __VA_ARGS__); \
    else if (C == 128 && K == 4) hipLaunchKernelGGL((KERNEL<128, 4>), g, t, 0, st, __VA_ARGS__); \
  } while (0)

void pixel_ce_fwd_launch(int C, int K, const float* H, const float* W, const float* bias, const int64_t* labels,
                         const float* wts, long long R, float* part, float* stats, float* loss, hipStream_t st) {
  if (R > 0) PH_DISPATCH(pixel_ce_fwd_kernel, H, W, bias, labels, wts, R, part);
  const int NS = 4 + 2 * K;
  hipLaunchKernelGGL(pixel_ce_finalize_kernel, dim3(1), dim3(64 * NS), 0, st, part, pixel_ce_blocks(R), NS, K, stats,
                     loss);
}

void pixel_ce_bwd_launch(int C, int K, const float* H, const float* W, const float* bias, const int64_t* labels,
                         const float* wts, const float* gout, const float* stats, long long R, float* dH, float* part,
                         float* dW, float* db, hipStream_t st) {
  if (R > 0) PH_DISPATCH(pixel_ce_bwd_kernel, H, W, bias, labels, wts, gout, stats, R, dH, part);
  const int NP = K * C + K;
  hipLaunchKernelGGL(pixel_ce_wgrad_kernel, dim3((NP + 63) / 64), dim3(1024), 0, st, part, pixel_ce_blocks(R), NP,
                     K * C, dW, db);
}
#undef PH_DISPATCH

}  // namespace pio
