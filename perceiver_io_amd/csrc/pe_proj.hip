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
