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

// one wave per input row r = b·M + m; lanes stride the O outputs four at a time
__global__ __launch_bounds__(256) void pe_proj_fwd_kernel(
    const float* __restrict__ pix, int nc, const float* __restrict__ P, const float* __restrict__ pes,
    const float* __restrict__ pesq, const float* __restrict__ wpg, const float* __restrict__ gw,
    const float* __restrict__ bw, long long R, int M, int O, float inv_k, float eps, uint16_t* __restrict__ y,
    float* __restrict__ mean, float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  const int O4 = O >> 2;
  for (long long r = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < R; r += nw) {
    const int m = (int)(r % M);
    float px[4] = {0.f, 0.f, 0.f, 0.f};
    float s = pes[m], sq = pesq[m];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c < nc) {
        const float v = pix[r * nc + c];
        px[c] = v;
        s += v;
        sq += v * v;
      }
    }
    const float mu = s * inv_k;
    const float var = fmaxf(sq * inv_k - mu * mu, 0.f);
    const float rs = rsqrtf(var + eps);
    const float mrs = mu * rs;
    if (lane == 0) {
      mean[r] = mu;
      rstd[r] = rs;
    }
    const float4* Pm = reinterpret_cast<const float4*>(P + (long long)m * O);
    uint2* yr = reinterpret_cast<uint2*>(y + r * O);
    for (int o4 = lane; o4 < O4; o4 += 64) {
      float4 a = Pm[o4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < nc) {
          const float4 w = reinterpret_cast<const float4*>(wpg + (long long)c * O)[o4];
          a.x += px[c] * w.x; a.y += px[c] * w.y; a.z += px[c] * w.z; a.w += px[c] * w.w;
        }
      }
      const float4 g = reinterpret_cast<const float4*>(gw)[o4];
      const float4 b = reinterpret_cast<const float4*>(bw)[o4];
      yr[o4] = make_uint2(pack2(a.x * rs - mrs * g.x + b.x, a.y * rs - mrs * g.y + b.y),
                          pack2(a.z * rs - mrs * g.z + b.z, a.w * rs - mrs * g.w + b.w));
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
#pragma unroll 4
    for (int b = 0; b < B; ++b) {
      const long long r = (long long)b * M + m;
      const float rs = rstd[r], mu = mean[r], mrs = mu * rs;
      float xh[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) xh[c] = c < nc ? (pix[r * nc + c] - mu) * rs : 0.f;
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
  long long blocks = (R + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(pe_proj_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, st, pix, nc, P, pes, pesq, wpg, gw,
                     bw, R, M, O, 1.f / (float)kin, eps, y, mean, rstd);
}

int pe_proj_bwd_blocks(int M) {
  int blocks = (M + 3) / 4;
  return blocks > 2048 ? 2048 : blocks;
}

void pe_proj_bwd_launch(const float* dy, const float* pix, int nc, const float* mean, const float* rstd, int B, int M,
                        int O, float* D, float* part, hipStream_t st) {
  const size_t lds = (size_t)4 * (2 + nc) * O * sizeof(float);
  hipLaunchKernelGGL(pe_proj_bwd_kernel, dim3((unsigned)pe_proj_bwd_blocks(M)), dim3(256), lds, st, dy, pix, nc, mean,
                     rstd, B, M, O, D, part);
}

}  // namespace pio
