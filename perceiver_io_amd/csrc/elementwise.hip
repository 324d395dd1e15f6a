// Memory-bound kernels: text embedding (+ scale + learned position table) forward/backward,
// BERT masking, fused multi-tensor AdamW over the flat parameter buffer.
//
// Reference parity:
//   TextInputAdapter  emb(x)·sqrt(C) + pos[:L]          perceiver/adapter.py:127-133  (SURVEY K-01)
//   TextMasking       80/10/10 BERT masking, labels      perceiver/model.py:265-293    (SURVEY K-02)
//   AdamW (torch.optim defaults, decoupled wd)           scripts/cli.py:43, lightning.py:44-55 (SURVEY K-15)
// MI355X notes: one launch each, vectorised 16-B accesses on the streaming paths; the
// masking kernel needs no host sync (the reference's nonzero/sum syncs disappear); AdamW
// reads hyper-parameters (lr, step, grad-norm clip factor) from device memory so the
// whole optimizer step can be captured in a hipGraph, and writes the bf16 weight shadow
// that the GEMM kernels consume in the same pass.
#include "common.h"

namespace pio {

// out[r, c] = E[ids[r], c] * scale + P[r % L, c]     (fp32), float4 vectorised over c
__global__ void embed_fwd_kernel(const int64_t* __restrict__ ids, const float* __restrict__ E,
                                 const float* __restrict__ P, float* __restrict__ out, long long rows, int L, int C,
                                 float scale) {
  const int c4 = C / 4;
  const long long n = rows * c4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / c4;
    const int c = (int)(i % c4) * 4;
    const int64_t id = ids[r];
    const float4 e = *reinterpret_cast<const float4*>(E + id * C + c);
    const float4 p = *reinterpret_cast<const float4*>(P + (r % L) * C + c);
    *reinterpret_cast<float4*>(out + r * C + c) =
        make_float4(e.x * scale + p.x, e.y * scale + p.y, e.z * scale + p.z, e.w * scale + p.w);
  }
}

// dE[ids[r]] += g[r] * scale, dP[l] += Σ_b g[b, l]  (both fp32 atomics)
// grid (L, ceil(B / EB)): block (l, j) handles batch rows j·EB .. j·EB+EB-1 of position l, one
// thread per channel; the EB loads per thread are issued together, then the EB scatter-adds
constexpr int EB = 16;
__global__ void embed_bwd_kernel(const int64_t* __restrict__ ids, const float* __restrict__ g, float* __restrict__ dE,
                                 float* __restrict__ dP, int B, int L, int C, float scale) {
  const int l = blockIdx.x, b0 = blockIdx.y * EB;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float v[EB];
    int64_t id[EB];
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      const long long r = (long long)(b0 + j) * L + l;
      const bool ok = b0 + j < B;
      v[j] = ok ? g[r * C + c] : 0.f;
      id[j] = ok ? ids[r] : -1;
    }
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < EB; ++j) {
      acc += v[j];
      if (dE && id[j] >= 0) atomicAdd(dE + id[j] * C + c, v[j] * scale);
    }
    if (dP) atomicAdd(dP + (long long)l * C + c, acc);
  }
}

// dE[id] += scale · Σ g rows with that id, over token positions SORTED by id (perm = the
// sort permutation): each 64-position chunk folds its runs of equal ids in registers and adds
// one row per run, so a frequent id ([MASK] is ~12 % of an MLM batch, [PAD] of a padded one)
// costs a few atomics per chunk instead of one per occurrence.  One thread per channel.
constexpr int ES = 64;
__global__ void embed_bwd_sorted_kernel(const int64_t* __restrict__ sorted_ids, const int64_t* __restrict__ perm,
                                        const float* __restrict__ g, float* __restrict__ dE, long long n, int C,
                                        float scale) {
  const long long j0 = (long long)blockIdx.x * ES;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float v[ES];
#pragma unroll
    for (int j = 0; j < ES; ++j) v[j] = j0 + j < n ? g[perm[j0 + j] * C + c] : 0.f;
    int64_t cur = sorted_ids[j0];
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < ES; ++j) {
      if (j0 + j >= n) break;
      const int64_t id = sorted_ids[j0 + j];
      if (id != cur) {
        atomicAdd(dE + cur * C + c, acc * scale);
        cur = id;
        acc = 0.f;
      }
      acc += v[j];
    }
    atomicAdd(dE + cur * C + c, acc * scale);
  }
}

// BERT masking from three uniform draws per token (torch.rand, graph-safe RNG):
//   sel = ~special & u0 < p ; msk = sel & u1 < 0.9 ; rnd = msk & u2 < 1/9
//   x' = rnd ? rid : (msk ? MASK : x) ; label = sel ? x : -100
__global__ void text_mask_kernel(const int64_t* __restrict__ x, const bool* __restrict__ pad,
                                 const float* __restrict__ u, const int64_t* __restrict__ rid, int64_t* __restrict__ xm,
                                 int64_t* __restrict__ labels, long long n, int unk_id, int mask_id, float p) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int64_t t = x[i];
    const bool special = (t == unk_id) || (pad && pad[i]);
    const bool sel = !special && (u[i] < p);
    const bool msk = sel && (u[n + i] < 0.9f);
    const bool rnd = msk && (u[2 * n + i] < (1.0f / 9.0f));
    xm[i] = rnd ? rid[i] : (msk ? (int64_t)mask_id : t);
    labels[i] = sel ? t : (int64_t)-100;
  }
}

// sum of squares of the flat gradient (for clip_grad_norm) → atomic into out[0]
__global__ void sumsq_kernel(const float* __restrict__ g, long long n, float* __restrict__ out) {
  float s = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = g[i];
    s += v * v;
  }
  s = wave_sum(s);
  __shared__ float red[16];
  if (lane_id() == 0) red[wave_id()] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    atomicAdd(out, t);
  }
}

// hyper[0] = lr, [1] = step (already incremented), [2] = grad sum of squares (if clip > 0),
// [3] = beta1, [4] = beta2 — read from device memory so schedulers can change them between
// replays of a captured step.
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, uint16_t* __restrict__ shadow, long long n,
                             const float* __restrict__ hyper, float eps, float wd, float clip, float gscale) {
  const float lr = hyper[0], step = hyper[1], beta1 = hyper[3], beta2 = hyper[4];
  const float bc1 = 1.f - powf(beta1, step), bc2 = 1.f - powf(beta2, step);
  float gs = gscale;
  if (clip > 0.f) {
    const float norm = sqrtf(hyper[2]);
    const float f = clip / (norm + 1e-6f);
    if (f < 1.f) gs *= f;
  }
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gs;
    float pi = p[i];
    pi *= 1.f - lr * wd;
    const float mi = beta1 * m[i] + (1.f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step_size * mi / (sqrtf(vi) / bc2s + eps);
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

__global__ void cast_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

static dim3 grid_for(long long n, int per = 256) {
  long long b = (n + per - 1) / per;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

void embed_fwd_launch(const int64_t* ids, const float* E, const float* P, float* out, long long rows, int L, int C,
                      float scale, hipStream_t st) {
  hipLaunchKernelGGL(embed_fwd_kernel, grid_for(rows * C / 4), dim3(256), 0, st, ids, E, P, out, rows, L, C, scale);
}
void embed_bwd_launch(const int64_t* ids, const float* g, float* dE, float* dP, int B, int L, int C, float scale,
                      hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(L, (B + EB - 1) / EB), dim3(C < 256 ? C : 256), 0, st, ids, g, dE, dP, B, L,
                     C, scale);
}
void embed_bwd_sorted_launch(const int64_t* sorted_ids, const int64_t* perm, const float* g, float* dE, long long n,
                             int C, float scale, hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_sorted_kernel, dim3((unsigned)((n + ES - 1) / ES)), dim3(C < 256 ? C : 256), 0, st,
                     sorted_ids, perm, g, dE, n, C, scale);
}
void text_mask_launch(const int64_t* x, const bool* pad, const float* u, const int64_t* rid, int64_t* xm,
                      int64_t* labels, long long n, int unk_id, int mask_id, float p, hipStream_t st) {
  hipLaunchKernelGGL(text_mask_kernel, grid_for(n), dim3(256), 0, st, x, pad, u, rid, xm, labels, n, unk_id, mask_id, p);
}
void sumsq_launch(const float* g, long long n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, grid_for(n, 1024), dim3(256), 0, st, g, n, out);
}
void adamw_launch(float* p, const float* g, float* m, float* v, uint16_t* shadow, long long n, const float* hyper,
                  float eps, float wd, float clip, float gscale, hipStream_t st) {
  hipLaunchKernelGGL(adamw_kernel, grid_for(n), dim3(256), 0, st, p, g, m, v, shadow, n, hyper, eps, wd, clip, gscale);
}
// grad[i] += Σ_r rep[r][i], rep[r][i] ← 0 (replicated gradient accumulators, see ops/optim.py)
__global__ void fold_replicas_kernel(float* __restrict__ grad, float* __restrict__ rep, long long n, int nrep) {
  const long long n4 = n >> 2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 acc = reinterpret_cast<float4*>(grad)[i];
    for (int r = 0; r < nrep; ++r) {
      float4* p = reinterpret_cast<float4*>(rep + r * n) + i;
      const float4 v = *p;
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      *p = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    reinterpret_cast<float4*>(grad)[i] = acc;
  }
  for (long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float acc = grad[i];
    for (int r = 0; r < nrep; ++r) { acc += rep[r * n + i]; rep[r * n + i] = 0.f; }
    grad[i] = acc;
  }
}
void fold_replicas_launch(float* grad, float* rep, long long n, int nrep, hipStream_t st) {
  hipLaunchKernelGGL(fold_replicas_kernel, grid_for((n + 3) / 4), dim3(256), 0, st, grad, rep, n, nrep);
}

// standalone form of a SlabJob (common.h): the reductions still pending at the end of a
// backward pass
__global__ __launch_bounds__(256) void slab_reduce_kernel(SlabJob job) {
  __shared__ float4 part[256];
  slab_reduce_block(job, blockIdx.x, part);
}
void slab_reduce_launch(const SlabJob& job, hipStream_t st) {
  if (job.slab == nullptr || job.nblk == 0) return;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(job.nblk), dim3(256), 0, st, job);
}

// one wave: the cross-lane reduction helpers of common.h on x[0..63] (numerics self-test)
__global__ void reduce_probe_kernel(const float* __restrict__ x, float* __restrict__ out) {
  const int l = threadIdx.x;
  const float v = x[l];
  out[l] = wave_sum(v);
  out[64 + l] = wave_max(v);
  out[128 + l] = half_sum(v);
  out[192 + l] = half_max(v);
  out[256 + l] = xor16_sum(v);
  out[320 + l] = xor32_sum(v);
}

void reduce_probe_launch(const float* x, float* out, hipStream_t st) {
  hipLaunchKernelGGL(reduce_probe_kernel, dim3(1), dim3(64), 0, st, x, out);
}

void cast_bf16_launch(const float* x, uint16_t* y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_bf16_kernel, grid_for(n), dim3(256), 0, st, x, y, n);
}

}  // namespace pio
