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
                                 float scale, long long V) {
  const int c4 = C / 4;
  const long long n = rows * c4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / c4;
    const int c = (int)(i % c4) * 4;
    int64_t id = ids[r];
#if PIO_CHECKS
    if (id < 0 || id >= V) {
      pio_flag(kErrEmbedId);
      id = id < 0 ? 0 : V - 1;
    }
#else
    (void)V;
#endif
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

// dE[id] += scale · Σ g rows with that id, with NO global sort: each workgroup takes 256
// consecutive token positions, bitonic-sorts their (id, slot) keys in LDS, and every wave walks
// a quarter of the sorted keys with its g rows' loads all in flight (lane = channel), adding
// one contiguous 256-B row per run of equal ids.  A hot id ([MASK] ≈ 12 % of an MLM batch,
// [PAD], frequent words) then costs ≤ 4 row atomics per 256 tokens instead of one per
// occurrence — the property the earlier sort-by-id pipeline (≈10 launches) paid for.
// Workgroups past the token blocks do the position-table gradient dP (batch sums per
// position, embed_bwd_kernel's layout): one launch for the whole text-embedding backward.
constexpr int ET = 256;
template <int C>
__global__ __launch_bounds__(256) void embed_bwd_local_kernel(const int64_t* __restrict__ ids,
                                                              const float* __restrict__ g, float* __restrict__ dE,
                                                              float* __restrict__ dP, long long n, int nblk_e, int B,
                                                              int L, float scale, int nblk_ep, SlabJob job) {
  __shared__ uint32_t sKey[ET];
  __shared__ __attribute__((aligned(16))) float4 sPart[256];  // a deterministic slab job's partials
  const int t = threadIdx.x;
  if ((int)blockIdx.x >= nblk_ep) {  // appended workgroups: the previous backward kernel's slab job
    slab_reduce_block(job, blockIdx.x - nblk_ep, sPart);
    return;
  }
  if ((int)blockIdx.x >= nblk_e) {  // position-table gradient: block (256 / C positions, batch group)
    constexpr int TPP = C < 256 ? C : 256, PPB = 256 / TPP;
    const int nlb = (L + PPB - 1) / PPB;
    const int pb = blockIdx.x - nblk_e, l = (pb % nlb) * PPB + t / TPP, b0 = (pb / nlb) * EB;
    if (l >= L) return;
    for (int c = t % TPP; c < C; c += TPP) {
      float v[EB];
#pragma unroll
      for (int j = 0; j < EB; ++j) v[j] = b0 + j < B ? g[((long long)(b0 + j) * L + l) * C + c] : 0.f;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < EB; ++j) acc += v[j];
      atomicAdd(dP + (long long)l * C + c, acc);
    }
    return;
  }
  const long long j0 = (long long)blockIdx.x * ET;
  sKey[t] = j0 + t < n ? ((uint32_t)ids[j0 + t] << 8) | (uint32_t)t : 0xFFFFFFFFu;  // ids < 2^24
  __syncthreads();
  for (int k = 2; k <= ET; k <<= 1) {
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      const int ix = t ^ jj;
      if (ix > t) {
        const uint32_t a = sKey[t], b = sKey[ix];
        if ((a > b) == ((t & k) == 0)) { sKey[t] = b; sKey[ix] = a; }
      }
      __syncthreads();
    }
  }
  if (dE == nullptr) return;
  constexpr int NC = C / 64;  // channels per lane (lane l: l, l + 64, ...)
  const int w = wave_id(), l = lane_id();
  const int e0 = 64 * w;
  for (int h = 0; h < 64; h += 32) {  // 32 sorted entries at a time: their loads all in flight
    float v[32][NC];
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      const uint32_t key = sKey[e0 + h + e];
      const long long row = j0 + (key & 255u);
#pragma unroll
      for (int q = 0; q < NC; ++q) v[e][q] = key != 0xFFFFFFFFu ? g[row * C + l + 64 * q] : 0.f;
    }
    uint32_t cur = sKey[e0 + h] >> 8;
    float acc[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) acc[q] = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      const uint32_t key = sKey[e0 + h + e];
      if (key == 0xFFFFFFFFu) break;  // padding past n sorts last (wave-uniform)
      if ((key >> 8) != cur) {
#pragma unroll
        for (int q = 0; q < NC; ++q) {
          atomicAdd(dE + (long long)cur * C + l + 64 * q, acc[q] * scale);
          acc[q] = 0.f;
        }
        cur = key >> 8;
      }
#pragma unroll
      for (int q = 0; q < NC; ++q) acc[q] += v[e][q];
    }
    if (cur != (0xFFFFFFFFu >> 8)) {
#pragma unroll
      for (int q = 0; q < NC; ++q) atomicAdd(dE + (long long)cur * C + l + 64 * q, acc[q] * scale);
    }
  }
}

// BERT masking with in-kernel counter-based randomness (no torch RNG kernels, no generator
// bookkeeping in a replayed graph).  Per token i, with key = hash3(seed, counter):
//   u_k = (hash3(key, k, i) >> 8) · 2^-24 (k = 0, 1, 2), rid = lo + mulhi(hash3(key, 3, i), range)
//   sel = ~special & u0 < p ; msk = sel & u1 < 0.9 ; rnd = msk & u2 < 1/9
//   x' = rnd ? rid : (msk ? MASK : x) ; label = sel ? x : -100
// state = {seed, counter, ticket}: with advance != 0 the last workgroup to finish (ticket
// count) increments the counter, so every launch — every replay of a captured step — draws
// fresh masks; every workgroup has read the counter before it takes its ticket.
__device__ __forceinline__ float unit24(uint32_t h) { return (float)(h >> 8) * (1.0f / 16777216.0f); }

__global__ void text_mask_kernel(const int64_t* __restrict__ x, const bool* __restrict__ pad, int64_t* __restrict__ state,
                                 int64_t* __restrict__ xm, int64_t* __restrict__ labels, long long n, int unk_id,
                                 int mask_id, float p, int lo, uint32_t range, int advance) {
  const uint64_t seed = (uint64_t)state[0];
  const int64_t ctr = state[1];
  const uint32_t key = hash3((uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ctr);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const uint32_t ii = (uint32_t)i;
    const int64_t t = x[i];
    const bool special = (t == unk_id) | (pad != nullptr && pad[i]);
    const bool sel = !special & (unit24(hash3(key, 0u, ii)) < p);
    const bool msk = sel & (unit24(hash3(key, 1u, ii)) < 0.9f);
    const bool rnd = msk & (unit24(hash3(key, 2u, ii)) < (1.0f / 9.0f));
    const int64_t rid = (int64_t)lo + (int64_t)__umulhi(hash3(key, 3u, ii), range);
    xm[i] = rnd ? rid : (msk ? (int64_t)mask_id : t);
    labels[i] = sel ? t : (int64_t)-100;
  }
  if (advance) {
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned* ticket = reinterpret_cast<unsigned*>(state + 2);
      if (atomicAdd(ticket, 1u) == gridDim.x - 1) {
        state[1] = ctr + 1;
        *ticket = 0u;
      }
    }
  }
}

// sum of squares of the flat gradient (clip_grad_norm): Σ g² in fixed order, no atomics: block b writes its partial to part[b] (kSumsqBlocks blocks,
// grid-stride, 8 independent 16-byte loads in flight per thread); the AdamW kernels sum the
// partials themselves (adam_clip_scale).  The previous single-address atomic per block put
// 2048 serialised adds at the end of an HBM-bound pass (36 µs for the 68 MB LArTPC gradient).
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, long long n, float* __restrict__ part) {
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const long long n4 = ((reinterpret_cast<uintptr_t>(g) & 15) == 0) ? n >> 2 : 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 7 * stride < n4; i += 8 * stride) {
    float4 a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = g4[i + k * stride];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      s[k] = fmaf(a[k].x, a[k].x, fmaf(a[k].y, a[k].y, fmaf(a[k].z, a[k].z, fmaf(a[k].w, a[k].w, s[k]))));
  }
  for (; i < n4; i += stride) {
    const float4 a = g4[i];
    s[0] = fmaf(a.x, a.x, fmaf(a.y, a.y, fmaf(a.z, a.z, fmaf(a.w, a.w, s[0]))));
  }
  for (long long j = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
    const float v = g[j];
    s[1] = fmaf(v, v, s[1]);
  }
  float t = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  t = wave_sum(t);
  __shared__ float red[4];
  if (lane_id() == 0) red[wave_id()] = t;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// the clip factor of a step from sumsq_kernel's partials, in a fixed order (every block of the
// AdamW grid the same value): wave 0 sums the kSumsqBlocks partials, LDS broadcast
__device__ __forceinline__ float adam_clip_scale(const float* __restrict__ part, float clip, float gscale) {
  __shared__ float s_norm2;
  if (threadIdx.x < 64) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kSumsqBlocks / 64; ++k) t += part[threadIdx.x + 64 * k];
    t = wave_sum(t);
    if (threadIdx.x == 0) s_norm2 = t;
  }
  __syncthreads();
  const float norm = sqrtf(s_norm2) * gscale;
  const float f = clip / (norm + 1e-6f);
  return f < 1.f ? f : 1.f;
}

// hyper[0] = lr, [1] = step (already incremented), [3] = beta1, [4] = beta2, [7] = loss-ring slot — read from device memory so schedulers can
// change them between replays of a captured step.
// loss_src (optional): the step's scalar loss, copied by thread 0 into loss_ring[hyper[7] % ring_n]
// (the step engine hands that slot back as the step's loss: no separate copy launch per step)
// zero_g: the gradient is cleared as it is consumed (a replayed step then needs no separate
// zero fill of the flat gradient buffer before its backward)
// clip > 0: the gradient's sum of squares comes as sumsq_kernel's per-block partials (norm_part)
__global__ void adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, uint16_t* __restrict__ shadow, long long n,
                             const float* __restrict__ hyper, float eps, float wd, float clip, float gscale,
                             int l2, int zero_g, const float* __restrict__ loss_src, float* __restrict__ loss_ring,
                             int ring_n, const float* __restrict__ norm_part) {
  const float lr = hyper[0], step = hyper[1], beta1 = hyper[3], beta2 = hyper[4];
  if (loss_src != nullptr && blockIdx.x == 0 && threadIdx.x == 0) loss_ring[(int)hyper[7] % ring_n] = *loss_src;
  const float bc1 = 1.f - powf(beta1, step), bc2 = 1.f - powf(beta2, step);
  // g holds the all-reduced SUM over ranks (gscale = 1 / world makes it the mean): the clip
  // threshold applies to the norm of the MEAN gradient, as in single-process training
  float gs = gscale;
  if (clip > 0.f) gs *= adam_clip_scale(norm_part, clip, gscale);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float pi = p[i];
    // l2 (torch.optim.Adam weight_decay): the decay joins the (clipped) gradient; else AdamW's
    // decoupled decay of the weights
    const float g0 = g[i];
    if (zero_g) g[i] = 0.f;
    const float gi = l2 ? fmaf(wd, pi, g0 * gs) : g0 * gs;
    if (!l2) pi *= 1.f - lr * wd;
    const float mi = beta1 * m[i] + (1.f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step_size * mi / (sqrtf(vi) / bc2s + eps);
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

// the same update on 4 elements per thread (16-byte loads / stores; every pointer 16-byte
// aligned, the shadow 8-byte aligned, n % 4 == 0 — checked by the launcher): a quarter of the
// memory instructions of the scalar loop, which is issue-bound at ≈40 % of HBM bandwidth
__global__ __launch_bounds__(256) void adamw4_kernel(float4* __restrict__ p, float4* __restrict__ g,
                                                     float4* __restrict__ m, float4* __restrict__ v,
                                                     uint2* __restrict__ shadow, long long n4,
                                                     const float* __restrict__ hyper, float eps, float wd, float clip,
                                                     float gscale, int l2, int zero_g, const float* __restrict__ loss_src,
                                                     float* __restrict__ loss_ring, int ring_n,
                                                     const float* __restrict__ norm_part) {
  const float lr = hyper[0], step = hyper[1], beta1 = hyper[3], beta2 = hyper[4];
  if (loss_src != nullptr && blockIdx.x == 0 && threadIdx.x == 0) loss_ring[(int)hyper[7] % ring_n] = *loss_src;
  const float bc1 = 1.f - powf(beta1, step), bc2 = 1.f - powf(beta2, step);
  float gs = gscale;
  if (clip > 0.f) gs *= adam_clip_scale(norm_part, clip, gscale);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const float4 p4 = p[i], g4 = g[i], m4 = m[i], v4 = v[i];
    if (zero_g) g[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float pa[4] = {p4.x, p4.y, p4.z, p4.w}, ga[4] = {g4.x, g4.y, g4.z, g4.w};
    const float ma[4] = {m4.x, m4.y, m4.z, m4.w}, va[4] = {v4.x, v4.y, v4.z, v4.w};
    float po[4], mo[4], vo[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // the scalar kernel's arithmetic, element by element
      float pi = pa[e];
      const float gi = l2 ? fmaf(wd, pi, ga[e] * gs) : ga[e] * gs;
      if (!l2) pi *= 1.f - lr * wd;
      mo[e] = beta1 * ma[e] + (1.f - beta1) * gi;
      vo[e] = beta2 * va[e] + (1.f - beta2) * gi * gi;
      po[e] = pi - step_size * mo[e] / (sqrtf(vo[e]) / bc2s + eps);
    }
    m[i] = make_float4(mo[0], mo[1], mo[2], mo[3]);
    v[i] = make_float4(vo[0], vo[1], vo[2], vo[3]);
    p[i] = make_float4(po[0], po[1], po[2], po[3]);
    if (shadow) shadow[i] = make_uint2(pack2(po[0], po[1]), pack2(po[2], po[3]));
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
                      float scale, long long V, hipStream_t st) {
  hipLaunchKernelGGL(embed_fwd_kernel, grid_for(rows * C / 4), dim3(256), 0, st, ids, E, P, out, rows, L, C, scale, V);
}
void embed_bwd_launch(const int64_t* ids, const float* g, float* dE, float* dP, int B, int L, int C, float scale,
                      hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(L, (B + EB - 1) / EB), dim3(C < 256 ? C : 256), 0, st, ids, g, dE, dP, B, L,
                     C, scale);
}
// C a multiple of 64 (≤ 256); dE and/or dP
// + the previous backward kernel's slab job in appended workgroups (small LDS: they share the CUs
// with the embedding blocks instead of running after them)
bool embed_bwd_local_launch(const int64_t* ids, const float* g, float* dE, float* dP, int B, int L, int C, float scale,
                            const SlabJob& job, hipStream_t st) {
  if (C != 64 && C != 128 && C != 256) return false;
  const long long n = (long long)B * L;
  const int nblk_e = dE ? (int)((n + ET - 1) / ET) : 0;
  const int ppb = 256 / (C < 256 ? C : 256);
  const int nblk_p = dP ? ((L + ppb - 1) / ppb) * ((B + EB - 1) / EB) : 0;
  const int nblk_ep = nblk_e + nblk_p;
  const dim3 grid(nblk_ep + (job.slab ? job.nblk : 0));
  if (grid.x == 0) return true;
  switch (C) {
    case 64: hipLaunchKernelGGL(embed_bwd_local_kernel<64>, grid, dim3(256), 0, st, ids, g, dE, dP, n, nblk_e, B, L, scale, nblk_ep, job); break;
    case 128: hipLaunchKernelGGL(embed_bwd_local_kernel<128>, grid, dim3(256), 0, st, ids, g, dE, dP, n, nblk_e, B, L, scale, nblk_ep, job); break;
    default: hipLaunchKernelGGL(embed_bwd_local_kernel<256>, grid, dim3(256), 0, st, ids, g, dE, dP, n, nblk_e, B, L, scale, nblk_ep, job); break;
  }
  return true;
}
void embed_bwd_sorted_launch(const int64_t* sorted_ids, const int64_t* perm, const float* g, float* dE, long long n,
                             int C, float scale, hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_sorted_kernel, dim3((unsigned)((n + ES - 1) / ES)), dim3(C < 256 ? C : 256), 0, st,
                     sorted_ids, perm, g, dE, n, C, scale);
}
void text_mask_launch(const int64_t* x, const bool* pad, int64_t* state, int64_t* xm, int64_t* labels, long long n,
                      int unk_id, int mask_id, float p, int lo, uint32_t range, int advance, hipStream_t st) {
  hipLaunchKernelGGL(text_mask_kernel, grid_for(n), dim3(256), 0, st, x, pad, state, xm, labels, n, unk_id, mask_id, p, lo,
                     range, advance);
}
void sumsq_launch(const float* g, long long n, float* part, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(kSumsqBlocks), dim3(256), 0, st, g, n, part);
}

// dst[idx[r]][:] += src[r][:] — the backward of a row gather (rows of idx may repeat: fp32
// atomics; an index outside dst is skipped).  One thread per 4 columns.
__global__ void index_add_rows_kernel(float* __restrict__ dst, long long nrows, const int64_t* __restrict__ idx,
                                      const float* __restrict__ src, long long R, int C) {
  const int c4 = C >> 2;
  const long long total = R * c4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / c4;
    const int c = (int)(i - r * c4) * 4;
    const long long d = idx[r];
#if PIO_CHECKS
    if (d < 0 || d >= nrows) pio_flag(kErrGatherRow);
#endif
    const float4 v = *reinterpret_cast<const float4*>(src + r * C + c);
    // all-zero quads (padding rows of a fixed-capacity gather) skip their atomics: padding
    // slots often share one destination row, whose serialised atomics would dominate
    const bool nz = v.x != 0.f || v.y != 0.f || v.z != 0.f || v.w != 0.f;
    if (nz && d >= 0 && d < nrows) {
      float* p = dst + d * C + c;
      atomicAdd(p, v.x);
      atomicAdd(p + 1, v.y);
      atomicAdd(p + 2, v.z);
      atomicAdd(p + 3, v.w);
    }
  }
}
void index_add_rows_launch(float* dst, long long nrows, const int64_t* idx, const float* src, long long R, int C,
                           hipStream_t st) {
  hipLaunchKernelGGL(index_add_rows_kernel, grid_for(R * (C / 4)), dim3(256), 0, st, dst, nrows, idx, src, R, C);
}
// out (R, C) = src[idx] (the forward of that gather: a decoder's output queries at the pixels of a
// sparse image); an index outside [0, nrows) yields a zero row
__global__ void gather_rows_kernel(float* __restrict__ out, const float* __restrict__ src, long long nrows,
                                   const int64_t* __restrict__ idx, long long R, int C) {
  const int c4 = C >> 2;
  const long long total = R * c4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / c4;
    const int c = (int)(i - r * c4) * 4;
    const long long d = idx[r];
#if PIO_CHECKS
    if (d < 0 || d >= nrows) pio_flag(kErrGatherRow);
#endif
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (d >= 0 && d < nrows) v = *reinterpret_cast<const float4*>(src + d * C + c);
    *reinterpret_cast<float4*>(out + r * C + c) = v;
  }
}
void gather_rows_launch(float* out, const float* src, long long nrows, const int64_t* idx, long long R, int C,
                        hipStream_t st) {
  hipLaunchKernelGGL(gather_rows_kernel, grid_for(R * (C / 4)), dim3(256), 0, st, out, src, nrows, idx, R, C);
}
// Σ over the batch of two (B, n) fp32 tensors in one launch: oa = Σ_b a[b], ob = Σ_b b[b] (the
// gradients of a batch-broadcast query stream: dQ and the residual dY of the first cross-attention
// over the shared latent array).  Block = 64 float4 columns × 4 batch groups, fixed summation
// order (deterministic).  n a multiple of 4, 16-byte aligned rows.
__global__ __launch_bounds__(256) void batch_sum2_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         float* __restrict__ oa, float* __restrict__ ob, int B,
                                                         long long na4, long long nb4, int acc_b) {
  __shared__ float4 part[4][64];
  const int l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long long c = (long long)blockIdx.x * 64 + l;  // float4 column of [a | b]
  const bool second = c >= na4;
  const long long cc = second ? c - na4 : c, n4 = second ? nb4 : na4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < na4 + nb4) {
    const float4* src = reinterpret_cast<const float4*>(second ? b : a) + cc;
#pragma unroll 8
    for (int bb = g; bb < B; bb += 4) {
      const float4 v = src[(long long)bb * n4];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  part[g][l] = acc;
  __syncthreads();
  if (g == 0 && c < na4 + nb4) {
    float4 r = part[0][l];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 v = part[k][l];
      r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    float4* dst = reinterpret_cast<float4*>(second ? ob : oa) + cc;
    if (second && acc_b) {  // ob += Σ_b b (e.g. straight into a parameter's gradient)
      const float4 o = *dst;
      r.x += o.x; r.y += o.y; r.z += o.z; r.w += o.w;
    }
    *dst = r;
  }
}
void batch_sum2_launch(const float* a, const float* b, float* oa, float* ob, int B, long long na, long long nb, int acc_b,
                       hipStream_t st) {
  const long long na4 = a ? na / 4 : 0, nb4 = nb / 4;
  hipLaunchKernelGGL(batch_sum2_kernel, dim3((unsigned)((na4 + nb4 + 63) / 64)), dim3(256), 0, st, a, b, oa, ob, B, na4,
                     nb4, acc_b);
}
void adamw_launch(float* p, float* g, float* m, float* v, uint16_t* shadow, long long n, const float* hyper,
                  float eps, float wd, float clip, float gscale, int l2, int zero_g, const float* loss_src,
                  float* loss_ring, int ring_n, const float* norm_part, hipStream_t st) {
  const bool vec = n % 4 == 0 && ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                                    reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v)) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(shadow) & 7) == 0;
  if (vec)
    hipLaunchKernelGGL(adamw4_kernel, grid_for(n / 4), dim3(256), 0, st, reinterpret_cast<float4*>(p),
                       reinterpret_cast<float4*>(g), reinterpret_cast<float4*>(m), reinterpret_cast<float4*>(v),
                       reinterpret_cast<uint2*>(shadow), n / 4, hyper, eps, wd, clip, gscale, l2, zero_g, loss_src,
                       loss_ring, ring_n, norm_part);
  else
    hipLaunchKernelGGL(adamw_kernel, grid_for(n), dim3(256), 0, st, p, g, m, v, shadow, n, hyper, eps, wd, clip, gscale,
                       l2, zero_g, loss_src, loss_ring, ring_n, norm_part);
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

// ------------------------------------------------------------------------------------------
// Per-step staging for a replayed hipGraph in ONE launch: the new batch's tensors are copied
// into the graph's static input buffers and the optimizer's per-step hyper-parameters (lr,
// step, betas, ...) arrive as kernel arguments (captured by value at launch, so no pinned
// staging ring and no host→device copy).  Replaces one copyBuffer per input tensor + one for
// the hyper-parameters.  Segments whose pointers and size are 16-byte multiples are copied in
// 16-byte units, the others byte-wise.
// ------------------------------------------------------------------------------------------
namespace pio {
constexpr int kStageSegs = 8, kStageHyper = 8, kStageSeeds = 64;
struct StageArgs {
  void* dst[kStageSegs];
  const void* src[kStageSegs];
  long long bytes[kStageSegs];
  int vec[kStageSegs];
  int nseg;
  float* hyper_dst;
  float hyper[kStageHyper];
  int nhyper;
  long long* seed_dst;  // a captured step's dropout seed slots (ops/fused.py static seeds)
  long long seeds[kStageSeeds];
  int nseeds;
};

__global__ __launch_bounds__(256) void stage_step_kernel(StageArgs a) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nt = (long long)gridDim.x * blockDim.x;
  if (blockIdx.x == 0 && threadIdx.x < a.nhyper && a.hyper_dst != nullptr) a.hyper_dst[threadIdx.x] = a.hyper[threadIdx.x];
  if (blockIdx.x == 0 && threadIdx.x < a.nseeds) a.seed_dst[threadIdx.x] = a.seeds[threadIdx.x];
  for (int s = 0; s < a.nseg; ++s) {
    if (a.vec[s]) {
      const long long n = a.bytes[s] >> 4;
      uint4* d = reinterpret_cast<uint4*>(a.dst[s]);
      const uint4* x = reinterpret_cast<const uint4*>(a.src[s]);
      for (long long i = tid; i < n; i += nt) d[i] = x[i];
    } else {
      uint8_t* d = reinterpret_cast<uint8_t*>(a.dst[s]);
      const uint8_t* x = reinterpret_cast<const uint8_t*>(a.src[s]);
      for (long long i = tid; i < a.bytes[s]; i += nt) d[i] = x[i];
    }
  }
}

int stage_step_launch(void* const* dst, const void* const* src, const long long* bytes, int nseg, float* hyper_dst,
                      const float* hyper, int nhyper, long long* seed_dst, const long long* seeds, int nseeds,
                      hipStream_t st) {
  if (nseg > kStageSegs || nhyper > kStageHyper || nseeds > kStageSeeds || (nseeds > 0 && seed_dst == nullptr)) return -1;
  StageArgs a{};
  a.seed_dst = seed_dst;
  a.nseeds = nseeds;
  for (int i = 0; i < nseeds; ++i) a.seeds[i] = seeds[i];
  long long units = 0;
  for (int s = 0; s < nseg; ++s) {
    a.dst[s] = dst[s];
    a.src[s] = src[s];
    a.bytes[s] = bytes[s];
    a.vec[s] = ((reinterpret_cast<uintptr_t>(dst[s]) | reinterpret_cast<uintptr_t>(src[s]) | (uintptr_t)bytes[s]) & 15) == 0;
    const long long u = a.vec[s] ? bytes[s] >> 4 : bytes[s];
    units = u > units ? u : units;
  }
  a.nseg = nseg;
  a.hyper_dst = hyper_dst;
  for (int i = 0; i < nhyper; ++i) a.hyper[i] = hyper[i];
  a.nhyper = hyper_dst ? nhyper : 0;
  long long blocks = (units + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
  hipLaunchKernelGGL(stage_step_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return 0;
}
}  // namespace pio

namespace pio {
unsigned check_errors_elementwise(bool reset) { return pio_read_errors(reset); }
}  // namespace pio

