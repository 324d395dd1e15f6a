// Per-sample latent self-attention block kernels for 32-latent stacks: C = 128 channels, H = 4 heads
// (d = 32) for the image configs (reference scripts/img_clf.py:14-22: 32×128 latents, 3 × (1 cross
// + 3 self-attention layers)) and C = 64 (d = 16) for the LArTPC experiment (run.py:72-112:
// 32×64 latents); model.py:36-44 self_attention_block.
//
// With 32 latents a sample's keys and values are its own 32 rows, so ONE workgroup can run every
// layer of a block for one sample — forward or backward — with no cross-workgroup dependency at
// all: one launch per block each way instead of 2 (forward) + 2 (backward) launches per layer,
// and no intermediate row ever leaves the CU between the kernels of a layer.
//
// Layout (NW = C / 32 waves per workgroup, wave w): every C-wide product is computed TRANSPOSED,
// Yᵀ = W·Xᵀ on v_mfma_f32_32x32x16_bf16 with the weight as the A operand (16-byte fragments
// straight from global memory / L2) and the activation image (bf16 [32 rows][C] in LDS) as B.
// The accumulator then holds, in lane l, row r = l & 31 and channels n0 + (i & 3) + 8(i >> 2) +
// 4(l >> 5) of the wave's 32-channel tile ("T layout"): a row's values are lane-local, row
// reductions are 16 local values + one lane swap (+ an NW-wave exchange for LayerNorm).  Wave w
// owns channels 32w .. 32w + 31 of every C-wide result and, of the packed QKV projection, exactly
// its HPW = 32 / d heads' Q, K and V — so those heads' attention (32 × 32 each) runs inside wave w:
// Sᵀ = K·Qᵀ from the packed T-layout registers (the contraction order of d is permuted identically
// on both operands; a head's d channels are register groups of 8), softmax over keys lane-locally,
// Oᵀ = Vᵀ·Pᵀ with Vᵀ read transposed from a wave-private LDS tile (with two heads per wave the rows
// of the other head are computed and dropped).
//
// Backward: the transposed products dXᵀ = Wᵀ·dYᵀ read the weight transposed from an LDS image
// (staged per C × C block, double-buffered), attention backward of the wave's heads again inside
// the wave.  Weight gradients are NOT formed here: the kernel stores the gradient rows (dQKV, dY,
// dU, dZ; bf16) and one grouped GEMM launch (sb_wgrad_kernel) forms dW = Σ Gᵀ·A for all weights of
// the block against the forward's saved operand rows (LN1(x), O, LN2(y), GELU(u)) — the row sums
// of a weight gradient need every sample, which no per-sample workgroup has.  LayerNorm γ/β
// gradients (C values per LN) are reduced over the sample's rows in registers and added atomically.
#include "common.h"
#include "sb_args.h"

namespace pio {
namespace sb {

constexpr int NR = 32, H = 4;
constexpr int LDA = 32 + 8;  // per-wave 32 × 32 attention tiles [32][40]

template <int C>
struct Shape {
  static constexpr int NW = C / 32;         // waves per workgroup (one sample)
  static constexpr int NT = 64 * NW;
  static constexpr int D = C / H;           // head width
  static constexpr int HPW = 32 / D;        // heads per wave
  static constexpr int KSD = D / 16;        // 16-wide k-steps per head
  static constexpr int KS = C / 16;         // k-steps of a C-deep product
  static constexpr int LDI = C + 8;         // activation images [32][C + 8]
  static constexpr int LDQ = 3 * C + 8;     // dQKV image [32][3C + 8]
  static constexpr int LDW = C + 8;         // staged weight block [C][C + 8]
  static constexpr int WCH = C / 16;        // 16-byte chunks per thread of a C × C weight block
};

__device__ __forceinline__ int tch(int i, int hh) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }

// KS A fragments (k-steps over K = C) of the 32-row tile n0.. of a row-major bf16 weight [N][C]
template <int C>
__device__ __forceinline__ void load_wtile(bf16x8 (&f)[C / 16], const uint16_t* W, int n0) {
  const int l = lane_id();
  const uint16_t* p = W + (long long)(n0 + (l & 31)) * C + 8 * (l >> 5);
#pragma unroll
  for (int t = 0; t < C / 16; ++t) f[t] = *reinterpret_cast<const bf16x8*>(p + 16 * t);
}
// Yᵀ tile = W tile · Xᵀ, X = an LDS image [32][ld]
template <int C>
__device__ __forceinline__ f32x16 gemm_t(const bf16x8 (&f)[C / 16], const uint16_t* sX, int ld) {
  const int l = lane_id();
  const uint16_t* p = sX + (l & 31) * ld + 8 * (l >> 5);
  f32x16 acc = f32x16{};
#pragma unroll
  for (int t = 0; t < C / 16; ++t) acc = mfma32(f[t], *reinterpret_cast<const bf16x8*>(p + 16 * t), acc);
  return acc;
}
// dXᵀ tile (output channels i0 .. i0 + 31) = Wᵀ · dYᵀ over a staged weight block sW [C n][LDW]
// (the contraction index n is the block's row) and dY = an LDS image [32][ld] (columns k0 ..)
template <int C>
__device__ __forceinline__ f32x16 gemm_tt(const uint16_t* sW, int i0, const uint16_t* sX, int ld, int k0, f32x16 acc) {
  const int l = lane_id();
  const uint16_t* p = sX + (l & 31) * ld + k0 + 8 * (l >> 5);
#pragma unroll
  for (int t = 0; t < C / 16; ++t)
    acc = mfma32(frag_ks(sW, Shape<C>::LDW, i0, 16 * t), *reinterpret_cast<const bf16x8*>(p + 16 * t), acc);
  return acc;
}
// T-layout values of this lane (row r, 16 channels of tile n0) → a row-major bf16 array / image
__device__ __forceinline__ void st_bf16(uint16_t* base, long long ld, long long row, int n0, const float (&v)[16]) {
  const int hh = lane_id() >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint2 pk;
    pk.x = pack2(v[4 * g], v[4 * g + 1]);
    pk.y = pack2(v[4 * g + 2], v[4 * g + 3]);
    *reinterpret_cast<uint2*>(base + row * ld + n0 + 8 * g + 4 * hh) = pk;
  }
}
__device__ __forceinline__ void st_f32(float* base, long long ld, long long row, int n0, const float (&v)[16]) {
  const int hh = lane_id() >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<float4*>(base + row * ld + n0 + 8 * g + 4 * hh) =
        make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
}
__device__ __forceinline__ void ld_f32(float (&v)[16], const float* base, long long ld, long long row, int n0) {
  const int hh = lane_id() >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 a = *reinterpret_cast<const float4*>(base + row * ld + n0 + 8 * g + 4 * hh);
    v[4 * g] = a.x; v[4 * g + 1] = a.y; v[4 * g + 2] = a.z; v[4 * g + 3] = a.w;
  }
}
// this lane's 16 bf16 values of tile n0 kept packed (4 × 8 bytes) until cvt_raw
__device__ __forceinline__ void ld_raw(uint2 (&v)[4], const uint16_t* base, long long ld, long long row, int n0) {
  const int hh = lane_id() >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) v[g] = *reinterpret_cast<const uint2*>(base + row * ld + n0 + 8 * g + 4 * hh);
}
__device__ __forceinline__ void cvt_raw(float (&v)[16], const uint2 (&a)[4]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    v[4 * g] = bf2f((uint16_t)(a[g].x & 0xFFFF)); v[4 * g + 1] = bf2f((uint16_t)(a[g].x >> 16));
    v[4 * g + 2] = bf2f((uint16_t)(a[g].y & 0xFFFF)); v[4 * g + 3] = bf2f((uint16_t)(a[g].y >> 16));
  }
}
__device__ __forceinline__ void ld_bf16(float (&v)[16], const uint16_t* base, long long ld, long long row, int n0) {
  const int hh = lane_id() >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const uint2 a = *reinterpret_cast<const uint2*>(base + row * ld + n0 + 8 * g + 4 * hh);
    v[4 * g] = bf2f((uint16_t)(a.x & 0xFFFF)); v[4 * g + 1] = bf2f((uint16_t)(a.x >> 16));
    v[4 * g + 2] = bf2f((uint16_t)(a.y & 0xFFFF)); v[4 * g + 3] = bf2f((uint16_t)(a.y >> 16));
  }
}
// whole-row copy of a staged LDS tile [32][ld] (W elements per row, 16-byte chunks) to the sample's
// 32 global rows (row stride gld), by every thread: a T-layout store from registers (8 or 16
// bytes per lane at a row stride) touches a cache line per lane, this one 4 lines per wave
template <int W, typename T>
__device__ __forceinline__ void copy_rows(T* g, long long gld, const T* img, int ld) {
  constexpr int E = 16 / sizeof(T), CPR = W / E;
  T* gb = g + (long long)blockIdx.x * NR * gld;
  for (int c = threadIdx.x; c < NR * CPR; c += blockDim.x) {
    const int rr = c / CPR, col = (c % CPR) * E;
    *reinterpret_cast<uint4*>(gb + rr * gld + col) = *reinterpret_cast<const uint4*>(img + rr * ld + col);
  }
}
// the sample's 32 global bf16 rows (row stride gld, W elements) → an LDS image [32][ld], by every
// thread in 16-byte chunks (no barrier)
template <int W>
__device__ __forceinline__ void load_rows(uint16_t* img, int ld, const uint16_t* g, long long gld) {
  constexpr int CPR = W / 8;
  const uint16_t* gb = g + (long long)blockIdx.x * NR * gld;
  for (int c = threadIdx.x; c < NR * CPR; c += blockDim.x) {
    const int rr = c / CPR, col = (c % CPR) * 8;
    *reinterpret_cast<uint4*>(img + rr * ld + col) = *reinterpret_cast<const uint4*>(gb + rr * gld + col);
  }
}
// T-layout fp32 values of this lane → an LDS fp32 tile [32][ld]
__device__ __forceinline__ void st_f32s(float* img, int ld, int r, int n0, const float (&v)[16]) {
  const int hh = lane_id() >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<float4*>(img + r * ld + n0 + 8 * g + 4 * hh) = make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
}
// per-channel vector (bias, γ, β) at this lane's 16 channels of tile n0 (from an LDS copy: vmcnt
// counts loads and stores together in issue order, so a global load consumed right after a
// phase's stores would wait for every one of them)
__device__ __forceinline__ void ld_vec(float (&v)[16], const float* p, int n0) { ld_f32(v, p, 0, 0, n0); }
// stage n (float4-aligned, 16-byte aligned) floats of global vectors into LDS: all threads, no barrier
__device__ __forceinline__ void stage_vec(float* dst, const float* src, int n) {
  for (int i = threadIdx.x; i < n / 4; i += blockDim.x)
    reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
}
__device__ __forceinline__ void to_f(float (&v)[16], const f32x16& a) {
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = a[i];
}
__device__ __forceinline__ bf16x8 pack8(const float (&v)[16], int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(v[8 * s + j]);
  return r;
}

// LayerNorm statistics of row r over the NW waves' 32-channel slices (Chan's combination of the
// per-wave (mean, M2)); one workgroup barrier
template <int C>
__device__ __forceinline__ void ln_stats(const float (&v)[16], float2* sRed, float eps, float& mean, float& rstd) {
  constexpr int NW = Shape<C>::NW;
  const int w = wave_id(), l = lane_id(), r = l & 31, hh = l >> 5;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += v[i];
  const float mw = xor32_sum(s) * (1.f / 32.f);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) { const float d = v[i] - mw; q = fmaf(d, d, q); }
  q = xor32_sum(q);
  if (hh == 0) sRed[w * NR + r] = make_float2(mw, q);
  lds_sync();
  float2 p[NW];
#pragma unroll
  for (int k = 0; k < NW; ++k) p[k] = sRed[k * NR + r];
  float sm = 0.f, m2 = 0.f;
#pragma unroll
  for (int k = 0; k < NW; ++k) { sm += p[k].x; m2 += p[k].y; }
  mean = sm * (1.f / NW);
#pragma unroll
  for (int k = 0; k < NW; ++k) { const float d = p[k].x - mean; m2 = fmaf(32.f * d, d, m2); }
  rstd = rsqrtf(m2 * (1.f / C) + eps);
}
// sums over the NW waves of two per-row partials (each lane-local over 16 channels); one barrier
template <int C>
__device__ __forceinline__ float2 row_sums2(float a, float b, float2* sRed) {
  constexpr int NW = Shape<C>::NW;
  const int w = wave_id(), l = lane_id(), r = l & 31, hh = l >> 5;
  a = xor32_sum(a);
  b = xor32_sum(b);
  if (hh == 0) sRed[w * NR + r] = make_float2(a, b);
  lds_sync();
  float2 t = make_float2(0.f, 0.f);
#pragma unroll
  for (int k = 0; k < NW; ++k) { const float2 p = sRed[k * NR + r]; t.x += p.x; t.y += p.y; }
  return t;
}

// Sᵀ (keys × queries, lane = query) of head hp of the wave, softmax over keys (probabilities
// normalised; `inv` = 1 / Σ)
template <int C>
__device__ __forceinline__ void softmax_t(const float (&q)[16], const float (&k)[16], int hp, float scale_log2,
                                          float (&p)[16], float& inv) {
  constexpr int KSD = Shape<C>::KSD;
  f32x16 s = f32x16{};
#pragma unroll
  for (int j = 0; j < KSD; ++j) s = mfma32(pack8(k, hp * KSD + j), pack8(q, hp * KSD + j), s);
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < 16; ++i) m = fmaxf(m, s[i]);
  m = xor32_max(m) * scale_log2;
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) { p[i] = fast_exp2(fmaf(s[i], scale_log2, -m)); sum += p[i]; }
  inv = 1.f / xor32_sum(sum);
}
// the registers of head hp in a wave's 32-channel T-layout tile
template <int C>
__device__ __forceinline__ bool head_reg(int i, int hp) { return (i >> 3) / Shape<C>::KSD == hp; }

// ------------------------------------------------------------------------------------
// forward: grid = B samples, NT threads
// ------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(2 * C) void sb_fwd_kernel(SBFwdArgs a) {
  using S = Shape<C>;
  constexpr int KS = S::KS, LDI = S::LDI;
  __shared__ __attribute__((aligned(16))) uint16_t sImg[2][NR * LDI];
  __shared__ __attribute__((aligned(16))) uint16_t sV[S::NW][NR * LDA];
  __shared__ __attribute__((aligned(16))) float2 sRed[S::NW * NR];
  // every layer's per-channel vectors, staged once before any store of the kernel:
  // [γ1 | β1 | bqkv (3C) | bo | γ2 | β2 | b1 | b2]
  constexpr int NV = 10 * C;
  __shared__ __attribute__((aligned(16))) float sVec[kSBMaxLayers + 1][NV];  // + the pre stage's
  // staging of the saved rows for whole-row stores: QKV then U (bf16 [32][3C + 8]), Y then Z (fp32)
  constexpr int LDS3 = 3 * C + 8, LDF = C + 4;
  __shared__ __attribute__((aligned(16))) uint16_t sS[NR * LDS3];
  __shared__ __attribute__((aligned(16))) float sF[NR * LDF];
  const int w = wave_id(), l = lane_id(), r = l & 31;
  const long long row = (long long)blockIdx.x * NR + r;
  const int n0 = 32 * w;  // this wave's channel tile
  for (int li = 0; li < a.L; ++li) {
    const SBLayer& y = a.ly[li];
    float* v = sVec[li];
    stage_vec(v, y.g1, C);
    stage_vec(v + C, y.be1, C);
    stage_vec(v + 2 * C, y.bqkv, 3 * C);
    stage_vec(v + 5 * C, y.bo, C);
    stage_vec(v + 6 * C, y.g2, C);
    stage_vec(v + 7 * C, y.be2, C);
    stage_vec(v + 8 * C, y.b1, C);
    stage_vec(v + 9 * C, y.b2, C);
  }
  if (a.has_post) {  // the query path's γ | β | bias (slot kSBMaxLayers, columns 0 .. 3C)
    stage_vec(sVec[kSBMaxLayers], a.post.g, C);
    stage_vec(sVec[kSBMaxLayers] + C, a.post.b, C);
    stage_vec(sVec[kSBMaxLayers] + 2 * C, a.post.bq, a.post.N);  // (≤ 4C: below the pre stage's 5C ..)
  }
  float x[16];
  bf16x8 wq[3][KS];
  if (a.has_pre) {
    // ---- pre: the cross layer's post-attention half, y = Wo·O + bo + x_q, z0 = y + MLP(LN2(y)),
    // the same phases as a layer's second half below; z0 is the block input ----
    const SBLayer& y = a.pre;
    float* vec = sVec[kSBMaxLayers];
    stage_vec(vec + 5 * C, y.bo, C);
    stage_vec(vec + 6 * C, y.g2, C);
    stage_vec(vec + 7 * C, y.be2, C);
    stage_vec(vec + 8 * C, y.b1, C);
    stage_vec(vec + 9 * C, y.b2, C);
    bf16x8 wo[KS], w1[KS];
    load_wtile<C>(wo, y.Wo, n0);
    load_rows<C>(sImg[1], LDI, a.preO, C);
    ld_f32(x, a.preX, C, (long long)(a.preX_bs ? (int)blockIdx.x * a.preX_bs : 0) + r, n0);
    load_wtile<C>(w1, y.W1, n0);
    lds_sync();  // the O image and every staged vector
    float yv[16], mu, rs, gv[16], bv[16], t[16];
    {
      float bb[16];
      const f32x16 acc = gemm_t<C>(wo, sImg[1], LDI);
      ld_vec(bb, vec + 5 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) yv[i] = acc[i] + bb[i] + x[i];
    }
    bf16x8 w2[KS];
    load_wtile<C>(w2, y.W2, n0);
    st_f32s(sF, LDF, r, n0, yv);
    ld_vec(gv, vec + 6 * C, n0);
    ld_vec(bv, vec + 7 * C, n0);
    ln_stats<C>(yv, sRed, a.eps, mu, rs);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = (yv[i] - mu) * rs * gv[i] + bv[i];
    if (w == 0 && l < 32) { y.mean2[row] = mu; y.rstd2[row] = rs; }
    st_bf16(sImg[0], LDI, r, n0, t);
    lds_sync();
    copy_rows<C>(y.Y, C, sF, LDF);
    copy_rows<C>(y.LN2Y, C, sImg[0], LDI);
    {
      float bb[16];
      const f32x16 acc = gemm_t<C>(w1, sImg[0], LDI);
      ld_vec(bb, vec + 8 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = acc[i] + bb[i];
    }
    float gu[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) gu[i] = gelu_f(t[i]);
    st_bf16(sImg[1], LDI, r, n0, gu);
    load_wtile<C>(wq[0], a.ly[0].Wqkv, n0);  // layer 0's QKV weights, in flight during the MLP
    load_wtile<C>(wq[1], a.ly[0].Wqkv, C + n0);
    load_wtile<C>(wq[2], a.ly[0].Wqkv, 2 * C + n0);
    st_bf16(sS, LDS3, r, n0, t);
    lds_sync();
    copy_rows<C>(y.U, C, sS, LDS3);
    copy_rows<C>(y.GU, C, sImg[1], LDI);
    {
      float bb[16];
      const f32x16 acc = gemm_t<C>(w2, sImg[1], LDI);
      ld_vec(bb, vec + 9 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = acc[i] + bb[i] + yv[i];
    }
    st_f32s(sF, LDF, r, n0, x);  // z0: copied out to X0 behind layer 0's first barrier
  } else {
    ld_f32(x, a.X0, C, row, n0);
    load_wtile<C>(wq[0], a.ly[0].Wqkv, n0);
    load_wtile<C>(wq[1], a.ly[0].Wqkv, C + n0);
    load_wtile<C>(wq[2], a.ly[0].Wqkv, 2 * C + n0);
  }
  for (int li = 0; li < a.L; ++li) {
    const SBLayer& y = a.ly[li];
    const float* vec = sVec[li];
    PIO_TS(12 * li);
    // ---- LN1 → image 0 (the QKV product's operand) ----
    float mu, rs, gv[16], bv[16], t[16];
    ln_stats<C>(x, sRed, a.eps, mu, rs);  // (its barrier also publishes the staged vectors)
    PIO_TS(12 * li + 1);
    ld_vec(gv, vec, n0);
    ld_vec(bv, vec + C, n0);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = (x[i] - mu) * rs * gv[i] + bv[i];
    st_bf16(sImg[0], LDI, r, n0, t);
    // each phase issues its weight prefetch before its global stores (vmcnt counts both in issue
    // order: a load behind the stores would make its consumer wait for them)
    bf16x8 wo[KS];
    load_wtile<C>(wo, y.Wo, n0);
    if (w == 0 && l < 32) { y.mean1[row] = mu; y.rstd1[row] = rs; }
    lds_sync();
    PIO_TS(12 * li + 2);
    copy_rows<C>(y.LN1X, C, sImg[0], LDI);
    if (li > 0) copy_rows<C>(a.ly[li - 1].Z, C, sF, LDF);  // the previous layer's output
    else if (a.has_pre) copy_rows<C>(a.pre.Z, C, sF, LDF);  // the pre stage's (the block input)
    // ---- Q, K, V of the wave's heads ----
    float q[16], k[16], v[16];
    {
      float bb[16];
      f32x16 acc = gemm_t<C>(wq[0], sImg[0], LDI);
      ld_vec(bb, vec + 2 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) q[i] = acc[i] + bb[i];
      acc = gemm_t<C>(wq[1], sImg[0], LDI);
      ld_vec(bb, vec + 3 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) k[i] = acc[i] + bb[i];
      acc = gemm_t<C>(wq[2], sImg[0], LDI);
      ld_vec(bb, vec + 4 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = acc[i] + bb[i];
    }
    PIO_TS(12 * li + 3);
    bf16x8 w1[KS];
    load_wtile<C>(w1, y.W1, n0);
    st_bf16(sS, LDS3, r, n0, q);
    st_bf16(sS, LDS3, r, C + n0, k);
    st_bf16(sS, LDS3, r, 2 * C + n0, v);
    // ---- attention of the wave's heads: Sᵀ = K·Qᵀ (lane = query), softmax over keys, Oᵀ = Vᵀ·Pᵀ
    // with Vᵀ read transposed from a wave-private LDS tile [key][32 channels] ----
    float o[16];
    {
      st_bf16(sV[w], LDA, r, 0, v);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's V tile written
#pragma unroll
      for (int hp = 0; hp < S::HPW; ++hp) {
        float p[16], inv;
        softmax_t<C>(q, k, hp, a.scale_log2, p, inv);
        f32x16 oa = f32x16{};
        oa = mfma32(frag_ks_perm(sV[w], LDA, 0, 0), pack8(p, 0), oa);
        oa = mfma32(frag_ks_perm(sV[w], LDA, 0, 16), pack8(p, 1), oa);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (head_reg<C>(i, hp)) o[i] = oa[i] * inv;
      }
    }
    PIO_TS(12 * li + 4);
    st_bf16(sImg[1], LDI, r, n0, o);
    bf16x8 w2[KS];
    load_wtile<C>(w2, y.W2, n0);
    lds_sync();
    PIO_TS(12 * li + 5);
    copy_rows<3 * C>(y.QKV, 3 * C, sS, LDS3);
    copy_rows<C>(y.O, C, sImg[1], LDI);
    // ---- out-projection + residual → y; LN2 → image 0 ----
    float yv[16];
    {
      float bb[16];
      const f32x16 acc = gemm_t<C>(wo, sImg[1], LDI);
      ld_vec(bb, vec + 5 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) yv[i] = acc[i] + bb[i] + x[i];
    }
    PIO_TS(12 * li + 6);
    st_f32s(sF, LDF, r, n0, yv);
    ld_vec(gv, vec + 6 * C, n0);
    ld_vec(bv, vec + 7 * C, n0);
    ln_stats<C>(yv, sRed, a.eps, mu, rs);
    PIO_TS(12 * li + 7);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = (yv[i] - mu) * rs * gv[i] + bv[i];
    if (w == 0 && l < 32) { y.mean2[row] = mu; y.rstd2[row] = rs; }
    st_bf16(sImg[0], LDI, r, n0, t);
    lds_sync();
    PIO_TS(12 * li + 8);
    copy_rows<C>(y.Y, C, sF, LDF);
    copy_rows<C>(y.LN2Y, C, sImg[0], LDI);
    // ---- MLP: u = W1·LN2(y) + b1, GELU → image 1, z = W2·GELU(u) + b2 + y ----
    {
      float bb[16];
      const f32x16 acc = gemm_t<C>(w1, sImg[0], LDI);
      ld_vec(bb, vec + 8 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = acc[i] + bb[i];
    }
    PIO_TS(12 * li + 9);
    float gu[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) gu[i] = gelu_f(t[i]);
    st_bf16(sImg[1], LDI, r, n0, gu);
    if (li + 1 < a.L) {  // the next layer's QKV weights, in flight during the MLP
      load_wtile<C>(wq[0], a.ly[li + 1].Wqkv, n0);
      load_wtile<C>(wq[1], a.ly[li + 1].Wqkv, C + n0);
      load_wtile<C>(wq[2], a.ly[li + 1].Wqkv, 2 * C + n0);
    } else if (a.has_post) {  // the query path's weight (K and V tiles for a 2C-wide projection)
      load_wtile<C>(wq[0], a.post.Wq, n0);
      if (a.post.N == 2 * C) load_wtile<C>(wq[1], a.post.Wq, C + n0);
    }
    st_bf16(sS, LDS3, r, n0, t);  // U (the QKV rows were copied out behind the last barrier)
    lds_sync();
    PIO_TS(12 * li + 10);
    copy_rows<C>(y.U, C, sS, LDS3);
    copy_rows<C>(y.GU, C, sImg[1], LDI);
    {
      float bb[16];
      const f32x16 acc = gemm_t<C>(w2, sImg[1], LDI);
      ld_vec(bb, vec + 9 * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = acc[i] + bb[i] + yv[i];
    }
    PIO_TS(12 * li + 11);
    // Z: staged (the Y rows were copied out behind the last barrier but one), copied out behind
    // the next layer's first barrier, or here after the last layer's
    st_f32s(sF, LDF, r, n0, x);
  }
  lds_sync();
  copy_rows<C>(a.ly[a.L - 1].Z, C, sF, LDF);
  if (a.has_post) {
    // ---- post: the next cross layer's LN + query projection of the block output ----
    const float* vec = sVec[kSBMaxLayers];
    float mu, rs, gv[16], bv[16], t[16];
    ln_stats<C>(x, sRed, a.eps, mu, rs);
    ld_vec(gv, vec, n0);
    ld_vec(bv, vec + C, n0);
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = (x[i] - mu) * rs * gv[i] + bv[i];
    if (w == 0 && l < 32) { a.post.mean[row] = mu; a.post.rstd[row] = rs; }
    st_bf16(sImg[0], LDI, r, n0, t);
    lds_sync();
    copy_rows<C>(a.post.LNX, C, sImg[0], LDI);
    auto out_tile = [&](const bf16x8(&wt)[KS], int j) {  // output tile j·C + n0 → the row image
      float bb[16];
      const f32x16 acc = gemm_t<C>(wt, sImg[0], LDI);
      ld_vec(bb, vec + 2 * C + j * C, n0);
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = acc[i] + bb[i];
      st_bf16(sS, LDS3, r, j * C + n0, t);
    };
    out_tile(wq[0], 0);
    if (a.post.N == 2 * C) out_tile(wq[1], 1);
    lds_sync();
    if (a.post.N == C) copy_rows<C>(a.post.Q, C, sS, LDS3);
    else copy_rows<2 * C>(a.post.Q, 2 * C, sS, LDS3);
  }
}

// ------------------------------------------------------------------------------------
// backward: grid = B samples, NT threads
// ------------------------------------------------------------------------------------
// one C × C block of a row-major bf16 weight (rows n0 ..) into registers, then into an LDS image
template <int C>
__device__ __forceinline__ void wblock_load(bf16x8 (&f)[C / 16], const uint16_t* W, int n0) {
#pragma unroll
  for (int k = 0; k < C / 16; ++k) {
    const int c = threadIdx.x + Shape<C>::NT * k, rr = c / (C / 8), col = (c % (C / 8)) * 8;
    f[k] = *reinterpret_cast<const bf16x8*>(W + (long long)(n0 + rr) * C + col);
  }
}
template <int C>
__device__ __forceinline__ void wblock_store(uint16_t* sW, const bf16x8 (&f)[C / 16]) {
#pragma unroll
  for (int k = 0; k < C / 16; ++k) {
    const int c = threadIdx.x + Shape<C>::NT * k, rr = c / (C / 8), col = (c % (C / 8)) * 8;
    *reinterpret_cast<bf16x8*>(sW + rr * Shape<C>::LDW + col) = f[k];
  }
}
// LayerNorm γ/β gradients of this sample: Σ_rows dxn·x̂ and Σ_rows dxn per channel (the 32 rows
// are the 32 lanes of each half), stored into the sample's slab row by lanes 0 and 32
__device__ __forceinline__ void ln_affine_grads(const float (&dxn)[16], const float (&xh)[16], float* dg, float* db, int n0) {
  const int l = lane_id(), hh = l >> 5;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float sg = half_sum(dxn[i] * xh[i]);
    const float sb = half_sum(dxn[i]);
    if ((l & 31) == 0) {
      dg[n0 + tch(i, hh)] = sg;
      db[n0 + tch(i, hh)] = sb;
    }
  }
}

template <int C>
__global__ __launch_bounds__(2 * C) void sb_bwd_kernel(SBBwdArgs a) {
  using S = Shape<C>;
  constexpr int KS = S::KS, LDI = S::LDI, LDQ = S::LDQ, LDW = S::LDW, NW = S::NW;
  __shared__ __attribute__((aligned(16))) uint16_t sW[2][C * LDW];
  __shared__ __attribute__((aligned(16))) uint16_t sImg[2][NR * LDI];
  __shared__ __attribute__((aligned(16))) uint16_t sQ[NR * LDQ];
  __shared__ __attribute__((aligned(16))) uint16_t sAt[NW][4][NR * LDA];  // per wave: K, Q, dO, P / dS
  __shared__ __attribute__((aligned(16))) float2 sRed[NW * NR];
  __shared__ __attribute__((aligned(16))) float sG[kSBMaxLayers + 1][2][C];  // γ1, γ2 of every layer (+ pre's γ2)
  const int w = wave_id(), l = lane_id(), r = l & 31;
  const long long row = (long long)blockIdx.x * NR + r;
  const int n0 = 32 * w;
  const float sc = a.scale_log2 * 0.69314718055994531f;  // the softmax scale 1/√d
  const long long lnr = (long long)blockIdx.x * a.ln_rs;  // this sample's LayerNorm partial row
  for (int li = 0; li < a.L; ++li) {
    stage_vec(sG[li][0], a.ly[li].g1, C);
    stage_vec(sG[li][1], a.ly[li].g2, C);
  }
  if (a.has_pre) stage_vec(sG[kSBMaxLayers][1], a.pre.g2, C);
  if (a.has_post) stage_vec(sG[kSBMaxLayers][0], a.post.g, C);
  if (a.zero_p != nullptr) {  // this workgroup's slice of the cross attention backward's accumulators
    const long long per = (a.zero_n4 + gridDim.x - 1) / gridDim.x;
    const long long z0 = (long long)blockIdx.x * per, z1 = z0 + per < a.zero_n4 ? z0 + per : a.zero_n4;
    for (long long i = z0 + threadIdx.x; i < z1; i += blockDim.x)
      reinterpret_cast<float4*>(a.zero_p)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float dz[16];
  bf16x8 pw[KS];
  if (a.has_post) {
    // ---- post: the next cross layer's query-path backward: dz = dres + LN_q backward of dQ·Wq ----
    const SBQPath& q = a.post;
    const bool two = q.N == 2 * C;
    wblock_load<C>(pw, q.Wq, 0);
    float dqv[16], dqv1[16], xz[16];
    ld_f32(dqv, q.dQ, q.N, row, n0);
    if (two) ld_f32(dqv1, q.dQ, q.N, row, C + n0);
    ld_f32(xz, a.ly[a.L - 1].Z, C, row, n0);
    if (q.dres != nullptr) ld_f32(dz, q.dres, C, row, n0);
    else
#pragma unroll
      for (int i = 0; i < 16; ++i) dz[i] = 0.f;
    const float mu = q.mean[row], rs = q.rstd[row];
    st_bf16(sQ, LDQ, r, n0, dqv);
    if (two) st_bf16(sQ, LDQ, r, C + n0, dqv1);
    wblock_store<C>(sW[1], pw);
    if (two) {  // the V block of the weight into the other buffer (free until the first layer)
      wblock_load<C>(pw, q.Wq, C);
      wblock_store<C>(sW[0], pw);
    }
    wblock_load<C>(pw, a.ly[a.L - 1].W2, 0);
    lds_sync();  // (also publishes the staged γ vectors)
    if (two) copy_rows<2 * C>(q.dQb, 2 * C, sQ, LDQ);
    else copy_rows<C>(q.dQb, C, sQ, LDQ);
    f32x16 acc = gemm_tt<C>(sW[1], n0, sQ, LDQ, 0, f32x16{});
    if (two) acc = gemm_tt<C>(sW[0], n0, sQ, LDQ, C, acc);
    float gv[16], gg[16], t[16], s1 = 0.f, s2 = 0.f;
    ld_vec(gv, sG[kSBMaxLayers][0], n0);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      t[i] = acc[i];               // dXn
      xz[i] = (xz[i] - mu) * rs;   // x̂
      gg[i] = acc[i] * gv[i];
      s1 += gg[i];
      s2 += gg[i] * xz[i];
    }
    const float2 sm = row_sums2<C>(s1, s2, sRed);  // (its barrier: every read of sImg[0] / sW[1] done)
    const float m1 = sm.x * (1.f / C), m2 = sm.y * (1.f / C);
#pragma unroll
    for (int i = 0; i < 16; ++i) dz[i] += rs * (gg[i] - m1 - xz[i] * m2);
    ln_affine_grads(t, xz, q.dg + lnr, q.db + lnr, n0);
  } else {
    ld_f32(dz, a.dZ, C, row, n0);
    wblock_load<C>(pw, a.ly[a.L - 1].W2, 0);
  }
  // Every phase issues its global loads (the next weight block, the layer's saved rows) BEFORE its
  // global stores: vmcnt counts both in issue order, so a load issued behind a phase's stores
  // would make its consumer wait for all of them
  for (int li = a.L - 1; li >= 0; --li) {
    const SBLayer& y = a.ly[li];
    const SBGrad& gd = a.gr[li];
    const float* X = li > 0 ? a.ly[li - 1].Z : a.X0;
    PIO_TS(16 * li);
    // ---- the layer's first saved rows; dZ image; W2 block ----
    uint2 ur[4];
    float yv[16];
    ld_raw(ur, y.U, C, row, n0);
    ld_f32(yv, y.Y, C, row, n0);
    const float mu2 = y.mean2[row], rs2 = y.rstd2[row];
    wblock_store<C>(sW[0], pw);
    wblock_load<C>(pw, y.W1, 0);
    st_bf16(sImg[0], LDI, r, n0, dz);
    lds_sync();
    PIO_TS(16 * li + 1);
    copy_rows<C>(gd.dZ, C, sImg[0], LDI);  // whole-row stores of the staged gradient rows
    // ---- dU = (W2ᵀ·dZ)∘GELU'(u) ----
    float t[16];
    {
      float uv[16];
      cvt_raw(uv, ur);
      const f32x16 acc = gemm_tt<C>(sW[0], n0, sImg[0], LDI, 0, f32x16{});
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = acc[i] * gelu_grad(uv[i]);
    }
    PIO_TS(16 * li + 2);
    st_bf16(sImg[1], LDI, r, n0, t);
    wblock_store<C>(sW[1], pw);
    wblock_load<C>(pw, y.Wo, 0);
    // the attention operands of the wave's heads (the forward's bf16 rows) and the LN1 input
    uint2 qr[4], kr[4], vr[4], orw[4];
    float xv[16];
    ld_raw(qr, y.QKV, 3 * C, row, n0);
    ld_raw(kr, y.QKV, 3 * C, row, C + n0);
    ld_raw(vr, y.QKV, 3 * C, row, 2 * C + n0);
    ld_raw(orw, y.O, C, row, n0);
    ld_f32(xv, X, C, row, n0);
    const float mu1 = y.mean1[row], rs1 = y.rstd1[row];
    lds_sync();
    PIO_TS(16 * li + 3);
    copy_rows<C>(gd.dU, C, sImg[1], LDI);
    // ---- dXn2 = W1ᵀ·dU; LN2 backward → dY ----
    float dy[16];
    {
      float gv[16];
      ld_vec(gv, sG[li][1], n0);
      const f32x16 acc = gemm_tt<C>(sW[1], n0, sImg[1], LDI, 0, f32x16{});
      PIO_TS(16 * li + 4);
      float s1 = 0.f, s2 = 0.f, gg[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        t[i] = acc[i];                     // dXn2
        yv[i] = (yv[i] - mu2) * rs2;       // ŷ
        gg[i] = acc[i] * gv[i];
        s1 += gg[i];
        s2 += gg[i] * yv[i];
      }
      const float2 s = row_sums2<C>(s1, s2, sRed);
      const float m1 = s.x * (1.f / C), m2 = s.y * (1.f / C);
#pragma unroll
      for (int i = 0; i < 16; ++i) dy[i] = dz[i] + rs2 * (gg[i] - m1 - yv[i] * m2);
    }
    PIO_TS(16 * li + 5);
    st_bf16(sImg[0], LDI, r, n0, dy);
    wblock_store<C>(sW[0], pw);
    wblock_load<C>(pw, y.Wqkv, 0);
    ln_affine_grads(t, yv, gd.dg2 + lnr, gd.dbe2 + lnr, n0);
    PIO_TS(16 * li + 6);
    lds_sync();
    PIO_TS(16 * li + 7);
    copy_rows<C>(gd.dY, C, sImg[0], LDI);
    // ---- dO = Woᵀ·dY (the wave's heads) ----
    float dov[16];
    to_f(dov, gemm_tt<C>(sW[0], n0, sImg[0], LDI, 0, f32x16{}));
    PIO_TS(16 * li + 8);
    // ---- attention backward of the wave's heads (wave-local) ----
    float gq[16], gk[16], gvv[16];
    {
      float qv[16], kv[16], vv[16], ov[16];
      cvt_raw(qv, qr);
      cvt_raw(kv, kr);
      cvt_raw(vv, vr);
      cvt_raw(ov, orw);
      uint16_t *tK = sAt[w][0], *tQ = sAt[w][1], *tdO = sAt[w][2], *tP = sAt[w][3];
      st_bf16(tK, LDA, r, 0, kv);
      st_bf16(tQ, LDA, r, 0, qv);
#pragma unroll
      for (int i = 0; i < 16; ++i) dov[i] = bf2f(f2bf(dov[i]));  // dO as bf16, as the products see it
      st_bf16(tdO, LDA, r, 0, dov);
#pragma unroll
      for (int hp = 0; hp < S::HPW; ++hp) {
        // Pᵀ exactly as the forward formed it, dPᵀ = V·dOᵀ, δ = rowsum(dO∘O) over the head
        float p[16], inv;
        softmax_t<C>(qv, kv, hp, a.scale_log2, p, inv);
#pragma unroll
        for (int i = 0; i < 16; ++i) p[i] *= inv;
        f32x16 dp = f32x16{};
#pragma unroll
        for (int j = 0; j < S::KSD; ++j) dp = mfma32(pack8(vv, hp * S::KSD + j), pack8(dov, hp * S::KSD + j), dp);
        float dl = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (head_reg<C>(i, hp)) dl = fmaf(dov[i], ov[i], dl);
        dl = xor32_sum(dl);
        float ds[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) ds[i] = p[i] * (dp[i] - dl);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous head's reads of tP done
        st_bf16(tP, LDA, r, 0, p);  // P as [query][key] (row = this lane's query) for dV
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // dVᵀ = dOᵀ·P, dQᵀ = Kᵀ·dSᵀ, dKᵀ = Qᵀ·dS: T layout (rows = keys / queries); the rows of
        // the wave's other head (two heads per wave) are dropped
        f32x16 dv = f32x16{}, dk = f32x16{}, dq = f32x16{};
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) dv = mfma32(frag_ks_perm(tdO, LDA, 0, 16 * ss), frag_ks_perm(tP, LDA, 0, 16 * ss), dv);
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) dq = mfma32(frag_ks_perm(tK, LDA, 0, 16 * ss), pack8(ds, ss), dq);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // P tile consumed: dS over it
        st_bf16(tP, LDA, r, 0, ds);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) dk = mfma32(frag_ks_perm(tQ, LDA, 0, 16 * ss), frag_ks_perm(tP, LDA, 0, 16 * ss), dk);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (head_reg<C>(i, hp)) { gq[i] = dq[i] * sc; gk[i] = dk[i] * sc; gvv[i] = dv[i]; }
      }
    }
    PIO_TS(16 * li + 9);
    st_bf16(sQ, LDQ, r, n0, gq);
    st_bf16(sQ, LDQ, r, C + n0, gk);
    st_bf16(sQ, LDQ, r, 2 * C + n0, gvv);
    wblock_store<C>(sW[1], pw);
    wblock_load<C>(pw, y.Wqkv, C);
    lds_sync();
    PIO_TS(16 * li + 10);
    copy_rows<3 * C>(gd.dQKV, 3 * C, sQ, LDQ);
    // ---- dXn1 = Wqkvᵀ·dQKV in three C-row blocks of Wqkv ----
    f32x16 acc = gemm_tt<C>(sW[1], n0, sQ, LDQ, 0, f32x16{});
    PIO_TS(16 * li + 11);
    wblock_store<C>(sW[0], pw);
    wblock_load<C>(pw, y.Wqkv, 2 * C);
    lds_sync();
    PIO_TS(16 * li + 12);
    acc = gemm_tt<C>(sW[0], n0, sQ, LDQ, C, acc);
    wblock_store<C>(sW[1], pw);
    if (li > 0) wblock_load<C>(pw, a.ly[li - 1].W2, 0);
    else if (a.has_pre) wblock_load<C>(pw, a.pre.W2, 0);
    lds_sync();
    PIO_TS(16 * li + 13);
    acc = gemm_tt<C>(sW[1], n0, sQ, LDQ, 2 * C, acc);
    // ---- LN1 backward → dX (the previous layer's dZ) ----
    {
      float gv[16];
      ld_vec(gv, sG[li][0], n0);
      float s1 = 0.f, s2 = 0.f, gg[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        t[i] = acc[i];                   // dXn1
        xv[i] = (xv[i] - mu1) * rs1;     // x̂
        gg[i] = acc[i] * gv[i];
        s1 += gg[i];
        s2 += gg[i] * xv[i];
      }
      const float2 s = row_sums2<C>(s1, s2, sRed);
      const float m1 = s.x * (1.f / C), m2 = s.y * (1.f / C);
#pragma unroll
      for (int i = 0; i < 16; ++i) dz[i] = dy[i] + rs1 * (gg[i] - m1 - xv[i] * m2);
    }
    PIO_TS(16 * li + 14);
    ln_affine_grads(t, xv, gd.dg1 + lnr, gd.dbe1 + lnr, n0);
    PIO_TS(16 * li + 15);
  }
  if (a.has_pre) {
    // ---- pre: the cross layer's post-attention backward (a layer's first half) → dO, δ of the
    // cross attention, dX = dY (the residual path to x_q) ----
    const SBLayer& y = a.pre;
    const SBGrad& gd = a.pgr;
    uint2 ur[4], orw[4];
    float yv[16];
    ld_raw(ur, y.U, C, row, n0);
    ld_f32(yv, y.Y, C, row, n0);
    const float mu2 = y.mean2[row], rs2 = y.rstd2[row];
    wblock_store<C>(sW[0], pw);
    wblock_load<C>(pw, y.W1, 0);
    st_bf16(sImg[0], LDI, r, n0, dz);
    lds_sync();
    copy_rows<C>(gd.dZ, C, sImg[0], LDI);
    float t[16];
    {
      float uv[16];
      cvt_raw(uv, ur);
      const f32x16 acc = gemm_tt<C>(sW[0], n0, sImg[0], LDI, 0, f32x16{});
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = acc[i] * gelu_grad(uv[i]);
    }
    st_bf16(sImg[1], LDI, r, n0, t);
    wblock_store<C>(sW[1], pw);
    wblock_load<C>(pw, y.Wo, 0);
    ld_raw(orw, y.O, C, row, n0);
    lds_sync();
    copy_rows<C>(gd.dU, C, sImg[1], LDI);
    float dy[16];
    {
      float gv[16];
      ld_vec(gv, sG[kSBMaxLayers][1], n0);
      const f32x16 acc = gemm_tt<C>(sW[1], n0, sImg[1], LDI, 0, f32x16{});
      float s1 = 0.f, s2 = 0.f, gg[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        t[i] = acc[i];                     // dXn2
        yv[i] = (yv[i] - mu2) * rs2;       // ŷ
        gg[i] = acc[i] * gv[i];
        s1 += gg[i];
        s2 += gg[i] * yv[i];
      }
      const float2 s = row_sums2<C>(s1, s2, sRed);
      const float m1 = s.x * (1.f / C), m2 = s.y * (1.f / C);
#pragma unroll
      for (int i = 0; i < 16; ++i) dy[i] = dz[i] + rs2 * (gg[i] - m1 - yv[i] * m2);
    }
    st_bf16(sImg[0], LDI, r, n0, dy);
    wblock_store<C>(sW[0], pw);
    ln_affine_grads(t, yv, gd.dg2 + lnr, gd.dbe2 + lnr, n0);
    lds_sync();
    copy_rows<C>(gd.dY, C, sImg[0], LDI);
    // dO = Woᵀ·dY as the attention backward reads it (bf16), δ = rowsum(dO∘O) per head
    float dov[16], ov[16];
    to_f(dov, gemm_tt<C>(sW[0], n0, sImg[0], LDI, 0, f32x16{}));
#pragma unroll
    for (int i = 0; i < 16; ++i) dov[i] = bf2f(f2bf(dov[i]));
    cvt_raw(ov, orw);
#pragma unroll
    for (int hp = 0; hp < S::HPW; ++hp) {
      float dl = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (head_reg<C>(i, hp)) dl = fmaf(dov[i], ov[i], dl);
      dl = xor32_sum(dl);
      if (l < 32) a.preDelta[row * H + w * S::HPW + hp] = dl;
    }
    st_bf16(sImg[1], LDI, r, n0, dov);
    lds_sync();
    copy_rows<C>(a.preDO, C, sImg[1], LDI);
#pragma unroll
    for (int i = 0; i < 16; ++i) dz[i] = dy[i];
  }
  st_f32(a.dX, C, row, n0, dz);
}

// ------------------------------------------------------------------------------------
// grouped weight gradients: grid (Σ_jobs N/64 column tiles, row splits), 256 threads.
// Workgroup (tile, split): dW[n0 .. n0 + 63][0 .. C) += Σ_{rows of the split} G[r][n]·A[r][k] and
// db[n] += Σ G[r][n]; wave w owns dW rows n0 + 32(w >> 1) .., columns (C/2)(w & 1) .. (C/64
// 32 × 32 MFMA tiles), the bias column sums by a ones operand.  Rows are staged 32 at a time in
// LDS (G tile [32][64], A tile [32][C]) with the next 32 register-prefetched.
// ------------------------------------------------------------------------------------
template <int C>
__global__ __launch_bounds__(256) void sb_wgrad_kernel(SBWgradArgs a, SlabJob sj, int tiles) {
  constexpr int LG = 64 + 8, LA = C + 8, TT = C / 64, AC = C / 64;  // A chunks (16 B) per thread
  __shared__ __attribute__((aligned(16))) uint16_t sG[2][NR * LG];
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][NR * LA];
  if ((int)blockIdx.x >= tiles) {  // appended: the block's LayerNorm partial slab
    const int jb = ((int)blockIdx.x - tiles) * (int)gridDim.y + (int)blockIdx.y;  // over every grid row
    if (jb < sj.nblk) slab_reduce_block(sj, jb, reinterpret_cast<float4*>(&sG[0][0]));
    return;
  }
  const int w = wave_id(), l = lane_id();
  int j = 0;
  while (j + 1 < a.njobs && (int)blockIdx.x >= a.job[j + 1].tile0) ++j;
  const SBWgradJob& jb = a.job[j];
  const int n0 = 64 * ((int)blockIdx.x - jb.tile0);
  const int r_begin = blockIdx.y * a.rows_per_split, r_end = min(a.R, r_begin + a.rows_per_split);
  // staging: thread t loads a G chunk (row t >> 3, 8 columns) and AC A chunks (row t >> 3)
  const int sr = threadIdx.x >> 3, gc = (threadIdx.x & 7) * 8, ac = (threadIdx.x & 7) * 8 * AC;
  bf16x8 g0, av[AC];
  auto fetch = [&](int r0) {
    const long long rr = r0 + sr;
    g0 = *reinterpret_cast<const bf16x8*>(jb.G + rr * jb.N + n0 + gc);
#pragma unroll
    for (int q = 0; q < AC; ++q) av[q] = *reinterpret_cast<const bf16x8*>(jb.A + rr * C + ac + 8 * q);
  };
  f32x16 acc[TT];
#pragma unroll
  for (int tt = 0; tt < TT; ++tt) acc[tt] = f32x16{};
  f32x16 bacc = f32x16{};
  const int mi = 32 * (w >> 1);        // dW rows (G columns) of this wave within the tile
  const int kc = (C / 2) * (w & 1);    // dW columns (A columns)
  const short one = (short)0x3F80;
  const bf16x8 ones = bf16x8{one, one, one, one, one, one, one, one};
  if (r_begin < r_end) fetch(r_begin);
  int buf = 0;
  for (int r0 = r_begin; r0 < r_end; r0 += NR, buf ^= 1) {
    *reinterpret_cast<bf16x8*>(sG[buf] + sr * LG + gc) = g0;
#pragma unroll
    for (int q = 0; q < AC; ++q) *reinterpret_cast<bf16x8*>(sA[buf] + sr * LA + ac + 8 * q) = av[q];
    lds_sync();
    if (r0 + NR < r_end) fetch(r0 + NR);
    // contraction over the 32 rows: A operand Gᵀ (element (n, r) at sG[r][n]), B operand A
    // (element (r, k) at sA[r][k]); two 16-row k-steps
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 ga = frag_ks(sG[buf], LG, mi, 16 * ks);
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) acc[tt] = mfma32(ga, frag_ks(sA[buf], LA, kc + 32 * tt, 16 * ks), acc[tt]);
      if ((w & 1) == 0) bacc = mfma32(ga, ones, bacc);
    }
  }
  // accumulator: col = k (lane), row = n = acc_row(i, hh)
  const int hh = l >> 5;
#pragma unroll
  for (int tt = 0; tt < TT; ++tt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = n0 + mi + acc_row(i, hh), k = kc + 32 * tt + (l & 31);
      atomicAdd(jb.dW + (long long)n * C + k, acc[tt][i]);
    }
  if ((w & 1) == 0 && (l & 31) == 0)  // every column of the ones product holds Σ_r G[r][n]
#pragma unroll
    for (int i = 0; i < 16; ++i) atomicAdd(jb.db + n0 + mi + acc_row(i, hh), bacc[i]);
}

}  // namespace sb

bool sb_fwd_launch(const SBFwdArgs& a, int C, hipStream_t st) {
  if (a.L < 1 || a.L > kSBMaxLayers || a.B < 1) return false;
  if (C == 128) hipLaunchKernelGGL(sb::sb_fwd_kernel<128>, dim3(a.B), dim3(256), 0, st, a);
  else if (C == 64) hipLaunchKernelGGL(sb::sb_fwd_kernel<64>, dim3(a.B), dim3(128), 0, st, a);
  else return false;
  return true;
}
bool sb_bwd_launch(const SBBwdArgs& a, int C, hipStream_t st) {
  if (a.L < 1 || a.L > kSBMaxLayers || a.B < 1) return false;
  if (C == 128) hipLaunchKernelGGL(sb::sb_bwd_kernel<128>, dim3(a.B), dim3(256), 0, st, a);
  else if (C == 64) hipLaunchKernelGGL(sb::sb_bwd_kernel<64>, dim3(a.B), dim3(128), 0, st, a);
  else return false;
  return true;
}
// rows per split: about 512 rows per workgroup (≥ 1 split; a multiple of 32)
// sj: a slab reduction (the sample-block backward's LayerNorm partials) run by appended workgroups
bool sb_wgrad_launch(SBWgradArgs a, int C, const SlabJob& sj, hipStream_t st) {
  if (a.njobs < 1 || a.njobs > kSBMaxJobs || a.R % sb::NR != 0 || (C != 64 && C != 128)) return false;
  int tiles = 0;
  for (int j = 0; j < a.njobs; ++j) {
    if (a.job[j].N % 64 != 0) return false;
    a.job[j].tile0 = tiles;
    tiles += a.job[j].N / 64;
  }
  int splits = (a.R + 511) / 512;
  a.rows_per_split = (a.R / sb::NR + splits - 1) / splits * sb::NR;
  splits = (a.R + a.rows_per_split - 1) / a.rows_per_split;
  const dim3 grid(tiles + (sj.slab ? (sj.nblk + splits - 1) / splits : 0), splits);
  if (C == 128) hipLaunchKernelGGL(sb::sb_wgrad_kernel<128>, grid, dim3(256), 0, st, a, sj, tiles);
  else hipLaunchKernelGGL(sb::sb_wgrad_kernel<64>, grid, dim3(256), 0, st, a, sj, tiles);
  return true;
}

}  // namespace pio
