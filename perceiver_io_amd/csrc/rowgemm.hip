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

// fp32 gradient targets of the post-attention block (views of the flat gradient buffer).
// Two sinks for a workgroup's parameter-gradient partials:
//  * atomic (slab = 0): targets may be replicated: workgroup i adds into replica
//    i % kGradReplicas, vrs floats apart (vrs = 0: one copy), folded once per step;
//  * slab (slab = 1): workgroup i STORES its partials into row i of a (tiles, P) fp32 slab
//    (vrs = P floats per row).  Float atomics execute at the memory side at ≈1.3 TB/s
//    chip-wide, so 256 tiles × 50 KB of partials per kernel cost ≈10 µs of a ≈25 µs kernel;
//    plain stores cost ≈0.3 µs per CU, and slab_reduce (elementwise.hip) sums the rows on a
//    side stream, overlapped with the rest of the backward chain.
__host__ __device__ __forceinline__ int round_up(int x, int m) { return (x + m - 1) / m * m; }

// ------------------------------------------------------------------------------------
// row-pass layout
// A 256-thread block owns a 64-row tile.  For row-wise work (LayerNorm statistics and
// backward, residual adds, vectorised loads/stores) thread t owns row t >> 2 and the
// 8-column chunks (t & 3) + 4j, j < NCH = ceil(K / 32).  Lanes 4r + p of wave w hold tile
// row 16w + r, so a row reduction is two DPP quad permutes and a column reduction over the
// wave's 16 rows is two DPP row rotations plus two cross-row shuffles.  Every global load of
// a phase is issued before its first use, so a kernel pays the memory latency once per
// phase instead of once per row.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ float quad_sum(float v) {  // over lanes 4r .. 4r+3
  v += dpp<0xB1>(v);                                    // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);                                    // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ float rows16_sum(float v) {  // over lanes ≡ l (mod 4)
  v += dpp<0x124>(v);                                     // row_ror:4
  v += dpp<0x128>(v);                                     // row_ror:8
  return xor32_sum(xor16_sum(v));
}
__device__ __forceinline__ int rp_row() { return threadIdx.x >> 2; }
__device__ __forceinline__ int rp_col(int j) { return 8 * ((threadIdx.x & 3) + 4 * j); }
__device__ __forceinline__ bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// row gr (< R) of a row-major [.. × K] matrix, this thread's chunks; zero outside
template <int NCH, typename T>
__device__ __forceinline__ void row_load(float (&v)[NCH][8], const T* __restrict__ base, long long rs, int gr, int R,
                                         int K, bool vec) {
  if (vec) {  // branch-free (vec ⇒ 16-B aligned base, rs and K multiples of 8): zeros outside
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = rp_col(j);
      const bool ok = gr < R && c < K;
      const T* src = ok ? base + (long long)gr * rs + c : reinterpret_cast<const T*>(kZero32B);
      if constexpr (sizeof(T) == 2) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(src);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[j][e] = bf2f(b[e]);
      } else {
        const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
        v[j][0] = a.x; v[j][1] = a.y; v[j][2] = a.z; v[j][3] = a.w;
        v[j][4] = b.x; v[j][5] = b.y; v[j][6] = b.z; v[j][7] = b.w;
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = rp_col(j);
    const T* src = base + (long long)gr * rs + c;
    if (vec && gr < R && c + 8 <= K) {
      if constexpr (sizeof(T) == 2) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(src);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[j][e] = bf2f(b[e]);
      } else {
        const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
        v[j][0] = a.x; v[j][1] = a.y; v[j][2] = a.z; v[j][3] = a.w;
        v[j][4] = b.x; v[j][5] = b.y; v[j][6] = b.z; v[j][7] = b.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][e] = (gr < R && c + e < K) ? ldf(src + e) : 0.f;
    }
  }
}

// Fourier-PE split input (SURVEY K-03): logical row r = pe[r mod M] (row stride pe_rs, a
// multiple of 8, with npix leading zero columns and zero padding past Kin) + the npix pixel
// values of row r in those leading columns.  The (B, M, npix + C_pe) concatenation is never
// materialised; the PE table stays L2/MALL-resident across the batch.  With idx given (sparse
// images: the LArTPC events' non-zero pixels, models/lartpc.py) row r reads pe[idx[r]] instead
// (clamped into the table), so the gathered [pixel ‖ PE] rows are not materialised either.
struct PeSplit {
  const float* pe;
  int pe_rs, M, npix;
  const long long* idx;
};
// An index outside the table is clamped (no fault); the eager PyTorch path (index_select) raises
// instead.  Checked builds flag it (kErrPeIndex: the launcher raises outside graph capture,
// ops.check_device_errors() after replays); the sparse collator only produces in-range indices.
__device__ __forceinline__ int pe_row(const PeSplit& ps, int gr) {
  if (ps.idx == nullptr) return gr % ps.M;
  const long long i = ps.idx[gr];
  if (i < 0 || i >= ps.M) pio_flag(kErrPeIndex);
  return i < 0 ? 0 : (i >= ps.M ? ps.M - 1 : (int)i);
}

// one fp32 vector of length K (an LN affine) at a 16-byte aligned base, K not a multiple of 8:
// 16-byte loads for the whole 8-column chunks, scalar loads for the tail (zeros past K)
template <int NCH>
__device__ __forceinline__ void vec_load_mixed(float (&v)[NCH][8], const float* __restrict__ base, int K) {
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = rp_col(j);
    if (c + 8 <= K) {
      const float4 a = *reinterpret_cast<const float4*>(base + c), b = *reinterpret_cast<const float4*>(base + c + 4);
      v[j][0] = a.x; v[j][1] = a.y; v[j][2] = a.z; v[j][3] = a.w;
      v[j][4] = b.x; v[j][5] = b.y; v[j][6] = b.z; v[j][7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[j][e] = c + e < K ? ldf(base + c + e) : 0.f;
    }
  }
}
// per-operand vector-load flags of a launch whose operands do not all qualify (AV = false), e.g.
// an odd input width (the LArTPC Fourier input, Kin = 131) with 8-aligned G / W rows
constexpr int kVecG = 1;   // G rows: 16-byte aligned, g_rs and N multiples of 8
constexpr int kVecW = 2;   // W rows: 16-byte aligned, w_rs a multiple of 8 and ≥ Kin
constexpr int kVecLn = 4;  // LN affine vectors 16-byte aligned (whole chunks vectorised)
template <int NCH>
__device__ __forceinline__ void ln_vec_load(float (&v)[NCH][8], const float* __restrict__ base, int K, bool av, int vf) {
  if (!av && (vf & kVecLn)) vec_load_mixed<NCH>(v, base, K);
  else row_load<NCH>(v, base, 0, 0, 1, K, av);
}

template <int NCH, typename T>
__device__ __forceinline__ void row_load_x(float (&v)[NCH][8], const T* __restrict__ X, long long x_rs, int gr, int R,
                                           int Kin, bool vec, const PeSplit& ps) {
  if (ps.pe == nullptr) {
    row_load<NCH>(v, X, x_rs, gr, R, Kin, vec);
    return;
  }
  row_load<NCH>(v, ps.pe, ps.pe_rs, gr < R ? pe_row(ps, gr) : 0, gr < R ? ps.M : 0, ps.pe_rs, true);
  if (gr < R) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = rp_col(j);
      if (c < ps.npix) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (c + e < ps.npix) v[j][e] += ldf(X + (long long)gr * x_rs + c + e);
      }
    }
  }
}

template <int NCH, typename T>
__device__ __forceinline__ void row_store(const float (&v)[NCH][8], T* __restrict__ base, long long rs, int gr, int R,
                                          int K, bool vec) {
  if (gr >= R) return;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = rp_col(j);
    if (c >= K) continue;
    T* dst = base + (long long)gr * rs + c;
    if (vec && c + 8 <= K) {
      if constexpr (sizeof(T) == 2) {
        bf16x8 b;
#pragma unroll
        for (int e = 0; e < 8; ++e) b[e] = (short)f2bf(v[j][e]);
        *reinterpret_cast<bf16x8*>(dst) = b;
      } else {
        *reinterpret_cast<float4*>(dst) = make_float4(v[j][0], v[j][1], v[j][2], v[j][3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(v[j][4], v[j][5], v[j][6], v[j][7]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c + e < K) stf(dst + e, v[j][e]);
    }
  }
}

// LDS row access (this thread's row and chunks); tiles are ≥ 32·NCH columns wide
template <int NCH>
__device__ __forceinline__ void lds_row_read(float (&v)[NCH][8], const float* s, int ld) {
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const float* p = s + rp_row() * ld + rp_col(j);
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[j][0] = a.x; v[j][1] = a.y; v[j][2] = a.z; v[j][3] = a.w;
    v[j][4] = b.x; v[j][5] = b.y; v[j][6] = b.z; v[j][7] = b.w;
  }
}
template <int NCH>
__device__ __forceinline__ void lds_row_write(float* s, int ld, const float (&v)[NCH][8]) {
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    float* p = s + rp_row() * ld + rp_col(j);
    *reinterpret_cast<float4*>(p) = make_float4(v[j][0], v[j][1], v[j][2], v[j][3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[j][4], v[j][5], v[j][6], v[j][7]);
  }
}
template <int NCH>
__device__ __forceinline__ void lds_row_write_bf16(uint16_t* s, int ld, const float (&v)[NCH][8]) {
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    bf16x8 b;
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = (short)f2bf(v[j][e]);
    *reinterpret_cast<bf16x8*>(s + rp_row() * ld + rp_col(j)) = b;
  }
}

// per-thread column values → per-wave column sums in sPart[w][·] (KP-strided); callers
// barrier, then colsum_flush adds the four wave partials into the fp32 gradient
template <int NCH>
__device__ __forceinline__ void colsum_partial(const float (&v)[NCH][8], float* sPart, int KP) {
  const int l = lane_id(), w = wave_id();
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float s = rows16_sum(v[j][e]);
      if (l < 4) sPart[w * KP + rp_col(j) + e] = s;
    }
}
__device__ __forceinline__ void colsum_flush(const float* sPart, int KP, float* __restrict__ dst, int K, int slab) {
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    gadd(dst + k, sPart[k] + sPart[KP + k] + sPart[2 * KP + k] + sPart[3 * KP + k], slab);
}

// rows [r0, r0 + rows) × cols [0, KP) of a bf16 row-major matrix → registers (zero beyond
// Rmax rows / K cols), then → an LDS tile [rows][ld]; NI = ceil(rows·KP / 2048)
template <int NI>
__device__ __forceinline__ void tile_fetch(bf16x8 (&b)[NI], const uint16_t* __restrict__ src, long long rs, int r0,
                                           int Rmax, int rows, int K, int KP, bool vec) {
  const int cpr = KP >> 3;
  if (vec) {  // branch-free (vec ⇒ 16-B aligned src, rs and K multiples of 8): zeros outside
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int e = threadIdx.x + 256 * i, rr = e / cpr, cc = (e - rr * cpr) * 8, gr = r0 + rr;
      const bool ok = rr < rows && gr < Rmax && cc < K;
      const uint16_t* p = ok ? src + (long long)gr * rs + cc : reinterpret_cast<const uint16_t*>(kZero32B);
      b[i] = *reinterpret_cast<const bf16x8*>(p);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int e = threadIdx.x + 256 * i, rr = e / cpr, cc = (e - rr * cpr) * 8, gr = r0 + rr;
    b[i] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (rr < rows && gr < Rmax && cc < K) {
      const uint16_t* p = src + (long long)gr * rs + cc;
      if (vec && cc + 8 <= K) {
        b[i] = *reinterpret_cast<const bf16x8*>(p);
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) b[i][q] = cc + q < K ? (short)p[q] : (short)0;
      }
    }
  }
}
template <int NI>
__device__ __forceinline__ void tile_store(const bf16x8 (&b)[NI], uint16_t* s, int ld, int rows, int KP) {
  const int cpr = KP >> 3;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int e = threadIdx.x + 256 * i, rr = e / cpr, cc = (e - rr * cpr) * 8;
    if (rr < rows) *reinterpret_cast<bf16x8*>(s + rr * ld + cc) = b[i];
  }
}

// 64 × 64 chunk of a gradient matrix G (cols [nc, nc+64)) in the staging layout
// (thread t: rows t>>3 and 32 + (t>>3), cols 8(t&7) .. +8), kept in fp32 for the bias sums
template <typename TG>
__device__ __forceinline__ void g_fetch(float (&v)[2][8], const TG* __restrict__ G, int g_rs, int m0, int R, int nc,
                                        int N, bool vec) {
  if (vec) {  // branch-free (vec ⇒ 16-B aligned G, g_rs and N multiples of 8): zeros outside
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = (threadIdx.x >> 3) + 32 * i, cc = (threadIdx.x & 7) * 8, gr = m0 + rr, gc = nc + cc;
      const TG* p = (gr < R && gc < N) ? G + (long long)gr * g_rs + gc : reinterpret_cast<const TG*>(kZero32B);
      if constexpr (sizeof(TG) == 2) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = bf2f(b[e]);
      } else {
        const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
        v[i][0] = a.x; v[i][1] = a.y; v[i][2] = a.z; v[i][3] = a.w;
        v[i][4] = b.x; v[i][5] = b.y; v[i][6] = b.z; v[i][7] = b.w;
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rr = (threadIdx.x >> 3) + 32 * i, cc = (threadIdx.x & 7) * 8, gr = m0 + rr, gc = nc + cc;
    const TG* p = G + (long long)gr * g_rs + gc;
    if (vec && gr < R && gc + 8 <= N) {
      if constexpr (sizeof(TG) == 2) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[i][e] = bf2f(b[e]);
      } else {
        const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
        v[i][0] = a.x; v[i][1] = a.y; v[i][2] = a.z; v[i][3] = a.w;
        v[i][4] = b.x; v[i][5] = b.y; v[i][6] = b.z; v[i][7] = b.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = (gr < R && gc + e < N) ? ldf(p + e) : 0.f;
    }
  }
}
__device__ __forceinline__ void g_store(const float (&v)[2][8], uint16_t* sG, int ldg) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    bf16x8 b;
#pragma unroll
    for (int e = 0; e < 8; ++e) b[e] = (short)f2bf(v[i][e]);
    *reinterpret_cast<bf16x8*>(sG + ((threadIdx.x >> 3) + 32 * i) * ldg + (threadIdx.x & 7) * 8) = b;
  }
}

// ------------------------------------------------------------------------------------
// LayerNorm(+)Linear forward: Y = act(LN(X)·Wᵀ + b) (+ res), one 64-row tile per block.
// Phase 0 issues the X rows, LN affine and the first 64-row W chunk together; LN runs in
// registers (row-pass layout) into a resident bf16 tile; W chunks are double-buffered
// through registers; each 64-column output chunk leaves through LDS as 16-byte row stores.
// ------------------------------------------------------------------------------------
// LN-Linear shared-memory footprint for NCH chunks: LN(X) tile, W chunk, fp32 output chunk
template <int NCH>
constexpr int ln_linear_fwd_smem() { return 2 * 64 * (32 * NCH + 8) * 2 + 64 * 68 * 4; }

// the LN + GEMM part of one 64-row tile: xv = this thread's rows (row-pass layout), wb = the
// prefetched first W chunk, gw/gb = LN affine (read when has_ln); smem ≥ ln_linear_fwd_smem
// AV: every operand meets the vector-load preconditions (checked on the host) — the loads are
// then straight-line code with no runtime layout branches (see kZero32B)
template <typename TOut, int NCH, bool AV>
__device__ __forceinline__ void ln_linear_fwd_tile(float (&xv)[NCH][8], bf16x8 (&wb)[NCH], const float (&gw)[NCH][8],
                                                   const float (&gb)[NCH][8], bool has_ln, int m0, int R, int Kin,
                                                   float eps, const uint16_t* __restrict__ W, int w_rs,
                                                   const float* __restrict__ bias, int N, int act,
                                                   const float* __restrict__ res, int res_rs, TOut* __restrict__ Y,
                                                   int y_rs, float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                   uint16_t* smem, int part = 0, int nparts = 1, bool wv = false) {
  // nparts > 1: workgroups sharing the tile; this one forms output chunks part, part + nparts, …
  // (wb must hold chunk `part`), the row statistics are the last part's to store
  constexpr int KP = 32 * NCH, LD = KP + 8, LDO = 64 + 4;
  uint16_t* sA = smem;                                  // [64][LD]  LN(X), bf16
  uint16_t* sW = sA + 64 * LD;                          // [64][LD]  W chunk
  float* sO = reinterpret_cast<float*>(sW + 64 * LD);   // [64][LDO] output chunk
  const int gr = m0 + rp_row(), w = wave_id(), l = lane_id();
  // W rows are w_rs apart (≥ Kin, zero padded): a multiple of 8 keeps the staging vectorised
  const bool wvec = AV || wv;
  const int wk = w_rs > Kin ? w_rs : Kin;
  const bool yvec = (N & 7) == 0 && (y_rs & 7) == 0 && aligned16(Y);
  if (has_ln) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) s += xv[j][e];
    const float mean = quad_sum(s) / Kin;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = rp_col(j) + e < Kin ? xv[j][e] - mean : 0.f;
        q += d * d;
      }
    const float rstd = rsqrtf(quad_sum(q) / Kin + eps);
    if ((threadIdx.x & 3) == 0 && gr < R && mean_out && part == nparts - 1) { mean_out[gr] = mean; rstd_out[gr] = rstd; }
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[j][e] = (xv[j][e] - mean) * rstd * gw[j][e] + gb[j][e];
  }
  lds_row_write_bf16<NCH>(sA, LD, xv);

  for (int n0 = 64 * part; n0 < N; n0 += 64 * nparts) {
    tile_store<NCH>(wb, sW, LD, 64, KP);
    lds_sync();
    if (n0 + 64 * nparts < N) tile_fetch<NCH>(wb, W, w_rs, n0 + 64 * nparts, N, 64, wk, KP, wvec);
    const int bc = n0 + 32 * (w & 1) + (l & 31);
    const float bv = (bias && bc < N) ? bias[bc] : 0.f;
    f32x16 acc[1] = {f32x16{}};
    tile_gemm<1, true, true>(sA, LD, sW, LD, 64, 64, KP, acc);
    for_acc<1>(64, 64, [&](int t, int m, int n, int i) {
      float v = acc[t][i] + bv;
      if (act == 1) v = gelu_f(v);
      sO[m * LDO + n] = v;
    });
    lds_sync();
    float ov[2][8];
    lds_row_read<2>(ov, sO, LDO);
    if (res) {
      float rv[2][8];
      row_load<2>(rv, res + n0, res_rs, gr, R, N - n0, false);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) ov[j][e] += rv[j][e];
    }
    row_store<2>(ov, Y + n0, y_rs, gr, R, N - n0, yvec && aligned16(Y + n0));
  }
}

template <typename TIn, typename TOut, int NCH, bool AV>
__global__ __launch_bounds__(256) void ln_linear_fwd_kernel(const TIn* __restrict__ X, int x_rs, int R, int Kin,
                                                            const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                            float eps, const uint16_t* __restrict__ W, int w_rs,
                                                            const float* __restrict__ bias, int N, int act,
                                                            const float* __restrict__ res, int res_rs,
                                                            TOut* __restrict__ Y, int y_rs, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out, PeSplit ps, int vf) {
  constexpr int KP = 32 * NCH;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int m0 = blockIdx.x * 64, gr = m0 + rp_row();
  const int part = (int)blockIdx.y, nparts = (int)gridDim.y;  // workgroups per tile (split_tiles)
  // phase 0: X rows, the first W chunk (of this part) and the LN affine in flight together
  float xv[NCH][8];
  row_load_x<NCH>(xv, X, x_rs, gr, R, Kin, AV, ps);
  bf16x8 wb[NCH];
  tile_fetch<NCH>(wb, W, w_rs, 64 * part, N, 64, w_rs > Kin ? w_rs : Kin, KP, AV || (vf & kVecW));
  float gw[NCH][8], gb[NCH][8];
  if (lnw) {
    ln_vec_load<NCH>(gw, lnw, Kin, AV, vf);
    ln_vec_load<NCH>(gb, lnb, Kin, AV, vf);
  }
  ln_linear_fwd_tile<TOut, NCH, AV>(xv, wb, gw, gb, lnw != nullptr, m0, R, Kin, eps, W, w_rs, bias, N, act, res, res_rs, Y,
                                y_rs, mean_out, rstd_out, smem, part, nparts, (vf & kVecW) != 0);
}

// ------------------------------------------------------------------------------------
// post-attention block forward: Z = Y + W2·gelu(W1·LN2(Y) + b1) + b2, Y = X + Wo·O + bo
// Phase 0 fetches the O tile, the X rows and (C ≤ 64) all three weights; the three GEMMs
// then run back to back on LDS with row-pass epilogues (LN2 in registers, 16-byte stores).
// For C = 128 the weights share one LDS buffer, each fetched during the previous GEMM.
// ------------------------------------------------------------------------------------
// phase-0 operands of the post-attention block that do not depend on the attention output:
// the weights (C ≤ 64: all three), the residual rows and the bias / LN2 vectors (thread k < C
// holds entry k) — issued before the attention in the fused self-attention layer kernel
template <int C>
struct PaPre {
  static constexpr int NCH = C / 32, NWB = C <= 64 ? 3 : 1, NIW = (C * C / 8 + 255) / 256;
  bf16x8 wr[NWB][NIW];
  float yv[NCH][8];
  float pp[5];
};
template <int C, bool AV>
__device__ __forceinline__ void post_attn_fwd_prefetch(PaPre<C>& pre, const float* __restrict__ X,
                                                       const uint16_t* __restrict__ Wo, const float* __restrict__ bo,
                                                       const float* __restrict__ g2, const float* __restrict__ be2,
                                                       const uint16_t* __restrict__ W1, const float* __restrict__ b1,
                                                       const uint16_t* __restrict__ W2, const float* __restrict__ b2,
                                                       int R, int Rx) {
  using P = PaPre<C>;
  const int gr = blockIdx.x * 64 + rp_row();
  tile_fetch<P::NIW>(pre.wr[0], Wo, C, 0, C, C, C, C, AV);
  if constexpr (P::NWB == 3) {
    tile_fetch<P::NIW>(pre.wr[1], W1, C, 0, C, C, C, C, AV);
    tile_fetch<P::NIW>(pre.wr[2], W2, C, 0, C, C, C, C, AV);
  }
  row_load<P::NCH>(pre.yv, X, C, gr < R ? gr % Rx : Rx, Rx, C, AV);
  // bias / LN2 vectors: address select (thread ≥ C reads a zero), no branch around the loads
  const int k = threadIdx.x < C ? (int)threadIdx.x : 0;
  pre.pp[0] = bo[k]; pre.pp[1] = b1[k]; pre.pp[2] = b2[k]; pre.pp[3] = g2[k]; pre.pp[4] = be2[k];
}

// one 64-row tile; Z is also left in z (row-pass registers) for a fused epilogue.  OLDS: the
// attention output tile is already in LDS (sO, [64][C + 8] bf16, written by the caller before a
// barrier); else it is fetched from O.
template <int C, bool AV, bool OLDS = false>
__device__ __forceinline__ void post_attn_fwd_body(
    const uint16_t* __restrict__ O, const float* __restrict__ X, const uint16_t* __restrict__ Wo,
    const float* __restrict__ bo, const float* __restrict__ g2, const float* __restrict__ be2, float eps,
    const uint16_t* __restrict__ W1, const float* __restrict__ b1, const uint16_t* __restrict__ W2,
    const float* __restrict__ b2, float* __restrict__ Z, float* __restrict__ Ysave, float* __restrict__ mean2,
    float* __restrict__ rstd2, uint16_t* __restrict__ Usave, int R, int Rx, const DropCfg& dr, float (&z)[C / 32][8],
    PaPre<C>& pre, const uint16_t* sO = nullptr, bool store_rows = true) {
  // store_rows = false: a workgroup sharing the tile with the one that stores Y, U, Z, the LN2
  // statistics (post_attn_ln_linear_fwd_kernel split over the next projection's columns)
  // X has Rx rows, row r of the tile adds X[r % Rx] (Rx < R: batch-broadcast residual).
  // Residual dropout (dr.thresh > 0): Y = X + drop₀(attn-out), Z = Y + drop₁(MLP(Y)), masks
  // hashed from (device seed, site, row·C + col) and regenerated by the backward.
  constexpr int LD = C + 8, LDF = C + 4, MAXT = (2 * C / 32 + 3) / 4, NCH = C / 32;
  constexpr int NWB = C <= 64 ? 3 : 1, NIW = (C * C / 8 + 255) / 256;
  __shared__ __attribute__((aligned(16))) uint16_t sA[64 * LD];   // O → LN2(Y) → GELU(U)
  __shared__ __attribute__((aligned(16))) uint16_t sW[NWB][C * LD];
  __shared__ __attribute__((aligned(16))) float sF[64 * LDF];
  __shared__ float sP[5][C];  // bo, b1, b2, γ2, β2
  const int m0 = blockIdx.x * 64, gr = m0 + rp_row();
  constexpr bool av = AV;  // O, X, Z, Ysave, Usave, Wo, W1, W2 16-B aligned (host-checked)

  bf16x8 (&wr)[NWB][NIW] = pre.wr;
  float (&yv)[NCH][8] = pre.yv;
  if constexpr (!OLDS) {
    bf16x8 ob[NCH];
    tile_fetch<NCH>(ob, O, C, m0, R, 64, C, C, av);
    tile_store<NCH>(ob, sA, LD, 64, C);
  }
  if (threadIdx.x < C) {
    const int k = threadIdx.x;
    sP[0][k] = pre.pp[0]; sP[1][k] = pre.pp[1]; sP[2][k] = pre.pp[2]; sP[3][k] = pre.pp[3]; sP[4][k] = pre.pp[4];
  }
#pragma unroll
  for (int b = 0; b < NWB; ++b) tile_store<NIW>(wr[b], sW[b], LD, C, C);
  lds_sync();
  if constexpr (NWB == 1) tile_fetch<NIW>(wr[0], W1, C, 0, C, C, C, C, av);
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, true>(OLDS ? sO : sA, LD, sW[0], LD, 64, C, C, acc);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) { sF[m * LDF + n] = acc[t][i] + sP[0][n]; });
  lds_sync();
  if constexpr (NWB == 1) tile_store<NIW>(wr[0], sW[0], LD, C, C);
  // Y = X + attn-out; LN2 → sA
  {
    float t[NCH][8];
    lds_row_read<NCH>(t, sF, LDF);
    drop_rows<NCH>(t, dr, 0u, gr, C);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) { yv[j][e] += t[j][e]; s += yv[j][e]; }
    if (store_rows) row_store<NCH>(yv, Ysave, C, gr, R, C, av);
    const float mean = quad_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = yv[j][e] - mean; q += d * d; }
    const float rstd = rsqrtf(quad_sum(q) / C + eps);
    if ((threadIdx.x & 3) == 0 && gr < R && store_rows) { mean2[gr] = mean; rstd2[gr] = rstd; }
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = rp_col(j) + e;
        t[j][e] = (yv[j][e] - mean) * rstd * sP[3][c] + sP[4][c];
      }
    lds_row_write_bf16<NCH>(sA, LD, t);
  }
  lds_sync();
  if constexpr (NWB == 1) tile_fetch<NIW>(wr[0], W2, C, 0, C, C, C, C, av);
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, true>(sA, LD, sW[NWB == 3 ? 1 : 0], LD, 64, C, C, acc);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) { sF[m * LDF + n] = acc[t][i] + sP[1][n]; });
  lds_sync();
  if constexpr (NWB == 1) tile_store<NIW>(wr[0], sW[0], LD, C, C);
  {
    float u[NCH][8];
    lds_row_read<NCH>(u, sF, LDF);
    if (store_rows) row_store<NCH>(u, Usave, C, gr, R, C, av);
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) u[j][e] = gelu_f(u[j][e]);
    lds_row_write_bf16<NCH>(sA, LD, u);
  }
  lds_sync();
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, true>(sA, LD, sW[NWB == 3 ? 2 : 0], LD, 64, C, C, acc);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) { sF[m * LDF + n] = acc[t][i] + sP[2][n]; });
  lds_sync();
  lds_row_read<NCH>(z, sF, LDF);
  drop_rows<NCH>(z, dr, 1u, gr, C);
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) z[j][e] += yv[j][e];
  if (store_rows) row_store<NCH>(z, Z, C, gr, R, C, av);
}

template <int C, bool AV>
__global__ __launch_bounds__(256) void post_attn_fwd_kernel(
    const uint16_t* __restrict__ O, const float* __restrict__ X, const uint16_t* __restrict__ Wo,
    const float* __restrict__ bo, const float* __restrict__ g2, const float* __restrict__ be2, float eps,
    const uint16_t* __restrict__ W1, const float* __restrict__ b1, const uint16_t* __restrict__ W2,
    const float* __restrict__ b2, float* __restrict__ Z, float* __restrict__ Ysave, float* __restrict__ mean2,
    float* __restrict__ rstd2, uint16_t* __restrict__ Usave, int R, int Rx, DropCfg dr) {
  float z[C / 32][8];
  PaPre<C> pre;
  post_attn_fwd_prefetch<C, AV>(pre, X, Wo, bo, g2, be2, W1, b1, W2, b2, R, Rx);
  post_attn_fwd_body<C, AV>(O, X, Wo, bo, g2, be2, eps, W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, Rx, dr, z,
                            pre);
}

// ------------------------------------------------------------------------------------
// cross-layer fusion inside a self-attention block (layer l → l+1, both row-local):
// post-attention block of layer l, then LayerNorm1 + packed QKV projection of layer l+1 on the
// same 64-row tile straight from the Z registers — one launch and one phase-0 latency fewer
// per layer boundary, and Z is never re-read.  The QKV chunk-0 weights and the LN1 affine are
// fetched in phase 0 with everything else.
// ------------------------------------------------------------------------------------
template <int C, bool AV>
__global__ __launch_bounds__(256) void post_attn_ln_linear_fwd_kernel(
    const uint16_t* __restrict__ O, const float* __restrict__ X, const uint16_t* __restrict__ Wo,
    const float* __restrict__ bo, const float* __restrict__ g2, const float* __restrict__ be2, float eps,
    const uint16_t* __restrict__ W1, const float* __restrict__ b1, const uint16_t* __restrict__ W2,
    const float* __restrict__ b2, float* __restrict__ Z, float* __restrict__ Ysave, float* __restrict__ mean2,
    float* __restrict__ rstd2, uint16_t* __restrict__ Usave, int R, int Rx, const float* __restrict__ lnw,
    const float* __restrict__ lnb, const uint16_t* __restrict__ Wq, const float* __restrict__ bq,
    uint16_t* __restrict__ QKV, float* __restrict__ mean1, float* __restrict__ rstd1, DropCfg dr) {
  constexpr int NCH = C / 32, KP = 32 * NCH;
  __shared__ __attribute__((aligned(16))) uint16_t smem[ln_linear_fwd_smem<NCH>() / 2];  // LN1+QKV half
  // gridDim.y workgroups per tile (split_tiles): each runs the post-attention chain and forms every
  // gridDim.y-th 64-column chunk of the next QKV; part 0 stores the chain's row outputs
  const int part = (int)blockIdx.y, nparts = (int)gridDim.y;
  bf16x8 wb[NCH];
  tile_fetch<NCH>(wb, Wq, C, 64 * part, 3 * C, 64, C, KP, AV);
  float gw[NCH][8], gb[NCH][8];
  row_load<NCH>(gw, lnw, 0, 0, 1, C, AV);
  row_load<NCH>(gb, lnb, 0, 0, 1, C, AV);
  float z[NCH][8];
  PaPre<C> pre;
  post_attn_fwd_prefetch<C, AV>(pre, X, Wo, bo, g2, be2, W1, b1, W2, b2, R, Rx);
  post_attn_fwd_body<C, AV>(O, X, Wo, bo, g2, be2, eps, W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, Rx, dr, z, pre,
                            nullptr, part == 0);
  ln_linear_fwd_tile<uint16_t, NCH, AV>(z, wb, gw, gb, true, blockIdx.x * 64, R, C, eps, Wq, C, bq, 3 * C, 0, nullptr, 0,
                                    QKV, 3 * C, mean1, rstd1, smem, part, nparts);
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
                                           int Nvalid, int Kvalid, float* __restrict__ dW, int dw_rs, int slab) {
  f32x16 acc[MAXW];
#pragma unroll
  for (int t = 0; t < MAXW; ++t) acc[t] = f32x16{};
  tile_gemm<MAXW, false, false>(sG, ldg, sX, ldx, NG, KX, 64, acc);
  for_acc<MAXW>(NG, KX, [&](int t, int m, int n, int i) {
    if (m < Nvalid && n < Kvalid) gadd(dW + (long long)m * dw_rs + n, acc[t][i], slab);
  });
}

// ------------------------------------------------------------------------------------
// post-attention block backward, one 64-row tile, weight gradients included:
//   dH = dZ·W2, dW2 += dZᵀ·GELU(U), db2 += Σ dZ
//   dU = dH∘GELU'(U), dXn2 = dU·W1, dW1 += dUᵀ·LN2(Y), db1 += Σ dU
//   dY = dZ + LN2_bwd(dXn2), dγ2 += Σ dXn2∘Ŷ, dβ2 += Σ dXn2
//   dO = dY·Wo, dWo += dYᵀ·O, dbo += Σ dY, delta = rowsum_head(dO∘O)
// The gradient tile (sG) and its matching activation tile (sX) sit side by side in LDS, so
// each weight gradient is one extra MFMA pass over resident tiles.  Phase 0 fetches dZ, Y,
// U, O and (C ≤ 64) all weights at once; the rest of the kernel touches global memory only
// to store results and to add parameter gradients.
// ------------------------------------------------------------------------------------
// which of the nparts workgroups sharing a tile stores output group g (0: dW2, 1: dW1, 2: dWo,
// 3: the row outputs, the vector and LayerNorm gradients); the QKV weight chunks of the fused
// boundary kernel go round-robin (chunk j → part j mod nparts)
__host__ __device__ constexpr int tile_part_owner(int g, int nparts) {
  return nparts == 1 ? 0 : nparts == 2 ? (g == 0 || g == 3 ? 0 : 1) : (g == 0 ? 0 : g == 1 ? 1 : g == 2 ? 2 : 3);
}

// workgroups per 64-row tile of the post-attention backward kernels when the tiles fill only a
// fraction of the chip (the C = 128 image latent stacks: 16-64 tiles): each runs the tile's row
// chain and stores its share of the outputs (tile_part_owner); measured: 2 per tile took the
// ImageNet step's boundary backward from 50 to 40 µs per launch
static inline unsigned split_tiles(int R) {
  const int t = (R + 63) / 64;
  return t <= 64 ? 4u : t < 128 ? 2u : 1u;
}

// LDS bytes of post_attn_bwd_body: sG, sX, sW[NWB], sF, sPart, sDb1, sP
template <int C>
constexpr int post_attn_bwd_smem() {
  return 2 * (2 * 64 * (C + 8) + (C <= 64 ? 3 : 1) * C * (C + 8)) + 4 * (64 * (C + 4) + 16 * C + 2 * C + 2 * C);
}

// dz: this thread's rows of dZ (row-pass layout), loaded by the caller or produced by a fused
// prologue (ln_linear_post_attn_bwd_kernel); smem ≥ post_attn_bwd_smem<C>() bytes, 16-B aligned
template <int C, bool AV>
__device__ __forceinline__ void post_attn_bwd_body(
    float (&dz)[C / 32][8], const float* __restrict__ Ysave, const float* __restrict__ mean2,
    const float* __restrict__ rstd2, const uint16_t* __restrict__ U, const uint16_t* __restrict__ O,
    const uint16_t* __restrict__ Wo, const uint16_t* __restrict__ W1, const uint16_t* __restrict__ W2,
    const float* __restrict__ g2, const float* __restrict__ be2, float* __restrict__ dY, uint16_t* __restrict__ dO,
    float* __restrict__ delta, int H, PostAttnGrads gr_out, int R, const DropCfg& dr, unsigned char* smem,
    int part = 0, int nparts = 1) {
  // residual dropout: the MLP output layer sees dZ∘m₁, the out-projection dY∘m₀; the residual
  // gradients (dZ into dY, dY out of the kernel) stay unmasked.
  // nparts > 1: that many workgroups share the tile (small row counts: more workgroups on the
  // chip); all run the whole row chain, each stores its share of the outputs (tile_part_owner) —
  // every output and gradient element keeps exactly one writer
  const bool own_w2 = tile_part_owner(0, nparts) == part, own_w1 = tile_part_owner(1, nparts) == part;
  const bool own_wo = tile_part_owner(2, nparts) == part, own_rows = tile_part_owner(3, nparts) == part;

  constexpr int LD = C + 8, LDF = C + 4, MAXT = (2 * C / 32 + 3) / 4, MAXW = ((C / 32) * (C / 32) + 3) / 4;
  constexpr int NCH = C / 32, NWB = C <= 64 ? 3 : 1, NIW = (C * C / 8 + 255) / 256;
  uint16_t* sG = reinterpret_cast<uint16_t*>(smem);  // [64][LD] dZ → dU → dY
  uint16_t* sX = sG + 64 * LD;                        // [64][LD] GELU(U) → LN2(Y) → O
  uint16_t(*sW)[C * LD] = reinterpret_cast<uint16_t(*)[C * LD]>(sX + 64 * LD);  // W2, W1, Wo
  float* sF = reinterpret_cast<float*>(sX + 64 * LD + NWB * C * LD);           // [64][LDF] GELU'(U) → dU → dXn2 → dO
  float(*sPart)[4 * C] = reinterpret_cast<float(*)[4 * C]>(sF + 64 * LDF);     // wave partials: Σ dZ, dγ2, dβ2, Σ dY
  float(*sDb1)[C] = reinterpret_cast<float(*)[C]>(sF + 64 * LDF + 16 * C);
  float(*sP)[C] = reinterpret_cast<float(*)[C]>(sF + 64 * LDF + 18 * C);       // γ2, β2
  const int m0 = blockIdx.x * 64, gr = m0 + rp_row(), w = wave_id(), l = lane_id();
  constexpr bool av = AV;  // Ysave, U, O, dY, dO, Wo, W1, W2 16-B aligned (host-checked)

  // ---- phase 0: every input of the tile in flight at once
  PIO_TS(0);
  float yv[NCH][8], t0[NCH][8];
  row_load<NCH>(yv, Ysave, C, gr, R, C, av);
  row_load<NCH>(t0, U, C, gr, R, C, av);
  bf16x8 ob[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const uint16_t* p = gr < R ? O + (long long)gr * C + rp_col(j) : reinterpret_cast<const uint16_t*>(kZero32B);
    ob[j] = *reinterpret_cast<const bf16x8*>(p);
  }
  const float mu = *(gr < R ? mean2 + gr : kZero32B), rs = *(gr < R ? rstd2 + gr : kZero32B);
  bf16x8 wr[NWB][NIW];
  tile_fetch<NIW>(wr[0], W2, C, 0, C, C, C, C, av);
  if constexpr (NWB == 3) {
    tile_fetch<NIW>(wr[1], W1, C, 0, C, C, C, C, av);
    tile_fetch<NIW>(wr[2], Wo, C, 0, C, C, C, C, av);
  }
  for (int k = threadIdx.x; k < C; k += blockDim.x) { sP[0][k] = g2[k]; sP[1][k] = be2[k]; }
  PIO_TS(1);
  float dzm[NCH][8];  // dZ∘m₁: the MLP output layer's gradient
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) dzm[j][e] = dz[j][e];
  drop_rows<NCH>(dzm, dr, 1u, gr, C);
  lds_row_write_bf16<NCH>(sG, LD, dzm);
  {
    float gp[NCH][8];
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) { gp[j][e] = gelu_grad(t0[j][e]); t0[j][e] = gelu_f(t0[j][e]); }
    lds_row_write_bf16<NCH>(sX, LD, t0);
    lds_row_write<NCH>(sF, LDF, gp);
  }
#pragma unroll
  for (int b = 0; b < NWB; ++b) tile_store<NIW>(wr[b], sW[b], LD, C, C);
  colsum_partial<NCH>(dzm, sPart[0], C);
  PIO_TS(2);
  lds_sync();
  PIO_TS(3);
  if constexpr (NWB == 1) tile_fetch<NIW>(wr[0], W1, C, 0, C, C, C, C, av);

  // ---- MLP output layer
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, false>(sG, LD, sW[0], LD, 64, C, C, acc);  // dH = dZ · W2
  PIO_TS(4);
  if (own_w2) wgrad_tile<MAXW>(sG, LD, sX, LD, C, C, C, C, rep(gr_out.dW2, gr_out.vrs, gr_out.slab), C, gr_out.slab);
  PIO_TS(5);
  {
    constexpr int NTN = C / 32;
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      const int tg = w + 4 * t;
      if (tg < 2 * NTN) {
        const int mt = tg / NTN, n0 = 32 * (tg % NTN), hh = l >> 5;
        float cs = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = 32 * mt + acc_row(i, hh), n = n0 + (l & 31);
          const float du = acc[t][i] * sF[m * LDF + n];
          sF[m * LDF + n] = du;
          cs += du;
        }
        cs = xor32_sum(cs);
        if (l < 32) sDb1[mt][n0 + l] = cs;
      }
    }
  }
  PIO_TS(6);
  lds_sync();
  PIO_TS(7);
  for (int k = threadIdx.x; k < (own_rows ? C : 0); k += blockDim.x) {
    gadd(rep(gr_out.db1, gr_out.vrs, gr_out.slab) + k,
         sDb1[0][k] + sDb1[1][k], gr_out.slab);
    gadd(rep(gr_out.db2, gr_out.vrs, gr_out.slab) + k,
         sPart[0][k] + sPart[0][C + k] + sPart[0][2 * C + k] + sPart[0][3 * C + k], gr_out.slab);
  }
  if constexpr (NWB == 1) tile_store<NIW>(wr[0], sW[0], LD, C, C);
  {
    float du[NCH][8];
    lds_row_read<NCH>(du, sF, LDF);
    lds_row_write_bf16<NCH>(sG, LD, du);
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = rp_col(j) + e;
        t0[j][e] = (yv[j][e] - mu) * rs * sP[0][c] + sP[1][c];
      }
    lds_row_write_bf16<NCH>(sX, LD, t0);
  }
  PIO_TS(8);
  lds_sync();
  PIO_TS(9);
  if constexpr (NWB == 1) tile_fetch<NIW>(wr[0], Wo, C, 0, C, C, C, C, av);

  // ---- MLP hidden layer
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, false>(sG, LD, sW[NWB == 3 ? 1 : 0], LD, 64, C, C, acc);  // dXn2 = dU · W1
  if (own_w1) wgrad_tile<MAXW>(sG, LD, sX, LD, C, C, C, C, rep(gr_out.dW1, gr_out.vrs, gr_out.slab), C, gr_out.slab);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) { sF[m * LDF + n] = acc[t][i]; });
  PIO_TS(10);
  lds_sync();
  PIO_TS(11);
  if constexpr (NWB == 1) tile_store<NIW>(wr[0], sW[0], LD, C, C);
  // ---- LN2 backward → dY = dZ + LN_bwd(dXn2); the O tile replaces LN2(Y) in sX
  {
    float dxn[NCH][8];
    lds_row_read<NCH>(dxn, sF, LDF);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        yv[j][e] = (yv[j][e] - mu) * rs;  // ŷ
        const float g = dxn[j][e] * sP[0][rp_col(j) + e];
        s1 += g;
        s2 += g * yv[j][e];
      }
    s1 = quad_sum(s1) / C;
    s2 = quad_sum(s2) / C;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dz[j][e] += rs * (dxn[j][e] * sP[0][rp_col(j) + e] - s1 - yv[j][e] * s2);  // dY
        yv[j][e] *= dxn[j][e];                                                      // dγ2 terms
      }
    colsum_partial<NCH>(yv, sPart[1], C);
    colsum_partial<NCH>(dxn, sPart[2], C);
    if (own_rows) row_store<NCH>(dz, dY, C, gr, R, C, av);
    drop_rows<NCH>(dz, dr, 0u, gr, C);  // dY∘m₀: the out-projection's gradient
    colsum_partial<NCH>(dz, sPart[3], C);
    lds_row_write_bf16<NCH>(sG, LD, dz);
#pragma unroll
    for (int j = 0; j < NCH; ++j) *reinterpret_cast<bf16x8*>(sX + rp_row() * LD + rp_col(j)) = ob[j];
  }
  PIO_TS(12);
  lds_sync();
  PIO_TS(13);
  for (int k = threadIdx.x; k < (own_rows ? C : 0); k += blockDim.x) {
    gadd(rep(gr_out.dg2, gr_out.vrs, gr_out.slab) + k,
         sPart[1][k] + sPart[1][C + k] + sPart[1][2 * C + k] + sPart[1][3 * C + k], gr_out.slab);
    gadd(rep(gr_out.dbe2, gr_out.vrs, gr_out.slab) + k,
         sPart[2][k] + sPart[2][C + k] + sPart[2][2 * C + k] + sPart[2][3 * C + k], gr_out.slab);
    gadd(rep(gr_out.dbo, gr_out.vrs, gr_out.slab) + k,
         sPart[3][k] + sPart[3][C + k] + sPart[3][2 * C + k] + sPart[3][3 * C + k], gr_out.slab);
  }

  // ---- out-projection
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  tile_gemm<MAXT, true, false>(sG, LD, sW[NWB == 3 ? 2 : 0], LD, 64, C, C, acc);  // dO = dY · Wo
  if (own_wo) wgrad_tile<MAXW>(sG, LD, sX, LD, C, C, C, C, rep(gr_out.dWo, gr_out.vrs, gr_out.slab), C, gr_out.slab);
  PIO_TS(14);
  for_acc<MAXT>(64, C, [&](int t, int m, int n, int i) { sF[m * LDF + n] = bf2f(f2bf(acc[t][i])); });
  lds_sync();
  PIO_TS(15);
  if (own_rows) {
    float dov[NCH][8];
    lds_row_read<NCH>(dov, sF, LDF);
    row_store<NCH>(dov, dO, C, gr, R, C, av);
    // delta[r, h] = Σ_d dO·O over head h's columns (bf16 values, as the attention sees them);
    // every 8-column chunk lies inside one head (D ≥ 8)
    const int D = C / H;
    for (int h = 0; h < H; ++h) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j)
        if (rp_col(j) / D == h) {
#pragma unroll
          for (int e = 0; e < 8; ++e) s += dov[j][e] * bf2f(ob[j][e]);
        }
      s = quad_sum(s);
      if ((threadIdx.x & 3) == 0 && gr < R) delta[(long long)gr * H + h] = s;
    }
  }
  PIO_TS(16);
}

template <int C, bool AV>
__global__ __launch_bounds__(256) void post_attn_bwd_kernel(
    const float* __restrict__ dZ, const float* __restrict__ Ysave, const float* __restrict__ mean2,
    const float* __restrict__ rstd2, const uint16_t* __restrict__ U, const uint16_t* __restrict__ O,
    const uint16_t* __restrict__ Wo, const uint16_t* __restrict__ W1, const uint16_t* __restrict__ W2,
    const float* __restrict__ g2, const float* __restrict__ be2, float* __restrict__ dY, uint16_t* __restrict__ dO,
    float* __restrict__ delta, int H, PostAttnGrads gr_out, int R, SlabJob job, DropCfg dr) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[post_attn_bwd_smem<C>()];
  if (blockIdx.y == 0) zero_span_block(job);
  if ((int)blockIdx.x >= (R + 63) / 64) {  // appended workgroups: the previous kernel's slab job
    {  // the appended job workgroups span every grid row: block (x − tiles)·gridDim.y + y
      const int jb = (int)(blockIdx.x - (R + 63) / 64) * (int)gridDim.y + (int)blockIdx.y;
      if (jb < job.nblk) slab_reduce_block(job, jb, reinterpret_cast<float4*>(smem));
    }
    return;
  }
  float dz[C / 32][8];
  row_load<C / 32>(dz, dZ, C, blockIdx.x * 64 + rp_row(), R, C, AV);
  post_attn_bwd_body<C, AV>(dz, Ysave, mean2, rstd2, U, O, Wo, W1, W2, g2, be2, dY, dO, delta, H, gr_out, R, dr, smem,
                            (int)blockIdx.y, (int)gridDim.y);
}

// ------------------------------------------------------------------------------------
// LayerNorm(+)Linear backward, one 64-row tile:
//   dXn = G·W (N streamed in 64-column chunks, double-buffered through registers),
//   dW += Gᵀ·LN(X), db += Σ G (per chunk, atomics), dX = LN_bwd(dXn) (+ dres), dγ/dβ.
// ------------------------------------------------------------------------------------
// bytes: sG | sW | sXn during the chunk loop, the fp32 dXn tile sF over the same bytes after it,
// then sPart | sPb (≈57 KB at 160 channels: two workgroups per CU)
template <int NCH>
constexpr int ln_linear_bwd_loop_smem() {
  return 64 * 72 * 2 + 2 * 64 * (32 * NCH + 8) * 2 > 64 * (32 * NCH + 4) * 4
             ? 64 * 72 * 2 + 2 * 64 * (32 * NCH + 8) * 2
             : 64 * (32 * NCH + 4) * 4;
}
template <int NCH>
constexpr int ln_linear_bwd_smem() {
  return ln_linear_bwd_loop_smem<NCH>() + 8 * 32 * NCH * 4 + 4 * 64 * 4;
}

// one 64-row tile; dX (incl. dres) is also left in dxo (row-pass registers) for a fused epilogue
template <typename TG, typename TX, int NCH, bool AV>
__device__ __forceinline__ void ln_linear_bwd_body(
    const TG* __restrict__ G, int g_rs, int N, const uint16_t* __restrict__ W, int w_rs, int Kin,
    const TX* __restrict__ X,
    int x_rs, const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ lnw,
    const float* __restrict__ lnb, const float* __restrict__ dres, int dres_rs, float* __restrict__ dX, int dx_rs,
    float* __restrict__ dlnw, float* __restrict__ dlnb, float* __restrict__ dW, float* __restrict__ db, int vrs,
    int wrs, int slab, int R, PeSplit ps, uint16_t* smem, float (&dxo)[NCH][8], int part = 0, int nparts = 1,
    int vf = 0) {
  // nparts > 1: workgroups sharing the tile; the weight / bias gradient of 64-column chunk j is
  // part (j mod nparts)'s, the LN gradients and dX the row-output owner's (tile_part_owner)
  const bool own_rows = tile_part_owner(3, nparts) == part;
  constexpr int KP = 32 * NCH, LD = KP + 8, LDG = 64 + 8, LDF = KP + 4;
  uint16_t* sG = smem;                                   // [64][LDG]  G chunk
  uint16_t* sW = sG + 64 * LDG;                          // [64][LD]   W chunk
  uint16_t* sXn = sW + 64 * LD;                          // [64][LD]   LN(X)
  float* sF = reinterpret_cast<float*>(smem);            // [64][LDF]  dXn, after the loop (over sG | sW | sXn)
  float* sPart = reinterpret_cast<float*>(smem + ln_linear_bwd_loop_smem<NCH>() / 2);  // [2][4][KP]
  float* sPb = sPart + 8 * KP;                           // [4][64]
  const int m0 = blockIdx.x * 64, gr = m0 + rp_row(), w = wave_id(), l = lane_id();
  // AV: G, W, X, the LN affine and dres meet the vector-load preconditions (host-checked);
  // otherwise vf names the operands that still do (kVecG / kVecW / kVecLn)
  const bool gvec = AV || (vf & kVecG), wvec = AV || (vf & kVecW);
  const int wk = w_rs > Kin ? w_rs : Kin;  // W rows zero padded to w_rs
  const bool kvec = (Kin & 7) == 0;

  // ---- phase 0
  float xv[NCH][8], gw[NCH][8];
  row_load_x<NCH>(xv, X, x_rs, gr, R, Kin, AV, ps);
  float mu = 0.f, rs = 1.f;
  if (lnw) {
    ln_vec_load<NCH>(gw, lnw, Kin, AV, vf);
    mu = *(gr < R ? mean + gr : kZero32B);  // address selects: no conditional loads
    rs = *(gr < R ? rstd + gr : kZero32B);
  }
  float gv[2][8];
  g_fetch<TG>(gv, G, g_rs, m0, R, 0, N, gvec);
  bf16x8 wb[NCH];
  tile_fetch<NCH>(wb, W, w_rs, 0, N, 64, wk, KP, wvec);
  if (dW) {  // LN(X), the forward GEMM's A operand, for the weight gradient
    float xn[NCH][8];
    if (lnw) {
      ln_vec_load<NCH>(xn, lnb, Kin, AV, vf);
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) xn[j][e] += (xv[j][e] - mu) * rs * gw[j][e];
    } else {
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) xn[j][e] = xv[j][e];
    }
    lds_row_write_bf16<NCH>(sXn, LD, xn);
  }

  constexpr int MAXT = 3;  // (64/32)·(KP/32) ≤ 10 sub-tiles (KP ≤ 160)
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  for (int nc = 0; nc < N; nc += 64) {
    g_store(gv, sG, LDG);
    tile_store<NCH>(wb, sW, LD, 64, KP);
    float cs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[e] = gv[0][e] + gv[1][e];
    lds_sync();
    if (nc + 64 < N) {
      g_fetch<TG>(gv, G, g_rs, m0, R, nc + 64, N, gvec);
      tile_fetch<NCH>(wb, W, w_rs, nc + 64, N, 64, wk, KP, wvec);
    }
    tile_gemm<MAXT, true, false>(sG, LDG, sW, LD, 64, KP, 64, acc);
    const bool mine = (nc >> 6) % nparts == part;
    if (dW && mine) {
      wgrad_tile<MAXT>(sG, LDG, sXn, LD, 64, KP, N - nc, Kin, rep(dW, wrs, slab) + (long long)nc * Kin, Kin, slab);
      if (db) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float s = xor32_sum(xor16_sum(cs[e] + dpp<0x128>(cs[e])));  // lanes ≡ l (mod 8)
          if (l < 8) sPb[w * 64 + 8 * l + e] = s;
        }
      }
    }
    lds_sync();
    if (dW && mine && db && threadIdx.x < 64 && nc + (int)threadIdx.x < N) {
      const int t = threadIdx.x;
      gadd(rep(db, vrs, slab) + nc + t, sPb[t] + sPb[64 + t] + sPb[128 + t] + sPb[192 + t], slab);
    }
  }
  for_acc<MAXT>(64, KP, [&](int t, int m, int n, int i) { sF[m * LDF + n] = acc[t][i]; });
  lds_sync();

  // ---- row pass: LN backward, residual gradient, LN parameter gradients
  float dr[NCH][8];
  if (dres) row_load<NCH>(dr, dres, dres_rs, gr, R, Kin, AV);
  float dxn[NCH][8];
  lds_row_read<NCH>(dxn, sF, LDF);
  if (lnw) {
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xv[j][e] = rp_col(j) + e < Kin ? (xv[j][e] - mu) * rs : 0.f;  // x̂
        const float g = dxn[j][e] * gw[j][e];
        s1 += g;
        s2 += g * xv[j][e];
      }
    s1 = quad_sum(s1) / Kin;
    s2 = quad_sum(s2) / Kin;
    if (dlnw) {
      colsum_partial<NCH>(dxn, sPart + 4 * KP, KP);
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) gw[j][e] = rs * (dxn[j][e] * gw[j][e] - s1 - xv[j][e] * s2);  // dX (LN part)
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) dxn[j][e] *= xv[j][e];
      colsum_partial<NCH>(dxn, sPart, KP);
    } else {
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) gw[j][e] = rs * (dxn[j][e] * gw[j][e] - s1 - xv[j][e] * s2);
    }
  } else {
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) gw[j][e] = dxn[j][e];
  }
  if (dres) {
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) gw[j][e] += dr[j][e];
  }
  if (dX && own_rows) row_store<NCH>(gw, dX, dx_rs, gr, R, Kin, kvec && (dx_rs & 7) == 0 && aligned16(dX));
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) dxo[j][e] = gw[j][e];
  if (lnw && dlnw && own_rows) {
    lds_sync();
    colsum_flush(sPart, KP, rep(dlnw, vrs, slab), Kin, slab);
    colsum_flush(sPart + 4 * KP, KP, rep(dlnb, vrs, slab), Kin, slab);
  }
}

template <typename TG, typename TX, int NCH, bool AV>
__global__ __launch_bounds__(256) void ln_linear_bwd_kernel(
    const TG* __restrict__ G, int g_rs, int N, const uint16_t* __restrict__ W, int w_rs, int Kin,
    const TX* __restrict__ X,
    int x_rs, const float* __restrict__ mean, const float* __restrict__ rstd, const float* __restrict__ lnw,
    const float* __restrict__ lnb, const float* __restrict__ dres, int dres_rs, float* __restrict__ dX, int dx_rs,
    float* __restrict__ dlnw, float* __restrict__ dlnb, float* __restrict__ dW, float* __restrict__ db, int vrs,
    int wrs, int slab, int R, PeSplit ps, SlabJob job, int vf) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  if ((int)blockIdx.x >= (R + 63) / 64) {  // appended workgroups: the previous kernel's slab job
    {  // the appended job workgroups span every grid row: block (x − tiles)·gridDim.y + y
      const int jb = (int)(blockIdx.x - (R + 63) / 64) * (int)gridDim.y + (int)blockIdx.y;
      if (jb < job.nblk) slab_reduce_block(job, jb, reinterpret_cast<float4*>(smem));
    }
    return;
  }
  float dxo[NCH][8];
  ln_linear_bwd_body<TG, TX, NCH, AV>(G, g_rs, N, W, w_rs, Kin, X, x_rs, mean, rstd, lnw, lnb, dres, dres_rs, dX, dx_rs,
                                  dlnw, dlnb, dW, db, vrs, wrs, slab, R, ps, smem, dxo, (int)blockIdx.y,
                                  (int)gridDim.y, vf);
}

// ------------------------------------------------------------------------------------
// cross-layer fusion inside a self-attention block, backward (layer l+1 → l, both row-local):
// LN1+QKV backward of layer l+1 (dX_{l+1} = LN1_bwd(dQKV·W) + dY_{l+1}) is dZ_l, which the
// post-attention backward of layer l consumes from registers on the same tile: dZ never
// touches memory, one launch and one phase-0 latency fewer per boundary.  Both halves store
// their parameter-gradient partials into ONE slab row per tile (12 segments).  C ≤ 64 (the
// two halves' LDS must coexist: ≈117 KB at C = 64).
// ------------------------------------------------------------------------------------
template <int C, bool AV, int NQ = 3>
__global__ __launch_bounds__(256) void ln_linear_post_attn_bwd_kernel(
    const float* __restrict__ G, const uint16_t* __restrict__ Wq, const float* __restrict__ X,
    const float* __restrict__ mean1, const float* __restrict__ rstd1, const float* __restrict__ lnw,
    const float* __restrict__ lnb, const float* __restrict__ dres, float* __restrict__ dlnw, float* __restrict__ dlnb,
    float* __restrict__ dWq, float* __restrict__ dbq, const float* __restrict__ Ysave, const float* __restrict__ mean2,
    const float* __restrict__ rstd2, const uint16_t* __restrict__ U, const uint16_t* __restrict__ O,
    const uint16_t* __restrict__ Wo, const uint16_t* __restrict__ W1, const uint16_t* __restrict__ W2,
    const float* __restrict__ g2, const float* __restrict__ be2, float* __restrict__ dY, uint16_t* __restrict__ dO,
    float* __restrict__ delta, int H, PostAttnGrads gr_out, int R, SlabJob job, DropCfg dr) {
  constexpr int NCH = C / 32, nq = NQ * C;  // NQ·C: rows of Wq (3C packed QKV, C a query projection)
  constexpr int SM = ln_linear_bwd_smem<NCH>() > post_attn_bwd_smem<C>() ? ln_linear_bwd_smem<NCH>()
                                                                          : post_attn_bwd_smem<C>();
  // ONE buffer for both halves (used one after the other): ≈69 KB at C = 64, two workgroups per
  // CU, so the appended slab-job workgroups run beside the tiles instead of after them
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM];
  if (blockIdx.y == 0) zero_span_block(job);
  if ((int)blockIdx.x >= (R + 63) / 64) {  // appended workgroups: the previous kernel's slab job
    {  // the appended job workgroups span every grid row: block (x − tiles)·gridDim.y + y
      const int jb = (int)(blockIdx.x - (R + 63) / 64) * (int)gridDim.y + (int)blockIdx.y;
      if (jb < job.nblk) slab_reduce_block(job, jb, reinterpret_cast<float4*>(smem));
    }
    return;
  }
  const int part = (int)blockIdx.y, nparts = (int)gridDim.y;  // workgroups per tile (split_tiles)
  float dz[NCH][8];
  ln_linear_bwd_body<float, float, NCH, AV>(G, nq, nq, Wq, C, C, X, C, mean1, rstd1, lnw, lnb, dres, C, nullptr, C,
                                        dlnw, dlnb, dWq, dbq, gr_out.vrs, gr_out.vrs, gr_out.slab, R, PeSplit{},
                                        reinterpret_cast<uint16_t*>(smem), dz, part, nparts);
  lds_sync();  // the ln_linear half's LDS traffic is done before the post-attention half reuses it
  post_attn_bwd_body<C, AV>(dz, Ysave, mean2, rstd2, U, O, Wo, W1, W2, g2, be2, dY, dO, delta, H, gr_out, R, dr, smem,
                            part, nparts);
}

// ------------------------------------------------------------------------------------
// tall weight gradient: dW[n][k] += Σ_rows G[r][n] · A'[r][k], db[n] += Σ_rows G[r][n]
// A' = A | LN(A) | GELU(A) recomputed on load (A may be a Fourier-PE split input).
// grid (N / 64, row splits); each workgroup streams its row range in 64-row tiles with the
// next tile register-prefetched, accumulates in MFMA registers and adds its partial once —
// the form for row counts (≥ 10⁵: image K/V projections) where per-tile atomics would cost
// more than the GEMM.
// ------------------------------------------------------------------------------------
template <typename TG, typename TA, int NCH>
__global__ __launch_bounds__(256) void wgrad_kernel(const TG* __restrict__ G, int g_rs, int N, const TA* __restrict__ A,
                                                    int a_rs, int Kin, int amode, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, const float* __restrict__ lnw,
                                                    const float* __restrict__ lnb, int R, int rows_per_split,
                                                    float* __restrict__ dW, float* __restrict__ db, int vrs, int wrs,
                                                    PeSplit ps) {
  constexpr int KP = 32 * NCH, LDA = KP + 8, LDG = 64 + 8, MAXT = 3;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* sG = smem;                                // [64 rows][64 n]
  uint16_t* sA = sG + 64 * LDG;                       // [64 rows][KP]
  float* sAff = reinterpret_cast<float*>(sA + 64 * LDA);  // [2][KP] LN affine
  float* sPb = sAff + 2 * KP;                         // [4][64] bias partials
  const int n0 = blockIdx.x * 64, s = blockIdx.y, l = lane_id(), w = wave_id();
  const int r_begin = s * rows_per_split, r_end = min(R, r_begin + rows_per_split);
  const bool gvec = (N & 7) == 0 && (g_rs & 7) == 0 && aligned16(G);
  const bool avec = (Kin & 7) == 0 && (a_rs & 7) == 0 && aligned16(A);
  for (int k = threadIdx.x; k < KP; k += blockDim.x) {
    sAff[k] = (amode == 1 && k < Kin) ? lnw[k] : 0.f;
    sAff[KP + k] = (amode == 1 && k < Kin) ? lnb[k] : 0.f;
  }
  f32x16 acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = f32x16{};
  float cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = 0.f;
  float gv[2][8], av[NCH][8], mu = 0.f, rs = 1.f;
  auto fetch = [&](int r0) {
    g_fetch<TG>(gv, G, g_rs, r0, r_end, n0, N, gvec);
    const int gr = r0 + rp_row();
    row_load_x<NCH>(av, A, a_rs, gr, r_end, Kin, avec, ps);
    if (amode == 1 && gr < r_end) { mu = mean[gr]; rs = rstd[gr]; }
  };
  if (r_begin < r_end) fetch(r_begin);
  for (int r0 = r_begin; r0 < r_end; r0 += 64) {
    lds_sync();  // previous tile's MFMAs done with sG / sA
    g_store(gv, sG, LDG);
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[e] += gv[0][e] + gv[1][e];
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = rp_col(j) + e;
        float v = av[j][e];
        if (amode == 1) v = c < Kin ? (v - mu) * rs * sAff[c] + sAff[KP + c] : 0.f;
        else if (amode == 2) v = gelu_f(v);
        av[j][e] = v;
      }
    lds_row_write_bf16<NCH>(sA, LDA, av);
    lds_sync();
    if (r0 + 64 < r_end) fetch(r0 + 64);
    tile_gemm<MAXT, false, false>(sG, LDG, sA, LDA, 64, KP, 64, acc);
  }
  float* dWr = rep(dW, wrs, 0);
  for_acc<MAXT>(64, KP, [&](int t, int m, int n, int i) {
    const int gn = n0 + m;
    if (gn < N && n < Kin) atomicAdd(dWr + (long long)gn * Kin + n, acc[t][i]);
  });
  if (db) {  // column sums: lanes ≡ l (mod 8) share a column group
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = xor32_sum(xor16_sum(cs[e] + dpp<0x128>(cs[e])));
      if (l < 8) sPb[w * 64 + 8 * l + e] = v;
    }
    lds_sync();
    if (threadIdx.x < 64 && n0 + (int)threadIdx.x < N) {
      const int t = threadIdx.x;
      atomicAdd(rep(db, vrs, 0) + n0 + t, sPb[t] + sPb[64 + t] + sPb[128 + t] + sPb[192 + t]);
    }
  }
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
// kernels whose dynamic LDS can exceed 64 KiB: raise the per-function limit once (gfx950: 160 KiB/CU)
static void set_smem_once(const void* fn) {
  static const void* done[256] = {nullptr};
  for (auto& d : done) {
    if (d == fn) return;
    if (d == nullptr) {
      (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      d = fn;
      return;
    }
  }
}

// row-pass chunk count for a K-wide row: K ≤ 32·NCH, NCH ∈ {1, 2, 4, 5, 8}
// host side of the AV template flag: every pointer 16-B aligned (nullptr allowed), every row
// stride / width a multiple of 8 elements
static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
// register-resident chain kernels (CL layout, chain.hip) for the C = 64, H = 4 shapes; the LDS row-pass kernels otherwise
bool sa_layer_fwd_chain_launch(const uint16_t* QKV, int N, float scale_log2, uint16_t* O, float* LSE, const float* X,
                               const uint16_t* Wo, const float* bo, const float* g2, const float* be2, float eps,
                               const uint16_t* W1, const float* b1, const uint16_t* W2, const float* b2, float* Z,
                               float* Ysave, float* mean2, float* rstd2, uint16_t* Usave, int R, const float* lnw,
                               const float* lnb, const uint16_t* Wq, const float* bq, uint16_t* QKVn, float* mean1,
                               float* rstd1, const DropCfg& dr, int nq, hipStream_t st);
bool ln_linear_post_attn_bwd_chain_launch(const void* G, bool g_bf16, const uint16_t* Wq, const float* X, const float* mean1,
                                          const float* rstd1, const float* lnw, const float* lnb, const float* dres,
                                          float* dlnw, float* dlnb, float* dWq, float* dbq, const float* Ysave,
                                          const float* mean2, const float* rstd2, const uint16_t* U, const uint16_t* O,
                                          const uint16_t* Wo, const uint16_t* W1, const uint16_t* W2, const float* g2,
                                          const float* be2, float* dY, uint16_t* dO, float* delta,
                                          const PostAttnGrads& grads, int R, const SlabJob& job, const DropCfg& dr,
                                          int nq, const uint16_t* att_qkv, const float* att_lse, uint16_t* att_out,
                                          float att_scale, hipStream_t st);
static bool av_ok(std::initializer_list<const void*> ptrs, std::initializer_list<long long> widths) {
  for (const void* p : ptrs)
    if (!al16(p)) return false;
  for (long long w : widths)
    if (w & 7) return false;
  return true;
}

// kVecG / kVecW / kVecLn for the operands of an AV = false launch that still meet their
// vector-load preconditions (G may be null: a forward)
static int vec_flags(const void* G, int g_rs, int N, const void* W, int w_rs, int Kin, const float* lnw,
                     const float* lnb) {
  int vf = 0;
  if (G && al16(G) && !(g_rs & 7) && !(N & 7)) vf |= kVecG;
  if (al16(W) && !(w_rs & 7) && w_rs >= Kin) vf |= kVecW;
  if (lnw && al16(lnw) && al16(lnb)) vf |= kVecLn;
  return vf;
}

static int pick_nch(int K) {
  const int n = (K + 31) / 32;
  return n <= 2 ? n : n <= 4 ? 4 : n <= 5 ? 5 : 8;
}

template <typename TI, typename TO, int NCH>
static void ln_linear_fwd_t(const void* X, int x_rs, int R, int Kin, const float* lnw, const float* lnb, float eps,
                            const uint16_t* W, int w_rs, const float* bias, int N, int act, const float* res, int res_rs,
                            void* Y, int y_rs, float* mean, float* rstd, const PeSplit& ps, hipStream_t st) {
  constexpr int KP = 32 * NCH;
  const size_t smem = ln_linear_fwd_smem<NCH>();
  const bool av = av_ok({X, W, lnw, lnb}, {Kin, x_rs, w_rs});
  const int vf = av ? 0 : vec_flags(nullptr, 0, 0, W, w_rs, Kin, lnw, lnb);
  auto fn = av ? ln_linear_fwd_kernel<TI, TO, NCH, true> : ln_linear_fwd_kernel<TI, TO, NCH, false>;
  set_smem_once((const void*)fn);
  // few tiles: several workgroups per tile, each forming every split_tiles(R)-th 64-column chunk
  hipLaunchKernelGGL(fn, dim3((R + 63) / 64, split_tiles(R)), dim3(256), smem, st, (const TI*)X, x_rs, R, Kin, lnw, lnb,
                     eps, W, w_rs, bias, N, act, res, res_rs, (TO*)Y, y_rs, mean, rstd, ps, vf);
}

template <typename TI, typename TO>
static void ln_linear_fwd_n(int nch, const void* X, int x_rs, int R, int Kin, const float* lnw, const float* lnb,
                            float eps, const uint16_t* W, int w_rs, const float* bias, int N, int act, const float* res,
                            int res_rs, void* Y, int y_rs, float* mean, float* rstd, const PeSplit& ps,
                            hipStream_t st) {
#define LNF(K) \
  ln_linear_fwd_t<TI, TO, K>(X, x_rs, R, Kin, lnw, lnb, eps, W, w_rs, bias, N, act, res, res_rs, Y, y_rs, mean, rstd, ps, st)
  switch (nch) {
    case 1: LNF(1); break;
    case 2: LNF(2); break;
    case 4: LNF(4); break;
    case 5: LNF(5); break;
    default: LNF(8); break;
  }
#undef LNF
}

void ln_linear_fwd_launch(const void* X, bool x_bf16, int x_rs, int R, int Kin, const float* lnw, const float* lnb,
                          float eps, const uint16_t* W, int w_rs, const float* bias, int N, int act, const float* res,
                          int res_rs, void* Y, bool y_bf16, int y_rs, float* mean, float* rstd, const float* pe, int pe_rs,
                          int pe_rows, int npix, const long long* pe_idx, hipStream_t st) {
  const int nch = pick_nch(Kin);
  const PeSplit ps{pe, pe_rs, pe_rows, npix, pe_idx};
#define LNL(TI, TO) \
  ln_linear_fwd_n<TI, TO>(nch, X, x_rs, R, Kin, lnw, lnb, eps, W, w_rs, bias, N, act, res, res_rs, Y, y_rs, mean, rstd, ps, st)
  if (x_bf16 && y_bf16) LNL(uint16_t, uint16_t);
  else if (x_bf16) LNL(uint16_t, float);
  else if (y_bf16) LNL(float, uint16_t);
  else LNL(float, float);
#undef LNL
}

void post_attn_fwd_launch(int C, const uint16_t* O, const float* X, const uint16_t* Wo, const float* bo,
                          const float* g2, const float* be2, float eps, const uint16_t* W1, const float* b1,
                          const uint16_t* W2, const float* b2, float* Z, float* Ysave, float* mean2, float* rstd2,
                          uint16_t* Usave, int R, int Rx, const DropCfg& dr, hipStream_t st) {
  const bool av = av_ok({O, X, Wo, W1, W2, Z, Ysave, Usave}, {});
  dim3 grid((R + 63) / 64);
#define PAF(CC)                                                                                                     \
  if (av) hipLaunchKernelGGL((post_attn_fwd_kernel<CC, true>), grid, dim3(256), 0, st, O, X, Wo, bo, g2, be2, eps, \
                             W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, Rx, dr);                         \
  else hipLaunchKernelGGL((post_attn_fwd_kernel<CC, false>), grid, dim3(256), 0, st, O, X, Wo, bo, g2, be2, eps,   \
                          W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, Rx, dr)
  if (C == 64) PAF(64);
  else if (C == 128) PAF(128);
  else if (C == 32) PAF(32);
#undef PAF
}

void post_attn_ln_linear_fwd_launch(int C, const uint16_t* O, const float* X, const uint16_t* Wo, const float* bo,
                                    const float* g2, const float* be2, float eps, const uint16_t* W1, const float* b1,
                                    const uint16_t* W2, const float* b2, float* Z, float* Ysave, float* mean2,
                                    float* rstd2, uint16_t* Usave, int R, int Rx, const float* lnw, const float* lnb,
                                    const uint16_t* Wq, const float* bq, uint16_t* QKV, float* mean1, float* rstd1,
                                    const DropCfg& dr, hipStream_t st) {
  const bool av = av_ok({O, X, Wo, W1, W2, Z, Ysave, Usave, Wq, lnw, lnb, QKV}, {});
  dim3 grid((R + 63) / 64, split_tiles(R));
#define PLF(CC)                                                                                                  \
  if (av) hipLaunchKernelGGL((post_attn_ln_linear_fwd_kernel<CC, true>), grid, dim3(256), 0, st, O, X, Wo, bo, g2, \
                             be2, eps, W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, Rx, lnw, lnb, Wq, bq, QKV,  \
                             mean1, rstd1, dr);                                                                    \
  else hipLaunchKernelGGL((post_attn_ln_linear_fwd_kernel<CC, false>), grid, dim3(256), 0, st, O, X, Wo, bo, g2,     \
                          be2, eps, W1, b1, W2, b2, Z, Ysave, mean2, rstd2, Usave, R, Rx, lnw, lnb, Wq, bq, QKV,     \
                          mean1, rstd1, dr)
  if (C == 64) PLF(64);
  else if (C == 128) PLF(128);
  else if (C == 32) PLF(32);
#undef PLF
}

// fused self-attention layer forward (C = 64, H = 4): the chain kernel (chain.hip
// sa_layer_fwd_chain8_kernel); false (nothing launched) when the operands do not qualify (every
// pointer 16-byte aligned, N <= 512) — the binding turns that into an error
bool sa_layer_fwd_launch(const uint16_t* QKV, int N, float scale_log2, uint16_t* O, float* LSE, const float* X,
                         const uint16_t* Wo, const float* bo, const float* g2, const float* be2, float eps,
                         const uint16_t* W1, const float* b1, const uint16_t* W2, const float* b2, float* Z,
                         float* Ysave, float* mean2, float* rstd2, uint16_t* Usave, int R, const float* lnw,
                         const float* lnb, const uint16_t* Wq, const float* bq, uint16_t* QKVn, float* mean1,
                         float* rstd1, const DropCfg& dr, int nq, hipStream_t st) {
  const bool av = av_ok({QKV, O, X, Wo, W1, W2, Z, Ysave, Usave, Wq, lnw, lnb, QKVn}, {});
  return av && sa_layer_fwd_chain_launch(QKV, N, scale_log2, O, LSE, X, Wo, bo, g2, be2, eps, W1, b1, W2, b2, Z, Ysave,
                                         mean2, rstd2, Usave, R, lnw, lnb, Wq, bq, QKVn, mean1, rstd1, dr, nq, st);
}

void post_attn_bwd_launch(int C, const float* dZ, const float* Ysave, const float* mean2, const float* rstd2,
                          const uint16_t* U, const uint16_t* O, const uint16_t* Wo, const uint16_t* W1,
                          const uint16_t* W2, const float* g2, const float* be2, float* dY, uint16_t* dO,
                          float* delta, int H, const PostAttnGrads& grads, int R, const SlabJob& job, const DropCfg& dr,
                          hipStream_t st) {
  const int spl = split_tiles(R);
  dim3 grid((R + 63) / 64 + (job.slab ? (job.nblk + spl - 1) / spl : 0), spl);
  const bool av = av_ok({dZ, Ysave, U, O, Wo, W1, W2, dY, dO}, {});
#define PAB(CC)                                                                                                  \
  if (av) hipLaunchKernelGGL((post_attn_bwd_kernel<CC, true>), grid, dim3(256), 0, st, dZ, Ysave, mean2, rstd2, U, \
                             O, Wo, W1, W2, g2, be2, dY, dO, delta, H, grads, R, job, dr);                        \
  else hipLaunchKernelGGL((post_attn_bwd_kernel<CC, false>), grid, dim3(256), 0, st, dZ, Ysave, mean2, rstd2, U, O,  \
                          Wo, W1, W2, g2, be2, dY, dO, delta, H, grads, R, job, dr)
  if (C == 64) PAB(64);
  else if (C == 128) PAB(128);
  else if (C == 32) PAB(32);
#undef PAB
}

// G: fp32, or (g_bf16) bf16 — taken by the chain-layout kernel only; returns false (nothing
// launched) for a bf16 G the chain kernel cannot take (the caller converts it to fp32)
bool ln_linear_post_attn_bwd_launch(int C, const void* Gv, bool g_bf16, const uint16_t* Wq, const float* X, const float* mean1,
                                    const float* rstd1, const float* lnw, const float* lnb, const float* dres,
                                    float* dlnw, float* dlnb, float* dWq, float* dbq, const float* Ysave,
                                    const float* mean2, const float* rstd2, const uint16_t* U, const uint16_t* O,
                                    const uint16_t* Wo, const uint16_t* W1, const uint16_t* W2, const float* g2,
                                    const float* be2, float* dY, uint16_t* dO, float* delta, int H,
                                    const PostAttnGrads& grads, int R, const SlabJob& job, const DropCfg& dr,
                                    int nq, const uint16_t* att_qkv, const float* att_lse, uint16_t* att_out,
                                    float att_scale, hipStream_t st) {
  dim3 grid((R + 63) / 64 + (job.slab ? job.nblk : 0));
  const float* G = static_cast<const float*>(Gv);
  const bool av = av_ok({Gv, Wq, X, lnw, lnb, dres, Ysave, U, O, Wo, W1, W2, dY, dO}, {});
  const bool att = att_out != nullptr;  // the fused attention backward (chain kernel only)
  if (att && !(av && al16(att_qkv) && al16(att_out) && al16(att_lse))) return false;
  if (av && C == 64 && H == 4 && grads.slab && (R % 64) == 0 &&
      ln_linear_post_attn_bwd_chain_launch(Gv, g_bf16, Wq, X, mean1, rstd1, lnw, lnb, dres, dlnw, dlnb, dWq, dbq, Ysave,
                                           mean2, rstd2, U, O, Wo, W1, W2, g2, be2, dY, dO, delta, grads, R, job, dr, nq,
                                           att_qkv, att_lse, att_out, att_scale, st))
    return true;
  if (g_bf16 || att) return false;
  grid.y = split_tiles(R);
  grid.x = (R + 63) / 64 + (job.slab ? (job.nblk + (int)grid.y - 1) / (int)grid.y : 0);
#define LPB(CC, NQ)                                                                                               \
  if (av) hipLaunchKernelGGL((ln_linear_post_attn_bwd_kernel<CC, true, NQ>), grid, dim3(256), 0, st, G, Wq, X, mean1, \
                             rstd1, lnw, lnb, dres, dlnw, dlnb, dWq, dbq, Ysave, mean2, rstd2, U, O, Wo, W1, W2, g2, \
                             be2, dY, dO, delta, H, grads, R, job, dr);                                            \
  else hipLaunchKernelGGL((ln_linear_post_attn_bwd_kernel<CC, false, NQ>), grid, dim3(256), 0, st, G, Wq, X, mean1,  \
                          rstd1, lnw, lnb, dres, dlnw, dlnb, dWq, dbq, Ysave, mean2, rstd2, U, O, Wo, W1, W2, g2,    \
                          be2, dY, dO, delta, H, grads, R, job, dr)
  if (C == 64 && nq == 3 * C) { LPB(64, 3); }
  else if (C == 64) { LPB(64, 1); }
  else if (C == 128 && nq == 3 * C) { LPB(128, 3); }
  else if (C == 128) { LPB(128, 1); }
  else if (nq == 3 * C) { LPB(32, 3); }
  else { LPB(32, 1); }
#undef LPB
  return true;
}

template <typename TG, typename TX, int NCH>
static void ln_linear_bwd_t(const void* G, int g_rs, int N, const uint16_t* W, int w_rs, int Kin, const void* X, int x_rs,
                            const float* mean, const float* rstd, const float* lnw, const float* lnb, const float* dres,
                            int dres_rs, float* dX, int dx_rs, float* dlnw, float* dlnb, float* dW, float* db, int vrs,
                            int wrs, int slab, int R, const PeSplit& ps, const SlabJob& job, hipStream_t st) {
  constexpr int KP = 32 * NCH;
  const size_t smem = ln_linear_bwd_smem<NCH>();
  const bool av = av_ok({G, W, X, lnw, lnb, dres}, {N, g_rs, w_rs, Kin, x_rs, dres ? dres_rs : 0});
  const int vf = av ? 0 : vec_flags(G, g_rs, N, W, w_rs, Kin, lnw, lnb);
  auto fn = av ? ln_linear_bwd_kernel<TG, TX, NCH, true> : ln_linear_bwd_kernel<TG, TX, NCH, false>;
  set_smem_once((const void*)fn);
  // + the appended slab-job workgroups; few tiles: several workgroups per tile (split_tiles)
  const int spl = split_tiles(R);
  const dim3 grid((R + 63) / 64 + (job.slab ? (job.nblk + spl - 1) / spl : 0), spl);
  hipLaunchKernelGGL(fn, grid, dim3(256), smem, st, (const TG*)G, g_rs, N, W, w_rs, Kin, (const TX*)X, x_rs,
                     mean, rstd, lnw, lnb, dres, dres_rs, dX, dx_rs, dlnw, dlnb, dW, db, vrs, wrs, slab, R, ps, job, vf);
}

template <typename TG, typename TX>
static void ln_linear_bwd_n(int nch, const void* G, int g_rs, int N, const uint16_t* W, int w_rs, int Kin, const void* X,
                            int x_rs, const float* mean, const float* rstd, const float* lnw, const float* lnb,
                            const float* dres, int dres_rs, float* dX, int dx_rs, float* dlnw, float* dlnb, float* dW,
                            float* db, int vrs, int wrs, int slab, int R, const PeSplit& ps, const SlabJob& job,
                            hipStream_t st) {
#define LNB(K)                                                                                                    \
  ln_linear_bwd_t<TG, TX, K>(G, g_rs, N, W, w_rs, Kin, X, x_rs, mean, rstd, lnw, lnb, dres, dres_rs, dX, dx_rs, dlnw, \
                             dlnb, dW, db, vrs, wrs, slab, R, ps, job, st)
  switch (nch) {
    case 1: LNB(1); break;
    case 2: LNB(2); break;
    case 4: LNB(4); break;
    default: LNB(5); break;
  }
#undef LNB
}

void ln_linear_bwd_launch(const void* G, bool g_bf16, int g_rs, int N, const uint16_t* W, int w_rs, int Kin, const void* X,
                          bool x_bf16, int x_rs, const float* mean, const float* rstd, const float* lnw,
                          const float* lnb, const float* dres, int dres_rs, float* dX, int dx_rs, float* dlnw,
                          float* dlnb, float* dW, float* db, int vrs, int wrs, int slab, int R, const float* pe,
                          int pe_rs, int pe_rows, int npix, const long long* pe_idx, const SlabJob& job, hipStream_t st) {
  const int nch = pick_nch(Kin);  // Kin ≤ 160 → ≤ 5
  const PeSplit ps{pe, pe_rs, pe_rows, npix, pe_idx};
#define LDG(TG, TX)                                                                                           \
  ln_linear_bwd_n<TG, TX>(nch, G, g_rs, N, W, w_rs, Kin, X, x_rs, mean, rstd, lnw, lnb, dres, dres_rs, dX, dx_rs, \
                          dlnw, dlnb, dW, db, vrs, wrs, slab, R, ps, job, st)
  if (g_bf16 && x_bf16) LDG(uint16_t, uint16_t);
  else if (g_bf16) LDG(uint16_t, float);
  else if (x_bf16) LDG(float, uint16_t);
  else LDG(float, float);
#undef LDG
}

template <typename TG, typename TA, int NCH>
static void wgrad_t(const void* G, int g_rs, int N, const void* A, int a_rs, int Kin, int amode, const float* mean,
                    const float* rstd, const float* lnw, const float* lnb, int R, int rps, float* dW, float* db,
                    int vrs, int wrs, const PeSplit& ps, hipStream_t st) {
  constexpr int KP = 32 * NCH;
  const size_t smem = (64 * (64 + 8) + 64 * (KP + 8)) * 2 + 2 * KP * 4 + 4 * 64 * 4;
  auto fn = wgrad_kernel<TG, TA, NCH>;
  set_smem_once((const void*)fn);
  dim3 grid((N + 63) / 64, (R + rps - 1) / rps);
  hipLaunchKernelGGL(fn, grid, dim3(256), smem, st, (const TG*)G, g_rs, N, (const TA*)A, a_rs, Kin, amode, mean, rstd,
                     lnw, lnb, R, rps, dW, db, vrs, wrs, ps);
}

template <typename TG, typename TA>
static void wgrad_n(int nch, const void* G, int g_rs, int N, const void* A, int a_rs, int Kin, int amode,
                    const float* mean, const float* rstd, const float* lnw, const float* lnb, int R, int rps, float* dW,
                    float* db, int vrs, int wrs, const PeSplit& ps, hipStream_t st) {
#define WGN(K) wgrad_t<TG, TA, K>(G, g_rs, N, A, a_rs, Kin, amode, mean, rstd, lnw, lnb, R, rps, dW, db, vrs, wrs, ps, st)
  switch (nch) {
    case 1: WGN(1); break;
    case 2: WGN(2); break;
    case 4: WGN(4); break;
    default: WGN(5); break;
  }
#undef WGN
}

// rows_per_wg ≤ 0: pick the split so that the launch has ≈ 512 workgroups
void wgrad_launch(const void* G, bool g_bf16, int g_rs, int N, const void* A, bool a_bf16, int a_rs, int Kin,
                  int amode, const float* mean, const float* rstd, const float* lnw, const float* lnb, int R,
                  int rows_per_wg, float* dW, float* db, int vrs, int wrs, const float* pe, int pe_rs, int pe_rows,
                  int npix, const long long* pe_idx, hipStream_t st) {
  const int nblk = (N + 63) / 64;
  int rps = rows_per_wg;
  if (rps <= 0) {
    const int splits = (512 + nblk - 1) / nblk;
    rps = (R + splits - 1) / splits;
  }
  rps = round_up(rps < 64 ? 64 : rps, 64);
  const PeSplit ps{pe, pe_rs, pe_rows, npix, pe_idx};
  const int nch = pick_nch(Kin);
#define WG(TG, TA) wgrad_n<TG, TA>(nch, G, g_rs, N, A, a_rs, Kin, amode, mean, rstd, lnw, lnb, R, rps, dW, db, vrs, wrs, ps, st)
  if (g_bf16 && a_bf16) WG(uint16_t, uint16_t);
  else if (g_bf16) WG(uint16_t, float);
  else if (a_bf16) WG(float, uint16_t);
  else WG(float, float);
#undef WG
}

}  // namespace pio

namespace pio {
unsigned check_errors_rowgemm(bool reset) { return pio_read_errors(reset); }
}  // namespace pio
