// Shared device helpers for the Perceiver IO CDNA4 (gfx950) kernels.
//
// Conventions (all kernels):
//   * wave = 64 lanes; blocks are multiples of 64 threads.
//   * matrix products use v_mfma_f32_32x32x16_bf16 (fp32 accumulate).
//     operand lane map (lane l, r = l & 31, h = l >> 5):
//        A[row r][k = 8h + j], B[k = 8h + j][col r], j = 0..7
//     accumulator map: col = l & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * h.
//   * an operand tile lives in LDS either "k-contiguous" (row-major with the
//     contraction index innermost → one ds_read_b128 per fragment) or
//     "k-strided" (contraction index = LDS row → two ds_read_b64_tr_b16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pio {

// ---- checked builds (python -m perceiver_io_amd.csrc.build --check → _C_check) ------------
// Index operands that come from user data (token ids, class labels, gather rows) are validated
// on the device: a violation sets a bit in this translation unit's error word (read and cleared
// by ext.check_errors()) and the access is clamped / skipped instead of faulting.  Release
// builds compile the checks out.
#ifndef PIO_CHECKS
#define PIO_CHECKS 0
#endif
enum : unsigned { kErrEmbedId = 1u, kErrGatherRow = 2u, kErrLabel = 4u, kErrPeIndex = 8u };
static __device__ unsigned pio_errors;
__device__ __forceinline__ void pio_flag(unsigned bit) {
#if PIO_CHECKS
  atomicOr(&pio_errors, bit);
#else
  (void)bit;
#endif
}
// this TU's error word (host side), optionally cleared
static inline unsigned pio_read_errors(bool reset) {
  unsigned h = 0;
  (void)hipMemcpyFromSymbol(&h, HIP_SYMBOL(pio_errors), sizeof(h), 0, hipMemcpyDeviceToHost);
  if (reset) {
    const unsigned z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(pio_errors), &z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  return h;
}

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ float bf2f(short v) { return bf2f((uint16_t)v); }

// round-to-nearest-even f32 -> bf16 (NaN stays NaN via the cast path hipcc lowers to v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<uint16_t*>(&b);
}
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// accumulator register -> row within the 32x32 tile
__device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// ---- LDS operand reads ------------------------------------------------------------
// k-contiguous: element (idx, k) at base[idx * ld + k]; fragment for tile origin (i0, k0)
__device__ __forceinline__ bf16x8 frag_kc(const uint16_t* lds, int ld, int i0, int k0) {
  const int l = lane_id();
  return *reinterpret_cast<const bf16x8*>(lds + (i0 + (l & 31)) * ld + k0 + 8 * (l >> 5));
}

// k-strided: element (idx, k) at base[k * ld + idx] — hardware transpose read.
// Lane group g = l>>4 covers idx i0 + 16*(g&1) + 0..15 and k rows k0 + 8*(g>>1) + 0..7.
__device__ __forceinline__ bf16x8 frag_ks(const uint16_t* lds, int ld, int i0, int k0) {
  const int l = lane_id();
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const uint16_t* base = lds + (k0 + 8 * (g >> 1) + q) * ld + i0 + 16 * (g & 1) + 4 * p;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + 4 * ld));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// A-operand read (attention backward: dV += Pᵀ·dO, dK += dSᵀ·Q) of V^T / dO^T / Q^T from an LDS tile stored [k][i] with the k order
// permuted to match an accumulator used as the other operand (see common.h).
__device__ __forceinline__ bf16x8 frag_ks_perm(const uint16_t* lds, int ld, int i0, int k0) {
  const int l = lane_id();
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const uint16_t* base = lds + (k0 + 4 * (g >> 1) + q) * ld + i0 + 16 * (g & 1) + 4 * p;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + 8 * ld));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// v_mfma_f32_16x16x32_bf16: lane l holds A[row l & 15][k = 8(l >> 4) + j], B[k = 8(l >> 4) + j][col l & 15];
// accumulator col = l & 15, row = 4(l >> 4) + reg
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// 16x16x32 operand from a k-strided LDS image (element (i, k) at base[k·ld + i]), natural k
__device__ __forceinline__ bf16x8 frag16_tr(const uint16_t* lds, int ld, int i0, int k0) {
  const int l = lane_id(), g = l >> 4, i = l & 15;
  const uint16_t* base = lds + (k0 + 8 * g + (i >> 2)) * ld + i0 + 4 * (i & 3);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(base + 4 * ld));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// pack accumulator registers 8s..8s+7 to a bf16 operand fragment
__device__ __forceinline__ bf16x8 pack_acc(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)f2bf(a[8 * s + j]);
  return r;
}

// ---- reductions (VALU only: DPP within 16-lane rows, gfx950 lane swaps across rows) --
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// v_permlane16_swap exchanges the odd 16-lane rows of its first operand with the even rows of
// its second, v_permlane32_swap the upper half of the first with the lower half of the second;
// with both operands = v the two registers end up holding v[l] and v[l ^ 16] (resp. v[l ^ 32])
// in some order.  Inline asm with two in/out operands: the instruction rewrites BOTH registers
// (with identical inputs the builtin lets the compiler merge them into one register, which
// swaps a register with itself).  s_nop 1 = the 2 wait states a VALU write of either operand
// needs before the swap reads it.
__device__ __forceinline__ void xor16_pair(float v, float& a, float& b) {
  a = v;
  b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void xor32_pair(float v, float& a, float& b) {
  a = v;
  b = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ float xor16_sum(float v) { float a, b; xor16_pair(v, a, b); return a + b; }
__device__ __forceinline__ float xor32_sum(float v) { float a, b; xor32_pair(v, a, b); return a + b; }
__device__ __forceinline__ float xor32_max(float v) { float a, b; xor32_pair(v, a, b); return fmaxf(a, b); }

// reductions over each 32-lane half (lanes l and l ^ 1..16)
__device__ __forceinline__ float half_sum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x124>(v);
  v += dpp<0x128>(v);
  return xor16_sum(v);
}
__device__ __forceinline__ float half_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x124>(v));
  v = fmaxf(v, dpp<0x128>(v));
  float a, b;
  xor16_pair(v, a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x124>(v);  // row_ror:4
  v += dpp<0x128>(v);  // row_ror:8
  return xor32_sum(xor16_sum(v));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x124>(v));
  v = fmaxf(v, dpp<0x128>(v));
  float a, b;
  xor16_pair(v, a, b);
  xor32_pair(fmaxf(a, b), a, b);
  return fmaxf(a, b);
}

// 2^x as one v_exp_f32 (no denormal-range fixup: results below 2^-126 flush to 0, -inf → 0)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// ---- XCD-aware workgroup order --------------------------------------------------------
// Workgroups are dealt round-robin over the 8 XCDs (observed placement; speed only, never
// correctness).  xcd_remap turns the dispatch-order id into a logical id such that
// consecutive logical ids share an XCD (and its L2) — bijective for any grid size.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}
// logical 3-D block index (x fastest) after the remap: the (x, y) blocks of one z are
// consecutive, i.e. all heads / key blocks of one batch element read their rows through one L2
struct Blk3 { int x, y, z; };
__device__ __forceinline__ Blk3 xcd_block3(int gz) {  // gz: the z extent of the remapped part of the grid
  const int gx = gridDim.x, gy = gridDim.y;
  const int nwg = gx * gy * gz;
  const int m = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), nwg);
  return Blk3{m % gx, (m / gx) % gy, m / (gx * gy)};
}
__device__ __forceinline__ Blk3 xcd_block3() { return xcd_block3(gridDim.z); }

// ---- phase timestamps (tools/trace only; compiled out unless PIO_TRACE is defined) ----
// PIO_TS(slot): lane 0 of every wave of workgroup (trace_bx, trace_by, trace_bz) records the
// shader clock into trace_buf[wave * 64 + slot]; slot 63 of every workgroup's wave 0 goes to
// trace_wg[2 * wg + {0, 1}] via PIO_WG_BEGIN / PIO_WG_END (dispatch timeline, on the 100 MHz
// s_memrealtime clock: the shader clocks of different XCDs are not aligned).
#ifdef PIO_TRACE
__device__ long long* trace_buf;
__device__ long long* trace_wg;
__device__ int trace_bx, trace_by, trace_bz;
#define PIO_TS(slot)                                                                                 \
  do {                                                                                               \
    if (blockIdx.x == (unsigned)trace_bx && blockIdx.y == (unsigned)trace_by &&                      \
        blockIdx.z == (unsigned)trace_bz && (threadIdx.x & 63) == 0)                                 \
      trace_buf[(threadIdx.x >> 6) * 64 + (slot)] = __builtin_amdgcn_s_memtime();                    \
  } while (0)
#define PIO_WG_MARK(which)                                                                           \
  do {                                                                                               \
    if (threadIdx.x == 0 && trace_wg)                                                                \
      trace_wg[2 * ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) + (which)] =     \
          __builtin_amdgcn_s_memrealtime();                                                          \
  } while (0)
#define PIO_WG_BEGIN() PIO_WG_MARK(0)
#define PIO_WG_END() PIO_WG_MARK(1)
#else
#define PIO_TS(slot) do {} while (0)
#define PIO_WG_BEGIN() do {} while (0)
#define PIO_WG_END() do {} while (0)
#endif

// ---- parameter-gradient slab reduction ----------------------------------------------
// A backward kernel in "slab" mode stores workgroup i's parameter-gradient partials into row
// i of an (S, P) fp32 slab (rowgemm.hip); a SlabJob sums the rows into the gradients:
// dst_j[k] += Σ_s slab[s][off_j + k] (P and every off_j multiples of 4).  The job runs as
// extra workgroups appended to the NEXT kernel of the backward chain (horizontal fusion: the
// latency-bound chain kernels leave most CU slots idle, and a separate node — or a side-stream
// branch, whose cross-queue hand-off costs 10–15 µs per fork in a replayed hipGraph — would sit
// on the critical path), or as a standalone launch at the end of the backward pass.
// Reduction block (x, y): 256 columns × slab rows [32y, 32y + 32); wave w sums rows w, w+4, …
// (all loads in flight), LDS combine, then wave w adds columns 64w..64w+63 with one
// contiguous 256-B no-return atomic instruction: S/32 adds per element in all.
constexpr int kMaxSlabSegs = 16;

// 32 bytes of zeros in global memory: the source of every out-of-range element of a fetch.  A
// load whose predicate is false reads here instead (an address select), so a phase's loads
// are straight-line code.  hipcc waits for a load at the first branch, phi copy or arithmetic
// that touches its result, and after a conditional load (even one skipped at run time) it can
// no longer count outstanding loads, so it falls back to vmcnt(0): one conditional load in a
// prefetch loop serialises the whole prefetch with the compute it was meant to overlap.
// (A writable __device__ array: a const one lands in the constant address space, and a select
// between it and a global pointer becomes a flat load, which also counts against lgkmcnt and
// so stalls every LDS wait behind the global loads.)  Never written.
static __device__ __attribute__((aligned(16))) float kZero32B[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup-scope fence and
// waits for every outstanding global load AND store of the thread (s_waitcnt vmcnt(0)), so a
// register prefetch issued before it, or a row store just before it, puts a full memory
// latency on the critical path at every LDS hand-off.  This barrier waits for LDS traffic only;
// global loads stay in flight until their registers are used (the compiler's own waits).
// Never use it where another thread of the workgroup reads global memory this thread wrote.
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct SlabJob {
  const float* slab;  // nullptr: no job
  int S, P, nbx, nblk;
  int det;            // deterministic mode: one block per column range sums ALL rows, plain add
  int n;
  float* dst[kMaxSlabSegs];
  int off[kMaxSlabSegs];
  int len[kMaxSlabSegs];
  // side job of the kernel that carries this struct: clear zero_n4 float4s at zero_p (the
  // accumulator of the NEXT kernel, e.g. the attention backward's atomic dQ), one slice per
  // workgroup — no separate fill launch on the chain
  float* zero_p;
  long long zero_n4;
};
// this workgroup's slice of a SlabJob zero span
__device__ __forceinline__ void zero_span_block(const SlabJob& j) {
  if (j.zero_p == nullptr) return;
  const long long nwg = gridDim.x, per = (j.zero_n4 + nwg - 1) / nwg;
  const long long z0 = (long long)blockIdx.x * per, z1 = z0 + per < j.zero_n4 ? z0 + per : j.zero_n4;
  for (long long i = z0 + threadIdx.x; i < z1; i += blockDim.x)
    reinterpret_cast<float4*>(j.zero_p)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}
// Column blocks of a SlabJob: kSlabColsPerBlock columns per workgroup (256 threads × 4).
// Non-deterministic mode: workgroup b sums rows [by·RB, (by + 1)·RB) of column block bx
// (b = by·nbx + bx, RB = ⌈S / (nblk / nbx)⌉, the host sizes nblk ≈ 128 workgroups) with
// every row's load in flight at once (16 per batch), and adds its 4 column sums per thread
// atomically — nblk / nbx partial sums per column.  A job carried by a one-workgroup-per-CU
// kernel (≈100 KB of LDS) runs in one round after the carrier's tiles.
// Deterministic mode: one workgroup per column block sums all S rows in a fixed order and
// adds once (single writer).
constexpr int kSlabColsPerBlock = 1024;
// blocks of the gradient sum-of-squares pass: one fp32 partial each (elementwise.hip sumsq_kernel)
constexpr int kSumsqBlocks = 512;
// part: ≥ 4 KiB of 16-B aligned LDS.  Deterministic mode runs on the first 256 threads of the
// carrier's workgroup (the others only join the barrier); the other mode splits the rows between
// the two halves of a 512-thread carrier.  NV: row loads in flight per thread (a one-workgroup-
// per-CU carrier has the registers for the whole share of its rows at once).
template <int NV = 16>
__device__ __forceinline__ void slab_reduce_block(const SlabJob& j, int b, float4* part) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int P = j.P;
  if (j.det) {  // fixed summation order, a single writer per element: bitwise reproducible
    const int cb = b * 256, c = cb + 4 * l;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < P && w < 4)
      for (int s = w; s < j.S; s += 4) {
        const float4 v = *reinterpret_cast<const float4*>(j.slab + (long long)s * P + c);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    if (w < 4) part[w * 64 + l] = acc;
    __syncthreads();
    if (w >= 4) return;
    const float* pf = reinterpret_cast<const float*>(part);
    const int k = 64 * w + l, col = cb + k;
    if (col >= P) return;
    const float sum = ((pf[k] + pf[256 + k]) + pf[512 + k]) + pf[768 + k];
    for (int q = 0; q < j.n; ++q) {
      const int lo = j.off[q];
      if (col >= lo && col < lo + j.len[q]) j.dst[q][col - lo] += sum;
    }
    return;
  }
  // a 512-thread carrier (the chain backward) splits the block's rows between its two halves:
  // twice the loads in flight per CU, the halves combined through LDS before the atomics
  const bool two = blockDim.x >= 512;
  const int t = threadIdx.x & 255, h = threadIdx.x >> 8;
  if (h > (two ? 1 : 0)) return;
  const int nsy = j.nblk / j.nbx, rb = (j.S + nsy - 1) / nsy;
  const int bx = b % j.nbx, by = b / j.nbx;
  const int c = bx * kSlabColsPerBlock + 4 * t;
  const int r0 = by * rb, r1 = min(j.S, r0 + rb), rm = two ? r0 + (r1 - r0 + 1) / 2 : r1;
  const int s0 = h ? rm : r0, s1 = h ? r1 : rm;
  const bool cin = c < P;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = s0; s < s1; s += NV) {
    float4 v[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {  // address selects: rows past s1 / columns past P read zeros
      const bool ok = cin && s + i < s1;
      v[i] = *reinterpret_cast<const float4*>(ok ? j.slab + (long long)(s + i) * P + c : kZero32B);
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      acc.x += v[i].x; acc.y += v[i].y; acc.z += v[i].z; acc.w += v[i].w;
    }
  }
  if (two) {
    if (h) part[t] = acc;
    __syncthreads();
    if (h) return;
    const float4 o = part[t];
    acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
  }
  if (!cin) return;
  const float a4[4] = {acc.x, acc.y, acc.z, acc.w};
  for (int q = 0; q < j.n; ++q) {
    const int lo = j.off[q], hi = lo + j.len[q];
    if (c + 4 <= lo || c >= hi) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (c + e >= lo && c + e < hi) atomicAdd(j.dst[q] + (c + e - lo), a4[e]);
  }
}

// fp32 gradient targets of the post-attention block (views of the flat gradient buffer).
// Two sinks for a workgroup's parameter-gradient partials:
//  * atomic (slab = 0): targets may be replicated: workgroup i adds into replica
//    i % kGradReplicas, vrs floats apart (vrs = 0: one copy), folded once per step;
//  * slab (slab = 1): workgroup i STORES its partials into row i of a (tiles, P) fp32 slab
//    (vrs = P floats per row).  Float atomics execute at the memory side at ≈1.3 TB/s
//    chip-wide, so 256 tiles × 50 KB of partials per kernel cost ≈10 µs of a ≈25 µs kernel;
//    plain stores cost ≈0.3 µs per CU, and the slab rows are summed by a SlabJob.
constexpr int kGradReplicas = 8;
struct PostAttnGrads {
  float *dWo, *dbo, *dg2, *dbe2, *dW1, *db1, *dW2, *db2;
  int vrs;
  int slab;
};
__device__ __forceinline__ float* rep(float* p, int vrs, int slab) {
  return p + (long long)(slab ? blockIdx.x : (blockIdx.x & (kGradReplicas - 1))) * vrs;
}
__device__ __forceinline__ void gadd(float* p, float v, int slab) {
  if (slab) *p = v;
  else atomicAdd(p, v);
}


// ---- GELU (erf form, nn.GELU default) ------------------------------------------------
// Branch-free: erf(|z|) = 1 − t·P(t)·exp(−z²), t = 1/(1 + 0.3275911·|z|) (Abramowitz & Stegun
// 7.1.26, |error| ≤ 1.5e-7), z = x/√2 — one v_rcp, one v_exp and five FMAs.  The device
// library's erff branches on |z| < 1 (both sides run when the lanes of a wave straddle it) and
// its expf adds a range reduction: ≈45 instructions per call against ≈12 here, and exp(−z²) is
// the Gaussian factor of the derivative too (gelu_pair: both for one exp).
__device__ __forceinline__ float gelu_cdf_e(float x, float& e) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  e = __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x);  // exp(−x²/2) = exp(−z²)
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float erf_abs = fmaf(-p * t, e, 1.f);
  return 0.5f + 0.5f * copysignf(erf_abs, x);  // Φ(x) = ½(1 + erf(x/√2))
}
__device__ __forceinline__ float gelu_f(float x) {
  float e;
  return x * gelu_cdf_e(x, e);
}
__device__ __forceinline__ float gelu_grad(float x) {
  float e;
  const float cdf = gelu_cdf_e(x, e);
  return fmaf(x * 0.39894228040143268f, e, cdf);  // Φ(x) + x·φ(x)
}
__device__ __forceinline__ void gelu_pair(float x, float& gelu, float& grad) {
  float e;
  const float cdf = gelu_cdf_e(x, e);
  gelu = x * cdf;
  grad = fmaf(x * 0.39894228040143268f, e, cdf);
}

// ---- counter-based RNG for dropout (regenerated in backward, no mask storage) -------
// hash3(a, b, c): a few rounds of a murmur-style mixer over (seed, stream, index); the text
// masking kernel (elementwise.hip) and ops/emulation.py use it as is
constexpr uint32_t kHashM1 = 0x85EBCA77u;
__device__ __forceinline__ uint32_t hash3_seed(uint32_t a, uint32_t b) { return a * 0x9E3779B1u ^ (b + 0x7F4A7C15u); }
__device__ __forceinline__ uint32_t hash3_mix(uint32_t h) {
  h ^= h >> 15; h *= 0x2C1B3C6Du;
  h ^= h >> 12; h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}
__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  return hash3_mix(hash3_seed(a, b) ^ c * kHashM1);
}
// dropout keep test (probability 1 − p, threshold p·2^32) of element c, called with
// hs = hash3_seed(seed, stream) and cm = c·kHashM1: the dropout kernels form cm as
// base·kHashM1 + offset·kHashM1 (mod 2^32, exact) with compile-time or wave-uniform offsets, so
// each element costs one full-rate add instead of a quarter-rate v_mul_lo_u32 — bit for bit
// hash3(seed, stream, c) >= thresh.  Each caller makes the base opaque (empty asm) inside its
// dropout branch: otherwise the compiler hoists the per-element multiplies (hundreds of
// quarter-rate v_mul_lo_u32) out of the loops and the branch into the kernel prologue, where
// they run even with dropout off.
__device__ __forceinline__ bool keep_elem_m(uint32_t hs, uint32_t cm, uint32_t thresh) {
  return hash3_mix(hs ^ cm) >= thresh;
}

// Dropout configuration of one fused call.  The 64-bit seed lives in DEVICE memory: it is
// drawn per forward call by torch's graph-safe generator (a 1-element randint on the step's
// stream), so a replayed hipGraph reads a fresh seed every step instead of a value frozen at
// capture time, and the backward regenerates the forward's masks from the same tensor.
// ``site`` separates the masks of one call: sub-stream 0 = residual after attention,
// 1 = residual after the MLP, 2 = attention probabilities (reference model.py:47-56, 66-71).
struct DropCfg {
  const int64_t* seed;  // nullptr or thresh == 0: dropout off
  uint32_t site;
  uint32_t thresh;      // p · 2^32
  float scale;          // 1 / (1 - p)
};
__device__ __forceinline__ uint32_t drop_key(const int64_t* seed, uint32_t site, uint32_t sub) {
  const uint64_t s = (uint64_t)*seed;
  return hash3((uint32_t)s, (uint32_t)(s >> 32), site * 4u + sub);
}
// this thread's row-pass elements (row gr, columns rp_col(j) + e of a C-wide row) × mask·scale
template <int NCH>
__device__ __forceinline__ void drop_rows(float (&v)[NCH][8], const DropCfg& d, uint32_t sub, int gr, int C) {
  if (d.thresh == 0u) return;
  const uint32_t key = drop_key(d.seed, d.site, sub);
  // element index gr·C + 8(t & 3) + (32j + e): base product once (keep_elem_m)
  uint32_t cm0 = ((uint32_t)gr * (uint32_t)C + (uint32_t)(8 * (threadIdx.x & 3))) * kHashM1;
  asm volatile("" : "+v"(cm0));
  const uint32_t hs = hash3_seed(key, 0u);
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[j][e] = keep_elem_m(hs, cm0 + (uint32_t)(32 * j + e) * kHashM1, d.thresh) ? v[j][e] * d.scale : 0.f;
}

}  // namespace pio
