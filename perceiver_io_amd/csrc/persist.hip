// Persistent latent self-attention block kernels (C = 64, H = 4, N ≤ 256 latents): ONE launch runs
// every layer of a block (reference model.py:36-44 self_attention_block, applied at
// model.py:185-187), instead of one launch per layer (chain.hip).
//
// Forward.  A workgroup owns one 64-row tile of one batch element for the whole block; its
// residual rows stay in registers (the CL2 chain layout of chain_cl.h) from the first layer to
// the last, and the next layer's weights are prefetched while it waits for its sample.  Self-
// attention only mixes the rows of one batch element, so the only cross-workgroup dependency is
// "the T = N / 64 tiles of my sample have published their next-layer QKV rows": a per-sample
// counter in global memory (one agent-scope add per tile and layer), polled by one lane.
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16, the write-through row of
// MI355X_MICROARCH.md § visibility): every published byte (the next layer's QKV rows) is stored
// sc1 (write-through) and every load of it is an sc1 buffer load (L1 bypass); every storing wave
// drains (s_waitcnt vmcnt(0)) before the workgroup barrier behind which one lane adds to the
// counter; the consumer polls relaxed (sc1 loads), then a workgroup barrier, then loads.
//
// Deadlock freedom without assuming co-residency (RCCL kernels may hold CUs under DDP): tiles
// are handed out by an atomic ticket in the order workgroups START, and the T tiles of a sample
// take consecutive tickets.  A workgroup holding a ticket is running, every lower ticket has
// been taken, so only the sample of the highest ticket taken can be incomplete; all others
// finish and free their CUs.  Every spin is bounded: a timeout sets a sticky error word
// (persist_errors) and the workgroup gives up waiting instead of hanging the GPU.
// The sync words (ticket, arrival count, per-sample counters) live in a persistent per-stream
// buffer that is zero before every launch: the LAST workgroup to finish (arrival count) resets
// them for the next launch on the stream.  No memset node (a hipMemsetAsync issued during stream
// capture is not replayed on this stack: measured, tools/persist_diag2.py) and no extra launch.
// The cross-workgroup hand-offs below rely on the write-through (sc1) store / L1-bypassing load
// behaviour measured on gfx950 (MI355X_MICROARCH.md, inter-workgroup visibility): no other target.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "this translation unit's sc1 hand-off protocol is validated on gfx950 (MI355X) only"
#endif
#include "chain_cl.h"
#include "persist_args.h"

namespace pio {

static __device__ unsigned pio_persist_err;  // sticky: bit 0 = a bounded spin timed out, bit 1 = bad ticket
// polls before a wait gives up (≈1 s); 0 (tests only) makes every wait time out at once
static __device__ unsigned pio_persist_spin_limit = 1u << 21;

void persist_set_spin_limit(unsigned n) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(pio_persist_spin_limit), &n, sizeof(n), 0, hipMemcpyHostToDevice);
}

unsigned persist_errors(bool reset) {
  unsigned h = 0;
  (void)hipMemcpyFromSymbol(&h, HIP_SYMBOL(pio_persist_err), sizeof(h), 0, hipMemcpyDeviceToHost);
  if (reset) {
    const unsigned z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(pio_persist_err), &z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  return h;
}

// buffer descriptor over [p, p + bytes) from wave-uniform values (kernel arguments)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pbuf(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// sc1 (L1-bypassing) 16-byte load; an offset past the descriptor's range reads zeros
__device__ __forceinline__ bf16x8 ld16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16));
}
// sc1 (write-through) 8-byte store
__device__ __forceinline__ void st8_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, uint2 v) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  u32x2 w;
  w[0] = v.x;
  w[1] = v.y;
  __builtin_amdgcn_raw_buffer_store_b64(w, r, (int)off, 0, 16);
}
// per-layer trace slots (tools/trace/persist_trace.hip): slot 10·layer + k
#define PTS(k) PIO_TS(10 * i + (k) < 63 ? 10 * i + (k) : 63)
constexpr unsigned kOffNone = 0x80000000u;  // past every descriptor: the load returns zeros
typedef __attribute__((address_space(1))) unsigned gu32;  // shared words: global (never flat) accesses

// one lane: poll *p (relaxed, sc1) until it reaches target; bounded (≈1 s), a timeout sets the
// sticky error word and returns false (the caller stops waiting for the rest of the launch)
__device__ __forceinline__ bool wait_count(unsigned* p, unsigned target) {
  const unsigned lim = pio_persist_spin_limit;
  if (lim == 0) {  // test hook (persist_set_spin_limit(0)): every wait times out
    atomicOr(&pio_persist_err, 1u);
    return false;
  }
  for (unsigned s = 0; __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++s) {
    if (s > lim) {
      atomicOr(&pio_persist_err, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}
// sync word layout (persist_args.h): [0] ticket, [1] finished workgroups, [4 ..) counters
constexpr int kSyncTicket = 0, kSyncDone = 1, kSyncCounters = 4;
// every workgroup, at its very end: count the arrival; the last one resets the nwords sync words
// (every other workgroup has taken its ticket and stopped polling) for the next launch
__device__ __forceinline__ void finish_launch(unsigned* sync, int nwords, int* sflag) {
  __syncthreads();
  if (threadIdx.x == 0)
    *sflag = __hip_atomic_fetch_add((gu32*)(sync + kSyncDone), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             gridDim.x * gridDim.y * gridDim.z - 1;
  __syncthreads();
  if (*sflag)
    for (int i = threadIdx.x; i < nwords; i += blockDim.x)
      __hip_atomic_store((gu32*)(sync + i), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every storing wave drained, then one lane signals the sample counter
__device__ __forceinline__ void publish_count(unsigned* p) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add((gu32*)p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------
// Forward: per layer exactly the math of sa_layer_fwd_chain8_kernel<NEXT, NQ, MAXKT> (chain.hip),
// so the block's outputs are bitwise those of the per-layer launches.
// ------------------------------------------------------------------------------------
// KLDS: the sample's K rows are staged in LDS once per workgroup (as V is) and every wave reads
// its head's fragments from there — the two query-block waves of a head no longer both fetch the
// head's K through the memory system (64 → 32 KB of K loads per workgroup and layer)
// LOCAL (N = 64: the workgroup's tile is the whole sample): layer i + 1's Q, K and V rows are
// also written into the workgroup's LDS images as layer i produces them, so layers ≥ 1 load
// nothing from global memory before their attention and need no drain before the hand-off (the
// rows still go to QKVn for the backward); MAXKT = 4 then (2 key tiles used).
template <int MAXKT, bool KLDS, bool ADROP, bool LOCAL = false>
__global__ __launch_bounds__(512) void sa_block_fwd_kernel(SABlockFwdArgs a) {
  constexpr int C = 64, H = 4, D = 16, LD = C + 8, LDV = C + 8, C3 = 3 * C, NT = 512;
  constexpr int NVI = MAXKT * 32 * 8 / NT;  // 16-byte V chunks per thread
  static_assert(MAXKT % 4 == 0 && MAXKT * 32 * 8 % NT == 0, "key tiles");
  constexpr int NWR = 6 * C;                // weight rows staged: Wo, W1, W2 | up to 3C rows of Wq
  constexpr int NWC = NWR * 8 / NT;         // 16-byte weight chunks per thread
  __shared__ __attribute__((aligned(16))) uint16_t sV[MAXKT * 32 * LDV + 64];
  __shared__ __attribute__((aligned(16))) uint16_t sK[KLDS ? MAXKT * 32 * LDV : 8];
  __shared__ __attribute__((aligned(16))) uint16_t sO[64 * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sW[NWR * LD];
  __shared__ __attribute__((aligned(16))) float sVec[10 * C];  // bo b1 b2 γ2 β2 γ1 β1 | bq (≤ 3C)
  __shared__ __attribute__((aligned(16))) bf16x8 sX[2][8 * 64];
  __shared__ __attribute__((aligned(16))) float2 sR[2][8 * 16];
  __shared__ __attribute__((aligned(16))) uint16_t sOnes[16 * 16];
  __shared__ __attribute__((aligned(16))) uint16_t sQl[LOCAL ? 64 * LD : 8];  // LOCAL: the next layer's Q rows
  __shared__ int sTicket, sLast;
  static_assert(!LOCAL || KLDS, "LOCAL keeps K in LDS");
  PIO_WG_BEGIN();
  if (threadIdx.x == 0)
    sTicket = (int)__hip_atomic_fetch_add((gu32*)(a.sync + kSyncTicket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < 128) reinterpret_cast<uint32_t*>(sOnes)[threadIdx.x] = 0x3F803F80u;
  __syncthreads();
  const int tile = sTicket;
  const int nsync = kSyncCounters + a.R / a.N;
  if (tile < 0 || tile >= a.R / 64) {  // never with a zeroed ticket and grid = R / 64 (uniform)
    if (threadIdx.x == 0) atomicOr(&pio_persist_err, 2u);
    finish_launch(a.sync, nsync, &sLast);
    return;
  }
  auto body = [&](auto hfc) {
  constexpr int hf = decltype(hfc)::value, qb = hf;
  const int w = wave_id(), l = lane_id(), hh = l >> 5, r = l & 31, g = l >> 4;
  const int N = a.N, T = N / 64, nkt = N / 32;
  const int m0 = tile * 64, b = m0 / N;
  const unsigned rb = (unsigned)(b * N);
  const int h = w & 3;
  const int gr = m0 + 16 * (w & 3) + (l & 15);  // this lane's chain row
  const int lr = 16 * (w & 3) + (l & 15);
  unsigned* cnt = a.sync + kSyncCounters + b;
  const unsigned qkv_bytes = (unsigned)a.R * C3 * 2u;
  bool live = true;  // false after a timed-out wait: stop waiting (results are garbage, flagged)

  // the residual rows, register-resident for the whole block (CL2: row gr, channels of half hf)
  float xr[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float4 v = *reinterpret_cast<const float4*>(a.X0 + (long long)gr * C + 16 * (2 * hf + i) + 4 * g);
    xr[i][0] = v.x; xr[i][1] = v.y; xr[i][2] = v.z; xr[i][3] = v.w;
  }
  // weight / vector prefetch of layer i into registers (plain loads: read-only in the launch)
  bf16x8 wr[NWC];
  float pv = 0.f, pq = 0.f;
  auto prefetch = [&](int i) {
    const SAFwdLayer& y = a.ly[i];
    const int nq = y.nq;
#pragma unroll
    for (int k = 0; k < NWC; ++k) {
      const int c = threadIdx.x + NT * k, row = c >> 3, col = (c & 7) * 8;
      const uint16_t* src = row < C ? y.Wo + row * C : row < 2 * C ? y.W1 + (row - C) * C
                          : row < 3 * C ? y.W2 + (row - 2 * C) * C : row < 3 * C + nq ? y.Wq + (row - 3 * C) * C : y.Wo;
      wr[k] = *reinterpret_cast<const bf16x8*>(src + col);
    }
    const int t = threadIdx.x, vi = t >> 6, kk = t & 63;
    const bool nx = nq > 0;
    const float* vs = vi == 0 ? y.bo : vi == 1 ? y.b1 : vi == 2 ? y.b2 : vi == 3 ? y.g2 : vi == 4 ? y.be2
                    : vi == 5 ? (nx ? y.lnw : y.bo) : vi == 6 ? (nx ? y.lnb : y.bo) : y.bo;
    pv = vs[kk];
    pq = nx ? y.bq[t < nq ? t : 0] : 0.f;
  };
  prefetch(0);

  for (int i = 0; i < a.L; ++i) {
    const SAFwdLayer& y = a.ly[i];
    const uint16_t* qkv = i == 0 ? a.QKV0 : a.ly[i - 1].QKVn;
    // ---- wait for the sample's tiles (layer i's QKV rows published), then every load ----
    PTS(0);
    if (i > 0 && T > 1) {
      if (threadIdx.x == 0 && live) live = wait_count(cnt, (unsigned)(T * i));
      __syncthreads();
    }
    const __amdgpu_buffer_rsrc_t rq = pbuf(qkv, qkv_bytes);
    bf16x8 kf[MAXKT], qf, vr[NVI], kr[KLDS ? NVI : 1];
    const bool gload = !(LOCAL && i > 0);  // LOCAL layers ≥ 1: Q / K / V are already in LDS (uniform)
    if (gload) {
      if constexpr (KLDS) {
#pragma unroll
        for (int k = 0; k < NVI; ++k) {
          const int c = threadIdx.x + NT * k, key = c >> 3, col = (c & 7) * 8;
          kr[k] = ld16_sc1(rq, key < N ? ((rb + key) * C3 + C + col) * 2u : kOffNone);
        }
      } else {
#pragma unroll
        for (int kt = 0; kt < MAXKT; ++kt)
          kf[kt] = ld16_sc1(rq, kt < nkt ? ((rb + 32 * kt + r) * C3 + C + h * D + 8 * hh) * 2u : kOffNone);
      }
      qf = ld16_sc1(rq, ((unsigned)(m0 + 32 * qb + r) * C3 + h * D + 8 * hh) * 2u);
#pragma unroll
      for (int k = 0; k < NVI; ++k) {
        const int c = threadIdx.x + NT * k, key = c >> 3, col = (c & 7) * 8;
        vr[k] = ld16_sc1(rq, key < N ? ((rb + key) * C3 + 2 * C + col) * 2u : kOffNone);
      }
    }
    PTS(1);
    // ---- stage this layer's weights / vectors (prefetched) and the sample's V rows ----
#pragma unroll
    for (int k = 0; k < NWC; ++k) {
      const int c = threadIdx.x + NT * k, row = c >> 3, col = (c & 7) * 8;
      cl_wstore(sW, LD, row, col, wr[k], row >= C);  // Wo natural, the rest permuted
    }
    if ((int)threadIdx.x < 7 * C) sVec[threadIdx.x] = pv;
    if ((int)threadIdx.x < 3 * C) sVec[7 * C + threadIdx.x] = pq;
    if (gload) {
#pragma unroll
      for (int k = 0; k < NVI; ++k) {
        const int c = threadIdx.x + NT * k, key = c >> 3, col = (c & 7) * 8;
        *reinterpret_cast<bf16x8*>(sV + key * LDV + col) = vr[k];
        if constexpr (KLDS) *reinterpret_cast<bf16x8*>(sK + key * LDV + col) = kr[k];
      }
    }
    PTS(2);
    lds_sync();
    PTS(3);
    if (!gload) qf = *reinterpret_cast<const bf16x8*>(sQl + (32 * qb + r) * LD + h * D + 8 * hh);


    // ---- attention: head h, query block qb (sa_layer_fwd_chain8_kernel) ----
    {
      float m_run = -INFINITY, l_run = 0.f;
      f32x16 o = f32x16{};
#pragma unroll
      for (int ch = 0; ch < MAXKT / 4; ++ch) {
        if (4 * ch < nkt) {
          f32x16 sc[4];
          float mt = -INFINITY;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int kt = 4 * ch + k;
            sc[k] = f32x16{};
            if (kt < nkt) {
              const bf16x8 kfr = KLDS ? *reinterpret_cast<const bf16x8*>(sK + (32 * kt + r) * LDV + h * D + 8 * hh)
                                      : kf[kt];
              sc[k] = mfma32(kfr, qf, sc[k]);
#pragma unroll
              for (int e = 0; e < 16; ++e) mt = fmaxf(mt, sc[k][e]);
            }
          }
          const float m_new = fmaxf(m_run, xor32_max(mt) * a.scale_log2);
          const float alpha = fast_exp2(m_run - m_new);
#pragma unroll
          for (int e = 0; e < 16; ++e) o[e] *= alpha;
          if constexpr (ADROP) l_run *= alpha;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (4 * ch + k < nkt) {
#pragma unroll
              for (int e = 0; e < 16; ++e) sc[k][e] = fast_exp2(fmaf(sc[k][e], a.scale_log2, -m_new));
              if constexpr (ADROP) {  // attention-probability dropout, as sa_layer_fwd_chain8_kernel
                const uint32_t dkey = drop_key(a.dr.seed, (uint32_t)i, 2u);
                // element index (row)·N + 32(4ch + k) + 4hh + acc_row(e, 0) (keep_elem_m)
                uint32_t cm0 = ((uint32_t)(m0 - (int)rb + 32 * qb + r) * (uint32_t)N + (uint32_t)(32 * (4 * ch + k) + 4 * hh)) * kHashM1;
                asm volatile("" : "+v"(cm0));
                const uint32_t hs = hash3_seed(dkey, (uint32_t)(b * H + h));
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                  l_run += sc[k][e];
                  sc[k][e] = keep_elem_m(hs, cm0 + (uint32_t)acc_row(e, 0) * kHashM1, a.dr.thresh) ? sc[k][e] * a.dr.scale : 0.f;
                }
              }
            }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int kt = 4 * ch + k;
            if (kt < nkt) {
#pragma unroll
              for (int ss = 0; ss < 2; ++ss)
                o = mfma32(frag_ks_perm_ones(sV, LDV, h * D, 32 * kt + 16 * ss, sOnes), pack_acc(sc[k], ss), o);
            }
          }
          m_run = m_new;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      const float ls = ADROP ? xor32_sum(l_run) : o[8];
      const float inv = 1.f / ls;
      const int row = 32 * qb + r;
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        uint2 pk;
        pk.x = pack2(o[4 * gg] * inv, o[4 * gg + 1] * inv);
        pk.y = pack2(o[4 * gg + 2] * inv, o[4 * gg + 3] * inv);
        *reinterpret_cast<uint2*>(sO + row * LD + h * D + 8 * gg + 4 * hh) = pk;
      }
      if (hh == 0) y.LSE[(long long)(m0 + row) * H + h] = m_run + __log2f(ls);
    }
    PTS(4);
    lds_sync();
    PTS(5);
    {
      const int row = threadIdx.x >> 3, col = (threadIdx.x & 7) * 8;
      *reinterpret_cast<bf16x8*>(y.O + (long long)(m0 + row) * C + col) = *reinterpret_cast<const bf16x8*>(sO + row * LD + col);
    }

    // ---- the post-attention chain (pair w & 3, channel half hf) ----
    DropCfg dr = a.dr;
    dr.site = (uint32_t)i;
    const uint16_t *sWo = sW, *sW1 = sW + C * LD, *sW2 = sW + 2 * C * LD, *sWq = sW + 3 * C * LD;
    f32x4 acc[2];
    {
      bf16x8 bo_[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) bo_[t] = *reinterpret_cast<const bf16x8*>(sO + lr * LD + 32 * t + 8 * g);
      cl2_gemm(sWo, LD, hf, bo_, acc);
    }
    PTS(6);
    float yv[2][4], t0[2][4];
    cl2_bias(t0, acc, sVec, hf);
    cl2_drop(t0, dr, 0u, gr, hf);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) { yv[p][j] = xr[p][j] + t0[p][j]; t0[p][j] = yv[p][j]; }
    cl2_store_f32(y.Y, C, gr, hf, yv);
    float mu, rs;
    cl2_layernorm(t0, sR[0], hf, sVec + 3 * C, sVec + 4 * C, a.eps, mu, rs);
    if (g == 0 && hf == 0) { y.mean2[gr] = mu; y.rstd2[gr] = rs; }
    PTS(7);
    {
      bf16x8 bb[2];
      cl2_swap_frag(sX[0], cl2_frag(t0), hf, bb);
      cl2_gemm(sW1, LD, hf, bb, acc);
    }
    cl2_bias(t0, acc, sVec + C, hf);
    cl2_store_bf16(y.U, C, gr, hf, t0);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) t0[p][j] = gelu_f(t0[p][j]);
    {
      bf16x8 bb[2];
      cl2_swap_frag(sX[1], cl2_frag(t0), hf, bb);
      cl2_gemm(sW2, LD, hf, bb, acc);
    }
    cl2_bias(t0, acc, sVec + 2 * C, hf);
    cl2_drop(t0, dr, 1u, gr, hf);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) { t0[p][j] += yv[p][j]; xr[p][j] = t0[p][j]; }
    cl2_store_f32(y.Z, C, gr, hf, t0);
    PTS(8);
    const int nq = y.nq;
    if (nq > 0) {  // the next LN1 + projection (uniform)
      cl2_layernorm(t0, sR[1], hf, sVec + 5 * C, sVec + 6 * C, a.eps, mu, rs);
      if (g == 0 && hf == 0) { y.mean1n[gr] = mu; y.rstd1n[gr] = rs; }
      bf16x8 bb[2];
      cl2_swap_frag(sX[0], cl2_frag(t0), hf, bb);
      const __amdgpu_buffer_rsrc_t rn = pbuf(y.QKVn, (unsigned)a.R * (unsigned)nq * 2u);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (q * C < nq) {
          f32x4 aq[2];
          cl2_gemm(sWq + q * C * LD, LD, hf, bb, aq);
          float v[2][4];
          cl2_bias(v, aq, sVec + 7 * C + q * C, hf);
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            uint2 pk;
            pk.x = pack2(v[p][0], v[p][1]);
            pk.y = pack2(v[p][2], v[p][3]);
            st8_sc1(rn, ((unsigned)gr * (unsigned)nq + q * C + 16 * (2 * hf + p) + 4 * g) * 2u, pk);
            if (LOCAL && i + 1 < a.L) {  // the next layer's row lr (= its key lr) into the LDS images;
              // every wave's reads of this layer's sK / sV ended at the barrier after the attention
              uint16_t* dst = q == 0 ? sQl + lr * LD : q == 1 ? sK + lr * LDV : sV + lr * LDV;
              *reinterpret_cast<uint2*>(dst + 16 * (2 * hf + p) + 4 * g) = pk;
            }
          }
        }
      }
    }
    PTS(9);
    if (i + 1 < a.L) {
      // publish the next layer's QKV rows to the sample; the barrier inside also ends every
      // wave's reads of this layer's LDS images (the next layer overwrites them).  LOCAL: no
      // other workgroup reads them — the barrier only, no drain of the stores
      if constexpr (LOCAL) lds_sync();
      else publish_count(cnt);
      prefetch(i + 1);
    }
  }
  };
  if (wave_id() >> 2) body(std::integral_constant<int, 1>{});
  else body(std::integral_constant<int, 0>{});
  finish_launch(a.sync, nsync, &sLast);
  PIO_WG_END();
}

int persist_sync_words(int B) { return kSyncCounters + 2 * B; }  // forward: B counters, backward: 2B

bool sa_block_fwd_launch(const SABlockFwdArgs& a, hipStream_t st) {
  if (a.L < 1 || a.L > kPersistMaxLayers || a.N <= 0 || a.N > 256 || a.N % 64 != 0 || a.R % a.N != 0) return false;
  for (int i = 0; i < a.L; ++i) {
    const int nq = a.ly[i].nq;
    if (nq != 0 && nq != 64 && nq != 128 && nq != 192) return false;
    if (i + 1 < a.L && nq != 192) return false;  // layers before the last feed the next layer's QKV
  }
  const dim3 grid(a.R / 64);  // the sample's K rows staged in LDS (KLDS; profiles/r5_persist.md)
  if (a.N == 64) {  // one tile per sample: the Q / K / V hand-off stays in the workgroup's LDS
    if (a.dr.thresh) hipLaunchKernelGGL((sa_block_fwd_kernel<4, true, true, true>), grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((sa_block_fwd_kernel<4, true, false, true>), grid, dim3(512), 0, st, a);
  } else if (a.dr.thresh) {
    hipLaunchKernelGGL((sa_block_fwd_kernel<8, true, true>), grid, dim3(512), 0, st, a);
  } else {
    hipLaunchKernelGGL((sa_block_fwd_kernel<8, true, false>), grid, dim3(512), 0, st, a);
  }
  return true;
}

}  // namespace pio
