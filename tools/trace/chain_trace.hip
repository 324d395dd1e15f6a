// Phase timelines of the chain-layout kernels at the headline self-attention shape (C = 64, H = 4,
// N = 256 latents; rows R = B·N, default 16384).  Standalone (no torch):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -munsafe-fp-atomics -DPIO_TRACE -mllvm -amdgpu-mfma-vgpr-form=1 \
//         -I perceiver_io_amd/csrc tools/trace/chain_trace.hip -o /tmp/chain_trace && /tmp/chain_trace [rows]
// sa_layer_fwd_chain slots: 1 loads issued, 2 LDS staging written, 3 barrier, 4 attention, 5 barrier,
//   6 out-proj GEMM, 7 LN2, 8 W1 GELU W2 residual + Z store, 9 LN1 + QKV stores.
// ln_linear_post_attn_bwd_chain slots: 1 loads issued, 2 staging written, 3 barrier, 4 dXn1 GEMM,
//   5 LN1 bwd + images, 6 barrier, 7 dH, 8 dU dXn2 LN2 bwd, 9 dO delta images, 10 barrier,
//   11 PA weight grads, 12 LL weight grads.
#include "../../perceiver_io_amd/csrc/rowgemm.hip"
#include "../../perceiver_io_amd/csrc/chain.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static uint16_t h_f2bf(float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16); }

template <typename T>
static T* dev_fill(size_t n, float scale, bool bf, float offset = 0.f) {
  T* p;
  CK(hipMalloc(&p, n * sizeof(T)));
  std::vector<T> h(n);
  for (size_t i = 0; i < n; ++i) {
    const float v = (rand() / (float)RAND_MAX - 0.5f) * scale + offset;
    if (bf) h[i] = (T)h_f2bf(v);
    else std::memcpy(&h[i], &v, sizeof(float));
  }
  CK(hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

static void wg_summary(const char* what, std::vector<double> st, std::vector<double> du) {
  if (st.empty()) return;
  std::sort(st.begin(), st.end());
  std::sort(du.begin(), du.end());
  const size_t n = st.size();
  printf("  %s (%zu WGs): start min %.2f p50 %.2f p90 %.2f max %.2f | duration min %.2f p50 %.2f p90 %.2f max %.2f us\n",
         what, n, st[0], st[n / 2], st[n * 9 / 10], st[n - 1], du[0], du[n / 2], du[n * 9 / 10], du[n - 1]);
}

template <typename F>
static void trace(const char* name, int R, F launch, int nwg_total = 0) {
  long long* tb;
  CK(hipMalloc(&tb, 16 * 64 * 8));
  long long* nul = nullptr;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_wg), &nul, sizeof(nul)));
  int bx = R / 128, by = 0, bz = 0;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_bx), &bx, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_by), &by, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_bz), &bz, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_buf), &tb, sizeof(tb)));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 200;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%s R=%d: %.2f us/launch\n", name, R, ms * 1e3 / iters);
  CK(hipMemset(tb, 0, 16 * 64 * 8));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<long long> t(16 * 64);
  CK(hipMemcpy(t.data(), tb, t.size() * 8, hipMemcpyDeviceToHost));
  for (int wv = 0; wv < 16; ++wv) {
    long long prev = t[wv * 64];
    if (!prev) continue;
    printf("  wave %d:", wv);
    for (int s = 1; s < 64; ++s) {
      if (!t[wv * 64 + s]) continue;
      printf(" [%d]%.2f", s, (t[wv * 64 + s] - prev) / 2400.0);
      prev = t[wv * 64 + s];
    }
    printf("  total %.2f\n", (prev - t[wv * 64]) / 2400.0);
  }
  // dispatch timeline (s_memrealtime, 100 MHz): tile workgroups and appended (slab job) ones
  const int tiles = R / 64, nwg = nwg_total > tiles ? nwg_total : tiles;
  long long* twg;
  CK(hipMalloc(&twg, (size_t)2 * nwg * 8));
  CK(hipMemset(twg, 0, (size_t)2 * nwg * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_wg), &twg, sizeof(twg)));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_wg), &nul, sizeof(nul)));
  std::vector<long long> w(2 * nwg);
  CK(hipMemcpy(w.data(), twg, w.size() * 8, hipMemcpyDeviceToHost));
  long long g0 = -1, g1 = 0;
  for (int i = 0; i < nwg; ++i)
    if (w[2 * i]) { g0 = g0 < 0 ? w[2 * i] : std::min(g0, w[2 * i]); g1 = std::max(g1, w[2 * i + 1]); }
  std::vector<double> st, du, st2, du2;
  for (int i = 0; i < nwg; ++i) {
    if (!w[2 * i]) continue;
    (i < tiles ? st : st2).push_back((w[2 * i] - g0) / 100.0);
    (i < tiles ? du : du2).push_back((w[2 * i + 1] - w[2 * i]) / 100.0);
  }
  printf("  grid span %.2f us\n", (g1 - g0) / 100.0);
  wg_summary("tiles", st, du);
  wg_summary("appended", st2, du2);
  CK(hipFree(twg));
  CK(hipFree(tb));
}

int main(int argc, char** argv) {
  const int C = 64, H = 4, N = 256, R = argc > 1 ? atoi(argv[1]) : 16384;
  srand(3);
  uint16_t* QKV = dev_fill<uint16_t>((size_t)R * 3 * C, 2.f, true);
  float* X = dev_fill<float>((size_t)R * C, 2.f, false);
  uint16_t* W[4];
  for (int i = 0; i < 4; ++i) W[i] = dev_fill<uint16_t>((size_t)3 * C * C, 0.2f, true);
  float* vec[8];
  for (int i = 0; i < 8; ++i) vec[i] = dev_fill<float>(3 * C, 0.2f, false, 1.f);
  uint16_t *O, *U, *QKVn, *dO;
  float *LSE, *Z, *Y, *m2, *r2, *m1, *r1, *dY, *delta, *slab;
  CK(hipMalloc(&O, (size_t)R * C * 2));
  CK(hipMalloc(&U, (size_t)R * C * 2));
  CK(hipMalloc(&QKVn, (size_t)R * 3 * C * 2));
  CK(hipMalloc(&dO, (size_t)R * C * 2));
  CK(hipMalloc(&LSE, (size_t)R * H * 4));
  CK(hipMalloc(&Z, (size_t)R * C * 4));
  CK(hipMalloc(&Y, (size_t)R * C * 4));
  CK(hipMalloc(&dY, (size_t)R * C * 4));
  CK(hipMalloc(&delta, (size_t)R * H * 4));
  CK(hipMalloc(&m2, R * 4)); CK(hipMalloc(&r2, R * 4)); CK(hipMalloc(&m1, R * 4)); CK(hipMalloc(&r1, R * 4));
  pio::DropCfg dr{};
  trace("sa_layer_fwd_chain", R, [&]() {
    pio::sa_layer_fwd_launch(QKV, N, 0.36f, O, LSE, X, W[0], vec[0], vec[1], vec[2], 1e-5f, W[1], vec[3], W[2], vec[4],
                             Z, Y, m2, r2, U, R, vec[5], vec[6], W[3], vec[7], QKVn, m1, r1, dr, 3 * C, 0);
  });
  // backward: inputs from the forward above
  float* G = dev_fill<float>((size_t)R * 3 * C, 1.f, false);
  float* dres = dev_fill<float>((size_t)R * C, 1.f, false);
  const int tiles = R / 64, P = (C + C + 3 * C * C + 3 * C) + (3 * C * C + 5 * C);
  CK(hipMalloc(&slab, (size_t)tiles * P * 4));
  float* s = slab;
  float *dg1 = s, *db1 = s + C, *dwq = s + 2 * C, *dbq = s + 2 * C + 3 * C * C;
  float* pa = s + 2 * C + 3 * C * C + 3 * C;
  pio::PostAttnGrads g{pa, pa + C * C, pa + C * C + C, pa + C * C + 2 * C, pa + C * C + 3 * C,
                       pa + 2 * C * C + 3 * C, pa + 2 * C * C + 4 * C, pa + 3 * C * C + 4 * C, P, 1};
  pio::SlabJob job{};
  trace("ln_linear_post_attn_bwd_chain", R, [&]() {
    pio::ln_linear_post_attn_bwd_launch(C, G, false, W[3], Z, m1, r1, vec[5], vec[6], dres, dg1, db1, dwq, dbq, Y, m2, r2, U, O,
                                        W[0], W[1], W[2], vec[3], vec[4], dY, dO, delta, H, g, R, job, dr, 3 * C, 0);
  });
  // the same launch carrying the previous boundary's slab reduction (what the step runs)
  float* slab2;
  CK(hipMalloc(&slab2, (size_t)tiles * P * 4));
  CK(hipMemset(slab2, 0, (size_t)tiles * P * 4));
  float* gdst;
  CK(hipMalloc(&gdst, (size_t)P * 4));
  pio::SlabJob job2{};
  job2.slab = slab2; job2.S = tiles; job2.P = P; job2.nbx = (P + pio::kSlabColsPerBlock - 1) / pio::kSlabColsPerBlock;
  { const int t = getenv("PIO_SLAB_WGS") ? atoi(getenv("PIO_SLAB_WGS")) : 128; int nsy = std::max(1, std::min(tiles, t / job2.nbx)); const int rb = (tiles + nsy - 1) / nsy; job2.nblk = job2.nbx * ((tiles + rb - 1) / rb); }
  job2.n = 1; job2.dst[0] = gdst; job2.off[0] = 0; job2.len[0] = P;
  trace("ln_linear_post_attn_bwd_chain + slab job", R, [&]() {
    pio::ln_linear_post_attn_bwd_launch(C, G, false, W[3], Z, m1, r1, vec[5], vec[6], dres, dg1, db1, dwq, dbq, Y, m2, r2, U, O,
                                        W[0], W[1], W[2], vec[3], vec[4], dY, dO, delta, H, g, R, job2, dr, 3 * C, 0);
  }, R / 64 + job2.nblk);
  // G as bf16 (the attention backward's bf16 dQKV)
  uint16_t* Gb = dev_fill<uint16_t>((size_t)R * 3 * C, 1.f, true);
  trace("ln_linear_post_attn_bwd_chain bf16 G + slab job", R, [&]() {
    pio::ln_linear_post_attn_bwd_launch(C, Gb, true, W[3], Z, m1, r1, vec[5], vec[6], dres, dg1, db1, dwq, dbq, Y, m2, r2,
                                        U, O, W[0], W[1], W[2], vec[3], vec[4], dY, dO, delta, H, g, R, job2, dr, 3 * C, 0);
  }, R / 64 + job2.nblk);
  return 0;
}
