// Per-layer phase timeline of the persistent self-attention block forward (csrc/persist.hip) at
// the headline shape (C = 64, H = 4, N = 256 latents, L = 6 layers; rows R = B·N, default 16384):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -munsafe-fp-atomics -DPIO_TRACE -mllvm -amdgpu-mfma-vgpr-form=1 \
//         -I perceiver_io_amd/csrc tools/trace/persist_trace.hip -o tools/trace/persist_trace && tools/trace/persist_trace [rows]
// slots per layer: 0 wait start, 1 loads issued (after the sample's hand-off), 2 LDS staging written,
//   3 barrier, 4 attention, 5 barrier, 6 out-proj GEMM, 7 LN2, 8 W1 GELU W2 residual + Z store, 9 LN1 + QKV stores.
#include "../../perceiver_io_amd/csrc/persist.hip"

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

int main(int argc, char** argv) {
  const int C = 64, H = 4, N = 256, L = 6, R = argc > 1 ? atoi(argv[1]) : 16384;
  srand(3);
  pio::SABlockFwdArgs a{};
  a.QKV0 = dev_fill<uint16_t>((size_t)R * 3 * C, 2.f, true);
  a.X0 = dev_fill<float>((size_t)R * C, 2.f, false);
  unsigned* sync;
  CK(hipMalloc(&sync, 1 << 16));
  CK(hipMemset(sync, 0, 1 << 16));
  a.sync = sync;
  a.L = L; a.N = N; a.R = R; a.scale_log2 = 0.36f; a.eps = 1e-5f;
  for (int i = 0; i < L; ++i) {
    pio::SAFwdLayer& y = a.ly[i];
    y.Wo = dev_fill<uint16_t>(C * C, 0.2f, true); y.W1 = dev_fill<uint16_t>(C * C, 0.2f, true);
    y.W2 = dev_fill<uint16_t>(C * C, 0.2f, true);
    y.bo = dev_fill<float>(C, 0.2f, false); y.g2 = dev_fill<float>(C, 0.2f, false, 1.f);
    y.be2 = dev_fill<float>(C, 0.2f, false); y.b1 = dev_fill<float>(C, 0.2f, false); y.b2 = dev_fill<float>(C, 0.2f, false);
    CK(hipMalloc(&y.O, (size_t)R * C * 2)); CK(hipMalloc(&y.U, (size_t)R * C * 2));
    CK(hipMalloc(&y.LSE, (size_t)R * H * 4)); CK(hipMalloc(&y.Z, (size_t)R * C * 4)); CK(hipMalloc(&y.Y, (size_t)R * C * 4));
    CK(hipMalloc(&y.mean2, R * 4)); CK(hipMalloc(&y.rstd2, R * 4));
    if (i + 1 < L) {
      y.nq = 3 * C;
      y.Wq = dev_fill<uint16_t>(3 * C * C, 0.2f, true);
      y.lnw = dev_fill<float>(C, 0.2f, false, 1.f); y.lnb = dev_fill<float>(C, 0.2f, false);
      y.bq = dev_fill<float>(3 * C, 0.2f, false);
      CK(hipMalloc(&y.QKVn, (size_t)R * 3 * C * 2)); CK(hipMalloc(&y.mean1n, R * 4)); CK(hipMalloc(&y.rstd1n, R * 4));
    }
  }
  long long* tb;
  CK(hipMalloc(&tb, 16 * 64 * 8));
  long long* nul = nullptr;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_wg), &nul, sizeof(nul)));
  int bx = argc > 2 ? atoi(argv[2]) : R / 128, by = 0, bz = 0;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_bx), &bx, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_by), &by, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_bz), &bz, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_buf), &tb, sizeof(tb)));
  auto launch = [&]() { if (!pio::sa_block_fwd_launch(a, 0)) { printf("launch refused\n"); exit(1); } };
  for (int i = 0; i < 20; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 100;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("sa_block_fwd L=%d R=%d: %.2f us/launch (%.2f us/layer)\n", L, R, ms * 1e3 / iters, ms * 1e3 / iters / L);
  unsigned err = pio::persist_errors(true);
  printf("persist errors: %u\n", err);
  CK(hipMemset(tb, 0, 16 * 64 * 8));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<long long> t(16 * 64);
  CK(hipMemcpy(t.data(), tb, t.size() * 8, hipMemcpyDeviceToHost));
  for (int wv = 0; wv < 8; ++wv) {
    long long first = 0;
    for (int s = 0; s < 63; ++s) if (t[wv * 64 + s]) { first = t[wv * 64 + s]; break; }
    if (!first) continue;
    printf("wave %d:\n", wv);
    long long prev = first;
    for (int l = 0; l < L; ++l) {
      printf("  layer %d:", l);
      for (int k = 0; k < 10; ++k) {
        const long long v = t[wv * 64 + 10 * l + k];
        if (!v) continue;
        printf(" [%d]%.2f", k, (v - prev) / 2400.0);
        prev = v;
      }
      printf("\n");
    }
    printf("  total %.2f us\n", (prev - first) / 2400.0);
  }
  return 0;
}
