// Phase timeline of post_attn_bwd_kernel at the headline self-attention shape (B·N = 16384 rows,
// C = 64, H = 4, slab gradients).  Standalone (no torch):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -munsafe-fp-atomics -DPIO_TRACE \
//         -I perceiver_io_amd/csrc tools/trace/post_attn_bwd_trace.hip -o /tmp/pab_trace && /tmp/pab_trace [rows]
// Prints µs per launch (events) and per-wave phase deltas (s_memtime shader-clock ticks at 2.4 GHz,
// as in attn_bwd_trace) of one mid-grid workgroup.  Slots: 0 start, 1 phase-0 loads issued,
// 2/3 before/after barrier 1, 4 dH GEMM, 5 dW2 partials stored, 6/7 barrier 2, 8/9 barrier 3,
// 10/11 barrier 4, 12/13 barrier 5, 14 dO GEMM + dWo partials, 15 barrier 6, 16 end.
#include "../../perceiver_io_amd/csrc/rowgemm.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static uint16_t h_f2bf(float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16); }

template <typename T>
static T* dev_fill(size_t n, float scale, bool bf) {
  T* p;
  CK(hipMalloc(&p, n * sizeof(T)));
  std::vector<T> h(n);
  for (size_t i = 0; i < n; ++i) {
    const float v = (rand() / (float)RAND_MAX - 0.5f) * scale;
    if (bf) h[i] = (T)h_f2bf(v);
    else std::memcpy(&h[i], &v, sizeof(float));
  }
  CK(hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
  return p;
}

int main(int argc, char** argv) {
  const int C = 64, H = 4, R = argc > 1 ? atoi(argv[1]) : 16384;
  srand(3);
  float* dZ = dev_fill<float>((size_t)R * C, 1.f, false);
  float* Y = dev_fill<float>((size_t)R * C, 2.f, false);
  float* m2 = dev_fill<float>(R, 0.1f, false);
  float* r2 = dev_fill<float>(R, 1.f, false);
  uint16_t* U = dev_fill<uint16_t>((size_t)R * C, 2.f, true);
  uint16_t* O = dev_fill<uint16_t>((size_t)R * C, 2.f, true);
  uint16_t* Wo = dev_fill<uint16_t>(C * C, 0.2f, true);
  uint16_t* W1 = dev_fill<uint16_t>(C * C, 0.2f, true);
  uint16_t* W2 = dev_fill<uint16_t>(C * C, 0.2f, true);
  float* g2 = dev_fill<float>(C, 1.f, false);
  float* be2 = dev_fill<float>(C, 1.f, false);
  float *dY, *delta, *slab;
  uint16_t* dO;
  CK(hipMalloc(&dY, (size_t)R * C * 4));
  CK(hipMalloc(&dO, (size_t)R * C * 2));
  CK(hipMalloc(&delta, (size_t)R * H * 4));
  const int tiles = (R + 63) / 64, P = 3 * C * C + 5 * C;
  CK(hipMalloc(&slab, (size_t)tiles * P * 4));
  pio::PostAttnGrads g{slab, slab + C * C, slab + C * C + C, slab + C * C + 2 * C, slab + C * C + 3 * C,
                       slab + 2 * C * C + 3 * C, slab + 2 * C * C + 4 * C, slab + 3 * C * C + 4 * C, P, 1};
  pio::SlabJob job{};
  pio::DropCfg dr{};
  auto launch = [&]() {
    pio::post_attn_bwd_launch(C, dZ, Y, m2, r2, U, O, Wo, W1, W2, g2, be2, dY, dO, delta, H, g, R, job, dr, 0);
  };
  long long* tb;
  CK(hipMalloc(&tb, 16 * 64 * 8));
  CK(hipMemset(tb, 0, 16 * 64 * 8));
  long long* nul = nullptr;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_wg), &nul, sizeof(nul)));
  int bx = tiles / 2, by = 0, bz = 0;
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
  printf("post_attn_bwd R=%d: %.2f us/launch\n", R, ms * 1e3 / iters);
  CK(hipMemset(tb, 0, 16 * 64 * 8));
  launch();
  CK(hipDeviceSynchronize());
  std::vector<long long> t(16 * 64);
  CK(hipMemcpy(t.data(), tb, t.size() * 8, hipMemcpyDeviceToHost));
  printf("per-wave phase deltas of WG %d in us (s_memtime shader clock at 2.4 GHz):\n", bx);
  for (int wv = 0; wv < 4; ++wv) {
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
  return 0;
}
