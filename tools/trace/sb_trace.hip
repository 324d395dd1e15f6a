// Per-layer phase timeline of the per-sample block kernels (csrc/sample_block.hip) at the image
// configs' shape (C = 128, H = 4, 32 latents, L = 3 layers; B samples, default 128 = MNIST):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -munsafe-fp-atomics -DPIO_TRACE \
//         -I perceiver_io_amd/csrc tools/trace/sb_trace.hip -o tools/trace/sb_trace && tools/trace/sb_trace [B] [C]
// forward slots per layer (12): 0 start, 1 LN1 stats, 2 barrier, 3 QKV GEMMs, 4 attention, 5 barrier,
//   6 out-proj, 7 LN2 stats, 8 barrier, 9 W1, 10 barrier, 11 W2.
// backward slots per layer (16): 0 start, 1 barrier, 2 dU, 3 barrier, 4 dXn2, 5 LN2 bwd, 6 LN2 partials,
//   7 barrier, 8 dO, 9 attention bwd, 10 barrier, 11 Wqkv block 0, 12 barrier, 13 barrier,
//   14 LN1 bwd, 15 LN1 partials.
#include "../../perceiver_io_amd/csrc/sample_block.hip"

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

static void report(const char* name, const long long* h, int L, int per, bool reverse) {
  printf("%s: per-layer phase durations (us at 100 MHz-equivalent shader clock ticks / 2.4e3), wave 0\n", name);
  for (int li = 0; li < L; ++li) {
    printf("  layer %d:", li);
    for (int k = 1; k < per; ++k) printf(" [%d]%.2f", k, (h[li * per + k] - h[li * per + k - 1]) / 2400.0);
    const int nx = reverse ? li - 1 : li + 1;  // the layer that runs next
    const long long end = (nx >= 0 && nx < L) ? h[nx * per] : h[li * per + per - 1];
    printf("  total %.2f\n", (end - h[li * per]) / 2400.0);
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 128, C = argc > 2 ? atoi(argv[2]) : 128, L = 3, R = B * 32;
  srand(3);
  pio::SBFwdArgs f{};
  pio::SBBwdArgs b{};
  f.X0 = b.X0 = dev_fill<float>((size_t)R * C, 2.f, false);
  f.L = b.L = L; f.B = b.B = B;
  f.scale_log2 = b.scale_log2 = 1.4426950f / sqrtf((float)(C / 4));
  f.eps = b.eps = 1e-5f;
  for (int i = 0; i < L; ++i) {
    pio::SBLayer& y = f.ly[i];
    y.Wqkv = dev_fill<uint16_t>(3 * C * C, 0.1f, true); y.Wo = dev_fill<uint16_t>(C * C, 0.1f, true);
    y.W1 = dev_fill<uint16_t>(C * C, 0.1f, true); y.W2 = dev_fill<uint16_t>(C * C, 0.1f, true);
    y.bqkv = dev_fill<float>(3 * C, 0.1f, false); y.g1 = dev_fill<float>(C, 0.1f, false, 1.f);
    y.be1 = dev_fill<float>(C, 0.1f, false); y.bo = dev_fill<float>(C, 0.1f, false);
    y.g2 = dev_fill<float>(C, 0.1f, false, 1.f); y.be2 = dev_fill<float>(C, 0.1f, false);
    y.b1 = dev_fill<float>(C, 0.1f, false); y.b2 = dev_fill<float>(C, 0.1f, false);
    uint16_t** bfs[6] = {&y.LN1X, &y.QKV, &y.O, &y.LN2Y, &y.U, &y.GU};
    for (int k = 0; k < 6; ++k) CK(hipMalloc(bfs[k], (size_t)R * (k == 1 ? 3 * C : C) * 2));
    CK(hipMalloc(&y.Y, (size_t)R * C * 4)); CK(hipMalloc(&y.Z, (size_t)R * C * 4));
    CK(hipMalloc(&y.mean1, R * 4)); CK(hipMalloc(&y.rstd1, R * 4)); CK(hipMalloc(&y.mean2, R * 4)); CK(hipMalloc(&y.rstd2, R * 4));
    b.ly[i] = y;
    pio::SBGrad& g = b.gr[i];
    CK(hipMalloc(&g.dQKV, (size_t)R * 3 * C * 2)); CK(hipMalloc(&g.dY, (size_t)R * C * 2));
    CK(hipMalloc(&g.dU, (size_t)R * C * 2)); CK(hipMalloc(&g.dZ, (size_t)R * C * 2));
  }
  float* lns;
  CK(hipMalloc(&lns, (size_t)B * 4 * L * C * 4));
  b.ln_rs = 4 * L * C;
  for (int i = 0; i < L; ++i) {
    b.gr[i].dg1 = lns + 4 * i * C; b.gr[i].dbe1 = lns + (4 * i + 1) * C;
    b.gr[i].dg2 = lns + (4 * i + 2) * C; b.gr[i].dbe2 = lns + (4 * i + 3) * C;
  }
  b.dZ = dev_fill<float>((size_t)R * C, 1.f, false);
  CK(hipMalloc(&b.dX, (size_t)R * C * 4));
  long long* tb;
  CK(hipMalloc(&tb, 16 * 64 * 8));
  long long* nul = nullptr;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_wg), &nul, sizeof(nul)));
  int bx = 0, by = 0, bz = 0;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_bx), &bx, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_by), &by, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_bz), &bz, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_buf), &tb, sizeof(tb)));
  std::vector<long long> h(16 * 64);
  for (int pass = 0; pass < 2; ++pass) {
    const bool fwd = pass == 0;
    auto launch = [&]() {
      const bool ok = fwd ? pio::sb_fwd_launch(f, C, 0) : pio::sb_bwd_launch(b, C, 0);
      if (!ok) { printf("launch refused\n"); exit(1); }
    };
    for (int i = 0; i < 10; ++i) launch();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemset(tb, 0, 16 * 64 * 8));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), tb, h.size() * 8, hipMemcpyDeviceToHost));
    printf("%s B=%d C=%d L=%d: %.2f us/launch\n", fwd ? "sb_fwd" : "sb_bwd", B, C, L, 1000.f * ms / iters);
    report(fwd ? "forward" : "backward", h.data(), L, fwd ? 12 : 16, !fwd);
  }
  return 0;
}
