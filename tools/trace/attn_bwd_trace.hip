// Phase timeline of attn_bwd_kernel at the headline self-attention shape (B=64, N=256, H=4,
// D=16, packed qkv rows).  Standalone (no torch):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPIO_TRACE -I perceiver_io_amd/csrc \
//         tools/trace/attn_bwd_trace.hip -o /tmp/attn_bwd_trace && /tmp/attn_bwd_trace
// Prints µs per launch (events), then per-wave phase times (shader clock, 100 MHz ticks on
// s_memtime are converted with the measured clock) of one mid-grid workgroup, and the spread
// of workgroup start / end times over the whole grid.
#include "../../perceiver_io_amd/csrc/attention.hip"

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static uint16_t h_f2bf(float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16); }

int main(int argc, char** argv) {
  const int B = 64, N = argc > 1 ? atoi(argv[1]) : 256, H = 4, D = 16, C = H * D;
  const int bz = argc > 2 ? atoi(argv[2]) : B / 2;
  std::vector<uint16_t> hqkv((size_t)B * N * 3 * C), hdo((size_t)B * N * C);
  srand(1);
  for (auto& v : hqkv) v = h_f2bf((rand() / (float)RAND_MAX - 0.5f));
  for (auto& v : hdo) v = h_f2bf((rand() / (float)RAND_MAX - 0.5f) * 0.1f);
  std::vector<float> hl((size_t)B * N * H, 8.f), hd((size_t)B * N * H, 0.01f);
  uint16_t *qkv, *dO;
  float *lse, *delta, *dqkv;
  CK(hipMalloc(&qkv, hqkv.size() * 2));
  CK(hipMalloc(&dO, hdo.size() * 2));
  CK(hipMalloc(&lse, hl.size() * 4));
  CK(hipMalloc(&delta, hd.size() * 4));
  CK(hipMalloc(&dqkv, (size_t)B * N * 3 * C * 4));
  CK(hipMemcpy(qkv, hqkv.data(), hqkv.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dO, hdo.data(), hdo.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(lse, hl.data(), hl.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(delta, hd.data(), hd.size() * 4, hipMemcpyHostToDevice));
  pio::AttnArgs a{};
  a.q = qkv; a.q_bs = (long long)N * 3 * C; a.q_rs = 3 * C;
  a.k = qkv + C; a.k_bs = a.q_bs; a.k_rs = 3 * C;
  a.v = qkv + 2 * C; a.v_bs = a.q_bs; a.v_rs = 3 * C;
  a.kmask = nullptr; a.B = B; a.H = H; a.Nq = N; a.Nk = N;
  a.scale = 0.25f; a.scale_log2 = 0.25f * 1.4426950408889634f;
  const long long bs = (long long)N * 3 * C;
  auto launch = [&]() {
    pio::attn_bwd_launch(a, D, nullptr, dO, lse, delta, dqkv, bs, 3 * C, dqkv + C, bs, 3 * C, dqkv + 2 * C, bs, 3 * C,
                         false, false, 0, 1, 0, 0);
  };
  long long *tb, *twg;
  const int nwg = B * H * ((N + 255) / 256);
  CK(hipMalloc(&tb, 16 * 64 * 8));
  CK(hipMalloc(&twg, 2 * nwg * 8 * 4));
  CK(hipMemset(tb, 0, 16 * 64 * 8));
  long long* nul = nullptr;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_wg), &nul, sizeof(nul)));
  int bx = 0, by = 1;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_bx), &bx, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_by), &by, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_bz), &bz, 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_buf), &tb, sizeof(tb)));
  for (int i = 0; i < 20; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  const int iters = 200;
  for (int i = 0; i < iters; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("attn_bwd N=%d: %.2f us/launch\n", N, ms * 1e3 / iters);
  {
    uint16_t* O;
    float* L;
    CK(hipMalloc(&O, (size_t)B * N * C * 2));
    CK(hipMalloc(&L, (size_t)B * N * H * 4));
    for (int i = 0; i < 20; ++i) pio::attn_fwd_launch(a, D, O, L, nullptr, nullptr, 1, 0);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) pio::attn_fwd_launch(a, D, O, L, nullptr, nullptr, 1, 0);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("attn_fwd N=%d: %.2f us/launch\n", N, ms * 1e3 / iters);
  }
  // clock rate of s_memtime: compare against events over one long launch sequence
  CK(hipMemset(tb, 0, 16 * 64 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(pio::trace_wg), &twg, sizeof(twg)));
  CK(hipMemset(twg, 0, 2 * nwg * 8));
  CK(hipEventRecord(e0));
  launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> t(16 * 64), w(2 * nwg);
  CK(hipMemcpy(t.data(), tb, t.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(w.data(), twg, w.size() * 8, hipMemcpyDeviceToHost));
  long long g0 = w[0], g1 = w[1];
  for (int i = 0; i < nwg; ++i) { g0 = std::min(g0, w[2 * i]); g1 = std::max(g1, w[2 * i + 1]); }
  printf("traced launch: %.2f us (events), WG span %.2f us (s_memrealtime, 100 MHz)\n", ms * 1e3, (g1 - g0) / 100.0);
  const double clk = 100.0;  // s_memtime counts the shader clock; report ticks and µs at 2.4 GHz
  (void)clk;
  auto us = [&](long long d) { return d / 2400.0; };
  printf("per-wave phase times of WG (0,%d,%d) in us at 2.4 GHz (slot: delta from previous recorded slot)\n", by, bz);
  for (int wv = 0; wv < 8; ++wv) {
    long long prev = t[wv * 64];
    if (!prev) continue;
    printf("  wave %d:", wv);
    for (int s = 1; s < 64; ++s) {
      if (!t[wv * 64 + s]) continue;
      printf(" [%d]%.2f", s, us(t[wv * 64 + s] - prev));
      prev = t[wv * 64 + s];
    }
    printf("  total %.2f\n", us(prev - t[wv * 64]));
  }
  printf("wave start skew vs wave 0 (us):");
  for (int wv = 0; wv < 8; ++wv)
    if (t[wv * 64]) printf(" %.2f", us(t[wv * 64] - t[0]));
  printf("\n");
  std::vector<double> st, du;
  auto rt = [](long long d) { return d / 100.0; };  // s_memrealtime ticks → µs
  for (int i = 0; i < nwg; ++i) { st.push_back(rt(w[2 * i] - g0)); du.push_back(rt(w[2 * i + 1] - w[2 * i])); }
  std::sort(st.begin(), st.end());
  std::sort(du.begin(), du.end());
  printf("WG start offsets (us): min %.2f p50 %.2f p90 %.2f max %.2f\n", st[0], st[nwg / 2], st[nwg * 9 / 10], st[nwg - 1]);
  printf("WG durations (us):     min %.2f p50 %.2f p90 %.2f max %.2f\n", du[0], du[nwg / 2], du[nwg * 9 / 10], du[nwg - 1]);
  printf("grid span (us): %.2f\n", rt(g1 - g0));
  return 0;
}
