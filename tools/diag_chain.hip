// Diagnostic build (not part of the library): phase accounting of the
// persistent faithful chain kernel at the bench shape (B=64, L=4693, T=1000).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -I <csrc> tools/diag_chain.hip <csrc>/encoder.hip <csrc>/head.hip -o tools/diag_chain
#define ERTD_CHAIN_STAMPS 1
#include "chain.hip"
#include <cstdio>
#include <vector>
#include <algorithm>
using namespace ertd;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 64, L = 4693, P = 29, T = argc > 2 ? atoi(argv[2]) : 1000;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2), R = argc > 3 ? atoi(argv[3]) : CHAIN_RING;
  std::vector<float> h((size_t)B * 14 * L + 1);
  for (size_t i = 0; i < h.size(); ++i) h[i] = ((i * 2654435761u) % 1000) / 1000.f;
  auto dev = [&](size_t n) { float* p; hipMalloc(&p, n * 4); hipMemcpy(p, h.data(), std::min(n, h.size()) * 4, hipMemcpyHostToDevice); return p; };
  for (auto& v : h) v = (v - 0.5f) * 0.1f;
  ertd_weights w{dev(32*42), dev(32), dev(64*96), dev(64), dev(128*64), dev(128), dev(128*128), dev(128),
                 dev(128*(P+256)), dev(128), dev(P*128), dev(P), P, 128};
  float* packed; CK(hipMalloc(&packed, PACKED_FLOATS_ALL * 4));
  CK(launch_pack(w, packed, 0));
  for (size_t i = 0; i < h.size(); ++i) h[i] = ((i * 2654435761u) % 1000) / 1000.f;
  float* cond = dev((size_t)B * 14 * L);
  std::vector<float> tabs(3 * T, 0.5f);
  float* tab = dev(3 * T); CK(hipMemcpy(tab, tabs.data(), 3 * T * 4, hipMemcpyHostToDevice));
  float* freq = dev(64); float* x = dev(B * P);
  float* ring = dev((size_t)R * B * S * 64);
  float* uring = dev((size_t)R * B * 128);
  float* Vc = dev((size_t)T * 128);
  const size_t zb = ((size_t)2 * R * B + 2 * B + 2) * SYNC_PAD * 4;
  char* zero; CK(hipMalloc(&zero, zb));
  FaithfulChainArgs fa{};
  fa.cond = cond; fa.cstride = 14LL * L; fa.L = L; fa.B = B; fa.S = S; fa.R = R;
  fa.n_run = T; fa.t_first = T - 1; fa.num_steps = T;
  fa.c1 = tab; fa.c2 = tab + T; fa.sigma = tab + 2 * T; fa.freq = freq; fa.noise = nullptr;
  fa.seed = 1; fa.member_offset = 0; fa.x = x; fa.part = ring;
  fa.cnt = (unsigned*)zero; fa.uflag = fa.cnt + (size_t)R * B * SYNC_PAD; fa.progress = fa.uflag + (size_t)R * B * SYNC_PAD;
  fa.claim = fa.progress + B * SYNC_PAD; fa.vready = fa.claim + B * SYNC_PAD; fa.status = fa.vready + SYNC_PAD;
  fa.uring = uring; fa.V = Vc;
  const int grid = faithful_chain_grid(B, S);
  printf("B=%d T=%d S=%d R=%d grid=%d (workers %d)\n", B, T, S, R, grid, grid - (B + CHAIN_MPB - 1) / CHAIN_MPB - 1);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    CK(launch_zero_words((unsigned*)zero, zb / 4, 0));
    hipEventRecord(e0, 0);
    CK(launch_faithful_chain(w, packed, fa, grid, 0));
    hipEventRecord(e1, 0);
    CK(hipEventSynchronize(e1));
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned st; CK(hipMemcpy(&st, fa.status, 4, hipMemcpyDeviceToHost));
    printf("rep %d: %.3f ms = %.2f us/step, status %u\n", rep, ms, ms * 1000.f / T, st);
  }
  static unsigned long long cst[8][1024][3], wacc[2048][8];
  CK(hipMemcpyFromSymbol(cst, HIP_SYMBOL(g_cst), sizeof(cst)));
  CK(hipMemcpyFromSymbol(wacc, HIP_SYMBOL(g_wacc), sizeof(wacc)));
  // chain block 0: wait vs compute per step (10 ns ticks)
  for (int b = 0; b < 2; ++b) {
    double wsum = 0, csum = 0, gsum = 0; int n = std::min(T, 1024);
    for (int i = 0; i < n; ++i) {
      wsum += (double)(cst[b][i][1] - cst[b][i][0]);
      csum += (double)(cst[b][i][2] - cst[b][i][1]);
      if (i) gsum += (double)(cst[b][i][0] - cst[b][i - 1][2]);
    }
    printf("chain b=%d: wait %.2f us/step, step body %.2f us/step, loop top %.2f us/step\n", b,
           wsum / n / 100, csum / n / 100, gsum / (n - 1) / 100);
    printf("   steps 0..9 wait(us):");
    for (int i = 0; i < 10; ++i) printf(" %.1f", (cst[b][i][1] - cst[b][i][0]) / 100.0);
    printf("\n   steps 500..509 wait(us):");
    for (int i = 500; i < 510 && i < n; ++i) printf(" %.1f", (cst[b][i][1] - cst[b][i][0]) / 100.0);
    printf("\n");
  }
  static unsigned long long pub[1024][3];
  CK(hipMemcpyFromSymbol(pub, HIP_SYMBOL(g_pub), sizeof(pub)));
  printf("step: chain0 wait start | u0 pub | chain0 ready (us rel. to chain0 step-0 wait start)\n");
  const unsigned long long z = cst[0][0][0];
  auto rl = [&](unsigned long long v) { return ((double)v - (double)z) / 100.0; };
  for (int i : {0, 1, 2, 3, 4, 5, 6, 7, 8, 100, 101, 102, 103, 104, 500, 501, 502, 503, 504, 505, 506, 507, 508, 509})
    if (i < T) printf("  %4d: %9.1f %9.1f %9.1f\n", i, rl(cst[0][i][0]), rl(pub[i][1]), rl(cst[0][i][1]));
  static unsigned long long it[4096][4];
  CK(hipMemcpyFromSymbol(it, HIP_SYMBOL(g_item), sizeof(it)));
  printf("member 0 items around step 100 (us rel. chain0 step-0 wait start): item step strip | start poll-done strip-done pub | chain0 step(i) wait-start ready end\n");
  const int NPS = (S + CHAIN_SPI - 1) / CHAIN_SPI;  // work items per step
  for (int k = NPS * 100; k < NPS * 104; ++k) {
    const int i = k / NPS;
    printf("  %5d %4d %2d | %9.1f %9.1f %9.1f %9.1f | %9.1f %9.1f %9.1f\n", k, i, (k % NPS) * CHAIN_SPI, rl(it[k][0]), rl(it[k][1]), rl(it[k][2]), rl(it[k][3]),
           rl(cst[0][i][0]), rl(cst[0][i][1]), rl(cst[0][i][2]));
  }
  double tot[8] = {}; int nw = grid - (B + CHAIN_MPB - 1) / CHAIN_MPB - 1;
  for (int k = 0; k < nw && k < 2048; ++k) for (int j = 0; j < 8; ++j) tot[j] += wacc[k][j];
  const double items = tot[5];
  printf("workers: items %.0f (%.1f/worker), last-arrivals %.0f, progress polls %.0f\n", items, items / nw, tot[6], tot[0]);
  printf("  per work item (%d strips): wait %.2f us, strip %.2f us, publish %.2f us; per last arrival cond row %.2f us\n", CHAIN_SPI,
         tot[1] / items / 100, tot[2] / items / 100, tot[3] / items / 100, tot[4] / std::max(1.0, tot[6]) / 100);
  printf("  worker span avg %.2f ms\n", tot[7] / nw / 1e5);
  return 0;
}
