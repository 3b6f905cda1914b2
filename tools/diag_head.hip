// Diagnostic build (not part of the library): phase timing of head_kernel and
// enc_fp32_kernel for the R2 shape with s_memrealtime stamps (100 MHz).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I <csrc> tools/diag_head.hip
#define ERTD_HEAD_STAMPS 1
#include "head.hip"
#include "encoder.hip"
#include <cstdio>
#include <vector>
#include <algorithm>
using namespace ertd;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
  const int B = 64, L = 4693, P = 29, T = 1000;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  std::vector<float> h(1 << 23);  // >= B*14*L floats
  for (size_t i = 0; i < h.size(); ++i) h[i] = ((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  auto dev = [&](size_t n) { float* p; hipMalloc(&p, n * 4); hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice); return p; };
  ertd_weights w{dev(32*42), dev(32), dev(64*96), dev(64), dev(128*64), dev(128), dev(128*128), dev(128),
                 dev(128*(P+256)), dev(128), dev(P*128), dev(P), P, 128};
  float* packed; CK(hipMalloc(&packed, PACKED_FLOATS_ALL * 4));
  CK(launch_pack(w, packed, 0));
  float* cond = dev((size_t)B * 14 * L);
  for (size_t i = 0; i < (size_t)B*14*L; i += 1) {}  // values in [-0.5,0.5)
  float *partial = dev((size_t)B * S * 64), *x = dev(B * P), *tabs = dev(128 * T), *freq = dev(64);
  HeadArgs a{};
  a.partial = partial; a.S = S; a.L2 = L2; a.freq = freq; a.x_in = x; a.c1 = tabs; a.c2 = tabs + T;
  a.sigma = tabs + 2 * T; a.num_steps = T; a.seed = 1; a.B = B; a.x_out = x;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 30; ++it) {
    a.t_scalar = T - 1 - it;
    CK(launch_encoder_strips(packed, w.enc0_b, w.enc2_b, cond, 14LL * L, B, L, 0, partial, 0));
    CK(launch_head_step(w, packed, a, tabs, 0));
  }
  CK(hipDeviceSynchronize());
  // time each kernel alone, back to back
  for (int which = 0; which < 2; ++which) {
    hipEventRecord(e0, 0);
    for (int it = 0; it < 100; ++it) {
      if (which == 0) launch_encoder_strips(packed, w.enc0_b, w.enc2_b, cond, 14LL * L, B, L, 0, partial, 0);
      else launch_head_step(w, packed, a, tabs, 0);
    }
    hipEventRecord(e1, 0); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%s: %.2f us per launch (100 back-to-back)\n", which ? "head" : "encoder", ms * 10.f);
  }
  unsigned long long st[1024][2][8];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_head_stamps), sizeof(st)));
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < B; ++b) t0 = std::min(t0, st[b][0][0]);
  const char* names[8] = {"start", "loads+pool barrier", "cond row done", "w barrier", "x bcast", "eps", "update", "-"};
  for (int ph = 0; ph < 7; ++ph) {
    double mn = 1e30, mx = 0, avg = 0; int n = 0;
    const int wv = 0;
    for (int b = 0; b < B; ++b) { double v = (st[b][wv][ph] - t0) / 100.0; mn = std::min(mn, v); mx = std::max(mx, v); avg += v; ++n; }
    printf("phase %d %-26s wave0: min %.2f avg %.2f max %.2f us (from first block start)\n", ph, names[ph], mn, avg / n, mx);
  }
  return 0;
}
