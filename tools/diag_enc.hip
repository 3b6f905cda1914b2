// Diagnostic build (not part of the library): enc_fp32_kernel launch time vs
// batch size, for ablation builds (-DERTD_ENC_ABLATE=mask, see encoder.hip).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -I <csrc> tools/diag_enc.hip
#include "head.hip"
#include "encoder.hip"
#include <cstdio>
#include <vector>
using namespace ertd;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
  const int BMAX = 128, L = 4693, P = 29;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  std::vector<float> h((size_t)BMAX * 14 * L);
  for (size_t i = 0; i < h.size(); ++i) h[i] = ((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  auto dev = [&](size_t n) { float* p; hipMalloc(&p, n * 4); hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice); return p; };
  ertd_weights w{dev(32*42), dev(32), dev(64*96), dev(64), dev(128*64), dev(128), dev(128*128), dev(128),
                 dev(128*(P+256)), dev(128), dev(P*128), dev(P), P, 128};
  float* packed; CK(hipMalloc(&packed, PACKED_FLOATS_ALL * 4));
  CK(launch_pack(w, packed, 0));
  float* cond = dev((size_t)BMAX * 14 * L);
  float* partial = dev((size_t)BMAX * S * 64);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int Bs[] = {1, 4, 14, 27, 40, 54, 64, 128};
  printf("ablate=%d\n", ERTD_ENC_ABLATE);
  for (int B : Bs) {
    for (int it = 0; it < 20; ++it)
      CK(launch_encoder_strips(packed, w.enc0_b, w.enc2_b, cond, 14LL * L, B, L, 0, partial, 0));
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(e0, 0);
      for (int it = 0; it < 200; ++it)
        launch_encoder_strips(packed, w.enc0_b, w.enc2_b, cond, 14LL * L, B, L, 0, partial, 0);
      hipEventRecord(e1, 0); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      best = std::min(best, ms * 5.f);
    }
    printf("  B=%4d blocks=%5d  %7.2f us/launch\n", B, B * S, best);
  }
  return 0;
}
