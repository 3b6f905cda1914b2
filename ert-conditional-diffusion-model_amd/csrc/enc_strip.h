// fp32 strip body of the condition encoder (see encoder.hip for the
// decomposition), shared by enc_fp32_kernel and the persistent faithful chain
// kernel (chain.hip).  Header-only.
#pragma once
#include "ertd_common.h"

namespace ertd {

// The cond image is dead once conv1's MFMAs have run, so the conv1 output
// images alias it: 17.9 KB per workgroup -> 8 workgroups (32 waves) per CU.
#ifndef ERTD_ENC_ABLATE
#define ERTD_ENC_ABLATE 0  // diagnostic builds only (tools/diag_enc.hip): bit mask of skipped phases
#endif

struct EncSmem {
  union {
    float X[4][CIN][XS];  // 4-phase cond image (15,232 B)
    struct {
      float E[C1][HS];    // conv1 output, even p (8,704 B)
      float O[C1][HS];    // conv1 output, odd p  (8,704 B) -- must follow E
    };
  };
  float red[2][C2];       // q-tile partial pool sums
};

template <int PAR>
__device__ __forceinline__ void conv1_tile(f32x16& acc, const float (&a1)[STEPS1], const float* xb) {
#pragma unroll
  for (int s = 0; s < STEPS1; ++s) {
    const int cp = s / 3, kk = s % 3;
    // even p=2m taps cond 4j0-3+4m+kk -> X[kk][c][m]
    // odd  p=2m+1 taps 4j0-1+4m+kk   -> X[2][c][m], X[3][c][m], X[0][c][m+1]
    const int arr = PAR == 0 ? kk : (kk == 2 ? 0 : kk + 2);
    const int add = (PAR == 1 && kk == 2) ? 1 : 0;
    const float bv = xb[(arr * CIN + cp) * XS + add];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], bv, acc, 0, 0, 0);
  }
}

// One strip (member b, conv2 outputs [strip*J, strip*J + J)) by the calling
// 256-thread workgroup: leaves the 64 channel sums in sm.red[0][c] + sm.red[1][c]
// (after a closing barrier).  tid = threadIdx.x (a persistent caller passes an
// opaque copy so the per-lane addresses are not hoisted out of its item loop).
// The training forward (train.hip enc_train_kernel) runs the same body on the
// raw weights and also stores the activations its backward reads.
__device__ __forceinline__ void enc_strip_fp32(EncSmem& sm, const float* __restrict__ packed,
                                               const float* __restrict__ b1,
                                               const float* __restrict__ b2,
                                               const float* __restrict__ cond, long long cstride,
                                               int L, int L1, int L2, int b, int crow, int strip,
                                               int tid) {
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int j0 = strip * J;

  float a1[STEPS1];
#pragma unroll
  for (int s = 0; s < STEPS1; ++s) a1[s] = packed[PACK_W1 + s * 64 + lane];

  // ---- stage cond[b][:, 4j0-3 : 4j0-3+260] into the 4-phase image (zero padded)
  const float* cb = cond + (long long)crow * cstride;   // crow: b, or b % ncond
  if constexpr ((ERTD_ENC_ABLATE & 1) != 0) {
    for (int c = 0; c < CIN; ++c) sm.X[tid & 3][c][tid >> 2] = (float)(c + b);
  } else {
    stage_cond(sm.X, cb, L, 4 * j0 - 3, tid, [](float v) { return v; });
  }
  __syncthreads();

  // ---- conv1 + bias + ReLU -> E / O (never leaves LDS; aliases X)
  {
    const int par = wave >> 1, mt = wave & 1;
    const int m = mt * 32 + l32;
    f32x16 acc = {};
    const float* xb = &sm.X[0][0][0] + 7 * h * XS + m;
    if constexpr ((ERTD_ENC_ABLATE & 2) != 0) {
      for (int r = 0; r < 16; ++r) acc[r] = xb[r];
    } else {
      if (par == 0) conv1_tile<0>(acc, a1, xb);
      else conv1_tile<1>(acc, a1, xb);
    }
    __syncthreads();  // every wave has read X: the images may now overwrite it
    if (tid < C1) sm.E[tid][64] = 0.f;  // read only by the pad row q=63
    float* dst = par ? &sm.O[0][0] : &sm.E[0][0];
    const int i = 2 * j0 - 1 + 2 * m + par;       // global conv1 position
    const bool valid = (i >= 0) && (i < L1);      // outside -> conv2's zero padding
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float v = fmaxf(acc[r] + b1[o], 0.f);
      dst[o * HS + m] = valid ? v : 0.f;
    }
  }
  __syncthreads();
  // ---- conv2 + bias + ReLU + masked column sum
  {
    const int qt = wave & 1, ot = wave >> 1;
    const int q = qt * 32 + l32;
    float w2r[STEPS2];
#pragma unroll
    for (int s = 0; s < STEPS2; ++s)
      w2r[s] = (ERTD_ENC_ABLATE & 8) ? (float)(s * lane) : packed[PACK_W2 + (ot * STEPS2 + s) * 64 + lane];
    const float* eb = &sm.E[0][0] + 16 * h * HS + q;
    f32x16 acc = {};
    if constexpr ((ERTD_ENC_ABLATE & 4) != 0) {
      for (int r = 0; r < 16; ++r) acc[r] = eb[r * HS] + w2r[r];
    } else {
#pragma unroll
      for (int s = 0; s < STEPS2; ++s) {
        const int cp = s / 3, kk = s % 3;
        const int off = (kk == 1 ? C1 * HS : 0) + cp * HS + (kk == 2 ? 1 : 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(eb[off], w2r[s], acc, 0, 0, 0);
      }
    }
    const int o = ot * 32 + l32;
    const float bias = b2[o];
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const bool valid = (qq < J) && (j0 + qq < L2);
      const float z = acc[r] + bias;
      const float v = fmaxf(z, 0.f);
      sum += valid ? v : 0.f;
    }
    sum += __shfl_xor(sum, 32);
    if (h == 0) sm.red[qt][o] = sum;
  }
  __syncthreads();
}

}  // namespace ertd
