// Fused condition encoder for gfx950:
//   Conv1d(14->32,k3,s2,p1) -> ReLU -> Conv1d(32->64,k3,s2,p1) -> ReLU -> partial
//   average-pool sums            (ERT_Conditional_Diffusion.py:133-138)
// The pool finish + Linear(64->128) + ReLU (:138-141) run in head.hip, which
// reduces the per-strip partial sums in a fixed order (deterministic for any
// grid).
//
// Work decomposition: one 256-thread workgroup (4 waves) per (member, strip of
// J=63 conv2 outputs).  Both convolutions are implicit GEMMs on the fp32-input
// MFMA v_mfma_f32_32x32x2_f32 (exact fp32 fma chains, 64 FLOP/clk/SIMD):
//   conv1:  D1[o=32][m]  = W1[o][k=42]  x X[k][m]      4 tiles: {even,odd} p x 2 m-tiles
//   conv2:  D2[q][o=64]  = A2[q][k=96]  x W2^T[k][o]   4 tiles: 2 q-tiles x 2 o-tiles
// conv1 outputs never leave LDS.  The cond strip is staged as a 4-phase image
// X[r][c][m] = cond[c][4*j0-3+4m+r] and the conv1 output as even/odd images
// E[c][m]=h1(p=2m), O[c][m]=h1(p=2m+1), so every stride-2 tap becomes a
// unit-stride, bank-conflict-free ds_read_b32 with a compile-time offset.
// The k-order inside each MFMA splits channels between the two half-waves
// (lanes 0-31: channels c, lanes 32-63: channels c+7 / c+16), which keeps the
// per-step LDS offset an immediate.
#include "enc_strip.h"

namespace ertd {

// ---------------------------------------------------------------------------
// Weight packing: fragment-order copies of the conv weights plus k-major
// (transposed) copies of the three dense layers the head streams.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pack_kernel(ertd_weights w, float* __restrict__ packed) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < PACK_W2) {  // W1f[s][lane]
    const int s = idx >> 6, l = idx & 63;
    const int o = l & 31, c = s / 3 + 7 * (l >> 5), kk = s % 3;
    packed[idx] = w.enc0_w[(o * CIN + c) * 3 + kk];
  } else if (idx < PACK_FLOATS) {  // W2f[ot][s][lane]
    const int j = idx - PACK_W2;
    const int ot = j / (STEPS2 * 64), r = j % (STEPS2 * 64);
    const int s = r >> 6, l = r & 63;
    const int o = ot * 32 + (l & 31), c = s / 3 + 16 * (l >> 5), kk = s % 3;
    packed[idx] = w.enc2_w[(o * C1 + c) * 3 + kk];
  } else if (idx < PACK_TOTAL) {  // bf16 fragments (see enc_bf16 below)
    const int j = idx - PACKH_OFF;       // float index -> 2 bf16 each
    const int frag = j >> 2, pair = j & 3;  // frag = (step, lane), 4 floats = 8 bf16
    const int l = frag & 63, st = frag >> 6;
    unsigned short hv[2];
    for (int e = 0; e < 2; ++e) {
      const int kk8 = pair * 2 + e;          // element 0..7 of the lane's fragment
      float v = 0.f;
      if (st < PACKH_W1_STEPS) {             // conv1: A = W1[o][k], k = 16*st + 8*(l>>5) + kk8
        const int k = 16 * st + 8 * (l >> 5) + kk8;
        const int o = l & 31;
        if (k < K1) v = w.enc0_w[o * K1 + k];
      } else {                               // conv2: B = W2^T[k][o]
        const int st2 = st - PACKH_W1_STEPS;
        const int ot = st2 / PACKH_W2_STEPS, s2 = st2 % PACKH_W2_STEPS;
        const int k = 16 * s2 + 8 * (l >> 5) + kk8;
        const int o = ot * 32 + (l & 31);
        v = w.enc2_w[o * K2 + k];
      }
      // round-to-nearest-even f32 -> bf16 (inputs are finite weights)
      const uint32_t u = __float_as_uint(v);
      hv[e] = (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
    }
    packed[idx] = __uint_as_float((uint32_t)hv[0] | ((uint32_t)hv[1] << 16));
  }
}

// k-major copies of condition_encoder.6 / time_embed.0 / mlp.0 weights:
// WT[k][j] = W[j][k], so a thread per output j streams coalesced rows.
__global__ __launch_bounds__(256) void pack_dense_kernel(ertd_weights w, float* __restrict__ packed) {
  const int P = w.param_dim;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int n3 = C2 * H, nt = H * H, n0 = (P + 2 * H) * H;
  float* W3T = packed + PACK_TOTAL;
  float* WtT = W3T + n3;
  float* W0T = WtT + nt;
  if (idx < n3) {
    const int k = idx / H, j = idx % H;
    W3T[idx] = w.enc6_w[j * C2 + k];
  } else if (idx < n3 + nt) {
    const int i = idx - n3, k = i / H, j = i % H;
    WtT[i] = w.time_w[j * H + k];
  } else if (idx < n3 + nt + n0) {
    const int i = idx - n3 - nt, k = i / H, j = i % H;
    W0T[i] = w.mlp0_w[j * (P + 2 * H) + k];
  }
}

__global__ __launch_bounds__(256) void pack_w2b_kernel(ertd_weights w, float* __restrict__ packed) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= W2B_FLOATS) {
    const int i = idx - W2B_FLOATS;
    if (i < W2F_FLOATS) {
      const int k = i >> 6, l = i & 63, o = l >> 1;
      packed[PACK_W2F + i] = o < w.param_dim ? w.mlp2_w[o * H + 64 * (l & 1) + k] : 0.f;
    } else if (i < W2F_FLOATS + W0XR_FLOATS) {
      const int r = i - W2F_FLOATS, jj = r / W0XR_PITCH, k = r % W0XR_PITCH;
      packed[PACK_W0XR + r] = k < w.param_dim ? w.mlp0_w[jj * (w.param_dim + 2 * H) + k] : 0.f;
    } else if (i < W2F_FLOATS + W0XR_FLOATS + W2L_FLOATS) {
      const int r = i - W2F_FLOATS - W0XR_FLOATS, l = r / W2L_PITCH, k = r % W2L_PITCH;
      const int o = l >> 1;
      packed[PACK_W2L + r] =
          (o < w.param_dim && k < H / 2) ? w.mlp2_w[o * H + 64 * (l & 1) + k] : 0.f;
    }
    return;
  }
  const int kk = idx / (32 * 64), r = idx % (32 * 64);
  const int st = r >> 6, l = r & 63;
  const int o = 2 * st + (l >> 5), c = l & 31;
  packed[PACK_W2B + idx] = w.enc2_w[(o * C1 + c) * 3 + kk];
}

// The U-Net train step's condition encoder (unet_train.hip): its train-mode
// forward / backward (train.hip) read the conv weights in their own layout, so
// the "packing" is a copy of the two tensors, W1 (32,14,3) at packed[0] and
// W2 (64,32,3) at packed[ENC_RAW_W2], taken once per tape: a second forward
// before that tape's backward must not change what the backward reads.
__global__ __launch_bounds__(256) void copy_encoder_convs_kernel(const float* __restrict__ w0,
                                                                 const float* __restrict__ w2,
                                                                 float* __restrict__ packed) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < C1 * K1) packed[i] = w0[i];
  else if (i < C1 * K1 + C2 * K2) packed[i] = w2[i - C1 * K1];
}

hipError_t launch_pack_encoder_convs(const float* w0, const float* w2, float* packed, hipStream_t s) {
  copy_encoder_convs_kernel<<<(C1 * K1 + C2 * K2 + 255) / 256, 256, 0, s>>>(w0, w2, packed);
  return hipGetLastError();
}

hipError_t launch_pack(const ertd_weights& w, float* packed, hipStream_t s) {
  pack_kernel<<<(PACK_TOTAL + 255) / 256, 256, 0, s>>>(w, packed);
  const int n = C2 * H + H * H + (w.param_dim + 2 * H) * H;
  pack_dense_kernel<<<(n + 255) / 256, 256, 0, s>>>(w, packed);
  pack_w2b_kernel<<<(W2B_FLOATS + W2F_FLOATS + W0XR_FLOATS + W2L_FLOATS + 255) / 256, 256, 0,
                    s>>>(w, packed);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// fp32 strip kernel (body: enc_strip.h)
// ---------------------------------------------------------------------------
// Optionally (tr.V != null) block number nstrip computes the time row v(tr.t)
// for the faithful sampler's next head launch (time_row_lean: few registers).
__global__ __launch_bounds__(256) void enc_fp32_kernel(const float* __restrict__ packed,
                                                       const float* __restrict__ b1,
                                                       const float* __restrict__ b2,
                                                       const float* __restrict__ cond,
                                                       long long cstride, int L, int L1, int L2,
                                                       int S, float* __restrict__ partial,
                                                       int nstrip, TimeRowArgs tr, int ncond) {
  __shared__ EncSmem sm;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= nstrip) {
    float* f = &sm.X[0][0][0];  // e[128] | te[128] | part[2][128]
    time_row_lean(tr.w, packed, tr.freq, tr.t, tr.V + (size_t)tr.t * H, f, f + H,
                  reinterpret_cast<float(*)[H]>(f + 2 * H), tid);
    return;
  }
  const int b = blockIdx.x / S, strip = blockIdx.x - b * S;
  enc_strip_fp32(sm, packed, b1, b2, cond, cstride, L, L1, L2, b, cond_row(b, ncond), strip, tid);
  if (tid < C2) partial[((size_t)b * S + strip) * C2 + tid] = sm.red[0][tid] + sm.red[1][tid];
  if (tr.V) {
    // Warm this XCD's L2 with a slice of the weights the next head_step reads
    // (W3T, the cond columns of W0T, the two step images: ~134 KB).  Blocks
    // b, b+8, ... share an XCD under the observed round-robin placement (a
    // speed hint only); together each XCD group touches every 64-B line.
    constexpr int L_W3 = C2 * H / 16, L_W0C = H * H / 16;
    constexpr int L_IMG = (W0XR_FLOATS + W2L_FLOATS) / 16;
    const int total = L_W3 + L_W0C + L_IMG;
    const int grp = blockIdx.x >> 3, ngrp = (nstrip + 7) >> 3;
    const int per = (total + ngrp - 1) / ngrp;
    if (tid < per) {
      const int line = grp * per + tid;
      if (line < total) {
        const float* src;
        if (line < L_W3) src = packed + PACK_TOTAL + line * 16;
        else if (line < L_W3 + L_W0C)
          src = packed + PACK_TOTAL + C2 * H + H * H + (size_t)(tr.w.param_dim + H) * H +
                (line - L_W3) * 16;
        else src = packed + PACK_W0XR + (line - L_W3 - L_W0C) * 16;  // W2L follows W0XR
        const float v = *src;  // plain load: allocates the line in this XCD's L2
        asm volatile("" ::"v"(v));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// bf16-operand strip kernel (R3/R5 configs): same decomposition on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation.  k-order: natural im2col
// order k = c*3 + kk (conv1 padded 42 -> 48).  The staged images are bf16.
// ---------------------------------------------------------------------------
using bf16x8 = __attribute__((ext_vector_type(8))) short;

__device__ __forceinline__ unsigned short f2bf(float v) {
  const uint32_t u = __float_as_uint(v);
  return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

struct EncSmemH {
  union {
    unsigned short X[4][CIN][XS];  // 4-phase cond image, bf16
    struct {
      unsigned short E[C1][HS];
      unsigned short O[C1][HS];
    };
  };
  float red[2][C2];
};

__global__ __launch_bounds__(256) void enc_bf16_kernel(const float* __restrict__ packed,
                                                       const float* __restrict__ b1,
                                                       const float* __restrict__ b2,
                                                       const float* __restrict__ cond,
                                                       long long cstride, int L, int L1, int L2,
                                                       int S,
                                                       float* __restrict__ partial, int ncond) {
  __shared__ EncSmemH sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.x / S, strip = blockIdx.x - b * S;
  const int j0 = strip * J;
  const bf16x8* ph = reinterpret_cast<const bf16x8*>(packed + PACKH_OFF);

  const float* cb = cond + (long long)cond_row(b, ncond) * cstride;
  stage_cond(sm.X, cb, L, 4 * j0 - 3, tid, [](float v) { return f2bf(v); });
  __syncthreads();

  // conv1: A = W1 (row o = l32, k = 16*st + 8h + e), B = X[k][m]
  {
    const int par = wave >> 1, mt = wave & 1;
    const int m = mt * 32 + l32;
    f32x16 acc = {};
#pragma unroll
    for (int st = 0; st < PACKH_W1_STEPS; ++st) {
      const bf16x8 a = ph[st * 64 + lane];
      bf16x8 bv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 16 * st + 8 * h + e;  // runtime in h only
        const int c = k / 3, kk = k - 3 * (k / 3);
        const int arr = par == 0 ? kk : (kk == 2 ? 0 : kk + 2);
        const int add = (par == 1 && kk == 2) ? 1 : 0;
        bv[e] = (k < K1) ? (short)sm.X[arr][c][m + add] : (short)0;
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, acc, 0, 0, 0);
    }
    __syncthreads();  // X fully consumed before the aliased images are written
    if (tid < C1) sm.E[tid][64] = 0;
    unsigned short* dst = par ? &sm.O[0][0] : &sm.E[0][0];
    const int i = 2 * j0 - 1 + 2 * m + par;
    const bool valid = (i >= 0) && (i < L1);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float v = fmaxf(acc[r] + b1[o], 0.f);
      dst[o * HS + m] = valid ? f2bf(v) : (unsigned short)0;
    }
  }
  __syncthreads();

  // conv2: A = im2col^T[q][k], B = W2^T[k][o], k = 16*s2 + 8h + e = c*3+kk
  {
    const int qt = wave & 1, ot = wave >> 1;
    const int q = qt * 32 + l32;
    f32x16 acc = {};
#pragma unroll
    for (int s2 = 0; s2 < PACKH_W2_STEPS; ++s2) {
      const bf16x8 bw = ph[(PACKH_W1_STEPS + ot * PACKH_W2_STEPS + s2) * 64 + lane];
      bf16x8 av;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = 16 * s2 + 8 * h + e;
        const int c = k / 3, kk = k - 3 * (k / 3);
        const unsigned short* src = kk == 1 ? &sm.O[c][q] : &sm.E[c][q + (kk == 2 ? 1 : 0)];
        av[e] = (short)*src;
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bw, acc, 0, 0, 0);
    }
    const int o = ot * 32 + l32;
    const float bias = b2[o];
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const bool valid = (qq < J) && (j0 + qq < L2);
      const float v = fmaxf(acc[r] + bias, 0.f);
      sum += valid ? v : 0.f;
    }
    sum += __shfl_xor(sum, 32);
    if (h == 0) sm.red[qt][o] = sum;
  }
  __syncthreads();
  if (tid < C2) partial[((size_t)b * S + strip) * C2 + tid] = sm.red[0][tid] + sm.red[1][tid];
}

hipError_t launch_encoder_strips(const float* packed, const float* b1, const float* b2,
                                 const float* cond, long long cstride, int B, int L, int precision,
                                 float* partial, hipStream_t s, int ncond) {
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  const dim3 grid((unsigned)(B * S));
  if (precision == ERTD_PREC_BF16)
    enc_bf16_kernel<<<grid, 256, 0, s>>>(packed, b1, b2, cond, cstride, L, L1, L2, S, partial, ncond);
  else
    enc_fp32_kernel<<<grid, 256, 0, s>>>(packed, b1, b2, cond, cstride, L, L1, L2, S, partial, B * S,
                                         TimeRowArgs{}, ncond);
  return hipGetLastError();
}

hipError_t launch_encoder_strips_t(const float* packed, const float* b1, const float* b2,
                                   const float* cond, long long cstride, int B, int L,
                                   int precision, float* partial, const TimeRowArgs& tr,
                                   hipStream_t s, int ncond) {
  if (precision == ERTD_PREC_BF16) {  // bf16 strips + the time row as its own launch
    hipError_t e = launch_encoder_strips(packed, b1, b2, cond, cstride, B, L, precision, partial, s, ncond);
    if (e != hipSuccess) return e;
    return launch_time_table(tr.w, packed, tr.freq, tr.t, 1, tr.V, s);
  }
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  enc_fp32_kernel<<<dim3((unsigned)(B * S + 1)), 256, 0, s>>>(packed, b1, b2, cond, cstride, L, L1,
                                                               L2, S, partial, B * S, tr, ncond);
  return hipGetLastError();
}

}  // namespace ertd
