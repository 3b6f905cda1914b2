// One-output-channel 3x3 convolution: the U-Net's conv_out (GroupNorm -> SiLU
// -> conv3x3 -> 1 channel, the predicted noise).
//
// The MFMA kernels (unet_conv.hip, unet_conv_bf16.hip) tile 64 output channels
// per wave, so a Cout = 1 layer there runs a whole 64-channel tile for one
// useful row (measured 187 us per U2 step, 1.6 TFLOP/s).  Here one thread owns
// one output pixel: the workgroup stages 16 input channels x (rows + halo) in
// LDS -- GroupNorm + SiLU applied on the way and the zero padding written after
// the transform, exactly as the MFMA kernels stage -- and every thread runs the
// 16 x 9 taps as an fp32 fma chain.  The input is read once (no output-channel
// tiles), so the layer is bounded by one pass over its input.
//
// Weights are gathered once per workgroup from the MFMA packing the model
// already holds (fp32 [co_tile32][chunk][step pair][lane][2] or bf16
// [co_tile32][chunk][step][lane][8]); the bf16 variant also rounds the staged
// activation to bf16 (RNE), so its products equal the bf16 MFMA's.
#include "unet.h"

namespace ertd {
namespace unet {

namespace {

constexpr int OCC = 16;  // input channels per staged chunk

__device__ __forceinline__ float round_bf16(float v) {  // RNE, finite v
  const uint32_t u = __float_as_uint(v);
  return __uint_as_float(((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16) << 16);
}

// W[0][ci][tap] in the fp32 packing (4-channel chunks, 18 steps, lane half = ci/2 % 2)
__device__ __forceinline__ float packed_w_f32(const float* w, int ci, int tap) {
  const int s = (ci & 1) * 9 + tap;
  return w[((size_t)(ci >> 2) * 9 + (s >> 1)) * 128 + ((ci & 3) >> 1) * 64 + (s & 1)];
}

// W[0][ci][tap] in the bf16 packing (16-channel chunks, step = tap, k = 8*half + j)
__device__ __forceinline__ float packed_w_bf16(const float* w, int ci, int tap) {
  const unsigned short* p = reinterpret_cast<const unsigned short*>(w);
  const unsigned short v = p[((size_t)(ci >> 4) * 9 + tap) * 512 + ((ci >> 3) & 1) * 256 + (ci & 7)];
  return __uint_as_float((unsigned)v << 16);
}

template <int WO>
struct OutGeom {
  static constexpr int ROWS = NTHR / WO;  // output rows per workgroup (one pixel per thread)
  static constexpr int IR = ROWS + 2;
  static constexpr int IP = WO + 2;       // zero column each side
  static constexpr int CSZ = IR * IP;
  static_assert(NTHR % WO == 0, "whole output rows per workgroup");
};

template <int ACT, int WO, bool BF>
__global__ __launch_bounds__(NTHR) void conv_out_kernel(ConvArgs a) {
  using G = OutGeom<WO>;
  extern __shared__ __attribute__((aligned(16))) float smo[];
  const int Cin = a.Cin, Ca = a.Ca;
  float* img = smo;                                   // [OCC][IR][IP]
  float* wl = smo + OCC * G::CSZ;                     // [Cin][9]
  float2* gtab = reinterpret_cast<float2*>(wl + ((Cin * 9 + 1) & ~1));  // [Cin]
  const int tid = threadIdx.x, b = blockIdx.z;
  const int oy0 = blockIdx.x * G::ROWS;
  constexpr size_t plane = (size_t)WO * WO;

  for (int i = tid; i < Cin * 9; i += NTHR) {
    const int ci = i / 9, tap = i - ci * 9;
    wl[i] = BF ? packed_w_bf16(a.wpk, ci, tap) : packed_w_f32(a.wpk, ci, tap);
  }
  if constexpr (ACT != ACT_NONE) {
    for (int c = tid; c < Cin; c += NTHR) gtab[c] = a.gn[(size_t)b * Cin + c];
  }
  for (int r = tid; r < OCC * G::IR; r += NTHR) {
    img[r * G::IP] = 0.f;
    img[r * G::IP + G::IP - 1] = 0.f;
  }

  const int py = tid / WO, px = tid - py * WO;
  float acc = 0.f;
  for (int c0 = 0; c0 < Cin; c0 += OCC) {
    __syncthreads();  // tables visible / previous chunk consumed
    constexpr int NE = (OCC * G::IR * WO + NTHR - 1) / NTHR;   // staged elements per thread
#pragma unroll
    for (int k = 0; k < NE; ++k) {
      const int e = tid + k * NTHR;
      if (OCC * G::IR * WO % NTHR != 0 && e >= OCC * G::IR * WO) break;
      const int c = e / (G::IR * WO), rem = e - c * (G::IR * WO);
      const int r = rem / WO, x = rem - r * WO;
      const int cg = c0 + c, iy = oy0 - 1 + r;
      float v = 0.f;
      if (cg < Cin && iy >= 0 && iy < WO) {
        const float* src = cg < Ca ? a.srcA + ((size_t)b * Ca + cg) * plane
                                   : a.srcB + ((size_t)b * a.Cb + (cg - Ca)) * plane;
        v = src[iy * WO + x];
        if constexpr (ACT != ACT_NONE) {
          const float2 g = gtab[cg];
          v = fmaf(v, g.x, g.y);
          if constexpr (ACT == ACT_GN_SILU) v = v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
        }
        if constexpr (BF) v = round_bf16(v);
      }
      img[(c * G::IR + r) * G::IP + x + 1] = v;
    }
    __syncthreads();
    const int nc = Cin - c0 < OCC ? Cin - c0 : OCC;
    for (int c = 0; c < nc; ++c) {
      const float* ip = img + (c * G::IR + py) * G::IP + px;
      const float* wp = wl + (c0 + c) * 9;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc = fmaf(wp[ky * 3 + kx], ip[ky * G::IP + kx], acc);
    }
  }

  // epilogue in the MFMA kernels' op order: conv + bias, + emb, + residual
  const size_t o = (size_t)b * plane + (size_t)(oy0 + py) * WO + px;
  float v = acc + a.bias[0];
  if (a.ebias) v = v + a.ebias[(size_t)b * a.eb_stride];
  if (a.res) v = v + a.res[o];
  a.out[o] = v;
}

template <int ACT, int WO, bool BF>
hipError_t launch_co(const ConvArgs& a, int B, hipStream_t s) {
  using G = OutGeom<WO>;
  const size_t lds = ((size_t)OCC * G::CSZ + (((size_t)a.Cin * 9 + 1) & ~(size_t)1)) * sizeof(float) +
                     (size_t)a.Cin * sizeof(float2);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)conv_out_kernel<ACT, WO, BF>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((unsigned)(WO / G::ROWS), 1u, (unsigned)B);
  conv_out_kernel<ACT, WO, BF><<<grid, NTHR, lds, s>>>(a);
  return hipGetLastError();
}

template <int ACT, bool BF>
hipError_t launch_co_w(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 16: return launch_co<ACT, 16, BF>(a, B, s);
    case 32: return launch_co<ACT, 32, BF>(a, B, s);
    case 64: return launch_co<ACT, 64, BF>(a, B, s);
    case 128: return launch_co<ACT, 128, BF>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_conv_out(int act, const ConvArgs& a, int B, bool bf16, hipStream_t s) {
  if (a.Cout != 1 || a.Ho != a.Wo || a.Hs != a.Ws || a.Ws != a.Wo || a.Cin != a.Ca + a.Cb)
    return hipErrorInvalidValue;
  if (act == ACT_GN_SILU) return bf16 ? launch_co_w<ACT_GN_SILU, true>(a, B, s)
                                      : launch_co_w<ACT_GN_SILU, false>(a, B, s);
  if (act == ACT_NONE) return bf16 ? launch_co_w<ACT_NONE, true>(a, B, s)
                                   : launch_co_w<ACT_NONE, false>(a, B, s);
  return hipErrorInvalidValue;
}

}  // namespace unet
}  // namespace ertd
