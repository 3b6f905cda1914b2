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
#include <cstdlib>

#include "unet.h"

namespace ertd {
namespace unet {

namespace {

__device__ __forceinline__ float round_bf16(float v) {  // RNE, finite v
  const uint32_t u = __float_as_uint(v);
  return __uint_as_float(((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16) << 16);
}

// W[0][ci][tap] in the fp32 packing (4-channel chunks, 18 steps, lane half = ci/2 % 2)
__device__ __forceinline__ float packed_w_f32(const float* w, int ci, int tap) {
  const int s = (ci & 1) * 9 + tap;
  return w[((size_t)(ci >> 2) * 9 + (s >> 1)) * 128 + ((ci & 3) >> 1) * 64 + (s & 1)];
}

// W[0][ci][tap] in the bf16 packing (16-channel chunks, step = tap, k = 8*half + j);
// split bf16: [chunk][hi | lo][9 steps], the weight is hi + lo
__device__ __forceinline__ float packed_w_bf16(const float* w, int ci, int tap, bool split) {
  const unsigned short* p = reinterpret_cast<const unsigned short*>(w);
  const size_t e = ((ci >> 3) & 1) * 256 + (ci & 7);
  if (!split) return __uint_as_float((unsigned)p[((size_t)(ci >> 4) * 9 + tap) * 512 + e] << 16);
  const float hi = __uint_as_float((unsigned)p[((size_t)(ci >> 4) * 18 + tap) * 512 + e] << 16);
  const float lo = __uint_as_float((unsigned)p[((size_t)(ci >> 4) * 18 + 9 + tap) * 512 + e] << 16);
  return hi + lo;
}

// Thread = 4 horizontally adjacent output pixels of one row; a workgroup owns
// ROWS whole rows (the whole image at W <= 32).  Staged rows: W + 8 floats,
// data at column 4 (16-B aligned float4 stores / loads), zero columns 3 and
// W + 4; the 3 taps of a kernel row read one float4 + two neighbours.
// NS channel groups: the workgroup is NS x NT threads, group g sweeps input
// channels [g Cq, (g + 1) Cq) (Cq = ceil(Cin / NS) rounded to OCC) through its
// own staging buffer, and the NS partial sums of a pixel are added in a fixed
// order at the end -- NS times the loads in flight per CU (one 4-wave
// workgroup per CU left the layer latency-bound: 42 us at U2 B=64)
template <int WO, int RWS, int NS>
struct OutGeom {
  static constexpr int TPR = WO / 4;                          // threads per output row
  static constexpr int ROWS = RWS;
  static constexpr int NT = TPR * ROWS;                       // threads per channel group
  static constexpr int IR = ROWS + 2;
  static constexpr int IP = WO + 8;
  static constexpr int CSZ = IR * IP;
  static constexpr int OCC = NS >= 4 ? 4 : 8;                 // channels per staged chunk
  static_assert(WO % ROWS == 0 && NT <= 256 && NT % 64 == 0, "whole output rows per workgroup");
};

template <int ACT, int WO, int RWS, int PK, int NS>
__global__ __launch_bounds__(1024) void conv_out_kernel(ConvArgs a) {
  constexpr bool BF = PK == PK_BF16;   // round the staged input to bf16
  using G = OutGeom<WO, RWS, NS>;
  constexpr int OCC = G::OCC;
  extern __shared__ __attribute__((aligned(16))) float smo[];
  const int Cin = a.Cin, Ca = a.Ca;
  const int tid = threadIdx.x, b = blockIdx.z;
  const int grp = tid / G::NT, tl = tid - grp * G::NT;
  float* img = smo + grp * OCC * G::CSZ;              // this group's [OCC][IR][IP]
  float* wl = smo + NS * OCC * G::CSZ;                // [Cin][9]
  float2* gtab = reinterpret_cast<float2*>(wl + ((Cin * 9 + 1) & ~1));  // [Cin]
  const int oy0 = blockIdx.x * G::ROWS;
  constexpr size_t plane = (size_t)WO * WO;
  const int cq = ((Cin + NS - 1) / NS + OCC - 1) / OCC * OCC;   // channels per group
  const int cbeg = grp * cq, cend = min(Cin, cbeg + cq);

  for (int i = tid; i < Cin * 9; i += NS * G::NT) {
    const int ci = i / 9, tap = i - ci * 9;
    wl[i] = PK == PK_F32 ? packed_w_f32(a.wpk, ci, tap) : packed_w_bf16(a.wpk, ci, tap, PK == PK_SPLIT);
  }
  if constexpr (ACT != ACT_NONE) {
    for (int c = tid; c < Cin; c += NS * G::NT) gtab[c] = a.gn[(size_t)b * Cin + c];
  }
  for (int r = tl; r < OCC * G::IR; r += G::NT) {
    img[r * G::IP + 3] = 0.f;
    img[r * G::IP + 4 + WO] = 0.f;
  }

  const int py = tl / G::TPR, px4 = tl - py * G::TPR;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // staging in two phases: the next chunk's float4 loads are issued into
  // registers before the current chunk's fma chains, so the global-load
  // latency hides behind them
  constexpr int NQ = OCC * G::IR * G::TPR;                   // float4 quads per chunk
  constexpr int NPT = (NQ + G::NT - 1) / G::NT;
  float4 raw[NPT];
  auto load = [&](int c0) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int e = tl + k * G::NT;
      const int c = e / (G::IR * G::TPR), rem = e - c * (G::IR * G::TPR);
      const int r = rem / G::TPR, q = rem - r * G::TPR;
      const int cg = c0 + c, iy = oy0 - 1 + r;
      raw[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < NQ && cg < cend && iy >= 0 && iy < WO) {
        const float* src = cg < Ca ? a.srcA + ((size_t)b * Ca + cg) * plane
                                   : a.srcB + ((size_t)b * a.Cb + (cg - Ca)) * plane;
        raw[k] = *reinterpret_cast<const float4*>(src + iy * WO + 4 * q);
      }
    }
  };
  auto stage = [&](int c0) {
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int e = tl + k * G::NT;
      if (e >= NQ) continue;
      const int c = e / (G::IR * G::TPR), rem = e - c * (G::IR * G::TPR);
      const int r = rem / G::TPR, q = rem - r * G::TPR;
      const int cg = c0 + c, iy = oy0 - 1 + r;
      float4 v = raw[k];
      if (cg < cend && iy >= 0 && iy < WO) {
        if constexpr (ACT != ACT_NONE) {
          const float2 g = gtab[cg];
          v.x = fmaf(v.x, g.x, g.y);
          v.y = fmaf(v.y, g.x, g.y);
          v.z = fmaf(v.z, g.x, g.y);
          v.w = fmaf(v.w, g.x, g.y);
          if constexpr (ACT == ACT_GN_SILU) {
            v.x = v.x * __builtin_amdgcn_rcpf(1.0f + __expf(-v.x));
            v.y = v.y * __builtin_amdgcn_rcpf(1.0f + __expf(-v.y));
            v.z = v.z * __builtin_amdgcn_rcpf(1.0f + __expf(-v.z));
            v.w = v.w * __builtin_amdgcn_rcpf(1.0f + __expf(-v.w));
          }
        }
        if constexpr (BF) {
          v.x = round_bf16(v.x);
          v.y = round_bf16(v.y);
          v.z = round_bf16(v.z);
          v.w = round_bf16(v.w);
        }
      }
      *reinterpret_cast<float4*>(img + (c * G::IR + r) * G::IP + 4 + 4 * q) = v;
    }
  };
  // every group runs the same number of chunks (workgroup-wide barriers); a
  // group past Cin stages zeros and skips the fma chains
  const int nchunk = cq / OCC;
  load(cbeg);
  for (int k = 0; k < nchunk; ++k) {
    const int c0 = cbeg + k * OCC;
    __syncthreads();  // tables visible / previous chunk consumed
    stage(c0);
    __syncthreads();
    if (k + 1 < nchunk) load(c0 + OCC);
    const int nc = cend - c0 < OCC ? cend - c0 : OCC;
    for (int c = 0; c < nc; ++c) {
      const float* wp = wl + (c0 + c) * 9;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const float* row = img + (c * G::IR + py + ky) * G::IP + 4 + 4 * px4;
        const float4 m = *reinterpret_cast<const float4*>(row);
        const float l = row[-1], rr = row[4];
        const float w0 = wp[ky * 3], w1 = wp[ky * 3 + 1], w2 = wp[ky * 3 + 2];
        // per output pixel the taps in the MFMA kernels' order (ky, kx)
        acc[0] = fmaf(w0, l, acc[0]);   acc[0] = fmaf(w1, m.x, acc[0]); acc[0] = fmaf(w2, m.y, acc[0]);
        acc[1] = fmaf(w0, m.x, acc[1]); acc[1] = fmaf(w1, m.y, acc[1]); acc[1] = fmaf(w2, m.z, acc[1]);
        acc[2] = fmaf(w0, m.y, acc[2]); acc[2] = fmaf(w1, m.z, acc[2]); acc[2] = fmaf(w2, m.w, acc[2]);
        acc[3] = fmaf(w0, m.z, acc[3]); acc[3] = fmaf(w1, m.w, acc[3]); acc[3] = fmaf(w2, rr, acc[3]);
      }
    }
  }
  if constexpr (NS > 1) {
    // the groups' partial sums through LDS (the staging buffers are free now),
    // added in a fixed order by group 0
    __syncthreads();
    float4* red = reinterpret_cast<float4*>(smo);
    red[grp * G::NT + tl] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    __syncthreads();
    if (grp != 0) return;
    float4 t[NS];
#pragma unroll
    for (int g2 = 0; g2 < NS; ++g2) t[g2] = red[g2 * G::NT + tl];
    if constexpr (NS == 2) {
      acc[0] = t[0].x + t[1].x; acc[1] = t[0].y + t[1].y; acc[2] = t[0].z + t[1].z; acc[3] = t[0].w + t[1].w;
    } else {
      acc[0] = (t[0].x + t[1].x) + (t[2].x + t[3].x);
      acc[1] = (t[0].y + t[1].y) + (t[2].y + t[3].y);
      acc[2] = (t[0].z + t[1].z) + (t[2].z + t[3].z);
      acc[3] = (t[0].w + t[1].w) + (t[2].w + t[3].w);
    }
  }

  // epilogue in the MFMA kernels' op order: conv + bias, + emb, + residual
  const size_t o = (size_t)b * plane + (size_t)(oy0 + py) * WO + 4 * px4;
  const float bb = a.bias ? a.bias[0] : 0.f;
  float4 v = make_float4(acc[0] + bb, acc[1] + bb, acc[2] + bb, acc[3] + bb);
  if (a.ebias) {
    const float e = a.ebias[(size_t)b * a.eb_stride];
    v.x = v.x + e; v.y = v.y + e; v.z = v.z + e; v.w = v.w + e;
  }
  if (a.res) {
    const float4 r = *reinterpret_cast<const float4*>(a.res + o);
    v.x = v.x + r.x; v.y = v.y + r.y; v.z = v.z + r.z; v.w = v.w + r.w;
  }
  *reinterpret_cast<float4*>(a.out + o) = v;
}

// W = 64 (U2 / U3): one wave per 64-pixel image row strip of CO64_R rows,
// lane = column, the column neighbours by full-wave DPP shifts (zero fill =
// the conv's padding); the 4 waves of a workgroup take channels w, w + 4, ...
// of the same strip and their sums meet in LDS in a fixed order.  Every input
// value is loaded and activated once per strip (R + 2 rows for R outputs), the
// loads of the next CO64_PF channels in flight over the current one's fmas.
// Per output and channel the 9 taps run in (ky, kx) order, as the MFMA kernels.
#ifndef CO64_R
#define CO64_R 8
#endif
#ifndef CO64_PF
#define CO64_PF 3
#endif
#ifndef CO64_PACK
#define CO64_PACK 1   // packed-fp32 activation pairs and output-row pairs (0: the scalar loop)
#endif
using f32x2 = __attribute__((ext_vector_type(2))) float;
__device__ __forceinline__ float wave_shr1(float v) {   // lane i <- lane i - 1, lane 0 <- 0
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_shl1(float v) {   // lane i <- lane i + 1, lane 63 <- 0
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, true));
}
template <int ACT, int PK>
__global__ __launch_bounds__(256) void conv_out64_kernel(ConvArgs a) {
  constexpr int W = 64, R = CO64_R, NR = R + 2, NW = 4, PF = CO64_PF;
  constexpr bool BF = PK == PK_BF16;
  extern __shared__ __attribute__((aligned(16))) float smo[];
  const int Cin = a.Cin, Ca = a.Ca;
  float* wl = smo;                                         // [Cin][9]
  float2* gtab = reinterpret_cast<float2*>(smo + ((Cin * 9 + 1) & ~1));   // [Cin]
  float* red = reinterpret_cast<float*>(gtab + Cin);       // [NW][R][64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.y, y0 = blockIdx.x * R;
  for (int i = tid; i < Cin * 9; i += 256) {
    const int ci = i / 9, tap = i - ci * 9;
    wl[i] = PK == PK_F32 ? packed_w_f32(a.wpk, ci, tap) : packed_w_bf16(a.wpk, ci, tap, PK == PK_SPLIT);
  }
  if constexpr (ACT != ACT_NONE) {
    for (int c = tid; c < Cin; c += 256) gtab[c] = a.gn[(size_t)b * Cin + c];
  }
  constexpr size_t plane = (size_t)W * W;
  auto ldrows = [&](int c, float (&v)[NR]) {
    if (c >= Cin) return;
    const float* src = c < Ca ? a.srcA + ((size_t)b * Ca + c) * plane : a.srcB + ((size_t)b * a.Cb + (c - Ca)) * plane;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      // clamped rows, no branches: the padding rows' values are replaced by
      // zero after the activation (the conv pads the activated tensor)
      const int iy = y0 - 1 + r;
      v[r] = src[(iy < 0 ? 0 : (iy >= W ? W - 1 : iy)) * W + lane];
    }
  };
  float ring[PF + 1][NR];
  float acc[R];
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.f;
#if CO64_PACK
  static_assert(R % 2 == 0 && NR % 2 == 0, "row pairs");
  f32x2 acc2[R / 2];
#pragma unroll
  for (int j = 0; j < R / 2; ++j) acc2[j] = f32x2{0.f, 0.f};
#endif
#pragma unroll
  for (int q = 0; q < PF; ++q) ldrows(wave + NW * q, ring[q]);
  __syncthreads();   // weights and the GroupNorm table
  const int nch = (Cin - wave + NW - 1) / NW;             // this wave's channels
  for (int k = 0; k < nch; k += PF + 1) {
#pragma unroll
    for (int q = 0; q <= PF; ++q) {
      // channel k + q in ring slot q; the load of channel k + q + PF into slot (q + PF) % (PF + 1)
      if (k + q >= nch) break;
      const int c = wave + NW * (k + q);
      ldrows(c + NW * PF, ring[(q + PF) % (PF + 1)]);
      const float* wp = wl + c * 9;
      float g0 = 1.f, g1 = 0.f;
      if constexpr (ACT != ACT_NONE) {
        const float2 g = gtab[c];
        g0 = g.x;
        g1 = g.y;
      }
      float w[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) w[t] = wp[t];
#if CO64_PACK
      // packed fp32 on row pairs (m, m + R/2): output rows j and j + 4 are one
      // v_pk_fma accumulator pair, and their ky-th input rows j + ky, j + 4 + ky
      // are the pair P[j + ky] -- rows 0-3 / 4-7 and 8 / 9 are activated as five
      // aligned pairs A, P[4] = {4, 8} and P[5] = {5, 9} are re-paired from them
      // (the same fma / mul / add per element as the scalar loop, so the same
      // bits; exp and rcp have no packed form; per output the taps still run in
      // (ky, kx) order)
      static_assert(R == 8, "row pairs (m, m + 4)");
      f32x2 A[5];
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        f32x2 v = m < 4 ? f32x2{ring[q][m], ring[q][m + 4]} : f32x2{ring[q][8], ring[q][9]};
        if constexpr (ACT != ACT_NONE) {
          v = __builtin_elementwise_fma(v, f32x2{g0, g0}, f32x2{g1, g1});
          if constexpr (ACT == ACT_GN_SILU) {
            // __expf(-y) = exp2(y * -log2 e): the same v_mul + v_exp as the scalar code
            f32x2 e = v * f32x2{-1.44269504088896340736f, -1.44269504088896340736f};
            e = f32x2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)} + f32x2{1.0f, 1.0f};
            v = v * f32x2{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
          }
        }
        if constexpr (BF) v = f32x2{round_bf16(v.x), round_bf16(v.y)};
        A[m] = v;
      }
      if (y0 == 0) A[0].x = 0.f;                           // the padding rows (after the activation)
      if (y0 + R == W) A[4].y = 0.f;
      f32x2 P[6], PL[6], PR[6];
#pragma unroll
      for (int m = 0; m < 4; ++m) P[m] = A[m];
      P[4] = f32x2{A[0].y, A[4].x};
      P[5] = f32x2{A[1].y, A[4].y};
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        PL[m] = f32x2{wave_shr1(P[m].x), wave_shr1(P[m].y)};
        PR[m] = f32x2{wave_shl1(P[m].x), wave_shl1(P[m].y)};
      }
#pragma unroll
      for (int j = 0; j < R / 2; ++j) {
        f32x2 s2 = acc2[j];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          s2 = __builtin_elementwise_fma(f32x2{w[ky * 3], w[ky * 3]}, PL[j + ky], s2);
          s2 = __builtin_elementwise_fma(f32x2{w[ky * 3 + 1], w[ky * 3 + 1]}, P[j + ky], s2);
          s2 = __builtin_elementwise_fma(f32x2{w[ky * 3 + 2], w[ky * 3 + 2]}, PR[j + ky], s2);
        }
        acc2[j] = s2;
      }
#else
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int iy = y0 - 1 + r;
        float v = ring[q][r];
        if constexpr (ACT != ACT_NONE) {
          v = fmaf(v, g0, g1);
          if constexpr (ACT == ACT_GN_SILU) v = v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
        }
        if constexpr (BF) v = round_bf16(v);
        v = (iy >= 0 && iy < W) ? v : 0.f;                 // the padding rows (after the activation)
        const float l = wave_shr1(v), rr = wave_shl1(v);
#pragma unroll
        for (int ky = 2; ky >= 0; --ky) {                  // output row j = r - ky: its ky-th input row
          const int j = r - ky;
          if (j >= 0 && j < R) {
            acc[j] = fmaf(w[ky * 3], l, acc[j]);
            acc[j] = fmaf(w[ky * 3 + 1], v, acc[j]);
            acc[j] = fmaf(w[ky * 3 + 2], rr, acc[j]);
          }
        }
      }
#endif
    }
  }
#if CO64_PACK
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = j < R / 2 ? acc2[j].x : acc2[j - R / 2].y;
#endif
#pragma unroll
  for (int j = 0; j < R; ++j) red[(wave * R + j) * 64 + lane] = acc[j];
  __syncthreads();
  // the waves' partial sums in wave order, then the MFMA kernels' epilogue order
  const float bb = a.bias ? a.bias[0] : 0.f;
  const float e = a.ebias ? a.ebias[(size_t)b * a.eb_stride] : 0.f;
  for (int o = tid; o < R * 64; o += 256) {
    const int j = o >> 6, x = o & 63;
    float v = (red[(0 * R + j) * 64 + x] + red[(1 * R + j) * 64 + x]) + (red[(2 * R + j) * 64 + x] + red[(3 * R + j) * 64 + x]);
    v = v + bb;
    if (a.ebias) v = v + e;
    const size_t oi = (size_t)b * plane + (size_t)(y0 + j) * W + x;
    if (a.res) v = v + a.res[oi];
    a.out[oi] = v;
  }
}

template <int ACT, int PK>
hipError_t launch_co64(const ConvArgs& a, int B, hipStream_t s) {
  constexpr int R = CO64_R;
  const size_t lds = (((size_t)a.Cin * 9 + 1) & ~(size_t)1) * 4 + (size_t)a.Cin * 8 + (size_t)4 * R * 64 * 4;
  if (lds > 65536) return hipErrorInvalidValue;
  conv_out64_kernel<ACT, PK><<<dim3(64 / R, (unsigned)B), 256, lds, s>>>(a);
  return hipGetLastError();
}

template <int ACT, int WO, int RWS, int BF, int NS>
hipError_t launch_co(const ConvArgs& a, int B, hipStream_t s) {
  using G = OutGeom<WO, RWS, NS>;
  const size_t lds = ((size_t)NS * G::OCC * G::CSZ + (((size_t)a.Cin * 9 + 1) & ~(size_t)1)) * sizeof(float) +
                     (size_t)a.Cin * sizeof(float2);
  static_assert((size_t)NS * G::NT * 16 <= (size_t)NS * G::OCC * G::CSZ * 4, "partials fit the staging buffers");
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)conv_out_kernel<ACT, WO, RWS, BF, NS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((unsigned)(WO / G::ROWS), 1u, (unsigned)B);
  conv_out_kernel<ACT, WO, RWS, BF, NS><<<grid, NS * G::NT, lds, s>>>(a);
  return hipGetLastError();
}

// channel groups per workgroup (ERTD_CONV_OUT_NS, A/B; 1 = one 256-thread group)
static int conv_out_ns() {
  static const int v = [] {
    const int n = ERTD_KNOB("CONV_OUT_NS", 4);
    return n == 1 || n == 2 ? n : 4;
  }();
  return v;
}

#ifndef CONV_OUT_RDIV
#define CONV_OUT_RDIV 1   // A/B: rows per workgroup divided by this (more, smaller workgroups)
#endif
// rows per workgroup: 256 threads per channel group (16 rows; 8 at W = 128;
// the whole image at W = 16).  Measured on a U2 B=64 step (64x64), one group:
// 16 rows (256 workgroups) 60.5 us, 4 rows (1024 one-wave workgroups) 70.5 us
// -- per-workgroup weight gathers and the halo re-reads cost more than the
// lost occupancy; U3 B=256: 163 us (the one-pixel-per-thread kernel before: 244 us).
template <int ACT, int WO, int BF>
hipError_t launch_co_r(const ConvArgs& a, int B, hipStream_t s) {
  constexpr int TPR = WO / 4;
  constexpr int R0 = (256 / TPR) < WO ? (256 / TPR) : WO;
  constexpr int R = CONV_OUT_RDIV > 1 && R0 / CONV_OUT_RDIV * TPR >= 64 ? R0 / CONV_OUT_RDIV : R0;
  const int ns = conv_out_ns();
  if (ns == 1) return launch_co<ACT, WO, R, BF, 1>(a, B, s);
  if (ns == 2) return launch_co<ACT, WO, R, BF, 2>(a, B, s);
  return launch_co<ACT, WO, R, BF, 4>(a, B, s);
}

// ERTD_CONV_OUT64=0 keeps the LDS-staged kernel at W = 64 (A/B)
static int conv_out64_env() {
  static const int v = [] {
    return ERTD_KNOB("CONV_OUT64", 1);
  }();
  return v;
}

template <int ACT, int BF>
hipError_t launch_co_w(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 16: return launch_co_r<ACT, 16, BF>(a, B, s);
    case 32: return launch_co_r<ACT, 32, BF>(a, B, s);
    case 64: return conv_out64_env() ? launch_co64<ACT, BF>(a, B, s) : launch_co_r<ACT, 64, BF>(a, B, s);
    case 128: return launch_co_r<ACT, 128, BF>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}

// ---- one-INPUT-channel 3x3 convolution (conv_in: x (B,1,H,W) -> (B,Cout,H,W)) ----
// The MFMA kernels pad Cin = 1 to a whole K chunk (4 / 16 channels): 31.9 us
// per U2 B=64 step at 6 % of the fp32 peak for a layer whose floor is its
// output write (67 MB).  Here a thread owns four consecutive output pixels:
// their 3 x 6 input window in registers (zero padding), the weights of the
// workgroup's 64 output channels in LDS (broadcast reads), one fp32 fma chain
// of 9 taps per pixel and channel in (ky, kx) order, and a float4 store per
// channel (consecutive lanes = consecutive pixels).  bf16: the input tap is rounded to bf16 (RNE) and the
// weights come from the bf16 packing, so the products equal the bf16 MFMA's.
// W[co][0][tap] in the fp32 packing (ks 3: 4-channel chunks, [tile][chunk][9 step pairs][lane][2])
__device__ __forceinline__ float packed_w0_f32(const float* w, int co, int tap) {
  return w[((size_t)(co >> 5) * 9 + (tap >> 1)) * 128 + (co & 31) * 2 + (tap & 1)];
}
// ... and in the bf16 packing ([tile][chunk][9 steps][lane][8], lane = co & 31 for ci 0..7;
// split: [tile][chunk][hi | lo][9 steps], the weight is hi + lo)
__device__ __forceinline__ float packed_w0_bf16(const float* w, int co, int tap, bool split) {
  const unsigned short* p = reinterpret_cast<const unsigned short*>(w);
  if (!split) return __uint_as_float((unsigned)p[((size_t)(co >> 5) * 9 + tap) * 512 + (co & 31) * 8] << 16);
  const float hi = __uint_as_float((unsigned)p[((size_t)(co >> 5) * 18 + tap) * 512 + (co & 31) * 8] << 16);
  const float lo = __uint_as_float((unsigned)p[((size_t)(co >> 5) * 18 + 9 + tap) * 512 + (co & 31) * 8] << 16);
  return hi + lo;
}

// wave sum, the same value in every lane: row16_sum, then the rows as (r0 + r1) + (r2 + r3)
__device__ __forceinline__ float wave_sum_rl(float v) {
  v = row16_sum(v);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

// A workgroup = one 256-pixel part (the GroupNorm partial's unit) x 64 output
// channels, 16 per wave; lane l owns pixels 4l .. 4l+3 of the part (one row
// segment: WO % 4 == 0), so each channel is one float4 store per lane.  With
// a.gnp the wave also emits the channel's partial {sum, M2 about the part
// mean} (DPP / readlane wave sums), and the walk needs no partials pass over
// the output.
template <int WO, int PK>
__global__ __launch_bounds__(256) void conv_in_kernel(ConvArgs a) {
  constexpr bool BF = PK == PK_BF16;
  constexpr int HW = WO * WO, NP = HW / 256;
  static_assert(HW % 256 == 0 && WO % 4 == 0, "whole 256-pixel parts of whole float4s");
  __shared__ float wl[64 * 9];        // [channel of the workgroup][tap]
  __shared__ float bl[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.y, part = blockIdx.x, cg = blockIdx.z * 64;
  const int Cout = a.Cout;
  for (int i = tid; i < 64 * 9; i += 256) {
    const int co = cg + i / 9, tap = i - (i / 9) * 9;
    wl[i] = co >= Cout ? 0.f
            : PK == PK_F32 ? packed_w0_f32(a.wpk, co, tap) : packed_w0_bf16(a.wpk, co, tap, PK == PK_SPLIT);
  }
  if (tid < 64) bl[tid] = (a.bias && cg + tid < Cout) ? a.bias[cg + tid] : 0.f;
  if (a.zero_words && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)   // the walk's GroupNorm-fold counters
    for (int i = tid; i < a.zero_n; i += 256) a.zero_words[i] = 0u;
  const int p = part * 256 + 4 * lane;
  const int y = p / WO, x0 = p - y * WO;
  const float* src = a.srcA + (size_t)b * HW;
  float v[3][6];      // rows y-1 .. y+1, columns x0-1 .. x0+4
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int iy = y - 1 + ky, ix = x0 - 1 + j;
      float t = (iy >= 0 && iy < WO && ix >= 0 && ix < WO) ? src[iy * WO + ix] : 0.f;
      if constexpr (BF) t = round_bf16(t);
      v[ky][j] = t;
    }
  __syncthreads();
  float* out = a.out + (size_t)b * Cout * HW + p;
  const int c0 = cg + wave * 16;
  const int nc = Cout - c0 < 16 ? Cout - c0 : 16;   // this wave's channels (wave-uniform)
  if (nc <= 0) return;
  float r[16][4];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k < nc) {
      const float* wp = wl + (wave * 16 + k) * 9;
      float w[9];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) w[tap] = wp[tap];
      const float bk = bl[wave * 16 + k];
#pragma unroll
      for (int px = 0; px < 4; ++px) {
        float acc = 0.f;   // one fma chain of the 9 taps in (ky, kx) order, then the bias
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) acc = fmaf(w[tap], v[tap / 3][tap % 3 + px], acc);
        r[k][px] = acc + bk;
      }
      *reinterpret_cast<float4*>(out + (size_t)(c0 + k) * HW) = make_float4(r[k][0], r[k][1], r[k][2], r[k][3]);
    }
  }
  if (!a.gnp) return;
  // per channel: wave sums by DPP row sums + the four rows' readlanes (VALU
  // only, no LDS round trips), {sum, M2 about the part mean}; lane k keeps
  // channel k's pair for one coalesced store
  float s_ = 0.f, q_ = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k < nc) {
      const float sm = wave_sum_rl((r[k][0] + r[k][1]) + (r[k][2] + r[k][3]));
      const float mu = sm * (1.0f / 256.0f);
      const float dx = r[k][0] - mu, dy = r[k][1] - mu, dz = r[k][2] - mu, dw = r[k][3] - mu;
      const float m2 = wave_sum_rl(fmaf(dx, dx, fmaf(dy, dy, fmaf(dz, dz, dw * dw))));
      if (lane == k) { s_ = sm; q_ = m2; }
    }
  }
  if (lane < nc) a.gnp[((size_t)b * Cout + c0 + lane) * NP + part] = make_float2(s_, q_);
}

// (measured: the same kernel looping over items with the next window prefetched,
// 1 / 2 / 4 workgroups per CU, ran 30.4 / 24.4 / 24.5 us against 24.4)
template <int WO, int BF>
hipError_t launch_ci(const ConvArgs& a, int B, hipStream_t s) {
  if (a.Cout < 1 || a.Cout > 1024) return hipErrorInvalidValue;
  conv_in_kernel<WO, BF><<<dim3((unsigned)(WO * WO / 256), (unsigned)B, (unsigned)((a.Cout + 63) / 64)), 256, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace

bool conv_in_ok(const ConvArgs& a, int ks, int mode, int act) {
  return a.Cin == 1 && a.Ca == 1 && ks == 3 && mode == MODE_S1 && act == ACT_NONE && !a.ebias &&
         !a.res && a.Ho == a.Wo && a.Hs == a.Ws && a.Ws == a.Wo &&
         (a.Wo == 16 || a.Wo == 32 || a.Wo == 64 || a.Wo == 128) && a.Cout <= 1024;
}

template <int PK>
static hipError_t launch_ci_w(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 16: return launch_ci<16, PK>(a, B, s);
    case 32: return launch_ci<32, PK>(a, B, s);
    case 64: return launch_ci<64, PK>(a, B, s);
    case 128: return launch_ci<128, PK>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_conv_in(const ConvArgs& a, int B, int pk, hipStream_t s) {
  switch (pk) {
    case PK_F32: return launch_ci_w<PK_F32>(a, B, s);
    case PK_BF16: return launch_ci_w<PK_BF16>(a, B, s);
    case PK_SPLIT: return launch_ci_w<PK_SPLIT>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}

template <int ACT>
static hipError_t launch_co_pk(const ConvArgs& a, int B, int pk, hipStream_t s) {
  switch (pk) {
    case PK_F32: return launch_co_w<ACT, PK_F32>(a, B, s);
    case PK_BF16: return launch_co_w<ACT, PK_BF16>(a, B, s);
    case PK_SPLIT: return launch_co_w<ACT, PK_SPLIT>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_conv_out(int act, const ConvArgs& a, int B, int pk, hipStream_t s) {
  if (a.Cout != 1 || a.Ho != a.Wo || a.Hs != a.Ws || a.Ws != a.Wo || a.Cin != a.Ca + a.Cb)
    return hipErrorInvalidValue;
  if (act == ACT_GN_SILU) return launch_co_pk<ACT_GN_SILU>(a, B, pk, s);
  if (act == ACT_NONE) return launch_co_pk<ACT_NONE>(a, B, pk, s);
  return hipErrorInvalidValue;
}

}  // namespace unet
}  // namespace ertd
