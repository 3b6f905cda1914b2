// fp32 conv weight packings as device functions shared by the per-layer pack
// kernels of unet_conv*.hip and the batched pack of unet_pack.hip, so both
// write the same bits.  Every packed value is a pure function of the source
// weight: a layer's packing can be rebuilt anywhere in a stream (e.g. once per
// optimizer step for every conv at once).
//
//   direct  W (Cout, Cin, ks, ks) -> [co_tile32][chunk][step pair][lane][2]
//   up      4 sub-pixel classes of 2x2 taps ([class][co_tile32][chunk][...])
//   wino    F(2x2,3x3): U = G g G^T, [cog][chunk][xi 16][cb 4][kk 4][c16][st]
//   wino4   F(4x4,3x3): U = G g G^T, [cog][chunk][xi/2 18][cb 4][kk 4][c16][xi&1]
// flipT: w is the forward conv's (cin', cout', ks, ks) weight and the packing
// is the input-gradient conv's W'[co][ci] = W[ci][co] spatially flipped.
#pragma once
#include "unet.h"

namespace ertd {
namespace unet {

// channels per K-chunk of the direct kernel: 4 for 3x3, 8 for the sub-pixel
// 2x2, 32 for 1x1
__host__ __device__ constexpr int conv_ck(int ks) { return ks == 3 ? 4 : (ks == 2 ? 8 : 32); }
constexpr int WINO_KC = 8;    // F(2x2) input channels per chunk
constexpr int WINO4_KC = 4;   // F(4x4) input channels per chunk

__device__ __forceinline__ float pack_conv_elem(const float* __restrict__ w, int cin, int cout, int ks,
                                                int nchunk, size_t i, bool flipT) {
  const int ck = conv_ck(ks), ch = ck / 2;
  const int spc = ks == 3 ? 9 * ch : ch;
  const int e = (int)(i & 1);
  const int lane = (int)((i >> 1) & 63);
  size_t rest = i >> 7;
  const int sp = (int)(rest % (spc / 2));
  rest /= (spc / 2);
  const int k = (int)(rest % nchunk);
  const int tile = (int)(rest / nchunk);
  const int s = 2 * sp + e;
  const int hh = lane >> 5;
  const int co = tile * 32 + (lane & 31);
  int ci, ky, kx;
  if (ks == 3) { ci = k * ck + hh * ch + s / 9; ky = (s % 9) / 3; kx = s % 3; }
  else { ci = k * ck + hh * ch + s; ky = 0; kx = 0; }
  if (co >= cout || ci >= cin) return 0.f;
  return flipT ? w[(((size_t)ci * cout + co) * ks + (ks - 1 - ky)) * ks + (ks - 1 - kx)]
               : w[(((size_t)co * cin + ci) * ks + ky) * ks + kx];
}

// Upsample conv: W (Cout, Cin, 3, 3) -> tap (ty, tx) of class (pa, pb) = sum of
// W[ky][kx] over ky in S(pa, ty), kx in S(pb, tx), S(0,0) = {0}, S(0,1) = {1,2},
// S(1,0) = {0,1}, S(1,1) = {2}
__device__ __forceinline__ float pack_conv_up_elem(const float* __restrict__ w, int cin, int cout, int nchunk,
                                                   size_t per_class, size_t gi) {
  const int cls = (int)(gi / per_class);
  const size_t i = gi - (size_t)cls * per_class;
  const int pa = cls >> 1, pb = cls & 1;
  constexpr int ck = conv_ck(2), ch = ck / 2, spc = 4 * ch;
  const int e = (int)(i & 1);
  const int lane = (int)((i >> 1) & 63);
  size_t rest = i >> 7;
  const int sp = (int)(rest % (spc / 2));
  rest /= (spc / 2);
  const int k = (int)(rest % nchunk);
  const int tile = (int)(rest / nchunk);
  const int st = 2 * sp + e;
  const int co = tile * 32 + (lane & 31);
  const int ci = k * ck + (lane >> 5) * ch + st / 4;
  const int ty = (st % 4) / 2, tx = st % 2;
  float v = 0.f;
  if (co < cout && ci < cin) {
    const float* wk = w + ((size_t)co * cin + ci) * 9;
    const int y0 = (pa == 0) ? (ty == 0 ? 0 : 1) : (ty == 0 ? 0 : 2);
    const int y1 = (pa == 0) ? (ty == 0 ? 0 : 2) : (ty == 0 ? 1 : 2);
    const int x0 = (pb == 0) ? (tx == 0 ? 0 : 1) : (tx == 0 ? 0 : 2);
    const int x1 = (pb == 0) ? (tx == 0 ? 0 : 2) : (tx == 0 ? 1 : 2);
    for (int ky = y0; ky <= y1; ++ky)
      for (int kx = x0; kx <= x1; ++kx) v += wk[ky * 3 + kx];
  }
  return v;
}

// The two Winograd packings, one thread per (co, ci): all xi of U = G g G^T
// in float64 (row_y = sum_x g[y][x] G[rj][x], then u = sum_y G[ri][y] row_y,
// rounded once to fp32; G g computed once per tile instead of per element).
// F(2x2) G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]; F(4x4) G = the rows of the
// points {0, 1, -1, 1/2, -2, inf}.  Thread j enumerates the packing's
// (co, ci) in its own index order, so consecutive lanes write consecutive
// floats of every xi.
// F(4x4): j = [cog][chunk][cb 4][kk 4][c16 16]; writes 18 float2 (xi pairs)
__device__ __forceinline__ void pack_wino4_tile(const float* __restrict__ w, int cin, int cout, int nchunk,
                                                size_t j, bool flipT, float* __restrict__ dst) {
  constexpr double GD[6][3] = {{1.0, 0.0, 0.0},
                               {1.0 / 3, 1.0 / 3, 1.0 / 3},
                               {-1.0 / 3, 1.0 / 3, -1.0 / 3},
                               {-16.0 / 15, -8.0 / 15, -4.0 / 15},
                               {1.0 / 15, -2.0 / 15, 4.0 / 15},
                               {0.0, 0.0, 1.0}};
  const int c16 = (int)(j & 15);
  const int kk = (int)((j >> 4) & 3);
  const int cb = (int)((j >> 6) & 3);
  const size_t rest = j >> 8;
  const int k = (int)(rest % nchunk);
  const int cog = (int)(rest / nchunk);
  const int co = cog * 64 + cb * 16 + c16;
  const int ci = k * WINO4_KC + kk;
  const float* g = flipT ? w + ((size_t)ci * cout + co) * 9 : w + ((size_t)co * cin + ci) * 9;
  double gv[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) gv[q] = (double)(flipT ? g[8 - q] : g[q]);
  double row[6][3];   // row[rj][y] = sum_x g[y][x] G[rj][x]
#pragma unroll
  for (int rj = 0; rj < 6; ++rj)
#pragma unroll
    for (int y = 0; y < 3; ++y) {
      double r = 0.0;
#pragma unroll
      for (int x = 0; x < 3; ++x) r += gv[y * 3 + x] * GD[rj][x];
      row[rj][y] = r;
    }
  // float index of xi pair p: ((((cog*nchunk + k)*18 + p)*4 + cb)*4 + kk)*16 + c16)*2
  float2* o = reinterpret_cast<float2*>(dst) + ((((size_t)(cog * nchunk + k) * 18) * 4 + cb) * 4 + kk) * 16 + c16;
#pragma unroll
  for (int pp = 0; pp < 18; ++pp) {
    float uv[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int xi = 2 * pp + e, ri = xi / 6, rj = xi % 6;
      double u = 0.0;
#pragma unroll
      for (int y = 0; y < 3; ++y) u += GD[ri][y] * row[rj][y];
      uv[e] = (float)u;
    }
    o[(size_t)pp * 256] = make_float2(uv[0], uv[1]);
  }
}

// F(2x2): j = [cog][chunk][cb 4][kk 4][c16 16][st 2]; writes 16 floats (one per xi)
__device__ __forceinline__ void pack_wino_tile(const float* __restrict__ w, int cin, int cout, int nchunk,
                                               size_t j, bool flipT, float* __restrict__ dst) {
  const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  const int st = (int)(j & 1);
  const int c16 = (int)((j >> 1) & 15);
  const int kk = (int)((j >> 5) & 3);
  const int cb = (int)((j >> 7) & 3);
  const size_t rest = j >> 9;
  const int k = (int)(rest % nchunk);
  const int cog = (int)(rest / nchunk);
  const int co = cog * 64 + cb * 16 + c16;
  const int ci = k * WINO_KC + 2 * kk + st;
  const float* g = flipT ? w + ((size_t)ci * cout + co) * 9 : w + ((size_t)co * cin + ci) * 9;
  double gv[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) gv[q] = (double)(flipT ? g[8 - q] : g[q]);
  double row[4][3];
#pragma unroll
  for (int rj = 0; rj < 4; ++rj)
#pragma unroll
    for (int y = 0; y < 3; ++y) {
      double r = 0.0;
#pragma unroll
      for (int x = 0; x < 3; ++x) r += gv[y * 3 + x] * G[rj][x];
      row[rj][y] = r;
    }
  // float index: (((((cog*nchunk + k)*16 + xi)*4 + cb)*4 + kk)*16 + c16)*2 + st
  float* o = dst + (((size_t)(cog * nchunk + k) * 16 * 4 + cb) * 4 + kk) * 32 + c16 * 2 + st;
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) {
    const int ri = xi >> 2, rj = xi & 3;
    double u = 0.0;
#pragma unroll
    for (int y = 0; y < 3; ++y) u += G[ri][y] * row[rj][y];
    o[(size_t)xi * 512] = (float)u;
  }
}

// threads of one packing in the tile forms (one per (co, ci)) / element forms
__host__ __device__ inline long long pack_work_items(int kind, long long total) {
  return kind == 3 ? total / 36 : (kind == 2 ? total / 16 : total);   // ERTD_PACK_WINO4 / _WINO
}

}  // namespace unet
}  // namespace ertd
