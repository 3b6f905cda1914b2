// Convolution weight gradient of the U-Net train step as an implicit GEMM on
// fp32 MFMA (SURVEY.md 8a' trainer; checked against torch autograd on
// oracle/unet_torch.py by tests/test_gpu_unet_train.py).
//
//   dW[co][ci][tap] = sum_{b, output pixel p} dY[b][co][p] * Xv[b][ci][p + off(tap)]
//
// Xv is the conv's (virtual) input: X itself (stride 1), the nearest-x2
// upsampled X (mode UP, never materialized), or X read at stride 2 (mode S2).
// GEMM view: M = Cout, N = Cin * taps, K = B * Ho * Wo (huge).  A workgroup
// owns a 64 (co) x 32 (ci) x taps output tile and a contiguous range of
// K-chunks (128 output pixels of one sample each); the per-range partials are
// summed in a fixed order by reduce_rows (bitwise reproducible, no atomics).
//
// Per chunk, dY (64 x 128) and the input rows the chunk's taps touch (32 ci x
// (R + 2) rows, zero halo; S2: even / odd columns de-interleaved) are staged
// in LDS.  The K order inside an MFMA is permuted so that lane group g feeds
// pixels 4g .. 4g+3 of a 16-pixel group over 4 consecutive MFMAs: every
// operand fetch is one ds_read_b128 (+ one b32 for a tap's left / right
// neighbour), and the 3 taps of a kernel row share one fetch.  Wave tile:
// 32 co x 16 ci x taps (2 x taps v_mfma_f32_16x16x4_f32 accumulators).
#include <algorithm>
#include <cstdlib>

#include "unet.h"

using namespace ertd;
using namespace ertd::unet;

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int TCO = 64, TCI = 32, PXC = 128, DYS = PXC + 4;

struct WgArgs {
  const float* dy;
  const float* xa;
  const float* xb;
  int Ca, Cb, Cout, H, Ho, R;
  const float2* gn;   // (B, Cin) {scale, shift} when the conv's input is act(GroupNorm(x)) (ACT)
  int ntiles, nco, nsplit, cps, nchunks;
  float* part;   // (nsplit, Cout, Cin * KK)
};

__host__ __device__ constexpr int round_cis(int n) { return n + ((4 - n) % 64 + 64) % 64; }

// LDS geometry per mode: rows of the staged input, row width, per-channel stride
struct Geo {
  int nr, roww, cis;
};
__host__ __device__ constexpr Geo geo(int mode, int ks, int Ho) {
  const int R = PXC / Ho;
  Geo g{};
  if (ks == 1) {
    g.nr = R; g.roww = Ho; g.cis = PXC + 4;
  } else if (mode == MODE_S2) {
    g.nr = 2 * R + 1; g.roww = 2 * Ho + 8; g.cis = round_cis(g.nr * g.roww);
  } else {
    g.nr = R + 2; g.roww = Ho + 8; g.cis = round_cis(g.nr * g.roww);
  }
  return g;
}

__device__ __forceinline__ const float* chan_ptr(const WgArgs& a, int b, int ci) {
  const size_t hw = (size_t)a.H * a.H;
  return ci < a.Ca ? a.xa + ((size_t)b * a.Ca + ci) * hw : a.xb + ((size_t)b * a.Cb + ci - a.Ca) * hw;
}

// ACT (stride 1 only): the conv's input is act(GroupNorm(x)) -- applied here
// while staging (x * scale + shift, then SiLU for ACT_GN_SILU), so the
// activated tensor never has to exist in HBM; padding stays zero
template <int ACT>
__device__ __forceinline__ f32x4 wg_act(f32x4 v, float2 g) {
  if constexpr (ACT != ACT_NONE) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = fmaf(v[e], g.x, g.y);
      if constexpr (ACT == ACT_GN_SILU) t = t * __builtin_amdgcn_rcpf(1.0f + __expf(-t));
      v[e] = t;
    }
  }
  return v;
}

template <int MODE, int KS, int HO, int ACT>
__global__ __launch_bounds__(256) void wgrad_conv_kernel(WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int KK = KS * KS;
  constexpr int Ho = HO, R = PXC / HO;
  const int Cin = a.Ca + a.Cb;
  constexpr Geo G = geo(MODE, KS, HO);
  float* dyL = smem;
  float* xL = smem + TCO * DYS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int tile = blockIdx.x % a.ntiles, split = blockIdx.x / a.ntiles;
  const int co0 = (tile % a.nco) * TCO, ci0 = (tile / a.nco) * TCI;
  const int cb0 = 2 * (w & 1), cib = w >> 1;
  // zero the staged input once: halo columns are never written by the loads
  for (int i = tid; i < TCI * G.cis; i += 256) xL[i] = 0.f;

  f32x4 acc[2][KK];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < KK; ++t) acc[i][t] = f32x4{};

  constexpr int rows_per_b = Ho / R;
  const int c_lo = split * a.cps, c_hi = min(a.nchunks, c_lo + a.cps);
  // Staging.  S1 / UP / 1x1: the next chunk's operands are loaded into
  // registers while the current chunk's MFMAs run (one LDS buffer, register
  // double buffering); S2 (two layers) loads synchronously.
  constexpr int NDY = TCO * PXC / 4 / 256;          // dY float4 per thread
  constexpr int q = Ho / 4;
  constexpr int nx = KS == 1 ? TCI * PXC / 4 : TCI * G.nr * q;
  constexpr int NXR = (nx + 255) / 256;
  f32x4 dyr[NDY];
  f32x4 xr[MODE == MODE_S2 ? 1 : NXR];
  // ACT: the activation is applied in store() (after the chunk's MFMAs), not
  // in load(), so the prefetch stays in flight; {scale, shift} ride along
  float2 gr[ACT != ACT_NONE && MODE != MODE_S2 ? NXR : 1];
  auto load = [&](int c) {
    const int b = c / rows_per_b, y0 = (c - b * rows_per_b) * R;
#pragma unroll
    for (int k = 0; k < NDY; ++k) {
      const int i = tid + 256 * k, r = i / (PXC / 4), c4 = i - r * (PXC / 4), co = co0 + r;
      dyr[k] = co < a.Cout
                   ? *(const f32x4*)(a.dy + ((size_t)b * a.Cout + co) * Ho * Ho + (size_t)y0 * Ho + 4 * c4)
                   : f32x4{};
    }
    if constexpr (MODE != MODE_S2) {
#pragma unroll
      for (int k = 0; k < NXR; ++k) {
        const int i = tid + 256 * k;
        f32x4 v = f32x4{};
        if constexpr (ACT != ACT_NONE) gr[k] = float2{0.f, 0.f};   // padding stays zero
        if (i < nx) {
          if constexpr (KS == 1) {
            const int r = i / (PXC / 4), c4 = i - r * (PXC / 4), ci = ci0 + r;
            if (ci < Cin) {
              v = *(const f32x4*)(chan_ptr(a, b, ci) + (size_t)y0 * Ho + 4 * c4);
              if constexpr (ACT != ACT_NONE) gr[k] = a.gn[(size_t)b * Cin + ci];
            }
          } else {
            const int r = i / q, c4 = i - r * q;
            const int cl = r / G.nr, rr = r - cl * G.nr;
            const int ci = ci0 + cl, vy = y0 - 1 + rr;
            if (ci < Cin && vy >= 0 && vy < Ho) {
              if constexpr (MODE == MODE_UP) {
                const float2 sv = *(const float2*)(chan_ptr(a, b, ci) + (size_t)(vy >> 1) * a.H + 2 * c4);
                v = f32x4{sv.x, sv.x, sv.y, sv.y};
              } else {
                v = *(const f32x4*)(chan_ptr(a, b, ci) + (size_t)vy * Ho + 4 * c4);
                if constexpr (ACT != ACT_NONE) gr[k] = a.gn[(size_t)b * Cin + ci];
              }
            }
          }
        }
        xr[k] = v;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int k = 0; k < NDY; ++k) {
      const int i = tid + 256 * k, r = i / (PXC / 4), c4 = i - r * (PXC / 4);
      *(f32x4*)(dyL + r * DYS + 4 * c4) = dyr[k];
    }
    if constexpr (MODE != MODE_S2) {
#pragma unroll
      for (int k = 0; k < NXR; ++k) {
        const int i = tid + 256 * k;
        if (i < nx) {
          f32x4 v = xr[k];
          if constexpr (ACT != ACT_NONE) v = wg_act<ACT>(v, gr[k]);
          if constexpr (KS == 1) {
            const int r = i / (PXC / 4), c4 = i - r * (PXC / 4);
            *(f32x4*)(xL + r * G.cis + 4 * c4) = v;
          } else {
            const int r = i / q, c4 = i - r * q;
            const int cl = r / G.nr, rr = r - cl * G.nr;
            *(f32x4*)(xL + cl * G.cis + rr * G.roww + 4 + 4 * c4) = v;
          }
        }
      }
    }
  };
  if (c_lo < c_hi) load(c_lo);
  for (int c = c_lo; c < c_hi; ++c) {
    __syncthreads();
    store();
    if constexpr (MODE == MODE_S2) {
      // input rows 2 y0 - 1 .. 2 (y0 + R - 1) + 1, width H = 2 Ho; E at col 4, O at col Ho + 8
      const int b = c / rows_per_b, y0 = (c - b * rows_per_b) * R;
      const int W = a.H, qw = W / 4;
      for (int i = tid; i < TCI * G.nr * qw; i += 256) {
        const int r = i / qw, c4 = i - r * qw;
        const int cl = r / G.nr, rr = r - cl * G.nr;
        const int ci = ci0 + cl, iy = 2 * y0 - 1 + rr;
        f32x4 v = f32x4{};
        if (ci < Cin && iy >= 0 && iy < W) v = *(const f32x4*)(chan_ptr(a, b, ci) + (size_t)iy * W + 4 * c4);
        float* row = xL + cl * G.cis + rr * G.roww;
        *(float2*)(row + 4 + 2 * c4) = float2{v.x, v.z};
        *(float2*)(row + Ho + 8 + 2 * c4) = float2{v.y, v.w};
      }
    }
    if (c + 1 < c_hi) load(c + 1);
    __syncthreads();
    // ---- MFMAs over the chunk's 128 pixels, 16 at a time
    const float* xw = xL + (cib * 16 + l16) * G.cis;
    const float* a0p = dyL + ((cb0 + 0) * 16 + l16) * DYS + 4 * g;
    const float* a1p = dyL + ((cb0 + 1) * 16 + l16) * DYS + 4 * g;
#pragma unroll 1
    for (int p16 = 0; p16 < PXC; p16 += 16) {
      const f32x4 A0 = *(const f32x4*)(a0p + p16);
      const f32x4 A1 = *(const f32x4*)(a1p + p16);
      if constexpr (KS == 1) {
        const f32x4 Bv = *(const f32x4*)(xw + p16 + 4 * g);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(A0[s], Bv[s], acc[0][0], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[s], Bv[s], acc[1][0], 0, 0, 0);
        }
      } else {
        const int yl = p16 / Ho, x0 = p16 - yl * Ho + 4 * g;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          f32x4 B0, B1, B2;
          if constexpr (MODE == MODE_S2) {
            const float* row = xw + (2 * yl + ky) * G.roww;
            const f32x4 E = *(const f32x4*)(row + 4 + x0);
            const f32x4 O = *(const f32x4*)(row + Ho + 8 + x0);
            const float ol = row[Ho + 7 + x0];
            B0 = f32x4{ol, O.x, O.y, O.z};
            B1 = E;
            B2 = O;
          } else {
            const float* row = xw + (yl + ky) * G.roww + 4 + x0;
            const f32x4 C = *(const f32x4*)row;
            const float lf = row[-1], rt = row[4];
            B0 = f32x4{lf, C.x, C.y, C.z};
            B1 = C;
            B2 = f32x4{C.y, C.z, C.w, rt};
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            acc[0][3 * ky + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(A0[s], B0[s], acc[0][3 * ky + 0], 0, 0, 0);
            acc[1][3 * ky + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[s], B0[s], acc[1][3 * ky + 0], 0, 0, 0);
            acc[0][3 * ky + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(A0[s], B1[s], acc[0][3 * ky + 1], 0, 0, 0);
            acc[1][3 * ky + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[s], B1[s], acc[1][3 * ky + 1], 0, 0, 0);
            acc[0][3 * ky + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(A0[s], B2[s], acc[0][3 * ky + 2], 0, 0, 0);
            acc[1][3 * ky + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[s], B2[s], acc[1][3 * ky + 2], 0, 0, 0);
          }
        }
      }
    }
  }
  // ---- partial tile out: D row 4 (lane / 16) + r of the 16-row block, column lane % 16
  const size_t ncol = (size_t)Cin * KK;
  const int ci = ci0 + cib * 16 + l16;
  if (ci >= Cin) return;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + (cb0 + i) * 16 + 4 * g + r;
      if (co >= a.Cout) continue;
      float* dst = a.part + ((size_t)split * a.Cout + co) * ncol + (size_t)ci * KK;
#pragma unroll
      for (int t = 0; t < KK; ++t) dst[t] = acc[i][t][r];
    }
}

#ifndef WG_REDUCE4
#define WG_REDUCE4 1  // 1: K-range partial sums on wgrad_reduce4_kernel where cols % 4 == 0 (A/B)
#endif

// dW[j] (+)= sum over ranges of part[r][j] (as reduce_rows_kernel in unet_train.hip)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int rows,
                                                           size_t cols, float* __restrict__ out,
                                                           int accumulate) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const size_t j = (size_t)blockIdx.x * 64 + tx;
  float s0 = 0.f, s1 = 0.f;
  if (j < cols) {
    int r = ty;
    for (; r + 4 < rows; r += 8) {
      s0 += part[(size_t)r * cols + j];
      s1 += part[(size_t)(r + 4) * cols + j];
    }
    if (r < rows) s0 += part[(size_t)r * cols + j];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty == 0 && j < cols) {
    const float s = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
    out[j] = accumulate ? out[j] + s : s;
  }
}

// the same sum for cols % 4 == 0: a workgroup owns 64 columns as 16 float4
// column quads x 16 row groups (rows r = g mod 16, two interleaved chains),
// the 16 group totals added in order -- 4x the loads in flight per lane of
// wgrad_reduce_kernel, whose 4 row groups left a 256-range sum latency-bound
__global__ __launch_bounds__(256) void wgrad_reduce4_kernel(const float* __restrict__ part, int rows,
                                                            size_t cols, float* __restrict__ out,
                                                            int accumulate) {
  __shared__ f32x4 red[16][16];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const size_t c4 = cols / 4, j = (size_t)blockIdx.x * 16 + tx;
  const f32x4* p = reinterpret_cast<const f32x4*>(part);
  f32x4 s0{}, s1{};
  if (j < c4) {
    int r = ty;
    for (; r + 16 < rows; r += 32) {
      s0 += p[(size_t)r * c4 + j];
      s1 += p[(size_t)(r + 16) * c4 + j];
    }
    if (r < rows) s0 += p[(size_t)r * c4 + j];
  }
  red[ty][tx] = s0 + s1;
  __syncthreads();
  if (ty == 0 && j < c4) {
    f32x4 s = red[0][tx];
#pragma unroll
    for (int g = 1; g < 16; ++g) s += red[g][tx];
    f32x4* o = reinterpret_cast<f32x4*>(out) + j;
    *o = accumulate ? *o + s : s;
  }
}

// dW (+)= the fixed-order sum of the rows x cols partials
hipError_t reduce_parts(const float* part, int rows, size_t cols, float* dw, int accumulate, hipStream_t s) {
  if (WG_REDUCE4 && cols % 4 == 0 && ((uintptr_t)dw & 15) == 0)
    wgrad_reduce4_kernel<<<(unsigned)((cols / 4 + 15) / 16), 256, 0, s>>>(part, rows, cols, dw, accumulate);
  else
    wgrad_reduce_kernel<<<(unsigned)((cols + 63) / 64), 256, 0, s>>>(part, rows, cols, dw, accumulate);
  return hipGetLastError();
}

#ifndef WG1_LDS
#define WG1_LDS 1  // 1: 1x1 weight gradients on wg1_lds_kernel; 0: wgrad_conv_kernel<S1, 1> (A/B)
#endif
#ifndef WG1_PD
#define WG1_PD 1   // wg1_lds_kernel global-load prefetch distance in 32-k blocks (1 or 2; A/B: 2 no faster)
#endif

// The 1x1 convs (the res-block skips) are a plain GEMM dW = dY Xᵀ over K =
// B * H * W with both operands already K-contiguous in NCHW: one workgroup
// per (co block 64 MB, ci block 64 NB, K range) stages the 16-k block's dY
// rows and X rows in LDS once (one float4 per lane per 256 row-quads, rows
// padded to 20 floats: conflict-free fragment reads) and the 2 x 2 waves
// multiply their 32 MB x 32 NB sub-tiles out of it -- the LDS-tiled GEMM of
// the Winograd weight gradient (unet_wgrad_wino.hip) with the NCHW sample
// stride folded into the K index (H W % 16 == 0: a 16-k block never spans
// two samples).  Partials per K range, summed in a fixed order by
// wgrad_reduce_kernel.
struct W1Args {
  const float* dy;
  const float* xa;
  const float* xb;
  int Ca, Cb, Cout, HW, nq, qpr;   // nq 32-k blocks, qpr per K range
  float* P;   // (nks, Cout, Cin)
};

// per stage a 32-k block: 8 row-quads per row (each row's 128 bytes one
// whole cache line, 8 lanes), two 16-k MFMA sub-blocks per barrier; the next
// block's loads are in flight during the current block's MFMAs (WG1_PD = 2:
// two blocks ahead).  Measured and not kept: an XCD-aware workgroup order
// putting a K range's tiles on one L2 (same time: the MALL absorbs the
// re-reads).
template <int MB, int NB>
__global__ __launch_bounds__(256) void wg1_lds_kernel(W1Args a) {
  constexpr int RA = 64 * MB, RB = 64 * NB, PITCH = 36, NU = 2 * (MB + NB);
  constexpr int WI = 2 * MB, WJ = 2 * NB;
  __shared__ __attribute__((aligned(16))) float lds[2][(RA + RB) * PITCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int Cin = a.Ca + a.Cb;
  const int ncb = Cin / RB, nmb = a.Cout / RA;
  int r = blockIdx.x;
  const int nb = r % ncb; r /= ncb;
  const int mb = r % nmb;
  const int ks = r / nmb;
  const int c16 = lane & 15, g = lane >> 4;
  const int q0 = ks * a.qpr, q1 = min(q0 + a.qpr, a.nq);
  // staging: thread tid moves row-quad f = tid + 256 u: row f >> 3, k-quad f & 7;
  // each row's sample-0 pointer is fixed for the workgroup
  const float* src[NU];
  long long bstride[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int f = tid + 256 * u;
    if (u < 2 * MB) {
      const int co = RA * mb + (f >> 3);
      src[u] = a.dy + (size_t)co * a.HW + 4 * (f & 7);
      bstride[u] = (long long)a.Cout * a.HW;
    } else {
      const int ci = RB * nb + ((f - 512 * MB) >> 3);
      const bool lo = ci < a.Ca;
      src[u] = (lo ? a.xa + (size_t)ci * a.HW : a.xb + (size_t)(ci - a.Ca) * a.HW) + 4 * (f & 7);
      bstride[u] = (long long)(lo ? a.Ca : a.Cb) * a.HW;
    }
  }
  auto gload = [&](int Q, f32x4 (&stg)[NU]) {
    const int t0 = 32 * Q, b = t0 / a.HW, p = t0 - b * a.HW;
#pragma unroll
    for (int u = 0; u < NU; ++u) stg[u] = *reinterpret_cast<const f32x4*>(src[u] + b * bstride[u] + p);
  };
  auto lstore = [&](int buf, const f32x4 (&stg)[NU]) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int f = tid + 256 * u;
      const int row = u < 2 * MB ? f >> 3 : RA + ((f - 512 * MB) >> 3);
      *reinterpret_cast<f32x4*>(&lds[buf][row * PITCH + 4 * (f & 7)]) = stg[u];
    }
  };
  f32x4 acc[WI][WJ];
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j) acc[i][j] = f32x4{};
  auto compute = [&](int buf) {
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      f32x4 av[WI], bv[WJ];
#pragma unroll
      for (int i = 0; i < WI; ++i)
        av[i] = *reinterpret_cast<const f32x4*>(
            &lds[buf][(32 * MB * wm + 16 * i + c16) * PITCH + 16 * sb + 4 * g]);
#pragma unroll
      for (int j = 0; j < WJ; ++j)
        bv[j] = *reinterpret_cast<const f32x4*>(
            &lds[buf][(RA + 32 * NB * wn + 16 * j + c16) * PITCH + 16 * sb + 4 * g]);
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < WI; ++i)
#pragma unroll
          for (int j = 0; j < WJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][k], bv[j][k], acc[i][j], 0, 0, 0);
    }
  };
  if (q0 < q1) {
    // two register stage sets: block Q + 2 is in flight while Q computes and
    // Q + 1 moves to LDS (2 blocks of compute hide each load)
    f32x4 s0[NU], s1[NU];
    gload(q0, s0);
    lstore(0, s0);
    if (WG1_PD > 1 && q0 + 1 < q1) gload(q0 + 1, s1);
    __syncthreads();
    auto step = [&](int Q, f32x4 (&mine)[NU], f32x4 (&next)[NU]) {
      const int buf = (Q - q0) & 1;
      if (WG1_PD > 1) {
        if (Q + 2 < q1) gload(Q + 2, mine);
      } else if (Q + 1 < q1) {
        gload(Q + 1, next);
      }
      compute(buf);
      if (Q + 1 < q1) lstore(buf ^ 1, next);
      __syncthreads();
    };
    for (int Q = q0; Q < q1; Q += 2) {
      step(Q, s0, s1);
      if (Q + 1 < q1) step(Q + 1, s1, s0);
    }
  }
  // lane holds rows co = RA mb + 32 MB wm + 16 i + 4 g + e, column ci = RB nb + 32 NB wn + 16 j + c16
  float* P = a.P + (size_t)ks * a.Cout * Cin;
  const int co0 = RA * mb + 32 * MB * wm, ci0 = RB * nb + 32 * NB * wn;
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        P[(size_t)(co0 + 16 * i + 4 * g + e) * Cin + ci0 + 16 * j + c16] = acc[i][j][e];
}

struct W1Plan {
  int mb, nb, nq, qpr, nks;   // tile 64 mb x 64 nb
  size_t part_floats;
};

// Tile and K split, as measured over forced plans at the U2 B = 32 skip
// shapes (tools/wgrad_probe.py --skip --sweep): 64 x 64 tiles (the most
// workgroups in flight) with 8 32-k blocks per K range, or 16 once that still
// leaves >= 512 workgroups -- 256 .. 768 workgroups, 256 .. 512 k per range,
// the best measured plan at every shape but one (within 4 %).  A pure
// function of the shape (bitwise reproducible); ERTD_WG1_MB / _NB / _QPR
// (diag build) force a plan.
bool wg1_plan(int Cin, int Cout, int B, int H, int ks, int mode, int act, W1Plan* p) {
  if (!WG1_LDS || ks != 1 || mode != MODE_S1 || act != ACT_NONE || Cin % 64 || Cout % 64 || B < 1 ||
      H < 4 || (H * H) % 32)
    return false;
  const long long K = (long long)B * H * H;
  if (K / 32 > (1 << 30)) return false;
  p->nq = (int)(K / 32);
  p->mb = ERTD_KNOB("WG1_MB", 1);
  p->nb = ERTD_KNOB("WG1_NB", 1);
  if (p->mb < 1 || p->mb > 2 || p->nb < 1 || p->nb > 2 || Cout % (64 * p->mb) || Cin % (64 * p->nb))
    return false;
  const long long tiles = (long long)(Cout / (64 * p->mb)) * (Cin / (64 * p->nb));
  int qpr = tiles * (p->nq / 16) >= 512 ? 16 : 8;
  qpr = ERTD_KNOB("WG1_QPR", qpr);
  p->qpr = std::max(1, std::min(qpr, p->nq));
  p->nks = (p->nq + p->qpr - 1) / p->qpr;
  p->part_floats = (size_t)p->nks * Cout * Cin;
  return true;
}

hipError_t launch_wg1(const W1Plan& pl, const float* dy, const float* x, int Ca, const float* x2, int Cb,
                      int HW, int Cout, float* part, hipStream_t s) {
  W1Args a{dy, x, x2, Ca, Cb, Cout, HW, pl.nq, pl.qpr, part};
  const unsigned nwg = (unsigned)((Cout / (64 * pl.mb)) * ((Ca + Cb) / (64 * pl.nb)) * pl.nks);
  if (pl.mb == 1 && pl.nb == 1) wg1_lds_kernel<1, 1><<<nwg, 256, 0, s>>>(a);
  else if (pl.mb == 1) wg1_lds_kernel<1, 2><<<nwg, 256, 0, s>>>(a);
  else if (pl.nb == 1) wg1_lds_kernel<2, 1><<<nwg, 256, 0, s>>>(a);
  else wg1_lds_kernel<2, 2><<<nwg, 256, 0, s>>>(a);
  return hipGetLastError();
}

#ifndef WGT_T
#define WGT_T 512  // wgt_kernel threads: 512 splits each row between two threads (256: one; A/B)
#endif
#ifndef WGT_ON
#define WGT_ON 1  // 1: 3x3 weight gradients with a single-channel side on wgt_kernel (0: implicit GEMM; A/B)
#endif

// The convs with one input or one output channel (conv_in: Cin = 1, conv_out:
// Cout = 1) leave 63 of 64 rows of the implicit GEMM's MFMA tile idle.  Their
// weight gradient dW[c][ky][kx] = sum_{b,y,x} P[y][x] Q[y + ky - 1][x + kx - 1]
// (conv_out: P = dy, Q = act(x[c]); conv_in: P = dy[c], Q = x) is C x 9 sums
// over B H W terms: one workgroup per (sample, band of R rows) stages P's R rows
// and Q's R + 2 rows (zero halo, the activation applied) in LDS, thread (c, ky)
// walks the band's pixels in order keeping the three kx sums (a sliding window:
// one Q read per pixel), and the per-band partials are summed in a fixed order.
struct WtArgs {
  const float* dy;
  const float* x;
  const float2* gn;   // (B, Cin) {scale, shift} of the activation on x, or null
  int C, H, R, cin1;  // C: the multi-channel side; cin1: conv_in (Cin = 1), else conv_out
  float* P;           // (B H / R, C * 9)
};

template <int ACT>
__global__ __launch_bounds__(WGT_T) void wgt_kernel(WtArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = a.H, W = a.H, R = a.R, C = a.C, QW = W + 2, W4 = W / 4;
  // odd per-channel strides: the lanes of a wave (21 channels x 3 ky) read
  // distinct banks (an even multiple of 32 put every channel on one bank)
  const int PS = R * W + 1, QS = (R + 2) * QW + 1;
  const int nband = H / R;
  const int b = blockIdx.x / nband, y0 = (blockIdx.x - b * nband) * R;
  const int CP = a.cin1 ? C : 1, CQ = a.cin1 ? 1 : C;
  float* Ps = sm;                     // [CP][PS]: R rows of W
  float* Qs = sm + CP * PS;           // [CQ][QS]: R + 2 rows of W + 2
  const int tid = threadIdx.x;
  constexpr int NB = 8;   // float4 loads in flight per lane while staging
  const int np4 = CP * R * W4;
  for (int i0 = tid; i0 < np4; i0 += WGT_T * NB) {
    f32x4 v[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int i = i0 + WGT_T * u, c = i / (R * W4), rem = i - c * (R * W4);
      v[u] = i < np4 ? *reinterpret_cast<const f32x4*>(a.dy + ((size_t)b * CP + c) * H * W + (size_t)y0 * W +
                                                      4 * rem)
                     : f32x4{};
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int i = i0 + WGT_T * u, c = i / (R * W4), rem = i - c * (R * W4);
      if (i < np4) {
        float* p = Ps + c * PS + 4 * rem;
        p[0] = v[u][0]; p[1] = v[u][1]; p[2] = v[u][2]; p[3] = v[u][3];
      }
    }
  }
  // Q: halo columns zero, rows outside the image zero
  for (int i = tid; i < CQ * (R + 2); i += WGT_T) {
    const int c = i / (R + 2), r = i - c * (R + 2);
    Qs[c * QS + r * QW] = 0.f;
    Qs[c * QS + r * QW + W + 1] = 0.f;
  }
  const int nq4 = CQ * (R + 2) * W4;
  for (int i0 = tid; i0 < nq4; i0 += WGT_T * NB) {
    f32x4 v[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int i = i0 + WGT_T * u, c = i / ((R + 2) * W4), rem = i - c * ((R + 2) * W4);
      const int r = rem / W4, x4 = rem - r * W4, y = y0 - 1 + r;
      v[u] = i < nq4 && y >= 0 && y < H
                 ? *reinterpret_cast<const f32x4*>(a.x + ((size_t)b * CQ + c) * H * W + (size_t)y * W + 4 * x4)
                 : f32x4{};
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int i = i0 + WGT_T * u, c = i / ((R + 2) * W4), rem = i - c * ((R + 2) * W4);
      const int r = rem / W4, x4 = rem - r * W4, y = y0 - 1 + r;
      if (i < nq4) {
        f32x4 t = v[u];
        if constexpr (ACT != ACT_NONE) {
          if (y >= 0 && y < H) t = wg_act<ACT>(t, a.gn[(size_t)b * CQ + c]);   // padding stays zero
        }
        float* q = Qs + c * QS + r * QW + 1 + 4 * x4;
        q[0] = t[0]; q[1] = t[1]; q[2] = t[2]; q[3] = t[3];
      }
    }
  }
  __syncthreads();
  // thread (xh, c, ky): the half xh of every row (WGT_T = 512: two halves,
  // their sums added in order below; 256: one)
  constexpr int NH = WGT_T / 256;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  const int xh = tid / (WGT_T / NH), tl = tid - xh * (WGT_T / NH);
  const int c = tl / 3, ky = tl - 3 * c;
  if (tl < 3 * C) {
    const float* pr = Ps + (a.cin1 ? c : 0) * PS;
    const float* qr = Qs + (a.cin1 ? 0 : c) * QS + ky * QW;
    const int xw = W / NH, x0 = xh * xw;
    for (int r = 0; r < R; ++r) {
      const float* pp = pr + r * W + x0;
      const float* qq = qr + r * QW + x0;
      float q0 = qq[0], q1 = qq[1];
#pragma unroll 8
      for (int x = 0; x < xw; ++x) {
        const float q2 = qq[x + 2], p = pp[x];
        s0 = fmaf(p, q0, s0);
        s1 = fmaf(p, q1, s1);
        s2 = fmaf(p, q2, s2);
        q0 = q1;
        q1 = q2;
      }
    }
  }
  if constexpr (NH > 1) {
    __syncthreads();   // the staging is free: the upper half's sums go through it
    if (xh == 1 && tl < 3 * C) {
      Ps[3 * tl] = s0; Ps[3 * tl + 1] = s1; Ps[3 * tl + 2] = s2;
    }
    __syncthreads();
    if (xh == 0 && tl < 3 * C) {
      s0 += Ps[3 * tl]; s1 += Ps[3 * tl + 1]; s2 += Ps[3 * tl + 2];
    }
  }
  if (xh == 0 && tl < 3 * C) {
    float* o = a.P + (size_t)blockIdx.x * C * 9 + c * 9 + 3 * ky;
    o[0] = s0;
    o[1] = s1;
    o[2] = s2;
  }
}

// rows per band (0: not this path): the largest of 8 / 4 / 2 dividing H whose
// staging fits 100 KB of LDS (two workgroups per CU; ERTD_WGT_LDSKB in the diag
// build: conv_out at 64x64 29.1 us with 4-row bands in 102 KB, 24.7 with 2-row)
int wgt_rows(int Cin, int Cout, int Cb, int H, int ks, int mode) {
  if (!WGT_ON || ks != 3 || mode != MODE_S1 || Cb != 0 || H < 4 || H % 4 || H > 128) return 0;
  const bool cin1 = Cin == 1 && Cout >= 1 && Cout <= 64, cout1 = Cout == 1 && Cin >= 2 && Cin <= 64;
  if (!cin1 && !cout1) return 0;
  const int C = cin1 ? Cout : Cin, CP = cin1 ? C : 1, CQ = cin1 ? 1 : C;
  const size_t cap = (size_t)ERTD_KNOB("WGT_LDSKB", 100) * 1024;
  for (int R = 8; R >= 2; R /= 2)
    if (H % R == 0 && (size_t)(CP * (R * H + 1) + CQ * ((R + 2) * (H + 2) + 1)) * sizeof(float) <= cap)
      return R;
  return 0;
}

size_t wgt_part_floats(int Cin, int Cout, int B, int H, int R) {
  return (size_t)B * (H / R) * std::max(Cin, Cout) * 9;
}

hipError_t launch_wgt(const float* dy, const float* x, int Cin, int Cout, int B, int H, int R, const float* gn,
                      int act, float* part, hipStream_t s) {
  const bool cin1 = Cin == 1;
  WtArgs a{dy, x, (const float2*)gn, cin1 ? Cout : Cin, H, R, cin1 ? 1 : 0, part};
  const int C = a.C, CP = cin1 ? C : 1, CQ = cin1 ? 1 : C;
  const size_t lds = (size_t)(CP * (R * H + 1) + CQ * ((R + 2) * (H + 2) + 1)) * sizeof(float);
  const unsigned nwg = (unsigned)(B * (H / R));
  if (act == ACT_GN_SILU) {
    static std::atomic<unsigned long long> at{0};
    set_max_lds_once((const void*)wgt_kernel<ACT_GN_SILU>, 160 * 1024, at);
    wgt_kernel<ACT_GN_SILU><<<nwg, WGT_T, lds, s>>>(a);
  } else if (act == ACT_GN) {
    static std::atomic<unsigned long long> at{0};
    set_max_lds_once((const void*)wgt_kernel<ACT_GN>, 160 * 1024, at);
    wgt_kernel<ACT_GN><<<nwg, WGT_T, lds, s>>>(a);
  } else {
    static std::atomic<unsigned long long> at{0};
    set_max_lds_once((const void*)wgt_kernel<ACT_NONE>, 160 * 1024, at);
    wgt_kernel<ACT_NONE><<<nwg, WGT_T, lds, s>>>(a);
  }
  return hipGetLastError();
}

int n_cu() {
  static int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    return n;
  }();
  return v;
}


struct Plan {
  int Ho, R, nco, nci, ntiles, nchunks, cps, nsplit;
  size_t lds, part_floats;
};

bool plan_of(int Cin, int Cout, int B, int H, int ks, int mode, Plan* p) {
  if (Cin < 1 || Cout < 1 || B < 1 || H < 1 || (ks != 1 && ks != 3) || mode < MODE_S1 ||
      mode > MODE_UP || (ks == 1 && mode != MODE_S1))
    return false;
  const int Ho = mode == MODE_S2 ? H / 2 : (mode == MODE_UP ? 2 * H : H);
  if ((Ho != 16 && Ho != 32 && Ho != 64 && Ho != 128) || (mode == MODE_S2 && H != 2 * Ho)) return false;
  if (ks == 3 && Ho < 16) return false;    // a 16-pixel group stays inside one row
  if (ks == 1 && Ho * Ho < 16) return false;
  const Geo G = geo(mode, ks, Ho);
  p->Ho = Ho;
  p->R = PXC / Ho;
  p->nco = (Cout + TCO - 1) / TCO;
  p->nci = (Cin + TCI - 1) / TCI;
  p->ntiles = p->nco * p->nci;
  p->nchunks = B * (Ho / p->R);
  if (ks == 1 && Ho * Ho < PXC) return false;
  // about 4 workgroups per CU, >= 2 chunks per range (the partial write +
  // reduce traffic vs occupancy; measured at U2 B=32 once the 3x3 stride-1 and
  // 1x1 convs had left this kernel: >= 4 chunks gave the stride-2 convs 128
  // workgroups, train step 10.19 -> 10.11 ms, tools/gpu_cps.sh)
  static const int wpc = ERTD_KNOB("WGRAD_WPC", 4), min_cps = ERTD_KNOB("WGRAD_CPS", 2);
  const int want = (wpc * n_cu() + p->ntiles - 1) / p->ntiles;
  int cps = (p->nchunks + want - 1) / want;
  if (cps < min_cps) cps = min_cps;
  if (cps > p->nchunks) cps = p->nchunks;
  p->cps = cps;
  p->nsplit = (p->nchunks + cps - 1) / cps;
  p->lds = ((size_t)TCO * DYS + (size_t)TCI * G.cis) * sizeof(float);
  p->part_floats = (size_t)p->nsplit * Cout * Cin * ks * ks;
  return true;
}

template <int MODE, int KS, int HO, int ACT>
hipError_t launch_t(const WgArgs& a, size_t lds, hipStream_t s) {
  static std::atomic<unsigned long long> attr{0};
  set_max_lds_once((const void*)wgrad_conv_kernel<MODE, KS, HO, ACT>, 160 * 1024, attr);
  wgrad_conv_kernel<MODE, KS, HO, ACT><<<(unsigned)(a.ntiles * a.nsplit), 256, lds, s>>>(a);
  return hipGetLastError();
}

template <int MODE, int KS, int ACT>
hipError_t launch_m(const WgArgs& a, size_t lds, hipStream_t s) {
  switch (a.Ho) {
    case 16: return launch_t<MODE, KS, 16, ACT>(a, lds, s);
    case 32: return launch_t<MODE, KS, 32, ACT>(a, lds, s);
    case 64: return launch_t<MODE, KS, 64, ACT>(a, lds, s);
    case 128: return launch_t<MODE, KS, 128, ACT>(a, lds, s);
    default: return hipErrorInvalidValue;
  }
}

template <int MODE, int KS>
hipError_t launch_a(const WgArgs& a, int act, size_t lds, hipStream_t s) {
  if constexpr (MODE == MODE_S1) {
    if (act == ACT_GN_SILU) return launch_m<MODE, KS, ACT_GN_SILU>(a, lds, s);
    if (act == ACT_GN) return launch_m<MODE, KS, ACT_GN>(a, lds, s);
  }
  if (act != ACT_NONE) return hipErrorInvalidValue;
  return launch_m<MODE, KS, ACT_NONE>(a, lds, s);
}

}  // namespace

extern "C" {

size_t ertd_conv_wgrad_ws_bytes(int Cin, int Cout, int B, int H, int ks, int mode) {
  Plan p;
  if (!plan_of(Cin, Cout, B, H, ks, mode, &p)) return 0;
  // the Winograd path (3x3 stride 1, unet_wgrad_wino.hip) and the 1x1 GEMM where eligible
  W1Plan w1;
  const size_t f1 = wg1_plan(Cin, Cout, B, H, ks, mode, ACT_NONE, &w1) ? w1.part_floats : 0;
  const int rt = wgt_rows(Cin, Cout, 0, H, ks, mode);
  const size_t ft = rt ? wgt_part_floats(Cin, Cout, B, H, rt) : 0;
  return std::max({p.part_floats, f1, ft, wgrad_wino_ws_floats(Cin, Cout, B, H, ks, mode)}) * sizeof(float);
}

int ertd_conv_wgrad(const float* dy, const float* x, int Ca, const float* x2, int Cb, int B, int H,
                    int Cout, int ks, int mode, const float* gn, int act, float* dw, int accumulate,
                    void* ws, size_t ws_bytes, void* stream) {
  if (!dy || !x || !dw || !ws || Ca < 1 || Cb < 0 || (Cb > 0 && !x2) || act < ACT_NONE ||
      act > ACT_GN || (act != ACT_NONE && (!gn || mode != MODE_S1)))
    return ERTD_EINVAL;
  Plan p;
  if (!plan_of(Ca + Cb, Cout, B, H, ks, mode, &p)) return ERTD_EINVAL;
  const size_t wf = wgrad_wino_ws_floats(Ca + Cb, Cout, B, H, ks, mode);
  if (wf > 0) {
    if (wf * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
    const hipError_t e = launch_wgrad_wino(dy, x, Ca, x2, Cb, B, H, Cout, mode, gn, act, dw, accumulate,
                                           (float*)ws, (hipStream_t)stream);
    return e == hipSuccess ? ERTD_OK : (int)e;
  }
  hipStream_t s = (hipStream_t)stream;
  if (const int rt = wgt_rows(Ca + Cb, Cout, Cb, H, ks, mode)) {
    const size_t nf = wgt_part_floats(Ca + Cb, Cout, B, H, rt);
    if (nf * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
    hipError_t e = launch_wgt(dy, x, Ca + Cb, Cout, B, H, rt, gn, act, (float*)ws, s);
    if (e != hipSuccess) return (int)e;
    e = reduce_parts((const float*)ws, B * (H / rt), (size_t)Cout * (Ca + Cb) * 9, dw, accumulate, s);
    return e == hipSuccess ? ERTD_OK : (int)e;
  }
  W1Plan w1;
  if (wg1_plan(Ca + Cb, Cout, B, H, ks, mode, act, &w1)) {
    if (w1.part_floats * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
    hipError_t e = launch_wg1(w1, dy, x, Ca, x2, Cb, H * H, Cout, (float*)ws, s);
    if (e != hipSuccess) return (int)e;
    e = reduce_parts((const float*)ws, w1.nks, (size_t)Cout * (Ca + Cb), dw, accumulate, s);
    return e == hipSuccess ? ERTD_OK : (int)e;
  }
  if (p.part_floats * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
  WgArgs a{dy, x, x2, Ca, Cb, Cout, H, p.Ho, p.R, (const float2*)gn, p.ntiles, p.nco, p.nsplit,
           p.cps, p.nchunks, (float*)ws};
  hipError_t e;
  if (ks == 1) e = launch_a<MODE_S1, 1>(a, act, p.lds, s);
  else if (mode == MODE_S2) e = launch_a<MODE_S2, 3>(a, act, p.lds, s);
  else if (mode == MODE_UP) e = launch_a<MODE_UP, 3>(a, act, p.lds, s);
  else e = launch_a<MODE_S1, 3>(a, act, p.lds, s);
  if (e != hipSuccess) return (int)e;
  e = reduce_parts((const float*)ws, p.nsplit, (size_t)Cout * (Ca + Cb) * ks * ks, dw, accumulate, s);
  return e == hipSuccess ? ERTD_OK : (int)e;
}

int ertd_conv_wgrad_bias(const float* dy, const float* x, int Ca, const float* x2, int Cb, int B, int H,
                         int Cout, int ks, int mode, const float* gn, int act, float* dw, int accumulate,
                         float* db, float* db2, void* ws, size_t ws_bytes, void* stream) {
  if (!dy || !x || !dw || !db || !ws || Ca < 1 || Cb < 0 || (Cb > 0 && !x2) || act < ACT_NONE ||
      act > ACT_GN || (act != ACT_NONE && (!gn || mode != MODE_S1)))
    return ERTD_EINVAL;
  if (!wgrad_wino_bias_ok(Ca + Cb, Cout, B, H, ks, mode)) return ERTD_EINVAL;
  if (ertd_conv_wgrad_ws_bytes(Ca + Cb, Cout, B, H, ks, mode) > ws_bytes) return ERTD_ENOSPC;
  const hipError_t e = launch_wgrad_wino(dy, x, Ca, x2, Cb, B, H, Cout, mode, gn, act, dw, accumulate,
                                         (float*)ws, (hipStream_t)stream, db, db2);
  return e == hipSuccess ? ERTD_OK : (int)e;
}

int ertd_conv_wgrad_bias_ok(int Cin, int Cout, int B, int H, int ks, int mode) {
  return wgrad_wino_bias_ok(Cin, Cout, B, H, ks, mode) ? 1 : 0;
}

}  // extern "C"
