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
  // about 4 workgroups per CU, >= 4 chunks per range (measured optimum at
  // U2 B=32 of the partial write + reduce traffic vs occupancy: tools/wgrad_sweep.sh)
  static const int wpc = ERTD_KNOB("WGRAD_WPC", 4), min_cps = ERTD_KNOB("WGRAD_CPS", 4);
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
  // the Winograd path (3x3 stride 1, unet_wgrad_wino.hip) where eligible
  return std::max(p.part_floats, wgrad_wino_ws_floats(Cin, Cout, B, H, ks, mode)) * sizeof(float);
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
  if (p.part_floats * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
  WgArgs a{dy, x, x2, Ca, Cb, Cout, H, p.Ho, p.R, (const float2*)gn, p.ntiles, p.nco, p.nsplit,
           p.cps, p.nchunks, (float*)ws};
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (ks == 1) e = launch_a<MODE_S1, 1>(a, act, p.lds, s);
  else if (mode == MODE_S2) e = launch_a<MODE_S2, 3>(a, act, p.lds, s);
  else if (mode == MODE_UP) e = launch_a<MODE_UP, 3>(a, act, p.lds, s);
  else e = launch_a<MODE_S1, 3>(a, act, p.lds, s);
  if (e != hipSuccess) return (int)e;
  const size_t cols = (size_t)Cout * (Ca + Cb) * ks * ks;
  wgrad_reduce_kernel<<<(unsigned)((cols + 63) / 64), 256, 0, s>>>((const float*)ws, p.nsplit, cols,
                                                                    dw, accumulate);
  e = hipGetLastError();
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
