// Training (backward) operators of the build-defined U-Net (SURVEY.md 8a';
// north_star "sampler/trainer", the reference train step
// ERT_Conditional_Diffusion.py:305-320 around the U-Net).  PARITY UNPINNED vs
// the reference (no U-Net there): checked against torch autograd on
// oracle/unet_torch.py (tests/test_gpu_unet_train.py).
//
// The host walk (ertdiff/unet_train.py) composes these with the forward
// operators (ertd_conv2d, ertd_group_norm_stats):
//   ertd_gn_stats_mr          GroupNorm statistics + (mean, rstd) per group
//   ertd_gn_act_apply         act(GroupNorm(cat(x, x2))) materialized (the conv input a wgrad needs)
//   ertd_gn_act_backward      dL/dx of act(GroupNorm(x)) (+ per-sample dgamma / dbeta partials)
//   ertd_im2col               the (C*k*k, Ho*Wo) patch matrix of a conv input (stride 1 / 2 /
//                             nearest-x2 upsample modes)
//   ertd_wgrad_gemm           dW = sum_b dY_b . Xcol_b^T on fp32 MFMA, split over samples,
//                             fixed-order reduction
//   ertd_conv_weight_flip     W'[ci][co] = W[co][ci] flipped: dX of a conv is a conv of dY
//   ertd_zero_insert / ertd_sum_pool2   stride-2 / upsample dX plumbing
//   ertd_channel_sums         per (sample, channel) and per channel sums (bias / emb grads)
//   ertd_reduce_rows          fixed-order sum over rows (per-sample partials -> grads)
//   ertd_reduce_rows_multi    many of those in one launch (bitwise equal)
//   ertd_gemm_small           strided batched fp32 GEMM (+ bias / accumulate): dense layers,
//                             attention forward / backward
//   ertd_softmax_rows / ertd_softmax_backward   attention softmax and its backward
//   ertd_eltwise              silu / silu-backward / relu-backward / add / scale / pool-mean
//   ertd_mse_loss             MSELoss(mean) and dL/deps
//   ertd_encoder_train_fwd / ertd_encoder_train_bwd   the reference condition encoder
//                             (conv strips with saved activations; backward reused from
//                             the reference train step, train.hip)
//   ertd_adam_multi           torch.optim.Adam over any number of tensors
// Every reduction has a fixed order: results are bitwise reproducible.
#include <cmath>
#include <cstring>

#include "unet.h"

using namespace ertd;
using namespace ertd::unet;

namespace {

inline int rcode(hipError_t e) { return e == hipSuccess ? ERTD_OK : (int)e; }

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return s * (1.0f + x * (1.0f - s));
}

// ---- GroupNorm (+SiLU) apply ------------------------------------------------------
__global__ void gn_act_apply_kernel(const float* __restrict__ xa, int Ca, const float* __restrict__ xb,
                                    int Cb, int HW, const float2* __restrict__ ss, int act, size_t n,
                                    float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int C = Ca + Cb;
  const size_t bc = i / HW;
  const int p = (int)(i - bc * HW);
  const int b = (int)(bc / C), c = (int)(bc - (size_t)b * C);
  const float x = c < Ca ? xa[((size_t)b * Ca + c) * HW + p] : xb[((size_t)b * Cb + c - Ca) * HW + p];
  const float2 g = ss[bc];
  float v = fmaf(x, g.x, g.y);
  if (act == ACT_GN_SILU) v = v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
  out[i] = v;
}

// ---- GroupNorm (+SiLU) backward: one 256-thread workgroup per (group, sample).
// xhat = (x - mean) rstd, xn = gamma xhat + beta, y = act(xn):
//   dxn = dy act'(xn); dgamma_c += sum dxn xhat, dbeta_c += sum dxn (per sample)
//   dx = rstd (dxhat - mean_g(dxhat) - xhat mean_g(dxhat xhat)),  dxhat = gamma dxn
__device__ __forceinline__ double wg_sum(double v, double* red, int tid) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Pass 1 reduces each channel's two sums within each wave (shuffles, no
// barrier) into LDS; one barrier per 64 channels; the wave partials are then
// added in a fixed order.  float4 loads throughout (HW % 4 == 0).  A channel
// gets min(4, HW / 256) waves (wpc): at 16x16 (64 float4s per
// channel) the four waves take four channels at once instead of one wave
// working while three idle.  The partial sums are the same values either way
// (a wave that held no pixels contributed exact zeros), so results are
// bitwise unchanged.
constexpr int GNB_CB = 64;
__global__ __launch_bounds__(256) void gn_act_bwd_kernel(
    const float* __restrict__ xa, int Ca, const float* __restrict__ xb, int Cb, int HW, int groups,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float2* __restrict__ mr,
    int act, const float* __restrict__ dy, float* __restrict__ dxa, float* __restrict__ dxb,
    int accumulate, float* __restrict__ dgb, float* __restrict__ csum, long long ldc,
    const float* __restrict__ addc) {
  __shared__ double part[2][GNB_CB][4];
  __shared__ float cred[GNB_CB][4];
  const int g = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int C = Ca + Cb, cpg = C / groups, HW4 = HW / 4;
  const int wpc = HW4 >= 256 ? 4 : (HW4 >= 128 ? 2 : 1);   // waves per channel
  const int cpi = 4 / wpc;                                  // channels in flight
  const int sub = w / wpc, wl = w - sub * wpc;
  const int p0 = wl * 64 + lane, pst = wpc * 64;
  const float2 m = mr[(size_t)b * groups + g];
  const float mean = m.x, rstd = m.y;
  auto xptr = [&](int c) {
    return c < Ca ? xa + ((size_t)b * Ca + c) * HW : xb + ((size_t)b * Cb + c - Ca) * HW;
  };
  auto dxn_of = [&](float xv, float dv, float ga, float be, float& xh) {
    xh = (xv - mean) * rstd;
    return act == ACT_GN_SILU ? dv * silu_grad(fmaf(ga, xh, be)) : dv;
  };
  double A = 0.0, Bs = 0.0;
  for (int c0 = 0; c0 < cpg; c0 += GNB_CB) {
    const int nc = cpg - c0 < GNB_CB ? cpg - c0 : GNB_CB;
    for (int cl = sub; cl < nc; cl += cpi) {
      const int c = g * cpg + c0 + cl;
      const float4* x = (const float4*)xptr(c);
      const float4* d = (const float4*)(dy + ((size_t)b * C + c) * HW);
      const float ga = gamma[c], be = beta[c];
      double sg = 0.0, sb = 0.0;
      for (int p = p0; p < HW4; p += pst) {
        const float4 xv = x[p], dv = d[p];
        float xh, dn;
        dn = dxn_of(xv.x, dv.x, ga, be, xh); sg += (double)dn * xh; sb += (double)dn;
        dn = dxn_of(xv.y, dv.y, ga, be, xh); sg += (double)dn * xh; sb += (double)dn;
        dn = dxn_of(xv.z, dv.z, ga, be, xh); sg += (double)dn * xh; sb += (double)dn;
        dn = dxn_of(xv.w, dv.w, ga, be, xh); sg += (double)dn * xh; sb += (double)dn;
      }
      sg = wave_sum_d(sg);
      sb = wave_sum_d(sb);
      if (lane == 0) {
        part[0][cl][wl] = sg;
        part[1][cl][wl] = sb;
      }
    }
    __syncthreads();
    for (int cl = 0; cl < nc; ++cl) {
      const int c = g * cpg + c0 + cl;
      double sg, sb;
      if (wpc == 4) {
        sg = (part[0][cl][0] + part[0][cl][1]) + (part[0][cl][2] + part[0][cl][3]);
        sb = (part[1][cl][0] + part[1][cl][1]) + (part[1][cl][2] + part[1][cl][3]);
      } else if (wpc == 2) {
        sg = part[0][cl][0] + part[0][cl][1];
        sb = part[1][cl][0] + part[1][cl][1];
      } else {
        sg = part[0][cl][0];
        sb = part[1][cl][0];
      }
      if (tid == 0) {
        dgb[(size_t)(2 * b) * C + c] = (float)sg;        // [b][0][c]: dgamma partial
        dgb[(size_t)(2 * b + 1) * C + c] = (float)sb;    // [b][1][c]: dbeta partial
      }
      const double ga = gamma[c];
      A += ga * sb;     // sum dxhat
      Bs += ga * sg;    // sum dxhat xhat
    }
    __syncthreads();
  }
  const double n = (double)cpg * HW;
  const float mA = (float)(A / n), mB = (float)(Bs / n);
  for (int cl = sub; cl < cpg; cl += cpi) {
    const int c = g * cpg + cl;
    const float4* x = (const float4*)xptr(c);
    float4* dx = (float4*)(c < Ca ? dxa + ((size_t)b * Ca + c) * HW : dxb + ((size_t)b * Cb + c - Ca) * HW);
    const float4* d = (const float4*)(dy + ((size_t)b * C + c) * HW);
    const float4* ad = addc ? (const float4*)(addc + ((size_t)b * C + c) * HW) : nullptr;
    const float ga = gamma[c], be = beta[c];
    float cs = 0.f;
    for (int p = p0; p < HW4; p += pst) {
      const float4 xv = x[p], dv = d[p];
      float4 o = accumulate ? dx[p] : float4{0.f, 0.f, 0.f, 0.f};
      if (ad) {   // (dx + addc) + the GroupNorm term: the order of a separate add before
        const float4 av = ad[p];
        o = accumulate ? float4{o.x + av.x, o.y + av.y, o.z + av.z, o.w + av.w} : av;
      }
      float xh, dn, q0, q1, q2, q3;
      dn = dxn_of(xv.x, dv.x, ga, be, xh); q0 = rstd * ((ga * dn - mA) - xh * mB); o.x += q0;
      dn = dxn_of(xv.y, dv.y, ga, be, xh); q1 = rstd * ((ga * dn - mA) - xh * mB); o.y += q1;
      dn = dxn_of(xv.z, dv.z, ga, be, xh); q2 = rstd * ((ga * dn - mA) - xh * mB); o.z += q2;
      dn = dxn_of(xv.w, dv.w, ga, be, xh); q3 = rstd * ((ga * dn - mA) - xh * mB); o.w += q3;
      dx[p] = o;
      cs += (q0 + q1) + (q2 + q3);
    }
    if (csum) {
      cs = wave_sum_f(cs);
      if (lane == 0) cred[cl][wl] = cs;   // cpg <= GNB_CB when csum is requested
    }
  }
  if (csum) {
    __syncthreads();
    if (tid < cpg) {
      const float s = wpc == 4 ? (cred[tid][0] + cred[tid][1]) + (cred[tid][2] + cred[tid][3])
                               : (wpc == 2 ? cred[tid][0] + cred[tid][1] : cred[tid][0]);
      csum[(size_t)b * ldc + g * cpg + tid] = s;
    }
  }
}

// ---- im2col: out[b][c*kk + tap][q] for output pixel q of the conv --------------------
__global__ void im2col_kernel(const float* __restrict__ x, int C, int H, int ks, int mode, int Ho,
                              size_t n, float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int HWo = Ho * Ho, kk = ks * ks;
  const size_t row = i / HWo;
  const int q = (int)(i - row * HWo);
  const int b = (int)(row / ((size_t)C * kk));
  const int r = (int)(row - (size_t)b * C * kk);
  const int c = r / kk, tap = r - c * kk;
  const int ky = tap / ks, kx = tap - ky * ks;
  const int oy = q / Ho, ox = q - oy * Ho;
  int iy, ix, lim = H;
  if (ks == 1) { iy = oy; ix = ox; }
  else if (mode == MODE_S2) { iy = 2 * oy - 1 + ky; ix = 2 * ox - 1 + kx; }
  else if (mode == MODE_UP) { iy = oy - 1 + ky; ix = ox - 1 + kx; lim = 2 * H; }
  else { iy = oy - 1 + ky; ix = ox - 1 + kx; }
  float v = 0.f;
  if (iy >= 0 && iy < lim && ix >= 0 && ix < lim) {
    if (mode == MODE_UP && ks == 3) { iy >>= 1; ix >>= 1; }
    v = x[((size_t)b * C + c) * H * H + (size_t)iy * H + ix];
  }
  out[i] = v;
}

// ---- dW partial of one sample: C[m][n] = sum_p A[m][p] B[n][p] on fp32 MFMA.
// WG = 4 waves, 64 (m) x 64 (n) tile, K chunks of 32 pixels staged in LDS.
__global__ __launch_bounds__(256) void wgrad_kernel(const float* __restrict__ A, const float* __restrict__ Bm,
                                                    int M, int N, int P, size_t bsA, size_t bsB,
                                                    float* __restrict__ part, int split_len,
                                                    int nsplit_per_b) {
  __shared__ float As[32][65];
  __shared__ float Bs[32][65];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int n0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
  const int split = blockIdx.z;
  const int b = split / nsplit_per_b, sp = split - b * nsplit_per_b;
  const int p_lo = sp * split_len, p_hi = min(P, p_lo + split_len);
  const float* Ab = A + (size_t)b * bsA;
  const float* Bb = Bm + (size_t)b * bsB;
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
  f32x16 acc = {};
  for (int p0 = p_lo; p0 < p_hi; p0 += 32) {
    for (int idx = tid; idx < 64 * 32; idx += 256) {
      const int r = idx >> 5, k = idx & 31;
      const int p = p0 + k;
      As[k][r] = (m0 + r < M && p < p_hi) ? Ab[(size_t)(m0 + r) * P + p] : 0.f;
      Bs[k][r] = (n0 + r < N && p < p_hi) ? Bb[(size_t)(n0 + r) * P + p] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int s = 0; s < 16; ++s) {
      const float a = As[2 * s + h][wm + l32];
      const float bb = Bs[2 * s + h][wn + l32];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  float* Cp = part + (size_t)split * M * N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * h, n = n0 + wn + l32;
    if (m < M && n < N) Cp[(size_t)m * N + n] = acc[r];
  }
}

// out[j] (+)= sum_r part[r][j]: 64 columns x 4 row-interleaved partial sums
// per workgroup (loads in flight), combined in a fixed order (reproducible)
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ part, int rows,
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

// Several reduce_rows_kernel problems in one launch (the train step's per-layer
// dgamma/dbeta and bias reductions, deferred to the end of the backward walk):
// workgroup -> (problem k, 64-column block) through the block prefix; the sum
// of every column in exactly reduce_rows_kernel's order (bitwise equal)
constexpr int RM_T = 48;
struct ReduceMulti {
  const float* part[RM_T];
  float* out[RM_T];
  long long cols[RM_T];
  int rows[RM_T];
  int acc[RM_T];
  int blk[RM_T + 1];
  int n;
};
__global__ __launch_bounds__(256) void reduce_rows_multi_kernel(ReduceMulti a) {
  __shared__ float red[4][64];
  const int bid = blockIdx.x;
  int k = 0;
  while (k + 1 < a.n && bid >= a.blk[k + 1]) ++k;
  const float* __restrict__ part = a.part[k];
  const int rows = a.rows[k];
  const size_t cols = (size_t)a.cols[k];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const size_t j = (size_t)(bid - a.blk[k]) * 64 + tx;
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
    const float sum = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
    float* out = a.out[k];
    out[j] = a.acc[k] ? out[j] + sum : sum;
  }
}

__global__ void weight_flip_kernel(const float* __restrict__ w, int Cout, int Cin, int ks,
                                   float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int kk = ks * ks;
  if (i >= Cout * Cin * kk) return;
  const int tap = i % kk, r = i / kk;
  const int co = r % Cout, ci = r / Cout;   // out is (Cin, Cout, ks, ks)
  const int ky = tap / ks, kx = tap % ks;
  out[i] = w[((size_t)co * Cin + ci) * kk + (ks - 1 - ky) * ks + (ks - 1 - kx)];
}

__global__ void zero_insert_kernel(const float* __restrict__ x, int Ho, size_t n, float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;   // over the 2Ho x 2Ho output
  if (i >= n) return;
  const int W2 = 2 * Ho;
  const size_t bc = i / ((size_t)W2 * W2);
  const int q = (int)(i - bc * W2 * W2);
  const int y = q / W2, xx = q - y * W2;
  out[i] = ((y | xx) & 1) ? 0.f : x[bc * Ho * Ho + (size_t)(y >> 1) * Ho + (xx >> 1)];
}

__global__ void sum_pool2_kernel(const float* __restrict__ x, int H, size_t n, float* __restrict__ out,
                                 int accumulate) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;   // over the H x H output
  if (i >= n) return;
  const size_t bc = i / ((size_t)H * H);
  const int q = (int)(i - bc * H * H);
  const int y = q / H, xx = q - y * H;
  const float* s = x + bc * 4 * H * H;
  const int W2 = 2 * H;
  const float v = (s[(size_t)(2 * y) * W2 + 2 * xx] + s[(size_t)(2 * y) * W2 + 2 * xx + 1]) +
                  (s[(size_t)(2 * y + 1) * W2 + 2 * xx] + s[(size_t)(2 * y + 1) * W2 + 2 * xx + 1]);
  out[i] = accumulate ? out[i] + v : v;
}

// per (sample, channel) sum over HW (one workgroup each, fixed order)
__global__ __launch_bounds__(256) void chan_sum_kernel(const float* __restrict__ x, int HW, int C,
                                                       int ldo, float* __restrict__ out) {
  __shared__ double red[4];
  const size_t bc = blockIdx.x;
  const float* s = x + bc * HW;
  double acc = 0.0;
  for (int p = threadIdx.x; p < HW; p += 256) acc += (double)s[p];
  acc = wg_sum(acc, red, threadIdx.x);
  if (threadIdx.x == 0) out[(bc / C) * ldo + bc % C] = (float)acc;
}

// ---- small strided batched GEMM (fp32 FMA, 32x32 tile per workgroup)
struct SmallGemm {
  const float* A; long long a_i, a_k, a_b;
  const float* Bm; long long b_k, b_j, b_b;
  float* C; long long c_i, c_j, c_b;
  const float* bias;   // per column j, or null
  int I, J, K;
  float alpha;
  int accumulate;
};

__global__ __launch_bounds__(256) void gemm_small_kernel(SmallGemm g) {
  __shared__ float As[32][33];
  __shared__ float Bs[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  const int i0 = blockIdx.y * 32, j0 = blockIdx.x * 32, bt = blockIdx.z;
  const float* A = g.A + bt * g.a_b;
  const float* Bm = g.Bm + bt * g.b_b;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // 32-k tiles are loaded into a ring of 4 register slots, 3 tiles ahead of
  // the FMAs (the small grids here -- 8 .. 86 workgroups -- leave each tile's
  // first-touch HBM load latency-bound: one tile ahead still waited per tile)
  constexpr int NS = 4;
  float ra[NS][4], rb[NS][4];
  auto gload = [&](float (&la)[4], float (&lb)[4], int k0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = ty + 8 * r;
      la[r] = (i0 + ii < g.I && k0 + tx < g.K) ? A[(i0 + ii) * g.a_i + (k0 + tx) * g.a_k] : 0.f;
      lb[r] = (k0 + ii < g.K && j0 + tx < g.J) ? Bm[(k0 + ii) * g.b_k + (j0 + tx) * g.b_j] : 0.f;
    }
  };
#pragma unroll
  for (int sl = 0; sl < NS; ++sl)
    if (32 * sl < g.K) gload(ra[sl], rb[sl], 32 * sl);
  for (int k00 = 0; k00 < g.K; k00 += 32 * NS) {
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
      const int k0 = k00 + 32 * sl;
      if (k0 >= g.K) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        As[ty + 8 * r][tx] = ra[sl][r];
        Bs[ty + 8 * r][tx] = rb[sl][r];
      }
      __syncthreads();
      if (k0 + 32 * NS < g.K) gload(ra[sl], rb[sl], k0 + 32 * NS);
#pragma unroll 8
      for (int k = 0; k < 32; ++k) {
        const float bv = Bs[k][tx];
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = fmaf(As[ty + 8 * r][k], bv, acc[r]);
      }
      __syncthreads();
    }
  }
  float* C = g.C + bt * g.c_b;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = i0 + ty + 8 * r, j = j0 + tx;
    if (i < g.I && j < g.J) {
      float v = g.alpha * acc[r];
      if (g.bias) v = v + g.bias[j];
      float* cp = C + i * g.c_i + j * g.c_j;
      *cp = g.accumulate ? *cp + v : v;
    }
  }
}

// softmax over rows of length N (one workgroup per row), P = softmax(scale * S)
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ S, int N, float scale,
                                                           float* __restrict__ P) {
  __shared__ float red[4];
  const size_t row = blockIdx.x;
  const float* s = S + row * N;
  float m = -INFINITY;
  for (int j = threadIdx.x; j < N; j += 256) m = fmaxf(m, s[j] * scale);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float sum = 0.f;
  for (int j = threadIdx.x; j < N; j += 256) sum += expf(s[j] * scale - m);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  sum = (red[0] + red[1]) + (red[2] + red[3]);
  for (int j = threadIdx.x; j < N; j += 256) P[row * N + j] = expf(s[j] * scale - m) / sum;
}

// dS = scale * P (dP - rowsum(dP P))
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const float* __restrict__ P,
                                                          const float* __restrict__ dP, int N,
                                                          float scale, float* __restrict__ dS) {
  __shared__ float red[4];
  const size_t row = blockIdx.x;
  const float* p = P + row * N;
  const float* d = dP + row * N;
  float acc = 0.f;
  for (int j = threadIdx.x; j < N; j += 256) acc = fmaf(p[j], d[j], acc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  const float dot = (red[0] + red[1]) + (red[2] + red[3]);
  for (int j = threadIdx.x; j < N; j += 256) dS[row * N + j] = scale * (p[j] * (d[j] - dot));
}

// elementwise ops (ertd_eltwise)
enum Elt { ELT_SILU = 0, ELT_SILU_BWD = 1, ELT_RELU = 2, ELT_RELU_BWD = 3, ELT_ADD = 4,
           ELT_SCALE = 5, ELT_COPY_STRIDED = 6 };
__global__ void eltwise_kernel(int op, const float* __restrict__ x, const float* __restrict__ y,
                               float* __restrict__ out, size_t n, float alpha, int accumulate) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float v;
  switch (op) {
    case ELT_SILU: v = silu_f(x[i]); break;
    case ELT_SILU_BWD: v = y[i] * silu_grad(x[i]); break;   // x = pre-activation, y = dL/dout
    case ELT_RELU: v = fmaxf(x[i], 0.f); break;
    case ELT_RELU_BWD: v = x[i] > 0.f ? y[i] : 0.f; break;
    case ELT_ADD: v = x[i] + y[i]; break;
    default: v = alpha * x[i]; break;
  }
  out[i] = accumulate ? out[i] + v : v;
}

// dst[b][d0 + c][p] (+)= src[b][c0 + c][p] for c < Cd: channel slices of (B, C, HW) tensors
__global__ void chan_slice_kernel(const float* __restrict__ src, int Cs, int c0, int Cd, int HW,
                                  size_t n, float* __restrict__ dst, int Cdst, int d0,
                                  int accumulate) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const size_t bc = i / HW;
  const int p = (int)(i - bc * HW);
  const int b = (int)(bc / Cd), c = (int)(bc - (size_t)b * Cd);
  const float v = src[((size_t)b * Cs + c0 + c) * HW + p];
  float* d = dst + ((size_t)b * Cdst + d0 + c) * HW + p;
  *d = accumulate ? *d + v : v;
}

// MSELoss(mean): per-workgroup double partial sums of (e - z)^2 (fixed
// ranges), then one workgroup adds them in order; dout = 2 (e - z) / n
constexpr int MSE_WG = 256;
__global__ __launch_bounds__(256) void mse_part_kernel(const float* __restrict__ e, const float* __restrict__ z,
                                                       size_t n, size_t per, double* __restrict__ part,
                                                       float* __restrict__ dout) {
  __shared__ double red[4];
  double acc = 0.0;
  const float two_n = (float)(2.0 / (double)n);
  const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (size_t i = lo + threadIdx.x; i < hi; i += 256) {
    const float d = e[i] - z[i];
    acc += (double)d * d;
    if (dout) dout[i] = two_n * d;
  }
  acc = wg_sum(acc, red, threadIdx.x);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}
__global__ __launch_bounds__(256) void mse_final_kernel(const double* __restrict__ part, int np, size_t n,
                                                        float* __restrict__ loss) {
  __shared__ double red[4];
  double acc = threadIdx.x < np ? part[threadIdx.x] : 0.0;
  acc = wg_sum(acc, red, threadIdx.x);
  if (threadIdx.x == 0) *loss = (float)(acc / (double)n);
}

// pool mean of the encoder strips' partial sums: m[b][c] = sum_s partial[b][s][c] / L2
__global__ void pool_mean_kernel(const float* __restrict__ partial, int S, int L2, int B,
                                 float* __restrict__ m) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * C2) return;
  const int b = i / C2, c = i - b * C2;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += partial[((size_t)b * S + k) * C2 + c];
  m[i] = s / (float)L2;
}

// torch.optim.Adam over up to 32 tensors per launch
constexpr int ADAM_T = 32;
struct AdamMulti {
  float* p[ADAM_T];
  const float* g[ADAM_T];
  float* m[ADAM_T];
  float* v[ADAM_T];
  long long n[ADAM_T];   // elements of tensor k
  int boff[ADAM_T + 1];  // first workgroup of tensor k (each tensor starts a workgroup)
  int nt;
  float one_minus_b1, b2, one_minus_b2, step_size_neg, bc2_sqrt, eps;
};
// one element, torch.optim.Adam's op order (the same bits as before)
__device__ __forceinline__ void adam_elem(const AdamMulti& a, float g, float& p, float& m, float& v) {
  m = m + a.one_minus_b1 * (g - m);                 // exp_avg.lerp_(grad, 1 - beta1)
  v = v * a.b2;                                     // exp_avg_sq.mul_(beta2)
  v = v + a.one_minus_b2 * g * g;                   //   .addcmul_(grad, grad, 1 - beta2)
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p + a.step_size_neg * (m / denom);
}
// A workgroup belongs to one tensor (found by a workgroup-uniform scan of
// boff: the per-element search over the tensor list cost more than the
// element's memory traffic) and a thread updates 4 consecutive elements with
// float4 accesses where they are whole and 16-B aligned.
__global__ __launch_bounds__(256) void adam_multi_kernel(AdamMulti a) {
  const int blk = blockIdx.x;
  int k = 0;
  while (k + 1 < a.nt && blk >= a.boff[k + 1]) ++k;
  const long long e0 = ((long long)(blk - a.boff[k]) * 256 + threadIdx.x) * 4;
  const long long n = a.n[k];
  if (e0 >= n) return;
  float* P = a.p[k];
  const float* Gp = a.g[k];
  float* M = a.m[k];
  float* V = a.v[k];
  const bool vec = e0 + 4 <= n && ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(Gp) |
                                    reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(V)) & 15) == 0;
  if (vec) {
    const float4 g4 = *reinterpret_cast<const float4*>(Gp + e0);
    float4 p4 = *reinterpret_cast<const float4*>(P + e0);
    float4 m4 = *reinterpret_cast<const float4*>(M + e0);
    float4 v4 = *reinterpret_cast<const float4*>(V + e0);
    adam_elem(a, g4.x, p4.x, m4.x, v4.x);
    adam_elem(a, g4.y, p4.y, m4.y, v4.y);
    adam_elem(a, g4.z, p4.z, m4.z, v4.z);
    adam_elem(a, g4.w, p4.w, m4.w, v4.w);
    *reinterpret_cast<float4*>(P + e0) = p4;
    *reinterpret_cast<float4*>(M + e0) = m4;
    *reinterpret_cast<float4*>(V + e0) = v4;
  } else {
    for (long long e = e0; e < e0 + 4 && e < n; ++e) {
      float p = P[e], m = M[e], v = V[e];
      adam_elem(a, Gp[e], p, m, v);
      P[e] = p;
      M[e] = m;
      V[e] = v;
    }
  }
}

// dst = cat(src[0], src[1], ...) over up to 64 contiguous tensors per launch
constexpr int CAT_T = 64;
struct CatMulti {
  const float* src[CAT_T];
  long long off[CAT_T + 1];
  int nt;
};
__global__ __launch_bounds__(256) void concat_kernel(CatMulti c, float* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= c.off[c.nt]) return;
  int k = 0;
  while (k + 1 < c.nt && i >= c.off[k + 1]) ++k;
  dst[i] = c.src[k][i - c.off[k]];
}

// dst[k] = alpha * src[off[k] .. off[k+1]) (the inverse of concat_kernel, scaled)
struct SplitMulti {
  float* dst[CAT_T];
  long long off[CAT_T + 1];
  int nt;
};
__global__ __launch_bounds__(256) void split_kernel(SplitMulti c, const float* __restrict__ src,
                                                    float alpha) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= c.off[c.nt]) return;
  int k = 0;
  while (k + 1 < c.nt && i >= c.off[k + 1]) ++k;
  c.dst[k][i - c.off[k]] = alpha * src[i];
}

inline unsigned nblk(size_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

namespace ertd {
namespace unet {
hipError_t launch_zero_insert(const float* x, int B, int C, int Ho, float* out, hipStream_t s) {
  const size_t n = (size_t)B * C * 4 * Ho * Ho;
  zero_insert_kernel<<<nblk(n), 256, 0, s>>>(x, Ho, n, out);
  return hipGetLastError();
}
hipError_t launch_sum_pool2(const float* x, int B, int C, int H, float* out, int accumulate,
                            hipStream_t s) {
  const size_t n = (size_t)B * C * H * H;
  sum_pool2_kernel<<<nblk(n), 256, 0, s>>>(x, H, n, out, accumulate);
  return hipGetLastError();
}
}  // namespace unet
}  // namespace ertd

extern "C" {

int ertd_gn_stats_mr(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                     const float* gamma, const float* beta, float* ss_out, float* mr_out,
                     void* stream) {
  const int C = Ca + Cb;
  if (!x || !gamma || !beta || !ss_out || B < 1 || Ca < 1 || Cb < 0 || (Cb > 0 && !x2) ||
      groups < 1 || C % groups || HW < 4 || HW % 4)
    return ERTD_EINVAL;
  GnArgs g{x, x2, Ca, Cb, HW, groups, gamma, beta, (float2*)ss_out, (float2*)mr_out};
  return rcode(launch_gn_stats(g, B, (hipStream_t)stream));
}

int ertd_gn_act_apply(const float* x, int Ca, const float* x2, int Cb, int B, int HW,
                      const float* ss, int act, float* out, void* stream) {
  if (!x || !ss || !out || B < 1 || Ca < 1 || Cb < 0 || (Cb > 0 && !x2) || HW < 1 ||
      (act != ACT_GN_SILU && act != ACT_GN))
    return ERTD_EINVAL;
  const size_t n = (size_t)B * (Ca + Cb) * HW;
  gn_act_apply_kernel<<<nblk(n), 256, 0, (hipStream_t)stream>>>(x, Ca, x2, Cb, HW, (const float2*)ss,
                                                                 act, n, out);
  return rcode(hipGetLastError());
}

static int gn_act_backward(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                           const float* gamma, const float* beta, const float* mr, int act,
                           const float* dy, float* dx, float* dx2, int accumulate, float* dgb_part,
                           float* csum, long long ldc, const float* addc, void* stream) {
  const int C = Ca + Cb;
  if (!x || !gamma || !beta || !mr || !dy || !dx || !dgb_part || B < 1 || Ca < 1 || Cb < 0 ||
      (Cb > 0 && (!x2 || !dx2)) || groups < 1 || C % groups || HW < 4 || HW % 4 ||
      (act != ACT_GN_SILU && act != ACT_GN) || (csum && (C / groups > GNB_CB || ldc < C)))
    return ERTD_EINVAL;
  const dim3 grid(groups, B);
  hipStream_t s = (hipStream_t)stream;
  gn_act_bwd_kernel<<<grid, 256, 0, s>>>(x, Ca, x2, Cb, HW, groups, gamma, beta, (const float2*)mr, act,
                                         dy, dx, dx2, accumulate, dgb_part, csum, ldc, addc);
  return rcode(hipGetLastError());
}

int ertd_gn_act_backward(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                         const float* gamma, const float* beta, const float* mr, int act,
                         const float* dy, float* dx, float* dx2, int accumulate, float* dgb_part,
                         void* stream) {
  return gn_act_backward(x, Ca, x2, Cb, B, HW, groups, gamma, beta, mr, act, dy, dx, dx2, accumulate,
                         dgb_part, nullptr, 0, nullptr, stream);
}

int ertd_gn_act_backward_csum(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                              const float* gamma, const float* beta, const float* mr, int act,
                              const float* dy, float* dx, float* dx2, int accumulate, float* dgb_part,
                              float* csum, long long ldc, void* stream) {
  if (!csum) return ERTD_EINVAL;
  return gn_act_backward(x, Ca, x2, Cb, B, HW, groups, gamma, beta, mr, act, dy, dx, dx2, accumulate,
                         dgb_part, csum, ldc, nullptr, stream);
}

int ertd_gn_act_backward_add(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                             const float* gamma, const float* beta, const float* mr, int act,
                             const float* dy, const float* addc, float* dx, float* dx2, int accumulate,
                             float* dgb_part, float* csum, long long ldc, void* stream) {
  if (!addc) return ERTD_EINVAL;
  return gn_act_backward(x, Ca, x2, Cb, B, HW, groups, gamma, beta, mr, act, dy, dx, dx2, accumulate,
                         dgb_part, csum, ldc, addc, stream);
}

int ertd_im2col(const float* x, int C, int B, int H, int ks, int mode, float* out, void* stream) {
  if (!x || !out || C < 1 || B < 1 || H < 1 || (ks != 1 && ks != 3) || mode < MODE_S1 ||
      mode > MODE_UP || (ks == 1 && mode != MODE_S1))
    return ERTD_EINVAL;
  const int Ho = mode == MODE_S2 ? H / 2 : (mode == MODE_UP ? 2 * H : H);
  const size_t n = (size_t)B * C * ks * ks * Ho * Ho;
  im2col_kernel<<<nblk(n), 256, 0, (hipStream_t)stream>>>(x, C, H, ks, mode, Ho, n, out);
  return rcode(hipGetLastError());
}

size_t ertd_wgrad_ws_bytes(int M, int N, int P, int B) {
  if (M < 1 || N < 1 || P < 1 || B < 1) return 0;
  const int nsp = (P + 4095) / 4096;
  return (size_t)B * nsp * M * N * sizeof(float);
}

int ertd_wgrad_gemm(const float* dY, const float* X, int M, int N, int P, int B, long long bsA,
                    long long bsB, float* dW, int accumulate, void* ws, size_t ws_bytes,
                    void* stream) {
  if (!dY || !X || !dW || !ws || M < 1 || N < 1 || P < 1 || B < 1) return ERTD_EINVAL;
  if (ertd_wgrad_ws_bytes(M, N, P, B) > ws_bytes) return ERTD_ENOSPC;
  const int split_len = 4096, nsp = (P + split_len - 1) / split_len;
  hipStream_t s = (hipStream_t)stream;
  wgrad_kernel<<<dim3((N + 63) / 64, (M + 63) / 64, B * nsp), 256, 0, s>>>(
      dY, X, M, N, P, (size_t)bsA, (size_t)bsB, (float*)ws, split_len, nsp);
  const size_t cols = (size_t)M * N;
  reduce_rows_kernel<<<(unsigned)((cols + 63) / 64), 256, 0, s>>>((const float*)ws, B * nsp, cols, dW,
                                                                   accumulate);
  return rcode(hipGetLastError());
}

int ertd_reduce_rows(const float* part, int rows, long long cols, float* out, int accumulate,
                     void* stream) {
  if (!part || !out || rows < 1 || cols < 1) return ERTD_EINVAL;
  reduce_rows_kernel<<<(unsigned)((cols + 63) / 64), 256, 0, (hipStream_t)stream>>>(part, rows, (size_t)cols,
                                                                                   out, accumulate);
  return rcode(hipGetLastError());
}

int ertd_reduce_rows_multi(const float* const* parts, const int* rows, const long long* cols,
                           float* const* outs, const int* accumulate, int n, void* stream) {
  if (!parts || !rows || !cols || !outs || !accumulate || n < 0) return ERTD_EINVAL;
  for (int i = 0; i < n; ++i)
    if (!parts[i] || !outs[i] || rows[i] < 1 || cols[i] < 1) return ERTD_EINVAL;
  for (int t0 = 0; t0 < n; t0 += RM_T) {
    ReduceMulti a{};
    a.n = n - t0 < RM_T ? n - t0 : RM_T;
    long long nb = 0;
    for (int i = 0; i < a.n; ++i) {
      a.part[i] = parts[t0 + i];
      a.out[i] = outs[t0 + i];
      a.rows[i] = rows[t0 + i];
      a.cols[i] = cols[t0 + i];
      a.acc[i] = accumulate[t0 + i];
      a.blk[i] = (int)nb;
      nb += (cols[t0 + i] + 63) / 64;
    }
    if (nb > 0x7fffffffLL) return ERTD_EINVAL;
    a.blk[a.n] = (int)nb;
    reduce_rows_multi_kernel<<<(unsigned)nb, 256, 0, (hipStream_t)stream>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return ERTD_OK;
}

int ertd_conv_weight_flip(const float* w, int Cout, int Cin, int ks, float* out, void* stream) {
  if (!w || !out || Cout < 1 || Cin < 1 || (ks != 1 && ks != 3)) return ERTD_EINVAL;
  weight_flip_kernel<<<nblk((size_t)Cout * Cin * ks * ks), 256, 0, (hipStream_t)stream>>>(w, Cout, Cin,
                                                                                          ks, out);
  return rcode(hipGetLastError());
}

int ertd_zero_insert(const float* x, int B, int C, int Ho, float* out, void* stream) {
  if (!x || !out || B < 1 || C < 1 || Ho < 1) return ERTD_EINVAL;
  const size_t n = (size_t)B * C * 4 * Ho * Ho;
  zero_insert_kernel<<<nblk(n), 256, 0, (hipStream_t)stream>>>(x, Ho, n, out);
  return rcode(hipGetLastError());
}

int ertd_sum_pool2(const float* x, int B, int C, int H, float* out, int accumulate, void* stream) {
  if (!x || !out || B < 1 || C < 1 || H < 1) return ERTD_EINVAL;
  const size_t n = (size_t)B * C * H * H;
  sum_pool2_kernel<<<nblk(n), 256, 0, (hipStream_t)stream>>>(x, H, n, out, accumulate);
  return rcode(hipGetLastError());
}

int ertd_channel_sums(const float* x, int B, int C, int HW, float* out_bc, int ldo, float* out_c,
                      int accumulate_c, void* stream) {
  if (ldo == 0) ldo = C;
  if (!x || !out_bc || B < 1 || C < 1 || HW < 1 || ldo < C || (out_c && ldo != C)) return ERTD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  chan_sum_kernel<<<(unsigned)((size_t)B * C), 256, 0, s>>>(x, HW, C, ldo, out_bc);
  if (out_c)
    reduce_rows_kernel<<<(unsigned)((C + 63) / 64), 256, 0, s>>>(out_bc, B, (size_t)C, out_c, accumulate_c);
  return rcode(hipGetLastError());
}

int ertd_gemm_small(const float* A, long long a_i, long long a_k, long long a_b, const float* Bm,
                    long long b_k, long long b_j, long long b_b, float* C, long long c_i,
                    long long c_j, long long c_b, const float* bias, int I, int J, int K, int batch,
                    float alpha, int accumulate, void* stream) {
  if (!A || !Bm || !C || I < 1 || J < 1 || K < 1 || batch < 1) return ERTD_EINVAL;
  SmallGemm g{A, a_i, a_k, a_b, Bm, b_k, b_j, b_b, C, c_i, c_j, c_b, bias, I, J, K, alpha, accumulate};
  gemm_small_kernel<<<dim3((J + 31) / 32, (I + 31) / 32, batch), 256, 0, (hipStream_t)stream>>>(g);
  return rcode(hipGetLastError());
}

int ertd_softmax_rows(const float* S, long long rows, int N, float scale, float* P, void* stream) {
  if (!S || !P || rows < 1 || N < 1) return ERTD_EINVAL;
  softmax_rows_kernel<<<(unsigned)rows, 256, 0, (hipStream_t)stream>>>(S, N, scale, P);
  return rcode(hipGetLastError());
}

int ertd_softmax_backward(const float* P, const float* dP, long long rows, int N, float scale,
                          float* dS, void* stream) {
  if (!P || !dP || !dS || rows < 1 || N < 1) return ERTD_EINVAL;
  softmax_bwd_kernel<<<(unsigned)rows, 256, 0, (hipStream_t)stream>>>(P, dP, N, scale, dS);
  return rcode(hipGetLastError());
}

int ertd_eltwise(int op, const float* x, const float* y, float* out, long long n, float alpha,
                 int accumulate, void* stream) {
  if (!x || !out || n < 1 || op < ELT_SILU || op > ELT_SCALE ||
      ((op == ELT_SILU_BWD || op == ELT_RELU_BWD || op == ELT_ADD) && !y))
    return ERTD_EINVAL;
  eltwise_kernel<<<nblk((size_t)n), 256, 0, (hipStream_t)stream>>>(op, x, y, out, (size_t)n, alpha,
                                                                   accumulate);
  return rcode(hipGetLastError());
}

int ertd_channel_slice(const float* src, int B, int Cs, int c0, int Cd, int HW, float* dst,
                       int Cdst, int d0, int accumulate, void* stream) {
  if (!src || !dst || B < 1 || Cd < 1 || c0 < 0 || c0 + Cd > Cs || d0 < 0 || d0 + Cd > Cdst ||
      HW < 1)
    return ERTD_EINVAL;
  const size_t n = (size_t)B * Cd * HW;
  chan_slice_kernel<<<nblk(n), 256, 0, (hipStream_t)stream>>>(src, Cs, c0, Cd, HW, n, dst, Cdst, d0,
                                                              accumulate);
  return rcode(hipGetLastError());
}

size_t ertd_mse_loss_ws_bytes(void) { return MSE_WG * sizeof(double); }

int ertd_mse_loss(const float* eps, const float* noise, long long n, float* loss, float* dout,
                  void* ws, size_t ws_bytes, void* stream) {
  if (!eps || !noise || !loss || n < 1 || !ws) return ERTD_EINVAL;
  if (ws_bytes < ertd_mse_loss_ws_bytes()) return ERTD_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  const size_t per = (((size_t)n + MSE_WG - 1) / MSE_WG + 255) / 256 * 256;
  const int np = (int)(((size_t)n + per - 1) / per);
  double* part = (double*)ws;   // caller-owned float64 partials (fixed-order final sum)
  mse_part_kernel<<<np, 256, 0, s>>>(eps, noise, (size_t)n, per, part, dout);
  mse_final_kernel<<<1, 256, 0, s>>>(part, np, (size_t)n, loss);
  return rcode(hipGetLastError());
}

// the reference condition encoder with saved activations (train.hip: pool
// partials, conv1 strip images, conv2 ReLU mask bits) and the backward's strip
// partial rows; packed = ertd_encoder_train_pack's copy of the conv weights
size_t ertd_encoder_train_ws_bytes(int B, int L) {
  if (B < 1 || L < 1) return 0;
  return encoder_train_ws_floats(B, L) * sizeof(float);
}

int ertd_encoder_train_pack(const float* w0, const float* w2, float* packed, void* stream) {
  if (!w0 || !w2 || !packed) return ERTD_EINVAL;
  return rcode(launch_pack_encoder_convs(w0, w2, packed, (hipStream_t)stream));
}

int ertd_encoder_train_fwd(const float* packed, const float* b1, const float* b2, const float* cond,
                           int B, int L, float* m_out, void* ws, size_t ws_bytes, void* stream) {
  if (!packed || !b1 || !b2 || !cond || !m_out || !ws || B < 1 || L < 1) return ERTD_EINVAL;
  if (ertd_encoder_train_ws_bytes(B, L) > ws_bytes) return ERTD_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  float* partial = nullptr;
  hipError_t e = launch_encoder_train(packed, b1, packed + ENC_RAW_W2, b2, cond, B, L, (float*)ws,
                                      &partial, s);
  if (e != hipSuccess) return (int)e;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  pool_mean_kernel<<<nblk((size_t)B * C2), 256, 0, s>>>(partial, S, L2, B, m_out);
  return rcode(hipGetLastError());
}

// g = dL/dm / L2 (B, 64) -> conv weight / bias grads of the encoder (after ertd_encoder_train_fwd on ws)
int ertd_encoder_train_bwd(const float* packed, const float* cond, const float* g, int B, int L,
                           float* dw1, float* db1, float* dw2, float* db2, void* ws,
                           size_t ws_bytes, void* stream) {
  if (!packed || !cond || !g || !dw1 || !db1 || !dw2 || !db2 || !ws || B < 1 || L < 1)
    return ERTD_EINVAL;
  if (ertd_encoder_train_ws_bytes(B, L) > ws_bytes) return ERTD_ENOSPC;
  return rcode(launch_encoder_conv_backward(packed + ENC_RAW_W2, cond, g, B, L, (float*)ws, dw1, db1,
                                            dw2, db2, (hipStream_t)stream));
}

int ertd_concat(const float* const* srcs, const long long* sizes, int n, float* dst, void* stream) {
  if (!srcs || !sizes || !dst || n < 1) return ERTD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  long long base = 0;
  for (int t0 = 0; t0 < n; t0 += CAT_T) {
    CatMulti c{};
    c.nt = n - t0 < CAT_T ? n - t0 : CAT_T;
    long long off = 0;
    for (int k = 0; k < c.nt; ++k) {
      if (!srcs[t0 + k] || sizes[t0 + k] < 0) return ERTD_EINVAL;
      c.src[k] = srcs[t0 + k];
      c.off[k] = off;
      off += sizes[t0 + k];
    }
    c.off[c.nt] = off;
    if (off > 0) concat_kernel<<<nblk((size_t)off), 256, 0, s>>>(c, dst + base);
    base += off;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return ERTD_OK;
}

int ertd_split(const float* src, float* const* dsts, const long long* sizes, int n, float alpha,
               void* stream) {
  if (!src || !dsts || !sizes || n < 1) return ERTD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  long long base = 0;
  for (int t0 = 0; t0 < n; t0 += CAT_T) {
    SplitMulti c{};
    c.nt = n - t0 < CAT_T ? n - t0 : CAT_T;
    long long off = 0;
    for (int k = 0; k < c.nt; ++k) {
      if (!dsts[t0 + k] || sizes[t0 + k] < 0) return ERTD_EINVAL;
      c.dst[k] = dsts[t0 + k];
      c.off[k] = off;
      off += sizes[t0 + k];
    }
    c.off[c.nt] = off;
    if (off > 0) split_kernel<<<nblk((size_t)off), 256, 0, s>>>(c, src + base, alpha);
    base += off;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return ERTD_OK;
}

int ertd_adam_multi(float* const* params, const float* const* grads, float* const* exp_avg,
                    float* const* exp_avg_sq, const long long* sizes, int ntensors, int step,
                    float lr, float beta1, float beta2, float eps, void* stream) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || !sizes || ntensors < 1 || step < 1)
    return ERTD_EINVAL;
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  hipStream_t s = (hipStream_t)stream;
  for (int t0 = 0; t0 < ntensors; t0 += ADAM_T) {
    AdamMulti a{};
    a.nt = ntensors - t0 < ADAM_T ? ntensors - t0 : ADAM_T;
    long long blocks = 0;
    for (int k = 0; k < a.nt; ++k) {
      if (sizes[t0 + k] < 0) return ERTD_EINVAL;
      a.p[k] = params[t0 + k];
      a.g[k] = grads[t0 + k];
      a.m[k] = exp_avg[t0 + k];
      a.v[k] = exp_avg_sq[t0 + k];
      a.n[k] = sizes[t0 + k];
      a.boff[k] = (int)blocks;
      blocks += (sizes[t0 + k] + 1023) / 1024;   // 256 threads x 4 elements
    }
    a.boff[a.nt] = (int)blocks;
    if (blocks == 0) continue;
    // scalars formed as torch does: Python floats (double), rounded when applied to fp32
    a.one_minus_b1 = (float)(1.0 - (double)beta1);
    a.b2 = beta2;
    a.one_minus_b2 = (float)(1.0 - (double)beta2);
    a.step_size_neg = (float)(-((double)lr / bc1));
    a.bc2_sqrt = (float)std::sqrt(bc2);
    a.eps = eps;
    adam_multi_kernel<<<(unsigned)blocks, 256, 0, s>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return ERTD_OK;
}

}  // extern "C"
