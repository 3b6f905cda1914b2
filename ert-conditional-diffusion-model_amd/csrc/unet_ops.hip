// Non-conv kernels of the build-defined U-Net (see unet.h): GroupNorm
// statistics, the small dense layers of the embedding path, the mid-block
// attention core, the DDPM update, and the step-counter words of a sampler
// step graph.
#include <cmath>

#include "head_dev.h"  // ddpm_update: the sampler update expression shared with head.hip
#include "unet.h"

namespace ertd {
namespace unet {

// ---- GroupNorm statistics -------------------------------------------------------
// One 256-thread workgroup per (group, sample).  Each thread accumulates its
// elements in float64 in a fixed order, the workgroup reduces in a fixed tree,
// so the result is deterministic; the output is ATen's folded form
// scale = gamma*rstd, shift = beta - mean*scale (per channel), which the conv
// prologue applies as x*scale + shift.
__global__ __launch_bounds__(256) void gn_stats_kernel(GnArgs a) {
  const int g = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int C = a.Ca + a.Cb;
  const int cpg = C / a.groups;
  const int HW = a.HW;
  double s = 0.0, ss = 0.0;
  auto acc4 = [&](const float4 v) {
    s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
    ss += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  };
  const int c0 = g * cpg;
  if (c0 + cpg <= a.Ca || c0 >= a.Ca) {
    // the group's channels are one contiguous run of cpg*HW floats: one flat
    // loop keeps every thread busy (cpg*HW/4 float4s), 4 loads in flight
    const float* src = c0 < a.Ca ? a.srcA + ((size_t)b * a.Ca + c0) * HW
                                 : a.srcB + ((size_t)b * a.Cb + (c0 - a.Ca)) * HW;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    const int n4 = cpg * HW / 4;
    int i = tid;
    for (; i + 3 * 256 < n4; i += 4 * 256) {
      const float4 v0 = s4[i], v1 = s4[i + 256], v2 = s4[i + 512], v3 = s4[i + 768];
      acc4(v0); acc4(v1); acc4(v2); acc4(v3);
    }
    for (; i < n4; i += 256) acc4(s4[i]);
  } else {
    for (int cl = 0; cl < cpg; ++cl) {   // a group split by the skip concatenation
      const int c = c0 + cl;
      const float* src = c < a.Ca ? a.srcA + ((size_t)b * a.Ca + c) * HW
                                  : a.srcB + ((size_t)b * a.Cb + (c - a.Ca)) * HW;
      const float4* s4 = reinterpret_cast<const float4*>(src);
      for (int i = tid; i < HW / 4; i += 256) acc4(s4[i]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    ss += __shfl_xor(ss, o);
  }
  __shared__ double red[2][4];
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = s;
    red[1][tid >> 6] = ss;
  }
  __syncthreads();
  const double n = (double)cpg * HW;
  const double S = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  const double SS = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  const double mean = S / n;
  double var = SS / n - mean * mean;
  var = var > 0.0 ? var : 0.0;
  const float rstd = (float)(1.0 / sqrt(var + GN_EPS));
  if (a.mr && tid == 0) a.mr[(size_t)b * a.groups + g] = make_float2((float)mean, rstd);
  // a group may hold more channels than the workgroup has threads (groups=1
  // at C=512): every channel of the group gets its {scale, shift}
  for (int cl = tid; cl < cpg; cl += 256) {
    const int c = g * cpg + cl;
    const float scale = rstd * a.gamma[c];
    const float shift = -scale * (float)mean + a.beta[c];
    a.out[(size_t)b * C + c] = make_float2(scale, shift);
  }
}

hipError_t launch_gn_stats(const GnArgs& a, int B, hipStream_t s) {
  gn_stats_kernel<<<dim3(a.groups, B), 256, 0, s>>>(a);
  return hipGetLastError();
}

// ---- GroupNorm statistics from partials (unet.h, GnPartArgs) ---------------------
// Partials of a tensor, parts of n = 256 pixels: one wave per 4 parts of one
// (sample, channel) plane, one float4 per lane and part, every load issued
// before the arithmetic; a butterfly over the wave (the same bits in every
// lane) gives the part sum, then the squared deviations from the part mean
// of the same registers.
__global__ __launch_bounds__(256) void gn_partials_kernel(const float* __restrict__ x, int np,
                                                          float2* __restrict__ out, long long nplanes) {
  const long long w = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);   // global wave
  const int lane = threadIdx.x & 63;
  const int groups4 = (np + 3) / 4;
  const long long plane = w / groups4;
  if (plane >= nplanes) return;
  const int p0 = (int)(w - plane * groups4) * 4;
  const float4* src = reinterpret_cast<const float4*>(x + plane * (long long)np * 256);
  float4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = p0 + j < np ? src[(p0 + j) * 64 + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (p0 + j >= np) break;
    float sm = (v[j].x + v[j].y) + (v[j].z + v[j].w);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sm += __shfl_xor(sm, o);
    const float mu = sm * (1.0f / 256.0f);
    const float dx = v[j].x - mu, dy = v[j].y - mu, dz = v[j].z - mu, dw = v[j].w - mu;
    float m2 = fmaf(dx, dx, fmaf(dy, dy, fmaf(dz, dz, dw * dw)));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m2 += __shfl_xor(m2, o);
    if (lane == 0) out[plane * np + p0 + j] = make_float2(sm, m2);
  }
}

hipError_t launch_gn_partials(const float* x, int C, int HW, int np, float2* out, int B, hipStream_t s) {
  if (C < 1 || np < 1 || HW != np * 256) return hipErrorInvalidValue;
  const long long nplanes = (long long)B * C;
  const long long waves = nplanes * ((np + 3) / 4);
  gn_partials_kernel<<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(x, np, out, nplanes);
  return hipGetLastError();
}

// float64 wave sum in a fixed order, the same bits in every lane: DPP row
// sums (row16_sum's pairing on both halves of the double), then the four row
// sums as (r0 + r1) + (r2 + r3) by readlane -- no LDS round trips (a
// __shfl_xor butterfly on doubles is 12 dependent ds_bpermutes)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// One wave per (sample, GN_LPG-group chunk): unet.h gn_group_finalize (the
// same arithmetic as the producing convs' GroupNorm fold): float64 Chan merge
// of the parts {sum, M2 about the part mean} in a fixed order, var = M2 / N
// (biased, as GroupNorm); {scale, shift} as gn_stats_kernel.
__global__ __launch_bounds__(256) void gn_finalize_kernel(GnPartArgs a, int B) {
  const int nparts = (a.groups + 64 / GN_LPG - 1) / (64 / GN_LPG);
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wv >= B * nparts) return;
  const int b = wv / nparts;
  gn_group_finalize<false>(a, b, lane, wv - b * nparts, nparts);
}

#ifdef GN_FIN_TWICE
__global__ void gn_fin_nop_kernel() {}
#endif

hipError_t launch_gn_finalize(const GnPartArgs& a, int B, hipStream_t s) {
  const int C = a.Ca + a.Cb;
  if (!a.pa || a.npa < 1 || a.Ca < 1 || (a.Cb > 0 && (!a.pb || a.npb < 1)) || a.groups < 1 ||
      C % a.groups || a.HW % a.npa || (a.Cb > 0 && a.HW % a.npb))
    return hipErrorInvalidValue;
  const int n = B * ((a.groups + 64 / GN_LPG - 1) / (64 / GN_LPG));   // one wave each
  gn_finalize_kernel<<<(n + 3) / 4, 256, 0, s>>>(a, B);
#ifdef GN_FIN_TWICE   // diagnostic variants only: the cost of one more launch in the step graph
#if GN_FIN_TWICE == 1
  gn_finalize_kernel<<<(n + 3) / 4, 256, 0, s>>>(a, B);
#else
  gn_fin_nop_kernel<<<1, 64, 0, s>>>();
#endif
#endif
  return hipGetLastError();
}

// ---- dense layers of the embedding path --------------------------------------------
// One workgroup per (256 outputs, sample); the input row is formed once in LDS
// (plain, SiLU, or the reference's sinusoid of t), then each thread runs one
// k-ordered fma chain over the k-major weights (coalesced across threads).
template <int DIN>
__global__ __launch_bounds__(256) void dense_kernel(DenseArgs a) {
  extern __shared__ float xin[];
  const int b = blockIdx.y, tid = threadIdx.x;
  const int K = a.K;
  if constexpr (DIN == DIN_SINUSOID) {
    const float tf = (float)(a.t ? a.t[b] : (int64_t)*a.t_dev);
    const int half = K / 2;
    for (int k = tid; k < K; k += 256)
      xin[k] = k < half ? sinf(tf * a.freq[k]) : cosf(tf * a.freq[k - half]);
  } else {
    for (int k = tid; k < K; k += 256) {
      const float v = a.x[(size_t)b * a.x_stride + k];
      xin[k] = DIN == DIN_SILU ? v / (1.0f + expf(-v)) : v;
    }
  }
  __syncthreads();
  // 64 outputs per workgroup, K split in four quarters (one per wave): each
  // thread runs one k-ordered fma chain over its quarter with every weight
  // load of a 64-step batch in flight (K = 256: one memory latency instead of
  // four), the quarters then added in order (q0 + q1) + (q2 + q3)
  __shared__ float part[4][64];
  const int ol = tid & 63, q = tid >> 6;
  const int o = blockIdx.x * 64 + ol;
  const int kq = (K + 3) / 4, kb = q * kq, ke = min(K, kb + kq);
  float acc = 0.f;
  if (o < a.O) {
    int k0 = kb;
    for (; k0 + 64 <= ke; k0 += 64) {
      float w[64];
#pragma unroll
      for (int j = 0; j < 64; ++j) w[j] = a.wt[(size_t)(k0 + j) * a.O + o];
#pragma unroll
      for (int j = 0; j < 64; ++j) acc = fmaf(xin[k0 + j], w[j], acc);
    }
    for (; k0 + 16 <= ke; k0 += 16) {
      float w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) w[j] = a.wt[(size_t)(k0 + j) * a.O + o];
#pragma unroll
      for (int j = 0; j < 16; ++j) acc = fmaf(xin[k0 + j], w[j], acc);
    }
    for (; k0 < ke; ++k0) acc = fmaf(xin[k0], a.wt[(size_t)k0 * a.O + o], acc);
  }
  part[q][ol] = acc;
  __syncthreads();
  if (q != 0 || o >= a.O) return;
  float v = (part[0][ol] + part[1][ol]) + (part[2][ol] + part[3][ol]);
  v = v + a.bias[o];
  if (a.add) v = v + a.add[(size_t)(a.add_bcast ? 0 : b) * a.add_stride + o];
  a.y[(size_t)b * a.y_stride + o] = v;
}

hipError_t launch_dense(int din, const DenseArgs& a, int B, hipStream_t s) {
  if (a.K < 1 || a.O < 1) return hipErrorInvalidValue;
  dim3 grid((a.O + 63) / 64, B);
  const size_t lds = (size_t)a.K * sizeof(float);
  if (din == DIN_PLAIN) dense_kernel<DIN_PLAIN><<<grid, 256, lds, s>>>(a);
  else if (din == DIN_SILU) dense_kernel<DIN_SILU><<<grid, 256, lds, s>>>(a);
  else if (din == DIN_SINUSOID) dense_kernel<DIN_SINUSOID><<<grid, 256, lds, s>>>(a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// W (O, K) row-major -> dst[k * dst_ld + o]
__global__ void transpose_kernel(const float* __restrict__ w, int O, int K, float* __restrict__ dst,
                                 int dst_ld) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= O * K) return;
  const int o = i / K, k = i - o * K;
  dst[(size_t)k * dst_ld + o] = w[i];
}

hipError_t launch_transpose(const float* w, int O, int K, float* dst, int dst_ld, hipStream_t s) {
  transpose_kernel<<<(O * K + 255) / 256, 256, 0, s>>>(w, O, K, dst, dst_ld);
  return hipGetLastError();
}

// ---- mid-block attention core (fp32 MFMA) -------------------------------------------------
// One workgroup per (64 queries, sample), 4 waves.  S = Q^T K over C (each
// wave 64 queries x 64 keys), scaled by 1/sqrt(C), row softmax across the 4
// waves (LDS), P^T kept in LDS, then O = V P^T (each wave 64 channels x 64
// queries per pass).  qkv: (B, 3C, N) = q | k | v channel blocks.
constexpr int AQ = 64;        // queries per workgroup
constexpr int APITCH = AQ + 1;

__global__ __launch_bounds__(256) void attention_kernel(const float* __restrict__ qkv, int C, int N,
                                                        float inv_scale_div,
                                                        float* __restrict__ out) {
  extern __shared__ float sm[];
  float* PT = sm;                       // [N][APITCH]: P^T (key-major)
  float* red = sm + (size_t)N * APITCH; // [4][AQ]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.y, i0 = blockIdx.x * AQ;
  const float* q = qkv + (size_t)b * 3 * C * N;
  const float* k = q + (size_t)C * N;
  const float* v = k + (size_t)C * N;

  for (int jb = 0; jb < N; jb += 256) {  // key blocks of 256 (N <= 256 supported: one block)
    const int j0 = jb + w * 64;
    f32x16 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = f32x16{};
    // operands straight from global memory (L2), in batches of 8 k-steps
    // whose 32 loads are all issued before the batch's MFMAs (one load
    // latency per batch instead of per k-step; same MFMA order)
    // (double-buffered: the next batch's loads are issued before this
    // batch's MFMAs; one wave per SIMD here, so the registers are there)
    constexpr int KBT = 8;
    float a0[2][KBT], a1[2][KBT], b0[2][KBT], b1[2][KBT];
    auto load_b = [&](const int buf, const int s0) {
#pragma unroll
      for (int u = 0; u < KBT; ++u) {
        const int c = 2 * (s0 + u) + h;
        const bool ok = s0 + u < C / 2;
        a0[buf][u] = ok ? q[(size_t)c * N + i0 + l32] : 0.f;
        a1[buf][u] = ok ? q[(size_t)c * N + i0 + 32 + l32] : 0.f;
        b0[buf][u] = ok ? k[(size_t)c * N + j0 + l32] : 0.f;
        b1[buf][u] = ok ? k[(size_t)c * N + j0 + 32 + l32] : 0.f;
      }
    };
    auto mfma_b = [&](const int buf, const int s0) {
#pragma unroll
      for (int u = 0; u < KBT; ++u) {
        if (s0 + u >= C / 2) break;
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[buf][u], b0[buf][u], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[buf][u], b1[buf][u], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[buf][u], b0[buf][u], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[buf][u], b1[buf][u], acc[1][1], 0, 0, 0);
      }
    };
    load_b(0, 0);
    for (int s0 = 0; s0 < C / 2; s0 += 2 * KBT) {
      load_b(1, s0 + KBT);            // past C/2: zero operands, MFMAs skipped
      mfma_b(0, s0);
      load_b(0, s0 + 2 * KBT);
      mfma_b(1, s0 + KBT);
    }
    // scale, row max over this wave's 64 keys
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[x][0][r] = acc[x][0][r] / inv_scale_div;
        acc[x][1][r] = acc[x][1][r] / inv_scale_div;
        float m = fmaxf(acc[x][0][r], acc[x][1][r]);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
        const int i = x * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (l32 == 0) red[w * AQ + i] = m;
      }
    __syncthreads();
    float rmax[2][16];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = x * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        rmax[x][r] = fmaxf(fmaxf(red[i], red[AQ + i]), fmaxf(red[2 * AQ + i], red[3 * AQ + i]));
      }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e0 = expf(acc[x][0][r] - rmax[x][r]);
        const float e1 = expf(acc[x][1][r] - rmax[x][r]);
        acc[x][0][r] = e0;
        acc[x][1][r] = e1;
        float sum = e0 + e1;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) sum += __shfl_xor(sum, o);
        const int i = x * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (l32 == 0) red[w * AQ + i] = sum;
      }
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = x * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float sum = (red[i] + red[AQ + i]) + (red[2 * AQ + i] + red[3 * AQ + i]);
        PT[(size_t)(j0 + l32) * APITCH + i] = acc[x][0][r] / sum;
        PT[(size_t)(j0 + 32 + l32) * APITCH + i] = acc[x][1][r] / sum;
      }
  }
  __syncthreads();

  // O[c][i] = sum_j V[c][j] P[i][j]; lane half h takes keys 8g+4h..8g+4h+3 over
  // steps 4g..4g+3, so its V operands are one float4 per 4 steps.
  for (int cb = 0; cb < C; cb += 256) {
    const int c0 = cb + w * 64;
    if (c0 >= C) break;
    f32x16 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = f32x16{};
    // V rows in batches of 4 groups (8 float4 loads in flight per lane)
    constexpr int GBT = 4;
    for (int g0 = 0; g0 < N / 8; g0 += GBT) {
      float4 va[GBT], vb[GBT];
#pragma unroll
      for (int u = 0; u < GBT; ++u) {
        const int g = g0 + u < N / 8 ? g0 + u : g0;
        va[u] = *reinterpret_cast<const float4*>(v + (size_t)(c0 + l32) * N + 8 * g + 4 * h);
        vb[u] = *reinterpret_cast<const float4*>(v + (size_t)(c0 + 32 + l32) * N + 8 * g + 4 * h);
      }
#pragma unroll
      for (int u = 0; u < GBT; ++u) {
        const int g = g0 + u;
        if (g >= N / 8) break;
        const float A0[4] = {va[u].x, va[u].y, va[u].z, va[u].w};
        const float A1[4] = {vb[u].x, vb[u].y, vb[u].z, vb[u].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = 8 * g + 4 * h + e;
          const float p0 = PT[(size_t)j * APITCH + l32];
          const float p1 = PT[(size_t)j * APITCH + 32 + l32];
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[e], p0, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[e], p1, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[e], p0, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[e], p1, acc[1][1], 0, 0, 0);
        }
      }
    }
    float* ob = out + (size_t)b * C * N;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = c0 + x * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        ob[(size_t)c * N + i0 + l32] = acc[x][0][r];
        ob[(size_t)c * N + i0 + 32 + l32] = acc[x][1][r];
      }
  }
}

hipError_t launch_attention(const float* qkv, int C, int N, float* o, float* /*scratch*/, int B,
                            hipStream_t s) {
  const size_t lds = ((size_t)N * APITCH + 4 * AQ) * sizeof(float);
  const float div = (float)std::sqrt((double)C);
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)attention_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  attention_kernel<<<dim3(N / AQ, B), 256, lds, s>>>(qkv, C, N, div, o);
  return hipGetLastError();
}

// ---- DDPM update (sample_model :111-118) on the U-Net's (B, P) state ----------------------
__global__ void unet_update_kernel(UpdateArgs a, int B) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)B * a.P;
  if (i >= n) return;
  const int t = *a.t_dev;
  const int b = (int)(i / a.P), o = (int)(i - (size_t)b * a.P);
  float z = 0.f;
  if (t > 0) {
    z = a.noise ? a.noise[((size_t)(a.num_steps - t) * B + b) * a.P + o]
                : philox_normal(a.seed, a.member_offset + (uint32_t)b, (uint32_t)t, 0u, o);
  }
  a.x[i] = ddpm_update(a.x[i], a.eps[i], a.c1[t], a.c2[t], a.sigma[t], z, t > 0);
}

hipError_t launch_unet_update(const UpdateArgs& a, int B, hipStream_t s) {
  const size_t n = (size_t)B * a.P;
  unet_update_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a, B);
  return hipGetLastError();
}

__global__ void set_word_kernel(int* w, int v) { *w = v; }
__global__ void dec_word_kernel(int* w) { *w = *w - 1; }

hipError_t launch_set_word(int* w, int v, hipStream_t s) {
  set_word_kernel<<<1, 1, 0, s>>>(w, v);
  return hipGetLastError();
}
hipError_t launch_dec_word(int* w, hipStream_t s) {
  dec_word_kernel<<<1, 1, 0, s>>>(w);
  return hipGetLastError();
}

}  // namespace unet
}  // namespace ertd
