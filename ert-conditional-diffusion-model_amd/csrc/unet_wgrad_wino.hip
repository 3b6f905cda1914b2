// Weight gradient of the fp32 3x3 stride-1 ResBlock convs by Winograd
// F(4x4,3x3) -- the transpose of the forward kernels' algorithm (same points
// {0, 1, -1, 1/2, -2, inf}, unet_conv_wino4.hip):
//
//   forward   y_tile = A^T [ (G g G^T) (.) (B^T d B) ] A
//   gradient  dg     = G^T [ sum_tiles (A dy_tile A^T) (.) (B^T d B) ] G
//
// (d = the 6x6 window of the ACTIVATED input, zero padding after the
// activation as in the spec; dy_tile the 4x4 output-gradient tile.)  The sum
// over tiles is 36 GEMMs dU[xi] = D[xi] V[xi]^T with M = Cout, N = Cin,
// K = B * tiles -- a quarter of the direct implicit GEMM's FLOP (36 per 16
// outputs instead of 144).  Four launches:
//   wgw_v_kernel   V[xi][ci][t] = B^T d B   (GroupNorm + SiLU on load)
//   wgw_d_kernel   D[xi][co][t] = A dy A^T
//   wgw_gemm_kernel  one wave per (xi, 64 co, 64 ci, K range): the operand
//                  fragments come straight from L2 as float4s (lane l = (row
//                  l & 15, k-quad l >> 4): four k-steps of v_mfma_f32_16x16x4_f32
//                  per load; K order permuted identically for both operands),
//                  4 x 4 accumulator blocks, loads two 16-k blocks ahead
//   wgw_sum_kernel / wgw_final_kernel  fixed-order sum of the K-range partials
//                  (one thread per (xi, co, ci)), then G^T dU G in float64 -> dW (= or +=)
// Bitwise reproducible (no atomics).  U2 B = 32 train step 13.95 -> 13.22 ms
// (same box); ERTD_WGRAD_WINO=0 keeps the implicit GEMM (A/B).  The Upsample
// convs (3x3 over the nearest-upsampled x) take the same path: only the V
// transform's loads change (ERTD_WGRAD_WINO=2 keeps them on the implicit GEMM).
#include <cstdlib>

#include "unet.h"

namespace ertd {
namespace unet {

namespace {

using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr int NX = 36;
#ifndef WGW_SETS
#define WGW_SETS 3
#endif

// o = B^T d (unet_conv_wino4.hip)
__device__ __forceinline__ void bt6(const float (&d)[6], float (&o)[6]) {
  const float c = d[4] - d[2], e = d[3] - d[1];
  const float u = d[4] - d[1], v = d[4] + d[1];
  o[0] = __builtin_fmaf(1.5f, e, __builtin_fmaf(-2.f, d[2], d[0] + d[4]));
  o[1] = __builtin_fmaf(2.5f, d[3], __builtin_fmaf(0.5f, d[2], u));
  o[2] = __builtin_fmaf(0.5f, d[3], __builtin_fmaf(-2.5f, d[2], v));
  o[3] = __builtin_fmaf(2.f, e, c);
  o[4] = __builtin_fmaf(-0.5f, e, c);
  o[5] = __builtin_fmaf(1.5f, c, __builtin_fmaf(-2.f, d[3], d[1] + d[5]));
}
// o = A v for a 4-vector v (A = the forward's A^T transposed, 6 x 4)
__device__ __forceinline__ void a4(const float (&v)[4], float (&o)[6]) {
  const float s = v[0] + v[2], d = v[1] + v[3];
  o[0] = v[0];
  o[1] = s + d;
  o[2] = s - d;
  o[3] = __builtin_fmaf(0.125f, v[3], __builtin_fmaf(0.25f, v[2], __builtin_fmaf(0.5f, v[1], v[0])));
  o[4] = __builtin_fmaf(-8.f, v[3], __builtin_fmaf(4.f, v[2], __builtin_fmaf(-2.f, v[1], v[0])));
  o[5] = v[3];
}

struct WgwArgs {
  const float* dy;      // (B, Cout, H, H)
  const float* xa;      // (B, Ca, H, H)
  const float* xb;      // (B, Cb, H, H) or null
  int Ca, Cb, Cout, H, B;
  const float2* gn;     // (B, Cin) {scale, shift} (ACT != NONE)
  float* V;             // [36][Cin][T]
  float* D;             // [36][Cout][T]
  float* P;             // [nks][36][Cout][Cin]
  int T, nks, kr;       // tiles (K), K ranges, K per range (multiple of 16)
  float* BP;            // [Cout][T / 256] bias-gradient partials (sums of dy), or null
};
// (H = the conv's output size; the Upsample convs read x at H / 2, nearest)

// one thread per (channel c, tile t), t fastest (coalesced stores per xi).
// UP: the conv reads the nearest-upsampled x -- window row iy, column ix is
// x[iy / 2][ix / 2] of the H / 2 plane (the 4 interior columns = 2 source
// pixels, each twice)
template <int ACT, bool UP>
__global__ __launch_bounds__(256) void wgw_v_kernel(WgwArgs a) {
  const int Cin = a.Ca + a.Cb;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)a.T * Cin) return;
  const int t = (int)(i % a.T);
  const int c = (int)(i / a.T);
  const int tpr = a.H / 4, ts = tpr * tpr;
  const int b = t / ts, tt = t - b * ts, ty = tt / tpr, tx = tt - ty * tpr;
  const int Hs = UP ? a.H / 2 : a.H;
  const float* src = c < a.Ca ? a.xa + ((size_t)b * a.Ca + c) * Hs * Hs
                              : a.xb + ((size_t)b * a.Cb + (c - a.Ca)) * Hs * Hs;
  float2 g = make_float2(1.f, 0.f);
  if constexpr (ACT != ACT_NONE) g = a.gn[(size_t)b * Cin + c];
  float d[6][6];
  const bool okl = tx > 0, okr = 4 * tx + 4 < a.H;
#pragma unroll
  for (int y = 0; y < 6; ++y) {
    const int iy = 4 * ty - 1 + y;
    const bool oky = iy >= 0 && iy < a.H;
    // the row's four interior columns as one float4 (UP: one float2), the two
    // halo columns alone
    float v[6];
    if constexpr (UP) {
      const float* row = src + (oky ? iy >> 1 : 0) * Hs + 2 * tx;
      const float2 m = *reinterpret_cast<const float2*>(row);
      v[0] = okl ? row[-1] : 0.f;
      v[1] = v[2] = m.x;
      v[3] = v[4] = m.y;
      v[5] = okr ? row[2] : 0.f;
    } else {
      const float* row = src + (oky ? iy : 0) * a.H + 4 * tx;
      const float4 m = *reinterpret_cast<const float4*>(row);
      v[0] = okl ? row[-1] : 0.f;
      v[1] = m.x;
      v[2] = m.y;
      v[3] = m.z;
      v[4] = m.w;
      v[5] = okr ? row[4] : 0.f;
    }
#pragma unroll
    for (int x = 0; x < 6; ++x) {
      const bool ok = oky && (x == 0 ? okl : (x == 5 ? okr : true));
      float u = v[x];
      if constexpr (ACT != ACT_NONE) {
        u = __builtin_fmaf(u, g.x, g.y);
        if constexpr (ACT == ACT_GN_SILU) u = u * __builtin_amdgcn_rcpf(1.0f + __expf(-u));
      }
      d[y][x] = ok ? u : 0.f;   // the padding pads the activated tensor
    }
  }
  // columns: B^T over the rows of each column, then rows
  float w[6][6];
#pragma unroll
  for (int x = 0; x < 6; ++x) {
    float col[6], o[6];
#pragma unroll
    for (int y = 0; y < 6; ++y) col[y] = d[y][x];
    bt6(col, o);
#pragma unroll
    for (int y = 0; y < 6; ++y) w[y][x] = o[y];
  }
  const size_t xs = (size_t)a.T * Cin;   // xi stride
  float* out = a.V + (size_t)c * a.T + t;
#pragma unroll
  for (int y = 0; y < 6; ++y) {
    float o[6];
    bt6(w[y], o);
#pragma unroll
    for (int x = 0; x < 6; ++x) out[(size_t)(6 * y + x) * xs] = o[x];
  }
}

__global__ __launch_bounds__(256) void wgw_d_kernel(WgwArgs a) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)a.T * a.Cout) return;
  const int t = (int)(i % a.T);
  const int co = (int)(i / a.T);
  const int tpr = a.H / 4, ts = tpr * tpr;
  const int b = t / ts, tt = t - b * ts, ty = tt / tpr, tx = tt - ty * tpr;
  const float* src = a.dy + ((size_t)b * a.Cout + co) * a.H * a.H + (4 * ty) * a.H + 4 * tx;
  float m[4][6];   // A applied along each row of the 4x4 tile
  float tsum = 0.f;  // the tile's sum of dy (the fused bias gradient)
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    const float4 q = *reinterpret_cast<const float4*>(src + y * a.H);
    const float v[4] = {q.x, q.y, q.z, q.w};
    a4(v, m[y]);
    tsum += (q.x + q.y) + (q.z + q.w);
  }
  const size_t xs = (size_t)a.T * a.Cout;
  float* out = a.D + (size_t)co * a.T + t;
#pragma unroll
  for (int x = 0; x < 6; ++x) {
    const float v[4] = {m[0][x], m[1][x], m[2][x], m[3][x]};
    float o[6];
    a4(v, o);
#pragma unroll
    for (int y = 0; y < 6; ++y) out[(size_t)(6 * y + x) * xs] = o[y];
  }
  if (a.BP) {
    // the conv's bias gradient rides along: the tile sums of the workgroup's
    // 256 tiles (T % 256 == 0: one output channel per workgroup, no early
    // return) in a fixed order
    float s = tsum;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) a.BP[(size_t)co * (a.T / 256) + t / 256] = (red[0] + red[1]) + (red[2] + red[3]);
  }
}

#ifndef WGW_LDS
#define WGW_LDS 1  // 1: LDS-staged workgroup tiles (wgw_gemm_lds_kernel); 0: wave tasks (A/B)
#endif

// one workgroup per (xi, co block 64 MB, ci block 64 NB, K range).  Per 16-k
// block the workgroup stages its D rows (64 MB) and V rows (64 NB) in LDS
// once -- each lane one float4 per 256 row-quads, rows padded to 20 floats so
// the fragment reads are conflict-free -- and wave (wm, wn) of the 2 x 2 wave
// grid multiplies rows [32 MB wm, +32 MB) by columns [32 NB wn, +32 NB): every
// operand byte crosses L2 -> CU once per workgroup instead of once per wave
// (wgw_gemm_kernel), and the four waves read it from LDS.  Same K permutation,
// fma order and K ranges as wgw_gemm_kernel: the partials are bitwise equal.
template <int MB, int NB>
__global__ __launch_bounds__(256) void wgw_gemm_lds_kernel(WgwArgs a) {
  constexpr int RA = 64 * MB, RB = 64 * NB, PITCH = 20;   // rows per operand, floats per LDS row
  constexpr int WI = 2 * MB, WJ = 2 * NB;                 // 16 x 16 blocks per wave
  __shared__ __attribute__((aligned(16))) float lds[2][(RA + RB) * PITCH];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int Cin = a.Ca + a.Cb;
  const int ncb = Cin / RB, nmb = a.Cout / RA;
  int r = blockIdx.x;
  const int nb = r % ncb; r /= ncb;
  const int mb = r % nmb; r /= nmb;
  const int xi = r % NX;
  const int ks = r / NX;
  const int c16 = lane & 15, g = lane >> 4;
  const int q0 = ks * (a.kr / 16), q1 = min(q0 + a.kr / 16, a.T / 16);
  // staging: thread tid moves row-quad f = tid + 256 u: row f >> 2, k-quad f & 3
  const f32x4* Dsrc = reinterpret_cast<const f32x4*>(a.D + ((size_t)xi * a.Cout + mb * RA) * a.T);
  const f32x4* Vsrc = reinterpret_cast<const f32x4*>(a.V + ((size_t)xi * Cin + nb * RB) * a.T);
  const size_t T4 = (size_t)a.T / 4;
  f32x4 stg[MB + NB];
  auto gload = [&](int Q) {
#pragma unroll
    for (int u = 0; u < MB + NB; ++u) {
      const int f = tid + 256 * u;
      const int row = u < MB ? f >> 2 : (f - 256 * MB) >> 2, kq = f & 3;
      stg[u] = (u < MB ? Dsrc : Vsrc)[(size_t)row * T4 + 4 * Q + kq];
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int u = 0; u < MB + NB; ++u) {
      const int f = tid + 256 * u;
      const int row = u < MB ? f >> 2 : RA + ((f - 256 * MB) >> 2), kq = f & 3;
      *reinterpret_cast<f32x4*>(&lds[buf][row * PITCH + 4 * kq]) = stg[u];
    }
  };
  f32x4 acc[WI][WJ];
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j) acc[i][j] = f32x4{};
  if (q0 < q1) {
    gload(q0);
    lstore(0);
    __syncthreads();
    for (int Q = q0; Q < q1; ++Q) {
      const int buf = (Q - q0) & 1;
      if (Q + 1 < q1) gload(Q + 1);
      f32x4 av[WI], bv[WJ];
#pragma unroll
      for (int i = 0; i < WI; ++i)
        av[i] = *reinterpret_cast<const f32x4*>(&lds[buf][(32 * MB * wm + 16 * i + c16) * PITCH + 4 * g]);
#pragma unroll
      for (int j = 0; j < WJ; ++j)
        bv[j] = *reinterpret_cast<const f32x4*>(&lds[buf][(RA + 32 * NB * wn + 16 * j + c16) * PITCH + 4 * g]);
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int i = 0; i < WI; ++i)
#pragma unroll
          for (int j = 0; j < WJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][k], bv[j][k], acc[i][j], 0, 0, 0);
      if (Q + 1 < q1) lstore(buf ^ 1);
      __syncthreads();
    }
  }
  // lane holds rows co = RA mb + 32 MB wm + 16 i + 4 g + e, column ci = RB nb + 32 NB wn + 16 j + c16
  float* P = a.P + (((size_t)ks * NX + xi) * a.Cout) * Cin;
  const int co0 = RA * mb + 32 * MB * wm, ci0 = RB * nb + 32 * NB * wn;
#pragma unroll
  for (int i = 0; i < WI; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        P[(size_t)(co0 + 16 * i + 4 * g + e) * Cin + ci0 + 16 * j + c16] = acc[i][j][e];
}

// one wave per task (xi, co block 64, ci block 64, K range); 4 waves per workgroup
__global__ __launch_bounds__(256) void wgw_gemm_kernel(WgwArgs a, int ntask) {
  const int lane = threadIdx.x & 63;
  const int task = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
  if (task >= ntask) return;
  const int Cin = a.Ca + a.Cb;
  const int ncb = Cin / 64, nmb = a.Cout / 64;
  int r = task;
  const int nb = r % ncb; r /= ncb;
  const int mb = r % nmb; r /= nmb;
  const int xi = r % NX;
  const int ks = r / NX;
  const int c16 = lane & 15, g = lane >> 4;
  // lane's float4 of 16-k block Q, row block i: [xi][row0 + 16 i + c16][16 Q + 4 g .. + 3]
  const f32x4* Db = reinterpret_cast<const f32x4*>(a.D + ((size_t)xi * a.Cout + mb * 64 + c16) * a.T) + g;
  const f32x4* Vb = reinterpret_cast<const f32x4*>(a.V + ((size_t)xi * Cin + nb * 64 + c16) * a.T) + g;
  const size_t rs = (size_t)16 * a.T / 4;        // 16 rows, in float4s
  const int q0 = ks * (a.kr / 16), q1 = min(q0 + a.kr / 16, a.T / 16);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};
  // WGW_SETS register sets: the loads run WGW_SETS - 1 16-k blocks ahead of
  // the MFMAs.  3 (176 VGPRs); 4 and 5 (192+ VGPRs, still two waves per SIMD)
  // measured 1.5 % / 2 % slower on the U2 B=32 train step (same box)
  constexpr int NS = WGW_SETS;
  f32x4 av[NS][4], bv[NS][4];
  auto load = [&](int Q, int s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) av[s][i] = Db[(size_t)4 * Q + i * rs];
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[s][j] = Vb[(size_t)4 * Q + j * rs];
  };
  auto step = [&](int s) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s][i][k], bv[s][j][k], acc[i][j], 0, 0, 0);
  };
  // blocks past q1 re-load the last block (unconditional loads keep the
  // compiler's vmcnt counting exact across the loop)
  auto qc = [&](int Q) { return Q < q1 ? Q : q1 - 1; };
  if (q0 < q1) {
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) load(qc(q0 + s), s);
  }
  // invariant at the loop head: set s holds block Q + s (s < NS - 1)
  int Q = q0;
  for (; Q + NS - 1 < q1; Q += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      load(qc(Q + s + NS - 1), (s + NS - 1) % NS);
      step(s);
    }
  }
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (Q + s < q1) step(s);
  // lane holds rows co = 64 mb + 16 i + 4 g + e, column ci = 64 nb + 16 j + c16
  float* P = a.P + (((size_t)ks * NX + xi) * a.Cout) * Cin;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        P[(size_t)(64 * mb + 16 * i + 4 * g + e) * Cin + 64 * nb + 16 * j + c16] = acc[i][j][e];
}

// G (6 x 3) of the points {0, 1, -1, 1/2, -2, inf}
__constant__ double kG[6][3] = {{1.0, 0.0, 0.0},
                                {1.0 / 3, 1.0 / 3, 1.0 / 3},
                                {-1.0 / 3, 1.0 / 3, -1.0 / 3},
                                {-16.0 / 15, -8.0 / 15, -4.0 / 15},
                                {1.0 / 15, -2.0 / 15, 4.0 / 15},
                                {0.0, 0.0, 1.0}};

// fixed-order sum of the K-range partials: one thread per (xi, co, ci), into
// partial slot 0
__global__ __launch_bounds__(256) void wgw_sum_kernel(WgwArgs a) {
  const size_t n = (size_t)NX * a.Cout * (a.Ca + a.Cb);
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float s = a.P[i];
  // batches of 8 independent loads, then the adds in k order (a serial
  // load-add chain was latency-bound: 11.0 us average per train-step launch;
  // batches of 8: 8.3 us; of 16: 11.7 us)
  for (int k = 1; k < a.nks; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = k + u < a.nks ? a.P[(size_t)(k + u) * n + i] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k + u < a.nks) s += v[u];
  }
  a.P[i] = s;
}

// dW[co][ci] = G^T dU G in float64 (one thread per (co, ci))
#ifndef WGW_FUSED_SUM
#define WGW_FUSED_SUM 4  // K ranges at most this many: summed by wgw_final_kernel (0: never)
#endif
__global__ __launch_bounds__(256) void wgw_final_kernel(WgwArgs a, float* dw, int accumulate, float* db,
                                                        float* db2, int nsum) {
  const int Cin = a.Ca + a.Cb;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t cc = (size_t)a.Cout * Cin;
  if (i >= cc) return;
  if (db && i % Cin == 0) {   // bias gradient of channel co: its T / 256 partials in order
    const size_t co = i / Cin;
    const int nb = a.T / 256;
    double s = 0.0;
    int k = 0;
    for (; k + 8 <= nb; k += 8) {   // 8 loads in flight, added in order
      float t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = a.BP[co * nb + k + j];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += (double)t[j];
    }
    for (; k < nb; ++k) s += (double)a.BP[co * nb + k];
    db[co] = (float)s;
    if (db2) db2[co] = (float)s;
  }
  // nsum > 1: the K-range partials are added here (the same k-ordered float
  // sum as wgw_sum_kernel, so the same bits) -- for small nks, saving a launch
  double u[NX];
  if (nsum > 1) {
    const size_t ks_stride = (size_t)NX * cc;
#pragma unroll
    for (int x = 0; x < NX; ++x) {
      float v[WGW_FUSED_SUM > 0 ? WGW_FUSED_SUM : 1];
#pragma unroll
      for (int k = 0; k < WGW_FUSED_SUM; ++k) v[k] = k < nsum ? a.P[(size_t)k * ks_stride + (size_t)x * cc + i] : 0.f;
      float s = v[0];
#pragma unroll
      for (int k = 1; k < WGW_FUSED_SUM; ++k)
        if (k < nsum) s += v[k];
      u[x] = (double)s;
    }
  } else {
#pragma unroll
    for (int x = 0; x < NX; ++x) u[x] = (double)a.P[(size_t)x * cc + i];
  }
  float* o = dw + i * 9;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      double v = 0.0;
#pragma unroll
      for (int p = 0; p < 6; ++p) {
        double rw = 0.0;
#pragma unroll
        for (int q = 0; q < 6; ++q) rw += u[6 * p + q] * kG[q][kx];
        v += kG[p][ky] * rw;
      }
      const float f = (float)v;
      o[3 * ky + kx] = accumulate ? o[3 * ky + kx] + f : f;
    }
}

int wgw_env() {
  static const int v = [] {
    return ERTD_KNOB("WGRAD_WINO", 1);
  }();
  return v;
}

struct WgwPlan {
  int T, nks, kr;
  int mb, nb;       // LDS path: workgroup tile (64 mb co) x (64 nb ci)
  size_t v, d, p;   // floats
  size_t bp;        // bias-gradient partials (0: T % 256 != 0, no fused bias gradient)
};

bool wgw_plan(int Cin, int Cout, int B, int H, WgwPlan* pl) {
  if (Cin % 64 || Cout % 64 || (H != 16 && H != 32 && H != 64) || B < 1) return false;
  const int T = B * (H / 4) * (H / 4);
  if (T % 16) return false;
  pl->mb = Cout % 128 == 0 ? 2 : 1;
  pl->nb = Cin % 128 == 0 ? 2 : 1;
  const int nq = T / 16;                         // 16-k blocks
#if WGW_LDS
  const int base = NX * (Cout / (64 * pl->mb)) * (Cin / (64 * pl->nb));
  // ERTD_WGW_TASKS: workgroup target (A/B; U2 B=32 train step, tools/gpu_knobs.sh:
  // 256 10.39, 320 10.21, 384 10.02-10.05, 448 10.05, 512 10.10-10.14 ms)
  static const int target = [] {
    const int v = ERTD_KNOB("WGW_TASKS", 384);
    return v > 0 ? v : 384;
  }();
#else
  const int base = NX * (Cout / 64) * (Cin / 64);
  static const int target = [] {                 // ERTD_WGW_TASKS: wave-task target (A/B)
    const int v = ERTD_KNOB("WGW_TASKS", 2048);
    return v > 0 ? v : 2048;
  }();
#endif
  int nks = (target + base - 1) / base;          // ~2 workgroups (8 waves) per CU
  if (nks > nq) nks = nq;
  if (nks < 1) nks = 1;
  const int qpr = (nq + nks - 1) / nks;
  nks = (nq + qpr - 1) / qpr;
  pl->T = T;
  pl->nks = nks;
  pl->kr = qpr * 16;
  pl->v = (size_t)NX * T * Cin;
  pl->d = (size_t)NX * T * Cout;
  pl->p = (size_t)nks * NX * Cout * Cin;
  pl->bp = T % 256 == 0 ? (size_t)Cout * (T / 256) : 0;
  return true;
}

}  // namespace

// H = the input size (the Upsample convs: Ho = 2 H)
size_t wgrad_wino_ws_floats(int Cin, int Cout, int B, int H, int ks, int mode) {
  WgwPlan pl;
  if (!wgw_env() || ks != 3 || (mode != MODE_S1 && mode != MODE_UP)) return 0;
  if (mode == MODE_UP && wgw_env() == 2) return 0;   // ERTD_WGRAD_WINO=2: stride-1 only (A/B)
  if (!wgw_plan(Cin, Cout, B, mode == MODE_UP ? 2 * H : H, &pl)) return 0;
  return pl.v + pl.d + pl.p + pl.bp;
}

bool wgrad_wino_bias_ok(int Cin, int Cout, int B, int H, int ks, int mode) {
  WgwPlan pl;
  return wgrad_wino_ws_floats(Cin, Cout, B, H, ks, mode) > 0 &&
         wgw_plan(Cin, Cout, B, mode == MODE_UP ? 2 * H : H, &pl) && pl.bp > 0;
}

hipError_t launch_wgrad_wino(const float* dy, const float* x, int Ca, const float* x2, int Cb, int B,
                             int H, int Cout, int mode, const float* gn, int act, float* dw,
                             int accumulate, float* ws, hipStream_t s, float* db, float* db2) {
  const bool up = mode == MODE_UP;
  if ((mode != MODE_S1 && !up) || (up && act != ACT_NONE)) return hipErrorInvalidValue;
  const int Ho = up ? 2 * H : H;
  WgwPlan pl;
  if (!wgw_plan(Ca + Cb, Cout, B, Ho, &pl)) return hipErrorInvalidValue;
  if ((db || db2) && (!db || !pl.bp)) return hipErrorInvalidValue;
  const int Cin = Ca + Cb;
  WgwArgs a{dy, x, x2, Ca, Cb, Cout, Ho, B, (const float2*)gn, ws, ws + pl.v, ws + pl.v + pl.d,
            pl.T, pl.nks, pl.kr, db ? ws + pl.v + pl.d + pl.p : nullptr};
  const size_t nv = (size_t)pl.T * Cin, nd = (size_t)pl.T * Cout;
  const unsigned gv = (unsigned)((nv + 255) / 256);
  if (up) wgw_v_kernel<ACT_NONE, true><<<gv, 256, 0, s>>>(a);
  else if (act == ACT_GN_SILU) wgw_v_kernel<ACT_GN_SILU, false><<<gv, 256, 0, s>>>(a);
  else if (act == ACT_GN) wgw_v_kernel<ACT_GN, false><<<gv, 256, 0, s>>>(a);
  else wgw_v_kernel<ACT_NONE, false><<<gv, 256, 0, s>>>(a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  wgw_d_kernel<<<(unsigned)((nd + 255) / 256), 256, 0, s>>>(a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
#if WGW_LDS
  const unsigned nwg = (unsigned)(pl.nks * NX * (Cout / (64 * pl.mb)) * (Cin / (64 * pl.nb)));
  if (pl.mb == 2 && pl.nb == 2) wgw_gemm_lds_kernel<2, 2><<<nwg, 256, 0, s>>>(a);
  else if (pl.mb == 2) wgw_gemm_lds_kernel<2, 1><<<nwg, 256, 0, s>>>(a);
  else if (pl.nb == 2) wgw_gemm_lds_kernel<1, 2><<<nwg, 256, 0, s>>>(a);
  else wgw_gemm_lds_kernel<1, 1><<<nwg, 256, 0, s>>>(a);
#else
  const int ntask = pl.nks * NX * (Cout / 64) * (Cin / 64);
  wgw_gemm_kernel<<<(unsigned)((ntask + 3) / 4), 256, 0, s>>>(a, ntask);
#endif
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const size_t nw = (size_t)Cout * Cin;
  const bool fuse = pl.nks > 1 && pl.nks <= WGW_FUSED_SUM;
  if (pl.nks > 1 && !fuse) {
    wgw_sum_kernel<<<(unsigned)((nw * NX + 255) / 256), 256, 0, s>>>(a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  wgw_final_kernel<<<(unsigned)((nw + 255) / 256), 256, 0, s>>>(a, dw, accumulate, db, db2,
                                                                  fuse ? pl.nks : 1);
  return hipGetLastError();
}

}  // namespace unet
}  // namespace ertd
