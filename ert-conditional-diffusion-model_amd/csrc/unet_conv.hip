// 2-D convolution of the build-defined U-Net as an implicit GEMM on fp32 MFMA
// (v_mfma_f32_32x32x2_f32: exact fp32 products, k-ordered fma chains).
//
//   out[b][co][p] = bias[co] (+ ebias[b][co]) (+ res[b][co][p])
//                 + sum_{ci, ky, kx} W[co][ci][ky][kx] * act(in[b][ci][.])
//
// GEMM view per sample: rows = output channels (A = packed weights), columns =
// output pixels (B = im2col of the staged input), K = Cin * ks * ks.
// Workgroup = 4 waves, each a 64 (cout) x 64 (pixel) tile = 2 x 2 MFMA tiles;
// WCO waves along cout, 4/WCO along pixels, so a workgroup covers BN = 64*WCO
// output channels x BM = 64*(4/WCO) consecutive output pixels of one sample.
//
// K is walked in chunks of CK = 8 input channels.  Per chunk the input rows the
// tile needs (with the 3x3 halo) are staged in LDS as an image [c][row][col]
// with a zero column on each side, AFTER the input transform (GroupNorm
// apply + SiLU for a ResBlock's convs, nothing for Downsample/Upsample/skip):
// zero padding therefore pads the activated tensor, as in the oracle.  The
// stage of chunk k+1 is loaded into registers while chunk k's MFMAs run
// (double-buffered LDS, one barrier per chunk).
//
// K order inside a chunk: lane half h takes channels 4h..4h+3, k-step s takes
// channel s/9 of that half and tap s%9, so a lane's LDS operand address is a
// per-lane base plus a per-step constant.  The host packs W in exactly this
// order ([co_tile32][chunk][group of 4 steps][lane][4]) so each lane streams
// its A operands as one coalesced float4 per 4 k-steps.
//
// Skip concatenations (the up path) are read from two source tensors in place
// (channels [0,Ca) from srcA, [Ca,Ca+Cb) from srcB); the nearest x2 Upsample is
// folded into the staging address (source row/col = staged row/col >> 1).
#include "unet.h"

namespace ertd {
namespace unet {

template <int MODE, int KS>
__device__ __forceinline__ int first_row(int oy0) {
  if constexpr (KS == 1) return oy0;
  else if constexpr (MODE == MODE_S2) return 2 * oy0 - 1;
  else return oy0 - 1;
}

template <int KS, int MODE, int ACT, int WCO>
__global__ __launch_bounds__(NTHR) void conv_kernel(ConvArgs a) {
  constexpr int WPX = 4 / WCO;
  constexpr int BM = 64 * WPX;           // output pixels per workgroup
  constexpr int BN = 64 * WCO;           // output channels per workgroup
  constexpr int NG = conv_groups(KS);    // weight groups (4 k-steps) per chunk
  constexpr int NIT = MODE == MODE_S2 ? 36 : 20;  // max staged rows per thread
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int wco = wave % WCO, wpx = wave / WCO;
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * BM;
  const int Wo = a.Wo;
  const int oy0 = p0 / Wo;
  const int IR = a.IR, IP = a.IP, ICH = IR * IP;
  const int CHB = CK * ICH;              // floats per LDS buffer
  const int Wst = MODE == MODE_UP ? 2 * a.Ws : a.Ws;   // staged image width
  const int Hst = MODE == MODE_UP ? 2 * a.Hs : a.Hs;
  const int Cin = a.Cin, Ca = a.Ca;

  // ---- zero the halo columns of both buffers (never written by staging)
  for (int r = tid; r < 2 * CK * IR; r += NTHR) {
    smem[r * IP] = 0.f;
    smem[r * IP + IP - 1] = 0.f;
  }

  // ---- staging geometry: thread -> (column, first row slot)
  const int col = tid % Wst;             // Wst is a power of two <= 256
  const int rstep = NTHR / Wst;
  const int rs0 = tid / Wst;
  const int nrows = CK * IR;
  const int row0 = first_row<MODE, KS>(oy0);
  const int sx = MODE == MODE_UP ? (col >> 1) : col;

  float stg[NIT];
  auto load_chunk = [&](int k) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int fr = rs0 + it * rstep;
      float v = 0.f;
      if (fr < nrows) {
        const int c = (int)(((unsigned)fr * (unsigned)a.ir_magic) >> 19), r = fr - c * IR;
        const int cg = k * CK + c;
        const int iy = row0 + r;
        if (cg < Cin && iy >= 0 && iy < Hst) {
          const int sy = MODE == MODE_UP ? (iy >> 1) : iy;
          const float* src = cg < Ca ? a.srcA + ((size_t)b * Ca + cg) * a.Hs * a.Ws
                                     : a.srcB + ((size_t)b * a.Cb + (cg - Ca)) * a.Hs * a.Ws;
          v = src[sy * a.Ws + sx];
        }
      }
      stg[it] = v;
    }
  };
  auto store_chunk = [&](int k, float* buf) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int fr = rs0 + it * rstep;
      if (fr < nrows) {
        const int c = (int)(((unsigned)fr * (unsigned)a.ir_magic) >> 19), r = fr - c * IR;
        const int cg = k * CK + c;
        const int iy = row0 + r;
        float v = stg[it];
        if constexpr (ACT != ACT_NONE) {
          if (cg < Cin && iy >= 0 && iy < Hst) {
            const float2 g = a.gn[(size_t)b * Cin + cg];
            v = v * g.x + g.y;  // ATen's folded GroupNorm: x*scale + shift
            if constexpr (ACT == ACT_GN_SILU) v = v / (1.0f + expf(-v));
          }
        }
        buf[fr * IP + col + 1] = v;
      }
    }
  };

  // ---- per-lane LDS operand bases (pixel tiles t = 0, 1 of this wave)
  int lbase[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int pl = wpx * 64 + t * 32 + l32;   // pixel within the workgroup tile
    const int oyl = pl / Wo, ox = pl - oyl * Wo;
    int rb, cb;
    if constexpr (KS == 1) { rb = oyl; cb = ox + 1; }
    else if constexpr (MODE == MODE_S2) { rb = 2 * oyl; cb = 2 * ox; }
    else { rb = oyl; cb = ox; }
    lbase[t] = h * 4 * ICH + rb * IP + cb;
  }

  // ---- weight stream of this wave's two 32-cout tiles
  const int nchunk = a.nchunk;
  const int tile0 = blockIdx.y * (BN / 32) + wco * 2;
  const float4* wp0 = reinterpret_cast<const float4*>(a.wpk) + (size_t)tile0 * nchunk * NG * 64 + lane;
  const float4* wp1 = wp0 + (size_t)nchunk * NG * 64;
  const int gtotal = nchunk * NG;
  int gnext = 0;
  float4 wn0 = wp0[0], wn1 = wp1[0];

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  load_chunk(0);
  store_chunk(0, smem);
  __syncthreads();

  for (int k = 0; k < nchunk; ++k) {
    const float* buf = smem + (k & 1) * CHB;
    if (k + 1 < nchunk) load_chunk(k + 1);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const float4 w0 = wn0, w1 = wn1;
      gnext = gnext + 1 < gtotal ? gnext + 1 : gnext;
      wn0 = wp0[(size_t)gnext * 64];
      wn1 = wp1[(size_t)gnext * 64];
      const float wa0[4] = {w0.x, w0.y, w0.z, w0.w};
      const float wa1[4] = {w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int s = g * 4 + s4;
        int off;
        if constexpr (KS == 1) off = s * ICH;
        else off = (s / 9) * ICH + ((s % 9) / 3) * IP + (s % 3);
        const float b0 = buf[lbase[0] + off];
        const float b1 = buf[lbase[1] + off];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa0[s4], b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa0[s4], b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa1[s4], b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa1[s4], b1, acc[1][1], 0, 0, 0);
      }
    }
    if (k + 1 < nchunk) store_chunk(k + 1, smem + ((k + 1) & 1) * CHB);
    __syncthreads();
  }

  // ---- epilogue: bias (+ per-sample channel add) (+ residual), NCHW store
  const size_t HWo = (size_t)a.Ho * Wo;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = (tile0 + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (co >= a.Cout) continue;
      const float bias = a.bias[co];
      const float eb = a.ebias ? a.ebias[(size_t)b * a.eb_stride + co] : 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const size_t p = (size_t)p0 + wpx * 64 + j * 32 + l32;
        const size_t o = ((size_t)b * a.Cout + co) * HWo + p;
        // the oracle's op order: conv(+bias), then + emb, then + residual
        float v = acc[i][j][r] + bias;
        if (a.ebias) v = v + eb;
        if (a.res) v = v + a.res[o];
        a.out[o] = v;
      }
    }
  }
}

template <int KS, int MODE, int ACT>
static hipError_t launch_t(const ConvArgs& a, int B, hipStream_t s) {
  const int wco = (a.Cout >= 128) ? 2 : 1;
  const int bm = 64 * (4 / wco), bn = 64 * wco;
  const size_t lds = (size_t)2 * CK * a.IR * a.IP * sizeof(float);
  dim3 grid((unsigned)((size_t)a.Ho * a.Wo / bm), (unsigned)((a.Cout + bn - 1) / bn), (unsigned)B);
  if (wco == 2) {
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)conv_kernel<KS, MODE, ACT, 2>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    conv_kernel<KS, MODE, ACT, 2><<<grid, NTHR, lds, s>>>(a);
  } else {
    if (lds > 65536)
      (void)hipFuncSetAttribute((const void*)conv_kernel<KS, MODE, ACT, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    conv_kernel<KS, MODE, ACT, 1><<<grid, NTHR, lds, s>>>(a);
  }
  return hipGetLastError();
}

hipError_t launch_conv(int ks, int mode, int act, const ConvArgs& a, int B, hipStream_t s) {
  if (ks == 3 && mode == MODE_S1 && act == ACT_NONE) return launch_t<3, MODE_S1, ACT_NONE>(a, B, s);
  if (ks == 3 && mode == MODE_S1 && act == ACT_GN_SILU) return launch_t<3, MODE_S1, ACT_GN_SILU>(a, B, s);
  if (ks == 3 && mode == MODE_S2 && act == ACT_NONE) return launch_t<3, MODE_S2, ACT_NONE>(a, B, s);
  if (ks == 3 && mode == MODE_UP && act == ACT_NONE) return launch_t<3, MODE_UP, ACT_NONE>(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_NONE) return launch_t<1, MODE_S1, ACT_NONE>(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_GN) return launch_t<1, MODE_S1, ACT_GN>(a, B, s);
  return hipErrorInvalidValue;
}

// ---- weight packing: W (Cout, Cin, ks, ks) -> [co_tile32][chunk][group][lane][4]
// Cout is padded to a multiple of 128 (so a 2-tile wave never reads past the
// end), Cin to a multiple of CK; padding is zero.
size_t conv_packed_floats(int cin, int cout, int ks) {
  const size_t tiles = (size_t)((cout + 127) / 128) * 4;
  const size_t nchunk = (size_t)((cin + CK - 1) / CK);
  return tiles * nchunk * conv_groups(ks) * 64 * 4;
}

__global__ void pack_conv_kernel(const float* __restrict__ w, int cin, int cout, int ks,
                                 int nchunk, size_t total, float* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int NG = conv_groups(ks);
  const int e = (int)(i & 3);
  const int lane = (int)((i >> 2) & 63);
  size_t rest = i >> 8;
  const int g = (int)(rest % NG);
  rest /= NG;
  const int k = (int)(rest % nchunk);
  const int tile = (int)(rest / nchunk);
  const int s = g * 4 + e;
  const int hh = lane >> 5;
  const int co = tile * 32 + (lane & 31);
  int ci, ky, kx;
  if (ks == 3) { ci = k * CK + hh * 4 + s / 9; ky = (s % 9) / 3; kx = s % 3; }
  else { ci = k * CK + hh * 4 + s; ky = 0; kx = 0; }
  float v = 0.f;
  if (co < cout && ci < cin) v = w[(((size_t)co * cin + ci) * ks + ky) * ks + kx];
  dst[i] = v;
}

hipError_t launch_pack_conv(const float* w, int cin, int cout, int ks, float* dst, hipStream_t s) {
  const size_t total = conv_packed_floats(cin, cout, ks);
  const int nchunk = (cin + CK - 1) / CK;
  pack_conv_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(w, cin, cout, ks, nchunk, total, dst);
  return hipGetLastError();
}

}  // namespace unet
}  // namespace ertd
