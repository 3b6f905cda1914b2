// bf16-operand variant of the U-Net convolution (BASELINE configs[2]/[4] are
// bf16): the same implicit GEMM as unet_conv.hip on v_mfma_f32_32x32x16_bf16
// (16x the fp32 MFMA rate), bf16 operands, fp32 accumulation; activations,
// GroupNorm statistics, bias/embedding/residual adds and outputs stay fp32 in
// HBM.  The input transform (GroupNorm apply + SiLU) runs in fp32 while the
// tile is staged, then rounds to bf16 (round-to-nearest-even).
//
// K order: a k-step is 16 channels at one tap; lane half h holds channels
// 8h..8h+7 (the MFMA's k = 8h + j).  So the staged input image is
// channel-innermost, [group of 16 ch][row][col][16 bf16] (32 B per pixel),
// and a lane's B operand is ONE ds_read_b128; the weights are packed as
// [co_tile32][chunk][step][lane][8 bf16] and arrive by LDS-DMA, A operand =
// one ds_read_b128.  Chunks: 16 channels x 9 taps for 3x3, 32 channels for 1x1.
// Workgroup = 4 waves along pixels, each 64 co x 32*TPX px.
#include <cstdlib>

#include "unet.h"

namespace ertd {
namespace unet {

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;

__device__ __forceinline__ unsigned bf16_bits(float v) {  // round to nearest even (finite v)
  const uint32_t u = __float_as_uint(v);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ unsigned lds_addr_h(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

__host__ __device__ constexpr int convh_ck(int ks) { return ks == 3 ? 16 : 32; }

template <int KS, int MODE, int WO, int TPX>
struct GeomH {
  static constexpr int BM = 128 * TPX;               // output pixels per workgroup
  static constexpr int BN = 64;                      // output channels per workgroup
  static constexpr int WST = MODE == MODE_S2 ? 2 * WO : WO;
  static constexpr int R = BM / WO;
  static constexpr int IR = KS == 1 ? R : (MODE == MODE_S2 ? 2 * R + 1 : R + 2);
  static constexpr int IP = WST + 2;                  // staged pixels per row
  static constexpr int CKB = convh_ck(KS);            // channels per chunk
  static constexpr int NG = CKB / 16;                 // 16-channel groups per chunk
  static constexpr int TAPS = KS * KS;
  static constexpr int SPC = TAPS * NG;               // k-steps per chunk
  static constexpr int GB = IR * IP * 32;             // bytes per 16-channel group image
  static constexpr int XB = NG * GB;                  // input image bytes per buffer
  static constexpr int TWB = SPC * 64 * 16;           // weight bytes per 32-co tile and chunk
  static constexpr int WBB = 2 * TWB;                 // 2 tiles per workgroup
  static constexpr int RSTEP = NTHR / WST;
  static constexpr int NR = 2 * NG * IR;              // (half-group, row) rows of 8-channel pixels
  static constexpr int NIT = (NR + RSTEP - 1) / RSTEP;
  static constexpr int NGL = WBB / 1024;              // 16-B-per-lane DMA instructions per chunk
  static constexpr size_t LDS = 2 * (size_t)XB + 2 * (size_t)WBB;
  static_assert(BM % WO == 0, "tile must hold whole output rows");
  static_assert(WST <= NTHR, "staged row wider than the workgroup");
  static_assert(XB % 16 == 0 && TWB % 1024 == 0, "alignment");
};

template <int KS, int MODE, int ACT, int WO, int TPX>
__global__ __launch_bounds__(NTHR) void conv_bf16_kernel(ConvArgs a) {
  using G = GeomH<KS, MODE, WO, TPX>;
  extern __shared__ __attribute__((aligned(16))) char smemh[];
  char* wim = smemh;                          // [2][WBB]
  char* xim = smemh + 2 * G::WBB;             // [2][XB]
  float2* gtab = reinterpret_cast<float2*>(smemh + 2 * G::WBB + 2 * G::XB);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * G::BM;
  const int oy0 = p0 / WO;
  const int Cin = a.Cin, Ca = a.Ca;
  constexpr int HS = MODE == MODE_UP ? WO / 2 : G::WST;
  constexpr int HST = MODE == MODE_UP ? WO : G::WST;
  constexpr int CK = G::CKB;
  const int nchunk = (Cin + CK - 1) / CK;

  if constexpr (ACT != ACT_NONE) {
    for (int c = tid; c < Cin; c += NTHR) gtab[c] = a.gn[(size_t)b * Cin + c];
  }
  // zero halo pixels (cols 0 and IP-1) of every row, group, buffer
  for (int r = tid; r < 2 * G::NG * G::IR * 2; r += NTHR) {
    const int side = r & 1, rest = r >> 1;
    const int buf = rest / (G::NG * G::IR), rem = rest - buf * (G::NG * G::IR);
    const int g = rem / G::IR, rr = rem - g * G::IR;
    u32x4* px = reinterpret_cast<u32x4*>(xim + buf * G::XB + g * G::GB +
                                         (rr * G::IP + (side ? G::IP - 1 : 0)) * 32);
    px[0] = u32x4{0u, 0u, 0u, 0u};
    px[1] = u32x4{0u, 0u, 0u, 0u};
  }

  const int col = tid % G::WST;
  const int rs0 = tid / G::WST;
  int row0;
  if constexpr (KS == 1) row0 = oy0;
  else if constexpr (MODE == MODE_S2) row0 = 2 * oy0 - 1;
  else row0 = oy0 - 1;
  const int sx = MODE == MODE_UP ? (col >> 1) : col;
  constexpr size_t plane = (size_t)HS * HS;

  float stg[G::NIT][8];
  auto load_chunk = [&](int k) {
#pragma unroll
    for (int it = 0; it < G::NIT; ++it) {
      const int fr = rs0 + it * G::RSTEP;
      const int hg = fr / G::IR, r = fr - hg * G::IR;
      const int iy = row0 + r;
      const bool rowok = fr < G::NR && iy >= 0 && iy < HST;
      const int sy = rowok ? (MODE == MODE_UP ? (iy >> 1) : iy) : 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cg = k * CK + hg * 8 + j;
        const int cgc = (rowok && cg < Cin) ? cg : 0;
        const float* src = cgc < Ca ? a.srcA + ((size_t)b * Ca + cgc) * plane
                                    : a.srcB + ((size_t)b * a.Cb + (cgc - Ca)) * plane;
        stg[it][j] = src[sy * HS + sx];
      }
    }
  };
  auto store_elem = [&](int it, int k, char* img) {
    const int fr = rs0 + it * G::RSTEP;
    if (fr < G::NR) {
      const int hg = fr / G::IR, r = fr - hg * G::IR;
      const int iy = row0 + r;
      const bool rowok = iy >= 0 && iy < HST;
      unsigned w[4];
#pragma unroll
      for (int j2 = 0; j2 < 4; ++j2) {
        unsigned bits[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int j = 2 * j2 + e;
          const int cg = k * CK + hg * 8 + j;
          const bool ok = rowok && cg < Cin;
          float v = stg[it][j];
          if constexpr (ACT != ACT_NONE) {
            const float2 g = gtab[ok ? cg : 0];
            v = fmaf(v, g.x, g.y);
            if constexpr (ACT == ACT_GN_SILU) v = v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
          }
          bits[e] = ok ? bf16_bits(v) : 0u;
        }
        w[j2] = bits[0] | (bits[1] << 16);
      }
      *reinterpret_cast<u32x4*>(img + (hg >> 1) * G::GB + (r * G::IP + col + 1) * 32 +
                                (hg & 1) * 16) = u32x4{w[0], w[1], w[2], w[3]};
    }
  };

  const int tile_wg = blockIdx.y * 2;
  auto dma_weights = [&](int k, char* wdst) {
#pragma unroll
    for (int j = 0; j < (G::NGL + 3) / 4; ++j) {
      const int ins = wave + 4 * j;
      if (ins < G::NGL) {
        const int byte = ins * 1024 + lane * 16;
        const int ti = byte / G::TWB, wi = byte - ti * G::TWB;
        const char* src = reinterpret_cast<const char*>(a.wpk) +
                          ((size_t)(tile_wg + ti) * nchunk + k) * G::TWB + wi;
        const unsigned dst = __builtin_amdgcn_readfirstlane(lds_addr_h(wdst + ins * 1024));
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(dst)
            : "memory");
      }
    }
  };
  auto dma_wait = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  int lbase[TPX];
#pragma unroll
  for (int t = 0; t < TPX; ++t) {
    const int pl = wave * 32 * TPX + t * 32 + l32;
    const int oyl = pl / WO, ox = pl - oyl * WO;
    int rb, cb;
    if constexpr (KS == 1) { rb = oyl; cb = ox + 1; }
    else if constexpr (MODE == MODE_S2) { rb = 2 * oyl; cb = 2 * ox; }
    else { rb = oyl; cb = ox; }
    lbase[t] = (rb * G::IP + cb) * 32 + h * 16;
  }
  const int abase = lane * 16;

  f32x16 acc[2][TPX];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < TPX; ++t) acc[i][t] = f32x16{};

  dma_weights(0, wim);
  if constexpr (ACT != ACT_NONE) __syncthreads();
  load_chunk(0);
#pragma unroll
  for (int it = 0; it < G::NIT; ++it) store_elem(it, 0, xim);
  if (nchunk > 1) load_chunk(1);
  dma_wait();
  __syncthreads();

  // rows two chunks ahead, stored at the top of the chunk (unet_conv.hip STG 1)
  for (int k = 0; k < nchunk; ++k) {
    const int cur = k & 1;
    const char* xb = xim + cur * G::XB;
    const char* wb = wim + cur * G::WBB;
    if (k + 1 < nchunk) {
#pragma unroll
      for (int it = 0; it < G::NIT; ++it) store_elem(it, k + 1, xim + (cur ^ 1) * G::XB);
      if (k + 2 < nchunk) load_chunk(k + 2);
      dma_weights(k + 1, wim + (cur ^ 1) * G::WBB);
    }
#pragma unroll
    for (int s = 0; s < G::SPC; ++s) {
      const int g = s / G::TAPS, tap = s % G::TAPS;
      int off;
      if constexpr (KS == 1) off = g * G::GB;
      else off = g * G::GB + ((tap / 3) * G::IP + (tap % 3)) * 32;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(wb + s * 1024 + abase);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(wb + G::TWB + s * 1024 + abase);
#pragma unroll
      for (int t = 0; t < TPX; ++t) {
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(xb + lbase[t] + off);
        acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bv, acc[0][t], 0, 0, 0);
        acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bv, acc[1][t], 0, 0, 0);
      }
    }
    dma_wait();
    __syncthreads();
  }

  // ---- epilogue (as unet_conv.hip): 8-row phases, loads before stores
  constexpr int HWo = WO * WO;
  const size_t lbase0 = (size_t)b * a.Cout * HWo + p0 + wave * 32 * TPX + l32;
  const float* __restrict__ resp = a.res ? a.res + lbase0 : nullptr;
  float* __restrict__ outp = a.out + lbase0;
  const float* ebp = a.ebias ? a.ebias + (size_t)b * a.eb_stride : nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
      float bias[8], eb[8], rv[8][TPX];
      int off[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = ph * 8 + q;
        int co = (tile_wg + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        co = co < a.Cout ? co : a.Cout - 1;
        off[q] = co * HWo;
        bias[q] = a.bias[co];
        eb[q] = ebp ? ebp[co] : 0.f;
#pragma unroll
        for (int t = 0; t < TPX; ++t) rv[q][t] = resp ? resp[off[q] + t * 32] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = ph * 8 + q;
        const int co = (tile_wg + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co >= a.Cout) continue;
#pragma unroll
        for (int t = 0; t < TPX; ++t) {
          float v = acc[i][t][r] + bias[q];
          if (ebp) v = v + eb[q];
          if (resp) v = v + rv[q][t];
          outp[off[q] + t * 32] = v;
        }
      }
    }
  }
}

template <int KS, int MODE, int ACT, int WO, int TPX>
static hipError_t launch_hg(const ConvArgs& a, int B, hipStream_t s) {
  using G = GeomH<KS, MODE, WO, TPX>;
  const size_t lds = G::LDS + (ACT != ACT_NONE ? (size_t)a.Cin * sizeof(float2) : 0);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)conv_bf16_kernel<KS, MODE, ACT, WO, TPX>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((unsigned)(WO * WO / G::BM), (unsigned)((a.Cout + G::BN - 1) / G::BN), (unsigned)B);
  conv_bf16_kernel<KS, MODE, ACT, WO, TPX><<<grid, NTHR, lds, s>>>(a);
  return hipGetLastError();
}

// ERTD_UNET_BF16_TPX=1 forces 128-pixel tiles for the 3x3 stride-1/upsample
// convs (diagnostics); 0 = automatic
static int convh_tpx_override() {
  static int v = [] {
    const char* e = getenv("ERTD_UNET_BF16_TPX");
    return e ? atoi(e) : 0;
  }();
  return v;
}

template <int KS, int MODE, int ACT, int TP>
static hipError_t launch_hwt(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 16: return launch_hg<KS, MODE, ACT, 16, TP>(a, B, s);
    case 32: return launch_hg<KS, MODE, ACT, 32, TP>(a, B, s);
    case 64: return launch_hg<KS, MODE, ACT, 64, TP>(a, B, s);
    case 128:
      if constexpr (MODE != MODE_S2) return launch_hg<KS, MODE, ACT, 128, TP>(a, B, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

template <int KS, int MODE, int ACT>
static hipError_t launch_hw(const ConvArgs& a, int B, hipStream_t s) {
  // TPX = 2 (256-pixel tiles) except stride 2 / 1x1 (staging registers)
  if constexpr (MODE == MODE_S2 || KS == 1) {
    return launch_hwt<KS, MODE, ACT, 1>(a, B, s);
  } else {
    if (convh_tpx_override() == 1) return launch_hwt<KS, MODE, ACT, 1>(a, B, s);
    return launch_hwt<KS, MODE, ACT, 2>(a, B, s);
  }
}

hipError_t launch_conv_bf16(int ks, int mode, int act, const ConvArgs& a, int B, hipStream_t s) {
  if (a.Ho != a.Wo || a.Hs != a.Ws || a.Cin != a.Ca + a.Cb) return hipErrorInvalidValue;
  const int expect = mode == MODE_S2 ? a.Ws / 2 : (mode == MODE_UP ? a.Ws * 2 : a.Ws);
  if (a.Wo != expect) return hipErrorInvalidValue;
  if (a.Cout == 1 && ks == 3 && mode == MODE_S1 && act != ACT_GN)
    return launch_conv_out(act, a, B, true, s);
  if (ks == 3 && mode == MODE_S1 && act == ACT_NONE) return launch_hw<3, MODE_S1, ACT_NONE>(a, B, s);
  if (ks == 3 && mode == MODE_S1 && act == ACT_GN_SILU) return launch_hw<3, MODE_S1, ACT_GN_SILU>(a, B, s);
  if (ks == 3 && mode == MODE_S2 && act == ACT_NONE) return launch_hw<3, MODE_S2, ACT_NONE>(a, B, s);
  if (ks == 3 && mode == MODE_UP && act == ACT_NONE) return launch_hw<3, MODE_UP, ACT_NONE>(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_NONE) return launch_hw<1, MODE_S1, ACT_NONE>(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_GN) return launch_hw<1, MODE_S1, ACT_GN>(a, B, s);
  return hipErrorInvalidValue;
}

// ---- bf16 weight packing: W (Cout, Cin, ks, ks) fp32 -> [co_tile32][chunk][step][lane][8] bf16
size_t conv_packed_floats_bf16(int cin, int cout, int ks) {
  const int ck = convh_ck(ks);
  const size_t tiles = (size_t)((cout + 127) / 128) * 4;
  const size_t nchunk = (size_t)((cin + ck - 1) / ck);
  const size_t steps = (size_t)ks * ks * (ck / 16);
  return tiles * nchunk * steps * 64 * 8 / 2;   // 8 bf16 per lane = 4 floats
}

__global__ void pack_conv_bf16_kernel(const float* __restrict__ w, int cin, int cout, int ks,
                                      int nchunk, size_t total, unsigned short* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // bf16 element
  if (i >= total) return;
  const int ck = convh_ck(ks), taps = ks * ks, spc = taps * (ck / 16);
  const int j = (int)(i & 7);
  const int lane = (int)((i >> 3) & 63);
  size_t rest = i >> 9;
  const int s = (int)(rest % spc);
  rest /= spc;
  const int k = (int)(rest % nchunk);
  const int tile = (int)(rest / nchunk);
  const int g = s / taps, tap = s % taps;
  const int co = tile * 32 + (lane & 31);
  const int ci = k * ck + g * 16 + 8 * (lane >> 5) + j;
  float v = 0.f;
  if (co < cout && ci < cin) v = w[((size_t)co * cin + ci) * taps + tap];
  const uint32_t u = __float_as_uint(v);
  dst[i] = (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

hipError_t launch_pack_conv_bf16(const float* w, int cin, int cout, int ks, float* dst,
                                 hipStream_t s) {
  const size_t total = conv_packed_floats_bf16(cin, cout, ks) * 2;
  const int nchunk = (cin + convh_ck(ks) - 1) / convh_ck(ks);
  pack_conv_bf16_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(
      w, cin, cout, ks, nchunk, total, reinterpret_cast<unsigned short*>(dst));
  return hipGetLastError();
}

}  // namespace unet
}  // namespace ertd
