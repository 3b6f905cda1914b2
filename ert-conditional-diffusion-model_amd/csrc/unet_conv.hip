// 2-D convolution of the build-defined U-Net as an implicit GEMM on fp32 MFMA
// (v_mfma_f32_32x32x2_f32: exact fp32 products, k-ordered fma chains).
//
//   out[b][co][p] = bias[co] (+ ebias[b][co]) (+ res[b][co][p])
//                 + sum_{ci, ky, kx} W[co][ci][ky][kx] * act(in[b][ci][.])
//
// GEMM view per sample: rows = output channels (A = packed weights), columns =
// output pixels (B = im2col of the staged input), K = Cin * ks * ks.
// Workgroup = 4 waves, each a 64 (cout) x 64 (pixel) tile = 2 x 2 MFMA tiles;
// WCO waves along cout, 4/WCO along pixels: a workgroup covers BN = 64*WCO
// output channels x BM = 64*(4/WCO) consecutive output pixels of one sample.
// The output width WO is a template parameter, so every LDS offset of the
// inner loop is an immediate.
//
// K is walked in chunks of 4 input channels (3x3; 32 for 1x1).  Per chunk:
//   * the weight slice (BN couts x 4 channels x 9 taps, pre-packed in MFMA
//     fragment order) is copied global -> LDS by LDS-DMA (global_load_lds,
//     16 B per lane) one chunk ahead, so the MFMA loop issues no global loads;
//   * the input rows the tile needs (with the 3x3 halo) are loaded into
//     registers one chunk ahead, transformed (GroupNorm apply + SiLU for a
//     ResBlock's convs, GroupNorm only for the attention qkv, nothing for
//     Downsample/Upsample/skip) and written as an LDS image [c][row][col]
//     with a zero column on each side; zero padding therefore pads the
//     activated tensor, as in the oracle.
// Both LDS images are double-buffered; one barrier per chunk.
//
// K order inside a chunk: lane half h takes channels 2h, 2h+1; k-step s takes
// channel s/9 of that pair and tap s%9, so a lane's LDS operand address is a
// per-lane base plus a per-step immediate.  The host packs W in exactly this
// order: [co_tile32][chunk][step pair][lane][2] (ds_read_b64 per 2 steps).
//
// Skip concatenations (the up path) are read from two source tensors in place
// (channels [0,Ca) from srcA, [Ca,Ca+Cb) from srcB); the nearest x2 Upsample is
// folded into the staging address (source row/col = staged row/col >> 1) for
// the bf16 kernel; the fp32 kernel runs the Upsample conv sub-pixel
// (MODE_UPP): output pixel (2i+a, 2j+b) of conv3x3(nearest_x2(x)) reads only
// source rows {i-1+a, i+a} and columns {j-1+b, j+b}, so each parity class
// (a, b) is a 2x2 conv at the SOURCE resolution with taps summed from the
// 3x3 kernel (a=0: row taps {W0, W1+W2}; a=1: {W0+W1, W2}; same for columns)
// -- 4 taps per output pixel instead of 9, exact up to the fp32 rounding of
// the summed weights.  grid.x = 4 classes x pixel tiles; the epilogue
// scatters each class to its output parity.
#include <cstdlib>
#include <type_traits>

#include "unet.h"
#include "unet_pack.h"

namespace ertd {
namespace unet {

// ERTD_UNET_TPX=1|2 forces the wave tile (diagnostics); 0 = automatic
static int conv_tpx_override() {
  static int v = [] {
    return ERTD_KNOB("UNET_TPX", 0);
  }();
  return v;
}

// LDS byte address of a pointer into dynamic shared memory (the M0 base of an
// LDS-DMA instruction)
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// channels per K-chunk: conv_ck (unet_pack.h) -- 4 for 3x3 (36-deep K per chunk), 32 for 1x1

template <int KS, int MODE, int WCO, int WO, int TPX>
struct ConvGeom {
  static constexpr int WPX = 4 / WCO;
  static constexpr int BM = 32 * TPX * WPX;           // output pixels per workgroup
  static constexpr int BN = 64 * WCO;                 // output channels per workgroup
  static constexpr int WST = MODE == MODE_S2 ? 2 * WO : WO;   // staged image width
  static constexpr int R = BM / WO;                   // output rows per workgroup
  static constexpr int IR = KS == 1 ? R : (KS == 2 ? R + 1 : (MODE == MODE_S2 ? 2 * R + 1 : R + 2));
  // 1x1: the chunk image is [channel][BM pixels] (no halo, no row pitch)
  static constexpr int IP = KS == 1 ? BM : WST + 2;   // LDS row pitch (zero column each side)
  static constexpr int CP = KS == 1 ? BM : IR * IP;   // channel pitch
  static constexpr int CKK = conv_ck(KS);             // input channels per chunk
  static constexpr int CH = CKK / 2;                  // channels per lane half
  static constexpr int HP = CH * CP + (MODE == MODE_S2 ? 1 : 0);  // lane-half pitch
  static constexpr int XB = (2 * HP + 3) / 4 * 4;     // input image floats per buffer
  static constexpr int SPC = KS == 3 ? 9 * CH : (KS == 2 ? 4 * CH : CH);   // k-steps per chunk
  static constexpr int TW = SPC * 64;                 // weight floats per 32-cout tile and chunk
  static constexpr int WB = (BN / 32) * TW;           // weight floats per buffer
  static constexpr int RSTEP = NTHR / WST;            // staged rows per thread pass
  static constexpr int NROWS = CKK * IR;
  static constexpr int NIT = KS == 1 ? CKK * BM / 4 / NTHR      // 1x1: float4s per thread
                                     : (NROWS + RSTEP - 1) / RSTEP;
  static constexpr int NGL = WB / 256;                // 16-B-per-lane DMA instructions per chunk
  static constexpr size_t LDS = (size_t)(2 * XB + 2 * WB) * sizeof(float);
  static_assert(BM % WO == 0, "tile must hold whole output rows");
  static_assert(WST <= NTHR, "staged row wider than the workgroup");
  static_assert(WB % 256 == 0, "weight slice must be whole DMA instructions");
  static_assert(KS != 1 || (CKK * BM / 4) % NTHR == 0, "1x1: whole float4s per thread");
};

// STG = input staging schedule: 0 = rows loaded one chunk ahead, LDS stores
// interleaved into the second 3/4 of the chunk's MFMAs; 1 = rows loaded two
// chunks ahead, stored at the top of the chunk.
template <int KS, int MODE, int ACT, int WCO, int WO, int TPX, int STG>
__global__ __launch_bounds__(NTHR) void conv_kernel(ConvArgs a) {
  using G = ConvGeom<KS, MODE, WCO, WO, TPX>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* wim = smem;                  // [2][WB] weight slices (DMA targets, 16-B aligned)
  float* xim = smem + 2 * G::WB;      // [2][XB] input images
  float2* gtab = reinterpret_cast<float2*>(smem + 2 * G::WB + 2 * G::XB);  // [Cin] GN scale/shift

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int wco = wave % WCO, wpx = wave / WCO;
  const int b = blockIdx.z;
  // MODE_UPP: parity class (pa, pb) of this workgroup's output pixels
  const int cls = MODE == MODE_UPP ? (int)(blockIdx.x & 3) : 0;
  const int pa = cls >> 1, pb = cls & 1;
  const int p0 = (MODE == MODE_UPP ? (int)(blockIdx.x >> 2) : (int)blockIdx.x) * G::BM;
  const int oy0 = p0 / WO;
  const int Cin = a.Cin, Ca = a.Ca;
  constexpr int HS = MODE == MODE_UP ? WO / 2 : G::WST;   // source height = width (square)
  constexpr int HST = MODE == MODE_UP ? WO : G::WST;      // staged image height
  constexpr int CK = G::CKK;
  const int nchunk = (Cin + CK - 1) / CK;

  // ---- GroupNorm table of this sample, zero halo columns of both images
  if constexpr (ACT != ACT_NONE) {
    for (int c = tid; c < Cin; c += NTHR) gtab[c] = a.gn[(size_t)b * Cin + c];
  }
  for (int r = tid; KS != 1 && r < 2 * CK * G::IR; r += NTHR) {  // rows of [buf][c][row]
    const int buf = r / (CK * G::IR), rem = r - buf * (CK * G::IR);
    const int c = rem / G::IR, rr = rem - c * G::IR;
    float* row = xim + buf * G::XB + (c / G::CH) * G::HP + (c % G::CH) * G::CP + rr * G::IP;
    row[0] = 0.f;
    row[G::IP - 1] = 0.f;
  }

  // ---- staging geometry: thread -> (column, first row slot)
  const int col = tid % G::WST;
  const int rs0 = tid / G::WST;
  int row0;
  if constexpr (KS == 1) row0 = oy0;
  else if constexpr (MODE == MODE_S2) row0 = 2 * oy0 - 1;
  else if constexpr (MODE == MODE_UPP) row0 = oy0 - 1 + pa;
  else row0 = oy0 - 1;
  const int sx = MODE == MODE_UP ? (col >> 1) : col;
  constexpr size_t plane = (size_t)HS * HS;

  // 1x1: a chunk is 32 channel rows of BM contiguous pixels -- float4 loads
  // and ds_write_b128 (4 per thread at BM = 128), no halo, no row arithmetic
  using StgT = std::conditional_t<KS == 1, float4, float>;
  StgT stg[G::NIT];
  // branch-free: out-of-image / padded-channel elements load a valid address
  // and are replaced by zero
  auto load_chunk = [&](int k) {
    if constexpr (KS == 1) {
#pragma unroll
      for (int it = 0; it < G::NIT; ++it) {
        const int q = tid + it * NTHR;                 // float4 of the chunk
        const int c = q / (G::BM / 4), p4 = q - c * (G::BM / 4);
        const int cg = k * CK + c;
        const int cgc = cg < Cin ? cg : 0;
        const float* src = cgc < Ca ? a.srcA + ((size_t)b * Ca + cgc) * plane
                                    : a.srcB + ((size_t)b * a.Cb + (cgc - Ca)) * plane;
        stg[it] = *reinterpret_cast<const float4*>(src + p0 + 4 * p4);
      }
      return;
    } else {
#pragma unroll
    for (int it = 0; it < G::NIT; ++it) {
      const int fr = rs0 + it * G::RSTEP;
      const int c = fr / G::IR, r = fr - c * G::IR;
      const int cg = k * CK + c;
      const int iy = row0 + r;
      const bool ok = (fr < G::NROWS) && cg < Cin && iy >= 0 && iy < HST;
      const int cgc = ok ? cg : 0;
      const int sy = ok ? (MODE == MODE_UP ? (iy >> 1) : iy) : 0;
      const float* src = cgc < Ca ? a.srcA + ((size_t)b * Ca + cgc) * plane
                                  : a.srcB + ((size_t)b * a.Cb + (cgc - Ca)) * plane;
      stg[it] = src[sy * HS + sx];   // raw; the zero select happens in store_chunk
    }
    }
  };
  // one staged element: GroupNorm(+SiLU) and the LDS write (element it of chunk k)
  auto store_elem = [&](int it, int k, float* img) {
    if constexpr (KS == 1) {
      const int q = tid + it * NTHR;
      const int c = q / (G::BM / 4), p4 = q - c * (G::BM / 4);
      const int cg = k * CK + c;
      float4 v = stg[it];
      if constexpr (ACT != ACT_NONE) {
        const float2 g = gtab[cg < Cin ? cg : 0];
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
      if (cg >= Cin) v = make_float4(0.f, 0.f, 0.f, 0.f);
      // channel c of the chunk is lane half c / CH's channel c % CH
      *reinterpret_cast<float4*>(img + (c / G::CH) * G::HP + (c % G::CH) * G::CP + 4 * p4) = v;
      return;
    } else {
    const int fr = rs0 + it * G::RSTEP;
    if (fr < G::NROWS) {
      const int c = fr / G::IR, r = fr - c * G::IR;
      const int cg = k * CK + c;
      const int iy = row0 + r;
      const bool ok = cg < Cin && iy >= 0 && iy < HST;
      float v = stg[it];
      if constexpr (ACT != ACT_NONE) {
        const float2 g = gtab[ok ? cg : 0];
        v = fmaf(v, g.x, g.y);  // ATen's folded GroupNorm: x*scale + shift
        if constexpr (ACT == ACT_GN_SILU) v = v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));
      }
      img[(c / G::CH) * G::HP + (c % G::CH) * G::CP + r * G::IP + col + 1] = ok ? v : 0.f;
    }
    }
  };
  auto store_chunk = [&](int k, float* img) {
#pragma unroll
    for (int it = 0; it < G::NIT; ++it) store_elem(it, k, img);
  };

  // ---- weight slice DMA: chunk k of this workgroup's BN/32 tiles -> wim[buf]
  const int tile_wg = blockIdx.y * (G::BN / 32);
  const size_t wcls = MODE == MODE_UPP
                          ? (size_t)cls * ((a.Cout + 127) / 128 * 4) * nchunk * G::TW : 0;
  // LDS-DMA by inline asm: hipcc's own global_load_lds bookkeeping waits
  // vmcnt(0) before every DMA (serialising them); here they are counted by
  // hand -- the single wait is the vmcnt(0) ahead of the chunk's barrier.
  auto dma_weights = [&](int k, float* wdst) {
#pragma unroll
    for (int j = 0; j < (G::NGL + 3) / 4; ++j) {
      const int ins = wave + 4 * j;                 // wave-uniform
      if (ins < G::NGL) {
        const int f = ins * 256 + lane * 4;          // float index in the slice
        const int ti = f / G::TW, wi = f - ti * G::TW;
        const float* src = a.wpk + wcls + ((size_t)(tile_wg + ti) * nchunk + k) * G::TW + wi;
        const unsigned dst = __builtin_amdgcn_readfirstlane(lds_addr(wdst + ins * 256));
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

  // ---- per-lane LDS operand bases (pixel tiles t < TPX of this wave)
  int lbase[TPX];
#pragma unroll
  for (int t = 0; t < TPX; ++t) {
    const int pl = wpx * 32 * TPX + t * 32 + l32;
    const int oyl = pl / WO, ox = pl - oyl * WO;
    int rb, cb;
    if constexpr (KS == 1) { rb = 0; cb = pl; }
    else if constexpr (KS == 2) { rb = oyl; cb = ox + pb; }
    else if constexpr (MODE == MODE_S2) { rb = 2 * oyl; cb = 2 * ox; }
    else { rb = oyl; cb = ox; }
    lbase[t] = h * G::HP + rb * G::IP + cb;
  }
  const int abase = (wco * 2) * G::TW + lane * 2;

  f32x16 acc[2][TPX];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TPX; ++j) acc[i][j] = f32x16{};

  dma_weights(0, wim);
  if constexpr (ACT != ACT_NONE) __syncthreads();  // gtab visible to store_chunk
  load_chunk(0);
  store_chunk(0, xim);
  if constexpr (STG == 1) {
    if (nchunk > 1) load_chunk(1);
  }
  dma_wait();
  __syncthreads();

  constexpr int H0 = G::SPC / 4;  // STG 0: first step pair that carries staging work
  for (int k = 0; k < nchunk; ++k) {
    const int cur = k & 1;
    const float* xb = xim + cur * G::XB;
    const float* wb = wim + cur * G::WB;
    if constexpr (STG == 1) {
      // input rows two chunks ahead: chunk k+1's registers were loaded during
      // chunk k-1 and completed at its closing vmcnt(0), so the stores below
      // never wait on memory; chunk k+2's loads and chunk k+1's weight DMA
      // then have a whole chunk of MFMAs to land.
      if (k + 1 < nchunk) {
        store_chunk(k + 1, xim + (cur ^ 1) * G::XB);
        if (k + 2 < nchunk) load_chunk(k + 2);
        dma_weights(k + 1, wim + (cur ^ 1) * G::WB);
      }
    } else if (k + 1 < nchunk) {
      dma_weights(k + 1, wim + (cur ^ 1) * G::WB);
      load_chunk(k + 1);
    }
#pragma unroll
    for (int sp = 0; sp < G::SPC / 2; ++sp) {
      const float2 w0 = *reinterpret_cast<const float2*>(wb + abase + sp * 128);
      const float2 w1 = *reinterpret_cast<const float2*>(wb + abase + G::TW + sp * 128);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int s = 2 * sp + e;
        int off;
        if constexpr (KS == 1) off = s * G::CP;
        else if constexpr (KS == 2) off = (s / 4) * G::CP + ((s % 4) / 2) * G::IP + (s % 2);
        else off = (s / 9) * G::CP + ((s % 9) / 3) * G::IP + (s % 3);
        float bv[TPX];
#pragma unroll
        for (int t = 0; t < TPX; ++t) bv[t] = xb[lbase[t] + off];
        const float a0 = e ? w0.y : w0.x;
        const float a1 = e ? w1.y : w1.x;
#pragma unroll
        for (int t = 0; t < TPX; ++t) {
          acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv[t], acc[0][t], 0, 0, 0);
          acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv[t], acc[1][t], 0, 0, 0);
        }
      }
      // the next chunk's staging work, spread over the second half of the
      // step pairs: its VALU issues in the gaps of this chunk's MFMAs
      // (a 32x32x2 f32 MFMA occupies the SIMD's matrix pipe for 64 cycles)
      if (STG == 0 && k + 1 < nchunk && sp >= H0) {
#pragma unroll
        for (int it = 0; it < G::NIT; ++it)
          if (H0 + it % (G::SPC / 2 - H0) == sp) store_elem(it, k + 1, xim + (cur ^ 1) * G::XB);
      }
    }
    dma_wait();
    __syncthreads();
  }

  // ---- epilogue: bias (+ per-sample channel add) (+ residual), NCHW store.
  // All loads of a 32-cout tile are issued before any of its stores: out and
  // res may not alias, but without the explicit phases hipcc must assume they
  // do and serialises every residual load behind the previous store.
  // Phases of 8 accumulator rows with 32-bit offsets from one per-lane base
  // keep the epilogue's live registers below the main loop's.
  if constexpr (MODE == MODE_UPP) {
    // scatter the class's pixels to their output parity (2i+pa, 2j+pb)
    constexpr int WOUT = 2 * WO, HWO = WOUT * WOUT;
    const int tile0 = tile_wg + wco * 2;
    int pix[TPX];
#pragma unroll
    for (int j = 0; j < TPX; ++j) {
      const int ps = p0 + wpx * 32 * TPX + j * 32 + l32;
      const int oy = ps / WO, ox = ps - oy * WO;
      pix[j] = (2 * oy + pa) * WOUT + 2 * ox + pb;
    }
    float* __restrict__ outb = a.out + (size_t)b * a.Cout * HWO;
    const float* __restrict__ resb = a.res ? a.res + (size_t)b * a.Cout * HWO : nullptr;
    const float* ebp = a.ebias ? a.ebias + (size_t)b * a.eb_stride : nullptr;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = (tile0 + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co >= a.Cout) continue;
        const float bias = a.bias ? a.bias[co] : 0.f;
#pragma unroll
        for (int j = 0; j < TPX; ++j) {
          float v = acc[i][j][r] + bias;
          if (ebp) v = v + ebp[co];
          if (resb) v = v + resb[(size_t)co * HWO + pix[j]];
          outb[(size_t)co * HWO + pix[j]] = v;
        }
      }
    }
    return;
  }
  constexpr int HWo = WO * WO;
  const int tile0 = tile_wg + wco * 2;
  const size_t lbase0 = (size_t)b * a.Cout * HWo + p0 + wpx * 32 * TPX + l32;
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
        int co = (tile0 + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        co = co < a.Cout ? co : a.Cout - 1;
        off[q] = co * HWo;
        bias[q] = a.bias ? a.bias[co] : 0.f;
        eb[q] = ebp ? ebp[co] : 0.f;
#pragma unroll
        for (int j = 0; j < TPX; ++j) rv[q][j] = resp ? resp[off[q] + j * 32] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = ph * 8 + q;
        const int co = (tile0 + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (co >= a.Cout) continue;
#pragma unroll
        for (int j = 0; j < TPX; ++j) {
          // the oracle's op order: conv(+bias), then + emb, then + residual
          float v = acc[i][j][r] + bias[q];
          if (ebp) v = v + eb[q];
          if (resp) v = v + rv[q][j];
          outp[off[q] + j * 32] = v;
        }
      }
    }
  }
}

// ERTD_UNET_STAGE=0|1 picks the staging schedule (diagnostics); default 1
static int conv_stage() {
  static int v = [] {
    return ERTD_KNOB("UNET_STAGE", 1);
  }();
  return v;
}

template <int KS, int MODE, int ACT, int WCO, int WO, int TPX, int STG>
static hipError_t launch_gs(const ConvArgs& a, int B, hipStream_t s) {
  using G = ConvGeom<KS, MODE, WCO, WO, TPX>;
  const size_t lds = G::LDS + (ACT != ACT_NONE ? (size_t)a.Cin * sizeof(float2) : 0);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)conv_kernel<KS, MODE, ACT, WCO, WO, TPX, STG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((unsigned)((MODE == MODE_UPP ? 4 : 1) * WO * WO / G::BM),
            (unsigned)((a.Cout + G::BN - 1) / G::BN), (unsigned)B);
  conv_kernel<KS, MODE, ACT, WCO, WO, TPX, STG><<<grid, NTHR, lds, s>>>(a);
  return hipGetLastError();
}

template <int KS, int MODE, int ACT, int WCO, int WO, int TPX>
static hipError_t launch_g(const ConvArgs& a, int B, hipStream_t s) {
  if (conv_stage() == 0) return launch_gs<KS, MODE, ACT, WCO, WO, TPX, 0>(a, B, s);
  return launch_gs<KS, MODE, ACT, WCO, WO, TPX, 1>(a, B, s);
}

// Wave tile 64 co x 32*TPX px: TPX = 2 (two 32-px accumulator pairs per wave,
// each staged weight fragment feeds twice the MFMAs) for the 3x3 stride-1 and
// sub-pixel convs; TPX = 1 (twice the workgroups, 5 waves/SIMD) for 1x1 and
// stride 2, whose short K or strided staging cannot feed the larger tile.
template <int KS, int MODE, int ACT, int WCO, int WO>
static hipError_t launch_p(const ConvArgs& a, int B, hipStream_t s) {
  const long long wg2 = (long long)(WO * WO / (64 * (4 / WCO))) * ((a.Cout + 64 * WCO - 1) / (64 * WCO)) * B;
  int tpx = conv_tpx_override();
  // measured per layer (U2 B=64, profiles/r01_unet_layers.txt era): TPX=2 wins
  // for the 3x3 stride-1 and sub-pixel Upsample convs (32x32 level -7..-9 %,
  // -270 us per step in all), TPX=1 for 1x1 (8x at 64x64) and stride 2
  // 1x1 since its float4 staging: TPX = 2 (U2 B=64 205.5 vs 202.9 steps/s, same box)
  if (tpx == 0) tpx = ((KS == 3 && MODE == MODE_S1) || MODE == MODE_UPP || KS == 1) ? 2 : 1;
  // ERTD_UNET_TPX1=1|2 picks the 1x1 convs' wave tile alone (A/B); 0 = the above
  static const int t1 = [] {
    return ERTD_KNOB("UNET_TPX1", 0);
  }();
  if (KS == 1 && t1 > 0) tpx = t1;
  (void)wg2;
  if constexpr (32 * (4 / WCO) >= WO) {
    if (tpx == 1) return launch_g<KS, MODE, ACT, WCO, WO, 1>(a, B, s);
  }
  return launch_g<KS, MODE, ACT, WCO, WO, 2>(a, B, s);
}

template <int KS, int MODE, int ACT, int WCO>
static hipError_t launch_w(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 16: return launch_p<KS, MODE, ACT, WCO, 16>(a, B, s);
    case 32: return launch_p<KS, MODE, ACT, WCO, 32>(a, B, s);
    case 64: return launch_p<KS, MODE, ACT, WCO, 64>(a, B, s);
    case 128:
      if constexpr (MODE != MODE_S2) return launch_p<KS, MODE, ACT, WCO, 128>(a, B, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

// ERTD_UNET_WCO=1 forces 64-cout workgroups everywhere (diagnostics); 0 = automatic
static int conv_wco_override() {
  static int v = [] {
    return ERTD_KNOB("UNET_WCO", 0);
  }();
  return v;
}

template <int KS, int MODE, int ACT>
static hipError_t launch_t(const ConvArgs& a, int B, hipStream_t s) {
  if (a.Cout >= 128 && conv_wco_override() != 1) return launch_w<KS, MODE, ACT, 2>(a, B, s);
  return launch_w<KS, MODE, ACT, 1>(a, B, s);
}

// the fp32 Upsample conv through the F(4x4) register-weight kernel
static bool wino4s_up_dispatchable(int ks, int mode, int act, const ConvArgs& a, int B) {
  return ks == 3 && mode == MODE_UP && act == ACT_NONE && a.wpk_wino4 && a.Hs * 2 == a.Ho &&
         wino4s_up_ok(a.Cin, a.Ca, a.Cout, a.Wo, B);
}

int conv_gn_parts(int ks, int mode, int act, const ConvArgs& a, int B) {
  if (a.Cout == 1 && ks == 3 && mode == MODE_S1 && act != ACT_GN) return 0;   // conv_out
#ifndef CONV_IN_PARTS
#define CONV_IN_PARTS 1   // 0 (A/B only): conv_in emits no partials, the walk runs a partials pass
#endif
  if (conv_in_ok(a, ks, mode, act)) return CONV_IN_PARTS ? a.Wo * a.Wo / 256 : 0;   // conv_in_kernel: one part per 256 px
  if (ks == 3 && mode == MODE_S1 && wino_dispatchable(a, B)) return wino_gn_parts(a, B);
  if (wino4s_up_dispatchable(ks, mode, act, a, B)) return (a.Wo / 4) * (a.Wo / 4) / 16;
  return 0;
}

bool conv_gn_fold_ok(int ks, int mode, int act, const ConvArgs& a, int B) {
  if (conv_gn_parts(ks, mode, act, a, B) == 0) return false;
  if (ks == 3 && mode == MODE_S1 && wino_dispatchable(a, B))
    return a.wpk_wino4 && wino4s_ok(a.Cin, a.Ca, a.Cout, a.Wo, B) && wino4s_fold_ok(a, false, B);
  if (wino4s_up_dispatchable(ks, mode, act, a, B)) return wino4s_fold_ok(a, true, B);
  return false;
}

bool conv_gn_consume_ok(int ks, int mode, int act, const ConvArgs& a, int B) {
  if (ks != 3 || mode != MODE_S1 || act == ACT_NONE || a.Cout == 1 || !a.wpk_wino4) return false;
  if (!wino_dispatchable(a, B) || !wino4s_ok(a.Cin, a.Ca, a.Cout, a.Wo, B)) return false;
  return wino4s_gnc_ok(a, B);
}

int conv_gn_fold_target(const ConvArgs& a, int B) {
  (void)B;
  return wino4s_fold_target(a);
}

hipError_t launch_conv(int ks, int mode, int act, const ConvArgs& a, int B, hipStream_t s) {
  if (a.Ho != a.Wo || a.Hs != a.Ws || a.Cin != a.Ca + a.Cb) return hipErrorInvalidValue;
  if (a.gnp && conv_gn_parts(ks, mode, act, a, B) == 0) return hipErrorInvalidValue;
  if (a.fold.cnt && (!a.gnp || a.fold.g.pa != a.gnp || !conv_gn_fold_ok(ks, mode, act, a, B)))
    return hipErrorInvalidValue;
  if (a.gnc.pa && (a.gnc.Ca + a.gnc.Cb != a.Cin || !conv_gn_consume_ok(ks, mode, act, a, B)))
    return hipErrorInvalidValue;
  const int expect = mode == MODE_S2 ? a.Ws / 2 : (mode == MODE_UP ? a.Ws * 2 : a.Ws);
  if (a.Wo != expect) return hipErrorInvalidValue;
  if (a.Cout == 1 && ks == 3 && mode == MODE_S1 && act != ACT_GN)
    return launch_conv_out(act, a, B, PK_F32, s);
  if (conv_in_ok(a, ks, mode, act)) return launch_conv_in(a, B, PK_F32, s);
  if (ks == 3 && mode == MODE_S1 && wino_dispatchable(a, B))
    return launch_conv_wino(act, a, B, s);
  if (ks == 3 && mode == MODE_S1 && act == ACT_NONE) return launch_t<3, MODE_S1, ACT_NONE>(a, B, s);
  if (ks == 3 && mode == MODE_S1 && act == ACT_GN_SILU) return launch_t<3, MODE_S1, ACT_GN_SILU>(a, B, s);
  if (ks == 3 && mode == MODE_S2 && act == ACT_NONE) return launch_t<3, MODE_S2, ACT_NONE>(a, B, s);
  if (wino4s_up_dispatchable(ks, mode, act, a, B)) return launch_conv_wino4s(act, a, B, s, device_cu_count());
  if (ks == 3 && mode == MODE_UP && act == ACT_NONE) {
    // sub-pixel: 2x2 taps per class at the source resolution (weights packed
    // by launch_pack_conv_up); the template width is the SOURCE width
    const bool w2 = a.Cout >= 128 && conv_wco_override() != 1;
    switch (a.Ws) {
      case 16: return w2 ? launch_p<2, MODE_UPP, ACT_NONE, 2, 16>(a, B, s) : launch_p<2, MODE_UPP, ACT_NONE, 1, 16>(a, B, s);
      case 32: return w2 ? launch_p<2, MODE_UPP, ACT_NONE, 2, 32>(a, B, s) : launch_p<2, MODE_UPP, ACT_NONE, 1, 32>(a, B, s);
      case 64: return w2 ? launch_p<2, MODE_UPP, ACT_NONE, 2, 64>(a, B, s) : launch_p<2, MODE_UPP, ACT_NONE, 1, 64>(a, B, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (skip_gemm_ok(a, ks, mode, act, B)) return launch_skip_gemm(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_NONE && conv1x1_ok(a, act, B)) return launch_conv1x1(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_NONE) return launch_t<1, MODE_S1, ACT_NONE>(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_GN) return launch_t<1, MODE_S1, ACT_GN>(a, B, s);
  return hipErrorInvalidValue;
}

// ---- weight packing: W (Cout, Cin, ks, ks) -> [co_tile32][chunk][step pair][lane][2]
// Cout is padded to a multiple of 128 (a workgroup's tiles never run past the
// end), Cin to a multiple of CK; padding is zero.
size_t conv_packed_floats(int cin, int cout, int ks) {
  const int ck = conv_ck(ks);
  const size_t tiles = (size_t)((cout + 127) / 128) * 4;
  const size_t nchunk = (size_t)((cin + ck - 1) / ck);
  return tiles * nchunk * (ks == 3 ? 9 * ck / 2 : (ks == 2 ? 4 * ck / 2 : ck / 2)) * 64;
}

__global__ void pack_conv_kernel(const float* __restrict__ w, int cin, int cout, int ks,
                                 int nchunk, size_t total, float* __restrict__ dst, bool flipT) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  dst[i] = pack_conv_elem(w, cin, cout, ks, nchunk, i, flipT);
}

// Upsample conv: W (Cout, Cin, 3, 3) -> 4 classes (pa, pb) of 2x2 taps in the
// ks = 2 packed order ([class][co_tile32][chunk][step pair][lane][2]); tap
// (ty, tx) of class (pa, pb) = sum of W[ky][kx] over ky in S(pa, ty), kx in
// S(pb, tx), S(0,0) = {0}, S(0,1) = {1,2}, S(1,0) = {0,1}, S(1,1) = {2}
size_t conv_packed_floats_up(int cin, int cout) { return 4 * conv_packed_floats(cin, cout, 2); }

__global__ void pack_conv_up_kernel(const float* __restrict__ w, int cin, int cout, int nchunk,
                                    size_t per_class, float* __restrict__ dst) {
  const size_t gi = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= 4 * per_class) return;
  dst[gi] = pack_conv_up_elem(w, cin, cout, nchunk, per_class, gi);
}

hipError_t launch_pack_conv_up(const float* w, int cin, int cout, float* dst, hipStream_t s) {
  const size_t per = conv_packed_floats(cin, cout, 2);
  const int nchunk = (cin + conv_ck(2) - 1) / conv_ck(2);
  pack_conv_up_kernel<<<(unsigned)((4 * per + 255) / 256), 256, 0, s>>>(w, cin, cout, nchunk, per, dst);
  return hipGetLastError();
}

hipError_t launch_pack_conv(const float* w, int cin, int cout, int ks, float* dst, hipStream_t s,
                            bool flipT) {
  const size_t total = conv_packed_floats(cin, cout, ks);
  const int nchunk = (cin + conv_ck(ks) - 1) / conv_ck(ks);
  pack_conv_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(w, cin, cout, ks, nchunk, total, dst,
                                                                    flipT);
  return hipGetLastError();
}

}  // namespace unet
}  // namespace ertd
