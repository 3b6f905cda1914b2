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
using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ unsigned bf16_bits(float v) {  // round to nearest even (finite v)
  const uint32_t u = __float_as_uint(v);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// the split-bf16 low part: bf16 RNE of v - hi (exact in fp32)
__device__ __forceinline__ unsigned bf16_lo_bits(float v, unsigned hi) {
  return bf16_bits(v - __uint_as_float(hi << 16));
}

__device__ __forceinline__ unsigned lds_addr_h(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

__host__ __device__ constexpr int convh_ck(int ks) { return ks == 3 ? 16 : 32; }

// fp32 sum over the 64 lanes of a wave in a fixed order, the same bits in
// every lane: row sums by DPP (row16_sum), then (r0 + r1) + (r2 + r3)
__device__ __forceinline__ float wave_sum_f(float v) {
  v = row16_sum(v);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

// SP = operand planes: 1 = bf16, 2 = split bf16 (x = hi + lo, both bf16 RNE;
// every product as lo_a*hi_b + hi_a*lo_b + hi_a*hi_b on the MFMA, fp32
// accumulate: ~2^-16 relative per product instead of bf16's 2^-8).  A split
// pixel record is [16 hi][16 lo] bf16 (64 B), a split weight slice [hi steps]
// [lo steps] per (co tile, chunk).
template <int KS, int MODE, int WO, int TPX, int SP = 1>
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
  static constexpr int PB = 32 * SP;                  // bytes per staged pixel record
  static constexpr int GB = IR * IP * PB;             // bytes per 16-channel group image
  static constexpr int XB = NG * GB;                  // input image bytes per buffer
  static constexpr int TWB = SPC * 64 * 16 * SP;      // weight bytes per 32-co tile and chunk
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

// PRE: the input was already transformed (GN/SiLU, bf16 RNE, channel padding)
// by act_bf16_kernel into a.bimg = [B][ceil(Cin/16)][H][W][16] bf16 -- the LDS
// image layout row by row -- so staging is LDS-DMA of whole rows (stride-1
// convs only): no staging VALU in the conv at all.
// DBG (diagnostics only, ERTD_BF16_DBG, 3x3 PRE path; results wrong): bit 0
// skips the epilogue's stores and residual loads, bit 1 the MFMAs, bit 2 the
// row DMA, bit 3 the weight DMA
template <int KS, int MODE, int ACT, int WO, int TPX, bool PRE, int DBG = 0, int SP = 1>
__global__ __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(2))) void conv_bf16_kernel(ConvArgs a) {
  using G = GeomH<KS, MODE, WO, TPX, SP>;
  extern __shared__ __attribute__((aligned(16))) char smemh[];
  char* wim = smemh;                          // [2][WBB]
  char* xim = smemh + 2 * G::WBB;             // [2][XB]
  // {bias, emb} of the workgroup's 64 output channels (read by the epilogue
  // from LDS: its only global loads are then the residual's), then the
  // GroupNorm table
  float2* etab = reinterpret_cast<float2*>(smemh + G::LDS);
  float2* gtab = reinterpret_cast<float2*>(smemh + G::LDS + 64 * sizeof(float2));

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
  if (tid < 64) {
    const int co = blockIdx.y * 64 + tid;
    const bool ok = co < a.Cout;
    etab[tid] = make_float2(ok && a.bias ? a.bias[co] : 0.f,
                            ok && a.ebias ? a.ebias[(size_t)b * a.eb_stride + co] : 0.f);
  }
  if constexpr (PRE) {
    // every LDS image byte starts at zero: halo columns and out-of-image rows
    // are never written by the row DMA
    for (int i = tid; i < 2 * G::XB / 16; i += NTHR)
      reinterpret_cast<u32x4*>(xim)[i] = u32x4{0u, 0u, 0u, 0u};
  }
  // zero halo pixels (cols 0 and IP-1) of every row, group, buffer
  for (int r = tid; !PRE && r < 2 * G::NG * G::IR * 2; r += NTHR) {
    const int side = r & 1, rest = r >> 1;
    const int buf = rest / (G::NG * G::IR), rem = rest - buf * (G::NG * G::IR);
    const int g = rem / G::IR, rr = rem - g * G::IR;
    u32x4* px = reinterpret_cast<u32x4*>(xim + buf * G::XB + g * G::GB +
                                         (rr * G::IP + (side ? G::IP - 1 : 0)) * G::PB);
#pragma unroll
    for (int q = 0; q < 2 * SP; ++q) px[q] = u32x4{0u, 0u, 0u, 0u};
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
      unsigned w[4], wl[4];
#pragma unroll
      for (int j2 = 0; j2 < 4; ++j2) {
        unsigned bits[2], lbits[2];
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
          if constexpr (SP == 2) lbits[e] = ok ? bf16_lo_bits(v, bits[e]) : 0u;
        }
        w[j2] = bits[0] | (bits[1] << 16);
        if constexpr (SP == 2) wl[j2] = lbits[0] | (lbits[1] << 16);
      }
      char* px = img + (hg >> 1) * G::GB + (r * G::IP + col + 1) * G::PB + (hg & 1) * 16;
      *reinterpret_cast<u32x4*>(px) = u32x4{w[0], w[1], w[2], w[3]};
      if constexpr (SP == 2) *reinterpret_cast<u32x4*>(px + 32) = u32x4{wl[0], wl[1], wl[2], wl[3]};
    }
  };

  const int tile_wg = blockIdx.y * 2;
  auto dma_weights = [&](int k, char* wdst) {
    if constexpr (DBG & 8) return;
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

  // PRE: chunk k's rows of the pre-transformed image -> img (LDS-DMA, 16 B per
  // lane, one instruction per 1 KB of a row; a 16-pixel row is half a wave)
  constexpr int RB = G::WST * G::PB;                       // bytes per image row
  constexpr int IPR = RB >= 1024 ? RB / 1024 : 1;          // DMA instructions per row
  const int G16 = (Cin + 15) / 16;
  auto dma_rows = [&](int k, char* img) {
    if constexpr (DBG & 4) return;
    for (int q = wave; q < G::NG * G::IR * IPR; q += 4) {  // wave-uniform
      const int g = q / (G::IR * IPR), rr = q - g * (G::IR * IPR);
      const int r = rr / IPR, part = rr - r * IPR;
      const int iy = row0 + r;
      const int gg = k * G::NG + g;
      if (iy < 0 || iy >= HST || gg >= G16) continue;
      if (RB < 1024 && lane >= RB / 16) continue;
      const char* src = reinterpret_cast<const char*>(a.bimg) +
                        (((size_t)b * G16 + gg) * HST + iy) * RB + part * 1024 + lane * 16;
      const unsigned dst = __builtin_amdgcn_readfirstlane(
          lds_addr_h(img + g * G::GB + (r * G::IP + 1) * G::PB + part * 1024));
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(src), "s"(dst)
          : "memory");
    }
  };

  int lbase[TPX];
#pragma unroll
  for (int t = 0; t < TPX; ++t) {
    const int pl = wave * 32 * TPX + t * 32 + l32;
    const int oyl = pl / WO, ox = pl - oyl * WO;
    int rb, cb;
    if constexpr (KS == 1) { rb = oyl; cb = ox + 1; }
    else if constexpr (MODE == MODE_S2) { rb = 2 * oyl; cb = 2 * ox; }
    else { rb = oyl; cb = ox; }
    lbase[t] = (rb * G::IP + cb) * G::PB + h * 16;
  }
  const int abase = lane * 16;

  f32x16 acc[2][TPX];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < TPX; ++t) acc[i][t] = f32x16{};

  if constexpr (PRE) {
    __syncthreads();                     // zeroed images before any DMA lands
    dma_weights(0, wim);
    dma_rows(0, xim);
  } else {
    dma_weights(0, wim);
    if constexpr (ACT != ACT_NONE) __syncthreads();
    load_chunk(0);
#pragma unroll
    for (int it = 0; it < G::NIT; ++it) store_elem(it, 0, xim);
    if (nchunk > 1) load_chunk(1);
  }
  dma_wait();
  __syncthreads();

  // rows two chunks ahead, stored at the top of the chunk (unet_conv.hip STG 1)
  for (int k = 0; k < nchunk; ++k) {
    const int cur = k & 1;
    const char* xb = xim + cur * G::XB;
    const char* wb = wim + cur * G::WBB;
    if (k + 1 < nchunk) {
      if constexpr (PRE) {
        dma_rows(k + 1, xim + (cur ^ 1) * G::XB);
      } else {
#pragma unroll
        for (int it = 0; it < G::NIT; ++it) store_elem(it, k + 1, xim + (cur ^ 1) * G::XB);
        if (k + 2 < nchunk) load_chunk(k + 2);
      }
      dma_weights(k + 1, wim + (cur ^ 1) * G::WBB);
    }
#pragma unroll
    for (int s = 0; s < G::SPC; ++s) {
      const int g = s / G::TAPS, tap = s % G::TAPS;
      int off;
      if constexpr (KS == 1) off = g * G::GB;
      else off = g * G::GB + ((tap / 3) * G::IP + (tap % 3)) * G::PB;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(wb + s * 1024 + abase);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(wb + G::TWB + s * 1024 + abase);
      bf16x8 a0l{}, a1l{};
      if constexpr (SP == 2) {
        a0l = *reinterpret_cast<const bf16x8*>(wb + (G::SPC + s) * 1024 + abase);
        a1l = *reinterpret_cast<const bf16x8*>(wb + G::TWB + (G::SPC + s) * 1024 + abase);
      }
#pragma unroll
      for (int t = 0; t < TPX; ++t) {
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(xb + lbase[t] + off);
        if constexpr (DBG & 2) {
          acc[0][t][0] += (float)a0[0] * (float)bv[0];
          acc[1][t][0] += (float)a1[1] * (float)bv[1];
        } else if constexpr (SP == 2) {
          // the two cross terms first (small), then hi*hi
          const bf16x8 bl = *reinterpret_cast<const bf16x8*>(xb + lbase[t] + off + 32);
          acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0l, bv, acc[0][t], 0, 0, 0);
          acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1l, bv, acc[1][t], 0, 0, 0);
          acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bl, acc[0][t], 0, 0, 0);
          acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bl, acc[1][t], 0, 0, 0);
          acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bv, acc[0][t], 0, 0, 0);
          acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bv, acc[1][t], 0, 0, 0);
        } else {
          acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bv, acc[0][t], 0, 0, 0);
          acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bv, acc[1][t], 0, 0, 0);
        }
      }
    }
    dma_wait();
    __syncthreads();
  }

  // ---- epilogue: every residual value of the tile is loaded before any
  // store (loads and stores share vmcnt: a load after a store would wait for
  // it), bias / emb from LDS
  constexpr int HWo = WO * WO;
  if constexpr (DBG & 1) {
    float sacc = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < TPX; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc += acc[i][t][r];
    if (sacc == 12345.f) a.out[tid] = sacc;
    return;
  }
  // the accumulators go through LDS (the image / weight buffers are free
  // now), one 32-channel tile at a time, so that every lane stores whole
  // float4s of one channel's pixel row (64 scalar stores per lane before:
  // store-issue-bound, ~30 % of a 64-channel layer); every residual value is
  // loaded before any store (loads and stores share vmcnt)
  constexpr int TP = G::BM + 4;                       // LDS row pitch (floats)
  constexpr int NQ4 = 32 * G::BM / 4 / NTHR;          // float4s per thread and tile
  static_assert(32 * TP * 4 <= 2 * G::XB + 2 * G::WBB, "epilogue tile fits the freed buffers");
  static_assert((32 * G::BM / 4) % NTHR == 0, "whole float4 rows per thread");
  float* et = reinterpret_cast<float*>(smemh);
  const bool has_eb = a.ebias != nullptr;
  const bool has_res = a.res != nullptr;
  // (TPX = 4: 2 x 16 float4 residual registers would cost a wave per SIMD;
  // the second tile's residual is loaded after the first tile's stores)
  constexpr int RV = TPX >= 4 ? 1 : 2;
  f32x4 rv[2][NQ4];
  auto load_res = [&](int i) {
#pragma unroll
    for (int j = 0; j < NQ4; ++j) {
      const int idx = tid + j * NTHR;
      const int cl = idx / (G::BM / 4), q = idx - cl * (G::BM / 4);
      int co = (tile_wg + i) * 32 + cl;
      co = co < a.Cout ? co : a.Cout - 1;
      rv[i % RV][j] = *reinterpret_cast<const f32x4*>(a.res + ((size_t)b * a.Cout + co) * HWo + p0 + 4 * q);
    }
  };
  if (has_res) {
#pragma unroll
    for (int i = 0; i < RV; ++i) load_res(i);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (RV == 1 && i == 1 && has_res) load_res(1);
    __syncthreads();   // the K loop's (or the previous tile's) LDS reads are done
#pragma unroll
    for (int t = 0; t < TPX; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int cl = (r & 3) + 8 * (r >> 2) + 4 * h;
        et[cl * TP + wave * 32 * TPX + t * 32 + l32] = acc[i][t][r];
      }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NQ4; ++j) {
      const int idx = tid + j * NTHR;
      const int cl = idx / (G::BM / 4), q = idx - cl * (G::BM / 4);
      const int co = (tile_wg + i) * 32 + cl;
      if (co >= a.Cout) continue;
      const float2 e = etab[i * 32 + cl];
      f32x4 v = *reinterpret_cast<const f32x4*>(et + cl * TP + 4 * q) + e.x;
      if (has_eb) v = v + e.y;
      if (has_res) v = v + rv[i % RV][j];
      *reinterpret_cast<f32x4*>(a.out + ((size_t)b * a.Cout + co) * HWo + p0 + 4 * q) = v;
      if constexpr (G::BM % 256 == 0 && (G::BM / 4) % 64 == 0) {
        // GroupNorm partials of the output (conv_bf16_gn_parts): with 256- or
        // 512-px tiles one wave's 64 lanes x 4 px are 256 px of one channel (cl
        // is wave-uniform); each 16-lane DPP row -- 64 consecutive px -- is one
        // part, {sum, M2 about the part mean} as the fp32 epilogues emit them
        // (row sums only: no cross-row readlanes, 4x the parts for the finalize)
        if (a.gnp) {
          const float sm = row16_sum((v[0] + v[1]) + (v[2] + v[3]));
          const float mu = sm * (1.0f / 64.0f);
          const float d0 = v[0] - mu, d1 = v[1] - mu, d2 = v[2] - mu, d3 = v[3] - mu;
          const float m2 = row16_sum(fmaf(d3, d3, fmaf(d2, d2, fmaf(d1, d1, d0 * d0))));
          if ((lane & 15) == 0)
            a.gnp[((size_t)b * a.Cout + co) * (HWo / 64) + (p0 + 4 * q) / 64] = make_float2(sm, m2);
        }
      }
    }
  }
}

// The input transform of the PRE path: x (srcA | srcB, fp32 NCHW) -> GN/SiLU
// (ATen's folded x*scale+shift, x*rcp(1+exp(-x))) -> bf16 RNE, written as
// [B][ceil(Cin/16)][H][W][16] with zero padding channels.  One thread per
// (sample, 16-channel group, pixel): 16 coalesced channel-plane loads, one
// 32-B store.  Applied once per activation instead of once per output-channel
// tile and halo row of every conv workgroup.
// UPS: nearest x2 upsample folded in (output pixel (y, x) reads source
// (y/2, x/2)), so an Upsample conv becomes a stride-1 conv on the image.
// SP = 2: split-bf16 records [16 hi][16 lo] (64 B per pixel)
#ifndef ACT_PXG
#define ACT_PXG 1
#endif
template <int ACT, bool UPS = false, int SP = 1>
__global__ __launch_bounds__(256) void act_bf16_kernel(ConvArgs a, int B, int G16, int HW) {
  // UPS: four horizontally adjacent output pixels per thread -- one float2 of
  // the source row per channel plane, four 32-B records stored contiguously
  // (U3 B=256 upsample images 129 -> 95 us); the GN(+SiLU) images keep one
  // pixel per thread (ACT_PXG: two measured 109.5 -> 99.5 U3 B=256 steps/s,
  // four 332 -> 384 us per image, longer chains)
  constexpr int PX = UPS ? 4 : ACT_PXG;
  const long long i4 = (long long)blockIdx.x * 256 + threadIdx.x;
  const int HW4 = HW / PX;
  if (i4 >= (long long)B * G16 * HW4) return;
  const int po = (int)(i4 % HW4) * PX;
  const int HWs = UPS ? a.Ws * a.Ws : HW;
  const int p = UPS ? ((po / a.Wo) >> 1) * a.Ws + ((po % a.Wo) >> 1) : po;
  const long long r = i4 / HW4;
  // a wave's 64 pixels lie in one (sample, 16-channel group) (HW4 % 64 == 0 for
  // every image here): (b, g) wave-uniform, so the GN table is read by scalar loads
  const int g = __builtin_amdgcn_readfirstlane((int)(r % G16));
  const int b = __builtin_amdgcn_readfirstlane((int)(r / G16));
  const int Cin = a.Cin, Ca = a.Ca;
  float v[16][PX];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = g * 16 + j;
#pragma unroll
    for (int k = 0; k < PX; ++k) v[j][k] = 0.f;
    if (c < Cin) {
      const float* src = c < Ca ? a.srcA + ((size_t)b * Ca + c) * HWs
                                : a.srcB + ((size_t)b * a.Cb + (c - Ca)) * HWs;
      if constexpr (UPS) {
        const float2 t = *reinterpret_cast<const float2*>(src + p);
        v[j][0] = v[j][1] = t.x;
        v[j][PX - 2] = v[j][PX - 1] = t.y;
      } else if constexpr (PX == 2) {
        const float2 t = *reinterpret_cast<const float2*>(src + p);
        v[j][0] = t.x;
        v[j][1] = t.y;
      } else {
        v[j][0] = src[p];
      }
    }
  }
  u32x4* dst = reinterpret_cast<u32x4*>(static_cast<char*>(a.bimg) + (size_t)i4 * 32 * SP * PX);
#pragma unroll
  for (int k = 0; k < PX; ++k) {
    unsigned w[8], wl[8];
#pragma unroll
    for (int j2 = 0; j2 < 8; ++j2) {
      unsigned bits[2], lbits[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int c = g * 16 + 2 * j2 + e;
        bits[e] = 0u;
        lbits[e] = 0u;
        if (c < Cin) {
          float x = v[2 * j2 + e][k];
          if constexpr (ACT != ACT_NONE) {
            const float2 gs = a.gn[(size_t)b * Cin + c];
            x = fmaf(x, gs.x, gs.y);
            if constexpr (ACT == ACT_GN_SILU) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
          }
          bits[e] = bf16_bits(x);
          if constexpr (SP == 2) lbits[e] = bf16_lo_bits(x, bits[e]);
        }
      }
      w[j2] = bits[0] | (bits[1] << 16);
      wl[j2] = lbits[0] | (lbits[1] << 16);
    }
    dst[2 * SP * k] = u32x4{w[0], w[1], w[2], w[3]};
    dst[2 * SP * k + 1] = u32x4{w[4], w[5], w[6], w[7]};
    if constexpr (SP == 2) {
      dst[4 * k + 2] = u32x4{wl[0], wl[1], wl[2], wl[3]};
      dst[4 * k + 3] = u32x4{wl[4], wl[5], wl[6], wl[7]};
    }
  }
}

// ---- fused GroupNorm statistics + apply + SiLU + bf16 image (3x3 GN convs) ----------
// One workgroup per (channel set, sample); a channel set is lcm(C/groups, 16)
// channels = NB 16-channel image blocks holding whole groups.  Thread t owns
// NREC pixels p = t + nthr*k and ALL of the set's channels at them, so:
//  - loads: per (channel, k) one coalesced 256-B row per wave, all issued up
//    front into registers (the activation is read from HBM once);
//  - statistics: the thread's values of one group are summed in float64 in
//    a fixed order, one wave reduction per group, then a fixed-order sum of
//    the waves' partials (the sum / sum-of-squares form of gn_stats_kernel);
//    {scale, shift} per channel also go to `gn` (for convs that stage fp32);
//  - output: x*scale+shift, SiLU, bf16 RNE, and the thread writes its whole
//    32-B pixel records of the [B][C/16][H][W][16] image (consecutive lanes =
//    consecutive records) -- no transpose.
// Replaces gn_stats_kernel + act_bf16_kernel: one fp32 read of the activation
// instead of two.
__host__ __device__ constexpr int ga_gcd(int a, int b) { return b == 0 ? a : ga_gcd(b, a % b); }

template <bool SILU, int NREC, int NB, int SP = 1>
__global__ __launch_bounds__(1024) void gn_act_bf16_kernel(GnArgs g, void* bimg) {
  constexpr int NCH = NB * 16;
  __shared__ double2 part[8][16];   // [group in set][wave]
  __shared__ float2 tab[NCH];
  const int C = g.Ca + g.Cb, HW = g.HW;
  const int cpg = C / g.groups;
  const int nthr = HW / NREC;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int set = blockIdx.x, b = blockIdx.y;
  const int c0 = set * NCH;

  float v[NCH][NREC];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int cg = c0 + c;
    const float* src = cg < g.Ca ? g.srcA + ((size_t)b * g.Ca + cg) * HW
                                 : g.srcB + ((size_t)b * g.Cb + (cg - g.Ca)) * HW;
#pragma unroll
    for (int k = 0; k < NREC; ++k) v[c][k] = src[tid + k * nthr];
  }
  double s = 0.0, ss = 0.0;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#pragma unroll
    for (int k = 0; k < NREC; ++k) {
      s += (double)v[c][k];
      ss += (double)v[c][k] * v[c][k];
    }
    if ((c + 1) % cpg == 0) {   // last channel of a group: reduce over the wave
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        ss += __shfl_xor(ss, o);
      }
      if (lane == 0) part[c / cpg][w] = make_double2(s, ss);
      s = 0.0;
      ss = 0.0;
    }
  }
  __syncthreads();
  if (tid < NCH) {
    const int gi = tid / cpg;
    const int nw = nthr / 64;
    double S = 0.0, SS = 0.0;
    for (int k = 0; k < nw; ++k) {
      S += part[gi][k].x;
      SS += part[gi][k].y;
    }
    const double n = (double)cpg * HW;
    const double mean = S / n;
    double var = SS / n - mean * mean;
    var = var > 0.0 ? var : 0.0;
    const float rstd = (float)(1.0 / sqrt(var + GN_EPS));
    const int cg = c0 + tid;
    const float scale = rstd * g.gamma[cg];
    const float shift = -scale * (float)mean + g.beta[cg];
    tab[tid] = make_float2(scale, shift);
    g.out[(size_t)b * C + cg] = make_float2(scale, shift);
  }
  __syncthreads();
  char* base = static_cast<char*>(bimg) + ((size_t)b * (C / 16) + (size_t)set * NB) * HW * 32 * SP;
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
#pragma unroll
    for (int k = 0; k < NREC; ++k) {
      unsigned u[8], ul[8];
#pragma unroll
      for (int j2 = 0; j2 < 8; ++j2) {
        unsigned bits[2], lbits[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int c = blk * 16 + 2 * j2 + e;
          const float2 t = tab[c];
          float x = fmaf(v[c][k], t.x, t.y);
          if constexpr (SILU) x = x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
          bits[e] = bf16_bits(x);
          lbits[e] = SP == 2 ? bf16_lo_bits(x, bits[e]) : 0u;
        }
        u[j2] = bits[0] | (bits[1] << 16);
        ul[j2] = lbits[0] | (lbits[1] << 16);
      }
      u32x4* dst = reinterpret_cast<u32x4*>(base + ((size_t)blk * HW + tid + k * nthr) * 32 * SP);
      dst[0] = u32x4{u[0], u[1], u[2], u[3]};
      dst[1] = u32x4{u[4], u[5], u[6], u[7]};
      if constexpr (SP == 2) {
        dst[2] = u32x4{ul[0], ul[1], ul[2], ul[3]};
        dst[3] = u32x4{ul[4], ul[5], ul[6], ul[7]};
      }
    }
  }
}

// shape plan of the fused path: records per thread (NREC) and image blocks per
// set (NB); false -> gn_stats + the conv's own transform
static bool ga_plan(int C, int groups, int HW, int* nrec, int* nb) {
  if (C % 16 || groups < 1 || C % groups || HW < 64 || HW % 64) return false;
  const int cpg = C / groups;
  const int bch = cpg / ga_gcd(cpg, 16) * 16;
  if (C % bch || bch / cpg > 8) return false;
  const int NB = bch / 16;
  const int NREC = HW <= 1024 ? 1 : HW / 1024;
  if (HW > 1024 && HW % 1024) return false;
  if (!((NB == 1 && (NREC == 1 || NREC == 2 || NREC == 4)) || (NB == 3 && NREC == 1)))
    return false;
  *nrec = NREC;
  *nb = NB;
  return true;
}

bool gn_act_bf16_fits(int C, int groups, int HW) {
  int r, n;
  return ga_plan(C, groups, HW, &r, &n);
}

template <bool SILU, int SP>
static hipError_t launch_ga(const GnArgs& g, int nrec, int nb, void* bimg, int B, hipStream_t s) {
  const int C = g.Ca + g.Cb;
  dim3 grid((unsigned)(C / (16 * nb)), (unsigned)B);
  const int thr = g.HW / nrec;
  if (nb == 3) gn_act_bf16_kernel<SILU, 1, 3, SP><<<grid, thr, 0, s>>>(g, bimg);
  else if (nrec == 1) gn_act_bf16_kernel<SILU, 1, 1, SP><<<grid, thr, 0, s>>>(g, bimg);
  else if (nrec == 2) gn_act_bf16_kernel<SILU, 2, 1, SP><<<grid, thr, 0, s>>>(g, bimg);
  else gn_act_bf16_kernel<SILU, 4, 1, SP><<<grid, thr, 0, s>>>(g, bimg);
  return hipGetLastError();
}

hipError_t launch_gn_act_bf16(const GnArgs& g, bool silu, void* bimg, int B, hipStream_t s, bool split) {
  int nrec, nb;
  if (!bimg || !ga_plan(g.Ca + g.Cb, g.groups, g.HW, &nrec, &nb)) return hipErrorInvalidValue;
  if (split)
    return silu ? launch_ga<true, 2>(g, nrec, nb, bimg, B, s) : launch_ga<false, 2>(g, nrec, nb, bimg, B, s);
  return silu ? launch_ga<true, 1>(g, nrec, nb, bimg, B, s) : launch_ga<false, 1>(g, nrec, nb, bimg, B, s);
}

size_t conv_bf16_image_bytes(int cin, int B, int H, int W, bool split) {
  return (size_t)B * ((cin + 15) / 16) * H * W * 32 * (split ? 2 : 1);
}

template <int KS, int MODE, int ACT, int WO, int TPX, bool PRE = false, int DBG = 0, int SP = 1>
static hipError_t launch_hgd(const ConvArgs& a, int B, hipStream_t s) {
  using G = GeomH<KS, MODE, WO, TPX, SP>;
  // the epilogue writes GroupNorm partials only for 256-multiple pixel tiles:
  // a caller asking for them (a.gnp) of any other tile would read unwritten memory
  if (a.gnp && !(G::BM % 256 == 0 && (G::BM / 4) % 64 == 0)) return hipErrorInvalidValue;
  const size_t lds = G::LDS + 64 * sizeof(float2) + (ACT != ACT_NONE ? (size_t)a.Cin * sizeof(float2) : 0);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)conv_bf16_kernel<KS, MODE, ACT, WO, TPX, PRE, DBG, SP>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  dim3 grid((unsigned)(WO * WO / G::BM), (unsigned)((a.Cout + G::BN - 1) / G::BN), (unsigned)B);
  conv_bf16_kernel<KS, MODE, ACT, WO, TPX, PRE, DBG, SP><<<grid, NTHR, lds, s>>>(a);
  return hipGetLastError();
}

#ifdef ERTD_DIAG
// ablation variants (results wrong): only in a diagnostic build of the library
// (tools/build_variant.sh ... "-DERTD_DIAG"), never in the shipped one
static int bf16_dbg() {
  static int v = [] {
    return ERTD_KNOB("BF16_DBG", 0);
  }();
  return v;
}
#endif

template <int KS, int MODE, int ACT, int WO, int TPX, bool PRE = false, int SP = 1>
static hipError_t launch_hg(const ConvArgs& a, int B, hipStream_t s) {
#ifdef ERTD_DIAG
  if constexpr (KS == 3 && PRE && WO == 64 && TPX == 2 && SP == 1) {
    switch (bf16_dbg()) {
      case 1: return launch_hgd<KS, MODE, ACT, WO, TPX, PRE, 1>(a, B, s);
      case 2: return launch_hgd<KS, MODE, ACT, WO, TPX, PRE, 2>(a, B, s);
      case 3: return launch_hgd<KS, MODE, ACT, WO, TPX, PRE, 3>(a, B, s);
      case 4: return launch_hgd<KS, MODE, ACT, WO, TPX, PRE, 4>(a, B, s);
      case 8: return launch_hgd<KS, MODE, ACT, WO, TPX, PRE, 8>(a, B, s);
      case 12: return launch_hgd<KS, MODE, ACT, WO, TPX, PRE, 12>(a, B, s);
      case 15: return launch_hgd<KS, MODE, ACT, WO, TPX, PRE, 15>(a, B, s);
      default: break;
    }
  }
#endif
  return launch_hgd<KS, MODE, ACT, WO, TPX, PRE, 0, SP>(a, B, s);
}

// ERTD_UNET_BF16_PRE=0 keeps the register staging for stride-1 convs (diagnostics)
static int convh_pre() {
  static int v = [] {
    return ERTD_KNOB("UNET_BF16_PRE", 1);
  }();
  return v;
}

// ERTD_UNET_BF16_TPX=1 / 2 forces 128- / 256-pixel tiles for the 3x3
// stride-1/upsample convs (diagnostics); 0 = automatic (512 at W = 32, 64)
static int convh_tpx_override() {
  static int v = [] {
    return ERTD_KNOB("UNET_BF16_TPX", 0);
  }();
  return v;
}

template <int KS, int TP, int SP>
static hipError_t launch_pre_w(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 16: return launch_hg<KS, MODE_S1, ACT_NONE, 16, TP, true, SP>(a, B, s);
    case 32: return launch_hg<KS, MODE_S1, ACT_NONE, 32, TP, true, SP>(a, B, s);
    case 64: return launch_hg<KS, MODE_S1, ACT_NONE, 64, TP, true, SP>(a, B, s);
    case 128: return launch_hg<KS, MODE_S1, ACT_NONE, 128, TP, true, SP>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}

// TPX = 4 (512-pixel tiles, 64 co x 128 px per wave: 6 LDS operand reads per
// 8 MFMAs instead of 4 per 4) where two workgroups still fit a CU (W = 32, 64);
// split bf16 (twice the LDS) fits one
template <int KS, int SP>
static hipError_t launch_pre_w4(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 32: return launch_hg<KS, MODE_S1, ACT_NONE, 32, 4, true, SP>(a, B, s);
    case 64: return launch_hg<KS, MODE_S1, ACT_NONE, 64, 4, true, SP>(a, B, s);
    default: return launch_pre_w<KS, 2, SP>(a, B, s);
  }
}

template <int SP>
static hipError_t launch_act_img(const ConvArgs& a, int act, bool up, int B, hipStream_t s) {
  const int HW = a.Wo * a.Wo, G16 = (a.Cin + 15) / 16;
  if ((HW / (up ? 4 : ACT_PXG)) % 64) return hipErrorInvalidValue;   // a wave = one (sample, group)
  const long long n = (long long)B * G16 * HW;
  const unsigned blocks = (unsigned)((n / ACT_PXG + 255) / 256);
  const unsigned blocks4 = (unsigned)((n / 4 + 255) / 256);   // the UPS kernel: 4 pixels per thread
  if (up) act_bf16_kernel<ACT_NONE, true, SP><<<blocks4, 256, 0, s>>>(a, B, G16, HW);
  else if (act == ACT_GN_SILU) act_bf16_kernel<ACT_GN_SILU, false, SP><<<blocks, 256, 0, s>>>(a, B, G16, HW);
  else if (act == ACT_GN) act_bf16_kernel<ACT_GN, false, SP><<<blocks, 256, 0, s>>>(a, B, G16, HW);
  else act_bf16_kernel<ACT_NONE, false, SP><<<blocks, 256, 0, s>>>(a, B, G16, HW);
  return hipGetLastError();
}

// stride-1 (or upsample) conv through the pre-transformed image: transform,
// then the conv as stride 1 on the image
template <int SP>
static hipError_t launch_conv_pre(int ks, int mode, int act, const ConvArgs& a, int B,
                                  hipStream_t s) {
  if (!a.bimg_ready) {   // else: image already written by gn_act_bf16_kernel
    const hipError_t e = launch_act_img<SP>(a, act, mode == MODE_UP, B, s);
    if (e != hipSuccess) return e;
  }
  ConvArgs c = a;
  c.Hs = c.Ws = a.Wo;   // the image is at the output resolution
  if (ks == 1) return launch_pre_w<1, 1, SP>(c, B, s);
  if (convh_tpx_override() == 1) return launch_pre_w<3, 1, SP>(c, B, s);
  if (convh_tpx_override() == 2) return launch_pre_w<3, 2, SP>(c, B, s);
  return launch_pre_w4<3, SP>(c, B, s);   // U3 B=256: 101.5 -> 103.1 steps/s over TPX = 2
}

template <int KS, int MODE, int ACT, int TP, int SP>
static hipError_t launch_hwt(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 16: return launch_hg<KS, MODE, ACT, 16, TP, false, SP>(a, B, s);
    case 32: return launch_hg<KS, MODE, ACT, 32, TP, false, SP>(a, B, s);
    case 64: return launch_hg<KS, MODE, ACT, 64, TP, false, SP>(a, B, s);
    case 128:
      if constexpr (MODE != MODE_S2) return launch_hg<KS, MODE, ACT, 128, TP, false, SP>(a, B, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

template <int KS, int MODE, int ACT, int SP>
static hipError_t launch_hw(const ConvArgs& a, int B, hipStream_t s) {
  // TPX = 2 (256-pixel tiles) except stride 2 / 1x1 (staging registers)
  if constexpr (KS == 1) {
    // ERTD_UNET_BF16_TPX1=2: 256-pixel tiles for the 1x1 convs (A/B)
    static const int t1 = [] {
      return ERTD_KNOB("UNET_BF16_TPX1", 1);
    }();
    if (t1 == 2) return launch_hwt<KS, MODE, ACT, 2, SP>(a, B, s);
    return launch_hwt<KS, MODE, ACT, 1, SP>(a, B, s);
  } else if constexpr (MODE == MODE_S2) {
    return launch_hwt<KS, MODE, ACT, 1, SP>(a, B, s);
  } else {
    if (convh_tpx_override() == 1) return launch_hwt<KS, MODE, ACT, 1, SP>(a, B, s);
    return launch_hwt<KS, MODE, ACT, 2, SP>(a, B, s);
  }
}

// the standalone image transform (act(GN(x)) or the nearest-x2 upsample of x
// -> the [B][C/16][H][W][16] bf16 image): ertd_act_bf16 (bench per-kernel GB/s)
hipError_t launch_act_bf16(const ConvArgs& a, int act, bool up, int B, hipStream_t s) {
  return a.split ? launch_act_img<2>(a, act, up, B, s) : launch_act_img<1>(a, act, up, B, s);
}

template <int SP>
static hipError_t launch_conv_h(int ks, int mode, int act, const ConvArgs& a, int B, hipStream_t s) {
  // the pre-transform pays where the staging VALU is heaviest: 3x3 convs with
  // a GroupNorm(+SiLU) prologue and the Upsample convs (measured on U3 B=256:
  // the extra read+write pass costs more than it saves for 1x1 convs)
  if (a.bimg && convh_pre() == 1 && ks == 3 &&
      ((mode == MODE_S1 && act != ACT_NONE) || (mode == MODE_UP && act == ACT_NONE)))
    return launch_conv_pre<SP>(ks, mode, act, a, B, s);
  if (ks == 3 && mode == MODE_S1 && act == ACT_NONE) return launch_hw<3, MODE_S1, ACT_NONE, SP>(a, B, s);
  if (ks == 3 && mode == MODE_S1 && act == ACT_GN_SILU) return launch_hw<3, MODE_S1, ACT_GN_SILU, SP>(a, B, s);
  if (ks == 3 && mode == MODE_S2 && act == ACT_NONE) return launch_hw<3, MODE_S2, ACT_NONE, SP>(a, B, s);
  if (ks == 3 && mode == MODE_UP && act == ACT_NONE) return launch_hw<3, MODE_UP, ACT_NONE, SP>(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_NONE) return launch_hw<1, MODE_S1, ACT_NONE, SP>(a, B, s);
  if (ks == 1 && mode == MODE_S1 && act == ACT_GN) return launch_hw<1, MODE_S1, ACT_GN, SP>(a, B, s);
  return hipErrorInvalidValue;
}

// parts per (sample, channel) of the GroupNorm partials the dispatched bf16
// conv emits (the pre-transformed-image 3x3 / Upsample convs: 256- and
// 512-px output tiles; parts of 64 px), 0 = none
int conv_bf16_gn_parts(int ks, int mode, int act, const ConvArgs& a, int B) {
  (void)B;
  if (a.Cout == 1 || ks != 3 || a.Ho != a.Wo || (a.Wo * a.Wo) % 256) return 0;
  const bool pre = convh_pre() == 1 && ((mode == MODE_S1 && act != ACT_NONE) || (mode == MODE_UP && act == ACT_NONE));
  if (!pre || convh_tpx_override() == 1) return 0;
  return a.Wo * a.Wo / 64;
}

hipError_t launch_conv_bf16(int ks, int mode, int act, const ConvArgs& a, int B, hipStream_t s) {
  if (a.fold.cnt || a.gnc.pa) return hipErrorInvalidValue;   // the fold rides on the fp32 Winograd kernels only
  if (a.Ho != a.Wo || a.Hs != a.Ws || a.Cin != a.Ca + a.Cb) return hipErrorInvalidValue;
  if (a.gnp && (!a.bimg || conv_bf16_gn_parts(ks, mode, act, a, B) == 0)) return hipErrorInvalidValue;
  const int expect = mode == MODE_S2 ? a.Ws / 2 : (mode == MODE_UP ? a.Ws * 2 : a.Ws);
  if (a.Wo != expect) return hipErrorInvalidValue;
  // conv_in / conv_out are fp32-VALU kernels: bf16 rounds their operands,
  // split bf16 reads hi + lo weights and keeps the activation fp32
  const int pk = a.split ? 2 : 1;
  if (a.Cout == 1 && ks == 3 && mode == MODE_S1 && act != ACT_GN) return launch_conv_out(act, a, B, pk, s);
  if (conv_in_ok(a, ks, mode, act)) return launch_conv_in(a, B, pk, s);
  return a.split ? launch_conv_h<2>(ks, mode, act, a, B, s) : launch_conv_h<1>(ks, mode, act, a, B, s);
}

// ---- bf16 weight packing: W (Cout, Cin, ks, ks) fp32 -> [co_tile32][chunk][step][lane][8] bf16
// (split: [co_tile32][chunk][hi | lo][step][lane][8])
size_t conv_packed_floats_bf16(int cin, int cout, int ks, bool split) {
  const int ck = convh_ck(ks);
  const size_t tiles = (size_t)((cout + 127) / 128) * 4;
  const size_t nchunk = (size_t)((cin + ck - 1) / ck);
  const size_t steps = (size_t)ks * ks * (ck / 16);
  return tiles * nchunk * steps * 64 * 8 / 2 * (split ? 2 : 1);   // 8 bf16 per lane = 4 floats
}

__global__ void pack_conv_bf16_kernel(const float* __restrict__ w, int cin, int cout, int ks,
                                      int nchunk, int planes, size_t total,
                                      unsigned short* __restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // bf16 element
  if (i >= total) return;
  const int ck = convh_ck(ks), taps = ks * ks, spc = taps * (ck / 16);
  const int j = (int)(i & 7);
  const int lane = (int)((i >> 3) & 63);
  size_t rest = i >> 9;
  const int s = (int)(rest % spc);
  rest /= spc;
  const int hl = (int)(rest % planes);
  rest /= planes;
  const int k = (int)(rest % nchunk);
  const int tile = (int)(rest / nchunk);
  const int g = s / taps, tap = s % taps;
  const int co = tile * 32 + (lane & 31);
  const int ci = k * ck + g * 16 + 8 * (lane >> 5) + j;
  float v = 0.f;
  if (co < cout && ci < cin) v = w[((size_t)co * cin + ci) * taps + tap];
  const uint32_t u = __float_as_uint(v);
  const uint32_t hi = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
  if (hl == 0) {
    dst[i] = (unsigned short)hi;
  } else {
    const uint32_t r = __float_as_uint(v - __uint_as_float(hi << 16));
    dst[i] = (unsigned short)((r + 0x7FFFu + ((r >> 16) & 1u)) >> 16);
  }
}

hipError_t launch_pack_conv_bf16(const float* w, int cin, int cout, int ks, float* dst,
                                 hipStream_t s, bool split) {
  const size_t total = conv_packed_floats_bf16(cin, cout, ks, split) * 2;
  const int nchunk = (cin + convh_ck(ks) - 1) / convh_ck(ks);
  pack_conv_bf16_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(
      w, cin, cout, ks, nchunk, split ? 2 : 1, total, reinterpret_cast<unsigned short*>(dst));
  return hipGetLastError();
}

}  // namespace unet
}  // namespace ertd
