// 3x3 stride-1 convolution of the U-Net ResBlocks by Winograd F(2x2, 3x3) on
// fp32 MFMA (v_mfma_f32_32x32x2_f32), GroupNorm + SiLU fused into the input
// transform, bias / embedding / residual into the output transform.
//
// Per 2x2 output tile and input channel c (d = the 4x4 input window at
// rows 2ty-1.., cols 2tx-1.., zero outside the image, AFTER the activation):
//   V = B^T d B        B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
//   U = G g G^T        G   = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1]
//   M[xi] = sum_c U[xi][co][c] V[xi][c][tile]          (16 GEMMs, xi = 4i + j)
//   Y = A^T M A        A^T = [1 1 1 0; 0 1 -1 -1]
// 16 multiplies per 4 outputs instead of 36: 2.25x less MFMA work than the
// direct implicit GEMM (unet_conv.hip), all of it fp32 (products exact, sums
// rounded in fp32; the transforms add a few roundings per value -- the
// forward stays within 1e-5 of the spec, tests/test_gpu_unet*.py).
//
// Work item = (64 output channels, 64 tiles = 256 output pixels, sample), all
// 16 xi, K walked in chunks of 8 input channels.  The kernel is PERSISTENT:
// one 768-thread workgroup per CU walks items bid, bid + grid, ... as one
// continuous chunk pipeline, so the next item's first chunks are staged
// while the current one finishes and its epilogue (stores) overlaps the
// next item's loads.  12 waves with fixed roles:
//   * 8 MFMA waves on v_mfma_f32_16x16x4_f32: wave w = (16-co block w & 3,
//     32-tile pair w >> 2) keeps ALL 16 xi of its 16 co x 32 tiles (2 x 16
//     accumulators of 4 VGPRs = 128), so the output transform needs no data
//     of any other wave; inside the K loop it only reads LDS (per xi: one
//     ds_read_b64 of U, two of V, 4 MFMAs);
//     They also LDS-DMA the weights U (pre-transformed at pack time in
//     fragment order: [xi 16][co block 4][k 4][co 16][k-step 2] = 32 KB per
//     chunk) two chunks ahead into a 3-slot ring;
//   * 4 producer waves: the input transform -- lane = tile, wave q owns the
//     channel pair (2q, 2q+1) = (k-step 0, k-step 1) of MFMA row k = q: the
//     two middle columns of the tile's 4x4 window are loaded four chunks
//     ahead into three register sets (one float2 per row, with the channels'
//     GroupNorm scale/shift), GroupNorm+SiLU applied, the outer columns taken
//     from the neighbouring lanes (DPP wave shifts), transformed -- both
//     channels at once in packed fp32 (v_pk_*) -- and written as
//     V [xi][tile block 4][k 4][tile 16][k-step 2] (32 KB, double-buffered):
//     one ds_write_b64 per xi, and one ds_read_b64 per xi and operand on the
//     MFMA side feeds both k-steps.
//   With 3 waves per SIMD (2 MFMA + 1 producer) the hardware interleaves the
//   producer's VALU / memory work with the MFMA waves' matrix-pipe time; one
//   barrier per chunk.
//   * Output transform (MFMA waves, in registers, right after an item's last
//     chunk): Y = A^T M A per (co, tile), + bias (+ emb) (+ residual), two
//     float2 stores per (co, tile); the next item's chunks are already staged.
// LDS 160 KB: one workgroup per CU.
#include <cstdlib>

#include "unet.h"
#include "unet_pack.h"

namespace ertd {
namespace unet {

namespace {

constexpr int NMW = 8;                        // MFMA waves
constexpr int NPW = 4;                        // producer waves
constexpr int WT = 64 * (NMW + NPW);          // threads per workgroup (768)
constexpr int WKC = 8;                        // input channels per K chunk
constexpr int WSP = WKC / 4;                  // MFMA step pairs per chunk
constexpr int U_FL = 16 * 2 * WSP * 128;      // U floats per chunk buffer (8192)
constexpr int V_FL = 16 * WSP * 2 * 128;      // V floats per chunk buffer (8192)
constexpr int NUB = 3;                        // U ring depth (DMA two chunks ahead)
constexpr int NRS = 3;                        // producer register sets (loads NRS+1 chunks ahead)
constexpr size_t WLDS = (size_t)(NUB * U_FL + 2 * V_FL) * sizeof(float);   // 160 KB
constexpr int XIF = WKC * 64;                 // U / V floats per xi (512)
#ifndef WINO_PPRIO
#define WINO_PPRIO 2                          // producer wave priority (s_setprio)
#endif
#ifndef WINO_PD
#define WINO_PD 2                             // MFMA operand read-ahead (xi)
#endif
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;

__device__ __forceinline__ unsigned wlds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

int wino_env() {
  static int v = [] {
    return ERTD_KNOB("UNET_WINO", 1);
  }();
  return v;
}

// item it -> (co block, tile block, sample): co block fastest, so the
// workgroups running at one time share few weight slices
struct Item {
  int cog, tblk, b;
};
__device__ __forceinline__ Item item_of(int it, int ncog, int ntblk) {
  Item r;
  r.cog = it % ncog;
  const int t = it / ncog;
  r.tblk = t % ntblk;
  r.b = t / ntblk;
  return r;
}

// DBG (diagnostics only, ERTD_WINO_DBG): bit 0 skips the activation VALU,
// bit 1 the input loads, bit 2 the weight DMA, bit 3 the MFMAs, bit 4 the
// producers' transform, bit 5 the MFMA waves' LDS reads, bit 6 the output
// transform and stores (all but one value per lane) -- the results are
// wrong, the timings show where a chunk's time goes
template <int WO, int ACT, int DBG = 0>
__global__ __launch_bounds__(WT) void conv_wino_kernel(ConvArgs a, int nitems, int ksp) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* ubuf = smem;                 // [3][U_FL] ring
  float* vbuf = smem + NUB * U_FL;    // [2][V_FL]

  constexpr int TPR = WO / 2;         // tiles per tile row
  constexpr int HW = WO * WO;
  constexpr int NTBLK = TPR * TPR / 64;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, l32 = lane & 31;
  const int Cin = a.Cin, Ca = a.Ca;
  const int nchunk = Cin / WKC;
  // ksp = 2 (K split, few items): work item it = 2 x (tile item) + half; half h
  // accumulates channel chunks [h nck, (h+1) nck) and writes its partial sum
  // to a.out (h = 0, with bias / emb / residual) or a.ksplit_buf (h = 1); the
  // launcher adds the two afterwards
  const int nck = nchunk / ksp;                                      // chunks per work item
  const int ncog = a.Cout / 64;
  const int bid = blockIdx.x, G = gridDim.x;
  const int nloc = bid < nitems ? (nitems - bid + G - 1) / G : 0;   // items of this workgroup
  const int gtot = nloc * nck;                                       // chunks of this workgroup

  if (wave >= NMW) {
    // =================== producer waves ===================
    // the producers issue ahead of the MFMA waves on a shared SIMD (as in the
    // F(4x4) kernel; U2 B=64 190.0 -> 191.6 steps/s)
    __builtin_amdgcn_s_setprio(WINO_PPRIO);
    const int q = wave - NMW;          // channels 2q (k-step 0), 2q+1 (k-step 1) of every chunk
    // V offset of (channel pair q, tile t = lane): [xi][t >> 4][q][t & 15][k-step]
    const int vwoff = (lane >> 4) * 128 + q * 32 + (lane & 15) * 2;
    // registers of the chunk in flight: the two middle columns of the 4x4
    // window (one float2 per row) of both channels, their GroupNorm
    // {scale, shift}, and the window's padding as 0 / 1 factors.  Each lane
    // loads its tile's middle columns; the outer columns are the neighbouring
    // tiles' (lanes t-1 / t+1) by DPP wave shifts -- across a tile-row
    // boundary they are padding (masked), so the shifted-in neighbour never
    // matters there.  Only rows 0 / 3 of a window can fall outside the image.
    float2 raw[NRS][2][4];   // [register set][channel][row]
    f32x4 gnv[NRS];          // {scale, shift} of channel 2q, then 2q+1
    f32x4 pad[NRS];          // row 0, row 3, left column, right column
    // the loads walk this workgroup's chunks in order (a cursor; the item's
    // geometry is derived once per item, not per chunk)
    int cur_g = 0, cur_k = 0, cur_k0 = 0, cur_b = 0, cur_il = 0;
    unsigned roff[4];        // byte offsets of the window's rows (global_load saddr + voffset)
    f32x4 cur_pad;
    auto set_item = [&](int il) {
      const int it = bid + il * G;
      cur_k0 = (it % ksp) * nck;
      const Item itm = item_of(it / ksp, ncog, NTBLK);
      cur_b = itm.b;
      const int tg = itm.tblk * 64 + lane;
      const int ty = tg / TPR, tx = tg - ty * TPR;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int iy = 2 * ty - 1 + r;
        roff[r] = (unsigned)(((iy >= 0 && iy < WO ? iy : 2 * ty) * WO + 2 * tx) * 4);
      }
      cur_pad = f32x4{ty > 0 ? 1.f : 0.f, ty < TPR - 1 ? 1.f : 0.f, tx > 0 ? 1.f : 0.f,
                      tx < TPR - 1 ? 1.f : 0.f};
    };
    const int glast = gtot - 1;
    // load the cursor's chunk into a register set and advance (past the last
    // chunk it stays put: the extra loads re-load the last chunk, unused, so
    // the steady-state loop has no conditional loads)
    auto load_next = [&](const int set) {
      const int cg = (cur_k0 + cur_k) * WKC + 2 * q;    // wave-uniform, channels cg, cg + 1
      pad[set] = cur_pad;
      if constexpr (ACT != ACT_NONE) gnv[set] = *reinterpret_cast<const f32x4*>(a.gn + (size_t)cur_b * Cin + cg);
      if constexpr (DBG & 2) {
#pragma unroll
        for (int hv = 0; hv < 2; ++hv)
#pragma unroll
          for (int r = 0; r < 4; ++r) raw[set][hv][r] = make_float2((float)(r + cur_k), (float)hv);
      } else {
        const float* p = cg < Ca ? a.srcA + ((size_t)cur_b * Ca + cg) * HW
                                 : a.srcB + ((size_t)cur_b * a.Cb + (cg - Ca)) * HW;
        // buffer loads: the channel pair's base in SGPRs, the row offset in one VGPR
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 2 * HW * 4, 0x00020000);
#pragma unroll
        for (int hv = 0; hv < 2; ++hv)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)roff[r], hv * HW * 4, 0);
            raw[set][hv][r] = make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
          }
      }
      if (cur_g < glast) {
        ++cur_g;
        if (++cur_k == nck) {
          cur_k = 0;
          set_item(++cur_il);
        }
      }
    };
    // both channels of the pair in the two halves of every f32x2: the
    // arithmetic is the same per channel, so it issues as packed fp32
    auto transform_chunk = [&](const int set, float* vb) {
      if constexpr (DBG & 16) return;
      const f32x2 gs = {gnv[set].x, gnv[set].z}, gh = {gnv[set].y, gnv[set].w};
      const float fl = pad[set].z, fr = pad[set].w;
      f32x2 d[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        f32x2 m0 = {raw[set][0][r].x, raw[set][1][r].x};
        f32x2 m1 = {raw[set][0][r].y, raw[set][1][r].y};
        if constexpr (ACT != ACT_NONE && !(DBG & 1)) {
          m0 = __builtin_elementwise_fma(m0, gs, gh);   // ATen's folded GroupNorm
          m1 = __builtin_elementwise_fma(m1, gs, gh);
          if constexpr (ACT == ACT_GN_SILU) {
            f32x2 e0 = {__expf(-m0.x), __expf(-m0.y)}, e1 = {__expf(-m1.x), __expf(-m1.y)};
            e0 = 1.0f + e0;
            e1 = 1.0f + e1;
            m0 = m0 * f32x2{__builtin_amdgcn_rcpf(e0.x), __builtin_amdgcn_rcpf(e0.y)};
            m1 = m1 * f32x2{__builtin_amdgcn_rcpf(e1.x), __builtin_amdgcn_rcpf(e1.y)};
          }
        }
        // the padding pads the activated tensor: rows outside the image and
        // the outer columns at the image's left / right edge are zero
        if (r == 0 || r == 3) {
          const float fy = r == 0 ? pad[set].x : pad[set].y;
          m0 = m0 * fy;
          m1 = m1 * fy;
        }
        // left neighbour's column 2tx-1 (lane t-1's m1), right's 2tx+2 (lane t+1's m0)
        f32x2 lf, rt;
        lf.x = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m1.x), 0x138, 0xf, 0xf, true));
        lf.y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m1.y), 0x138, 0xf, 0xf, true));
        rt.x = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m0.x), 0x130, 0xf, 0xf, true));
        rt.y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m0.y), 0x130, 0xf, 0xf, true));
        d[r][0] = lf * fl;
        d[r][1] = m0;
        d[r][2] = m1;
        d[r][3] = rt * fr;
      }
      f32x2 tm[4][4];   // B^T d
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        tm[0][s] = d[0][s] - d[2][s];
        tm[1][s] = d[1][s] + d[2][s];
        tm[2][s] = d[2][s] - d[1][s];
        tm[3][s] = d[1][s] - d[3][s];
      }
      float* o = vb + vwoff;
#pragma unroll
      for (int i = 0; i < 4; ++i) {   // (B^T d) B
        *reinterpret_cast<f32x2*>(o + (4 * i + 0) * XIF) = tm[i][0] - tm[i][2];
        *reinterpret_cast<f32x2*>(o + (4 * i + 1) * XIF) = tm[i][1] + tm[i][2];
        *reinterpret_cast<f32x2*>(o + (4 * i + 2) * XIF) = tm[i][2] - tm[i][1];
        *reinterpret_cast<f32x2*>(o + (4 * i + 3) * XIF) = tm[i][1] - tm[i][3];
      }
    };

    // NRS = 3 register sets (chunk c in set c % 3), loads four chunks ahead
    // of the MFMAs: in the slot of chunk g the producers transform chunk g+1
    // (loaded three slots earlier -- the compiler's own vmcnt waits, which
    // count only these loads) into V[(g+1) & 1] and issue chunk g+4's loads
    // into the set just freed.  (With two sets, loads three chunks ahead, the
    // producers waited on their loads: the layer ran as long as the producers
    // alone.)  Loads past the last chunk re-load the last one (clamped,
    // unused): the steady-state loop has no conditional loads, and the
    // compiler's vmcnt bookkeeping across its back edge stays exact.
    auto slot = [&](const int set, int g) {   // set = (g + 1) % NRS
      transform_chunk(set, vbuf + ((g + 1) & 1) * V_FL);
      load_next(set);    // chunk g + 1 + NRS
      __syncthreads();   // (B) end of slot g
    };
    if (gtot > 0) {
      set_item(0);
      load_next(0);
      load_next(1);
      load_next(2);
      transform_chunk(0, vbuf);
      load_next(0);
    }
    __syncthreads();   // (A) chunk 0 staged
    int g = 0;
    for (; g + 2 < gtot; g += 3) {
      slot(1, g);
      slot(2, g + 1);
      slot(0, g + 2);
    }
    if (g < gtot) slot(1, g);
    if (g + 1 < gtot) slot(2, g + 1);
    return;
  }

  // =================== MFMA waves ===================
#ifdef WINO_PRIO
  __builtin_amdgcn_s_setprio(WINO_PRIO);   // issue ahead of the producer on a shared SIMD
#endif
  const int cb = wave & 3, tbp = wave >> 2;
  // operands: U at cb*64 + lane, V at (2 tbp)*64 + lane (+64: second tile
  // block), + xi*XIF + s*256 (derived per chunk in the K loop)
  f32x4 acc[16][2];

  // U slice DMA of chunk g into ring slot g % 3, issued two slots ahead by the
  // MFMA waves themselves (4 x 1 KB per wave): they issue no other vector
  // memory operation in the K loop, so "all but this slot's 4 DMAs done"
  // (vmcnt(4)) is exactly "chunk g+1's slice has landed"
  auto dma_u = [&](int g) {
    if constexpr (DBG & 4) return;
    const int il = g / nck, it = bid + il * G;
    const int k = (it % ksp) * nck + (g - il * nck);
    const int cog = (it / ksp) % ncog;
    const float* usrc = a.wpk_wino + ((size_t)cog * nchunk + k) * U_FL;
    float* dst = ubuf + (g % NUB) * U_FL;
#pragma unroll
    for (int j = 0; j < U_FL / (NMW * 256); ++j) {
      const int ins = wave * (U_FL / (NMW * 256)) + j;   // wave-uniform, 1 KB each
      const float* src = usrc + ins * 256 + lane * 4;
      const unsigned ldst = __builtin_amdgcn_readfirstlane(wlds_addr(dst + ins * 256));
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(src), "s"(ldst)
          : "memory");
    }
  };
  static_assert(U_FL / (NMW * 256) == 4, "vmcnt(4) below counts the DMAs of one slot");
  if (gtot > 0) dma_u(0);
  if (gtot > 1) dma_u(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // (A)
  for (int il = 0; il < nloc; ++il) {
#pragma unroll
    for (int x = 0; x < 16; ++x) acc[x][0] = acc[x][1] = f32x4{};
    for (int k = 0; k < nck; ++k) {
      const int g = il * nck + k;
      const bool dma = g + 2 < gtot;
      if (dma) dma_u(g + 2);
      // the lane-dependent operand offsets are re-derived per chunk from a
      // fresh lane id (opaque to the compiler): held across the loop they
      // were spilled to scratch, and the reload's vmcnt(0) waited for the
      // U DMA just issued for chunk g + 2 -- every chunk
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      const float* ub = ubuf + (g % NUB) * U_FL + cb * 128 + 2 * ln;
      const float* vb = vbuf + (g & 1) * V_FL + (2 * tbp) * 128 + 2 * ln;
      // 16 xi: one ds_read_b64 per operand gives both k-steps (4 MFMAs per
      // xi); operands read PD xi ahead into a register ring, each xi's three
      // ds_reads grouped with the MFMAs of an earlier xi (the compiler
      // otherwise spends the few free registers on A operands and waits a
      // full LDS latency before every MFMA group)
      constexpr int PD = WINO_PD;
      f32x2 ra[PD + 1], rb0[PD + 1], rb1[PD + 1];
      auto ld = [&](const int x) {
        const int r = x % (PD + 1);
        if constexpr (DBG & 32) {
          ra[r] = f32x2{(float)(lane + x), (float)(lane - x)};
          rb0[r] = f32x2{(float)(lane - x + k), (float)x};
          rb1[r] = rb0[r] + 1.f;
        } else {
          ra[r] = *reinterpret_cast<const f32x2*>(ub + x * XIF);
          rb0[r] = *reinterpret_cast<const f32x2*>(vb + x * XIF);
          rb1[r] = *reinterpret_cast<const f32x2*>(vb + x * XIF + 128);
        }
      };
#pragma unroll
      for (int x = 0; x < PD; ++x) ld(x);
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        if (x + PD < 16) ld(x + PD);
        const int r = x % (PD + 1);
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          if constexpr (DBG & 8) {
            acc[x][0][0] += ra[r][st] * rb0[r][st];
            acc[x][1][0] += ra[r][st] * rb1[r][st];
          } else {
            acc[x][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[r][st], rb0[r][st], acc[x][0], 0, 0, 0);
            acc[x][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[r][st], rb1[r][st], acc[x][1], 0, 0, 0);
          }
        }
        if (x + PD < 16) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);   // DS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                     // MFMAs
      }
      // keep the chunk's MFMAs ahead of the barrier (hipcc would sink them:
      // they touch no memory)
#pragma unroll
      for (int x = 0; x < 16; ++x) asm volatile("" : "+v"(acc[x][0]), "+v"(acc[x][1]));
      if (dma) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();   // (B)
    }

    // ---- output transform of this wave's 16 co x 32 tiles, in registers:
    // lane l holds M[xi] of co = 16 cb + 4 (l >> 4) + i (acc element i) and
    // tile 16 j + (l & 15) of its tile pair (accumulator j)
    if constexpr (DBG & 64) {   // no output transform / stores
      if (il == nloc - 1)
        for (int x = 0; x < 16; ++x) a.out[(size_t)bid * 64 + lane] += acc[x][0][0] + acc[x][1][1];
      continue;
    }
    const int itg = bid + il * G;
    const Item itm = item_of(itg / ksp, ncog, NTBLK);
    const bool part2 = (itg % ksp) != 0;   // second K half: raw partial sum only
    // wave-uniform flags (a per-lane null test on a derived pointer made the
    // compiler mask every load)
    const bool has_eb = a.ebias && !part2, has_res = a.res && !part2, has_bias = a.bias && !part2;
    // buffer loads / stores: the sample's base in SGPRs, one 32-bit offset
    // per tile block (64-bit addresses per store spilled)
    const unsigned smp = (unsigned)(a.Cout * HW * 4);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (part2 ? a.ksplit_buf : a.out) + (size_t)itm.b * a.Cout * HW, (short)0, smp, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        has_res ? const_cast<float*>(a.res) + (size_t)itm.b * a.Cout * HW : nullptr, (short)0, smp, 0x00020000);
    // a fresh lane id (as in the K loop): lane-derived values held across the
    // loop were spilled, and each reload's vmcnt(0) waited for this item's
    // stores
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    const int co0 = itm.cog * 64 + cb * 16 + 4 * (ln >> 4);
    int vo[2];   // byte offset of (co0, the tile's top-left pixel)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tg = itm.tblk * 64 + (2 * tbp + j) * 16 + (ln & 15);
      const int ty = tg / TPR, tx = tg - ty * TPR;
      vo[j] = (co0 * HW + 2 * ty * WO + 2 * tx) * 4;
    }
    float bias[4], eb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bias[i] = has_bias ? a.bias[co0 + i] : 0.f;
      eb[i] = has_eb ? a.ebias[(size_t)itm.b * a.eb_stride + co0 + i] : 0.f;
    }
    // Y = A^T (M A) of tile block j, then the spec's op order: conv + bias,
    // + emb (the residual is added by the caller)
    auto out_tile = [&](const int j, f32x2 (&y)[4][2]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float Pm[4][2];   // P = M A, per row of M
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float m0 = acc[4 * r + 0][j][i], m1 = acc[4 * r + 1][j][i];
          const float m2 = acc[4 * r + 2][j][i], m3 = acc[4 * r + 3][j][i];
          Pm[r][0] = (m0 + m1) + m2;
          Pm[r][1] = (m1 - m2) - m3;
        }
        y[i][0] = f32x2{(Pm[0][0] + Pm[1][0]) + Pm[2][0], (Pm[0][1] + Pm[1][1]) + Pm[2][1]} + bias[i];
        y[i][1] = f32x2{(Pm[1][0] - Pm[2][0]) - Pm[3][0], (Pm[1][1] - Pm[2][1]) - Pm[3][1]} + bias[i];
        if (has_eb) {
          y[i][0] = y[i][0] + eb[i];
          y[i][1] = y[i][1] + eb[i];
        }
      }
    };
    auto store_tile = [&](const int j, const f32x2 (&y)[4][2]) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 2; ++r)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, y[i][r]),
                                                ro, vo[j] + r * WO * 4, i * HW * 4, 0);
    };
    // all outputs first (frees the accumulators), then the residual of both
    // tile blocks into the freed registers, then the stores: no load is
    // issued after a store (loads and stores share vmcnt, so it would wait
    // for the store)
    f32x2 y[2][4][2];
    out_tile(0, y[0]);
    out_tile(1, y[1]);
    __builtin_amdgcn_sched_barrier(0);
    if (has_res) {
      f32x2 rv[2][4][2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 2; ++r)
            rv[j][i][r] = __builtin_bit_cast(
                f32x2, __builtin_amdgcn_raw_buffer_load_b64(rr, vo[j] + r * WO * 4, i * HW * 4, 0));
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 2; ++r) y[j][i][r] = y[j][i][r] + rv[j][i][r];
    }
    store_tile(0, y[0]);
    store_tile(1, y[1]);
    // GroupNorm partials of the stored output: the 16 lanes of a DPP row hold
    // 2 x 16 tiles x 4 px = 128 pixels of sample itm.b for the same 4 channels
    if (a.gnp && ksp == 1) {
      float2 pr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float sm = ((y[0][i][0][0] + y[0][i][0][1]) + (y[0][i][1][0] + y[0][i][1][1])) +
                   ((y[1][i][0][0] + y[1][i][0][1]) + (y[1][i][1][0] + y[1][i][1][1]));
        sm = row16_sum(sm);
        const float mu = sm * (1.0f / 128.0f);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int x = 0; x < 2; ++x) {
              const float d = y[j][i][r][x] - mu;
              q = __builtin_fmaf(d, d, q);
            }
        pr[i] = make_float2(sm, row16_sum(q));
      }
      if ((ln & 15) == 0) {
        constexpr int np = TPR * TPR / 32;
        const int part = 2 * itm.tblk + tbp;
#pragma unroll
        for (int i = 0; i < 4; ++i) a.gnp[((size_t)itm.b * a.Cout + co0 + i) * np + part] = pr[i];
      }
    }
  }
}

#ifdef ERTD_DIAG
// ablation variants (results wrong): only in a diagnostic build of the library
// (tools/build_variant.sh ... "-DERTD_DIAG"), never in the shipped one
int wino_dbg() {
  static int v = [] {
    return ERTD_KNOB("WINO_DBG", 0);
  }();
  return v;
}
#endif

// out += part (float4): the K-split halves' fixed-order sum
__global__ void add_inplace_kernel(float* __restrict__ out, const float* __restrict__ part, size_t n4) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 o = reinterpret_cast<float4*>(out)[i];
  const float4 p = reinterpret_cast<const float4*>(part)[i];
  o.x = o.x + p.x; o.y = o.y + p.y; o.z = o.z + p.z; o.w = o.w + p.w;
  reinterpret_cast<float4*>(out)[i] = o;
}

// K split when a layer has fewer tile items than ERTD_WINO_KSPLIT x CUs (default 1)
int ksplit_items() {
  static int v = [] {
    return ERTD_KNOB("WINO_KSPLIT", 1);
  }();
  return v;
}

int cu_count() { return device_cu_count(); }

template <int WO, int ACT, int DBG>
hipError_t launch_wod(const ConvArgs& a, int B, hipStream_t s) {
  static std::atomic<unsigned long long> attr{0};
  set_max_lds_once((const void*)conv_wino_kernel<WO, ACT, DBG>, (int)WLDS, attr);
  const int base = (WO / 2) * (WO / 2) / 64 * (a.Cout / 64) * B;
  // fewer tile items than the split threshold (x CUs) -> K split in two halves
  const int nchunk = a.Cin / WKC;
  const int ksp = (a.ksplit_buf && nchunk % 2 == 0 && nchunk >= 4 &&
                   base < ksplit_items() * cu_count()) ? 2 : 1;
  const int nitems = base * ksp;
  const int grid = nitems < cu_count() ? nitems : cu_count();
  conv_wino_kernel<WO, ACT, DBG><<<grid, WT, WLDS, s>>>(a, nitems, ksp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || ksp == 1) return e;
  const size_t n = (size_t)B * a.Cout * WO * WO;
  return launch_add_inplace(a.out, a.ksplit_buf, n, s);
}

template <int WO, int ACT>
hipError_t launch_wo(const ConvArgs& a, int B, hipStream_t s) {
#ifdef ERTD_DIAG
  if constexpr (WO == 64 && ACT == ACT_GN_SILU) {
    switch (wino_dbg()) {
      case 1: return launch_wod<WO, ACT, 1>(a, B, s);
      case 2: return launch_wod<WO, ACT, 2>(a, B, s);
      case 4: return launch_wod<WO, ACT, 4>(a, B, s);
      case 8: return launch_wod<WO, ACT, 8>(a, B, s);
      case 7: return launch_wod<WO, ACT, 7>(a, B, s);
      case 16: return launch_wod<WO, ACT, 16>(a, B, s);
      case 32: return launch_wod<WO, ACT, 32>(a, B, s);
      case 64: return launch_wod<WO, ACT, 64>(a, B, s);
      case 23: return launch_wod<WO, ACT, 23>(a, B, s);
      case 55: return launch_wod<WO, ACT, 55>(a, B, s);
      default: break;
    }
  }
#endif
  return launch_wod<WO, ACT, 0>(a, B, s);
}

template <int ACT>
hipError_t launch_act(const ConvArgs& a, int B, hipStream_t s) {
  switch (a.Wo) {
    case 16: return launch_wo<16, ACT>(a, B, s);
    case 32: return launch_wo<32, ACT>(a, B, s);
    case 64: return launch_wo<64, ACT>(a, B, s);
    case 128: return launch_wo<128, ACT>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}

// ---- packing: W (Cout, Cin, 3, 3) -> U = G g G^T in [cog][chunk][xi][cb][kk][c16][st]
// (computed in float64, rounded once): the A-operand fragments of
// v_mfma_f32_16x16x4_f32 for co block cb (16 co), both k-steps st in one
// float2, lane l = 16 kk + c16 -> co = 16 cb + c16, channel 2 kk + st of the chunk
// one thread per (co, ci): all 16 xi (pack_wino_tile)
__global__ void pack_wino_kernel(const float* __restrict__ w, int cin, int cout, int nchunk,
                                 size_t items, float* __restrict__ dst, bool flipT) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= items) return;
  pack_wino_tile(w, cin, cout, nchunk, j, flipT, dst);
}

}  // namespace

hipError_t launch_add_inplace(float* out, const float* part, size_t n, hipStream_t s) {
  add_inplace_kernel<<<(unsigned)((n / 4 + 255) / 256), 256, 0, s>>>(out, part, n / 4);
  return hipGetLastError();
}

// W = 16 takes F(4x4) only when its tile items fill the CUs without a K split
// (U2 B=64: 128 items; split in two halves it measured no faster than F(2x2))
// ERTD_WINO4_W16=1: F(4x4) at 16x16 for every even batch (K split), A/B only
static int wino4_w16_env() {
  static int v = [] {
    return ERTD_KNOB("WINO4_W16", 0);
  }();
  return v;
}

// ERTD_WINO4S (A/B): 0 off, 1 the 16x16 level (where its items fill the CUs),
// 2 every eligible level, 3 the 32x32 / 64x64 levels only, 4 (default) the
// 32x32 / 64x64 levels and 16x16 where its items fill the CUs.  U2 B=64
// (same box): 204.3 steps/s off, 222.1 (1), 224.2 (2), 205.9 (3).
static int wino4s_env() {
  static int v = [] {
    return ERTD_KNOB("WINO4S", 4);
  }();
  return v;
}

bool wino4s_ok(int cin, int ca, int cout, int wo, int B) {
  const int e = wino4s_env();
  if (e == 0 || wino_env() != 1 || cin % 8 || ca % 2 || cout % 64) return false;
  if (wo != 16 && wo != 32 && wo != 64) return false;
  if (e == 2) return true;
  if (e == 3) return wo != 16;
  if (e == 4 && wo != 16) return true;
  if (wo != 16) return false;
  if (wino4s_items(cout, wo, B) >= cu_count()) return true;
  // the K-split schedule (half the CUs' worth of items): only where every caller
  // that sizes scratch (want_split: conv_wino_ok && wino_ksplit_wanted) hands the
  // kernel its ksplit_buf -- a concatenated input with Ca % 8 != 0 runs F(2x2)
  return wino4s_ksplit(cin, cout, wo, B) && conv_wino_ok(cin, ca, cout, wo);
}

bool wino4_ok(int cin, int ca, int cout, int wo, int B) {
  if (wino_env() != 1 || cin % 4 || ca % 4 || cout % 64) return false;
  if (wino4s_ok(cin, ca, cout, wo, B)) return true;
  if (wo == 16)
    return B % 2 == 0 && (wino4_w16_env() == 1 || wino4_tile_items(cout, wo, B) >= cu_count());
  return wo == 32 || wo == 64 || wo == 128;
}

bool wino4_ksplit(int cin, int cout, int wo, int B) {
  if (wino4s_ok(cin, cin, cout, wo, B)) return wino4s_ksplit(cin, cout, wo, B);
  const int nchunk = cin / 4;
  return nchunk % 2 == 0 && nchunk >= 4 && wino4_tile_items(cout, wo, B) < ksplit_items() * cu_count();
}

bool wino_dispatchable(const ConvArgs& a, int B) {
  if (a.Ho != a.Wo || a.Hs != a.Ho || a.Ws != a.Wo) return false;
  return (a.wpk_wino4 && wino4_ok(a.Cin, a.Ca, a.Cout, a.Wo, B)) ||
         (a.wpk_wino && conv_wino_ok(a.Cin, a.Ca, a.Cout, a.Wo));
}

bool wino_ksplit_wanted(int cin, int cout, int wo, int B) {
  if (wino4_ok(cin, cin, cout, wo, B)) return wino4_ksplit(cin, cout, wo, B);
  const int base = (wo / 2) * (wo / 2) / 64 * (cout / 64) * B;
  const int nchunk = cin / WKC;
  return nchunk % 2 == 0 && nchunk >= 4 && base < ksplit_items() * cu_count();
}

bool conv_wino_ok(int cin, int ca, int cout, int wo) {
  return wino_env() != 0 && cin % WKC == 0 && ca % WKC == 0 && cout % 64 == 0 &&
         (wo == 16 || wo == 32 || wo == 64 || wo == 128);
}

size_t conv_packed_floats_wino(int cin, int cout) {
  if (cin % WKC || cout % 64) return 0;
  return (size_t)16 * cout * cin;
}

hipError_t launch_pack_conv_wino(const float* w, int cin, int cout, float* dst, hipStream_t s,
                                 bool flipT) {
  const size_t total = conv_packed_floats_wino(cin, cout);
  if (!total) return hipErrorInvalidValue;
  const size_t items = total / 16;
  pack_wino_kernel<<<(unsigned)((items + 255) / 256), 256, 0, s>>>(w, cin, cout, cin / WKC, items, dst,
                                                                    flipT);
  return hipGetLastError();
}

// parts per (sample, channel) of the GroupNorm partials the dispatched
// Winograd kernel emits (none when it splits its K: the halves are summed by
// a separate pass after the epilogue)
int wino_gn_parts(const ConvArgs& a, int B) {
  if (!wino_dispatchable(a, B)) return 0;
  if (a.wpk_wino4 && wino4_ok(a.Cin, a.Ca, a.Cout, a.Wo, B)) {
    if (a.ksplit_buf && wino4_ksplit(a.Cin, a.Cout, a.Wo, B)) return 0;
    return (a.Wo / 4) * (a.Wo / 4) / 16;
  }
  const int base = (a.Wo / 2) * (a.Wo / 2) / 64 * (a.Cout / 64) * B;
  const int nchunk = a.Cin / WKC;
  if (a.ksplit_buf && nchunk % 2 == 0 && nchunk >= 4 && base < ksplit_items() * cu_count()) return 0;
  return (a.Wo / 2) * (a.Wo / 2) / 32;
}

hipError_t launch_conv_wino(int act, const ConvArgs& a, int B, hipStream_t s) {
  if (a.wpk_wino4 && wino4s_ok(a.Cin, a.Ca, a.Cout, a.Wo, B) && a.Ho == a.Wo && a.Hs == a.Ho &&
      a.Ws == a.Wo)
    return launch_conv_wino4s(act, a, B, s, cu_count());
  if (a.wpk_wino4 && wino4_ok(a.Cin, a.Ca, a.Cout, a.Wo, B) && a.Ho == a.Wo && a.Hs == a.Ho &&
      a.Ws == a.Wo)
    return launch_conv_wino4(act, a, B, s, cu_count());
  if (!a.wpk_wino || !conv_wino_ok(a.Cin, a.Ca, a.Cout, a.Wo) || a.Ho != a.Wo || a.Hs != a.Ho ||
      a.Ws != a.Wo)
    return hipErrorInvalidValue;
  switch (act) {
    case ACT_NONE: return launch_act<ACT_NONE>(a, B, s);
    case ACT_GN_SILU: return launch_act<ACT_GN_SILU>(a, B, s);
    case ACT_GN: return launch_act<ACT_GN>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet
}  // namespace ertd
