// Winograd F(4x4,3x3) with register-resident weights: the variant of
// conv_wino4_kernel (unet_conv_wino4.hip, same points, same U packing, same
// fp32 arithmetic) for work items of 64 output channels x 16 tiles.
//
// Why a second schedule: conv_wino4_kernel stages the transformed weights U
// through a 108 KB LDS ring and feeds BOTH MFMA operands from LDS; its items
// are 64 co x 32 tiles, so at 16x16 (16 tiles per sample) a B = 64 batch has
// 128 items for 256 CUs and the level ran F(2x2) instead.  Here
//   * each of the 4 MFMA waves (one per SIMD) owns 16 co x 16 tiles x all 36 xi
//     (144 accumulator VGPRs) and streams ITS OWN U fragments from L2 straight
//     into VGPRs (18 buffer_load_dwordx2 per k-step, one k-step ahead, double
//     buffered: the A operand never touches LDS, no LDS-DMA issue on the MFMA
//     waves) -- no other wave reads them, so nothing is lost by not sharing;
//   * LDS holds only V (the transformed input, 18 KB per 8-channel chunk,
//     double-buffered): one ds_read_b64 per xi pair feeds two MFMAs;
//   * 4 producer waves, each two channels of the chunk (lane = channel bit 5,
//     column half bit 4, tile bits 0-3), do GroupNorm + SiLU + B^T d B exactly
//     as conv_wino4_kernel's producers (the half exchange is v_permlane16_swap:
//     the halves are 16 lanes apart here);
//   * XS = 1: 512 threads, 256 VGPRs per wave (2 waves per SIMD), 36 KB of LDS;
//   * XS = 2 (the default): each co block's 36 xi are split over two MFMA
//     waves (8 MFMA waves, 768 threads, 163 VGPRs, 36 + 64 KB of LDS); the
//     halves' partial output tiles meet in an LDS exchange buffer (below).
// Item = (co group of 64, block of 16 consecutive tiles of one sample); the
// output transform, bias / emb / residual epilogue and the GroupNorm partials
// (one part per 16 tiles, as conv_wino4_kernel) are per MFMA wave.
// K split (ksp = 2, XS = 2 only, never for the Upsample convs): where the items
// fill half the CUs or more but not all (wino4s_ksplit: the 16x16 level of the
// B = 32 train step), an item is (K half, co group, block) with the two halves
// of a (co group, block) adjacent; half 0 sweeps channels [0, Cin/2) and writes
// out with bias / emb / residual, half 1 sweeps [Cin/2, Cin) and writes its raw
// sums to ksplit_buf (no bias / emb / residual, no GroupNorm partials: a split
// layer emits none), and add_inplace_kernel adds them afterwards.
#include <cstdlib>
#include <type_traits>

#include "unet.h"

namespace ertd {
namespace unet {

namespace {

constexpr int NMW = 4;                        // co blocks (MFMA waves at XS = 1, one per SIMD)
constexpr int NPW = 4;                        // producer waves
constexpr int CCH = 8;                        // input channels per chunk (2 MFMA k-steps)
constexpr int NX = 36;
constexpr int VKS = 18 * 128;                 // V floats per k-step: [xi/2 18][k 4][tile 16][xi&1]
constexpr int V_FL = 2 * VKS;                 // per chunk (4608 floats = 18 KB)
constexpr size_t WLDS = (size_t)2 * V_FL * sizeof(float);   // 36 KB
constexpr int NRS = 3;                        // producer register sets
constexpr int GNC_JM = 4;                     // consumer-side finalize: jobs per MFMA wave
constexpr int GNC_KM = 6;                     //   parts per lane and group
constexpr int GNC_TAB = 4096;                 //   table entries (item x channel): 32 KB of LDS
#ifndef WINO4S_PPRIO
#define WINO4S_PPRIO 2
#endif
#ifndef WINO4S_PD
#define WINO4S_PD 2                           // V operand read-ahead (xi pairs)
#endif
#ifndef WINO4S_MPRIO
#define WINO4S_MPRIO 1                        // s_setprio of the xh = 1 MFMA waves (0 = none): +0.3-0.7 % U2 B=64
#endif
#ifndef WINO4S_XCD
#define WINO4S_XCD 1                          // XCD-aware item walk (0: blockIdx order)
#endif
#ifndef WINO4S_XCDMAX
#define WINO4S_XCDMAX 2                       // ... for layers of at most this many co groups
#endif
#ifndef WINO4S_PACK
#define WINO4S_PACK 1                         // producer stage on packed fp32 pairs
#endif
#ifndef WINO4S_RPF
#define WINO4S_RPF 0                          // residual L2 prefetch this many chunks before the epilogue
                                              // (0: none; 2: 250.2 vs 252.2 steps/s U2 B=64, same box)
#endif
// Ablations for a diagnostic build only (tools/build_variant.sh ... -DWINO4S_ABL=n;
// results WRONG, never in the shipped library): bit 0 the producers skip the
// activation and transform, bit 1 every U load reads the first k-step (L2-hot),
// bit 2 the MFMAs become one VALU fma, bit 3 the output transform / stores are skipped,
// bit 4 no per-chunk barrier (either role), bit 5 the MFMA waves issue no U loads
#ifndef WINO4S_ABL
#define WINO4S_ABL 0
#endif
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
using u32x2 = __attribute__((ext_vector_type(2))) unsigned;

__device__ __forceinline__ f32x2 fmac(f32x2 x, float c, f32x2 s) {
  return __builtin_elementwise_fma(x, f32x2{c, c}, s);
}
// B^T d and A^T m of the points {0, 1, -1, 1/2, -2, inf} (unet_conv_wino4.hip)
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
// bt6 on two columns at once (packed fp32: the same fma / add sequence per
// element as bt6, so the same bits)
__device__ __forceinline__ f32x2 pfma(f32x2 a, float c, f32x2 b) {
  return __builtin_elementwise_fma(a, f32x2{c, c}, b);
}
__device__ __forceinline__ void bt6p(const f32x2 (&d)[6], f32x2 (&o)[6]) {
  const f32x2 c = d[4] - d[2], e = d[3] - d[1];
  const f32x2 u = d[4] - d[1], v = d[4] + d[1];
  o[0] = pfma(e, 1.5f, pfma(d[2], -2.f, d[0] + d[4]));
  o[1] = pfma(d[3], 2.5f, pfma(d[2], 0.5f, u));
  o[2] = pfma(d[3], 0.5f, pfma(d[2], -2.5f, v));
  o[3] = pfma(e, 2.f, c);
  o[4] = pfma(e, -0.5f, c);
  o[5] = pfma(c, 1.5f, pfma(d[3], -2.f, d[1] + d[5]));
}
__device__ __forceinline__ void at6(const f32x2 (&m)[6], f32x2 (&y)[4]) {
  const f32x2 s = m[1] + m[2], d = m[1] - m[2];
  y[0] = (m[0] + s) + (m[3] + m[4]);
  y[1] = fmac(m[3], 0.5f, fmac(m[4], -2.f, d));
  y[2] = fmac(m[3], 0.25f, fmac(m[4], 4.f, s));
  y[3] = fmac(m[3], 0.125f, fmac(m[4], -8.f, d + m[5]));
}

// the GroupNorm fold's finalizes, after the MFMA waves' last item (the
// producer waves have exited: the barrier counts the MFMA waves): samples
// bid, bid + grid, ... -- wave 0 waits for the sample's item count (all
// workgroups are resident: one per CU, grid <= CUs) and re-arms the counter,
// then every MFMA wave finalizes its share of the sample's groups
__device__ __forceinline__ void wino4s_fold_tail(const GnFold& f, int lane, int wave, int nmw) {
  for (int b = blockIdx.x; b < f.B; b += gridDim.x) {
    if (wave == 0 && lane == 0) {
      const unsigned* c = f.cnt + b;
      while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (unsigned)f.target)
        __builtin_amdgcn_s_sleep(2);
      __hip_atomic_store(f.cnt + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    gn_group_finalize<true>(f.g, b, lane, wave, nmw);
  }
}

#ifdef WINO4S_STAMP
// Diagnostic build only (tools/wino4s_stamps.py): per-wave s_memtime stamps of
// workgroups 0..255, stored by lane 0 with vector stores.  Per wave (S4_SPW
// words): [0] s_memrealtime at entry (low 32 bits), [1] s_memtime at entry,
// [2] barrier (A) passed; MFMA waves: per item il < 8 [3 + 3 il] item start,
// [4 + 3 il] last chunk barrier passed, [5 + 3 il] epilogue stores issued;
// [27] exit; [28 + g] chunk g's barrier passed (g < 32, the first item(s));
// producer waves: [3] prologue staged (before (A)), [27] exit; GNC: [25]
// table done (MFMA) / first loads issued (producers), [26] barrier (A0) passed.
constexpr int S4_SPW = 64;
__device__ unsigned g_w4s_stamps[256 * 12 * S4_SPW];
#define W4S_STAMP(slot)                                                                            \
  do {                                                                                             \
    if (blockIdx.x < 256 && lane == 0)                                                             \
      g_w4s_stamps[(blockIdx.x * 12 + wave) * S4_SPW + (slot)] = (unsigned)__builtin_amdgcn_s_memtime(); \
  } while (0)
#define W4S_STAMP_ENTRY()                                                                          \
  do {                                                                                             \
    if (blockIdx.x < 256 && lane == 0) {                                                           \
      g_w4s_stamps[(blockIdx.x * 12 + wave) * S4_SPW] = (unsigned)__builtin_amdgcn_s_memrealtime(); \
      g_w4s_stamps[(blockIdx.x * 12 + wave) * S4_SPW + 1] = (unsigned)__builtin_amdgcn_s_memtime(); \
    }                                                                                              \
  } while (0)
#else
#define W4S_STAMP(slot) \
  do {                  \
  } while (0)
#define W4S_STAMP_ENTRY() \
  do {                    \
  } while (0)
#endif

// item it -> (K half, co group, 16-tile block): the K halves of a (co group,
// block) adjacent, then co group, then block
struct Item {
  int cog, blk, half;
};
__device__ __forceinline__ Item item_of(int it, int ncog, int ksp) {
  Item r;
  r.half = it % ksp;
  const int pr = it / ksp;
  r.cog = pr % ncog;
  r.blk = pr / ncog;
  return r;
}

// a workgroup's items in walk order: item base + il stride
struct ItemWalk {
  int base, stride, ncog, ksp;
  __device__ __forceinline__ Item at(int il) const { return item_of(base + il * stride, ncog, ksp); }
};
__device__ __forceinline__ int itm_half(const ItemWalk& w, int il) { return w.at(il).half; }

// UP: the Upsample conv, conv3x3 of the nearest-x2 upsampled source (WO / 2)^2:
// the window rows 4ty-1 .. 4ty+4 of the upsampled image are source rows 2ty-1,
// 2ty, 2ty, 2ty+1, 2ty+1, 2ty+2 and a lane's two columns one source column, so
// a producer lane loads 4 source values instead of 12 (36 of the 144
// multiplies per 4x4 output tile, against 64 for the sub-pixel direct kernel)
// XS = 2: each co block's 36 xi are split over two MFMA waves (xi 0-17 / 18-35:
// Winograd rows 0-2 / 3-5) -- two MFMA waves per SIMD hide each other's
// operand-read and issue stalls; each computes the partial output transform
// of its rows, the halves are exchanged through LDS across the item's last
// barrier, and each wave finishes two of the lane's four channels
// FOLD (diagnostic builds only, ERTD_UNET_GNFOLD): the GroupNorm fold's
// write-through partial stores, arrival counts and finalize tail.  The shipped
// instantiation (FOLD = false) has none of it: no static LDS word in front of
// the dynamic V buffers, no per-item branches.
// GNC: the input's GroupNorm finalize runs in this kernel's prologue
// (ConvArgs::gnc, conv_gn_consume_ok): before the first chunk the 8 MFMA waves
// -- idle until the producers stage chunk 0 -- merge the partials of every
// item's sample into an LDS table of {scale, shift} per (item, channel)
// (gn_group_finalize_regs: the arithmetic of gn_finalize_kernel, so the same
// bits, with all loads issued first), while the producers' first input loads
// are in flight; the producers read the table instead of ConvArgs::gn.  One
// launch (3.3 us of the step graph, measured) per GroupNorm fewer.
// cw > 0 (diagnostic A/B only): contiguous walk -- workgroup bid runs items
// bid * cw .. bid * cw + cw - 1 (nitems == grid * cw); 0: items bid, bid + grid, ...
template <int WO, int ACT, bool UP, int XS, bool FOLD, bool GNC>
__global__ __launch_bounds__(64 * (4 * XS + NPW)) void conv_wino4s_kernel(ConvArgs a, int nitems, int ksp, int cw) {
  static_assert(!GNC || (XS == 2 && !UP && ACT != ACT_NONE && !FOLD), "GNC: the xi-split GN+act kernel");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* vbuf = smem;                  // [2][V_FL]
  int* fold_items = nullptr;           // GroupNorm fold: MFMA waves done with the current item
  if constexpr (FOLD) {
    __shared__ int fold_lds;
    fold_items = &fold_lds;
    if (threadIdx.x == 0) fold_lds = 0;
  }

  constexpr int TPR = WO / 4;
  constexpr int HW = WO * WO;
  constexpr int TS = TPR * TPR;        // tiles per sample (a multiple of 16)
  constexpr int WS = UP ? WO / 2 : WO; // source width
  constexpr int HWS = WS * WS;
  static_assert(TS % 16 == 0 && TPR <= 16, "a 16-tile block is whole tile rows of one sample");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  W4S_STAMP_ENTRY();
  const int Cin = a.Cin, Ca = a.Ca;
  // ksp = 2 (XS = 2 only): an item runs half of the input channels, the
  // second half's sums go to a.ksplit_buf (no bias / emb / residual) and are
  // added by a separate pass -- layers whose items would fill only half the CUs
  const int nchunk = Cin / CCH / ksp;          // chunks per item
  const int ncog = a.Cout / 64;
  // XCD-aware item walk for layers of one or two co groups: workgroups are
  // dealt round-robin to the 8 XCDs (blockIdx % 8); the remap hands each XCD
  // runs of consecutive items (a sample's tile rows and its co groups), so the
  // tile-row halos and the input both co groups read come from that XCD's L2.
  // With 4-8 co groups (the 16x16 level, the 16 -> 32 Upsample conv) the
  // blockIdx order keeps one co group's transformed weights (2.4-9.4 MB of
  // them) per XCD (cog = bid % ncog), which saves more (PMC, U2 B=64:
  // profiles/r05_u2_layer_traffic.txt).
  const int G = gridDim.x;
  const int bid = (WINO4S_XCD && G % 8 == 0 && ncog <= WINO4S_XCDMAX)
                      ? (int)(blockIdx.x % 8) * (G / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const ItemWalk wk = cw ? ItemWalk{bid * cw, 1, ncog, ksp} : ItemWalk{bid, G, ncog, ksp};
  const int nloc = cw ? (bid * cw < nitems ? min(cw, nitems - bid * cw) : 0)
                      : (bid < nitems ? (nitems - bid + G - 1) / G : 0);
  float2* const gtab = reinterpret_cast<float2*>(smem + 2 * V_FL + 4 * 2 * 8 * 256);   // GNC: [item][Cin]
  const int gtot = nloc * nchunk;

  if (wave >= 4 * XS) {
    // =================== producer waves ===================
    __builtin_amdgcn_s_setprio(WINO4S_PPRIO);
    const int q = wave - 4 * XS;              // channels 2q, 2q+1 of every chunk
    const int chb = lane >> 5, h = (lane >> 4) & 1, t = lane & 15;
    const int cl = 2 * q + chb;               // channel of the chunk: k-step cl >> 2, k = cl & 3
    const int vwoff = ((((cl >> 2) * 18 + 9 * h) * 4 + (cl & 3)) * 16 + t) * 2;
    // the outer window column from the neighbouring tile's other half (16 lanes apart)
    const int nbaddr = (lane + 15 - 30 * h) * 4;
    const unsigned choff = (unsigned)(chb * HWS * 4);
    float2 raw[NRS][6];
    float2 gnv[NRS];
    int gch[NRS];
    f32x4 pad[NRS];
    int cur_g = 0, cur_k = 0, cur_b = 0, cur_il = 0, cur_k0 = 0;
    unsigned roff[6];   // per window row (UP: per distinct source row, 4)
    f32x4 cur_pad;
    auto set_item = [&](int il) {
      const Item itm = wk.at(il);
      cur_k0 = itm.half * nchunk;
      const int flat0 = itm.blk * 16;
      cur_b = flat0 / TS;
      const int tg = flat0 % TS + t;
      const int ty = tg / TPR, tx = tg - ty * TPR;
      if constexpr (UP) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int sy = 2 * ty - 1 + r;
          roff[r] = (unsigned)(((sy >= 0 && sy < WS ? sy : 2 * ty) * WS + 2 * tx + h) * 4) + choff;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          const int iy = 4 * ty - 1 + r;
          roff[r] = (unsigned)(((iy >= 0 && iy < WO ? iy : 4 * ty) * WO + 4 * tx + 2 * h) * 4) + choff;
        }
      }
      cur_pad = f32x4{ty > 0 ? 1.f : 0.f, ty < TPR - 1 ? 1.f : 0.f,
                      (h ? tx < TPR - 1 : tx > 0) ? 1.f : 0.f, 0.f};
    };
    const int glast = gtot - 1;
    auto load_next = [&](const int set) {
      const int cg = (cur_k0 + cur_k) * CCH + 2 * q;   // wave-uniform first channel of the pair
      pad[set] = cur_pad;
      if constexpr (GNC) gch[set] = cur_il * Cin + cg + chb;   // the table entry, read at the activation
      else if constexpr (ACT != ACT_NONE) gnv[set] = a.gn[(size_t)cur_b * Cin + cg + chb];
      const bool inA = cg < Ca;               // Ca even: both channels on one side
      const float* p = inA ? a.srcA + ((size_t)cur_b * Ca + cg) * HWS
                           : a.srcB + ((size_t)cur_b * a.Cb + (cg - Ca)) * HWS;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 2 * HWS * 4, 0x00020000);
      if constexpr (UP) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)roff[r], 0, 0));
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          const float u = v[(r + 1) >> 1];
          raw[set][r] = make_float2(u, u);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 6; ++r) {
          const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)roff[r], 0, 0);
          raw[set][r] = make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
        }
      }
      if (cur_g < glast) {
        ++cur_g;
        if (++cur_k == nchunk) {
          cur_k = 0;
          set_item(++cur_il);
        }
      }
    };
    // act[ab][c][i]: row i of B^T d for local column c (window columns 1+2h,
    // 2+2h and the outer one): the lane transforms its own two columns and takes
    // the outer column's transform from the neighbouring tile's lane (B^T is
    // linear, so transforming before the exchange skips the third column's bt6)
#if WINO4S_PACK
    // the lane's two own columns as one packed pair through GroupNorm, SiLU,
    // the row padding and the column transform (v_pk_* on f32x2: the same fma /
    // mul / add per element as the scalar form, so the same bits); exp and rcp
    // have no packed form.  act2[ab][i] = transformed row i of (col a, col b),
    // actn[ab][i] = that of the outer column (from the neighbour lane)
    f32x2 act2[2][6];
    float actn[2][6];
    auto act_stage = [&](const int set, const int ab) {
      if constexpr (GNC) gnv[set] = gtab[gch[set]];
      f32x2 m[6];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        m[r] = f32x2{raw[set][r].x, raw[set][r].y};
        if constexpr (ACT != ACT_NONE) {
          m[r] = __builtin_elementwise_fma(m[r], f32x2{gnv[set].x, gnv[set].x}, f32x2{gnv[set].y, gnv[set].y});
          if constexpr (ACT == ACT_GN_SILU) {
            // __expf(-y) = exp2(y * -log2 e): the same v_mul + v_exp as the scalar code
            f32x2 e = m[r] * f32x2{-1.44269504088896340736f, -1.44269504088896340736f};
            e = f32x2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)} + f32x2{1.0f, 1.0f};
            m[r] = m[r] * f32x2{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
          }
        }
      }
      m[0] = m[0] * f32x2{pad[set].x, pad[set].x};
      m[5] = m[5] * f32x2{pad[set].y, pad[set].y};
      bt6p(m, act2[ab]);
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const float give = h ? act2[ab][i].y : act2[ab][i].x;
        const float nb = __int_as_float(__builtin_amdgcn_ds_bpermute(nbaddr, __float_as_int(give)));
        actn[ab][i] = nb * pad[set].z;
      }
    };
#else
    float act[2][3][6];
    auto act_stage = [&](const int set, const int ab) {
      if constexpr (GNC) gnv[set] = gtab[gch[set]];
      float cx[6], cy[6];
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        float2 m = raw[set][r];
        if constexpr (ACT != ACT_NONE) {
          m.x = __builtin_fmaf(m.x, gnv[set].x, gnv[set].y);
          m.y = __builtin_fmaf(m.y, gnv[set].x, gnv[set].y);
          if constexpr (ACT == ACT_GN_SILU) {
            m.x = m.x * __builtin_amdgcn_rcpf(1.0f + __expf(-m.x));
            m.y = m.y * __builtin_amdgcn_rcpf(1.0f + __expf(-m.y));
          }
        }
        if (r == 0 || r == 5) {
          const float fy = r == 0 ? pad[set].x : pad[set].y;
          m.x *= fy;
          m.y *= fy;
        }
        cx[r] = m.x;
        cy[r] = m.y;
      }
      bt6(cx, act[ab][0]);
      bt6(cy, act[ab][1]);
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const float give = h ? act[ab][1][i] : act[ab][0][i];
        const float nb = __int_as_float(__builtin_amdgcn_ds_bpermute(nbaddr, __float_as_int(give)));
        act[ab][2][i] = nb * pad[set].z;
      }
    };
#endif
    auto tr_stage = [&](const int ab, float* vb) {
      float w[6][3];
#if WINO4S_PACK
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        w[i][0] = act2[ab][i].x;
        w[i][1] = act2[ab][i].y;
        w[i][2] = actn[ab][i];
      }
#else
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int i = 0; i < 6; ++i) w[i][c] = act[ab][c][i];
#endif
      // rows 0-2 to the lower half (h = 0), 3-5 to the upper: the rows of 16
      // lanes pair (0,1), (2,3) -- afterwards row[a][j] is row 3h+a of window column j
      float row[3][6];
#pragma unroll
      for (int aa = 0; aa < 3; ++aa)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[aa][c]),
                                                           __float_as_uint(w[3 + aa][c]), false, false);
          const int jl = c == 0 ? 1 : (c == 1 ? 2 : 0);
          row[aa][jl] = __uint_as_float(sw[0]);
          row[aa][3 + c] = __uint_as_float(sw[1]);
        }
      float* o = vb + vwoff;
#pragma unroll
      for (int aa = 0; aa < 3; ++aa) {
        float vv[6];
        bt6(row[aa], vv);
#pragma unroll
        for (int jp = 0; jp < 6; jp += 2)
          *reinterpret_cast<f32x2*>(o + (aa * 3 + jp / 2) * 128) = f32x2{vv[jp], vv[jp + 1]};
      }
    };
    auto slot = [&](auto sa, auto ab, int g) {
      constexpr int SA = decltype(sa)::value, AB = decltype(ab)::value;
      if constexpr (!(WINO4S_ABL & 1)) {
        tr_stage(AB ^ 1, vbuf + ((g + 1) & 1) * V_FL);
        act_stage(SA, AB);
      }
      load_next(SA);
      if constexpr (!(WINO4S_ABL & 16)) __syncthreads();   // (B) end of slot g
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    if (gtot > 0) {
      set_item(0);
      load_next(0);
      load_next(1);
      load_next(2);
    }
    if constexpr (GNC) {
      W4S_STAMP(25);
      __syncthreads();   // (A0) the MFMA waves' GroupNorm table is in LDS
      W4S_STAMP(26);
    }
    if (gtot > 0) {
      act_stage(0, 0);
      tr_stage(0, vbuf);
      load_next(0);      // chunk 3
      act_stage(1, 1);
      load_next(1);      // chunk 4
    }
    W4S_STAMP(3);
    __syncthreads();   // (A) chunk 0 staged
    W4S_STAMP(2);
    int g = 0;
    for (; g + 5 < gtot; g += 6) {
      slot(I2{}, I0{}, g);
      slot(I0{}, I1{}, g + 1);
      slot(I1{}, I0{}, g + 2);
      slot(I2{}, I1{}, g + 3);
      slot(I0{}, I0{}, g + 4);
      slot(I1{}, I1{}, g + 5);
    }
    if (g < gtot) slot(I2{}, I0{}, g);
    if (g + 1 < gtot) slot(I0{}, I1{}, g + 1);
    if (g + 2 < gtot) slot(I1{}, I0{}, g + 2);
    if (g + 3 < gtot) slot(I2{}, I1{}, g + 3);
    if (g + 4 < gtot) slot(I0{}, I0{}, g + 4);
    W4S_STAMP(27);
    return;
  }

  if constexpr (XS == 1) {
  // =================== MFMA waves ===================
  const int cb = wave;                         // co block of 16
  f32x4 acc[NX];
  // U fragments of (co group, 4-channel k-step ks, xi pair p, co block cb):
  // 128 floats at byte ((cog * nks + ks) * 18 + p) * 2048 + cb * 512 of wpk_wino4
  // (launch_pack_conv_wino4's layout); lane l reads the float2 at l * 8
  const int nks = Cin / 4;
  const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.wpk_wino4), (short)0, (int)((size_t)NX * a.Cout * Cin * 4), 0x00020000);
  // U cursor: the k-step whose fragments load next (clamped at the last one)
  int u_il = 0, u_ks = 0;
  int u_base = 0;                              // byte offset of (cog, ks = 0) of item u_il
  auto u_item = [&](int il) {
    const Item itm = wk.at(il);
    u_base = itm.cog * nks * 36864;
  };
  auto u_advance = [&]() {
    if (++u_ks == nks) {
      if (u_il + 1 < nloc) {
        u_ks = 0;
        u_item(++u_il);
      } else {
        u_ks = nks - 1;                        // past the end: re-load the last k-step
      }
    }
  };
  if (nloc > 0) u_item(0);
  f32x2 ub[2][18];
  const int uvoff = lane * 8 + cb * 512;
  auto u_load = [&](f32x2 (&u)[18], const int p) {
    if constexpr ((WINO4S_ABL & 32) != 0) {
      u[p] = u[p] + f32x2{1.f, 1.f};
      return;
    }
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(
        ru, uvoff, (WINO4S_ABL & 2) ? p * 2048 : u_base + u_ks * 36864 + p * 2048, 0);
    u[p] = f32x2{__uint_as_float(v[0]), __uint_as_float(v[1])};
  };
  if (nloc > 0) {
#pragma unroll
    for (int p = 0; p < 18; ++p) u_load(ub[0], p);
    u_advance();
  }
  __syncthreads();   // (A)
#ifndef WINO4S_XK
#define WINO4S_XK 1                           // V read-ahead continues across the chunk's two k-steps
#endif
  // one k-step: 36 MFMAs on V (LDS) and U (registers u), the next k-step's U
  // fragments loaded into nx, one per xi pair
  auto kstep = [&](const f32x2 (&u)[18], f32x2 (&nx)[18], const float* vs) {
    constexpr int PD = WINO4S_PD;
    f32x2 rb[PD + 1];
#pragma unroll
    for (int p = 0; p < PD; ++p) rb[p] = *reinterpret_cast<const f32x2*>(vs + p * 128);
#pragma unroll
    for (int p = 0; p < 18; ++p) {
      if (p + PD < 18) rb[(p + PD) % (PD + 1)] = *reinterpret_cast<const f32x2*>(vs + (p + PD) * 128);
      const int r = p % (PD + 1);
      if constexpr (WINO4S_ABL & 4) {
        acc[2 * p][0] = __builtin_fmaf(u[p].x, rb[r].x, acc[2 * p][0]);
        acc[2 * p + 1][0] = __builtin_fmaf(u[p].y, rb[r].y, acc[2 * p + 1][0]);
      } else {
        acc[2 * p] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[p].x, rb[r].x, acc[2 * p], 0, 0, 0);
        acc[2 * p + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[p].y, rb[r].y, acc[2 * p + 1], 0, 0, 0);
      }
      u_load(nx, p);
      if (p + PD < 18) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                      // MFMAs
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                      // VMEM read
    }
    u_advance();
  };
  // a whole chunk (both k-steps) as one stream: the V operand reads run PD xi
  // pairs ahead across the k-step boundary too
  auto chunk2 = [&](const float* vs) {
    constexpr int PD = WINO4S_PD;
    f32x2 rb[PD + 1];
#pragma unroll
    for (int q = 0; q < PD; ++q) rb[q] = *reinterpret_cast<const f32x2*>(vs + q * 128);
#pragma unroll
    for (int q = 0; q < 36; ++q) {
      const int st = q / 18, p = q % 18;
      const int qn = q + PD;
      if (qn < 36) rb[qn % (PD + 1)] = *reinterpret_cast<const f32x2*>(vs + (qn / 18) * VKS + (qn % 18) * 128);
      const int r = q % (PD + 1);
      const f32x2 u = st == 0 ? ub[0][p] : ub[1][p];
      acc[2 * p] = __builtin_amdgcn_mfma_f32_16x16x4f32(u.x, rb[r].x, acc[2 * p], 0, 0, 0);
      acc[2 * p + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u.y, rb[r].y, acc[2 * p + 1], 0, 0, 0);
      if (st == 0) u_load(ub[1], p);
      else u_load(ub[0], p);
      if (qn < 36) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                  // MFMAs
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                  // VMEM read
      if (p == 17) u_advance();
    }
  };
  for (int il = 0; il < nloc; ++il) {
#pragma unroll
    for (int x = 0; x < NX; ++x) acc[x] = f32x4{};
    for (int k = 0; k < nchunk; ++k) {
      const int g = il * nchunk + k;
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      const float* vb = vbuf + (g & 1) * V_FL + ln * 2;
      if constexpr (WINO4S_XK && !(WINO4S_ABL & 4)) {
        chunk2(vb);
      } else {
        kstep(ub[0], ub[1], vb);
        kstep(ub[1], ub[0], vb + VKS);
      }
#pragma unroll
      for (int x = 0; x < NX; ++x) asm volatile("" : "+v"(acc[x]));
      if constexpr (!(WINO4S_ABL & 16)) __syncthreads();   // (B)
    }

    if constexpr ((WINO4S_ABL & 8) != 0) {
      if (il == nloc - 1) {
        float sacc = 0.f;
        for (int x = 0; x < NX; ++x) sacc += acc[x][0] + acc[x][3];
        a.out[(size_t)bid * 64 + lane] = sacc;
      }
      continue;
    }
    // ---- output transform: lane l holds M[xi] of co = 16 cb + 4 (l >> 4) + i, tile l & 15
    const Item itm = wk.at(il);
    const int flatw = itm.blk * 16;
    const int smpl = flatw / TS;
    const bool has_eb = a.ebias != nullptr, has_res = a.res != nullptr, has_bias = a.bias != nullptr;
    const unsigned smp = (unsigned)(a.Cout * HW * 4);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        a.out + (size_t)smpl * a.Cout * HW, (short)0, smp, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        has_res ? const_cast<float*>(a.res) + (size_t)smpl * a.Cout * HW : nullptr, (short)0, smp,
        0x00020000);
    f32x4 y[4][4];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      f32x2 P[6][4];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        f32x2 m[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) m[j] = f32x2{acc[6 * i + j][2 * pp], acc[6 * i + j][2 * pp + 1]};
        at6(m, P[i]);
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        f32x2 col[6], yc[4];
#pragma unroll
        for (int i = 0; i < 6; ++i) col[i] = P[i][x];
        at6(col, yc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          y[2 * pp][r][x] = yc[r].x;
          y[2 * pp + 1][r][x] = yc[r].y;
        }
      }
    }
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    const int co0 = itm.cog * 64 + cb * 16 + 4 * (ln >> 4);
    const int tg = flatw % TS + (ln & 15);
    const int ty = tg / TPR, tx = tg - ty * TPR;
    const int vo = (co0 * HW + 4 * ty * WO + 4 * tx) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float bi = has_bias ? a.bias[co0 + i] : 0.f;
      const float ei = has_eb ? a.ebias[(size_t)smpl * a.eb_stride + co0 + i] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        y[i][r] = y[i][r] + bi;
        if (has_eb) y[i][r] = y[i][r] + ei;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (has_res) {
      f32x4 rv[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          rv[i][r] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, vo, i * HW * 4 + r * WO * 4, 0));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) y[i][r] = y[i][r] + rv[i][r];
    }
    if (a.gnp) {
      float2 pr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float sm = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) sm += (y[i][r][0] + y[i][r][1]) + (y[i][r][2] + y[i][r][3]);
        sm = row16_sum(sm);
        const float mu = sm * (1.0f / 256.0f);
        float qq = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            const float d = y[i][r][x] - mu;
            qq = __builtin_fmaf(d, d, qq);
          }
        pr[i] = make_float2(sm, row16_sum(qq));
      }
      if ((ln & 15) == 0) {
        const int np = TS / 16, part = (flatw % TS) / 16;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float2* d = a.gnp + ((size_t)smpl * a.Cout + co0 + i) * np + part;
          if constexpr (FOLD) st_f2_wt(d, pr[i]);
          else *d = pr[i];
        }
      }
      if constexpr (FOLD) gn_fold_item_done(a.fold, smpl, fold_items, NMW, ln);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y[i][r]), ro, vo,
                                               i * HW * 4 + r * WO * 4, 0);
  }
  if constexpr (FOLD) wino4s_fold_tail(a.fold, lane, wave, NMW);
  } else {
  // =================== MFMA waves, xi split over two waves ===================
  constexpr int NP = 9;                        // xi pairs per wave
  const int cb = wave & 3, xh = wave >> 2;
#if WINO4S_MPRIO
  if (xh) __builtin_amdgcn_s_setprio(WINO4S_MPRIO);   // static priority for the younger MFMA half
#endif
  float* xbuf = smem + 2 * V_FL;               // [4 cb][2 receiver][8][64 lanes][4]
  f32x4 acc[2 * NP];
  const int nks = Cin / 4;
  const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.wpk_wino4), (short)0, (int)((size_t)NX * a.Cout * Cin * 4), 0x00020000);
  // U cursor over the item's k-steps [u_ks0, u_end) (its K half)
  int u_il = 0, u_ks = 0, u_end = 0, u_base = 0;
  auto u_item = [&](int il) {
    const Item itm = wk.at(il);
    u_base = itm.cog * nks * 36864;
    u_ks = itm.half * nchunk * 2;
    u_end = u_ks + nchunk * 2;
  };
  auto u_advance = [&]() {
    if (++u_ks == u_end) {
      if (u_il + 1 < nloc) {
        u_item(++u_il);
      } else {
        u_ks = u_end - 1;
      }
    }
  };
  if (nloc > 0) u_item(0);
  f32x2 ub[2][NP];
  const int uvoff = lane * 8 + cb * 512;
  const int psoff = xh * NP * 2048;
  auto u_load = [&](f32x2 (&u)[NP], const int p) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(ru, uvoff, u_base + u_ks * 36864 + psoff + p * 2048, 0);
    u[p] = f32x2{__uint_as_float(v[0]), __uint_as_float(v[1])};
  };
  if (nloc > 0) {
#pragma unroll
    for (int p = 0; p < NP; ++p) u_load(ub[0], p);
    u_advance();
  }
  if constexpr (GNC) {
    // job j = item il, groups 4 jg .. 4 jg + 3 (ng4 = ceil(G / 4) jobs per item):
    // wave w of the 8 takes jobs w, w + 8, ... (conv_gn_consume_ok: <= 4 each)
    constexpr int JM = GNC_JM;
    const int ng4 = (a.gnc.groups + 3) / 4;
    int smp[JM], jg[JM], row[JM];
    bool jl[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      const int job = wave + 4 * XS * j, il = job / ng4;
      jl[j] = il < nloc;
      row[j] = jl[j] ? il : 0;
      jg[j] = job - il * ng4;
      smp[j] = jl[j] ? wk.at(il).blk * 16 / TS : 0;
    }
    gn_group_finalize_regs<JM, GNC_KM>(a.gnc, smp, jg, row, jl, lane, gtab);
    W4S_STAMP(25);
    __syncthreads();   // (A0)
    W4S_STAMP(26);
  }
  __syncthreads();   // (A)
  W4S_STAMP(2);
  auto chunk2 = [&](const float* vs) {
    constexpr int PD = WINO4S_PD;
    f32x2 rb[PD + 1];
#pragma unroll
    for (int q = 0; q < PD; ++q) rb[q] = *reinterpret_cast<const f32x2*>(vs + (xh * NP + q) * 128);
#pragma unroll
    for (int q = 0; q < 2 * NP; ++q) {
      const int st = q / NP, p = q % NP;
      const int qn = q + PD;
      if (qn < 2 * NP)
        rb[qn % (PD + 1)] = *reinterpret_cast<const f32x2*>(vs + (qn / NP) * VKS + (xh * NP + qn % NP) * 128);
      const int r = q % (PD + 1);
      const f32x2 u = st == 0 ? ub[0][p] : ub[1][p];
      acc[2 * p] = __builtin_amdgcn_mfma_f32_16x16x4f32(u.x, rb[r].x, acc[2 * p], 0, 0, 0);
      acc[2 * p + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(u.y, rb[r].y, acc[2 * p + 1], 0, 0, 0);
      if (st == 0) u_load(ub[1], p);
      else u_load(ub[0], p);
      if (qn < 2 * NP) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      if (p == NP - 1) u_advance();
    }
  };
  for (int il = 0; il < nloc; ++il) {
#pragma unroll
    for (int x = 0; x < 2 * NP; ++x) acc[x] = f32x4{};
    f32x2 own[4][4];     // this wave's partial Y of its channel pair (pp = xh): [row][col]
    if (il < 8) W4S_STAMP(3 + 3 * il);
    unsigned rpf[2] = {0u, 0u};   // the residual prefetch's destinations (kept until the epilogue)
    for (int k = 0; k < nchunk; ++k) {
      const int g = il * nchunk + k;
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#if WINO4S_RPF
      // the epilogue's residual tile into L2 WINO4S_RPF chunks ahead (its HBM
      // latency was the epilogue's critical path): one dword per 16-B segment of
      // tiles 0, 8 / 4, 12 of each (channel, row) -- every 128-B line of the
      // wave's residual rows at 64x64, 32x32 and 16x16
      if (k == (nchunk > WINO4S_RPF ? nchunk - WINO4S_RPF : 0) && a.res && itm_half(wk, il) == 0) {
        const Item pit = wk.at(il);
        const int pflat = pit.blk * 16, psm = pflat / TS;
        const int pco = pit.cog * 64 + cb * 16 + 4 * (ln >> 4) + 2 * xh + ((ln >> 3) & 1);
        const int pr = (ln >> 1) & 3;
        const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.res) + (size_t)psm * a.Cout * HW, (short)0, (unsigned)(a.Cout * HW * 4), 0x00020000);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ptg = pflat % TS + (ln & 1) * 8 + h * 4;
          const int pty = ptg / TPR, ptx = ptg - pty * TPR;
          rpf[h] = __builtin_amdgcn_raw_buffer_load_b32(rp, (pco * HW + (4 * pty + pr) * WO + 4 * ptx) * 4, 0, 0);
        }
      }
#endif
      chunk2(vbuf + (g & 1) * V_FL + ln * 2);
#pragma unroll
      for (int x = 0; x < 2 * NP; ++x) asm volatile("" : "+v"(acc[x]));
      if (k == nchunk - 1) {
        // partial output transform of rows 3 xh .. 3 xh + 2:  P = M A per row,
        // then Y[r] = sum_i A^T[r][3 xh + i] P[i]; the partner's channel pair to LDS
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          f32x2 P[3][4];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            f32x2 m[6];
#pragma unroll
            for (int j = 0; j < 6; ++j) m[j] = f32x2{acc[6 * i + j][2 * pp], acc[6 * i + j][2 * pp + 1]};
            at6(m, P[i]);
          }
          f32x2 Y[4][4];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            if (xh == 0) {
              const f32x2 s12 = P[1][x] + P[2][x], d12 = P[1][x] - P[2][x];
              Y[0][x] = P[0][x] + s12;
              Y[1][x] = d12;
              Y[2][x] = s12;
              Y[3][x] = d12;
            } else {
              Y[0][x] = P[0][x] + P[1][x];
              Y[1][x] = fmac(P[0][x], 0.5f, P[1][x] * f32x2{-2.f, -2.f});
              Y[2][x] = fmac(P[0][x], 0.25f, P[1][x] * f32x2{4.f, 4.f});
              Y[3][x] = fmac(P[0][x], 0.125f, fmac(P[1][x], -8.f, P[2][x]));
            }
          }
          if (pp == xh) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int x = 0; x < 4; ++x) own[r][x] = Y[r][x];
          } else {
            float* xw = xbuf + ((cb * 2 + (xh ^ 1)) * 8) * 256 + lane * 4;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
              for (int x = 0; x < 4; x += 2)
                *reinterpret_cast<f32x4*>(xw + (r * 2 + x / 2) * 256) =
                    f32x4{Y[r][x].x, Y[r][x].y, Y[r][x + 1].x, Y[r][x + 1].y};
          }
        }
      }
      __syncthreads();   // (B)
#ifdef WINO4S_STAMP
      if (g < 32) W4S_STAMP(28 + g);
#endif
    }
    if (il < 8) W4S_STAMP(4 + 3 * il);
    // ---- finish this wave's channel pair: own partial + the partner's
    int ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    f32x4 y[2][4];   // [channel of the pair][output row]: 4 pixels
    {
      const float* xr = xbuf + ((cb * 2 + xh) * 8) * 256 + ln * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int x = 0; x < 4; x += 2) {
          const f32x4 o = *reinterpret_cast<const f32x4*>(xr + (r * 2 + x / 2) * 256);
          const f32x2 q0 = own[r][x] + f32x2{o[0], o[1]}, q1 = own[r][x + 1] + f32x2{o[2], o[3]};
          y[0][r][x] = q0.x;
          y[1][r][x] = q0.y;
          y[0][r][x + 1] = q1.x;
          y[1][r][x + 1] = q1.y;
        }
    }
    const Item itm = wk.at(il);
    const int flatw = itm.blk * 16;
    const int smpl = flatw / TS;
    const bool part2 = itm.half != 0;          // second K half: raw sums to ksplit_buf
    const bool has_eb = !part2 && a.ebias != nullptr, has_res = !part2 && a.res != nullptr,
               has_bias = !part2 && a.bias != nullptr;
    const unsigned smp = (unsigned)(a.Cout * HW * 4);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (part2 ? a.ksplit_buf : a.out) + (size_t)smpl * a.Cout * HW, (short)0, smp, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        has_res ? const_cast<float*>(a.res) + (size_t)smpl * a.Cout * HW : nullptr, (short)0, smp,
        0x00020000);
    const int co0 = itm.cog * 64 + cb * 16 + 4 * (ln >> 4) + 2 * xh;
    const int tg = flatw % TS + (ln & 15);
    const int ty = tg / TPR, tx = tg - ty * TPR;
    const int vo = (co0 * HW + 4 * ty * WO + 4 * tx) * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float bi = has_bias ? a.bias[co0 + i] : 0.f;
      const float ei = has_eb ? a.ebias[(size_t)smpl * a.eb_stride + co0 + i] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        y[i][r] = y[i][r] + bi;
        if (has_eb) y[i][r] = y[i][r] + ei;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (has_res) {
      f32x4 rv[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          rv[i][r] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, vo, i * HW * 4 + r * WO * 4, 0));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) y[i][r] = y[i][r] + rv[i][r];
    }
    asm volatile("" ::"v"(rpf[0]), "v"(rpf[1]));   // (younger than the prefetch: it has landed)
    if (a.gnp && !part2) {
      float2 pr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float sm = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) sm += (y[i][r][0] + y[i][r][1]) + (y[i][r][2] + y[i][r][3]);
        sm = row16_sum(sm);
        const float mu = sm * (1.0f / 256.0f);
        float qq = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            const float d = y[i][r][x] - mu;
            qq = __builtin_fmaf(d, d, qq);
          }
        pr[i] = make_float2(sm, row16_sum(qq));
      }
      if ((ln & 15) == 0) {
        const int np = TS / 16, part = (flatw % TS) / 16;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          float2* d = a.gnp + ((size_t)smpl * a.Cout + co0 + i) * np + part;
          if constexpr (FOLD) st_f2_wt(d, pr[i]);
          else *d = pr[i];
        }
      }
      if constexpr (FOLD) gn_fold_item_done(a.fold, smpl, fold_items, 4 * XS, ln);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y[i][r]), ro, vo,
                                               i * HW * 4 + r * WO * 4, 0);
    if (il < 8) W4S_STAMP(5 + 3 * il);
  }
  W4S_STAMP(27);
  if constexpr (FOLD) wino4s_fold_tail(a.fold, lane, wave, 4 * XS);
  }

}

// xi split over two MFMA waves per co block (default; ERTD_WINO4S_XS=1 keeps
// one wave with all 36 xi, A/B): U2 B=64 240.5 -> 243.0 steps/s (same box,
// two alternations).  Needs Cin >= 16: the exchange buffer is reused across an
// item boundary only after a barrier that every wave passes between the two uses
static int wino4s_xs() {
  static const int v = [] {
    return ERTD_KNOB("WINO4S_XS", 2);
  }();
  return v;
}

}  // namespace

#ifdef WINO4S_STAMP
extern "C" int ertd_diag_wino4s_stamps(unsigned* host, size_t n) {
  const size_t cap = sizeof(g_w4s_stamps) / sizeof(unsigned);
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_w4s_stamps), (n < cap ? n : cap) * sizeof(unsigned), 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int ertd_diag_wino4s_stamps_clear() {
  static unsigned zero[256 * 12 * S4_SPW];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_w4s_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif

// ERTD_WINO4S_KSPLIT=0: no K split (a 16x16 layer whose items fill only half
// the CUs then runs F(2x2), as before)
static int wino4s_ks_env() {
  static const int v = [] {
    return ERTD_KNOB("WINO4S_KSPLIT", 1);
  }();
  return v;
}

// the xi-split kernel splits its K in two halves when its items fill half the
// CUs or more but not all of them (the 16x16 level of the B = 32 train step:
// 128 items of 64 co x 16 tiles for 256 CUs), given an even chunk count >= 4
bool wino4s_ksplit(int cin, int cout, int wo, int B) {
  if (!wino4s_ks_env() || wino4s_xs() != 2 || wo != 16 || cin % CCH || cout % 64) return false;
  const int nchunk = cin / CCH;
  const int items = wino4s_items(cout, wo, B), cus = device_cu_count();
  return nchunk % 2 == 0 && nchunk >= 4 && items < cus && 2 * items >= cus;
}

// contiguous walk (items bid * cw ...), diagnostic builds only:
// ERTD_WINO4S_CWALK=1 takes it for every xi-split layer that can.  Measured
// (U2 B=64, same box): 249.4 -> 243.8 steps/s -- the strided walk keeps the
// concurrently running items in a few samples (16 of 64 at 64x64), the
// contiguous one spreads them over all 64 at a 1-MB sample stride
static int wino4s_cwalk_env() {
  static const int v = [] {
    return ERTD_KNOB("WINO4S_CWALK", 0);
  }();
  return v;
}

// items per workgroup of the contiguous walk, or 0 where it does not apply:
// the xi-split kernel (Cin >= 16) without a K split, items an exact multiple of
// the grid, each workgroup's run inside one sample
static int wino4s_cw_geom(const ConvArgs& a, int wo, int B, int ksp, int cus) {
  if (ksp != 1 || wino4s_xs() != 2 || a.Cin < 16 || a.Cout % 64) return 0;
  const int nitems = wino4s_items(a.Cout, wo, B);
  const int grid = nitems < cus ? nitems : cus;
  if (grid < 1 || nitems % grid) return 0;
  const int cw = nitems / grid;
  const int per_sample = (wo / 4) * (wo / 4) / 16 * (a.Cout / 64);
  return per_sample % cw == 0 ? cw : 0;
}

namespace {

int wino4s_cwalk(const ConvArgs& a, int wo, int B, int ksp, int cus) {
  if (wino4s_cwalk_env() == 0 || a.fold.cnt) return 0;
  return wino4s_cw_geom(a, wo, B, ksp, cus);
}

template <int WO, int ACT, bool UP, int XS>
hipError_t launch_wo4x(const ConvArgs& a, int B, hipStream_t s, int cus, int ksp) {
  constexpr size_t lds = WLDS + (XS == 2 ? (size_t)4 * 2 * 8 * 256 * sizeof(float) : 0);
  const int nitems = wino4s_items(a.Cout, WO, B) * ksp;
  const int grid = nitems < cus ? nitems : cus;
  const int cw = wino4s_cwalk(a, WO, B, ksp, cus);
#ifdef ERTD_DIAG
  if (a.fold.cnt) {
    static std::atomic<unsigned long long> attr{0};
    set_max_lds_once((const void*)conv_wino4s_kernel<WO, ACT, UP, XS, true, false>, (int)lds, attr);
    conv_wino4s_kernel<WO, ACT, UP, XS, true, false><<<grid, 64 * (4 * XS + NPW), lds, s>>>(a, nitems, ksp, cw);
  } else
#else
  if (a.fold.cnt) return hipErrorInvalidValue;   // the fold is built into diagnostic libraries only
#endif
  if constexpr (XS == 2 && !UP && ACT != ACT_NONE) {
    if (a.gnc.pa) {
      const int nlocmax = (nitems + grid - 1) / grid;
      const size_t ldsg = lds + (size_t)(cw ? cw : nlocmax) * a.Cin * sizeof(float2);
      static std::atomic<unsigned long long> attr{0};
      set_max_lds_once((const void*)conv_wino4s_kernel<WO, ACT, UP, XS, false, true>,
                       (int)(lds + GNC_TAB * sizeof(float2)), attr);
      conv_wino4s_kernel<WO, ACT, UP, XS, false, true><<<grid, 64 * (4 * XS + NPW), ldsg, s>>>(a, nitems, ksp, cw);
      return hipGetLastError();
    }
  }
  if (a.gnc.pa) return hipErrorInvalidValue;
  {
    static std::atomic<unsigned long long> attr{0};
    set_max_lds_once((const void*)conv_wino4s_kernel<WO, ACT, UP, XS, false, false>, (int)lds, attr);
    conv_wino4s_kernel<WO, ACT, UP, XS, false, false><<<grid, 64 * (4 * XS + NPW), lds, s>>>(a, nitems, ksp, cw);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || ksp == 1) return e;
  return launch_add_inplace(a.out, a.ksplit_buf, (size_t)B * a.Cout * WO * WO, s);
}

template <int WO, int ACT, bool UP>
hipError_t launch_wo4s(const ConvArgs& a, int B, hipStream_t s, int cus) {
  if (wino4s_xs() == 2 && a.Cin >= 16) {
    // the split geometry (wino4s_ok's second case) always comes with its buffer:
    // without one the kernel would run unsplit on half the CUs -- refuse instead
    const bool spl = !UP && wino4s_ksplit(a.Cin, a.Cout, WO, B) && wino4s_items(a.Cout, WO, B) < cus;
    if (spl && !a.ksplit_buf) return hipErrorInvalidValue;
    const int ksp = spl ? 2 : 1;
    return launch_wo4x<WO, ACT, UP, 2>(a, B, s, cus, ksp);
  }
  return launch_wo4x<WO, ACT, UP, 1>(a, B, s, cus, 1);
}

template <int ACT>
hipError_t launch_act4s(const ConvArgs& a, int B, hipStream_t s, int cus) {
  switch (a.Wo) {
    case 16: return launch_wo4s<16, ACT, false>(a, B, s, cus);
    case 32: return launch_wo4s<32, ACT, false>(a, B, s, cus);
    case 64: return launch_wo4s<64, ACT, false>(a, B, s, cus);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

int wino4s_items(int cout, int wo, int B) { return (wo / 4) * (wo / 4) / 16 * B * (cout / 64); }

// the GroupNorm fold (ConvArgs::fold) rides on the emitted partials: items
// without a K split; every MFMA wave of an item arrives once
bool wino4s_fold_ok(const ConvArgs& a, bool up, int B) {
  if (a.Cin % CCH || a.Ca % 2 || a.Cout % 64) return false;
  (void)B;
  const int xs = wino4s_xs() == 2 && a.Cin >= 16 ? 2 : 1;
  if (xs == 2 && !up && wino4s_ksplit(a.Cin, a.Cout, a.Wo, B) && wino4s_items(a.Cout, a.Wo, B) < device_cu_count())
    return false;
  return true;
}
int wino4s_fold_target(const ConvArgs& a) { return (a.Wo / 4) * (a.Wo / 4) / 16 * (a.Cout / 64); }

// the consumer-side GroupNorm finalize (ConvArgs::gnc): a GN+act layer of the
// xi-split kernel without a K split (stride-1 only: the Upsample convs take no
// activation) whose finalize jobs fit the MFMA waves' registers and whose
// per-item tables fit the LDS, and whose workgroups run at most two items: the
// table costs the MFMA waves' prologue 2-4 us at four items per workgroup (the
// 64x64 layers, U2 B=64), more than the 3.3 us launch it replaces.  Same box,
// U2 B=64, three alternations: 250.1 steps/s without (ERTD_UNET_GNC=0), 251.9
// on every eligible layer (1), 252.1 at <= 2 items (3, the default; 2: one item)
bool wino4s_gnc_ok(const ConvArgs& a, int B) {
  static const int env = [] {
    return ERTD_KNOB("UNET_GNC", 3);
  }();
  const GnPartArgs& g = a.gnc;
  if (!env || wino4s_xs() != 2 || a.Cin < 16 || a.Cin % CCH || a.Ca % 2 || a.Cout % 64) return false;
  if (a.Wo != 16 && a.Wo != 32 && a.Wo != 64) return false;
  if (!g.pa || g.groups < 1 || g.Ca + g.Cb != a.Cin || a.Cin % g.groups || g.npa < 1 ||
      (g.Cb > 0 && (!g.pb || g.npb < 1)) || g.HW != a.Wo * a.Wo || g.HW % g.npa ||
      (g.Cb > 0 && g.HW % g.npb))
    return false;
  const int cus = device_cu_count();
  const bool spl = wino4s_ksplit(a.Cin, a.Cout, a.Wo, B) && wino4s_items(a.Cout, a.Wo, B) < cus;
  if (spl) return false;
  const int nitems = wino4s_items(a.Cout, a.Wo, B);
  const int grid = nitems < cus ? nitems : cus;
  const int nloc = wino4s_cwalk_env() ? wino4s_cw_geom(a, a.Wo, B, 1, cus) : (nitems + grid - 1) / grid;
  const int cpg = a.Cin / g.groups;
  const int np = g.npa > g.npb ? g.npa : g.npb;
  if (env == 2 && nloc > 1) return false;   // (diagnostic: single-item workgroups only)
  if (env == 3 && nloc > 2) return false;   // (diagnostic: at most two items per workgroup)
  return nloc > 0 && nloc * ((g.groups + 3) / 4) <= 8 * GNC_JM && cpg <= GN_LPG &&
         cpg * np <= GN_LPG * GNC_KM && nloc * a.Cin <= GNC_TAB;
}

// ERTD_WINO4S_UP=0 keeps the sub-pixel direct kernel for the Upsample convs (A/B)
bool wino4s_up_ok(int cin, int ca, int cout, int wo, int B) {
  static const int env = [] {
    return ERTD_KNOB("WINO4S_UP", 1);
  }();
  // (at 16x16 only where the items fill the CUs: the Upsample conv has no K split)
  return env != 0 && wino4s_ok(cin, ca, cout, wo, B) && (wo == 16 || wo == 32 || wo == 64) &&
         (wo != 16 || wino4s_items(cout, wo, B) >= device_cu_count());
}

hipError_t launch_conv_wino4s(int act, const ConvArgs& a, int B, hipStream_t s, int cus) {
  if (a.Cin % CCH || a.Ca % 2 || a.Cout % 64 || !a.wpk_wino4 || a.Ho != a.Wo || a.Hs != a.Ws)
    return hipErrorInvalidValue;
  if (a.Hs * 2 == a.Wo) {   // Upsample conv (no activation)
    if (act != ACT_NONE) return hipErrorInvalidValue;
    switch (a.Wo) {
      case 16: return launch_wo4s<16, ACT_NONE, true>(a, B, s, cus);
      case 32: return launch_wo4s<32, ACT_NONE, true>(a, B, s, cus);
      case 64: return launch_wo4s<64, ACT_NONE, true>(a, B, s, cus);
      default: return hipErrorInvalidValue;
    }
  }
  if (a.Hs != a.Wo) return hipErrorInvalidValue;
  switch (act) {
    case ACT_NONE: return launch_act4s<ACT_NONE>(a, B, s, cus);
    case ACT_GN_SILU: return launch_act4s<ACT_GN_SILU>(a, B, s, cus);
    case ACT_GN: return launch_act4s<ACT_GN>(a, B, s, cus);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet
}  // namespace ertd
