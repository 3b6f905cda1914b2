// 3x3 stride-1 convolution of the U-Net ResBlocks by Winograd F(4x4, 3x3) on
// fp32 MFMA (v_mfma_f32_16x16x4_f32): 36 multiplies per 16 outputs instead of
// F(2x2,3x3)'s 16 per 4 (unet_conv_wino.hip) -- 1.78x less MFMA work, 4x less
// than the direct implicit GEMM.  GroupNorm + SiLU fused into the input
// transform, bias / embedding / residual into the output transform, as in the
// F(2x2) kernel.
//
// Interpolation points {0, 1, -1, 1/2, -2, inf} (Toom-Cook): the best fp32
// accuracy of the F(4,3) point sets we measured (1.5e-6 rel-L2 per layer vs
// 2.3e-6 for {0, +-1, +-2}; F(2x2) 3.5e-7, direct 2.1e-7):
//   V = B^T d B (d = the 6x6 input window at rows 4ty-1.., cols 4tx-1.., zero
//       outside the image, AFTER the activation)
//   U = G g G^T (3x3 kernel, float64 at pack time, rounded once)
//   M[xi] = sum_c U[xi][co][c] V[xi][c][tile]            (36 GEMMs)
//   Y = A^T M A
// All arithmetic fp32; the forward stays within 1e-5 of the spec (tests).
//
// Work item = (64 output channels, 32 tiles = 512 output pixels: one sample's,
// or two samples' at W = 16), all
// 36 xi, K walked in chunks of 4 input channels (one MFMA k-step).  Persistent
// and warp-specialized like the F(2x2) kernel: one 768-thread workgroup per CU
// walks items bid, bid + grid, ... as one continuous chunk pipeline.
//   * 8 MFMA waves: wave w = (16-co block w & 3, 16-tile block w >> 2) keeps
//     ALL 36 xi of its 16 co x 16 tiles in 36 accumulators (144 VGPRs); per
//     chunk and xi one ds_read_b32 of U, one of V, one MFMA (consecutive MFMAs
//     are independent; the U / V layouts keep xi pairs adjacent, so one
//     ds_read_b64 per operand feeds two MFMAs).  They LDS-DMA the U slices
//     ([xi/2 18][co block 4][k 4][co 16][xi&1] = 36 KB per chunk) two chunks
//     ahead into a 3-slot ring.
//   * 4 producer waves: wave q = channel q of every chunk; lane = (tile t =
//     lane & 31, column half h = lane >> 5).  A lane loads its tile's window
//     columns 1+2h, 2+2h (one float2 per row, six rows, four chunks ahead in
//     three register sets), applies GroupNorm+SiLU, takes the outer column
//     from the neighbouring tile's other half (ds_bpermute), transforms its
//     three columns over the rows (B^T d), swaps rows with the other half
//     (v_permlane32_swap: afterwards lane half h holds xi rows 3h..3h+2 of all
//     six columns) and finishes (.. B): 18 V values, one ds_write_b64 per
//     xi pair, into V [xi/2][tile block 2][k 4][tile 16][xi&1] (18 KB,
//     double-buffered).
//   * Output transform (MFMA waves, registers, packed fp32 over co pairs):
//     Y = A^T M A per (co, tile), + bias (+ emb) (+ residual), float4 stores.
// LDS 144 KB: one workgroup per CU.
#include <cstdlib>
#include <type_traits>

#include "unet.h"

namespace ertd {
namespace unet {

namespace {

constexpr int NMW = 8;                        // MFMA waves
constexpr int NPW = 4;                        // producer waves
constexpr int WT = 64 * (NMW + NPW);          // threads per workgroup (768)
constexpr int WKC = 4;                        // input channels per K chunk
constexpr int NX = 36;                        // transformed positions
constexpr int U_FL = NX * 256;                // U floats per chunk (9216)
constexpr int V_FL = NX * 128;                // V floats per chunk (4608)
constexpr int NUB = 3;                        // U ring depth (DMA two chunks ahead)
constexpr int NRS = 3;                        // producer register sets
constexpr size_t WLDS = (size_t)(NUB * U_FL + 2 * V_FL) * sizeof(float);   // 144 KB
constexpr int NDMA = U_FL / 256;              // 1-KB DMA instructions per chunk (36)
static_assert(NDMA == 4 * 5 + 4 * 4, "waves 0-3 issue 5 DMAs per chunk, waves 4-7 issue 4");
#ifndef WINO4_PPRIO
#define WINO4_PPRIO 2                         // producer wave priority (s_setprio)
#endif
#ifndef WINO4_PD
#define WINO4_PD 2                            // MFMA operand read-ahead (xi pairs)
#endif
#ifndef WINO4_DMAI
#define WINO4_DMAI 1                          // U DMA interleaved with the MFMAs (0: all after the barrier)
#endif
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;

// Transforms of the points {0, 1, -1, 1/2, -2, inf} (bt6 / at6 below apply them):
//   B^T = [1 -1.5 -2  1.5 1   0]     A^T = [1 1  1 1     1  0]
//         [0 -1   0.5 2.5 1   0]           [0 1 -1 0.5  -2  0]
//         [0  1  -2.5 0.5 1   0]           [0 1  1 0.25  4  0]
//         [0 -2  -1   2   1   0]           [0 1 -1 0.125 -8 1]
//         [0  0.5 -1 -0.5 1   0]
//         [0  1  -1.5 -2  1.5 1]
// G (float64, pack time): rows of the same points
constexpr double GD[6][3] = {{1.0, 0.0, 0.0},
                             {1.0 / 3, 1.0 / 3, 1.0 / 3},
                             {-1.0 / 3, 1.0 / 3, -1.0 / 3},
                             {-16.0 / 15, -8.0 / 15, -4.0 / 15},
                             {1.0 / 15, -2.0 / 15, 4.0 / 15},
                             {0.0, 0.0, 1.0}};

__device__ __forceinline__ f32x2 fmac(f32x2 x, float c, f32x2 s) {
  return __builtin_elementwise_fma(x, f32x2{c, c}, s);
}
// o = B^T d for one 6-vector, common subexpressions shared (16 ops, not 20)
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
// y = A^T m for one 6-vector (packed over a co pair)
__device__ __forceinline__ void at6(const f32x2 (&m)[6], f32x2 (&y)[4]) {
  const f32x2 s = m[1] + m[2], d = m[1] - m[2];
  y[0] = (m[0] + s) + (m[3] + m[4]);
  y[1] = fmac(m[3], 0.5f, fmac(m[4], -2.f, d));
  y[2] = fmac(m[3], 0.25f, fmac(m[4], 4.f, s));
  y[3] = fmac(m[3], 0.125f, fmac(m[4], -8.f, d + m[5]));
}

__device__ __forceinline__ unsigned wlds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

#ifdef WINO4_STAMP
// Diagnostic build only (tools/wino4_stamps.py): per-wave s_memtime stamps of
// the first NSS chunks, staged in the 16 KB of LDS above the ring and copied to
// g_w4stamps at the end.  Per wave: [0] s_memrealtime, [1] s_memtime at entry,
// then NSS x 5 events.
constexpr int NSS = 64;
constexpr int SPW = 2 + NSS * 5;
__device__ unsigned g_w4stamps[256 * 12 * SPW];
#define W4STAMP(ev, sl)                                                                  \
  do {                                                                                   \
    if (lane == 0 && (sl) < NSS)                                                         \
      stamps[wave * SPW + 2 + (sl) * 5 + (ev)] = (unsigned)__builtin_amdgcn_s_memtime(); \
  } while (0)
constexpr size_t WLDS_LAUNCH = WLDS + 12 * SPW * sizeof(unsigned);
#else
#define W4STAMP(ev, sl) \
  do {                  \
  } while (0)
constexpr size_t WLDS_LAUNCH = WLDS;
#endif

// item it -> (co block, tile block): co block fastest; tile block blk covers
// tiles [32 blk, 32 blk + 32) of the batch's tiles in (sample, row, column)
// order -- within one sample at W >= 32, two whole samples at W = 16
struct Item {
  int cog, blk;
};
__device__ __forceinline__ Item item_of(int it, int ncog) {
  Item r;
  r.cog = it % ncog;
  r.blk = it / ncog;
  return r;
}

// DBG (diagnostics only, ERTD_WINO4_DBG; results wrong): bit 0 skips the
// producers' transform, bit 1 their loads, bit 2 the U DMA, bit 3 the MFMAs,
// bit 4 the MFMA waves' LDS reads, bit 5 the output transform and stores
template <int WO, int ACT, int DBG = 0>
__global__ __launch_bounds__(WT) void conv_wino4_kernel(ConvArgs a, int nitems, int ksp) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* ubuf = smem;                 // [3][U_FL] ring
  float* vbuf = smem + NUB * U_FL;    // [2][V_FL]

  constexpr int TPR = WO / 4;         // tiles per tile row
  constexpr int HW = WO * WO;
  constexpr int TS = TPR * TPR;       // tiles per sample
  static_assert(TPR >= 4 && (TS % 32 == 0 || 32 % TS == 0), "a 32-tile block is whole tile rows");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int Cin = a.Cin, Ca = a.Ca;
  const int nchunk = Cin / WKC;
  // ksp = 2: work item it = 2 x (tile item) + half, as in conv_wino_kernel
  const int nck = nchunk / ksp;
  const int ncog = a.Cout / 64;
  const int bid = blockIdx.x, G = gridDim.x;
  const int nloc = bid < nitems ? (nitems - bid + G - 1) / G : 0;
  const int gtot = nloc * nck;
#ifdef WINO4_STAMP
  unsigned* stamps = reinterpret_cast<unsigned*>(smem + NUB * U_FL + 2 * V_FL);
  if (lane == 0) {
    stamps[wave * SPW] = (unsigned)__builtin_amdgcn_s_memrealtime();
    stamps[wave * SPW + 1] = (unsigned)__builtin_amdgcn_s_memtime();
  }
  auto stamp_flush = [&]() {
    __builtin_amdgcn_s_waitcnt(0);
    for (int i = lane; i < SPW; i += 64)
      g_w4stamps[((size_t)bid * 12 + wave) * SPW + i] = stamps[wave * SPW + i];
  };
#endif

  if (wave >= NMW) {
    // =================== producer waves ===================
    // the producers issue ahead of the MFMA waves on a shared SIMD: their
    // transform is the chunk's critical path (U2 B=64: 185.0 -> 189.2 steps/s)
    __builtin_amdgcn_s_setprio(WINO4_PPRIO);
    const int q = wave - NMW;          // channel q of every chunk (MFMA k row q)
    const int h = lane >> 5, t = lane & 31;
    // V offset of (xi pair 9h, tile t, k q): [xi/2][t >> 4][q][t & 15][xi&1]
    const int vwoff = ((h * 18 + (t >> 4)) * 64 + q * 16 + (t & 15)) * 2;
    // the outer window column: lower half (left, column 0) from tile t-1's
    // upper half, upper half (right, column 5) from tile t+1's lower half
    const int nbaddr = (lane + 31 - 62 * h) * 4;
    float2 raw[NRS][6];      // [register set][row]: window columns 1+2h, 2+2h
    float2 gnv[NRS];         // {scale, shift} of the channel
    f32x4 pad[NRS];          // row 0, row 5, outer column, -
    int cur_g = 0, cur_k = 0, cur_k0 = 0, cur_b = 0, cur_il = 0;
    unsigned roff[6];
    unsigned soffA = 0, soffB = 0;   // W = 16: lanes 16..31 read the block's second sample
    f32x4 cur_pad;
    auto set_item = [&](int il) {
      const int it = bid + il * G;
      cur_k0 = (it % ksp) * nck;
      const Item itm = item_of(it / ksp, ncog);
      const int flat0 = itm.blk * 32;
      cur_b = flat0 / TS;                       // the block's first sample
      const int tg = (flat0 + t) % TS;          // tile within its sample
      if constexpr (TS < 32) {
        const int ls = (flat0 + t) / TS - cur_b;
        soffA = (unsigned)(ls * Ca * HW * 4);
        soffB = (unsigned)(ls * a.Cb * HW * 4);
      }
      const int ty = tg / TPR, tx = tg - ty * TPR;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const int iy = 4 * ty - 1 + r;
        roff[r] = (unsigned)(((iy >= 0 && iy < WO ? iy : 4 * ty) * WO + 4 * tx + 2 * h) * 4);
      }
      cur_pad = f32x4{ty > 0 ? 1.f : 0.f, ty < TPR - 1 ? 1.f : 0.f,
                      (h ? tx < TPR - 1 : tx > 0) ? 1.f : 0.f, 0.f};
    };
    const int glast = gtot - 1;
    auto load_next = [&](const int set) {
      const int cg = (cur_k0 + cur_k) * WKC + q;     // wave-uniform channel
      pad[set] = cur_pad;
      if constexpr (ACT != ACT_NONE) {
        if constexpr (TS < 32) gnv[set] = a.gn[(size_t)(cur_b + (t >= TS)) * Cin + cg];
        else gnv[set] = a.gn[(size_t)cur_b * Cin + cg];
      }
      const bool inA = cg < Ca;
      const float* p = inA ? a.srcA + ((size_t)cur_b * Ca + cg) * HW
                           : a.srcB + ((size_t)cur_b * a.Cb + (cg - Ca)) * HW;
      const unsigned soff = TS < 32 ? (inA ? soffA : soffB) : 0u;
      const int nrec = TS < 32 ? ((inA ? Ca : a.Cb) + 1) * HW * 4 : HW * 4;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, nrec, 0x00020000);
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        if constexpr (DBG & 2) {
          raw[set][r] = make_float2((float)(r + cur_k), (float)lane);
        } else {
          const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(roff[r] + soff), 0, 0);
          raw[set][r] = make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
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
    // Two stages, software-pipelined one chunk apart so that each slot holds
    // two independent dependency chains (a lone producer wave per SIMD is
    // latency-bound otherwise): act (GroupNorm + SiLU + padding + the outer
    // column by ds_bpermute: 18 values into an act buffer) for chunk g+2 and
    // tr (the transform, the row swap, the V stores) for chunk g+1.
    float act[2][3][6];      // [buffer][local column (1+2h, 2+2h, outer)][row]
    auto act_stage = [&](const int set, const int ab) {
      if constexpr (DBG & 1) return;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        float2 m = raw[set][r];
        if constexpr (ACT != ACT_NONE) {
          m.x = __builtin_fmaf(m.x, gnv[set].x, gnv[set].y);   // ATen's folded GroupNorm
          m.y = __builtin_fmaf(m.y, gnv[set].x, gnv[set].y);
          if constexpr (ACT == ACT_GN_SILU) {
            m.x = m.x * __builtin_amdgcn_rcpf(1.0f + __expf(-m.x));
            m.y = m.y * __builtin_amdgcn_rcpf(1.0f + __expf(-m.y));
          }
        }
        // the padding pads the activated tensor
        if (r == 0 || r == 5) {
          const float fy = r == 0 ? pad[set].x : pad[set].y;
          m.x *= fy;
          m.y *= fy;
        }
        const float give = h ? m.y : m.x;
        const float nb = __int_as_float(__builtin_amdgcn_ds_bpermute(nbaddr, __float_as_int(give)));
        act[ab][0][r] = m.x;
        act[ab][1][r] = m.y;
        act[ab][2][r] = nb * pad[set].z;
      }
    };
    auto tr_stage = [&](const int ab, float* vb) {
      if constexpr (DBG & 1) return;
      // B^T d on the three local columns
      float w[6][3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float o[6];
        bt6(act[ab][c], o);
#pragma unroll
        for (int i = 0; i < 6; ++i) w[i][c] = o[i];
      }
      // rows 0-2 to the lower half, 3-5 to the upper: afterwards row[a][j] is
      // row 3h+a of window column j (the lower half's local columns are
      // window columns {1,2,0}, the upper half's 3,4,5)
      float row[3][6];
#pragma unroll
      for (int aa = 0; aa < 3; ++aa)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(w[aa][c]),
                                                           __float_as_uint(w[3 + aa][c]), false, false);
          const int jl = c == 0 ? 1 : (c == 1 ? 2 : 0);
          row[aa][jl] = __uint_as_float(sw[0]);
          row[aa][3 + c] = __uint_as_float(sw[1]);
        }
      // (B^T d) B: V[3h+a][j'] = sum_j B^T[j'][j] row[a][j]
      float* o = vb + vwoff;
#pragma unroll
      for (int aa = 0; aa < 3; ++aa) {
        float vv[6];
        bt6(row[aa], vv);
#pragma unroll
        for (int jp = 0; jp < 6; jp += 2)
          *reinterpret_cast<f32x2*>(o + (aa * 3 + jp / 2) * 256) = f32x2{vv[jp], vv[jp + 1]};
      }
    };
    // slot g: tr(chunk g+1) -> V[(g+1)&1]; act(chunk g+2, register set (g+2)%3)
    // -> act[g&1]; reload that set with chunk g+5; barrier.  Register sets and
    // act buffers are compile-time indices: the loop is unrolled by 6.
    auto slot = [&](auto sa, auto ab, int g) {
      constexpr int SA = decltype(sa)::value, AB = decltype(ab)::value;
      W4STAMP(0, g);
      tr_stage(AB ^ 1, vbuf + ((g + 1) & 1) * V_FL);
      W4STAMP(1, g);
      act_stage(SA, AB);
      W4STAMP(4, g);
      load_next(SA);
      W4STAMP(2, g);
      __syncthreads();   // (B) end of slot g
      W4STAMP(3, g);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    if (gtot > 0) {
      set_item(0);
      load_next(0);
      load_next(1);
      load_next(2);
      act_stage(0, 0);
      tr_stage(0, vbuf);
      load_next(0);      // chunk 3
      act_stage(1, 1);
      load_next(1);      // chunk 4
    }
    __syncthreads();   // (A) chunk 0 staged
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
#ifdef WINO4_STAMP
    stamp_flush();
#endif
    return;
  }

  // =================== MFMA waves ===================
#ifdef WINO4_MPRIO
  __builtin_amdgcn_s_setprio(WINO4_MPRIO);
#endif
  const int cb = wave & 3, tb = wave >> 2;
  f32x4 acc[NX];
  // U slice DMA of chunk g into ring slot g % 3 (36 x 1 KB: waves 0-3 five,
  // waves 4-7 four); the MFMA waves issue no other vector memory operation in
  // the K loop, so vmcnt(own count) = "the previous slot's slice has landed"
  const int ndma = wave < 4 ? 5 : 4;
  const int dfirst = wave < 4 ? wave * 5 : 20 + (wave - 4) * 4;
  // DMA cursor (wave-uniform, scalar): the chunk whose U slice goes out next
  // (chunk g + 2 while chunk g computes): item d_il, chunk d_k of its K range.
  // The item's base pointer is formed once per item -- per chunk only an add
  // (the per-chunk integer divisions cost ~700 cycles of issue per chunk).
  int d_k = 0, d_il = 0;
  const float* d_src = a.wpk_wino4;
  auto d_item = [&](int il) {
    const int it = bid + il * G;
    d_src = a.wpk_wino4 + ((size_t)((it / ksp) % ncog) * nchunk + (size_t)(it % ksp) * nck) * U_FL;
  };
  if (nloc > 0) d_item(0);
  // DMA instruction j (1 KB) of the cursor's chunk into ring slot `slot`
  auto dma_one = [&](const int j, const int slot) {
    if constexpr (DBG & 4) return;
    int ln;   // a fresh lane id: one held across the item loop was spilled
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    const int ins = dfirst + j;
    const float* src = d_src + (size_t)d_k * U_FL + ins * 256 + ln * 4;
    const unsigned ldst = __builtin_amdgcn_readfirstlane(wlds_addr(ubuf + slot * U_FL + ins * 256));
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(ldst)
        : "memory");
  };
  auto dma_advance = [&]() {
    if (++d_k == nck) {
      d_k = 0;
      if (++d_il < nloc) d_item(d_il);
    }
  };
  auto dma_all = [&](const int slot) {
#pragma unroll
    for (int j = 0; j < 5; ++j)
      if (j < 4 || wave < 4) dma_one(j, slot);
    dma_advance();
  };
  if (gtot > 0) dma_all(0);
  if (gtot > 1) dma_all(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // (A)
  int su = 0, sd = 2;   // ring slots of the computed chunk (g % 3) and of the DMA'd one ((g + 2) % 3)
  for (int il = 0; il < nloc; ++il) {
#pragma unroll
    for (int x = 0; x < NX; ++x) acc[x] = f32x4{};
    for (int k = 0; k < nck; ++k) {
      const int g = il * nck + k;
      const bool dma = g + 2 < gtot;
      W4STAMP(0, g);
#if !WINO4_DMAI
      if (dma) dma_all(sd);
#endif
      W4STAMP(1, g);
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      const float* ub = ubuf + su * U_FL + (cb * 64 + ln) * 2;
      const float* vb = vbuf + (g & 1) * V_FL + (tb * 64 + ln) * 2;
      constexpr int PD = WINO4_PD;   // xi pairs read ahead
      f32x2 ra[PD + 1], rb[PD + 1];
      auto ld = [&](const int xp) {
        const int r = xp % (PD + 1);
        if constexpr (DBG & 16) {
          ra[r] = f32x2{(float)(ln + xp), (float)k};
          rb[r] = f32x2{(float)(xp - ln), 1.f};
        } else {
          ra[r] = *reinterpret_cast<const f32x2*>(ub + xp * 512);
          rb[r] = *reinterpret_cast<const f32x2*>(vb + xp * 256);
        }
      };
#pragma unroll
      for (int xp = 0; xp < PD; ++xp) ld(xp);
#pragma unroll
      for (int xp = 0; xp < NX / 2; ++xp) {
        if (xp + PD < NX / 2) ld(xp + PD);
        const int r = xp % (PD + 1);
        if constexpr (DBG & 8) {
          acc[2 * xp][0] += ra[r].x * rb[r].x;
          acc[2 * xp + 1][0] += ra[r].y * rb[r].y;
        } else {
          acc[2 * xp] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[r].x, rb[r].x, acc[2 * xp], 0, 0, 0);
          acc[2 * xp + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[r].y, rb[r].y, acc[2 * xp + 1], 0, 0, 0);
        }
        if (xp + PD < NX / 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);   // DS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                          // MFMAs
#if WINO4_DMAI
        // the next-but-one chunk's U slice, one 1-KB DMA after each of the
        // first MFMA pairs: its issue cost (~140 cycles each) hides behind the
        // MFMAs instead of holding every MFMA wave for ~700 cycles after the
        // barrier, when no MFMA is in flight
        if (xp >= 1 && xp <= 5 && (xp <= 4 || wave < 4))
          if (dma) dma_one(xp - 1, sd);
#endif
      }
#if WINO4_DMAI
      if (dma) dma_advance();
#endif
      su = su == NUB - 1 ? 0 : su + 1;
      sd = sd == NUB - 1 ? 0 : sd + 1;
#pragma unroll
      for (int x = 0; x < NX; ++x) asm volatile("" : "+v"(acc[x]));
      W4STAMP(2, g);
      if (dma) {
        if (wave < 4) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      W4STAMP(4, g);
      __syncthreads();   // (B)
      W4STAMP(3, g);
    }

    if constexpr (DBG & 32) {
      if (il == nloc - 1) {
        float sacc = 0.f;
        for (int x = 0; x < NX; ++x) sacc += acc[x][0] + acc[x][3];
        a.out[(size_t)bid * 64 + lane] = sacc;
      }
      continue;
    }
    // ---- output transform: lane l holds M[xi] of co = 16 cb + 4 (l >> 4) + i
    // (accumulator element i) and tile 16 tb + (l & 15)
    const int itg = bid + il * G;
    const Item itm = item_of(itg / ksp, ncog);
    const int flatw = itm.blk * 32 + tb * 16;   // this wave's 16 tiles: one sample
    const int smpl = flatw / TS;
    const bool part2 = (itg % ksp) != 0;
    const bool has_eb = a.ebias && !part2, has_res = a.res && !part2, has_bias = a.bias && !part2;
    const unsigned smp = (unsigned)(a.Cout * HW * 4);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (part2 ? a.ksplit_buf : a.out) + (size_t)smpl * a.Cout * HW, (short)0, smp, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        has_res ? const_cast<float*>(a.res) + (size_t)smpl * a.Cout * HW : nullptr, (short)0, smp,
        0x00020000);
    // the transform first (bias, emb and addresses after it: fewer live
    // registers while the accumulators drain); y[i][r] = output row r
    // (4 pixels) of co0 + i; co pairs (0,1), (2,3) as packed fp32
    f32x4 y[4][4];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      f32x2 P[6][4];   // P = M A, per xi row
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
    // conv + bias, + emb (the spec's op order; the residual is added by the caller)
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
    // residual loads all issued before any store (loads and stores share vmcnt)
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
    // GroupNorm partials of the output: the 16 lanes of a DPP row hold 16 tiles
    // x 16 px = 256 pixels of one sample for the same 4 channels.  Before the
    // output stores: anything after them that reloads a spilled value waits
    // (shared vmcnt) for every store of the item
    if (a.gnp && ksp == 1) {
      float2 pr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float sm = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) sm += (y[i][r][0] + y[i][r][1]) + (y[i][r][2] + y[i][r][3]);
        sm = row16_sum(sm);
        const float mu = sm * (1.0f / 256.0f);
        float q = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            const float d = y[i][r][x] - mu;
            q = __builtin_fmaf(d, d, q);
          }
        pr[i] = make_float2(sm, row16_sum(q));
      }
      if ((ln & 15) == 0) {
        const int np = TS / 16, part = (flatw % TS) / 16;
#pragma unroll
        for (int i = 0; i < 4; ++i) a.gnp[((size_t)smpl * a.Cout + co0 + i) * np + part] = pr[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y[i][r]), ro, vo,
                                               i * HW * 4 + r * WO * 4, 0);
  }
#ifdef WINO4_STAMP
  stamp_flush();
#endif
}

// ---- packing: W (Cout, Cin, 3, 3) -> U = G g G^T in [cog][chunk][xi/2 18][cb 4][k 4][co 16][xi&1]
// (float64, rounded once): the A-operand fragments of v_mfma_f32_16x16x4_f32,
// lane l = 16 k + c16 -> co = 16 cb + c16, channel k of the chunk
__global__ void pack_wino4_kernel(const float* __restrict__ w, int cin, int cout, int nchunk,
                                  size_t total, float* __restrict__ dst, bool flipT) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int e = (int)(i & 1);
  const int c16 = (int)((i >> 1) & 15);
  const int kk = (int)((i >> 5) & 3);
  const int cb = (int)((i >> 7) & 3);
  size_t rest = i >> 9;
  const int xi = 2 * (int)(rest % (NX / 2)) + e;
  rest /= NX / 2;
  const int k = (int)(rest % nchunk);
  const int cog = (int)(rest / nchunk);
  const int co = cog * 64 + cb * 16 + c16;
  const int ci = k * WKC + kk;
  const int ri = xi / 6, rj = xi % 6;
  const float* g = flipT ? w + ((size_t)ci * cout + co) * 9 : w + ((size_t)co * cin + ci) * 9;
  double u = 0.0;
#pragma unroll
  for (int y = 0; y < 3; ++y) {
    double row = 0.0;
#pragma unroll
    for (int x = 0; x < 3; ++x) row += (double)(flipT ? g[8 - (y * 3 + x)] : g[y * 3 + x]) * GD[rj][x];
    u += GD[ri][y] * row;
  }
  dst[i] = (float)u;
}

template <int WO, int ACT, int DBG>
hipError_t launch_wo4d(const ConvArgs& a, int B, hipStream_t s, int cus) {
  static std::atomic<unsigned long long> attr{0};
  set_max_lds_once((const void*)conv_wino4_kernel<WO, ACT, DBG>, (int)WLDS_LAUNCH, attr);
  const int base = wino4_tile_items(a.Cout, a.Wo, B);
  const int ksp = wino4_ksplit(a.Cin, a.Cout, a.Wo, B) && a.ksplit_buf ? 2 : 1;
  const int nitems = base * ksp;
  const int grid = nitems < cus ? nitems : cus;
  conv_wino4_kernel<WO, ACT, DBG><<<grid, WT, WLDS_LAUNCH, s>>>(a, nitems, ksp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || ksp == 1) return e;
  const size_t n = (size_t)B * a.Cout * WO * WO;
  return launch_add_inplace(a.out, a.ksplit_buf, n, s);
}

#ifdef ERTD_DIAG
// ablation variants (results wrong): only in a diagnostic build of the library
// (tools/build_variant.sh ... "-DERTD_DIAG"), never in the shipped one
int wino4_dbg() {
  static int v = [] {
    return ERTD_KNOB("WINO4_DBG", 0);
  }();
  return v;
}
#endif

template <int WO, int ACT>
hipError_t launch_wo4(const ConvArgs& a, int B, hipStream_t s, int cus) {
#ifdef ERTD_DIAG
  if constexpr (WO == 64 && ACT == ACT_GN_SILU) {
    switch (wino4_dbg()) {
      case 1: return launch_wo4d<WO, ACT, 1>(a, B, s, cus);
      case 2: return launch_wo4d<WO, ACT, 2>(a, B, s, cus);
      case 3: return launch_wo4d<WO, ACT, 3>(a, B, s, cus);
      case 4: return launch_wo4d<WO, ACT, 4>(a, B, s, cus);
      case 8: return launch_wo4d<WO, ACT, 8>(a, B, s, cus);
      case 16: return launch_wo4d<WO, ACT, 16>(a, B, s, cus);
      case 32: return launch_wo4d<WO, ACT, 32>(a, B, s, cus);
      case 7: return launch_wo4d<WO, ACT, 7>(a, B, s, cus);
      case 23: return launch_wo4d<WO, ACT, 23>(a, B, s, cus);
      default: break;
    }
  }
#endif
  return launch_wo4d<WO, ACT, 0>(a, B, s, cus);
}

template <int ACT>
hipError_t launch_act4(const ConvArgs& a, int B, hipStream_t s, int cus) {
  switch (a.Wo) {
    case 16: return launch_wo4<16, ACT>(a, B, s, cus);
    case 32: return launch_wo4<32, ACT>(a, B, s, cus);
    case 64: return launch_wo4<64, ACT>(a, B, s, cus);
    case 128: return launch_wo4<128, ACT>(a, B, s, cus);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

#ifdef WINO4_STAMP
extern "C" int ertd_diag_wino4_stamps(unsigned* host, size_t n) {
  const size_t cap = sizeof(g_w4stamps) / sizeof(unsigned);
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_w4stamps), (n < cap ? n : cap) * sizeof(unsigned), 0,
                                  hipMemcpyDeviceToHost);
}
#endif

int wino4_tile_items(int cout, int wo, int B) { return (wo / 4) * (wo / 4) * B / 32 * (cout / 64); }

size_t conv_packed_floats_wino4(int cin, int cout) {
  if (cin % WKC || cout % 64) return 0;
  return (size_t)NX * cout * cin;
}

hipError_t launch_pack_conv_wino4(const float* w, int cin, int cout, float* dst, hipStream_t s,
                                  bool flipT) {
  const size_t total = conv_packed_floats_wino4(cin, cout);
  if (!total) return hipErrorInvalidValue;
  pack_wino4_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(w, cin, cout, cin / WKC, total, dst,
                                                                     flipT);
  return hipGetLastError();
}

hipError_t launch_conv_wino4(int act, const ConvArgs& a, int B, hipStream_t s, int cus) {
  switch (act) {
    case ACT_NONE: return launch_act4<ACT_NONE>(a, B, s, cus);
    case ACT_GN_SILU: return launch_act4<ACT_GN_SILU>(a, B, s, cus);
    case ACT_GN: return launch_act4<ACT_GN>(a, B, s, cus);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet
}  // namespace ertd
