// 1x1 convolution (the ResBlock skip projections, SURVEY 8a') as a batched
// GEMM on v_mfma_f32_32x32x2_f32:
//   out[b][co][p] = bias[co] + sum_ci W[co][ci] x[b][ci][p]      (x = cat(srcA, srcB))
//
// Persistent workgroups (two per CU) walk (MT co x NT px) output tiles of one
// sample each, 4 waves in a 2 x 2 grid, wave tile (MT/2 x NT/2) = TI x TJ blocks of 32 x 32 (TI * TJ * 16
// accumulator VGPRs).  K runs in chunks of 32 input channels, double-buffered
// in LDS:
//   * X chunk [32 ci][NT px], float4 rows straight from the NCHW input (the two
//     inputs of a skip concatenation read in place);
//   * W chunk: the direct packing's [co tile 32][chunk][step pair 8][lane 64][2]
//     block (unet_pack.h, 4 KB per 32 co) copied as is -- its K order is the
//     MFMA's: k-step s of lane half h is channel 32 chunk + 16 h + s, so a
//     lane's A operands of two consecutive k-steps are one ds_read_b64 and its
//     B operand of k-step s is row 16 h + s of the X chunk (conflict-free).
// The next chunk's global loads are in flight during the current chunk's
// MFMAs and land in the other buffer after them (one barrier per chunk).
// Round 1-5 kernels for these shapes (the implicit GEMM conv_kernel<1, ...>
// and conv1x1_kernel) ran the U2 skips at 48-56 % of the fp32 peak.
// Exact fp32 products; per output the accumulation runs over the channels in
// the fixed order above, the same for every batch size and member offset.
#include "unet.h"
#include "unet_pack.h"

namespace ertd {
namespace unet {

namespace {

constexpr int KC = 32;                      // input channels per chunk
constexpr int SG_THREADS = 256;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int MT, int NT>
struct SgGeom {
  static constexpr int TI = MT / 64, TJ = NT / 64;      // 32x32 blocks per wave (2 x 2 waves)
  static constexpr int XF = KC * NT;                    // X floats per chunk
  static constexpr int WF = MT / 32 * 1024;             // W floats per chunk
  static constexpr int XV = XF / 4 / SG_THREADS;        // float4 loads per thread
  static constexpr int WV = WF / 4 / SG_THREADS;
  static constexpr size_t LDS = (size_t)2 * (XF + WF) * sizeof(float);
  static_assert(TI >= 1 && TJ >= 1 && XV >= 1 && WV >= 1, "tile");
};

template <int MT, int NT>
__global__ __launch_bounds__(SG_THREADS, 2) void skip_gemm_kernel(ConvArgs a, int HW, int ntiles) {
  using G = SgGeom<MT, NT>;
  constexpr int TI = G::TI, TJ = G::TJ;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* xs = smem;                         // [2][KC][NT]
  float* ws = smem + 2 * G::XF;             // [2][MT/32][8][64][2]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, l32 = lane & 31;
  const int Cin = a.Cin, Ca = a.Ca, Cout = a.Cout;
  const int nchunk = Cin / KC;
  const int nN = HW / NT, nM = (Cout + MT - 1) / MT;
  // persistent: workgroup bid runs tiles bid, bid + grid, ... (tile = (sample,
  // pixel tile, co tile), co fastest: concurrent neighbours share the X tile),
  // as one chunk stream -- the next tile's first chunk is loaded during the
  // current tile's last chunk, so the per-tile load latency is paid once
  const int nloc = (int)blockIdx.x < ntiles ? (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int gtot = nloc * nchunk;
  struct Tile { int b, m0, p0; };
  auto tile_of = [&](int il) {
    const int t = (int)blockIdx.x + il * (int)gridDim.x;
    const int mt = t % nM, r = t / nM;
    return Tile{r / nN, mt * MT, (r % nN) * NT};
  };

  f32x4 xr[G::XV], wr[G::WV];
  auto load = [&](int g) {
    const int il = g / nchunk, k = g - il * nchunk;
    const Tile tl = tile_of(il);
    const float* __restrict__ wp = a.wpk + (size_t)(tl.m0 / 32) * nchunk * 1024;
#pragma unroll
    for (int i = 0; i < G::XV; ++i) {
      const int idx = tid + SG_THREADS * i;
      const int row = idx / (NT / 4), c4 = idx - row * (NT / 4);
      const int ci = k * KC + row;
      const float* src = ci < Ca ? a.srcA + ((size_t)tl.b * Ca + ci) * HW
                                 : a.srcB + ((size_t)tl.b * a.Cb + (ci - Ca)) * HW;
      xr[i] = *reinterpret_cast<const f32x4*>(src + tl.p0 + 4 * c4);
    }
#pragma unroll
    for (int i = 0; i < G::WV; ++i) {
      const int idx = tid + SG_THREADS * i;
      const int t = idx >> 8, j = idx & 255;                 // co tile, float4 within its 4 KB block
      wr[i] = *reinterpret_cast<const f32x4*>(wp + ((size_t)t * nchunk + k) * 1024 + 4 * j);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < G::XV; ++i) {
      const int idx = tid + SG_THREADS * i;
      *reinterpret_cast<f32x4*>(xs + buf * G::XF + 4 * idx) = xr[i];   // [row][NT] order = idx order
    }
#pragma unroll
    for (int i = 0; i < G::WV; ++i) {
      const int idx = tid + SG_THREADS * i;
      *reinterpret_cast<f32x4*>(ws + buf * G::WF + 4 * idx) = wr[i];
    }
  };

  f32x16 acc[TI][TJ];
  if (gtot > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int g = 0; g < gtot; ++g) {
    const int buf = g & 1;
    const int il = g / nchunk, k = g - il * nchunk;
    if (g + 1 < gtot) load(g + 1);
    if (k == 0) {
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = f32x16{};
    }
    const float* xb = xs + buf * G::XF + h * 16 * NT + wn * (NT / 2) + l32;
    const float* wb = ws + buf * G::WF + (wm * TI) * 1024 + lane * 2;
#pragma unroll
    for (int sp = 0; sp < 8; ++sp) {
      float2 av[TI];
#pragma unroll
      for (int i = 0; i < TI; ++i) av[i] = *reinterpret_cast<const float2*>(wb + i * 1024 + sp * 128);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int s = 2 * sp + e;
        float bv[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) bv[j] = xb[s * NT + j * 32];
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(e ? av[i].y : av[i].x, bv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (g + 1 < gtot) store(buf ^ 1);
    if (k == nchunk - 1) {
      // epilogue: lane holds rows 8 (r / 4) + 4 h + (r % 4) of each 32 x 32 block, column l32
      const Tile tl = tile_of(il);
      float* out = a.out + (size_t)tl.b * Cout * HW + tl.p0 + wn * (NT / 2) + l32;
      const float* res = a.res ? a.res + (size_t)tl.b * Cout * HW + tl.p0 + wn * (NT / 2) + l32 : nullptr;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = tl.m0 + wm * (MT / 2) + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
          if (co >= Cout) continue;
          const float bi = a.bias ? a.bias[co] : 0.f;
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            float v = acc[i][j][r] + bi;
            if (res) v = v + res[(size_t)co * HW + j * 32];
            out[(size_t)co * HW + j * 32] = v;
          }
        }
      }
    }
    __syncthreads();
  }
}

template <int MT, int NT>
hipError_t launch_sg(const ConvArgs& a, int B, hipStream_t s) {
  using G = SgGeom<MT, NT>;
  const int HW = a.Ho * a.Wo;
  static std::atomic<unsigned long long> attr{0};
  set_max_lds_once((const void*)skip_gemm_kernel<MT, NT>, (int)G::LDS, attr);
  const int ntiles = HW / NT * ((a.Cout + MT - 1) / MT) * B;
  const int cap = 2 * device_cu_count();                 // two workgroups per CU (LDS)
  skip_gemm_kernel<MT, NT><<<ntiles < cap ? ntiles : cap, SG_THREADS, G::LDS, s>>>(a, HW, ntiles);
  return hipGetLastError();
}

// ERTD_SKIPGEMM=0 (diagnostic builds) keeps the round-5 kernels for A/B
int skip_gemm_env() {
  static const int v = [] {
    return ERTD_KNOB("SKIPGEMM", 1);
  }();
  return v;
}

}  // namespace

// tile per shape (ERTD_SG_TILE, diagnostic builds: 1 = 128 x 64, 2 = 128 x 128,
// 3 = 64 x 256, 4 = 64 x 128 where it divides).  Default 128 x 128 and only
// for Cout >= 128: per-layer serialized trace of the U2 B=64 step (same box,
// profiles/r06_skip_gemm_tiles.txt), the 11 skips take 534.8 us on the round-5
// kernels, 558.1 with 128 x 128 everywhere -- faster at every Cout >= 128 layer
// (u2r0 54.3 -> 51.8, u1r0 70.7 -> 67.3 us) but slower at Cout = 64 (u0r0
// 71.0 -> 87.7), which keeps conv1x1_kernel; smaller tiles (two or more per
// persistent workgroup) measured slower still (610.8-673.3 us)
static int sg_tile_env() {
  static const int v = [] {
    return ERTD_KNOB("SG_TILE", 0);
  }();
  return v;
}
static bool sg_tile(const ConvArgs& a, int B, int& mt, int& nt) {
  (void)B;
  const int HW = a.Ho * a.Wo;
  if (a.Cout % 64) return false;
  switch (sg_tile_env()) {
    case 1: mt = 128; nt = 64; break;
    case 2: mt = 128; nt = 128; break;
    case 3: mt = 64; nt = 256; break;
    case 4: mt = 64; nt = 128; break;
    default:
      if (a.Cout < 128) return false;
      mt = 128; nt = 128;
  }
  if (mt == 128 && a.Cout % 128) mt = 64;
  return HW % nt == 0;
}

bool skip_gemm_ok(const ConvArgs& a, int ks, int mode, int act, int B) {
  int mt, nt;
  return skip_gemm_env() != 0 && ks == 1 && mode == MODE_S1 && act == ACT_NONE && !a.ebias && !a.gnp &&
         a.Cin % KC == 0 && a.Ca % 4 == 0 && a.Cin == a.Ca + a.Cb && a.Ho == a.Hs && a.Wo == a.Ws &&
         a.wpk && sg_tile(a, B, mt, nt);
}

hipError_t launch_skip_gemm(const ConvArgs& a, int B, hipStream_t s) {
  int mt, nt;
  if (!sg_tile(a, B, mt, nt)) return hipErrorInvalidValue;
  if (mt == 64 && nt == 256) return launch_sg<64, 256>(a, B, s);
  if (mt == 64 && nt == 128) return launch_sg<64, 128>(a, B, s);
  if (mt == 64) return launch_sg<64, 64>(a, B, s);
  if (nt == 64) return launch_sg<128, 64>(a, B, s);
  return launch_sg<128, 128>(a, B, s);
}

}  // namespace unet
}  // namespace ertd
