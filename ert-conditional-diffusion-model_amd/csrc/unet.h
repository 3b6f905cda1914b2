// Build-defined conditional U-Net denoiser (SURVEY.md 8a', BASELINE north_star):
// shared declarations of its kernels (unet_conv.hip, unet_ops.hip) and the
// layer plan (unet_capi.hip).  PARITY UNPINNED vs the reference, which has
// no U-Net; the specification is oracle/unet_torch.py.
//
// Layout in HBM: every activation is NCHW fp32, one buffer per layer output
// (B, C, H, W), contiguous.  The sampled variable x stays (B, H*W) = (B, P),
// the reference's (B, param_dim) contract.
#pragma once
#include <cstdlib>

#include "ertd_common.h"

// Schedule knobs for same-box A/B: the shipped library compiles every default
// in and reads no environment variable; only a diagnostic build (-DERTD_DIAG:
// build.py --diag, tools/build_variant.sh) reads ERTD_<name> at first use.
#ifdef ERTD_DIAG
#define ERTD_KNOB(name, dflt) (::ertd::unet::diag_knob("ERTD_" name, (dflt)))
#else
#define ERTD_KNOB(name, dflt) (dflt)
#endif

namespace ertd {
namespace unet {

#ifdef ERTD_DIAG
inline int diag_knob(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
#endif

constexpr int NTHR = 256;   // conv workgroup: 4 waves, each a 64 (cout) x 64 (pixel) tile
constexpr double GN_EPS = 1e-5;   // GroupNorm eps (oracle/unet_torch.py)

// Activation applied to the conv input while it is staged into LDS.
enum Act { ACT_NONE = 0, ACT_GN_SILU = 1, ACT_GN = 2 };
// Spatial mode of a 3x3 conv: stride 1, stride 2 (Downsample), nearest x2
// upsample of the source followed by the stride-1 conv (Upsample).
enum Mode { MODE_S1 = 0, MODE_S2 = 1, MODE_UP = 2,
            // fp32 kernel only (internal): the Upsample conv as 4 sub-pixel
            // 2x2 convs at the source resolution (launch_pack_conv_up weights)
            MODE_UPP = 3 };

// GroupNorm partials per (sample, channel, part) -> {scale, shift} (see launch_gn_finalize below)
struct GnPartArgs {
  const float2* pa; int npa; int Ca;   // (B, Ca, npa) partials of channels [0, Ca)
  const float2* pb; int npb; int Cb;   // (B, Cb, npb) of channels [Ca, Ca+Cb), or null
  int HW, groups;
  const float* gamma; const float* beta;
  float2* out;           // (B, Ca+Cb) {gamma*rstd, beta - mean*gamma*rstd}
  float2* mr;            // optional (B, groups) {mean, rstd}
};

// The consumer GroupNorm's finalize folded into the producing conv: the MFMA
// waves store their partials write-through, every finished item adds one to
// its sample's counter, and once its items are done, workgroup w waits for
// the counts of samples w, w + grid, ... and finalizes them -- no finalize launch.
struct GnFold {
  GnPartArgs g;          // g.pa = the conv's own partials (ConvArgs::gnp), g.out the consumer's {scale, shift}
  unsigned* cnt;         // (B) arrival counters: zero before the launch, left zero by it
  int target;            // arrivals (items) per sample
  int B;                 // samples: workgroup w finalizes samples w, w + grid, ...
};

struct ConvArgs {
  const float* srcA;     // (B, Ca, Hs, Ws)  channels [0, Ca)
  const float* srcB;     // (B, Cb, Hs, Ws)  channels [Ca, Ca+Cb) (skip concat) or null
  int Ca, Cb;
  const float2* gn;      // (B, Cin) {scale, shift}: GroupNorm(x) = x*scale + shift (ACT_GN*)
  const float* wpk;      // packed weights: [co_tile32][chunk][step pair][64 lanes][2]
  const float* bias;     // (Cout), or null (no bias: the training input-gradient convs)
  const float* ebias;    // (B, eb_stride) per-sample per-channel add (offset applied) or null
  int eb_stride;
  const float* res;      // (B, Cout, Ho, Wo) residual add, or null
  float* out;            // (B, Cout, Ho, Wo)
  int Cin, Cout;
  int Hs, Ws;            // source spatial size
  int Ho, Wo;            // output spatial size
  void* bimg;            // bf16 3x3 GN / Upsample convs: scratch for the pre-transformed
                         // input, conv_bf16_image_bytes(Cin, B, Ho, Wo) bytes (null: stage fp32)
  int bimg_ready;        // 1: bimg already holds the transformed input (launch_gn_act_bf16)
  const float* wpk_wino; // fp32 3x3 stride-1: Winograd-transformed weights (launch_pack_conv_wino)
                         // or null (direct implicit GEMM)
  float* ksplit_buf;     // Winograd, optional: (B, Cout, Ho, Wo) scratch that lets a layer with
                         // fewer tile items than CUs split its K (input channels) in two halves
  const float* wpk_wino4;// fp32 3x3 stride-1 at W >= 32: Winograd F(4x4,3x3) weights
                         // (launch_pack_conv_wino4), preferred over wpk_wino where eligible
  float2* gnp;           // optional (B, Cout, np): GroupNorm partials of the OUTPUT (after
                         // bias / emb / residual), np = conv_gn_parts(...) (0: the dispatched
                         // kernel emits none and gnp must be null)
  int split;             // bf16 kernels: 1 = split-bf16 operands (hi + lo planes: weights
                         // packed with split = true, images of conv_bf16_image_bytes(.., true))
  GnFold fold;           // fp32 Winograd F(4x4) kernels with gnp: the next GroupNorm's finalize
                         // (fold.cnt null: none; conv_gn_fold_ok says where it is taken)
  unsigned* zero_words;  // conv_in: zero these zero_n words (the fold counters of the walk)
  int zero_n;
};

// GroupNorm statistics without a second read of the activation: the fp32
// Winograd convs emit, per (sample, channel, part of n = HW/np pixels), the
// partial {sum, M2 = sum (x - sum/n)^2} of their output from the epilogue
// registers; launch_gn_partials computes the same from a tensor (the outputs
// of the other kernels); launch_gn_finalize combines a group's parts in a
// fixed order in float64 (Chan's parallel formula) into the conv prologue's
// {scale, shift} (and {mean, rstd}) -- the 35 full-tensor reads of
// gn_stats_kernel per U2 step become 5.
hipError_t launch_gn_finalize(const GnPartArgs& a, int B, hipStream_t s);
// x (B, C, HW) -> (B, C, np) partials of 256 pixels: HW == 256 np
hipError_t launch_gn_partials(const float* x, int C, int HW, int np, float2* out, int B, hipStream_t s);
// parts per (sample, channel) the kernel launch_conv would dispatch emits into
// ConvArgs::gnp (0 = none: the Winograd layers without a K split do)
int conv_gn_parts(int ks, int mode, int act, const ConvArgs& a, int B);
// the same for the bf16 / split-bf16 convs (unet_conv_bf16.hip)
int conv_bf16_gn_parts(int ks, int mode, int act, const ConvArgs& a, int B);
int wino_gn_parts(const ConvArgs& a, int B);
// true where the kernel launch_conv would dispatch (fp32) takes ConvArgs::fold:
// the Winograd F(4x4) register-weight kernel without a K split
bool conv_gn_fold_ok(int ks, int mode, int act, const ConvArgs& a, int B);
// its MFMA-wave arrivals per sample (GnFold::target)
int conv_gn_fold_target(const ConvArgs& a, int B);

// sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15), the same bits in
// every lane of the row (fixed pairing: quad swaps, then the half-row and row
// mirrors; fp32 addition is commutative)
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

// ---- the GroupNorm finalize folded into the producing conv (GnFold) --------------
// write-through (agent-coherent) float2 store / load of the partials: the
// arriving waves of other workgroups (other XCDs' L2s) see them
__device__ __forceinline__ void st_f2_wt(float2* p, float2 v) {
  unsigned* u = reinterpret_cast<unsigned*>(p);
  __hip_atomic_store(u, __float_as_uint(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(u + 1, __float_as_uint(v.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_f2_wt(const float2* p) {
  const unsigned* u = reinterpret_cast<const unsigned*>(p);
  return make_float2(__uint_as_float(__hip_atomic_load(u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                     __uint_as_float(__hip_atomic_load(u + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
// running {count, mean, M2} in float64; chan_add merges a part (Chan et al.)
#ifndef FOLD_BATCH
#define FOLD_BATCH 4   // parts loaded per round trip and lane (registers: the producer's epilogue)
#endif
struct ChanAcc {
  double n, mean, m2;
};
__device__ __forceinline__ void chan_add(ChanAcc& a, double nb, double meanb, double m2b) {
  const double n = a.n + nb;
  const double d = meanb - a.mean;
  const double f = n > 0.0 ? nb / n : 0.0;   // two empty states stay empty
  a.mean = a.mean + d * f;
  a.m2 = a.m2 + m2b + d * d * a.n * f;
  a.n = n;
}
// Groups [part * ceil(G / nparts), ...) of sample b finalized by the calling
// wave -- the one GroupNorm finalize of the fp32 U-Net, run by
// gn_finalize_kernel and by the producing convs' fold alike, so a group's
// {scale, shift} has the same bits whichever runs it: GN_LPG lanes per group,
// each streaming the group's parts k = sub, sub + GN_LPG, ... (channel-major,
// A then B) through chan_add, then the lanes' states merged in a fixed
// butterfly (the lower lane's state first, so every lane holds the same bits).
// WT: the A partials were written in this launch (write-through loads).
constexpr int GN_LPG = 16;
template <bool WT>
__device__ __forceinline__ void gn_group_finalize(const GnPartArgs& g, int b, int lane, int part,
                                                  int nparts) {
  const int G = g.groups, C = g.Ca + g.Cb, cpg = C / G;
  const int gper = (G + nparts - 1) / nparts, gfirst = part * gper;
  const int gcnt = G - gfirst < gper ? G - gfirst : gper;
  if (gcnt <= 0) return;
  constexpr int LPG = GN_LPG;
  const double na = (double)(g.HW / g.npa), nb = g.Cb > 0 ? (double)(g.HW / g.npb) : 1.0;
  for (int gbase = 0; gbase < gcnt; gbase += 64 / LPG) {
    const int gl = gbase + lane / LPG, sub = lane % LPG;
    const bool live = gl < gcnt;
    const int gi = gfirst + gl;
    const int c0 = live ? gi * cpg : 0;
    const int nA = !live ? 0 : (c0 < g.Ca ? (g.Ca - c0 < cpg ? g.Ca - c0 : cpg) : 0);
    const int itemsA = nA * g.npa, items = !live ? 0 : itemsA + (cpg - nA) * (g.Cb > 0 ? g.npb : 0);
    const float2* pa = g.pa + ((size_t)b * g.Ca + c0) * g.npa;
    const float2* pb = g.Cb > 0 && live ? g.pb + ((size_t)b * g.Cb + (c0 + nA - g.Ca)) * g.npb : nullptr;
    ChanAcc acc{0.0, 0.0, 0.0};
    for (int k0 = sub; k0 < items; k0 += FOLD_BATCH * LPG) {
      float2 v[FOLD_BATCH];
#pragma unroll
      for (int j = 0; j < FOLD_BATCH; ++j) {
        const int k = k0 + j * LPG;
        v[j] = k >= items ? make_float2(0.f, 0.f) : (k < itemsA ? (WT ? ld_f2_wt(pa + k) : pa[k]) : pb[k - itemsA]);
      }
#pragma unroll
      for (int j = 0; j < FOLD_BATCH; ++j) {
        const int k = k0 + j * LPG;
        if (k < items) {
          const double n = k < itemsA ? na : nb;
          chan_add(acc, n, (double)v[j].x / n, (double)v[j].y);
        }
      }
    }
    for (int m = 1; m < LPG; m <<= 1) {
      ChanAcc o{__shfl_xor(acc.n, m), __shfl_xor(acc.mean, m), __shfl_xor(acc.m2, m)};
      const bool lower = (sub & m) == 0;
      ChanAcc x = lower ? acc : o;
      const ChanAcc y = lower ? o : acc;
      chan_add(x, y.n, y.mean, y.m2);
      acc = x;
    }
    if (!live) continue;
    double var = acc.m2 / acc.n;
    var = var > 0.0 ? var : 0.0;
    const float rstd = (float)(1.0 / sqrt(var + GN_EPS));
    const float mean = (float)acc.mean;
    if (g.mr && sub == 0) g.mr[(size_t)b * G + gi] = make_float2(mean, rstd);
    for (int cl = sub; cl < cpg; cl += LPG) {
      const int c = c0 + cl;
      const float scale = rstd * g.gamma[c];
      const float shift = -scale * mean + g.beta[c];
      g.out[(size_t)b * C + c] = make_float2(scale, shift);
    }
  }
}
// called by every MFMA wave of a producing conv once per item, after its
// partials of sample b are stored with st_f2_wt (whole wave active): the
// item's last wave (an LDS count over the nw MFMA waves) adds the item's one
// arrival to the sample's counter -- without waiting for the atomic's return
// (same-address device atomics serialize: the count is read at the tail)
__device__ __forceinline__ void gn_fold_item_done(const GnFold& f, int b, int* lds_cnt, int nw, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = atomicAdd(lds_cnt, 1);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old == nw - 1 && lane == 0) {
    *lds_cnt = 0;
    (void)__hip_atomic_fetch_add(f.cnt + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

hipError_t launch_conv(int ks, int mode, int act, const ConvArgs& a, int B, hipStream_t s);
// bf16-operand variant (unet_conv_bf16.hip): same arguments, wpk packed by
// launch_pack_conv_bf16
hipError_t launch_conv_bf16(int ks, int mode, int act, const ConvArgs& a, int B, hipStream_t s);
// split: the split-bf16 layouts (two bf16 planes, hi and lo = RNE(x - hi))
size_t conv_packed_floats_bf16(int cin, int cout, int ks, bool split = false);
hipError_t launch_act_bf16(const ConvArgs& a, int act, bool up, int B, hipStream_t s);
size_t conv_bf16_image_bytes(int cin, int B, int H, int W, bool split = false);
hipError_t launch_pack_conv_bf16(const float* w, int cin, int cout, int ks, float* dst,
                                 hipStream_t s, bool split = false);
// weight packing a conv_in / conv_out launch reads: 0 fp32, 1 bf16 (the staged
// input is rounded to bf16 too), 2 split bf16 (weight = hi + lo, fp32 input)
enum PackKind { PK_F32 = 0, PK_BF16 = 1, PK_SPLIT = 2 };
// Cout = 1, 3x3 stride 1 (conv_out; unet_conv_out.hip): per-pixel fp32 fma
// chains, weights read from the model's packing
hipError_t launch_conv_out(int act, const ConvArgs& a, int B, int pk, hipStream_t s);
// Cin = 1, 3x3 stride 1, no activation / emb / residual (conv_in; unet_conv_out.hip):
// one thread per output pixel, every output channel's 9-tap fp32 fma chain
bool conv_in_ok(const ConvArgs& a, int ks, int mode, int act);
hipError_t launch_conv_in(const ConvArgs& a, int B, int pk, hipStream_t s);
// fp32 3x3 stride-1 convs by Winograd F(2x2,3x3) (unet_conv_wino.hip): eligible
// shapes (Cin, Ca multiples of 8, Cout of 64, W in 16..128; ERTD_UNET_WINO=0
// disables), the U = G g G^T packing (0 floats: shape not eligible), launch
hipError_t launch_conv_wino(int act, const ConvArgs& a, int B, hipStream_t s);
bool conv_wino_ok(int cin, int ca, int cout, int wo);
// a Winograd layer with this geometry splits its K when given ConvArgs::ksplit_buf
bool wino_ksplit_wanted(int cin, int cout, int wo, int B);
size_t conv_packed_floats_wino(int cin, int cout);
// Winograd F(4x4,3x3) (unet_conv_wino4.hip): Cin, Ca multiples of 4, Cout of 64,
// W in {32, 64, 128} (16 with an even batch); ERTD_UNET_WINO=2 keeps F(2x2) everywhere.  A Winograd
// launch (launch_conv_wino) takes it when wino4_ok and ConvArgs::wpk_wino4 is set.
bool wino4_ok(int cin, int ca, int cout, int wo, int B);
bool wino_dispatchable(const ConvArgs& a, int B);
size_t conv_packed_floats_wino4(int cin, int cout);
hipError_t launch_pack_conv_wino4(const float* w, int cin, int cout, float* dst, hipStream_t s,
                                  bool flipT = false);
hipError_t launch_conv_wino4(int act, const ConvArgs& a, int B, hipStream_t s, int cus);
int wino4_tile_items(int cout, int wo, int B);
// the F(4x4) register-weight kernel splits its K (given ConvArgs::ksplit_buf)
bool wino4s_ksplit(int cin, int cout, int wo, int B);
bool wino4_ksplit(int cin, int cout, int wo, int B);
// F(4x4) with register-resident weights (unet_conv_wino4s.hip): items of 64 co x
// 16 tiles (the 16x16 level fills the CUs at B = 64 without a K split); same
// wpk_wino4 packing; Cin a multiple of 8, Ca even, W in {16, 32, 64}.  wino4_ok
// is true where wino4s_ok is, and launch_conv_wino then dispatches it.
bool wino4s_ok(int cin, int ca, int cout, int wo, int B);
int wino4s_items(int cout, int wo, int B);
bool wino4s_fold_ok(const ConvArgs& a, bool up, int B);
int wino4s_fold_target(const ConvArgs& a);
// the same kernel for the fp32 Upsample conv (MODE_UP, no activation; wo = the
// OUTPUT width): conv3x3 of the nearest-x2 source through the F(4x4) packing
bool wino4s_up_ok(int cin, int ca, int cout, int wo, int B);
hipError_t launch_conv_wino4s(int act, const ConvArgs& a, int B, hipStream_t s, int cus);
hipError_t launch_add_inplace(float* out, const float* part, size_t n, hipStream_t s);
// flipT: w is a forward conv's (cin, cout, 3, 3) weight; pack the input-gradient
// conv's weight W'[co][ci] = W[ci][co] spatially flipped (training)
hipError_t launch_pack_conv_wino(const float* w, int cin, int cout, float* dst, hipStream_t s,
                                 bool flipT = false);
// fp32 1x1 conv without activation / emb / residual (the ResBlock skips;
// unet_conv1x1.hip): per-sample GEMM, weights and input by LDS-DMA
bool conv1x1_ok(const ConvArgs& a, int act, int B);
hipError_t launch_conv1x1(const ConvArgs& a, int B, hipStream_t s);
// training: the fp32 3x3 stride-1 weight gradient by Winograd F(4x4,3x3)
// (unet_wgrad_wino.hip); scratch floats it needs (0 = not eligible: Cin, Cout
// multiples of 64, H in {16, 32, 64}; ERTD_WGRAD_WINO=0 disables)
size_t wgrad_wino_ws_floats(int Cin, int Cout, int B, int H, int ks, int mode);
hipError_t launch_wgrad_wino(const float* dy, const float* x, int Ca, const float* x2, int Cb, int B,
                             int H, int Cout, int mode, const float* gn, int act, float* dw,
                             int accumulate, float* ws, hipStream_t s, float* db = nullptr,
                             float* db2 = nullptr);
// the Winograd path can also return the conv's bias gradient (sum of dy)
bool wgrad_wino_bias_ok(int Cin, int Cout, int B, int H, int ks, int mode);
// packed floats of one conv's weights
size_t conv_packed_floats(int cin, int cout, int ks);
hipError_t launch_pack_conv(const float* w, int cin, int cout, int ks, float* dst, hipStream_t s,
                            bool flipT = false);
// every packing of a prepared ertd_pack_desc table (device copy) in one launch (unet_pack.hip)
hipError_t launch_pack_batch(const ertd_pack_desc* d, int n, int blocks, hipStream_t s);
// fp32 Upsample conv weights: 4 parity classes of combined 2x2 taps
size_t conv_packed_floats_up(int cin, int cout);
hipError_t launch_pack_conv_up(const float* w, int cin, int cout, float* dst, hipStream_t s);

struct GnArgs {
  const float* srcA; const float* srcB; int Ca, Cb;
  int HW, groups;
  const float* gamma; const float* beta;
  float2* out;           // (B, Ca+Cb) {gamma*rstd, beta - mean*gamma*rstd}
  float2* mr;            // optional (B, groups) {mean, rstd} (training: GroupNorm backward)
};
hipError_t launch_gn_stats(const GnArgs& a, int B, hipStream_t s);
// GroupNorm statistics + apply (+ SiLU) + bf16 image of a 3x3 stride-1 bf16
// conv's input in one pass (unet_conv_bf16.hip); writes a.out like
// launch_gn_stats and the [B][C/16][H][W][16] image; shapes gated by
// gn_act_bf16_fits (C/16 whole, <= 64 activations per thread)
bool gn_act_bf16_fits(int C, int groups, int HW);
hipError_t launch_gn_act_bf16(const GnArgs& a, bool silu, void* bimg, int B, hipStream_t s,
                              bool split = false);

// y[b][o] = bias[o] (+ add[b][o]) + sum_k Wt[k][o] * in(b, k)
enum DenseIn { DIN_PLAIN = 0, DIN_SILU = 1, DIN_SINUSOID = 2 };
struct DenseArgs {
  const float* x; int x_stride;     // (B, K) input (DIN_PLAIN / DIN_SILU)
  const int64_t* t;                 // DIN_SINUSOID: per-sample t (B), or null -> *t_dev
  const int* t_dev;
  const float* freq;                // DIN_SINUSOID: (K/2) frequencies
  const float* wt;                  // (K, O) k-major
  const float* bias;                // (O)
  const float* add; int add_stride; // optional (B, O) add (row stride), or null
  int add_bcast;                    // add row 0 for every b
  float* y; int y_stride;
  int K, O;
};
hipError_t launch_dense(int din, const DenseArgs& a, int B, hipStream_t s);
hipError_t launch_transpose(const float* w, int O, int K, float* dst, int dst_ld, hipStream_t s);

// single-head self-attention core: o[b][c][i] = sum_j softmax_j(q_i . k_j / sqrt(C)) v[c][j]
// qkv (B, 3C, N) -> o (B, C, N)
hipError_t launch_attention(const float* qkv, int C, int N, float* o, float* scratch, int B,
                            hipStream_t s);

struct UpdateArgs {
  float* x;             // (B, P) in/out
  const float* eps;     // (B, P)
  const float* c1; const float* c2; const float* sigma;   // per-step tables (index t)
  const float* noise;   // injected (num_steps, B, P) or null -> Philox
  int num_steps;
  const int* t_dev;
  uint64_t seed; uint32_t member_offset;
  int P;
};
hipError_t launch_unet_update(const UpdateArgs& a, int B, hipStream_t s);
// training plumbing (unet_train.hip): stride-2 input-gradient zero insertion
// (x (B,C,Ho,Ho) -> (B,C,2Ho,2Ho)) and the upsample input gradient's 2x2 sums
hipError_t launch_zero_insert(const float* x, int B, int C, int Ho, float* out, hipStream_t s);
hipError_t launch_sum_pool2(const float* x, int B, int C, int H, float* out, int accumulate,
                            hipStream_t s);
hipError_t launch_set_word(int* w, int v, hipStream_t s);
hipError_t launch_dec_word(int* w, hipStream_t s);

}  // namespace unet
}  // namespace ertd
