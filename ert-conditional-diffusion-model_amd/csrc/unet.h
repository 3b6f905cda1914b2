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
  GnPartArgs gnc;        // fp32 Winograd F(4x4) consumers (gnc.pa non-null): the input's
                         // GroupNorm finalize in the conv's own prologue (conv_gn_consume_ok):
                         // the {scale, shift} of the sample the workgroup runs are merged from
                         // these partials into LDS -- no finalize launch, gn unused
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
// true where the kernel launch_conv would dispatch (fp32) takes ConvArgs::gnc:
// the Winograd F(4x4) register-weight kernel without a K split whose items
// divide evenly over its workgroups with each workgroup's items in one sample
bool conv_gn_consume_ok(int ks, int mode, int act, const ConvArgs& a, int B);

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
// GroupNorm statistics of one group from its parts' {sum, M2 about the part
// mean}, in float64 and a fixed order -- two passes over the parts:
//   S = sum_k sum_k,  mean = S / N,  M2 = sum_k (M2_k + n_k (sum_k / n_k - mean)^2)
// (N = cpg * HW pixels; n_k = HW / np pixels per part, 256 for every producer
// here, so sum_k / n_k is exact).  GN_LPG lanes per group: lane sub takes the
// parts k = sub + GN_LPG i (channel-major, A then B) in ascending i, and the
// lanes' totals meet in an xor butterfly (a + b == b + a, so every lane ends
// with the same bits).  gn_finalize_kernel, the consumer-side finalize of the
// F(4x4) conv (gn_group_finalize_regs) and the diagnostic fold all run this
// arithmetic, so a group's {scale, shift} has the same bits whichever runs it.
// (Rounds 3-5 merged the parts with Chan's pairwise update: a float64
// division per part and per butterfly level.)
#ifndef FOLD_BATCH
#define FOLD_BATCH 4   // parts loaded per round trip and lane
#endif
constexpr int GN_LPG = 16;
struct GnGroupGeom {
  int c0, itemsA, items;          // first channel, parts of tensor A, all parts (0: dead lane group)
  const float2* pa;               // (b, c0) of A
  const float2* pb;               // (b, c0 + nA - Ca) of B
};
__device__ __forceinline__ GnGroupGeom gn_group_geom(const GnPartArgs& g, int b, int gi, bool live) {
  const int cpg = (g.Ca + g.Cb) / g.groups;
  GnGroupGeom q{};
  if (!live) return q;
  q.c0 = gi * cpg;
  const int nA = q.c0 < g.Ca ? (g.Ca - q.c0 < cpg ? g.Ca - q.c0 : cpg) : 0;
  q.itemsA = nA * g.npa;
  q.items = q.itemsA + (cpg - nA) * (g.Cb > 0 ? g.npb : 0);
  q.pa = g.pa + ((size_t)b * g.Ca + q.c0) * g.npa;
  q.pb = g.Cb > 0 ? g.pb + ((size_t)b * g.Cb + (q.c0 + nA - g.Ca)) * g.npb : nullptr;
  return q;
}
// sum over the 16 lanes of a DPP row in float64, the same bits in every lane
// (row16_sum's pairing: quad swaps, then the half-row and row mirrors; each
// level adds a lane's value and its partner's, and a + b == b + a)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double gn_lpg_sum(double v) {
  static_assert(GN_LPG == 16, "one DPP row per group");
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  v += dpp_f64<0x140>(v);
  return v;
}
// pass-2 term of part k: its M2 plus its mean's deviation, weighted by its
// count n (inv_n = 1 / n: exact for the 256-pixel parts)
__device__ __forceinline__ double gn_part_q(float2 v, double n, double inv_n, double mean) {
  const double d = (double)v.x * inv_n - mean;
  return (double)v.y + n * (d * d);
}
// {mean, rstd} of the group from the lanes' S and Q totals
__device__ __forceinline__ float2 gn_mean_rstd(double mean, double Q, double N) {
  double var = Q / N;
  var = var > 0.0 ? var : 0.0;
  return make_float2((float)mean, (float)(1.0 / sqrt(var + GN_EPS)));
}
template <bool WT>
__device__ __forceinline__ float2 gn_ld_part(const GnGroupGeom& q, int k) {
  return k < q.itemsA ? (WT ? ld_f2_wt(q.pa + k) : q.pa[k]) : q.pb[k - q.itemsA];
}
// Groups [part * ceil(G / nparts), ...) of sample b finalized by the calling
// wave, parts streamed FOLD_BATCH per lane and round trip (the second pass
// re-reads them: L2-hot).  WT: the A partials were written in this launch
// (write-through loads).  orow: where {scale, shift} of sample b's channels go
// (null: g.out + b * C).
template <bool WT>
__device__ __forceinline__ void gn_group_finalize(const GnPartArgs& g, int b, int lane, int part,
                                                  int nparts, float2* orow = nullptr) {
  const int G = g.groups, C = g.Ca + g.Cb, cpg = C / G;
  const int gper = (G + nparts - 1) / nparts, gfirst = part * gper;
  const int gcnt = G - gfirst < gper ? G - gfirst : gper;
  if (gcnt <= 0) return;
  constexpr int LPG = GN_LPG;
  const double na = (double)(g.HW / g.npa), nb = g.Cb > 0 ? (double)(g.HW / g.npb) : 1.0;
  const double ina = 1.0 / na, inb = 1.0 / nb;
  const double N = (double)cpg * (double)g.HW;
  for (int gbase = 0; gbase < gcnt; gbase += 64 / LPG) {
    const int gl = gbase + lane / LPG, sub = lane % LPG;
    const bool live = gl < gcnt;
    const int gi = gfirst + gl;
    const GnGroupGeom q = gn_group_geom(g, b, gi, live);
    double S = 0.0;
    for (int k0 = sub; k0 < q.items; k0 += FOLD_BATCH * LPG) {
      float2 v[FOLD_BATCH];
#pragma unroll
      for (int j = 0; j < FOLD_BATCH; ++j) {
        const int k = k0 + j * LPG;
        v[j] = k < q.items ? gn_ld_part<WT>(q, k) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < FOLD_BATCH; ++j)
        if (k0 + j * LPG < q.items) S += (double)v[j].x;
    }
    S = gn_lpg_sum(S);
    const double mean = S / N;
    double Q = 0.0;
    for (int k0 = sub; k0 < q.items; k0 += FOLD_BATCH * LPG) {
      float2 v[FOLD_BATCH];
#pragma unroll
      for (int j = 0; j < FOLD_BATCH; ++j) {
        const int k = k0 + j * LPG;
        v[j] = k < q.items ? gn_ld_part<WT>(q, k) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < FOLD_BATCH; ++j) {
        const int k = k0 + j * LPG;
        if (k < q.items) Q += k < q.itemsA ? gn_part_q(v[j], na, ina, mean) : gn_part_q(v[j], nb, inb, mean);
      }
    }
    Q = gn_lpg_sum(Q);
    if (!live) continue;
    const float2 mr = gn_mean_rstd(mean, Q, N);
    if (g.mr && sub == 0) g.mr[(size_t)b * G + gi] = mr;
    for (int cl = sub; cl < cpg; cl += LPG) {
      const int c = q.c0 + cl;
      const float scale = mr.y * g.gamma[c];
      const float shift = -scale * mr.x + g.beta[c];
      if (orow) orow[c] = make_float2(scale, shift);
      else g.out[(size_t)b * C + c] = make_float2(scale, shift);
    }
  }
}
// The same finalize with every load issued before any arithmetic (one memory
// latency for all of a wave's groups): the consumer conv's prologue.  Job j of
// the calling wave (jobs wave, wave + nw, ... < njobs, at most JM) finalizes
// groups 4 jg .. 4 jg + 3 of sample smp[j] into tab[row[j] * C + c]; the
// caller guarantees cpg <= GN_LPG and at most KM parts per lane.
template <int JM, int KM>
__device__ __forceinline__ void gn_group_finalize_regs(const GnPartArgs& g, const int (&smp)[JM],
                                                       const int (&jg)[JM], const int (&row)[JM],
                                                       const bool (&jl)[JM], int lane, float2* tab) {
  constexpr int LPG = GN_LPG;
  const int G = g.groups, C = g.Ca + g.Cb, cpg = C / G, sub = lane % LPG;
  const double na = (double)(g.HW / g.npa), nb = g.Cb > 0 ? (double)(g.HW / g.npb) : 1.0;
  const double ina = 1.0 / na, inb = 1.0 / nb;
  const double N = (double)cpg * (double)g.HW;
  GnGroupGeom q[JM];
  float2 v[JM][KM];
  float ga[JM], be[JM];
  bool live[JM];
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    const int gi = jg[j] * 4 + lane / LPG;
    live[j] = jl[j] && gi < G;
    q[j] = gn_group_geom(g, smp[j], gi, live[j]);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int kk = sub + LPG * k;
      v[j][k] = kk < q[j].items ? gn_ld_part<false>(q[j], kk) : make_float2(0.f, 0.f);
    }
    const bool ch = live[j] && sub < cpg;
    ga[j] = ch ? g.gamma[q[j].c0 + sub] : 0.f;
    be[j] = ch ? g.beta[q[j].c0 + sub] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < JM; ++j) {
    double S = 0.0;
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (sub + LPG * k < q[j].items) S += (double)v[j][k].x;
    S = gn_lpg_sum(S);
    const double mean = S / N;
    double Q = 0.0;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int kk = sub + LPG * k;
      if (kk < q[j].items)
        Q += kk < q[j].itemsA ? gn_part_q(v[j][k], na, ina, mean) : gn_part_q(v[j][k], nb, inb, mean);
    }
    Q = gn_lpg_sum(Q);
    if (live[j] && sub < cpg) {
      const float2 mr = gn_mean_rstd(mean, Q, N);
      const float scale = mr.y * ga[j];
      const float shift = -scale * mr.x + be[j];
      tab[(size_t)row[j] * C + q[j].c0 + sub] = make_float2(scale, shift);
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
bool wino4s_gnc_ok(const ConvArgs& a, int B);
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
// the 1x1 skip convs as a batched GEMM on 32x32x2 fp32 MFMAs (unet_skip_gemm.hip)
bool skip_gemm_ok(const ConvArgs& a, int ks, int mode, int act, int B);
hipError_t launch_skip_gemm(const ConvArgs& a, int B, hipStream_t s);
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
