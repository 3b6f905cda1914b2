// C ABI of the build-defined conditional U-Net (include/ertdiff.h, "U-Net"
// section): parameter enumeration, weight packing, forward and the T-step
// sampler.  The layer walk below restates oracle/unet_torch.py (the
// specification; PARITY UNPINNED vs the reference, which has no U-Net).
//
// Everything is enqueued on the caller's stream; the library allocates
// nothing.  Workspace = one NCHW buffer per layer output (bump allocator over
// the caller's ws), so a whole step can be captured into a hipGraph.
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <map>
#include <string>
#include <vector>

#include "unet.h"
#include "unet_pack.h"

using namespace ertd;
using namespace ertd::unet;

namespace {

struct Param {
  std::string name;
  std::vector<int> shape;
  size_t numel() const {
    size_t n = 1;
    for (int d : shape) n *= (size_t)d;
    return n;
  }
};

bool cfg_ok(const ertd_unet_config* c) {
  if (!c) return false;
  if (c->image < 16 || c->image > 128 || (c->image & (c->image - 1))) return false;
  if (c->n_levels < 1 || c->n_levels > 4 || c->num_res < 1 || c->num_res > 4) return false;
  if (c->groups < 1 || c->ch < 8) return false;
  if ((c->image >> (c->n_levels - 1)) < 16) return false;  // every level >= 16x16
  for (int i = 0; i < c->n_levels; ++i) {
    const int C = c->ch * c->ch_mult[i];
    if (c->ch_mult[i] < 1 || C % c->groups) return false;
  }
  if (c->ch % c->groups) return false;
  if (c->precision != ERTD_PREC_FP32 && c->precision != ERTD_PREC_BF16 &&
      c->precision != ERTD_PREC_BF16X3)
    return false;
  if (c->attn) {
    const int Cm = c->ch * c->ch_mult[c->n_levels - 1];
    const int r = c->image >> (c->n_levels - 1);
    if (r * r != 256 || Cm % 256) return false;  // attention kernel: N = 256, C multiple of 256
  }
  return true;
}

int temb(const ertd_unet_config* c) { return 4 * c->ch; }

// the bf16-operand conv kernels (plain or split): bf16 packings and images
bool bf_prec(int p) { return p == ERTD_PREC_BF16 || p == ERTD_PREC_BF16X3; }

std::vector<Param> enumerate(const ertd_unet_config* c) {
  std::vector<Param> P;
  auto lin = [&](const std::string& n, int i, int o) {
    P.push_back({n + ".weight", {o, i}});
    P.push_back({n + ".bias", {o}});
  };
  auto conv = [&](const std::string& n, int i, int o, int k) {
    P.push_back({n + ".weight", {o, i, k, k}});
    P.push_back({n + ".bias", {o}});
  };
  auto gn = [&](const std::string& n, int ch) {
    P.push_back({n + ".weight", {ch}});
    P.push_back({n + ".bias", {ch}});
  };
  auto res = [&](const std::string& n, int i, int o) {
    gn(n + ".norm1", i);
    conv(n + ".conv1", i, o, 3);
    lin(n + ".emb", temb(c), o);
    gn(n + ".norm2", o);
    conv(n + ".conv2", o, o, 3);
    if (i != o) conv(n + ".skip", i, o, 1);
  };
  P.push_back({"condition_encoder.0.weight", {C1, CIN, 3}});
  P.push_back({"condition_encoder.0.bias", {C1}});
  P.push_back({"condition_encoder.2.weight", {C2, C1, 3}});
  P.push_back({"condition_encoder.2.bias", {C2}});
  P.push_back({"condition_encoder.6.weight", {H, C2}});
  P.push_back({"condition_encoder.6.bias", {H}});
  lin("time_embed.0", c->ch, temb(c));
  lin("time_embed.2", temb(c), temb(c));
  lin("cond_proj", H, temb(c));
  conv("conv_in", 1, c->ch, 3);
  std::vector<int> chans{c->ch};
  int ch = c->ch;
  const int nl = c->n_levels;
  for (int i = 0; i < nl; ++i) {
    for (int r = 0; r < c->num_res; ++r) {
      const int o = c->ch * c->ch_mult[i];
      res("down." + std::to_string(i) + ".res." + std::to_string(r), ch, o);
      ch = o;
      chans.push_back(ch);
    }
    if (i != nl - 1) {
      conv("down." + std::to_string(i) + ".downsample", ch, ch, 3);
      chans.push_back(ch);
    }
  }
  res("mid.res1", ch, ch);
  if (c->attn) {
    gn("mid.attn.norm", ch);
    conv("mid.attn.qkv", ch, 3 * ch, 1);
    conv("mid.attn.proj", ch, ch, 1);
  }
  res("mid.res2", ch, ch);
  for (int i = nl - 1; i >= 0; --i) {
    for (int r = 0; r <= c->num_res; ++r) {
      const int o = c->ch * c->ch_mult[i];
      const int skip = chans.back();
      chans.pop_back();
      res("up." + std::to_string(i) + ".res." + std::to_string(r), ch + skip, o);
      ch = o;
    }
    if (i != 0) conv("up." + std::to_string(i) + ".upsample", ch, ch, 3);
  }
  gn("norm_out", ch);
  conv("conv_out", ch, 1, 3);
  return P;
}

bool ends_with(const std::string& s, const char* suf) {
  const size_t n = strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

// ---- packed layout ------------------------------------------------------------
// [encoder pack (ertd_pack_weights layout)] [zero head dummy] then, per
// parameter in enumeration order: conv weights in conv fragment order, the
// three embedding-path linears transposed (K, O), every ResBlock's emb linear
// into one concatenated transposed matrix Wall^T (temb, sum C) + bias vector,
// everything else verbatim.
constexpr size_t DUMMY_FLOATS = (size_t)H * H + H + (size_t)H * (1 + 2 * H) + H + H + 1;

struct Layout {
  std::vector<Param> params;
  std::map<std::string, size_t> off;  // packed offset per parameter name
  std::map<std::string, size_t> offw; // fp32: Winograd-packed copy of eligible 3x3 weights
  std::map<std::string, size_t> offw4;// ... and the F(4x4,3x3) packing (layers at W >= 32 use it)
  std::map<std::string, int> eboff;   // ResBlock name -> column offset in Wall
  size_t enc = 0, dummy = 0, wall = 0, ball = 0, total = 0;
  int ebtotal = 0;
};

size_t a64(size_t n) { return (n + 63) / 64 * 64; }

Layout layout(const ertd_unet_config* c) {
  Layout L;
  L.params = enumerate(c);
  size_t o = 0;
  L.enc = o;
  o += a64(PACKED_FLOATS_ALL);
  L.dummy = o;
  o += a64(DUMMY_FLOATS);
  for (const Param& p : L.params)
    if (ends_with(p.name, ".emb.weight")) {
      L.eboff[p.name.substr(0, p.name.size() - 11)] = L.ebtotal;
      L.ebtotal += p.shape[0];
    }
  L.wall = o;
  o += a64((size_t)temb(c) * L.ebtotal);
  L.ball = o;
  o += a64((size_t)L.ebtotal);
  for (const Param& p : L.params) {
    if (p.name.rfind("condition_encoder.", 0) == 0) continue;
    if (ends_with(p.name, ".emb.weight") || ends_with(p.name, ".emb.bias")) continue;
    L.off[p.name] = o;
    if (p.shape.size() == 4)
      o += a64(bf_prec(c->precision)
                   ? conv_packed_floats_bf16(p.shape[1], p.shape[0], p.shape[2],
                                             c->precision == ERTD_PREC_BF16X3)
                   : (ends_with(p.name, ".upsample.weight")
                          ? conv_packed_floats_up(p.shape[1], p.shape[0])
                          : conv_packed_floats(p.shape[1], p.shape[0], p.shape[2])));
    else o += a64(p.numel());
    // fp32 ResBlock 3x3 convs also get the Winograd F(2x2,3x3) packing
    // (dispatch picks it when conv_wino_ok; ERTD_UNET_WINO=0 keeps the direct one)
    if (c->precision == ERTD_PREC_FP32 && p.shape.size() == 4 && p.shape[2] == 3 &&
        ends_with(p.name, ".upsample.weight") && conv_packed_floats_wino4(p.shape[1], p.shape[0]) > 0) {
      // ... and the Upsample convs the F(4x4) packing (wino4s_up_ok dispatch)
      L.offw4[p.name] = o;
      o += a64(conv_packed_floats_wino4(p.shape[1], p.shape[0]));
    }
    if (c->precision == ERTD_PREC_FP32 && p.shape.size() == 4 && p.shape[2] == 3 &&
        (ends_with(p.name, ".conv1.weight") || ends_with(p.name, ".conv2.weight")) &&
        conv_packed_floats_wino(p.shape[1], p.shape[0]) > 0) {
      L.offw[p.name] = o;
      o += a64(conv_packed_floats_wino(p.shape[1], p.shape[0]));
      if (conv_packed_floats_wino4(p.shape[1], p.shape[0]) > 0) {
        L.offw4[p.name] = o;
        o += a64(conv_packed_floats_wino4(p.shape[1], p.shape[0]));
      }
    }
  }
  L.total = o;
  return L;
}


// ---- forward walk -----------------------------------------------------------------
struct Walk {
  const ertd_unet_config* c;
  const Layout* L;
  const float* pk;       // packed
  char* ws;              // workspace base (null: size only)
  size_t used = 0;
  int B;
  hipStream_t s;
  bool dry;
  hipError_t err = hipSuccess;

  // dry (sizing) walks hand out distinct fake addresses -- never dereferenced,
  // but tensors are keyed by address (GroupNorm partials): a shared null would
  // merge their records and under-count the workspace
  float* alloc(size_t floats) {
    float* p = dry ? reinterpret_cast<float*>((uintptr_t)4096 + used) : (float*)(ws + used);
    used += (floats * sizeof(float) + 255) / 256 * 256;
    if (!dry && cap && used > cap) {   // never launch past the caller's workspace
      if (err == hipSuccess) err = hipErrorOutOfMemory;
      return (float*)ws;
    }
    return p;
  }
  size_t cap = 0;        // real walks: the caller's workspace bytes (checked by alloc)
  const float* P(const std::string& n) const { return pk + L->off.at(n); }
  void chk(hipError_t e) {
    if (err == hipSuccess && e != hipSuccess) err = e;
  }

  float2* gnbuf = nullptr;  // the {scale, shift} the next GN+act conv reads: one of gnb
  float2* gnb[2] = {nullptr, nullptr};   // alternated per GroupNorm (a folded finalize writes
                                         // the other one while its producer still reads this one)
  // ---- GroupNorm finalize folded into the producing conv (unet.h GnFold) ----
  // OFF by default (ERTD_UNET_GNFOLD=1 in a diagnostic build): measured on one
  // box, U2 B=64, 248.2 steps/s without vs 238.4 with -- the per-item
  // write-through partials + arrival and the tail's count wait and finalize
  // add ~6 us per producing conv, more than the ~5 us finalize launch they
  // replace (profiles/r05_gnfold_ab.txt).
  // The walk's conv and GroupNorm calls are recorded as events; a dry pass of
  // the same walk (plan_folds) finds each fold-capable conv whose output is
  // the A input of the very next GroupNorm, and the real walk hands that conv
  // the GroupNorm's finalize (the GroupNorm then launches nothing).
  struct Ev {
    bool gn;            // GroupNorm (else conv)
    bool foldable;      // conv: its dispatched kernel takes ConvArgs::fold
    int prod = -1;      // GroupNorm: the conv event that produced A (-1: none)
    int prodB = -2;     // GroupNorm: ... produced Bs (-2: no Bs, -1: unknown)
    int Cb = 0, HW = 0;
    std::string name;
  };
  std::vector<Ev> evs;
  std::vector<const float*> ev_out;          // event -> the conv's output tensor (null: GroupNorm)
  std::map<const float*, int> producer;      // tensor -> conv event
  std::vector<int> fold_at;                  // real walk: conv event -> folded GroupNorm event
  std::vector<Ev> plan_evs;
  unsigned* fold_cnt = nullptr;              // (B) arrival counters (fixed(); zeroed by conv_in)
  bool cnt_zeroed = false;                   // conv_in ran with the zeroing: folds may follow
  struct PendFold {
    int gn_ev = -1;
    float2* buf = nullptr;
  } pfold;
  static int fold_env() {
    static const int v = [] {
      return ERTD_KNOB("UNET_GNFOLD", 0);
    }();
    return v;
  }
  float2* next_gnbuf() const { return gnbuf == gnb[0] ? gnb[1] : gnb[0]; }
  void plan_folds() {
    Walk d{c, L, pk, nullptr, 0, B, nullptr, true};
    d.fold_cnt = reinterpret_cast<unsigned*>(16);   // plan as the real walk (never dereferenced)
    d.unet(nullptr, nullptr, nullptr);
    plan_evs = d.evs;
    fold_at.assign(plan_evs.size(), -1);
    for (size_t i = 0; i < plan_evs.size(); ++i) {
      if (plan_evs[i].gn || !plan_evs[i].foldable) continue;
      size_t j = i + 1;
      while (j < plan_evs.size() && !plan_evs[j].gn) ++j;
      if (j == plan_evs.size() || plan_evs[j].prod != (int)i || plan_evs[j].prodB == -1) continue;
      fold_at[i] = (int)j;
    }
  }
  // plan capture only: a side stream (forked/joined with events) on which a
  // ResBlock's 1x1 skip conv runs concurrently with its conv1 -- a branch of
  // the step graph that fills conv1's tail
  hipStream_t s2 = nullptr;
  hipEvent_t evf = nullptr, evj = nullptr;
  hipEvent_t emb_join = nullptr;   // embedding branch not yet joined (first conv1 waits)

  // bf16: the statistics of a 3x3 GN+SiLU conv's input are computed by the
  // fused gn_act_bf16_kernel together with its bf16 image (one read of the
  // activation); the launch is deferred to conv()
  GnArgs pend{};
  bool has_pend = false;
  static bool fuse_gn_env() {
    static const bool v = [] {
      return ERTD_KNOB("UNET_BF16_FUSEGN", 1) != 0;
    }();
    return v;
  }

  // fp32: a GroupNorm finalize not yet launched -- the next conv either takes
  // it into its prologue (conv_gn_consume_ok) or launches it first
  GnPartArgs pend_fin{};
  bool has_pend_fin = false;
  void flush_fin() {
    if (!has_pend_fin) return;
    has_pend_fin = false;
    chk(launch_gn_finalize(pend_fin, B, s));
  }

  // fp32: GroupNorm partials per activation tensor (unet.h, GnPartArgs) --
  // emitted by the Winograd convs' epilogues, else computed once by a
  // partials pass (conv_in, Downsample, Upsample outputs) -- so a GroupNorm
  // costs a finalize over B x C x np partials instead of a read of the tensor
  struct PartRec {
    float2* p;
    int np;
  };
  std::map<const float*, PartRec> parts;
  static bool gn_fuse_env() {
    static const bool v = [] {
      return ERTD_KNOB("UNET_GNFUSE", 1) != 0;
    }();
    return v;
  }
  // every precision: the fp32 Winograd and the bf16 pre-transformed-image
  // convs emit partials of their outputs; bf16 then applies GN(+SiLU) in the
  // image pass (act_bf16_kernel) without reading the activation for statistics
  bool gn_parts_on() const { return gn_fuse_env(); }
  const PartRec& parts_of(const float* X, int C, int HW) {
    auto it = parts.find(X);
    if (it != parts.end()) return it->second;
    const int np = HW / 256;   // gn_stats only takes this path when HW % 256 == 0
    float2* p = (float2*)alloc((size_t)B * C * np * 2);
    if (!dry) chk(launch_gn_partials(X, C, HW, np, p, B, s));
    return parts[X] = PartRec{p, np};
  }

  void gn_stats(const float* A, int Ca, const float* Bs, int Cb, int HW, const std::string& n,
                bool fusable = false) {
    {
      Ev e{true, false};
      const auto pa = producer.find(A);
      e.prod = pa != producer.end() ? pa->second : -1;
      if (Cb > 0) {
        const auto pb = producer.find(Bs);
        e.prodB = pb != producer.end() ? pb->second : -1;
      }
      e.Cb = Cb;
      e.HW = HW;
      e.name = n;
      evs.push_back(e);
      ev_out.push_back(nullptr);
    }
    if (pfold.gn_ev >= 0) {   // finalized by its producer's last arrivals
      const bool mine = pfold.gn_ev == (int)evs.size() - 1;
      if (!mine) chk(hipErrorInvalidValue);   // the plan and the walk disagree
      gnbuf = pfold.buf;
      pfold = PendFold{};
      if (mine && fold_env() < 2) return;
      // diagnostic builds: the finalize launched as well, into the other buffer
      // (ERTD_UNET_GNFOLD=2) or over the folded one (3)
      if (fold_env() == 2) gnbuf = next_gnbuf();
    } else {
      gnbuf = next_gnbuf();
    }
    float2* const out = gnbuf;
    if (gn_parts_on() && HW % 256 == 0) {
      const PartRec ra = parts_of(A, Ca, HW);
      const PartRec rb = Cb > 0 ? parts_of(Bs, Cb, HW) : PartRec{nullptr, 0};
      if (dry) return;
      GnPartArgs g{ra.p, ra.np, Ca, rb.p, rb.np, Cb, HW, c->groups, P(n + ".weight"), P(n + ".bias"),
                   out, nullptr};
      // deferred to the consuming conv: its own prologue finalizes (fp32
      // Winograd F(4x4) consumers, ConvArgs::gnc), else it launches this first
      flush_fin();
      pend_fin = g;
      has_pend_fin = true;
      return;
    }
    if (dry) return;
    GnArgs g{A, Bs, Ca, Cb, HW, c->groups, P(n + ".weight"), P(n + ".bias"), out};
    if (fusable && bf_prec(c->precision) && fuse_gn_env() &&
        gn_act_bf16_fits(Ca + Cb, c->groups, HW)) {
      pend = g;
      has_pend = true;
      return;
    }
    chk(launch_gn_stats(g, B, s));
  }

  // conv over input (A: Ca ch, Bs: Cb ch) at source size Hs x Ws
  float* conv(const std::string& n, int ks, int mode, int act, const float* A, int Ca,
              const float* Bs, int Cb, int Hs, int Ws, const float* ebias, const float* res,
              float* out = nullptr, bool gn_out = true) {
    const Param* wp = nullptr;
    for (const Param& p : L->params)
      if (p.name == n + ".weight") { wp = &p; break; }
    const int Cout = wp->shape[0], Cin = wp->shape[1];
    int Ho = Hs, Wo = Ws;
    if (mode == MODE_S2) { Ho = Hs / 2; Wo = Ws / 2; }
    if (mode == MODE_UP) { Ho = Hs * 2; Wo = Ws * 2; }
    if (!out) out = alloc((size_t)B * Cout * Ho * Wo);
    // fp32 Winograd layers with fewer tile items than CUs split their K
    const bool want_split = c->precision == ERTD_PREC_FP32 && ks == 3 && mode == MODE_S1 &&
                            (L->offw.count(n + ".weight") || L->offw4.count(n + ".weight")) &&
                            conv_wino_ok(Cin, Ca, Cout, Wo) && wino_ksplit_wanted(Cin, Cout, Wo, B);
    float* kbuf = want_split ? alloc((size_t)B * Cout * Ho * Wo) : nullptr;
    // bf16 stride-1 convs stage a pre-transformed bf16 copy of their input
    float* bimg = nullptr;
    const bool split = c->precision == ERTD_PREC_BF16X3;
    if (bf_prec(c->precision) && ks == 3 && Cout > 1 &&
        ((mode == MODE_S1 && act != ACT_NONE) || (mode == MODE_UP && act == ACT_NONE)))
      bimg = alloc((conv_bf16_image_bytes(Ca + Cb, B, Ho, Wo, split) + 3) / 4);
    // fp32: GroupNorm partials of the output, when the dispatched kernel emits
    // them (the geometry-only part of the dispatch: sentinel pointers in dry runs)
    float2* gnp = nullptr;
    int gnp_np = 0;
    ConvArgs q{};   // the dispatch geometry (sentinel pointers)
    q.Ca = Ca; q.Cb = Cb; q.Cin = Cin; q.Cout = Cout;
    q.Hs = Hs; q.Ws = Ws; q.Ho = Ho; q.Wo = Wo;
    q.ebias = ebias; q.res = res;
    q.wpk_wino = L->offw.count(n + ".weight") ? reinterpret_cast<const float*>(16) : nullptr;
    q.wpk_wino4 = L->offw4.count(n + ".weight") ? reinterpret_cast<const float*>(16) : nullptr;
    q.ksplit_buf = want_split ? reinterpret_cast<float*>(16) : nullptr;
    if (gn_parts_on() && gn_out) {
      const int np = bf_prec(c->precision) ? conv_bf16_gn_parts(ks, mode, act, q, B)
                                           : conv_gn_parts(ks, mode, act, q, B);
      if (np > 0) {
        gnp = (float2*)alloc((size_t)B * Cout * np * 2);
        gnp_np = np;
        parts[out] = PartRec{gnp, np};
      }
    }
    const bool fp32 = c->precision == ERTD_PREC_FP32;
    const bool zero_cnt = fp32 && fold_cnt && fold_env() && conv_in_ok(q, ks, mode, act);
    if (zero_cnt) cnt_zeroed = true;
    const int ev = (int)evs.size();
    {
      Ev e{false, false};
      e.foldable = gnp && fp32 && fold_cnt && cnt_zeroed && fold_env() &&
                   conv_gn_fold_ok(ks, mode, act, q, B);
      evs.push_back(e);
      ev_out.push_back(out);
      producer[out] = ev;
    }
    if (dry) return out;
    if (Cin != Ca + Cb) {
      chk(hipErrorInvalidValue);
      return out;
    }
    ConvArgs a{};
    a.srcA = A; a.srcB = Bs; a.Ca = Ca; a.Cb = Cb;
    a.gn = act != ACT_NONE ? gnbuf : nullptr;
    a.wpk = P(n + ".weight");
    {
      const auto it = L->offw.find(n + ".weight");
      a.wpk_wino = it != L->offw.end() ? pk + it->second : nullptr;
      const auto it4 = L->offw4.find(n + ".weight");
      a.wpk_wino4 = it4 != L->offw4.end() ? pk + it4->second : nullptr;
    }
    a.bias = P(n + ".bias");
    a.ebias = ebias; a.eb_stride = L->ebtotal;
    a.res = res; a.out = out;
    a.Cin = Cin; a.Cout = Cout;
    a.Hs = Hs; a.Ws = Ws; a.Ho = Ho; a.Wo = Wo;
    a.bimg = bimg;
    a.ksplit_buf = kbuf;
    a.gnp = gnp;
    a.split = split ? 1 : 0;
    if (zero_cnt) {
      a.zero_words = fold_cnt;
      a.zero_n = B;
    }
    if (ev < (int)fold_at.size() && fold_at[ev] >= 0 && gnp) {
      const Ev& g = plan_evs[fold_at[ev]];
      const float* Bs2 = g.Cb > 0 ? ev_out[g.prodB] : nullptr;
      const PartRec rb = g.Cb > 0 ? parts_of(Bs2, g.Cb, g.HW) : PartRec{nullptr, 0};
      float2* const tgt = next_gnbuf();
      a.fold.g = GnPartArgs{gnp, gnp_np, Cout, rb.p, rb.np, g.Cb, g.HW, c->groups,
                            P(g.name + ".weight"), P(g.name + ".bias"), tgt, nullptr};
      a.fold.cnt = fold_cnt;
      a.fold.target = conv_gn_fold_target(a, B);
      a.fold.B = B;
      pfold = PendFold{fold_at[ev], tgt};
    }
    if (has_pend_fin) {
      ConvArgs t = a;
      t.gnc = pend_fin;
      t.gnc.out = nullptr;
      t.gn = nullptr;
      if (act != ACT_NONE && a.gn == pend_fin.out && conv_gn_consume_ok(ks, mode, act, t, B)) {
        a = t;
        has_pend_fin = false;
      } else {
        flush_fin();
      }
    }
    if (has_pend) {
      has_pend = false;
      if (bimg && ks == 3 && mode == MODE_S1 && act == ACT_GN_SILU) {
        chk(launch_gn_act_bf16(pend, true, bimg, B, s, split));
        a.bimg_ready = 1;
      } else {
        chk(launch_gn_stats(pend, B, s));
      }
    }
    chk(bf_prec(c->precision) ? launch_conv_bf16(ks, mode, act, a, B, s)
                              : launch_conv(ks, mode, act, a, B, s));
    return out;
  }

  float* resblock(const std::string& n, const float* A, int Ca, const float* Bs, int Cb, int Hh,
                  int Ww, int cout, const float* ebias_all) {
    const int HW = Hh * Ww;
    const float* eb = ebias_all ? ebias_all + L->eboff.at(n) : nullptr;
    gn_stats(A, Ca, Bs, Cb, HW, n + ".norm1", true);
    const bool skip = Ca + Cb != cout;
    const bool side = skip && s2 && !dry;
    if (side) {   // fork: the skip conv only needs the block input
      chk(hipEventRecord(evf, s));
      chk(hipStreamWaitEvent(s2, evf, 0));
    }
    if (emb_join && !dry) {   // conv1's epilogue adds the embedding bias
      chk(hipStreamWaitEvent(s, emb_join, 0));
      emb_join = nullptr;
    }
    float* h1 = conv(n + ".conv1", 3, MODE_S1, ACT_GN_SILU, A, Ca, Bs, Cb, Hh, Ww, eb, nullptr);
    const float* resid = A;
    if (skip) {
      const hipStream_t s0 = s;
      if (side) s = s2;
      resid = conv(n + ".skip", 1, MODE_S1, ACT_NONE, A, Ca, Bs, Cb, Hh, Ww, nullptr, nullptr);
      s = s0;
      if (side) chk(hipEventRecord(evj, s2));
    }
    gn_stats(h1, cout, nullptr, 0, HW, n + ".norm2", true);
    if (side) chk(hipStreamWaitEvent(s, evj, 0));   // join before conv2 reads the residual
    return conv(n + ".conv2", 3, MODE_S1, ACT_GN_SILU, h1, cout, nullptr, 0, Hh, Ww, nullptr, resid);
  }

  // x (B, image^2) -> eps (B, image^2); emb_act source = ebias_all (B, ebtotal)
  void unet(const float* x, const float* ebias_all, float* eps) {
    if (!dry && fold_cnt && fold_env() && c->precision == ERTD_PREC_FP32) plan_folds();
    const int nl = c->n_levels;
    int Hh = c->image;
    std::vector<std::pair<const float*, int>> hs;
    const float* h = conv("conv_in", 3, MODE_S1, ACT_NONE, x, 1, nullptr, 0, Hh, Hh, nullptr,
                          nullptr);
    int ch = c->ch;
    hs.push_back({h, ch});
    for (int i = 0; i < nl; ++i) {
      for (int r = 0; r < c->num_res; ++r) {
        const int o = c->ch * c->ch_mult[i];
        h = resblock("down." + std::to_string(i) + ".res." + std::to_string(r), h, ch, nullptr, 0,
                     Hh, Hh, o, ebias_all);
        ch = o;
        hs.push_back({h, ch});
      }
      if (i != nl - 1) {
        h = conv("down." + std::to_string(i) + ".downsample", 3, MODE_S2, ACT_NONE, h, ch, nullptr,
                 0, Hh, Hh, nullptr, nullptr);
        Hh /= 2;
        hs.push_back({h, ch});
      }
    }
    h = resblock("mid.res1", h, ch, nullptr, 0, Hh, Hh, ch, ebias_all);
    if (c->attn) {
      gn_stats(h, ch, nullptr, 0, Hh * Hh, "mid.attn.norm");
      float* qkv = conv("mid.attn.qkv", 1, MODE_S1, ACT_GN, h, ch, nullptr, 0, Hh, Hh, nullptr,
                        nullptr);
      float* o = alloc((size_t)B * ch * Hh * Hh);
      if (!dry) chk(launch_attention(qkv, ch, Hh * Hh, o, nullptr, B, s));
      h = conv("mid.attn.proj", 1, MODE_S1, ACT_NONE, o, ch, nullptr, 0, Hh, Hh, nullptr, h);
    }
    h = resblock("mid.res2", h, ch, nullptr, 0, Hh, Hh, ch, ebias_all);
    for (int i = nl - 1; i >= 0; --i) {
      for (int r = 0; r <= c->num_res; ++r) {
        const int o = c->ch * c->ch_mult[i];
        const auto sk = hs.back();
        hs.pop_back();
        h = resblock("up." + std::to_string(i) + ".res." + std::to_string(r), h, ch, sk.first,
                     sk.second, Hh, Hh, o, ebias_all);
        ch = o;
      }
      if (i != 0) {
        h = conv("up." + std::to_string(i) + ".upsample", 3, MODE_UP, ACT_NONE, h, ch, nullptr, 0,
                 Hh, Hh, nullptr, nullptr);
        Hh *= 2;
      }
    }
    gn_stats(h, ch, nullptr, 0, Hh * Hh, "norm_out");
    conv("conv_out", 3, MODE_S1, ACT_GN_SILU, h, ch, nullptr, 0, Hh, Hh, nullptr, nullptr, eps);
    if (!dry) flush_fin();   // (every GroupNorm has its consumer: nothing is pending here)
  }

  int max_cin() const {
    int m = 1;
    for (const Param& p : L->params)
      if (p.shape.size() == 4 && p.shape[1] > m) m = p.shape[1];
    return m;
  }

  void dense(int din, const float* xin, int xs, const int64_t* t, const int* tdev,
             const float* freq, const std::string& n, int K, int O, const float* add, int adds,
             float* y, int ys, const float* wt = nullptr, const float* bias = nullptr) {
    if (dry) return;
    DenseArgs d{};
    d.x = xin; d.x_stride = xs; d.t = t; d.t_dev = tdev; d.freq = freq;
    d.wt = wt ? wt : P(n + ".weight");
    d.bias = bias ? bias : P(n + ".bias");
    d.add = add; d.add_stride = adds; d.add_bcast = 0;
    d.y = y; d.y_stride = ys; d.K = K; d.O = O;
    chk(launch_dense(din, d, B, s));
  }
};

// Persistent per-call buffers at the head of the workspace.
struct Fixed {
  float* cond_emb;   // (B, 128)
  float* cproj;      // (B, temb)
  float* e1;         // (B, temb)
  float* emb;        // (B, temb)
  float* ebias;      // (B, ebtotal)
  float* eps;        // (B, P)
  float* freq;       // (ch/2)
  float* partial;    // encoder strips (B, S, 64)
  float* Uscr;       // (B, 128)
  int* tdev;         // step counter word
};

Fixed fixed(Walk& w, int L) {
  Fixed f{};
  const int B = w.B, tb = temb(w.c);
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  f.cond_emb = w.alloc((size_t)B * H);
  f.cproj = w.alloc((size_t)B * tb);
  f.e1 = w.alloc((size_t)B * tb);
  f.emb = w.alloc((size_t)B * tb);
  f.ebias = w.alloc((size_t)B * w.L->ebtotal);
  f.eps = w.alloc((size_t)B * w.c->image * w.c->image);
  f.freq = w.alloc((size_t)w.c->ch / 2);
  f.partial = w.alloc((size_t)B * S * C2);
  f.Uscr = w.alloc((size_t)B * H);
  f.tdev = (int*)w.alloc(64);
  w.gnb[0] = (float2*)w.alloc((size_t)B * w.max_cin() * 2);
  w.gnb[1] = (float2*)w.alloc((size_t)B * w.max_cin() * 2);
  w.gnbuf = w.gnb[0];
  w.fold_cnt = (unsigned*)w.alloc((size_t)B);
  return f;
}

ertd_weights enc_weights(const Layout& L, const float* pk, const float* const* params) {
  ertd_weights e{};
  e.enc0_w = params[0]; e.enc0_b = params[1];
  e.enc2_w = params[2]; e.enc2_b = params[3];
  e.enc6_w = params[4]; e.enc6_b = params[5];
  const float* d = pk + L.dummy;
  e.time_w = d; d += H * H;
  e.time_b = d; d += H;
  e.mlp0_w = d; d += (size_t)H * (1 + 2 * H);
  e.mlp0_b = d; d += H;
  e.mlp2_w = d; d += H;
  e.mlp2_b = d;
  e.param_dim = 1;
  e.hidden_dim = H;
  return e;
}

// encoder weights as seen by the strip/pool kernels after packing: the biases
// and enc6 are read from the packed copies (no params pointer needed at run time)
ertd_weights enc_weights_packed(const Layout& L, const float* pk) {
  const float* const* none = nullptr;
  (void)none;
  ertd_weights e{};
  const float* d = pk + L.dummy;
  e.time_w = d; d += H * H;
  e.time_b = d; d += H;
  e.mlp0_w = d; d += (size_t)H * (1 + 2 * H);
  e.mlp0_b = d; d += H;
  e.mlp2_w = d; d += H;
  e.mlp2_b = d;
  e.enc0_w = pk + L.off.at("enc.0.weight");
  e.enc0_b = pk + L.off.at("enc.0.bias");
  e.enc2_w = pk + L.off.at("enc.2.weight");
  e.enc2_b = pk + L.off.at("enc.2.bias");
  e.enc6_w = pk + L.off.at("enc.6.weight");
  e.enc6_b = pk + L.off.at("enc.6.bias");
  e.param_dim = 1;
  e.hidden_dim = H;
  return e;
}

Layout layout_full(const ertd_unet_config* c) {
  Layout L = layout(c);
  // verbatim copies of the encoder parameters (the encoder kernels read its
  // biases and enc6 directly), appended at the end
  const char* names[6] = {"enc.0.weight", "enc.0.bias", "enc.2.weight",
                          "enc.2.bias", "enc.6.weight", "enc.6.bias"};
  for (int i = 0; i < 6; ++i) {
    L.off[names[i]] = L.total;
    L.total += a64(L.params[i].numel());
  }
  return L;
}

// cond (B,14,Lc) -> cond_emb -> cproj; once per forward / sampler call
int prologue(Walk& w, const Fixed& f, const float* cond, long long cstride, int Lc) {
  const float* pk = w.pk;
  const ertd_weights e = enc_weights_packed(*w.L, pk);
  const int L2 = conv_len(conv_len(Lc)), S = n_strips(L2);
  w.chk(launch_encoder_strips(pk + w.L->enc, e.enc0_b, e.enc2_b, cond, cstride, w.B, Lc,
                              ERTD_PREC_FP32, f.partial, w.s));
  w.chk(launch_hoist_prep(e, pk + w.L->enc, f.partial, S, L2, w.B, f.Uscr, f.cond_emb, w.s));
  w.dense(DIN_PLAIN, f.cond_emb, H, nullptr, nullptr, nullptr, "cond_proj", H, temb(w.c), nullptr,
          0, f.cproj, temb(w.c));
  // sinusoid frequencies exp(-i*ln(1e4)/(half-1)) (float32, as the reference's
  // get_timestep_embedding) are packed on the host side into "freq"
  return w.err == hipSuccess ? ERTD_OK : (int)w.err;
}

// t (per-sample) or *tdev -> emb -> all ResBlock emb biases
void embed(Walk& w, const Fixed& f, const int64_t* t) {
  const int tb = temb(w.c);
  w.dense(DIN_SINUSOID, nullptr, 0, t, f.tdev, w.pk + w.L->off.at("freq"), "time_embed.0", w.c->ch,
          tb, nullptr, 0, f.e1, tb);
  w.dense(DIN_SILU, f.e1, tb, nullptr, nullptr, nullptr, "time_embed.2", tb, tb, f.cproj, tb, f.emb,
          tb);
  w.dense(DIN_SILU, f.emb, tb, nullptr, nullptr, nullptr, "", tb, w.L->ebtotal, nullptr, 0, f.ebias,
          w.L->ebtotal, w.pk + w.L->wall, w.pk + w.L->ball);
}

Layout layout_with_freq(const ertd_unet_config* c) {
  Layout L = layout_full(c);
  L.off["freq"] = L.total;
  L.total += a64((size_t)c->ch / 2);
  return L;
}

size_t ws_bytes_for(const ertd_unet_config* c, const Layout& L, int B, int Lc) {
  Walk w{c, &L, nullptr, nullptr, 0, B, nullptr, true};
  fixed(w, Lc);
  w.unet(nullptr, nullptr, nullptr);
  return w.used;
}

inline int rcode(hipError_t e) { return e == hipSuccess ? ERTD_OK : (int)e; }

// One sampler call: head = encoder + cond_proj + t := t_first; step = one
// reverse step (embedding, U-Net, update, t := t - 1) reading t from the
// workspace word, so the same step can be replayed as a graph.
struct SampleCall {
  const ertd_unet_config* c;
  const float* packed; const float* cond; long long cond_stride; int L; int B;
  int num_steps; int t_first; int n_run;
  const float* c1; const float* c2; const float* sigma; const float* noise;
  uint64_t seed; uint32_t member_offset; float* x; void* ws; size_t ws_bytes;

  int check() const {
    if (!cfg_ok(c) || !packed || !cond || !c1 || !c2 || !sigma || !x || !ws || B < 1 || L < 1 ||
        num_steps < 1 || t_first < 0 || t_first >= num_steps || n_run < 0 || n_run > t_first + 1)
      return ERTD_EINVAL;
    const Layout Lo = layout_with_freq(c);
    if (ws_bytes_for(c, Lo, B, L) > ws_bytes) return ERTD_ENOSPC;
    return ERTD_OK;
  }
  int head(hipStream_t s) const {
    const Layout Lo = layout_with_freq(c);
    Walk w{c, &Lo, packed, (char*)ws, 0, B, s, false};
    w.cap = ws_bytes;
    const Fixed f = fixed(w, L);
    const int r = prologue(w, f, cond, cond_stride, L);
    if (r != ERTD_OK) return r;
    w.chk(launch_set_word(f.tdev, t_first, s));
    return rcode(w.err);
  }
  // skip_side: the ResBlock skip convs on s2 too (else only the embedding branch)
  int step(hipStream_t s, hipStream_t s2 = nullptr, hipEvent_t evf = nullptr,
           hipEvent_t evj = nullptr, hipEvent_t eve = nullptr, bool skip_side = true) const {
    const Layout Lo = layout_with_freq(c);
    Walk w{c, &Lo, packed, (char*)ws, 0, B, s, false};
    w.cap = ws_bytes;
    w.s2 = skip_side ? s2 : nullptr;
    w.evf = evf;
    w.evj = evj;
    const Fixed f = fixed(w, L);
    const int P = c->image * c->image;
    if (s2 && eve) {
      // the embedding dense layers run beside conv_in and the first norm1
      w.chk(hipEventRecord(evf, s));
      w.chk(hipStreamWaitEvent(s2, evf, 0));
      w.s = s2;
      embed(w, f, nullptr);
      w.s = s;
      w.chk(hipEventRecord(eve, s2));
      w.emb_join = eve;
    } else {
      embed(w, f, nullptr);
    }
    w.unet(x, f.ebias, f.eps);
    UpdateArgs u{x, f.eps, c1, c2, sigma, noise, num_steps, f.tdev, seed, member_offset, P};
    w.chk(launch_unet_update(u, B, s));
    w.chk(launch_dec_word(f.tdev, s));
    return rcode(w.err);
  }
};

}  // namespace

struct ertd_unet_plan {
  ertd_unet_config cfg{};
  SampleCall call{};
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;            // skip-conv branch of the step graph
  hipEvent_t evf = nullptr, evj = nullptr, eve = nullptr;
  hipGraph_t g_head = nullptr, g_step = nullptr;
  hipGraphExec_t x_head = nullptr, x_step = nullptr;
  // MULTI consecutive steps captured as one graph: one launch (and its ~8 us
  // graph-boundary gap) per MULTI steps instead of per step
  hipGraph_t g_multi = nullptr;
  hipGraphExec_t x_multi = nullptr;
  int multi = 0;
  bool skip_side = false;                // the skip convs on the side stream too
};

extern "C" {

// ---- single operators of the U-Net (the SURVEY 8a' operator rows), for
// per-operator parity tests and microbenchmarks -----------------------------
}  // extern "C"

namespace {
// Caller-owned workspace of one ertd_conv2d call: the packed weights (every
// layout the dispatch may read), then the stream-ordered scratch the launch
// needs -- a Winograd K split's second half (fp32) or the pre-transformed bf16
// input image -- so the library never allocates (include/ertdiff.h).
struct Conv2dWs {
  size_t pack_floats = 0;   // packed weights (floats, 64-aligned)
  size_t kbuf_floats = 0;   // fp32 Winograd K-split partial (B, Cout, Ho, Ho)
  size_t bimg_bytes = 0;    // bf16 image
  size_t total() const { return a64(pack_floats) * sizeof(float) + a64(kbuf_floats) * sizeof(float) +
                                (bimg_bytes + 255) / 256 * 256; }
};

bool conv2d_geom_ok(int cin, int cout, int ks, int precision, int B, int H, int mode) {
  return cin >= 1 && cout >= 1 && (ks == 1 || ks == 3) && B >= 1 && H >= 1 && mode >= MODE_S1 &&
         mode <= MODE_UP && !(ks == 1 && mode != MODE_S1) &&
         (precision == ERTD_PREC_FP32 || bf_prec(precision));
}

Conv2dWs conv2d_ws(int cin, int ca, int cout, int ks, int precision, int B, int H, int mode, int act) {
  Conv2dWs w;
  const bool bf = bf_prec(precision), split = precision == ERTD_PREC_BF16X3;
  size_t f = bf ? conv_packed_floats_bf16(cin, cout, ks, split) : conv_packed_floats(cin, cout, ks);
  // fp32 3x3 convs may be Upsample convs (sub-pixel packing)
  if (!bf && ks == 3 && conv_packed_floats_up(cin, cout) > f)
    f = conv_packed_floats_up(cin, cout);
  // ... and stride-1 ones carry the Winograd packing behind the direct one
  if (!bf && ks == 3)
    f = a64(f) + std::max(conv_packed_floats_wino(cin, cout), conv_packed_floats_wino4(cin, cout));
  w.pack_floats = f;
  const int Ho = mode == MODE_S2 ? H / 2 : (mode == MODE_UP ? 2 * H : H);
  if (!bf && ks == 3 && mode == MODE_S1 && cout > 1 &&
      (conv_packed_floats_wino(cin, cout) > 0 || conv_packed_floats_wino4(cin, cout) > 0) &&
      conv_wino_ok(cin, ca, cout, Ho) && wino_ksplit_wanted(cin, cout, Ho, B))
    w.kbuf_floats = (size_t)B * cout * Ho * Ho;
  if (bf && ks == 3 && cout > 1 &&
      ((mode == MODE_S1 && act != ACT_NONE) || (mode == MODE_UP && act == ACT_NONE)))
    w.bimg_bytes = conv_bf16_image_bytes(cin, B, Ho, Ho, split);
  return w;
}

}  // namespace

extern "C" {

size_t ertd_conv2d_workspace_bytes(int cin, int cout, int ks, int precision, int B, int H, int mode) {
  if (!conv2d_geom_ok(cin, cout, ks, precision, B, H, mode)) return 0;
  // the K-split / image scratch does not depend on the activation except for
  // the bf16 image, which stride-1 convs need only with an activation: size
  // for the larger of the two cases (ca = cin: the split depends on Cin only)
  const Conv2dWs a = conv2d_ws(cin, cin, cout, ks, precision, B, H, mode, ACT_GN_SILU);
  const Conv2dWs b = conv2d_ws(cin, cin, cout, ks, precision, B, H, mode, ACT_NONE);
  return std::max(a.total(), b.total());
}

namespace {
// which Winograd layout ertd_conv2d dispatches (geometry only)
void conv2d_wino_flags(int Cin, int Ca, int Cout, int ks, int mode, int act, int precision, int B, int Ho,
                       bool* wino, bool* wino4) {
  const bool bf = bf_prec(precision);
  *wino4 = !bf && ks == 3 && Cout > 1 && conv_packed_floats_wino4(Cin, Cout) > 0 &&
           ((mode == MODE_S1 && wino4_ok(Cin, Ca, Cout, Ho, B)) ||
            (mode == MODE_UP && act == ACT_NONE && wino4s_up_ok(Cin, Ca, Cout, Ho, B)));
  *wino = *wino4 || (!bf && ks == 3 && mode == MODE_S1 && Cout > 1 &&
                     conv_packed_floats_wino(Cin, Cout) > 0 && conv_wino_ok(Cin, Ca, Cout, Ho));
}

// ertd_conv2d: pack (unless `pack` is false: ws already holds this shape's
// packing from an earlier call) and launch; gnp (B, Cout, gn_np) float2: the
// GroupNorm partials of the output from the epilogue (gn_np must be what
// ertd_conv2d_gn_parts returns for the call, > 0)
int conv2d_impl(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* w,
                const float* bias, int Cout, int ks, int mode, const float* gn, int act,
                const float* ebias, int eb_stride, const float* res, float* out, int precision,
                void* ws, size_t ws_bytes, void* stream, bool pack, float* gnp = nullptr, int gn_np = 0) {
  const int Cin = Ca + Cb;
  if (!x || (pack && !w) || !bias || !out || !ws || B < 1 || Ca < 1 || Cb < 0 || (Cb > 0 && !x2) ||
      !conv2d_geom_ok(Cin, Cout, ks, precision, B, H, mode) || act < ACT_NONE || act > ACT_GN ||
      (act != ACT_NONE && !gn))
    return ERTD_EINVAL;
  const Conv2dWs need = conv2d_ws(Cin, Ca, Cout, ks, precision, B, H, mode, act);
  if (need.total() > ws_bytes) return ERTD_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  float* pk = (float*)ws;
  // caller-owned scratch behind the packing (stream-ordered: reused by the next call)
  float* kbuf = need.kbuf_floats ? pk + a64(need.pack_floats) : nullptr;
  void* bimg = need.bimg_bytes ? (void*)(pk + a64(need.pack_floats) + a64(need.kbuf_floats)) : nullptr;
  // the Winograd path reads only its own packing: skip the direct one then
  const int Ho_ = mode == MODE_S2 ? H / 2 : (mode == MODE_UP ? 2 * H : H);
  const bool bf = bf_prec(precision), split = precision == ERTD_PREC_BF16X3;
  bool wino, wino4;
  conv2d_wino_flags(Cin, Ca, Cout, ks, mode, act, precision, B, Ho_, &wino, &wino4);
  if (gnp && (bf || gn_np < 1)) return ERTD_EINVAL;
  hipError_t e = hipSuccess;
  if (!wino && pack)
    e = bf ? launch_pack_conv_bf16(w, Cin, Cout, ks, pk, s, split)
        : (ks == 3 && mode == MODE_UP) ? launch_pack_conv_up(w, Cin, Cout, pk, s)
                                       : launch_pack_conv(w, Cin, Cout, ks, pk, s);
  if (e != hipSuccess) return (int)e;
  ConvArgs a{};
  a.srcA = x; a.srcB = x2; a.Ca = Ca; a.Cb = Cb;
  a.gn = (const float2*)gn;
  a.wpk = pk; a.bias = bias; a.ebias = ebias; a.eb_stride = eb_stride; a.res = res; a.out = out;
  a.Cin = Cin; a.Cout = Cout; a.Hs = H; a.Ws = H;
  a.Ho = Ho_;
  a.Wo = a.Ho;
  if (wino) {
    float* pw = pk + a64(std::max(conv_packed_floats(Cin, Cout, ks), conv_packed_floats_up(Cin, Cout)));
    if (pack && (e = wino4 ? launch_pack_conv_wino4(w, Cin, Cout, pw, s)
                           : launch_pack_conv_wino(w, Cin, Cout, pw, s)) != hipSuccess)
      return (int)e;
    if (wino4) a.wpk_wino4 = pw; else a.wpk_wino = pw;
    a.ksplit_buf = kbuf;
  }
  a.bimg = bimg;
  a.split = split ? 1 : 0;
  if (gnp) {
    if (conv_gn_parts(ks, mode, act, a, B) != gn_np) return ERTD_EINVAL;
    a.gnp = (float2*)gnp;
  }
  e = bf ? launch_conv_bf16(ks, mode, act, a, B, s) : launch_conv(ks, mode, act, a, B, s);
  return e == hipErrorInvalidValue ? ERTD_EINVAL : rcode(e);
}
}  // namespace

int ertd_conv2d(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* w,
                const float* bias, int Cout, int ks, int mode, const float* gn, int act,
                const float* ebias, int eb_stride, const float* res, float* out, int precision,
                void* ws, size_t ws_bytes, void* stream) {
  return conv2d_impl(x, Ca, x2, Cb, B, H, w, bias, Cout, ks, mode, gn, act, ebias, eb_stride, res, out,
                     precision, ws, ws_bytes, stream, true);
}

int ertd_conv2d_run(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* bias,
                    int Cout, int ks, int mode, const float* gn, int act, const float* ebias,
                    int eb_stride, const float* res, float* out, int precision, void* ws,
                    size_t ws_bytes, void* stream) {
  return conv2d_impl(x, Ca, x2, Cb, B, H, nullptr, bias, Cout, ks, mode, gn, act, ebias, eb_stride, res,
                     out, precision, ws, ws_bytes, stream, false);
}

int ertd_conv2d_gn_parts(int Ca, int Cb, int Cout, int ks, int mode, int act, int precision, int B, int H) {
  const int Cin = Ca + Cb;
  if (Ca < 1 || Cb < 0 || !conv2d_geom_ok(Cin, Cout, ks, precision, B, H, mode) || bf_prec(precision) ||
      act < ACT_NONE || act > ACT_GN)
    return 0;
  const int Ho = mode == MODE_S2 ? H / 2 : (mode == MODE_UP ? 2 * H : H);
  bool wino, wino4;
  conv2d_wino_flags(Cin, Ca, Cout, ks, mode, act, precision, B, Ho, &wino, &wino4);
  const Conv2dWs need = conv2d_ws(Cin, Ca, Cout, ks, precision, B, H, mode, act);
  // the dispatch reads only which pointers are set: sentinels, as the walk's dry run
  const float* sent = reinterpret_cast<const float*>(16);
  ConvArgs q{};
  q.Ca = Ca; q.Cb = Cb; q.Cin = Cin; q.Cout = Cout;
  q.Hs = H; q.Ws = H; q.Ho = Ho; q.Wo = Ho;
  q.wpk_wino4 = wino4 ? sent : nullptr;
  q.wpk_wino = wino && !wino4 ? sent : nullptr;
  q.ksplit_buf = wino && need.kbuf_floats ? const_cast<float*>(sent) : nullptr;
  return conv_gn_parts(ks, mode, act, q, B);
}

int ertd_conv2d_gn(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* w,
                   const float* bias, int Cout, int ks, int mode, const float* gn, int act,
                   const float* ebias, int eb_stride, const float* res, float* out, int precision,
                   void* ws, size_t ws_bytes, float* gn_parts, int gn_np, void* stream) {
  if (!gn_parts) return ERTD_EINVAL;
  return conv2d_impl(x, Ca, x2, Cb, B, H, w, bias, Cout, ks, mode, gn, act, ebias, eb_stride, res, out,
                     precision, ws, ws_bytes, stream, true, gn_parts, gn_np);
}

int ertd_conv2d_run_gn(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* bias,
                       int Cout, int ks, int mode, const float* gn, int act, const float* ebias,
                       int eb_stride, const float* res, float* out, int precision, void* ws,
                       size_t ws_bytes, float* gn_parts, int gn_np, void* stream) {
  if (!gn_parts) return ERTD_EINVAL;
  return conv2d_impl(x, Ca, x2, Cb, B, H, nullptr, bias, Cout, ks, mode, gn, act, ebias, eb_stride, res,
                     out, precision, ws, ws_bytes, stream, false, gn_parts, gn_np);
}

// dX (B, Cin, H, H) (+)= the input gradient of y = conv(x) (Cout, Cin, ks, ks; mode as
// ertd_conv2d) given dY (B, Cout, Ho, Ho): a stride-1 conv of dY (stride 2: of dY
// zero-inserted to H; upsample: at 2H, then 2x2 sum-pooled) with the weight
// transposed and flipped -- packed straight from w (Winograd where eligible).
size_t ertd_conv_input_grad_ws_bytes(int Cin, int Cout, int B, int H, int ks, int mode) {
  if (Cin < 1 || Cout < 1 || B < 1 || H < 1 || (ks != 1 && ks != 3) || mode < MODE_S1 ||
      mode > MODE_UP || (ks == 1 && mode != MODE_S1))
    return 0;
  // packing (either layout) + the zero-inserted dY (stride 2) or the 2H gradient (upsample)
  size_t n = a64(std::max(conv_packed_floats(Cout, Cin, ks),
                          std::max(conv_packed_floats_wino(Cout, Cin), conv_packed_floats_wino4(Cout, Cin))));
  if (mode == MODE_S2) n += a64((size_t)B * Cout * H * H);
  if (mode == MODE_UP) n += a64((size_t)B * Cin * 4 * H * H);
  const int Hg = mode == MODE_UP ? 2 * H : H;
  if (ks == 3) n += a64((size_t)B * Cin * Hg * Hg);   // a Winograd K split's second half
  return n * sizeof(float);
}

}  // extern "C"

namespace {
// the gradient conv's packing: Winograd F(4x4) / F(2x2) where eligible, else direct,
// at the head of ws (flipped, transposed)
int input_grad_kind(int Cin, int Cout, int B, int H, int ks, int mode) {
  const int Hg = mode == MODE_UP ? 2 * H : H;
  if (ks == 3 && Cin > 1 && conv_packed_floats_wino4(Cout, Cin) > 0 && wino4_ok(Cout, Cout, Cin, Hg, B))
    return ERTD_PACK_WINO4;
  if (ks == 3 && Cin > 1 && conv_packed_floats_wino(Cout, Cin) > 0 && conv_wino_ok(Cout, Cout, Cin, Hg))
    return ERTD_PACK_WINO;
  return ERTD_PACK_DIRECT;
}

int input_grad_impl(const float* dy, int B, int H, const float* w, int Cout, int Cin, int ks, int mode,
                    float* dx, int accumulate, void* ws, size_t ws_bytes, void* stream, bool pack) {
  const size_t need = ertd_conv_input_grad_ws_bytes(Cin, Cout, B, H, ks, mode);
  if (!dy || (pack && !w) || !dx || !ws || need == 0) return ERTD_EINVAL;
  if (need > ws_bytes) return ERTD_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  float* pk = (float*)ws;
  float* scratch = pk + a64(std::max(conv_packed_floats(Cout, Cin, ks),
                                     std::max(conv_packed_floats_wino(Cout, Cin),
                                              conv_packed_floats_wino4(Cout, Cin))));
  // the gradient conv: Cin_g = Cout, Cout_g = Cin, at resolution Hg
  const int Hg = mode == MODE_UP ? 2 * H : H;
  const float* src = dy;
  if (mode == MODE_S2) {
    hipError_t e = launch_zero_insert(dy, B, Cout, H / 2, scratch, s);
    if (e != hipSuccess) return (int)e;
    src = scratch;
  }
  ConvArgs a{};
  a.srcA = src; a.Ca = Cout; a.Cb = 0;
  a.Cin = Cout; a.Cout = Cin;
  a.Hs = a.Ws = a.Ho = a.Wo = Hg;
  const int kind = input_grad_kind(Cin, Cout, B, H, ks, mode);
  const bool wino4 = kind == ERTD_PACK_WINO4, wino = wino4 || kind == ERTD_PACK_WINO;
  hipError_t e = hipSuccess;
  if (pack)
    e = wino4 ? launch_pack_conv_wino4(w, Cout, Cin, pk, s, true)
        : wino ? launch_pack_conv_wino(w, Cout, Cin, pk, s, true)
               : launch_pack_conv(w, Cout, Cin, ks, pk, s, true);
  if (e != hipSuccess) return (int)e;
  if (wino4) a.wpk_wino4 = pk; else if (wino) a.wpk_wino = pk; else a.wpk = pk;
  if (wino && wino_ksplit_wanted(Cout, Cin, Hg, B)) {
    const size_t sc = mode == MODE_S2 ? a64((size_t)B * Cout * H * H)
                      : (mode == MODE_UP ? a64((size_t)B * Cin * 4 * H * H) : 0);
    a.ksplit_buf = scratch + sc;
  }
  a.bias = nullptr;   // no bias term in a gradient
  float* out = mode == MODE_UP ? scratch : dx;
  a.res = (mode != MODE_UP && accumulate) ? dx : nullptr;   // dx += conv(...) via the residual add
  a.out = out;
  if ((e = launch_conv(ks, MODE_S1, ACT_NONE, a, B, s)) != hipSuccess) return rcode(e);
  if (mode == MODE_UP) return rcode(launch_sum_pool2(scratch, B, Cin, H, dx, accumulate, s));
  return ERTD_OK;
}

void fill_desc(ertd_pack_desc* d, const float* w, float* dst, int cin, int cout, int ks, int kind, int flip) {
  *d = ertd_pack_desc{};
  d->w = w; d->dst = dst; d->cin = cin; d->cout = cout; d->ks = ks; d->kind = kind; d->flip = flip;
  switch (kind) {
    case ERTD_PACK_DIRECT:
      d->total = (long long)conv_packed_floats(cin, cout, ks);
      d->nchunk = (cin + conv_ck(ks) - 1) / conv_ck(ks);
      break;
    case ERTD_PACK_UP:
      d->total = (long long)conv_packed_floats_up(cin, cout);
      d->nchunk = (cin + conv_ck(2) - 1) / conv_ck(2);
      break;
    case ERTD_PACK_WINO:
      d->total = (long long)conv_packed_floats_wino(cin, cout);
      d->nchunk = cin / WINO_KC;
      break;
    default:
      d->total = (long long)conv_packed_floats_wino4(cin, cout);
      d->nchunk = cin / WINO4_KC;
      break;
  }
}
}  // namespace

extern "C" {

int ertd_conv_input_grad(const float* dy, int B, int H, const float* w, int Cout, int Cin, int ks,
                         int mode, float* dx, int accumulate, void* ws, size_t ws_bytes,
                         void* stream) {
  return input_grad_impl(dy, B, H, w, Cout, Cin, ks, mode, dx, accumulate, ws, ws_bytes, stream, true);
}

int ertd_conv_input_grad_run(const float* dy, int B, int H, int Cout, int Cin, int ks, int mode,
                             float* dx, int accumulate, void* ws, size_t ws_bytes, void* stream) {
  return input_grad_impl(dy, B, H, nullptr, Cout, Cin, ks, mode, dx, accumulate, ws, ws_bytes, stream,
                         false);
}

int ertd_conv_input_grad_pack_desc(int Cin, int Cout, int B, int H, int ks, int mode, const float* w,
                                   void* ws, ertd_pack_desc* out) {
  if (!w || !ws || !out || ertd_conv_input_grad_ws_bytes(Cin, Cout, B, H, ks, mode) == 0)
    return ERTD_EINVAL;
  fill_desc(out, w, (float*)ws, Cout, Cin, ks, input_grad_kind(Cin, Cout, B, H, ks, mode), 1);
  return ERTD_OK;
}

// the packing ertd_conv2d_run on this ws reads (fp32; the dispatch of conv2d_impl)
int ertd_conv2d_pack_desc(int Cin, int Ca, int Cout, int ks, int mode, int precision, int B, int H,
                          const float* w, void* ws, ertd_pack_desc* out) {
  if (!w || !ws || !out || precision != ERTD_PREC_FP32 || Ca < 1 || Ca > Cin ||
      !conv2d_geom_ok(Cin, Cout, ks, precision, B, H, mode))
    return ERTD_EINVAL;
  const int Ho = mode == MODE_S2 ? H / 2 : (mode == MODE_UP ? 2 * H : H);
  float* pk = (float*)ws;
  // (the fp32 Upsample conv has no activation: ertd_conv2d_run dispatches it with ACT_NONE)
  const bool wino4 = ks == 3 && Cout > 1 && conv_packed_floats_wino4(Cin, Cout) > 0 &&
                     ((mode == MODE_S1 && wino4_ok(Cin, Ca, Cout, Ho, B)) ||
                      (mode == MODE_UP && wino4s_up_ok(Cin, Ca, Cout, Ho, B)));
  const bool wino = wino4 || (ks == 3 && mode == MODE_S1 && Cout > 1 && conv_packed_floats_wino(Cin, Cout) > 0 &&
                              conv_wino_ok(Cin, Ca, Cout, Ho));
  if (wino) {
    float* pw = pk + a64(std::max(conv_packed_floats(Cin, Cout, ks), conv_packed_floats_up(Cin, Cout)));
    fill_desc(out, w, pw, Cin, Cout, ks, wino4 ? ERTD_PACK_WINO4 : ERTD_PACK_WINO, 0);
  } else if (ks == 3 && mode == MODE_UP) {
    fill_desc(out, w, pk, Cin, Cout, ks, ERTD_PACK_UP, 0);
  } else {
    fill_desc(out, w, pk, Cin, Cout, ks, ERTD_PACK_DIRECT, 0);
  }
  return ERTD_OK;
}

int ertd_conv_pack_batch_prepare(ertd_pack_desc* d, int n) {
  if (!d || n < 1) return ERTD_EINVAL;
  long long blocks = 0;
  for (int k = 0; k < n; ++k) {
    if (!d[k].w || !d[k].dst || d[k].total < 1 || d[k].kind < ERTD_PACK_DIRECT || d[k].kind > ERTD_PACK_WINO4)
      return ERTD_EINVAL;
    d[k].block0 = (int)blocks;
    blocks += (pack_work_items(d[k].kind, d[k].total) + 255) / 256;
    if (blocks > (1LL << 30)) return ERTD_EINVAL;
  }
  return (int)blocks;
}

int ertd_conv_pack_batch(const ertd_pack_desc* descs, int n, int blocks, void* stream) {
  if (!descs || n < 1 || blocks < 1) return ERTD_EINVAL;
  return rcode(launch_pack_batch(descs, n, blocks, (hipStream_t)stream));
}

int ertd_group_norm_stats(const float* x, int Ca, const float* x2, int Cb, int B, int HW,
                          int groups, const float* gamma, const float* beta, float* out,
                          void* stream) {
  const int C = Ca + Cb;
  if (!x || !gamma || !beta || !out || B < 1 || Ca < 1 || Cb < 0 || (Cb > 0 && !x2) ||
      groups < 1 || C % groups || HW < 4 || HW % 4)
    return ERTD_EINVAL;
  GnArgs g{x, x2, Ca, Cb, HW, groups, gamma, beta, (float2*)out};
  return rcode(launch_gn_stats(g, B, (hipStream_t)stream));
}

int ertd_group_norm_partials(const float* x, int C, int B, int HW, int np, float* parts, void* stream) {
  if (!x || !parts || C < 1 || B < 1 || np < 1 || HW != np * 256) return ERTD_EINVAL;
  return rcode(launch_gn_partials(x, C, HW, np, (float2*)parts, B, (hipStream_t)stream));
}

int ertd_group_norm_finalize(const float* pa, int npa, int Ca, const float* pb, int npb, int Cb, int B,
                             int HW, int groups, const float* gamma, const float* beta, float* out,
                             float* mr, void* stream) {
  const int C = Ca + Cb;
  if (!pa || !gamma || !beta || !out || B < 1 || Ca < 1 || Cb < 0 || npa < 1 || HW < 1 || groups < 1 ||
      C % groups || HW % npa || (Cb > 0 && (!pb || npb < 1 || HW % npb)))
    return ERTD_EINVAL;
  GnPartArgs g{(const float2*)pa, npa, Ca, (const float2*)pb, npb, Cb, HW, groups, gamma, beta,
               (float2*)out, (float2*)mr};
  return rcode(launch_gn_finalize(g, B, (hipStream_t)stream));
}

int ertd_group_norm_act_bf16(const float* x, int Ca, const float* x2, int Cb, int B, int H,
                             int groups, const float* gamma, const float* beta, float* out,
                             void* img, int silu, void* stream) {
  const int C = Ca + Cb;
  if (!x || !gamma || !beta || !out || !img || B < 1 || Ca < 1 || Cb < 0 || (Cb > 0 && !x2) ||
      groups < 1 || H < 1 || !gn_act_bf16_fits(C, groups, H * H))
    return ERTD_EINVAL;
  GnArgs g{x, x2, Ca, Cb, H * H, groups, gamma, beta, (float2*)out};
  return rcode(launch_gn_act_bf16(g, silu != 0, img, B, (hipStream_t)stream));
}

int ertd_act_bf16(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* ss,
                  int act, int up, void* img, void* stream) {
  if (!x || !img || B < 1 || Ca < 1 || Cb < 0 || (Cb > 0 && !x2) || H < 1 ||
      act < ACT_NONE || act > ACT_GN || (act != ACT_NONE && !ss) || (up && act != ACT_NONE))
    return ERTD_EINVAL;
  ConvArgs a{};
  a.srcA = x;
  a.srcB = x2;
  a.Ca = Ca;
  a.Cb = Cb;
  a.Cin = Ca + Cb;
  a.gn = (const float2*)ss;
  a.Hs = a.Ws = H;
  a.Ho = a.Wo = up ? 2 * H : H;
  a.bimg = img;
  return rcode(launch_act_bf16(a, act, up != 0, B, (hipStream_t)stream));
}

int ertd_unet_update(float* x, const float* eps, const float* c1, const float* c2,
                     const float* sigma, const float* noise, int num_steps, const int* t_dev,
                     uint64_t seed, uint32_t member_offset, int B, int P, void* stream) {
  if (!x || !eps || !c1 || !c2 || !sigma || !t_dev || B < 1 || P < 1 || (noise && num_steps < 1))
    return ERTD_EINVAL;
  UpdateArgs u{x, eps, c1, c2, sigma, noise, num_steps, t_dev, seed, member_offset, P};
  return rcode(launch_unet_update(u, B, (hipStream_t)stream));
}

int ertd_attention(const float* qkv, int B, int C, int N, float* out, void* stream) {
  if (!qkv || !out || B < 1 || N != 256 || C < 2 || C % 256) return ERTD_EINVAL;
  return rcode(launch_attention(qkv, C, N, out, nullptr, B, (hipStream_t)stream));
}

int ertd_unet_n_params(const ertd_unet_config* c) {
  if (!cfg_ok(c)) return ERTD_EINVAL;
  return (int)enumerate(c).size();
}

int ertd_unet_param_info(const ertd_unet_config* c, int idx, char* name, int name_len,
                         int64_t* shape, int* ndim) {
  if (!cfg_ok(c) || !name || name_len < 2 || !shape || !ndim) return ERTD_EINVAL;
  const std::vector<Param> P = enumerate(c);
  if (idx < 0 || idx >= (int)P.size()) return ERTD_EINVAL;
  const Param& p = P[idx];
  strncpy(name, p.name.c_str(), (size_t)name_len - 1);
  name[name_len - 1] = 0;
  *ndim = (int)p.shape.size();
  for (int i = 0; i < *ndim; ++i) shape[i] = p.shape[i];
  return ERTD_OK;
}

size_t ertd_unet_packed_floats(const ertd_unet_config* c) {
  if (!cfg_ok(c)) return 0;
  return layout_with_freq(c).total;
}

size_t ertd_unet_workspace_bytes(const ertd_unet_config* c, int B, int L) {
  if (!cfg_ok(c) || B < 1 || L < 1) return 0;
  const Layout Lo = layout_with_freq(c);
  return ws_bytes_for(c, Lo, B, L);
}

int ertd_unet_pack(const ertd_unet_config* c, const float* const* params, const float* freq,
                   float* packed, void* stream) {
  if (!cfg_ok(c) || !params || !freq || !packed) return ERTD_EINVAL;
  const Layout L = layout_with_freq(c);
  for (size_t i = 0; i < L.params.size(); ++i)
    if (!params[i]) return ERTD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(packed + L.dummy, 0, DUMMY_FLOATS * sizeof(float), s);
  if (e != hipSuccess) return (int)e;
  const ertd_weights ew = enc_weights(L, packed, params);
  if ((e = launch_pack(ew, packed + L.enc, s)) != hipSuccess) return (int)e;
  const int tb = temb(c);
  for (size_t i = 0; i < L.params.size(); ++i) {
    const Param& p = L.params[i];
    const float* src = params[i];
    if (p.name.rfind("condition_encoder.", 0) == 0) {
      static const char* map[6] = {"enc.0.weight", "enc.0.bias", "enc.2.weight",
                                   "enc.2.bias", "enc.6.weight", "enc.6.bias"};
      e = hipMemcpyAsync(packed + L.off.at(map[i]), src, p.numel() * sizeof(float),
                         hipMemcpyDeviceToDevice, s);
    } else if (ends_with(p.name, ".emb.weight")) {
      const int col = L.eboff.at(p.name.substr(0, p.name.size() - 11));
      e = launch_transpose(src, p.shape[0], p.shape[1], packed + L.wall + col, L.ebtotal, s);
    } else if (ends_with(p.name, ".emb.bias")) {
      const int col = L.eboff.at(p.name.substr(0, p.name.size() - 9));
      e = hipMemcpyAsync(packed + L.ball + col, src, p.numel() * sizeof(float),
                         hipMemcpyDeviceToDevice, s);
    } else if (p.shape.size() == 4) {
      e = bf_prec(c->precision)
              ? launch_pack_conv_bf16(src, p.shape[1], p.shape[0], p.shape[2],
                                      packed + L.off.at(p.name), s, c->precision == ERTD_PREC_BF16X3)
              : (ends_with(p.name, ".upsample.weight")
                     ? launch_pack_conv_up(src, p.shape[1], p.shape[0], packed + L.off.at(p.name), s)
                     : launch_pack_conv(src, p.shape[1], p.shape[0], p.shape[2],
                                        packed + L.off.at(p.name), s));
      const auto itw = L.offw.find(p.name);
      if (e == hipSuccess && itw != L.offw.end())
        e = launch_pack_conv_wino(src, p.shape[1], p.shape[0], packed + itw->second, s);
      const auto itw4 = L.offw4.find(p.name);
      if (e == hipSuccess && itw4 != L.offw4.end())
        e = launch_pack_conv_wino4(src, p.shape[1], p.shape[0], packed + itw4->second, s);
    } else if (p.shape.size() == 2) {
      e = launch_transpose(src, p.shape[0], p.shape[1], packed + L.off.at(p.name), p.shape[0], s);
    } else {
      e = hipMemcpyAsync(packed + L.off.at(p.name), src, p.numel() * sizeof(float),
                         hipMemcpyDeviceToDevice, s);
    }
    if (e != hipSuccess) return (int)e;
  }
  (void)tb;
  e = hipMemcpyAsync(packed + L.off.at("freq"), freq, (size_t)c->ch / 2 * sizeof(float),
                     hipMemcpyDeviceToDevice, s);
  return rcode(e);
}

int ertd_unet_forward(const ertd_unet_config* c, const float* packed, const float* x,
                      const int64_t* t, const float* cond, long long cond_stride, int L, int B,
                      float* out, float* cond_emb_out, void* ws, size_t ws_bytes, void* stream) {
  if (!cfg_ok(c) || !packed || !x || !t || !cond || !out || !ws || B < 1 || L < 1)
    return ERTD_EINVAL;
  const Layout Lo = layout_with_freq(c);
  if (ws_bytes_for(c, Lo, B, L) > ws_bytes) return ERTD_ENOSPC;
  Walk w{c, &Lo, packed, (char*)ws, 0, B, (hipStream_t)stream, false};
  w.cap = ws_bytes;
  const Fixed f = fixed(w, L);
  int r = prologue(w, f, cond, cond_stride, L);
  if (r != ERTD_OK) return r;
  embed(w, f, t);
  w.unet(x, f.ebias, out);
  if (cond_emb_out && w.err == hipSuccess)
    w.chk(hipMemcpyAsync(cond_emb_out, f.cond_emb, (size_t)B * H * sizeof(float),
                         hipMemcpyDeviceToDevice, w.s));
  return rcode(w.err);
}

int ertd_unet_sample(const ertd_unet_config* c, const float* packed, const float* cond,
                     long long cond_stride, int L, int B, int num_steps, int t_first, int n_run,
                     const float* c1, const float* c2, const float* sigma, const float* noise,
                     uint64_t seed, uint32_t member_offset, float* x_inout, void* ws,
                     size_t ws_bytes, void* stream) {
  SampleCall sc{c, packed, cond, cond_stride, L, B, num_steps, t_first, n_run, c1, c2, sigma,
                noise, seed, member_offset, x_inout, ws, ws_bytes};
  int r = sc.check();
  if (r != ERTD_OK) return r;
  hipStream_t s = (hipStream_t)stream;
  if ((r = sc.head(s)) != ERTD_OK) return r;
  for (int i = 0; i < n_run; ++i)
    if ((r = sc.step(s)) != ERTD_OK) return r;
  return ERTD_OK;
}

int ertd_unet_sample_plan_create(const ertd_unet_config* c, const float* packed, const float* cond,
                                 long long cond_stride, int L, int B, int num_steps, int t_first,
                                 int n_run, const float* c1, const float* c2, const float* sigma,
                                 const float* noise, uint64_t seed, uint32_t member_offset,
                                 float* x_inout, void* ws, size_t ws_bytes,
                                 ertd_unet_plan** plan) {
  if (!plan) return ERTD_EINVAL;
  *plan = nullptr;
  ertd_unet_plan* p = new (std::nothrow) ertd_unet_plan();
  if (!p) return ERTD_EINVAL;
  p->call = SampleCall{c, packed, cond, cond_stride, L, B, num_steps, t_first, n_run, c1, c2,
                       sigma, noise, seed, member_offset, x_inout, ws, ws_bytes};
  p->cfg = *c;
  p->call.c = &p->cfg;
  int r = p->call.check();
  if (r != ERTD_OK) {
    delete p;
    return r;
  }
  hipError_t e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
  // The forked skip-conv branch pays only where the convs leave CUs free: the
  // fp32 Winograd kernel is persistent (one workgroup on every CU), so the side
  // branch's convs queue behind it and slow it (U2 B=64: 154.9 steps/s single
  // chain vs 152.6 forked); the bf16 path keeps it (U3 B=256: 94.0 vs 93.1).
  // ERTD_UNET_SIDE=0/1 overrides (A/B).
  const int sv = ERTD_KNOB("UNET_SIDE", -1);
  const bool side = sv >= 0 ? sv != 0 : bf_prec(c->precision);
  // the embedding branch alone beside conv_in and the first GroupNorm
  // (ERTD_UNET_SIDE_EMB=1, A/B): slower, U2 B=64 246.1 vs 249.7 steps/s -- the
  // cross-queue event waits of a forked graph cost more than the overlap
  const bool side_emb = ERTD_KNOB("UNET_SIDE_EMB", 0) != 0;
  p->skip_side = side;
  if (e == hipSuccess && (side || side_emb)) {
    e = hipStreamCreateWithFlags(&p->side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->evf, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->evj, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->eve, hipEventDisableTiming);
  }
  const int multi = ERTD_KNOB("UNET_MULTI", 8);   // U2 B=64: 248.6 (1) vs 249.0 (4) vs 249.4 (8) steps/s
  const int ngraphs = multi > 1 && n_run >= 2 * multi ? 3 : 2;
  for (int k = 0; e == hipSuccess && k < ngraphs; ++k) {
    e = hipStreamBeginCapture(p->stream, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) break;
    if (k == 0) {
      r = p->call.head(p->stream);
    } else {
      for (int i = 0; r == ERTD_OK && i < (k == 1 ? 1 : multi); ++i)
        r = p->call.step(p->stream, p->side, p->evf, p->evj, p->eve, p->skip_side);
    }
    hipGraph_t g = nullptr;
    e = hipStreamEndCapture(p->stream, &g);
    (k == 0 ? p->g_head : k == 1 ? p->g_step : p->g_multi) = g;
    if (r != ERTD_OK) break;
    if (e == hipSuccess)
      e = hipGraphInstantiate(k == 0 ? &p->x_head : k == 1 ? &p->x_step : &p->x_multi, g, nullptr, nullptr, 0);
    if (k == 2 && e == hipSuccess) p->multi = multi;
  }
  if (r != ERTD_OK || e != hipSuccess) {
    ertd_unet_plan_destroy(p);
    return r != ERTD_OK ? r : (int)e;
  }
  *plan = p;
  return ERTD_OK;
}

int ertd_unet_plan_launch_steps(ertd_unet_plan* p, int n_steps, void* stream) {
  if (!p || !p->x_head || !p->x_step || n_steps < 0 || n_steps > p->call.n_run) return ERTD_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipGraphLaunch(p->x_head, s);
  int i = 0;
  if (p->x_multi)
    for (; e == hipSuccess && i + p->multi <= n_steps; i += p->multi) e = hipGraphLaunch(p->x_multi, s);
  for (; e == hipSuccess && i < n_steps; ++i) e = hipGraphLaunch(p->x_step, s);
  return rcode(e);
}

int ertd_unet_plan_launch(ertd_unet_plan* p, void* stream) {
  if (!p) return ERTD_EINVAL;
  return ertd_unet_plan_launch_steps(p, p->call.n_run, stream);
}

int ertd_unet_plan_destroy(ertd_unet_plan* p) {
  if (!p) return ERTD_OK;
  if (p->x_head) (void)hipGraphExecDestroy(p->x_head);
  if (p->x_step) (void)hipGraphExecDestroy(p->x_step);
  if (p->x_multi) (void)hipGraphExecDestroy(p->x_multi);
  if (p->g_multi) (void)hipGraphDestroy(p->g_multi);
  if (p->g_head) (void)hipGraphDestroy(p->g_head);
  if (p->g_step) (void)hipGraphDestroy(p->g_step);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  if (p->side) (void)hipStreamDestroy(p->side);
  if (p->evf) (void)hipEventDestroy(p->evf);
  if (p->evj) (void)hipEventDestroy(p->evj);
  if (p->eve) (void)hipEventDestroy(p->eve);
  delete p;
  return ERTD_OK;
}

}  // extern "C"
