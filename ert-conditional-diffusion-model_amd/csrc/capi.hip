// extern "C" entry points of libertdiff_hip.so (declared in include/ertdiff.h).
// Every shape is validated on the host before anything is enqueued.
#include <cstdlib>
#include <cstring>
#include <new>

#include "ertd_common.h"

using namespace ertd;

namespace {

constexpr size_t ALIGN = 256;
inline size_t align_up(size_t n) { return (n + ALIGN - 1) / ALIGN * ALIGN; }

struct Ws {
  float* partial;   // (B, S, 64) per-strip pool sums
  float* U;
  float* V;
  float* cond_emb;
  size_t partial_floats;
  // persistent faithful chain (OP_SAMPLE only)
  float* ring;                  // CHAIN_RING x (B, S, 64)
  unsigned* sync;               // zeroed per call (sync_words)
  float* uring;                 // (R, B, 128) condition rows
  float* Vc;                    // (T, 128) time rows of the chain
  size_t zero_bytes;
  unsigned* status;             // sampler status word (every faithful schedule)
};

// sync block (zeroed per call), one word per SYNC_PAD-word line:
// cnt (R,B) | uflag (R,B) | progress (B) | claim (B) | vready | status
inline size_t sync_words(int B) {
  return ((size_t)2 * CHAIN_RING * B + 2 * (size_t)B + 2) * SYNC_PAD;
}
inline unsigned* status_word(unsigned* sync, int B) {
  return sync + ((size_t)2 * CHAIN_RING * B + 2 * (size_t)B + 1) * SYNC_PAD;
}

size_t ws_layout(int B, int L, int T, int op, void* base, Ws* out) {
  const int L2 = conv_len(conv_len(L));
  const size_t S = (size_t)n_strips(L2);
  size_t off = 0;
  char* p = (char*)base;
  Ws w{};
  w.partial = (float*)(p + off);
  w.partial_floats = (size_t)B * S * C2;
  off += align_up((size_t)B * S * C2 * sizeof(float));
  if (op == ERTD_OP_SAMPLE) {
    w.U = (float*)(p + off);
    off += align_up((size_t)B * H * sizeof(float));
    w.V = (float*)(p + off);
    off += align_up((size_t)(T > 0 ? T : 1) * H * sizeof(float));
    w.cond_emb = (float*)(p + off);
    off += align_up((size_t)B * H * sizeof(float));
    if (!faithful_chain_may_run(B)) {
      // the persistent chain cannot be resident at this B: no ring, no sync
      // block (faithful mode runs the per-step schedule), just the status word
      w.status = (unsigned*)(p + off);
      off += align_up(SYNC_PAD * sizeof(unsigned));
      if (out) *out = w;
      return off;
    }
    w.ring = (float*)(p + off);
    off += align_up((size_t)CHAIN_RING * B * S * C2 * sizeof(float));
    w.sync = (unsigned*)(p + off);
    w.zero_bytes = sync_words(B) * sizeof(unsigned);
    w.status = status_word(w.sync, B);
    off += align_up(w.zero_bytes);
    w.uring = (float*)(p + off);
    off += align_up((size_t)CHAIN_RING * B * H * sizeof(float));
    w.Vc = (float*)(p + off);
    off += align_up((size_t)(T > 0 ? T : 1) * H * sizeof(float));
  }
  if (out) *out = w;
  return off;
}

bool weights_ok(const ertd_weights* w) {
  if (!w) return false;
  if (!w->enc0_w || !w->enc0_b || !w->enc2_w || !w->enc2_b || !w->enc6_w || !w->enc6_b ||
      !w->time_w || !w->time_b || !w->mlp0_w || !w->mlp0_b || !w->mlp2_w || !w->mlp2_b)
    return false;
  return w->param_dim >= 1 && w->param_dim <= PMAX && w->hidden_dim == H;
}

inline int rc(hipError_t e) { return e == hipSuccess ? ERTD_OK : (int)e; }

#define ERTD_TRY(expr)                  \
  do {                                  \
    const hipError_t e_ = (expr);       \
    if (e_ != hipSuccess) return (int)e_; \
  } while (0)

int enqueue_sample(const ertd_weights* w, const float* packed, const float* cond,
                   long long cstride, int B, int L, int num_steps, int t_first, int n_run,
                   const float* c1, const float* c2, const float* sigma, const float* freq,
                   const float* noise, uint64_t seed, uint32_t member_offset, int mode,
                   int precision, float* x_inout, void* ws, size_t ws_bytes, hipStream_t s,
                   int ncond = 0, int id_period = 0) {
  if (!weights_ok(w) || !packed || !cond || !c1 || !c2 || !sigma || !freq || !x_inout || !ws)
    return ERTD_EINVAL;
  // ncond > 0 (ertd_sample_conditions): member b = realisation b / ncond of
  // condition b % ncond, Philox id member_id(member_offset, b, ncond, id_period)
  if (ncond < 0 || (ncond > 0 && (B % ncond || id_period < ncond || cstride == 0))) return ERTD_EINVAL;
  if (B < 1 || L < 1 || num_steps < 1 ||
      (mode != ERTD_MODE_HOISTED && mode != ERTD_MODE_FAITHFUL && mode != ERTD_MODE_FAITHFUL_STEPS))
    return ERTD_EINVAL;
  if (precision != ERTD_PREC_FP32 && precision != ERTD_PREC_BF16) return ERTD_EINVAL;
  if (t_first < 0 || t_first >= num_steps || n_run < 1 || n_run > t_first + 1) return ERTD_EINVAL;
  if (cstride != 0 && cstride < (long long)CIN * L) return ERTD_EINVAL;
  Ws W;
  if (ws_layout(B, L, num_steps, ERTD_OP_SAMPLE, ws, &W) > ws_bytes) return ERTD_ENOSPC;
  const int t_last = t_first - n_run + 1;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  if (mode == ERTD_MODE_HOISTED) {
    // the encoder depends on the condition only: once per condition (ncond
    // rows, each member reads row b % ncond) -- bitwise the rows it would
    // compute per member
    const int nenc = ncond > 0 ? ncond : B;
    ERTD_TRY(launch_encoder_strips(packed, w->enc0_b, w->enc2_b, cond, cstride, nenc, L, precision,
                                   W.partial, s));
    ERTD_TRY(launch_hoist_prep(*w, packed, W.partial, S, L2, nenc, W.U, W.cond_emb, s));
    ERTD_TRY(launch_time_table(*w, packed, freq, t_last, n_run, W.V, s));
    ERTD_TRY(launch_hoisted_sampler(*w, packed, W.U, W.V, c1, c2, sigma, noise, num_steps, t_first,
                                    n_run, seed, member_offset, B, x_inout, s, ncond, id_period,
                                    ncond));
    return ERTD_OK;
  }
  // Faithful mode: every step re-runs the full condition encoder and the
  // member heads, as the reference does.  Preferred schedule: one persistent
  // launch for the whole chain (chain.hip); it needs every block resident, so
  // it is used when the grid fits (and for fp32, the precision it implements).
  if (mode == ERTD_MODE_FAITHFUL && precision == ERTD_PREC_FP32) {
    const int grid = W.ring ? faithful_chain_grid(B, S) : 0;
    if (grid > 0) {
      ERTD_TRY(launch_zero_words(W.sync, W.zero_bytes / sizeof(unsigned), s));
      FaithfulChainArgs fa{};
      fa.cond = cond;
      fa.cstride = cstride;
      fa.L = L;
      fa.B = B;
      fa.S = S;
      fa.R = CHAIN_RING;
      fa.n_run = n_run;
      fa.t_first = t_first;
      fa.num_steps = num_steps;
      fa.c1 = c1;
      fa.c2 = c2;
      fa.sigma = sigma;
      fa.freq = freq;
      fa.noise = noise;
      fa.seed = seed;
      fa.member_offset = member_offset;
      fa.ncond = ncond;
      fa.id_period = id_period;
      fa.x = x_inout;
      fa.part = W.ring;
      fa.cnt = W.sync;
      fa.uflag = fa.cnt + (size_t)CHAIN_RING * B * SYNC_PAD;
      fa.progress = fa.uflag + (size_t)CHAIN_RING * B * SYNC_PAD;
      fa.claim = fa.progress + (size_t)B * SYNC_PAD;
      fa.vready = fa.claim + (size_t)B * SYNC_PAD;
      fa.status = W.status;
      fa.uring = W.uring;
      fa.V = W.Vc;
      return rc(launch_faithful_chain(*w, packed, fa, grid, s));
    }
  }
  // Per-step schedule (ERTD_MODE_FAITHFUL_STEPS, bf16, or grids too large to
  // be resident): encoder(t), head(t), encoder(t-1), ... on one stream.
  // (The status word is cleared so ertd_sample_status reads ok.)
  ERTD_TRY(launch_zero_words(W.status, 1, s));
  // A pipeline over several streams was measured and rejected: cross-queue
  // event hops inside a graph cost ~10 us each on ROCm 7.
  HeadArgs a{};
  a.partial = W.partial;
  a.S = S;
  a.L2 = L2;
  a.freq = freq;
  a.x_in = x_inout;
  a.c1 = c1;
  a.c2 = c2;
  a.sigma = sigma;
  a.noise = noise;
  a.num_steps = num_steps;
  a.seed = seed;
  a.member_offset = member_offset;
  a.ncond = ncond;
  a.id_period = id_period;
  a.B = B;
  a.x_out = x_inout;
  // Each step's encoder launch also computes v(t) (the time branch, identical
  // for every member of a step) in one extra block; head_step consumes it.
  TimeRowArgs tr{*w, freq, 0, W.V};
  for (int t = t_first; t >= t_last; --t) {
    a.t_scalar = t;
    tr.t = t;
    ERTD_TRY(launch_encoder_strips_t(packed, w->enc0_b, w->enc2_b, cond, cstride, B, L, precision,
                                     W.partial, tr, s, ncond));
    ERTD_TRY(launch_head_step(*w, packed, a, W.V, s));
  }
  return ERTD_OK;
}

}  // namespace

struct ertd_plan {
  hipStream_t stream = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
};

extern "C" {

int ertd_version(void) { return 1; }

const char* ertd_error_string(int code) {
  switch (code) {
    case ERTD_OK: return "ok";
    case ERTD_EINVAL: return "invalid argument (shape, null pointer or unsupported dimension)";
    case ERTD_ENOSPC: return "workspace too small";
    case ERTD_ENOGPU: return "no usable gfx950 device";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
  }
}

int ertd_device_ok(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

size_t ertd_workspace_bytes(int B, int L, int P, int T, int op) {
  (void)P;
  if (B < 1 || L < 1) return 0;
  if (op == ERTD_OP_TRAIN) return train_ws_floats(B, L) * sizeof(float);
  return ws_layout(B, L, T, op, nullptr, nullptr);
}

size_t ertd_packed_floats(void) { return (size_t)PACKED_FLOATS_ALL; }

int ertd_pack_weights(const ertd_weights* w, float* packed, void* stream) {
  if (!weights_ok(w) || !packed) return ERTD_EINVAL;
  return rc(launch_pack(*w, packed, (hipStream_t)stream));
}

int ertd_timestep_embedding(const int64_t* t, int B, int dim, const float* freq, float* out,
                            void* stream) {
  if (!t || !freq || !out || B < 1 || dim < 4) return ERTD_EINVAL;
  return rc(launch_timestep_embedding(t, B, dim, freq, out, (hipStream_t)stream));
}

int ertd_q_sample(const float* x0, const int64_t* t, const float* noise, const float* alpha_bar,
                  int B, int P, float* out, void* stream) {
  if (!x0 || !t || !noise || !alpha_bar || !out || B < 1 || P < 1) return ERTD_EINVAL;
  return rc(launch_q_sample(x0, t, noise, alpha_bar, B, P, out, (hipStream_t)stream));
}

int ertd_encoder_fwd(const ertd_weights* w, const float* packed, const float* cond, int B, int L,
                     int precision, float* cond_emb, void* ws, size_t ws_bytes, void* stream) {
  if (!weights_ok(w) || !packed || !cond || !cond_emb || !ws || B < 1 || L < 1) return ERTD_EINVAL;
  if (precision != ERTD_PREC_FP32 && precision != ERTD_PREC_BF16) return ERTD_EINVAL;
  // the hoisted-mode prep kernel also yields cond_emb; U goes to a scratch slot after partial
  const size_t need = ws_layout(B, L, 1, ERTD_OP_SAMPLE, nullptr, nullptr);
  if (need > ws_bytes) return ERTD_ENOSPC;
  Ws W;
  ws_layout(B, L, 1, ERTD_OP_SAMPLE, ws, &W);
  hipStream_t s = (hipStream_t)stream;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  ERTD_TRY(launch_encoder_strips(packed, w->enc0_b, w->enc2_b, cond, (long long)CIN * L, B, L,
                                 precision, W.partial, s));
  return rc(launch_hoist_prep(*w, packed, W.partial, S, L2, B, W.U, cond_emb, s));
}

int ertd_encoder_strips(const ertd_weights* w, const float* packed, const float* cond,
                        long long cond_stride, int B, int L, int precision, void* ws,
                        size_t ws_bytes, void* stream) {
  if (!weights_ok(w) || !packed || !cond || !ws || B < 1 || L < 1) return ERTD_EINVAL;
  if (precision != ERTD_PREC_FP32 && precision != ERTD_PREC_BF16) return ERTD_EINVAL;
  if (cond_stride != 0 && cond_stride < (long long)CIN * L) return ERTD_EINVAL;
  Ws W;
  if (ws_layout(B, L, 0, ERTD_OP_FORWARD, ws, &W) > ws_bytes) return ERTD_ENOSPC;
  return rc(launch_encoder_strips(packed, w->enc0_b, w->enc2_b, cond, cond_stride, B, L, precision,
                                  W.partial, (hipStream_t)stream));
}

int ertd_forward(const ertd_weights* w, const float* packed, const float* x, const int64_t* t,
                 const float* cond, int B, int L, const float* freq, int precision, float* out,
                 float* cond_emb_out, float* t_emb_out, void* ws, size_t ws_bytes, void* stream) {
  if (!weights_ok(w) || !packed || !x || !t || !cond || !freq || !out || !ws || B < 1 || L < 1)
    return ERTD_EINVAL;
  if (precision != ERTD_PREC_FP32 && precision != ERTD_PREC_BF16) return ERTD_EINVAL;
  Ws W;
  if (ws_layout(B, L, 0, ERTD_OP_FORWARD, ws, &W) > ws_bytes) return ERTD_ENOSPC;
  hipStream_t s = (hipStream_t)stream;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  ERTD_TRY(launch_encoder_strips(packed, w->enc0_b, w->enc2_b, cond, (long long)CIN * L, B, L,
                                 precision, W.partial, s));
  HeadArgs a{};
  a.partial = W.partial;
  a.S = S;
  a.L2 = L2;
  a.freq = freq;
  a.x_in = x;
  a.t_vec = t;
  a.B = B;
  a.eps_out = out;
  a.cond_emb_out = cond_emb_out;
  a.t_emb_out = t_emb_out;
  return rc(launch_head(*w, packed, a, s));
}

int ertd_sample(const ertd_weights* w, const float* packed, const float* cond,
                long long cond_stride, int B, int L, int num_steps, int t_first, int n_run,
                const float* c1, const float* c2, const float* sigma, const float* freq,
                const float* noise, uint64_t seed, uint32_t member_offset, int mode,
                int precision, float* x_inout, void* ws, size_t ws_bytes, void* stream) {
  return enqueue_sample(w, packed, cond, cond_stride, B, L, num_steps, t_first, n_run, c1, c2,
                        sigma, freq, noise, seed, member_offset, mode, precision, x_inout, ws,
                        ws_bytes, (hipStream_t)stream);
}

int ertd_sample_status(const void* ws, int B, int L, int num_steps, int* status, void* stream) {
  if (!ws || !status || B < 1 || L < 1 || num_steps < 1) return ERTD_EINVAL;
  Ws W;
  ws_layout(B, L, num_steps, ERTD_OP_SAMPLE, const_cast<void*>(ws), &W);
  const unsigned* dev = W.status;
  unsigned v = 0;
  ERTD_TRY(hipMemcpyAsync(&v, dev, sizeof(v), hipMemcpyDeviceToHost, (hipStream_t)stream));
  ERTD_TRY(hipStreamSynchronize((hipStream_t)stream));
  *status = (int)v;
  return v == 0 ? ERTD_OK : ERTD_ETIMEOUT;
}

int ertd_philox_normal(uint64_t seed, uint32_t member_offset, int B, int P, int t, int tag,
                       float* out, void* stream) {
  if (!out || B < 1 || P < 1 || (long long)B * P > (1LL << 31) || t < 0) return ERTD_EINVAL;
  return rc(launch_philox_normal(seed, member_offset, B, P, t, tag, out, (hipStream_t)stream));
}

int ertd_postprocess(const float* u, long long rows, int P, double a, double b,
                     const double* min_, const double* scale_, const double* limits, float* out,
                     uint8_t* valid, void* stream) {
  if (!u || !min_ || !scale_ || !limits || !out || !valid || rows < 0 || P < 1 || P > PMAX)
    return ERTD_EINVAL;
  if (rows == 0) return ERTD_OK;
  if (rows > (long long)8 * 0x7fffffff) return ERTD_EINVAL;
  return rc(launch_postproc(u, rows, P, (float)a, (float)(b - a), min_, scale_, limits, out, valid,
                            (hipStream_t)stream));
}

}  // extern "C"

namespace {

// one sampler call captured as a graph on the plan's own stream
template <class Enqueue>
int capture_plan(ertd_plan** plan, Enqueue&& enqueue) {
  if (!plan) return ERTD_EINVAL;
  *plan = nullptr;
  ertd_plan* p = new (std::nothrow) ertd_plan();
  if (!p) return ERTD_EINVAL;
  hipError_t e = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete p;
    return (int)e;
  }
  e = hipStreamBeginCapture(p->stream, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    ertd_plan_destroy(p);
    return (int)e;
  }
  const int r = enqueue(p->stream);
  e = hipStreamEndCapture(p->stream, &p->graph);
  if (r != ERTD_OK || e != hipSuccess) {
    ertd_plan_destroy(p);
    return r != ERTD_OK ? r : (int)e;
  }
  e = hipGraphInstantiate(&p->exec, p->graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    ertd_plan_destroy(p);
    return (int)e;
  }
  *plan = p;
  return ERTD_OK;
}

// ertd_sample_conditions' geometry checks; returns B = n_cond * n_samples or 0.
// member_id() computes member_offset + r * id_period + c in uint32: the slice
// must fit one period (member_offset + n_cond <= id_period, as the Python
// wrapper enforces) and the largest id must not wrap, or Philox ids of
// different members (ranks, realisations) would coincide.
int conditions_batch(int n_cond, int n_samples, long long id_period, uint32_t member_offset) {
  if (n_cond < 1 || n_samples < 1 || id_period < n_cond || id_period > 0x7fffffff) return 0;
  if ((long long)member_offset + n_cond > id_period) return 0;
  if ((unsigned long long)member_offset + (unsigned long long)(n_samples - 1) * (unsigned long long)id_period +
          (unsigned long long)n_cond > 0x100000000ull)
    return 0;
  const long long B = (long long)n_cond * n_samples;
  return B > (1 << 30) ? 0 : (int)B;
}

}  // namespace

extern "C" {

int ertd_sample_plan_create(const ertd_weights* w, const float* packed, const float* cond,
                            long long cond_stride, int B, int L, int num_steps, int t_first,
                            int n_run, const float* c1, const float* c2, const float* sigma,
                            const float* freq, const float* noise, uint64_t seed,
                            uint32_t member_offset, int mode, int precision, float* x_inout,
                            void* ws, size_t ws_bytes, ertd_plan** plan) {
  return capture_plan(plan, [&](hipStream_t s) {
    return enqueue_sample(w, packed, cond, cond_stride, B, L, num_steps, t_first, n_run, c1, c2,
                          sigma, freq, noise, seed, member_offset, mode, precision, x_inout, ws,
                          ws_bytes, s);
  });
}

int ertd_sample_conditions(const ertd_weights* w, const float* packed, const float* cond, int n_cond,
                           int n_samples, long long id_period, int L, int num_steps, int t_first,
                           int n_run, const float* c1, const float* c2, const float* sigma,
                           const float* freq, const float* noise, uint64_t seed,
                           uint32_t member_offset, int mode, int precision, float* x_inout, void* ws,
                           size_t ws_bytes, void* stream) {
  const int B = conditions_batch(n_cond, n_samples, id_period, member_offset);
  if (!B) return ERTD_EINVAL;
  return enqueue_sample(w, packed, cond, (long long)CIN * L, B, L, num_steps, t_first, n_run, c1, c2,
                        sigma, freq, noise, seed, member_offset, mode, precision, x_inout, ws,
                        ws_bytes, (hipStream_t)stream, n_cond, (int)id_period);
}

int ertd_sample_conditions_plan_create(const ertd_weights* w, const float* packed, const float* cond,
                                       int n_cond, int n_samples, long long id_period, int L,
                                       int num_steps, int t_first, int n_run, const float* c1,
                                       const float* c2, const float* sigma, const float* freq,
                                       const float* noise, uint64_t seed, uint32_t member_offset,
                                       int mode, int precision, float* x_inout, void* ws,
                                       size_t ws_bytes, ertd_plan** plan) {
  const int B = conditions_batch(n_cond, n_samples, id_period, member_offset);
  if (!B) {
    if (plan) *plan = nullptr;
    return ERTD_EINVAL;
  }
  return capture_plan(plan, [&](hipStream_t s) {
    return enqueue_sample(w, packed, cond, (long long)CIN * L, B, L, num_steps, t_first, n_run, c1,
                          c2, sigma, freq, noise, seed, member_offset, mode, precision, x_inout, ws,
                          ws_bytes, s, n_cond, (int)id_period);
  });
}

int ertd_plan_launch(ertd_plan* plan, void* stream) {
  if (!plan || !plan->exec) return ERTD_EINVAL;
  return rc(hipGraphLaunch(plan->exec, (hipStream_t)stream));
}

int ertd_plan_destroy(ertd_plan* plan) {
  if (!plan) return ERTD_OK;
  if (plan->exec) (void)hipGraphExecDestroy(plan->exec);
  if (plan->graph) (void)hipGraphDestroy(plan->graph);
  if (plan->stream) (void)hipStreamDestroy(plan->stream);
  delete plan;
  return ERTD_OK;
}

static bool grads_ok(float* const* g) {
  if (!g) return false;
  for (int k = 0; k < 12; ++k)
    if (!g[k]) return false;
  return true;
}

int ertd_train_forward(const ertd_weights* w, float* packed, const float* x, const float* x0,
                       const float* noise, const float* alpha_bar, const int64_t* t,
                       const float* cond, int B, int L, const float* freq, float* eps_out,
                       void* ws, size_t ws_bytes, void* stream) {
  (void)packed;  // the train kernels read the parameters in place
  if (!weights_ok(w) || !t || !cond || !freq || !ws || B < 1 || L < 1) return ERTD_EINVAL;
  if (!x && (!x0 || !noise || !alpha_bar)) return ERTD_EINVAL;
  if (train_ws_floats(B, L) * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
  return rc(launch_train_forward(*w, x, x0, noise, alpha_bar, t, cond, B, L, freq, eps_out,
                                 (float*)ws, (hipStream_t)stream));
}

int ertd_train_backward(const ertd_weights* w, const float* packed, const float* dout,
                        const float* noise, const float* cond, int B, int L, float* const* grads,
                        float* loss_out, float* dx_out, void* ws, size_t ws_bytes, void* stream) {
  (void)packed;
  if (!weights_ok(w) || !cond || !grads_ok(grads) || !ws || B < 1 || L < 1) return ERTD_EINVAL;
  if (!dout && (!noise || !loss_out)) return ERTD_EINVAL;
  if (train_ws_floats(B, L) * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
  return rc(launch_train_backward(*w, dout, noise, cond, B, L, grads, loss_out, dx_out, (float*)ws,
                                  (hipStream_t)stream));
}

int ertd_adam(const ertd_weights* w, float* const* grads, float* const* exp_avg,
              float* const* exp_avg_sq, int step, float lr, float beta1, float beta2, float eps,
              void* stream) {
  if (!weights_ok(w) || !grads_ok(grads) || !grads_ok(exp_avg) || !grads_ok(exp_avg_sq) || step < 1)
    return ERTD_EINVAL;
  return rc(launch_adam(*w, grads, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps,
                        (hipStream_t)stream));
}

static int train_step_args_ok(const ertd_weights* w, const float* x0, const int64_t* t,
                              const float* noise, const float* cond, const float* alpha_bar, int B,
                              int L, const float* freq, float* const* grads, float* const* exp_avg,
                              float* const* exp_avg_sq, float* loss_out, void* ws, size_t ws_bytes) {
  if (!weights_ok(w) || !x0 || !t || !noise || !cond || !alpha_bar || !freq || !loss_out || !ws ||
      B < 1 || L < 1)
    return ERTD_EINVAL;
  if (!grads_ok(grads) || !grads_ok(exp_avg) || !grads_ok(exp_avg_sq)) return ERTD_EINVAL;
  if (train_ws_floats(B, L) * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
  return ERTD_OK;
}

int ertd_train_step(const ertd_weights* w, float* packed, const float* x0, const int64_t* t,
                    const float* noise, const float* cond, const float* alpha_bar, int B, int L,
                    const float* freq, float* const* grads, float* const* exp_avg,
                    float* const* exp_avg_sq, int step, float lr, float beta1, float beta2,
                    float eps, float* loss_out, void* ws, size_t ws_bytes, void* stream) {
  (void)packed;
  const int r = train_step_args_ok(w, x0, t, noise, cond, alpha_bar, B, L, freq, grads, exp_avg,
                                   exp_avg_sq, loss_out, ws, ws_bytes);
  if (r != ERTD_OK) return r;
  if (step < 1) return ERTD_EINVAL;
  const TrainAdam adam{step, lr, beta1, beta2, eps, nullptr, nullptr, 0, 0, 0, 0, 0};
  return rc(launch_train_step(*w, x0, t, noise, cond, alpha_bar, B, L, freq, grads, exp_avg,
                              exp_avg_sq, adam, loss_out, (float*)ws, (hipStream_t)stream));
}

int ertd_train_conv_backward(const float* cond, int B, int L, void* ws, size_t ws_bytes,
                             void* stream) {
  if (!cond || !ws || B < 1 || L < 1) return ERTD_EINVAL;
  if (train_ws_floats(B, L) * sizeof(float) > ws_bytes) return ERTD_ENOSPC;
  return rc(launch_train_conv_backward(cond, B, L, (float*)ws, (hipStream_t)stream));
}

int ertd_adam_table(int step_first, int n, float lr, float beta1, float beta2, float eps,
                    float* out) {
  if (!out || step_first < 1 || n < 1) return ERTD_EINVAL;
  adam_table_host(step_first, n, lr, beta1, beta2, eps, out);
  return ERTD_OK;
}

int ertd_train_step_dev(const ertd_weights* w, const float* x0, int64_t* t, float* noise,
                        const float* cond, const float* alpha_bar, int B, int L, const float* freq,
                        float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                        int* step_dev, const float* adam_table, int table_first, int table_len,
                        int draw, int T, uint64_t seed, float* loss_out, void* ws, size_t ws_bytes,
                        void* stream) {
  const int r = train_step_args_ok(w, x0, t, noise, cond, alpha_bar, B, L, freq, grads, exp_avg,
                                   exp_avg_sq, loss_out, ws, ws_bytes);
  if (r != ERTD_OK) return r;
  if (!step_dev || !adam_table || table_first < 1 || table_len < 1) return ERTD_EINVAL;
  if (draw && T < 1) return ERTD_EINVAL;
  const TrainAdam adam{0, 0.f, 0.f, 0.f, 0.f, adam_table, step_dev, table_first, table_len, seed,
                       draw ? 1 : 0, T};
  return rc(launch_train_step(*w, x0, t, noise, cond, alpha_bar, B, L, freq, grads, exp_avg,
                              exp_avg_sq, adam, loss_out, (float*)ws, (hipStream_t)stream));
}

int ertd_train_steps_dev(const ertd_weights* w, const float* x0, int64_t* t, float* noise,
                         const float* cond, const float* alpha_bar, int B, int L, const float* freq,
                         float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                         int* step_dev, const float* adam_table, int table_first, int table_len,
                         int draw, int T, uint64_t seed, int nsteps, float* loss_out, void* ws,
                         size_t ws_bytes, void* stream) {
  if (nsteps < 1 || !draw) return ERTD_EINVAL;
  for (int i = 0; i < nsteps; ++i) {
    const int r = ertd_train_step_dev(w, x0, t, noise, cond, alpha_bar, B, L, freq, grads, exp_avg,
                                      exp_avg_sq, step_dev, adam_table, table_first, table_len, draw,
                                      T, seed, loss_out, ws, ws_bytes, stream);
    if (r != ERTD_OK) return r;
  }
  return ERTD_OK;
}

}  // extern "C"
