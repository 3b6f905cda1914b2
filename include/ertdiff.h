/*
 * ertdiff.h -- C ABI of libertdiff_hip.so, the MI355X (gfx950) implementation
 * of the conditional-DDPM denoising hot path of pnnl/ERT-Conditional-Diffusion-Model.
 *
 * The reference has no native code and no FFI: its hot path is the Python call
 * surface in ERT_Conditional_Diffusion.py.  Each entry point below replaces the
 * ATen work behind one of those Python functions; the Python drop-in module
 * (ert-conditional-diffusion-model_amd/ertdiff) binds them with ctypes, see
 * INTEGRATION.md.
 *
 * Conventions (all entry points):
 *   - every pointer is DEVICE memory owned by the caller (torch tensors);
 *     the library never allocates or frees device memory on these paths and
 *     keeps no global state besides cached kernel handles;
 *   - float tensors are fp32, row-major contiguous; timesteps are int64;
 *   - work is enqueued on `stream` (a hipStream_t passed as void*) with no
 *     host synchronisation, so calls may be captured into a hipGraph;
 *   - return 0 on success, a negative ERTD_E* code for bad arguments (checked
 *     on the host BEFORE anything is launched), or a positive hipError_t.
 *
 * Shapes: B = batch (members), L = measurements per survey (4693 in the
 * reference), C_in = 14 surveys, P = param_dim (29 in the reference, 1..32
 * supported), H = hidden_dim (128; the only value the reference uses).
 */
#ifndef ERTDIFF_H
#define ERTDIFF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ERTD_OK 0
#define ERTD_EINVAL (-1)   /* bad shape / null pointer / unsupported dim */
#define ERTD_ENOSPC (-2)   /* workspace too small */
#define ERTD_ENOGPU (-3)   /* no gfx950 device / kernel image unavailable */
#define ERTD_ETIMEOUT (-4) /* a persistent sampler wait timed out (see ertd_sample_status) */

#define ERTD_CIN 14
#define ERTD_HIDDEN 128
#define ERTD_PMAX 32

/* Pointers to the 12 state_dict tensors of ConditionalDiffusionModel
 * (ERT_Conditional_Diffusion.py:133-153), in state_dict order.          */
typedef struct ertd_weights {
  const float* enc0_w; /* condition_encoder.0.weight (32,14,3)   */
  const float* enc0_b; /* condition_encoder.0.bias   (32)        */
  const float* enc2_w; /* condition_encoder.2.weight (64,32,3)   */
  const float* enc2_b; /* condition_encoder.2.bias   (64)        */
  const float* enc6_w; /* condition_encoder.6.weight (128,64)    */
  const float* enc6_b; /* condition_encoder.6.bias   (128)       */
  const float* time_w; /* time_embed.0.weight        (128,128)   */
  const float* time_b; /* time_embed.0.bias          (128)       */
  const float* mlp0_w; /* mlp.0.weight               (128,P+256) */
  const float* mlp0_b; /* mlp.0.bias                 (128)       */
  const float* mlp2_w; /* mlp.2.weight               (P,128)     */
  const float* mlp2_b; /* mlp.2.bias                 (P)         */
  int param_dim;       /* P */
  int hidden_dim;      /* H, must be 128 */
} ertd_weights;

/* Workspace ops for ertd_workspace_bytes(). */
#define ERTD_OP_FORWARD 0
#define ERTD_OP_SAMPLE 1
#define ERTD_OP_TRAIN 2

/* Sampler modes. */
#define ERTD_MODE_HOISTED 0  /* condition encoder once, persistent T-loop   */
#define ERTD_MODE_FAITHFUL 1 /* encoder re-evaluated every step (reference):
                                one persistent launch per chain when the grid
                                fits, else the per-step schedule            */
#define ERTD_MODE_FAITHFUL_STEPS 2 /* faithful, forced per-step schedule:
                                      encoder + head launch per step        */

/* Encoder operand precision. */
#define ERTD_PREC_FP32 0
#define ERTD_PREC_BF16 1 /* bf16 conv operands, fp32 accumulate/state */
/* U-Net only: split-bf16 conv operands -- x = hi + lo (two bf16 RNE planes),
   products lo*hi + hi*lo + hi*hi on the bf16 MFMA, fp32 accumulate/state
   (about 2^-16 relative per product: within the north star's 1e-4) */
#define ERTD_PREC_BF16X3 2

int ertd_version(void);
const char* ertd_error_string(int code);
/* 1 when a gfx950 device is visible and the kernels load, else 0. */
int ertd_device_ok(void);

/* Bytes of caller-provided device workspace an op needs.
 * T = number of sampler steps (ignored for FORWARD).                      */
size_t ertd_workspace_bytes(int B, int L, int P, int T, int op);
/* Floats of packed (MFMA fragment-order) encoder weights. */
size_t ertd_packed_floats(void);

/* Re-lay the two Conv1d weights into MFMA fragment order (once per weight
 * update).  packed: ertd_packed_floats() floats.                          */
int ertd_pack_weights(const ertd_weights* w, float* packed, void* stream);

/* get_timestep_embedding (ERT_Conditional_Diffusion.py:80-88) on device.
 * freq: (dim/2) float32 frequencies exp(-i*ln(1e4)/(dim/2-1)) computed on the
 * host with the reference's float32 expression; out: (B, dim).            */
int ertd_timestep_embedding(const int64_t* t, int B, int dim, const float* freq,
                            float* out, void* stream);

/* q_sample (ERT_Conditional_Diffusion.py:96-99): out = sqrt(ab[t])*x0 + sqrt(1-ab[t])*noise. */
int ertd_q_sample(const float* x0, const int64_t* t, const float* noise,
                  const float* alpha_bar, int B, int P, float* out, void* stream);

/* condition_encoder (ERT_Conditional_Diffusion.py:133-142): cond (B,14,L) ->
 * cond_emb (B,128).                                                       */
int ertd_encoder_fwd(const ertd_weights* w, const float* packed, const float* cond,
                     int B, int L, int precision, float* cond_emb,
                     void* ws, size_t ws_bytes, void* stream);

/* The encoder's strip kernel alone (conv1 -> ReLU -> conv2 -> ReLU -> per-strip
 * pool sums), writing partial (B, n_strips, 64) into ws.  This is the hot
 * kernel of every step; exposed so callers can time it in isolation.      */
int ertd_encoder_strips(const ertd_weights* w, const float* packed, const float* cond,
                        long long cond_stride, int B, int L, int precision,
                        void* ws, size_t ws_bytes, void* stream);

/* ConditionalDiffusionModel.forward (ERT_Conditional_Diffusion.py:155-164):
 * x (B,P), t (B,) int64, cond (B,14,L) -> out (B,P).  freq as above (H/2).
 * cond_emb_out / t_emb_out: optional (B,128) intermediates (NULL to skip). */
int ertd_forward(const ertd_weights* w, const float* packed, const float* x,
                 const int64_t* t, const float* cond, int B, int L, const float* freq,
                 int precision, float* out, float* cond_emb_out, float* t_emb_out,
                 void* ws, size_t ws_bytes, void* stream);

/* sample_model's reverse loop (ERT_Conditional_Diffusion.py:107-119).
 *   cond (B,14,L) with member stride cond_stride floats (14*L when each
 *     member has its own condition, 0 when all members share one).
 *   num_steps: schedule length n of the call (reference: num_steps or T).
 *   Runs steps t = t_first, t_first-1, ..., t_first-n_run+1 (reference:
 *     t_first = n-1, n_run = n); x_inout (B,P) carries the state in/out, so a
 *     chain may be split into segments.
 *   c1, c2, sigma: (num_steps) float32 per-step scalars, index t, formed on
 *     the host with the reference's expressions (:111-118; sigma already
 *     multiplied by temperature).
 *   noise: NULL -> counter-based Philox keyed by (seed, member_offset+b, t);
 *     else (num_steps, B, P) injected draws in reference order: noise[k] is
 *     the z used at t = num_steps-k (noise[0] = x_T is not read).
 *   mode: ERTD_MODE_HOISTED / ERTD_MODE_FAITHFUL / ERTD_MODE_FAITHFUL_STEPS
 *     (bit-identical outputs).                                            */
int ertd_sample(const ertd_weights* w, const float* packed, const float* cond,
                long long cond_stride, int B, int L, int num_steps, int t_first, int n_run,
                const float* c1, const float* c2, const float* sigma, const float* freq,
                const float* noise, uint64_t seed, uint32_t member_offset, int mode,
                int precision, float* x_inout, void* ws, size_t ws_bytes, void* stream);

/* Status word of the last persistent faithful chain run on `ws` (same B, L,
 * num_steps as the ertd_sample call): synchronizes `stream`; *status = 0 and
 * ERTD_OK, or the code of the wait that timed out and ERTD_ETIMEOUT (the
 * launch then drained without finishing; x_inout is not valid).           */
int ertd_sample_status(const void* ws, int B, int L, int num_steps, int* status, void* stream);

/* Standard normals from the sampler's Philox stream: out (B,P) for members
 * member_offset..+B-1 at step `t`, stream tag `tag` (0 = step noise z_t,
 * 1 = initial x_T).                                                       */
int ertd_philox_normal(uint64_t seed, uint32_t member_offset, int B, int P, int t,
                       int tag, float* out, void* stream);

/* Ensemble post-processing (ERT_Conditional_Diffusion.py:400-406, :1054-1060):
 * u (rows, P) unconstrained samples (sample_model output) ->
 *   out (rows, P) = param_scaler.inverse_transform(inverse_transform(u, a, b))
 *     (sigmoid in float32; then MinMaxScaler's float64 min_/scale_ applied as
 *      x -= min_; x /= scale_ on the float32 array, each op rounded to float32)
 *   valid (rows) uint8 = 1 unless check_param_bounds (:183-218) rejects the row
 *     (any value < limits[p][0] or > limits[p][1], compared in float64).
 * min_, scale_: (P) float64 (a fitted MinMaxScaler's min_ and scale_);
 * limits: (P, 2) float64 [min, max] (Generate_ERT_utils.ParameterLimits.plims). */
int ertd_postprocess(const float* u, long long rows, int P, double a, double b,
                     const double* min_, const double* scale_, const double* limits, float* out,
                     uint8_t* valid, void* stream);

/* hipGraph plans: capture one full ertd_sample call (all kernels of all
 * steps) once, replay with ertd_plan_launch.  Buffers are bound at creation. */
typedef struct ertd_plan ertd_plan;
int ertd_sample_plan_create(const ertd_weights* w, const float* packed, const float* cond,
                            long long cond_stride, int B, int L, int num_steps, int t_first,
                            int n_run, const float* c1, const float* c2, const float* sigma,
                            const float* freq, const float* noise, uint64_t seed,
                            uint32_t member_offset, int mode, int precision, float* x_inout,
                            void* ws, size_t ws_bytes, ertd_plan** plan);
int ertd_plan_launch(ertd_plan* plan, void* stream);
int ertd_plan_destroy(ertd_plan* plan);

/* The reference's test-set uncertainty evaluation (ERT_Conditional_Diffusion.py
 * :1042-1069: every test condition x `uncertainty_samples` calls of
 * sample_model) as ONE sampler launch of B = n_cond * n_samples members.
 *   cond (n_cond, 14, L) contiguous; member j = realisation r = j / n_cond of
 *     condition c = j % n_cond, so x_inout (B, P) is the (n_samples, n_cond, P)
 *     `Uncertainty_params` layout (:1073) as it fills.
 *   Philox id of member j: member_offset + r * id_period + c.  One device:
 *     id_period = n_cond, member_offset = 0 (ids 0..B-1, realisation r's
 *     members r*N .. r*N+N-1: the same draws as sample_model with
 *     member_offset = r*N).  A rank holding conditions [c0, c0+n_cond) of N
 *     passes member_offset = c0, id_period = N: every member keeps its global
 *     id, so the result is bitwise invariant to how the conditions are split.
 *   ERTD_MODE_HOISTED runs the condition encoder once per CONDITION (n_cond
 *     strip sets, not B); the faithful modes re-run it per member and step as
 *     the reference does.  Workspace: ertd_workspace_bytes(B, L, P, num_steps,
 *     ERTD_OP_SAMPLE).  Other arguments as ertd_sample.                      */
int ertd_sample_conditions(const ertd_weights* w, const float* packed, const float* cond, int n_cond,
                           int n_samples, long long id_period, int L, int num_steps, int t_first,
                           int n_run, const float* c1, const float* c2, const float* sigma,
                           const float* freq, const float* noise, uint64_t seed,
                           uint32_t member_offset, int mode, int precision, float* x_inout, void* ws,
                           size_t ws_bytes, void* stream);
int ertd_sample_conditions_plan_create(const ertd_weights* w, const float* packed, const float* cond,
                                       int n_cond, int n_samples, long long id_period, int L,
                                       int num_steps, int t_first, int n_run, const float* c1,
                                       const float* c2, const float* sigma, const float* freq,
                                       const float* noise, uint64_t seed, uint32_t member_offset,
                                       int mode, int precision, float* x_inout, void* ws,
                                       size_t ws_bytes, ertd_plan** plan);

/* ---- training (ERT_Conditional_Diffusion.py:305-320) ---------------------------
 * Workspace: ertd_workspace_bytes(B, L, P, 0, ERTD_OP_TRAIN).  The forward
 * stores the activations the backward reads there: keep it between the two.
 * grads / exp_avg / exp_avg_sq: 12 device buffers in state_dict order with the
 * parameters' shapes.  The parameters are the (mutable) pointers of `w`.    */

/* Training forward: eps = model(x, t, cond) with activations saved in ws.
 * x (B,P), or x == NULL and x0/noise/alpha_bar given: x = q_sample(x0, t, noise)
 * (:314).  The train kernels read the parameters of `w` in place: `packed` is
 * unused (kept for ABI compatibility; may be NULL), here and below.          */
int ertd_train_forward(const ertd_weights* w, float* packed, const float* x, const float* x0,
                       const float* noise, const float* alpha_bar, const int64_t* t,
                       const float* cond, int B, int L, const float* freq, float* eps_out,
                       void* ws, size_t ws_bytes, void* stream);

/* Backward of the last ertd_train_forward on `ws`.  dout (B,P) = dL/deps, or
 * NULL with `noise`: L = MSELoss(mean)(eps, noise) (:295, :316), loss_out (1).
 * dx_out (B,P) optional.  grads are overwritten (not accumulated).          */
int ertd_train_backward(const ertd_weights* w, const float* packed, const float* dout,
                        const float* noise, const float* cond, int B, int L, float* const* grads,
                        float* loss_out, float* dx_out, void* ws, size_t ws_bytes, void* stream);

/* torch.optim.Adam step (no weight decay / amsgrad) on the 12 parameters of w,
 * in place.  step = the step count after this update (>= 1).               */
int ertd_adam(const ertd_weights* w, float* const* grads, float* const* exp_avg,
              float* const* exp_avg_sq, int step, float lr, float beta1, float beta2, float eps,
              void* stream);

/* The reference train step (:309-319) in one call: q_sample -> forward ->
 * MSELoss -> backward -> Adam.  loss_out (1) float32 on device; grads receive
 * the gradients (the reference's p.grad after loss.backward()).            */
int ertd_train_step(const ertd_weights* w, float* packed, const float* x0, const int64_t* t,
                    const float* noise, const float* cond, const float* alpha_bar, int B, int L,
                    const float* freq, float* const* grads, float* const* exp_avg,
                    float* const* exp_avg_sq, int step, float lr, float beta1, float beta2,
                    float eps, float* loss_out, void* ws, size_t ws_bytes, void* stream);

/* ertd_train_step with no host scalars, for graph capture (ertdiff.TrainPlan):
 * the step advances the device counter *step_dev (int32; the count of Adam
 * steps applied, as torch's state["step"]) and the update of step s uses the
 * 6-float entry adam_table[s - table_first] (device copy of ertd_adam_table's
 * output); s must lie in [table_first, table_first + table_len).  The device
 * cannot report a step outside the table: it CLAMPS s to the nearest entry
 * (wrong bias corrections, no error), so the caller re-builds the table before
 * it runs out (ertdiff.TrainPlan does).  With draw = 1, alpha_bar must hold at
 * least T entries (t is drawn in [0, T) and alpha_bar[t] read on the device).
 * draw = 0: t (B) / noise (B,P) are inputs.  draw = 1: the step draws them
 * itself into the same buffers (t ~ U{0..T-1}, noise ~ N(0,1), Philox4x32-10
 * keyed by (seed, member, step s): reproducible, independent of the grid).  */
int ertd_train_step_dev(const ertd_weights* w, const float* x0, int64_t* t, float* noise,
                        const float* cond, const float* alpha_bar, int B, int L, const float* freq,
                        float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                        int* step_dev, const float* adam_table, int table_first, int table_len,
                        int draw, int T, uint64_t seed, float* loss_out, void* ws, size_t ws_bytes,
                        void* stream);

/* nsteps consecutive ertd_train_step_dev steps (draw = 1 only: each step draws
 * its own t / noise from the device step count) in one call.  For graph
 * capture: a graph holding n steps of ONE call replays them back to back,
 * where n single-step calls captured one after another leave an ~8 us gap at
 * every call boundary of the graph (rocprofv3 trace, B = 32 -- measured, cause
 * in the runtime's graph, not in the kernels).  ertdiff.TrainPlan.run.  */
int ertd_train_steps_dev(const ertd_weights* w, const float* x0, int64_t* t, float* noise,
                         const float* cond, const float* alpha_bar, int B, int L, const float* freq,
                         float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                         int* step_dev, const float* adam_table, int table_first, int table_len,
                         int draw, int T, uint64_t seed, int nsteps, float* loss_out, void* ws,
                         size_t ws_bytes, void* stream);

/* The condition encoder's conv backward alone (the Conv1d part of
 * loss.backward(), :317), re-run on the state the last ertd_train_step /
 * ertd_train_step_dev / ertd_train_backward left in ws (same B, L, cond): it
 * rewrites the per-strip gradient rows in ws and nothing else.  For timing the
 * step's dominant kernel on its own (bench.py train_roofline).               */
int ertd_train_conv_backward(const float* cond, int B, int L, void* ws, size_t ws_bytes,
                             void* stream);

/* host: the Adam scalars of steps step_first ... step_first + n - 1 (6 floats
 * each), formed as torch.optim.Adam forms them (Python-float bias corrections). */
int ertd_adam_table(int step_first, int n, float lr, float beta1, float beta2, float eps,
                    float* out);

/* ---- build-defined conditional U-Net (SURVEY.md 8a'; north_star) -----------------
 * PARITY UNPINNED vs the reference: ERT_Conditional_Diffusion.py has no U-Net
 * (SURVEY.md 0.3).  The specification is oracle/unet_torch.py: x (B, image^2)
 * viewed as (B,1,image,image); emb = time MLP(sinusoid(t, ch)) + Linear(128->4ch)
 * of the reference's condition encoder (:133-142); ResBlocks of GroupNorm ->
 * SiLU -> 3x3 conv (+emb) -> GroupNorm -> SiLU -> 3x3 conv (+1x1 skip);
 * stride-2 Downsample, nearest-x2 Upsample + 3x3 conv, optional single-head
 * mid-block attention; GroupNorm -> SiLU -> 3x3 conv out.  fp32 throughout
 * (convs on fp32 MFMA).  Activations NCHW in the caller's workspace.         */
typedef struct ertd_unet_config {
  int image;       /* H = W: 16..128, power of two                          */
  int ch;          /* base channels                                         */
  int n_levels;    /* 1..4; every level >= 16x16                           */
  int ch_mult[4];  /* channel multiplier per level                          */
  int num_res;     /* ResBlocks per level on the way down (num_res+1 up)    */
  int attn;        /* 1: mid-block attention (needs 16x16 and C % 256 == 0) */
  int groups;      /* GroupNorm groups (32)                                 */
  int precision;   /* ERTD_PREC_FP32 (fp32 MFMA convs), ERTD_PREC_BF16
                      (bf16 conv operands, fp32 accumulate/activations) or
                      ERTD_PREC_BF16X3 (split-bf16 conv operands)          */
} ertd_unet_config;

/* Single U-Net operators (the SURVEY 8a' operator rows; used by per-operator
 * parity tests and microbenchmarks).
 * ertd_conv2d: out (B,Cout,Ho,Ho) = conv(act(cat(x (B,Ca,H,H), x2 (B,Cb,H,H))))
 *   + bias (+ ebias[b][co], row stride eb_stride) (+ res), ks 1|3, mode
 *   0 stride 1 / 1 stride 2 (Downsample) / 2 nearest-x2 upsample then conv;
 *   act 0 none / 1 GroupNorm+SiLU / 2 GroupNorm, gn = (B, Cin) float2
 *   {scale, shift} from ertd_group_norm_stats; precision FP32 | BF16 | BF16X3;
 *   H in {16,32,64,128} (Ho likewise); ws >= ertd_conv2d_workspace_bytes(Cin,
 *   Cout, ks, precision, B, H, mode): the packed weights plus the launch's
 *   scratch (a Winograd K split's partial sums, the bf16 pre-transformed
 *   input image), all caller-owned -- the call allocates nothing.  fp32 3x3 stride-1 convs with Cout % 64 == 0 run as
 *   Winograd F(4x4,3x3) (Cin, Ca % 4 == 0; H >= 32, or 16 when the tile items
 *   fill the device) or F(2x2,3x3) (Cin, Ca % 8 == 0), the rest as direct
 *   implicit GEMMs; ERTD_UNET_WINO=2 keeps F(2x2), 0 disables Winograd.
 * ertd_group_norm_stats: per (sample, channel) {gamma*rstd, beta-mean*gamma*rstd}
 *   of cat(x, x2) over `groups` groups (eps 1e-5), out (B, Ca+Cb) float2.
 * ertd_attention: qkv (B, 3C, N) -> out (B, C, N) = v softmax(q^T k / sqrt C)^T, N = 256.
 * ertd_group_norm_partials: parts (B, C, np, 2) = per (sample, channel, part of n = 256
 *   pixels) {sum, sum (x - sum/n)^2} of x (B, C, HW); HW = 256 np.  The fp32
 *   Winograd convs of the U-Net walk emit the same partials of their output from the
 *   epilogue, so a GroupNorm does not re-read its input.
 * ertd_group_norm_finalize: out (B, Ca+Cb) {scale, shift} exactly as ertd_group_norm_stats
 *   (and mr (B, groups) {mean, rstd}, optional) from the partials of the two concatenated
 *   inputs (pb = null when Cb = 0), combined per group in a fixed order in float64.  */
size_t ertd_conv2d_workspace_bytes(int cin, int cout, int ks, int precision, int B, int H,
                                   int mode);
int ertd_conv2d(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* w,
                const float* bias, int Cout, int ks, int mode, const float* gn, int act,
                const float* ebias, int eb_stride, const float* res, float* out, int precision,
                void* ws, size_t ws_bytes, void* stream);
/* ertd_conv2d_run: the same conv reusing the packing a previous ertd_conv2d call with the
 * same (Ca, Cb, B, H, Cout, ks, mode, act, precision) and weights left at the head of ws
 * (no weight read, no pack kernel: the conv kernel alone, e.g. for per-kernel timing). */
int ertd_conv2d_run(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* bias,
                    int Cout, int ks, int mode, const float* gn, int act, const float* ebias,
                    int eb_stride, const float* res, float* out, int precision, void* ws,
                    size_t ws_bytes, void* stream);
/* ertd_conv2d_gn_parts: np > 0 when the fp32 conv ertd_conv2d dispatches for this geometry
 *   emits the GroupNorm partials of its output from the epilogue ((B, Cout, np) float2
 *   {sum, M2} over HW / np pixels each, the ertd_group_norm_partials format), else 0.
 * ertd_conv2d_gn / ertd_conv2d_run_gn: ertd_conv2d / ertd_conv2d_run that also write those
 *   partials (gn_np = that np), for ertd_group_norm_finalize without re-reading the output
 *   (the train walk).  */
int ertd_conv2d_gn_parts(int Ca, int Cb, int Cout, int ks, int mode, int act, int precision, int B, int H);
int ertd_conv2d_gn(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* w,
                   const float* bias, int Cout, int ks, int mode, const float* gn, int act,
                   const float* ebias, int eb_stride, const float* res, float* out, int precision,
                   void* ws, size_t ws_bytes, float* gn_parts, int gn_np, void* stream);
int ertd_conv2d_run_gn(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* bias,
                       int Cout, int ks, int mode, const float* gn, int act, const float* ebias,
                       int eb_stride, const float* res, float* out, int precision, void* ws,
                       size_t ws_bytes, float* gn_parts, int gn_np, void* stream);
int ertd_group_norm_stats(const float* x, int Ca, const float* x2, int Cb, int B, int HW,
                          int groups, const float* gamma, const float* beta, float* out,
                          void* stream);
int ertd_attention(const float* qkv, int B, int C, int N, float* out, void* stream);
int ertd_group_norm_partials(const float* x, int C, int B, int HW, int np, float* parts, void* stream);
int ertd_group_norm_finalize(const float* pa, int npa, int Ca, const float* pb, int npb, int Cb, int B,
                             int HW, int groups, const float* gamma, const float* beta, float* out,
                             float* mr, void* stream);
/* ertd_act_bf16: img [B][ceil(C/16)][Ho][Ho][16] bf16 (RNE) of act(cat(x, x2)*ss.x + ss.y)
 *   (act 0 none / 1 GN+SiLU / 2 GN; ss (B, C, 2) as ertd_group_norm_stats) or, with up = 1
 *   (act 0), of the nearest-x2 upsample of cat(x, x2) (Ho = 2H): the bf16 path's standalone
 *   image transform (act_bf16_kernel).
 * ertd_unet_update: the U-Net sampler's DDPM update (sample_model :111-118) of x (B, P) given
 *   eps, per-step tables c1/c2/sigma (index t = *t_dev) and injected noise
 *   (num_steps, B, P) or Philox (noise = null; seed, member ids from member_offset). */
int ertd_act_bf16(const float* x, int Ca, const float* x2, int Cb, int B, int H, const float* ss,
                  int act, int up, void* img, void* stream);
int ertd_unet_update(float* x, const float* eps, const float* c1, const float* c2,
                     const float* sigma, const float* noise, int num_steps, const int* t_dev,
                     uint64_t seed, uint32_t member_offset, int B, int P, void* stream);
/* ertd_group_norm_act_bf16: the bf16 path's fused prologue of a 3x3 GN conv
 *   in one pass -- out as ertd_group_norm_stats, and img = bf16 RNE of
 *   act(GroupNorm(cat(x, x2))) (act: silu=1 SiLU, 0 none) in the conv's
 *   [B][C/16][H][H][16] layout (C*H*H*2 bytes per sample).  ERTD_EINVAL
 *   unless C % 16 == 0, lcm(C/groups, 16) * H*H <= 65536 (and a multiple of
 *   1024), H*H % 64 == 0.                                                    */
int ertd_group_norm_act_bf16(const float* x, int Ca, const float* x2, int Cb, int B, int H,
                             int groups, const float* gamma, const float* beta, float* out,
                             void* img, int silu, void* stream);

/* Parameter tensors in state_dict order: count, and (name, shape) of one.  */
int ertd_unet_n_params(const ertd_unet_config* cfg);
int ertd_unet_param_info(const ertd_unet_config* cfg, int idx, char* name, int name_len,
                         int64_t* shape, int* ndim);
/* Packed device weights (floats) and their packing from the params array
 * (ertd_unet_n_params device pointers, state_dict order).  freq: (ch/2)
 * float32 sinusoid frequencies computed on the host with the reference's
 * get_timestep_embedding expression (:80-88) at dim = ch.                 */
size_t ertd_unet_packed_floats(const ertd_unet_config* cfg);
int ertd_unet_pack(const ertd_unet_config* cfg, const float* const* params, const float* freq,
                   float* packed, void* stream);
/* Workspace bytes for batch B and condition length L (forward and sampler). */
size_t ertd_unet_workspace_bytes(const ertd_unet_config* cfg, int B, int L);
/* eps = unet(x (B, image^2), t (B,) int64, cond (B,14,L) with member stride
 * cond_stride floats (0: one shared condition)); cond_emb_out (B,128) optional. */
int ertd_unet_forward(const ertd_unet_config* cfg, const float* packed, const float* x,
                      const int64_t* t, const float* cond, long long cond_stride, int L, int B,
                      float* out, float* cond_emb_out, void* ws, size_t ws_bytes, void* stream);
/* sample_model (:102-119) around the U-Net: steps t = t_first .. t_first-n_run+1 on
 * x_inout (B, image^2); c1/c2/sigma/noise/seed/member_offset as in ertd_sample.
 * The condition embedding is computed once per call (it does not depend on x
 * or t; recomputing it per step would give identical bits).               */
int ertd_unet_sample(const ertd_unet_config* cfg, const float* packed, const float* cond,
                     long long cond_stride, int L, int B, int num_steps, int t_first, int n_run,
                     const float* c1, const float* c2, const float* sigma, const float* noise,
                     uint64_t seed, uint32_t member_offset, float* x_inout, void* ws,
                     size_t ws_bytes, void* stream);
/* The same call as a plan: the head and one step are captured as hipGraphs
 * once; a launch replays head + n_run x step on `stream`.  For bf16
 * precision the step graph is not a single chain: the embedding dense layers
 * and each ResBlock's 1x1 skip conv are captured on a plan-owned side stream
 * (event fork/join), so they run beside conv_in / conv1 (fp32 captures one
 * chain: its persistent Winograd convs occupy every CU); results equal the
 * eager call bit for bit either way.  The plan owns its capture streams and
 * events (ertd_unet_plan_destroy frees them); ERTD_UNET_SIDE=0/1 in the
 * environment forces one chain / the forked graph.                          */
typedef struct ertd_unet_plan ertd_unet_plan;
int ertd_unet_sample_plan_create(const ertd_unet_config* cfg, const float* packed, const float* cond,
                                 long long cond_stride, int L, int B, int num_steps, int t_first,
                                 int n_run, const float* c1, const float* c2, const float* sigma,
                                 const float* noise, uint64_t seed, uint32_t member_offset,
                                 float* x_inout, void* ws, size_t ws_bytes, ertd_unet_plan** plan);
int ertd_unet_plan_launch(ertd_unet_plan* plan, void* stream);
/* head + the first n_steps (0 <= n_steps <= n_run) steps only: warms both
 * graphs (first-launch upload) without running the whole plan.            */
int ertd_unet_plan_launch_steps(ertd_unet_plan* plan, int n_steps, void* stream);
int ertd_unet_plan_destroy(ertd_unet_plan* plan);

/* ---- U-Net training operators (csrc/unet_train.hip; the reference train step
 * ERT_Conditional_Diffusion.py:305-320 around the build-defined U-Net, walked
 * by ertdiff/unet_train.py).  PARITY UNPINNED vs the reference (no U-Net
 * there): checked against torch autograd on oracle/unet_torch.py.  All device
 * pointers, enqueued on `stream`; `accumulate` = add into the output.
 * ertd_gn_stats_mr: ertd_group_norm_stats + mr_out (B, groups) {mean, rstd}.
 * ertd_gn_act_apply: out (B, Ca+Cb, HW) = act(cat(x, x2) * ss.x + ss.y), act 1 GN+SiLU / 2 GN.
 * ertd_gn_act_backward: dx / dx2 of act(GroupNorm(cat(x, x2))) given dy (B, C, HW);
 *   dgb_part (B, 2, C): per-sample sum dxn*xhat ([b][0]) and sum dxn ([b][1]) ->
 *   (dgamma | dbeta) by one ertd_reduce_rows (rows B, cols 2C).
 * ertd_gn_act_backward_csum: the same, plus csum[b * ldc + c] = sum over the HW pixels
 *   of the gradient this call adds to channel c of sample b (a ResBlock's emb-projection
 *   gradient when dx is the conv1 output's gradient; channels per group <= 64).
 * ertd_gn_act_backward_add: the same with an addend: dx / dx2 (+)= addc + the GroupNorm
 *   gradient, addc (B, C, HW) in the concatenated channel order (a ResBlock's skip / identity
 *   gradient of the same input), added first (as a separate add before the call would); csum
 *   optional (null: none), and when given it sums the GroupNorm term only.
 * ertd_im2col: out (B, C*ks*ks, Ho*Ho) patches of x (B, C, H, H), mode 0 s1 / 1 s2 / 2 upsample.
 * ertd_wgrad_gemm: dW (M, N) = sum_b dY_b (M, P) . X_b (N, P)^T (batch strides bsA, bsB),
 *   fp32 MFMA, split per sample + fixed-order reduction; ws >= ertd_wgrad_ws_bytes.
 * ertd_conv_weight_flip: out (Cin, Cout, ks, ks) = w (Cout, Cin, ks, ks) spatially flipped.
 * ertd_zero_insert: out (B, C, 2Ho, 2Ho) with x at even positions; ertd_sum_pool2: 2x2 sums.
 * ertd_channel_sums: out_bc (B, C; row stride ldo, 0 = C) sums over HW; out_c (C) = sum over b
 *   (optional, ldo = C).
 * ertd_concat: dst = cat(srcs[0..n)) of contiguous fp32 tensors (sizes in elements).
 * ertd_encoder_train_pack: copies condition_encoder.0 / .2 weights into an
 *   ertd_packed_floats() buffer (the layout ertd_encoder_train_fwd / _bwd read).
 * ertd_gemm_small: C[b][i][j] = alpha sum_k A[b][i][k] B[b][k][j] (+ bias[j]) with element
 *   strides (a_i, a_k, a_b, b_k, b_j, b_b, c_i, c_j, c_b).
 * ertd_softmax_rows: P = softmax(scale S) per row; ertd_softmax_backward: dS = scale P (dP - <dP, P>).
 * ertd_eltwise: op 0 silu(x), 1 y silu'(x), 2 relu(x), 3 y [x > 0], 4 x + y, 5 alpha x.
 * ertd_channel_slice: dst (B, Cdst, HW) channels [d0, d0+Cd) (+)= src (B, Cs, HW) channels
 *   [c0, c0+Cd).
 * ertd_mse_loss: loss (1) = mean (eps - noise)^2, dout = 2 (eps - noise) / n (optional);
 *   ws >= ertd_mse_loss_ws_bytes() (float64 partial sums, caller-owned).
 * ertd_encoder_train_fwd / _bwd: the reference condition encoder (:133-142) with saved
 *   activations in ws (pool mean m (B, 64) out) / conv-parameter grads from g = dL/dm / L.
 * ertd_adam_multi: torch.optim.Adam step (no weight decay) over ntensors tensors.        */
int ertd_gn_stats_mr(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                     const float* gamma, const float* beta, float* ss_out, float* mr_out,
                     void* stream);
int ertd_gn_act_apply(const float* x, int Ca, const float* x2, int Cb, int B, int HW,
                      const float* ss, int act, float* out, void* stream);
int ertd_gn_act_backward(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                         const float* gamma, const float* beta, const float* mr, int act,
                         const float* dy, float* dx, float* dx2, int accumulate, float* dgb_part,
                         void* stream);
int ertd_gn_act_backward_csum(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                              const float* gamma, const float* beta, const float* mr, int act,
                              const float* dy, float* dx, float* dx2, int accumulate, float* dgb_part,
                              float* csum, long long ldc, void* stream);
int ertd_gn_act_backward_add(const float* x, int Ca, const float* x2, int Cb, int B, int HW, int groups,
                             const float* gamma, const float* beta, const float* mr, int act,
                             const float* dy, const float* addc, float* dx, float* dx2, int accumulate,
                             float* dgb_part, float* csum, long long ldc, void* stream);
int ertd_im2col(const float* x, int C, int B, int H, int ks, int mode, float* out, void* stream);
size_t ertd_wgrad_ws_bytes(int M, int N, int P, int B);
int ertd_wgrad_gemm(const float* dY, const float* X, int M, int N, int P, int B, long long bsA,
                    long long bsB, float* dW, int accumulate, void* ws, size_t ws_bytes,
                    void* stream);
int ertd_reduce_rows(const float* part, int rows, long long cols, float* out, int accumulate,
                     void* stream);
/* ertd_reduce_rows_multi: n independent ertd_reduce_rows problems (host arrays of
 * their arguments) in ceil(n / 48) launches; every output bitwise equal to the
 * single call's.  The U-Net train walk defers its per-layer dgamma/dbeta and
 * linear-bias reductions (no other kernel reads them before the optimizer) to one
 * such call at the end of the backward.                                         */
int ertd_reduce_rows_multi(const float* const* parts, const int* rows, const long long* cols,
                           float* const* outs, const int* accumulate, int n, void* stream);
int ertd_conv_weight_flip(const float* w, int Cout, int Cin, int ks, float* out, void* stream);
int ertd_zero_insert(const float* x, int B, int C, int Ho, float* out, void* stream);
int ertd_sum_pool2(const float* x, int B, int C, int H, float* out, int accumulate, void* stream);
int ertd_channel_sums(const float* x, int B, int C, int HW, float* out_bc, int ldo, float* out_c,
                      int accumulate_c, void* stream);
int ertd_gemm_small(const float* A, long long a_i, long long a_k, long long a_b, const float* Bm,
                    long long b_k, long long b_j, long long b_b, float* C, long long c_i,
                    long long c_j, long long c_b, const float* bias, int I, int J, int K, int batch,
                    float alpha, int accumulate, void* stream);
int ertd_softmax_rows(const float* S, long long rows, int N, float scale, float* P, void* stream);
int ertd_softmax_backward(const float* P, const float* dP, long long rows, int N, float scale,
                          float* dS, void* stream);
int ertd_eltwise(int op, const float* x, const float* y, float* out, long long n, float alpha,
                 int accumulate, void* stream);
int ertd_channel_slice(const float* src, int B, int Cs, int c0, int Cd, int HW, float* dst,
                       int Cdst, int d0, int accumulate, void* stream);
size_t ertd_mse_loss_ws_bytes(void);
int ertd_mse_loss(const float* eps, const float* noise, long long n, float* loss, float* dout,
                  void* ws, size_t ws_bytes, void* stream);
/* ertd_conv_wgrad: dW (Cout, Ca+Cb, ks, ks) (+)= the weight gradient of
 *   y = conv(cat(x, x2)) (mode 0 stride 1 / 1 stride 2 / 2 nearest-x2 upsample,
 *   as ertd_conv2d) given dy (B, Cout, Ho, Ho): implicit GEMM on fp32 MFMA,
 *   fixed-order split reduction; ws >= ertd_conv_wgrad_ws_bytes (0 = unsupported
 *   geometry: output side not a power of two in [16, 128]).  csrc/unet_wgrad.hip. */
size_t ertd_conv_wgrad_ws_bytes(int Cin, int Cout, int B, int H, int ks, int mode);
/* ertd_conv_input_grad: dx (B, Cin, H, H) (+)= dL/dx of y = conv(x) (weight w (Cout, Cin, ks, ks),
 *   mode as ertd_conv2d) given dy (B, Cout, Ho, Ho): a stride-1 conv of dy (stride 2:
 *   zero-inserted; upsample: at 2H then 2x2 sum-pooled) with w transposed and flipped, packed
 *   straight from w (Winograd where eligible); ws >= ertd_conv_input_grad_ws_bytes.       */
size_t ertd_conv_input_grad_ws_bytes(int Cin, int Cout, int B, int H, int ks, int mode);
int ertd_conv_input_grad(const float* dy, int B, int H, const float* w, int Cout, int Cin, int ks,
                         int mode, float* dx, int accumulate, void* ws, size_t ws_bytes,
                         void* stream);
/* ertd_conv_input_grad_run: the same, reusing the flipped packing an earlier
 *   ertd_conv_input_grad (or ertd_conv_pack_batch with the descriptor of
 *   ertd_conv_input_grad_pack_desc) left at the head of ws.                    */
int ertd_conv_input_grad_run(const float* dy, int B, int H, int Cout, int Cin, int ks, int mode,
                             float* dx, int accumulate, void* ws, size_t ws_bytes, void* stream);
int ertd_conv_wgrad(const float* dy, const float* x, int Ca, const float* x2, int Cb, int B, int H,
                    int Cout, int ks, int mode, const float* gn, int act, float* dw, int accumulate,
                    void* ws, size_t ws_bytes, void* stream);
/* ertd_conv_wgrad_bias: ertd_conv_wgrad plus the conv's bias gradient db (Cout) = sum of dy
 *   over samples and pixels (written, not accumulated; also into db2 when non-null, e.g.
 *   a 1x1 skip conv fed the same dy), fused into the Winograd path's dy transform.  Only
 *   where ertd_conv_wgrad_bias_ok (3x3 stride 1 / upsample on the Winograd path, B * tiles
 *   a multiple of 256); ws as ertd_conv_wgrad_ws_bytes.                                  */
int ertd_conv_wgrad_bias_ok(int Cin, int Cout, int B, int H, int ks, int mode);
int ertd_conv_wgrad_bias(const float* dy, const float* x, int Ca, const float* x2, int Cb, int B, int H,
                         int Cout, int ks, int mode, const float* gn, int act, float* dw, int accumulate,
                         float* db, float* db2, void* ws, size_t ws_bytes, void* stream);

/* Batched fp32 weight packing (the train step packs every conv once per
 * optimizer step, in one launch).  A descriptor names one packing: the source
 * weight, its destination, and the layout a later ertd_conv2d_run /
 * ertd_conv_input_grad_run on that workspace reads -- filled by the two
 * *_pack_desc queries from the same dispatch decisions as ertd_conv2d /
 * ertd_conv_input_grad, so the batch writes exactly their packings, bit for bit. */
#define ERTD_PACK_DIRECT 0 /* implicit-GEMM fragment order (1x1 / 3x3)   */
#define ERTD_PACK_UP 1     /* sub-pixel Upsample classes                 */
#define ERTD_PACK_WINO 2   /* Winograd F(2x2,3x3) U = G g G^T            */
#define ERTD_PACK_WINO4 3  /* Winograd F(4x4,3x3)                        */
typedef struct {
  const float* w;      /* source weight (Cout, Cin, ks, ks) of the FORWARD conv    */
  float* dst;          /* destination (inside the conv's workspace)               */
  long long total;     /* packed floats                                           */
  int cin, cout, ks;   /* of the packed conv (flip: the input-gradient conv's)    */
  int kind;            /* ERTD_PACK_*                                             */
  int flip;            /* 1: the input-gradient conv's transposed, flipped weight */
  int nchunk;          /* K chunks of the layout                                  */
  int block0;          /* first 256-thread block (ertd_conv_pack_batch_prepare)   */
  int reserved;
} ertd_pack_desc;
int ertd_conv2d_pack_desc(int Cin, int Ca, int Cout, int ks, int mode, int precision, int B, int H,
                          const float* w, void* ws, ertd_pack_desc* out);
int ertd_conv_input_grad_pack_desc(int Cin, int Cout, int B, int H, int ks, int mode, const float* w,
                                   void* ws, ertd_pack_desc* out);
/* host: fills block0 of descs[0..n) in order; returns the batch's block count (< 0: error) */
int ertd_conv_pack_batch_prepare(ertd_pack_desc* descs, int n);
/* one launch packing all n descriptors (descs: DEVICE copy of the prepared table) */
int ertd_conv_pack_batch(const ertd_pack_desc* descs, int n, int blocks, void* stream);
int ertd_concat(const float* const* srcs, const long long* sizes, int n, float* dst, void* stream);
/* ertd_split: dsts[k] = alpha * src[sum(sizes[<k]) ...] (the inverse of ertd_concat, scaled):
 *   the data-parallel train step's gradient bucket back into the per-tensor gradients. */
int ertd_split(const float* src, float* const* dsts, const long long* sizes, int n, float alpha,
               void* stream);
int ertd_encoder_train_pack(const float* w0, const float* w2, float* packed, void* stream);
size_t ertd_encoder_train_ws_bytes(int B, int L);
int ertd_encoder_train_fwd(const float* packed, const float* b1, const float* b2, const float* cond,
                           int B, int L, float* m_out, void* ws, size_t ws_bytes, void* stream);
int ertd_encoder_train_bwd(const float* packed, const float* cond, const float* g, int B, int L,
                           float* dw1, float* db1, float* dw2, float* db2, void* ws,
                           size_t ws_bytes, void* stream);
int ertd_adam_multi(float* const* params, const float* const* grads, float* const* exp_avg,
                    float* const* exp_avg_sq, const long long* sizes, int ntensors, int step,
                    float lr, float beta1, float beta2, float eps, void* stream);

/* ---- Ensemble KDE mode (csrc/kde.hip) -------------
 * Replaces the reference's per-cell loop ERT_Conditional_Diffusion.py:747-762
 * (scipy.stats.gaussian_kde per cell of sim_data, evaluated on
 * np.linspace(lo, hi, grid), mode = grid point of the first maximum) and
 * mode_kde_calculation :166-181 (one array, its own range, 1000 points).
 * x: (n, ld) float64 row-major on the device, cell c = column c < cells.
 * range_mode 0: grid over [lo, hi]; 1: each cell's own [min, max];
 * 2: [lo, hi] read from range_dev (2 doubles, e.g. ertd_minmax_f64's output).
 * mode (cells) receives the mode; index (cells, optional) the grid index, -1
 * where the cell's variance is 0 (gaussian_kde raises there); density
 * (cells, optional) the KDE value at the mode.  Requires 2 <= n <= 20480.   */
int ertd_kde_mode(const double* x, int n, long long cells, long long ld, int grid, int range_mode,
                  double lo, double hi, const double* range_dev, double* mode, int* index,
                  double* density, void* stream);

/* min and max of count float64 values: out2 = {min, max} (device);
 * work: 2 * ERTD_MINMAX_BLOCKS doubles of device scratch.                  */
#define ERTD_MINMAX_BLOCKS 1024
int ertd_minmax_f64(const double* x, long long count, double* work, double* out2, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ERTDIFF_H */
