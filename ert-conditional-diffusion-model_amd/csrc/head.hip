// Head of ConditionalDiffusionModel and the reverse-diffusion update.
//
//   pool finish + condition_encoder.6 Linear(64->128)+ReLU  (ERT_Conditional_Diffusion.py:138-141)
//   sinusoid + time_embed Linear(128->128)+ReLU            (:80-88, :144-147, :159-160)
//   mlp: Linear(P+256 -> 128)+ReLU -> Linear(128 -> P)     (:149-153, :162-163)
//   x <- c1_t (x - c2_t eps) + sigma_t z                   (:111-118)
//
// mlp.0 is evaluated as  h = relu( (u + v) + W0x.x )  with
//   u = b0 + W0c.cond_emb   (per member; constant over the T loop)
//   v = W0t.t_emb           (per timestep; identical for all members)
// and every dot product is a sequential fma chain in a fixed k order.  The
// faithful kernel (head_kernel, encoder re-run every step) and the hoisted
// persistent sampler call the same device functions and the same per-wave
// step body, so both modes produce bit-identical trajectories.
#include "head_dev.h"

namespace ertd {


struct HeadSmem {
  float pg[POOL_GROUPS][C2];   // pool group sums
  float m[C2];
  float e[H];
  float c[H];
  float te[H];
  float part[2][2][H];         // [branch][q][j] split-k partials
  float w[H];                  // u + v
  float hbuf[H];               // step body scratch (wave 0)
  float xbuf[PMAX];
  alignas(16) float w0xr[H * W0XR_PITCH];
  alignas(16) float w2l[64 * W2L_PITCH];
};

// waves 0-3: condition branch, 4-7: time branch; wave 0 then runs the step.
constexpr int HEAD_THREADS = 512;

// ---------------------------------------------------------------------------
// head_kernel: one 512-thread workgroup per member; full head for timestep t.
//   forward mode (eps_out != null): eps_out = model(x, t, cond)
//   step mode    (x_out  != null): one faithful DDPM step
// Threads 0..255: condition branch (j = tid&127, q = tid>>7), 256..511: time
// branch.  Every weight a thread needs is requested at kernel start.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(HEAD_THREADS) void head_kernel(ertd_weights w,
                                                            const float* __restrict__ packed,
                                                            HeadArgs a) {
  __shared__ HeadSmem sm;
  const int P = w.param_dim;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool cond_br = tid < 256;
  const int j = tid & (H - 1), q = (tid >> 7) & 1;
  const DenseT d = dense_ptrs(packed);
  const int64_t t = a.t_vec ? a.t_vec[b] : (int64_t)a.t_scalar;
  const int ts = (int)t;
  const int o = lane >> 1;
  HEAD_STAMP(0);

  // ---- issue every load up front ------------------------------------------------
  CondW cw;
  TimeW tw;
  if (cond_br) load_cond_w(cw, d, P, j, q);
  else load_time_w(tw, d, P, j, q);
  float xv = 0.f, z = 0.f, c1 = 0.f, c2 = 0.f, sig = 0.f, bo = 0.f;
  if (wave == 0) {  // the step's own inputs, off the critical path
    xv = o < P ? a.x_in[(size_t)b * P + o] : 0.f;
    bo = o < P ? w.mlp2_b[o] : 0.f;
    if (!a.eps_out) {
      z = step_noise(a.noise, a.num_steps, ts, a.B, b, P, o, a.seed, member_id(a.member_offset, b, a.ncond, a.id_period));
      c1 = a.c1[ts];
      c2 = a.c2[ts];
      sig = a.sigma[ts];
    }
  }
  {  // verbatim copies of the packed step images (float4, coalesced)
    const float4* s0 = reinterpret_cast<const float4*>(packed + PACK_W0XR);
    const float4* s1 = reinterpret_cast<const float4*>(packed + PACK_W2L);
    float4* d0 = reinterpret_cast<float4*>(sm.w0xr);
    float4* d1 = reinterpret_cast<float4*>(sm.w2l);
    for (int i = tid; i < W0XR_FLOATS / 4; i += HEAD_THREADS) d0[i] = s0[i];
    for (int i = tid; i < W2L_FLOATS / 4; i += HEAD_THREADS) d1[i] = s1[i];
  }
  {
    const int c = tid & (C2 - 1), g = tid >> 6;
    sm.pg[g][c] = pool_group(a.partial, b, a.S, c, g);
  }
  const float bias_c = (cond_br && q == 0) ? w.enc6_b[j] : 0.f;
  const float bias_u = (cond_br && q == 0) ? w.mlp0_b[j] : 0.f;
  const float bias_t = (!cond_br && q == 0) ? w.time_b[j] : 0.f;
  if (!cond_br && q == 0) sm.e[j] = sinusoid((float)t, a.freq, j);
  __syncthreads();
  HEAD_STAMP(1);

  // ---- layer 1: cond_emb (64 -> 128), t_emb (128 -> 128) -------------------------
  if (tid < C2) sm.m[tid] = pool_combine(sm.pg, tid, a.L2);
  __syncthreads();
  HEAD_STAMP(2);
  if (cond_br) sm.part[0][q][j] = chain_half<C2>(cw.w3, sm.m, bias_c, q);
  else sm.part[1][q][j] = chain_half<H>(tw.wt, sm.e, bias_t, q);
  __syncthreads();
  HEAD_STAMP(3);
  if (tid < H) {
    const float c = fmaxf(sm.part[0][0][j] + sm.part[0][1][j], 0.f);
    sm.c[j] = c;
    if (a.cond_emb_out) a.cond_emb_out[(size_t)b * H + j] = c;
  } else if (tid >= 256 && tid < 256 + H) {
    const float te = fmaxf(sm.part[1][0][j] + sm.part[1][1][j], 0.f);
    sm.te[j] = te;
    if (a.t_emb_out) a.t_emb_out[(size_t)b * H + j] = te;
  }
  __syncthreads();

  // ---- layer 2: u = b0 + W0c.c, v = W0t.te --------------------------------------
  if (cond_br) sm.part[0][q][j] = chain_half<H>(cw.w0c, sm.c, bias_u, q);
  else sm.part[1][q][j] = chain_half<H>(tw.w0t, sm.te, 0.f, q);
  __syncthreads();
  if (tid < H) {
    const float u = sm.part[0][0][j] + sm.part[0][1][j];
    const float v = sm.part[1][0][j] + sm.part[1][1][j];
    sm.w[j] = u + v;
  }
  __syncthreads();
  HEAD_STAMP(4);
  if (wave != 0) return;

  // ---- step body (wave 0), weights read from LDS inside the chains -----------------
  float xs[PMAX];
  broadcast_x(xs, xv, P, lane, sm.xbuf);
  HEAD_STAMP(5);
  const LdsSrc src{sm.w0xr + lane * W0XR_PITCH, sm.w0xr + (lane + 64) * W0XR_PITCH,
                   sm.w2l + lane * W2L_PITCH, bo};
  const float eps = step_eps(src, sm.w[lane], sm.w[lane + 64], xs, P, lane, sm.hbuf);
  HEAD_STAMP(6);
  if (a.eps_out) {
    if (!(lane & 1) && o < P) a.eps_out[(size_t)b * P + o] = eps;
    return;
  }
  xv = ddpm_update(xv, eps, c1, c2, sig, z, ts > 0);
  if (!(lane & 1) && o < P) a.x_out[(size_t)b * P + o] = xv;
  HEAD_STAMP(7);
}

hipError_t launch_head(const ertd_weights& w, const float* packed, const HeadArgs& a, hipStream_t s) {
  head_kernel<<<a.B, HEAD_THREADS, 0, s>>>(w, packed, a);
  return hipGetLastError();
}



// ---- hoisted-mode precomputation ------------------------------------------------
__global__ __launch_bounds__(256) void hoist_prep_kernel(ertd_weights w, const float* __restrict__ packed,
                                                         const float* __restrict__ partial, int S,
                                                         int L2, float* __restrict__ U,
                                                         float* __restrict__ cond_emb_out) {
  __shared__ CondScratch sc;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int j = tid & (H - 1), q = tid >> 7;
  const DenseT d = dense_ptrs(packed);
  CondW cw;
  load_cond_w(cw, d, w.param_dim, j, q);
  cond_row_pool(sc, partial, b, S, tid);
  const float bias_c = q == 0 ? w.enc6_b[j] : 0.f;
  const float bias_u = q == 0 ? w.mlp0_b[j] : 0.f;
  __syncthreads();
  const float u = cond_row_finish(sc, cw, bias_c, bias_u, L2, tid, j, q,
                                  cond_emb_out ? cond_emb_out + (size_t)b * H : nullptr);
  if (tid < H) U[(size_t)b * H + j] = u;
}

__global__ __launch_bounds__(256) void time_table_kernel(ertd_weights w, const float* __restrict__ packed,
                                                         const float* __restrict__ freq, int t_lo,
                                                         float* __restrict__ V) {
  __shared__ TimeScratch sc;
  const int t = t_lo + (int)blockIdx.x;
  time_row(sc, w, dense_ptrs(packed), freq, t, V + (size_t)t * H, threadIdx.x);
}

hipError_t launch_hoist_prep(const ertd_weights& w, const float* packed, const float* partial,
                             int S, int L2, int B, float* U, float* cond_emb_out, hipStream_t s) {
  hoist_prep_kernel<<<B, 256, 0, s>>>(w, packed, partial, S, L2, U, cond_emb_out);
  return hipGetLastError();
}

hipError_t launch_time_table(const ertd_weights& w, const float* packed, const float* freq,
                             int t_lo, int n, float* V, hipStream_t s) {
  time_table_kernel<<<n, 256, 0, s>>>(w, packed, freq, t_lo, V);
  return hipGetLastError();
}

// ---- faithful per-step head -------------------------------------------------------
// One block per member: the condition branch for this step's pool partials,
// w = u + v(t), then wave 0 runs the step.  v(t) -- the time branch, identical
// for every member of a step -- is computed once per step by an extra block of
// the step's encoder launch (time_row_lean: the same fma chains as the
// hoisted time table, so both modes stay bit-identical).
struct HeadStepSmem {
  CondScratch cond;
  float w[H];
  alignas(16) float hbuf[H];
  alignas(16) float xbuf[PMAX];
};
constexpr int HEAD_STEP_THREADS = 320;  // waves 0-3: condition branch, wave 4: step

__global__ __launch_bounds__(HEAD_STEP_THREADS) void head_step_kernel(
    ertd_weights w, const float* __restrict__ packed, HeadArgs a, const float* __restrict__ V) {
  __shared__ HeadStepSmem sm;
  const int tid = threadIdx.x, lane = tid & 63;
  const bool step_wave = tid >= 256;
  const DenseT d = dense_ptrs(packed);
  const int P = w.param_dim, b = blockIdx.x, ts = a.t_scalar;
  const int j = tid & (H - 1), q = (tid >> 7) & 1, o = lane >> 1;
  HEAD_STAMP(0);
  CondW cw;
  StepRegs R;
  float xv = 0.f, z = 0.f, c1 = 0.f, c2 = 0.f, sig = 0.f;
  if (step_wave) {  // the step's weights and inputs, requested at kernel start
    load_step_regs(R, packed, w.mlp2_b, P, lane);
    xv = o < P ? a.x_in[(size_t)b * P + o] : 0.f;
    z = step_noise(a.noise, a.num_steps, ts, a.B, b, P, o, a.seed, member_id(a.member_offset, b, a.ncond, a.id_period));
    c1 = a.c1[ts];
    c2 = a.c2[ts];
    sig = a.sigma[ts];
  } else {
    load_cond_w(cw, d, P, j, q);
    cond_row_pool(sm.cond, a.partial, b, a.S, tid);
  }
  const float bias_c = q == 0 ? w.enc6_b[j] : 0.f;
  const float bias_u = q == 0 ? w.mlp0_b[j] : 0.f;
  const float vj = tid < H ? V[(size_t)ts * H + j] : 0.f;
  __syncthreads();
  HEAD_STAMP(1);
  // cond_row_finish's barriers are block-wide: the step wave joins them idle
  float u = 0.f;
  if (!step_wave) u = cond_row_finish_nb(sm.cond, cw, bias_c, bias_u, a.L2, tid, j, q);
  else cond_row_idle();
  HEAD_STAMP(2);
  if (tid < H) sm.w[j] = u + vj;
  __syncthreads();
  HEAD_STAMP(3);
  if (!step_wave) return;
  float xs[PMAX];
  broadcast_x(xs, xv, P, lane, sm.xbuf);
  HEAD_STAMP(4);
  const RegSrc src{R, R.bo};
  const float eps = step_eps(src, sm.w[lane], sm.w[lane + 64], xs, P, lane, sm.hbuf);
  HEAD_STAMP(5);
  xv = ddpm_update(xv, eps, c1, c2, sig, z, ts > 0);
  if (!(lane & 1) && o < P) a.x_out[(size_t)b * P + o] = xv;
  HEAD_STAMP(6);
}

hipError_t launch_head_step(const ertd_weights& w, const float* packed, const HeadArgs& a,
                            const float* V, hipStream_t s) {
  head_step_kernel<<<a.B, HEAD_STEP_THREADS, 0, s>>>(w, packed, a, V);
  return hipGetLastError();
}

// ---- persistent hoisted sampler ---------------------------------------------------
// One wave per member runs all num_steps steps; x lives in registers (lane 2o
// and 2o+1 hold x[o]; a readlane broadcast feeds the next step's W0x.x as
// scalar operands).  Members are independent: no inter-wave communication.
__global__ __launch_bounds__(256) void hoisted_sampler_kernel(
    ertd_weights w, const float* __restrict__ packed, const float* __restrict__ U,
    const float* __restrict__ V, const float* __restrict__ c1, const float* __restrict__ c2,
    const float* __restrict__ sigma, const float* __restrict__ noise, int num_steps, int t_first,
    int n_run, uint64_t seed, uint32_t member_offset, int B, float* __restrict__ x, int ncond,
    int id_period, int u_rows) {
  __shared__ float hbuf[4][H];
  __shared__ float xbuf[4][PMAX];
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave exits together (no block barriers below)
  const int P = w.param_dim;
  StepRegs R;
  load_step_regs(R, packed, w.mlp2_b, P, lane);
  // u_rows > 0: one condition row per condition (the encoder ran once per
  // condition), member b reads row b % u_rows
  const int ur = u_rows > 0 ? b % u_rows : b;
  const float u_lo = U[(size_t)ur * H + lane];
  const float u_hi = U[(size_t)ur * H + 64 + lane];
  const int o = lane >> 1;
  const uint32_t member = member_id(member_offset, b, ncond, id_period);
  float xv = o < P ? x[(size_t)b * P + o] : 0.f;
  float xs[PMAX];
  for (int t = t_first; t > t_first - n_run; --t) {
    broadcast_x(xs, xv, P, lane, xbuf[threadIdx.x >> 6]);
    const float w_lo = u_lo + V[(size_t)t * H + lane];
    const float w_hi = u_hi + V[(size_t)t * H + 64 + lane];
    const float z = step_noise(noise, num_steps, t, B, b, P, o, seed, member);
    const RegSrc src{R, R.bo};
    const float eps = step_eps(src, w_lo, w_hi, xs, P, lane, hbuf[threadIdx.x >> 6]);
    xv = ddpm_update(xv, eps, c1[t], c2[t], sigma[t], z, t > 0);
  }
  if (!(lane & 1) && o < P) x[(size_t)b * P + o] = xv;
}

hipError_t launch_hoisted_sampler(const ertd_weights& w, const float* packed, const float* U,
                                  const float* V, const float* c1, const float* c2,
                                  const float* sigma, const float* noise, int num_steps,
                                  int t_first, int n_run, uint64_t seed, uint32_t member_offset,
                                  int B, float* x, hipStream_t s, int ncond, int id_period,
                                  int u_rows) {
  hoisted_sampler_kernel<<<(B + 3) / 4, 256, 0, s>>>(w, packed, U, V, c1, c2, sigma, noise,
                                                      num_steps, t_first, n_run, seed,
                                                      member_offset, B, x, ncond, id_period, u_rows);
  return hipGetLastError();
}

// ---- small API kernels -------------------------------------------------------------
__global__ void timestep_embedding_kernel(const int64_t* __restrict__ t, int B, int dim,
                                          const float* __restrict__ freq, float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * dim) return;
  const int b = idx / dim, k = idx - b * dim;
  const int half = dim / 2;
  const float tf = (float)t[b];
  float v = 0.f;  // odd-dim zero pad (:86-87)
  if (k < half) v = sinf(tf * freq[k]);
  else if (k < 2 * half) v = cosf(tf * freq[k - half]);
  out[idx] = v;
}

__global__ void q_sample_kernel(const float* __restrict__ x0, const int64_t* __restrict__ t,
                                const float* __restrict__ noise, const float* __restrict__ ab,
                                int B, int P, float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * P) return;
  const float abt = ab[t[idx / P]];
  const float sa = sqrtf(abt);
  const float sb = sqrtf(1.0f - abt);
  out[idx] = sa * x0[idx] + sb * noise[idx];
}

__global__ void philox_normal_kernel(uint64_t seed, uint32_t member_offset, int B, int P, int t,
                                     int tag, float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * P) return;
  const int b = idx / P, o = idx - b * P;
  out[idx] = philox_normal(seed, member_offset + (uint32_t)b, (uint32_t)t, (uint32_t)tag, o);
}

hipError_t launch_timestep_embedding(const int64_t* t, int B, int dim, const float* freq,
                                     float* out, hipStream_t s) {
  const int n = B * dim;
  timestep_embedding_kernel<<<(n + 255) / 256, 256, 0, s>>>(t, B, dim, freq, out);
  return hipGetLastError();
}

hipError_t launch_q_sample(const float* x0, const int64_t* t, const float* noise,
                           const float* alpha_bar, int B, int P, float* out, hipStream_t s) {
  const int n = B * P;
  q_sample_kernel<<<(n + 255) / 256, 256, 0, s>>>(x0, t, noise, alpha_bar, B, P, out);
  return hipGetLastError();
}

hipError_t launch_philox_normal(uint64_t seed, uint32_t member_offset, int B, int P, int t,
                                int tag, float* out, hipStream_t s) {
  const int n = B * P;
  philox_normal_kernel<<<(n + 255) / 256, 256, 0, s>>>(seed, member_offset, B, P, t, tag, out);
  return hipGetLastError();
}

}  // namespace ertd
