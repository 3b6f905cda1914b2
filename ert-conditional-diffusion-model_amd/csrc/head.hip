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
#include "ertd_common.h"

namespace ertd {

// k-major dense weights behind the conv fragments (see pack_dense_kernel)
struct DenseT {
  const float* W3T;  // [64][128]
  const float* WtT;  // [128][128]
  const float* W0T;  // [P+256][128]: rows 0..P-1 x part, P..P+127 t part, P+128.. c part
};
__device__ __forceinline__ DenseT dense_ptrs(const float* packed) {
  DenseT d;
  d.W3T = packed + PACK_TOTAL;
  d.WtT = d.W3T + C2 * H;
  d.W0T = d.WtT + H * H;
  return d;
}

// out_j = init + sum_{k<N} WT[k][j] * v[k]: sequential fma chain in k.
template <int N>
__device__ __forceinline__ float dotT(const float* __restrict__ WT, const float* v, float init, int j) {
  float acc = init;
#pragma unroll 16
  for (int k = 0; k < N; ++k) acc = fmaf(WT[k * H + j], v[k], acc);
  return acc;
}

// Pool finish: mean over L2 of the per-strip sums, strips summed in order.
__device__ __forceinline__ float pool_mean(const float* __restrict__ partial, int b, int S, int L2, int c) {
  float acc = 0.f;
  for (int s = 0; s < S; ++s) acc += partial[((size_t)b * S + s) * C2 + c];
  return acc / (float)L2;
}

// Sinusoidal embedding element k (< 128) of timestep t (:82-85).
__device__ __forceinline__ float sinusoid(float tf, const float* __restrict__ freq, int k) {
  constexpr int half = H / 2;
  const float a = tf * freq[k < half ? k : k - half];
  return k < half ? sinf(a) : cosf(a);
}

// cond_emb_j and u_j (thread j < 128); m in LDS.
__device__ __forceinline__ float cond_emb_j(const DenseT& d, const ertd_weights& w, const float* m, int j) {
  return fmaxf(dotT<C2>(d.W3T, m, w.enc6_b[j], j), 0.f);
}
__device__ __forceinline__ float u_j(const DenseT& d, const ertd_weights& w, const float* c, int j) {
  return dotT<H>(d.W0T + (size_t)(w.param_dim + H) * H, c, w.mlp0_b[j], j);
}
// t_emb_j and v_j (thread j < 128); e / te in LDS.
__device__ __forceinline__ float t_emb_j(const DenseT& d, const ertd_weights& w, const float* e, int j) {
  return fmaxf(dotT<H>(d.WtT, e, w.time_b[j], j), 0.f);
}
__device__ __forceinline__ float v_j(const DenseT& d, const ertd_weights& w, const float* te, int j) {
  return dotT<H>(d.W0T + (size_t)w.param_dim * H, te, 0.f, j);
}

// ---- per-wave step body --------------------------------------------------------
struct StepRegs {
  float w0x_lo[PMAX], w0x_hi[PMAX];  // W0[lane][k], W0[lane+64][k]  (k < P)
  float w2_lo[PMAX], w2_hi[PMAX];    // W2[o][lane], W2[o][lane+64]  (o < P)
  float bo;                          // b2[lane>>1]
};

__device__ __forceinline__ void load_step_regs(StepRegs& R, const float* __restrict__ W0T,
                                               const float* __restrict__ W2,
                                               const float* __restrict__ b2, int P, int lane) {
#pragma unroll
  for (int k = 0; k < PMAX; ++k) {
    R.w0x_lo[k] = k < P ? W0T[k * H + lane] : 0.f;
    R.w0x_hi[k] = k < P ? W0T[k * H + 64 + lane] : 0.f;
    R.w2_lo[k] = k < P ? W2[k * H + lane] : 0.f;
    R.w2_hi[k] = k < P ? W2[k * H + 64 + lane] : 0.f;
  }
  const int o = lane >> 1;
  R.bo = o < P ? b2[o] : 0.f;
}

// xs[k] = x[k], held by lanes 2k and 2k+1 (wave-uniform result).
__device__ __forceinline__ void broadcast_x(float (&xs)[PMAX], float xv, int P) {
#pragma unroll
  for (int k = 0; k < PMAX; ++k)
    xs[k] = k < P ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), 2 * k)) : 0.f;
}

// eps for o = lane>>1 given the pre-activations of hidden units lane, lane+64.
__device__ __forceinline__ float step_eps(const StepRegs& R, float w_lo, float w_hi,
                                          const float (&xs)[PMAX], int P, int lane) {
  float a_lo = w_lo, a_hi = w_hi;
#pragma unroll
  for (int k = 0; k < PMAX; ++k) {
    if (k < P) {
      a_lo = fmaf(R.w0x_lo[k], xs[k], a_lo);
      a_hi = fmaf(R.w0x_hi[k], xs[k], a_hi);
    }
  }
  const float h_lo = fmaxf(a_lo, 0.f), h_hi = fmaxf(a_hi, 0.f);
  // per-lane partials of all 32 outputs, then a fixed butterfly reduce-scatter:
  // level i pairs lane bit (5-i) with output bit (4-i); lane l ends with o = l>>1.
  float v[32];
#pragma unroll
  for (int o = 0; o < 32; ++o) v[o] = fmaf(R.w2_hi[o], h_hi, R.w2_lo[o] * h_lo);
#pragma unroll
  for (int lvl = 0; lvl < 5; ++lvl) {
    const int n = 16 >> lvl;
    const int lb = 5 - lvl;
    const bool up = (lane >> lb) & 1;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const float keep = up ? v[n + i] : v[i];
      const float send = up ? v[i] : v[n + i];
      v[i] = keep + __shfl_xor(send, 1 << lb);
    }
  }
  const float e = v[0] + __shfl_xor(v[0], 1);
  return e + R.bo;
}

// x <- c1*(x - c2*eps) [+ sig*z], one fp32 rounding per reference op (:113-118).
__device__ __forceinline__ float ddpm_update(float xv, float eps, float c1, float c2, float sig,
                                             float z, bool add_noise) {
  const float t1 = c2 * eps;
  const float t2 = xv - t1;
  const float t3 = c1 * t2;
  return add_noise ? t3 + sig * z : t3;
}

__device__ __forceinline__ float step_noise(const float* __restrict__ noise, int num_steps, int t,
                                            int B, int b, int P, int o, uint64_t seed,
                                            uint32_t member) {
  if (o >= P || t == 0) return 0.f;
  if (noise) return noise[((size_t)(num_steps - t) * B + b) * P + o];
  return philox_normal(seed, member, (uint32_t)t, 0u, o);
}

struct HeadSmem {
  float m[C2];
  float e[H];
  float c[H];
  float te[H];
  float u[H];
  float v[H];
};

// ---------------------------------------------------------------------------
// head_kernel: one workgroup per member; full head for timestep t.
//   forward mode (eps_out != null): eps_out = model(x, t, cond)
//   step mode    (x_out  != null): one faithful DDPM step
// Threads 0..127 run the condition branch, 128..255 the time branch.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void head_kernel(ertd_weights w, const float* __restrict__ packed,
                                                   HeadArgs a) {
  __shared__ HeadSmem sm;
  const int P = w.param_dim;
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const DenseT d = dense_ptrs(packed);
  const int64_t t = a.t_vec ? a.t_vec[b] : (int64_t)a.t_scalar;

  if (tid < C2) sm.m[tid] = pool_mean(a.partial, b, a.S, a.L2, tid);
  if (tid >= H) sm.e[tid - H] = sinusoid((float)t, a.freq, tid - H);
  __syncthreads();
  if (tid < H) {
    const float c = cond_emb_j(d, w, sm.m, tid);
    sm.c[tid] = c;
    if (a.cond_emb_out) a.cond_emb_out[(size_t)b * H + tid] = c;
  } else {
    const int j = tid - H;
    const float te = t_emb_j(d, w, sm.e, j);
    sm.te[j] = te;
    if (a.t_emb_out) a.t_emb_out[(size_t)b * H + j] = te;
  }
  __syncthreads();
  if (tid < H) sm.u[tid] = u_j(d, w, sm.c, tid);
  else sm.v[tid - H] = v_j(d, w, sm.te, tid - H);
  __syncthreads();
  if (wave != 0) return;

  StepRegs R;
  load_step_regs(R, d.W0T, w.mlp2_w, w.mlp2_b, P, lane);
  const int o = lane >> 1;
  float xv = o < P ? a.x_in[(size_t)b * P + o] : 0.f;
  float xs[PMAX];
  broadcast_x(xs, xv, P);
  const float w_lo = sm.u[lane] + sm.v[lane];
  const float w_hi = sm.u[lane + 64] + sm.v[lane + 64];
  const float eps = step_eps(R, w_lo, w_hi, xs, P, lane);
  if (a.eps_out) {
    if (!(lane & 1) && o < P) a.eps_out[(size_t)b * P + o] = eps;
    return;
  }
  const int ts = (int)t;
  const float z = step_noise(a.noise, a.num_steps, ts, a.B, b, P, o, a.seed,
                             a.member_offset + (uint32_t)b);
  xv = ddpm_update(xv, eps, a.c1[ts], a.c2[ts], a.sigma[ts], z, ts > 0);
  if (!(lane & 1) && o < P) a.x_out[(size_t)b * P + o] = xv;
}

hipError_t launch_head(const ertd_weights& w, const float* packed, const HeadArgs& a, hipStream_t s) {
  head_kernel<<<a.B, 256, 0, s>>>(w, packed, a);
  return hipGetLastError();
}

// ---- hoisted-mode precomputation ------------------------------------------------
// U[b][j] = b0_j + W0c.relu(W3.mean + b3)   (one 128-thread block per member)
__global__ __launch_bounds__(128) void hoist_prep_kernel(ertd_weights w, const float* __restrict__ packed,
                                                         const float* __restrict__ partial, int S,
                                                         int L2, float* __restrict__ U,
                                                         float* __restrict__ cond_emb_out) {
  __shared__ float m[C2];
  __shared__ float c[H];
  const int b = blockIdx.x, j = threadIdx.x;
  const DenseT d = dense_ptrs(packed);
  if (j < C2) m[j] = pool_mean(partial, b, S, L2, j);
  __syncthreads();
  const float cj = cond_emb_j(d, w, m, j);
  c[j] = cj;
  if (cond_emb_out) cond_emb_out[(size_t)b * H + j] = cj;
  __syncthreads();
  U[(size_t)b * H + j] = u_j(d, w, c, j);
}

// V[t][j] = W0t.relu(Wt.sinusoid(t) + bt)   (one 128-thread block per timestep)
__global__ __launch_bounds__(128) void time_table_kernel(ertd_weights w, const float* __restrict__ packed,
                                                         const float* __restrict__ freq, int t_lo,
                                                         float* __restrict__ V) {
  __shared__ float e[H];
  __shared__ float te[H];
  const int t = t_lo + (int)blockIdx.x, j = threadIdx.x;
  const DenseT d = dense_ptrs(packed);
  e[j] = sinusoid((float)t, freq, j);
  __syncthreads();
  te[j] = t_emb_j(d, w, e, j);
  __syncthreads();
  V[(size_t)t * H + j] = v_j(d, w, te, j);
}

hipError_t launch_hoist_prep(const ertd_weights& w, const float* packed, const float* partial,
                             int S, int L2, int B, float* U, float* cond_emb_out, hipStream_t s) {
  hoist_prep_kernel<<<B, 128, 0, s>>>(w, packed, partial, S, L2, U, cond_emb_out);
  return hipGetLastError();
}

hipError_t launch_time_table(const ertd_weights& w, const float* packed, const float* freq,
                             int t_lo, int n, float* V, hipStream_t s) {
  time_table_kernel<<<n, 128, 0, s>>>(w, packed, freq, t_lo, V);
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
    int n_run, uint64_t seed, uint32_t member_offset, int B, float* __restrict__ x) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave exits together
  const int P = w.param_dim;
  const DenseT d = dense_ptrs(packed);
  StepRegs R;
  load_step_regs(R, d.W0T, w.mlp2_w, w.mlp2_b, P, lane);
  const float u_lo = U[(size_t)b * H + lane];
  const float u_hi = U[(size_t)b * H + 64 + lane];
  const int o = lane >> 1;
  const uint32_t member = member_offset + (uint32_t)b;
  float xv = o < P ? x[(size_t)b * P + o] : 0.f;
  float xs[PMAX];
  for (int t = t_first; t > t_first - n_run; --t) {
    broadcast_x(xs, xv, P);
    const float w_lo = u_lo + V[(size_t)t * H + lane];
    const float w_hi = u_hi + V[(size_t)t * H + 64 + lane];
    const float z = step_noise(noise, num_steps, t, B, b, P, o, seed, member);
    const float eps = step_eps(R, w_lo, w_hi, xs, P, lane);
    xv = ddpm_update(xv, eps, c1[t], c2[t], sigma[t], z, t > 0);
  }
  if (!(lane & 1) && o < P) x[(size_t)b * P + o] = xv;
}

hipError_t launch_hoisted_sampler(const ertd_weights& w, const float* packed, const float* U,
                                  const float* V, const float* c1, const float* c2,
                                  const float* sigma, const float* noise, int num_steps,
                                  int t_first, int n_run, uint64_t seed, uint32_t member_offset,
                                  int B, float* x, hipStream_t s) {
  hoisted_sampler_kernel<<<(B + 3) / 4, 256, 0, s>>>(w, packed, U, V, c1, c2, sigma, noise,
                                                      num_steps, t_first, n_run, seed,
                                                      member_offset, B, x);
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
