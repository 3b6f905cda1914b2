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

// Phase stamps for the diagnostic build only (tools/diag_head.hip defines
// ERTD_HEAD_STAMPS); the library build compiles them out.
#ifdef ERTD_HEAD_STAMPS
__device__ unsigned long long g_head_stamps[1024][2][8];
#define HEAD_STAMP(i)                                                                   \
  do {                                                                                  \
    if ((threadIdx.x & 255) == 0)                                                       \
      g_head_stamps[blockIdx.x][threadIdx.x >> 8][i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define HEAD_STAMP(i) \
  do {                \
  } while (0)
#endif

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

// ---- dense layers: 2-way split-k ------------------------------------------------
// Each output j of a 128-wide layer is produced by two threads q = 0, 1: thread q
// runs a sequential fma chain over k in [q*N/2, (q+1)*N/2) (q = 0 starts from the
// bias), the two partials are added (p0 + p1).  The weights of a thread's half
// are loaded into registers at kernel start, so a whole layer costs one global
// latency round.  Faithful head, hoist_prep and time_table all use these
// functions with the same (j, q) layout: bit-identical results.
template <int N>
struct HalfW {
  float w[N / 2];
};
template <int N>
__device__ __forceinline__ void load_half(HalfW<N>& r, const float* __restrict__ WT, int j, int q) {
#pragma unroll
  for (int k = 0; k < N / 2; ++k) r.w[k] = WT[(q * (N / 2) + k) * H + j];
}
template <int N>
__device__ __forceinline__ float chain_half(const HalfW<N>& r, const float* v, float init, int q) {
  float acc = init;
#pragma unroll
  for (int k = 0; k < N / 2; ++k) acc = fmaf(r.w[k], v[q * (N / 2) + k], acc);
  return acc;
}

// Pool finish: 8 interleaved strip groups (group g sums strips g, g+8, ...),
// combined in group order, divided by L2.
constexpr int POOL_GROUPS = 8;
__device__ __forceinline__ float pool_group(const float* __restrict__ partial, int b, int S, int c,
                                            int g) {
  // loads of 4 strips issued together, then added in strip order
  const float* p = partial + (size_t)b * S * C2 + c;
  float acc = 0.f;
  int s = g;
  for (; s + 3 * POOL_GROUPS < S; s += 4 * POOL_GROUPS) {
    const float v0 = p[(size_t)s * C2], v1 = p[(size_t)(s + POOL_GROUPS) * C2];
    const float v2 = p[(size_t)(s + 2 * POOL_GROUPS) * C2], v3 = p[(size_t)(s + 3 * POOL_GROUPS) * C2];
    acc += v0;
    acc += v1;
    acc += v2;
    acc += v3;
  }
  float v[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) v[i] = s + i * POOL_GROUPS < S ? p[(size_t)(s + i * POOL_GROUPS) * C2] : 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (s + i * POOL_GROUPS < S) acc += v[i];
  return acc;
}
__device__ __forceinline__ float pool_combine(const float (*pg)[C2], int c, int L2) {
  float acc = pg[0][c];
#pragma unroll
  for (int g = 1; g < POOL_GROUPS; ++g) acc += pg[g][c];
  return acc / (float)L2;
}

// Sinusoidal embedding element k (< 128) of timestep t (:82-85).
__device__ __forceinline__ float sinusoid(float tf, const float* __restrict__ freq, int k) {
  constexpr int half = H / 2;
  const float a = tf * freq[k < half ? k : k - half];
  return k < half ? sinf(a) : cosf(a);
}

// Weights of the condition branch (cond_emb, u) and of the time branch (t_emb, v).
struct CondW {
  HalfW<C2> w3;  // condition_encoder.6
  HalfW<H> w0c;  // mlp.0, cond_emb columns
};
struct TimeW {
  HalfW<H> wt;   // time_embed.0
  HalfW<H> w0t;  // mlp.0, t_emb columns
};
__device__ __forceinline__ void load_cond_w(CondW& r, const DenseT& d, int P, int j, int q) {
  load_half<C2>(r.w3, d.W3T, j, q);
  load_half<H>(r.w0c, d.W0T + (size_t)(P + H) * H, j, q);
}
__device__ __forceinline__ void load_time_w(TimeW& r, const DenseT& d, int P, int j, int q) {
  load_half<H>(r.wt, d.WtT, j, q);
  load_half<H>(r.w0t, d.W0T + (size_t)P * H, j, q);
}

// ---- per-wave step body --------------------------------------------------------
// One wave per member.  Lane l holds hidden units l and l+64 of mlp.0 and, for
// mlp.2, output o = l>>1 over the k-half (l&1): eps_o is one 64-term fma chain
// per half against h broadcast from LDS, the halves joined by one lane swap
// (a commutative add, so both lanes of a pair hold identical bits).
struct StepRegs {
  float w0x_lo[PMAX], w0x_hi[PMAX];  // W0[lane][k], W0[lane+64][k]  (k < P)
  float w2h[H / 2];                  // W2[lane>>1][64*(lane&1) + k]  (o < P)
  float bo;                          // b2[lane>>1]
};

// All loads coalesced: W0T rows (k-major) and the lane-major W2F copy.
__device__ __forceinline__ void load_step_regs(StepRegs& R, const float* __restrict__ packed,
                                               const float* __restrict__ b2, int P, int lane) {
  const float* W0T = packed + PACK_TOTAL + C2 * H + H * H;
  const float* W2F = packed + PACK_W2F;
  const int o = lane >> 1;
#pragma unroll
  for (int k = 0; k < PMAX; ++k) {
    R.w0x_lo[k] = k < P ? W0T[k * H + lane] : 0.f;
    R.w0x_hi[k] = k < P ? W0T[k * H + 64 + lane] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < H / 2; ++k) R.w2h[k] = W2F[k * 64 + lane];
  R.bo = o < P ? b2[o] : 0.f;
}

// xs[k] = x[k] for every lane: lanes 2k write x[k] to this wave's LDS slot,
// then every lane reads the slot back (uniform-address broadcast reads).
__device__ __forceinline__ void broadcast_x(float (&xs)[PMAX], float xv, int P, int lane,
                                            float* xbuf) {
  if (!(lane & 1) && (lane >> 1) < P) xbuf[lane >> 1] = xv;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int k = 0; k < PMAX; ++k) xs[k] = k < P ? xbuf[k] : 0.f;
}

// eps for o = lane>>1 given the pre-activations of hidden units lane, lane+64.
// hbuf: this wave's 128-float LDS scratch.  Src supplies the weights (registers
// in the persistent sampler, LDS images in the per-step head): same fma order.
template <class Src>
__device__ __forceinline__ float step_eps(const Src& W, float w_lo, float w_hi,
                                          const float (&xs)[PMAX], int P, int lane, float* hbuf) {
  // mlp.0 x-part: two chains per hidden unit (k < 16, k >= 16), joined in order
  float a_lo = w_lo, a_hi = w_hi, b_lo = 0.f, b_hi = 0.f;
#pragma unroll
  for (int k = 0; k < PMAX / 2; ++k) {
    if (k < P) {
      a_lo = fmaf(W.w0x_lo(k), xs[k], a_lo);
      a_hi = fmaf(W.w0x_hi(k), xs[k], a_hi);
    }
    if (k + PMAX / 2 < P) {
      b_lo = fmaf(W.w0x_lo(k + PMAX / 2), xs[k + PMAX / 2], b_lo);
      b_hi = fmaf(W.w0x_hi(k + PMAX / 2), xs[k + PMAX / 2], b_hi);
    }
  }
  hbuf[lane] = fmaxf(a_lo + b_lo, 0.f);
  hbuf[64 + lane] = fmaxf(a_hi + b_hi, 0.f);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // mlp.2: four 16-term chains over this lane's k-half, joined (c0+c1)+(c2+c3)
  const float4* hh4 = reinterpret_cast<const float4*>(hbuf + 64 * (lane & 1));
  float hv[H / 2];  // all 16 LDS reads in flight before the chains start
#pragma unroll
  for (int i = 0; i < H / 8; ++i) {
    const float4 q4 = hh4[i];
    hv[4 * i] = q4.x;
    hv[4 * i + 1] = q4.y;
    hv[4 * i + 2] = q4.z;
    hv[4 * i + 3] = q4.w;
  }
  float c[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = fmaf(W.w2h(16 * i + k), hv[16 * i + k], c[i]);
  }
  const float acc = (c[0] + c[1]) + (c[2] + c[3]);
  const float e = acc + __shfl_xor(acc, 1);
  return e + W.bo;
}

struct RegSrc {  // StepRegs in registers
  const StepRegs& R;
  float bo;
  __device__ float w0x_lo(int k) const { return R.w0x_lo[k]; }
  __device__ float w0x_hi(int k) const { return R.w0x_hi[k]; }
  __device__ float w2h(int k) const { return R.w2h[k]; }
};
struct LdsSrc {  // the packed W0XR / W2L images copied into LDS (16-B aligned rows)
  const float* w0x_row_lo;  // &W0XR[lane][0]
  const float* w0x_row_hi;  // &W0XR[lane + 64][0]
  const float* w2_row;      // &W2L[lane][0]
  float bo;
  __device__ float w0x_lo(int k) const { return w0x_row_lo[k]; }
  __device__ float w0x_hi(int k) const { return w0x_row_hi[k]; }
  __device__ float w2h(int k) const { return w2_row[k]; }
};

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
      z = step_noise(a.noise, a.num_steps, ts, a.B, b, P, o, a.seed, a.member_offset + (uint32_t)b);
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


// ---- condition branch row and time row (shared by every mode) ---------------------
// cond_row: U[j] = b0_j + W0c.relu(W3.mean + b3) for one member, 256 threads
// (j = tid&127, q = tid>>7).  Weights must already be in `cw` (loaded early).
struct CondScratch {
  float pg[POOL_GROUPS][C2];
  float m[C2];
  float c[H];
  float part[2][H];
};
__device__ __forceinline__ void cond_row_pool(CondScratch& sc, const float* partial, int b, int S,
                                              int tid) {
  for (int i = tid; i < POOL_GROUPS * C2; i += 256) {
    const int cc = i & (C2 - 1), g = i >> 6;
    sc.pg[g][cc] = pool_group(partial, b, S, cc, g);
  }
}
// after cond_row_pool + __syncthreads(); returns u_j on threads < 128 (else 0).
// Four block barriers; cond_row_idle() mirrors them for waves that sit it out.
__device__ __forceinline__ float cond_row_finish_nb(CondScratch& sc, const CondW& cw, float bias_c,
                                                    float bias_u, int L2, int tid, int j, int q,
                                                    float* cond_emb_out = nullptr) {
  if (tid < C2) sc.m[tid] = pool_combine(sc.pg, tid, L2);
  __syncthreads();
  sc.part[q][j] = chain_half<C2>(cw.w3, sc.m, bias_c, q);
  __syncthreads();
  if (tid < H) {
    const float cj = fmaxf(sc.part[0][j] + sc.part[1][j], 0.f);
    sc.c[j] = cj;
    if (cond_emb_out) cond_emb_out[j] = cj;
  }
  __syncthreads();
  sc.part[q][j] = chain_half<H>(cw.w0c, sc.c, bias_u, q);
  __syncthreads();
  return tid < H ? sc.part[0][j] + sc.part[1][j] : 0.f;
}
__device__ __forceinline__ void cond_row_idle() {
#pragma unroll
  for (int i = 0; i < 4; ++i) __syncthreads();
}
__device__ __forceinline__ float cond_row_finish(CondScratch& sc, const CondW& cw, float bias_c,
                                                 float bias_u, int L2, int tid, int j, int q,
                                                 float* cond_emb_out) {
  return cond_row_finish_nb(sc, cw, bias_c, bias_u, L2, tid, j, q, cond_emb_out);
}

// time_row: V[t][j] = W0t.relu(Wt.sinusoid(t) + bt), 256 threads.
struct TimeScratch {
  float e[H];
  float te[H];
  float part[2][H];
};
__device__ __forceinline__ void time_row(TimeScratch& sc, const ertd_weights& w, const DenseT& d,
                                         const float* freq, int t, float* vrow, int tid) {
  const int j = tid & (H - 1), q = tid >> 7;
  TimeW tw;
  load_time_w(tw, d, w.param_dim, j, q);
  const float bias_t = q == 0 ? w.time_b[j] : 0.f;
  if (q == 0) sc.e[j] = sinusoid((float)t, freq, j);
  __syncthreads();
  sc.part[q][j] = chain_half<H>(tw.wt, sc.e, bias_t, q);
  __syncthreads();
  if (tid < H) sc.te[j] = fmaxf(sc.part[0][j] + sc.part[1][j], 0.f);
  __syncthreads();
  sc.part[q][j] = chain_half<H>(tw.w0t, sc.te, 0.f, q);
  __syncthreads();
  if (tid < H) vrow[j] = sc.part[0][j] + sc.part[1][j];
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
    z = step_noise(a.noise, a.num_steps, ts, a.B, b, P, o, a.seed, a.member_offset + (uint32_t)b);
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
    int n_run, uint64_t seed, uint32_t member_offset, int B, float* __restrict__ x) {
  __shared__ float hbuf[4][H];
  __shared__ float xbuf[4][PMAX];
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave exits together (no block barriers below)
  const int P = w.param_dim;
  StepRegs R;
  load_step_regs(R, packed, w.mlp2_b, P, lane);
  const float u_lo = U[(size_t)b * H + lane];
  const float u_hi = U[(size_t)b * H + 64 + lane];
  const int o = lane >> 1;
  const uint32_t member = member_offset + (uint32_t)b;
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
