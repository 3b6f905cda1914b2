// Device helpers of the head (pool finish, dense split-k chains, the per-wave
// step body, condition/time rows), shared by head.hip and the fused faithful
// step kernel (step.hip).  Header-only; every function is inlined.
#pragma once
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
struct PlainLoad {
  __device__ float operator()(const float* p) const { return *p; }
};
template <class Ld = PlainLoad>
__device__ __forceinline__ float pool_group(const float* __restrict__ partial, int b, int S, int c,
                                            int g, Ld ld = Ld()) {
  // loads of 4 strips issued together, then added in strip order
  const float* p = partial + (size_t)b * S * C2 + c;
  float acc = 0.f;
  int s = g;
  for (; s + 3 * POOL_GROUPS < S; s += 4 * POOL_GROUPS) {
    const float v0 = ld(p + (size_t)s * C2), v1 = ld(p + (size_t)(s + POOL_GROUPS) * C2);
    const float v2 = ld(p + (size_t)(s + 2 * POOL_GROUPS) * C2);
    const float v3 = ld(p + (size_t)(s + 3 * POOL_GROUPS) * C2);
    acc += v0;
    acc += v1;
    acc += v2;
    acc += v3;
  }
  float v[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    v[i] = s + i * POOL_GROUPS < S ? ld(p + (size_t)(s + i * POOL_GROUPS) * C2) : 0.f;
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

// ---- condition branch row and time row (shared by every mode) ---------------------
// cond_row: U[j] = b0_j + W0c.relu(W3.mean + b3) for one member, 256 threads
// (j = tid&127, q = tid>>7).  Weights must already be in `cw` (loaded early).
struct CondScratch {
  float pg[POOL_GROUPS][C2];
  float m[C2];
  float c[H];
  float part[2][H];
};
template <class Ld = PlainLoad>
__device__ __forceinline__ void cond_row_pool(CondScratch& sc, const float* partial, int b, int S,
                                              int tid, Ld ld = Ld()) {
  for (int i = tid; i < POOL_GROUPS * C2; i += 256) {
    const int cc = i & (C2 - 1), g = i >> 6;
    sc.pg[g][cc] = pool_group(partial, b, S, cc, g, ld);
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

}  // namespace ertd
