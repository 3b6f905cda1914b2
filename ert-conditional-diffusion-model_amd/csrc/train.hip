// Training step on gfx950: ERT_Conditional_Diffusion.py:309-319
//   x_noisy = q_sample(x0, t, noise)               (:96-99, :314)
//   pred = model(x_noisy, t, cond)                  (:155-164, :315)
//   loss = MSELoss(pred, noise)  (mean)             (:295, :316)
//   loss.backward(); Adam(lr=1e-4).step()           (:294, :318-319)
//
// Four kernels per step; every kernel reads the parameters in place (no
// packing pass), every reduction has a fixed order (bitwise reproducible for
// any grid):
//   enc_train_kernel    per (member, strip of J conv2 outputs): conv1 -> ReLU ->
//                       conv2 -> ReLU -> pool partial sums (the sampler's strip
//                       body, enc_strip.h), plus what the backward reads: the
//                       strip's conv1 images (a1s, float4 rows) and the conv2
//                       ReLU mask as bits (m2w, one ballot per accumulator row)
//   train_head_kernel   per member: q_sample, pool finish, dense forward, MSE
//                       gradient, dense backward down to g = dL/dm / L2 (the
//                       forward and backward halves alone for the autograd path)
//   conv_bwd_kernel     per (member, strip): dz2 = g * mask -> da1 (transposed
//                       conv2, MFMA) -> dz1; dW2 / dW1 / db1 / db2 partial row
//   train_final_kernel  dense-layer gradients (chains over members), the strip
//                       partial rows reduced in order, the loss, and in the
//                       train step the Adam update of every element
#include <cmath>
#include <cstring>

#include "enc_strip.h"

namespace ertd {

// ---- per-member saved vectors (one row of TV floats per member) ------------------
constexpr int TV_HCAT = 0;          // [x (P) | t_emb (128) | cond_emb (128)], P+256 <= 288
constexpr int TV_E = 288;           // sinusoid (128)
constexpr int TV_M = TV_E + H;      // pooled mean (64)
constexpr int TV_H = TV_M + C2;     // relu(z5) (128)
constexpr int TV_EPS = TV_H + H;    // prediction (32)
constexpr int TV_DOUT = TV_EPS + 32;  // dL/dpred (32)
constexpr int TV_DZ5 = TV_DOUT + 32;  // (128)
constexpr int TV_DZ4 = TV_DZ5 + H;    // (128)
constexpr int TV_DZ3 = TV_DZ4 + H;    // (128)
constexpr int TV_G = TV_DZ3 + H;      // dm / L2 (64)
constexpr int TV_SQ = TV_G + C2;      // sum of squared errors (1)
constexpr int TV = TV_SQ + 16;        // row pitch (floats)

// conv-gradient partial row: [dW1 32x42 | dW2 64x96 | db1 32 | db2 64]
constexpr int NG_W1 = 0;
constexpr int NG_W2 = C1 * K1;
constexpr int NG_B1 = NG_W2 + C2 * K2;
constexpr int NG_B2 = NG_B1 + C1;
constexpr int NG = NG_B2 + C2;  // 7584 (every region a multiple of 4 floats)
// the reference train step splits the row: conv_bwd's chain rows [dW1 | db1]
// (NG1) per (member, strip), and w2m_body's rows [M | mask counts] (NG2) per
// (member, group of W2M_NS strips) with dW2 = sum_b g_b[o] M_b[o][n] (dz2 =
// g * mask: dW2 is linear in g, so M needs no g and runs beside the head)
constexpr int NG1 = C1 * K1 + C1;   // 1376
constexpr int NG2 = C2 * K2 + C2;   // 6208
constexpr int W2M_NS = 3;           // strips per w2m workgroup
__host__ __device__ inline int w2m_groups(int S) { return (S + W2M_NS - 1) / W2M_NS; }

// saved activations per (member, strip): the conv1 images E[c][m] = a1(p = 2m),
// O[c][m] = a1(p = 2m+1) at conv1 positions i = 2*j0 - 1 + p, p < 128 (zero
// outside [0, L1)), and the conv2 ReLU mask word [q][o >> 5] (bit o & 31) of
// conv2 output j0 + q (0 for q >= J or j0 + q >= L2)
constexpr int A1S_FLOATS = 2 * C1 * 64;
constexpr int M2W_WORDS = 64 * 2;

// k-major copies of the dense weights (written by enc_train_kernel each step)
constexpr int WT_W3 = 0;                    // [64][128]   W3T[k][j] = W3[j][k]
constexpr int WT_WT = WT_W3 + C2 * H;       // [128][128]  time_embed.0
constexpr int WT_W0 = WT_WT + H * H;        // [K0][128]   mlp.0 (K0 = P + 256 <= 288)
constexpr int WT_W2 = WT_W0 + (PMAX + 2 * H) * H;  // [128][32] mlp.2: W2T[k][o]
constexpr int WT_W0B = WT_W2 + H * PMAX;    // [128][256]  mlp.0 columns P.. (16-B aligned rows): W0[j][P + k]
constexpr int WT_W5 = WT_W0B + H * 2 * H;   // [PMAX][128]  mlp.2 rows, zero past P
constexpr int WT_FLOATS = WT_W5 + PMAX * H;

constexpr int W2B_FRAG = 3 * 32 * 64;  // transposed-conv2 fragments (conv_bwd)
#ifndef ENC_ABL
#define ENC_ABL 0  // diagnostic variants only: bit 0 no a1s stores, 1 no mask words, 2 no weight copies, 3 no LDS weight staging
#endif
// train_final_kernel's conv-column reduction (see there)
constexpr int FIN_CB_COLS = 64;                                  // float4 columns per block
constexpr int FIN_NCB = (NG / 4 + FIN_CB_COLS - 1) / FIN_CB_COLS;  // 30 column blocks
#ifndef FIN_RB_N
#define FIN_RB_N 4
#endif
constexpr int FIN_RB = FIN_RB_N;                                 // row blocks
constexpr int FIN_MAXR = FIN_RB < 8 ? 48 : 384 / FIN_RB;   // rows per wave held in flight
constexpr int FIN_CNT_WORDS = 64;
static_assert(FIN_NCB <= FIN_CNT_WORDS, "counter words");
static_assert(NG1 + NG2 == NG, "split rows cover the gradient row");

// ---------------------------------------------------------------------------
// training forward of the condition encoder
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void enc_train_kernel(
    const float* __restrict__ w1, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ cond, int L, int L1, int L2, int S,
    float* __restrict__ partial, float* __restrict__ a1s, uint32_t* __restrict__ m2w,
    unsigned* __restrict__ fin_cnt, int* __restrict__ step_ctr, ertd_weights wd,
    float* __restrict__ wt, float* __restrict__ w2b) {
  __shared__ __attribute__((aligned(16))) EncSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int item = blockIdx.x;
  if (item == 0) {  // the step's bookkeeping words (read only by later kernels of the stream)
    if (tid < FIN_CNT_WORDS) fin_cnt[tid] = 0u;   // train_final_kernel's arrival counters
    if (tid == 0 && step_ctr) step_ctr[0] += 1;   // the Adam step of this train step
  }
  // this step's transposed-conv2 fragments (conv_bwd's da1 A operand, one
  // coalesced 256-B row per wave load): W2B[kk][s][lane] = W2[2s + (lane >> 5)][lane & 31][kk]
  if constexpr ((ENC_ABL & 4) == 0)
  for (int e = item * 256 + tid; e < W2B_FRAG; e += gridDim.x * 256) {
    const int kk = e >> 11, sl = e & 2047, st = sl >> 6, l = sl & 63;
    w2b[e] = w2[((2 * st + (l >> 5)) * C1 + (l & 31)) * 3 + kk];
  }
  if ((ENC_ABL & 4) == 0 && wt) {  // this step's k-major copies of the dense weights (the head's forward reads them)
    const int P = wd.param_dim, K0 = P + 2 * H;
    for (int e = item * 256 + tid; e < WT_FLOATS; e += gridDim.x * 256) {
      float v;
      if (e < WT_WT) {
        v = wd.enc6_w[(e & (H - 1)) * C2 + (e >> 7)];
      } else if (e < WT_W0) {
        const int i = e - WT_WT;
        v = wd.time_w[(i & (H - 1)) * H + (i >> 7)];
      } else if (e < WT_W2) {
        const int i = e - WT_W0, k = i >> 7;
        v = k < K0 ? wd.mlp0_w[(size_t)(i & (H - 1)) * K0 + k] : 0.f;
      } else if (e < WT_W0B) {
        const int i = e - WT_W2, o = i & (PMAX - 1);
        v = o < P ? wd.mlp2_w[o * H + (i >> 5)] : 0.f;
      } else if (e < WT_W5) {
        const int i = e - WT_W0B;
        v = wd.mlp0_w[(size_t)(i >> 8) * K0 + P + (i & 255)];
      } else {
        const int i = e - WT_W5, o = i >> 7;
        v = o < P ? wd.mlp2_w[i] : 0.f;
      }
      wt[e] = v;
    }
  }
  const int b = item / S, strip = item - b * S;
  const int j0 = strip * J;

  // the conv weights through LDS (coalesced float4 loads; the fragment reads
  // below are one ds_read_b32 each): W1 (32,42) and W2 (64,96), odd row pitches
  __shared__ float w1s[C1][K1 + 1];
  __shared__ float w2s[C2][K2 + 1];
  if constexpr ((ENC_ABL & 8) == 0) {
    float4 v2[6], v1[2];
#pragma unroll
    for (int k = 0; k < 6; ++k) v2[k] = reinterpret_cast<const float4*>(w2)[tid + 256 * k];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + 256 * k;
      v1[k] = i < C1 * K1 / 4 ? reinterpret_cast<const float4*>(w1)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int e = 4 * (tid + 256 * k), o = e / K2, c = e - o * K2;
      w2s[o][c] = v2[k].x; w2s[o][c + 1] = v2[k].y; w2s[o][c + 2] = v2[k].z; w2s[o][c + 3] = v2[k].w;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = 4 * (tid + 256 * k);
      if (e < C1 * K1) {
        const float vv[4] = {v1[k].x, v1[k].y, v1[k].z, v1[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) w1s[(e + j) / K1][(e + j) % K1] = vv[j];
      }
    }
  }
  stage_cond_f32(sm.X, cond + (size_t)b * CIN * L, L, 4 * j0 - 3, tid);
  __syncthreads();
  // conv1 fragment s of lane (o = l32, h): W1[o][c = s/3 + 7h][s % 3], contiguous in s
  float wa[STEPS1];
#pragma unroll
  for (int s = 0; s < STEPS1; ++s) wa[s] = w1s[l32][21 * h + s];

  {  // conv1 + bias + ReLU -> E / O (aliases X)
    const int par = wave >> 1, mt = wave & 1;
    const int m = mt * 32 + l32;
    f32x16 acc = {};
    const float* xb = &sm.X[0][0][0] + 7 * h * XS + m;
    if (par == 0) conv1_tile<0>(acc, wa, xb);
    else conv1_tile<1>(acc, wa, xb);
    __syncthreads();
    if (tid < C1) sm.E[tid][64] = 0.f;
    float* dst = par ? &sm.O[0][0] : &sm.E[0][0];
    const int i = 2 * j0 - 1 + 2 * m + par;
    const bool valid = (i >= 0) && (i < L1);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = (r & 3) + 8 * (r >> 2) + 4 * h;
      const float v = fmaxf(acc[r] + b1[o], 0.f);
      dst[o * HS + m] = valid ? v : 0.f;
    }
  }
  __syncthreads();
  if constexpr ((ENC_ABL & 1) == 0) {  // the strip's conv1 images -> a1s: 1,024 float4 rows, 4 per thread
    float4* dst = reinterpret_cast<float4*>(a1s + (size_t)item * A1S_FLOATS);
    const float* img = &sm.E[0][0];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = tid + 256 * k;
      const int plane = idx >> 9, c = (idx >> 4) & 31, m4 = idx & 15;
      dst[idx] = *reinterpret_cast<const float4*>(img + (plane * C1 + c) * HS + 4 * m4);
    }
  }
  {  // conv2 + bias + ReLU + masked column sums; the ReLU mask as ballot words
    const int qt = wave & 1, ot = wave >> 1;
    const int q = qt * 32 + l32, o = ot * 32 + l32;
    // conv2 fragment s of lane (o, h): W2[o][c = s/3 + 16h][s % 3], contiguous in s
    float w2r[STEPS2];
#pragma unroll
    for (int s = 0; s < STEPS2; ++s) w2r[s] = w2s[o][48 * h + s];
    const float* eb = &sm.E[0][0] + 16 * h * HS + q;
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < STEPS2; ++s) {
      const int cp = s / 3, kk = s % 3;
      const int off = (kk == 1 ? C1 * HS : 0) + cp * HS + (kk == 2 ? 1 : 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(eb[off], w2r[s], acc, 0, 0, 0);
    }
    const float bias = b2[o];
    float sum = 0.f;
    uint32_t word = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const bool valid = (qq < J) && (j0 + qq < L2);
      const float z = acc[r] + bias;
      sum += valid ? fmaxf(z, 0.f) : 0.f;
      // bit (h*32 + l32): row qq of this lane half, channel ot*32 + l32
      const uint64_t bal = __ballot(valid && z > 0.f);
      if (lane == r) word = (uint32_t)bal;
      if (lane == 16 + r) word = (uint32_t)(bal >> 32);
    }
    if ((ENC_ABL & 2) == 0 && lane < 32) {
      const int rr = lane & 15, hh = lane >> 4;
      const int qw = qt * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * hh;
      m2w[(size_t)item * M2W_WORDS + qw * 2 + ot] = word;
    }
    sum += __shfl_xor(sum, 32);
    if (h == 0) sm.red[qt][o] = sum;
  }
  __syncthreads();
  if (tid < C2) partial[(size_t)item * C2 + tid] = sm.red[0][tid] + sm.red[1][tid];
}

// ---------------------------------------------------------------------------
// head forward / backward (one 1024-thread block per member)
// Every layer is split-k: thread (q, j) sums k in group q's range for output
// j, the groups' partials are added in q order through LDS, so no dependent
// chain is longer than 64 loads.  Forward layers y = W x read the k-major
// copies WT[k][j] the encoder kernel wrote this step (coalesced across j);
// backward layers y = W^T x read W itself (row j of W is contiguous in the
// output index).
// ---------------------------------------------------------------------------
constexpr int HT = 1024;  // head block threads
#ifndef HEAD_ABL
#define HEAD_ABL 0  // diagnostic variants only: bit 0 no sin/cos, bit 1 no V stores, bit 2 no weight loads
#endif
#ifdef HEAD_STAMPS   // diagnostic build only: phase times of block 0 (tools/train_ref_probe.py)
__device__ unsigned long long g_hstamp[64];
#define HSTAMP(i) \
  do { if (blockIdx.x == 0 && threadIdx.x == 0) g_hstamp[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define HSTAMP(i) do { } while (0)
#endif
struct HeadSmem {
  float m[C2], e[H], c[H], te[H], hc[PMAX + 2 * H], h[H], eps[PMAX], nz[PMAX];
  float dout[PMAX], dz5[H], dhc[PMAX + 2 * H], dz3[H], red[PMAX];
  float part[HT];
  float4 part4[HT];
};

// part[tid] = sum over k in group q's range of W(k, j) * x[k], (q, j) = (tid / NOUT, tid % NOUT),
// W(k, j) = Wp[k * sk + j * sj]; j >= nout or an empty range gives 0
template <int NOUT>
__device__ __forceinline__ void splitk_part(const float* __restrict__ Wp, int sk, int sj, int K,
                                            const float* x, int nout, float* part, int tid) {
  constexpr int NQ = HT / NOUT;
  const int j = tid % NOUT, q = tid / NOUT;
  const int kc = (K + NQ - 1) / NQ, k0 = q * kc, k1 = min(K, k0 + kc);
  float acc = 0.f;
  if (j < nout) {
    const float* wp = Wp + (size_t)j * sj;
#pragma unroll 16
    for (int k = k0; k < k1; ++k) acc = fmaf(wp[(size_t)k * sk], x[k], acc);
  }
  part[tid] = acc;
}
// the same split with the weight slice loaded into registers ahead of time
// (the weights do not depend on the activations: a layer's loads are issued
// before the layers it waits for); the same fma order as splitk_part
template <int NOUT, int KCM>
struct SplitK {
  float w[KCM];
  int k0, k1;
  __device__ __forceinline__ void load(const float* __restrict__ Wp, int sk, int sj, int K, int nout,
                                       int tid) {
    constexpr int NQ = HT / NOUT;
    const int j = tid % NOUT, q = tid / NOUT;
    const int kc = (K + NQ - 1) / NQ;
    k0 = q * kc;
    k1 = min(K, k0 + kc);
    if (j >= nout) k1 = k0;
    const float* wp = Wp + (size_t)(j < nout ? j : 0) * sj;
#pragma unroll
    for (int i = 0; i < KCM; ++i) {
      const int k = k0 + i;
      if constexpr ((HEAD_ABL & 4) != 0) w[i] = k < k1 ? 1e-3f * (float)(k + j) : 0.f;
      else w[i] = k < k1 ? wp[(size_t)k * sk] : 0.f;
    }
  }
  __device__ __forceinline__ void part(const float* x, float* part, int tid) const {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < KCM; ++i)
      if (k0 + i < k1) acc = fmaf(w[i], x[k0 + i], acc);
    part[tid] = acc;
  }
};
// float4 form: thread (q, j4) owns outputs 4 j4 .. 4 j4 + 3 and the k range of
// group q (NQ groups, NOUT / 4 * NQ <= HT threads active); the weights are
// rows W[k][0 .. NOUT) with a 16-B aligned pitch sk, loaded ahead as float4s
// (a quarter of the load instructions of the scalar form); partials to part4
template <int NOUT, int NQ, int KCM>
struct SplitK4 {
  static_assert(NOUT / 4 * NQ <= HT, "threads");
  float4 w[KCM];
  int k0, k1, kb;
  // every load unconditional: the KCM rows from kb = min(k0, K - KCM) (rows
  // outside [k0, k1) are never read by part(); idle threads load the last
  // rows at one common address) -- no select on a loaded value, so nothing
  // waits for the loads before their use, and one base address per slice
  // (R >= KCM rows of Wp are readable; R >= K)
  __device__ __forceinline__ void load(const float* __restrict__ Wp, int sk, int K, int R, int tid) {
    constexpr int NJ = NOUT / 4;
    const int j4 = tid % NJ, q = tid / NJ;
    const int kc = (K + NQ - 1) / NQ;
    k0 = q * kc;
    k1 = q < NQ ? min(K, k0 + kc) : k0;
    kb = min(k0, R - KCM);
    const float* wp = Wp + (q < NQ ? 4 * j4 : 0) + (size_t)kb * sk;
#pragma unroll
    for (int i = 0; i < KCM; ++i) w[i] = *reinterpret_cast<const float4*>(wp + (size_t)i * sk);
  }
  __device__ __forceinline__ void part(const float* x, float4* part4, int tid) const {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < KCM; ++i) {
      const int k = kb + i;
      if (k >= k0 && k < k1) {
        const float xv = x[k];
        acc.x = fmaf(w[i].x, xv, acc.x);
        acc.y = fmaf(w[i].y, xv, acc.y);
        acc.z = fmaf(w[i].z, xv, acc.z);
        acc.w = fmaf(w[i].w, xv, acc.w);
      }
    }
    if (tid < NOUT / 4 * NQ) part4[tid] = acc;
  }
  // output j: the NQ group partials in group order
  __device__ __forceinline__ static float sum(const float4* part4, int j) {
    constexpr int NJ = NOUT / 4;
    const float* p = reinterpret_cast<const float*>(part4) + 4 * (j >> 2) + (j & 3);
    float s = p[0];
#pragma unroll
    for (int q = 1; q < NQ; ++q) s += p[4 * NJ * q];
    return s;
  }
};
// the NQ group partials of output j, in group order
template <int NOUT>
__device__ __forceinline__ float splitk_sum(const float* part, int j) {
  constexpr int NQ = HT / NOUT;
  float s = part[j];
#pragma unroll
  for (int q = 1; q < NQ; ++q) s += part[q * NOUT + j];
  return s;
}

struct HeadRng {  // the train step's own draws (TrainPlan): t ~ U{0..T-1}, noise ~ N(0,1)
  uint64_t seed;
  const int* step;  // device step counter (already advanced for this step)
  int T;
  int64_t* t_out;   // (B) the drawn t
  float* noise_out; // (B, P) the drawn noise
};
constexpr uint32_t RNG_TAG_T = 0x7A11u, RNG_TAG_NOISE = 0x7A12u;

// the backward layers' weight slices (W itself: rows contiguous in the output index)
struct HeadBwdW {
  SplitK4<H, 8, PMAX / 8> w5;      // dz5: W2 rows (o), 128 columns (the zero-padded copy)
  SplitK4<2 * H, 16, H / 16> w0;   // dhcat: W0B rows (j), 256 columns
  SplitK4<C2, 16, H / 16> w3;      // g: W3 rows (j), 64 columns
};

template <bool PRE>
__device__ __forceinline__ void head_forward(
    const ertd_weights& w, const float* __restrict__ wt, const float* __restrict__ x_in,
    const float* __restrict__ x0, const float* __restrict__ noise,
    const float* __restrict__ alpha_bar, const int64_t* __restrict__ t_vec,
    const float* __restrict__ freq, const float* __restrict__ partial, int S, int L2,
    float* __restrict__ V, float* __restrict__ eps_out, HeadRng rng, HeadSmem& s, int b,
    int tid, HeadBwdW& bw) {
  HSTAMP(0);
  const int P = w.param_dim;
  // the pool partials first (the first barrier waits for these loads only):
  // strips k = q, q + 16, ... of channel c summed per group q, the groups in order
  const int pc = tid & 63, pq = tid >> 6;
  float pv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = pq + (HT / 64) * u;
    pv[u] = 0.f;
    if (k < S) pv[u] = partial[((size_t)b * S + k) * C2 + pc];
  }
  // this member's t, known to every thread (no LDS round trip before the
  // loads that depend on it)
  int tme;
  if (rng.step) {  // Philox keyed (seed, member, step): independent of the grid and of the schedule
    const uint32_t st = (uint32_t)*rng.step;
    const u32x4 r = philox4x32_10(u32x4{0u, (uint32_t)b, st, RNG_TAG_T}, (uint32_t)rng.seed,
                                  (uint32_t)(rng.seed >> 32));
    tme = (int)(((uint64_t)r.x * (uint64_t)rng.T) >> 32);
    if (tid == 0) rng.t_out[b] = tme;
    if (tid >= 64 && tid < 64 + P) {
      const int o = tid - 64;
      const float z = philox_normal(rng.seed, (uint32_t)b, st, RNG_TAG_NOISE, o);
      s.nz[o] = z;
      rng.noise_out[(size_t)b * P + o] = z;
    }
  } else {
    tme = (int)t_vec[b];
    if (tid >= 64 && tid < 64 + P && noise) s.nz[tid - 64] = noise[(size_t)b * P + tid - 64];
  }
  // the loads of the later phases that need no activation, issued now
  float ab = 0.f, x0v = 0.f, frq = 0.f, bce = 0.f, bh = 0.f, be = 0.f;
  if (tid < P) {
    if (x_in) x0v = x_in[(size_t)b * P + tid];
    else {
      ab = alpha_bar[tme];
      x0v = x0[(size_t)b * P + tid];
    }
    be = w.mlp2_b[tid];
  }
  if (tid >= 256 && tid < 256 + H) frq = freq[(tid - 256) & 63];
  if (tid < 2 * H) bce = tid < H ? w.enc6_b[tid] : w.time_b[tid - H];
  if (tid < H) bh = w.mlp0_b[tid];
  // every forward layer's weight slice into registers now (k-major copies)
  const int K0 = P + 2 * H;
  // cond_emb (j4 < 32: outputs 0-127, K 64) and t_emb (j4 >= 32: 128-255, K 128) in one split:
  // 16 groups of 4 / 8 k each
  SplitK4<256, 16, 8> wce;
  {
    const bool ce = (tid & 63) < 32;
    wce.load(ce ? wt + WT_W3 : wt + WT_WT - H, H, ce ? C2 : H, ce ? C2 : H, tid);
  }
  SplitK4<128, 32, (PMAX + 2 * H + 31) / 32> wh;
  wh.load(wt + WT_W0, H, K0, K0, tid);
  {  // pool: the group sums (strips past 4 * 16: a plain loop)
    float acc = pv[0];
#pragma unroll
    for (int u = 1; u < 4; ++u) acc += pv[u];
    for (int k = pq + 4 * (HT / 64); k < S; k += HT / 64) acc += partial[((size_t)b * S + k) * C2 + pc];
    s.part[tid] = acc;
  }
  __syncthreads(); HSTAMP(1);
  if (tid < C2) {
    float acc = s.part[tid];
#pragma unroll
    for (int q = 1; q < HT / 64; ++q) acc += s.part[q * 64 + tid];
    s.m[tid] = acc / (float)L2;
  }
  if (tid < P) {
    float xv = x0v;
    if (!x_in) {  // q_sample (:97-99): one rounding per op
      const float sa = sqrtf(ab), sb = sqrtf(1.0f - ab);
      xv = sa * x0v + sb * s.nz[tid];
    }
    s.hc[tid] = xv;
  } else if (tid >= 256 && tid < 256 + H) {
    const int k = tid - 256;
    const float a = (float)tme * frq;
    if constexpr ((HEAD_ABL & 1) != 0) s.e[k] = a * 1e-3f;
    else s.e[k] = k < 64 ? sinf(a) : cosf(a);
  }
  __syncthreads(); HSTAMP(2);
  // cond_emb = relu(W3 m + b3) (outputs 0-127), t_emb = relu(Wt e + bt) (128-255)
  wce.part((tid & 63) < 32 ? s.m : s.e, s.part4, tid);
  // the later layers' slices into the registers wce leaves (each load lands
  // during the phases before its use; a barrier waits for LDS only)
  SplitK4<PMAX, 32, H / 32> we;
  we.load(wt + WT_W2, PMAX, H, H, tid);
  if constexpr (PRE) bw.w5.load(wt + WT_W5, H, P, PMAX, tid);
  __syncthreads(); HSTAMP(3);
  if (tid < 2 * H) {
    const float y = SplitK4<256, 16, 8>::sum(s.part4, tid);
    if (tid < H) {
      s.c[tid] = fmaxf(y + bce, 0.f);
      s.hc[P + H + tid] = s.c[tid];
    } else {
      const int j = tid - H;
      s.te[j] = fmaxf(y + bce, 0.f);
      s.hc[P + j] = s.te[j];
    }
  }
  __syncthreads(); HSTAMP(4);
  wh.part(s.hc, s.part4, tid);   // h = relu(W0 hcat + b0)
  if constexpr (PRE) bw.w0.load(wt + WT_W0B, 2 * H, H, H, tid);
  __syncthreads(); HSTAMP(5);
  if (tid < H) s.h[tid] = fmaxf(SplitK4<128, 32, (PMAX + 2 * H + 31) / 32>::sum(s.part4, tid) + bh, 0.f);
  __syncthreads(); HSTAMP(6);
  we.part(s.h, s.part4, tid);    // eps = W2 h + b2
  if constexpr (PRE) bw.w3.load(w.enc6_w, C2, H, H, tid);
  __syncthreads(); HSTAMP(7);
  if (tid < P) {
    const float y = SplitK4<PMAX, 32, H / 32>::sum(s.part4, tid) + be;
    s.eps[tid] = y;
    V[TV_EPS + tid] = y;
    if (eps_out) eps_out[(size_t)b * P + tid] = y;
  }
  if constexpr ((HEAD_ABL & 2) != 0) return;
  for (int i = tid; i < K0; i += HT) V[TV_HCAT + i] = s.hc[i];
  if (tid >= 512 && tid < 512 + H) {
    V[TV_E + tid - 512] = s.e[tid - 512];
    V[TV_H + tid - 512] = s.h[tid - 512];
  }
  if (tid >= 768 && tid < 768 + C2) V[TV_M + tid - 768] = s.m[tid - 768];
}

//   dout: given (autograd) or MSE: (pred - noise) * (2/(B*P))   (mse_loss backward)
// eps_v / h_v / hcat_v / nz_v: the forward's prediction, relu(z5), [x | t_emb |
// cond_emb] and noise (LDS in the fused kernel; the saved row / the noise input otherwise)
__device__ __forceinline__ void head_backward(
    const ertd_weights& w, const float* __restrict__ wt, const float* __restrict__ dout_in,
    const float* nz_v, float two_over_n,
    int L2, float* __restrict__ V, float* __restrict__ dx_out, const float* eps_v, const float* h_v,
    const float* hcat_v, HeadSmem& s, int b, int tid, HeadBwdW& bw, bool loaded) {
  const int P = w.param_dim;
  const int K0 = P + 2 * H;
  // every backward layer's weight slice into registers (the fused step issued
  // them during the forward)
  if (!loaded) {
    bw.w5.load(wt + WT_W5, H, P, PMAX, tid);
    bw.w0.load(wt + WT_W0B, 2 * H, H, H, tid);
    bw.w3.load(w.enc6_w, C2, H, H, tid);
  }
  const auto& w5 = bw.w5;
  const auto& w0 = bw.w0;
  const auto& w3 = bw.w3;
  if (tid < PMAX) {
    float d = 0.f, sq = 0.f;
    if (tid < P) {
      if (dout_in) {
        d = dout_in[(size_t)b * P + tid];
      } else {
        const float diff = eps_v[tid] - nz_v[tid];
        sq = diff * diff;
        d = diff * two_over_n;
      }
    }
    s.dout[tid] = d;
    s.red[tid] = sq;
    V[TV_DOUT + tid] = d;
  }
  __syncthreads(); HSTAMP(8);
  if (tid == 0) {
    float acc = 0.f;
    for (int o = 0; o < P; ++o) acc += s.red[o];
    V[TV_SQ] = acc;
  }
  w5.part(s.dout, s.part4, tid);   // dz5 = (W2^T dout) * [h > 0]
  __syncthreads(); HSTAMP(9);
  if (tid < H) {
    const float d = h_v[tid] > 0.f ? SplitK4<H, 8, PMAX / 8>::sum(s.part4, tid) : 0.f;
    s.dz5[tid] = d;
    V[TV_DZ5 + tid] = d;
  }
  __syncthreads(); HSTAMP(10);
  // dhcat[P + k] = (W0^T dz5)[P + k] for the t_emb / cond_emb columns
  w0.part(s.dz5, s.part4, tid);
  __syncthreads(); HSTAMP(11);
  if (tid < 2 * H) s.dhc[tid] = SplitK4<2 * H, 16, H / 16>::sum(s.part4, tid);
  if (dx_out) {  // dx = W0x^T dz5 (autograd w.r.t. the model input)
    __syncthreads(); HSTAMP(12);
    splitk_part<32>(w.mlp0_w, K0, 1, H, s.dz5, P, s.part, tid);
    __syncthreads(); HSTAMP(13);
    if (tid < P) dx_out[(size_t)b * P + tid] = splitk_sum<32>(s.part, tid);
  }
  __syncthreads(); HSTAMP(14);
  if (tid < H) {
    const float te = hcat_v[P + tid];
    V[TV_DZ4 + tid] = te > 0.f ? s.dhc[tid] : 0.f;
  } else if (tid < 2 * H) {
    const int j = tid - H;
    const float c = hcat_v[P + H + j];
    const float d = c > 0.f ? s.dhc[tid] : 0.f;
    s.dz3[j] = d;
    V[TV_DZ3 + j] = d;
  }
  __syncthreads(); HSTAMP(15);
  w3.part(s.dz3, s.part4, tid);   // g = (W3^T dz3) / L2
  __syncthreads(); HSTAMP(16);
  if (tid < C2) V[TV_G + tid] = SplitK4<C2, 16, H / 16>::sum(s.part4, tid) / (float)L2;
}

// ---------------------------------------------------------------------------
// conv backward: two 256-thread workgroups per (member, strip of J conv2
// outputs), one launch -- the first B*S blocks the dz1 chain, the next B*S the
// rest of dW2 (the two touch disjoint columns of the strip's gradient row):
//   chain, phase A: dz2 = g * mask -> da1 (transposed conv2) -> dz1 = da1 * [a1 > 0]
//            (waves 0-1: even conv1 positions, 1 tap + one dW2 tile each;
//            waves 2-3: odd positions, 2 taps) -- 64 MFMAs per wave
//   chain, phase B: dW1 = dz1 x cond (+ db1 from a ones column of the padded N), 32 per wave
//   dW2 blocks: dz2 -> dW2 tiles 2-5 (one per wave, 32 MFMAs) and db2
// Every wave of a chain block runs 96 MFMAs (128 before the split, in one
// block per item: 608 blocks for 768 slots at B = 32 left the CUs that got
// three blocks as the critical path); the short dW2 blocks fill the gaps.
// LDS: phase A's dz2 / a1 images are dead in phase B, where the cond image and
// the dW1 halves take their place: 51.6 KB -> 3 workgroups per CU.
// ---------------------------------------------------------------------------
#ifndef CBW_ABL
#define CBW_ABL 0  // diagnostic variants only (tools/cbw_abl.sh): bit mask of skipped phases (16: no dW2 blocks)
#endif
constexpr int DZ2P = 65;   // dz2 row pitch (column reads conflict-free)
constexpr int DZ1P = 129;  // dz1 row pitch
struct ConvBwdSmem {
  union {
    float DZ2[C2][DZ2P];     // phase A: dz2[o][q'], q' = j - j0 in [0, 65)
    float X[4][CIN][XS];     // phase B: cond image (the forward's 4-phase layout)
  };
  union {
    struct {
      float AE[C1][HS];      // phase A: a1 at p = 2m   (i = 2*j0 - 1 + p)
      float AO[C1][HS];      //          a1 at p = 2m+1
    };
    float red[4][32][33];    // phase B: the dW1 r-halves
  };
  float DZ1[C1][DZ1P];       // dz1[c][r], r = i - 2*j0 in [0, 128)
  float db2p[4][C2];         // db2 partial sums of the four q' classes
};

// acc += sum_s A(s) x B(s) over N k-steps of v_mfma_f32_32x32x2_f32, the
// operands of step s + AHEAD fetched (LDS reads) before step s's MFMA: a
// read's latency hides behind AHEAD MFMAs instead of stalling the next one
template <int N, int AHEAD, class FA, class FB>
__device__ __forceinline__ void mfma_pipe(f32x16& acc, FA fa, FB fb) {
  float ra[AHEAD], rb[AHEAD];
#pragma unroll
  for (int i = 0; i < AHEAD; ++i) {
    ra[i] = fa(i);
    rb[i] = fb(i);
  }
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const float a = ra[s % AHEAD], b = rb[s % AHEAD];
    if (s + AHEAD < N) {
      ra[s % AHEAD] = fa(s + AHEAD);
      rb[s % AHEAD] = fb(s + AHEAD);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    // keep the order: this step's reads (for s + AHEAD), then its MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
  }
}
#ifndef CBW_ORDER
#define CBW_ORDER 0   // 1: chain items two per CU first (A/B: 21.8 vs 19.5 us, slower)
#endif
#ifndef CBW_AHEAD
#define CBW_AHEAD 6
#endif
#ifndef CBW_PB16
#define CBW_PB16 1   // phase B: 32x32 tile + 16x16x4 edge tiles (0: two padded 32x32 tiles)
#endif
using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ void store_tile_rows(float (*red)[33], const f32x16& acc, int h, int l32) {
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(r & 3) + 8 * (r >> 2) + 4 * h][l32] = acc[r];
}

// dW2 tile tt = (ot, nt): rows o = 32 ot + ., columns n = c*3 + kk = 32 nt + .
//   dW2[o][n] += sum_{q < J} dz2[o][q] * a1[c][p = 2q + kk]
__device__ __forceinline__ void dw2_tile(const ConvBwdSmem& sm, int tt, int h, int l32,
                                         float* __restrict__ G) {
  const int ot = tt / 3, nt = tt - 3 * (tt / 3);
  const int n = nt * 32 + l32, c = n / 3, kk = n - 3 * (n / 3);
  const float* ab = kk == 1 ? &sm.AO[c][h] : &sm.AE[c][h + (kk == 2 ? 1 : 0)];
  const float* zb = &sm.DZ2[ot * 32 + l32][h];
  f32x16 acc = {};
  mfma_pipe<32, CBW_AHEAD>(acc, [&](int s) { return zb[2 * s]; },
                           // q' = 63 is the halo: excluded
                           [&](int s) { return (2 * s + h < J) ? ab[2 * s] : 0.f; });
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int o = ot * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    G[NG_W2 + o * K2 + n] = acc[r];
  }
}

// the a1 images (the forward's float4 rows) and dz2 = g * mask (+ the db2
// partial sums of the four q' classes) into LDS
template <bool ONES = false, class SM>
__device__ __forceinline__ void conv_bwd_images(SM& sm, const float* __restrict__ a1s,
                                                const uint32_t* __restrict__ m2w,
                                                const float* __restrict__ g, int g_stride, int b,
                                                int item, int strip, int S, int tid) {
  {
    const float4* src = reinterpret_cast<const float4*>(a1s + (size_t)item * A1S_FLOATS);
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = src[tid + 256 * k];
    float* img = &sm.AE[0][0];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = tid + 256 * k;
      const int plane = idx >> 9, c = (idx >> 4) & 31, m4 = idx & 15;
      *reinterpret_cast<float4*>(img + (plane * C1 + c) * HS + 4 * m4) = v[k];
    }
  }
  {
    const int o = tid & 63, qb = tid >> 6;
    const float go = ONES ? 1.f : g[(size_t)b * g_stride + o];
    const uint32_t* mw = m2w + (size_t)item * M2W_WORDS + (o >> 5);
    const bool next = strip + 1 < S;
    uint32_t wd[17];  // every word loaded up front (unconditional, clamped), then used
#pragma unroll
    for (int k = 0; k < 17; ++k) {
      const int q = qb + 4 * k;
      wd[k] = mw[q < J ? q * 2 : (q == J && next ? M2W_WORDS : 0)];  // q = J: the next strip's q = 0
    }
    float dsum = 0.f;
#pragma unroll
    for (int k = 0; k < 17; ++k) {
      const int q = qb + 4 * k;
      if (q < DZ2P) {
        const bool on = (q < J || (q == J && next)) && ((wd[k] >> (o & 31)) & 1u);
        const float v = on ? go : 0.f;
        sm.DZ2[o][q] = v;
        if (q < J) dsum += v;
      }
    }
    sm.db2p[qb][o] = dsum;
  }
}

// W2: the dW2 work too (dW2 blocks + two tiles per chain block, rows of NG);
// else the chain alone, rows [dW1 | db1] of NG1 (the reference train step)
template <bool W2>
__global__ __launch_bounds__(256, 3) void conv_bwd_kernel(
    const float* __restrict__ w2b, const float* __restrict__ cond, const float* __restrict__ a1s,
    const uint32_t* __restrict__ m2w, const float* __restrict__ g, int g_stride, int L, int L1,
    int L2, int S, float* __restrict__ gpart, int c1, int c2) {
  __shared__ __attribute__((aligned(16))) ConvBwdSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  // dispatch order: all chain blocks, then all dW2 blocks (CBW_ORDER = 1: chain
  // items [0, c1), dW2 items [0, c2), the remaining chain items, the remaining
  // dW2 items, c1 = 2 and c2 = 1 per CU -- measured slower)
  constexpr bool WB = W2 && (CBW_ABL & 16) == 0;   // dW2 blocks in the grid
  const int nit = WB ? (int)gridDim.x / 2 : (int)gridDim.x, bi = (int)blockIdx.x;
  const bool w2blk = !WB ? false : CBW_ORDER ? (bi >= c1 && bi < c1 + c2) || bi >= nit + c2 : bi >= nit;
  const int item = !CBW_ORDER ? (w2blk ? bi - nit : bi)
                 : bi < c1 ? bi : bi < c1 + c2 ? bi - c1 : bi < nit + c2 ? bi - c2 : bi - nit;
  const int b = item / S, strip = item - b * S;
  const int j0 = strip * J;
  float* G = gpart + (size_t)item * (W2 ? NG : NG1);
  constexpr int GB1 = W2 ? NG_B1 : C1 * K1;   // db1 offset in the row

  if (w2blk) {
    conv_bwd_images(sm, a1s, m2w, g, g_stride, b, item, strip, S, tid);
    __syncthreads();
    if constexpr ((CBW_ABL & 2) == 0) dw2_tile(sm, 2 + wave, h, l32, G);
    if (tid < C2) G[NG_B2 + tid] = sm.db2p[0][tid] + sm.db2p[1][tid] + sm.db2p[2][tid] + sm.db2p[3][tid];
    return;
  }

  // ---- transposed-conv2 fragments (the da1 A operand) first, into registers:
  //   W2B[kk][s][lane] = W2[o = 2s + h][c = l32][kk]; even waves tap 1, odd waves taps 0 and 2
  const bool oddw = wave >= 2;
  float wt0[32], wt1[32];
  {
    const float* base = w2b + lane;
    const int k0 = oddw ? 0 : 1;
#pragma unroll
    for (int s = 0; s < 32; ++s) wt0[s] = base[(k0 * 32 + s) * 64];
#pragma unroll
    for (int s = 0; s < 32; ++s) wt1[s] = oddw ? base[(2 * 32 + s) * 64] : 0.f;
  }
  // ---- the cond strip (phase B's image), loaded now, stored after phase A
  const float* cb = cond + (size_t)b * CIN * L;
  const int pos = 4 * j0 - 3 + tid;
  const bool cin = pos >= 0 && pos < L;
  float cv[CIN];
  {
    const int pc = pos < 0 ? 0 : (pos >= L ? L - 1 : pos);
#pragma unroll
    for (int c = 0; c < CIN; ++c) cv[c] = cb[(size_t)c * L + pc];
  }
  const int tc = tid >> 2, tu = 256 + (tid & 3);
  const int pt = 4 * j0 - 3 + tu;
  float cvt = 0.f;
  if (tid < CIN * 4) cvt = cb[(size_t)tc * L + (pt < 0 ? 0 : (pt >= L ? L - 1 : pt))];

  conv_bwd_images(sm, a1s, m2w, g, g_stride, b, item, strip, S, tid);
  __syncthreads();

  // ---- phase A
  {
    const int mt = wave & 1;
    const int mcol = mt * 32 + l32;
    const float* db = &sm.DZ2[0][0] + h * DZ2P + mcol;
    f32x16 acc = {};
    if ((CBW_ABL & 1) != 0) {
      for (int k = 0; k < 16; ++k) acc[k] = db[k] + wt0[k] + wt1[k];
    } else if (!oddw) {
      // r = 2m: da1 = sum_o W2[o][c][1] dz2[o][m]
      mfma_pipe<32, CBW_AHEAD>(acc, [&](int s) { return wt0[s]; }, [&](int s) { return db[2 * s * DZ2P]; });
    } else {
      // r = 2m+1: da1 = sum_o W2[o][c][0] dz2[o][m+1] + W2[o][c][2] dz2[o][m]
      mfma_pipe<32, CBW_AHEAD>(acc, [&](int s) { return wt0[s]; },
                               [&](int s) { return db[2 * s * DZ2P + 1]; });
      mfma_pipe<32, CBW_AHEAD>(acc, [&](int s) { return wt1[s]; }, [&](int s) { return db[2 * s * DZ2P]; });
    }
    const int odd = oddw ? 1 : 0;
    const int r = 2 * mcol + odd;
    const bool owned = r < 2 * J && 2 * j0 + r < L1;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int c = (k & 3) + 8 * (k >> 2) + 4 * h;
      const float act = odd ? sm.AE[c][mcol + 1] : sm.AO[c][mcol];  // a1 at p = r + 1
      sm.DZ1[c][r] = (owned && act > 0.f) ? acc[k] : 0.f;
    }
  }
  if constexpr (W2 && (CBW_ABL & 2) == 0) {
    if (!oddw) dw2_tile(sm, wave, h, l32, G);   // tiles 0, 1 (2-5: the dW2 blocks)
  }
  __syncthreads();

  // ---- cond image into the dead dz2 region
#pragma unroll
  for (int c = 0; c < CIN; ++c) sm.X[tid & 3][c][tid >> 2] = cin ? cv[c] : 0.f;
  if (tid < CIN * 4) sm.X[tu & 3][tc][tu >> 2] = (pt >= 0 && pt < L) ? cvt : 0.f;
  __syncthreads();

  // ---- phase B: dW1[o][n = c*3+kk] = sum_r dz1[o][r] * cond[c][4*j0 + 2r - 1 + kk];
  //      column n = 42 (padding) multiplies by ones: db1[o] = sum_r dz1[o][r]
#if CBW_PB16
  // columns 0-31: one 32x32x2 tile, its 64 k-steps split 24/24/8/8 over the
  // four waves; columns 32-47 (the 10 remaining weights and the db1 column):
  // 16x16x4 tiles, rows 0-15 in wave 2, 16-31 in wave 3 (32 k-steps each, two
  // accumulators) -- 1536 MFMA cycles per wave instead of 2048 for a 64-wide
  // N padded to two 32x32 tiles
  f32x4 acc1 = {};
  {
    const int c = l32 / 3, kk = l32 - 3 * (l32 / 3);
    const int u0 = 2 * h + 2 + kk;  // u = 4s + u0 for r = 2s + h
    const int s0 = wave < 2 ? 24 * wave : 48 + 8 * (wave - 2);
    const float* xr = &sm.X[u0 & 3][c][u0 >> 2] + s0;
    const float* zr = &sm.DZ1[l32][h] + 2 * s0;
    f32x16 acc = {};
    if (wave < 2) {
      mfma_pipe<24, CBW_AHEAD>(acc, [&](int s) { return zr[2 * s]; }, [&](int s) { return xr[s]; });
    } else {
      mfma_pipe<8, CBW_AHEAD>(acc, [&](int s) { return zr[2 * s]; }, [&](int s) { return xr[s]; });
      // lane: row o = 16 (wave - 2) + q, column n = 32 + q, k: r = 64 half + 16 kq + s
      // (DZ1 reads conflict-free: bank = q + 16 kq + s)
      const int q = lane & 15, kq = lane >> 4;
      const int n1 = 32 + q;
      const bool nv = n1 < K1;
      const float pad = n1 == K1 ? 1.f : 0.f;
      const int cc = nv ? n1 / 3 : 0, k1 = nv ? n1 - 3 * (n1 / 3) : 0;
      // u = 2r + 2 + k1 = 128 half + 32 kq + 4 (s >> 1) + w, w = 2 + k1 + 2 (s & 1)
      const int w0 = 2 + k1, w1 = 4 + k1;
      const float* xe = &sm.X[w0 & 3][cc][8 * kq + (w0 >> 2)];
      const float* xo = &sm.X[w1 & 3][cc][8 * kq + (w1 >> 2)];
      const float* zq = &sm.DZ1[16 * (wave - 2) + q][16 * kq];
      f32x4 a0 = {}, a1 = {};
      float ra[4], rb[4];
      auto fa = [&](int t) { return zq[64 * (t >> 4) + (t & 15)]; };
      auto fb = [&](int t) {
        const int s = t & 15, off = 32 * (t >> 4) + (s >> 1);
        return nv ? ((s & 1) ? xo[off] : xe[off]) : pad;
      };
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ra[i] = fa(i);
        rb[i] = fb(i);
      }
#pragma unroll
      for (int t = 0; t < 32; ++t) {
        const float a = ra[t & 3], b = rb[t & 3];
        if (t + 4 < 32) {
          ra[t & 3] = fa(t + 4);
          rb[t & 3] = fb(t + 4);
        }
        if (t & 1) a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, a1, 0, 0, 0);
        else a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, a0, 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      acc1 = a0 + a1;
    }
    store_tile_rows(sm.red[wave], acc, h, l32);  // red aliases the dead a1 images
  }
  if (wave >= 2) {  // rows o = 16 (wave - 2) + 4 (lane >> 4) + i, column 32 + (lane & 15)
    const int n1 = 32 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 16 * (wave - 2) + 4 * (lane >> 4) + i;
      if (n1 < K1) G[NG_W1 + o * K1 + n1] = acc1[i];
      else if (n1 == K1) G[GB1 + o] = acc1[i];
    }
  }
  __syncthreads();
  for (int idx = tid; idx < C1 * 32; idx += 256) {  // the k-quarters combined in order
    const int o = idx >> 5, col = idx & 31;
    G[NG_W1 + o * K1 + col] = (sm.red[0][o][col] + sm.red[1][o][col]) + (sm.red[2][o][col] + sm.red[3][o][col]);
  }
#else
  {
    const int nt = wave & 1, rh = wave >> 1;
    const int n = nt * 32 + l32;
    const bool nvalid = n < K1;
    const float pad = n == K1 ? 1.f : 0.f;
    const int c = nvalid ? n / 3 : 0, kk = nvalid ? n - 3 * (n / 3) : 0;
    const int u0 = 2 * h + 2 + kk;  // u = 4s + u0 for r = 2s + h
    const float* xb = &sm.X[u0 & 3][c][u0 >> 2];
    const float* zb = &sm.DZ1[l32][h];
    f32x16 acc = {};
    if constexpr ((CBW_ABL & 4) != 0) {
      for (int k = 0; k < 16; ++k) acc[k] = zb[2 * k] + xb[k] + pad;
    } else {
      const float* zr = zb + 64 * rh;
      const float* xr = xb + 32 * rh;
      mfma_pipe<32, CBW_AHEAD>(acc, [&](int s) { return zr[2 * s]; },
                               [&](int s) { return nvalid ? xr[s] : pad; });
    }
    store_tile_rows(sm.red[wave], acc, h, l32);  // red aliases the dead a1 images
  }
  __syncthreads();
  if constexpr ((CBW_ABL & 8) != 0) {
    if (item >= 0x7fffffff) G[tid] = sm.red[0][0][tid & 31];
    return;
  }
  for (int idx = tid; idx < C1 * K1; idx += 256) {  // r-halves combined in order
    const int o = idx / K1, n = idx - o * K1;
    const int nt = n >> 5, col = n & 31;
    G[NG_W1 + idx] = sm.red[nt][o][col] + sm.red[2 + nt][o][col];
  }
  if (tid < C1) G[GB1 + tid] = sm.red[1][tid][K1 - 32] + sm.red[3][tid][K1 - 32];
#endif
}

// k-half kh of dW2 tile tt (k-steps 16 kh .. 16 kh + 15 of dw2_tile), added to acc
template <class SM>
__device__ __forceinline__ void dw2_half(const SM& sm, int tt, int kh, int h, int l32,
                                         f32x16& acc) {
  const int ot = tt / 3, nt = tt - 3 * (tt / 3);
  const int n = nt * 32 + l32, c = n / 3, kk = n - 3 * (n / 3);
  const float* ab = (kk == 1 ? &sm.AO[c][h] : &sm.AE[c][h + (kk == 2 ? 1 : 0)]) + 32 * kh;
  const float* zb = &sm.DZ2[ot * 32 + l32][h] + 32 * kh;
  const int qb = 32 * kh + h;
  mfma_pipe<16, CBW_AHEAD>(acc, [&](int s) { return zb[2 * s]; },
                           // q' = 63 is the halo: excluded
                           [&](int s) { return (qb + 2 * s < J) ? ab[2 * s] : 0.f; });
}

// M = dW2 / g of a group of W2M_NS strips of one member (dz2 = mask: the same
// images and tiles as the dW2 blocks with g = 1), and the mask counts (db2 /
// g).  Three slots of 4 waves take one strip each; a slot's 6 tiles x 2
// k-halves: wave w owns half tiles w, w + 4, w + 8 (tile hv / 2, half hv % 2).
// The odd waves' halves go to their partner through LDS, then slots 1 and 2
// to slot 0, in a fixed order.  Reads only the forward's a1s / m2w: workgroups
// of the head kernel's launch run it beside the per-member head blocks.
struct W2mSmem {
  float AE[C1][HS];
  float AO[C1][HS];
  float DZ2[C2][DZ2P];
  float db2p[4][C2];
};
static_assert(W2M_NS == 3, "one slot per strip");
static_assert(sizeof(W2mSmem) >= (6 * 1024 + C2) * sizeof(float), "exchange buffer");
__device__ __forceinline__ void w2m_body(W2mSmem (&msm)[W2M_NS], const float* __restrict__ a1s,
                                         const uint32_t* __restrict__ m2w, int S,
                                         float* __restrict__ mrows, int mb, int tid) {
  const int slot = tid >> 8, t = tid & 255, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int ng = w2m_groups(S);
  const int b = mb / ng;
  const int st = (mb - b * ng) * W2M_NS + slot;   // this slot's strip
  const bool act = st < S;
  W2mSmem& sm = msm[slot];
  f32x16 acc[3] = {};
  float cnt = 0.f;
  if (act) conv_bwd_images<true>(sm, a1s, m2w, nullptr, 0, b, b * S + st, st, S, t);
  __syncthreads();
  if (act) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int hv = wave + 4 * u;
      dw2_half(sm, hv >> 1, hv & 1, h, l32, acc[u]);
    }
    if (t < C2) cnt = (sm.db2p[0][t] + sm.db2p[1][t]) + (sm.db2p[2][t] + sm.db2p[3][t]);
  }
  __syncthreads();
  float* xb = reinterpret_cast<float*>(&sm);   // the slot's dead images
  const int pair = wave >> 1;
  if (wave & 1) {
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) xb[(pair * 3 + u) * 1024 + r * 64 + lane] = acc[u][r];
  }
  __syncthreads();
  if ((wave & 1) == 0) {
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[u][r] += xb[(pair * 3 + u) * 1024 + r * 64 + lane];
  }
  __syncthreads();
  if (slot > 0) {
    if ((wave & 1) == 0) {
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int r = 0; r < 16; ++r) xb[(pair * 3 + u) * 1024 + r * 64 + lane] = acc[u][r];
    }
    if (t < C2) xb[6 * 1024 + t] = cnt;
  }
  __syncthreads();
  if (slot != 0) return;
  const float* x1 = reinterpret_cast<const float*>(&msm[1]);
  const float* x2 = reinterpret_cast<const float*>(&msm[2]);
  float* M = mrows + (size_t)mb * NG2;
  if ((wave & 1) == 0) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int tt = (wave + 4 * u) >> 1, ot = tt / 3, nt = tt - 3 * (tt / 3);
      const int n = nt * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = ot * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int xi = (pair * 3 + u) * 1024 + r * 64 + lane;
        M[o * K2 + n] = (acc[u][r] + x1[xi]) + x2[xi];
      }
    }
  }
  if (t < C2) M[C2 * K2 + t] = (cnt + x1[6 * 1024 + t]) + x2[6 * 1024 + t];
}

// MODE 1 / 2 with mw.mrows: workgroups B .. B + B * w2m_groups(S) - 1 of the
// launch run w2m_body (waves 0-11; the others leave at once) on the CUs the B
// head blocks leave idle
struct W2mArgs {
  const float* a1s;
  const uint32_t* m2w;
  float* mrows;   // null: head blocks only
  int nb;         // head blocks (B)
};
template <int MODE>
__global__ __launch_bounds__(HT) void train_head_kernel(
    ertd_weights w, const float* __restrict__ wt, const float* __restrict__ x_in,
    const float* __restrict__ x0, const float* __restrict__ noise,
    const float* __restrict__ alpha_bar, const int64_t* __restrict__ t_vec,
    const float* __restrict__ freq, const float* __restrict__ partial, int S, int L2,
    float* __restrict__ vec, float* __restrict__ eps_out, const float* __restrict__ dout_in,
    float two_over_n, float* __restrict__ dx_out, HeadRng rng, W2mArgs mw) {
  const int b = blockIdx.x, tid = threadIdx.x;
  if constexpr (MODE != 0) {
    if (mw.mrows && b >= mw.nb) {
      __shared__ __attribute__((aligned(16))) W2mSmem msm[W2M_NS];
      if (tid >= 256 * W2M_NS) return;
      w2m_body(msm, mw.a1s, mw.m2w, S, mw.mrows, b - mw.nb, tid);
      return;
    }
  }
  __shared__ HeadSmem s;
  float* V = vec + (size_t)b * TV;
  HeadBwdW bw;
  if constexpr (MODE != 1)
    head_forward<MODE == 2>(w, wt, x_in, x0, noise, alpha_bar, t_vec, freq, partial, S, L2, V, eps_out, rng,
                            s, b, tid, bw);
  if constexpr (MODE == 2) {
    __syncthreads(); HSTAMP(17);
    head_backward(w, wt, dout_in, s.nz, two_over_n, L2, V, dx_out, s.eps, s.h, s.hc, s, b, tid, bw, true);
  }
  if constexpr (MODE == 1) {
    head_backward(w, wt, dout_in, noise ? noise + (size_t)b * w.param_dim : nullptr, two_over_n, L2, V,
                  dx_out, V + TV_EPS, V + TV_H, V + TV_HCAT, s, b, tid, bw, false);
  }
}

// ---------------------------------------------------------------------------
// gradients (+ Adam): conv columns from the strip partial rows, dense layers
// from the saved member rows, the loss
// ---------------------------------------------------------------------------
struct AdamHyper {
  float one_minus_b1, b2, one_minus_b2, step_size_neg, bc2_sqrt, eps;
};
static_assert(sizeof(AdamHyper) == ADAM_TABLE_FLOATS * sizeof(float), "AdamHyper layout");

// torch.optim.Adam's single-tensor update (no weight decay / amsgrad), as torch
// forms it: exp_avg.lerp_(grad, 1-b1); exp_avg_sq.mul_(b2).addcmul_(grad, grad,
// 1-b2); denom = sqrt(exp_avg_sq) / sqrt(bc2) + eps; param.addcdiv_(exp_avg, denom, -lr/bc1)
__device__ __forceinline__ void adam_vals(float& p, float& m, float& v, float g, const AdamHyper& a) {
  m = m + a.one_minus_b1 * (g - m);
  v = v * a.b2;
  v = v + a.one_minus_b2 * g * g;
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p + a.step_size_neg * (m / denom);
}
__device__ __forceinline__ void adam_elem(float* __restrict__ p, float* __restrict__ m,
                                          float* __restrict__ v, int e, float g, const AdamHyper& a) {
  float pp = p[e], mm = m[e], vv = v[e];
  adam_vals(pp, mm, vv, g, a);
  p[e] = pp;
  m[e] = mm;
  v[e] = vv;
}

// Conv columns: a two-level fixed-order reduction of the (rows, NG) strip
// partial rows.  Block (cb, rb) sums rows [rb*rpb, (rb+1)*rpb) of 64 float4
// columns (wave w takes rows w, w+4, ...: one coalesced 1-KB row segment per
// load, all of a lane's loads in flight), writes its sum write-through (sc1)
// to fin[rb], drains, and arrives on the column block's counter; the last of
// the FIN_RB arrivals reads the FIN_RB sums (sc1 loads) in rb order, writes the
// gradient and applies Adam, and resets the counter (no fences: the hand-off
// form of MI355X_MICROARCH.md "Valid forms", row 1).

struct FinalArgs {
  const float* gpart;    // (rows, NG) strip partial rows
  int rows;
  float* fin;            // (FIN_RB, NG) row-block sums
  unsigned* cnt;         // (FIN_CNT_WORDS) arrival counters, 0 between launches
  const float* vec;      // (B, TV) saved member rows (dense part; null: conv part only)
  int B, P;
  float inv_n;
  float* grad[12];       // state_dict order; the conv part writes 0..3 only
  float* loss;           // null: no loss
  float* param[12];      // Adam: null = gradients only
  float* m[12];
  float* v[12];
  AdamHyper hyper;       // host-formed scalars, or (hyper_tab != null) the entry
  const float* hyper_tab;  //   of step *step_ctr: hyper_tab[(s - tab_first)], clamped
  const int* step_ctr;
  int tab_first, tab_len;
  int conv_off;          // diagnostic variants only (FIN_ABL): block index offset
  // split rows (the reference train step): gpart rows are [dW1 | db1] (NG1),
  // mpart's rows2 rows [M | counts] (NG2) of member row / ngrp, weighted by
  // that member's g = vec[TV_G ..]
  const float* mpart;
  int rows2, ngrp;
};

__device__ __forceinline__ AdamHyper fetch_hyper(const FinalArgs& a) {
  if (!a.hyper_tab) return a.hyper;
  int k = *a.step_ctr - a.tab_first;
  k = k < 0 ? 0 : (k >= a.tab_len ? a.tab_len - 1 : k);
  const float* t = a.hyper_tab + (size_t)k * ADAM_TABLE_FLOATS;
  return AdamHyper{t[0], t[1], t[2], t[3], t[4], t[5]};
}

__device__ __forceinline__ void st_wt(float* p, float v) {  // write-through (sc1) store
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {    // sc1 load (L2, not L1)
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}

// Split rows (the reference train step): one level.  Workgroup = 16 float4
// columns of one segment ([dW1 | db1] over the rows chain rows, or [M |
// counts] over the rows2 M rows weighted by their member's g); thread (rg,
// col) sums rows rg, rg + 16, ... (all of its loads in flight), the 16 row
// groups are added in order, and the same thread applies Adam.
constexpr int FS_COLS = 16;
constexpr int FS_NCB1 = (NG1 / 4 + FS_COLS - 1) / FS_COLS;   // 22
constexpr int FS_NCB2 = (NG2 / 4 + FS_COLS - 1) / FS_COLS;   // 97
constexpr int FS_NR = 40;                                      // rows per thread in flight
__device__ __forceinline__ void final_split_conv(const FinalArgs& a, const AdamHyper& hy, int cb, int tid,
                                                 float4 (*red)[FS_COLS]) {
  const bool seg2 = cb >= FS_NCB1;
  const int cl = tid & (FS_COLS - 1), rg = tid >> 4;
  const int col4 = (seg2 ? cb - FS_NCB1 : cb) * FS_COLS + cl;
  const int ncol4 = seg2 ? NG2 / 4 : NG1 / 4;
  const bool ok = col4 < ncol4;
  const int e0 = col4 * 4;
  int k, off;
  if (!seg2) {
    if (e0 < C1 * K1) { k = 0; off = e0; } else { k = 1; off = e0 - C1 * K1; }
  } else {
    if (e0 < C2 * K2) { k = 2; off = e0; } else { k = 3; off = e0 - C2 * K2; }
  }
  // Adam's operands of the column's 4 elements, prefetched by the row group 0 threads
  float pv[4] = {}, mv[4] = {}, vv[4] = {};
  if (a.param[0] && ok && rg == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pv[q] = a.param[k][off + q];
      mv[q] = a.m[k][off + q];
      vv[q] = a.v[k][off + q];
    }
  }
  const int rows = seg2 ? a.rows2 : a.rows;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok && !seg2) {
    const float4* src = reinterpret_cast<const float4*>(a.gpart) + col4;
    for (int rbase = rg; rbase < rows; rbase += 16 * FS_NR) {
      float4 x[FS_NR];
#pragma unroll
      for (int i = 0; i < FS_NR; ++i) {
        const int r = rbase + 16 * i;
        x[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < rows) x[i] = src[(size_t)r * ncol4];
      }
#pragma unroll
      for (int i = 0; i < FS_NR; ++i) {
        acc.x += x[i].x; acc.y += x[i].y; acc.z += x[i].z; acc.w += x[i].w;
      }
    }
  } else if (ok) {   // M rows times the member's g: one o for 4 weight columns, o .. o+3 for counts
    constexpr int NR = 16;
    const float4* src = reinterpret_cast<const float4*>(a.mpart) + col4;
    const bool wcol = e0 < C2 * K2;
    const int o0 = wcol ? e0 / K2 : e0 - C2 * K2, od = wcol ? 0 : 1;
    const float* gv = a.vec + TV_G + o0;
    for (int rbase = rg; rbase < rows; rbase += 16 * NR) {
      float4 x[NR], gq[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int r = rbase + 16 * i;
        x[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        gq[i] = x[i];
        if (r < rows) {
          x[i] = src[(size_t)r * ncol4];
          const float* gp = gv + (size_t)(r / a.ngrp) * TV;
          gq[i] = make_float4(gp[0], gp[od], gp[2 * od], gp[3 * od]);
        }
      }
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        acc.x += x[i].x * gq[i].x; acc.y += x[i].y * gq[i].y;
        acc.z += x[i].z * gq[i].z; acc.w += x[i].w * gq[i].w;
      }
    }
  }
  red[rg][cl] = acc;
  __syncthreads();
  if (rg != 0 || !ok) return;
  float4 sm4 = red[0][cl];
#pragma unroll
  for (int q = 1; q < 16; ++q) {
    const float4 x = red[q][cl];
    sm4.x += x.x; sm4.y += x.y; sm4.z += x.z; sm4.w += x.w;
  }
  const float gvv[4] = {sm4.x, sm4.y, sm4.z, sm4.w};
  float* gd = a.grad[k];
#pragma unroll
  for (int q = 0; q < 4; ++q) gd[off + q] = gvv[q];
  if (a.param[0]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float mm = mv[q];
      adam_vals(pv[q], mm, vv[q], gvv[q], hy);
      a.param[k][off + q] = pv[q];
      a.m[k][off + q] = mm;
      a.v[k][off + q] = vv[q];
    }
  }
}

template <bool SPLIT>
__global__ __launch_bounds__(256) void train_final_kernel(FinalArgs a) {
  __shared__ float4 red[4][FIN_CB_COLS];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // Adam's scalars first: their (dependent) loads overlap the gradient loads
  const AdamHyper hy = a.param[0] ? fetch_hyper(a) : AdamHyper{};
  constexpr int NCB = SPLIT ? FS_NCB1 + FS_NCB2 : FIN_NCB * FIN_RB;   // conv workgroups
  const int bx = blockIdx.x + a.conv_off;
  if constexpr (SPLIT) {
    if (bx < NCB) {
      __shared__ float4 reds[16][FS_COLS];
      final_split_conv(a, hy, bx, tid, reds);
      return;
    }
  }
  if (!SPLIT && bx < NCB) {
    const int cb = bx / FIN_RB, rb = bx - cb * FIN_RB;
    const int col4 = cb * FIN_CB_COLS + lane;
    const int ncol4 = NG / 4;   // row pitch (float4)
    const bool ok = col4 < ncol4;
    const int e0 = col4 * 4;
    const int fcol = e0;        // column of the row-block sums
    int k, off;
    if (e0 < NG_W2) { k = 0; off = e0 - NG_W1; }        // condition_encoder.0.weight
    else if (e0 < NG_B1) { k = 2; off = e0 - NG_W2; }   // condition_encoder.2.weight
    else if (e0 < NG_B2) { k = 1; off = e0 - NG_B1; }   // condition_encoder.0.bias
    else { k = 3; off = e0 - NG_B2; }                   // condition_encoder.2.bias
    // Adam's operands of the lane's 4 elements, prefetched (used by the last block only)
    float pv[4] = {}, mv[4] = {}, vv[4] = {};
    if (a.param[0] && ok && wave == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pv[q] = a.param[k][off + q];
        mv[q] = a.m[k][off + q];
        vv[q] = a.v[k][off + q];
      }
    }
    const int rpb = (a.rows + FIN_RB - 1) / FIN_RB;
    const int r0 = rb * rpb, r1 = min(a.rows, r0 + rpb);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
      const float4* src = reinterpret_cast<const float4*>(a.gpart) + col4;
      for (int rbase = r0 + wave; rbase < r1; rbase += 4 * FIN_MAXR) {
        float4 x[FIN_MAXR];
#pragma unroll
        for (int i = 0; i < FIN_MAXR; ++i) {
          const int r = rbase + 4 * i;
          x[i] = r < r1 ? src[(size_t)r * ncol4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < FIN_MAXR; ++i) {
          acc.x += x[i].x; acc.y += x[i].y; acc.z += x[i].z; acc.w += x[i].w;
        }
      }
    }
    red[wave][lane] = acc;
    __syncthreads();
    if (wave == 0) {
      float4 s = red[0][lane];
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const float4 x = red[q][lane];
        s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
      }
      if (ok) {
        float* f = a.fin + (size_t)rb * NG + fcol;
        st_wt(f, s.x); st_wt(f + 1, s.y); st_wt(f + 2, s.z); st_wt(f + 3, s.w);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.cnt + cb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old == FIN_RB - 1;
    }
    __syncthreads();
    if (!last || wave != 0) return;
    if (lane == 0)   // every arrival of this launch is in: ready for the next launch
      __hip_atomic_store(a.cnt + cb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!ok) return;
    float gv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < FIN_RB; ++q) {
      const float* f = a.fin + (size_t)q * NG + fcol;
#pragma unroll
      for (int e = 0; e < 4; ++e) gv[e] += ld_wt(f + e);
    }
    float* gd = a.grad[k];
#pragma unroll
    for (int q = 0; q < 4; ++q) gd[off + q] = gv[q];
    if (a.param[0]) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float mm = mv[q];
        adam_vals(pv[q], mm, vv[q], gv[q], hy);
        a.param[k][off + q] = pv[q];
        a.m[k][off + q] = mm;
        a.v[k][off + q] = vv[q];
      }
    }
    return;
  }
  // dense layers: one thread per element, a chain over the members
  const int H0 = a.P + 2 * H;
  int i = (bx - NCB) * 256 + tid;
  int dz_off, in_off, kdim, k;
  bool bias = false;
  if (i < H * C2) { dz_off = TV_DZ3; in_off = TV_M; kdim = C2; k = 4; }
  else if ((i -= H * C2) < H) { dz_off = TV_DZ3; bias = true; k = 5; kdim = 1; in_off = 0; }
  else if ((i -= H) < H * H) { dz_off = TV_DZ4; in_off = TV_E; kdim = H; k = 6; }
  else if ((i -= H * H) < H) { dz_off = TV_DZ4; bias = true; k = 7; kdim = 1; in_off = 0; }
  else if ((i -= H) < H * H0) { dz_off = TV_DZ5; in_off = TV_HCAT; kdim = H0; k = 8; }
  else if ((i -= H * H0) < H) { dz_off = TV_DZ5; bias = true; k = 9; kdim = 1; in_off = 0; }
  else if ((i -= H) < a.P * H) { dz_off = TV_DOUT; in_off = TV_H; kdim = H; k = 10; }
  else if ((i -= a.P * H) < a.P) { dz_off = TV_DOUT; bias = true; k = 11; kdim = 1; in_off = 0; }
  else if (i - a.P == 0) {  // loss = sum of squared errors / (B*P)
    if (!a.loss) return;    // autograd backward: the loss lives in torch
    float acc = 0.f;
    for (int b = 0; b < a.B; ++b) acc += a.vec[(size_t)b * TV + TV_SQ];
    *a.loss = acc * a.inv_n;
    return;
  } else {
    return;
  }
  float pv = 0.f, mv = 0.f, vv = 0.f;
  if (a.param[0]) {   // Adam's operands first: their loads overlap the chain's
    pv = a.param[k][i];
    mv = a.m[k][i];
    vv = a.v[k][i];
  }
  const int row = bias ? i : i / kdim, col = bias ? 0 : i - row * kdim;
  const float* pd = a.vec + dz_off + row;
  const float* pi = a.vec + (bias ? dz_off + row : in_off + col);
  float acc = 0.f;
  // 32 members' operands in flight at a time (clamped rows past B, never used)
  for (int b0 = 0; b0 < a.B; b0 += 32) {
    float xd[32], xi[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const size_t r = (size_t)min(b0 + u, a.B - 1) * TV;
      xd[u] = pd[r];
      xi[u] = pi[r];
    }
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (b0 + u < a.B) acc = bias ? acc + xd[u] : fmaf(xd[u], xi[u], acc);
  }
  a.grad[k][i] = acc;
  if (a.param[0]) {
    adam_vals(pv, mv, vv, acc, hy);
    a.param[k][i] = pv;
    a.m[k][i] = mv;
    a.v[k][i] = vv;
  }
}

// ---------------------------------------------------------------------------
// Adam alone (ertd_adam: torch.optim.Adam on gradients computed elsewhere)
// ---------------------------------------------------------------------------
struct AdamArgs {
  float* p[12];
  const float* g[12];
  float* m[12];
  float* v[12];
  int off[13];
  AdamHyper hy;
};

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.off[12]) return;
  int k = 0;
#pragma unroll
  for (int q = 1; q < 12; ++q) k += (i >= a.off[q]) ? 1 : 0;
  const int e = i - a.off[k];
  adam_elem(a.p[k], a.m[k], a.v[k], e, a.g[k][e], a.hy);
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
namespace {

// scalars formed as torch does: Python floats (double), rounded when applied to fp32
AdamHyper adam_hyper(int step, float lr, float beta1, float beta2, float eps) {
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  AdamHyper a;
  a.one_minus_b1 = (float)(1.0 - (double)beta1);
  a.b2 = beta2;
  a.one_minus_b2 = (float)(1.0 - (double)beta2);
  a.step_size_neg = (float)(-((double)lr / bc1));
  a.bc2_sqrt = (float)std::sqrt(bc2);
  a.eps = eps;
  return a;
}

void param_list(const ertd_weights& w, float* out[12]) {
  const float* ps[12] = {w.enc0_w, w.enc0_b, w.enc2_w, w.enc2_b, w.enc6_w, w.enc6_b,
                         w.time_w, w.time_b, w.mlp0_w, w.mlp0_b, w.mlp2_w, w.mlp2_b};
  for (int k = 0; k < 12; ++k) out[k] = const_cast<float*>(ps[k]);
}

struct TrainWs {
  float* partial;  // (B, S, 64)
  float* a1s;      // (B*S, A1S_FLOATS)
  uint32_t* m2w;   // (B*S, M2W_WORDS)
  float* gpart;    // (B*S, NG)
  float* fin;      // (FIN_RB, NG)
  unsigned* cnt;   // (FIN_CNT_WORDS)
  float* vec;      // (B, TV); the reference train step only
  float* wt;       // (WT_FLOATS) k-major dense weights; the reference train step only
  float* w2b;      // (W2B_FRAG) transposed-conv2 fragments
  float* mpart;    // (B * w2m_groups(S), NG2) w2m rows; the reference train step only
};

// the encoder part (also the U-Net's condition branch), then the member rows
size_t ws_layout(int B, int L, bool with_vec, float* base, TrainWs* out) {
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  const size_t items = (size_t)B * S;
  auto al = [](size_t n) { return (n + 63) / 64 * 64; };
  size_t o = 0;
  TrainWs w{};
  w.partial = base + o; o += al(items * C2);
  w.a1s = base + o; o += al(items * A1S_FLOATS);
  w.m2w = reinterpret_cast<uint32_t*>(base + o); o += al(items * M2W_WORDS);
  w.gpart = base + o; o += al(items * NG);
  w.fin = base + o; o += al((size_t)FIN_RB * NG);
  w.cnt = reinterpret_cast<unsigned*>(base + o); o += al(FIN_CNT_WORDS);
  w.w2b = base + o; o += al(W2B_FRAG);
  if (with_vec) {
    w.vec = base + o; o += al((size_t)B * TV);
    w.wt = base + o; o += al(WT_FLOATS);
    w.mpart = base + o; o += al((size_t)B * w2m_groups(S) * NG2);
  }
  if (out) *out = w;
  return o;
}

int dense_count(int P) { return H * C2 + H + H * H + H + H * (P + 2 * H) + H + P * H + P + 1; }

// conv_grads: FIN_NCB * FIN_RB conv blocks; dense: the member-row part too
#ifndef FIN_ABL
#define FIN_ABL 0  // diagnostic variants only: 1 = conv part only, 2 = dense part only
#endif
hipError_t launch_final(FinalArgs& a, bool dense, hipStream_t s) {
  if ((FIN_ABL & 1) != 0) dense = false;
  const bool split = a.mpart != nullptr;
  const int ncb = split ? FS_NCB1 + FS_NCB2 : FIN_NCB * FIN_RB;
  int blocks = ncb + (dense ? (dense_count(a.P) + 255) / 256 : 0);
  if ((FIN_ABL & 2) != 0) { a.conv_off = ncb; blocks -= ncb; }
  if (split) train_final_kernel<true><<<blocks, 256, 0, s>>>(a);
  else train_final_kernel<false><<<blocks, 256, 0, s>>>(a);
  return hipGetLastError();
}

FinalArgs final_args(const TrainWs& W, int rows) {
  FinalArgs a{};
  a.gpart = W.gpart;
  a.rows = rows;
  a.fin = W.fin;
  a.cnt = W.cnt;
  return a;
}

void set_dense(FinalArgs& a, const ertd_weights& w, const TrainWs& W, int B, float* const* grads,
               float* loss_out) {
  a.vec = W.vec;
  a.B = B;
  a.P = w.param_dim;
  a.inv_n = (float)(1.0 / ((double)B * w.param_dim));
  for (int k = 0; k < 12; ++k) a.grad[k] = grads[k];
  a.loss = loss_out;
}

// wd: the model's dense weights (their k-major copies go to W.wt), or null
hipError_t launch_enc(const float* w1, const float* b1, const float* w2, const float* b2,
                      const float* cond, int B, int L, const TrainWs& W, int* step_ctr,
                      const ertd_weights* wd, hipStream_t s) {
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  enc_train_kernel<<<dim3((unsigned)(B * S)), 256, 0, s>>>(w1, b1, w2, b2, cond, L, L1, L2, S, W.partial,
                                                         W.a1s, W.m2w, W.cnt, step_ctr,
                                                         wd ? *wd : ertd_weights{}, wd ? W.wt : nullptr,
                                                         W.w2b);
  return hipGetLastError();
}

// (the W2 fragments are the ones the forward on this workspace wrote)
// w2: with the dW2 work (rows of NG); else the chain alone (rows of NG1)
hipError_t launch_conv_bwd(const float* cond, const TrainWs& W, const float* g, int g_stride, int B,
                           int L, bool w2, hipStream_t s) {
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  const int nit = B * S, cus = device_cu_count();
  const int c1 = nit < 2 * cus ? nit : 2 * cus, c2 = nit < cus ? nit : cus;
  if (w2)
    conv_bwd_kernel<true><<<dim3((unsigned)((CBW_ABL & 16) ? nit : 2 * nit)), 256, 0, s>>>(
        W.w2b, cond, W.a1s, W.m2w, g, g_stride, L, L1, L2, S, W.gpart, c1, c2);
  else
    conv_bwd_kernel<false><<<dim3((unsigned)nit), 256, 0, s>>>(W.w2b, cond, W.a1s, W.m2w, g, g_stride,
                                                              L, L1, L2, S, W.gpart, c1, c2);
  return hipGetLastError();
}

W2mArgs w2m_args(const TrainWs& W, int B) { return W2mArgs{W.a1s, W.m2w, W.mpart, B}; }
int head_grid(int B, int L) { return B + B * w2m_groups(n_strips(conv_len(conv_len(L)))); }

void set_split(FinalArgs& a, const TrainWs& W, int B, int L) {
  const int S = n_strips(conv_len(conv_len(L)));
  a.mpart = W.mpart;
  a.ngrp = w2m_groups(S);
  a.rows2 = B * a.ngrp;
}

}  // namespace

size_t train_ws_floats(int B, int L) { return ws_layout(B, L, true, nullptr, nullptr); }

// the encoder-conv backward kernel alone, on the state the last train forward /
// step left in ws (its dL/dpooled rows): per-kernel timing (bench.py train_roofline)
hipError_t launch_train_conv_backward(const float* cond, int B, int L, float* ws, hipStream_t s) {
  TrainWs W;
  ws_layout(B, L, true, ws, &W);
  return launch_conv_bwd(cond, W, W.vec + TV_G, TV, B, L, false, s);
}

void adam_table_host(int step_first, int n, float lr, float beta1, float beta2, float eps,
                     float* out) {
  for (int i = 0; i < n; ++i) {
    const AdamHyper a = adam_hyper(step_first + i, lr, beta1, beta2, eps);
    std::memcpy(out + (size_t)i * ADAM_TABLE_FLOATS, &a, sizeof(a));
  }
}

hipError_t launch_train_forward(const ertd_weights& w, const float* x_in, const float* x0,
                                const float* noise, const float* alpha_bar, const int64_t* t,
                                const float* cond, int B, int L, const float* freq, float* eps_out,
                                float* ws, hipStream_t s) {
  TrainWs W;
  ws_layout(B, L, true, ws, &W);
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  hipError_t e = launch_enc(w.enc0_w, w.enc0_b, w.enc2_w, w.enc2_b, cond, B, L, W, nullptr, &w, s);
  if (e != hipSuccess) return e;
  train_head_kernel<0><<<B, HT, 0, s>>>(w, W.wt, x_in, x0, noise, alpha_bar, t, freq, W.partial, S, L2,
                                        W.vec, eps_out, nullptr, 0.f, nullptr, HeadRng{}, W2mArgs{});
  return hipGetLastError();
}

hipError_t launch_train_backward(const ertd_weights& w, const float* dout, const float* noise,
                                 const float* cond, int B, int L, float* const* grads,
                                 float* loss_out, float* dx_out, float* ws, hipStream_t s) {
  TrainWs W;
  ws_layout(B, L, true, ws, &W);
  const int P = w.param_dim;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  const float two_over_n = (float)(2.0 / ((double)B * P));
  train_head_kernel<1><<<head_grid(B, L), HT, 0, s>>>(w, W.wt, nullptr, nullptr, noise, nullptr, nullptr,
                                                      nullptr, nullptr, S, L2, W.vec, nullptr, dout,
                                                      two_over_n, dx_out, HeadRng{}, w2m_args(W, B));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_conv_bwd(cond, W, W.vec + TV_G, TV, B, L, false, s);
  if (e != hipSuccess) return e;
  FinalArgs a = final_args(W, B * S);
  set_dense(a, w, W, B, grads, loss_out);
  set_split(a, W, B, L);
  return launch_final(a, true, s);
}

hipError_t launch_train_step(const ertd_weights& w, const float* x0, const int64_t* t,
                             const float* noise, const float* cond, const float* alpha_bar, int B,
                             int L, const float* freq, float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, const TrainAdam& adam, float* loss_out,
                             float* ws, hipStream_t s) {
  TrainWs W;
  ws_layout(B, L, true, ws, &W);

  const int P = w.param_dim;
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  const float two_over_n = (float)(2.0 / ((double)B * P));
  hipError_t e =
      launch_enc(w.enc0_w, w.enc0_b, w.enc2_w, w.enc2_b, cond, B, L, W, adam.step_dev, &w, s);
  if (e != hipSuccess) return e;
  HeadRng rng{};
  if (adam.draw) {
    rng.seed = adam.seed;
    rng.step = adam.step_dev;
    rng.T = adam.T;
    rng.t_out = const_cast<int64_t*>(t);
    rng.noise_out = const_cast<float*>(noise);
  }
  train_head_kernel<2><<<head_grid(B, L), HT, 0, s>>>(w, W.wt, nullptr, x0, noise, alpha_bar, t, freq,
                                                      W.partial, S, L2, W.vec, nullptr, nullptr,
                                                      two_over_n, nullptr, rng, w2m_args(W, B));
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_conv_bwd(cond, W, W.vec + TV_G, TV, B, L, false, s);
  if (e != hipSuccess) return e;
  FinalArgs a = final_args(W, B * S);
  set_dense(a, w, W, B, grads, loss_out);
  set_split(a, W, B, L);
  param_list(w, a.param);
  for (int k = 0; k < 12; ++k) {
    a.m[k] = exp_avg[k];
    a.v[k] = exp_avg_sq[k];
  }
  if (adam.table) {
    a.hyper_tab = adam.table;
    a.step_ctr = adam.step_dev;
    a.tab_first = adam.table_first;
    a.tab_len = adam.table_len;
  } else {
    a.hyper = adam_hyper(adam.step, adam.lr, adam.beta1, adam.beta2, adam.eps);
  }
  return launch_final(a, true, s);
}

// ---------------------------------------------------------------------------
// The reference condition encoder alone with saved activations (the U-Net
// train step's condition branch, unet_train.hip): the same kernels on the raw
// conv weights w1 (32,14,3) / w2 (64,32,3); the backward from g = dL/dm / L2.
// ---------------------------------------------------------------------------
size_t encoder_train_ws_floats(int B, int L) { return ws_layout(B, L, false, nullptr, nullptr); }

hipError_t launch_encoder_train(const float* w1, const float* b1, const float* w2, const float* b2,
                                const float* cond, int B, int L, float* ws, float** partial_out,
                                hipStream_t s) {
  TrainWs W;
  ws_layout(B, L, false, ws, &W);
  *partial_out = W.partial;
  return launch_enc(w1, b1, w2, b2, cond, B, L, W, nullptr, nullptr, s);
}

hipError_t launch_encoder_conv_backward(const float* w2, const float* cond, const float* g, int B,
                                        int L, float* ws, float* dw1, float* db1, float* dw2,
                                        float* db2, hipStream_t s) {
  TrainWs W;
  ws_layout(B, L, false, ws, &W);
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  (void)w2;  // the fragments of the forward on this workspace
  hipError_t e = launch_conv_bwd(cond, W, g, C2, B, L, true, s);
  if (e != hipSuccess) return e;
  FinalArgs a = final_args(W, B * S);
  a.grad[0] = dw1;
  a.grad[1] = db1;
  a.grad[2] = dw2;
  a.grad[3] = db2;
  return launch_final(a, false, s);
}

hipError_t launch_adam(const ertd_weights& w, float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, int step, float lr, float beta1, float beta2,
                       float eps, hipStream_t s) {
  const int P = w.param_dim;
  const int sizes[12] = {C1 * K1, C1, C2 * K2, C2, H * C2, H, H * H, H, H * (P + 2 * H), H, P * H, P};
  float* ps[12];
  param_list(w, ps);
  AdamArgs a{};
  int off = 0;
  for (int k = 0; k < 12; ++k) {
    a.p[k] = ps[k];
    a.g[k] = grads[k];
    a.m[k] = exp_avg[k];
    a.v[k] = exp_avg_sq[k];
    a.off[k] = off;
    off += sizes[k];
  }
  a.off[12] = off;
  a.hy = adam_hyper(step, lr, beta1, beta2, eps);
  adam_kernel<<<(off + 255) / 256, 256, 0, s>>>(a);
  return hipGetLastError();
}

#ifdef HEAD_STAMPS
extern "C" int ertd_diag_head_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hstamp), sizeof(g_hstamp));
}
#endif

}  // namespace ertd
