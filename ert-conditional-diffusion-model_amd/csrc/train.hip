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

// saved activations per (member, strip): the conv1 images E[c][m] = a1(p = 2m),
// O[c][m] = a1(p = 2m+1) at conv1 positions i = 2*j0 - 1 + p, p < 128 (zero
// outside [0, L1)), and the conv2 ReLU mask word [q][o >> 5] (bit o & 31) of
// conv2 output j0 + q (0 for q >= J or j0 + q >= L2)
constexpr int A1S_FLOATS = 2 * C1 * 64;
constexpr int M2W_WORDS = 64 * 2;

// train_final_kernel's conv-column reduction (see there)
constexpr int FIN_CB_COLS = 64;                                  // float4 columns per block
constexpr int FIN_NCB = (NG / 4 + FIN_CB_COLS - 1) / FIN_CB_COLS;  // 30 column blocks
constexpr int FIN_RB = 8;                                        // row blocks
constexpr int FIN_MAXR = 48;                                     // rows per wave held in flight
constexpr int FIN_CNT_WORDS = 64;
static_assert(FIN_NCB <= FIN_CNT_WORDS, "counter words");

// ---------------------------------------------------------------------------
// training forward of the condition encoder
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void enc_train_kernel(
    const float* __restrict__ w1, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ cond, int L, int L1, int L2, int S,
    float* __restrict__ partial, float* __restrict__ a1s, uint32_t* __restrict__ m2w,
    unsigned* __restrict__ fin_cnt, int* __restrict__ step_ctr) {
  __shared__ __attribute__((aligned(16))) EncSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int item = blockIdx.x;
  if (item == 0) {  // the step's bookkeeping words (read only by later kernels of the stream)
    if (tid < FIN_CNT_WORDS) fin_cnt[tid] = 0u;   // train_final_kernel's arrival counters
    if (tid == 0 && step_ctr) step_ctr[0] += 1;   // the Adam step of this train step
  }
  const int b = item / S, strip = item - b * S;
  const int j0 = strip * J;

  // conv1 fragment s of lane (o = l32, h): W1[o][c = s/3 + 7h][s % 3], contiguous in s
  float wa[STEPS1];
  {
    const float* src = w1 + l32 * K1 + 21 * h;
#pragma unroll
    for (int s = 0; s < STEPS1; ++s) wa[s] = src[s];
  }
  stage_cond_f32(sm.X, cond + (size_t)b * CIN * L, L, 4 * j0 - 3, tid);
  __syncthreads();

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
  {  // the strip's conv1 images -> a1s: 1,024 float4 rows, 4 per thread
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
    const float* src = w2 + o * K2 + 48 * h;
#pragma unroll
    for (int s = 0; s < STEPS2; ++s) w2r[s] = src[s];
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
    if (lane < 32) {
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
// head forward / backward (one 256-thread block per member)
// Forward layers y = W x + b (W row-major, as the parameters lie): a wave owns
// 32 (or 8) rows, lane l the columns k = l + 64 i, so every weight load is a
// coalesced 256-B row segment; the 64 lane partials of all its rows are summed
// by one reduce-scatter (rows_reduce: 32 shuffles for 32 rows).  Backward
// layers y = W^T x: a thread per output, the loads coalesced across threads,
// 16 of them in flight.
// ---------------------------------------------------------------------------
struct HeadSmem {
  float m[C2], e[H], c[H], te[H], hc[PMAX + 2 * H], h[H], eps[PMAX], nz[PMAX];
  float dout[PMAX], dz5[H], dhc[2 * H], dz3[H], red[PMAX];
  int t;
};

// v[r] holds this lane's partial of row r (NR = 2^m <= 32 rows): returns the
// sum over all 64 lanes of row (lane >> (6 - m)) & (NR - 1), in a fixed order
template <int NR>
__device__ __forceinline__ float rows_reduce(float (&v)[NR], int lane) {
  constexpr int LEVELS = NR == 32 ? 5 : NR == 16 ? 4 : NR == 8 ? 3 : NR == 4 ? 2 : NR == 2 ? 1 : 0;
#pragma unroll
  for (int lev = 0; lev < LEVELS; ++lev) {
    const int msk = 32 >> lev, half = NR >> (lev + 1);
    const bool hi = (lane & msk) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float send = hi ? v[i] : v[half + i];
      const float keep = hi ? v[half + i] : v[i];
      v[i] = keep + __shfl_xor(send, msk);
    }
  }
  float s = v[0];
#pragma unroll
  for (int msk = 32 >> LEVELS; msk >= 1; msk >>= 1) s += __shfl_xor(s, msk);
  return s;
}

// out[row0 + r] = act(bias + W[row0 + r][0:K] . x[0:K]) for r < NR, rows < nrows;
// x in LDS; KC = ceil(K / 64) column chunks
template <int NR, int KC, bool RELU>
__device__ __forceinline__ void rows_layer(const float* __restrict__ W, int ldw, int K,
                                           const float* __restrict__ bias, const float* x, int row0,
                                           int nrows, float* out, int lane) {
  float xv[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) xv[i] = (lane + 64 * i < K) ? x[lane + 64 * i] : 0.f;
  float v[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int row = row0 + r < nrows ? row0 + r : nrows - 1;   // clamped: rows past nrows unused
    const float* wr = W + (size_t)row * ldw;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const int k = lane + 64 * i;
      acc = fmaf(k < K ? wr[k] : 0.f, xv[i], acc);
    }
    v[r] = acc;
  }
  constexpr int SH = NR == 32 ? 1 : NR == 16 ? 2 : NR == 8 ? 3 : NR == 4 ? 4 : 5;
  const float s = rows_reduce<NR>(v, lane);
  const int row = row0 + ((lane >> SH) & (NR - 1));
  if ((lane & ((1 << SH) - 1)) == 0 && row < nrows) {
    const float y = s + bias[row];
    out[row] = RELU ? fmaxf(y, 0.f) : y;
  }
}

struct HeadRng {  // the train step's own draws (TrainPlan): t ~ U{0..T-1}, noise ~ N(0,1)
  uint64_t seed;
  const int* step;  // device step counter (already advanced for this step)
  int T;
  int64_t* t_out;   // (B) the drawn t
  float* noise_out; // (B, P) the drawn noise
};
constexpr uint32_t RNG_TAG_T = 0x7A11u, RNG_TAG_NOISE = 0x7A12u;

__device__ __forceinline__ void head_forward(
    const ertd_weights& w, const float* __restrict__ x_in, const float* __restrict__ x0,
    const float* __restrict__ noise, const float* __restrict__ alpha_bar,
    const int64_t* __restrict__ t_vec, const float* __restrict__ freq,
    const float* __restrict__ partial, int S, int L2, float* __restrict__ V,
    float* __restrict__ eps_out, const HeadRng* rng, HeadSmem& s, int b, int tid) {
  const int P = w.param_dim, lane = tid & 63, wave = tid >> 6;
  if (rng) {  // Philox keyed (seed, member, step): independent of the grid and of the schedule
    const uint32_t st = (uint32_t)*rng->step;
    if (tid == 0) {
      const u32x4 r = philox4x32_10(u32x4{0u, (uint32_t)b, st, RNG_TAG_T}, (uint32_t)rng->seed,
                                    (uint32_t)(rng->seed >> 32));
      const int tv = (int)(((uint64_t)r.x * (uint64_t)rng->T) >> 32);
      s.t = tv;
      rng->t_out[b] = tv;
    }
    if (tid < P) {
      const float z = philox_normal(rng->seed, (uint32_t)b, st, RNG_TAG_NOISE, tid);
      s.nz[tid] = z;
      rng->noise_out[(size_t)b * P + tid] = z;
    }
  } else {
    if (tid == 0) s.t = (int)t_vec[b];
    if (tid < P && noise) s.nz[tid] = noise[(size_t)b * P + tid];
  }
  if (tid < C2) {
    float acc = 0.f;
    for (int k = 0; k < S; ++k) acc += partial[((size_t)b * S + k) * C2 + tid];
    s.m[tid] = acc / (float)L2;
  }
  __syncthreads();
  const int t = s.t;
  if (tid < P) {
    float xv;
    if (x_in) {
      xv = x_in[(size_t)b * P + tid];
    } else {  // q_sample (:97-99): one rounding per op
      const float ab = alpha_bar[t];
      const float sa = sqrtf(ab), sb = sqrtf(1.0f - ab);
      xv = sa * x0[(size_t)b * P + tid] + sb * s.nz[tid];
    }
    s.hc[tid] = xv;
  }
  if (tid >= H) {
    const int k = tid - H;
    const float a = (float)t * freq[k < 64 ? k : k - 64];
    s.e[k] = k < 64 ? sinf(a) : cosf(a);
  }
  __syncthreads();
  // cond_emb = relu(W3 m + b3) (waves 0-1), t_emb = relu(Wt e + bt) (waves 2-3)
  if (wave < 2) {
    rows_layer<32, 1, true>(w.enc6_w, C2, C2, w.enc6_b, s.m, wave * 64, H, s.c, lane);
    rows_layer<32, 1, true>(w.enc6_w, C2, C2, w.enc6_b, s.m, wave * 64 + 32, H, s.c, lane);
  } else {
    rows_layer<32, 2, true>(w.time_w, H, H, w.time_b, s.e, (wave - 2) * 64, H, s.te, lane);
    rows_layer<32, 2, true>(w.time_w, H, H, w.time_b, s.e, (wave - 2) * 64 + 32, H, s.te, lane);
  }
  __syncthreads();
  if (tid < H) {
    s.hc[P + tid] = s.te[tid];
    s.hc[P + H + tid] = s.c[tid];
  }
  __syncthreads();
  const int K0 = P + 2 * H;
  // h = relu(W0 hcat + b0)
  rows_layer<32, (PMAX + 2 * H + 63) / 64, true>(w.mlp0_w, K0, K0, w.mlp0_b, s.hc, wave * 32, H, s.h,
                                                 lane);
  __syncthreads();
  // eps = W2 h + b2
  rows_layer<8, 2, false>(w.mlp2_w, H, H, w.mlp2_b, s.h, wave * 8, P, s.eps, lane);
  __syncthreads();
  if (tid < P) {
    V[TV_EPS + tid] = s.eps[tid];
    if (eps_out) eps_out[(size_t)b * P + tid] = s.eps[tid];
  }
  for (int i = tid; i < K0; i += 256) V[TV_HCAT + i] = s.hc[i];
  if (tid < H) {
    V[TV_E + tid] = s.e[tid];
    V[TV_H + tid] = s.h[tid];
  }
  if (tid < C2) V[TV_M + tid] = s.m[tid];
}

//   dout: given (autograd) or MSE: (pred - noise) * (2/(B*P))   (mse_loss backward)
// eps_v / h_v / hcat_v / nz_v: the forward's prediction, relu(z5), [x | t_emb |
// cond_emb] and noise (LDS in the fused kernel; the saved row / the noise input otherwise)
__device__ __forceinline__ void head_backward(
    const ertd_weights& w, const float* __restrict__ dout_in, const float* nz_v, float two_over_n,
    int L2, float* __restrict__ V, float* __restrict__ dx_out, const float* eps_v, const float* h_v,
    const float* hcat_v, HeadSmem& s, int b, int tid) {
  const int P = w.param_dim;
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
  __syncthreads();
  if (tid == 0) {
    float acc = 0.f;
    for (int o = 0; o < P; ++o) acc += s.red[o];
    V[TV_SQ] = acc;
  }
  if (tid < H) {  // dz5 = (W2^T dout) * [h > 0]
    float acc = 0.f;
#pragma unroll 8
    for (int o = 0; o < P; ++o) acc = fmaf(w.mlp2_w[o * H + tid], s.dout[o], acc);
    const float d = h_v[tid] > 0.f ? acc : 0.f;
    s.dz5[tid] = d;
    V[TV_DZ5 + tid] = d;
  }
  __syncthreads();
  const int K0 = P + 2 * H;
  {  // dhcat[P + k] for k < 256 (t_emb and cond_emb columns)
    float acc = 0.f;
#pragma unroll 16
    for (int j = 0; j < H; ++j) acc = fmaf(w.mlp0_w[(size_t)j * K0 + P + tid], s.dz5[j], acc);
    s.dhc[tid] = acc;
  }
  if (dx_out && tid < P) {  // dx = W0x^T dz5 (autograd w.r.t. the model input)
    float acc = 0.f;
#pragma unroll 16
    for (int j = 0; j < H; ++j) acc = fmaf(w.mlp0_w[(size_t)j * K0 + tid], s.dz5[j], acc);
    dx_out[(size_t)b * P + tid] = acc;
  }
  __syncthreads();
  if (tid < H) {
    const float te = hcat_v[P + tid];
    V[TV_DZ4 + tid] = te > 0.f ? s.dhc[tid] : 0.f;
  } else {
    const int j = tid - H;
    const float c = hcat_v[P + H + j];
    const float d = c > 0.f ? s.dhc[tid] : 0.f;
    s.dz3[j] = d;
    V[TV_DZ3 + j] = d;
  }
  __syncthreads();
  if (tid < C2) {  // g = (W3^T dz3) / L2  (AdaptiveAvgPool backward)
    float acc = 0.f;
#pragma unroll 16
    for (int j = 0; j < H; ++j) acc = fmaf(w.enc6_w[j * C2 + tid], s.dz3[j], acc);
    V[TV_G + tid] = acc / (float)L2;
  }
}

// MODE 0: forward only; 1: backward only (of the last forward's saved row);
// 2: both (the train step; rng != null: the step draws its own t and noise)
template <int MODE>
__global__ __launch_bounds__(256) void train_head_kernel(
    ertd_weights w, const float* __restrict__ x_in, const float* __restrict__ x0,
    const float* __restrict__ noise, const float* __restrict__ alpha_bar,
    const int64_t* __restrict__ t_vec, const float* __restrict__ freq,
    const float* __restrict__ partial, int S, int L2, float* __restrict__ vec,
    float* __restrict__ eps_out, const float* __restrict__ dout_in, float two_over_n,
    float* __restrict__ dx_out, HeadRng rng) {
  __shared__ HeadSmem s;
  const int b = blockIdx.x, tid = threadIdx.x;
  float* V = vec + (size_t)b * TV;
  const HeadRng* rp = rng.step ? &rng : nullptr;
  if constexpr (MODE != 1)
    head_forward(w, x_in, x0, noise, alpha_bar, t_vec, freq, partial, S, L2, V, eps_out, rp, s, b, tid);
  if constexpr (MODE == 2) {
    __syncthreads();
    head_backward(w, dout_in, s.nz, two_over_n, L2, V, dx_out, s.eps, s.h, s.hc, s, b, tid);
  }
  if constexpr (MODE == 1) {
    head_backward(w, dout_in, noise ? noise + (size_t)b * w.param_dim : nullptr, two_over_n, L2, V,
                  dx_out, V + TV_EPS, V + TV_H, V + TV_HCAT, s, b, tid);
  }
}

// ---------------------------------------------------------------------------
// conv backward, one 256-thread workgroup per (member, strip of J conv2 outputs)
//   phase A: dz2 = g * mask -> da1 (transposed conv2) -> dz1 = da1 * [a1 > 0]
//            (waves 0-1: even conv1 positions, 1 tap; waves 2-3: odd, 2 taps)
//            and dW2 = dz2 x a1 (6 tiles: 2 + 2 + 1 + 1) -- 96 MFMAs per wave
//   phase B: dW1 = dz1 x cond (+ db1 from a ones column of the padded N), 32 per wave
// LDS: phase A's dz2 / a1 images are dead in phase B, where the cond image and
// the dW1 halves take their place: 51.6 KB -> 3 workgroups per CU.
// ---------------------------------------------------------------------------
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
#pragma unroll 8
  for (int s = 0; s < 32; ++s) {
    const float bv = (2 * s + h < J) ? ab[2 * s] : 0.f;  // q' = 63 is the halo: excluded
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(zb[2 * s], bv, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int o = ot * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    G[NG_W2 + o * K2 + n] = acc[r];
  }
}

__global__ __launch_bounds__(256, 3) void conv_bwd_kernel(
    const float* __restrict__ w2, const float* __restrict__ cond, const float* __restrict__ a1s,
    const uint32_t* __restrict__ m2w, const float* __restrict__ g, int g_stride, int L, int L1,
    int L2, int S, float* __restrict__ gpart) {
  __shared__ __attribute__((aligned(16))) ConvBwdSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int item = blockIdx.x;
  const int b = item / S, strip = item - b * S;
  const int j0 = strip * J;
  float* G = gpart + (size_t)item * NG;

  // ---- transposed-conv2 fragments (the da1 A operand) first, into registers:
  //   T_kk[s][lane] = W2[o = 2s + h][c = l32][kk]; even waves tap 1, odd waves taps 0 and 2
  const bool oddw = wave >= 2;
  float wt0[32], wt1[32];
  {
    const float* base = w2 + h * K2 + l32 * 3;
    const int k0 = oddw ? 0 : 1;
#pragma unroll
    for (int s = 0; s < 32; ++s) wt0[s] = base[s * 2 * K2 + k0];
#pragma unroll
    for (int s = 0; s < 32; ++s) wt1[s] = oddw ? base[s * 2 * K2 + 2] : 0.f;
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

  // ---- a1 images (the forward's float4 rows) and dz2 = g * mask
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
    const float go = g[(size_t)b * g_stride + o];
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
  __syncthreads();

  // ---- phase A
  {
    const int mt = wave & 1;
    const int mcol = mt * 32 + l32;
    const float* db = &sm.DZ2[0][0] + h * DZ2P + mcol;
    f32x16 acc = {};
    if (!oddw) {
      // r = 2m: da1 = sum_o W2[o][c][1] dz2[o][m]
#pragma unroll 8
      for (int s = 0; s < 32; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wt0[s], db[2 * s * DZ2P], acc, 0, 0, 0);
    } else {
      // r = 2m+1: da1 = sum_o W2[o][c][0] dz2[o][m+1] + W2[o][c][2] dz2[o][m]
#pragma unroll 8
      for (int s = 0; s < 32; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wt0[s], db[2 * s * DZ2P + 1], acc, 0, 0, 0);
#pragma unroll 8
      for (int s = 0; s < 32; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wt1[s], db[2 * s * DZ2P], acc, 0, 0, 0);
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
  if (wave == 0) { dw2_tile(sm, 0, h, l32, G); dw2_tile(sm, 1, h, l32, G); }
  else if (wave == 1) { dw2_tile(sm, 2, h, l32, G); dw2_tile(sm, 3, h, l32, G); }
  else dw2_tile(sm, 2 + wave, h, l32, G);
  __syncthreads();

  // ---- cond image into the dead dz2 region; db2
#pragma unroll
  for (int c = 0; c < CIN; ++c) sm.X[tid & 3][c][tid >> 2] = cin ? cv[c] : 0.f;
  if (tid < CIN * 4) sm.X[tu & 3][tc][tu >> 2] = (pt >= 0 && pt < L) ? cvt : 0.f;
  if (tid < C2) G[NG_B2 + tid] = sm.db2p[0][tid] + sm.db2p[1][tid] + sm.db2p[2][tid] + sm.db2p[3][tid];
  __syncthreads();

  // ---- phase B: dW1[o][n = c*3+kk] = sum_r dz1[o][r] * cond[c][4*j0 + 2r - 1 + kk];
  //      column n = 42 (padding) multiplies by ones: db1[o] = sum_r dz1[o][r]
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
#pragma unroll 8
    for (int s = rh * 32; s < rh * 32 + 32; ++s) {
      const float bv = nvalid ? xb[s] : pad;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(zb[2 * s], bv, acc, 0, 0, 0);
    }
    store_tile_rows(sm.red[wave], acc, h, l32);  // red aliases the dead a1 images
  }
  __syncthreads();
  for (int idx = tid; idx < C1 * K1; idx += 256) {  // r-halves combined in order
    const int o = idx / K1, n = idx - o * K1;
    const int nt = n >> 5, col = n & 31;
    G[NG_W1 + idx] = sm.red[nt][o][col] + sm.red[2 + nt][o][col];
  }
  if (tid < C1) G[NG_B1 + tid] = sm.red[1][tid][K1 - 32] + sm.red[3][tid][K1 - 32];
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
__device__ __forceinline__ void adam_elem(float* __restrict__ p, float* __restrict__ m,
                                          float* __restrict__ v, int e, float g, const AdamHyper& a) {
  float mm = m[e];
  mm = mm + a.one_minus_b1 * (g - mm);
  float vv = v[e] * a.b2;
  vv = vv + a.one_minus_b2 * g * g;
  const float denom = sqrtf(vv) / a.bc2_sqrt + a.eps;
  p[e] = p[e] + a.step_size_neg * (mm / denom);
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

__global__ __launch_bounds__(256) void train_final_kernel(FinalArgs a) {
  __shared__ float4 red[4][FIN_CB_COLS];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if ((int)blockIdx.x < FIN_NCB * FIN_RB) {
    const int cb = blockIdx.x / FIN_RB, rb = blockIdx.x - cb * FIN_RB;
    const int col4 = cb * FIN_CB_COLS + lane;
    const bool ok = col4 < NG / 4;
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
          x[i] = r < r1 ? src[(size_t)r * (NG / 4)] : make_float4(0.f, 0.f, 0.f, 0.f);
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
        float* f = a.fin + (size_t)rb * NG + col4 * 4;
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
      const float* f = a.fin + (size_t)q * NG + col4 * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) gv[e] += ld_wt(f + e);
    }
    const int e0 = col4 * 4;
    int k, off;
    if (e0 < NG_W2) { k = 0; off = e0 - NG_W1; }        // condition_encoder.0.weight
    else if (e0 < NG_B1) { k = 2; off = e0 - NG_W2; }   // condition_encoder.2.weight
    else if (e0 < NG_B2) { k = 1; off = e0 - NG_B1; }   // condition_encoder.0.bias
    else { k = 3; off = e0 - NG_B2; }                   // condition_encoder.2.bias
    float* gd = a.grad[k];
#pragma unroll
    for (int q = 0; q < 4; ++q) gd[off + q] = gv[q];
    if (a.param[0]) {
      const AdamHyper hy = fetch_hyper(a);
#pragma unroll
      for (int q = 0; q < 4; ++q) adam_elem(a.param[k], a.m[k], a.v[k], off + q, gv[q], hy);
    }
    return;
  }
  // dense layers: one thread per element, a chain over the members
  const int H0 = a.P + 2 * H;
  int i = (blockIdx.x - FIN_NCB * FIN_RB) * 256 + tid;
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
  const int row = bias ? i : i / kdim, col = bias ? 0 : i - row * kdim;
  const float* pd = a.vec + dz_off + row;
  const float* pi = a.vec + in_off + col;
  float acc = 0.f;
  if (bias) {
#pragma unroll 16
    for (int b = 0; b < a.B; ++b) acc = acc + pd[(size_t)b * TV];
  } else {
#pragma unroll 16
    for (int b = 0; b < a.B; ++b) acc = fmaf(pd[(size_t)b * TV], pi[(size_t)b * TV], acc);
  }
  a.grad[k][i] = acc;
  if (a.param[0]) adam_elem(a.param[k], a.m[k], a.v[k], i, acc, fetch_hyper(a));
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
  if (with_vec) { w.vec = base + o; o += al((size_t)B * TV); }
  if (out) *out = w;
  return o;
}

int dense_count(int P) { return H * C2 + H + H * H + H + H * (P + 2 * H) + H + P * H + P + 1; }

// conv_grads: FIN_NCB * FIN_RB conv blocks; dense: the member-row part too
hipError_t launch_final(FinalArgs& a, bool dense, hipStream_t s) {
  const int blocks = FIN_NCB * FIN_RB + (dense ? (dense_count(a.P) + 255) / 256 : 0);
  train_final_kernel<<<blocks, 256, 0, s>>>(a);
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

hipError_t launch_enc(const float* w1, const float* b1, const float* w2, const float* b2,
                      const float* cond, int B, int L, const TrainWs& W, int* step_ctr, hipStream_t s) {
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  enc_train_kernel<<<dim3((unsigned)(B * S)), 256, 0, s>>>(w1, b1, w2, b2, cond, L, L1, L2, S, W.partial,
                                                         W.a1s, W.m2w, W.cnt, step_ctr);
  return hipGetLastError();
}

hipError_t launch_conv_bwd(const float* w2, const float* cond, const TrainWs& W, const float* g,
                           int g_stride, int B, int L, hipStream_t s) {
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  conv_bwd_kernel<<<dim3((unsigned)(B * S)), 256, 0, s>>>(w2, cond, W.a1s, W.m2w, g, g_stride, L, L1,
                                                        L2, S, W.gpart);
  return hipGetLastError();
}

}  // namespace

size_t train_ws_floats(int B, int L) { return ws_layout(B, L, true, nullptr, nullptr); }

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
  hipError_t e = launch_enc(w.enc0_w, w.enc0_b, w.enc2_w, w.enc2_b, cond, B, L, W, nullptr, s);
  if (e != hipSuccess) return e;
  train_head_kernel<0><<<B, 256, 0, s>>>(w, x_in, x0, noise, alpha_bar, t, freq, W.partial, S, L2,
                                         W.vec, eps_out, nullptr, 0.f, nullptr, HeadRng{});
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
  train_head_kernel<1><<<B, 256, 0, s>>>(w, nullptr, nullptr, noise, nullptr, nullptr, nullptr,
                                         nullptr, S, L2, W.vec, nullptr, dout, two_over_n, dx_out,
                                         HeadRng{});
  hipError_t e = launch_conv_bwd(w.enc2_w, cond, W, W.vec + TV_G, TV, B, L, s);
  if (e != hipSuccess) return e;
  FinalArgs a = final_args(W, B * S);
  set_dense(a, w, W, B, grads, loss_out);
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
  hipError_t e = launch_enc(w.enc0_w, w.enc0_b, w.enc2_w, w.enc2_b, cond, B, L, W, adam.step_dev, s);
  if (e != hipSuccess) return e;
  HeadRng rng{};
  if (adam.draw) {
    rng.seed = adam.seed;
    rng.step = adam.step_dev;
    rng.T = adam.T;
    rng.t_out = const_cast<int64_t*>(t);
    rng.noise_out = const_cast<float*>(noise);
  }
  train_head_kernel<2><<<B, 256, 0, s>>>(w, nullptr, x0, noise, alpha_bar, t, freq, W.partial, S, L2,
                                         W.vec, nullptr, nullptr, two_over_n, nullptr, rng);
  e = launch_conv_bwd(w.enc2_w, cond, W, W.vec + TV_G, TV, B, L, s);
  if (e != hipSuccess) return e;
  FinalArgs a = final_args(W, B * S);
  set_dense(a, w, W, B, grads, loss_out);
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
  return launch_enc(w1, b1, w2, b2, cond, B, L, W, nullptr, s);
}

hipError_t launch_encoder_conv_backward(const float* w2, const float* cond, const float* g, int B,
                                        int L, float* ws, float* dw1, float* db1, float* dw2,
                                        float* db2, hipStream_t s) {
  TrainWs W;
  ws_layout(B, L, false, ws, &W);
  const int L2 = conv_len(conv_len(L)), S = n_strips(L2);
  hipError_t e = launch_conv_bwd(w2, cond, W, g, C2, B, L, s);
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

}  // namespace ertd
