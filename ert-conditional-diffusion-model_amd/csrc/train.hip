// Training step on gfx950: ERT_Conditional_Diffusion.py:309-319
//   x_noisy = q_sample(x0, t, noise)               (:96-99, :314)
//   pred = model(x_noisy, t, cond)                  (:155-164, :315)
//   loss = MSELoss(pred, noise)  (mean)             (:295, :316)
//   loss.backward(); Adam(lr=1e-4).step()           (:294, :318-319)
//
// Kernels (all reductions in a fixed order: bitwise reproducible for any grid):
//   enc_fp32_kernel<true>   conv forward, stores a1 (conv1 act.) + m2 (conv2 ReLU mask)
//   train_head_fwd_kernel   per member: q_sample, pool, dense forward, saves vectors
//   train_head_bwd_kernel   per member: dout (MSE or given), dense backward to g = dm/L2
//   dense_grad_kernel       dW/db of the four Linear layers = sum_b dZ_b (x) IN_b, loss
//   conv_bwd_kernel         per (member, strip): dz2 = g*m2 -> da1 (transposed conv,
//                           MFMA) -> dz1; dW1 / dW2 / db partials (MFMA)
//   conv_grad_reduce_kernel partials -> dW1, dW2, db1, db2
//   adam_kernel             torch.optim.Adam update (lerp / addcmul / addcdiv form)
#include <cmath>

#include "ertd_common.h"

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
constexpr int NG = NG_B2 + C2;  // 7584

// ---------------------------------------------------------------------------
// head forward (one 256-thread block per member)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void train_head_fwd_kernel(
    ertd_weights w, const float* __restrict__ x_in, const float* __restrict__ x0,
    const float* __restrict__ noise, const float* __restrict__ alpha_bar,
    const int64_t* __restrict__ t_vec, const float* __restrict__ freq,
    const float* __restrict__ partial, int S, int L2, float* __restrict__ vec,
    float* __restrict__ eps_out) {
  __shared__ float m[C2], e[H], c[H], te[H], hc[PMAX + 2 * H], h[H];
  const int P = w.param_dim, b = blockIdx.x, tid = threadIdx.x;
  float* V = vec + (size_t)b * TV;
  const int64_t t = t_vec[b];
  if (tid < P) {
    float xv;
    if (x_in) {
      xv = x_in[(size_t)b * P + tid];
    } else {  // q_sample (:97-99): one rounding per op
      const float ab = alpha_bar[t];
      const float sa = sqrtf(ab), sb = sqrtf(1.0f - ab);
      xv = sa * x0[(size_t)b * P + tid] + sb * noise[(size_t)b * P + tid];
    }
    hc[tid] = xv;
  }
  if (tid < C2) {
    float acc = 0.f;
    for (int s = 0; s < S; ++s) acc += partial[((size_t)b * S + s) * C2 + tid];
    m[tid] = acc / (float)L2;
  }
  if (tid >= H) {
    const int k = tid - H;
    const float a = (float)t * freq[k < 64 ? k : k - 64];
    e[k] = k < 64 ? sinf(a) : cosf(a);
  }
  __syncthreads();
  if (tid < H) {  // cond_emb = relu(W3 m + b3)
    float acc = w.enc6_b[tid];
    for (int k = 0; k < C2; ++k) acc = fmaf(w.enc6_w[tid * C2 + k], m[k], acc);
    c[tid] = fmaxf(acc, 0.f);
  } else {  // t_emb = relu(Wt e + bt)
    const int j = tid - H;
    float acc = w.time_b[j];
    for (int k = 0; k < H; ++k) acc = fmaf(w.time_w[j * H + k], e[k], acc);
    te[j] = fmaxf(acc, 0.f);
  }
  __syncthreads();
  if (tid < H) {
    hc[P + tid] = te[tid];
    hc[P + H + tid] = c[tid];
  }
  __syncthreads();
  const int K0 = P + 2 * H;
  if (tid < H) {  // h = relu(W0 hcat + b0)
    float acc = w.mlp0_b[tid];
    const float* wr = w.mlp0_w + (size_t)tid * K0;
    for (int k = 0; k < K0; ++k) acc = fmaf(wr[k], hc[k], acc);
    h[tid] = fmaxf(acc, 0.f);
  }
  __syncthreads();
  if (tid < P) {  // eps = W2 h + b2
    float acc = w.mlp2_b[tid];
    for (int k = 0; k < H; ++k) acc = fmaf(w.mlp2_w[tid * H + k], h[k], acc);
    V[TV_EPS + tid] = acc;
    if (eps_out) eps_out[(size_t)b * P + tid] = acc;
  }
  for (int i = tid; i < K0; i += 256) V[TV_HCAT + i] = hc[i];
  if (tid < H) {
    V[TV_E + tid] = e[tid];
    V[TV_H + tid] = h[tid];
  }
  if (tid < C2) V[TV_M + tid] = m[tid];
}

// ---------------------------------------------------------------------------
// head backward (one 256-thread block per member)
//   dout: given (autograd) or MSE: (pred - noise) * (2/(B*P))   (mse_loss backward)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void train_head_bwd_kernel(
    ertd_weights w, const float* __restrict__ dout_in, const float* __restrict__ noise,
    float two_over_n, int L2, float* __restrict__ vec, float* __restrict__ dx_out) {
  __shared__ float dout[PMAX], dz5[H], dhc[2 * H], dz3[H];
  __shared__ float red[256];
  const int P = w.param_dim, b = blockIdx.x, tid = threadIdx.x;
  float* V = vec + (size_t)b * TV;
  if (tid < PMAX) {
    float d = 0.f, sq = 0.f;
    if (tid < P) {
      if (dout_in) {
        d = dout_in[(size_t)b * P + tid];
      } else {
        const float diff = V[TV_EPS + tid] - noise[(size_t)b * P + tid];
        sq = diff * diff;
        d = diff * two_over_n;
      }
    }
    dout[tid] = d;
    red[tid] = sq;
    V[TV_DOUT + tid] = d;
  }
  __syncthreads();
  if (tid == 0) {
    float acc = 0.f;
    for (int o = 0; o < P; ++o) acc += red[o];
    V[TV_SQ] = acc;
  }
  if (tid < H) {  // dz5 = (W2^T dout) * [h > 0]
    float acc = 0.f;
    for (int o = 0; o < P; ++o) acc = fmaf(w.mlp2_w[o * H + tid], dout[o], acc);
    const float d = V[TV_H + tid] > 0.f ? acc : 0.f;
    dz5[tid] = d;
    V[TV_DZ5 + tid] = d;
  }
  __syncthreads();
  const int K0 = P + 2 * H;
  {  // dhcat[P + k] for k < 256 (t_emb and cond_emb columns)
    float acc = 0.f;
    for (int j = 0; j < H; ++j) acc = fmaf(w.mlp0_w[(size_t)j * K0 + P + tid], dz5[j], acc);
    dhc[tid] = acc;
  }
  if (dx_out && tid < P) {  // dx = W0x^T dz5 (autograd w.r.t. the model input)
    float acc = 0.f;
    for (int j = 0; j < H; ++j) acc = fmaf(w.mlp0_w[(size_t)j * K0 + tid], dz5[j], acc);
    dx_out[(size_t)b * P + tid] = acc;
  }
  __syncthreads();
  if (tid < H) {
    const float te = V[TV_HCAT + P + tid];
    const float dz4 = te > 0.f ? dhc[tid] : 0.f;
    V[TV_DZ4 + tid] = dz4;
  } else {
    const int j = tid - H;
    const float c = V[TV_HCAT + P + H + j];
    const float d = c > 0.f ? dhc[tid] : 0.f;
    dz3[j] = d;
    V[TV_DZ3 + j] = d;
  }
  __syncthreads();
  if (tid < C2) {  // g = (W3^T dz3) / L2  (AdaptiveAvgPool backward)
    float acc = 0.f;
    for (int j = 0; j < H; ++j) acc = fmaf(w.enc6_w[j * C2 + tid], dz3[j], acc);
    V[TV_G + tid] = acc / (float)L2;
  }
}

// ---------------------------------------------------------------------------
// dense-layer gradients: one thread per output element, chain over members
// ---------------------------------------------------------------------------
struct DenseGradOut {
  float* w3; float* b3; float* wt; float* bt; float* w0; float* b0; float* w2; float* b2;
  float* loss;
};

__global__ __launch_bounds__(256) void dense_grad_kernel(const float* __restrict__ vec, int B, int P,
                                                         float inv_n, DenseGradOut g) {
  const int K0 = P + 2 * H;
  int i = blockIdx.x * 256 + threadIdx.x;
  int dz_off, in_off, kdim;
  float* dst;
  bool bias = false;
  if (i < H * C2) { dz_off = TV_DZ3; in_off = TV_M; kdim = C2; dst = g.w3; }
  else if ((i -= H * C2) < H) { dz_off = TV_DZ3; bias = true; dst = g.b3; kdim = 1; in_off = 0; }
  else if ((i -= H) < H * H) { dz_off = TV_DZ4; in_off = TV_E; kdim = H; dst = g.wt; }
  else if ((i -= H * H) < H) { dz_off = TV_DZ4; bias = true; dst = g.bt; kdim = 1; in_off = 0; }
  else if ((i -= H) < H * K0) { dz_off = TV_DZ5; in_off = TV_HCAT; kdim = K0; dst = g.w0; }
  else if ((i -= H * K0) < H) { dz_off = TV_DZ5; bias = true; dst = g.b0; kdim = 1; in_off = 0; }
  else if ((i -= H) < P * H) { dz_off = TV_DOUT; in_off = TV_H; kdim = H; dst = g.w2; }
  else if ((i -= P * H) < P) { dz_off = TV_DOUT; bias = true; dst = g.b2; kdim = 1; in_off = 0; }
  else if (i - P == 0) {  // loss = sum of squared errors / (B*P)
    if (!g.loss) return;      // autograd backward: the loss lives in torch
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += vec[(size_t)b * TV + TV_SQ];
    *g.loss = acc * inv_n;
    return;
  } else {
    return;
  }
  const int row = bias ? i : i / kdim, col = bias ? 0 : i - row * kdim;
  float acc = 0.f;
  for (int b = 0; b < B; ++b) {
    const float* V = vec + (size_t)b * TV;
    acc = bias ? acc + V[dz_off + row] : fmaf(V[dz_off + row], V[in_off + col], acc);
  }
  dst[i] = acc;
}

// ---------------------------------------------------------------------------
// conv backward, one 256-thread workgroup per (member, strip of J conv2 outputs)
// ---------------------------------------------------------------------------
constexpr int DZ2P = 65;   // dz2 row pitch (column reads conflict-free)
constexpr int DZ1P = 129;  // dz1 row pitch
struct ConvBwdSmem {
  union {
    float X[4][CIN][XS];   // cond image (forward's 4-phase layout) ...
    float red[4][32][33];  // ... reused for the cross-wave combine once dW1's MFMAs are done
  };
  float AE[C1][HS];        // a1 at p = 2m   (i = 2*j0 - 1 + p)
  float AO[C1][HS];        // a1 at p = 2m+1
  float DZ2[C2][DZ2P];     // dz2[o][q'], q' = j - j0 in [0, 64)
  float DZ1[C1][DZ1P];     // dz1[c][r],  r = i - 2*j0 in [0, 128)
};

__device__ __forceinline__ void store_tile_rows(float (*red)[33], const f32x16& acc, int h, int l32) {
#pragma unroll
  for (int r = 0; r < 16; ++r) red[(r & 3) + 8 * (r >> 2) + 4 * h][l32] = acc[r];
}

__global__ __launch_bounds__(256) void conv_bwd_kernel(
    const float* __restrict__ packed, const float* __restrict__ cond, const float* __restrict__ a1,
    const unsigned char* __restrict__ m2, const float* __restrict__ vec, int L, int L1, int L2,
    int S, float* __restrict__ gpart) {
  __shared__ ConvBwdSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int b = blockIdx.x / S, strip = blockIdx.x - b * S;
  const int j0 = strip * J;
  float* G = gpart + (size_t)blockIdx.x * NG;

  // ---- staging: cond image, a1 images, dz2 = g * m2 (q' = 63 is the next strip's halo)
  stage_cond_f32(sm.X, cond + (size_t)b * CIN * L, L, 4 * j0 - 3, tid);
  const float* a1b = a1 + (size_t)b * C1 * L1;
  for (int idx = tid; idx < C1 * 128; idx += 256) {
    const int c = idx >> 7, p = idx & 127;
    const int i = 2 * j0 - 1 + p;
    const float v = (i >= 0 && i < L1) ? a1b[(size_t)c * L1 + i] : 0.f;
    if (p & 1) sm.AO[c][p >> 1] = v;
    else sm.AE[c][p >> 1] = v;
  }
  const float* gv = vec + (size_t)b * TV + TV_G;
  for (int idx = tid; idx < C2 * DZ2P; idx += 256) {
    const int o = idx / DZ2P, q = idx - o * DZ2P;
    const int j = j0 + q;
    float v = 0.f;
    if (q < 64 && j < L2 && m2[((size_t)b * C2 + o) * L2 + j]) v = gv[o];
    sm.DZ2[o][q] = v;
  }
  __syncthreads();

  // ---- da1 (transposed conv2) -> dz1 over the owned conv1 positions i = 2*j0 + r
  //   r = 2m  : da1 = sum_o W2[o][c][1] dz2[o][m]
  //   r = 2m+1: da1 = sum_o W2[o][c][0] dz2[o][m+1] + W2[o][c][2] dz2[o][m]
  {
    const float* W2B = packed + PACK_W2B;
    const int odd = wave >> 1, mt = wave & 1;
    const int mcol = mt * 32 + l32;
    f32x16 acc = {};
    const float* db = &sm.DZ2[0][0] + h * DZ2P + mcol;
    if (!odd) {
#pragma unroll 8
      for (int s = 0; s < 32; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(W2B[(1 * 32 + s) * 64 + lane], db[2 * s * DZ2P],
                                                   acc, 0, 0, 0);
    } else {
#pragma unroll 8
      for (int s = 0; s < 32; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(W2B[(0 * 32 + s) * 64 + lane],
                                                   db[2 * s * DZ2P + 1], acc, 0, 0, 0);
#pragma unroll 8
      for (int s = 0; s < 32; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(W2B[(2 * 32 + s) * 64 + lane], db[2 * s * DZ2P],
                                                   acc, 0, 0, 0);
    }
    const int r = 2 * mcol + odd;
    const int i = 2 * j0 + r;
    const bool owned = r < 2 * J && i < L1;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int c = (k & 3) + 8 * (k >> 2) + 4 * h;
      const float act = odd ? sm.AE[c][mcol + 1] : sm.AO[c][mcol];  // a1 at p = r + 1
      sm.DZ1[c][r] = (owned && act > 0.f) ? acc[k] : 0.f;
    }
  }
  __syncthreads();

  // ---- dW1[o][n = c*3+kk] = sum_r dz1[o][r] * cond[c][4*j0 + 2r - 1 + kk]
  {
    const int nt = wave & 1, rh = wave >> 1;  // n-tile, r-half
    const int n = nt * 32 + l32;
    const bool nvalid = n < K1;
    const int c = nvalid ? n / 3 : 0, kk = nvalid ? n - 3 * (n / 3) : 0;
    const int u0 = 2 * h + 2 + kk;  // u = 4s + u0 for r = 2s + h
    const float* xb = &sm.X[u0 & 3][c][u0 >> 2];
    const float* zb = &sm.DZ1[l32][h];
    f32x16 acc = {};
#pragma unroll 8
    for (int s = rh * 32; s < rh * 32 + 32; ++s) {
      const float bv = nvalid ? xb[s] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(zb[2 * s], bv, acc, 0, 0, 0);
    }
    __syncthreads();  // X (aliased by red) fully read
    store_tile_rows(sm.red[wave], acc, h, l32);
  }
  __syncthreads();
  for (int idx = tid; idx < C1 * K1; idx += 256) {  // r-halves combined in order
    const int o = idx / K1, n = idx - o * K1;
    const int nt = n >> 5, col = n & 31;
    G[NG_W1 + idx] = sm.red[nt][o][col] + sm.red[2 + nt][o][col];
  }
  if (tid < C1) {
    float acc = 0.f;
    for (int r = 0; r < 2 * J; ++r) acc += sm.DZ1[tid][r];
    G[NG_B1 + tid] = acc;
  }
  if (tid >= 64 && tid < 64 + C2) {
    const int o = tid - 64;
    float acc = 0.f;
    for (int q = 0; q < J; ++q) acc += sm.DZ2[o][q];
    G[NG_B2 + o] = acc;
  }
  __syncthreads();

  // ---- dW2[o][n = c*3+kk] = sum_{q < J} dz2[o][q] * a1[c][p = 2q + kk]
  for (int tt = wave; tt < 6; tt += 4) {
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
}

__global__ __launch_bounds__(256) void conv_grad_reduce_kernel(const float* __restrict__ gpart,
                                                               int rows, float* __restrict__ dw1,
                                                               float* __restrict__ dw2,
                                                               float* __restrict__ db1,
                                                               float* __restrict__ db2) {
  __shared__ float red[8][32];
  const int col = blockIdx.x * 32 + (threadIdx.x & 31), grp = threadIdx.x >> 5;
  float acc = 0.f;
  if (col < NG)
    for (int r = grp; r < rows; r += 8) acc += gpart[(size_t)r * NG + col];
  red[grp][threadIdx.x & 31] = acc;
  __syncthreads();
  if (grp == 0 && col < NG) {
    float s = red[0][threadIdx.x];
#pragma unroll
    for (int g = 1; g < 8; ++g) s += red[g][threadIdx.x];
    if (col < NG_W2) dw1[col - NG_W1] = s;
    else if (col < NG_B1) dw2[col - NG_W2] = s;
    else if (col < NG_B2) db1[col - NG_B1] = s;
    else db2[col - NG_B2] = s;
  }
}

// ---------------------------------------------------------------------------
// Adam (torch.optim.Adam, no weight decay / amsgrad): 12 tensors in one launch
// ---------------------------------------------------------------------------
struct AdamArgs {
  float* p[12];
  const float* g[12];
  float* m[12];
  float* v[12];
  int n[12];
  int off[13];
  float one_minus_b1, b2, one_minus_b2, step_size_neg, bc2_sqrt, eps;
};

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.off[12]) return;
  int k = 0;
#pragma unroll
  for (int q = 1; q < 12; ++q) k += (i >= a.off[q]) ? 1 : 0;
  const int e = i - a.off[k];
  const float g = a.g[k][e];
  float m = a.m[k][e];
  m = m + a.one_minus_b1 * (g - m);                 // exp_avg.lerp_(grad, 1 - beta1)
  float v = a.v[k][e] * a.b2;                       // exp_avg_sq.mul_(beta2)
  v = v + a.one_minus_b2 * g * g;                   //   .addcmul_(grad, grad, 1 - beta2)
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  a.p[k][e] = a.p[k][e] + a.step_size_neg * (m / denom);  // param.addcdiv_(m, denom, -lr/bc1)
  a.m[k][e] = m;
  a.v[k][e] = v;
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
size_t train_ws_floats(int B, int L, int* offs) {
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  auto al = [](size_t n) { return (n + 63) / 64 * 64; };
  size_t o = 0;
  offs[0] = 0; o += al((size_t)B * S * C2);          // partial
  offs[1] = (int)o; o += al((size_t)B * C1 * L1);    // a1
  offs[2] = (int)o; o += al(((size_t)B * C2 * L2 + 3) / 4);  // m2 (bytes)
  offs[3] = (int)o; o += al((size_t)B * TV);         // vec
  offs[4] = (int)o; o += al((size_t)B * S * NG);     // conv gradient partials
  return o;
}

hipError_t launch_train_forward(const ertd_weights& w, const float* packed, const float* x_in,
                                const float* x0, const float* noise, const float* alpha_bar,
                                const int64_t* t, const float* cond, int B, int L,
                                const float* freq, float* eps_out, float* ws, hipStream_t s) {
  int off[5];
  train_ws_floats(B, L, off);
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  hipError_t e = launch_encoder_train(packed, w.enc0_b, w.enc2_b, cond, B, L, ws + off[0],
                                      ws + off[1], (unsigned char*)(ws + off[2]), s);
  if (e != hipSuccess) return e;
  train_head_fwd_kernel<<<B, 256, 0, s>>>(w, x_in, x0, noise, alpha_bar, t, freq, ws + off[0], S,
                                          L2, ws + off[3], eps_out);
  return hipGetLastError();
}

hipError_t launch_train_backward(const ertd_weights& w, const float* packed, const float* dout,
                                 const float* noise, const float* cond, int B, int L,
                                 float* const* grads, float* loss_out, float* dx_out, float* ws,
                                 hipStream_t s) {
  int off[5];
  train_ws_floats(B, L, off);
  const int P = w.param_dim;
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  const float two_over_n = (float)(2.0 / ((double)B * P));
  train_head_bwd_kernel<<<B, 256, 0, s>>>(w, dout, noise, two_over_n, L2, ws + off[3], dx_out);
  DenseGradOut g{grads[4], grads[5], grads[6], grads[7], grads[8], grads[9], grads[10], grads[11],
                 loss_out};
  const int nd = H * C2 + H + H * H + H + H * (P + 2 * H) + H + P * H + P + 1;
  dense_grad_kernel<<<(nd + 255) / 256, 256, 0, s>>>(ws + off[3], B, P,
                                                     (float)(1.0 / ((double)B * P)), g);
  conv_bwd_kernel<<<dim3((unsigned)(B * S)), 256, 0, s>>>(
      packed, cond, ws + off[1], (const unsigned char*)(ws + off[2]), ws + off[3], L, L1, L2, S,
      ws + off[4]);
  conv_grad_reduce_kernel<<<(NG + 31) / 32, 256, 0, s>>>(ws + off[4], B * S, grads[0], grads[2],
                                                         grads[1], grads[3]);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Encoder backward for another head (the U-Net's cond_proj): the conv part of
// the reference encoder's backward given g = dL/d(pool mean) / L2 per member
// (B, 64) -- the same conv_bwd / reduce kernels as the reference train step.
// ws: encoder_bwd_ws_floats(B, L) floats.
// ---------------------------------------------------------------------------
__global__ void put_g_kernel(const float* __restrict__ g, int B, float* __restrict__ vec) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * C2) return;
  const int b = i / C2, c = i - b * C2;
  vec[(size_t)b * TV + TV_G + c] = g[i];
}

size_t encoder_bwd_ws_floats(int B, int L) {
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  return ((size_t)B * TV + 63) / 64 * 64 + (size_t)B * S * NG;
}

hipError_t launch_encoder_conv_backward(const float* packed, const float* cond, const float* a1,
                                        const unsigned char* m2, const float* g, int B, int L,
                                        float* ws, float* dw1, float* db1, float* dw2, float* db2,
                                        hipStream_t s) {
  const int L1 = conv_len(L), L2 = conv_len(L1), S = n_strips(L2);
  float* vec = ws;
  float* gpart = ws + ((size_t)B * TV + 63) / 64 * 64;
  put_g_kernel<<<(B * C2 + 255) / 256, 256, 0, s>>>(g, B, vec);
  conv_bwd_kernel<<<dim3((unsigned)(B * S)), 256, 0, s>>>(packed, cond, a1, m2, vec, L, L1, L2, S,
                                                          gpart);
  conv_grad_reduce_kernel<<<(NG + 31) / 32, 256, 0, s>>>(gpart, B * S, dw1, dw2, db1, db2);
  return hipGetLastError();
}

hipError_t launch_adam(const ertd_weights& w, float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, int step, float lr, float beta1, float beta2,
                       float eps, hipStream_t s) {
  const int P = w.param_dim;
  const int sizes[12] = {C1 * K1, C1, C2 * K2, C2, H * C2, H, H * H, H, H * (P + 2 * H), H, P * H, P};
  const float* ps[12] = {w.enc0_w, w.enc0_b, w.enc2_w, w.enc2_b, w.enc6_w, w.enc6_b,
                         w.time_w, w.time_b, w.mlp0_w, w.mlp0_b, w.mlp2_w, w.mlp2_b};
  AdamArgs a{};
  int off = 0;
  for (int k = 0; k < 12; ++k) {
    a.p[k] = const_cast<float*>(ps[k]);
    a.g[k] = grads[k];
    a.m[k] = exp_avg[k];
    a.v[k] = exp_avg_sq[k];
    a.n[k] = sizes[k];
    a.off[k] = off;
    off += sizes[k];
  }
  a.off[12] = off;
  // scalars formed as torch does: Python floats (double), rounded when applied to fp32
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  a.one_minus_b1 = (float)(1.0 - (double)beta1);
  a.b2 = beta2;
  a.one_minus_b2 = (float)(1.0 - (double)beta2);
  a.step_size_neg = (float)(-((double)lr / bc1));
  a.bc2_sqrt = (float)std::sqrt(bc2);
  a.eps = eps;
  adam_kernel<<<(off + 255) / 256, 256, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace ertd
