// Shared device helpers and launch declarations for libertdiff_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "ertdiff.h"

namespace ertd {

// ---- model geometry (ERT_Conditional_Diffusion.py:133-153) -------------------
constexpr int CIN = 14;        // ERT surveys = Conv1d in_channels
constexpr int C1 = 32;         // conv1 out channels
constexpr int C2 = 64;         // conv2 out channels
constexpr int H = 128;         // hidden_dim
constexpr int PMAX = 32;       // largest supported param_dim
constexpr int K1 = CIN * 3;    // conv1 contraction (42)
constexpr int K2 = C1 * 3;     // conv2 contraction (96)

// ---- encoder strip geometry ---------------------------------------------------
// One workgroup (4 waves) turns a strip of J conv2 outputs of one member into a
// 64-channel partial pool sum.  conv2 output j needs conv1 outputs 2j-1..2j+1,
// which need cond positions 4j-3..4j+3, so a strip starting at j0 reads cond
// positions [4*j0-3, 4*j0-3+XU).
constexpr int J = 63;          // conv2 outputs per strip (64-wide MFMA tile, 1 pad row)
constexpr int XU = 4 * 65;     // cond positions staged per strip (260)
constexpr int XS = 68;         // LDS row stride of the 4-phase cond image (floats)
constexpr int HS = 68;         // LDS row stride of the conv1 even/odd images (floats)
constexpr int STEPS1 = K1 / 2; // 32x32x2 MFMA k-steps for conv1 (21)
constexpr int STEPS2 = K2 / 2; // ... for conv2 (48)
// packed fragment-order weights: W1f[21][64] then W2f[2][48][64] (floats)
constexpr int PACK_W1 = 0;
constexpr int PACK_W2 = STEPS1 * 64;
constexpr int PACK_FLOATS = PACK_W2 + 2 * STEPS2 * 64;
// bf16 packing (second region): W1h[3][64] x 8 bf16, W2h[2][6][64] x 8 bf16
constexpr int PACKH_OFF = PACK_FLOATS;                    // in floats
constexpr int PACKH_W1_STEPS = 3;                         // ceil(42/16)
constexpr int PACKH_W2_STEPS = 6;                         // 96/16
constexpr int PACKH_FLOATS = (PACKH_W1_STEPS + 2 * PACKH_W2_STEPS) * 64 * 4;  // 8 bf16 = 4 floats
constexpr int PACK_TOTAL = PACK_FLOATS + PACKH_FLOATS;

// ---- per-device host state ----------------------------------------------------
// A process may drive several GPUs (of different kinds) from several threads:
// the dynamic-LDS opt-in of a kernel and the CU count are kept per device.
constexpr int MAX_DEVICES = 64;
inline int current_device() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= MAX_DEVICES) d = 0;
  return d;
}
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device);
// `done` is the kernel's own flag word (one bit per device).  Two threads
// racing both set the attribute, which is idempotent.
inline void set_max_lds_once(const void* kernel, int bytes, std::atomic<unsigned long long>& done) {
  const unsigned long long bit = 1ull << current_device();
  if (done.load(std::memory_order_acquire) & bit) return;
  (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  done.fetch_or(bit, std::memory_order_acq_rel);
}
// compute units of the current device (grid sizing of persistent kernels)
inline int device_cu_count() {
  static std::atomic<int> cache[MAX_DEVICES];
  const int d = current_device();
  int n = cache[d].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n < 1) n = 256;
  cache[d].store(n, std::memory_order_relaxed);
  return n;
}

__host__ __device__ constexpr int conv_len(int L) { return (L - 1) / 2 + 1; }
__host__ __device__ constexpr int n_strips(int L2) { return (L2 + J - 1) / J; }

using f32x16 = __attribute__((ext_vector_type(16))) float;

// ---- Philox4x32-10 counter RNG --------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// Standard normal for element `o` of member `member` at step `t`.  Counter
// (o/4, member, t, tag), key = seed; Box-Muller on (x,y) and (z,w).
__device__ inline float philox_normal(uint64_t seed, uint32_t member, uint32_t t, uint32_t tag, int o) {
  const u32x4 r = philox4x32_10(u32x4{(uint32_t)(o >> 2), member, t, tag}, (uint32_t)seed,
                                (uint32_t)(seed >> 32));
  const bool second = (o & 2) != 0;
  const uint32_t a = second ? r.z : r.x;
  const uint32_t b = second ? r.w : r.y;
  const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0,1]
  const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);           // [0,1)
  const float rad = sqrtf(-2.0f * logf(u1));
  float s, c;
  sincospif(2.0f * u2, &s, &c);
  return (o & 1) ? rad * s : rad * c;
}

// Stage cond[b][:, pos0 : pos0+260] into X[u&3][c][u>>2] (zero outside [0,L)).
// Thread tid owns u = tid for all 14 channels (+ u = 256..259 on threads 0..55):
// every load is issued before the first LDS write.
template <typename Tx, typename Cvt>
__device__ __forceinline__ void stage_cond(Tx (*X)[CIN][XS], const float* __restrict__ cb, int L,
                                           int pos0, int tid, Cvt cvt) {
  // addresses are clamped into the row and the value selected afterwards:
  // unconditional loads, no branches (the loads may not be speculable)
  float v[CIN];
  const int pos = pos0 + tid;
  const bool in = pos >= 0 && pos < L;
  const int pc = pos < 0 ? 0 : (pos >= L ? L - 1 : pos);
#pragma unroll
  for (int c = 0; c < CIN; ++c) v[c] = cb[(size_t)c * L + pc];
#pragma unroll
  for (int c = 0; c < CIN; ++c) v[c] = in ? v[c] : 0.f;
  float vt = 0.f;
  const int tc = tid >> 2, tu = 256 + (tid & 3);
  if (tid < CIN * 4) {
    const int p2 = pos0 + tu;
    const int p2c = p2 < 0 ? 0 : (p2 >= L ? L - 1 : p2);
    vt = cb[(size_t)tc * L + p2c];
    vt = (p2 >= 0 && p2 < L) ? vt : 0.f;
  }
#pragma unroll
  for (int c = 0; c < CIN; ++c) X[tid & 3][c][tid >> 2] = cvt(v[c]);
  if (tid < CIN * 4) X[tu & 3][tc][tu >> 2] = cvt(vt);
}

// Time row with streamed weights (low register use; for blocks living inside a
// high-occupancy kernel).  Arithmetic identical to the split-k chain_half code
// of head.hip: thread (j = tid&127, q = tid>>7) runs acc = init; acc = fma(W, v,
// acc) over k in [64q, 64q+64) in order; outputs p0 + p1.  256 threads.
__device__ __forceinline__ void time_row_lean(const ertd_weights& w, const float* packed,
                                              const float* freq, int t, float* vrow, float* e,
                                              float* te, float (*part)[H], int tid) {
  const float* WtT = packed + PACK_TOTAL + C2 * H;
  const float* W0tT = WtT + H * H + (size_t)w.param_dim * H;
  const int j = tid & (H - 1), q = tid >> 7;
  if (q == 0) {
    constexpr int half = H / 2;
    const float a = (float)t * freq[j < half ? j : j - half];
    e[j] = j < half ? sinf(a) : cosf(a);
  }
  __syncthreads();
  float acc = q == 0 ? w.time_b[j] : 0.f;
#pragma unroll 8
  for (int k = 0; k < H / 2; ++k) acc = fmaf(WtT[(q * (H / 2) + k) * H + j], e[q * (H / 2) + k], acc);
  part[q][j] = acc;
  __syncthreads();
  if (tid < H) te[j] = fmaxf(part[0][j] + part[1][j], 0.f);
  __syncthreads();
  acc = 0.f;
#pragma unroll 8
  for (int k = 0; k < H / 2; ++k) acc = fmaf(W0tT[(q * (H / 2) + k) * H + j], te[q * (H / 2) + k], acc);
  part[q][j] = acc;
  __syncthreads();
  if (tid < H) vrow[j] = part[0][j] + part[1][j];
}

__device__ __forceinline__ void stage_cond_f32(float (*X)[CIN][XS], const float* __restrict__ cb,
                                               int L, int pos0, int tid) {
  stage_cond(X, cb, L, pos0, tid, [](float v) { return v; });
}

// ---- launch declarations (defined in encoder.hip / head.hip / train.hip) ------
// `packed` is the ertd_pack_weights() buffer (conv fragments + k-major dense weights).
constexpr int DENSE_FLOATS = C2 * H + H * H + (PMAX + 2 * H) * H;
// conv2 transposed-conv fragments for the backward (train.hip):
// W2B[kk][s][lane] = W2[o = 2s + (lane>>5)][c = lane&31][kk]
constexpr int PACK_W2B = PACK_TOTAL + DENSE_FLOATS;
constexpr int W2B_FLOATS = 3 * 32 * 64;
// mlp.2 in step-lane order: W2F[k][lane] = W2[lane>>1][64*(lane&1) + k] (0 for o >= P)
constexpr int PACK_W2F = PACK_W2B + W2B_FLOATS;
constexpr int W2F_FLOATS = (H / 2) * 64;
// Step-body LDS images (copied verbatim into LDS, read with ds_read_b128,
// conflict-free): W0XR[j][k] = W0[j][k] (k < P, row pitch 36) and
// W2L[lane][k] = W2[lane>>1][64*(lane&1) + k] (row pitch 68).
constexpr int W0XR_PITCH = 36;
constexpr int W2L_PITCH = 68;
constexpr int PACK_W0XR = PACK_W2F + W2F_FLOATS;
constexpr int W0XR_FLOATS = H * W0XR_PITCH;
constexpr int PACK_W2L = PACK_W0XR + W0XR_FLOATS;
constexpr int W2L_FLOATS = 64 * W2L_PITCH;
constexpr int PACKED_FLOATS_ALL = PACK_W2L + W2L_FLOATS;

hipError_t launch_pack(const ertd_weights& w, float* packed, hipStream_t s);
// the U-Net train step's encoder weights: W1 raw at packed[0], W2 raw at packed[ENC_RAW_W2]
constexpr int ENC_RAW_W2 = C1 * K1;
hipError_t launch_pack_encoder_convs(const float* w0, const float* w2, float* packed, hipStream_t s);
// ncond > 0: member b reads condition row b % ncond (a many-condition launch,
// ertd_sample_conditions); 0: row b
hipError_t launch_encoder_strips(const float* packed, const float* b1, const float* b2,
                                 const float* cond, long long cstride, int B, int L,
                                 int precision, float* partial, hipStream_t s, int ncond = 0);
// Same, plus one extra block computing the time row v(t) = W0t.relu(Wt.e(t)+bt)
// into V[t] (faithful sampler: the row the next head_step launch consumes).
// Member b of a many-condition launch (ertd_sample_conditions): realisation
// r = b / ncond of local condition b % ncond; its Philox member id is
// member_offset + r * id_period + b % ncond (id_period = the global condition
// count, so a rank holding a slice of the conditions keeps every member's
// global id).  ncond <= 0: a plain launch, id = member_offset + b.
__host__ __device__ inline uint32_t member_id(uint32_t member_offset, int b, int ncond, int id_period) {
  if (ncond <= 0) return member_offset + (uint32_t)b;
  const int r = b / ncond;
  return member_offset + (uint32_t)r * (uint32_t)id_period + (uint32_t)(b - r * ncond);
}
__host__ __device__ inline int cond_row(int b, int ncond) { return ncond > 0 ? b % ncond : b; }
struct TimeRowArgs {
  ertd_weights w;
  const float* freq;
  int t;
  float* V;
};
hipError_t launch_encoder_strips_t(const float* packed, const float* b1, const float* b2,
                                   const float* cond, long long cstride, int B, int L,
                                   int precision, float* partial, const TimeRowArgs& tr,
                                   hipStream_t s, int ncond = 0);
struct HeadArgs {
  const float* partial; int S; int L2;
  const float* freq;
  const float* x_in; const int64_t* t_vec; int t_scalar;
  const float* c1; const float* c2; const float* sigma; const float* noise;
  int num_steps; uint64_t seed; uint32_t member_offset; int B;
  float* x_out; float* eps_out; float* cond_emb_out; float* t_emb_out;
  int ncond; int id_period;      // Philox ids of a many-condition launch (member_id); 0 = plain
};
hipError_t launch_head(const ertd_weights& w, const float* packed, const HeadArgs& a, hipStream_t s);
// faithful step: per-member condition branch + step for a.t_scalar using V[t]
hipError_t launch_head_step(const ertd_weights& w, const float* packed, const HeadArgs& a,
                            const float* V, hipStream_t s);
hipError_t launch_hoist_prep(const ertd_weights& w, const float* packed, const float* partial,
                             int S, int L2, int B, float* U, float* cond_emb_out, hipStream_t s);
hipError_t launch_time_table(const ertd_weights& w, const float* packed, const float* freq,
                             int t_lo, int n, float* V, hipStream_t s);
hipError_t launch_hoisted_sampler(const ertd_weights& w, const float* packed, const float* U,
                                  const float* V, const float* c1, const float* c2,
                                  const float* sigma, const float* noise, int num_steps,
                                  int t_first, int n_run, uint64_t seed, uint32_t member_offset,
                                  int B, float* x, hipStream_t s, int ncond = 0, int id_period = 0,
                                  int u_rows = 0);
hipError_t launch_timestep_embedding(const int64_t* t, int B, int dim, const float* freq,
                                     float* out, hipStream_t s);
hipError_t launch_q_sample(const float* x0, const int64_t* t, const float* noise,
                           const float* alpha_bar, int B, int P, float* out, hipStream_t s);
hipError_t launch_postproc(const float* u, long long rows, int P, float a, float bma,
                           const double* min_, const double* scale_, const double* limits,
                           float* out, uint8_t* valid, hipStream_t s);
hipError_t launch_philox_normal(uint64_t seed, uint32_t member_offset, int B, int P, int t,
                                int tag, float* out, hipStream_t s);
// chain.hip: persistent faithful sampler (one launch per chain)
struct FaithfulChainArgs {
  const float* cond; long long cstride; int L; int B; int S; int R;
  int n_run; int t_first; int num_steps;
  const float* c1; const float* c2; const float* sigma; const float* freq; const float* noise;
  uint64_t seed; uint32_t member_offset;
  int ncond; int id_period;      // condition row b % ncond, Philox member_id (0 = plain)
  float* x;                      // (B, P) in/out
  float* part;                   // R ring slots of (B, S, 64) strip partials
  // sync words, one per SYNC_PAD-word line:
  unsigned* cnt;                 // (R, B) monotonic strip arrival counters
  unsigned* progress;            // (B) steps consumed by each chain
  unsigned* claim;               // (B) next strip item of each member (worker tickets)
  unsigned* status;              // 0 = ok, else the code of the wait that timed out
  unsigned* uflag;               // (R, B) step+1 of the u row in each ring slot
  unsigned* vready;              // (1) time rows published so far
  float* uring;                  // (R, B, 128) condition rows u_i[b]
  float* V;                      // (n_run, 128) time rows v(t_first - i)
};
#ifndef ERTD_CHAIN_RING
#define ERTD_CHAIN_RING 16  // (a -D override is for same-box variant A/Bs only)
#endif
constexpr int CHAIN_RING = ERTD_CHAIN_RING;
// Every sync word of the chain sits alone in a 128-B line: words polled or
// updated by hundreds of blocks serialize per line (measured: progress words
// of 16 members sharing one line slowed every memory access on the chip 3-5x).
constexpr int SYNC_PAD = 32;
// grid for launch_faithful_chain (0: B too large for a resident grid)
int faithful_chain_grid(int B, int S);
// false where faithful_chain_grid(B, .) is 0 on any gfx950 device (device-
// independent: sizes the sampler workspace's ring and sync block)
bool faithful_chain_may_run(int B);
hipError_t launch_zero_words(unsigned* p, size_t n, hipStream_t s);
hipError_t launch_faithful_chain(const ertd_weights& w, const float* packed,
                                 const FaithfulChainArgs& a, int grid, hipStream_t s);
// train.hip (every kernel reads the parameters of w in place: no packing)
size_t train_ws_floats(int B, int L);
// Adam hyper-parameters of a train step: host scalars (table == nullptr), or
// the device step counter *step_dev (advanced by the step itself) indexing a
// table of adam_table_host() entries for steps [table_first, table_first + table_len)
// draw != 0 (with step_dev): the step draws t ~ U{0..T-1} and noise ~ N(0,1)
// itself (Philox keyed (seed, member, step)) into the t / noise buffers
struct TrainAdam {
  int step; float lr, beta1, beta2, eps;
  const float* table; int* step_dev; int table_first, table_len;
  uint64_t seed; int draw; int T;
};
constexpr int ADAM_TABLE_FLOATS = 6;  // floats per step entry
void adam_table_host(int step_first, int n, float lr, float beta1, float beta2, float eps, float* out);
hipError_t launch_train_conv_backward(const float* cond, int B, int L, float* ws, hipStream_t s);
hipError_t launch_train_forward(const ertd_weights& w, const float* x_in, const float* x0,
                                const float* noise, const float* alpha_bar, const int64_t* t,
                                const float* cond, int B, int L, const float* freq, float* eps_out,
                                float* ws, hipStream_t s);
hipError_t launch_train_backward(const ertd_weights& w, const float* dout, const float* noise,
                                 const float* cond, int B, int L, float* const* grads,
                                 float* loss_out, float* dx_out, float* ws, hipStream_t s);
hipError_t launch_train_step(const ertd_weights& w, const float* x0, const int64_t* t,
                             const float* noise, const float* cond, const float* alpha_bar, int B,
                             int L, const float* freq, float* const* grads, float* const* exp_avg,
                             float* const* exp_avg_sq, const TrainAdam& adam, float* loss_out,
                             float* ws, hipStream_t s);
hipError_t launch_adam(const ertd_weights& w, float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, int step, float lr, float beta1, float beta2,
                       float eps, hipStream_t s);
// the reference condition encoder alone (the U-Net's condition branch): forward
// with saved activations (partial_out = the (B, S, 64) pool partials in ws) and
// the conv-parameter backward from g = dL/dm / L2 (B, 64); raw weights w1 (32,14,3), w2 (64,32,3)
size_t encoder_train_ws_floats(int B, int L);
hipError_t launch_encoder_train(const float* w1, const float* b1, const float* w2, const float* b2,
                                const float* cond, int B, int L, float* ws, float** partial_out,
                                hipStream_t s);
hipError_t launch_encoder_conv_backward(const float* w2, const float* cond, const float* g, int B,
                                        int L, float* ws, float* dw1, float* db1, float* dw2,
                                        float* db2, hipStream_t s);

}  // namespace ertd
