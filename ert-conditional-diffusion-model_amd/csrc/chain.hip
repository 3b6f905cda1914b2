// Persistent faithful sampler: the whole T-step chain of sample_model
// (ERT_Conditional_Diffusion.py:102-119) in ONE launch, the full model
// evaluated at every step as the reference does.
//
// The encoder's output does not depend on x, only the step body does.  So
// instead of encoder(t) -> head(t) -> encoder(t-1) ... as 2T dependent
// launches, one launch runs three roles side by side:
//
//   chain blocks   (block b < B)   member b's x-chain: per step, wait for the
//                                  step's condition row u_i[b] and time row
//                                  v(t), then mlp.0 x-part -> ReLU -> mlp.2
//                                  -> DDPM update.  x stays on chip.
//   time-row block (block B)       v(t) = W0t.relu(Wt.e(t) + bt) for every
//                                  step of the call in order, published as
//                                  it goes (identical for all members).
//   worker blocks  (the rest)      member-affine: the workers w with
//                                  w % B == b run member b's encoder strips
//                                  (enc_strip.h) of every step, claimed in
//                                  step-major order from a per-member ticket
//                                  counter (one claim in flight ahead).  The
//                                  last of a step's S strips to arrive
//                                  reduces the pool partials and computes the
//                                  condition row u_i[b] (pool -> Linear ->
//                                  ReLU -> W0c).
//
// Members never share a worker, so a stalled member pipeline cannot hold up
// another one (a step-major round-robin over all members did: one blocked
// worker delayed other members' strips, whose chains then stalled more
// workers -- measured as 180-340 us convoys).  Claims rather than a static
// split: with a static split one slow worker per member held every step, and
// as the last arriver it also took every condition row, so it stayed last.
//
// Workers run up to R steps ahead of the chains (ring slots i % R for the
// partials and u); a worker about to overwrite slot i % R for member b waits
// until chain b has consumed step i - R.  Deadlock-free for any timing as long
// as every block is resident: the grid is sized from the occupancy query with
// a one-block-per-CU margin, and every spin is bounded (a timeout sets the
// status word and every waiter gives up, so the launch always drains).
//
// Hand-offs (cdna_hip_programming.md Guideline 16):
//   strip partials -> last arriver: write-through (sc1) stores drained by
//     every storing wave, a relaxed arrival counter; the last arriver reads
//     them with sc1 loads (no fences: Guideline 16, form R1).
//   u_i[b], v(t) -> chain: write-through (sc1) row stores drained by every
//     storing wave, a barrier, then ONE flag word (u: per slot and member,
//     tag = step + 1; v: a monotonic count of published rows).  One lane of
//     the chain polls the flag word(s); the rows are read with sc1 loads.
//     (Per-lane granule polling was tried: 128 lanes x 64 chains re-reading
//     8-byte tags every ~100 clocks is ~1 TB/s of poll traffic.)
//   chain progress -> workers: relaxed store / relaxed poll (no payload).
//
// Arithmetic: the strip, pool, condition row, time row and step body use the
// same fma chains in the same order as the per-step kernels and the hoisted
// sampler, so all faithful schedules and the hoisted mode are bit-identical.
#include "enc_strip.h"
#include "head_dev.h"

namespace ertd {

namespace {

typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

#ifndef CHAIN_MAX_BPC
#define CHAIN_MAX_BPC 5  // resident blocks per CU used at most
#endif
// strips per claimed work item: a worker runs SPI consecutive strips of one
// (member, step) back to back and publishes them with ONE drain + arrival
// (the publish -- write-through stores, vmcnt(0), a barrier, an atomic round
// trip -- cost ~1.4 us per strip, ~10 % of a worker's time, at SPI = 1)
#ifndef CHAIN_SPI
#define CHAIN_SPI 2
#endif
// members per chain block: a member's step body is ~1.5 us of a ~15 us step,
// so one block runs the steps of CHAIN_MPB members in turn and the slots the
// other chain blocks would hold go to strip workers
#ifndef CHAIN_MPB
#define CHAIN_MPB 2
#endif
constexpr uint64_t SPIN_TIMEOUT_TICKS = 50000000ull;  // 0.5 s of s_memrealtime (100 MHz)

// A zero the compiler cannot see through: loads addressed with it stay inside
// the worker loop instead of being hoisted (and held in registers) across items.
__device__ __forceinline__ int opaque0() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}

__device__ __forceinline__ int opaque_tid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"((int)threadIdx.x));
  return t;
}

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ unsigned ld_relaxed(unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// write-through (sc1) 4-byte store / load: the hand-off of the strip partials
struct Sc1Load {
  __device__ float operator()(const float* p) const {
    return __uint_as_float(__hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
};
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Spin (one lane) until *word >= target; `seen` gets the value observed.
// fast = 1: latency-critical waiter (a chain), short sleeps.  fast = 0: a
// worker held by the ring, backing off to ~4 us between polls -- hundreds of
// idle workers polling at full rate slow every memory access on the chip.
// false: timed out or aborted.
__device__ bool wait_ge(unsigned* word, unsigned target, unsigned* status, unsigned code,
                        unsigned& seen, int fast) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned n = 0;; ++n) {
    seen = ld_relaxed(word);
    if (seen >= target) return true;
    if ((n & 15) == 15) {
      if (ld_relaxed(status) != 0) return false;
      if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TIMEOUT_TICKS) {
        atomicCAS(status, 0u, code);
        return false;
      }
    }
    if (fast || n < 2) __builtin_amdgcn_s_sleep(2);
    else if (n < 8) __builtin_amdgcn_s_sleep(16);
    else __builtin_amdgcn_s_sleep(127);  // 127 x 64 clocks
  }
}

// chain_half with the weights streamed from L2 in batches of 16 (same fma
// order; a rolled loop, so one batch of weights and operands is live).
template <int N>
__device__ __forceinline__ float chain_half_stream(const float* __restrict__ WT, const float* v,
                                                   float init, int j, int q) {
  constexpr int BATCH = 16;
  const float* src = WT + (size_t)(q * (N / 2)) * H + j;
  float acc = init;
#pragma unroll 1
  for (int kb = 0; kb < N / 2; kb += BATCH) {
    const float* bsrc = src + opaque0();  // not hoistable above this batch
    float wv[BATCH];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) wv[k] = bsrc[(size_t)(kb + k) * H];
#pragma unroll
    for (int k = 0; k < BATCH; ++k) acc = fmaf(wv[k], v[q * (N / 2) + kb + k], acc);
  }
  return acc;
}

// time_row_lean's arithmetic (same chains) with bounded register use:
// vrow[j] = W0t.relu(Wt.e(t) + bt), 256 threads, scratch f[4*H].
__device__ __forceinline__ void time_row_stream(const ertd_weights& w, const float* packed,
                                                const float* freq, int t, float* vrow, float* f,
                                                int tid) {
  float* e = f;
  float* te = f + H;
  float(*part)[H] = reinterpret_cast<float(*)[H]>(f + 2 * H);
  const float* WtT = packed + PACK_TOTAL + C2 * H;
  const float* W0tT = WtT + H * H + (size_t)w.param_dim * H;
  const int j = tid & (H - 1), q = tid >> 7;
  if (q == 0) {
    constexpr int half = H / 2;
    const float ang = (float)t * freq[j < half ? j : j - half];
    e[j] = j < half ? sinf(ang) : cosf(ang);
  }
  __syncthreads();
  part[q][j] = chain_half_stream<H>(WtT, e, q == 0 ? w.time_b[j] : 0.f, j, q);
  __syncthreads();
  if (tid < H) te[j] = fmaxf(part[0][j] + part[1][j], 0.f);
  __syncthreads();
  part[q][j] = chain_half_stream<H>(W0tT, te, 0.f, j, q);
  __syncthreads();
  if (tid < H) vrow[j] = part[0][j] + part[1][j];
}

// Phase stamps for the diagnostic build only (tools/diag_chain.hip defines
// ERTD_CHAIN_STAMPS): chain blocks 0..7 stamp every step, worker tid 0
// accumulates time per phase.  Compiled out of the library.
#ifdef ERTD_CHAIN_STAMPS
__device__ unsigned long long g_cst[8][1024][3];
__device__ unsigned long long g_wacc[2048][8];
__device__ unsigned long long g_pub[1024][3];
__device__ unsigned long long g_item[4096][4];  // member 0 items: start, polled-done, strip done, published  // step i: v published, u[0] published, v worker id
#define CST(k)                                                              \
  do {                                                                      \
    if (tid == 0 && b < 8 && i < 1024) g_cst[b][i][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define WT0() const unsigned long long wt0_ = __builtin_amdgcn_s_memrealtime()
#define WACC(k, t0) \
  do {              \
    if (tid == 0) wacc[k] += __builtin_amdgcn_s_memrealtime() - (t0); \
  } while (0)
#else
#define CST(k) do {} while (0)
#define WT0() do {} while (0)
#define WACC(k, t0) do {} while (0)
#endif

struct ChainStepSmem {
  float w[H];
  alignas(16) float h[H];
  float x[CHAIN_MPB][PMAX];
};
struct ChainSmem {
  union {
    EncSmem enc;
    CondScratch cond;
    float trow[5 * H];  // time row scratch: e | te | part[2] | v
    ChainStepSmem step;
  };
  int flag;   // chain: per-step abort vote; worker: "this block arrived last"
  int abort;  // worker: set once, never cleared
  int seen;   // worker: chain progress last observed by lane 0 (written before a barrier)
  int next;   // worker: the item claimed for after the current one
  float keep[CHAIN_SPI][C2];  // worker: each strip's channel sums until the item's publish
};

}  // namespace

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void faithful_chain_kernel(ertd_weights w,
                                                             const float* __restrict__ packed,
                                                             FaithfulChainArgs a) {
  __shared__ ChainSmem sm;
  const int tid = threadIdx.x;
  const int P = w.param_dim, B = a.B, S = a.S, R = a.R;
  const size_t ring_part = (size_t)B * S * C2;  // floats per ring slot

  const int NCH = (B + CHAIN_MPB - 1) / CHAIN_MPB;   // chain blocks
  if ((int)blockIdx.x < NCH) {
    // ============ chain block: members b0 .. b0 + nm - 1, one step each in turn ============
    const int b0 = blockIdx.x * CHAIN_MPB;
    const int nm = B - b0 < CHAIN_MPB ? B - b0 : CHAIN_MPB;
    const int xj = tid >> 1, xc = tid & 1;                             // mlp.0 x-part
    const int eo = tid >> 3, ehf = (tid >> 2) & 1, ei = tid & 3;       // mlp.2 chains
    const bool updater = ehf == 0 && ei == 0 && eo < P;
    // this thread's mlp.0 x-part row slice and mlp.2 chain slice (16 floats
    // each, 16-B aligned image rows), re-read from L2 every step: holding
    // them would cost 32 registers in every role of this kernel
    const float4* wx_src = reinterpret_cast<const float4*>(packed + PACK_W0XR + xj * W0XR_PITCH + 16 * xc);
    const float4* w2_src = reinterpret_cast<const float4*>(packed + PACK_W2L + (2 * eo + ehf) * W2L_PITCH + 16 * ei);
    const float bo = eo < P ? w.mlp2_b[eo] : 0.f;
    float xv[CHAIN_MPB];
#pragma unroll
    for (int m = 0; m < CHAIN_MPB; ++m) {
      xv[m] = updater && m < nm ? a.x[(size_t)(b0 + m) * P + eo] : 0.f;
      if (tid < P && m < nm) sm.step.x[m][tid] = a.x[(size_t)(b0 + m) * P + tid];
    }
    unsigned vseen = 0;  // lane 0: time rows known to be published
    __syncthreads();
    for (int i = 0; i < a.n_run; ++i) {
      const int t = a.t_first - i;
      const int slot = i % R;
      float c1 = 0.f, c2 = 0.f, sig = 0.f;
      if (updater) {
        c1 = a.c1[t];
        c2 = a.c2[t];
        sig = a.sigma[t];
      }
#pragma unroll
      for (int m = 0; m < CHAIN_MPB; ++m) {
        if (m >= nm) break;
        const int b = b0 + m;
        // inputs that do not depend on this step's u (noise first: its Philox
        // and Box-Muller temporaries are dead before the x-part operands load)
        const float z = updater ? step_noise(a.noise, a.num_steps, t, B, b, P, eo, a.seed,
                                             member_id(a.member_offset, b, a.ncond, a.id_period))
                                : 0.f;
        float wx[16];
        {
          const float4* src = wx_src + opaque0();
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const float4 v4 = src[q4];
            wx[4 * q4] = v4.x;
            wx[4 * q4 + 1] = v4.y;
            wx[4 * q4 + 2] = v4.z;
            wx[4 * q4 + 3] = v4.w;
          }
        }
        float xs[16];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) xs[kk] = (16 * xc + kk < P) ? sm.step.x[m][16 * xc + kk] : 0.f;
        float bsum = 0.f;  // second x-part chain (k >= 16), from zero
        if (xc == 1) {
#pragma unroll
          for (int kk = 0; kk < 16; ++kk)
            if (16 + kk < P) bsum = fmaf(wx[kk], xs[kk], bsum);
        }
        // this step's condition row and time row: lane 0 polls the two flags
        CST(0);
        if (tid == 0) {
          bool ok = true;
          if (vseen < (unsigned)(i + 1)) ok = wait_ge(a.vready, (unsigned)(i + 1), a.status, 1u, vseen, 1);
          unsigned useen = 0;
          if (ok) ok = wait_ge(a.uflag + ((size_t)slot * B + b) * SYNC_PAD, (unsigned)(i + 1), a.status, 1u, useen, 1);
          sm.flag = ok ? 0 : 1;
        }
        __syncthreads();
        if (sm.flag) return;  // aborted: every waiter gives up
        if (tid < H) {
          const float u = Sc1Load()(a.uring + ((size_t)slot * B + b) * H + tid);
          const float v = Sc1Load()(a.V + (size_t)i * H + tid);
          sm.step.w[tid] = u + v;
        }
        __syncthreads();
        CST(1);
        if (tid == 0) st_relaxed(a.progress + (size_t)b * SYNC_PAD, (unsigned)(i + 1));  // slot i%R consumed
        // mlp.0: h_j = relu((w_j + W0x[j][0:16].x) + W0x[j][16:P].x)
        float av = bsum;
        if (xc == 0) {
          av = sm.step.w[xj];
#pragma unroll
          for (int kk = 0; kk < 16; ++kk)
            if (kk < P) av = fmaf(wx[kk], xs[kk], av);
        }
        const float other = __shfl_xor(av, 1);
        if (xc == 0) sm.step.h[xj] = fmaxf(av + other, 0.f);
        float w2[16];
        {
          const float4* src = w2_src + opaque0();
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const float4 v4 = src[q4];
            w2[4 * q4] = v4.x;
            w2[4 * q4 + 1] = v4.y;
            w2[4 * q4 + 2] = v4.z;
            w2[4 * q4 + 3] = v4.w;
          }
        }
        __syncthreads();
        // mlp.2: four 16-term chains per k-half, joined (c0+c1)+(c2+c3), halves added
        const float4* h4 = reinterpret_cast<const float4*>(sm.step.h + 64 * ehf + 16 * ei);
        float hv[16];
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const float4 v4 = h4[q4];
          hv[4 * q4] = v4.x;
          hv[4 * q4 + 1] = v4.y;
          hv[4 * q4 + 2] = v4.z;
          hv[4 * q4 + 3] = v4.w;
        }
        float c = 0.f;
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) c = fmaf(w2[kk], hv[kk], c);
        const float s1 = c + __shfl_xor(c, 1);
        const float s2 = s1 + __shfl_xor(s1, 2);
        const float e = s2 + __shfl_xor(s2, 4);
        if (updater) {
          xv[m] = ddpm_update(xv[m], e + bo, c1, c2, sig, z, t > 0);
          sm.step.x[m][eo] = xv[m];
        }
        __syncthreads();
        CST(2);
      }
    }
#pragma unroll
    for (int m = 0; m < CHAIN_MPB; ++m)
      if (updater && m < nm) a.x[(size_t)(b0 + m) * P + eo] = xv[m];
    return;
  }

  if ((int)blockIdx.x == NCH) {
    // ======================= time-row block =======================
    for (int i = 0; i < a.n_run; ++i) {
      float* f = sm.trow;
      time_row_stream(w, packed + opaque0(), a.freq, a.t_first - i, f + 4 * H, f, opaque_tid());
      __syncthreads();
      if (tid < H) st_sc1(a.V + (size_t)i * H + tid, f[4 * H + tid]);
      drain();
      __syncthreads();
      if (tid == 0) st_relaxed(a.vready, (unsigned)(i + 1));
    }
    return;
  }

  // ======================= worker block =======================
  if (tid == 0) {
    sm.abort = 0;
    sm.seen = 0;
  }
  unsigned seen_reg = 0;  // lane 0's copy
  __syncthreads();
  const int wid = blockIdx.x - NCH - 1;
  const int b = wid % B;
  const int NPS = (S + CHAIN_SPI - 1) / CHAIN_SPI;   // work items per step
  const unsigned n_items = (unsigned)a.n_run * (unsigned)NPS;
  const int L1 = conv_len(a.L), L2 = conv_len(L1);
  gu32* claim = (gu32*)(a.claim + (size_t)b * SYNC_PAD);
  if (tid == 0)
    sm.next = (int)__hip_atomic_fetch_add(claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
#ifdef ERTD_CHAIN_STAMPS
  unsigned long long wacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long wstart = __builtin_amdgcn_s_memrealtime();
#endif
  for (unsigned item = (unsigned)sm.next; item < n_items; item = (unsigned)sm.next) {
    // claim the following item now; its ticket returns while this one runs
    unsigned nxt = 0;
    if (tid == 0) nxt = __hip_atomic_fetch_add(claim, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int i = (int)(item / (unsigned)NPS);
    const int s0 = (int)(item - (unsigned)i * NPS) * CHAIN_SPI;
    const int ns = S - s0 < CHAIN_SPI ? S - s0 : CHAIN_SPI;   // strips of this item
    const int z0 = opaque0();
    const int tid_i = opaque_tid();
    const float* pk = packed + z0;
    WT0();
    const int slot = i % R;
    // slot i%R of member b is free once chain b has consumed step i-R.  The
    // progress word is re-read with every arrival (below), so the poll (a
    // memory round trip and a barrier) runs only when that copy is too old.
#ifdef ERTD_CHAIN_STAMPS
    if (tid == 0 && b == 0 && item < 4096) g_item[item][0] = __builtin_amdgcn_s_memrealtime();
#endif
    if (i >= R && sm.seen < i - R + 1) {
#ifdef ERTD_CHAIN_STAMPS
      if (tid == 0) wacc[0] += 1;
#endif
      if (tid == 0 && !wait_ge(a.progress + (size_t)b * SYNC_PAD, (unsigned)(i - R + 1), a.status, 2u, seen_reg, 0))
        sm.abort = 1;
      __syncthreads();
      if (sm.abort) return;
    }
    WACC(1, wt0_);
#ifdef ERTD_CHAIN_STAMPS
    const unsigned long long wt1_ = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && b == 0 && item < 4096) g_item[item][1] = wt1_;
#endif
    // one inlined strip body (a second inlined copy spills), run ns times,
    // with fresh opaque offsets so its weight loads are not hoisted out of the
    // loop; keep[u][tid] is written and later read by the same thread
#pragma unroll 1
    for (int u = 0; u < ns; ++u) {
      const int zu = opaque0(), tu = opaque_tid();
      enc_strip_fp32(sm.enc, packed + zu, w.enc0_b + zu, w.enc2_b + zu, a.cond, a.cstride, a.L, L1, L2, b,
                     cond_row(b, a.ncond), s0 + u, tu);
      if (tid < C2) sm.keep[u][tid] = sm.enc.red[0][tid] + sm.enc.red[1][tid];
    }
    WACC(2, wt1_);
#ifdef ERTD_CHAIN_STAMPS
    const unsigned long long wt2_ = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) wacc[5] += 1;
    if (tid == 0 && b == 0 && item < 4096) g_item[item][2] = wt2_;
#endif
    float* part = a.part + (size_t)slot * ring_part;
    // publish: write-through partial stores, drained by every storing wave,
    // then one relaxed arrival; the last arriver reads them with sc1 loads
    // (no release/acquire fences: Guideline 16, form R1)
    if (tid < C2) {
#pragma unroll 1
      for (int u = 0; u < ns; ++u) st_sc1(part + ((size_t)b * S + s0 + u) * C2 + tid, sm.keep[u][tid]);
    }
    drain();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add((gu32*)(a.cnt + ((size_t)slot * B + b) * SYNC_PAD), (unsigned)ns,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned pv = ld_relaxed(a.progress + (size_t)b * SYNC_PAD);  // same round trip as the arrival
      seen_reg = pv > seen_reg ? pv : seen_reg;
      sm.seen = (int)seen_reg;
      sm.next = (int)nxt;
      sm.flag = old + (unsigned)ns == (unsigned)(S * (i / R + 1));
    }
    __syncthreads();
    WACC(3, wt2_);
#ifdef ERTD_CHAIN_STAMPS
    if (tid == 0 && b == 0 && item < 4096) g_item[item][3] = __builtin_amdgcn_s_memrealtime();
#endif
    if (!sm.flag) continue;
#ifdef ERTD_CHAIN_STAMPS
    const unsigned long long wt3_ = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) wacc[6] += 1;
#endif
    // ---- last arriver: condition row u_i[b] = b0 + W0c.relu(W3.mean + b3)
    {
      const DenseT d = dense_ptrs(pk);
      const int j = tid_i & (H - 1), q = tid_i >> 7;
      CondScratch& sc = sm.cond;
      cond_row_pool(sc, part, b, S, tid_i, Sc1Load());
      const float bias_c = q == 0 ? w.enc6_b[j + z0] : 0.f;
      const float bias_u = q == 0 ? w.mlp0_b[j + z0] : 0.f;
      __syncthreads();
      if (tid < C2) sc.m[tid] = pool_combine(sc.pg, tid, L2);
      __syncthreads();
      sc.part[q][j] = chain_half_stream<C2>(d.W3T, sc.m, bias_c, j, q);
      __syncthreads();
      if (tid < H) sc.c[j] = fmaxf(sc.part[0][j] + sc.part[1][j], 0.f);
      __syncthreads();
      sc.part[q][j] = chain_half_stream<H>(d.W0T + (size_t)(P + H) * H, sc.c, bias_u, j, q);
      __syncthreads();
      if (tid < H) st_sc1(a.uring + ((size_t)slot * B + b) * H + j, sc.part[0][j] + sc.part[1][j]);
      drain();
      __syncthreads();  // (also: scratch is reused by the next item)
      if (tid == 0) st_relaxed(a.uflag + ((size_t)slot * B + b) * SYNC_PAD, (unsigned)(i + 1));
#ifdef ERTD_CHAIN_STAMPS
      if (tid == 0 && b == 0 && i < 1024) g_pub[i][1] = __builtin_amdgcn_s_memrealtime();
#endif
    }
    WACC(4, wt3_);
  }
#ifdef ERTD_CHAIN_STAMPS
  if (tid == 0 && wid < 2048) {
    wacc[7] = __builtin_amdgcn_s_memrealtime() - wstart;
    for (int k = 0; k < 8; ++k) g_wacc[wid][k] = wacc[k];
  }
#endif
}

bool faithful_chain_may_run(int B) {
  constexpr int MAX_CUS = 256;  // MI355X (gfx950): the most CUs a device of this target has
  const long long nch = (B + CHAIN_MPB - 1) / CHAIN_MPB;
  return B >= 1 && nch + 1 + B <= (long long)CHAIN_MAX_BPC * MAX_CUS;
}

int faithful_chain_grid(int B, int S) {
  static int cached[64];  // resident blocks per device (0 = not yet queried)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (cached[dev] == 0) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, faithful_chain_kernel, 256, 0) !=
        hipSuccess)
      return 0;
    // VGPRs (<= 96 -> 5 waves/SIMD) bind before SGPRs (106 -> 6) and LDS (8),
    // so the query is exact here; at most 5 per CU (MICROARCH: the query can
    // read one high only where SGPRs are the binding limit)
    const int use = per_cu < CHAIN_MAX_BPC ? per_cu : CHAIN_MAX_BPC;
    cached[dev] = use > 0 ? use * cus : -1;
  }
  // the chain blocks + the time-row block + workers; every block must be
  // resident.  At most 2S workers per member: more only poll (and slow the chip).
  const int nch = (B + CHAIN_MPB - 1) / CHAIN_MPB;
  const long long want = (long long)nch + 1 + (long long)B * 2 * S;
  if (cached[dev] < nch + 1 + B) return 0;
  return (int)(want < cached[dev] ? want : cached[dev]);
}

// Clears the chain's sync words before each launch.  Our own kernel rather
// than hipMemsetAsync: a memset node replayed from a hipGraph was observed to
// fill the block with a stale non-zero pattern (0xA5251C00 in every word)
// after unrelated launches on the stream (ROCm 7.x runtime, MI355X).
__global__ __launch_bounds__(256) void zero_words_kernel(unsigned* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = 0u;
}

hipError_t launch_zero_words(unsigned* p, size_t n, hipStream_t s) {
  const size_t blocks = (n + 255) / 256;
  zero_words_kernel<<<(unsigned)(blocks < 1024 ? blocks : 1024), 256, 0, s>>>(p, n);
  return hipGetLastError();
}

hipError_t launch_faithful_chain(const ertd_weights& w, const float* packed,
                                 const FaithfulChainArgs& a, int grid, hipStream_t s) {
  faithful_chain_kernel<<<grid, 256, 0, s>>>(w, packed, a);
  return hipGetLastError();
}

}  // namespace ertd
