// Per-cell Gaussian-KDE mode of an ensemble.
//
// Reference: ERT_Conditional_Diffusion.py:747-762, the ensemble-mode loop --
// for every cell (i, j) of sim_data (n, 4693, 14) one scipy.stats.gaussian_kde
// of the n values sim_data[:, i, j], evaluated on
// x_range = np.linspace(min(sim_data), max(sim_data), 5000), mode =
// x_range[np.argmax(kde(x_range))] -- and :166-181 mode_kde_calculation (one
// array, its own min/max, 1000 points).
//
// gaussian_kde (scipy/stats/_kde.py, 1-D, equal weights w = 1/n, Scott's
// factor neff^(-1/5), neff = 1/sum(w^2)):
//   avg = sum(w x) / sum(w)
//   var = sum((x-avg) * ((x-avg) w)) * (1 / (sum(w) - sum(w w)/sum(w)))   (np.cov)
//   L   = sqrt(var) * factor                                             (cho_cov)
//   kde(q) = sum_i  w * (exp(-((x_i/L - q/L)^2) / 2) * norm),  norm = (2 pi)^(-1/2) / L
// accumulated in float64, i ascending (scipy's gaussian_kernel_estimate loop).
// The grid is numpy's linspace: q_j = j*step + lo, q_{G-1} = hi, step = (hi-lo)/(G-1).
//
// One workgroup per cell.  The n samples are staged in LDS already divided by
// L; each thread owns grid points j = tid, tid + 256, ... and runs the i-loop
// in order, so every density value is the reference's ordered float64 sum.
// A pair whose exponent underflows (arg > 1491: exp(-745.5) is 0 in binary64)
// adds an exact zero and is skipped -- typically most of the grid, which spans
// the whole ensemble's range while one cell's kernel is narrow.  The argmax
// keeps the lowest index among equal maxima (np.argmax).  Bound: fp64 VALU
// (the exp of the near pairs); the input is read once.
#include "ertd_common.h"

#include <cmath>

#include "ertdiff.h"

namespace ertd {
namespace {

constexpr int KT = 256;
constexpr double ARG_ZERO = 1491.0;   // exp(-arg/2) == 0.0 for arg > 1490.3

struct KdeArgs {
  const double* x;       // (n, ld) row-major, cell c at column c
  int n;
  long long cells, ld;
  int G;
  int range_mode;        // 0: [lo, hi] args, 1: per cell, 2: [lo, hi] from range_dev
  double lo, hi;
  const double* range_dev;
  double factor;         // Scott's factor neff^(-1/5)
  double norm0;          // (2 pi)^(-1/2)
  double* mode;          // (cells)
  int* index;            // (cells) or null; -1 = singular covariance
  double* density;       // (cells) or null: kde value at the mode
};

__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

__device__ __forceinline__ double block_min(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double s = fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
  __syncthreads();
  return s;
}

__device__ __forceinline__ double block_max(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double s = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  return s;
}

__device__ __forceinline__ double grid_point(int j, int G, double lo, double hi, double step) {
  if (j == G - 1 && G > 1) return hi;
  return (double)j * step + lo;   // -ffp-contract=off: numpy's y*step, then + start
}

__global__ __launch_bounds__(KT) void kde_mode_kernel(KdeArgs a) {
  extern __shared__ double xs[];   // [n]
  __shared__ double red[4];
  __shared__ double bv_s[4];
  __shared__ int bi_s[4];
  const long long c = blockIdx.x;
  const int tid = threadIdx.x;
  const int n = a.n;
  const double w = 1.0 / (double)n;

  double s1 = 0.0, sw = 0.0, sww = 0.0, mn = INFINITY, mx = -INFINITY;
  for (int i = tid; i < n; i += KT) {
    const double v = a.x[(size_t)i * a.ld + c];
    xs[i] = v;
    s1 += v * w;
    sw += w;
    sww += w * w;
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
  const double S1 = block_sum(s1, red), SW = block_sum(sw, red), SWW = block_sum(sww, red);
  double lo = a.lo, hi = a.hi;
  if (a.range_mode == 1) {
    lo = block_min(mn, red);
    hi = block_max(mx, red);
  } else if (a.range_mode == 2) {
    lo = a.range_dev[0];
    hi = a.range_dev[1];
  }
  const double avg = S1 / SW;
  double s2 = 0.0;
  for (int i = tid; i < n; i += KT) {
    const double d = xs[i] - avg;
    s2 += d * (d * w);
  }
  const double S2 = block_sum(s2, red);
  const double fact = SW - SWW / SW;
  const double var = S2 * (1.0 / fact);
  const double L = sqrt(var) * a.factor;
  const int G = a.G;
  const double step = G > 1 ? (hi - lo) / (double)(G - 1) : 0.0;
  if (!(L > 0.0) || !isfinite(L)) {
    // var == 0: gaussian_kde raises (singular covariance); NaN data: every
    // density is NaN and np.argmax returns 0
    if (tid == 0) {
      const bool singular = var == 0.0;
      a.mode[c] = singular ? NAN : grid_point(0, G, lo, hi, step);
      if (a.index) a.index[c] = singular ? -1 : 0;
      if (a.density) a.density[c] = NAN;
    }
    return;
  }
  for (int i = tid; i < n; i += KT) xs[i] = xs[i] / L;   // solve_triangular(cho_cov, x)
  __syncthreads();
  const double norm = a.norm0 / L;

  double bv = -1.0;
  int bi = 0x7fffffff;
  for (int j = tid; j < G; j += KT) {
    const double qw = grid_point(j, G, lo, hi, step) / L;
    double est = 0.0;
    for (int i = 0; i < n; ++i) {
      const double r = xs[i] - qw;
      const double arg = r * r;
      if (arg <= ARG_ZERO) est += w * (exp(-arg / 2.0) * norm);
    }
    if (est > bv) { bv = est; bi = j; }   // ascending j: first maximum kept
  }
  // workgroup argmax, lowest index on ties
  for (int o = 32; o > 0; o >>= 1) {
    const double ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  if ((tid & 63) == 0) { bv_s[tid >> 6] = bv; bi_s[tid >> 6] = bi; }
  __syncthreads();
  if (tid == 0) {
    for (int q = 1; q < 4; ++q)
      if (bv_s[q] > bv || (bv_s[q] == bv && bi_s[q] < bi)) { bv = bv_s[q]; bi = bi_s[q]; }
    a.mode[c] = grid_point(bi, G, lo, hi, step);
    if (a.index) a.index[c] = bi;
    if (a.density) a.density[c] = bv;
  }
}

// min / max over a float64 array: per-block partials, then one block
__global__ __launch_bounds__(KT) void minmax_partial_kernel(const double* x, long long count,
                                                            double* part) {
  __shared__ double red[4];
  double mn = INFINITY, mx = -INFINITY;
  for (long long i = (long long)blockIdx.x * KT + threadIdx.x; i < count;
       i += (long long)gridDim.x * KT) {
    const double v = x[i];
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
  mn = block_min(mn, red);
  mx = block_max(mx, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = mn;
    part[2 * blockIdx.x + 1] = mx;
  }
}

__global__ __launch_bounds__(KT) void minmax_final_kernel(const double* part, int nb, double* out2) {
  __shared__ double red[4];
  double mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < nb; i += KT) {
    mn = fmin(mn, part[2 * i]);
    mx = fmax(mx, part[2 * i + 1]);
  }
  mn = block_min(mn, red);
  mx = block_max(mx, red);
  if (threadIdx.x == 0) {
    out2[0] = mn;
    out2[1] = mx;
  }
}

inline int kde_rc(hipError_t e) { return e == hipSuccess ? ERTD_OK : (int)e; }

}  // namespace
}  // namespace ertd

extern "C" {

int ertd_minmax_f64(const double* x, long long count, double* work, double* out2, void* stream) {
  if (!x || !work || !out2 || count < 1) return ERTD_EINVAL;
  const hipStream_t s = (hipStream_t)stream;
  const long long want = (count + ertd::KT - 1) / ertd::KT;
  const int nb = (int)(want < ERTD_MINMAX_BLOCKS ? want : ERTD_MINMAX_BLOCKS);
  ertd::minmax_partial_kernel<<<nb, ertd::KT, 0, s>>>(x, count, work);
  ertd::minmax_final_kernel<<<1, ertd::KT, 0, s>>>(work, nb, out2);
  return ertd::kde_rc(hipGetLastError());
}

int ertd_kde_mode(const double* x, int n, long long cells, long long ld, int grid, int range_mode,
                  double lo, double hi, const double* range_dev, double* mode, int* index,
                  double* density, void* stream) {
  if (!x || !mode || n < 2 || cells < 1 || ld < cells || grid < 1 || cells > 0x7fffffffLL)
    return ERTD_EINVAL;
  if (range_mode < 0 || range_mode > 2 || (range_mode == 2 && !range_dev)) return ERTD_EINVAL;
  const size_t lds = (size_t)n * sizeof(double);
  if (lds > 160 * 1024) return ERTD_EINVAL;
  if (lds > 65536)
    (void)hipFuncSetAttribute((const void*)ertd::kde_mode_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  ertd::KdeArgs a{};
  a.x = x; a.n = n; a.cells = cells; a.ld = ld; a.G = grid;
  a.range_mode = range_mode; a.lo = lo; a.hi = hi; a.range_dev = range_dev;
  // scipy: neff = 1/sum(w**2) with w = ones(n)/n; factor = neff**(-1/(d+4))
  const double w = 1.0 / (double)n;
  double sww = 0.0;
  for (int i = 0; i < n; ++i) sww += w * w;
  a.factor = std::pow(1.0 / sww, -1.0 / 5.0);
  a.norm0 = std::pow(2.0 * M_PI, -0.5);
  a.mode = mode; a.index = index; a.density = density;
  ertd::kde_mode_kernel<<<(unsigned)cells, ertd::KT, lds, (hipStream_t)stream>>>(a);
  return ertd::kde_rc(hipGetLastError());
}

}  // extern "C"
