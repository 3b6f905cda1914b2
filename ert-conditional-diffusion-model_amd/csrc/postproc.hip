// Ensemble post-processing on device: the chain the
// reference runs on every realisation after sample_model returns
// (ERT_Conditional_Diffusion.py:400-406 and :1054-1060):
//
//   inverse_transform(u, a, b)            :42-53   a + (b-a)*sigmoid(u), fp32 tensor op
//   .cpu().numpy()
//   param_scaler.inverse_transform(x)     sklearn MinMaxScaler: x -= min_; x /= scale_
//                                         (float64 vectors applied in place to the
//                                          float32 array: each op in float64, rounded
//                                          back to float32)
//   check_param_bounds(x, limits)         :183-218  a row is dropped when any value
//                                         v satisfies v < lo or v > hi (float64
//                                         compare; a NaN passes, as in the reference)
//
// One 32-lane half-wave per parameter row (P <= 32): each lane maps one
// parameter, the row verdict is a ballot over the half-wave.  The output keeps
// the reference's Uncertainty_params layout (n_samples, n_rows, P) when the
// caller points `out` at realisation r's slice.
#include "ertd_common.h"

namespace ertd {

__global__ __launch_bounds__(256) void postproc_kernel(const float* __restrict__ u, long long rows,
                                                       int P, float a, float bma,
                                                       const double* __restrict__ min_,
                                                       const double* __restrict__ scale_,
                                                       const double* __restrict__ limits,
                                                       float* __restrict__ out,
                                                       uint8_t* __restrict__ valid) {
  const long long row = (long long)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int p = threadIdx.x & 31;
  const bool act = row < rows && p < P;
  bool bad = false;
  if (act) {
    const float v = u[row * P + p];
    // torch.sigmoid(u) on float32: 1/(1+exp(-u)), each op rounded to float32
    // (exp formed in float64 and rounded once: the correctly rounded expf)
    const float e = (float)exp(-(double)v);
    const float s = __fdiv_rn(1.0f, __fadd_rn(1.0f, e));
    const float x = __fadd_rn(a, __fmul_rn(bma, s));
    const float y = (float)((double)x - min_[p]);
    const float z = (float)((double)y / scale_[p]);
    out[row * P + p] = z;
    const double zd = (double)z;
    bad = (zd < limits[2 * p]) || (zd > limits[2 * p + 1]);
  }
  const uint64_t m = __ballot(bad);
  const uint32_t half = (threadIdx.x & 32) ? (uint32_t)(m >> 32) : (uint32_t)m;
  if (p == 0 && row < rows) valid[row] = half == 0u ? 1 : 0;
}

hipError_t launch_postproc(const float* u, long long rows, int P, float a, float bma,
                           const double* min_, const double* scale_, const double* limits,
                           float* out, uint8_t* valid, hipStream_t s) {
  const long long blocks = (rows + 7) / 8;
  postproc_kernel<<<(unsigned)blocks, 256, 0, s>>>(u, rows, P, a, bma, min_, scale_, limits, out,
                                                   valid);
  return hipGetLastError();
}

}  // namespace ertd
