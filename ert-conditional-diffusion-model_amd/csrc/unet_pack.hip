// Batched fp32 conv weight packing (include/ertdiff.h, ertd_conv_pack_batch):
// the U-Net train step re-packs every conv's forward and input-gradient
// weights once per optimizer step -- ~100 packings for U2 -- in ONE launch
// instead of one small launch per conv call.  Block b finds its descriptor
// by binary search over the prepared block offsets; each work item is the
// same device function the per-layer pack kernels call (unet_pack.h: one
// element of a direct / Upsample packing, one (co, ci) tile of a Winograd
// one), so the bits are identical.
#include "unet_pack.h"

namespace ertd {
namespace unet {

namespace {

__global__ __launch_bounds__(256) void pack_batch_kernel(const ertd_pack_desc* __restrict__ d, int n) {
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {   // last descriptor with block0 <= b
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].block0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const ertd_pack_desc q = d[lo];
  const size_t i = (size_t)(b - q.block0) * 256 + threadIdx.x;   // work item of this packing
  if (i >= (size_t)pack_work_items(q.kind, q.total)) return;
  switch (q.kind) {
    case ERTD_PACK_DIRECT: q.dst[i] = pack_conv_elem(q.w, q.cin, q.cout, q.ks, q.nchunk, i, q.flip != 0); break;
    case ERTD_PACK_UP: q.dst[i] = pack_conv_up_elem(q.w, q.cin, q.cout, q.nchunk, (size_t)q.total / 4, i); break;
    case ERTD_PACK_WINO: pack_wino_tile(q.w, q.cin, q.cout, q.nchunk, i, q.flip != 0, q.dst); break;
    default: pack_wino4_tile(q.w, q.cin, q.cout, q.nchunk, i, q.flip != 0, q.dst); break;
  }
}

}  // namespace

hipError_t launch_pack_batch(const ertd_pack_desc* d, int n, int blocks, hipStream_t s) {
  pack_batch_kernel<<<(unsigned)blocks, 256, 0, s>>>(d, n);
  return hipGetLastError();
}

}  // namespace unet
}  // namespace ertd
