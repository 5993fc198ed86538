// pgp_train.hip — AdamW (utils.py:65: torch.optim.AdamW, single-tensor
// semantics) over the master weights of the online training steps.  The
// steps themselves: pgp_tune.hip (tuning step), pgp_gantrain.hip (GAN step).
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_train.hpp"

namespace pgp {
namespace {

// AdamW (adamw_elem, pgp_train.hpp) over the tensors of a.t on a flat grid:
// tensor i owns blocks [g.bx0[i], g.bx0[i+1]), kAdamChunk elements each (a
// grid of one row per tensor sized by the largest dispatched ~1,000 idle
// workgroups per small tensor: 17-20 us per call for the tuning step's
// section).  Each element's update is independent, so the results are the
// same as any other order.
constexpr int kAdamChunk = 1024;
struct AdamGrid {
  int bx0[kMaxTensors + 1];
};
__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a, AdamGrid g) {
  const int bx = blockIdx.x;
  int lo = 0, hi = a.ntensors - 1;  // the last tensor whose first block is <= bx
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (bx >= g.bx0[mid]) lo = mid;
    else hi = mid - 1;
  }
  const AdamTensor& t = a.t[lo];
  float step_size = t.step_size, bc2_sqrt = t.bc2_sqrt;
  if (a.sched && (t.active & kAdamFromTable)) {  // per-step scalars from the device (graph-captured loops)
    const float* r = a.sched + 3 * lo;
    if (r[0] == 0.f) return;
    step_size = r[1];
    bc2_sqrt = r[2];
  } else if (!t.active) {
    return;
  }
  const long base = (long)(bx - g.bx0[lo]) * kAdamChunk;
#pragma unroll
  for (int k = 0; k < kAdamChunk / 256; ++k) {
    const long i = base + k * 256 + threadIdx.x;
    if (i < t.n) adamw_elem(a, t.off + i, step_size, bc2_sqrt);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
hipError_t launch_adamw(const AdamArgs& a, hipStream_t st) {
  AdamGrid g{};
  int nb = 0;
  for (int i = 0; i < a.ntensors; ++i) {
    g.bx0[i] = nb;
    nb += (int)((a.t[i].n + kAdamChunk - 1) / kAdamChunk);
  }
  g.bx0[a.ntensors] = nb;
  if (nb == 0) return hipSuccess;
  adamw_kernel<<<nb, 256, 0, st>>>(a, g);
  return hipGetLastError();
}

}  // namespace pgp
