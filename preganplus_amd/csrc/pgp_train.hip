// pgp_train.hip — AdamW (utils.py:65: torch.optim.AdamW, single-tensor
// semantics) over the master weights of the online training steps.  The
// steps themselves: pgp_tune.hip (tuning step), pgp_gantrain.hip (GAN step).
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_train.hpp"

namespace pgp {
namespace {

// AdamW (adamw_elem, pgp_train.hpp) over the tensors of a.t, one grid row each
__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
  const AdamTensor& t = a.t[blockIdx.y];
  float step_size = t.step_size, bc2_sqrt = t.bc2_sqrt;
  if (a.sched) {  // per-step scalars from the device (graph-captured loops)
    const float* r = a.sched + 3 * blockIdx.y;
    if (r[0] == 0.f) return;
    step_size = r[1];
    bc2_sqrt = r[2];
  } else if (!t.active) {
    return;
  }
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < t.n; i += (long)gridDim.x * 256)
    adamw_elem(a, t.off + i, step_size, bc2_sqrt);
}

}  // namespace

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
hipError_t launch_adamw(const AdamArgs& a, hipStream_t st) {
  long maxn = 0;
  for (int i = 0; i < a.ntensors; ++i) maxn = a.t[i].n > maxn ? a.t[i].n : maxn;
  int gx = (int)((maxn + 255) / 256);
  gx = gx > 1024 ? 1024 : (gx < 1 ? 1 : gx);
  adamw_kernel<<<dim3(gx, a.ntensors), 256, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace pgp
