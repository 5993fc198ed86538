// pgp_tunetargets.hpp — custom_loss / triplet_loss bookkeeping of ONE window
// (train.py:13-40) as a device function, shared by tune_targets_kernel
// (pgp_tune.hip) and the fused batch-1 step (pgp_tune1.hip).  The logic is
// inherently sequential (the prototype EMA of host i feeds the targets of host
// i+1), so one lane runs it, in fp64 and in the reference's operation order,
// with FMA contraction off: every value matches the numpy restatement
// (train.loss_targets) bit for bit, except the reported loss values, which go
// through device log/exp.
//   state [2K+3] fp64: prototypes [K][2] (model.prototype, K = n_hosts for the
//                   Transformer, models.py:373; triplet_loss reads and updates
//                   rows 0-2 only), PROTO_UPDATE_FACTOR, num_zero, num_ones
//                   (train.py's module globals)
//   outputs: mult [H] and tgt [H][2] (fp32, as the backward takes them),
//            loss [2] fp64 = (aloss, tloss) of the window
#pragma once
#include <hip/hip_runtime.h>

namespace pgp {

// CrossEntropyLoss of one host's logits row (train.py:28-32), fp64
__device__ inline double tune_ce_term(float l0f, float l1f, int yi) {
#pragma clang fp contract(off)
  const double l0 = l0f, l1 = l1f;
  const double m = fmax(l0, l1);
  const double lse = log(exp(l0 - m) + exp(l1 - m)) + m;
  return lse - (yi ? l1 : l0);
}

// ce: the hosts' tune_ce_term values computed ahead in parallel, or nullptr
// (computed here).  Prototype rows 0-2 and the counters live in registers for
// the sequential loop (one read and one write of state).
__device__ inline void tune_targets_one(int H, int K, const float* __restrict__ logits,
                                        const float* __restrict__ protos, const int* __restrict__ y,
                                        const int* __restrict__ cls, double* __restrict__ state, double update_min,
                                        double decay, float* __restrict__ mult, float* __restrict__ tgt,
                                        double* __restrict__ loss, const double* __restrict__ ce = nullptr) {
#pragma clang fp contract(off)
  double* pr = state;          // [K][2]
  double* sc = state + 2 * K;  // factor, num_zero, num_ones
  double p00 = pr[0], p01 = pr[1], p10 = pr[2], p11 = pr[3], p20 = pr[4], p21 = pr[5];
  const double factor = sc[0], nz = sc[1], no = sc[2];
  const double ratio = nz / no;  // num_zero / num_ones (exact integers in fp64)
  double aloss = 0.0;
  long ones = 0;
  for (int i = 0; i < H; ++i) {  // train.py:28-32
    const int yi = y[i];
    const double mu = yi == 0 ? 1.0 : ratio;
    mult[i] = (float)mu;
    ones += yi == 1 ? 1 : 0;
    aloss += (ce ? ce[i] : tune_ce_term(logits[2 * i], logits[2 * i + 1], yi)) * mu;
  }
  double tloss = 0.0;
  for (int i = 0; i < H; ++i) {  // train.py:33-35 -> triplet_loss (:13-24)
    if (y[i] > 0) {
      const int cc = cls[i];
      const double a0 = protos[2 * i], a1 = protos[2 * i + 1];
      const double c0 = cc == 0 ? p00 : (cc == 1 ? p10 : p20);
      const double c1 = cc == 0 ? p01 : (cc == 1 ? p11 : p21);
      tgt[2 * i] = (float)c0;
      tgt[2 * i + 1] = (float)c1;
      const double m0 = ((a0 - p00) * (a0 - p00) + (a1 - p01) * (a1 - p01)) / 2.0;  // MSELoss over 2 values
      const double m1 = ((a0 - p10) * (a0 - p10) + (a1 - p11) * (a1 - p11)) / 2.0;
      const double m2 = ((a0 - p20) * (a0 - p20) + (a1 - p21) * (a1 - p21)) / 2.0;
      const double pos = cc == 0 ? m0 : (cc == 1 ? m1 : m2);
      const double n0 = cc == 0 ? m1 : m0, n1 = cc == 2 ? m1 : m2;  // negatives in class order
      tloss += pos - (n0 + n1);
      if (pos <= n0 && pos <= n1) {
        const double f = factor + update_min;
        const double u0 = f * a0 + (1.0 - f) * c0, u1 = f * a1 + (1.0 - f) * c1;
        if (cc == 0) {
          p00 = u0;
          p01 = u1;
        } else if (cc == 1) {
          p10 = u0;
          p11 = u1;
        } else {
          p20 = u0;
          p21 = u1;
        }
      }
    } else {
      tgt[2 * i] = 0.f;
      tgt[2 * i + 1] = 0.f;
    }
  }
  pr[0] = p00;
  pr[1] = p01;
  pr[2] = p10;
  pr[3] = p11;
  pr[4] = p20;
  pr[5] = p21;
  sc[0] = factor * decay;  // PROTO_UPDATE_FACTOR *= PROTO_FACTOR_DECAY
  sc[1] = nz + (double)H;  // nz counts every host (train.py:31)
  sc[2] = no + (double)ones;
  loss[0] = aloss;
  loss[1] = tloss;
}

}  // namespace pgp
