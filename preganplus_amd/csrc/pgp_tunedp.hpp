// pgp_tunedp.hpp — launchers of the data-parallel tuning bookkeeping
// (pgp_tunedp.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace pgp {

constexpr int kMaxTuneRows = 16;  // on-the-fly dataset rows (LATEST_WINDOW_SIZE = 10, constants.py:16)
constexpr int kDpInc = 10;        // per-block partials: delta[3][2], count[3], ones
constexpr int kMaxCond = 4;       // AdamW rows whose activity is decided on the device

struct CondRows {
  int n;
  int row[kMaxCond];
};

// The decoders' pre-activation gradient of one (window, host) [2 anomaly | 2
// prototype entries]: CE(logits, y) * mult (train.py:28-36) and the positive
// triplet MSE toward tgt through the sigmoid (train.py:15-21; the negative
// terms are detached there and carry no gradient).  fp32, the compiler's
// default contraction; shared by tune_loss_kernel (pgp_tune.hip) and the DP
// targets kernel (pgp_tunedp.hip) so both write the same bits.
#ifdef __HIPCC__
__device__ __forceinline__ void dpre_host(float l0, float l1, int yy, float mu, float p0, float p1, float t0, float t1,
                                          float* d_anom, float* d_proto) {
  const float m = fmaxf(l0, l1), e0 = expf(l0 - m), e1 = expf(l1 - m), inv = 1.0f / (e0 + e1);
  d_anom[0] = mu * (e0 * inv - (yy == 0 ? 1.f : 0.f));
  d_anom[1] = mu * (e1 * inv - (yy == 1 ? 1.f : 0.f));
  const float g0 = yy > 0 ? (p0 - t0) : 0.f, g1 = yy > 0 ? (p1 - t1) : 0.f;  // d/dp mean_k (p - t)^2
  d_proto[0] = g0 * p0 * (1.f - p0);                                          // through the sigmoid
  d_proto[1] = g1 * p1 * (1.f - p1);
}
#endif

hipError_t launch_tune_dataset(int H, int E, int R, const double* series, const double* train_max, float* windows,
                               int* y, int* cls, float* infer, hipStream_t st, hipEvent_t stop = nullptr);
long tune_dp_workspace_doubles(int B);
// the state update (pgp_tune_state_apply) done by the targets kernel's last
// workgroup, when the step has no exchange between the two (world size 1)
struct StateApplyArgs {
  int on;
  double decay;
  CondRows cr;
  double* dsteps;
  float* table;
  double lr, b1, b2;
};
hipError_t launch_tune_targets_dp(int H, int K, int B, const float* logits, const float* protos, const int* y,
                                  const int* cls, double* state, double update_min, float* mult, float* tgt,
                                  double* loss, double* inc, double* ws, hipStream_t st, float* dpre = nullptr,
                                  int nop = 0, const StateApplyArgs* apply = nullptr, hipEvent_t stop = nullptr);
hipError_t launch_tune_state_apply(int K, double* state, const double* inc, double decay, const CondRows& cr,
                                   double* dsteps, float* table, double lr, double b1, double b2, hipStream_t st);

}  // namespace pgp
