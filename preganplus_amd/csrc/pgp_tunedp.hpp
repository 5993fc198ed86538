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

hipError_t launch_tune_dataset(int H, int E, int R, const double* series, const double* train_max, float* windows,
                               int* y, int* cls, float* infer, hipStream_t st);
long tune_dp_workspace_doubles(int B);
hipError_t launch_tune_targets_dp(int H, int K, int B, const float* logits, const float* protos, const int* y,
                                  const int* cls, const double* state, double update_min, float* mult, float* tgt,
                                  double* loss, double* inc, double* ws, hipStream_t st);
hipError_t launch_tune_state_apply(int K, double* state, const double* inc, double decay, const CondRows& cr,
                                   double* dsteps, float* table, double lr, double b1, double b2, hipStream_t st);

}  // namespace pgp
