// pgp_tune.hpp — geometry and workspace plan of the tuning step (train.py:42-57).
//
// The buffers between its kernels are row-major [M][ld] arrays over the batch's
// M = B * 3H tokens, token row m = b*3H + w*H + h (the reference's [S=W, N=H, d]
// order per window, models.py:387-396), feature widths zero-padded to multiples
// of 16 (d = H -> DP, 3d -> Q3P).  The encoder layers themselves run as fused
// per-unit kernels (pgp_tunef.hip) that keep a layer's activations in registers;
// only layer inputs, norm1's x-hat / rstd and the gradients between layers
// cross HBM.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "pgp_layout.hpp"

namespace pgp {

template <int H>
struct TuneGeo {
  static constexpr int D = H, DP = round_up(H, 16), T = 3 * H, HD = H / 2;
  static constexpr int Q3 = 3 * H, Q3P = round_up(3 * H, 16), FF = 64;
  static constexpr int NO = 4 * H, NOP = round_up(4 * H, 16);  // decoder outputs: anomaly 2H | prototype 2H
  static constexpr long KD = (long)T * DP;                     // decoder contraction in token layout
  static constexpr int XBP = 16;                               // GAT aggregated raw features, padded
};

// The workspace starts with kTuneCounters floats of device counters (the
// last-part finishes of the backward's reductions; zero in a fresh workspace,
// each left at zero by the launch that uses it), then the regions below.
constexpr long kTuneCounters = 1024;
// counters [0, 2 * 3H): the decoder weight gradient's per-(token, half) parts;
// kCtrGatTail: the GAT parameter tail of the fused reduction
constexpr int kCtrGatTail = 1000;
static_assert(kCtrGatTail < kTuneCounters, "GAT tail counter inside the counter head");
#define PGP_CTR_FITS(h) static_assert(2 * 3 * (h) <= kCtrGatTail, "decoder dW counters reach kCtrGatTail");
PGP_FOR_EACH_H(PGP_CTR_FITS)
#undef PGP_CTR_FITS
constexpr int kMaxDecDws = 4;  // decoder weight-gradient parts (windows split over up to 4)
// Workspace regions (float offsets) for one (H, B); region-major, so the same
// (H, B) must be used by the forward and the backward of one step.
struct TunePlan {
  int H = 0, B = 0;
  long M = 0;  // tokens
  int DP = 0, Q3P = 0, NOP = 0;
  long KD = 0;
  long win = 0;                                          // [B][9H] copy of the input windows
  long g = 0, xb = 0, gs = 0;                            // GAT out [M][DP], x-bar [M][16], (max, Z) [3B][4]
  long x[3] = {0, 0, 0};                                 // layer inputs; x[2] = encoder output [M][DP]
  long xh1[2] = {0, 0}, rs1[2] = {0, 0};                 // norm1 x-hat [M][DP], rstd [M] (checkpoints)
  long da = 0, db = 0, dq[2] = {0, 0};                   // backward temporaries ([M][DP], [M][DP], 2 x [M][3][DP])
  long gsx = 0, dpre = 0, wp = 0, wpt = 0, part = 0, total = 0;  // wp: Wp [NOP][KD], wpt: WpT [T][DP][NOP]
  long fcd = 0;  // sum over tokens of dX0 (x) x-bar [H][3] (the fc gradient before W_TE, gat_param_kernel)
  long mt = 0;   // W_TE fc [64][3] (the forward's packing launch, read by gat_bwd_kernel)
  long tff = 0;                                          // fused-kernel weight fragments (pgp_tunef.hpp)
  long tfs[2][2] = {{0, 0}, {0, 0}};                     // [layer][ffn | attention] weight-gradient slabs
  long pool = 0, pool_len = 0;  // the backward's deferred-reduction regions (RedBatch)
  int lin_grid = 0, dw_grid = 0, dec_s = 0, dec_dws = 1, tf_grid = 0;
};

bool tune_plan(int H, int B, TunePlan* p);
// a backward over the first B windows of a forward of B_fwd (same workspace)
bool tune_plan_prefix(int H, int B_fwd, int B, TunePlan* p);
// live timing of the six fused encoder launches of a forward + backward
// (pgp_tune_timing / pgp_tune_fused_ms)
hipError_t tune_timing(bool on);
// the tuning backward's side stream on the current device: `s`, or the
// library's own low-priority stream when null (pgp_tune_set_side_stream)
hipError_t tune_set_side_stream(hipStream_t s);
// whether a step of that many tokens forks side work (a capture, or a side
// stream override equal to the step's stream, can still keep it on one stream)
bool tune_side_active(long tokens);
hipError_t tune_fused_ms(float* out6);

// decoder GEMMs (pgp_dec.hip): split-K forward into part[S][B][NOP] and the
// backward into the encoder output's gradient [M][DP]
int dec_fwd_splits(int H, int B);
hipError_t launch_dec_fwd(int H, int B, int S, const float* X2, const float* Wp, float* part, hipStream_t st);
hipError_t launch_dec_dx(int H, int B, const float* dpre, const float* WpT, float* dX, hipStream_t st);

// post: signalled when the logits / prototypes are written (the forward's last
// launch's stop event)
hipError_t launch_tune_forward(const TunePlan& p, const float* windows, const float* P, float* ws, float* latent,
                               float* logits, float* protos, hipStream_t st, hipEvent_t post = nullptr);
// dpre_ready: the decoder pre-activation gradient [B][NOP] at ws + p.dpre was
// already written (launch_tune_targets_dp with dpre), so the loss kernel is
// skipped; pre (with dpre_ready): an event the caller's last launch on `st`
// signals at its end, which the first fork of the side work waits on instead
// of an event recorded here
hipError_t launch_tune_backward(const TunePlan& p, const float* P, float* G, float* ws, const float* logits,
                                const float* protos, const int* y, const float* mult, const float* tgt,
                                hipStream_t st, bool dpre_ready = false, hipEvent_t pre = nullptr);
hipError_t launch_tune_targets(int H, int K, const float* logits, const float* protos, const int* y, const int* cls,
                               double* state, double update_min, double decay, float* mult, float* tgt, double* loss,
                               hipStream_t st);

// one fused batch-1 tuning step (pgp_tune1.hip): forward + targets + backward
// writing the transformer section of G; H in {8, 16}
bool tune1_supported(int H);
hipError_t launch_tune1(int H, int K, const float* win, const int* y, const int* cls, const float* P, float* G,
                        double* state, double update_min, double decay, float* logits, float* protos, double* loss,
                        hipStream_t st);
// n independent batch-1 forwards (accuracy()'s batch), fp64 logits / protos [n][H][2]
hipError_t launch_fwd_many(int H, int n, const float* win, const float* P, double* logits, double* protos,
                           hipStream_t st);
// batch-1 inference of run_model from the master weights (pgp_tune1.hip)
hipError_t launch_infer1(int H, int K, const float* win, const float* sched, const float* P, const double* protos,
                         float* logits, float* protos_out, int* cls, int* any_anom, float* probs, int* keep,
                         int* final_t, int* gen_t, hipStream_t st);

}  // namespace pgp
