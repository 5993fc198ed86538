// pgp_tunedp.hip — the data-parallel tuning step's bookkeeping on the device
// (BASELINE config C3), so that one step of the semi-supervised
// tuning (tune_model, PreGANPlus.py:51-58) over a batch of environments needs
// no host round trip:
//
//   tune_dataset_kernel     load_on_the_fly_dataset (utils.py:40-47): the last
//                           n rows of each environment's series, normalised by
//                           the training series' column max (utils.py:94-95),
//                           cut into windows (convert_to_windows, utils.py:7-14)
//                           and labelled by form_test_dataset (utils.py:16-24:
//                           98th percentile per column, numpy 'linear'
//                           interpolation; class = first argmax of the host's 3
//                           columns); plus run_encoder's inference window of the
//                           same rows (PreGANPlus.py:107-112)
//   tune_targets_dp_kernel  custom_loss / triplet_loss (train.py:13-40) in the
//                           data-parallel form of train.loss_targets_dp: every
//                           window scored against the step-START state; CE
//                           weights, positive targets, per-window losses and the
//                           state increments (prototype-EMA deltas f(a - P[c]) and
//                           counts, num_zero / num_ones, windows)
//                           summed over the batch in a fixed order by its last
//                           workgroup (deterministic; the rank's buffer for the
//                           all-reduce)
//   tune_state_apply_kernel train.dp_state_update after the all-reduce: each
//                           prototype moves by the mean of its deltas, counters
//                           add, the factor decays once per window; and the AdamW
//                           table rows of the prototype decoder, which torch skips
//                           when no window of the global batch has a positive
//                           label (their step counts live on the device)
//
// All fp64 with FMA contraction off, in the numpy restatement's operation order
// per value (labels and CE weights bit-identical to it; sums over the batch are
// tree-ordered, equal to fp64 rounding).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_tunedp.hpp"

namespace pgp {
namespace {

constexpr int kWin = 3;  // models.py:320 n_window
// state apply lane map: prototypes 0..K-1 (K <= kMaxProtos = 64), the counters /
// factor on thread 64, the conditional AdamW rows' lanes from thread 66 (wave 1)
constexpr int kStateCountLane = 64, kStateCondLane0 = 66, kStateThreads = 128;

// ---------------------------------------------------------------------------
// dataset: one thread per (environment, host, column, row): a workgroup holds
// kDsP (environment, host) pairs x 3 columns x kMaxTuneRows rows, lanes
// ordered column-fastest so a row's loads are contiguous.  Each thread divides
// its value by the column max and finds that value's stable rank among the
// column's rows (LDS); the rows of rank ilo / ihi publish the order statistics
// of the 98th percentile; then each thread writes its windows and the column-0
// threads form the labels.  Every value goes through the same operations as
// in the one-thread-per-column version (bit-identical outputs); the rows now
// run side by side instead of in one thread's chain (C3: 81 workgroups of
// dependent fp64 divisions and 256 comparisons per thread before).
// ---------------------------------------------------------------------------
constexpr int kDsP = 16;                           // pairs per workgroup
constexpr int kDsThreads = kDsP * 3 * kMaxTuneRows;  // 768
__global__ __launch_bounds__(kDsThreads) void tune_dataset_kernel(int H, int E, int R,
                                                                  const double* __restrict__ series,
                                                                  const double* __restrict__ train_max,
                                                                  float* __restrict__ windows, int* __restrict__ y,
                                                                  int* __restrict__ cls, float* __restrict__ infer) {
#pragma clang fp contract(off)
  __shared__ double sv[3][kMaxTuneRows][kDsP];  // normalised rows
  __shared__ double sab[3][2][kDsP];            // the percentile's order statistics (ranks ilo, ihi)
  const int c = threadIdx.x % 3, q = (threadIdx.x / 3) % kDsP, r = threadIdx.x / (3 * kDsP);
  const long t = (long)blockIdx.x * kDsP + q;
  const bool ok = t < (long)E * H;
  const int e = ok ? (int)(t / H) : 0, h = ok ? (int)(t % H) : 0;
  const int F = 3 * H;
  const bool live = ok && r < R;
  const double den = train_max[3 * h + c] + 1e-8;  // np.max(train, axis=0) + 1e-8
  const double v = live ? series[((long)e * R + r) * F + 3 * h + c] / den : 0.0;
  sv[c][r][q] = v;
  // 98th percentile of the column, numpy 'linear': virtual index (R-1)*0.98,
  // gamma = frac, lerp(a, b, g) = g >= 0.5 ? b - (b-a)(1-g) : a + (b-a) g.
  // The order statistics ilo, ihi are found by stable rank (the element with
  // rank p is sorted[p]) instead of sorting.
  const double vi = (double)(R - 1) * (98.0 / 100.0);
  const double lo = floor(vi);
  const double gm = vi - lo;
  const int ilo = (int)lo, ihi = ilo + 1 < R ? ilo + 1 : R - 1;
  __syncthreads();
  if (live) {
    int rank = 0;
#pragma unroll
    for (int j = 0; j < kMaxTuneRows; ++j) {
      const double vj = sv[c][j][q];
      if (j != r && j < R) rank += (vj < v || (j < r && vj == v)) ? 1 : 0;
    }
    if (rank == ilo) sab[c][0][q] = v;
    if (rank == ihi) sab[c][1][q] = v;
  }
  __syncthreads();
  auto thr_of = [&](int cc) {
    const double a = sab[cc][0][q], b = sab[cc][1][q];
    const double d = b - a;
    return gm >= 0.5 ? b - d * (1.0 - gm) : a + d * gm;
  };
  if (!live) return;  // (no barrier below)
  // convert_to_windows: window r = rows r-3..r-1, row 0 repeated for r < 3
#pragma unroll
  for (int w = 0; w < kWin; ++w) {
    const int src = r >= kWin ? r - kWin + w : (w < kWin - r ? 0 : w - (kWin - r));
    windows[(((long)e * R + r) * kWin + w) * F + 3 * h + c] = (float)sv[c][src][q];
  }
  if (infer && r == 0) {  // run_encoder: last 3 rows -> convert_to_windows(...)[-1] = [R-3, R-3, R-2];
                          // a shorter series (R = 1, 2: the first intervals) keeps all its rows and
                          // its last window is row 0 three times
    const int ra = R >= kWin ? R - 3 : 0, rb = R >= kWin ? R - 2 : 0;
    const double u0 = sv[c][ra][q], u1 = sv[c][rb][q];
#pragma unroll
    for (int w = 0; w < kWin; ++w) infer[((long)e * kWin + w) * F + 3 * h + c] = (float)(w < 2 ? u0 : u1);
  }
  if (c == 0) {  // labels: all three columns of the row
    const double x0 = sv[0][r][q], x1 = sv[1][r][q], x2 = sv[2][r][q];
    const bool an = x0 > thr_of(0) || x1 > thr_of(1) || x2 > thr_of(2);
    int am = 0;  // np.argmax: first maximum
    double best = x0;
    if (x1 > best) {
      am = 1;
      best = x1;
    }
    if (x2 > best) am = 2;
    y[((long)e * R + r) * H + h] = an ? 1 : 0;
    cls[((long)e * R + r) * H + h] = am;
  }
}

// ---------------------------------------------------------------------------
// targets: one wave per window (lane = host), kWpb windows per workgroup.  The
// per-host terms (the fp64 log-sum-exp of the CE, the triplet MSEs) run across
// the lanes; lane 0 then folds them in host order, so each window's losses and
// increments are summed exactly as the one-thread-per-window loop would
// (train.loss_targets_dp's per-window order); windows are combined in a fixed
// tree per workgroup, and the LAST workgroup to finish (a device-scope
// counter in the workspace, reset by it) sums the workgroups' partials in
// index order into inc: the former tune_dp_finish_kernel's order, bit for bit,
// one launch fewer on the C3 step's critical path.  With dpre != nullptr each
// lane also writes its host's decoder pre-activation gradient [B][nop] (the
// former tune_loss_kernel of pgp_tune.hip, same fp32 expressions, from the
// mult / tgt values it has just written): CE(logits, y) * mult
// (train.py:28-36) and the positive triplet MSE toward tgt through the
// sigmoid (train.py:15-21; the negative terms are detached there).
// ---------------------------------------------------------------------------
constexpr int kWpb = 4, kTB = 64 * kWpb;
// (the caller's last workgroup, after its agent-scope acquire on the counter:
// the other workgroups' rows are read with plain loads; sh != nullptr also
// keeps the finished increments in LDS for the fused state update)
__device__ __forceinline__ void dp_finish(int tid, int H, int B, int K, int nblk, const double* part, double* inc,
                                          double* sh = nullptr) {
#pragma clang fp contract(off)
  __shared__ double red[kDpInc][kTB];
  const int t = tid;
  double v[kDpInc] = {};
  for (int i = t; i < nblk; i += kTB) {
    double r[kDpInc];
    for (int k = 0; k < kDpInc; ++k) r[k] = part[(long)i * kDpInc + k];  // all of the row's loads in flight
    for (int k = 0; k < kDpInc; ++k) v[k] += r[k];
  }
  for (int k = 0; k < kDpInc; ++k) red[k][t] = v[k];
  __syncthreads();
  for (int s = kTB / 2; s > 0; s >>= 1) {
    if (t < s)
      for (int k = 0; k < kDpInc; ++k) red[k][t] += red[k][t + s];
    __syncthreads();
  }
  for (int k = t; k < 3 * K + 3; k += kTB) {
    int src = -1;
    if (k < 6) src = k;                                           // delta rows 0-2 (triplet classes)
    else if (k >= 2 * K && k < 2 * K + 3) src = 6 + (k - 2 * K);  // counts 0-2
    else if (k == 3 * K + 1) src = 9;                             // num_ones
    double x = src >= 0 ? red[src][0] : 0.0;
    if (k == 3 * K) x = (double)H * (double)B;  // num_zero: every host counts (train.py:31)
    if (k == 3 * K + 2) x = (double)B;          // windows
    inc[k] = x;
    if (sh) sh[k] = x;
  }
}

// One lane per independent value (K prototypes, the counters / factor, and
// each conditional AdamW row's two bias corrections), each computed exactly as
// the single-thread version did: the fp64 pow calls run side by side instead
// of one after another (13 -> a few us on the C3 step's critical path).
// A row's two lanes are in one wave: its step count is read by both before
// the even lane writes it back.
// (inc: global, or the finishing workgroup's LDS copy)
__device__ __forceinline__ void state_apply_body(int t, int K, double* state, const double* inc,
                                                 const StateApplyArgs& sa) {
#pragma clang fp contract(off)
  auto in = [&](int k) { return inc[k]; };
  const CondRows& cr = sa.cr;
  const bool active = in(3 * K + 1) > 0;  // a positive label somewhere in the global batch
  if (t < K) {
    const double n = in(2 * K + t);
    if (n > 0) {
      state[2 * t] += in(2 * t) / n;
      state[2 * t + 1] += in(2 * t + 1) / n;
    }
  } else if (t == kStateCountLane) {
    state[2 * K + 1] += in(3 * K);
    state[2 * K + 2] += in(3 * K + 1);
    state[2 * K] *= pow(sa.decay, in(3 * K + 2));
  }
  const int u = t - kStateCondLane0;  // threads kStateCondLane0.. : row u / 2, bias correction u % 2
  if (u >= 0 && u < 2 * cr.n) {
    const int i = u >> 1;
    const double ds = active ? sa.dsteps[i] + 1.0 : sa.dsteps[i];
    const double s = ds > 1.0 ? ds : 1.0;
    float* r = sa.table + 3 * cr.row[i];
    if ((u & 1) == 0) {
      r[0] = active ? 1.f : 0.f;
      r[1] = (float)(sa.lr / (1.0 - pow(sa.b1, s)));
    } else {
      r[2] = (float)sqrt(1.0 - pow(sa.b2, s));
    }
    __builtin_amdgcn_wave_barrier();
    if ((u & 1) == 0) sa.dsteps[i] = ds;
  }
}
__global__ __launch_bounds__(kTB) void tune_targets_dp_kernel(int H, int B, const float* __restrict__ logits,
                                                              const float* __restrict__ protos,
                                                              const int* __restrict__ y, const int* __restrict__ cls,
                                                              double* state, int K, double update_min,
                                                              float* __restrict__ mult, float* __restrict__ tgt,
                                                              double* __restrict__ loss, double* __restrict__ part,
                                                              unsigned* __restrict__ counter, double* __restrict__ inc,
                                                              float* __restrict__ dpre, int nop, StateApplyArgs sa) {
#pragma clang fp contract(off)
  __shared__ double s_ce[kWpb][64], s_tl[kWpb][64], s_d0[kWpb][64], s_d1[kWpb][64];
  __shared__ int s_code[kWpb][64];  // -1: negative label; 0-2: class, +4 when the window's prototype moves
  __shared__ double red[kWpb][kDpInc];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * kWpb + wv;
  double acc[kDpInc] = {};  // delta[3][2], count[3], ones (lane 0)
  const bool live = b < B;
  const double* P = state;
  const double ratio = state[2 * K + 1] / state[2 * K + 2];  // num_zero / num_ones at the step start
  const double f = state[2 * K] + update_min;               // PROTO_UPDATE_FACTOR + PROTO_UPDATE_MIN
  double aloss = 0.0, tloss = 0.0;
  for (int i0 = 0; i0 < H; i0 += 64) {  // uniform trip count: every wave reaches the barriers
    const int i = i0 + lane;
    if (live && i < H) {
      const long o = (long)b * H + i;
      const int yi = y[o];
      const double mu = yi == 0 ? 1.0 : ratio;
      mult[o] = (float)mu;
      const double l0 = logits[2 * o], l1 = logits[2 * o + 1];
      const double m = fmax(l0, l1);
      // log(exp(l0 - m) + exp(l1 - m)): the larger logit's term is exp(0) = 1
      // exactly, so one exp (the sum is the same either way round)
      const double em = exp((l0 >= l1 ? l1 : l0) - m);
      s_ce[wv][lane] = (log(1.0 + em) + m - (yi ? l1 : l0)) * mu;
      int code = -1;
      if (yi > 0) {
        const int cc = cls[o];
        const double a0 = protos[2 * o], a1 = protos[2 * o + 1];
        tgt[2 * o] = (float)P[2 * cc];
        tgt[2 * o + 1] = (float)P[2 * cc + 1];
        double mse[3];
        for (int k = 0; k < 3; ++k) {
          const double d0 = a0 - P[2 * k], d1 = a1 - P[2 * k + 1];
          mse[k] = (d0 * d0 + d1 * d1) / 2.0;
        }
        const double pos = mse[cc];
        const double n0 = mse[cc == 0 ? 1 : 0], n1 = mse[cc == 2 ? 1 : 2];
        s_tl[wv][lane] = pos - (n0 + n1);
        code = cc;
        if (pos <= n0 && pos <= n1) {
          s_d0[wv][lane] = f * (a0 - P[2 * cc]);
          s_d1[wv][lane] = f * (a1 - P[2 * cc + 1]);
          code += 4;
        }
      } else {
        tgt[2 * o] = 0.f;
        tgt[2 * o + 1] = 0.f;
      }
      s_code[wv][lane] = code;
      if (dpre) {  // tune_loss's function on the values just written (mult, tgt)
        float* d = dpre + (long)b * nop;
        const int cc = yi > 0 ? cls[o] : 0;
        dpre_host(logits[2 * o], logits[2 * o + 1], yi, (float)mu, protos[2 * o], protos[2 * o + 1],
                  yi > 0 ? (float)P[2 * cc] : 0.f, yi > 0 ? (float)P[2 * cc + 1] : 0.f, d + 2 * i, d + 2 * H + 2 * i);
      }
    }
    __syncthreads();
    if (live && lane == 0) {  // host order, as the per-window loop
      // 8 hosts' LDS values read together (clamped index: no branch around a
      // read), then their adds in host order: one LDS round trip per 8 hosts
      // instead of two dependent ones per host (the loop was LDS-latency-bound:
      // the kernel 22.6 us at H = 50)
      const int n = H - i0 < 64 ? H - i0 : 64;
      for (int j0 = 0; j0 < n; j0 += 8) {
        int cd[8];
        double ce[8], tl[8], e0[8], e1[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int jj = j0 + q < n ? j0 + q : n - 1;
          cd[q] = s_code[wv][jj];
          ce[q] = s_ce[wv][jj];
          tl[q] = s_tl[wv][jj];
          e0[q] = s_d0[wv][jj];
          e1[q] = s_d1[wv][jj];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (j0 + q >= n) break;
          const int code = cd[q];
          aloss += ce[q];
          acc[9] += code >= 0 ? 1.0 : 0.0;
          if (code >= 0) {
            tloss += tl[q];
            if (code == 4) {
              acc[0] += e0[q];
              acc[1] += e1[q];
              acc[6] += 1.0;
            } else if (code == 5) {
              acc[2] += e0[q];
              acc[3] += e1[q];
              acc[7] += 1.0;
            } else if (code == 6) {
              acc[4] += e0[q];
              acc[5] += e1[q];
              acc[8] += 1.0;
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if (live && lane == 0) {
    loss[2 * b] = aloss;
    loss[2 * b + 1] = tloss;
  }
  if (lane == 0)
    for (int k = 0; k < kDpInc; ++k) red[wv][k] = acc[k];
  __syncthreads();
  if (threadIdx.x < kDpInc) {  // fixed tree over the workgroup's windows
    const int k = threadIdx.x;
    __hip_atomic_store(part + (long)blockIdx.x * kDpInc + k, (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the last workgroup sums every workgroup's partials (rows stored
  // write-through above; arrive_last resets the counter)
  __shared__ int s_last;
  if (!arrive_last(counter, gridDim.x, &s_last)) return;
  __shared__ double s_inc[3 * kMaxProtos + 3];
  dp_finish(threadIdx.x, H, B, K, (int)gridDim.x, part, inc, s_inc);
  if (sa.on) {
    // world size 1: the state update right here (every other workgroup read
    // the step-start state before it counted itself done), one launch fewer;
    // the increments from this workgroup's LDS copy
    __syncthreads();
    if (threadIdx.x < kStateThreads) state_apply_body(threadIdx.x, K, state, s_inc, sa);
  }
}

__global__ void tune_state_apply_kernel(int K, double* __restrict__ state, const double* __restrict__ inc,
                                        StateApplyArgs sa) {
  state_apply_body(threadIdx.x, K, state, inc, sa);
}

}  // namespace

hipError_t launch_tune_dataset(int H, int E, int R, const double* series, const double* train_max, float* windows,
                               int* y, int* cls, float* infer, hipStream_t st, hipEvent_t stop) {
  const long n = (long)E * H;
  const int grid = (int)((n + kDsP - 1) / kDsP);
  if (stop) {  // the launch signals `stop` at its end (a fork right after it)
    void* args[] = {&H, &E, &R, &series, &train_max, &windows, &y, &cls, &infer};
    return hipExtLaunchKernel(reinterpret_cast<const void*>(tune_dataset_kernel), dim3(grid), dim3(kDsThreads), args,
                              0, st, nullptr, stop, 0);
  }
  tune_dataset_kernel<<<grid, kDsThreads, 0, st>>>(H, E, R, series, train_max, windows, y, cls, infer);
  return hipGetLastError();
}

// the finishing counter (slot 0: zero in a fresh workspace, reset by the last
// workgroup of every launch), then the partials [nblk][kDpInc]
long tune_dp_workspace_doubles(int B) { return (long)((B + kWpb - 1) / kWpb) * kDpInc + 1; }

hipError_t launch_tune_targets_dp(int H, int K, int B, const float* logits, const float* protos, const int* y,
                                  const int* cls, double* state, double update_min, float* mult, float* tgt,
                                  double* loss, double* inc, double* ws, hipStream_t st, float* dpre, int nop,
                                  const StateApplyArgs* apply, hipEvent_t stop) {
  const int nblk = (B + kWpb - 1) / kWpb;
  unsigned* counter = reinterpret_cast<unsigned*>(ws);   // slot 0 (any batch), the partials after it
  StateApplyArgs sa{};
  if (apply) {
    if (K < 0 || K > kMaxProtos || apply->cr.n < 0 || apply->cr.n > kMaxCond) return hipErrorInvalidValue;
    sa = *apply;
    sa.on = 1;
  }
  if (stop) {  // the launch signals `stop` at its end (a fork right after it)
    double* part = ws + 1;
    void* args[] = {&H, &B, &logits, &protos, &y, &cls, &state, &K, &update_min, &mult, &tgt, &loss, &part,
                    &counter, &inc, &dpre, &nop, &sa};
    return hipExtLaunchKernel(reinterpret_cast<const void*>(tune_targets_dp_kernel), dim3(nblk), dim3(kTB), args, 0,
                              st, nullptr, stop, 0);
  }
  tune_targets_dp_kernel<<<nblk, kTB, 0, st>>>(H, B, logits, protos, y, cls, state, K, update_min, mult, tgt, loss,
                                               ws + 1, counter, inc, dpre, nop, sa);
  return hipGetLastError();
}

hipError_t launch_tune_state_apply(int K, double* state, const double* inc, double decay, const CondRows& cr,
                                   double* dsteps, float* table, double lr, double b1, double b2, hipStream_t st) {
  static_assert(kMaxProtos <= kStateCountLane && kStateCondLane0 + 2 * kMaxCond <= kStateThreads &&
                    kStateThreads <= kTB &&
                    kStateCondLane0 / 64 == (kStateCondLane0 + 2 * kMaxCond - 1) / 64,
                "state apply lane map (a row's two lanes in one wave)");
  if (K < 0 || K > kMaxProtos || cr.n < 0 || cr.n > kMaxCond) return hipErrorInvalidValue;
  tune_state_apply_kernel<<<1, kStateThreads, 0, st>>>(K, state, inc,
                                                       StateApplyArgs{1, decay, cr, dsteps, table, lr, b1, b2});
  return hipGetLastError();
}

}  // namespace pgp
