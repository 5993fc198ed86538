// pgp_sim.hip — the GAN-label simulation: Stats.runSimulation
// (stats/Stats.py:154-177) scored for a batch of environments, and the BCE
// target of PreGANPlus.py:65-66 (run_simulation, recovery/PreGANSrc/src/utils.py:97-100).
//
// One 128-thread workgroup per environment: both schedules are staged into
// LDS rows (coalesced, 8 loads in flight per thread; odd row stride), then
// wave 0 scores the generator's schedule and wave 1 the original.  Lane c is
// container c and host c: its record fields are read lane-indexed into
// registers up front; a row's argmax is a per-lane scan of its LDS row, and
// cross-lane reads (target host availability, ranks) are shuffles.  Integer
// and fp64 bookkeeping, reproducing the reference's order of operations so the
// scores are bit-identical to Python's:
//   * first argmax of each placed container's row (list.index(max(list)));
//   * a move is applied when it changes the host and getPlacementPossible
//     (simulator/Simulator.py:89-105) admits it against the host's CURRENT
//     availability (filter_placement, scheduler/Scheduler.py:22-27, keeps every
//     such decision);
//   * host h's IPS = its staying containers in containerlist order, then the
//     containers moved in, in decision order (= placed containers sorted by
//     (old host, id), the np.concatenate(host_alloc) order), summed left to right;
//   * PM.powerFromCPU (metrics/powermodels/PM.py:11-16) with Python's floor,
//     float modulo and negative list indexing (an index the reference would
//     raise IndexError on gives NaN); energy summed over hosts in order.
// No FMA contraction anywhere (Python rounds every operation).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "../../include/preganplus.h"
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kMaxH = 64, kNP = 11;

struct SimLds {  // one per wave (schedule)
  int hid[kMaxH];                // by container
  int stay[kMaxH], into[kMaxH];  // by position in np.concatenate(host_alloc): host it stays on / moves to (-1)
  double app[kMaxH], pw[kMaxH];  // apparent IPS by position; power by host
};

__device__ double py_power(const double* __restrict__ pl, double cpu) {
#pragma clang fp contract(off)
  const double q = cpu / 10.0;
  if (!(fabs(q) < 1e15)) return NAN;  // math.floor(nan / inf) raises in the reference
  const double fl = floor(q);
  const long idx = (long)fl;
  const long ri = cpu != 10.0 * fl ? idx + 1 : idx;  // cpu % 10 != 0 (10*fl is exact: a multiple of 10)
  if (idx < -kNP || idx >= kNP || ri < -kNP || ri >= kNP) return NAN;  // IndexError in the reference
  const double left = pl[idx < 0 ? idx + kNP : idx];
  const double right = pl[ri < 0 ? ri + kNP : ri];
  const double alpha = q - fl;
  return alpha * right + (1.0 - alpha) * left;
}

__host__ __device__ inline int sched_stride(int H) { return H | 1; }  // odd row stride: row-per-lane LDS reads conflict-free
inline size_t sim_lds_bytes(int H) { return sizeof(float) * 2 * H * sched_stride(H); }

__global__ __launch_bounds__(128) void simulate_kernel(int H, int E, const double* __restrict__ envs,
                                                       const float* __restrict__ sn, const float* __restrict__ so,
                                                       double* __restrict__ out, float* __restrict__ target) {
#pragma clang fp contract(off)
  __shared__ SimLds S[2];
  __shared__ double sc[2];
  extern __shared__ __attribute__((aligned(16))) float sch_all[];
  const int e = blockIdx.x;
  if (e >= E) return;  // whole workgroup
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int HS = sched_stride(H), HH = H * H;
  const double* v = envs + (size_t)e * (2 + 20 * H);
  const bool lane_ok = l < H;
  // the record, lane-indexed (container l / host l), loads issued up front
  const int hid = lane_ok ? (int)v[2 + l] : -1;
  const double base = lane_ok ? v[2 + H + l] : 0.0, ram = lane_ok ? v[2 + 2 * H + l] : 0.0;
  const double disk = lane_ok ? v[2 + 3 * H + l] : 0.0, app = lane_ok ? v[2 + 4 * H + l] : 0.0;
  const double ipsav = lane_ok ? v[2 + 5 * H + l] : 0.0, ramav = lane_ok ? v[2 + 6 * H + l] : 0.0;
  const double diskav = lane_ok ? v[2 + 7 * H + l] : 0.0, cap = lane_ok ? v[2 + 8 * H + l] : 1.0;
  double pl[kNP];
#pragma unroll
  for (int k = 0; k < kNP; ++k) pl[k] = lane_ok ? v[2 + 9 * H + l * kNP + k] : 0.0;
  SimLds& L = S[w];
  L.hid[l] = hid;
  {  // both schedules -> LDS rows (coalesced reads, 8 in flight per thread)
    constexpr int U = 8;
    const float* g0 = sn + (size_t)e * HH;
    const float* g1 = so + (size_t)e * HH;
    for (int i0 = threadIdx.x; i0 < HH; i0 += 128 * U) {
      float a[U], b[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * 128;
        a[u] = i < HH ? g0[i] : 0.f;
        b[u] = i < HH ? g1[i] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * 128;
        if (i < HH) {
          const int r = i / H, j = i - r * H;
          sch_all[r * HS + j] = a[u];
          sch_all[H * HS + r * HS + j] = b[u];
        }
      }
    }
  }
  __syncthreads();
  int nh = -1;
  if (hid >= 0) {  // first argmax of the container's row: max() keeps the first maximal item, index() finds it
    const float* row = sch_all + w * H * HS + l * HS;
    float best = row[0];
    int bi = 0;
#pragma unroll 8
    for (int j = 1; j < H; ++j) {
      const float x = row[j];
      if (x > best) {
        best = x;
        bi = j;
      }
    }
    nh = bi;
  }
  int moved = 0;
  {  // getPlacementPossible against the target host's current availability (held by lane nh)
    const int src = nh < 0 ? 0 : nh;
    const double iav = __shfl(ipsav, src), rav = __shfl(ramav, src), dav = __shfl(diskav, src);
    if (hid >= 0 && nh != hid) moved = base <= iav && ram <= rav && disk <= dav;
  }
  const bool placed = hid >= 0;
  const int np = __popcll(__ballot(placed));
  {  // position in np.concatenate(host_alloc): sorted by (host, id)
    int rank = 0;
#pragma unroll 8
    for (int c = 0; c < H; ++c) {
      const int hc = L.hid[c];
      rank += hc >= 0 && (hc < hid || (hc == hid && c < l));
    }
    if (placed) {
      L.stay[rank] = moved ? -1 : hid;
      L.into[rank] = moved ? nh : -1;
      L.app[rank] = app;
    }
  }
  __syncthreads();
  if (lane_ok) {  // lane = host
    double ips = 0.0;
#pragma unroll 4
    for (int k = 0; k < np; ++k)  // staying containers, containerlist order
      if (L.stay[k] == l) ips = ips + L.app[k];
#pragma unroll 4
    for (int k = 0; k < np; ++k)  // moved in, decision order
      if (L.into[k] == l) ips = ips + L.app[k];
    const double xc = 100.0 * (ips / cap);
    L.pw[l] = py_power(pl, xc < 100.0 ? xc : 100.0);  // min(100, x)
  }
  __syncthreads();
  if (l == 0) {
    double en = 0.0;
#pragma unroll 8
    for (int h = 0; h < H; ++h) en = en + L.pw[h];
    en = en * v[0];
    const double score = 0.8 * en + 0.2 * v[1];
    out[(size_t)e * 4 + 2 * w] = en;
    out[(size_t)e * 4 + 2 * w + 1] = score;
    sc[w] = score;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // PreGANPlus.py:66: [0, 1] if new_score <= orig_score else [1, 0]
    const bool le = sc[0] <= sc[1];
    target[2 * e] = le ? 0.f : 1.f;
    target[2 * e + 1] = le ? 1.f : 0.f;
  }
}

}  // namespace

hipError_t launch_simulate(int H, int E, const double* envs, const float* new_sched, const float* orig_sched,
                           double* out, float* target, hipStream_t st) {
  if (H < 1 || H > kMaxH || E < 0) return hipErrorInvalidValue;
  if (E == 0) return hipSuccess;
  simulate_kernel<<<E, 128, sim_lds_bytes(H), st>>>(H, E, envs, new_sched, orig_sched, out, target);
  return hipGetLastError();
}

}  // namespace pgp

using namespace pgp;

extern "C" {

size_t pgp_sim_env_len(int n_hosts) { return n_hosts > 0 ? (size_t)(2 + 20 * n_hosts) : 0; }

int pgp_simulate(int n_hosts, int n_env, const double* envs, const float* new_sched, const float* orig_sched,
                 double* out, float* target, void* stream) {
  if (n_hosts < 1 || n_hosts > kMaxH)
    return set_error(PGP_ERR_UNSUPPORTED, "pgp_simulate: 1 <= hosts <= 64 (one lane per container)");
  if (n_env < 0) return set_error(PGP_ERR_ARG, "pgp_simulate: negative batch");
  if (n_env == 0) return PGP_OK;
  if (!envs || !new_sched || !orig_sched || !out || !target)
    return set_error(PGP_ERR_ARG, "pgp_simulate: NULL pointer");
  simulate_kernel<<<n_env, 128, sim_lds_bytes(n_hosts), reinterpret_cast<hipStream_t>(stream)>>>(
      n_hosts, n_env, envs, new_sched, orig_sched, out, target);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(PGP_ERR_HIP, std::string("simulate_kernel: ") + hipGetErrorString(e));
  return PGP_OK;
}

}  // extern "C"
