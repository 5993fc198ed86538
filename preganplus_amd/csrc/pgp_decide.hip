// pgp_decide.hip — K5: the per-container decision of recover_decision
// (recovery/PreGANPlus.py:87-105, recovery/PreGAN.py:77-95) for a batch of
// windows, from K3's keep_orig / final_target and the current placement.
//   keep_orig[b]          -> no change (the original decision stands)
//   cur_host[b,c] == -1   -> unplaced / None container: not considered (so is any
//                            host index outside [0, C): it is never written through)
//   final_target != cur   -> moves[b,c] = final_target, hosts_from[b,cur] = 1
// Integer work over C = H containers per window: one lane per (window,
// container); hosts_from is a per-window OR, one atomicOr per moving container
// (after a zeroing pass).
#include "pgp_device.hpp"

namespace pgp {
namespace {

__global__ __launch_bounds__(256) void decide_kernel(int B, int C, const int* __restrict__ keep,
                                                     const int* __restrict__ target, const int* __restrict__ cur,
                                                     int* __restrict__ moves, int* __restrict__ hosts_from) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * C) return;
  const long b = i / C;
  const int h = cur[i];
  const int t = target[i];
  const bool mv = !keep[b] && h >= 0 && h < C && t != h;
  moves[i] = mv ? t : -1;
  if (mv) atomicOr(hosts_from + b * C + h, 1);
}

// run_model's embedding (PreGANPlus.py:129): emb[b,h] = protos[b,h] where the
// host is flagged (argmax of its logits = 1, ties -> 0) else 0
__global__ __launch_bounds__(256) void embed_kernel(long n, const float* __restrict__ logits,
                                                    const float* __restrict__ protos, float* __restrict__ emb) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const f32x2 l = *reinterpret_cast<const f32x2*>(logits + 2 * i);
  const f32x2 p = *reinterpret_cast<const f32x2*>(protos + 2 * i);
  *reinterpret_cast<f32x2*>(emb + 2 * i) = l[1] > l[0] ? p : f32x2{0.f, 0.f};
}

__global__ __launch_bounds__(256) void zero_kernel(long n, int* __restrict__ p) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0;
}

// one-hot schedule rows from per-container host indices: one lane per
// output float, consecutive lanes consecutive floats of a row (coalesced)
__global__ __launch_bounds__(256) void onehot_kernel(long n, int H, const unsigned char* __restrict__ idx,
                                                     float* __restrict__ sched) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long row = i / H;
  sched[i] = (int)idx[row] == (int)(i - row * H) ? 1.f : 0.f;
}

}  // namespace

hipError_t launch_onehot(int H, long rows, const unsigned char* idx, float* sched, hipStream_t st) {
  const long n = rows * H;
  if (n > 0) onehot_kernel<<<(int)((n + 255) / 256), 256, 0, st>>>(n, H, idx, sched);
  return hipGetLastError();
}

hipError_t launch_decide(int B, int C, const int* keep, const int* target, const int* cur, int* moves,
                         int* hosts_from, hipStream_t st) {
  const long n = (long)B * C;
  const int grid = (int)((n + 255) / 256);
  zero_kernel<<<grid, 256, 0, st>>>(n, hosts_from);
  decide_kernel<<<grid, 256, 0, st>>>(B, C, keep, target, cur, moves, hosts_from);
  return hipGetLastError();
}

hipError_t launch_embed(long n, const float* logits, const float* protos, float* emb, hipStream_t st) {
  if (n > 0) embed_kernel<<<(int)((n + 255) / 256), 256, 0, st>>>(n, logits, protos, emb);
  return hipGetLastError();
}

}  // namespace pgp
