// pgp_train.hip — HIP kernels of the online training steps:
//   * the GAN step (PreGANPlus.py:60-81): Gen/Disc forward, Disc BCE backward,
//     Gen BCE backward through the updated Disc;
//   * batched weight-gradient outer products and AdamW (utils.py:65).
// (The tuning step's forward/backward is pgp_tune.hip.)  The GAN step runs one
// 256-thread workgroup per window on the VALU (the reference steps one window
// per call, PreGANPlus.py:60-81); Gen/Disc weight gradients are batched outer
// products over the windows (dw_outer_kernel).
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_train.hpp"

namespace pgp {
namespace {

constexpr int kTW = 256;

// dW[n][k] += sum_b A[b*lda + n] * X[b*ldx + k] (+ db[n] += sum_b A)
__global__ __launch_bounds__(256) void dw_outer_kernel(int B, int N, int K, const float* __restrict__ A, long lda,
                                                       const float* __restrict__ X, long ldx, float* __restrict__ dW,
                                                       float* __restrict__ db) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx < (long)N * K) {
    const int n = (int)(idx / K), k = (int)(idx - (long)n * K);
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc = fmaf(A[b * lda + n], X[b * ldx + k], acc);
    dW[idx] += acc;
  }
  if (db && idx < N) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += A[b * lda + idx];
    db[idx] += acc;
  }
}

// AdamW, torch single-tensor semantics (torch/optim/adamw.py): p *= 1 - lr*wd;
// m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
  const AdamTensor& t = a.t[blockIdx.y];
  if (!t.active) return;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < t.n; i += (long)gridDim.x * 256) {
    const long o = t.off + i;
    const float g = a.grad[o];
    float p = a.param[o] * (1.0f - a.lr_wd);
    const float m = a.m[o] + (1.0f - a.b1) * (g - a.m[o]);
    const float v = a.b2 * a.v[o] + (1.0f - a.b2) * g * g;
    p -= t.step_size * m / (sqrtf(v) / t.bc2_sqrt + a.eps);
    a.param[o] = p;
    a.m[o] = m;
    a.v[o] = v;
  }
}

// ============================================================================
// GAN: forward (saves activations), Disc BCE backward, Gen BCE backward.
// P points at the gen section (Pg) and disc section (Pd) of the master buffer.
// ============================================================================
template <int H>
__device__ void gan_disc_fwd(float* S, const float* Pd, float* red) {
  using G = TGeo<H>;
  const int tid = threadIdx.x;
  for (int o = tid; o < 64; o += kTW) {
    float acc = Pd[G::D_B1 + o];
    const float* w = Pd + G::D_W1 + (long)o * G::DIN;
    for (int k = 0; k < G::DIN; ++k) acc = fmaf(w[k], S[G::GS_Z + k], acc);
    S[G::GS_DD + o] = acc;  // LeakyReLU(True) = identity
  }
  __syncthreads();
  if (tid < 2) {
    float acc = Pd[G::D_B2 + tid];
    for (int k = 0; k < 64; ++k) acc = fmaf(Pd[G::D_W2 + tid * 64 + k], S[G::GS_DD + k], acc);
    red[tid] = acc;
  }
  __syncthreads();
  if (tid == 0) {
    const float m = fmaxf(red[0], red[1]), e0 = expf(red[0] - m), e1 = expf(red[1] - m);
    S[G::GS_P] = e0 / (e0 + e1);
    S[G::GS_P + 1] = e1 / (e0 + e1);
  }
  __syncthreads();
}

// nn.BCELoss (mean over the 2 probs) -> softmax -> Disc2 -> Disc1 hidden
template <int H>
__device__ void gan_disc_bwd_local(float* S, const float* Pd, float t0, float t1) {
  using G = TGeo<H>;
  const int tid = threadIdx.x;
  if (tid == 0) {
    const float p0 = S[G::GS_P], p1 = S[G::GS_P + 1];
    // torch BCE grad: (p - t) / max(p (1 - p), 1e-12) / N
    const float dp0 = (p0 - t0) / fmaxf(p0 * (1.f - p0), 1e-12f) * 0.5f;
    const float dp1 = (p1 - t1) / fmaxf(p1 * (1.f - p1), 1e-12f) * 0.5f;
    const float s = p0 * dp0 + p1 * dp1;
    S[G::GS_DO] = p0 * (dp0 - s);
    S[G::GS_DO + 1] = p1 * (dp1 - s);
  }
  __syncthreads();
  for (int k = tid; k < 64; k += kTW)
    S[G::GS_DDD + k] = Pd[G::D_W2 + k] * S[G::GS_DO] + Pd[G::D_W2 + 64 + k] * S[G::GS_DO + 1];
  __syncthreads();
}

template <int H>
__global__ __launch_bounds__(kTW) void gan_fwd_kernel(int B, const float* __restrict__ emb /*[B][2H]*/,
                                                      const float* __restrict__ sched, const float* __restrict__ Pg,
                                                      const float* __restrict__ Pd, float* __restrict__ scr,
                                                      float* __restrict__ ns_out, float* __restrict__ probs) {
  using G = TGeo<H>;
  __shared__ float red[16];
  const int b = blockIdx.x;
  if (b >= B) return;
  float* S = scr + (long)b * G::GS_SIZE;
  const int tid = threadIdx.x;
  for (int k = tid; k < 2 * H; k += kTW) S[G::GS_X + k] = emb[(long)b * 2 * H + k];
  for (int k = tid; k < H * H; k += kTW) {
    const float s = sched[(long)b * H * H + k];
    S[G::GS_X + 2 * H + k] = s;
    S[G::GS_Z + k] = s;
  }
  __syncthreads();
  for (int o = tid; o < 64; o += kTW) {
    float acc = Pg[G::G_B1 + o];
    const float* w = Pg + G::G_W1 + (long)o * G::GIN;
    for (int k = 0; k < G::GIN; ++k) acc = fmaf(w[k], S[G::GS_X + k], acc);
    S[G::GS_H + o] = acc;
  }
  __syncthreads();
  for (int o = tid; o < H * H; o += kTW) {
    float acc = Pg[G::G_B2 + o];
    const float* w = Pg + G::G_W2 + (long)o * 64;
    for (int k = 0; k < 64; ++k) acc = fmaf(w[k], S[G::GS_H + k], acc);
    const float t = tanhf(acc);
    S[G::GS_T + o] = t;
    const float nv = S[G::GS_Z + o] + 4.0f * t;
    S[G::GS_Z + H * H + o] = nv;
    ns_out[(long)b * H * H + o] = nv;
  }
  __syncthreads();
  gan_disc_fwd<H>(S, Pd, red);
  if (tid < 2) probs[(long)b * 2 + tid] = S[G::GS_P + tid];
}

// Disc step: target [B][2] -> GS_DO, GS_DDD (weight grads by dw_outer over the batch)
template <int H>
__global__ __launch_bounds__(kTW) void gan_disc_bwd_kernel(int B, const float* __restrict__ target,
                                                           const float* __restrict__ Pd, float* __restrict__ scr) {
  using G = TGeo<H>;
  const int b = blockIdx.x;
  if (b >= B) return;
  gan_disc_bwd_local<H>(scr + (long)b * G::GS_SIZE, Pd, target[2 * b], target[2 * b + 1]);
}

// Gen step: Disc forward with the UPDATED Disc, BCE toward [0,1], back through
// Disc into the new schedule, tanh, Gen2 -> GS_DY, GS_DH.
template <int H>
__global__ __launch_bounds__(kTW) void gan_gen_bwd_kernel(int B, const float* __restrict__ Pg,
                                                          const float* __restrict__ Pd, float* __restrict__ scr) {
  using G = TGeo<H>;
  __shared__ float red[16];
  const int b = blockIdx.x;
  if (b >= B) return;
  float* S = scr + (long)b * G::GS_SIZE;
  const int tid = threadIdx.x;
  gan_disc_fwd<H>(S, Pd, red);
  gan_disc_bwd_local<H>(S, Pd, 0.f, 1.f);
  for (int k = tid; k < H * H; k += kTW) {
    float dz = 0.f;  // d(ns_k) = sum_o Wd1[o][H^2 + k] dDD[o]
    for (int o = 0; o < 64; ++o) dz = fmaf(Pd[G::D_W1 + (long)o * G::DIN + H * H + k], S[G::GS_DDD + o], dz);
    const float t = S[G::GS_T + k];
    S[G::GS_DY + k] = 4.0f * dz * (1.f - t * t);
  }
  __syncthreads();
  for (int u = tid; u < 64; u += kTW) {
    float acc = 0.f;
    for (int k = 0; k < H * H; ++k) acc = fmaf(Pg[G::G_W2 + (long)k * 64 + u], S[G::GS_DY + k], acc);
    S[G::GS_DH + u] = acc;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
long gan_scratch_floats(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return TGeo<h>::GS_SIZE;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

hipError_t launch_dw_outer(int B, int N, int K, const float* A, long lda, const float* X, long ldx, float* dW,
                           float* db, hipStream_t st) {
  const long n = (long)N * K;
  const long nb = (n > N ? n : N);
  dw_outer_kernel<<<(int)((nb + 255) / 256), 256, 0, st>>>(B, N, K, A, lda, X, ldx, dW, db);
  return hipGetLastError();
}

hipError_t launch_adamw(const AdamArgs& a, hipStream_t st) {
  long maxn = 0;
  for (int i = 0; i < a.ntensors; ++i) maxn = a.t[i].n > maxn ? a.t[i].n : maxn;
  int gx = (int)((maxn + 255) / 256);
  gx = gx > 1024 ? 1024 : (gx < 1 ? 1 : gx);
  adamw_kernel<<<dim3(gx, a.ntensors), 256, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_gan_fwd(int H, int B, const float* emb, const float* sched, const float* Pg, const float* Pd,
                          float* scr, float* ns_out, float* probs, hipStream_t st) {
  switch (H) {
#define CASE(h)                                                                         \
  case h:                                                                               \
    gan_fwd_kernel<h><<<B, kTW, 0, st>>>(B, emb, sched, Pg, Pd, scr, ns_out, probs);    \
    return hipGetLastError();
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_disc_bwd(int H, int B, const float* target, const float* Pd, float* Gdd, float* scr,
                               hipStream_t st) {
  switch (H) {
#define CASE(h)                                                                                              \
  case h: {                                                                                                  \
    using G = TGeo<h>;                                                                                       \
    gan_disc_bwd_kernel<h><<<B, kTW, 0, st>>>(B, target, Pd, scr);                                           \
    hipError_t e = hipGetLastError();                                                                        \
    if (e != hipSuccess) return e;                                                                           \
    e = launch_dw_outer(B, 2, 64, scr + G::GS_DO, G::GS_SIZE, scr + G::GS_DD, G::GS_SIZE, Gdd + G::D_W2,     \
                        Gdd + G::D_B2, st);                                                                  \
    if (e != hipSuccess) return e;                                                                           \
    return launch_dw_outer(B, 64, G::DIN, scr + G::GS_DDD, G::GS_SIZE, scr + G::GS_Z, G::GS_SIZE,            \
                           Gdd + G::D_W1, Gdd + G::D_B1, st);                                                \
  }
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_gen_bwd(int H, int B, const float* Pg, const float* Pd, float* Gdg, float* scr,
                              hipStream_t st) {
  switch (H) {
#define CASE(h)                                                                                             \
  case h: {                                                                                                 \
    using G = TGeo<h>;                                                                                      \
    gan_gen_bwd_kernel<h><<<B, kTW, 0, st>>>(B, Pg, Pd, scr);                                               \
    hipError_t e = hipGetLastError();                                                                       \
    if (e != hipSuccess) return e;                                                                          \
    e = launch_dw_outer(B, h * h, 64, scr + G::GS_DY, G::GS_SIZE, scr + G::GS_H, G::GS_SIZE, Gdg + G::G_W2, \
                        Gdg + G::G_B2, st);                                                                 \
    if (e != hipSuccess) return e;                                                                          \
    return launch_dw_outer(B, 64, G::GIN, scr + G::GS_DH, G::GS_SIZE, scr + G::GS_X, G::GS_SIZE,            \
                           Gdg + G::G_W1, Gdg + G::G_B1, st);                                               \
  }
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
