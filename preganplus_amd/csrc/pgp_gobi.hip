// pgp_gobi.hip — GOBI, the schedule producer of the decision path (SURVEY §8f
// row f3): scheduler/GOBI.py:19-42 -> scheduler/BaGTI/src/opt.py:17-33 over
// the energy_latency_16 surrogate (scheduler/BaGTI/src/models.py:8-27), for a
// batch of independent environments.
//
// One 1024-thread workgroup per environment runs the whole optimisation
// in-kernel (the reference's loop: up to 200 AdamW steps on the input matrix,
// one-hot projection after each, stop after 31 unchanged steps).  Thread t < 256
// owns allocation entry t = (container t/16, host t%16): its AdamW moments live
// in registers, and a row's first-argmax is a 16-lane reduction inside one wave.
// The MLP (288-128-128-64-2) and its input gradient are VALU dot products split
// 4-16 ways over the threads; layer 1 (60% of the work, used in both
// directions) sits in LDS as one copy with a 289-float row stride, so row reads
// (forward) and column reads (input gradient) are both bank-conflict-free;
// layers 2-3 are read from L2, forward from transposed copies, backward from
// the natural rows, both coalesced.  Elementwise semantics follow torch's
// CPU kernels (softplus threshold 20, tanhshrink = x - tanh x composite,
// sigmoid backward g(1-y)y, AdamW single-tensor op order); per-iteration AdamW
// scalars (cosine lr) are computed on the host in double, as torch does.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/preganplus.h"
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kH = 16, kF = 2 + kH, kIn = kH * kF;  // 16 containers x [cpu, ips, one-hot 16] = 288
constexpr int kN1 = 128, kN2 = 128, kN3 = 64;
constexpr int kMaxIt = 200, kPatience = 30;

struct GobiW {  // device offsets (floats) into one buffer
  static constexpr int W1T = 0;                    // [288][128]
  static constexpr int W1 = W1T + kIn * kN1;       // [128][288]
  static constexpr int B1 = W1 + kN1 * kIn;        // [128]
  static constexpr int W2T = B1 + kN1;             // [128][128]
  static constexpr int W2 = W2T + kN1 * kN2;       // [128][128]
  static constexpr int B2 = W2 + kN2 * kN1;
  static constexpr int W3T = B2 + kN2;             // [128][64]
  static constexpr int W3 = W3T + kN2 * kN3;       // [64][128]
  static constexpr int B3 = W3 + kN3 * kN2;
  static constexpr int W4 = B3 + kN3;              // [2][64]
  static constexpr int B4 = W4 + 2 * kN3;
  static constexpr int ADAM = B4 + 4;              // [200][4]: decay, step size, sqrt(bc2), lr
  static constexpr int SIZE = ADAM + kMaxIt * 4;
};

__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

constexpr int kT = 1024;          // threads per environment
constexpr int kW1S = kIn + 1;      // LDS row stride of W1: 289 = 33 (mod 64) banks -> row and column reads conflict-free

struct GobiLds {
  float w1[kN1 * kW1S];  // layer-1 weights, natural [128][288] rows padded to 289 (147,968 B)
  float x[kIn];
  float h1[kN1], h2[kN2];
  float g1[kN1], g2[kN2], g3[kN3];
  float part[1024];
  float adam[kMaxIt * 4];  // per-iteration AdamW scalars (GobiW::ADAM)
  int hs[kH];              // each container's host (the one-hot column of its allocation row)
  int dense;               // 1 while the allocation may not be one-hot (a non-one-hot init, iteration 0)
  float o[4];
  int flag[2];
};

// this thread's slices of layers 2-3, loaded once and kept in registers for
// every iteration (forward: W2^T/W3^T column blocks; backward: W2/W3 row blocks)
struct GobiRegs {
  float w2f[16], w3f[8], w3b[8], w2b[16];
  float b1, b2, b3, w40, w41, b40, b41;  // biases (threads < 128 / < 64) and the head, off the critical path
};

__device__ void load_regs(const float* __restrict__ W, GobiRegs& R) {
  const int t = threadIdx.x, o = t & 127, sp = t >> 7, o3 = t & 63, sp3 = t >> 6;
#pragma unroll
  for (int j = 0; j < 16; ++j) R.w2f[j] = W[GobiW::W2T + (sp * 16 + j) * kN2 + o];
#pragma unroll
  for (int j = 0; j < 8; ++j) R.w3f[j] = W[GobiW::W3T + (sp3 * 8 + j) * kN3 + o3];
#pragma unroll
  for (int j = 0; j < 8; ++j) R.w3b[j] = W[GobiW::W3 + (sp * 8 + j) * kN2 + o];
#pragma unroll
  for (int j = 0; j < 16; ++j) R.w2b[j] = W[GobiW::W2 + (sp * 16 + j) * kN1 + o];
  R.b1 = W[GobiW::B1 + o];
  R.b2 = W[GobiW::B2 + o];
  R.b3 = W[GobiW::B3 + o3];
  R.w40 = W[GobiW::W4 + o3];
  R.w41 = W[GobiW::W4 + kN3 + o3];
  R.b40 = W[GobiW::B4];
  R.b41 = W[GobiW::B4 + 1];
}

// pre-activations and their exp / tanh, kept in the registers of the threads
// that own them in both directions (t < 128 for layers 1-2, t < 64 for layer 3),
// so the backward's derivatives need no transcendental
struct FwdKeep {
  float a1, z1, a2, z2, th3;
};
__device__ __forceinline__ float softplus_keep(float a, float& z) {  // softplus (threshold 20), z = exp(a)
  z = expf(a);
  return a > 20.f ? a : log1pf(z);
}
__device__ __forceinline__ float softplus_grad(float g, float a, float z) {  // torch: g * z / (z + 1)
  return a > 20.f ? g : g * z / (z + 1.f);
}

// forward of the surrogate on L.x (all 1024 threads); z in L.o[2]
__device__ void surrogate_fwd(const float* __restrict__ W, const GobiRegs& R, GobiLds& L, FwdKeep& K, bool grad) {
  const int t = threadIdx.x;
  if (L.dense) {  // layer 1, dense: 128 outputs x 8 splits of K = 288 (36 each), W1 rows from LDS
    const int o = t & 127, sp = t >> 7;
    float acc = 0.f;
    const float* wr = L.w1 + o * kW1S + sp * 36;
    const float* xr = L.x + sp * 36;
#pragma unroll 6
    for (int k = 0; k < 36; ++k) acc = fmaf(wr[k], xr[k], acc);
    L.part[t] = acc;
    __syncthreads();
    if (t < kN1) {
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) a += L.part[q * 128 + t];
      a += R.b1;
      K.a1 = a;
      L.h1[t] = softplus_keep(a, K.z1);
    }
    __syncthreads();
  } else {  // layer 1 on a one-hot allocation: per container 2 FMAs (cpu, ips) + its host's column
    if (t < kN1) {
      const float* wr = L.w1 + t * kW1S;
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < kH; ++c) {
        a = fmaf(wr[c * kF], L.x[c * kF], a);
        a = fmaf(wr[c * kF + 1], L.x[c * kF + 1], a);
        a = a + wr[c * kF + 2 + L.hs[c]];  // w * 1.0; the other 15 columns multiply 0
      }
      a += R.b1;
      K.a1 = a;
      L.h1[t] = softplus_keep(a, K.z1);
    }
    __syncthreads();
  }
  {  // layer 2: 128 outputs x 8 splits of K = 128 (16 each)
    const int sp = t >> 7;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = fmaf(R.w2f[j], L.h1[sp * 16 + j], acc);
    L.part[t] = acc;
    __syncthreads();
    if (t < kN2) {
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) a += L.part[q * 128 + t];
      a += R.b2;
      K.a2 = a;
      L.h2[t] = softplus_keep(a, K.z2);
    }
    __syncthreads();
  }
  {  // layer 3: 64 outputs x 16 splits of K = 128 (8 each)
    const int sp = t >> 6;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = fmaf(R.w3f[j], L.h2[sp * 8 + j], acc);
    L.part[t] = acc;
    __syncthreads();
    if (t < kN3) {
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) a += L.part[q * 64 + t];
      a += R.b3;
      K.th3 = tanhf(a);
      const float h3 = a - K.th3;  // Tanhshrink
      // layer 4 (2 outputs) in the same wave 0 (no barrier), sigmoid, z = 0.8 e + 0.2 l
      float p0 = R.w40 * h3, p1 = R.w41 * h3;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        p0 += __shfl_xor(p0, off);
        p1 += __shfl_xor(p1, off);
      }
      // every lane holds the same sums (the butterfly adds commute exactly)
      const float o0 = sigmoid_f(p0 + R.b40), o1 = sigmoid_f(p1 + R.b41);
      if (t == 0) {
        L.o[0] = o0;
        L.o[1] = o1;
        L.o[2] = 0.8f * o0 + 0.2f * o1;
      }
      if (grad) {  // backward start in the same wave: dz/do = (0.8, 0.2) through the sigmoids,
                   // dh3 = W4^T do, through Tanhshrink
        const float d0 = 0.8f * (1.f - o0) * o0, d1 = 0.2f * (1.f - o1) * o1;
        const float gh = R.w40 * d0 + R.w41 * d1;
        L.g3[t] = gh - gh * (1.f - K.th3 * K.th3);
      }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kT) void gobi_kernel(int E, const float* __restrict__ W, const float* __restrict__ init,
                                                  float* __restrict__ result, int* __restrict__ iterations,
                                                  float* __restrict__ fitness, int max_it, float* __restrict__ pre) {
#pragma clang fp contract(off)  // elementwise steps as torch's separate mul/add
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  GobiLds& L = *reinterpret_cast<GobiLds*>(lds_raw);
  const int e = blockIdx.x;
  if (e >= E) return;  // whole workgroup
  const int t = threadIdx.x, c = (t & 255) >> 4, hcol = t & 15;
  const int xi = c * kF + 2 + hcol;  // threads < 256: this thread's allocation entry in the flattened input
  for (int k = t; k < kN1 * kIn; k += kT) {
    const int o = k / kIn, j = k - o * kIn;
    L.w1[o * kW1S + j] = W[GobiW::W1 + k];
  }
  for (int k = t; k < kIn; k += kT) L.x[k] = init[(long)e * kIn + k];
  for (int k = t; k < kMaxIt * 4; k += kT) L.adam[k] = W[GobiW::ADAM + k];
  if (t < 2) L.flag[t] = 0;
  if (t == 0) L.dense = 0;
  GobiRegs R;
  load_regs(W, R);
  __syncthreads();
  if (t < kH) {  // is the init's allocation one-hot?  (then layer 1 is a column gather)
    int ones = 0, other = 0, h = 0;
    for (int j = 0; j < kH; ++j) {
      const float xv = L.x[t * kF + 2 + j];
      if (xv == 1.f) {
        ++ones;
        h = j;
      } else if (xv != 0.f) {
        ++other;
      }
    }
    L.hs[t] = h;
    if (ones != 1 || other) L.dense = 1;
  }
  __syncthreads();
  float m = 0.f, v = 0.f;
  FwdKeep K{0.f, 0.f, 0.f, 0.f, 0.f};
  int equal = 0, it = 0;
  while (it < max_it) {
    surrogate_fwd(W, R, L, K, true);
    // ---- backward to the input (autograd of z; g3 came with the forward) ----
    {  // dh2 = W3^T g3 (128 x K=64, 8 splits of 8), through softplus
      const int sp = t >> 7;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf(R.w3b[j], L.g3[sp * 8 + j], acc);
      L.part[t] = acc;
      __syncthreads();
      if (t == 0) L.flag[(it + 1) & 1] = 0;  // next iteration's flag; its last readers passed barriers since
      if (t < kN2) {
        float a = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) a += L.part[q * 128 + t];
        L.g2[t] = softplus_grad(a, K.a2, K.z2);
      }
      __syncthreads();
    }
    {  // dh1 = W2^T g2 (128 x K=128, 8 splits of 16), through softplus
      const int sp = t >> 7;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) acc = fmaf(R.w2b[j], L.g2[sp * 16 + j], acc);
      L.part[t] = acc;
      __syncthreads();
      if (t < kN1) {
        float a = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) a += L.part[q * 128 + t];
        L.g1[t] = softplus_grad(a, K.a1, K.z1);
      }
      __syncthreads();
    }
    {  // dx for the 256 allocation entries: W1[:, xi] . g1, 4 splits of 32 over the LDS copy
      const int sp = t >> 8;
      float acc = 0.f;
#pragma unroll 8
      for (int o = sp * 32; o < sp * 32 + 32; ++o) acc = fmaf(L.w1[o * kW1S + xi], L.g1[o], acc);
      L.part[t] = acc;
      __syncthreads();
    }
    int changed = 0;
    if (t < 256) {
      const float gx = (L.part[t] + L.part[t + 256]) + (L.part[t + 512] + L.part[t + 768]);
      // ---- AdamW (torch single-tensor, opt.py:18 defaults) on the entry ----
      const float* ad = L.adam + it * 4;
      const float xold = L.x[xi];
      float xv = xold * ad[0];
      m = m + 0.1f * (gx - m);            // exp_avg.lerp_(grad, 1 - beta1)
      v = v * 0.999f + 0.001f * gx * gx;  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
      const float denom = sqrtf(v) / ad[2] + 1e-8f;
      xv = xv + (-ad[1]) * m / denom;     // addcdiv_: self + value * t1 / t2 (ATen's order)
      // ---- one-hot of the row's first argmax (opt.py:9-15) ----
      float best = xv;
      int bi = hcol;
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) {
        const float ov = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        if (ov > best || (ov == best && oi < bi)) {
          best = ov;
          bi = oi;
        }
      }
      if (pre) pre[(long)e * kH * kH + t] = xv;  // test tap: the step's values before the projection
      const float nv = bi == hcol ? 1.f : 0.f;
      changed = nv != xold;
      L.x[xi] = nv;
      if (bi == hcol) L.hs[c] = hcol;
      if (t == 0) L.dense = 0;  // one-hot from here on
    }
    if (changed) L.flag[it & 1] = 1;  // benign race: every writer stores 1
    __syncthreads();
    equal = L.flag[it & 1] ? 0 : equal + 1;
    if (equal > kPatience) break;
    ++it;
  }
  surrogate_fwd(W, R, L, K, false);
  for (int k = t; k < kIn; k += kT) result[(long)e * kIn + k] = L.x[k];
  if (t == 0) {
    iterations[e] = it;
    fitness[e] = L.o[2];
  }
}

}  // namespace
}  // namespace pgp

using namespace pgp;

struct pgp_gobi {
  int H = 0;
  float* d_w = nullptr;
};

namespace {
thread_local std::string g_gerr;
int gfail(int code, const std::string& msg) {
  g_gerr = msg;
  return code;
}
}  // namespace

extern "C" {

size_t pgp_gobi_weight_len(int n_hosts) {
  if (n_hosts != kH) return 0;
  return (size_t)kN1 * kIn + kN1 + kN2 * kN1 + kN2 + kN3 * kN2 + kN3 + 2 * kN3 + 2;
}

int pgp_gobi_create(int n_hosts, const float* weights, size_t len, pgp_gobi** out) {
  if (!out) return gfail(PGP_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (n_hosts != kH) return gfail(PGP_ERR_UNSUPPORTED, "GOBI surrogate: only energy_latency_16 exists (16 hosts)");
  if (!weights || len != pgp_gobi_weight_len(n_hosts)) return gfail(PGP_ERR_ARG, "GOBI weight length mismatch");
  // state-dict order: find.0.weight [128,288], find.0.bias, find.2.weight [128,128], find.2.bias,
  //                   find.4.weight [64,128], find.4.bias, find.6.weight [2,64], find.6.bias
  const float* w1 = weights;
  const float* b1 = w1 + kN1 * kIn;
  const float* w2 = b1 + kN1;
  const float* b2 = w2 + kN2 * kN1;
  const float* w3 = b2 + kN2;
  const float* b3 = w3 + kN3 * kN2;
  const float* w4 = b3 + kN3;
  const float* b4 = w4 + 2 * kN3;
  std::vector<float> h(GobiW::SIZE, 0.f);
  for (int o = 0; o < kN1; ++o)
    for (int k = 0; k < kIn; ++k) {
      h[GobiW::W1 + o * kIn + k] = w1[o * kIn + k];
      h[GobiW::W1T + k * kN1 + o] = w1[o * kIn + k];
    }
  for (int o = 0; o < kN2; ++o)
    for (int k = 0; k < kN1; ++k) {
      h[GobiW::W2 + o * kN1 + k] = w2[o * kN1 + k];
      h[GobiW::W2T + k * kN2 + o] = w2[o * kN1 + k];
    }
  for (int o = 0; o < kN3; ++o)
    for (int k = 0; k < kN2; ++k) {
      h[GobiW::W3 + o * kN2 + k] = w3[o * kN2 + k];
      h[GobiW::W3T + k * kN3 + o] = w3[o * kN2 + k];
    }
  for (int i = 0; i < kN1; ++i) h[GobiW::B1 + i] = b1[i];
  for (int i = 0; i < kN2; ++i) h[GobiW::B2 + i] = b2[i];
  for (int i = 0; i < kN3; ++i) h[GobiW::B3 + i] = b3[i];
  for (int i = 0; i < 2 * kN3; ++i) h[GobiW::W4 + i] = w4[i];
  h[GobiW::B4] = b4[0];
  h[GobiW::B4 + 1] = b4[1];
  // AdamW(lr=0.8, betas (0.9, 0.999), eps 1e-8, weight_decay 1e-2) under
  // CosineAnnealingLR(T_max=10), torch's recursive update, in double as torch does
  const double base = 0.8, wd = 1e-2, T = 10.0;
  double lr = base;
  for (int i = 0; i < kMaxIt; ++i) {
    const int step = i + 1;
    h[GobiW::ADAM + i * 4 + 0] = (float)(1.0 - lr * wd);
    h[GobiW::ADAM + i * 4 + 1] = (float)(lr / (1.0 - std::pow(0.9, step)));
    h[GobiW::ADAM + i * 4 + 2] = (float)std::sqrt(1.0 - std::pow(0.999, step));
    h[GobiW::ADAM + i * 4 + 3] = (float)lr;
    const int ep = i + 1;
    if ((ep - 1 - 10) % 20 == 0)
      lr = lr + base * (1 - std::cos(M_PI / T)) / 2;
    else
      lr = (1 + std::cos(M_PI * ep / T)) / (1 + std::cos(M_PI * (ep - 1) / T)) * lr;
  }
  pgp_gobi* g = new pgp_gobi();
  g->H = n_hosts;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gobi_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)sizeof(GobiLds)) != hipSuccess) {
    delete g;
    return gfail(PGP_ERR_HIP, "GOBI: cannot reserve LDS");
  }
  if (hipMalloc(&g->d_w, h.size() * sizeof(float)) != hipSuccess ||
      hipMemcpy(g->d_w, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
    if (g->d_w) (void)hipFree(g->d_w);
    delete g;
    return gfail(PGP_ERR_HIP, "GOBI weight upload failed");
  }
  *out = g;
  return PGP_OK;
}

int pgp_gobi_destroy(pgp_gobi* g) {
  if (!g) return PGP_OK;
  if (g->d_w) (void)hipFree(g->d_w);
  delete g;
  return PGP_OK;
}

const char* pgp_gobi_last_error(void) { return g_gerr.c_str(); }

int pgp_gobi_optimize(pgp_gobi* g, int n_env, const float* init, float* result, int* iterations, float* fitness,
                      int max_iters, float* pre, void* stream) {
  if (!g) return gfail(PGP_ERR_ARG, "NULL optimiser");
  if (n_env < 0) return gfail(PGP_ERR_ARG, "negative batch");
  if (n_env == 0) return PGP_OK;
  if (!init || !result || !iterations || !fitness) return gfail(PGP_ERR_ARG, "NULL input/output pointer");
  const int mi = (max_iters <= 0 || max_iters > kMaxIt) ? kMaxIt : max_iters;
  gobi_kernel<<<n_env, kT, sizeof(GobiLds), reinterpret_cast<hipStream_t>(stream)>>>(n_env, g->d_w, init, result,
                                                                                     iterations, fitness, mi, pre);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return gfail(PGP_ERR_HIP, std::string("gobi_kernel: ") + hipGetErrorString(e));
  return PGP_OK;
}

}  // extern "C"
