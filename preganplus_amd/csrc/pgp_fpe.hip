// pgp_fpe.hip — K4: PreGAN's FPE_16 encoder, decoders and diagnosis, one
// window per lane, for H = 16 (shipped FPE_16) and H = 50 (the same reference
// code at n_hosts = 50, BASELINE config C4; reference
// recovery/PreGANSrc/src/models.py:10-115, recovery/PreGAN.py:97-120).
//
// Per window the work after the GAT is tiny once folded (pgp_pack.cpp,
// FpeGeo): the GAT node mean has rank 3, so every MHA token is P u_w with
// u_w = [GRU state; r-weighted raw features] (6 floats) and the MHA, V,
// out_proj, encoder and both decoders collapse to a 6x6 score form and one
// [4H x 18] affine map.  The GAT's graph-wise edge softmax is the only H^2
// term; it stays on the VALU (an indicator-weighted sum, not a GEMM), one
// window per lane, weights at wave-uniform addresses (scalar loads).
//   GRU(3H -> 3), 3 steps, torch gate order (r, z, n), h0 supplied by the caller
//   GAT node mean: r_i = sum_j softmax_ij over all H^2 edges; the edge term
//     exp(lrelu(s_i + t_j) - m) factorises per branch into node exponentials
//     A_j = 2^(t_j - tmax), C_j = 2^(0.01 (t_j - tmax)):
//       r_i = E1_i sum_{j: s_i + t_j > 0} A_j + E2_i (sum_j C_j - sum_{j: s_i + t_j > 0} C_j)
//     so an edge costs one add with output clamp (the 0/1 branch indicator:
//     2^64 (s_i + t_j) clamped to [0, 1]) and one packed FMA into {SA, SC}.
//     r_i >= E2_i sum_j C_j, so the subtraction loses no relative accuracy.
//   MHA (1 head) as scores u_s^T M6 u_t + beta6.u_t, softmax over t
//   [4H x 18] map -> per host {a0, a1, p0, p1}: softmax / sigmoid, detect
//   (argmax, ties -> 0), embed, nearest of K = 3 prototypes (utils.py
//   get_classes), any-anomaly flag.
// The embedding goes to the workspace row K3 (pgp_gan.hip) reads.
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kFpeThreads = 64;
// 2^64: (s + t) * 2^64 >= 1 for every positive sum the scores produce (|s|,
// |t| < 2^60); a positive sum below 2^-64 gets a fraction, i.e. a convex
// combination of two edge values that agree to ~2^-64 there
constexpr float kBig = 18446744073709551616.0f;

PGP_DEV float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

template <int H>
__global__ __launch_bounds__(kFpeThreads) void fpe_kernel(FpeArgs a) {
  using F = FpeGeo<H>;
  constexpr int NIN = F::NIN;
  const float* __restrict__ T = a.tab;
  const long b = (long)blockIdx.x * kFpeThreads + threadIdx.x;
  if (b >= a.B) return;
  const float* __restrict__ xb = a.windows + b * 3 * NIN;

  float hs[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) hs[k] = a.h0[b * 3 + k];
  float u[3][6] = {};  // per step: GRU state after the step, r-weighted raw features

  for (int w = 0; w < 3; ++w) {
    const float* __restrict__ xw = xb + w * NIN;
    // ---- pass 1: GRU input product, node scores s / t (log2e-scaled) ----
    float gi[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) gi[i] = 0.f;
    float t[H];
    float smax = -INFINITY, tmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float x0 = xw[3 * i], x1 = xw[3 * i + 1], x2 = xw[3 * i + 2];
#pragma unroll
      for (int g = 0; g < 9; ++g)
        gi[g] = fmaf(T[F::F_WIH + g * NIN + 3 * i + 2], x2,
                     fmaf(T[F::F_WIH + g * NIN + 3 * i + 1], x1, fmaf(T[F::F_WIH + g * NIN + 3 * i], x0, gi[g])));
      const float s = fmaf(T[F::F_UV], x0, fmaf(T[F::F_UV + 1], x1, T[F::F_UV + 2] * x2));
      t[i] = fmaf(T[F::F_UV + 4], x0, fmaf(T[F::F_UV + 5], x1, T[F::F_UV + 6] * x2));
      smax = fmaxf(smax, s);
      tmax = fmaxf(tmax, t[i]);
    }
    // ---- GRU cell (torch.nn.GRU, gates r, z, n) ----
    {
      float gh[9];
#pragma unroll
      for (int i = 0; i < 9; ++i)
        gh[i] = fmaf(T[F::F_WHH + 3 * i], hs[0], fmaf(T[F::F_WHH + 3 * i + 1], hs[1], T[F::F_WHH + 3 * i + 2] * hs[2]));
      float hn[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float r = sigm(gi[k] + gh[k] + T[F::F_BRZ + k]);
        const float z = sigm(gi[3 + k] + gh[3 + k] + T[F::F_BRZ + 3 + k]);
        const float n = tanhf(gi[6 + k] + T[F::F_BIN + k] + r * (gh[6 + k] + T[F::F_BHN + k]));
        hn[k] = (1.f - z) * n + z * hs[k];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) hs[k] = hn[k];
    }
    // ---- GAT, mean over nodes ----
    const float mraw = smax + tmax;
    const float m = fmaxf(mraw, 0.01f * mraw);  // max over edges of lrelu(s_i + t_j)
    const float k1 = __builtin_amdgcn_exp2f(mraw - m);
    const float k2 = __builtin_amdgcn_exp2f(0.01f * mraw - m);
    f32x2 ac[H];
    float ctot = 0.f;
#pragma unroll
    for (int j = 0; j < H; ++j) {
      ac[j] = f32x2{__builtin_amdgcn_exp2f(t[j] - tmax), __builtin_amdgcn_exp2f(0.01f * (t[j] - tmax))};
      ctot += ac[j][1];
      t[j] *= kBig;
    }
    float Z = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f;
    const float us0 = T[F::F_UV], us1 = T[F::F_UV + 1], us2 = T[F::F_UV + 2];
    // two source nodes per trip: their feature loads (L1/L2 hits; with one
    // window per lane no other wave on the SIMD hides them) share one wait
    static_assert(H % 2 == 0, "node pairs");
#pragma unroll 1
    for (int i = 0; i < H; i += 2) {
      float xs[2][3], sv[2];
      f32x2 pa[2], pb[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        xs[q][0] = xw[3 * (i + q)];
        xs[q][1] = xw[3 * (i + q) + 1];
        xs[q][2] = xw[3 * (i + q) + 2];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        sv[q] = fmaf(us0, xs[q][0], fmaf(us1, xs[q][1], us2 * xs[q][2]));
        pa[q] = f32x2{0.f, 0.f};
        pb[q] = f32x2{0.f, 0.f};
      }
#pragma unroll
      for (int j = 0; j < H; j += 2) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float m0 = __builtin_amdgcn_fmed3f(sv[q] * kBig + t[j], 0.f, 1.f);
          pa[q] = __builtin_elementwise_fma(f32x2{m0, m0}, ac[j], pa[q]);
          const float m1 = __builtin_amdgcn_fmed3f(sv[q] * kBig + t[j + 1], 0.f, 1.f);
          pb[q] = __builtin_elementwise_fma(f32x2{m1, m1}, ac[j + 1], pb[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x2 p = pa[q] + pb[q];
        const float s = sv[q];
        const float r = __builtin_amdgcn_exp2f(s - smax) * k1 * p[0] +
                        __builtin_amdgcn_exp2f(0.01f * (s - smax)) * k2 * (ctot - p[1]);
        Z += r;
        g0 = fmaf(r, xs[q][0], g0);
        g1 = fmaf(r, xs[q][1], g1);
        g2 = fmaf(r, xs[q][2], g2);
      }
    }
    const float iz = 1.0f / Z;
    // shift register over the steps (static indices)
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      u[0][k] = u[1][k];
      u[1][k] = u[2][k];
    }
    u[2][0] = hs[0];
    u[2][1] = hs[1];
    u[2][2] = hs[2];
    u[2][3] = g0 * iz;
    u[2][4] = g1 * iz;
    u[2][5] = g2 * iz;
  }

  // ---- single-head attention over the 3 steps, in u-space ----
  float ub[3][6];
  {
    float mt[3][6], bt[3];
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) {
      float bb = 0.f;
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        float acc = 0.f;
#pragma unroll
        for (int f = 0; f < 6; ++f) acc = fmaf(T[F::F_M6 + e * 6 + f], u[tt][f], acc);
        mt[tt][e] = acc;
        bb = fmaf(T[F::F_BETA6 + e], u[tt][e], bb);
      }
      bt[tt] = bb;
    }
#pragma unroll
    for (int ss = 0; ss < 3; ++ss) {
      float sc[3];
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) {
        float acc = bt[tt];
#pragma unroll
        for (int e = 0; e < 6; ++e) acc = fmaf(u[ss][e], mt[tt][e], acc);
        sc[tt] = acc;
      }
      const float mx = fmaxf(sc[0], fmaxf(sc[1], sc[2]));
      float p[3], ps = 0.f;
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) {
        p[tt] = __builtin_amdgcn_exp2f(sc[tt] - mx);
        ps += p[tt];
      }
      const float ip = 1.0f / ps;
#pragma unroll
      for (int e = 0; e < 6; ++e) ub[ss][e] = (p[0] * u[0][e] + p[1] * u[1][e] + p[2] * u[2][e]) * ip;
    }
  }

  // ---- folded encoder + decoders, softmax / sigmoid, detect, diagnose ----
  const float* P = T + F::F_PROTO;
  int anyf = 0;
  float* emb = a.emb + b * Geo<H>::EP;
#pragma unroll 2
  for (int h = 0; h < H; ++h) {
    float o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = 4 * h + q;
      float acc = T[F::F_B2 + n];
#pragma unroll
      for (int ss = 0; ss < 3; ++ss)
#pragma unroll
        for (int e = 0; e < 6; ++e) acc = fmaf(T[F::F_W6 + n * F::KU + ss * 6 + e], ub[ss][e], acc);
      o[q] = acc;
    }
    const float mx = fmaxf(o[0], o[1]);
    const float e0 = __expf(o[0] - mx), e1 = __expf(o[1] - mx);
    const float is = 1.0f / (e0 + e1);
    const float s0 = e0 * is, s1 = e1 * is;
    const float p0 = sigm(o[2]), p1 = sigm(o[3]);
    const bool an = s1 > s0;  // torch.argmax of the softmax: ties -> 0 (PreGAN.py:111, :119)
    const float m0 = an ? p0 : 0.f, m1 = an ? p1 : 0.f;
    int cl = -1;
    if (!(m0 == 0.f && m1 == 0.f)) {
      float best = INFINITY;
#pragma unroll
      for (int k = 0; k < F::K; ++k) {
        const float d0 = m0 - P[2 * k], d1 = m1 - P[2 * k + 1];
        const float dist = (d0 * d0 + d1 * d1) * 0.5f;
        if (dist < best) {
          best = dist;
          cl = k;
        }
      }
    }
    anyf |= an ? 1 : 0;
    *reinterpret_cast<float2*>(a.scores + (b * H + h) * 2) = make_float2(s0, s1);
    *reinterpret_cast<float2*>(a.protos + (b * H + h) * 2) = make_float2(p0, p1);
    *reinterpret_cast<float2*>(emb + 2 * h) = make_float2(m0, m1);
    a.cls[b * H + h] = cl;
  }
  a.any_anom[b] = anyf;
}

template <int H>
hipError_t launch(const FpeArgs& a, hipStream_t st) {
  const int grid = (a.B + kFpeThreads - 1) / kFpeThreads;
  fpe_kernel<H><<<grid, kFpeThreads, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_fpe(int H, const FpeArgs& a, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return launch<h>(a, st);
    PGP_FOR_EACH_FPE_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
