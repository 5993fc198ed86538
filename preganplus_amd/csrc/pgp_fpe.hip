// pgp_fpe.hip — K4: PreGAN's FPE_16 encoder, decoders and diagnosis, one
// window per lane (BASELINE config C4; reference recovery/PreGANSrc/src/models.py:10-115,
// recovery/PreGAN.py:97-120).
//
// Per window the whole model is ~10k multiply-adds over a 576-byte input: far too
// little per window to amortise an MFMA tiling's operand shuffles, so each lane
// owns one window and the folded weights (pgp_pack.cpp, FpeGeo) are read at
// wave-uniform addresses (scalar loads, shared by the 64 windows of a wave).
//   GRU(3H -> 3), 3 steps, torch gate order (r, z, n), h0 supplied by the caller
//   GAT node mean: r_i = sum_j softmax_ij over all H^2 edges; the edge term
//     exp(lrelu(s_i + t_j) - m) factorises per branch into node exponentials,
//     so a step costs 4H exp2 and H^2 compare/selects instead of H^2 exp
//   MHA (1 head, E = 3 + H) as scores c_s^T M c_t + beta.c_t, softmax over t
//   one [4H x 3E] matrix (V, out_proj, encoder, decoders folded) -> per host
//   {a0, a1, p0, p1}: softmax / sigmoid, detect (argmax, ties -> 0), embed,
//   nearest of K = 3 prototypes (utils.py get_classes), any-anomaly flag.
// The embedding goes to the workspace row K3 (pgp_gan.hip) reads.
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kFpeThreads = 64;

PGP_DEV float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

template <int H>
__global__ __launch_bounds__(kFpeThreads) void fpe_kernel(FpeArgs a) {
  using F = FpeGeo<H>;
  constexpr int E = F::E, NIN = F::NIN;
  const float* __restrict__ T = a.tab;
  const long b = (long)blockIdx.x * kFpeThreads + threadIdx.x;
  if (b >= a.B) return;
  const float* __restrict__ xw = a.windows + b * 3 * NIN;

  float hs[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) hs[k] = a.h0[b * 3 + k];
  float c[3][E];

#pragma unroll
  for (int w = 0; w < 3; ++w) {
    float x[NIN];
#pragma unroll
    for (int q = 0; q < NIN / 4; ++q) {
      const f32x4 v = ld4(xw + w * NIN + 4 * q);
      x[4 * q] = v[0];
      x[4 * q + 1] = v[1];
      x[4 * q + 2] = v[2];
      x[4 * q + 3] = v[3];
    }
    // ---- GRU cell (torch.nn.GRU, gates r, z, n) ----
    float gi[9], gh[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < NIN; ++k) acc = fmaf(T[F::F_WIH + i * NIN + k], x[k], acc);
      gi[i] = acc;
      gh[i] = fmaf(T[F::F_WHH + 3 * i], hs[0], fmaf(T[F::F_WHH + 3 * i + 1], hs[1], T[F::F_WHH + 3 * i + 2] * hs[2]));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float r = sigm(gi[k] + gh[k] + T[F::F_BRZ + k]);
      const float z = sigm(gi[3 + k] + gh[3 + k] + T[F::F_BRZ + 3 + k]);
      const float n = tanhf(gi[6 + k] + T[F::F_BIN + k] + r * (gh[6 + k] + T[F::F_BHN + k]));
      hs[k] = (1.f - z) * n + z * hs[k];
    }
    // ---- GAT, mean over nodes (log2e-scaled scores) ----
    float s[H], t[H];
    float smax = -INFINITY, tmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      s[i] = fmaf(T[F::F_UV], x[3 * i], fmaf(T[F::F_UV + 1], x[3 * i + 1], T[F::F_UV + 2] * x[3 * i + 2]));
      t[i] = fmaf(T[F::F_UV + 4], x[3 * i], fmaf(T[F::F_UV + 5], x[3 * i + 1], T[F::F_UV + 6] * x[3 * i + 2]));
      smax = fmaxf(smax, s[i]);
      tmax = fmaxf(tmax, t[i]);
    }
    const float mraw = smax + tmax;
    const float m = fmaxf(mraw, 0.01f * mraw);  // max over edges of lrelu(s_i + t_j)
    const float k1 = __builtin_amdgcn_exp2f(mraw - m);
    const float k2 = __builtin_amdgcn_exp2f(0.01f * mraw - m);
    float A[H], C[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
      A[j] = __builtin_amdgcn_exp2f(t[j] - tmax);
      C[j] = __builtin_amdgcn_exp2f(0.01f * (t[j] - tmax));
    }
    float Z = 0.f, g0 = 0.f, g1 = 0.f, g2 = 0.f;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      float sa = 0.f, scn = 0.f;
      const float ns = -s[i];
#pragma unroll
      for (int j = 0; j < H; ++j) {
        const bool pos = t[j] > ns;
        sa += pos ? A[j] : 0.f;
        scn += pos ? 0.f : C[j];
      }
      const float r = __builtin_amdgcn_exp2f(s[i] - smax) * k1 * sa +
                      __builtin_amdgcn_exp2f(0.01f * (s[i] - smax)) * k2 * scn;
      Z += r;
      g0 = fmaf(r, x[3 * i], g0);
      g1 = fmaf(r, x[3 * i + 1], g1);
      g2 = fmaf(r, x[3 * i + 2], g2);
    }
    const float iz = 1.0f / Z;
    g0 *= iz;
    g1 *= iz;
    g2 *= iz;
    c[w][0] = hs[0];
    c[w][1] = hs[1];
    c[w][2] = hs[2];
#pragma unroll
    for (int dd = 0; dd < H; ++dd)
      c[w][3 + dd] = fmaf(T[F::F_FC + 3 * dd], g0, fmaf(T[F::F_FC + 3 * dd + 1], g1, T[F::F_FC + 3 * dd + 2] * g2));
  }

  // ---- single-head attention over the 3 steps ----
  float sc[3][3];
  {
    float mt[3][E], bt[3];
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) {
      float bb = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float acc = 0.f;
#pragma unroll
        for (int f = 0; f < E; ++f) acc = fmaf(T[F::F_M + e * E + f], c[tt][f], acc);
        mt[tt][e] = acc;
        bb = fmaf(T[F::F_BETA + e], c[tt][e], bb);
      }
      bt[tt] = bb;
    }
#pragma unroll
    for (int ss = 0; ss < 3; ++ss)
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) {
        float acc = bt[tt];
#pragma unroll
        for (int e = 0; e < E; ++e) acc = fmaf(c[ss][e], mt[tt][e], acc);
        sc[ss][tt] = acc;
      }
  }
  float ch[3][E];
#pragma unroll
  for (int ss = 0; ss < 3; ++ss) {
    const float mx = fmaxf(sc[ss][0], fmaxf(sc[ss][1], sc[ss][2]));
    float p[3], ps = 0.f;
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) {
      p[tt] = __builtin_amdgcn_exp2f(sc[ss][tt] - mx);
      ps += p[tt];
    }
    const float ip = 1.0f / ps;
#pragma unroll
    for (int e = 0; e < E; ++e) ch[ss][e] = (p[0] * c[0][e] + p[1] * c[1][e] + p[2] * c[2][e]) * ip;
  }

  // ---- folded encoder + decoders, softmax / sigmoid, detect, diagnose ----
  const float* P = T + F::F_PROTO;
  int anyf = 0;
  float* emb = a.emb + b * Geo<H>::EP;
#pragma unroll
  for (int h = 0; h < H; ++h) {
    float o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = 4 * h + q;
      float acc = T[F::F_B2 + n];
#pragma unroll
      for (int ss = 0; ss < 3; ++ss)
#pragma unroll
        for (int e = 0; e < E; ++e) acc = fmaf(T[F::F_W2 + n * F::KC + ss * E + e], ch[ss][e], acc);
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
