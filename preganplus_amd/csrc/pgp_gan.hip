// pgp_gan.hip — K3: generator + discriminator + decision argmaxes
// (models.py:118-151, 258-291; PreGANPlus.py:84-105; stats/Stats.py:162-166).
//
// One wave = 16 windows on lanes.  Gen1 [64 x (2H+H^2)] and the schedule half
// of Disc1 [64 x H^2] share one pass over the schedule (shared B operand);
// Gen2 is produced one container row at a time, tanh'd, added to the schedule,
// arg-maxed, and immediately consumed as B operand by the new-schedule half of
// Disc1 — the new schedule never leaves registers.
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kGanWaves = 4;

template <int H>
__global__ __launch_bounds__(kGanWaves * 64) void gan_kernel(FwdArgs a) {
  const int B = a.B;
  const float* __restrict__ emb = a.emb;
  const float* __restrict__ sched = a.sched;
  const float* __restrict__ frags = a.frags;
  const float* __restrict__ gt = a.gtab;
  float* __restrict__ probs = a.probs;
  int* __restrict__ keep = a.keep;
  int* __restrict__ final_t = a.final_t;
  int* __restrict__ gen_t = a.gen_t;
  using G = Geo<H>;
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const long blk = (long)blockIdx.x * kGanWaves + (threadIdx.x >> 6);
  const long nblk = (B + 15) / 16;
  if (blk >= nblk) return;
  const long b = blk * 16 + j;
  const bool valid = b < B;
  const float* sw = sched + (valid ? b : 0) * G::H2;
  const float* ew = emb + (valid ? b : 0) * G::EP;

  f32x4 hg[G::MT_G], hd[G::MT_G];
#pragma unroll
  for (int mt = 0; mt < G::MT_G; ++mt) {
    hg[mt] = ld4(gt + G::G_B1 + 16 * mt + 4 * g);
    hd[mt] = ld4(gt + G::G_BD1 + 16 * mt + 4 * g);
  }
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  // ---- Gen1, embedding half ----
  const f32x4* A1e = reinterpret_cast<const f32x4*>(frags + G::OFF_G1E);
#pragma unroll
  for (int q = 0; q < G::EQ; ++q) {
    const f32x4 bv = valid ? ld4(ew + 16 * q + 4 * g) : zero4;
#pragma unroll
    for (int mt = 0; mt < G::MT_G; ++mt) {
      const f32x4 a = A1e[(mt * G::EQ + q) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) hg[mt] = mfma(a[e], bv[e], hg[mt]);
    }
  }
  // ---- Gen1 schedule half + Disc1 schedule half (shared B operand) ----
  const f32x4* A1s = reinterpret_cast<const f32x4*>(frags + G::OFF_G1S);
  const f32x4* Ad1s = reinterpret_cast<const f32x4*>(frags + G::OFF_D1S);
#pragma unroll 2
  for (int q = 0; q < G::SQ; ++q) {
    const int idx = 16 * q + 4 * g;
    const f32x4 bv = (valid && idx < G::H2) ? ld4(sw + idx) : zero4;
#pragma unroll
    for (int mt = 0; mt < G::MT_G; ++mt) {
      const f32x4 a = A1s[(mt * G::SQ + q) * 64 + lane];
      const f32x4 ad = Ad1s[(mt * G::SQ + q) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hg[mt] = mfma(a[e], bv[e], hg[mt]);
        hd[mt] = mfma(ad[e], bv[e], hd[mt]);
      }
    }
  }
  // (LeakyReLU(True) is the identity: hg is the hidden layer as is)
  // ---- per container row: Gen2 -> tanh -> ns -> argmaxes -> Disc1 ns half ----
  const f32x4* A2 = reinterpret_cast<const f32x4*>(frags + G::OFF_G2);
  const f32x4* Ad1n = reinterpret_cast<const f32x4*>(frags + G::OFF_D1N);
  for (int c = 0; c < G::C; ++c) {
    f32x4 ns[G::MT_N];
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t) {
      ns[t] = ld4(gt + G::G_B2 + c * G::MT_N * 16 + 16 * t + 4 * g);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const f32x4 a = A2[(((long)c * G::MT_N + t) * 4 + q4) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) ns[t] = mfma(a[e], hg[q4][e], ns[t]);
      }
    }
    float bn = -INFINITY, bs = -INFINITY;
    int bni = 0, bsi = 0;
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hh = 16 * t + 4 * g + r;
        if (hh < H) {
          const float sv = valid ? sw[c * H + hh] : 0.f;
          const float nv = sv + 4.0f * tanhf(ns[t][r]);
          ns[t][r] = nv;
          if (nv > bn) {
            bn = nv;
            bni = hh;
          }
          if (sv > bs) {
            bs = sv;
            bsi = hh;
          }
        } else {
          ns[t][r] = 0.f;
        }
      }
#pragma unroll
    for (int mt = 0; mt < G::MT_G; ++mt)
#pragma unroll
      for (int q4 = 0; q4 < G::MT_N; ++q4) {
        const f32x4 a = Ad1n[(((long)c * G::MT_G + mt) * G::MT_N + q4) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) hd[mt] = mfma(a[e], ns[q4][e], hd[mt]);
      }
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float ov = __shfl_xor(bn, off), os = __shfl_xor(bs, off);
      const int oi = __shfl_xor(bni, off), osi = __shfl_xor(bsi, off);
      if (ov > bn || (ov == bn && oi < bni)) {
        bn = ov;
        bni = oi;
      }
      if (os > bs || (os == bs && osi < bsi)) {
        bs = os;
        bsi = osi;
      }
    }
    if (valid && g == 0) {
      gen_t[b * G::C + c] = bni;
      final_t[b * G::C + c] = bsi;
    }
  }
  // ---- Disc2 + softmax + gate ----
  float z0 = 0.f, z1 = 0.f;
#pragma unroll
  for (int mt = 0; mt < G::MT_G; ++mt) {
    const f32x4 w0 = ld4(gt + G::G_WD2 + 16 * mt + 4 * g), w1 = ld4(gt + G::G_WD2 + 64 + 16 * mt + 4 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      z0 += hd[mt][r] * w0[r];
      z1 += hd[mt][r] * w1[r];
    }
  }
  z0 = xsum(z0, true) + gt[G::G_BD2];
  z1 = xsum(z1, true) + gt[G::G_BD2 + 1];
  const float m = fmaxf(z0, z1);
  const float e0 = expf(z0 - m), e1 = expf(z1 - m);
  const float inv = 1.0f / (e0 + e1);
  const float p0 = e0 * inv, p1 = e1 * inv;
  if (valid && g == 0) {
    probs[2 * b] = p0;
    probs[2 * b + 1] = p1;
    keep[b] = p0 > p1 ? 1 : 0;
  }
}


template <int H>
hipError_t launch(const FwdArgs& a, hipStream_t st) {
  const long nblk = (a.B + 15) / 16;
  const int grid = (int)((nblk + kGanWaves - 1) / kGanWaves);
  gan_kernel<H><<<grid, kGanWaves * 64, 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_gan(const FwdArgs& a, hipStream_t st) {
  switch (a.H) {
#define CASE(h) \
  case h:       \
    return launch<h>(a, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
