// pgp_packcore.hpp — the PreGAN+ weight packing (natural blob -> the kernels'
// fragment / table layouts of pgp_layout.hpp), written once for both sides:
//   * host: pgp_pack.cpp (pgp_load_weights, fp64 reference blob);
//   * device: pgp_repack.hip (pgp_repack_master: straight from the training
//     master weights P and the device prototype state after an optimizer step,
//     no host round trip — the reference's AdamW updates the modules in place,
//     utils.py:64-65).
// Every loop nest is a flat parallel-for over its output elements (`ex.par`):
// a serial loop on the host, a grid-stride loop on the device.  The source is
// an accessor src(i) = blob element i as fp64; FP contraction is off, so host
// and device produce the same bits.  Three phases (device: three launches):
//   0: A = Wte Wfc (d x 3) and the GAT constants;
//   1: the fold of every layer-0 in_proj row onto the raw features (needs A);
//   2: everything else (reads A and the fold table).
// Folds (all fp64, results rounded once to fp32) — see pgp_pack.cpp's header.
#pragma once
#include <cmath>

#include "pgp_layout.hpp"

#pragma STDC FP_CONTRACT OFF

#if defined(__HIP__)
#define PGP_HD __host__ __device__
#else
#define PGP_HD
#endif

namespace pgp {
namespace packcore {

// feature of d-space row R (see pgp_layout.hpp): R = 16t+4g+r <-> c = 16t+4r+g
PGP_HD inline int featX(int R) { return 16 * (R / 16) + 4 * (R % 4) + (R % 16) / 4; }

template <class Src>
struct View {
  Src s;
  long o;
  PGP_HD double operator[](long i) const { return s(o + i); }
};

// element offsets of the natural blob (transformer | gen | disc | prototypes),
// the order of pgp_load_weights and of the training master (pgp_train.hpp)
template <int H>
struct BlobOff {
  struct Ly {
    long inW, inB, outW, outB, l1W, l1B, l2W, l2B, n1w, n1b, n2w, n2b;
  };
  long fcW, attn, teW, teB, pe;
  Ly ly[kLayers];
  long anW, anB, prW, prB, g0W, g0B, g2W, g2B, d0W, d0B, d2W, d2B, protos, end;
  PGP_HD explicit BlobOff(int K) {
    const long d = H, L = 3L * H * H, GIN = 2 * d + d * d;
    long o = 0;
    auto take = [&](long n) {
      const long r = o;
      o += n;
      return r;
    };
    fcW = take(d * 3);
    attn = take(2 * d);
    teW = take(d * d);
    teB = take(d);
    pe = take(3 * d);
    for (int l = 0; l < kLayers; ++l) {
      ly[l].inW = take(3 * d * d);
      ly[l].inB = take(3 * d);
      ly[l].outW = take(d * d);
      ly[l].outB = take(d);
      ly[l].l1W = take(64 * d);
      ly[l].l1B = take(64);
      ly[l].l2W = take(d * 64);
      ly[l].l2B = take(d);
      ly[l].n1w = take(d);
      ly[l].n1b = take(d);
      ly[l].n2w = take(d);
      ly[l].n2b = take(d);
    }
    anW = take(2 * d * L);
    anB = take(2 * d);
    prW = take(2 * d * L);
    prB = take(2 * d);
    g0W = take(64 * GIN);
    g0B = take(64);
    g2W = take(d * d * 64);
    g2B = take(d * d);
    d0W = take(64 * 2 * d * d);
    d0B = take(64);
    d2W = take(2 * 64);
    d2B = take(2);
    protos = take(2L * K);
    end = o;
  }
};

// scratch (fp64): A [d][3], then the fold table [3d][6] (wf[3] | bw[3 steps])
template <int H>
struct Scratch {
  static constexpr long A = 0;
  static constexpr long FOLD = 3L * H;
  static constexpr long DECC = FOLD + 3L * H * 6;  // [dec row][feature][step]: sum over hosts of W
  static constexpr long SIZE = DECC + (long)Geo<H>::MT_O * 16 * H * 3;
};

// Gen / Disc (models.py:118-151) into the K3 chunk layout (pgp_gan.hip).
template <int H, class V, class Ex>
PGP_HD void pack_gan(const V& g0W, const V& g0B, const V& g2W, const V& g2B, const V& d0W, const V& d0B,
                     const V& d2W, const V& d2B, const Ex& ex, float* F, float* GT) {
  using G = Geo<H>;
  constexpr int d = H, GIN = 2 * d + d * d;
  ex.par((long)G::MT_G * 64 * 4, [&](long idx) {
    const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), mt = (int)(idx / 256);
    const int i = lane & 15, g = lane >> 4, row = 16 * mt + i;
    for (int q = 0; q < G::EQ; ++q) {
      const int k = 16 * q + 4 * g + e4;
      if (k < 2 * d) F[G::OFF_GE + (long)(mt * G::EQ + q) * G::FQ + lane * 4 + e4] = (float)g0W[(long)row * GIN + k];
    }
    for (int q = 0; q < G::SQ; ++q) {
      const int k = 16 * q + 4 * g + e4;
      if (k >= d * d) continue;
      F[G::OFF_GS + ((long)q * G::GS_G + mt) * G::FQ + lane * 4 + e4] = (float)g0W[(long)row * GIN + 2 * d + k];
      F[G::OFF_GS + ((long)q * G::GS_G + G::MT_G + mt) * G::FQ + lane * 4 + e4] = (float)d0W[(long)row * 2 * d * d + k];
    }
  });
  ex.par((long)d * G::MT_N * 4 * 256, [&](long idx) {
    const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % 4);
    const int t = (int)(idx / 1024 % G::MT_N), c = (int)(idx / (1024L * G::MT_N));
    const int i = lane & 15, g = lane >> 4, u = 16 * q4 + 4 * g + e4, hh = 16 * t + i;
    if (hh >= d) return;
    float* FC = F + G::OFF_GC + (long)c * G::GC_G * G::FQ;
    FC[(t * 4 + q4) * G::FQ + lane * 4 + e4] = (float)g2W[(long)(c * d + hh) * 64 + u];
  });
  ex.par((long)d * G::MT_G * G::MT_N * 256, [&](long idx) {
    const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % G::MT_N);
    const int mt = (int)(idx / (256L * G::MT_N) % G::MT_G), c = (int)(idx / (256L * G::MT_N * G::MT_G));
    const int i = lane & 15, g = lane >> 4, hh = 16 * q4 + 4 * g + e4;
    if (hh >= d) return;
    float* FC = F + G::OFF_GC + (long)c * G::GC_G * G::FQ;
    FC[(G::GC_G2 + mt * G::MT_N + q4) * G::FQ + lane * 4 + e4] =
        (float)d0W[(long)(16 * mt + i) * 2 * d * d + d * d + c * d + hh];
  });
  ex.par((long)d * d, [&](long idx) {
    const int c = (int)(idx / d), R = (int)(idx % d);
    GT[G::G_B2 + c * G::MT_N * 16 + R] = (float)g2B[c * d + R];
  });
  ex.par(64, [&](long u) {
    GT[G::G_B1 + u] = (float)g0B[u];
    GT[G::G_BD1 + u] = (float)d0B[u];
    GT[G::G_WD2 + u] = (float)d2W[u];
    GT[G::G_WD2 + 64 + u] = (float)d2W[64 + u];
    if (u < 2) GT[G::G_BD2 + u] = (float)d2B[u];
  });
}

// Tail mode (Geo<H>::TAIL): q/k/v tile t, C-row i -> (head, dim).  Slot
// sigma = 4*(i%4) + i/4 (the B-operand order of the row); tiles [0,HF) head 0,
// [HF,2HF) head 1, tile 2HF: sigma < HT head 0's tail, else head 1's tail.
// Head 1's last SR tail dims are VALU rows n: dim 16*HF + 16 - HT + n.
template <int H>
PGP_HD bool tail_slot(int t, int i, int* hh, int* e) {
  using G = Geo<H>;
  const int sg = 4 * (i % 4) + i / 4;
  if (t < G::HF) {
    *hh = 0;
    *e = 16 * t + sg;
  } else if (t < 2 * G::HF) {
    *hh = 1;
    *e = 16 * (t - G::HF) + sg;
  } else if (sg < G::HT) {
    *hh = 0;
    *e = 16 * G::HF + sg;
  } else {
    *hh = 1;
    *e = 16 * G::HF + sg - G::HT;
  }
  return *e < G::HD;
}

// out_proj k-step s, lane group g -> the (head, dim) of the O slot it reads
template <int H>
PGP_HD bool tail_oslot(int s, int g, int* hh, int* e) {
  using G = Geo<H>;
  if (s < 4 * G::TQ) return tail_slot<H>(s / 4, 4 * g + s % 4, hh, e);
  if (s == 4 * G::TQ && g < G::SR) {
    *hh = 1;
    *e = 16 * G::HF + 16 - G::HT + g;
    return true;
  }
  return false;
}

// head-space row R within a pass block -> (head, dim), valid? (non-tail modes)
template <int H>
PGP_HD bool head_row(int p, int R, int* hh, int* e) {
  using G = Geo<H>;
  if (G::P8) {
    const int g = (R % 16) / 4, r = R % 4;
    *hh = g >> 1;
    *e = 4 * (g & 1) + r;
  } else {
    *hh = p;
    *e = featX(R);
  }
  return *e < G::HD;
}

// layer-0 q/k/v output tile T0, C-row i -> source row of in_proj, or -1
template <int H>
PGP_HD int tile_src(int T0, int i) {
  using G = Geo<H>;
  int hh, e, m;
  if constexpr (G::TAIL) {
    m = T0 / G::TQ;
    if (!tail_slot<H>(T0 % G::TQ, i, &hh, &e)) return -1;
  } else {
    const int p = T0 / (3 * G::TP), r = T0 % (3 * G::TP), tp = r % G::TP;
    m = r / G::TP;
    if (!head_row<H>(p, 16 * tp + i, &hh, &e)) return -1;
  }
  return m * H + hh * G::HD + e;
}

template <int H, class V, class Ex>
PGP_HD void pack_tail_attention(const V& inW, const V& inB, const V& outW, double scale, const Ex& ex, float* FL,
                                float* TL, bool fold, const V& gam, const V& bet) {
  using G = Geo<H>;
  constexpr int d = H;
  // fold: the layer's input is the previous norm2's x-hat, so in_proj's columns
  // take that norm's gamma and its rows add in_proj . beta (fp64, one rounding)
  auto wcol = [&](long src, int c) { return inW[src * d + c] * (fold ? gam[c] : 1.0); };
  auto brow = [&](long src) {
    double b = inB[src];
    if (fold)
      for (int c = 0; c < d; ++c) b += inW[src * d + c] * bet[c];
    return b;
  };
  // q, k tiles (stage 0) and v tiles (stage 1): [m][t][q4] groups over X k-steps
  ex.par(3L * G::TQ * G::KQ_D * 256, [&](long idx) {
    const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % G::KQ_D);
    const int t = (int)(idx / (256L * G::KQ_D) % G::TQ), m = (int)(idx / (256L * G::KQ_D * G::TQ));
    const long base = m < 2 ? (long)(m * G::TQ + t) * G::KQ_D : G::P_V + (long)t * G::KQ_D;
    const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4, c = 4 * s + g;
    int hh, e;
    if (s >= G::KS_D || c >= d || !tail_slot<H>(t, i, &hh, &e)) return;
    const int src = m * d + hh * G::HD + e;
    FL[(base + q4) * G::FQ + lane * 4 + e4] = (float)(wcol(src, c) * (m == 0 ? scale : 1.0));
  });
  ex.par(3L * G::TQ * 16, [&](long idx) {
    const int i = (int)(idx % 16), t = (int)(idx / 16 % G::TQ), m = (int)(idx / (16 * G::TQ));
    int hh, e;
    if (!tail_slot<H>(t, i, &hh, &e)) return;
    TL[G::TL_QKV + (m * G::TQ + t) * 16 + i] = (float)(brow(m * d + hh * G::HD + e) * (m == 0 ? scale : 1.0));
  });
  // VALU rows of head 1's tail
  ex.par(3L * G::SR * G::KQ_D * 16, [&](long idx) {
    const int e4 = (int)(idx % 4), g = (int)(idx / 4 % 4), q4 = (int)(idx / 16 % G::KQ_D);
    const int n = (int)(idx / (16L * G::KQ_D) % G::SR), m = (int)(idx / (16L * G::KQ_D * G::SR));
    const int src = m * d + G::HD + 16 * G::HF + 16 - G::HT + n;
    const int s = 4 * q4 + e4, c = 4 * s + g;
    if (s >= G::KS_D || c >= d) return;
    TL[G::TL_RQ + (((m * G::SR + n) * G::KQ_D + q4) * 4 + g) * 4 + e4] =
        (float)(wcol(src, c) * (m == 0 ? scale : 1.0));
  });
  ex.par(3L * G::SR, [&](long idx) {
    const int n = (int)(idx % G::SR), m = (int)(idx / G::SR);
    const int src = m * d + G::HD + 16 * G::HF + 16 - G::HT + n;
    TL[G::TL_RQB + m * G::SR + n] = (float)(brow(src) * (m == 0 ? scale : 1.0));
  });
  // out_proj: MT_X output tiles over the O slots (+ VALU rows 16*MT_X + n)
  ex.par((long)G::MT_X * G::KQ_OT * 256, [&](long idx) {
    const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % G::KQ_OT);
    const int mt = (int)(idx / (256L * G::KQ_OT));
    const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4;
    const int co = featX(16 * mt + i);
    int hh, e;
    if (co >= d || !tail_oslot<H>(s, g, &hh, &e)) return;
    FL[(G::P_OT + mt * G::KQ_OT + q4) * G::FQ + lane * 4 + e4] = (float)outW[(long)co * d + hh * G::HD + e];
  });
  ex.par((long)G::XR * G::KQ_OT * 16, [&](long idx) {
    const int e4 = (int)(idx % 4), g = (int)(idx / 4 % 4), q4 = (int)(idx / 16 % G::KQ_OT);
    const int n = (int)(idx / (16L * G::KQ_OT));
    int hh, e;
    if (!tail_oslot<H>(4 * q4 + e4, g, &hh, &e)) return;
    TL[G::TL_RO + ((n * G::KQ_OT + q4) * 4 + g) * 4 + e4] = (float)outW[(long)(16 * G::MT_X + n) * d + hh * G::HD + e];
  });
}

// phase 0: A = Wte Wfc and the GAT constants gatc = [u, 0, v, 0] (log2(e)-scaled:
// leaky_relu is positively homogeneous, so the kernel evaluates exp(e - M) as
// exp2(e' - M') with one v_exp_f32)
template <int H, class Src, class Ex>
PGP_HD void pack_phase0(int K, const Src& src, const Ex& ex, double* scr, float* gatc) {
  constexpr int d = H;
  const BlobOff<H> B(K);
  const View<Src> fcW{src, B.fcW}, attn{src, B.attn}, teW{src, B.teW};
  double* A = scr + Scratch<H>::A;
  ex.par(3L * d, [&](long idx) {
    const int c = (int)(idx / 3), f = (int)(idx % 3);
    double acc = 0;
    for (int k = 0; k < d; ++k) acc += teW[(long)c * d + k] * fcW[k * 3 + f];
    A[c * 3 + f] = acc;
  });
  ex.par(4, [&](long f) {
    if (f == 3) {
      gatc[3] = gatc[7] = 0.f;
      return;
    }
    double u = 0, v = 0;
    for (int c = 0; c < d; ++c) {
      u += fcW[c * 3 + f] * attn[c];
      v += fcW[c * 3 + f] * attn[d + c];
    }
    gatc[f] = (float)(u * 1.4426950408889634);
    gatc[4 + f] = (float)(v * 1.4426950408889634);
  });
}

// phase 1: layer 0's q/k/v folded onto the aggregated raw features.
// X0[c] = sum_f A[c][f] agg[f] + teB[c] + pe[w][c], so for in_proj row src
//   wf[f] = sc (Win A)[src][f],  bw[w] = sc (inB + Win (teB + pe[w]))[src]
// (sc = the attention scale for q rows, 1 otherwise)
template <int H, class Src, class Ex>
PGP_HD void pack_phase1(int K, const Src& src, const Ex& ex, double scale, double* scr) {
  constexpr int d = H;
  const BlobOff<H> B(K);
  const View<Src> teB{src, B.teB}, pe{src, B.pe}, inW{src, B.ly[0].inW}, inB{src, B.ly[0].inB};
  const double* A = scr + Scratch<H>::A;
  double* FT = scr + Scratch<H>::FOLD;
  ex.par(3L * d * 6, [&](long idx) {  // one (row, column) of the fold table per item
    const long s = idx / 6;
    const int k = (int)(idx % 6);
    const double sc = s < d ? scale : 1.0;
    if (k < 3) {
      double acc = 0;
      for (int c = 0; c < d; ++c) acc += inW[s * d + c] * A[c * 3 + k];
      FT[s * 6 + k] = acc * sc;
    } else {
      const int w = k - 3;
      double acc = inB[s];
      for (int c = 0; c < d; ++c) acc += inW[s * d + c] * (teB[c] + pe[w * d + c]);
      FT[s * 6 + 3 + w] = acc * sc;
    }
  });
  // decoder rows n = 4*host + {l0, l1, p0, p1}: per (feature c, step w) the sum
  // over the H host columns (the last norm2's beta fold, phase 2)
  using G = Geo<H>;
  constexpr long L = 3L * H * H;
  const View<Src> anW{src, B.anW}, prW{src, B.prW};
  double* DC = scr + Scratch<H>::DECC;
  ex.par((long)G::MT_O * 16 * d * 3, [&](long idx) {  // [row][feature][step]: a sum over hosts
    const int w = (int)(idx % 3), c = (int)(idx / 3 % d), n = (int)(idx / (3L * d)), host = n / 4, q = n % 4;
    double acc = 0;
    if (host < d)
#pragma unroll 8
      for (int h = 0; h < d; ++h) {
        const long col = (long)h * 3 * d + w * d + c;
        acc += q < 2 ? anW[(long)(2 * host + q) * L + col] : prW[(long)(2 * host + q - 2) * L + col];
      }
    DC[idx] = acc;
  });
}

// phase 2: everything else.  sections: bit 0 the PreGAN+ encoder / decoder
// layouts (which read phases 0 / 1's scratch), bit 1 the GAN's (pack_gan, from
// its own weights only); independent outputs, so either order
template <int H, class Src, class Ex>
PGP_HD void pack_phase2(int K, const Src& src, const Ex& ex, double scale, const double* scr, float* F, float* T,
                        float* GT, int sections = 3) {
  using G = Geo<H>;
  using Ly = typename BlobOff<H>::Ly;
  constexpr int d = H;
  constexpr long L = 3L * H * H;
  const BlobOff<H> B(K);
  auto V = [&](long o) { return View<Src>{src, o}; };
  if (sections & 2)
    pack_gan<H>(V(B.g0W), V(B.g0B), V(B.g2W), V(B.g2B), V(B.d0W), V(B.d0B), V(B.d2W), V(B.d2B), ex, F, GT);
  if (!(sections & 1)) return;
  const View<Src> teB = V(B.teB), pe = V(B.pe);
  const double* A = scr + Scratch<H>::A;
  const double* FT = scr + Scratch<H>::FOLD;

  // ---- time encoder (folded with GAT fc): A's columns 0..2 as K=4 A fragments ----
  ex.par((long)G::MT_D * 64, [&](long idx) {
    const int mt = (int)(idx / 64), lane = (int)(idx % 64);
    const int i = lane & 15, g = lane >> 4;
    const int c = featX(16 * mt + i);
    if (c >= d || g >= 3) return;
    T[G::T_TEW + mt * 64 + lane] = (float)A[c * 3 + g];
  });
  ex.par(3L * G::DP, [&](long idx) {
    const int w = (int)(idx / G::DP), R = (int)(idx % G::DP);
    const int c = featX(R);
    if (c < d) T[G::T_TE + w * G::DP + R] = (float)(teB[c] + pe[w * d + c]);
  });

  // ---- encoder layers ----
  for (int l = 0; l < kLayers; ++l) {
    const Ly& O = B.ly[l];
    const View<Src> inW = V(O.inW), inB = V(O.inB), outW = V(O.outW), outB = V(O.outB), l1W = V(O.l1W),
                    l1B = V(O.l1B), l2W = V(O.l2W), l2B = V(O.l2B), n1w = V(O.n1w), n1b = V(O.n1b),
                    n2w = V(O.n2w), n2b = V(O.n2b);
    float* FL = F + G::OFF_ENC + (long)l * G::LAYER_G * G::FQ;
    float* TL = T + G::T_L0 + l * G::TL_SIZE;
    // layer 0's norm2 gamma / beta folded into layer 1's in_proj and residual
    // (the kernel passes layer 1 x-hat; residual = gamma * x-hat + (bo + beta))
    const bool fold0 = l > 0;
    const View<Src> pn2w = V(B.ly[l > 0 ? l - 1 : 0].n2w), pn2b = V(B.ly[l > 0 ? l - 1 : 0].n2b);
    if constexpr (G::TAIL) {
      pack_tail_attention<H>(inW, inB, outW, scale, ex, FL, TL, fold0, pn2w, pn2b);
    } else {
      ex.par((long)G::NPASS * 3 * G::TP * G::KQ_D * 256, [&](long idx) {
        const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % G::KQ_D);
        long r = idx / (256L * G::KQ_D);
        const int tp = (int)(r % G::TP);
        r /= G::TP;
        const int m = (int)(r % 3), p = (int)(r / 3);
        const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4;
        const int c = 4 * s + g;
        int hh, e;
        if (s >= G::KS_D || c >= d || !head_row<H>(p, 16 * tp + i, &hh, &e)) return;
        const int sr = m * d + hh * G::HD + e;
        const double v = inW[(long)sr * d + c] * (fold0 ? pn2w[c] : 1.0) * (m == 0 ? scale : 1.0);
        FL[(G::P_QKV(p) + (m * G::TP + tp) * G::KQ_D + q4) * G::FQ + lane * 4 + e4] = (float)v;
      });
      ex.par((long)G::NPASS * 3 * G::TP * 16, [&](long idx) {
        const int i = (int)(idx % 16), tp = (int)(idx / 16 % G::TP), m = (int)(idx / (16L * G::TP) % 3);
        const int p = (int)(idx / (48L * G::TP));
        int hh, e;
        if (!head_row<H>(p, 16 * tp + i, &hh, &e)) return;
        const int sr = m * d + hh * G::HD + e;
        double bb = inB[sr];
        if (fold0)
          for (int c = 0; c < d; ++c) bb += inW[(long)sr * d + c] * pn2b[c];
        TL[G::TL_QKV + (p * 3 + m) * G::TP * 16 + 16 * tp + i] = (float)(bb * (m == 0 ? scale : 1.0));
      });
      // out_proj
      ex.par((long)G::NPASS * G::MT_D * G::KQ_O * 256, [&](long idx) {
        const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % G::KQ_O);
        const int mt = (int)(idx / (256L * G::KQ_O) % G::MT_D), p = (int)(idx / (256L * G::KQ_O * G::MT_D));
        const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4;
        const int co = featX(16 * mt + i);
        if (s >= G::KS_O || co >= d) return;
        int hh, e;
        if (G::P8) {
          hh = g >> 1;
          e = 4 * (g & 1) + s;
        } else {
          hh = p;
          e = 4 * s + g;
        }
        if (e >= G::HD) return;
        FL[(G::P_O(p) + mt * G::KQ_O + q4) * G::FQ + lane * 4 + e4] = (float)outW[(long)co * d + hh * G::HD + e];
      });
    }
    // FFN; norm1's gamma folded into linear1 (the kernel feeds it the un-scaled x-hat)
    ex.par((long)G::MT_F * G::KQ_D * 256, [&](long idx) {
      const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % G::KQ_D);
      const int mt = (int)(idx / (256L * G::KQ_D));
      const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4, c = 4 * s + g;
      if (s >= G::KS_D || c >= d) return;
      FL[(G::P_F1 + mt * G::KQ_D + q4) * G::FQ + lane * 4 + e4] = (float)(l1W[(long)(16 * mt + i) * d + c] * n1w[c]);
    });
    ex.par((long)G::MT_X * G::KQ_F * 256, [&](long idx) {
      const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % G::KQ_F);
      const int mt = (int)(idx / (256L * G::KQ_F));
      const int i = lane & 15, g = lane >> 4, u = 16 * q4 + 4 * g + e4;
      const int co = featX(16 * mt + i);
      if (co >= d) return;
      FL[(G::P_F2 + mt * G::KQ_F + q4) * G::FQ + lane * 4 + e4] = (float)l2W[(long)co * 64 + u];
    });
    ex.par((long)G::DP, [&](long R) {
      const int c = featX((int)R);
      if (c >= d) return;
      TL[G::TL_BO + R] = (float)(outB[c] + (fold0 ? pn2b[c] : 0.0));
      TL[G::TL_LN1G + R] = (float)n1w[c];
      TL[G::TL_LN1B + R] = (float)n1b[c];
      TL[G::TL_B2 + R] = (float)(l2B[c] + n1b[c]);  // + norm1's beta: the residual is gamma*x-hat + beta
      TL[G::TL_LN2G + R] = (float)n2w[c];
      TL[G::TL_LN2B + R] = (float)n2b[c];
    });
    ex.par(64, [&](long u) {  // linear1 bias + linear1 . norm1's beta
      double b = l1B[u];
      for (int c = 0; c < d; ++c) b += l1W[u * d + c] * n1b[c];
      TL[G::TL_B1 + u] = (float)b;
    });
    // tail mode: linear2 rows of the VALU d-rows (feature 16*MT_X + n)
    ex.par((long)G::XR * G::KQ_F * 16, [&](long idx) {
      const int e = (int)(idx % 4), g = (int)(idx / 4 % 4), q4 = (int)(idx / 16 % G::KQ_F);
      const int n = (int)(idx / (16L * G::KQ_F));
      TL[G::TL_RF + ((n * G::KQ_F + q4) * 4 + g) * 4 + e] =
          (float)l2W[(long)(16 * G::MT_X + n) * 64 + 16 * q4 + 4 * g + e];
    });
  }

  // ---- layer 0's q/k/v folded onto the aggregated raw features (fold table) ----
  ex.par(3L * G::NQT * 16, [&](long idx) {
    const int T0 = (int)(idx / 16), i = (int)(idx % 16);
    const int s = tile_src<H>(T0, i);
    if (s < 0) return;
    for (int g = 0; g < 3; ++g) T[G::T_F0 + T0 * 64 + 16 * g + i] = (float)FT[s * 6 + g];
    for (int w = 0; w < 3; ++w) T[G::T_F0B + (w * 3 * G::NQT + T0) * 16 + i] = (float)FT[s * 6 + 3 + w];
  });
  if constexpr (G::TAIL) {
    const View<Src> outW = V(B.ly[0].outW);
    // out_proj through the attention, per head hh and output c:
    //   Gh[c][f] = sum_e Wo[c][hh*HD+e] Fv[e][f], Ch[c][w'] = sum_e Wo[c][hh*HD+e] bv_w'[e]
    auto gc = [&](int hh, int c, int g, double* gm, double* cm) {
      double a = 0, b = 0;
      for (int e = 0; e < G::HD; ++e) {
        const long s = 2 * d + hh * G::HD + e;
        const double wo = outW[(long)c * d + hh * G::HD + e];
        a += wo * FT[s * 6 + g];
        b += wo * FT[s * 6 + 3 + g];
      }
      *gm = a;
      *cm = b;
    };
    ex.par(2L * G::MT_X * 16 * 3, [&](long idx) {
      const int g = (int)(idx % 3), i = (int)(idx / 3 % 16), mt = (int)(idx / 48 % G::MT_X);
      const int hh = (int)(idx / (48L * G::MT_X));
      const int c = featX(16 * mt + i);
      if (c >= d) return;
      double gm, cm;
      gc(hh, c, g, &gm, &cm);
      T[G::T_F0O + ((hh * 2 + 0) * G::MT_X + mt) * 64 + 16 * g + i] = (float)gm;
      T[G::T_F0O + ((hh * 2 + 1) * G::MT_X + mt) * 64 + 16 * g + i] = (float)cm;
    });
    ex.par((long)G::XR * 2 * 3, [&](long idx) {
      const int g = (int)(idx % 3), hh = (int)(idx / 3 % 2), n = (int)(idx / 6);
      double gm, cm;
      gc(hh, 16 * G::MT_X + n, g, &gm, &cm);
      T[G::T_F0OR + n * 16 + (hh * 2 + 0) * 4 + g] = (float)gm;
      T[G::T_F0OR + n * 16 + (hh * 2 + 1) * 4 + g] = (float)cm;
    });
    // layer 0's scores per head as bilinear forms of the raw features:
    // M = sum_e qf kf^T, U = qf kb^T (f, key step), V = qb kf^T (query step, f), S = qb kb^T
    ex.par(2L * 9, [&](long idx) {
      const int hh = (int)(idx / 9), a = (int)(idx % 9) / 3, b = (int)(idx % 3);
      double M = 0, U = 0, Vv = 0, Sc = 0;
      for (int e = 0; e < G::HD; ++e) {
        const double* q = FT + (long)(hh * G::HD + e) * 6;      // q (attention scale folded in)
        const double* k = FT + (long)(d + hh * G::HD + e) * 6;  // k
        M += q[a] * k[b];
        U += q[a] * k[3 + b];
        Vv += q[3 + a] * k[b];
        Sc += q[3 + a] * k[3 + b];
      }
      T[G::T_F0S + hh * 36 + a * 3 + b] = (float)M;
      T[G::T_F0S + hh * 36 + 9 + a * 3 + b] = (float)U;
      T[G::T_F0S + hh * 36 + 18 + a * 3 + b] = (float)Vv;
      T[G::T_F0S + hh * 36 + 27 + a * 3 + b] = (float)Sc;
    });
  }
  if constexpr (G::SR > 0)
    ex.par(3L * G::SR, [&](long idx) {
      const int m = (int)(idx / G::SR), n = (int)(idx % G::SR);
      const int s = m * d + G::HD + 16 * G::HF + 16 - G::HT + n;
      for (int g = 0; g < 3; ++g) T[G::T_F0R + (m * G::SR + n) * 4 + g] = (float)FT[s * 6 + g];
      for (int w = 0; w < 3; ++w) T[G::T_F0RB + w * 3 * G::SR + m * G::SR + n] = (float)FT[s * 6 + 3 + w];
    });

  // ---- decoders: rows n = 4*host + {l0, l1, p0, p1} ----
  // The encoder hands over the last norm2's x-hat: its gamma scales the decoder
  // columns and W . beta joins the decoder bias (fp64, one rounding)
  const View<Src> anW = V(B.anW), prW = V(B.prW), anB = V(B.anB), prB = V(B.prB);
  const View<Src> n2wL = V(B.ly[kLayers - 1].n2w), n2bL = V(B.ly[kLayers - 1].n2b);
  ex.par((long)d * 3 * G::MT_O * G::KQ_D * 256, [&](long idx) {
    const int e4 = (int)(idx % 4), lane = (int)(idx / 4 % 64), q4 = (int)(idx / 256 % G::KQ_D);
    long r = idx / (256L * G::KQ_D);
    const int mt = (int)(r % G::MT_O);
    r /= G::MT_O;
    const int w = (int)(r % 3), h = (int)(r / 3);
    const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4, c = 4 * s + g;
    const int n = 16 * mt + i, host = n / 4, q = n % 4;
    if (s >= G::KS_D || c >= d || host >= d) return;
    const long col = (long)h * 3 * d + w * d + c;
    const double v =
        (q < 2 ? anW[(long)(2 * host + q) * L + col] : prW[(long)(2 * host + q - 2) * L + col]) * n2wL[c];
    F[G::OFF_DEC + ((long)(h * 3 + w) * G::DEC_G + mt * G::KQ_D + q4) * G::FQ + lane * 4 + e4] = (float)v;
  });
  ex.par((long)G::MT_O * 16, [&](long n) {
    const int host = (int)(n / 4), q = (int)(n % 4);
    if (host >= d) return;
    double b = q < 2 ? anB[2 * host + q] : prB[2 * host + q - 2];
    const double* DC = scr + Scratch<H>::DECC + n * d * 3;  // phase 1's column sums
#pragma unroll 4
    for (int c = 0; c < d; ++c) b += ((DC[3 * c] + DC[3 * c + 1]) + DC[3 * c + 2]) * n2bL[c];
    T[G::T_DEC + n] = (float)b;
  });
  const View<Src> protos = V(B.protos);
  ex.par(2L * K, [&](long k) { T[G::T_PROTO + k] = (float)protos[k]; });
}

}  // namespace packcore
}  // namespace pgp
