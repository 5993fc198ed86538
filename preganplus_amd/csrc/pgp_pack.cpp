// pgp_pack.cpp — pack the reference's fp64 tensors into the kernels' layouts.
//
// Source tensors and their reference definitions:
//   GAT fc / attn_fc            dlutils.py:301-302 (no bias)
//   time_encoder, pos_encoder   models.py:344-347, 297-311
//   encoder layers              models.py:350-356 (torch TransformerEncoderLayer)
//   anomaly/prototype decoders  models.py:359-370
//   Gen / Disc                  models.py:118-151, 258-291
//   prototypes                  models.py:373-374, utils.py:70
// Algebraic folds done here in fp64 (results then rounded once to fp32):
//   GAT + time encoder: the GAT aggregates z_i = Wfc x_i linearly, so
//     te(h_j) = Wte (Wfc sum_i a_ij x_i) + b = (Wte Wfc) agg_j + b
//   edge scores: a . [z_i || z_j] = (Wfc^T a_src) . x_i + (Wfc^T a_dst) . x_j
//   attention scale 1/sqrt(head_dim) folded into Wq, bq.
//   layer 0's q/k/v: X0 is affine in the aggregated raw features, so
//     Win X0 + bin = (Win Wte Wfc) agg + (Win (bte + pe[w]) + bin), one K=3
//     product per output row and per-step biases; in tail mode its out_proj
//     too: Wo P V = sum_head (Wo Fv)(P agg) + (Wo bv_w') P (v affine in agg).
#include "pgp_pack.hpp"

#include "pgp_packcore.hpp"

#include <cmath>
#include <cstring>
#include <vector>

namespace pgp {
namespace {

using packcore::View;

struct HostSrc {
  const double* p;
  double operator()(long i) const { return p[i]; }
};
struct HostEx {
  template <class F>
  void par(long n, F&& f) const {
    for (long i = 0; i < n; ++i) f(i);
  }
};

struct Reader {
  const double* p;
  size_t len, off = 0;
  const double* take(size_t n) {
    const double* r = p + off;
    off += n;
    return r;
  }
};

template <int H>
size_t blob_len_t(int K) {
  return (size_t)packcore::BlobOff<H>(K).end;
}

// The PreGAN+ packing (pgp_packcore.hpp) run serially on the host.
template <int H>
std::string pack_t(int K, const double* blob, size_t len, Packed* P) {
  using G = Geo<H>;
  if (len != blob_len_t<H>(K)) return "weight blob length mismatch";
  P->frags.assign(G::SZ_FRAGS, 0.0f);
  P->enc_tab.assign(G::t_size(K), 0.0f);
  P->gan_tab.assign(G::G_SIZE, 0.0f);
  std::vector<double> scr(packcore::Scratch<H>::SIZE, 0.0);
  float gatc[8] = {};
  const HostSrc src{blob};
  const HostEx ex;
  const double scale = 1.0 / std::sqrt((double)G::HD);
  packcore::pack_phase0<H>(K, src, ex, scr.data(), gatc);
  packcore::pack_phase1<H>(K, src, ex, scale, scr.data());
  packcore::pack_phase2<H>(K, src, ex, scale, scr.data(), P->frags.data(), P->enc_tab.data(), P->gan_tab.data());
  for (int f = 0; f < 4; ++f) {
    P->gat.u[f] = gatc[f];
    P->gat.v[f] = gatc[4 + f];
  }
  return "";
}

// ---------------------------------------------------------------------------
// PreGAN FPE_16 variant (models.py:10-115).  Folds, all in fp64:
//   GAT node mean: mean_j sum_i a_ij Wfc x_i = (Wfc / H) sum_i r_i x_i, r_i = sum_j a_ij,
//     so each MHA token is c_w = P u_w, u_w = [h_w; g_w] (GRU state, r-weighted
//     raw features / Z), P = blockdiag(I3, Wfc / H) [E x 6]
//   edge scores as above (u, v), pre-scaled by log2(e)
//   MHA scores: q_s.k_t = c_s^T (Wq^T Wk) c_t + (Wk^T bq).c_t + (terms constant in t,
//     which cancel in the softmax over t) = u_s^T M6 u_t + beta6.u_t with
//     M6 = P^T Wq^T Wk P, beta6 = P^T Wk^T bq; 1/sqrt(E) and log2(e) folded in
//   V, out_proj, encoder Linear (identity LeakyReLU(True)) and both decoders are
//     affine maps applied after a convex combination (sum_t p_st = 1), so
//     [a0 a1 p0 p1]_host = W6 . [sum_t p_st u_t]_s + b2 with
//     W6 = Dec . Wenc . blockdiag_s(Wout Wv P), b2 = Dec (Wenc (Wout bv + bout)_s + benc) + bdec
// ---------------------------------------------------------------------------
template <int H>
std::string pack_fpe_t(const double* blob, size_t len, Packed* P) {
  using FG = FpeGeo<H>;
  using G = Geo<H>;
  const int d = H, E = FG::E, KC = FG::KC, L = 10;
  const size_t gan_len = (size_t)64 * (2 * d + d * d) + 64 + (size_t)d * d * 64 + d * d + 64 * 2 * d * d + 64 +
                         2 * 64 + 2;
  if (len != FG::blob_len() + gan_len + 2 * FG::K) return "FPE weight blob length mismatch";
  Reader rd{blob, len};
  const double* Wih = rd.take(9 * FG::NIN);
  const double* Whh = rd.take(27);
  const double* bih = rd.take(9);
  const double* bhh = rd.take(9);
  const double* fcW = rd.take(d * 3);
  const double* attn = rd.take(2 * d);
  const double* inW = rd.take(3 * E * E);
  const double* inB = rd.take(3 * E);
  const double* outW = rd.take(E * E);
  const double* outB = rd.take(E);
  const double* encW = rd.take((size_t)L * d * KC);
  const double* encB = rd.take(L * d);
  const double* anW = rd.take(2 * L);
  const double* anB = rd.take(2);
  const double* prW = rd.take(2 * L);
  const double* prB = rd.take(2);
  const int GIN = 2 * d + d * d;
  const double* g0W = rd.take((size_t)64 * GIN);
  const double* g0B = rd.take(64);
  const double* g2W = rd.take((size_t)d * d * 64);
  const double* g2B = rd.take(d * d);
  const double* d0W = rd.take((size_t)64 * 2 * d * d);
  const double* d0B = rd.take(64);
  const double* d2W = rd.take(2 * 64);
  const double* d2B = rd.take(2);
  const double* protos = rd.take(2 * FG::K);
  if (rd.off != len) return "FPE weight blob parse error";

  P->frags.assign(G::SZ_FRAGS, 0.0f);
  P->enc_tab.assign(FG::F_SIZE, 0.0f);
  P->gan_tab.assign(G::G_SIZE, 0.0f);
  float* T = P->enc_tab.data();
  const double log2e = 1.4426950408889634;
  for (int i = 0; i < 9 * FG::NIN; ++i) T[FG::F_WIH + i] = (float)Wih[i];
  for (int i = 0; i < 27; ++i) T[FG::F_WHH + i] = (float)Whh[i];
  for (int i = 0; i < 6; ++i) T[FG::F_BRZ + i] = (float)(bih[i] + bhh[i]);
  for (int i = 0; i < 3; ++i) {
    T[FG::F_BIN + i] = (float)bih[6 + i];
    T[FG::F_BHN + i] = (float)bhh[6 + i];
  }
  for (int f = 0; f < 3; ++f) {
    double u = 0, v = 0;
    for (int k = 0; k < d; ++k) {
      u += fcW[k * 3 + f] * attn[k];
      v += fcW[k * 3 + f] * attn[d + k];
    }
    T[FG::F_UV + f] = (float)(u * log2e);
    T[FG::F_UV + 4 + f] = (float)(v * log2e);
  }
  // P [E][6]: rows 0-2 the identity on the GRU state, rows 3.. Wfc / H
  std::vector<double> Pm((size_t)E * 6, 0.0);
  for (int k = 0; k < 3; ++k) Pm[(size_t)k * 6 + k] = 1.0;
  for (int dd = 0; dd < d; ++dd)
    for (int f = 0; f < 3; ++f) Pm[(size_t)(3 + dd) * 6 + 3 + f] = fcW[dd * 3 + f] / d;
  const double* Wq = inW;
  const double* Wk = inW + E * E;
  const double* Wv = inW + 2 * E * E;
  const double* bq = inB;
  const double* bv = inB + 2 * E;
  const double sc = log2e / std::sqrt((double)E);
  std::vector<double> M((size_t)E * E), beta(E);  // Wq^T Wk, Wk^T bq
  for (int a = 0; a < E; ++a) {
    for (int b = 0; b < E; ++b) {
      double m = 0;
      for (int e = 0; e < E; ++e) m += Wq[e * E + a] * Wk[e * E + b];
      M[(size_t)a * E + b] = m;
    }
    double bb = 0;
    for (int e = 0; e < E; ++e) bb += Wk[e * E + a] * bq[e];
    beta[a] = bb;
  }
  std::vector<double> MP((size_t)E * 6, 0.0);  // M P
  for (int a = 0; a < E; ++a)
    for (int k = 0; k < 6; ++k) {
      double acc = 0;
      for (int b = 0; b < E; ++b) acc += M[(size_t)a * E + b] * Pm[(size_t)b * 6 + k];
      MP[(size_t)a * 6 + k] = acc;
    }
  for (int j = 0; j < 6; ++j) {
    for (int k = 0; k < 6; ++k) {
      double acc = 0;
      for (int a = 0; a < E; ++a) acc += Pm[(size_t)a * 6 + j] * MP[(size_t)a * 6 + k];
      T[FG::F_M6 + j * 6 + k] = (float)(acc * sc);
    }
    double bb = 0;
    for (int a = 0; a < E; ++a) bb += Pm[(size_t)a * 6 + j] * beta[a];
    T[FG::F_BETA6 + j] = (float)(bb * sc);
  }
  std::vector<double> A((size_t)E * 6), a0(E);  // A = Wout Wv P, a0 = Wout bv + bout
  {
    std::vector<double> OV((size_t)E * E);
    for (int f = 0; f < E; ++f) {
      double acc0 = outB[f];
      for (int g = 0; g < E; ++g) acc0 += outW[f * E + g] * bv[g];
      a0[f] = acc0;
      for (int e = 0; e < E; ++e) {
        double acc = 0;
        for (int g = 0; g < E; ++g) acc += outW[f * E + g] * Wv[g * E + e];
        OV[(size_t)f * E + e] = acc;
      }
    }
    for (int f = 0; f < E; ++f)
      for (int k = 0; k < 6; ++k) {
        double acc = 0;
        for (int e = 0; e < E; ++e) acc += OV[(size_t)f * E + e] * Pm[(size_t)e * 6 + k];
        A[(size_t)f * 6 + k] = acc;
      }
  }
  // encoder rows composed with A:  WA[row][s*6+k] = sum_f Wenc[row][s*E+f] A[f][k]
  const int KU = FG::KU;
  std::vector<double> WA((size_t)L * d * KU), bA((size_t)L * d);
  for (int row = 0; row < L * d; ++row) {
    double bb = encB[row];
    for (int s = 0; s < 3; ++s) {
      for (int f = 0; f < E; ++f) bb += encW[(size_t)row * KC + s * E + f] * a0[f];
      for (int k = 0; k < 6; ++k) {
        double acc = 0;
        for (int f = 0; f < E; ++f) acc += encW[(size_t)row * KC + s * E + f] * A[(size_t)f * 6 + k];
        WA[(size_t)row * KU + s * 6 + k] = acc;
      }
    }
    bA[row] = bb;
  }
  for (int h = 0; h < d; ++h)
    for (int q = 0; q < 4; ++q) {
      const double* dw = q < 2 ? anW + q * L : prW + (q - 2) * L;
      double bb = q < 2 ? anB[q] : prB[q - 2];
      for (int l = 0; l < L; ++l) bb += dw[l] * bA[h * L + l];
      T[FG::F_B2 + 4 * h + q] = (float)bb;
      for (int k = 0; k < KU; ++k) {
        double acc = 0;
        for (int l = 0; l < L; ++l) acc += dw[l] * WA[(size_t)(h * L + l) * KU + k];
        T[FG::F_W6 + (4 * h + q) * KU + k] = (float)acc;
      }
    }
  for (int k = 0; k < 2 * FG::K; ++k) T[FG::F_PROTO + k] = (float)protos[k];
  const HostSrc src{blob};
  auto V = [&](const double* q) { return View<HostSrc>{src, (long)(q - blob)}; };
  packcore::pack_gan<H>(V(g0W), V(g0B), V(g2W), V(g2B), V(d0W), V(d0B), V(d2W), V(d2B), HostEx{}, P->frags.data(),
                        P->gan_tab.data());
  P->gat = GatConst{};
  return "";
}

}  // namespace

size_t blob_len(int H, int K) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return blob_len_t<h>(K);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

std::string pack_weights(int H, int K, const double* blob, size_t len, Packed* out) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return pack_t<h>(K, blob, len, out);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return "unsupported host count";
}

size_t fpe_blob_len(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return FpeGeo<h>::blob_len() + (size_t)64 * (2 * h + h * h) + 64 + (size_t)h * h * 64 + h * h + \
           64 * 2 * h * h + 64 + 2 * 64 + 2 + 2 * FpeGeo<h>::K;
    PGP_FOR_EACH_FPE_H(CASE)
#undef CASE
  }
  return 0;
}

std::string pack_fpe_weights(int H, const double* blob, size_t len, Packed* out) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return pack_fpe_t<h>(blob, len, out);
    PGP_FOR_EACH_FPE_H(CASE)
#undef CASE
  }
  return "FPE variant: unsupported host count";
}

}  // namespace pgp
