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

#include <cmath>
#include <cstring>
#include <vector>

namespace pgp {
namespace {

struct Reader {
  const double* p;
  size_t len, off = 0;
  const double* take(size_t n) {
    const double* r = p + off;
    off += n;
    return r;
  }
};

// feature of d-space row R (see pgp_layout.hpp): R = 16t+4g+r <-> c = 16t+4r+g
inline int featX(int R) { return 16 * (R / 16) + 4 * (R % 4) + (R % 16) / 4; }

// Gen / Disc (models.py:118-151) into the K3 chunk layout (pgp_gan.hip).
template <int H>
void pack_gan(const double* g0W, const double* g0B, const double* g2W, const double* g2B, const double* d0W,
              const double* d0B, const double* d2W, const double* d2B, float* F, float* GT) {
  using G = Geo<H>;
  const int d = H, GIN = 2 * d + d * d;
  for (int mt = 0; mt < G::MT_G; ++mt)
    for (int lane = 0; lane < 64; ++lane)
      for (int e4 = 0; e4 < 4; ++e4) {
        const int i = lane & 15, g = lane >> 4, row = 16 * mt + i;
        for (int q = 0; q < G::EQ; ++q) {
          const int k = 16 * q + 4 * g + e4;
          if (k < 2 * d)
            F[G::OFF_GE + (long)(mt * G::EQ + q) * G::FQ + lane * 4 + e4] = (float)g0W[(size_t)row * GIN + k];
        }
        for (int q = 0; q < G::SQ; ++q) {
          const int k = 16 * q + 4 * g + e4;
          if (k >= d * d) continue;
          F[G::OFF_GS + ((long)q * G::GS_G + mt) * G::FQ + lane * 4 + e4] =
              (float)g0W[(size_t)row * GIN + 2 * d + k];
          F[G::OFF_GS + ((long)q * G::GS_G + G::MT_G + mt) * G::FQ + lane * 4 + e4] =
              (float)d0W[(size_t)row * 2 * d * d + k];
        }
      }
  for (int c = 0; c < d; ++c) {
    float* FC = F + G::OFF_GC + (long)c * G::GC_G * G::FQ;
    for (int t = 0; t < G::MT_N; ++t)
      for (int q4 = 0; q4 < 4; ++q4)
        for (int lane = 0; lane < 64; ++lane)
          for (int e4 = 0; e4 < 4; ++e4) {
            const int i = lane & 15, g = lane >> 4, u = 16 * q4 + 4 * g + e4, hh = 16 * t + i;
            if (hh >= d) continue;
            FC[(t * 4 + q4) * G::FQ + lane * 4 + e4] = (float)g2W[(size_t)(c * d + hh) * 64 + u];
          }
    for (int mt = 0; mt < G::MT_G; ++mt)
      for (int q4 = 0; q4 < G::MT_N; ++q4)
        for (int lane = 0; lane < 64; ++lane)
          for (int e4 = 0; e4 < 4; ++e4) {
            const int i = lane & 15, g = lane >> 4, hh = 16 * q4 + 4 * g + e4;
            if (hh >= d) continue;
            FC[(G::GC_G2 + mt * G::MT_N + q4) * G::FQ + lane * 4 + e4] =
                (float)d0W[(size_t)(16 * mt + i) * 2 * d * d + d * d + c * d + hh];
          }
    for (int R = 0; R < G::MT_N * 16; ++R)
      if (R < d) GT[G::G_B2 + c * G::MT_N * 16 + R] = (float)g2B[c * d + R];
  }
  for (int u = 0; u < 64; ++u) {
    GT[G::G_B1 + u] = (float)g0B[u];
    GT[G::G_BD1 + u] = (float)d0B[u];
    GT[G::G_WD2 + u] = (float)d2W[u];
    GT[G::G_WD2 + 64 + u] = (float)d2W[64 + u];
  }
  GT[G::G_BD2 + 0] = (float)d2B[0];
  GT[G::G_BD2 + 1] = (float)d2B[1];
}

// Tail mode (Geo<H>::TAIL): q/k/v tile t, C-row i -> (head, dim).  Slot
// sigma = 4*(i%4) + i/4 (the B-operand order of the row); tiles [0,HF) head 0,
// [HF,2HF) head 1, tile 2HF: sigma < HT head 0's tail, else head 1's tail.
// Head 1's last SR tail dims are VALU rows n: dim 16*HF + 16 - HT + n.
template <int H>
bool tail_slot(int t, int i, int* hh, int* e) {
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
bool tail_oslot(int s, int g, int* hh, int* e) {
  using G = Geo<H>;
  if (s < 4 * G::TQ) return tail_slot<H>(s / 4, 4 * g + s % 4, hh, e);
  if (s == 4 * G::TQ && g < G::SR) {
    *hh = 1;
    *e = 16 * G::HF + 16 - G::HT + g;
    return true;
  }
  return false;
}

template <int H>
void pack_tail_attention(const double* inW, const double* inB, const double* outW, double scale, float* FL,
                         float* TL) {
  using G = Geo<H>;
  const int d = H;
  // q, k tiles (stage 0) and v tiles (stage 1): [m][t][q4] groups over X k-steps
  for (int m = 0; m < 3; ++m)
    for (int t = 0; t < G::TQ; ++t) {
      const long base = m < 2 ? (long)(m * G::TQ + t) * G::KQ_D : G::P_V + (long)t * G::KQ_D;
      for (int q4 = 0; q4 < G::KQ_D; ++q4)
        for (int lane = 0; lane < 64; ++lane)
          for (int e4 = 0; e4 < 4; ++e4) {
            const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4, c = 4 * s + g;
            int hh, e;
            if (s >= G::KS_D || c >= d || !tail_slot<H>(t, i, &hh, &e)) continue;
            const int src = m * d + hh * G::HD + e;
            FL[(base + q4) * G::FQ + lane * 4 + e4] = (float)(inW[src * d + c] * (m == 0 ? scale : 1.0));
          }
      for (int i = 0; i < 16; ++i) {
        int hh, e;
        if (!tail_slot<H>(t, i, &hh, &e)) continue;
        TL[G::TL_QKV + (m * G::TQ + t) * 16 + i] = (float)(inB[m * d + hh * G::HD + e] * (m == 0 ? scale : 1.0));
      }
      // VALU rows of head 1's tail
      if (t == 0)
        for (int n = 0; n < G::SR; ++n) {
          const int src = m * d + G::HD + 16 * G::HF + 16 - G::HT + n;
          for (int q4 = 0; q4 < G::KQ_D; ++q4)
            for (int g = 0; g < 4; ++g)
              for (int e4 = 0; e4 < 4; ++e4) {
                const int s = 4 * q4 + e4, c = 4 * s + g;
                if (s >= G::KS_D || c >= d) continue;
                TL[G::TL_RQ + (((m * G::SR + n) * G::KQ_D + q4) * 4 + g) * 4 + e4] =
                    (float)(inW[src * d + c] * (m == 0 ? scale : 1.0));
              }
          TL[G::TL_RQB + m * G::SR + n] = (float)(inB[src] * (m == 0 ? scale : 1.0));
        }
    }
  // out_proj: MT_X output tiles over the O slots (+ VALU rows 16*MT_X + n)
  for (int mt = 0; mt < G::MT_X; ++mt)
    for (int q4 = 0; q4 < G::KQ_OT; ++q4)
      for (int lane = 0; lane < 64; ++lane)
        for (int e4 = 0; e4 < 4; ++e4) {
          const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4;
          const int co = featX(16 * mt + i);
          int hh, e;
          if (co >= d || !tail_oslot<H>(s, g, &hh, &e)) continue;
          FL[(G::P_OT + mt * G::KQ_OT + q4) * G::FQ + lane * 4 + e4] = (float)outW[co * d + hh * G::HD + e];
        }
  for (int n = 0; n < G::XR; ++n)
    for (int q4 = 0; q4 < G::KQ_OT; ++q4)
      for (int g = 0; g < 4; ++g)
        for (int e4 = 0; e4 < 4; ++e4) {
          int hh, e;
          if (!tail_oslot<H>(4 * q4 + e4, g, &hh, &e)) continue;
          TL[G::TL_RO + ((n * G::KQ_OT + q4) * 4 + g) * 4 + e4] =
              (float)outW[(16 * G::MT_X + n) * d + hh * G::HD + e];
        }
}

template <int H>
size_t blob_len_t(int K) {
  const size_t d = H, L = 3 * H * H;
  size_t n = d * 3 + 2 * d + d * d + d + 3 * d;
  n += 2 * (3 * d * d + 3 * d + d * d + d + 64 * d + 64 + d * 64 + d + 4 * d);
  n += 2 * (2 * d * L + 2 * d);
  n += 64 * (2 * d + d * d) + 64 + d * d * 64 + d * d;
  n += 64 * 2 * d * d + 64 + 2 * 64 + 2;
  n += (size_t)K * 2;
  return n;
}

template <int H>
std::string pack_t(int K, const double* blob, size_t len, Packed* P) {
  using G = Geo<H>;
  if (len != blob_len_t<H>(K)) return "weight blob length mismatch";
  Reader rd{blob, len};
  const int d = H, L = 3 * H * H;
  const double* fcW = rd.take(d * 3);
  const double* attn = rd.take(2 * d);
  const double* teW = rd.take(d * d);
  const double* teB = rd.take(d);
  const double* pe = rd.take(3 * d);
  struct LayerSrc {
    const double *inW, *inB, *outW, *outB, *l1W, *l1B, *l2W, *l2B, *n1w, *n1b, *n2w, *n2b;
  } ly[kLayers];
  for (int l = 0; l < kLayers; ++l) {
    ly[l].inW = rd.take(3 * d * d);
    ly[l].inB = rd.take(3 * d);
    ly[l].outW = rd.take(d * d);
    ly[l].outB = rd.take(d);
    ly[l].l1W = rd.take(64 * d);
    ly[l].l1B = rd.take(64);
    ly[l].l2W = rd.take(d * 64);
    ly[l].l2B = rd.take(d);
    ly[l].n1w = rd.take(d);
    ly[l].n1b = rd.take(d);
    ly[l].n2w = rd.take(d);
    ly[l].n2b = rd.take(d);
  }
  const double* anW = rd.take((size_t)2 * d * L);
  const double* anB = rd.take(2 * d);
  const double* prW = rd.take((size_t)2 * d * L);
  const double* prB = rd.take(2 * d);
  const int GIN = 2 * d + d * d;
  const double* g0W = rd.take((size_t)64 * GIN);
  const double* g0B = rd.take(64);
  const double* g2W = rd.take((size_t)d * d * 64);
  const double* g2B = rd.take(d * d);
  const double* d0W = rd.take((size_t)64 * 2 * d * d);
  const double* d0B = rd.take(64);
  const double* d2W = rd.take(2 * 64);
  const double* d2B = rd.take(2);
  const double* protos = rd.take(2 * K);
  if (rd.off != len) return "weight blob parse error";
  (void)GIN;

  P->frags.assign(G::SZ_FRAGS, 0.0f);
  P->enc_tab.assign(G::t_size(K), 0.0f);
  P->gan_tab.assign(G::G_SIZE, 0.0f);
  float* F = P->frags.data();
  float* T = P->enc_tab.data();
  float* GT = P->gan_tab.data();

  // ---- GAT constants ----
  for (int f = 0; f < 3; ++f) {
    double u = 0, v = 0;
    for (int c = 0; c < d; ++c) {
      u += fcW[c * 3 + f] * attn[c];
      v += fcW[c * 3 + f] * attn[d + c];
    }
    // pre-scaled by log2(e): leaky_relu is positively homogeneous, so the kernel
    // evaluates exp(e - M) as exp2(e' - M') with one v_exp_f32
    P->gat.u[f] = (float)(u * 1.4426950408889634);
    P->gat.v[f] = (float)(v * 1.4426950408889634);
  }
  P->gat.u[3] = P->gat.v[3] = 0.f;

  // ---- time encoder (folded with GAT fc) ----
  for (int mt = 0; mt < G::MT_D; ++mt)
    for (int lane = 0; lane < 64; ++lane) {
      const int i = lane & 15, g = lane >> 4;
      const int c = featX(16 * mt + i);
      if (c >= d || g >= 3) continue;
      double acc = 0;
      for (int k = 0; k < d; ++k) acc += teW[c * d + k] * fcW[k * 3 + g];
      T[G::T_TEW + mt * 64 + lane] = (float)acc;
    }
  for (int w = 0; w < 3; ++w)
    for (int R = 0; R < G::DP; ++R) {
      const int c = featX(R);
      if (c < d) T[G::T_TE + w * G::DP + R] = (float)(teB[c] + pe[w * d + c]);
    }

  // ---- encoder layers ----
  const double scale = 1.0 / std::sqrt((double)G::HD);
  for (int l = 0; l < kLayers; ++l) {
    const LayerSrc& S = ly[l];
    float* FL = F + G::OFF_ENC + (long)l * G::LAYER_G * G::FQ;
    float* TL = T + G::T_L0 + l * G::TL_SIZE;
    if constexpr (G::TAIL) {
      pack_tail_attention<H>(S.inW, S.inB, S.outW, scale, FL, TL);
    } else {
      // head-space row R within a pass block -> (head, dim), valid?
      auto head_row = [&](int p, int R, int* hh, int* e) -> bool {
        if (G::P8) {
          const int g = (R % 16) / 4, r = R % 4;
          *hh = g >> 1;
          *e = 4 * (g & 1) + r;
        } else {
          *hh = p;
          *e = featX(R);
        }
        return *e < G::HD;
      };
      for (int p = 0; p < G::NPASS; ++p)
        for (int m = 0; m < 3; ++m)
          for (int tp = 0; tp < G::TP; ++tp) {
            for (int q4 = 0; q4 < G::KQ_D; ++q4)
              for (int lane = 0; lane < 64; ++lane)
                for (int e4 = 0; e4 < 4; ++e4) {
                  const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4;
                  const int c = 4 * s + g;
                  int hh, e;
                  if (s >= G::KS_D || c >= d || !head_row(p, 16 * tp + i, &hh, &e)) continue;
                  const int src = m * d + hh * G::HD + e;
                  const double v = S.inW[src * d + c] * (m == 0 ? scale : 1.0);
                  FL[(G::P_QKV(p) + (m * G::TP + tp) * G::KQ_D + q4) * G::FQ + lane * 4 + e4] = (float)v;
                }
            for (int i = 0; i < 16; ++i) {
              int hh, e;
              if (!head_row(p, 16 * tp + i, &hh, &e)) continue;
              const int src = m * d + hh * G::HD + e;
              TL[G::TL_QKV + (p * 3 + m) * G::TP * 16 + 16 * tp + i] =
                  (float)(S.inB[src] * (m == 0 ? scale : 1.0));
            }
          }
      // out_proj
      for (int p = 0; p < G::NPASS; ++p)
        for (int mt = 0; mt < G::MT_D; ++mt)
          for (int q4 = 0; q4 < G::KQ_O; ++q4)
            for (int lane = 0; lane < 64; ++lane)
              for (int e4 = 0; e4 < 4; ++e4) {
                const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4;
                const int co = featX(16 * mt + i);
                if (s >= G::KS_O || co >= d) continue;
                int hh, e;
                if (G::P8) {
                  hh = g >> 1;
                  e = 4 * (g & 1) + s;
                } else {
                  hh = p;
                  e = 4 * s + g;
                }
                if (e >= G::HD) continue;
                FL[(G::P_O(p) + mt * G::KQ_O + q4) * G::FQ + lane * 4 + e4] =
                    (float)S.outW[co * d + hh * G::HD + e];
              }
    }
    // FFN
    for (int mt = 0; mt < G::MT_F; ++mt)
      for (int q4 = 0; q4 < G::KQ_D; ++q4)
        for (int lane = 0; lane < 64; ++lane)
          for (int e4 = 0; e4 < 4; ++e4) {
            const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4, c = 4 * s + g;
            if (s >= G::KS_D || c >= d) continue;
            // norm1's gamma folded into linear1 (the kernel feeds it the un-scaled x-hat)
            FL[(G::P_F1 + mt * G::KQ_D + q4) * G::FQ + lane * 4 + e4] =
                (float)(S.l1W[(16 * mt + i) * d + c] * S.n1w[c]);
          }
    for (int mt = 0; mt < G::MT_X; ++mt)
      for (int q4 = 0; q4 < G::KQ_F; ++q4)
        for (int lane = 0; lane < 64; ++lane)
          for (int e4 = 0; e4 < 4; ++e4) {
            const int i = lane & 15, g = lane >> 4, u = 16 * q4 + 4 * g + e4;
            const int co = featX(16 * mt + i);
            if (co >= d) continue;
            FL[(G::P_F2 + mt * G::KQ_F + q4) * G::FQ + lane * 4 + e4] = (float)S.l2W[co * 64 + u];
          }
    for (int R = 0; R < G::DP; ++R) {
      const int c = featX(R);
      if (c >= d) continue;
      TL[G::TL_BO + R] = (float)S.outB[c];
      TL[G::TL_LN1G + R] = (float)S.n1w[c];
      TL[G::TL_LN1B + R] = (float)S.n1b[c];
      TL[G::TL_B2 + R] = (float)(S.l2B[c] + S.n1b[c]);  // + norm1's beta: the residual is gamma*x-hat + beta
      TL[G::TL_LN2G + R] = (float)S.n2w[c];
      TL[G::TL_LN2B + R] = (float)S.n2b[c];
    }
    for (int u = 0; u < 64; ++u) {  // linear1 bias + linear1 . norm1's beta
      double b = S.l1B[u];
      for (int c = 0; c < d; ++c) b += S.l1W[u * d + c] * S.n1b[c];
      TL[G::TL_B1 + u] = (float)b;
    }
    // tail mode: linear2 rows of the VALU d-rows (feature 16*MT_X + n)
    for (int n = 0; n < G::XR; ++n)
      for (int q4 = 0; q4 < G::KQ_F; ++q4)
        for (int g = 0; g < 4; ++g)
          for (int e = 0; e < 4; ++e)
            TL[G::TL_RF + ((n * G::KQ_F + q4) * 4 + g) * 4 + e] =
                (float)S.l2W[(16 * G::MT_X + n) * 64 + 16 * q4 + 4 * g + e];
  }

  // ---- layer 0's q/k/v folded onto the aggregated raw features ----
  // X0[c] = sum_f A[c][f] agg[f] + teB[c] + pe[w][c], A = Wte Wfc, so
  // qkv[src] = sum_f (Win A)[src][f] agg[f] + (inB + Win (teB + pe[w]))[src]
  {
    const LayerSrc& S = ly[0];
    std::vector<double> A((size_t)d * 3, 0.0);
    for (int c = 0; c < d; ++c)
      for (int f = 0; f < 3; ++f)
        for (int k = 0; k < d; ++k) A[c * 3 + f] += teW[c * d + k] * fcW[k * 3 + f];
    auto fold = [&](int src, double* wf, double* bw) {  // wf[3], bw[3 steps]
      const double sc = src < d ? scale : 1.0;
      for (int f = 0; f < 3; ++f) {
        double acc = 0;
        for (int c = 0; c < d; ++c) acc += S.inW[(size_t)src * d + c] * A[c * 3 + f];
        wf[f] = acc * sc;
      }
      for (int w = 0; w < 3; ++w) {
        double acc = S.inB[src];
        for (int c = 0; c < d; ++c) acc += S.inW[(size_t)src * d + c] * (teB[c] + pe[w * d + c]);
        bw[w] = acc * sc;
      }
    };
    // (tile, C-row) -> source row of in_proj, or -1
    auto tile_src = [&](int T, int i) -> int {
      int hh, e, m;
      if constexpr (G::TAIL) {
        m = T / G::TQ;
        if (!tail_slot<H>(T % G::TQ, i, &hh, &e)) return -1;
      } else {
        const int p = T / (3 * G::TP), r = T % (3 * G::TP), tp = r % G::TP;
        m = r / G::TP;
        const int R = 16 * tp + i;
        if (G::P8) {
          const int g = (R % 16) / 4, rr = R % 4;
          hh = g >> 1;
          e = 4 * (g & 1) + rr;
        } else {
          hh = p;
          e = featX(R);
        }
        if (e >= G::HD) return -1;
      }
      return m * d + hh * G::HD + e;
    };
    for (int T0 = 0; T0 < 3 * G::NQT; ++T0)
      for (int i = 0; i < 16; ++i) {
        const int src = tile_src(T0, i);
        if (src < 0) continue;
        double wf[3], bw[3];
        fold(src, wf, bw);
        for (int g = 0; g < 3; ++g) T[G::T_F0 + T0 * 64 + 16 * g + i] = (float)wf[g];
        for (int w = 0; w < 3; ++w) T[G::T_F0B + (w * 3 * G::NQT + T0) * 16 + i] = (float)bw[w];
      }
    if constexpr (G::TAIL) {  // out_proj through the attention: per head hh and output c
      // Gh[c][f] = sum_e Wo[c][hh*HD+e] Fv[e][f], Ch[c][w'] = sum_e Wo[c][hh*HD+e] bv_w'[e]
      std::vector<double> Gm((size_t)2 * d * 3, 0.0), Cm((size_t)2 * d * 3, 0.0);
      for (int hh = 0; hh < 2; ++hh)
        for (int e = 0; e < G::HD; ++e) {
          double wf[3], bw[3];
          fold(2 * d + hh * G::HD + e, wf, bw);
          for (int c = 0; c < d; ++c) {
            const double wo = S.outW[(size_t)c * d + hh * G::HD + e];
            for (int f = 0; f < 3; ++f) {
              Gm[((size_t)hh * d + c) * 3 + f] += wo * wf[f];
              Cm[((size_t)hh * d + c) * 3 + f] += wo * bw[f];
            }
          }
        }
      for (int hh = 0; hh < 2; ++hh)
        for (int mt = 0; mt < G::MT_X; ++mt)
          for (int i = 0; i < 16; ++i) {
            const int c = featX(16 * mt + i);
            if (c >= d) continue;
            for (int g = 0; g < 3; ++g) {
              T[G::T_F0O + ((hh * 2 + 0) * G::MT_X + mt) * 64 + 16 * g + i] = (float)Gm[((size_t)hh * d + c) * 3 + g];
              T[G::T_F0O + ((hh * 2 + 1) * G::MT_X + mt) * 64 + 16 * g + i] = (float)Cm[((size_t)hh * d + c) * 3 + g];
            }
          }
      for (int n = 0; n < G::XR; ++n) {
        const int c = 16 * G::MT_X + n;
        for (int hh = 0; hh < 2; ++hh)
          for (int g = 0; g < 3; ++g) {
            T[G::T_F0OR + n * 16 + (hh * 2 + 0) * 4 + g] = (float)Gm[((size_t)hh * d + c) * 3 + g];
            T[G::T_F0OR + n * 16 + (hh * 2 + 1) * 4 + g] = (float)Cm[((size_t)hh * d + c) * 3 + g];
          }
      }
    }
    if constexpr (G::TAIL) {  // layer 0's scores per head as bilinear forms of the raw features
      for (int hh = 0; hh < 2; ++hh) {
        double M[9] = {}, U[9] = {}, V[9] = {}, Sc[9] = {};
        for (int e = 0; e < G::HD; ++e) {
          double qf[3], qb[3], kf[3], kb[3];
          fold(hh * G::HD + e, qf, qb);      // q (attention scale folded in)
          fold(d + hh * G::HD + e, kf, kb);  // k
          for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
              M[a * 3 + b] += qf[a] * kf[b];
              U[a * 3 + b] += qf[a] * kb[b];   // (f, key step)
              V[a * 3 + b] += qb[a] * kf[b];   // (query step, f)
              Sc[a * 3 + b] += qb[a] * kb[b];  // (query step, key step)
            }
        }
        for (int i = 0; i < 9; ++i) {
          T[G::T_F0S + hh * 36 + i] = (float)M[i];
          T[G::T_F0S + hh * 36 + 9 + i] = (float)U[i];
          T[G::T_F0S + hh * 36 + 18 + i] = (float)V[i];
          T[G::T_F0S + hh * 36 + 27 + i] = (float)Sc[i];
        }
      }
    }
    for (int m = 0; m < 3; ++m)
      for (int n = 0; n < G::SR; ++n) {
        const int src = m * d + G::HD + 16 * G::HF + 16 - G::HT + n;
        double wf[3], bw[3];
        fold(src, wf, bw);
        for (int g = 0; g < 3; ++g) T[G::T_F0R + (m * G::SR + n) * 4 + g] = (float)wf[g];
        for (int w = 0; w < 3; ++w) T[G::T_F0RB + w * 3 * G::SR + m * G::SR + n] = (float)bw[w];
      }
  }

  // ---- decoders: rows n = 4*host + {l0, l1, p0, p1} ----
  for (int h = 0; h < d; ++h)
    for (int w = 0; w < 3; ++w)
      for (int mt = 0; mt < G::MT_O; ++mt)
        for (int q4 = 0; q4 < G::KQ_D; ++q4)
          for (int lane = 0; lane < 64; ++lane)
            for (int e4 = 0; e4 < 4; ++e4) {
              const int i = lane & 15, g = lane >> 4, s = 4 * q4 + e4, c = 4 * s + g;
              const int n = 16 * mt + i, host = n / 4, q = n % 4;
              if (s >= G::KS_D || c >= d || host >= d) continue;
              const size_t col = (size_t)h * 3 * d + w * d + c;
              const double v = q < 2 ? anW[(size_t)(2 * host + q) * L + col]
                                     : prW[(size_t)(2 * host + q - 2) * L + col];
              F[G::OFF_DEC + ((long)(h * 3 + w) * G::DEC_G + mt * G::KQ_D + q4) * G::FQ + lane * 4 + e4] =
                  (float)v;
            }
  for (int n = 0; n < G::MT_O * 16; ++n) {
    const int host = n / 4, q = n % 4;
    if (host >= d) continue;
    T[G::T_DEC + n] = (float)(q < 2 ? anB[2 * host + q] : prB[2 * host + q - 2]);
  }
  for (int k = 0; k < 2 * K; ++k) T[G::T_PROTO + k] = (float)protos[k];

  pack_gan<H>(g0W, g0B, g2W, g2B, d0W, d0B, d2W, d2B, F, GT);
  return "";
}


// ---------------------------------------------------------------------------
// PreGAN FPE_16 variant (models.py:10-115).  Folds, all in fp64:
//   GAT node mean: mean_j sum_i a_ij Wfc x_i = (Wfc / H) sum_i r_i x_i, r_i = sum_j a_ij
//   edge scores as above (u, v), pre-scaled by log2(e)
//   MHA scores: q_s.k_t = c_s^T (Wq^T Wk) c_t + (Wk^T bq).c_t + (terms constant in t,
//     which cancel in the softmax over t); 1/sqrt(E) and log2(e) folded in
//   V, out_proj, encoder Linear (identity LeakyReLU(True)) and both decoders are
//     affine maps applied after a convex combination (sum_t p_st = 1), so
//     [a0 a1 p0 p1]_host = W2 . [sum_t p_st c_t]_s + b2 with
//     W2 = Dec . Wenc . blockdiag_s(Wout Wv), b2 = Dec (Wenc (Wout bv + bout)_s + benc) + bdec
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
  for (int i = 0; i < 3 * d; ++i) T[FG::F_FC + i] = (float)(fcW[i] / d);
  const double* Wq = inW;
  const double* Wk = inW + E * E;
  const double* Wv = inW + 2 * E * E;
  const double* bq = inB;
  const double* bv = inB + 2 * E;
  const double sc = log2e / std::sqrt((double)E);
  for (int a = 0; a < E; ++a) {
    for (int b = 0; b < E; ++b) {
      double m = 0;
      for (int e = 0; e < E; ++e) m += Wq[e * E + a] * Wk[e * E + b];
      T[FG::F_M + a * E + b] = (float)(m * sc);
    }
    double beta = 0;
    for (int e = 0; e < E; ++e) beta += Wk[e * E + a] * bq[e];
    T[FG::F_BETA + a] = (float)(beta * sc);
  }
  std::vector<double> A((size_t)E * E), a0(E);  // A = Wout Wv, a0 = Wout bv + bout
  for (int f = 0; f < E; ++f) {
    double acc0 = outB[f];
    for (int g = 0; g < E; ++g) acc0 += outW[f * E + g] * bv[g];
    a0[f] = acc0;
    for (int e = 0; e < E; ++e) {
      double acc = 0;
      for (int g = 0; g < E; ++g) acc += outW[f * E + g] * Wv[g * E + e];
      A[(size_t)f * E + e] = acc;
    }
  }
  // encoder rows composed with A:  WA[row][s*E+e] = sum_f Wenc[row][s*E+f] A[f][e]
  std::vector<double> WA((size_t)L * d * KC), bA((size_t)L * d);
  for (int row = 0; row < L * d; ++row) {
    double bb = encB[row];
    for (int s = 0; s < 3; ++s) {
      for (int f = 0; f < E; ++f) bb += encW[(size_t)row * KC + s * E + f] * a0[f];
      for (int e = 0; e < E; ++e) {
        double acc = 0;
        for (int f = 0; f < E; ++f) acc += encW[(size_t)row * KC + s * E + f] * A[(size_t)f * E + e];
        WA[(size_t)row * KC + s * E + e] = acc;
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
      for (int k = 0; k < KC; ++k) {
        double acc = 0;
        for (int l = 0; l < L; ++l) acc += dw[l] * WA[(size_t)(h * L + l) * KC + k];
        T[FG::F_W2 + (4 * h + q) * KC + k] = (float)acc;
      }
    }
  for (int k = 0; k < 2 * FG::K; ++k) T[FG::F_PROTO + k] = (float)protos[k];
  pack_gan<H>(g0W, g0B, g2W, g2B, d0W, d0B, d2W, d2B, P->frags.data(), P->gan_tab.data());
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
