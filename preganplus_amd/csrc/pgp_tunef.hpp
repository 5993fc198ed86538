// pgp_tunef.hpp — geometry and launch interface of the fused tuning-encoder
// kernels (pgp_tunef.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_layout.hpp"
#include "pgp_train.hpp"

#ifndef PGP_TF_SPLIT
#define PGP_TF_SPLIT 1  // split-bf16 feed-forward GEMMs in the fused kernels at H = 50 (A/B: -DPGP_TF_SPLIT=0)
#endif

namespace pgp {

// weight fragment matrices (A operands; "T" = transposed for the backward)
enum TfMat : int { TFM_TE = 0, TFM_IN, TFM_O, TFM_F1, TFM_F2, TFM_F2T, TFM_F1T, TFM_INT, TFM_OT };

template <int H>
struct TF {
  static constexpr int D = H, DP = round_up(H, 16), NT = DP / 16, HD = H / 2;
  // k-steps over d in the natural row map (feature 16t + 4g + r of k-step (t, r))
  static constexpr int KS = 4 * (H / 16) + ((H % 16) == 0 ? 0 : ((H % 16) < 4 ? (H % 16) : 4));
  static constexpr int KG = (KS + 3) / 4;
  static constexpr int NQ = 3 * NT;          // q | k | v output tiles
  static constexpr int KSQ = 3 * KS, KGQ = (KSQ + 3) / 4;
  static constexpr int KGF = 4;              // 16 k-steps over the FFN hidden (64)
  static constexpr int Q3P = round_up(3 * H, 16);
  // fragment groups (1 KiB = 64 lanes x 4 k-steps) per matrix
  static constexpr int G_TE = NT * KG, G_IN = NQ * KG, G_O = NT * KG, G_F1 = 4 * KG, G_F2 = NT * KGF,
                       G_F2T = 4 * KG, G_F1T = NT * KGF, G_INT = NT * KGQ, G_OT = NT * KG;
  // per-layer block order: IN O F1 F2 F2T F1T INT OT (forward | ffn backward | attention backward)
  static constexpr int LG = G_IN + G_O + G_F1 + G_F2 + G_F2T + G_F1T + G_INT + G_OT;
  static constexpr long OFF_IN = 0, OFF_O = OFF_IN + G_IN * 256L, OFF_F1 = OFF_O + G_O * 256L,
                        OFF_F2 = OFF_F1 + G_F1 * 256L, OFF_F2T = OFF_F2 + G_F2 * 256L,
                        OFF_F1T = OFF_F2T + G_F2T * 256L, OFF_INT = OFF_F1T + G_F1T * 256L,
                        OFF_OT = OFF_INT + G_INT * 256L;
  static constexpr long TE_OFF = 0;
  static constexpr long layer_off(int l) { return (G_TE + (long)l * LG) * 256L; }
  static constexpr long FP32_FLOATS = (G_TE + 2L * LG) * 256L;
  // Split-bf16 planes (SPLIT, H = 50): the feed-forward matrices F1 F2 F2T F1T
  // and out_proj's transpose OT of each layer also as exact three-part bf16 splits (pgp_device.hpp split8)
  // for v_mfma_f32_16x16x32_bf16: a 32-k block b pairs fragment groups 2b, 2b + 1
  // lane-locally (element e of a lane's 8 <-> k-step 8b + e), 1-KiB fragments
  // [tile][block][plane], after the fp32 fragments in the same buffer
  static constexpr bool SPLIT = PGP_TF_SPLIT && H == 50;
  static constexpr int NBD = (KS + 7) / 8;  // 32-k blocks over d
  static constexpr int NBH = 2;             // over the hidden 64
  static constexpr int P_F1 = 4 * NBD * 3, P_F2 = NT * NBH * 3, P_F2T = 4 * NBD * 3, P_F1T = NT * NBH * 3,
                       P_OT = NT * NBD * 3;
  static constexpr int PL = P_F1 + P_F2 + P_F2T + P_F1T + P_OT;  // per layer
  static constexpr int PO_OT = P_F1 + P_F2 + P_F2T + P_F1T;      // OT's first fragment in the layer block
  static constexpr long pl_off(int l) { return FP32_FLOATS + (long)l * PL * 256L; }
  static constexpr long TRIPLES = SPLIT ? 2L * PL / 3 : 0;
  static constexpr long TOTAL_FLOATS = FP32_FLOATS + TRIPLES * 768L;
  static constexpr long PACK_ITEMS = FP32_FLOATS + TRIPLES * 64L;  // tf_pack_elem's index range
  static constexpr int mat_kg(int m) {
    return m == TFM_F2 || m == TFM_F1T ? KGF : m == TFM_INT ? KGQ : KG;
  }
  __host__ __device__ static void locate(long grp, int& layer, int& mat, long& gi) {
    if (grp < G_TE) {
      layer = -1;
      mat = TFM_TE;
      gi = grp;
      return;
    }
    long r = grp - G_TE;
    layer = (int)(r / LG);
    r -= (long)layer * LG;
    const int cnt[8] = {G_IN, G_O, G_F1, G_F2, G_F2T, G_F1T, G_INT, G_OT};
    const int ids[8] = {TFM_IN, TFM_O, TFM_F1, TFM_F2, TFM_F2T, TFM_F1T, TFM_INT, TFM_OT};
    int k = 0;
    while (k < 7 && r >= cnt[k]) r -= cnt[k++];
    mat = ids[k];
    gi = r;
  }
};

// arguments of the fused kernels (unused pointers may be null); every [M][*]
// buffer a fused kernel writes has a spare row M (lanes outside the batch)
struct TfArgs {
  int layer, B;
  const float* P;      // master weights (natural blob)
  float* frags;        // packed fragments [TE][layer 0][layer 1] (tf_frag_floats)
  const float* in;     // fwd: layer input (layer 0: GAT output); ffn bwd: dOut; att bwd: dR1   [M][DP]
  float* out;          // fwd: layer output; ffn bwd: dR1; att bwd: dX                          [M][DP]
  float* x0;           // fwd layer 0: X0 (time-encoder output)                                  [M][DP]
  const float* x;      // att bwd: the layer input X                                             [M][DP]
  float* xh1;          // norm1 x-hat [M][DP] (fwd writes, ffn bwd reads)
  float* rs1;          // norm1 rstd [M]
  float* dqkv;         // att bwd: dQKV [M][3][DP] (q | k | v, each zero-padded)
  float* part;         // bwd: one weight-gradient slab per workgroup
};

#ifdef __HIPCC__
// fragment group of matrix `mat`: float offset ((tile * KG + q) * 64 + lane) * 4 + e
// holds A[i = lane & 15][k = lane >> 4] of k-step 4q + e of output tile `tile`
template <int H>
PGP_DEV float tf_frag_value(const float* __restrict__ P, int layer, int mat, int tile, int ks, int lane) {
  using F = TF<H>;
  using G = TGeo<H>;
  const int i = lane & 15, g = lane >> 4;
  const float* L = P + G::LAY0 + (long)layer * G::L_SIZE;
  auto dfeat = [&](int s) { return 16 * (s >> 2) + 4 * g + (s & 3); };  // d-space k-step -> feature
  switch (mat) {
    case TFM_TE: {  // out d, in d
      if (ks >= F::KS) return 0.f;
      const int n = 16 * tile + i, c = dfeat(ks);
      return (n < H && c < H) ? P[G::W_TE + n * H + c] : 0.f;
    }
    case TFM_IN: {  // out q|k|v tiles, in d
      if (ks >= F::KS) return 0.f;
      const int part = tile / F::NT, n = 16 * (tile - part * F::NT) + i, c = dfeat(ks);
      return (n < H && c < H) ? L[G::L_IN + (long)(part * H + n) * H + c] : 0.f;
    }
    case TFM_O: {  // out d, in d
      if (ks >= F::KS) return 0.f;
      const int n = 16 * tile + i, c = dfeat(ks);
      return (n < H && c < H) ? L[G::L_OUT + n * H + c] : 0.f;
    }
    case TFM_F1: {  // out hidden, in d
      if (ks >= F::KS) return 0.f;
      const int u = 16 * tile + i, c = dfeat(ks);
      return c < H ? L[G::L_W1 + u * H + c] : 0.f;
    }
    case TFM_F2: {  // out d, in hidden
      const int n = 16 * tile + i, u = dfeat(ks);
      return n < H ? L[G::L_W2 + n * 64 + u] : 0.f;
    }
    case TFM_F2T: {  // out hidden, in d: W2^T
      if (ks >= F::KS) return 0.f;
      const int u = 16 * tile + i, n = dfeat(ks);
      return n < H ? L[G::L_W2 + n * 64 + u] : 0.f;
    }
    case TFM_F1T: {  // out d, in hidden: W1^T
      const int c = 16 * tile + i, u = dfeat(ks);
      return c < H ? L[G::L_W1 + u * H + c] : 0.f;
    }
    case TFM_INT: {  // out d, in q|k|v rows: Win^T
      if (ks >= F::KSQ) return 0.f;
      const int part = ks / F::KS, s = ks - part * F::KS, n = dfeat(s), c = 16 * tile + i;
      return (n < H && c < H) ? L[G::L_IN + (long)(part * H + n) * H + c] : 0.f;
    }
    case TFM_OT: {  // out d (attention output feature), in d (dR1 feature): Wo^T
      if (ks >= F::KS) return 0.f;
      const int c = 16 * tile + i, n = dfeat(ks);
      return (n < H && c < H) ? L[G::L_OUT + n * H + c] : 0.f;
    }
  }
  return 0.f;
}

// one plane triple (SPLIT): item = triple * 64 + lane; the lane's 8 values of
// fragment groups 2b, 2b + 1 split into three bf16 planes (u32x4 each)
template <int H>
PGP_DEV void tf_split_item(const float* __restrict__ P, float* __restrict__ frags, long item) {
  using F = TF<H>;
  const int lane = (int)(item & 63);
  const long tr = item >> 6;
  const int layer = (int)(tr / (F::PL / 3));
  int t = (int)(tr - (long)layer * (F::PL / 3));
  const int cnt[5] = {F::P_F1 / 3, F::P_F2 / 3, F::P_F2T / 3, F::P_F1T / 3, F::P_OT / 3};
  const int mats[5] = {TFM_F1, TFM_F2, TFM_F2T, TFM_F1T, TFM_OT};
  const int nbs[5] = {F::NBD, F::NBH, F::NBD, F::NBH, F::NBD};
  int k = 0;
  while (k < 4 && t >= cnt[k]) t -= cnt[k++];
  const int tile = t / nbs[k], b = t - tile * nbs[k];
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = tf_frag_value<H>(P, layer, mats[k], tile, 8 * b + e, lane);
  u32x4 pl[3];
  split8(v, pl);
  u32x4* dst = reinterpret_cast<u32x4*>(frags + F::FP32_FLOATS + tr * 768L) + lane;
#pragma unroll
  for (int q = 0; q < 3; ++q) dst[q * 64] = pl[q];
}

// one element of the fragment buffer (tf_pack_kernel; the C3 step's merged
// packing launch in pgp_tune.hip); indices past the fp32 fragments are plane
// triple items (tf_split_item)
template <int H>
PGP_DEV void tf_pack_elem(const float* __restrict__ P, float* __restrict__ frags, long idx) {
  using F = TF<H>;
  if (idx >= F::PACK_ITEMS) return;
  if (idx >= F::FP32_FLOATS) {
    if constexpr (F::SPLIT) tf_split_item<H>(P, frags, idx - F::FP32_FLOATS);
    return;
  }
  const int e = (int)(idx & 3), lane = (int)((idx >> 2) & 63);
  const long grp = idx >> 8;  // 1-KiB group
  int layer, mat;
  long gi;
  F::locate(grp, layer, mat, gi);
  const int kg = F::mat_kg(mat);
  const int tile = (int)(gi / kg), q = (int)(gi - (long)tile * kg);
  frags[idx] = tf_frag_value<H>(P, layer < 0 ? 0 : layer, mat, tile, 4 * q + e, lane);
}
#endif

long tf_frag_floats(int H);
long tf_pack_items(int H);  // tf_pack_elem's index range (>= tf_frag_floats' fp32 part)
long tf_slab_floats(int H, int kind);  // kind 2: ffn backward, 3: attention backward
int tf_max_grid();                      // the most workgroups a fused launch uses (one per CU)
int tf_bwd_grid(int H, int B);          // workgroups (= weight-gradient slabs) of a backward launch
void tf_reserve_cus(int n);             // CUs the fused launches leave to other streams
// kind 0: pack fragments from P; 1: forward of a.layer; 2: ffn backward; 3: attention backward
// stop != nullptr: the launch signals that event at its end (hipExtLaunchKernel)
hipError_t launch_tf(int H, int kind, const TfArgs& a, hipStream_t st, hipEvent_t stop = nullptr);

}  // namespace pgp
