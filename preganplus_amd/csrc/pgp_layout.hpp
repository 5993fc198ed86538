// pgp_layout.hpp — compile-time geometry of the PreGAN+ kernels for H hosts,
// shared by the host-side packer (pgp_pack.cpp) and the gfx950 kernels.
//
// Execution layout: every kernel runs "windows on lanes".
// One wave owns 16 windows.  Activations are kept as the accumulators of
// v_mfma_f32_16x16x4_f32 with the TOKEN (window) on the lane column j = lane&15
// and FEATURES on the rows: lane group g = lane>>4, register r hold row
// 16*t + 4*g + r of tile t.  Such an accumulator register is directly the B
// operand of the next GEMM's k-step (t, r): lane group g supplies k-row
// 16t+4g+r.  Weights are the A operand, pre-packed into per-lane fragments.
//
// Row <-> feature maps (all chosen so padding sits in whole k-steps):
//   d-space (X, residual stream), feature c:  X row (t,g,r)  <-> c = 16t+4r+g
//     consumed as B: k-step s, group g  <-> c = 4s+g   (KS_D = ceil(H/4) steps)
//   head space, HP >= 16 (per head block of HP rows): same formula with the
//     head dim e in place of c; P8 mode (head dim <= 8, H <= 16): one tile holds
//     both heads, row (g,r) <-> head g>>1, dim 4(g&1)+r.
//   FFN hidden (64) and GAN hidden (64): natural rows u = 16t+4g+r.
//   decoder outputs: row n = 4*host + q, q = {logit0, logit1, proto0, proto1}.
#pragma once
#include <cstddef>

// host counts compiled into the library (d_model = H split over 2 heads: H even)
#define PGP_FOR_EACH_H(X) X(8) X(16) X(32) X(50) X(64)

namespace pgp {

constexpr int round_up(int x, int m) { return (x + m - 1) / m * m; }
constexpr int cdiv(int x, int m) { return (x + m - 1) / m; }

constexpr int kWindow = 3;     // models.py:320
constexpr int kFeat = 3;       // models.py:321
constexpr int kFF = 64;        // models.py:325
constexpr int kLayers = 2;     // models.py:326
constexpr int kGanHidden = 64; // models.py:124,142
constexpr int kProtoDim = 2;   // constants.py:12
constexpr int kFrag = 64;      // floats per MFMA A fragment (one per lane)

template <int H>
struct Geo {
  static_assert(H % 2 == 0, "H must be even (2 heads)");
  static constexpr int D = H;                 // d_model
  static constexpr int DP = round_up(H, 16);  // padded d rows
  static constexpr int MT_D = DP / 16;        // d-space M tiles
  static constexpr int KS_D = cdiv(H, 4);     // k-steps over d-space
  static constexpr int KQ_D = cdiv(KS_D, 4);  // float4 groups of k-steps
  static constexpr int HD = H / 2;            // head dim
  static constexpr bool P8 = HD <= 8;
  static constexpr int HP = P8 ? 8 : round_up(HD, 16);
  static constexpr int NPASS = P8 ? 1 : 2;    // attention passes (heads per pass: 2 or 1)
  static constexpr int TP = P8 ? 1 : HP / 16; // tiles per Q/K/V per pass
  static constexpr int KS_O = P8 ? 4 : cdiv(HD, 4);
  static constexpr int KQ_O = cdiv(KS_O, 4);
  static constexpr int MT_F = kFF / 16;       // 4
  static constexpr int KQ_F = kFF / 16;       // 16 k-steps -> 4 groups
  static constexpr int MT_O = cdiv(H, 4);     // decoder output tiles (4H rows)
  static constexpr int LAT = H * kWindow * H; // latent length 3H^2
  // GAN
  static constexpr int C = H;                 // containers (main.py:80)
  static constexpr int H2 = H * H;
  static constexpr int EP = round_up(2 * H, 16);  // padded embedding row
  static constexpr int EQ = EP / 16;
  static constexpr int SQ = cdiv(H2, 16);
  static constexpr int MT_G = kGanHidden / 16;    // 4
  static constexpr int MT_N = cdiv(H, 16);        // Gen2 tiles per container row

  // ---------------- device weight buffer ----------------
  // Fragments are stored as 1-KiB "groups" [..][q][lane][4]: 64 lanes x one
  // float4 = 4 consecutive k-steps of one 16-row tile; a group is one
  // global_load_lds_dwordx4 wave-instruction and one ds_read_b128 per lane.
  static constexpr int FQ = kFrag * 4;  // floats per group
  // ---- tail mode (H = 50): no padded 16-row output tile ----
  // d = 16*MT_X + XR with XR <= 4 and head dim = 16*HF + HT with 16 < 2*HT <= 20.
  // The XR last d-rows (X tile MT_X, register 0, lane groups < XR) are produced
  // by a VALU GEMV + cross-group sum instead of a 16-row MFMA tile; q/k/v of
  // both heads share TQ = 2*HF+1 tiles per pass (head-0 full tiles, head-1 full
  // tiles, one tile holding both tails) and the SR head-1 tail rows that do
  // not fit are VALU rows too.
  static constexpr int HF = HD / 16, HT = HD % 16;
  static constexpr bool TAIL = !P8 && (H % 16) != 0 && (H % 16) <= 4 && 2 * HT > 16 && 2 * HT - 16 <= 4;
  static constexpr int MT_X = TAIL ? H / 16 : MT_D;   // MFMA output tiles of d-space GEMMs
  static constexpr int XR = TAIL ? H % 16 : 0;        // VALU d-rows
  static constexpr int TQ = 2 * HF + 1;               // q (k, v) tiles, tail mode
  static constexpr int SR = TAIL ? 2 * HT - 16 : 0;   // VALU q/k/v rows (head 1)
  static constexpr int KS_OT = 4 * TQ + (SR > 0 ? 1 : 0);
  static constexpr int KQ_OT = cdiv(KS_OT, 4);

  // encoder stream of one layer, in consumption order:
  //   for p: qkv(p) [m][tp][q4], o(p) [mt][q4];  f1 [mt][q4];  f2 [mt][q4]
  //   tail mode: qk [m][t][q4] | v [t][q4], o [mt][q4] | f1 [mt][q4], f2 [mt][q4]
  static constexpr int G_QKV = 3 * TP * KQ_D;
  static constexpr int G_O = MT_D * KQ_O;
  static constexpr int G_F1 = MT_F * KQ_D;
  static constexpr int G_F2 = MT_X * KQ_F;
  static constexpr int G_QK = 2 * TQ * KQ_D;          // tail mode
  static constexpr int G_V = TQ * KQ_D;
  static constexpr int G_OT = MT_X * KQ_OT;
  static constexpr int P_QKV(int p) { return p * (G_QKV + G_O); }
  static constexpr int P_O(int p) { return p * (G_QKV + G_O) + G_QKV; }
  static constexpr int P_V = G_QK;                    // tail mode
  static constexpr int P_OT = G_QK + G_V;
  static constexpr int P_F1 = TAIL ? P_OT + G_OT : NPASS * (G_QKV + G_O);
  static constexpr int P_F2 = P_F1 + G_F1;
  static constexpr int LAYER_G = P_F2 + G_F2;
  // LDS stages of a layer: NPASS=2: [qkv0] [o0 qkv1] [o1 f1] [f2]
  //                        NPASS=1: [qkv0] [o0 f1] [f2]
  //                        tail:    [qk] [v o] [f1 f2]
  static constexpr int NST = TAIL ? 3 : NPASS + 2;
  static constexpr int st_begin(int k) {
    return TAIL ? (k == 0 ? 0 : k == 1 ? P_V : P_F1)
                : NPASS == 2 ? (k == 0 ? 0 : k == 1 ? P_O(0) : k == 2 ? P_O(1) : P_F2)
                             : (k == 0 ? 0 : k == 1 ? P_O(0) : P_F2);
  }
  static constexpr int st_end(int k) { return k + 1 < NST ? st_begin(k + 1) : LAYER_G; }
  static constexpr int max_stage() {
    int m = 0;
    for (int k = 0; k < NST; ++k) m = st_end(k) - st_begin(k) > m ? st_end(k) - st_begin(k) : m;
    return m;
  }
  static constexpr int SLOT_G = max_stage();      // groups per LDS slot (encoder)
  // decoder chunk per (host, step): [mt][q4]
  static constexpr int DEC_G = MT_O * KQ_D;

  static constexpr long OFF_ENC = 0;                                   // [layer][LAYER_G groups]
  static constexpr long OFF_DEC = OFF_ENC + (long)kLayers * LAYER_G * FQ;  // [h][w][DEC_G]
  // GAN (K3) chunks, each contiguous:
  //   emb chunk   [mt][q]  MT_G x EQ groups           (Gen1, embedding columns)
  //   sched q     [q][8]   Gen1 mt0..3 | Disc1 mt0..3 (schedule columns 16q..16q+15)
  //   container c [G2: t][q4] (MT_N x 4) | [D1N: mt][q4] (MT_G x MT_N)
  static constexpr int GE_G = MT_G * EQ;
  static constexpr int GS_G = 2 * MT_G;                       // per schedule q
  static constexpr int GC_G2 = MT_N * 4;
  static constexpr int GC_G = GC_G2 + MT_G * MT_N;            // per container
  static constexpr long OFF_GE = OFF_DEC + (long)H * kWindow * DEC_G * FQ;
  static constexpr long OFF_GS = OFF_GE + (long)GE_G * FQ;
  static constexpr long OFF_GC = OFF_GS + (long)SQ * GS_G * FQ;
  static constexpr long SZ_FRAGS = OFF_GC + (long)C * GC_G * FQ;

  // latent workspace (encoder -> decoder): per 16-window block
  //   [H][3][KS_D][64]: X tile registers as the decoder's B operand
  static constexpr long LAT_BLK = (long)H * kWindow * KS_D * 64;
  // within a (host, step) chunk of KS_D x 64 floats: LAT_FG full groups of 4
  // k-steps stored [group][lane][4] (16 B per lane), then the KS_D - 4 LAT_FG
  // remaining k-steps [k][lane]
  static constexpr int LAT_FG = KS_D / 4;

  // ---------------- encoder/decoder tables (staged into LDS) ----------------
  static constexpr int T_TEW = 0;                   // [MT_D][64] time-encoder A fragments (K=4)
  static constexpr int T_TE = T_TEW + MT_D * 64;    // [3][DP] time-encoder bias + pe[w]
  static constexpr int T_L0 = T_TE + kWindow * DP;
  static constexpr int TL_QKV = 0;                  // [NPASS][3][TP*16]; tail: [3][TQ*16]
  static constexpr int TL_BO = TAIL ? 3 * TQ * 16 : NPASS * 3 * TP * 16;
  static constexpr int TL_LN1G = TL_BO + DP;
  static constexpr int TL_LN1B = TL_LN1G + DP;
  static constexpr int TL_B1 = TL_LN1B + DP;
  static constexpr int TL_B2 = TL_B1 + kFF;
  static constexpr int TL_LN2G = TL_B2 + DP;
  static constexpr int TL_LN2B = TL_LN2G + DP;
  // tail-mode VALU rows: weights [.][n][q4][g][4] (k-step 4*q4+e, lane group g)
  static constexpr int TL_RQ = TL_LN2B + DP;                 // [3][SR][KQ_D][4][4] q/k/v rows
  static constexpr int TL_RQB = TL_RQ + 3 * SR * KQ_D * 16;  // [3*SR] (pad 8) their biases
  static constexpr int TL_RO = TL_RQB + (TAIL ? 8 : 0);      // [XR][KQ_OT][4][4] out_proj rows
  static constexpr int TL_RF = TL_RO + XR * KQ_OT * 16;      // [XR][KQ_F][4][4] linear2 rows
  static constexpr int TL_SIZE = TL_RF + XR * KQ_F * 16;
  // layer 0's q/k/v folded onto the aggregated raw features (X0 is affine in
  // them): one K=4 A fragment per q/k/v output tile (k = raw feature, lane
  // groups 0..2) and per-step biases; tail-mode VALU rows likewise
  static constexpr int NQT = TAIL ? TQ : NPASS * TP;       // tiles per q / k / v
  static constexpr int T_F0 = T_L0 + kLayers * TL_SIZE;    // [3*NQT][64] A fragments
  static constexpr int T_F0B = T_F0 + 3 * NQT * 64;        // [3 steps][3*NQT*16] biases
  static constexpr int T_F0R = T_F0B + 9 * NQT * 16;       // [3][SR][4] VALU-row weights
  static constexpr int T_F0RB = T_F0R + 3 * SR * 4;        // [3 steps][3*SR] VALU-row biases
  // tail mode, layer 0's out_proj folded through the attention (v affine in the
  // raw features too): out = sum_head (Wo Fv) (P x-bar) + (Wo bv_w') P + bo, as
  // K=4 A fragments [head][G|C][MT_X][64] and VALU rows [XR][head][G|C][4]
  static constexpr int T_F0O = T_F0RB + round_up(9 * SR, 4);
  static constexpr int T_F0OR = T_F0O + (TAIL ? 4 * MT_X * 64 : 0);
  // tail mode, layer 0's attention scores as bilinear forms of the raw features
  // (q and k are affine in them): per head [M 3x3 | U 3x3 (f, key step) | V 3x3
  // (query step, f) | S 3x3 (query, key step)], score(w, w2) = x_w^T M x_w2 +
  // x_w . U[:, w2] + V[w] . x_w2 + S[w][w2]
  static constexpr int T_F0S = T_F0OR + (TAIL ? XR * 16 : 0);
  static constexpr int T_DEC = T_F0S + (TAIL ? 72 : 0);     // [MT_O*16] decoder bias
  static constexpr int T_PROTO = T_DEC + MT_O * 16;         // [K][2]
  static constexpr int t_size(int K) { return T_PROTO + round_up(2 * K, 4); }

  // ---------------- GAN tables (global) ----------------
  static constexpr int G_B1 = 0;                  // [64] gen hidden bias
  static constexpr int G_BD1 = G_B1 + 64;         // [64] disc hidden bias
  static constexpr int G_WD2 = G_BD1 + 64;        // [2][64]
  static constexpr int G_BD2 = G_WD2 + 128;       // [4] (2 used)
  static constexpr int G_B2 = G_BD2 + 4;          // [C][MT_N*16] gen output bias
  // + one 1-KiB group of zero padding: K3 copies a ring chunk's biases to LDS
  // as a whole group (global_load_lds), which may run past the last container
  static constexpr int G_SIZE = G_B2 + C * MT_N * 16 + 256;
};

// PreGAN's FPE_16 encoder (models.py:10-115), folded table of K4 (pgp_fpe.hip).
// FPE_16's encode/forward are host-count generic (every shape comes from
// n_hosts); H = 50 is that code at n_hosts = 50 (tests/golden/make_golden_fpe50.py),
// an extrapolation of the FPE_16 architecture: the reference's own FPE_50
// (models.py:156-210) raises in its GAT call (dlutils.py:306).
#define PGP_FOR_EACH_FPE_H(X) X(16) X(50)
template <int H>
struct FpeGeo {
  static constexpr int W = 3;          // window rows = GRU steps = GRU state size
  static constexpr int NIN = 3 * H;    // features per window row
  static constexpr int E = W + H;      // MHA embedding: GRU state ++ GAT node-mean
  static constexpr int KC = W * E;     // flattened attention output (encoder input)
  static constexpr int NO = 4 * H;     // outputs per window: per host {a0, a1, p0, p1}
  static constexpr int K = 3;          // prototypes (models.py:62)
  // The GAT node mean is Wfc (sum_i r_i x_i) / (H Z): rank 3.  So each MHA
  // token c_w = P u_w with u_w = [GRU state (3); node-weighted raw features
  // g_w (3)] and P = blockdiag(I3, Wfc / H): every map after the GAT acts on
  // the 6-vector u_w (pgp_pack.cpp pack_fpe_t).
  static constexpr int U = 6;
  static constexpr int KU = W * U;     // 18: the attention output in u-space
  static constexpr int F_WIH = 0;                                 // [9][NIN] GRU input weights (r,z,n)
  static constexpr int F_WHH = F_WIH + round_up(9 * NIN, 4);      // [9][3]
  static constexpr int F_BRZ = F_WHH + round_up(27, 4);           // [6] b_ih + b_hh for r, z
  static constexpr int F_BIN = F_BRZ + 8;                         // [3] b_ih of n
  static constexpr int F_BHN = F_BIN + 4;                         // [3] b_hh of n
  static constexpr int F_UV = F_BHN + 4;                          // u[3] (+pad), v[3] (+pad), log2e-scaled
  static constexpr int F_M6 = F_UV + 8;                           // [6][6] log2e P^T Wq^T Wk P / sqrt(E)
  static constexpr int F_BETA6 = F_M6 + 36;                       // [6]    log2e P^T Wk^T bq / sqrt(E)
  static constexpr int F_W6 = F_BETA6 + 8;                        // [NO][KU] Dec . Wenc . (Wout Wv P)_s
  static constexpr int F_B2 = F_W6 + round_up(NO * KU, 4);        // [NO]
  static constexpr int F_PROTO = F_B2 + round_up(NO, 4);          // [K][2]
  static constexpr int F_SIZE = F_PROTO + round_up(2 * K, 4);
  static constexpr size_t blob_len() {
    return 9 * NIN + 27 + 9 + 9 + 3 * H + 2 * H + 3 * E * E + 3 * E + E * E + E + (size_t)10 * H * KC + 10 * H +
           20 + 2 + 20 + 2;
  }
};

// GAT constants passed by value: u = Wfc^T a_src, v = Wfc^T a_dst (fp64-composed)
struct GatConst {
  float u[4];
  float v[4];
};

}  // namespace pgp
