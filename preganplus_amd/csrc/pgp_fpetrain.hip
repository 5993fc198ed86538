// pgp_fpetrain.hip — offline training of PreGAN's FPE_16 encoder
// (PreGAN.py:26-27, 39-49: a new FPE is trained for num_epochs when no
// checkpoint exists; train.py:42-57 backprop, sequential batch-1 steps).
//
// fpe_step_kernel: ONE window per workgroup (256 threads), the whole step:
//   forward of FPE_16 (models.py:65-115) from the natural fp32 master P —
//     GRU(48 -> 3) over the 3 window rows from the given h0 (the reference
//     draws it with torch.randn inside encode, models.py:70; the host draws it
//     the same way and passes it in), GAT on each row (16 nodes, graph-wise
//     edge softmax, node mean), concat, MultiheadAttention(19, 1 head) over
//     the 3 rows, encoder Linear(57 -> 160) (LeakyReLU(True) = identity),
//     per host Softmax(Linear(10, 2)) and Sigmoid(Linear(10, 2));
//   custom_loss / triplet_loss bookkeeping of the window on the device state
//     (pgp_tunetargets.hpp, fp64, the reference's order; the anomaly decoder
//     ends in a Softmax, so CrossEntropyLoss sees probabilities);
//   the backward of aloss + tloss into G (every element written).
// With train = 0 the kernel stops after the forward and writes the window's
// probabilities / prototypes (fp64), one workgroup per window: accuracy()'s
// forwards (train.py:94-109) after an epoch.
// The model is tiny (11,401 parameters, ~10^5 MACs per window): every phase is
// a few hundred independent dot products over LDS-resident activations, so
// one workgroup per step is latency-bound by construction; the step count
// (windows x epochs) is what the offline training costs.
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_tunetargets.hpp"

namespace pgp {
namespace {

// natural parameter blob (state_dict order, weights.fpe_shapes)
struct FP {
  static constexpr int H = 16, F = 48, W = 3, G3 = 9, E = 19, L = 10, D = 16, Q = 3 * E, NL = H * L, NF = W * E;
  static constexpr int IH = 0, HH = IH + G3 * F, BIH = HH + G3 * 3, BHH = BIH + G3, FC = BHH + G3, ATT = FC + D * 3,
                       IN = ATT + 2 * D, INB = IN + Q * E, OUT = INB + Q, OUTB = OUT + E * E, ENC = OUTB + E,
                       ENCB = ENC + NL * NF, AN = ENCB + NL, ANB = AN + 2 * L, PR = ANB + 2, PRB = PR + 2 * L,
                       SIZE = PRB + 2;
};
static_assert(FP::SIZE == 11401, "FPE_16 parameter count");

constexpr int kFT = 256;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ __launch_bounds__(kFT) void fpe_step_kernel(int train, int K, const float* __restrict__ wins,
                                                       const float* __restrict__ h0s, const int* __restrict__ ys,
                                                       const int* __restrict__ clss, const float* __restrict__ P,
                                                       float* __restrict__ G, double* __restrict__ state,
                                                       double update_min, double decay, double* __restrict__ loss,
                                                       double* __restrict__ probs_out, double* __restrict__ protos_out) {
  using C = FP;
  constexpr int H = C::H, W = C::W, E = C::E, D = C::D, L = C::L;
  const int t = threadIdx.x;
  const int b = blockIdx.x;  // window (forward-only launches: one per window; training: 0)
  __shared__ float x[W][C::F];
  __shared__ float hs[W + 1][3];           // GRU states h_0 .. h_3
  __shared__ float gi[W][9], gh[W][9], gr[W][3], gz[W][3], gn[W][3];
  __shared__ float z[W][H][D + 1];         // GAT fc outputs
  __shared__ float sv[W][H], tv[W][H];     // attention halves a1.z_i, a2.z_j
  __shared__ float al[W][H][H + 1];        // edge softmax
  __shared__ float red[W][H];
  __shared__ float mx[W], sm[W];
  __shared__ float c[W][E];                // concat
  __shared__ float qkv[W][C::Q];
  __shared__ float pa[W][W];               // attention probabilities
  __shared__ float ao[W][E];               // attention output before out_proj
  __shared__ float fl[C::NF];              // out_proj output, flattened
  __shared__ float lat[C::NL];
  __shared__ float pr[H][2], an[H][2];     // prototypes (sigmoid), anomaly probs
  // backward
  __shared__ float mult[H], tgt[H][2];
  __shared__ double lsum[2];
  __shared__ float dan[H][2], dpr[H][2];
  __shared__ float dlat[C::NL];
  __shared__ float dfl[C::NF];
  __shared__ float dao[W][E], dP[W][W], dS[W][W];
  __shared__ float dqkv[W][C::Q];
  __shared__ float dc[W][E];
  __shared__ float dh[W + 1][3];
  __shared__ float dgi[W][9], dgh[W][9];
  __shared__ float dz[W][H][D + 1];
  __shared__ float dal[W][H][H + 1];
  __shared__ float dsv[W][H], dtv[W][H];

  const float* win = wins + (long)b * W * C::F;
  for (int k = t; k < W * C::F; k += kFT) x[k / C::F][k % C::F] = win[k];
  if (t < 3) hs[0][t] = h0s[(long)b * 3 + t];
  __syncthreads();

  // ---- GRU (torch gate order r, z, n), one row at a time ----
  for (int w = 0; w < W; ++w) {
    if (t < 9) {
      float a = P[C::BIH + t];
      for (int k = 0; k < C::F; ++k) a = fmaf(P[C::IH + t * C::F + k], x[w][k], a);
      gi[w][t] = a;
    } else if (t < 18) {
      const int o = t - 9;
      float a = P[C::BHH + o];
      for (int k = 0; k < 3; ++k) a = fmaf(P[C::HH + o * 3 + k], hs[w][k], a);
      gh[w][o] = a;
    }
    __syncthreads();
    if (t < 3) {
      const float r = sigm(gi[w][t] + gh[w][t]);
      const float zz = sigm(gi[w][3 + t] + gh[w][3 + t]);
      const float n = tanhf(gi[w][6 + t] + r * gh[w][6 + t]);
      gr[w][t] = r;
      gz[w][t] = zz;
      gn[w][t] = n;
      hs[w + 1][t] = (1.f - zz) * n + zz * hs[w][t];
    }
    __syncthreads();
  }

  // ---- GAT on every row (dlutils.py:304-348), node mean ----
  for (int k = t; k < W * H * D; k += kFT) {  // z = fc x
    const int w = k / (H * D), i = (k / D) % H, d = k % D;
    const float* fc = P + C::FC + d * 3;
    z[w][i][d] = fc[0] * x[w][3 * i] + fc[1] * x[w][3 * i + 1] + fc[2] * x[w][3 * i + 2];
  }
  __syncthreads();
  if (t < 2 * W * H) {
    const int half = t / (W * H), w = (t / H) % W, i = t % H;
    const float* a = P + C::ATT + half * D;
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(a[d], z[w][i][d], s);
    (half ? tv : sv)[w][i] = s;
  }
  __syncthreads();
  for (int k = t; k < W * H * H; k += kFT) {  // e_ij = lrelu(a1.z_i + a2.z_j), src i -> dst j
    const int w = k / (H * H), i = (k / H) % H, j = k % H;
    const float e = sv[w][i] + tv[w][j];
    al[w][i][j] = e > 0.f ? e : 0.01f * e;
  }
  __syncthreads();
  if (t < W * H) {  // softmax over all H^2 edges of the row's graph: max, then sum
    const int w = t / H, i = t % H;
    float m = -INFINITY;
    for (int j = 0; j < H; ++j) m = fmaxf(m, al[w][i][j]);
    red[w][i] = m;
  }
  __syncthreads();
  if (t < W) {
    float m = -INFINITY;
    for (int i = 0; i < H; ++i) m = fmaxf(m, red[t][i]);
    mx[t] = m;
  }
  __syncthreads();
  for (int k = t; k < W * H * H; k += kFT) {
    const int w = k / (H * H), i = (k / H) % H, j = k % H;
    al[w][i][j] = expf(al[w][i][j] - mx[w]);
  }
  __syncthreads();
  if (t < W * H) {
    const int w = t / H, i = t % H;
    float s = 0.f;
    for (int j = 0; j < H; ++j) s += al[w][i][j];
    red[w][i] = s;
  }
  __syncthreads();
  if (t < W) {
    float s = 0.f;
    for (int i = 0; i < H; ++i) s += red[t][i];
    sm[t] = s;
  }
  __syncthreads();
  for (int k = t; k < W * H * H; k += kFT) {
    const int w = k / (H * H), i = (k / H) % H, j = k % H;
    al[w][i][j] = al[w][i][j] / sm[w];
  }
  __syncthreads();
  if (t < W * H) {  // column weight of source i: sum_j a_ij
    const int w = t / H, i = t % H;
    float s = 0.f;
    for (int j = 0; j < H; ++j) s += al[w][i][j];
    red[w][i] = s;
  }
  __syncthreads();
  if (t < W * D) {  // gat_w[d] = mean_j sum_i a_ij z_i[d] = (1/H) sum_i red_i z_i[d]
    const int w = t / D, d = t % D;
    float s = 0.f;
    for (int i = 0; i < H; ++i) s = fmaf(red[w][i], z[w][i][d], s);
    c[w][3 + d] = s / (float)H;
  } else if (t < W * D + W * 3) {
    const int k = t - W * D, w = k / 3, o = k % 3;
    c[w][o] = hs[w + 1][o];
  }
  __syncthreads();

  // ---- MultiheadAttention(19, 1 head) over the 3 rows ----
  for (int k = t; k < W * C::Q; k += kFT) {
    const int w = k / C::Q, o = k % C::Q;
    float a = P[C::INB + o];
    for (int e = 0; e < E; ++e) a = fmaf(P[C::IN + o * E + e], c[w][e], a);
    qkv[w][o] = a;
  }
  __syncthreads();
  const float isq = 1.0f / sqrtf((float)E);
  if (t < W * W) {
    const int w = t / W, v = t % W;
    float s = 0.f;
    for (int e = 0; e < E; ++e) s = fmaf(qkv[w][e], qkv[v][E + e], s);
    pa[w][v] = s * isq;
  }
  __syncthreads();
  if (t < W) {
    const float m = fmaxf(pa[t][0], fmaxf(pa[t][1], pa[t][2]));
    const float e0 = expf(pa[t][0] - m), e1 = expf(pa[t][1] - m), e2 = expf(pa[t][2] - m);
    const float s = e0 + e1 + e2;
    pa[t][0] = e0 / s;
    pa[t][1] = e1 / s;
    pa[t][2] = e2 / s;
  }
  __syncthreads();
  if (t < W * E) {
    const int w = t / E, e = t % E;
    ao[w][e] = pa[w][0] * qkv[0][2 * E + e] + pa[w][1] * qkv[1][2 * E + e] + pa[w][2] * qkv[2][2 * E + e];
  }
  __syncthreads();
  if (t < W * E) {
    const int w = t / E, o = t % E;
    float a = P[C::OUTB + o];
    for (int e = 0; e < E; ++e) a = fmaf(P[C::OUT + o * E + e], ao[w][e], a);
    fl[w * E + o] = a;
  }
  __syncthreads();
  // ---- encoder Linear(57 -> 160) ----
  if (t < C::NL) {
    float a = P[C::ENCB + t];
    for (int k = 0; k < C::NF; ++k) a = fmaf(P[C::ENC + t * C::NF + k], fl[k], a);
    lat[t] = a;
  }
  __syncthreads();
  // ---- per-host decoders ----
  if (t < 4 * H) {
    const int h = t >> 2, which = (t >> 1) & 1, o = t & 1;
    const float* Wd = P + (which ? C::PR : C::AN) + o * L;
    float a = P[(which ? C::PRB : C::ANB) + o];
    for (int l = 0; l < L; ++l) a = fmaf(Wd[l], lat[h * L + l], a);
    (which ? pr : an)[h][o] = a;
  }
  __syncthreads();
  if (t < H) {
    const float a0 = an[t][0], a1 = an[t][1], m = fmaxf(a0, a1);
    const float e0 = expf(a0 - m), e1 = expf(a1 - m);
    an[t][0] = e0 / (e0 + e1);
    an[t][1] = e1 / (e0 + e1);
    pr[t][0] = sigm(pr[t][0]);
    pr[t][1] = sigm(pr[t][1]);
  }
  __syncthreads();
  if (!train) {
    if (t < 2 * H) {
      probs_out[(long)b * 2 * H + t] = (double)an[t >> 1][t & 1];
      protos_out[(long)b * 2 * H + t] = (double)pr[t >> 1][t & 1];
    }
    return;
  }

  // ---- custom_loss / triplet_loss bookkeeping (fp64, sequential, one lane) ----
  if (t == 0) {
    double ls[2];
    tune_targets_one(H, K, &an[0][0], &pr[0][0], ys, clss, state, update_min, decay, mult, &tgt[0][0], ls);
    lsum[0] = ls[0];
    lsum[1] = ls[1];
    loss[0] = ls[0];
    loss[1] = ls[1];
  }
  __syncthreads();

  // ---- loss gradients at the decoder outputs ----
  if (t < H) {
    // aloss: mult * CrossEntropy(probs as logits, y): d/dp = mult (softmax(p) - e_y);
    // through the decoder's Softmax: da = p (dp - p . dp)
    const int y = ys[t];
    const float p0 = an[t][0], p1 = an[t][1], m = fmaxf(p0, p1);
    const float e0 = expf(p0 - m), e1 = expf(p1 - m);
    const float q0 = e0 / (e0 + e1), q1 = e1 / (e0 + e1);
    const float dp0 = mult[t] * (q0 - (y == 0 ? 1.f : 0.f)), dp1 = mult[t] * (q1 - (y == 1 ? 1.f : 0.f));
    const float s = p0 * dp0 + p1 * dp1;
    dan[t][0] = p0 * (dp0 - s);
    dan[t][1] = p1 * (dp1 - s);
    // tloss: MSE(anchor, P[c]) over 2 values (negatives are constants): d = (a - P[c]); through the Sigmoid
    const bool pos = y > 0;
    const float a0 = pr[t][0], a1 = pr[t][1];
    dpr[t][0] = pos ? (a0 - tgt[t][0]) * a0 * (1.f - a0) : 0.f;
    dpr[t][1] = pos ? (a1 - tgt[t][1]) * a1 * (1.f - a1) : 0.f;
  }
  __syncthreads();
  // decoder weight gradients (sum over hosts) and d latent
  if (t < 2 * 2 * (L + 1)) {
    const int which = t / (2 * (L + 1)), o = (t / (L + 1)) % 2, l = t % (L + 1);
    float s = 0.f;
    for (int h = 0; h < H; ++h) {
      const float d = which ? dpr[h][o] : dan[h][o];
      s = fmaf(d, l < L ? lat[h * L + l] : 1.f, s);
    }
    if (l < L)
      G[(which ? C::PR : C::AN) + o * L + l] = s;
    else
      G[(which ? C::PRB : C::ANB) + o] = s;
  }
  if (t < C::NL) {
    const int h = t / L, l = t % L;
    dlat[t] = P[C::AN + l] * dan[h][0] + P[C::AN + L + l] * dan[h][1] + P[C::PR + l] * dpr[h][0] +
              P[C::PR + L + l] * dpr[h][1];
  }
  __syncthreads();
  // encoder
  for (int k = t; k < C::NL * C::NF; k += kFT) G[C::ENC + k] = dlat[k / C::NF] * fl[k % C::NF];
  if (t < C::NL) G[C::ENCB + t] = dlat[t];
  if (t < C::NF) {
    float s = 0.f;
    for (int r = 0; r < C::NL; ++r) s = fmaf(P[C::ENC + r * C::NF + t], dlat[r], s);
    dfl[t] = s;
  }
  __syncthreads();
  // out_proj: d ao = Wo^T d out; dWo = sum_w d out_w ao_w^T
  for (int k = t; k < E * E; k += kFT) {
    const int o = k / E, e = k % E;
    G[C::OUT + k] = dfl[o] * ao[0][e] + dfl[E + o] * ao[1][e] + dfl[2 * E + o] * ao[2][e];
  }
  if (t < E) G[C::OUTB + t] = dfl[t] + dfl[E + t] + dfl[2 * E + t];
  if (t < W * E) {
    const int w = t / E, e = t % E;
    float s = 0.f;
    for (int o = 0; o < E; ++o) s = fmaf(P[C::OUT + o * E + e], dfl[w * E + o], s);
    dao[w][e] = s;
  }
  __syncthreads();
  // attention: dP[w][v] = dao_w . v_v; dv_v = sum_w P[w][v] dao_w
  if (t < W * W) {
    const int w = t / W, v = t % W;
    float s = 0.f;
    for (int e = 0; e < E; ++e) s = fmaf(dao[w][e], qkv[v][2 * E + e], s);
    dP[w][v] = s;
  }
  if (t >= 64 && t < 64 + W * E) {
    const int k = t - 64, v = k / E, e = k % E;
    dqkv[v][2 * E + e] = pa[0][v] * dao[0][e] + pa[1][v] * dao[1][e] + pa[2][v] * dao[2][e];
  }
  __syncthreads();
  if (t < W) {  // softmax backward per query row, then the 1/sqrt(E) scale
    const float s = pa[t][0] * dP[t][0] + pa[t][1] * dP[t][1] + pa[t][2] * dP[t][2];
    for (int v = 0; v < W; ++v) dS[t][v] = pa[t][v] * (dP[t][v] - s) * isq;
  }
  __syncthreads();
  if (t < 2 * W * E) {  // dq_w = sum_v dS[w][v] k_v; dk_v = sum_w dS[w][v] q_w
    const int part = t / (W * E), w = (t / E) % W, e = t % E;
    if (part == 0)
      dqkv[w][e] = dS[w][0] * qkv[0][E + e] + dS[w][1] * qkv[1][E + e] + dS[w][2] * qkv[2][E + e];
    else
      dqkv[w][E + e] = dS[0][w] * qkv[0][e] + dS[1][w] * qkv[1][e] + dS[2][w] * qkv[2][e];
  }
  __syncthreads();
  // in_proj: dWin = sum_w dqkv_w c_w^T, dc_w = Win^T dqkv_w
  for (int k = t; k < C::Q * E; k += kFT) {
    const int o = k / E, e = k % E;
    G[C::IN + k] = dqkv[0][o] * c[0][e] + dqkv[1][o] * c[1][e] + dqkv[2][o] * c[2][e];
  }
  if (t < C::Q) G[C::INB + t] = dqkv[0][t] + dqkv[1][t] + dqkv[2][t];
  if (t >= 64 && t < 64 + W * E) {
    const int k = t - 64, w = k / E, e = k % E;
    float s = 0.f;
    for (int o = 0; o < C::Q; ++o) s = fmaf(P[C::IN + o * E + e], dqkv[w][o], s);
    dc[w][e] = s;
  }
  __syncthreads();

  // ---- GRU backward through the rows (h0 gets no gradient) ----
  if (t < 3) dh[W][t] = 0.f;
  __syncthreads();
  for (int w = W - 1; w >= 0; --w) {
    if (t < 3) {
      const float d = dh[w + 1][t] + dc[w][t];   // grad of h_{w+1}
      const float r = gr[w][t], zz = gz[w][t], n = gn[w][t];
      const float dn = d * (1.f - zz), dzz = d * (hs[w][t] - n);
      const float dan_ = dn * (1.f - n * n);
      const float dr = dan_ * gh[w][6 + t];
      const float dar = dr * r * (1.f - r), daz = dzz * zz * (1.f - zz);
      dgi[w][t] = dar;
      dgi[w][3 + t] = daz;
      dgi[w][6 + t] = dan_;
      dgh[w][t] = dar;
      dgh[w][3 + t] = daz;
      dgh[w][6 + t] = dan_ * r;
      dh[w][t] = d * zz;   // + Whh^T dgh below
    }
    __syncthreads();
    if (t < 3) {
      float s = dh[w][t];
      for (int o = 0; o < 9; ++o) s = fmaf(P[C::HH + o * 3 + t], dgh[w][o], s);
      dh[w][t] = s;
    }
    __syncthreads();
  }
  for (int k = t; k < 9 * C::F; k += kFT) {
    const int o = k / C::F, f = k % C::F;
    G[C::IH + k] = dgi[0][o] * x[0][f] + dgi[1][o] * x[1][f] + dgi[2][o] * x[2][f];
  }
  if (t < 27) {
    const int o = t / 3, k = t % 3;
    G[C::HH + t] = dgh[0][o] * hs[0][k] + dgh[1][o] * hs[1][k] + dgh[2][o] * hs[2][k];
  } else if (t >= 32 && t < 41) {
    const int o = t - 32;
    G[C::BIH + o] = dgi[0][o] + dgi[1][o] + dgi[2][o];
    G[C::BHH + o] = dgh[0][o] + dgh[1][o] + dgh[2][o];
  }

  // ---- GAT backward: gat_w = (1/H) sum_i (sum_j a_ij) z_i ----
  // d a_ij = (1/H) z_i . dgat_w; d z_i = (1/H)(sum_j a_ij) dgat_w (+ the score terms)
  for (int k = t; k < W * H * H; k += kFT) {
    const int w = k / (H * H), i = (k / H) % H, j = k % H;
    float s = 0.f;
    for (int d = 0; d < D; ++d) s = fmaf(z[w][i][d], dc[w][3 + d], s);
    dal[w][i][j] = s / (float)H;   // independent of j
  }
  __syncthreads();
  if (t < W) {  // sum over edges of a . da
    float s = 0.f;
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < H; ++j) s = fmaf(al[t][i][j], dal[t][i][j], s);
    sm[t] = s;
  }
  __syncthreads();
  for (int k = t; k < W * H * H; k += kFT) {  // softmax backward, then the LeakyReLU
    const int w = k / (H * H), i = (k / H) % H, j = k % H;
    const float de = al[w][i][j] * (dal[w][i][j] - sm[w]);
    const float e = sv[w][i] + tv[w][j];
    dal[w][i][j] = e > 0.f ? de : 0.01f * de;
  }
  __syncthreads();
  if (t < 2 * W * H) {  // d s_i = sum_j de_ij, d t_j = sum_i de_ij
    const int half = t / (W * H), w = (t / H) % W, i = t % H;
    float s = 0.f;
    for (int k = 0; k < H; ++k) s += half ? dal[w][k][i] : dal[w][i][k];
    (half ? dtv : dsv)[w][i] = s;
  }
  __syncthreads();
  for (int k = t; k < W * H * D; k += kFT) {
    const int w = k / (H * D), i = (k / D) % H, d = k % D;
    dz[w][i][d] = red[w][i] / (float)H * dc[w][3 + d] + dsv[w][i] * P[C::ATT + d] + dtv[w][i] * P[C::ATT + D + d];
  }
  if (t < 2 * D) {  // attn_fc: sum over rows and nodes of (d s_i) z_i | (d t_j) z_j
    const int half = t / D, d = t % D;
    float s = 0.f;
    for (int w = 0; w < W; ++w)
      for (int i = 0; i < H; ++i) s = fmaf(half ? dtv[w][i] : dsv[w][i], z[w][i][d], s);
    G[C::ATT + t] = s;
  }
  __syncthreads();
  if (t < D * 3) {  // fc: sum over rows and nodes of dz_i x_i^T
    const int d = t / 3, f = t % 3;
    float s = 0.f;
    for (int w = 0; w < W; ++w)
      for (int i = 0; i < H; ++i) s = fmaf(dz[w][i][d], x[w][3 * i + f], s);
    G[C::FC + t] = s;
  }
}

}  // namespace

int fpe_param_count() { return FP::SIZE; }

hipError_t launch_fpe_step(const float* win, const float* h0, const int* y, const int* cls, const float* P, float* G,
                           int K, double* state, double update_min, double decay, double* loss, hipStream_t st) {
  fpe_step_kernel<<<1, kFT, 0, st>>>(1, K, win, h0, y, cls, P, G, state, update_min, decay, loss, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_fpe_forward_many(int n, const float* wins, const float* h0s, const float* P, double* probs,
                                   double* protos, hipStream_t st) {
  fpe_step_kernel<<<n, kFT, 0, st>>>(0, 3, wins, h0s, nullptr, nullptr, P, nullptr, nullptr, 0.0, 0.0, nullptr, probs,
                                     protos);
  return hipGetLastError();
}

}  // namespace pgp
