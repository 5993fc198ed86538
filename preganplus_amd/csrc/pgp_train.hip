// pgp_train.hip — HIP kernels of the online training steps:
//   * the semi-supervised tuning step (train.py:42-57): forward with saved
//     activations, loss gradient (custom_loss / triplet_loss, train.py:13-40),
//     backward through decoders, 2 encoder layers, time encoder and GAT;
//   * the GAN step (PreGANPlus.py:60-81): Gen/Disc forward, Disc BCE backward,
//     Gen BCE backward through the updated Disc;
//   * batched weight-gradient outer products and AdamW (utils.py:65).
// Correctness-first design: one 256-thread workgroup per window,
// VALU, activations in a per-window global scratch; parameter gradients of the
// small per-token matrices are accumulated with one atomicAdd per element per
// window, the large ones (decoders, Gen, Disc) by dw_outer_kernel over the batch.
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_train.hpp"

namespace pgp {
namespace {

constexpr int kTW = 256;

// Y[m][n] = sum_k X[m*ldx+k] * Wt[n*K+k] + b[n]     (nn.Linear, W row-major [N][K])
__device__ void wg_linear(float* Y, int ldy, const float* X, int ldx, const float* Wt, const float* b, int M,
                          int N, int K) {
  for (int idx = threadIdx.x; idx < M * N; idx += blockDim.x) {
    const int m = idx / N, n = idx - m * N;
    float acc = b ? b[n] : 0.f;
    const float* x = X + (long)m * ldx;
    const float* w = Wt + (long)n * K;
    for (int k = 0; k < K; ++k) acc = fmaf(x[k], w[k], acc);
    Y[(long)m * ldy + n] = acc;
  }
}
// dX[m][k] (+)= sum_n dY[m*ldy+n] * W[n][k]
__device__ void wg_linear_dx(float* dX, int ldd, const float* dY, int ldy, const float* W, int M, int N, int K,
                             bool acc_into) {
  for (int idx = threadIdx.x; idx < M * K; idx += blockDim.x) {
    const int m = idx / K, k = idx - m * K;
    float acc = acc_into ? dX[(long)m * ldd + k] : 0.f;
    const float* dy = dY + (long)m * ldy;
    for (int n = 0; n < N; ++n) acc = fmaf(dy[n], W[(long)n * K + k], acc);
    dX[(long)m * ldd + k] = acc;
  }
}
// dW[n][k] += sum_m dY[m][n] X[m][k];  db[n] += sum_m dY[m][n]   (atomics: one per element per window)
__device__ void wg_linear_dw(float* dW, float* db, const float* dY, int ldy, const float* X, int ldx, int M, int N,
                             int K) {
  for (int idx = threadIdx.x; idx < N * K; idx += blockDim.x) {
    const int n = idx / K, k = idx - n * K;
    float acc = 0.f;
    for (int m = 0; m < M; ++m) acc = fmaf(dY[(long)m * ldy + n], X[(long)m * ldx + k], acc);
    atomicAdd(dW + idx, acc);
  }
  if (db)
    for (int n = threadIdx.x; n < N; n += blockDim.x) {
      float acc = 0.f;
      for (int m = 0; m < M; ++m) acc += dY[(long)m * ldy + n];
      atomicAdd(db + n, acc);
    }
}
__device__ float block_sum(float v, float* red) {
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wv] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}
__device__ float block_max(float v, float* red) {
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wv] = v;
  __syncthreads();
  float s = -INFINITY;
  for (int i = 0; i < nw; ++i) s = fmaxf(s, red[i]);
  return s;
}

// ============================================================================
// Tuning forward: one workgroup per window.  Writes logits/protos [B][H][2],
// the latent in reference order lat[B][3H^2], and the saved activations.
// ============================================================================
template <int H>
__global__ __launch_bounds__(kTW) void tune_fwd_kernel(int B, const float* __restrict__ win,
                                                       const float* __restrict__ P, float* __restrict__ scr,
                                                       float* __restrict__ lat, float* __restrict__ logits,
                                                       float* __restrict__ protos) {
  using G = TGeo<H>;
  constexpr int d = G::D, T = G::T, HD = G::HD;
  __shared__ float red[16];
  const int b = blockIdx.x;
  if (b >= B) return;
  float* S = scr + (long)b * G::S_SIZE;
  const int tid = threadIdx.x;
  for (int i = tid; i < 9 * H; i += kTW) S[G::S_X + i] = win[(long)b * 9 * H + i];
  __syncthreads();
  // ---- GAT (dlutils.py:304-348) ----
  wg_linear(S + G::S_Z, d, S + G::S_X, 3, P + G::W_FC, nullptr, T, d, 3);
  __syncthreads();
  for (int t = tid; t < T; t += kTW) {
    float s = 0.f, u = 0.f;
    for (int c = 0; c < d; ++c) {
      s = fmaf(S[G::S_Z + t * d + c], P[G::W_ATT + c], s);
      u = fmaf(S[G::S_Z + t * d + c], P[G::W_ATT + d + c], u);
    }
    S[G::S_SS + t] = s;
    S[G::S_TT + t] = u;
  }
  __syncthreads();
  for (int w = 0; w < 3; ++w) {
    float mx = -INFINITY;
    for (int e = tid; e < H * H; e += kTW) {
      const int i = e / H, j = e - i * H;
      float v = S[G::S_SS + w * H + i] + S[G::S_TT + w * H + j];
      v = v > 0.f ? v : 0.01f * v;
      mx = fmaxf(mx, v);
    }
    mx = block_max(mx, red);
    float sum = 0.f;
    for (int e = tid; e < H * H; e += kTW) {
      const int i = e / H, j = e - i * H;
      float v = S[G::S_SS + w * H + i] + S[G::S_TT + w * H + j];
      v = v > 0.f ? v : 0.01f * v;
      const float p = expf(v - mx);
      S[G::S_A + (long)w * H * H + e] = p;
      sum += p;
    }
    sum = block_sum(sum, red);
    const float inv = 1.0f / sum;
    for (int e = tid; e < H * H; e += kTW) S[G::S_A + (long)w * H * H + e] *= inv;
    __syncthreads();
  }
  // g[w][j][c] = sum_i a[w][i][j] z[w][i][c]
  for (int idx = tid; idx < T * d; idx += kTW) {
    const int w = idx / (H * d), r = idx - w * H * d, jj = r / d, c = r - jj * d;
    float acc = 0.f;
    for (int i = 0; i < H; ++i)
      acc = fmaf(S[G::S_A + (long)w * H * H + i * H + jj], S[G::S_Z + (w * H + i) * d + c], acc);
    S[G::S_G + idx] = acc;
  }
  __syncthreads();
  // ---- time encoder + PE (models.py:390-393) -> layer 0 input ----
  float* X0 = S + G::S_LAY + G::LS_X;
  wg_linear(X0, d, S + G::S_G, d, P + G::W_TE, P + G::B_TE, T, d, d);
  __syncthreads();
  for (int idx = tid; idx < T * d; idx += kTW) X0[idx] += P[G::PE + (idx / (H * d)) * d + idx % d];
  __syncthreads();
  // ---- encoder layers (models.py:350-356) ----
  const float scale = 1.0f / sqrtf((float)HD);
  for (int l = 0; l < 2; ++l) {
    float* Ls = S + G::S_LAY + l * G::LS_SIZE;
    const float* Lp = P + G::LAY0 + l * G::L_SIZE;
    float* Xout = (l == 0) ? S + G::S_LAY + G::LS_SIZE + G::LS_X : S + G::S_XL;
    wg_linear(Ls + G::LS_QKV, 3 * d, Ls + G::LS_X, d, Lp + G::L_IN, Lp + G::L_INB, T, 3 * d, d);
    __syncthreads();
    for (int idx = tid; idx < 2 * H; idx += kTW) {  // (host, head)
      const int h = idx >> 1, hh = idx & 1;
      float pr[3][3];
      for (int w = 0; w < 3; ++w) {
        float sc[3], m = -INFINITY;
        for (int w2 = 0; w2 < 3; ++w2) {
          float acc = 0.f;
          for (int e = 0; e < HD; ++e)
            acc = fmaf(Ls[G::LS_QKV + (w * H + h) * 3 * d + hh * HD + e],
                       Ls[G::LS_QKV + (w2 * H + h) * 3 * d + d + hh * HD + e], acc);
          sc[w2] = acc * scale;
          m = fmaxf(m, sc[w2]);
        }
        float s = 0.f;
        for (int w2 = 0; w2 < 3; ++w2) {
          sc[w2] = expf(sc[w2] - m);
          s += sc[w2];
        }
        for (int w2 = 0; w2 < 3; ++w2) {
          pr[w][w2] = sc[w2] / s;
          Ls[G::LS_P + ((h * 2 + hh) * 3 + w) * 3 + w2] = pr[w][w2];
        }
      }
      for (int w = 0; w < 3; ++w)
        for (int e = 0; e < HD; ++e) {
          float acc = 0.f;
          for (int w2 = 0; w2 < 3; ++w2)
            acc = fmaf(pr[w][w2], Ls[G::LS_QKV + (w2 * H + h) * 3 * d + 2 * d + hh * HD + e], acc);
          Ls[G::LS_O + (w * H + h) * d + hh * HD + e] = acc;
        }
    }
    __syncthreads();
    wg_linear(Ls + G::LS_R1, d, Ls + G::LS_O, d, Lp + G::L_OUT, Lp + G::L_OUTB, T, d, d);
    __syncthreads();
    for (int idx = tid; idx < T * d; idx += kTW) Ls[G::LS_R1 + idx] += Ls[G::LS_X + idx];
    __syncthreads();
    for (int t = tid; t < T; t += kTW) {  // LN1
      float mu = 0.f;
      for (int c = 0; c < d; ++c) mu += Ls[G::LS_R1 + t * d + c];
      mu /= d;
      float var = 0.f;
      for (int c = 0; c < d; ++c) {
        const float dv = Ls[G::LS_R1 + t * d + c] - mu;
        var += dv * dv;
      }
      const float rs = 1.0f / sqrtf(var / d + 1e-5f);
      Ls[G::LS_M1 + t] = mu;
      Ls[G::LS_S1 + t] = rs;
      for (int c = 0; c < d; ++c)
        Ls[G::LS_Y1 + t * d + c] = (Ls[G::LS_R1 + t * d + c] - mu) * rs * Lp[G::L_N1W + c] + Lp[G::L_N1B + c];
    }
    __syncthreads();
    wg_linear(Ls + G::LS_F, G::FF, Ls + G::LS_Y1, d, Lp + G::L_W1, Lp + G::L_B1, T, G::FF, d);
    __syncthreads();
    // R2 = Y1 + relu(F) W2^T + b2
    for (int idx = tid; idx < T * d; idx += kTW) {
      const int t = idx / d, c = idx - t * d;
      float acc = Lp[G::L_B2 + c];
      for (int u = 0; u < G::FF; ++u) acc = fmaf(fmaxf(Ls[G::LS_F + t * G::FF + u], 0.f), Lp[G::L_W2 + c * G::FF + u], acc);
      Ls[G::LS_R2 + idx] = acc + Ls[G::LS_Y1 + idx];
    }
    __syncthreads();
    for (int t = tid; t < T; t += kTW) {  // LN2 -> next input
      float mu = 0.f;
      for (int c = 0; c < d; ++c) mu += Ls[G::LS_R2 + t * d + c];
      mu /= d;
      float var = 0.f;
      for (int c = 0; c < d; ++c) {
        const float dv = Ls[G::LS_R2 + t * d + c] - mu;
        var += dv * dv;
      }
      const float rs = 1.0f / sqrtf(var / d + 1e-5f);
      Ls[G::LS_M2 + t] = mu;
      Ls[G::LS_S2 + t] = rs;
      for (int c = 0; c < d; ++c)
        Xout[t * d + c] = (Ls[G::LS_R2 + t * d + c] - mu) * rs * Lp[G::L_N2W + c] + Lp[G::L_N2B + c];
    }
    __syncthreads();
  }
  // ---- latent (h, w, c) order (models.py:399) + decoders (models.py:359-370) ----
  float* lt = lat + (long)b * G::L;
  for (int idx = tid; idx < G::L; idx += kTW) {
    const int h = idx / (3 * d), r = idx - h * 3 * d, w = r / d, c = r - w * d;
    lt[idx] = S[G::S_XL + (w * H + h) * d + c];
  }
  __syncthreads();
  for (int n = tid; n < 4 * H; n += kTW) {
    const bool an = n < 2 * H;
    const int row = an ? n : n - 2 * H;
    const float* Wr = P + (an ? G::W_AN : G::W_PR) + (long)row * G::L;
    float acc = P[(an ? G::B_AN : G::B_PR) + row];
    for (int k = 0; k < G::L; ++k) acc = fmaf(Wr[k], lt[k], acc);
    if (an)
      logits[(long)b * 2 * H + row] = acc;
    else
      protos[(long)b * 2 * H + row] = 1.0f / (1.0f + expf(-acc));
  }
}

// ============================================================================
// Loss gradient + backward.  Per window inputs (host-computed sequential
// custom_loss state, train.py:27-40): y [B][H] labels, mult [B][H] CE weights,
// tgt [B][H][2] positive prototypes (prototype value when host h is reached),
// tmask [B][H] (y>0).  dpre [B][4H] = d(decoder pre-activations) (anomaly rows,
// then prototype rows) is written for dw_outer_kernel.
// ============================================================================
template <int H>
__global__ __launch_bounds__(kTW) void tune_bwd_kernel(int B, const float* __restrict__ P, float* __restrict__ Gd,
                                                       float* __restrict__ scr, const float* __restrict__ lat,
                                                       const float* __restrict__ logits,
                                                       const float* __restrict__ protos, const int* __restrict__ y,
                                                       const float* __restrict__ mult, const float* __restrict__ tgt,
                                                       float* __restrict__ dpre) {
  using G = TGeo<H>;
  constexpr int d = G::D, T = G::T, HD = G::HD;
  __shared__ float red[16];
  __shared__ float sd[4 * H];
  const int b = blockIdx.x;
  if (b >= B) return;
  float* S = scr + (long)b * G::S_SIZE;
  const int tid = threadIdx.x;
  // ---- loss gradients (CE * mult; positive-MSE of the triplet term) ----
  for (int h = tid; h < H; h += kTW) {
    const float l0 = logits[(long)b * 2 * H + 2 * h], l1 = logits[(long)b * 2 * H + 2 * h + 1];
    const float m = fmaxf(l0, l1), e0 = expf(l0 - m), e1 = expf(l1 - m), inv = 1.0f / (e0 + e1);
    const int yy = y[(long)b * H + h];
    const float mu = mult[(long)b * H + h];
    sd[2 * h] = mu * (e0 * inv - (yy == 0 ? 1.f : 0.f));
    sd[2 * h + 1] = mu * (e1 * inv - (yy == 1 ? 1.f : 0.f));
    for (int k = 0; k < 2; ++k) {
      const float p = protos[(long)b * 2 * H + 2 * h + k];
      const float g = yy > 0 ? (p - tgt[((long)b * H + h) * 2 + k]) : 0.f;  // d/dp mean_k (p-t)^2
      sd[2 * H + 2 * h + k] = g * p * (1.f - p);                              // through sigmoid
    }
  }
  __syncthreads();
  for (int n = tid; n < 4 * H; n += kTW) dpre[(long)b * 4 * H + n] = sd[n];
  // ---- dlatent = Wa^T da + Wp^T dp -> dX (token layout) ----
  float* dX = S + G::S_DX;
  for (int k = tid; k < G::L; k += kTW) {
    float acc = 0.f;
    for (int n = 0; n < 2 * H; ++n) {
      acc = fmaf(P[G::W_AN + (long)n * G::L + k], sd[n], acc);
      acc = fmaf(P[G::W_PR + (long)n * G::L + k], sd[2 * H + n], acc);
    }
    const int h = k / (3 * d), r = k - h * 3 * d, w = r / d, c = r - w * d;
    dX[(w * H + h) * d + c] = acc;
  }
  __syncthreads();
  // ---- encoder layers, last to first ----
  const float scale = 1.0f / sqrtf((float)HD);
  float* dY = S + G::S_DY;
  float* dF = S + G::S_DF;
  float* dQ = S + G::S_DQKV;
  float* dO = S + G::S_DO;
  for (int l = 1; l >= 0; --l) {
    float* Ls = S + G::S_LAY + l * G::LS_SIZE;
    const float* Lp = P + G::LAY0 + l * G::L_SIZE;
    float* Lg = Gd + G::LAY0 + l * G::L_SIZE;
    // LN2 backward: dX (grad of LN2 output) -> dY (grad of R2)
    for (int t = tid; t < T; t += kTW) {
      const float mu = Ls[G::LS_M2 + t], rs = Ls[G::LS_S2 + t];
      float s1 = 0.f, s2 = 0.f;
      for (int c = 0; c < d; ++c) {
        const float xh = (Ls[G::LS_R2 + t * d + c] - mu) * rs;
        const float dyh = dX[t * d + c] * Lp[G::L_N2W + c];
        s1 += dyh;
        s2 += dyh * xh;
      }
      for (int c = 0; c < d; ++c) {
        const float xh = (Ls[G::LS_R2 + t * d + c] - mu) * rs;
        const float dyh = dX[t * d + c] * Lp[G::L_N2W + c];
        dY[t * d + c] = rs * (dyh - s1 / d - xh * s2 / d);
      }
    }
    for (int c = tid; c < d; c += kTW) {
      float gw = 0.f, gb = 0.f;
      for (int t = 0; t < T; ++t) {
        const float xh = (Ls[G::LS_R2 + t * d + c] - Ls[G::LS_M2 + t]) * Ls[G::LS_S2 + t];
        gw = fmaf(dX[t * d + c], xh, gw);
        gb += dX[t * d + c];
      }
      atomicAdd(Lg + G::L_N2W + c, gw);
      atomicAdd(Lg + G::L_N2B + c, gb);
    }
    __syncthreads();
    // R2 = Y1 + relu(F) W2^T + b2: dF = (dY W2) * (F > 0); dW2 += dY^T relu(F); db2
    for (int idx = tid; idx < T * G::FF; idx += kTW) {
      const int t = idx / G::FF, u = idx - t * G::FF;
      float acc = 0.f;
      for (int c = 0; c < d; ++c) acc = fmaf(dY[t * d + c], Lp[G::L_W2 + c * G::FF + u], acc);
      dF[idx] = Ls[G::LS_F + idx] > 0.f ? acc : 0.f;
    }
    for (int idx = tid; idx < d * G::FF; idx += kTW) {
      const int c = idx / G::FF, u = idx - c * G::FF;
      float acc = 0.f;
      for (int t = 0; t < T; ++t) acc = fmaf(dY[t * d + c], fmaxf(Ls[G::LS_F + t * G::FF + u], 0.f), acc);
      atomicAdd(Lg + G::L_W2 + idx, acc);
    }
    for (int c = tid; c < d; c += kTW) {
      float acc = 0.f;
      for (int t = 0; t < T; ++t) acc += dY[t * d + c];
      atomicAdd(Lg + G::L_B2 + c, acc);
    }
    __syncthreads();
    // F = Y1 W1^T + b1: dW1 += dF^T Y1; db1; dY1 = dY (residual) + dF W1
    wg_linear_dw(Lg + G::L_W1, Lg + G::L_B1, dF, G::FF, Ls + G::LS_Y1, d, T, G::FF, d);
    wg_linear_dx(dY, d, dF, G::FF, Lp + G::L_W1, T, G::FF, d, true);
    __syncthreads();
    // LN1 backward: dY (grad of Y1) -> dX (grad of R1)
    for (int t = tid; t < T; t += kTW) {
      const float mu = Ls[G::LS_M1 + t], rs = Ls[G::LS_S1 + t];
      float s1 = 0.f, s2 = 0.f;
      for (int c = 0; c < d; ++c) {
        const float xh = (Ls[G::LS_R1 + t * d + c] - mu) * rs;
        const float dyh = dY[t * d + c] * Lp[G::L_N1W + c];
        s1 += dyh;
        s2 += dyh * xh;
      }
      for (int c = 0; c < d; ++c) {
        const float xh = (Ls[G::LS_R1 + t * d + c] - mu) * rs;
        const float dyh = dY[t * d + c] * Lp[G::L_N1W + c];
        dX[t * d + c] = rs * (dyh - s1 / d - xh * s2 / d);
      }
    }
    for (int c = tid; c < d; c += kTW) {
      float gw = 0.f, gb = 0.f;
      for (int t = 0; t < T; ++t) {
        const float xh = (Ls[G::LS_R1 + t * d + c] - Ls[G::LS_M1 + t]) * Ls[G::LS_S1 + t];
        gw = fmaf(dY[t * d + c], xh, gw);
        gb += dY[t * d + c];
      }
      atomicAdd(Lg + G::L_N1W + c, gw);
      atomicAdd(Lg + G::L_N1B + c, gb);
    }
    __syncthreads();
    // R1 = X + O Wo^T + bo: dWo += dR1^T O; dbo; dO = dR1 Wo; dX (residual) stays
    wg_linear_dw(Lg + G::L_OUT, Lg + G::L_OUTB, dX, d, Ls + G::LS_O, d, T, d, d);
    wg_linear_dx(dO, d, dX, d, Lp + G::L_OUT, T, d, d, false);
    __syncthreads();
    // attention backward per (host, head)
    for (int idx = tid; idx < 2 * H; idx += kTW) {
      const int h = idx >> 1, hh = idx & 1;
      const float* pr = Ls + G::LS_P + (h * 2 + hh) * 9;
      float dP[3][3], dS[3][3];
      for (int w = 0; w < 3; ++w)
        for (int w2 = 0; w2 < 3; ++w2) {
          float acc = 0.f;
          for (int e = 0; e < HD; ++e)
            acc = fmaf(dO[(w * H + h) * d + hh * HD + e], Ls[G::LS_QKV + (w2 * H + h) * 3 * d + 2 * d + hh * HD + e], acc);
          dP[w][w2] = acc;
        }
      for (int w = 0; w < 3; ++w) {
        const float sdot = pr[w * 3 + 0] * dP[w][0] + pr[w * 3 + 1] * dP[w][1] + pr[w * 3 + 2] * dP[w][2];
        for (int w2 = 0; w2 < 3; ++w2) dS[w][w2] = pr[w * 3 + w2] * (dP[w][w2] - sdot) * scale;
      }
      for (int w = 0; w < 3; ++w)
        for (int e = 0; e < HD; ++e) {
          float dq = 0.f, dk = 0.f, dv = 0.f;
          for (int w2 = 0; w2 < 3; ++w2) {
            dq = fmaf(dS[w][w2], Ls[G::LS_QKV + (w2 * H + h) * 3 * d + d + hh * HD + e], dq);
            dk = fmaf(dS[w2][w], Ls[G::LS_QKV + (w2 * H + h) * 3 * d + hh * HD + e], dk);
            dv = fmaf(pr[w2 * 3 + w], dO[(w2 * H + h) * d + hh * HD + e], dv);
          }
          dQ[(w * H + h) * 3 * d + hh * HD + e] = dq;
          dQ[(w * H + h) * 3 * d + d + hh * HD + e] = dk;
          dQ[(w * H + h) * 3 * d + 2 * d + hh * HD + e] = dv;
        }
    }
    __syncthreads();
    // QKV = X Win^T + bin: dWin += dQKV^T X; dbin; dX += dQKV Win
    wg_linear_dw(Lg + G::L_IN, Lg + G::L_INB, dQ, 3 * d, Ls + G::LS_X, d, T, 3 * d, d);
    wg_linear_dx(dX, d, dQ, 3 * d, Lp + G::L_IN, T, 3 * d, d, true);
    __syncthreads();
  }
  // ---- time encoder: X0 = G Wte^T + bte + pe ----
  float* dG = dO;  // reuse
  wg_linear_dw(Gd + G::W_TE, Gd + G::B_TE, dX, d, S + G::S_G, d, T, d, d);
  wg_linear_dx(dG, d, dX, d, P + G::W_TE, T, d, d, false);
  __syncthreads();
  // ---- GAT backward ----
  float* dZ = dY;  // reuse
  float* dA = S + G::S_DA;
  for (int idx = tid; idx < T * d; idx += kTW) {  // dz[w][i][c] = sum_j a[w][i][j] dg[w][j][c]
    const int w = idx / (H * d), r = idx - w * H * d, i = r / d, c = r - i * d;
    float acc = 0.f;
    for (int jj = 0; jj < H; ++jj)
      acc = fmaf(S[G::S_A + (long)w * H * H + i * H + jj], dG[(w * H + jj) * d + c], acc);
    dZ[idx] = acc;
  }
  for (int e = tid; e < 3 * H * H; e += kTW) {  // da[w][i][j] = dg[w][j] . z[w][i]
    const int w = e / (H * H), r = e - w * H * H, i = r / H, jj = r - i * H;
    float acc = 0.f;
    for (int c = 0; c < d; ++c) acc = fmaf(dG[(w * H + jj) * d + c], S[G::S_Z + (w * H + i) * d + c], acc);
    dA[e] = acc;
  }
  __syncthreads();
  for (int w = 0; w < 3; ++w) {  // softmax over all H^2 edges, then leaky_relu'
    float part = 0.f;
    for (int e = tid; e < H * H; e += kTW) part += S[G::S_A + (long)w * H * H + e] * dA[(long)w * H * H + e];
    const float sdot = block_sum(part, red);
    for (int e = tid; e < H * H; e += kTW) {
      const int i = e / H, jj = e - i * H;
      const float a = S[G::S_A + (long)w * H * H + e];
      const float pre = S[G::S_SS + w * H + i] + S[G::S_TT + w * H + jj];
      dA[(long)w * H * H + e] = a * (dA[(long)w * H * H + e] - sdot) * (pre > 0.f ? 1.f : 0.01f);
    }
    __syncthreads();
  }
  float* dSs = S + G::S_DS;
  float* dTt = S + G::S_DT;
  for (int t = tid; t < T; t += kTW) {
    const int w = t / H, n = t - w * H;
    float ds = 0.f, dt = 0.f;
    for (int k = 0; k < H; ++k) {
      ds += dA[(long)w * H * H + n * H + k];  // n as source i
      dt += dA[(long)w * H * H + k * H + n];  // n as destination j
    }
    dSs[t] = ds;
    dTt[t] = dt;
  }
  __syncthreads();
  for (int c = tid; c < d; c += kTW) {
    float g1 = 0.f, g2 = 0.f;
    for (int t = 0; t < T; ++t) {
      g1 = fmaf(dSs[t], S[G::S_Z + t * d + c], g1);
      g2 = fmaf(dTt[t], S[G::S_Z + t * d + c], g2);
    }
    atomicAdd(Gd + G::W_ATT + c, g1);
    atomicAdd(Gd + G::W_ATT + d + c, g2);
  }
  for (int idx = tid; idx < T * d; idx += kTW) {
    const int t = idx / d, c = idx - t * d;
    dZ[idx] += dSs[t] * P[G::W_ATT + c] + dTt[t] * P[G::W_ATT + d + c];
  }
  __syncthreads();
  wg_linear_dw(Gd + G::W_FC, nullptr, dZ, d, S + G::S_X, 3, T, d, 3);
}

// dW[n][k] += sum_b A[b*lda + n] * X[b*ldx + k] (+ db[n] += sum_b A)
__global__ __launch_bounds__(256) void dw_outer_kernel(int B, int N, int K, const float* __restrict__ A, long lda,
                                                       const float* __restrict__ X, long ldx, float* __restrict__ dW,
                                                       float* __restrict__ db) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx < (long)N * K) {
    const int n = (int)(idx / K), k = (int)(idx - (long)n * K);
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc = fmaf(A[b * lda + n], X[b * ldx + k], acc);
    dW[idx] += acc;
  }
  if (db && idx < N) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += A[b * lda + idx];
    db[idx] += acc;
  }
}

// AdamW, torch single-tensor semantics (torch/optim/adamw.py): p *= 1 - lr*wd;
// m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
  const AdamTensor& t = a.t[blockIdx.y];
  if (!t.active) return;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < t.n; i += (long)gridDim.x * 256) {
    const long o = t.off + i;
    const float g = a.grad[o];
    float p = a.param[o] * (1.0f - a.lr_wd);
    const float m = a.m[o] + (1.0f - a.b1) * (g - a.m[o]);
    const float v = a.b2 * a.v[o] + (1.0f - a.b2) * g * g;
    p -= t.step_size * m / (sqrtf(v) / t.bc2_sqrt + a.eps);
    a.param[o] = p;
    a.m[o] = m;
    a.v[o] = v;
  }
}

// ============================================================================
// GAN: forward (saves activations), Disc BCE backward, Gen BCE backward.
// P points at the gen section (Pg) and disc section (Pd) of the master buffer.
// ============================================================================
template <int H>
__device__ void gan_disc_fwd(float* S, const float* Pd, float* red) {
  using G = TGeo<H>;
  const int tid = threadIdx.x;
  for (int o = tid; o < 64; o += kTW) {
    float acc = Pd[G::D_B1 + o];
    const float* w = Pd + G::D_W1 + (long)o * G::DIN;
    for (int k = 0; k < G::DIN; ++k) acc = fmaf(w[k], S[G::GS_Z + k], acc);
    S[G::GS_DD + o] = acc;  // LeakyReLU(True) = identity
  }
  __syncthreads();
  if (tid < 2) {
    float acc = Pd[G::D_B2 + tid];
    for (int k = 0; k < 64; ++k) acc = fmaf(Pd[G::D_W2 + tid * 64 + k], S[G::GS_DD + k], acc);
    red[tid] = acc;
  }
  __syncthreads();
  if (tid == 0) {
    const float m = fmaxf(red[0], red[1]), e0 = expf(red[0] - m), e1 = expf(red[1] - m);
    S[G::GS_P] = e0 / (e0 + e1);
    S[G::GS_P + 1] = e1 / (e0 + e1);
  }
  __syncthreads();
}

// nn.BCELoss (mean over the 2 probs) -> softmax -> Disc2 -> Disc1 hidden
template <int H>
__device__ void gan_disc_bwd_local(float* S, const float* Pd, float t0, float t1) {
  using G = TGeo<H>;
  const int tid = threadIdx.x;
  if (tid == 0) {
    const float p0 = S[G::GS_P], p1 = S[G::GS_P + 1];
    // torch BCE grad: (p - t) / max(p (1 - p), 1e-12) / N
    const float dp0 = (p0 - t0) / fmaxf(p0 * (1.f - p0), 1e-12f) * 0.5f;
    const float dp1 = (p1 - t1) / fmaxf(p1 * (1.f - p1), 1e-12f) * 0.5f;
    const float s = p0 * dp0 + p1 * dp1;
    S[G::GS_DO] = p0 * (dp0 - s);
    S[G::GS_DO + 1] = p1 * (dp1 - s);
  }
  __syncthreads();
  for (int k = tid; k < 64; k += kTW)
    S[G::GS_DDD + k] = Pd[G::D_W2 + k] * S[G::GS_DO] + Pd[G::D_W2 + 64 + k] * S[G::GS_DO + 1];
  __syncthreads();
}

template <int H>
__global__ __launch_bounds__(kTW) void gan_fwd_kernel(int B, const float* __restrict__ emb /*[B][2H]*/,
                                                      const float* __restrict__ sched, const float* __restrict__ Pg,
                                                      const float* __restrict__ Pd, float* __restrict__ scr,
                                                      float* __restrict__ ns_out, float* __restrict__ probs) {
  using G = TGeo<H>;
  __shared__ float red[16];
  const int b = blockIdx.x;
  if (b >= B) return;
  float* S = scr + (long)b * G::GS_SIZE;
  const int tid = threadIdx.x;
  for (int k = tid; k < 2 * H; k += kTW) S[G::GS_X + k] = emb[(long)b * 2 * H + k];
  for (int k = tid; k < H * H; k += kTW) {
    const float s = sched[(long)b * H * H + k];
    S[G::GS_X + 2 * H + k] = s;
    S[G::GS_Z + k] = s;
  }
  __syncthreads();
  for (int o = tid; o < 64; o += kTW) {
    float acc = Pg[G::G_B1 + o];
    const float* w = Pg + G::G_W1 + (long)o * G::GIN;
    for (int k = 0; k < G::GIN; ++k) acc = fmaf(w[k], S[G::GS_X + k], acc);
    S[G::GS_H + o] = acc;
  }
  __syncthreads();
  for (int o = tid; o < H * H; o += kTW) {
    float acc = Pg[G::G_B2 + o];
    const float* w = Pg + G::G_W2 + (long)o * 64;
    for (int k = 0; k < 64; ++k) acc = fmaf(w[k], S[G::GS_H + k], acc);
    const float t = tanhf(acc);
    S[G::GS_T + o] = t;
    const float nv = S[G::GS_Z + o] + 4.0f * t;
    S[G::GS_Z + H * H + o] = nv;
    ns_out[(long)b * H * H + o] = nv;
  }
  __syncthreads();
  gan_disc_fwd<H>(S, Pd, red);
  if (tid < 2) probs[(long)b * 2 + tid] = S[G::GS_P + tid];
}

// Disc step: target [B][2] -> GS_DO, GS_DDD (weight grads by dw_outer over the batch)
template <int H>
__global__ __launch_bounds__(kTW) void gan_disc_bwd_kernel(int B, const float* __restrict__ target,
                                                           const float* __restrict__ Pd, float* __restrict__ scr) {
  using G = TGeo<H>;
  const int b = blockIdx.x;
  if (b >= B) return;
  gan_disc_bwd_local<H>(scr + (long)b * G::GS_SIZE, Pd, target[2 * b], target[2 * b + 1]);
}

// Gen step: Disc forward with the UPDATED Disc, BCE toward [0,1], back through
// Disc into the new schedule, tanh, Gen2 -> GS_DY, GS_DH.
template <int H>
__global__ __launch_bounds__(kTW) void gan_gen_bwd_kernel(int B, const float* __restrict__ Pg,
                                                          const float* __restrict__ Pd, float* __restrict__ scr) {
  using G = TGeo<H>;
  __shared__ float red[16];
  const int b = blockIdx.x;
  if (b >= B) return;
  float* S = scr + (long)b * G::GS_SIZE;
  const int tid = threadIdx.x;
  gan_disc_fwd<H>(S, Pd, red);
  gan_disc_bwd_local<H>(S, Pd, 0.f, 1.f);
  for (int k = tid; k < H * H; k += kTW) {
    float dz = 0.f;  // d(ns_k) = sum_o Wd1[o][H^2 + k] dDD[o]
    for (int o = 0; o < 64; ++o) dz = fmaf(Pd[G::D_W1 + (long)o * G::DIN + H * H + k], S[G::GS_DDD + o], dz);
    const float t = S[G::GS_T + k];
    S[G::GS_DY + k] = 4.0f * dz * (1.f - t * t);
  }
  __syncthreads();
  for (int u = tid; u < 64; u += kTW) {
    float acc = 0.f;
    for (int k = 0; k < H * H; ++k) acc = fmaf(Pg[G::G_W2 + (long)k * 64 + u], S[G::GS_DY + k], acc);
    S[G::GS_DH + u] = acc;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
long train_scratch_floats(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return TGeo<h>::S_SIZE;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}
long gan_scratch_floats(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return TGeo<h>::GS_SIZE;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

hipError_t launch_tune_fwd(int H, int B, const float* win, const float* P, float* scr, float* lat, float* logits,
                           float* protos, hipStream_t st) {
  switch (H) {
#define CASE(h)                                                                               \
  case h:                                                                                     \
    tune_fwd_kernel<h><<<B, kTW, 0, st>>>(B, win, P, scr, lat, logits, protos);               \
    return hipGetLastError();
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_dw_outer(int B, int N, int K, const float* A, long lda, const float* X, long ldx, float* dW,
                           float* db, hipStream_t st) {
  const long n = (long)N * K;
  const long nb = (n > N ? n : N);
  dw_outer_kernel<<<(int)((nb + 255) / 256), 256, 0, st>>>(B, N, K, A, lda, X, ldx, dW, db);
  return hipGetLastError();
}

hipError_t launch_tune_bwd(int H, int B, const float* P, float* Gd, float* scr, const float* lat, const float* logits,
                           const float* protos, const int* y, const float* mult, const float* tgt, float* dpre,
                           hipStream_t st) {
  switch (H) {
#define CASE(h)                                                                                          \
  case h: {                                                                                              \
    using G = TGeo<h>;                                                                                   \
    tune_bwd_kernel<h><<<B, kTW, 0, st>>>(B, P, Gd, scr, lat, logits, protos, y, mult, tgt, dpre);       \
    hipError_t e = hipGetLastError();                                                                    \
    if (e != hipSuccess) return e;                                                                       \
    e = launch_dw_outer(B, 2 * h, G::L, dpre, 4 * h, lat, G::L, Gd + G::W_AN, Gd + G::B_AN, st);          \
    if (e != hipSuccess) return e;                                                                       \
    return launch_dw_outer(B, 2 * h, G::L, dpre + 2 * h, 4 * h, lat, G::L, Gd + G::W_PR, Gd + G::B_PR, st); \
  }
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_adamw(const AdamArgs& a, hipStream_t st) {
  long maxn = 0;
  for (int i = 0; i < a.ntensors; ++i) maxn = a.t[i].n > maxn ? a.t[i].n : maxn;
  int gx = (int)((maxn + 255) / 256);
  gx = gx > 1024 ? 1024 : (gx < 1 ? 1 : gx);
  adamw_kernel<<<dim3(gx, a.ntensors), 256, 0, st>>>(a);
  return hipGetLastError();
}

hipError_t launch_gan_fwd(int H, int B, const float* emb, const float* sched, const float* Pg, const float* Pd,
                          float* scr, float* ns_out, float* probs, hipStream_t st) {
  switch (H) {
#define CASE(h)                                                                         \
  case h:                                                                               \
    gan_fwd_kernel<h><<<B, kTW, 0, st>>>(B, emb, sched, Pg, Pd, scr, ns_out, probs);    \
    return hipGetLastError();
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_disc_bwd(int H, int B, const float* target, const float* Pd, float* Gdd, float* scr,
                               hipStream_t st) {
  switch (H) {
#define CASE(h)                                                                                              \
  case h: {                                                                                                  \
    using G = TGeo<h>;                                                                                       \
    gan_disc_bwd_kernel<h><<<B, kTW, 0, st>>>(B, target, Pd, scr);                                           \
    hipError_t e = hipGetLastError();                                                                        \
    if (e != hipSuccess) return e;                                                                           \
    e = launch_dw_outer(B, 2, 64, scr + G::GS_DO, G::GS_SIZE, scr + G::GS_DD, G::GS_SIZE, Gdd + G::D_W2,     \
                        Gdd + G::D_B2, st);                                                                  \
    if (e != hipSuccess) return e;                                                                           \
    return launch_dw_outer(B, 64, G::DIN, scr + G::GS_DDD, G::GS_SIZE, scr + G::GS_Z, G::GS_SIZE,            \
                           Gdd + G::D_W1, Gdd + G::D_B1, st);                                                \
  }
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_gen_bwd(int H, int B, const float* Pg, const float* Pd, float* Gdg, float* scr,
                              hipStream_t st) {
  switch (H) {
#define CASE(h)                                                                                             \
  case h: {                                                                                                 \
    using G = TGeo<h>;                                                                                      \
    gan_gen_bwd_kernel<h><<<B, kTW, 0, st>>>(B, Pg, Pd, scr);                                               \
    hipError_t e = hipGetLastError();                                                                       \
    if (e != hipSuccess) return e;                                                                          \
    e = launch_dw_outer(B, h * h, 64, scr + G::GS_DY, G::GS_SIZE, scr + G::GS_H, G::GS_SIZE, Gdg + G::G_W2, \
                        Gdg + G::G_B2, st);                                                                 \
    if (e != hipSuccess) return e;                                                                          \
    return launch_dw_outer(B, 64, G::GIN, scr + G::GS_DH, G::GS_SIZE, scr + G::GS_X, G::GS_SIZE,            \
                           Gdg + G::G_W1, Gdg + G::G_B1, st);                                               \
  }
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
