// pgp_tune1.hip — ONE batch-1 tuning step of backprop (train.py:46-54) as a
// single workgroup: the Transformer forward of one window with every
// activation in LDS, custom_loss / triplet_loss bookkeeping (fp64,
// tune_targets_one; the per-host cross-entropy terms in parallel lanes), the
// loss gradient and the whole backward, writing the transformer section of G.
// The plugin's tune_model runs 10 such steps strictly in sequence (each step's
// forward sees the previous AdamW), so the token-major batched kernels of
// pgp_tune.hip (~45 launches of a few µs each per step at batch 1) are
// replaced by this kernel + the AdamW launch.
//
// Small H only (d = H <= 16: 3H = 48 tokens): every phase is a plain loop over
// its outputs across the workgroup's 1024 threads, phases separated by
// barriers; weight-gradient sums over the 48 tokens run in a fixed order per
// output (deterministic).  Latency-bound by construction (one CU), so the
// layout is chosen for LDS bank behaviour and memory-level parallelism:
//   * the non-decoder weights (GAT, time encoder, pe, both layers: 28 KB at
//     H=16) are copied to LDS once at the start, all loads in flight together;
//   * activation rows have an ODD stride (features + 1), and linear layers map
//     consecutive lanes to consecutive tokens: activation reads are
//     conflict-free, weight reads are broadcasts;
//   * the decoders (2 x [2H][3H^2], 196 KB at H=16) stay in HBM / L2: forward
//     one wave per output row (contiguous 256 B loads, 12 per lane, then a
//     wave sum), backward one lane per latent element (the weight-gradient
//     row writes and the latent gradient share the lane's loads).
// Same math as pgp_tune.hip (GAT aggregating the raw features with
// u = fc^T a_src, v = fc^T a_dst; post-norm layers with LayerNorm on the
// residual sum; decoders over the latent in the reference's (host, step,
// channel) order, models.py:399).
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_gemm.hpp"
#include "pgp_train.hpp"
#include "pgp_tunetargets.hpp"

// phase timing study (variant builds only): -DPGP_T1_PROF records the wall
// clock after every barrier of the kernel; pgp_tune1_prof_read copies it out
#ifdef PGP_T1_PROF
__device__ unsigned long long g_t1_prof[128];
#define T1MARK()                                           \
  do {                                                     \
    if (threadIdx.x == 0) g_t1_prof[mk_] = wall_clock64(); \
    ++mk_;                                                 \
  } while (0)
#else
#define T1MARK() \
  do {           \
  } while (0)
#endif
#define T1SYNC()   \
  __syncthreads(); \
  T1MARK()

namespace pgp {
namespace {

constexpr int kT1Threads = 1024;

template <int H>
struct T1 {
  using G = TGeo<H>;
  static constexpr int D = H, T = 3 * H, HD = H / 2, FF = 64, Q3 = 3 * H, NO = 4 * H, L = 3 * H * H;
  // odd row strides (LDS bank spread)
  static constexpr int DS = D + 1, QS = Q3 + 1, FS = FF + 1;
  // LDS layout (floats)
  static constexpr int S_WIN = 0;                  // [3][3H] window
  static constexpr int S_UV = S_WIN + 9 * H;       // u[3], v[3], pad
  static constexpr int S_ST = S_UV + 8;            // s, t per (step, node) [3][H][2]
  static constexpr int S_GS = S_ST + 6 * H;        // per step: max, Z  [3][2] (pad 8)
  static constexpr int S_RS = S_GS + 8;            // GAT row sums [3][H]
  static constexpr int S_XB = S_RS + 3 * H;        // x-bar [T][3]
  static constexpr int S_G = S_XB + 3 * T;         // GAT output [T][DS]
  static constexpr int S_X0 = S_G + T * DS;        // layer inputs x[0..2] [3][T][DS]
  static constexpr int S_QKV = S_X0 + 3 * T * DS;  // [2][T][QS]
  static constexpr int S_PR = S_QKV + 2 * T * QS;  // probs [2][T][2 heads][3]
  static constexpr int S_O = S_PR + 2 * T * 6;     // attention output [2][T][DS]
  static constexpr int S_XH1 = S_O + 2 * T * DS;   // LN1 x-hat [2][T][DS]
  static constexpr int S_RS1 = S_XH1 + 2 * T * DS; // [2][T]
  static constexpr int S_Y1 = S_RS1 + 2 * T;       // LN1 output [2][T][DS]
  static constexpr int S_F = S_Y1 + 2 * T * DS;    // FFN pre-activation [2][T][FS]
  static constexpr int S_XH2 = S_F + 2 * T * FS;   // LN2 x-hat [2][T][DS]
  static constexpr int S_RS2 = S_XH2 + 2 * T * DS; // [2][T]
  static constexpr int S_Z = S_RS2 + 2 * T;        // pre-LN scratch [T][DS]
  static constexpr int S_OUT = S_Z + T * DS;       // decoder outputs [NO] (logits | protos)
  static constexpr int S_DPRE = S_OUT + NO;        // their gradients [NO]
  static constexpr int S_CE = S_DPRE + NO;         // per-host cross-entropy terms, fp64 [H] (8-byte aligned)
  static constexpr int S_DA = S_CE + 2 * H;        // backward scratch [T][DS]
  static constexpr int S_DB = S_DA + T * DS;       // [T][DS]
  static constexpr int S_DF = S_DB + T * DS;       // [T][FS]
  static constexpr int S_DQ = S_DF + T * FS;       // [T][QS]
  static constexpr int S_MT = S_DQ + T * QS;       // mult [H], tgt [H][2], y [H] (int), cls [H] (int)
  static constexpr int S_GSX = S_MT + 5 * H;       // per step: Xs[3], Xt[3] [3][8]
  static constexpr int WN = (int)(G::LAY0 + 2 * G::L_SIZE);  // GAT, time encoder, pe, both layers
  static constexpr int S_PW = S_GSX + 24;          // LDS copy of those weights
  static constexpr int TOTAL = S_PW + WN;
  static_assert(S_CE % 2 == 0, "fp64 scratch alignment");
  static_assert(TOTAL * 4 <= 160 * 1024, "LDS budget");
  static_assert(L % 64 == 0 && NO <= 64, "decoder wave mapping");
};

// y[t][n] = b[n] + sum_k W[n][k] act(x[t][k]) (+ R[t][n]) for t < T, n < N;
// lanes run over tokens (odd strides: conflict-free), W is a broadcast
template <int K, bool RELU>
PGP_DEV void t1_linear(const float* W, const float* b, const float* x, int xs, int T, int N, float* y, int ys,
                       const float* R, int rs, int tid) {
  for (int i = tid; i < T * N; i += kT1Threads) {
    const int n = i / T, t = i - n * T;
    float acc = b[n];
    const float* w = W + n * K;
    const float* xr = x + t * xs;
#pragma unroll 16
    for (int k = 0; k < K; ++k) acc = fmaf(w[k], RELU ? fmaxf(xr[k], 0.f) : xr[k], acc);
    if (R) acc += R[t * rs + n];
    y[t * ys + n] = acc;
  }
}

// LayerNorm over D features of T tokens (eps 1e-5, biased variance): xh, rs,
// y = xh * gamma + beta (rows of stride DS)
template <int D, int DS>
PGP_DEV void t1_ln(const float* z, int T, const float* gam, const float* bet, float* xh, float* rs, float* y,
                   int tid) {
  for (int t = tid; t < T; t += kT1Threads) {
    const float* zr = z + t * DS;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) s += zr[c];
    const float mu = s / (float)D;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) q = fmaf(zr[c] - mu, zr[c] - mu, q);
    const float r = 1.0f / sqrtf(q / (float)D + 1e-5f);
    rs[t] = r;
#pragma unroll
    for (int c = 0; c < D; ++c) {
      const float v = (zr[c] - mu) * r;
      xh[t * DS + c] = v;
      y[t * DS + c] = fmaf(v, gam[c], bet[c]);
    }
  }
}

// LayerNorm backward: dy [T][DS] -> dx (in place), gamma / beta grads summed
// over the T tokens (written to global)
template <int D, int DS>
PGP_DEV void t1_ln_bwd(float* dy, const float* xh, const float* rs, const float* gam, int T, float* __restrict__ gg,
                       float* __restrict__ gb, int tid) {
  for (int c = tid; c < D; c += kT1Threads) {  // parameter grads first (dy still the output grad)
    float sw = 0.f, sb = 0.f;
    for (int t = 0; t < T; ++t) {
      sw = fmaf(dy[t * DS + c], xh[t * DS + c], sw);
      sb += dy[t * DS + c];
    }
    gg[c] = sw;
    gb[c] = sb;
  }
  __syncthreads();
  for (int t = tid; t < T; t += kT1Threads) {
    float* d = dy + t * DS;
    const float* x = xh + t * DS;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < D; ++c) {
      const float dxh = d[c] * gam[c];
      s1 += dxh;
      s2 = fmaf(dxh, x[c], s2);
    }
    s1 /= (float)D;
    s2 /= (float)D;
    const float r = rs[t];
#pragma unroll
    for (int c = 0; c < D; ++c) d[c] = r * (d[c] * gam[c] - s1 - x[c] * s2);
  }
}

// dW[n][k] = sum_t dy[t][n] act(x[t][k]), db[n] = sum_t dy[t][n]  (to global)
template <int K, bool RELU>
PGP_DEV void t1_dw(const float* dy, int dys, int N, const float* x, int xs, int T, float* __restrict__ dW,
                   float* __restrict__ db, int tid) {
  for (int i = tid; i < N * K; i += kT1Threads) {
    const int n = i / K, k = i - n * K;
    float acc = 0.f;
    for (int t = 0; t < T; ++t) {
      float xv = x[t * xs + k];
      if (RELU) xv = fmaxf(xv, 0.f);
      acc = fmaf(dy[t * dys + n], xv, acc);
    }
    dW[i] = acc;
  }
  if (db)
    for (int n = tid; n < N; n += kT1Threads) {
      float s = 0.f;
      for (int t = 0; t < T; ++t) s += dy[t * dys + n];
      db[n] = s;
    }
}

// dx[t][k] = sum_n W[n][k] dy[t][n] (+ R[t][k]); optional ReLU mask (m[t][k] > 0)
template <int N>
PGP_DEV void t1_dx(const float* W, int K, const float* dy, int dys, int T, float* dx, int dxs, const float* R,
                   int rs, const float* mask, int ms, int tid) {
  for (int i = tid; i < T * K; i += kT1Threads) {
    const int t = i / K, k = i - t * K;
    float acc = 0.f;
    const float* d = dy + t * dys;
#pragma unroll 16
    for (int n = 0; n < N; ++n) acc = fmaf(W[n * K + k], d[n], acc);
    if (R) acc += R[t * rs + k];
    if (mask) acc = mask[t * ms + k] > 0.f ? acc : 0.f;
    dx[t * dxs + k] = acc;
  }
}

// The forward of one window (GAT, time encoder, 2 layers, decoders) with every
// activation left in LDS (T1<H> layout) for the backward; the decoder outputs
// (logits | sigmoid protos) end in sm[S_OUT] and, when given, in global memory.
// Shared by the tuning step (tune1_kernel) and the batch-1 inference (infer1_kernel).
template <int H>
PGP_DEV void t1_forward(float* sm, const float* __restrict__ P, const float* __restrict__ win,
                        float* __restrict__ logits_out, float* __restrict__ protos_out, int& mk_,
                        double* __restrict__ logits64 = nullptr, double* __restrict__ protos64 = nullptr) {
  using S = T1<H>;
  using G = TGeo<H>;
  constexpr int D = S::D, T = S::T, HD = S::HD, FF = S::FF, Q3 = S::Q3, NO = S::NO, L = S::L;
  constexpr int DS = S::DS, QS = S::QS, FS = S::FS;
  (void)mk_;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float* win_s = sm + S::S_WIN;
  float* uv = sm + S::S_UV;
  float* st = sm + S::S_ST;
  float* gs = sm + S::S_GS;
  float* rsum = sm + S::S_RS;
  float* xb = sm + S::S_XB;
  float* g = sm + S::S_G;
  float* xs = sm + S::S_X0;  // x[l] = xs + l*T*DS
  float* Pw = sm + S::S_PW;
  for (int i = tid; i < S::WN; i += kT1Threads) Pw[i] = P[i];
  for (int i = tid; i < 9 * H; i += kT1Threads) win_s[i] = win[i];
  T1SYNC();
  if (tid < 6) {  // u = fc^T a_src, v = fc^T a_dst (dlutils.py:315-329, algebraically)
    const int k = tid % 3;
    const float* a = Pw + G::W_ATT + (tid < 3 ? 0 : D);
    float acc = 0.f;
    for (int c = 0; c < D; ++c) acc = fmaf(a[c], Pw[G::W_FC + c * 3 + k], acc);
    uv[tid] = acc;
  }
  T1SYNC();
  for (int i = tid; i < 3 * H; i += kT1Threads) {  // per (step, node): s = u.x, t = v.x
    const float* x = win_s + (i / H) * 3 * H + 3 * (i % H);
    st[2 * i] = uv[0] * x[0] + uv[1] * x[1] + uv[2] * x[2];
    st[2 * i + 1] = uv[3] * x[0] + uv[4] * x[1] + uv[5] * x[2];
  }
  T1SYNC();
  if (tid < 3) {  // graph-wise softmax max over the H^2 edges of step w: lrelu(max s + max t)
    float ms = -INFINITY, mt = -INFINITY;
    for (int j = 0; j < H; ++j) {
      ms = fmaxf(ms, st[2 * (tid * H + j)]);
      mt = fmaxf(mt, st[2 * (tid * H + j) + 1]);
    }
    const float m = ms + mt;
    gs[2 * tid] = m > 0.f ? m : 0.01f * m;
  }
  T1SYNC();
  for (int i = tid; i < 3 * H; i += kT1Threads) {  // destination j of step w: row sum and x-bar (unnormalised)
    const int w = i / H;
    const float tj = st[2 * i + 1], mx = gs[2 * w];
    float sum = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int s = 0; s < H; ++s) {
      const float e = st[2 * (w * H + s)] + tj;
      const float p = expf((e > 0.f ? e : 0.01f * e) - mx);
      sum += p;
      const float* x = win_s + w * 3 * H + 3 * s;
      a0 = fmaf(p, x[0], a0);
      a1 = fmaf(p, x[1], a1);
      a2 = fmaf(p, x[2], a2);
    }
    rsum[i] = sum;
    xb[3 * i] = a0;
    xb[3 * i + 1] = a1;
    xb[3 * i + 2] = a2;
  }
  T1SYNC();
  if (tid < 3) {
    float z = 0.f;
    for (int j = 0; j < H; ++j) z += rsum[tid * H + j];
    gs[2 * tid + 1] = z;
  }
  T1SYNC();
  for (int i = tid; i < 3 * T; i += kT1Threads) xb[i] *= 1.0f / gs[2 * ((i / 3) / H) + 1];
  T1SYNC();
  for (int i = tid; i < T * D; i += kT1Threads) {  // g = fc(x-bar)
    const int c = i / T, t = i - c * T;
    const float* fc = Pw + G::W_FC + c * 3;
    g[t * DS + c] = fmaf(fc[0], xb[3 * t], fmaf(fc[1], xb[3 * t + 1], fc[2] * xb[3 * t + 2]));
  }
  T1SYNC();
  for (int i = tid; i < T * D; i += kT1Threads) {  // time encoder + pe (models.py:390-393)
    const int c = i / T, t = i - c * T;
    float acc = Pw[G::B_TE + c];
    const float* wr = Pw + G::W_TE + c * D;
    const float* gr = g + t * DS;
#pragma unroll
    for (int k = 0; k < D; ++k) acc = fmaf(wr[k], gr[k], acc);
    xs[t * DS + c] = acc + Pw[G::PE + (t / H) * D + c];
  }
  T1SYNC();
  const float scale = 1.0f / sqrtf((float)HD);
  for (int l = 0; l < 2; ++l) {
    const float* Lp = Pw + G::LAY0 + l * G::L_SIZE;
    float* x = xs + l * T * DS;
    float* qkv = sm + S::S_QKV + l * T * QS;
    float* pr = sm + S::S_PR + l * T * 6;
    float* o = sm + S::S_O + l * T * DS;
    float* xh1 = sm + S::S_XH1 + l * T * DS;
    float* rs1 = sm + S::S_RS1 + l * T;
    float* y1 = sm + S::S_Y1 + l * T * DS;
    float* f = sm + S::S_F + l * T * FS;
    float* xh2 = sm + S::S_XH2 + l * T * DS;
    float* rs2 = sm + S::S_RS2 + l * T;
    float* z = sm + S::S_Z;
    t1_linear<D, false>(Lp + G::L_IN, Lp + G::L_INB, x, DS, T, Q3, qkv, QS, nullptr, 0, tid);
    T1SYNC();
    for (int i = tid; i < H * 2 * 3; i += kT1Threads) {  // (query step, head, host)
      const int w = i / (2 * H), hh = (i / H) % 2, h = i % H;
      const float* q = qkv + (w * H + h) * QS + hh * HD;
      float sc[3];
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) {
        const float* k = qkv + (w2 * H + h) * QS + D + hh * HD;
        float a = 0.f;
#pragma unroll
        for (int e = 0; e < HD; ++e) a = fmaf(q[e], k[e], a);
        sc[w2] = a * scale;
      }
      const float mx = fmaxf(sc[0], fmaxf(sc[1], sc[2]));
      const float e0 = expf(sc[0] - mx), e1 = expf(sc[1] - mx), e2 = expf(sc[2] - mx);
      const float inv = 1.0f / (e0 + e1 + e2);
      float* p = pr + (w * H + h) * 6 + hh * 3;
      p[0] = e0 * inv;
      p[1] = e1 * inv;
      p[2] = e2 * inv;
    }
    T1SYNC();
    for (int i = tid; i < T * D; i += kT1Threads) {  // o = P v
      const int c = i / T, t = i - c * T, h = t % H, hh = c / HD;
      const float* p = pr + t * 6 + hh * 3;
      float acc = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) acc = fmaf(p[w2], qkv[(w2 * H + h) * QS + 2 * D + c], acc);
      o[t * DS + c] = acc;
    }
    T1SYNC();
    t1_linear<D, false>(Lp + G::L_OUT, Lp + G::L_OUTB, o, DS, T, D, z, DS, x, DS, tid);  // out_proj + residual
    T1SYNC();
    t1_ln<D, DS>(z, T, Lp + G::L_N1W, Lp + G::L_N1B, xh1, rs1, y1, tid);
    T1SYNC();
    t1_linear<D, false>(Lp + G::L_W1, Lp + G::L_B1, y1, DS, T, FF, f, FS, nullptr, 0, tid);
    T1SYNC();
    t1_linear<FF, true>(Lp + G::L_W2, Lp + G::L_B2, f, FS, T, D, z, DS, y1, DS, tid);  // linear2(relu f) + y1
    T1SYNC();
    t1_ln<D, DS>(z, T, Lp + G::L_N2W, Lp + G::L_N2B, xh2, rs2, x + T * DS, tid);
    T1SYNC();
  }
  // decoders (models.py:359-370): out[n] = b[n] + sum_L W[n][L] lat[L], lat[h*3H + w*H + c] = x2[w*H + h][c];
  // one wave per output row n (rows wv, wv+16, ...), lane l over L = l + 64j
  const float* x2 = xs + 2 * T * DS;
  float* out = sm + S::S_OUT;
  {
    constexpr int NJ = L / 64;
    float lat[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int Lc = lane + 64 * j, h = Lc / (3 * H), w = (Lc / H) % 3, c = Lc % H;
      lat[j] = x2[(w * H + h) * DS + c];
    }
    for (int n = wv; n < NO; n += kT1Threads / 64) {
      const float* W = n < 2 * H ? P + G::W_AN + (long)n * L : P + G::W_PR + (long)(n - 2 * H) * L;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc = fmaf(W[lane + 64 * j], lat[j], acc);
      acc = wave_sum(acc);
      if (lane == 0) {
        float s;
        if (n < 2 * H) {
          s = acc + P[G::B_AN + n];  // LeakyReLU(True) = identity (models.py:361)
          if (logits_out) logits_out[n] = s;
          if (logits64) logits64[n] = (double)s;
        } else {
          s = 1.0f / (1.0f + expf(-(acc + P[G::B_PR + n - 2 * H])));
          if (protos_out) protos_out[n - 2 * H] = s;
          if (protos64) protos64[n - 2 * H] = (double)s;
        }
        out[n] = s;
      }
    }
  }
  T1SYNC();
}

template <int H>
__global__ __launch_bounds__(kT1Threads) void tune1_kernel(int K, const float* __restrict__ win,
                                                           const int* __restrict__ yv, const int* __restrict__ cv,
                                                           const float* __restrict__ P, float* __restrict__ Gd,
                                                           double* __restrict__ state, double update_min,
                                                           double decay, float* __restrict__ logits_out,
                                                           float* __restrict__ protos_out, double* __restrict__ loss) {
  using S = T1<H>;
  using G = TGeo<H>;
  constexpr int D = S::D, T = S::T, HD = S::HD, FF = S::FF, Q3 = S::Q3, NO = S::NO, L = S::L;
  constexpr int DS = S::DS, QS = S::QS, FS = S::FS;
  __shared__ __attribute__((aligned(16))) float sm[S::TOTAL];
  const int tid = threadIdx.x;
  float* win_s = sm + S::S_WIN;
  float* st = sm + S::S_ST;
  float* gs = sm + S::S_GS;
  float* xb = sm + S::S_XB;
  float* g = sm + S::S_G;
  float* xs = sm + S::S_X0;  // x[l] = xs + l*T*DS
  float* mult = sm + S::S_MT;
  float* tgt = sm + S::S_MT + H;
  int* ys = reinterpret_cast<int*>(sm + S::S_MT + 3 * H);
  int* cs = reinterpret_cast<int*>(sm + S::S_MT + 4 * H);
  double* ce = reinterpret_cast<double*>(sm + S::S_CE);
  float* Pw = sm + S::S_PW;
  int mk_ = 0;
  (void)mk_;
  T1MARK();

  // ---------------- forward ----------------
  for (int i = tid; i < H; i += kT1Threads) {
    ys[i] = yv[i];
    cs[i] = cv[i];
  }
  t1_forward<H>(sm, P, win, logits_out, protos_out, mk_);
  const float* x2 = xs + 2 * T * DS;
  float* out = sm + S::S_OUT;
  const float scale = 1.0f / sqrtf((float)HD);
  // custom_loss / triplet_loss bookkeeping (train.py:13-40): the per-host CE
  // terms in parallel, then the sequential part on one lane, fp64
  if (tid < H) ce[tid] = tune_ce_term(out[2 * tid], out[2 * tid + 1], ys[tid]);
  T1SYNC();
  if (tid == 0) tune_targets_one(H, K, out, out + 2 * H, ys, cs, state, update_min, decay, mult, tgt, loss, ce);
  T1SYNC();

  // ---------------- backward ----------------
  float* dpre = sm + S::S_DPRE;
  for (int h = tid; h < H; h += kT1Threads) {  // CE * mult and the positive MSE through the sigmoid
    const float l0 = out[2 * h], l1 = out[2 * h + 1];
    const float m = fmaxf(l0, l1), e0 = expf(l0 - m), e1 = expf(l1 - m), inv = 1.0f / (e0 + e1);
    const int yy = ys[h];
    const float mu = mult[h];
    dpre[2 * h] = mu * (e0 * inv - (yy == 0 ? 1.f : 0.f));
    dpre[2 * h + 1] = mu * (e1 * inv - (yy == 1 ? 1.f : 0.f));
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float p = out[2 * H + 2 * h + k];
      const float gk = yy > 0 ? (p - tgt[2 * h + k]) : 0.f;
      dpre[2 * H + 2 * h + k] = gk * p * (1.f - p);
    }
  }
  T1SYNC();
  float* da = sm + S::S_DA;
  float* db = sm + S::S_DB;
  float* df = sm + S::S_DF;
  float* dq = sm + S::S_DQ;
  // decoders: one lane per latent element Lc — weight-gradient column Lc of
  // every row (dpre[n] lat[Lc]) and the latent gradient sum_n W[n][Lc] dpre[n]
  for (int Lc = tid; Lc < L; Lc += kT1Threads) {
    const int h = Lc / (3 * H), w = (Lc / H) % 3, c = Lc % H;
    const int r = (w * H + h) * DS + c;
    const float xv = x2[r];
    float acc = 0.f;
#pragma unroll 16
    for (int n = 0; n < NO; ++n) {
      const long off = n < 2 * H ? G::W_AN + (long)n * L : G::W_PR + (long)(n - 2 * H) * L;
      acc = fmaf(P[off + Lc], dpre[n], acc);
      Gd[off + Lc] = dpre[n] * xv;
    }
    da[r] = acc;
  }
  for (int n = tid; n < NO; n += kT1Threads) Gd[n < 2 * H ? G::B_AN + n : G::B_PR + n - 2 * H] = dpre[n];
  T1SYNC();
  for (int l = 1; l >= 0; --l) {
    const float* Lp = Pw + G::LAY0 + l * G::L_SIZE;
    float* Lg = Gd + G::LAY0 + l * G::L_SIZE;
    const float* x = xs + l * T * DS;
    const float* qkv = sm + S::S_QKV + l * T * QS;
    const float* pr = sm + S::S_PR + l * T * 6;
    const float* o = sm + S::S_O + l * T * DS;
    const float* xh1 = sm + S::S_XH1 + l * T * DS;
    const float* rs1 = sm + S::S_RS1 + l * T;
    const float* y1 = sm + S::S_Y1 + l * T * DS;
    const float* f = sm + S::S_F + l * T * FS;
    const float* xh2 = sm + S::S_XH2 + l * T * DS;
    const float* rs2 = sm + S::S_RS2 + l * T;
    // norm2 backward: da (grad of the layer output) -> grad of z2 = y1 + ffn
    t1_ln_bwd<D, DS>(da, xh2, rs2, Lp + G::L_N2W, T, Lg + G::L_N2W, Lg + G::L_N2B, tid);
    T1SYNC();
    t1_dw<FF, true>(da, DS, D, f, FS, T, Lg + G::L_W2, Lg + G::L_B2, tid);         // linear2
    t1_dx<D>(Lp + G::L_W2, FF, da, DS, T, df, FS, nullptr, 0, f, FS, tid);         // d relu(f) (mask f > 0)
    T1SYNC();
    t1_dw<D, false>(df, FS, FF, y1, DS, T, Lg + G::L_W1, Lg + G::L_B1, tid);       // linear1
    t1_dx<FF>(Lp + G::L_W1, D, df, FS, T, db, DS, da, DS, nullptr, 0, tid);        // dy1 = W1^T df + dz2
    T1SYNC();
    t1_ln_bwd<D, DS>(db, xh1, rs1, Lp + G::L_N1W, T, Lg + G::L_N1W, Lg + G::L_N1B, tid);  // -> grad of z1
    T1SYNC();
    t1_dw<D, false>(db, DS, D, o, DS, T, Lg + G::L_OUT, Lg + G::L_OUTB, tid);      // out_proj
    t1_dx<D>(Lp + G::L_OUT, D, db, DS, T, da, DS, nullptr, 0, nullptr, 0, tid);    // d o
    T1SYNC();
    for (int i = tid; i < H * 2 * HD; i += kT1Threads) {  // attention backward per (host, head, e)
      const int h = i / (2 * HD), hh = (i / HD) % 2, e = i % HD;
      float q[3], k[3], v[3], dov[3], p[3][3];
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        const float* rr = qkv + (w * H + h) * QS + hh * HD + e;
        q[w] = rr[0];
        k[w] = rr[D];
        v[w] = rr[2 * D];
        dov[w] = da[(w * H + h) * DS + hh * HD + e];
#pragma unroll
        for (int w2 = 0; w2 < 3; ++w2) p[w][w2] = pr[(w * H + h) * 6 + hh * 3 + w2];
      }
      float dS[3][3];
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        float dp[3];
#pragma unroll
        for (int w2 = 0; w2 < 3; ++w2) {  // dp[w2] = sum_e' dO[w][e'] v[w2][e'] (full head dot product)
          float a = 0.f;
#pragma unroll
          for (int e2 = 0; e2 < HD; ++e2)
            a = fmaf(da[(w * H + h) * DS + hh * HD + e2], qkv[(w2 * H + h) * QS + 2 * D + hh * HD + e2], a);
          dp[w2] = a;
        }
        const float sd = p[w][0] * dp[0] + p[w][1] * dp[1] + p[w][2] * dp[2];
#pragma unroll
        for (int w2 = 0; w2 < 3; ++w2) dS[w][w2] = p[w][w2] * (dp[w2] - sd) * scale;
      }
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        float* rr = dq + (w * H + h) * QS + hh * HD + e;
        rr[0] = dS[w][0] * k[0] + dS[w][1] * k[1] + dS[w][2] * k[2];
        rr[D] = dS[0][w] * q[0] + dS[1][w] * q[1] + dS[2][w] * q[2];
        rr[2 * D] = p[0][w] * dov[0] + p[1][w] * dov[1] + p[2][w] * dov[2];
      }
    }
    T1SYNC();
    t1_dw<D, false>(dq, QS, Q3, x, DS, T, Lg + G::L_IN, Lg + G::L_INB, tid);       // in_proj
    t1_dx<Q3>(Lp + G::L_IN, D, dq, QS, T, da, DS, db, DS, nullptr, 0, tid);        // Win^T dqkv + dz1 (residual)
    T1SYNC();
  }
  // time encoder: da = grad of X0
  t1_dw<D, false>(da, DS, D, g, DS, T, Gd + G::W_TE, Gd + G::B_TE, tid);
  t1_dx<D>(Pw + G::W_TE, D, da, DS, T, db, DS, nullptr, 0, nullptr, 0, tid);  // db = grad of the GAT output g
  for (int i = tid; i < 3 * D; i += kT1Threads) Gd[G::PE + i] = 0.f;  // buffer, not a parameter
  T1SYNC();
  // GAT: g = fc(x-bar): dfc (aggregation part) and dx-bar
  float* dxb = dq;  // [T][3]
  for (int i = tid; i < 3 * T; i += kT1Threads) {
    const int t = i / 3, k = i % 3;
    float acc = 0.f;
    for (int c = 0; c < D; ++c) acc = fmaf(Pw[G::W_FC + c * 3 + k], db[t * DS + c], acc);
    dxb[i] = acc;
  }
  T1SYNC();
  float* gsx = sm + S::S_GSX;
  // edge-softmax backward per step (as gat_bwd_kernel): ds_i, dt_j, then
  // Xs = sum_i ds_i x_i, Xt = sum_j dt_j x_j
  float* dst = df;            // [3][H][2]: ds, dt
  float* dot = df + 6 * H;    // [3]
  float* dpart = df + 8 * H;  // [3][H]
  for (int i = tid; i < 3 * H; i += kT1Threads) {  // per destination j: sum_i a_ij (dxb_j . x_i)
    const int w = i / H;
    const float mx = gs[2 * w], iz = 1.0f / gs[2 * w + 1], tj = st[2 * i + 1];
    const float* dx = dxb + 3 * i;
    float part = 0.f;
    for (int s2 = 0; s2 < H; ++s2) {
      const float e = st[2 * (w * H + s2)] + tj;
      const float a = expf((e > 0.f ? e : 0.01f * e) - mx) * iz;
      const float* xx = win_s + w * 3 * H + 3 * s2;
      part = fmaf(a, dx[0] * xx[0] + dx[1] * xx[1] + dx[2] * xx[2], part);
    }
    dpart[i] = part;
  }
  T1SYNC();
  if (tid < 3) {
    float sum = 0.f;
    for (int j = 0; j < H; ++j) sum += dpart[tid * H + j];
    dot[tid] = sum;
  }
  T1SYNC();
  for (int i = tid; i < 3 * H; i += kT1Threads) {
    const int w = i / H, j = i % H;
    const float mx = gs[2 * w], iz = 1.0f / gs[2 * w + 1], dtt = dot[w];
    const float s = st[2 * i], t = st[2 * i + 1];
    const float* dxj = dxb + 3 * i;
    const float* xj = win_s + w * 3 * H + 3 * j;
    float dt = 0.f, ds = 0.f;
    for (int s2 = 0; s2 < H; ++s2) {  // j as destination
      const float pre = st[2 * (w * H + s2)] + t;
      const float a = expf((pre > 0.f ? pre : 0.01f * pre) - mx) * iz;
      const float* xx = win_s + w * 3 * H + 3 * s2;
      const float d = dxj[0] * xx[0] + dxj[1] * xx[1] + dxj[2] * xx[2];
      dt = fmaf(a * (d - dtt), pre > 0.f ? 1.f : 0.01f, dt);
    }
    for (int d2 = 0; d2 < H; ++d2) {  // j as source
      const float pre = s + st[2 * (w * H + d2) + 1];
      const float a = expf((pre > 0.f ? pre : 0.01f * pre) - mx) * iz;
      const float* dx = dxb + 3 * (w * H + d2);
      const float d = dx[0] * xj[0] + dx[1] * xj[1] + dx[2] * xj[2];
      ds = fmaf(a * (d - dtt), pre > 0.f ? 1.f : 0.01f, ds);
    }
    dst[2 * i] = ds;
    dst[2 * i + 1] = dt;
  }
  T1SYNC();
  if (tid < 18) {  // (step, Xs/Xt, k)
    const int w = tid / 6, which = (tid / 3) % 2, k = tid % 3;
    float acc = 0.f;
    for (int j = 0; j < H; ++j) acc = fmaf(dst[2 * (w * H + j) + which], win_s[w * 3 * H + 3 * j + k], acc);
    gsx[w * 8 + which * 3 + k] = acc;
  }
  T1SYNC();
  for (int c = tid; c < D; c += kT1Threads) {
    float xs_[3] = {0.f, 0.f, 0.f}, xt_[3] = {0.f, 0.f, 0.f};
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        xs_[k] += gsx[w * 8 + k];
        xt_[k] += gsx[w * 8 + 3 + k];
      }
    const float a1 = Pw[G::W_ATT + c], a2 = Pw[G::W_ATT + D + c];
    const float* fc = Pw + G::W_FC + c * 3;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float agg = 0.f;  // aggregation part: sum_t db[t][c] x-bar[t][k]
      for (int t = 0; t < T; ++t) agg = fmaf(db[t * DS + c], xb[3 * t + k], agg);
      Gd[G::W_FC + c * 3 + k] = agg + (a1 * xs_[k] + a2 * xt_[k]);
    }
    Gd[G::W_ATT + c] = fc[0] * xs_[0] + fc[1] * xs_[1] + fc[2] * xs_[2];
    Gd[G::W_ATT + D + c] = fc[0] * xt_[0] + fc[1] * xt_[1] + fc[2] * xt_[2];
  }
#ifdef PGP_T1_PROF
  T1SYNC();
#endif
}

// ---------------------------------------------------------------------------
// Batch-1 inference of run_model (PreGANPlus.py:115-136: run_encoder, detect /
// embed / get_classes, Gen + Disc, the recover_decision gate and targets) in ONE
// workgroup, from the training master weights P (natural layout) and the
// prototypes (fp64, device) — the plugin's per-interval forward without the
// batch-tiled K1-K3 (built for 65,536-window batches).  Outputs as pgp_forward
// at B = 1.  Gen / Disc (models.py:131-151): hg = W1 [emb; s] + b1 (LeakyReLU
// slope 1 = identity), ns = s + 4 tanh(W2 hg + b2); hd = Wd1 [s; ns] + bd1,
// probs = softmax(Wd2 hd + bd2).
// ---------------------------------------------------------------------------
template <int H>
__global__ __launch_bounds__(kT1Threads) void infer1_kernel(int K, const float* __restrict__ win,
                                                            const float* __restrict__ sched,
                                                            const float* __restrict__ P,
                                                            const double* __restrict__ protos_dev,
                                                            float* __restrict__ logits, float* __restrict__ protos,
                                                            int* __restrict__ cls, int* __restrict__ any_anom,
                                                            float* __restrict__ probs, int* __restrict__ keep,
                                                            int* __restrict__ final_t, int* __restrict__ gen_t) {
  using S = T1<H>;
  using G = TGeo<H>;
  constexpr int H2 = H * H, GIN = G::GIN, DIN = G::DIN;
  __shared__ __attribute__((aligned(16))) float sm[S::TOTAL];
  const int tid = threadIdx.x, lane = tid & 63;
  int mk_ = 0;
  t1_forward<H>(sm, P, win, logits, protos, mk_);  // ends with a barrier; outputs in sm[S_OUT]
  const float* out = sm + S::S_OUT;
  // reuse the (now dead) backward scratch regions for the GAN
  float* xin = sm + S::S_DA;       // [GIN] Gen input [emb; s]
  float* sd = xin + GIN;           // [DIN] Disc input [s; ns]
  float* hg = sm + S::S_DF;        // [64]
  float* hd = hg + 64;             // [64]
  int* anyf = reinterpret_cast<int*>(hd + 64);
  const float* Gp = P + G::OFF_GEN;
  const float* Dp = P + G::OFF_DISC;
  if (tid == 0) anyf[0] = 0;
  __syncthreads();
  // detect + embed + get_classes (as K2b's epilogue): first-argmax of the logits,
  // embedding = prototype output where anomalous, class = first argmin of the MSE
  for (int h = tid; h < H; h += kT1Threads) {
    const float l0 = out[2 * h], l1 = out[2 * h + 1], p0 = out[2 * H + 2 * h], p1 = out[2 * H + 2 * h + 1];
    const bool an = l1 > l0;  // torch.argmax: ties -> index 0
    const float e0 = an ? p0 : 0.f, e1 = an ? p1 : 0.f;
    int cl = -1;
    if (!(e0 == 0.f && e1 == 0.f)) {
      float best = INFINITY;
      for (int k = 0; k < K; ++k) {
        const float d0 = e0 - (float)protos_dev[2 * k], d1 = e1 - (float)protos_dev[2 * k + 1];
        const float dist = (d0 * d0 + d1 * d1) * 0.5f;  // torch.mean over PROTO_DIM = 2
        if (dist < best) {                              // np.argmin: first minimum
          best = dist;
          cl = k;
        }
      }
    }
    cls[h] = cl;
    xin[2 * h] = e0;
    xin[2 * h + 1] = e1;
    if (an) anyf[0] = 1;  // benign race: every writer stores 1
  }
  for (int i = tid; i < H2; i += kT1Threads) {
    xin[2 * H + i] = sched[i];
    sd[i] = sched[i];
  }
  __syncthreads();
  // Gen1: 64 outputs, 16 lanes each (k-chunks), xor-butterfly sum
  {
    const int o = tid >> 4, sp = tid & 15;
    constexpr int KC = (GIN + 15) / 16;
    float acc = 0.f;
    for (int k = sp * KC; k < sp * KC + KC && k < GIN; ++k) acc = fmaf(Gp[G::G_W1 + o * GIN + k], xin[k], acc);
    acc = xadd<8>(xadd<4>(xadd<2>(xadd<1>(acc))));  // xor 1, 2, 4, 8 (DPP, pgp_gemm.hpp)
    if (sp == 0) hg[o] = acc + Gp[G::G_B1 + o];  // LeakyReLU(True): identity
  }
  __syncthreads();
  // Gen2: H^2 outputs, ns = s + 4 tanh(W2 hg + b2)
  for (int i = tid; i < 4 * H2; i += kT1Threads) {
    const int o = i >> 2, sp = i & 3;
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc = fmaf(Gp[G::G_W2 + o * 64 + sp * 16 + k], hg[sp * 16 + k], acc);
    acc = xadd<2>(xadd<1>(acc));
    if (sp == 0) sd[H2 + o] = xin[2 * H + o] + 4.0f * tanhf(acc + Gp[G::G_B2 + o]);
  }
  __syncthreads();
  // Disc1: 64 outputs over [s; ns], 16 lanes each
  {
    const int o = tid >> 4, sp = tid & 15;
    constexpr int KC = DIN / 16;
    float acc = 0.f;
    for (int k = sp * KC; k < sp * KC + KC; ++k) acc = fmaf(Dp[G::D_W1 + o * DIN + k], sd[k], acc);
    acc = xadd<8>(xadd<4>(xadd<2>(xadd<1>(acc))));
    if (sp == 0) hd[o] = acc + Dp[G::D_B1 + o];
  }
  __syncthreads();
  if (tid < 64) {  // Disc2 + softmax + gate (PreGANPlus.py:87), one wave
    float z0 = Dp[G::D_W2 + lane] * hd[lane], z1 = Dp[G::D_W2 + 64 + lane] * hd[lane];
    z0 = wave_sum(z0);  // xor 32 .. 1
    z1 = wave_sum(z1);
    z0 += Dp[G::D_B2];
    z1 += Dp[G::D_B2 + 1];
    const float m = fmaxf(z0, z1), e0 = expf(z0 - m), e1 = expf(z1 - m), inv = 1.0f / (e0 + e1);
    if (lane == 0) {
      probs[0] = e0 * inv;
      probs[1] = e1 * inv;
      keep[0] = e0 * inv > e1 * inv ? 1 : 0;
      any_anom[0] = anyf[0];
    }
  }
  for (int c = tid; c < H; c += kT1Threads) {  // first-argmax of each schedule row (original / generated)
    float bs = -INFINITY, bn = -INFINITY;
    int is = 0, in = 0;
    for (int h = 0; h < H; ++h) {
      const float v = sd[c * H + h], w = sd[H2 + c * H + h];
      if (v > bs) {
        bs = v;
        is = h;
      }
      if (w > bn) {
        bn = w;
        in = h;
      }
    }
    final_t[c] = is;
    gen_t[c] = in;
  }
}

}  // namespace

// n independent batch-1 forwards (one workgroup each, t1_forward): the
// batched forward accuracy() runs on the tuning windows (train.py:94-109),
// logits / prototype outputs written as fp64 [n][2H] each
template <int H>
__global__ __launch_bounds__(kT1Threads) void fwd_many_kernel(const float* __restrict__ win,
                                                              const float* __restrict__ P,
                                                              double* __restrict__ logits,
                                                              double* __restrict__ protos) {
  using S = T1<H>;
  __shared__ __attribute__((aligned(16))) float sm[S::TOTAL];
  const long b = blockIdx.x;
  int mk_ = 0;
  t1_forward<H>(sm, P, win + b * 9 * H, nullptr, nullptr, mk_, logits + b * 2 * H, protos + b * 2 * H);
}

#ifdef PGP_T1_PROF
extern "C" int pgp_tune1_prof_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_prof), sizeof(g_t1_prof)) == hipSuccess ? 0 : -1;
}
#endif

bool tune1_supported(int H) { return H == 8 || H == 16; }

hipError_t launch_infer1(int H, int K, const float* win, const float* sched, const float* P, const double* protos,
                         float* logits, float* protos_out, int* cls, int* any_anom, float* probs, int* keep,
                         int* final_t, int* gen_t, hipStream_t st) {
  switch (H) {
    case 8:
      infer1_kernel<8><<<1, kT1Threads, 0, st>>>(K, win, sched, P, protos, logits, protos_out, cls, any_anom, probs,
                                                 keep, final_t, gen_t);
      break;
    case 16:
      infer1_kernel<16><<<1, kT1Threads, 0, st>>>(K, win, sched, P, protos, logits, protos_out, cls, any_anom, probs,
                                                  keep, final_t, gen_t);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_fwd_many(int H, int n, const float* win, const float* P, double* logits, double* protos,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  switch (H) {
    case 8:
      fwd_many_kernel<8><<<n, kT1Threads, 0, st>>>(win, P, logits, protos);
      break;
    case 16:
      fwd_many_kernel<16><<<n, kT1Threads, 0, st>>>(win, P, logits, protos);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_tune1(int H, int K, const float* win, const int* y, const int* cls, const float* P, float* G,
                        double* state, double update_min, double decay, float* logits, float* protos, double* loss,
                        hipStream_t st) {
  switch (H) {
    case 8:
      tune1_kernel<8><<<1, kT1Threads, 0, st>>>(K, win, y, cls, P, G, state, update_min, decay, logits, protos, loss);
      break;
    case 16:
      tune1_kernel<16><<<1, kT1Threads, 0, st>>>(K, win, y, cls, P, G, state, update_min, decay, logits, protos,
                                                  loss);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace pgp
