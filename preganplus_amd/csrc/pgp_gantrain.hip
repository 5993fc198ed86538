// pgp_gantrain.hip — the GAN step (PreGANPlus.py:60-81) over a batch of
// windows as fp32 MFMA GEMMs: Gen + Disc forward (models.py:118-151,
// 258-291), Disc BCE backward, then Gen BCE backward through the updated Disc.
//
// Layout: one scratch row per window (row stride GS_SIZE, pgp_train.hpp) holds
// that window's activations, every segment 16-byte aligned, so the batch's
// rows of one segment form a strided [B][width] matrix:
//   X  = [emb; s] (GIN = 2H + H^2), Z = [s; ns] (DIN = 2H^2), Hg (64), T = tanh
//   (H^2), DD (64), P (2), dOut (2), dDD (64), dY (H^2), dHg (64).
// Products with a long contraction (Gen1 over GIN, Disc1 over DIN, dHg over H^2)
// are split-K GEMMs (gemm_nt_kernel, partial slabs summed in a fixed order by
// the epilogue kernel); the wide ones (Gen2, dZ over H^2 outputs) tile the
// outputs.  Weight gradients sum over the batch's windows with the LDS-staged
// MFMA core shared with the tuning step (dw_accumulate): one workgroup per
// 64x64 output block, written once into G (deterministic).  The 2-way Disc
// head, its softmax and the BCE gradient are one wave per window.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pgp_device.hpp"
#include "pgp_gemm.hpp"
#include "pgp_train.hpp"

namespace pgp {
namespace {

// part[s][m][n0 + n] = sum over k in split s of X[m][k] W[n0 + n][k], n < 64 of
// output group blockIdx.y; 4 waves x 16 rows; K a multiple of 4.
__global__ __launch_bounds__(256) void gemm_nt_kernel(int M, int N, int K, const float* __restrict__ X, long ldx,
                                                      const float* __restrict__ W, long ldw, int S, int ldp,
                                                      float* __restrict__ part) {
  constexpr int NT = 4;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  const long m = ((long)blockIdx.x * 4 + wv) * 16 + i;
  const bool ok = m < M;
  const int n0 = blockIdx.y * 64, s = blockIdx.z;
  const int kbt = (K + 15) / 16;
  const int kb0 = (int)((long)kbt * s / S), kb1 = (int)((long)kbt * (s + 1) / S);
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = zero4();
  const float* xr = X + m * ldx + 4 * g;
  bool nok[NT];
  const float* wr[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    nok[t] = n0 + 16 * t + i < N;
    wr[t] = W + (long)(n0 + 16 * t + i) * ldw + 4 * g;
  }
  for (int kb = kb0; kb < kb1; ++kb) {
    const bool kok = 16 * kb + 4 * g < K;
    const f32x4 xv = (ok && kok) ? ld4(xr + 16 * kb) : zero4();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 wf = (nok[t] && kok) ? ld4(wr[t] + 16 * kb) : zero4();
      acc[t] = mfma(wf[0], xv[0], acc[t]);
      acc[t] = mfma(wf[1], xv[1], acc[t]);
      acc[t] = mfma(wf[2], xv[2], acc[t]);
      acc[t] = mfma(wf[3], xv[3], acc[t]);
    }
  }
  if (ok) {
#pragma unroll
    for (int t = 0; t < NT; ++t) st4(part + ((long)s * M + m) * ldp + n0 + 16 * t + 4 * g, acc[t]);
  }
}

enum : int { GE_BIAS = 0, GE_TANH = 1, GE_DY = 2 };

// epilogue of a split GEMM: v = sum_s part[s][m][n] (+ bias[n]), n < N, then
//   GE_BIAS: out[m*ldo + n] = v
//   GE_TANH: t = tanh(v) -> out (T);  ns = sched + 4 t -> out2 (Z's ns half) and ns_out
//   GE_DY:   out = 4 v (1 - T^2), T read from aux
__global__ __launch_bounds__(256) void gemm_epi_kernel(int mode, int M, int N, int S, int ldp,
                                                       const float* __restrict__ part, const float* __restrict__ bias,
                                                       float* __restrict__ out, long ldo, const float* __restrict__ aux,
                                                       float* __restrict__ out2, float* __restrict__ ns_out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)M * N) return;
  const long m = idx / N;
  const int n = (int)(idx - m * N);
  // the S split partials in split order, loads issued 8 at a time (one
  // dependent round trip per split made this latency-bound at S = 128)
  const float* pp = part + m * ldp + n;
  const long ss = (long)M * ldp;
  float v = 0.f;
  int s = 0;
  for (; s + 8 <= S; s += 8) {
    float q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = pp[(s + j) * ss];
#pragma unroll
    for (int j = 0; j < 8; ++j) v += q[j];
  }
  for (; s < S; ++s) v += pp[s * ss];
  if (bias) v += bias[n];  // LeakyReLU(True) = identity (models.py:127,145)
  if (mode == GE_BIAS) {
    out[m * ldo + n] = v;
  } else if (mode == GE_TANH) {
    const float t = tanhf(v);
    out[m * ldo + n] = t;
    const float nv = aux[m * ldo + n] + 4.0f * t;  // aux: the schedule half of Z
    out2[m * ldo + n] = nv;
    ns_out[m * N + n] = nv;
  } else {
    const float t = aux[m * ldo + n];
    out[m * ldo + n] = 4.0f * v * (1.f - t * t);
  }
}

// one wave per window: the Disc head (models.py:146-151: Linear(64,2), Softmax),
// then (mode >= 1) nn.BCELoss's gradient toward the target (mean over the 2
// probabilities, PreGANPlus.py:66-67,72-73) back through the softmax and the
// head: dOut (2) and dDD = D2^T dOut (64).  mode 1: target from tgt[b]; mode 2: [0,1].
template <int H>
__global__ __launch_bounds__(256) void disc_head_kernel(int B, int mode, const float* __restrict__ Pd,
                                                        float* __restrict__ scr, const float* __restrict__ tgt,
                                                        float* __restrict__ probs) {
  using G = TGeo<H>;
  const int lane = threadIdx.x & 63;
  const long b = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave
  float* S = scr + b * G::GS_SIZE;
  const float dd = S[G::GS_DD + lane];
  const float z0 = wave_sum(Pd[G::D_W2 + lane] * dd) + Pd[G::D_B2];
  const float z1 = wave_sum(Pd[G::D_W2 + 64 + lane] * dd) + Pd[G::D_B2 + 1];
  const float mx = fmaxf(z0, z1), e0 = expf(z0 - mx), e1 = expf(z1 - mx);
  const float p0 = e0 / (e0 + e1), p1 = e1 / (e0 + e1);
  if (lane == 0) {
    S[G::GS_P] = p0;
    S[G::GS_P + 1] = p1;
    if (probs) {
      probs[2 * b] = p0;
      probs[2 * b + 1] = p1;
    }
  }
  if (mode == 0) return;
  const float t0 = mode == 1 ? tgt[2 * b] : 0.f, t1 = mode == 1 ? tgt[2 * b + 1] : 1.f;
  // torch BCE grad: (p - t) / max(p (1 - p), 1e-12) / N
  const float dp0 = (p0 - t0) / fmaxf(p0 * (1.f - p0), 1e-12f) * 0.5f;
  const float dp1 = (p1 - t1) / fmaxf(p1 * (1.f - p1), 1e-12f) * 0.5f;
  const float sd = p0 * dp0 + p1 * dp1;
  const float do0 = p0 * (dp0 - sd), do1 = p1 * (dp1 - sd);
  if (lane == 0) {
    S[G::GS_DO] = do0;
    S[G::GS_DO + 1] = do1;
  }
  S[G::GS_DDD + lane] = Pd[G::D_W2 + lane] * do0 + Pd[G::D_W2 + 64 + lane] * do1;
}

// write the Gen input [emb; s] and Z's schedule half
template <int H>
__global__ __launch_bounds__(256) void gan_in_kernel(int B, const float* __restrict__ emb,
                                                     const float* __restrict__ sched, float* __restrict__ scr) {
  using G = TGeo<H>;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * G::GIN) return;
  const long b = idx / G::GIN;
  const int k = (int)(idx - b * G::GIN);
  float* S = scr + b * G::GS_SIZE;
  if (k < 2 * H) {
    S[G::GS_X + k] = emb[b * 2 * H + k];
  } else {
    const float s = sched[b * H * H + k - 2 * H];
    S[G::GS_X + k] = s;
    S[G::GS_Z + k - 2 * H] = s;
  }
}

// out[c][r] = in[r*ldi + c] for r < R, c < C (small weight transposes)
__global__ __launch_bounds__(256) void transpose_kernel(int R, int C, const float* __restrict__ in, long ldi,
                                                        float* __restrict__ out) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)R * C) return;
  const int c = (int)(idx / R), r = (int)(idx - (long)c * R);
  out[idx] = in[(long)r * ldi + c];
}

// dW[n][k] += sum_b Y[b][n] X[b][k] for the 64x64 block (blockIdx.y, blockIdx.x);
// db[n] += sum_b Y[b][n] by the blockIdx.x == 0 blocks.  With gridDim.z > 1 the
// batch is split: split z sums its rows into part[z] ([N][K] then [N]) and
// dw_part_reduce adds the splits in order.
__global__ __launch_bounds__(256) void dw_block_kernel(int B, int N, int K, const float* __restrict__ Y, long ldy,
                                                       const float* __restrict__ X, long ldx, float* __restrict__ dW,
                                                       float* __restrict__ db, float* __restrict__ part) {
  constexpr int NP = 64, KP = 64, KT = 4, NTW = 1;
  __shared__ __attribute__((aligned(16))) float ys[kDwRows * lds_stride(NP)];
  __shared__ __attribute__((aligned(16))) float xs[kDwRows * lds_stride(KP)];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  const int k0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  f32x4 acc[NTW][KT];
  float pb[NTW] = {0.f};
#pragma unroll
  for (int u = 0; u < KT; ++u) acc[0][u] = zero4();
  const int S = gridDim.z, z = blockIdx.z;
  const long nch = (B + kDwRows - 1) / kDwRows;
  const long r0 = nch * z / S * kDwRows, r1 = std::min<long>(B, nch * (z + 1) / S * kDwRows);
  dw_accumulate<NP, KP, NTW>(r0, r1, Y + n0, ldy, X + k0, ldx, 0, 0, 4, ys, xs, acc, pb, std::min(NP, N - n0),
                             std::min(KP, K - k0));
  float* oW = S > 1 ? part + (long)z * ((long)N * K + N) : dW;
  float* ob = S > 1 ? part + (long)z * ((long)N * K + N) + (long)N * K : db;
  const int t = wv;  // n-tile of this wave
#pragma unroll
  for (int u = 0; u < KT; ++u)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 16 * t + 4 * g + r, k = k0 + 16 * u + i;
      if (n < N && k < K) {
        if (S > 1)
          oW[(long)n * K + k] = acc[0][u][r];
        else
          oW[(long)n * K + k] += acc[0][u][r];
      }
    }
  if (db && blockIdx.x == 0) {
    const float s = xsum(pb[0], true);
    const int n = n0 + 16 * t + i;
    if (g == 0 && n < N) {
      if (S > 1)
        ob[n] = s;
      else
        ob[n] += s;
    }
  }
}

// dW[o] += sum_z part[z][o] (o < N*K), db[n] += sum_z part[z][N*K + n], z ascending
__global__ __launch_bounds__(256) void dw_part_reduce(int S, int N, int K, const float* __restrict__ part,
                                                      float* __restrict__ dW, float* __restrict__ db) {
  const long o = (long)blockIdx.x * 256 + threadIdx.x;
  const long nk = (long)N * K, stride = nk + N;
  if (o < nk) {
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += part[z * stride + o];
    dW[o] += s;
  } else if (db && o < nk + N) {
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += part[z * stride + o];
    db[o - nk] += s;
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
#define GCK(expr)                            \
  do {                                       \
    expr;                                    \
    const hipError_t e_ = hipGetLastError(); \
    if (e_ != hipSuccess) return e_;         \
  } while (0)

struct GanPlan {
  long rows = 0;   // [B][GS_SIZE] window rows
  long part = 0;   // split-K partial slabs
  long tr = 0;     // weight transposes (D1's ns half, W2)
  long total = 0;
};

template <int H>
GanPlan gan_plan_h(int B) {
  using G = TGeo<H>;
  GanPlan p;
  long off = 0;
  auto take = [&](long n) {
    const long o = off;
    off += (n + 63) / 64 * 64;
    return o;
  };
  p.rows = take((long)B * G::GS_SIZE);
  const long wide = (long)B * round_up(H * H, 64);  // S = 1 GEMMs over H^2 outputs
  // split GEMMs: S * ceil(B/64)*64 <= 256*64 rows x 64; weight-gradient splits <= 8 x the largest [N][K] + [N]
  const long dwmax = 8L * (std::max({64L * G::DIN, (long)H * H * 64, 64L * G::GIN}) + (long)H * H);
  p.part = take(std::max({256L * 64 * 64, wide, dwmax}));
  p.tr = take(2L * H * H * 64);
  p.total = off;
  return p;
}

// split factor for an M x 64 output over K: ~256 workgroups
inline int split_for(int M, int K) {
  const int mb = (M + 63) / 64, kbt = (K + 15) / 16;
  return std::max(1, std::min(kbt, 256 / mb));
}

// out (row stride ldo) <- X[M][K] . W[N][K]^T (+ bias) through the epilogue
hipError_t gemm(int M, int N, int K, const float* X, long ldx, const float* W, long ldw, int S, float* part, int mode,
                const float* bias, float* out, long ldo, const float* aux, float* out2, float* ns_out,
                hipStream_t st) {
  const int ng = (N + 63) / 64, ldp = ng * 64;
  GCK((gemm_nt_kernel<<<dim3((M + 63) / 64, ng, S), 256, 0, st>>>(M, N, K, X, ldx, W, ldw, S, ldp, part)));
  GCK((gemm_epi_kernel<<<(int)(((long)M * N + 255) / 256), 256, 0, st>>>(mode, M, N, S, ldp, part, bias, out, ldo,
                                                                           aux, out2, ns_out)));
  return hipSuccess;
}

hipError_t dw_blocks(int B, int N, int K, const float* Y, long ldy, const float* X, long ldx, float* dW, float* db,
                     float* part, hipStream_t st) {
  const int nb = ((K + 63) / 64) * ((N + 63) / 64);
  const int S = std::max(1, std::min({8, 256 / nb, (B + kDwRows - 1) / kDwRows}));
  GCK((dw_block_kernel<<<dim3((K + 63) / 64, (N + 63) / 64, S), 256, 0, st>>>(B, N, K, Y, ldy, X, ldx, dW, db,
                                                                                part)));
  if (S > 1) {
    const long n = (long)N * K + N;
    GCK((dw_part_reduce<<<(int)((n + 255) / 256), 256, 0, st>>>(S, N, K, part, dW, db)));
  }
  return hipSuccess;
}

// Disc1 hidden: DD = Z . D1^T + db1
template <int H>
hipError_t disc_hidden(int B, const float* Pd, float* ws, const GanPlan& gp, hipStream_t st) {
  using G = TGeo<H>;
  float* R = ws + gp.rows;
  return gemm(B, 64, G::DIN, R + G::GS_Z, G::GS_SIZE, Pd + G::D_W1, G::DIN, split_for(B, G::DIN), ws + gp.part,
              GE_BIAS, Pd + G::D_B1, R + G::GS_DD, G::GS_SIZE, nullptr, nullptr, nullptr, st);
}

template <int H>
hipError_t gan_fwd_h(int B, const float* emb, const float* sched, const float* Pg, const float* Pd, float* ws,
                     float* ns_out, float* probs, hipStream_t st) {
  using G = TGeo<H>;
  const GanPlan gp = gan_plan_h<H>(B);
  float* R = ws + gp.rows;
  hipError_t e;
  GCK((gan_in_kernel<H><<<(int)(((long)B * G::GIN + 255) / 256), 256, 0, st>>>(B, emb, sched, R)));
  // Gen1 (models.py:124-127): Hg = W1 [emb; s] + b1
  if ((e = gemm(B, 64, G::GIN, R + G::GS_X, G::GS_SIZE, Pg + G::G_W1, G::GIN, split_for(B, G::GIN), ws + gp.part,
                GE_BIAS, Pg + G::G_B1, R + G::GS_H, G::GS_SIZE, nullptr, nullptr, nullptr, st)) != hipSuccess)
    return e;
  // Gen2 + tanh, ns = s + 4 tanh(.) (models.py:128-133)
  if ((e = gemm(B, H * H, 64, R + G::GS_H, G::GS_SIZE, Pg + G::G_W2, 64, 1, ws + gp.part, GE_TANH, Pg + G::G_B2,
                R + G::GS_T, G::GS_SIZE, R + G::GS_Z, R + G::GS_Z + H * H, ns_out, st)) != hipSuccess)
    return e;
  if ((e = disc_hidden<H>(B, Pd, ws, gp, st)) != hipSuccess) return e;
  GCK((disc_head_kernel<H><<<(B + 3) / 4, 256, 0, st>>>(B, 0, Pd, R, nullptr, probs)));
  return hipSuccess;
}

template <int H>
hipError_t gan_disc_bwd_h(int B, const float* target, const float* Pd, float* Gdd, float* ws, hipStream_t st) {
  using G = TGeo<H>;
  const GanPlan gp = gan_plan_h<H>(B);
  float* R = ws + gp.rows;
  hipError_t e;
  GCK((disc_head_kernel<H><<<(B + 3) / 4, 256, 0, st>>>(B, 1, Pd, R, target, nullptr)));
  if ((e = dw_blocks(B, 2, 64, R + G::GS_DO, G::GS_SIZE, R + G::GS_DD, G::GS_SIZE, Gdd + G::D_W2, Gdd + G::D_B2,
                     ws + gp.part, st)) != hipSuccess)
    return e;
  return dw_blocks(B, 64, G::DIN, R + G::GS_DDD, G::GS_SIZE, R + G::GS_Z, G::GS_SIZE, Gdd + G::D_W1, Gdd + G::D_B1,
                   ws + gp.part, st);
}

template <int H>
hipError_t gan_gen_bwd_h(int B, const float* Pg, const float* Pd, float* Gdg, float* ws, hipStream_t st) {
  using G = TGeo<H>;
  constexpr int HH = H * H;
  const GanPlan gp = gan_plan_h<H>(B);
  float* R = ws + gp.rows;
  float* D1nsT = ws + gp.tr;        // [H^2][64] = D1[:, H^2:]^T
  float* W2T = ws + gp.tr + HH * 64;  // [64][H^2] = W2^T
  hipError_t e;
  // Disc forward with the updated Disc, BCE toward [0,1] (PreGANPlus.py:69-73)
  if ((e = disc_hidden<H>(B, Pd, ws, gp, st)) != hipSuccess) return e;
  GCK((disc_head_kernel<H><<<(B + 3) / 4, 256, 0, st>>>(B, 2, Pd, R, nullptr, nullptr)));
  // d ns = D1[:, H^2:]^T dDD; through 4 tanh: dY = 4 dns (1 - T^2)
  GCK((transpose_kernel<<<(int)((64L * HH + 255) / 256), 256, 0, st>>>(64, HH, Pd + G::D_W1 + HH, G::DIN, D1nsT)));
  if ((e = gemm(B, HH, 64, R + G::GS_DDD, G::GS_SIZE, D1nsT, 64, 1, ws + gp.part, GE_DY, nullptr, R + G::GS_DY,
                G::GS_SIZE, R + G::GS_T, nullptr, nullptr, st)) != hipSuccess)
    return e;
  if ((e = dw_blocks(B, HH, 64, R + G::GS_DY, G::GS_SIZE, R + G::GS_H, G::GS_SIZE, Gdg + G::G_W2, Gdg + G::G_B2,
                     ws + gp.part, st)) != hipSuccess)
    return e;
  // dHg = W2^T dY, then Gen1's gradients
  GCK((transpose_kernel<<<(int)((64L * HH + 255) / 256), 256, 0, st>>>(HH, 64, Pg + G::G_W2, 64, W2T)));
  if ((e = gemm(B, 64, HH, R + G::GS_DY, G::GS_SIZE, W2T, HH, split_for(B, HH), ws + gp.part, GE_BIAS, nullptr,
                R + G::GS_DH, G::GS_SIZE, nullptr, nullptr, nullptr, st)) != hipSuccess)
    return e;
  return dw_blocks(B, 64, G::GIN, R + G::GS_DH, G::GS_SIZE, R + G::GS_X, G::GS_SIZE, Gdg + G::G_W1, Gdg + G::G_B1,
                   ws + gp.part, st);
}

// the Disc probabilities the last disc_head_kernel left in the window rows (after
// pgp_gan_gen_backward: the updated Disc's, i.e. gen_loss's, PreGANPlus.py:71-73)
template <int H>
__global__ void gan_probs_kernel(int B, const float* __restrict__ scr, float* __restrict__ probs) {
  using G = TGeo<H>;
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  probs[2 * b] = scr[b * G::GS_SIZE + G::GS_P];
  probs[2 * b + 1] = scr[b * G::GS_SIZE + G::GS_P + 1];
}

template <int H>
hipError_t gan_probs_h(int B, const float* ws, float* probs, hipStream_t st) {
  const GanPlan gp = gan_plan_h<H>(B);
  GCK((gan_probs_kernel<H><<<(B + 255) / 256, 256, 0, st>>>(B, ws + gp.rows, probs)));
  return hipSuccess;
}

}  // namespace

hipError_t launch_gan_probs(int H, int B, const float* ws, float* probs, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_probs_h<h>(B, ws, probs, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

long gan_workspace_floats(int H, int B) {
  if (B < 1) return 0;
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_plan_h<h>(B).total;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

hipError_t launch_gan_fwd(int H, int B, const float* emb, const float* sched, const float* Pg, const float* Pd,
                          float* ws, float* ns_out, float* probs, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_fwd_h<h>(B, emb, sched, Pg, Pd, ws, ns_out, probs, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_disc_bwd(int H, int B, const float* target, const float* Pd, float* Gdd, float* ws,
                               hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_disc_bwd_h<h>(B, target, Pd, Gdd, ws, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_gen_bwd(int H, int B, const float* Pg, const float* Pd, float* Gdg, float* ws,
                              hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_gen_bwd_h<h>(B, Pg, Pd, Gdg, ws, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
