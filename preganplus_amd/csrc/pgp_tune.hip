// pgp_tune.hip — the semi-supervised tuning step (train.py:42-57): forward with
// saved activations and backward of the PreGAN+ Transformer (models.py:376-416)
// over a batch of windows, as token-major fp32 MFMA GEMMs.
//
// Layout (pgp_tune.hpp): activations are [M][ld] over the batch's M = B*3H
// tokens.  A linear layer runs with one wave per 16 tokens x all N outputs on
// v_mfma_f32_16x16x4_f32: the weights are the A operand (the whole [N][K]
// matrix is staged once per workgroup in LDS as per-lane fragments), the 16
// token rows the B operand (one float4 per lane per 16-deep k-block straight
// from HBM).  A lane then holds outputs n = 16t + 4g + r of token row
// (lane & 15), g = lane >> 4 — whole rows per wave, so LayerNorm forward and
// backward run in the GEMM epilogue with two cross-lane-group sums.  Weight
// gradients [N][K] = sum over tokens are split over workgroups into partial
// slabs that one reduction adds up in a fixed order (deterministic).  The
// decoders contract over a window's whole encoder output (3H x DP, token
// layout) as split-K GEMMs on a permuted copy of their weights.
//
// Deviations from the reference's op order are algebraic only: the GAT
// aggregates the raw features (sum_i a_ij x_i, then fc) instead of fc(x_i)
// (dlutils.py:315-342), and the edge scores use u.x_i + v.x_j with u = fc^T a_1
// (dlutils.py:326-329); the result is the same function, rounded once in fp32.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pgp_device.hpp"
#include "pgp_gemm.hpp"
#include "pgp_train.hpp"
#include "pgp_tune.hpp"
#include "pgp_tunetargets.hpp"

// workgroups of the token-major GEMMs / weight-gradient kernels (grid-stride loops)
#ifndef PGP_LIN_CAP
#define PGP_LIN_CAP 512
#endif
#ifndef PGP_DW_CAP
#define PGP_DW_CAP 512
#endif

namespace pgp {
namespace {

enum : int { EPI_STORE = 0, EPI_PE = 1, EPI_LN = 2, EPI_MASK = 3, EPI_RES = 4, EPI_LNB = 5 };

// LayerNorm (eps 1e-5, biased variance; models.py:350-356 norm1/norm2) of rows
// held as v[t][r] = feature 16t+4g+r of token (lane & 15); features >= N are 0
// on entry.  v becomes x-hat (pads 0); returns rstd.
template <int NT>
PGP_DEV float ln_rows(f32x4 (&v)[NT], int g, int N) {
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t) s += (v[t][0] + v[t][1]) + (v[t][2] + v[t][3]);
  const float mu = xsum(s, true) / (float)N;
  float q = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float dv = (16 * t + 4 * g + r < N) ? v[t][r] - mu : 0.f;
      v[t][r] = dv;
      q += dv * dv;
    }
  const float rs = 1.0f / sqrtf(xsum(q, true) / (float)N + 1e-5f);
#pragma unroll
  for (int t = 0; t < NT; ++t) v[t] = v[t] * rs;
  return rs;
}

// LayerNorm backward: dy (grad of the output) -> grad of the input, from the
// saved x-hat and rstd and gamma w (pads 0); accumulates dy*xh and dy (the
// gamma / beta gradients) into pw / pb.
template <int NT>
PGP_DEV void ln_bwd_rows(f32x4 (&dy)[NT], const f32x4 (&xh)[NT], const f32x4 (&w)[NT], float rs, int g, int N,
                         f32x4 (&pw)[NT], f32x4 (&pb)[NT]) {
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pw[t][r] = fmaf(dy[t][r], xh[t][r], pw[t][r]);
      pb[t][r] += dy[t][r];
      const float dxh = dy[t][r] * w[t][r];
      s1 += dxh;
      s2 = fmaf(dxh, xh[t][r], s2);
      dy[t][r] = dxh;
    }
  s1 = xsum(s1, true) / (float)N;
  s2 = xsum(s2, true) / (float)N;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      dy[t][r] = (16 * t + 4 * g + r < N) ? rs * (dy[t][r] - s1 - xh[t][r] * s2) : 0.f;
}

// ============================================================================
// Linear layer over all tokens: Y = epilogue(X . W'^T + bias), W' = W (trans 0,
// W[n][k] = W[n*ldw+k]) or W^T (trans 1, W'[n][k] = W[k*ldw+n]).
// ============================================================================
struct LinArgs {
  long M;
  const float* X;
  int ldx, relu_x;
  const float* W;
  int ldw, N, K, trans;
  const float* bias;
  float* Y;
  int ldy;
  const float* R;  // residual (LN, RES, LNB) or mask source (MASK)
  int ldr;
  const float* lnw;
  const float* lnb;
  float* XH;  // LN: x-hat out; LNB: saved x-hat in   (row stride ldy)
  float* RS;  // LN: rstd out;  LNB: saved rstd in
  const float* pe;  // PE: positional encoding [3][N]
  int H;
  float* part;  // LNB: per-workgroup gamma/beta partials [grid.y][grid.x][2][NP]
  // batched launch (grid.y = batch index): offsets of W, Y, XH and RS per
  // batch entry; RS is read / written at RS[m * rss]
  long bw, by, bxh, brs;
  int rss;
  int frag;  // W points at W' pre-packed as [NP/16][KP/16][64 lanes][4] fragments
};

template <int NP, int KP, int EPI>
__global__ __launch_bounds__(256, 2) void linear_kernel(LinArgs a) {
  constexpr int NT = NP / 16, KB = KP / 16;
  __shared__ f32x4 wl[NT * KB * 64];
  __shared__ float cb[NP], cw[NP], cbb[NP];
  __shared__ float lred[EPI == EPI_LNB ? 8 * NP : 1];
  float* wf_flat = reinterpret_cast<float*>(wl);
  const float* Wb = a.W + blockIdx.y * a.bw;
  float* Yb = a.Y + blockIdx.y * a.by;
  float* XHb = a.XH ? a.XH + blockIdx.y * a.bxh : nullptr;
  float* RSb = a.RS ? a.RS + blockIdx.y * a.brs : nullptr;
  if (a.frag) {  // W' already packed in fragment order for this (NP, KP): a straight copy
    const f32x4* src = reinterpret_cast<const f32x4*>(Wb);
    for (int i = threadIdx.x; i < NT * KB * 64; i += 256) wl[i] = src[i];
  } else {  // fragment (t, j), lane l, register r <- W'[16t + l%16][16j + 4(l/16) + r]
    for (int i = threadIdx.x; i < NT * KB * 256; i += 256) {
      const int r = i & 3, l = (i >> 2) & 63, f = i >> 8;
      const int t = f / KB, j = f - t * KB;
      const int n = 16 * t + (l & 15), k = 16 * j + 4 * (l >> 4) + r;
      float v = 0.f;
      if (n < a.N && k < a.K) v = a.trans ? Wb[(long)k * a.ldw + n] : Wb[(long)n * a.ldw + k];
      wf_flat[i] = v;
    }
  }
  for (int n = threadIdx.x; n < NP; n += 256) {
    cb[n] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
    cw[n] = (a.lnw && n < a.N) ? a.lnw[n] : 0.f;
    cbb[n] = (a.lnb && n < a.N) ? a.lnb[n] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, mi = lane & 15;
  const long nrb = (a.M + 15) >> 4;
  f32x4 pw[NT], pb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) pw[t] = pb[t] = zero4();
  // B-operand k-blocks are prefetched PF ahead (a ring of registers), so a
  // wave keeps several HBM loads in flight; wide layers (NT > 4) keep the LDS
  // fragments out of registers with a short unroll.  The next row block's first
  // PF k-blocks are loaded while the current one computes.
  constexpr int PF = NT > 4 ? (KB < 2 ? KB : 2) : (KB < 4 ? KB : 4);
  const long rstep = (long)gridDim.x * 4;
  f32x4 xq[PF];
  {
    const long m0 = ((long)blockIdx.x * 4 + wv) * 16 + mi;
#pragma unroll
    for (int j = 0; j < PF; ++j) xq[j] = m0 < a.M ? ld4(a.X + m0 * a.ldx + 4 * g + 16 * j) : zero4();
  }
  for (long rb = (long)blockIdx.x * 4 + wv; rb < nrb; rb += rstep) {
    const long m = rb * 16 + mi;
    const bool ok = m < a.M;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = *reinterpret_cast<const f32x4*>(&cb[16 * t + 4 * g]);
    const float* xr = a.X + m * a.ldx + 4 * g;
    f32x4 xn[PF];
    {
      const long mn = m + rstep * 16;
#pragma unroll
      for (int j = 0; j < PF; ++j) xn[j] = mn < a.M ? ld4(a.X + mn * a.ldx + 4 * g + 16 * j) : zero4();
    }
#pragma unroll 1
    for (int j0 = 0; j0 < KB; j0 += PF) {
#pragma unroll
      for (int jj = 0; jj < PF; ++jj) {
        const int j = j0 + jj;
        if (j < KB) {
          f32x4 xv = xq[jj];
          if (j + PF < KB) xq[jj] = ok ? ld4(xr + 16 * (j + PF)) : zero4();
          if (a.relu_x) {
#pragma unroll
            for (int r = 0; r < 4; ++r) xv[r] = fmaxf(xv[r], 0.f);
          }
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const f32x4 wf = wl[(t * KB + j) * 64 + lane];
            acc[t] = mfma(wf[0], xv[0], acc[t]);
            acc[t] = mfma(wf[1], xv[1], acc[t]);
            acc[t] = mfma(wf[2], xv[2], acc[t]);
            acc[t] = mfma(wf[3], xv[3], acc[t]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < PF; ++j) xq[j] = xn[j];
    float* yr = Yb + m * a.ldy + 4 * g;
    if constexpr (EPI == EPI_PE) {
      const int w = (int)((m % (3L * a.H)) / a.H);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * t + 4 * g + r;
          if (n < a.N) acc[t][r] += a.pe[w * a.N + n];
        }
    }
    if (EPI == EPI_LN || EPI == EPI_MASK || EPI == EPI_RES || (EPI == EPI_LNB && a.R)) {
      const float* rr = a.R + m * a.ldr + 4 * g;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f32x4 rv = ok ? ld4(rr + 16 * t) : zero4();
        if constexpr (EPI == EPI_MASK) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[t][r] = rv[r] > 0.f ? acc[t][r] : 0.f;
        } else {
          acc[t] += rv;
        }
      }
    }
    if constexpr (EPI == EPI_LN) {
      const float rs = ln_rows<NT>(acc, g, a.N);
      if (ok) {
        float* xh = XHb + m * a.ldy + 4 * g;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          st4(xh + 16 * t, acc[t]);
          f32x4 y;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = 16 * t + 4 * g + r;
            y[r] = fmaf(acc[t][r], cw[n], cbb[n]);
          }
          st4(yr + 16 * t, y);
        }
        if (g == 0) RSb[m * a.rss] = rs;
      }
    } else if constexpr (EPI == EPI_LNB) {
      f32x4 xh[NT], w[NT];
      const float* xhr = XHb + m * a.ldy + 4 * g;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        xh[t] = ok ? ld4(xhr + 16 * t) : zero4();
        w[t] = *reinterpret_cast<const f32x4*>(&cw[16 * t + 4 * g]);
      }
      const float rs = ok ? RSb[m * a.rss] : 0.f;
      ln_bwd_rows<NT>(acc, xh, w, rs, g, a.N, pw, pb);
      if (ok) {
#pragma unroll
        for (int t = 0; t < NT; ++t) st4(yr + 16 * t, acc[t]);
      }
    } else {
      if (ok) {
#pragma unroll
        for (int t = 0; t < NT; ++t) st4(yr + 16 * t, acc[t]);
      }
    }
  }
  if constexpr (EPI == EPI_LNB) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sw = row16_sum(pw[t][r]), sb = row16_sum(pb[t][r]);
        if (mi == 0) {
          lred[wv * 2 * NP + 16 * t + 4 * g + r] = sw;
          lred[wv * 2 * NP + NP + 16 * t + 4 * g + r] = sb;
        }
      }
    __syncthreads();
    float* pp = a.part + ((long)blockIdx.y * gridDim.x + blockIdx.x) * 2 * NP;
    for (int k = threadIdx.x; k < 2 * NP; k += 256)
      pp[k] = (lred[k] + lred[2 * NP + k]) + (lred[4 * NP + k] + lred[6 * NP + k]);
  }
}

// part[blk] = [ sum_{rows of blk} Y[m][n] X[m][k] ]_{n<NP,k<KP} ++ [ sum Y[m][n] ]_{n<NP}
struct DwArgs {
  long M;
  const float* Y;
  int ldy;
  const float* X;
  int ldx, relu_x;
  float* part;
};

template <int NP, int KP>
__global__ __launch_bounds__(256) void dw_kernel(DwArgs a) {
  constexpr int NT = NP / 16, KT = KP / 16, NTW = (NT + 3) / 4;
  __shared__ __attribute__((aligned(16))) float ys[kDwRows * lds_stride(NP)];
  __shared__ __attribute__((aligned(16))) float xs[kDwRows * lds_stride(KP)];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  f32x4 acc[NTW][KT];
  float pb[NTW];
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    pb[q] = 0.f;
#pragma unroll
    for (int u = 0; u < KT; ++u) acc[q][u] = zero4();
  }
  const long nch = (a.M + kDwRows - 1) / kDwRows;
  const long r0 = nch * blockIdx.x / gridDim.x * kDwRows;
  const long r1 = std::min<long>(a.M, nch * (blockIdx.x + 1) / gridDim.x * kDwRows);
  dw_accumulate<NP, KP, NTW>(r0, r1, a.Y, a.ldy, a.X, a.ldx, a.relu_x, 0, 4, ys, xs, acc, pb);
  float* P = a.part + (long)blockIdx.x * (NP * KP + NP);
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    const int t = wv + 4 * q;
    if (t < NT) {
#pragma unroll
      for (int u = 0; u < KT; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) P[(16 * t + 4 * g + r) * KP + 16 * u + i] = acc[q][u][r];
      const float sb = xsum(pb[q], true);
      if (g == 0) P[NP * KP + 16 * t + i] = sb;
    }
  }
}

// Deterministic reduction of partial slabs.  Outputs: segment A, rows x cols
// (source i*ldp + j, destination outA[i*ldo + j]) then segment B, nb values
// (source srcb + j, destination outB[j]); each sums part[p*pstride + src] over
// p in [y*pc, (y+1)*pc) of this block's split y — 4 lane groups x 4 independent
// chains, a fixed order — and adds into the destination (one split) or writes
// lvl2[y][o] for a second pass.
constexpr int kRedChunk = 256;
struct RedArgs {
  int nparts, pc;
  long pstride;
  const float* part;
  int rows, cols, ldp, ldo, nb;
  long srcb;
  float* outA;
  float* outB;
  float* lvl2;
};
PGP_DEV void reduce_block(const RedArgs& a, int bx, int by) {
  __shared__ float red[4][65];
  const int jl = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const long na = (long)a.rows * a.cols, nout = na + a.nb;
  const long o = (long)bx * 64 + jl;
  const bool ok = o < nout;
  long src = 0;
  if (ok) {
    if (o < na) {
      const int i = (int)(o / a.cols), j = (int)(o - (long)i * a.cols);
      src = (long)i * a.ldp + j;
    } else {
      src = a.srcb + (o - na);
    }
  }
  const int p0 = by * a.pc, p1 = min(a.nparts, p0 + a.pc);
  const float* sp = a.part + src;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (ok) {
    int p = p0 + pg;
    for (; p + 12 < p1; p += 16) {
      s0 += sp[p * a.pstride];
      s1 += sp[(p + 4) * a.pstride];
      s2 += sp[(p + 8) * a.pstride];
      s3 += sp[(p + 12) * a.pstride];
    }
    for (; p < p1; p += 4) s0 += sp[p * a.pstride];
  }
  red[pg][jl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (pg == 0 && ok) {
    const float t = (red[0][jl] + red[1][jl]) + (red[2][jl] + red[3][jl]);
    if (a.lvl2) {
      a.lvl2[by * nout + o] = t;
    } else if (o < na) {
      const int i = (int)(o / a.cols), j = (int)(o - (long)i * a.cols);
      a.outA[(long)i * a.ldo + j] += t;
    } else {
      a.outB[o - na] += t;
    }
  }
}
__global__ __launch_bounds__(256) void reduce_kernel(RedArgs a) { reduce_block(a, blockIdx.x, blockIdx.y); }

// Up to kMaxRedSeg reductions in one launch (the backward defers every weight-
// gradient reduction to its end): block x -> (segment, local block) by the
// prefix table, y = split; a segment's blocks run reduce_block exactly as its own
// reduce_kernel launch would, so the sums are bit-identical.
constexpr int kMaxRedSeg = 16;
struct RedTable {
  int n;
  int bx0[kMaxRedSeg + 1];
  int nsplit[kMaxRedSeg];
  RedArgs seg[kMaxRedSeg];
};
__global__ __launch_bounds__(256) void reduce_multi_kernel(RedTable t) {
  const int bx = blockIdx.x;
  int s = 0;
  while (s + 1 < t.n && bx >= t.bx0[s + 1]) ++s;
  if ((int)blockIdx.y >= t.nsplit[s]) return;  // whole block
  reduce_block(t.seg[s], bx - t.bx0[s], blockIdx.y);
}


// ============================================================================
// GAT (dlutils.py:296-369), one wave per (window, step), lane = host.
// ============================================================================
template <int H>
struct GatFold {
  float u[3], v[3];  // u = fc^T a_src, v = fc^T a_dst
};
template <int H>
PGP_DEV GatFold<H> gat_fold(const float* P) {
  using G = TGeo<H>;
  GatFold<H> f;
#pragma unroll
  for (int k = 0; k < 3; ++k) f.u[k] = f.v[k] = 0.f;
  for (int c = 0; c < H; ++c)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      f.u[k] = fmaf(P[G::W_ATT + c], P[G::W_FC + c * 3 + k], f.u[k]);
      f.v[k] = fmaf(P[G::W_ATT + H + c], P[G::W_FC + c * 3 + k], f.v[k]);
    }
  return f;
}

template <int H>
__global__ __launch_bounds__(256) void gat_fwd_kernel(int B, const float* __restrict__ win,
                                                      const float* __restrict__ P, float* __restrict__ wcopy,
                                                      float* __restrict__ Gout, float* __restrict__ XB,
                                                      float* __restrict__ GS) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  __shared__ float ss[4][64], sx[4][64][3];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long pw = (long)blockIdx.x * 4 + wv;  // (window, step)
  const bool okw = pw < 3L * B;
  const long b = okw ? pw / 3 : 0;
  const int w = okw ? (int)(pw - b * 3) : 0;
  const int j = lane;
  const bool okj = okw && j < H;
  const GatFold<H> fo = gat_fold<H>(P);
  float x[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) x[k] = okj ? win[(b * 3 + w) * 3 * H + 3 * j + k] : 0.f;
  if (okj) {
#pragma unroll
    for (int k = 0; k < 3; ++k) wcopy[(b * 3 + w) * 3 * H + 3 * j + k] = x[k];
  }
  const float s = fo.u[0] * x[0] + fo.u[1] * x[1] + fo.u[2] * x[2];
  const float t = fo.v[0] * x[0] + fo.v[1] * x[1] + fo.v[2] * x[2];
  const float smax = wave_max(okj ? s : -INFINITY), tmax = wave_max(okj ? t : -INFINITY);
  const float mx = lrelu(smax + tmax);  // max over all H^2 edges (leaky_relu is monotone)
  ss[wv][j] = s;
#pragma unroll
  for (int k = 0; k < 3; ++k) sx[wv][j][k] = x[k];
  __syncthreads();
  float sum = 0.f, xb[3] = {0.f, 0.f, 0.f};
  if (okj)
    for (int i = 0; i < H; ++i) {
      const float p = expf(lrelu(ss[wv][i] + t) - mx);  // graph-wise softmax_edges (dlutils.py:335)
      sum += p;
#pragma unroll
      for (int k = 0; k < 3; ++k) xb[k] = fmaf(p, sx[wv][i][k], xb[k]);
    }
  const float Z = wave_sum(sum);
  const float iz = 1.0f / Z;
  if (okj) {
#pragma unroll
    for (int k = 0; k < 3; ++k) xb[k] *= iz;
    const long m = b * Q::T + (long)w * H + j;
    float* gr = Gout + m * Q::DP;
    for (int c = 0; c < H; ++c)
      gr[c] = fmaf(P[G::W_FC + c * 3], xb[0], fmaf(P[G::W_FC + c * 3 + 1], xb[1], P[G::W_FC + c * 3 + 2] * xb[2]));
#pragma unroll
    for (int k = 0; k < 3; ++k) XB[m * Q::XBP + k] = xb[k];
  }
  if (okw && lane == 0) {
    GS[pw * 4] = mx;
    GS[pw * 4 + 1] = Z;
  }
}

// GAT backward from dG (grad of the GAT output): the fc gradient through the
// aggregation is a dW GEMM over (dG, x-bar); this kernel back-propagates into
// the edge softmax and writes, per (window, step), Xs = sum_i ds_i x_i and
// Xt = sum_j dt_j x_j (ds, dt: grads of the per-node source / destination
// scores), from which gat_param_kernel forms the attn_fc and remaining fc grads.
template <int H>
__global__ __launch_bounds__(256) void gat_bwd_kernel(int B, const float* __restrict__ wcopy,
                                                      const float* __restrict__ P, const float* __restrict__ dG,
                                                      const float* __restrict__ GS, float* __restrict__ GSX) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  __shared__ float ss[4][64], st[4][64], sx[4][64][3], sdx[4][64][3];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long pw = (long)blockIdx.x * 4 + wv;
  const bool okw = pw < 3L * B;
  const long b = okw ? pw / 3 : 0;
  const int w = okw ? (int)(pw - b * 3) : 0;
  const int j = lane;
  const bool okj = okw && j < H;
  const GatFold<H> fo = gat_fold<H>(P);
  float x[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) x[k] = okj ? wcopy[(b * 3 + w) * 3 * H + 3 * j + k] : 0.f;
  const float s = fo.u[0] * x[0] + fo.u[1] * x[1] + fo.u[2] * x[2];
  const float t = fo.v[0] * x[0] + fo.v[1] * x[1] + fo.v[2] * x[2];
  const float mx = okw ? GS[pw * 4] : 0.f, iz = okw ? 1.0f / GS[pw * 4 + 1] : 0.f;
  float dxb[3] = {0.f, 0.f, 0.f};  // grad of x-bar_j = fc^T dG_j
  if (okj) {
    const float* gr = dG + (b * Q::T + (long)w * H + j) * Q::DP;
    for (int c = 0; c < H; ++c) {
      const float gv = gr[c];
#pragma unroll
      for (int k = 0; k < 3; ++k) dxb[k] = fmaf(P[G::W_FC + c * 3 + k], gv, dxb[k]);
    }
  }
  ss[wv][j] = s;
  st[wv][j] = t;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    sx[wv][j][k] = x[k];
    sdx[wv][j][k] = dxb[k];
  }
  __syncthreads();
  // softmax backward: da_ij = dxb_j . x_i ; dot = sum_ij a_ij da_ij
  float part = 0.f;
  if (okj)
    for (int i = 0; i < H; ++i) {
      const float a = expf(lrelu(ss[wv][i] + t) - mx) * iz;
      const float da = dxb[0] * sx[wv][i][0] + dxb[1] * sx[wv][i][1] + dxb[2] * sx[wv][i][2];
      part = fmaf(a, da, part);
    }
  const float dot = wave_sum(part);
  float dt = 0.f, ds = 0.f;
  if (okj) {
    for (int i = 0; i < H; ++i) {  // this lane as destination
      const float pre = ss[wv][i] + t;
      const float a = expf(lrelu(pre) - mx) * iz;
      const float da = dxb[0] * sx[wv][i][0] + dxb[1] * sx[wv][i][1] + dxb[2] * sx[wv][i][2];
      dt = fmaf(a * (da - dot), pre > 0.f ? 1.f : 0.01f, dt);
    }
    for (int jj = 0; jj < H; ++jj) {  // this lane as source
      const float pre = s + st[wv][jj];
      const float a = expf(lrelu(pre) - mx) * iz;
      const float da = sdx[wv][jj][0] * x[0] + sdx[wv][jj][1] * x[1] + sdx[wv][jj][2] * x[2];
      ds = fmaf(a * (da - dot), pre > 0.f ? 1.f : 0.01f, ds);
    }
  }
  float xs[3], xt[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    xs[k] = wave_sum(ds * x[k]);
    xt[k] = wave_sum(dt * x[k]);
  }
  if (okw && lane == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      GSX[pw * 8 + k] = xs[k];
      GSX[pw * 8 + 3 + k] = xt[k];
    }
  }
}

// attn_fc and the score part of the fc gradient: s_i = a_1 . fc x_i, so
// d a_1 = fc Xs, d fc += a_1 Xs^T (and likewise a_2, Xt), summed over all
// (window, step) in a fixed order.
template <int H>
__global__ __launch_bounds__(256) void gat_param_kernel(int n, const float* __restrict__ GSX,
                                                        const float* __restrict__ P, float* __restrict__ Gd) {
  using G = TGeo<H>;
  __shared__ float red[256][7];
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = threadIdx.x; p < n; p += 256)
#pragma unroll
    for (int k = 0; k < 6; ++k) acc[k] += GSX[(long)p * 8 + k];
#pragma unroll
  for (int k = 0; k < 6; ++k) red[threadIdx.x][k] = acc[k];
  __syncthreads();
  for (int s = 128; s >= 1; s >>= 1) {
    if (threadIdx.x < s)
#pragma unroll
      for (int k = 0; k < 6; ++k) red[threadIdx.x][k] += red[threadIdx.x + s][k];
    __syncthreads();
  }
  const float* xs = red[0];
  const float* xt = red[0] + 3;
  for (int c = threadIdx.x; c < H; c += 256) {
    const float* fc = P + G::W_FC + c * 3;
    const float a1 = P[G::W_ATT + c], a2 = P[G::W_ATT + H + c];
#pragma unroll
    for (int k = 0; k < 3; ++k) Gd[G::W_FC + c * 3 + k] += a1 * xs[k] + a2 * xt[k];
    Gd[G::W_ATT + c] += fc[0] * xs[0] + fc[1] * xs[1] + fc[2] * xs[2];
    Gd[G::W_ATT + H + c] += fc[0] * xt[0] + fc[1] * xt[1] + fc[2] * xt[2];
  }
}

// ============================================================================
// Self-attention over the 3 window steps (models.py:350-356, 2 heads), one
// 32-lane half wave per (window, host): lane e = head dimension.
// ============================================================================
template <int H>
__global__ __launch_bounds__(256) void attn_fwd_kernel(int B, const float* __restrict__ QKV, float* __restrict__ O,
                                                       float* __restrict__ PR) {
  using Q = TuneGeo<H>;
  constexpr int HD = Q::HD;
  const long hw = ((long)blockIdx.x * 256 + threadIdx.x) >> 5;
  const int e = threadIdx.x & 31;
  const bool okp = hw < (long)B * H;
  const long b = okp ? hw / H : 0;
  const int h = okp ? (int)(hw - b * H) : 0;
  const bool oke = okp && e < HD;
  const float scale = 1.0f / sqrtf((float)HD);
  long mr[3];
#pragma unroll
  for (int w = 0; w < 3; ++w) mr[w] = b * Q::T + (long)w * H + h;
  float q[2][3], k[2][3], v[2][3];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const float* rw = QKV + mr[w] * Q::Q3P + hh * HD + e;
      q[hh][w] = oke ? rw[0] : 0.f;
      k[hh][w] = oke ? rw[H] : 0.f;
      v[hh][w] = oke ? rw[2 * H] : 0.f;
    }
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      float sc[3];
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) sc[w2] = half_sum(q[hh][w] * k[hh][w2]) * scale;
      const float mx = fmaxf(sc[0], fmaxf(sc[1], sc[2]));
      const float e0 = expf(sc[0] - mx), e1 = expf(sc[1] - mx), e2 = expf(sc[2] - mx);
      const float inv = 1.0f / (e0 + e1 + e2);
      const float p0 = e0 * inv, p1 = e1 * inv, p2 = e2 * inv;
      if (oke) O[mr[w] * Q::DP + hh * HD + e] = fmaf(p0, v[hh][0], fmaf(p1, v[hh][1], p2 * v[hh][2]));
      if (okp && e < 3) PR[mr[w] * 8 + hh * 3 + e] = e == 0 ? p0 : (e == 1 ? p1 : p2);
    }
}

template <int H>
__global__ __launch_bounds__(256) void attn_bwd_kernel(int B, const float* __restrict__ QKV,
                                                       const float* __restrict__ PR, const float* __restrict__ dO,
                                                       float* __restrict__ dQKV) {
  using Q = TuneGeo<H>;
  constexpr int HD = Q::HD;
  const long hw = ((long)blockIdx.x * 256 + threadIdx.x) >> 5;
  const int e = threadIdx.x & 31;
  const bool okp = hw < (long)B * H;
  const long b = okp ? hw / H : 0;
  const int h = okp ? (int)(hw - b * H) : 0;
  const bool oke = okp && e < HD;
  const float scale = 1.0f / sqrtf((float)HD);
  long mr[3];
#pragma unroll
  for (int w = 0; w < 3; ++w) mr[w] = b * Q::T + (long)w * H + h;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    float q[3], k[3], v[3], dov[3], p[3][3];
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const float* rw = QKV + mr[w] * Q::Q3P + hh * HD + e;
      q[w] = oke ? rw[0] : 0.f;
      k[w] = oke ? rw[H] : 0.f;
      v[w] = oke ? rw[2 * H] : 0.f;
      dov[w] = oke ? dO[mr[w] * Q::DP + hh * HD + e] : 0.f;
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) p[w][w2] = okp ? PR[mr[w] * 8 + hh * 3 + w2] : 0.f;
    }
    float dS[3][3];
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      float dp[3];
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) dp[w2] = half_sum(dov[w] * v[w2]);
      const float sd = p[w][0] * dp[0] + p[w][1] * dp[1] + p[w][2] * dp[2];
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) dS[w][w2] = p[w][w2] * (dp[w2] - sd) * scale;
    }
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const float dq = dS[w][0] * k[0] + dS[w][1] * k[1] + dS[w][2] * k[2];
      const float dk = dS[0][w] * q[0] + dS[1][w] * q[1] + dS[2][w] * q[2];
      const float dv = p[0][w] * dov[0] + p[1][w] * dov[1] + p[2][w] * dov[2];
      if (oke) {
        float* o = dQKV + mr[w] * Q::Q3P + hh * HD + e;
        o[0] = dq;
        o[H] = dk;
        o[2 * H] = dv;
      }
    }
  }
}

// ============================================================================
// Decoders (models.py:359-370, 399) and the loss gradient (train.py:27-40).
// ============================================================================
// Decoder weights permuted to the token layout: Wp[n][k'] with k' = tok*DP + c,
// tok = w*H + h, natural column h*3H + w*H + c (the latent order, models.py:399);
// rows n: anomaly 0..2H-1, prototype 2H..4H-1, zero pads.  WpF holds, per token,
// the transposed slab W'[c][n] = Wp[n][tok*DP + c] as linear_kernel<DP, NOP>
// fragments (the decoder backward into the encoder output).
template <int H>
__global__ __launch_bounds__(256) void dec_pack_kernel(const float* __restrict__ P, float* __restrict__ Wp,
                                                       float* __restrict__ WpF) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  constexpr int KB = Q::NOP / 16;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)Q::NOP * Q::KD) return;
  const int n = (int)(idx / Q::KD);
  const long k = idx - (long)n * Q::KD;
  const int tok = (int)(k / Q::DP), c = (int)(k - (long)tok * Q::DP);
  const int w = tok / H, h = tok - w * H;
  float v = 0.f;
  if (n < 4 * H && c < H) {
    const long col = (long)h * 3 * H + w * H + c;
    v = n < 2 * H ? P[G::W_AN + (long)n * G::L + col] : P[G::W_PR + (long)(n - 2 * H) * G::L + col];
  }
  Wp[idx] = v;
  const int f = (c >> 4) * KB + (n >> 4), l = (c & 15) + 16 * ((n & 15) >> 2);
  WpF[(long)tok * Q::DP * Q::NOP + ((long)f * 64 + l) * 4 + (n & 3)] = v;
}

// split-K decoder GEMM: part[s][b][n] = sum over k-blocks of split s of X2[b] . Wp[n]
template <int H>
__global__ __launch_bounds__(256) void dec_fwd_kernel(int B, int S, const float* __restrict__ X2,
                                                      const float* __restrict__ Wp, float* __restrict__ part) {
  using Q = TuneGeo<H>;
  constexpr int NT = Q::NOP / 16;
  constexpr long KBT = Q::KD / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  const long b = ((long)blockIdx.x * 4 + wv) * 16 + i;
  const bool ok = b < B;
  const int s = blockIdx.y;
  const long kb0 = KBT * s / S, kb1 = KBT * (s + 1) / S;
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = zero4();
  const float* xr = X2 + b * Q::KD + 4 * g;
  const float* wr = Wp + (long)i * Q::KD + 4 * g;
  for (long kb = kb0; kb < kb1; ++kb) {
    const f32x4 xv = ok ? ld4(xr + 16 * kb) : zero4();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 wf = ld4(wr + (long)16 * t * Q::KD + 16 * kb);
      acc[t] = mfma(wf[0], xv[0], acc[t]);
      acc[t] = mfma(wf[1], xv[1], acc[t]);
      acc[t] = mfma(wf[2], xv[2], acc[t]);
      acc[t] = mfma(wf[3], xv[3], acc[t]);
    }
  }
  if (ok) {
#pragma unroll
    for (int t = 0; t < NT; ++t) st4(part + ((long)s * B + b) * Q::NOP + 16 * t + 4 * g, acc[t]);
  }
}

template <int H>
__global__ __launch_bounds__(256) void dec_fin_kernel(int B, int S, const float* __restrict__ part,
                                                      const float* __restrict__ P, float* __restrict__ logits,
                                                      float* __restrict__ protos) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * 4 * H) return;
  const long b = idx / (4 * H);
  const int n = (int)(idx - b * 4 * H);
  // the S partials in split order; loads issued 8 at a time so the adds wait
  // on one batch instead of one round trip per split
  const float* pp = part + b * Q::NOP + n;
  const long qs = (long)B * Q::NOP;
  float s = 0.f;
  int q = 0;
  for (; q + 8 <= S; q += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = pp[(q + j) * qs];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
  }
  for (; q < S; ++q) s += pp[q * qs];
  if (n < 2 * H)
    logits[b * 2 * H + n] = s + P[G::B_AN + n];  // LeakyReLU(True) = identity (models.py:361)
  else
    protos[b * 2 * H + n - 2 * H] = 1.0f / (1.0f + expf(-(s + P[G::B_PR + n - 2 * H])));
}

// latent in the reference's (host, step, channel) order (models.py:399), a test tap
template <int H>
__global__ __launch_bounds__(256) void latent_kernel(int B, const float* __restrict__ X2, float* __restrict__ lat) {
  using Q = TuneGeo<H>;
  constexpr long L = 3L * H * H;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * L) return;
  const long b = idx / L;
  const int r = (int)(idx - b * L), h = r / (3 * H), w = (r % (3 * H)) / H, c = r % H;
  lat[idx] = X2[(b * Q::T + (long)w * H + h) * Q::DP + c];
}

// d(decoder pre-activations) [B][NOP]: CE(logits, y) * mult (train.py:28-36)
// and the positive triplet MSE toward tgt through the sigmoid (train.py:15-21;
// the negative terms are detached there and carry no gradient).
__global__ __launch_bounds__(256) void tune_loss_kernel(int B, int H, int NOP, const float* __restrict__ logits,
                                                        const float* __restrict__ protos, const int* __restrict__ y,
                                                        const float* __restrict__ mult,
                                                        const float* __restrict__ tgt, float* __restrict__ dpre) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * H) return;
  const long b = idx / H;
  const int h = (int)(idx - b * H);
  const float l0 = logits[b * 2 * H + 2 * h], l1 = logits[b * 2 * H + 2 * h + 1];
  const float m = fmaxf(l0, l1), e0 = expf(l0 - m), e1 = expf(l1 - m), inv = 1.0f / (e0 + e1);
  const int yy = y[idx];
  const float mu = mult[idx];
  float* d = dpre + b * NOP;
  d[2 * h] = mu * (e0 * inv - (yy == 0 ? 1.f : 0.f));
  d[2 * h + 1] = mu * (e1 * inv - (yy == 1 ? 1.f : 0.f));
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float p = protos[b * 2 * H + 2 * h + k];
    const float gk = yy > 0 ? (p - tgt[idx * 2 + k]) : 0.f;  // d/dp mean_k (p - t)^2
    d[2 * H + 2 * h + k] = gk * p * (1.f - p);                // through the sigmoid
  }
}

// decoder weight / bias gradients straight into G (natural layout): one
// workgroup per (token, n-half); the contraction runs over the batch's windows
// (rows: dpre[b], X2 row b*T + tok), staged through LDS like dw_kernel.
// Decoder weight gradient: for token tok (grid.x) and output-tile half y,
// sum over windows of dpre[b] (x) X2[b][tok].  The windows are split over
// grid.z = S parts (latency: one part is a short chain of LDS-staged chunks);
// S = 1 adds straight into G, otherwise each part writes its [NOP][DP] slab
// (and tok 0 its bias column) to `part` and dec_dw_sum adds them in part order.
template <int H>
__global__ __launch_bounds__(256) void dec_dw_kernel(int B, const float* __restrict__ dpre,
                                                     const float* __restrict__ X2, float* __restrict__ Gd,
                                                     float* __restrict__ part) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  constexpr int NP = Q::NOP, KP = Q::DP, NT = NP / 16, NTW = (NT + 7) / 8, KT = KP / 16;
  __shared__ __attribute__((aligned(16))) float ys[kDwRows * lds_stride(NP)];
  __shared__ __attribute__((aligned(16))) float xs[kDwRows * lds_stride(KP)];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  const int tok = blockIdx.x, y = blockIdx.y, z = blockIdx.z, S = gridDim.z;
  f32x4 acc[NTW][KT];
  float pb[NTW];
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    pb[q] = 0.f;
#pragma unroll
    for (int u = 0; u < KT; ++u) acc[q][u] = zero4();
  }
  const long nch = (B + kDwRows - 1) / kDwRows;
  const long r0 = nch * z / S * kDwRows, r1 = std::min<long>(B, nch * (z + 1) / S * kDwRows);
  dw_accumulate<NP, KP, NTW>(r0, r1, dpre, Q::NOP, X2 + (long)tok * Q::DP, (long)Q::T * Q::DP, 0, 4 * y, 8, ys, xs,
                             acc, pb);
  const int w = tok / H, h = tok - w * H;
  float* ps = part + ((long)z * Q::T + tok) * NP * KP;
  float* pbias = part + (long)S * Q::T * NP * KP + (long)z * NP;
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    const int t = 4 * y + wv + 8 * q;
    if (t < NT) {
#pragma unroll
      for (int u = 0; u < KT; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * t + 4 * g + r, c = 16 * u + i;
          if (S > 1) {
            ps[n * KP + c] = acc[q][u][r];
          } else if (n < 4 * H && c < H) {
            const long col = (long)h * 3 * H + w * H + c;
            Gd[(n < 2 * H ? G::W_AN + (long)n * G::L : G::W_PR + (long)(n - 2 * H) * G::L) + col] += acc[q][u][r];
          }
        }
      if (tok == 0) {
        const float sb = xsum(pb[q], true);
        const int n = 16 * t + i;
        if (S > 1) {
          if (g == 0) pbias[n] = sb;
        } else if (g == 0 && n < 4 * H) {
          Gd[n < 2 * H ? G::B_AN + n : G::B_PR + n - 2 * H] += sb;
        }
      }
    }
  }
}

// G += the S parts of dec_dw_kernel, summed in part order (one thread per
// decoder weight in G's own layout, so the adds into G are coalesced)
template <int H>
__global__ __launch_bounds__(256) void dec_dw_sum_kernel(int S, const float* __restrict__ part, float* __restrict__ Gd) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  constexpr int NP = Q::NOP, KP = Q::DP;
  constexpr long NW = 4L * H * G::L;  // anomaly rows then prototype rows, each [2H][L]
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx < NW) {
    const int n = (int)(idx / G::L);
    const long col = idx - (long)n * G::L;  // h*3H + w*H + c
    const int h = (int)(col / (3 * H)), rem = (int)(col - (long)h * 3 * H), w = rem / H, c = rem - w * H;
    const int tok = w * H + h;
    const float* src = part + ((long)tok * NP + n) * KP + c;
    float v = 0.f;
    for (int z = 0; z < S; ++z) v += src[(long)z * Q::T * NP * KP];
    Gd[(n < 2 * H ? G::W_AN + (long)n * G::L : G::W_PR + (long)(n - 2 * H) * G::L) + col] += v;
  } else if (idx < NW + 4 * H) {
    const int n = (int)(idx - NW);
    const float* src = part + (long)S * Q::T * NP * KP + n;
    float v = 0.f;
    for (int z = 0; z < S; ++z) v += src[(long)z * NP];
    Gd[n < 2 * H ? G::B_AN + n : G::B_PR + n - 2 * H] += v;
  }
}

// ============================================================================
// host side
// ============================================================================
#define TCK(expr)                          \
  do {                                     \
    expr;                                  \
    const hipError_t e_ = hipGetLastError(); \
    if (e_ != hipSuccess) return e_;       \
  } while (0)

LinArgs lin_args(long M, const float* X, int ldx, const float* W, int ldw, int N, int K, int trans, const float* bias,
                 float* Y, int ldy) {
  LinArgs a{};
  a.M = M;
  a.X = X;
  a.ldx = ldx;
  a.W = W;
  a.ldw = ldw;
  a.N = N;
  a.K = K;
  a.trans = trans;
  a.bias = bias;
  a.Y = Y;
  a.ldy = ldy;
  a.rss = 1;
  return a;
}

template <int NP, int KP, int EPI>
hipError_t lin(const TunePlan& p, const LinArgs& a, hipStream_t st) {
  TCK((linear_kernel<NP, KP, EPI><<<p.lin_grid, 256, 0, st>>>(a)));
  return hipSuccess;
}

// The backward's weight-gradient reductions, deferred to one pair of launches at
// its end (nothing in the backward reads a weight gradient).  Each deferred
// reduction gets its own partial and level-2 regions from the plan's pool.
struct RedBatch {
  float* pool;
  long cap;
  long used = 0;
  RedTable l1{}, l2{};
  int gx1 = 0, gx2 = 0, ny1 = 1;
  float* take(long n) {
    float* r = pool + used;
    used += (n + 63) / 64 * 64;
    return r;
  }
  bool add(int nparts, long pstride, const float* part, int rows, int cols, int ldp, float* outA, int ldo, int nb,
           long srcb, float* outB) {
    if (l1.n >= kMaxRedSeg) return false;
    const long nout = (long)rows * cols + nb;
    const int gx = (int)((nout + 63) / 64);
    const int nsplit = (nparts + kRedChunk - 1) / kRedChunk;
    RedArgs a{nparts, nparts, pstride, part, rows, cols, ldp, ldo, nb, srcb, outA, outB, nullptr};
    if (nsplit > 1) {
      a.pc = kRedChunk;
      a.lvl2 = take((long)nsplit * nout);
      l2.seg[l2.n] = RedArgs{nsplit, nsplit, nout, a.lvl2, rows, cols, cols, ldo, nb, (long)rows * cols,
                             outA, outB, nullptr};
      l2.nsplit[l2.n] = 1;
      l2.bx0[l2.n] = gx2;
      gx2 += gx;
      ++l2.n;
    }
    l1.seg[l1.n] = a;
    l1.nsplit[l1.n] = nsplit;
    l1.bx0[l1.n] = gx1;
    gx1 += gx;
    ny1 = std::max(ny1, nsplit);
    ++l1.n;
    return used <= cap;
  }
  hipError_t flush(hipStream_t st) {
    if (used > cap) return hipErrorInvalidValue;  // the plan's pool is too small (a bug): fail loudly
    l1.bx0[l1.n] = gx1;
    l2.bx0[l2.n] = gx2;
    if (l1.n) TCK((reduce_multi_kernel<<<dim3(gx1, ny1), 256, 0, st>>>(l1)));
    if (l2.n) TCK((reduce_multi_kernel<<<gx2, 256, 0, st>>>(l2)));
    return hipSuccess;
  }
};

// dW[N][K] (row stride K) += sum_m Y[m][n] X[m][k];  db[N] += sum_m Y[m][n]
// (partial slabs from the pool; the reduction is deferred to rb.flush)
template <int NP, int KP>
hipError_t dw(const TunePlan& p, RedBatch& rb, const float* Y, int ldy, const float* X, int ldx, int relu, int N,
              int K, float* gW, float* gb, hipStream_t st) {
  const long pstride = (long)NP * KP + NP;
  float* part = rb.take((long)p.dw_grid * pstride);
  DwArgs a{p.M, Y, ldy, X, ldx, relu, part};
  TCK((dw_kernel<NP, KP><<<p.dw_grid, 256, 0, st>>>(a)));
  return rb.add(p.dw_grid, pstride, part, N, K, KP, gW, K, gb ? N : 0, (long)NP * KP, gb) ? hipSuccess
                                                                                          : hipErrorInvalidValue;
}

// gamma / beta gradients from LNB partials [nparts][2][DP] (deferred)
hipError_t ln_grads(const TunePlan& p, RedBatch& rb, int nparts, const float* part, int N, float* gw, float* gb) {
  return rb.add(nparts, 2L * p.DP, part, 1, N, 0, gw, 0, N, p.DP, gb) ? hipSuccess : hipErrorInvalidValue;
}

template <int H>
bool plan_h(int B, TunePlan* out) {
  using Q = TuneGeo<H>;
  TunePlan q;
  q.H = H;
  q.B = B;
  q.M = (long)B * Q::T;
  q.DP = Q::DP;
  q.Q3P = Q::Q3P;
  q.NOP = Q::NOP;
  q.KD = Q::KD;
  long off = 0;
  auto take = [&](long n) {
    const long o = off;
    off += (n + 63) / 64 * 64;
    return o;
  };
  const long M = q.M;
  q.win = take((long)B * 9 * H);
  q.g = take(M * Q::DP);
  q.xb = take(M * Q::XBP);
  q.gs = take(3L * B * 4);
  for (int i = 0; i < 3; ++i) q.x[i] = take(M * Q::DP);
  for (int l = 0; l < 2; ++l) {
    q.qkv[l] = take(M * Q::Q3P);
    q.o[l] = take(M * Q::DP);
    q.pr[l] = take(M * 8);
    q.xh1[l] = take(M * Q::DP);
    q.rs1[l] = take(M);
    q.y1[l] = take(M * Q::DP);
    q.f[l] = take(M * Q::FF);
    q.xh2[l] = take(M * Q::DP);
    q.rs2[l] = take(M);
  }
  q.da = take(M * Q::DP);
  q.db = take(M * Q::DP);
  q.dq = take(M * Q::Q3P);
  q.df = take(M * Q::FF);
  q.gsx = take(3L * B * 8);
  q.dpre = take((long)B * Q::NOP);
  q.wp = take((long)Q::NOP * Q::KD);
  q.wpt = take((long)Q::NOP * Q::KD);
  const long nrb = (M + 15) / 16;
  q.lin_grid = (int)std::min<long>(PGP_LIN_CAP, std::max<long>(1, (nrb + 3) / 4));
  q.dw_grid = (int)std::min<long>(PGP_DW_CAP, std::max<long>(1, (nrb + 7) / 8));
  q.dec_bg = (B + 63) / 64;
  q.dec_dxg = (int)std::min<long>(4, (B + 63) / 64);
  const long kbt = Q::KD / 16;
  q.dec_s = (int)std::max<long>(1, std::min<long>(kbt, 512 / q.dec_bg));
  // partial slabs; every bound grows with B, so a workspace sized for B_max serves any B <= B_max
  const long np_max = std::max(Q::Q3P, 64);
  long part = (long)PGP_LIN_CAP * 2 * Q::DP;                             // linear LNB, one per workgroup
  part = std::max(part, (long)PGP_DW_CAP * (np_max * 64 + np_max));       // dW slabs
  part = std::max(part, std::max(512L, (long)q.dec_bg) * 64 * Q::NOP);    // decoder split-K
  part = std::max(part, (long)Q::T * 8 * 2 * Q::DP);                      // decoder dX LNB (<= 8 x T groups)
  // decoder weight gradient: windows split over up to 4 parts of >= 8 chunks
  q.dec_dws = (int)std::max<long>(1, std::min<long>(4, (B + kDwRows - 1) / kDwRows / 8));
  if (q.dec_dws > 1) part = std::max(part, (long)q.dec_dws * (Q::T * Q::NOP * Q::DP + Q::NOP));
  q.part = take(part);
  // the backward's deferred reductions (RedBatch): each dW / LN-gradient partial
  // region plus its level-2 region, in the order tune_bwd_h takes them
  {
    long pool = 0;
    auto r64 = [](long n) { return (n + 63) / 64 * 64; };
    auto red = [&](long nparts, long slab, long nout) {
      pool += r64(nparts * slab);
      const long ns = (nparts + 255) / 256;
      if (ns > 1) pool += r64(ns * nout);
    };
    auto dwr = [&](long np, long kp, long n, long k, bool bias) { red(q.dw_grid, np * kp + np, n * k + (bias ? n : 0)); };
    const long DPl = Q::DP, FFl = Q::FF, Q3Pl = Q::Q3P, Hl = H;
    red((long)q.dec_dxg * Q::T, 2 * DPl, 2 * Hl);  // decoder dX through layer 1's norm2
    for (int l = 1; l >= 0; --l) {
      dwr(DPl, FFl, Hl, FFl, true);        // W2
      dwr(FFl, DPl, FFl, Hl, true);        // W1
      red(q.lin_grid, 2 * DPl, 2 * Hl);    // norm1
      dwr(DPl, DPl, Hl, Hl, true);         // out_proj
      dwr(Q3Pl, DPl, 3 * Hl, Hl, true);    // in_proj
      if (l == 1) red(q.lin_grid, 2 * DPl, 2 * Hl);  // layer 0's norm2
    }
    dwr(DPl, DPl, Hl, Hl, true);           // time encoder
    dwr(DPl, Q::XBP, Hl, 3, false);        // GAT fc
    q.pool = take(pool);
    q.pool_len = pool;
  }
  q.total = off;
  *out = q;
  return true;
}

template <int H>
hipError_t tune_fwd_h(const TunePlan& p, const float* win, const float* P, float* ws, float* latent, float* logits,
                      float* protos, hipStream_t st) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  constexpr int DP = Q::DP, Q3P = Q::Q3P, FF = Q::FF;
  const int B = p.B;
  const long M = p.M;
  hipError_t e;
  TCK((dec_pack_kernel<H><<<(int)((Q::NOP * Q::KD + 255) / 256), 256, 0, st>>>(P, ws + p.wp, ws + p.wpt)));
  TCK((gat_fwd_kernel<H><<<(3 * B + 3) / 4, 256, 0, st>>>(B, win, P, ws + p.win, ws + p.g, ws + p.xb, ws + p.gs)));
  {  // time encoder + positional encoding (models.py:390-393)
    LinArgs a = lin_args(M, ws + p.g, DP, P + G::W_TE, H, H, H, 0, P + G::B_TE, ws + p.x[0], DP);
    a.pe = P + G::PE;
    a.H = H;
    if ((e = lin<DP, DP, EPI_PE>(p, a, st)) != hipSuccess) return e;
  }
  for (int l = 0; l < 2; ++l) {
    const float* Lp = P + G::LAY0 + l * G::L_SIZE;
    LinArgs a = lin_args(M, ws + p.x[l], DP, Lp + G::L_IN, H, 3 * H, H, 0, Lp + G::L_INB, ws + p.qkv[l], Q3P);
    if ((e = lin<Q3P, DP, EPI_STORE>(p, a, st)) != hipSuccess) return e;
    TCK((attn_fwd_kernel<H><<<(int)(((long)B * H * 32 + 255) / 256), 256, 0, st>>>(B, ws + p.qkv[l], ws + p.o[l],
                                                                                      ws + p.pr[l])));
    a = lin_args(M, ws + p.o[l], DP, Lp + G::L_OUT, H, H, H, 0, Lp + G::L_OUTB, ws + p.y1[l], DP);
    a.R = ws + p.x[l];
    a.ldr = DP;
    a.lnw = Lp + G::L_N1W;
    a.lnb = Lp + G::L_N1B;
    a.XH = ws + p.xh1[l];
    a.RS = ws + p.rs1[l];
    if ((e = lin<DP, DP, EPI_LN>(p, a, st)) != hipSuccess) return e;
    a = lin_args(M, ws + p.y1[l], DP, Lp + G::L_W1, H, FF, H, 0, Lp + G::L_B1, ws + p.f[l], FF);
    if ((e = lin<FF, DP, EPI_STORE>(p, a, st)) != hipSuccess) return e;
    a = lin_args(M, ws + p.f[l], FF, Lp + G::L_W2, FF, H, FF, 0, Lp + G::L_B2, ws + p.x[l + 1], DP);
    a.relu_x = 1;
    a.R = ws + p.y1[l];
    a.ldr = DP;
    a.lnw = Lp + G::L_N2W;
    a.lnb = Lp + G::L_N2B;
    a.XH = ws + p.xh2[l];
    a.RS = ws + p.rs2[l];
    if ((e = lin<DP, FF, EPI_LN>(p, a, st)) != hipSuccess) return e;
  }
  TCK((dec_fwd_kernel<H><<<dim3(p.dec_bg, p.dec_s), 256, 0, st>>>(B, p.dec_s, ws + p.x[2], ws + p.wp,
                                                                   ws + p.part)));
  TCK((dec_fin_kernel<H><<<(int)(((long)B * 4 * H + 255) / 256), 256, 0, st>>>(B, p.dec_s, ws + p.part, P, logits,
                                                                                protos)));
  if (latent)
    TCK((latent_kernel<H><<<(int)(((long)B * 3 * H * H + 255) / 256), 256, 0, st>>>(B, ws + p.x[2], latent)));
  return hipSuccess;
}

template <int H>
hipError_t tune_bwd_h(const TunePlan& p, const float* P, float* Gd, float* ws, const float* logits,
                      const float* protos, const int* y, const float* mult, const float* tgt, hipStream_t st) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  constexpr int DP = Q::DP, Q3P = Q::Q3P, FF = Q::FF;
  const int B = p.B;
  const long M = p.M;
  hipError_t e;
  RedBatch rb{ws + p.pool, p.pool_len};
  TCK((tune_loss_kernel<<<(int)(((long)B * H + 255) / 256), 256, 0, st>>>(B, H, Q::NOP, logits, protos, y, mult,
                                                                           tgt, ws + p.dpre)));
  TCK((dec_dw_kernel<H><<<dim3(Q::T, 2, p.dec_dws), 256, 0, st>>>(B, ws + p.dpre, ws + p.x[2], Gd, ws + p.part)));
  if (p.dec_dws > 1) {
    const long nw = 4L * H * G::L + 4 * H;
    TCK((dec_dw_sum_kernel<H><<<(int)((nw + 255) / 256), 256, 0, st>>>(p.dec_dws, ws + p.part, Gd)));
  }
  {  // grad of the encoder output = dpre . Wp (token layout), through layer 1's norm2: one
     // linear layer per token (grid.y) with that token's [DP][NOP] slab of Wp^T in LDS
    const float* L1 = P + G::LAY0 + G::L_SIZE;
    float* L1g = Gd + G::LAY0 + G::L_SIZE;
    LinArgs a = lin_args(B, ws + p.dpre, Q::NOP, ws + p.wpt, Q::NOP, H, 4 * H, 0, nullptr, ws + p.da, Q::T * DP);
    a.frag = 1;
    a.XH = ws + p.xh2[1];
    a.RS = ws + p.rs2[1];
    a.rss = Q::T;
    a.lnw = L1 + G::L_N2W;
    a.part = rb.take((long)p.dec_dxg * Q::T * 2 * DP);
    a.bw = (long)DP * Q::NOP;
    a.by = a.bxh = DP;
    a.brs = 1;
    TCK((linear_kernel<DP, Q::NOP, EPI_LNB><<<dim3(p.dec_dxg, Q::T), 256, 0, st>>>(a)));
    if ((e = ln_grads(p, rb, p.dec_dxg * Q::T, a.part, H, L1g + G::L_N2W, L1g + G::L_N2B)) != hipSuccess) return e;
  }
  const int lnb_parts = p.lin_grid;
  for (int l = 1; l >= 0; --l) {
    const float* Lp = P + G::LAY0 + l * G::L_SIZE;
    float* Lg = Gd + G::LAY0 + l * G::L_SIZE;
    // da = grad of R2 = Y1 + relu(F) W2^T + b2
    if ((e = dw<DP, FF>(p, rb, ws + p.da, DP, ws + p.f[l], FF, 1, H, FF, Lg + G::L_W2, Lg + G::L_B2, st)) !=
        hipSuccess)
      return e;
    LinArgs a = lin_args(M, ws + p.da, DP, Lp + G::L_W2, FF, FF, H, 1, nullptr, ws + p.df, FF);
    a.R = ws + p.f[l];
    a.ldr = FF;
    if ((e = lin<FF, DP, EPI_MASK>(p, a, st)) != hipSuccess) return e;
    if ((e = dw<FF, DP>(p, rb, ws + p.df, FF, ws + p.y1[l], DP, 0, FF, H, Lg + G::L_W1, Lg + G::L_B1, st)) !=
        hipSuccess)
      return e;
    // db = grad of R1: (dF W1 + dR2) through norm1
    a = lin_args(M, ws + p.df, FF, Lp + G::L_W1, H, H, FF, 1, nullptr, ws + p.db, DP);
    a.R = ws + p.da;
    a.ldr = DP;
    a.XH = ws + p.xh1[l];
    a.RS = ws + p.rs1[l];
    a.lnw = Lp + G::L_N1W;
    a.part = rb.take((long)lnb_parts * 2 * DP);
    if ((e = lin<DP, FF, EPI_LNB>(p, a, st)) != hipSuccess) return e;
    if ((e = ln_grads(p, rb, lnb_parts, a.part, H, Lg + G::L_N1W, Lg + G::L_N1B)) != hipSuccess) return e;
    if ((e = dw<DP, DP>(p, rb, ws + p.db, DP, ws + p.o[l], DP, 0, H, H, Lg + G::L_OUT, Lg + G::L_OUTB, st)) !=
        hipSuccess)
      return e;
    // da = grad of the attention output
    a = lin_args(M, ws + p.db, DP, Lp + G::L_OUT, H, H, H, 1, nullptr, ws + p.da, DP);
    if ((e = lin<DP, DP, EPI_STORE>(p, a, st)) != hipSuccess) return e;
    TCK((attn_bwd_kernel<H><<<(int)(((long)B * H * 32 + 255) / 256), 256, 0, st>>>(B, ws + p.qkv[l], ws + p.pr[l],
                                                                                       ws + p.da, ws + p.dq)));
    if ((e = dw<Q3P, DP>(p, rb, ws + p.dq, Q3P, ws + p.x[l], DP, 0, 3 * H, H, Lg + G::L_IN, Lg + G::L_INB, st)) !=
        hipSuccess)
      return e;
    // grad of the layer input: dQKV Win + dR1 (residual); for l = 1 through layer 0's norm2
    a = lin_args(M, ws + p.dq, Q3P, Lp + G::L_IN, H, H, 3 * H, 1, nullptr, ws + p.da, DP);
    a.R = ws + p.db;
    a.ldr = DP;
    if (l == 1) {
      const float* L0 = P + G::LAY0;
      float* L0g = Gd + G::LAY0;
      a.XH = ws + p.xh2[0];
      a.RS = ws + p.rs2[0];
      a.lnw = L0 + G::L_N2W;
      a.part = rb.take((long)lnb_parts * 2 * DP);
      if ((e = lin<DP, Q3P, EPI_LNB>(p, a, st)) != hipSuccess) return e;
      if ((e = ln_grads(p, rb, lnb_parts, a.part, H, L0g + G::L_N2W, L0g + G::L_N2B)) != hipSuccess) return e;
    } else {
      if ((e = lin<DP, Q3P, EPI_RES>(p, a, st)) != hipSuccess) return e;
    }
  }
  // time encoder: da = grad of X0
  if ((e = dw<DP, DP>(p, rb, ws + p.da, DP, ws + p.g, DP, 0, H, H, Gd + G::W_TE, Gd + G::B_TE, st)) != hipSuccess)
    return e;
  {
    LinArgs a = lin_args(M, ws + p.da, DP, P + G::W_TE, H, H, H, 1, nullptr, ws + p.db, DP);
    if ((e = lin<DP, DP, EPI_STORE>(p, a, st)) != hipSuccess) return e;
  }
  // GAT: db = grad of the GAT output
  TCK((gat_bwd_kernel<H><<<(3 * B + 3) / 4, 256, 0, st>>>(B, ws + p.win, P, ws + p.db, ws + p.gs, ws + p.gsx)));
  if ((e = dw<DP, Q::XBP>(p, rb, ws + p.db, DP, ws + p.xb, Q::XBP, 0, H, 3, Gd + G::W_FC, nullptr, st)) !=
      hipSuccess)
    return e;
  TCK((gat_param_kernel<H><<<1, 256, 0, st>>>(3 * B, ws + p.gsx, P, Gd)));
  return rb.flush(st);  // every deferred weight-gradient reduction: 2 launches
}

}  // namespace

bool tune_plan(int H, int B, TunePlan* p) {
  if (B < 1) return false;
  switch (H) {
#define CASE(h) \
  case h:       \
    return plan_h<h>(B, p);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return false;
}

hipError_t launch_tune_forward(const TunePlan& p, const float* windows, const float* P, float* ws, float* latent,
                               float* logits, float* protos, hipStream_t st) {
  switch (p.H) {
#define CASE(h) \
  case h:       \
    return tune_fwd_h<h>(p, windows, P, ws, latent, logits, protos, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_tune_backward(const TunePlan& p, const float* P, float* G, float* ws, const float* logits,
                                const float* protos, const int* y, const float* mult, const float* tgt,
                                hipStream_t st) {
  switch (p.H) {
#define CASE(h) \
  case h:       \
    return tune_bwd_h<h>(p, P, G, ws, logits, protos, y, mult, tgt, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// custom_loss / triplet_loss host bookkeeping of ONE window (train.py:13-40),
// on the device so that a backprop() loop of sequential batch-1 steps needs no
// host round trip between steps.  The logic is inherently sequential (the
// prototype EMA of host i feeds the targets of host i+1), so one lane runs it,
// in fp64 and in the reference's operation order, with FMA contraction off:
// every value matches the numpy restatement (train.loss_targets) bit for bit,
// except the reported loss values, which go through device log/exp.
//   state [2K+3] fp64: prototypes [K][2] (model.prototype, K = n_hosts for the
//                   Transformer, models.py:373; triplet_loss reads and updates
//                   rows 0-2 only), PROTO_UPDATE_FACTOR, num_zero, num_ones
//                   (train.py's module globals)
//   outputs: mult [H] and tgt [H][2] (fp32, as pgp_tune_backward takes them),
//            loss [2] fp64 = (aloss, tloss) of the window
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void tune_targets_kernel(int H, int K, const float* __restrict__ logits,
                                                          const float* __restrict__ protos, const int* __restrict__ y,
                                                          const int* __restrict__ cls, double* __restrict__ state,
                                                          double update_min, double decay, float* __restrict__ mult,
                                                          float* __restrict__ tgt, double* __restrict__ loss) {
  if (threadIdx.x != 0) return;
  tune_targets_one(H, K, logits, protos, y, cls, state, update_min, decay, mult, tgt, loss);
}

hipError_t launch_tune_targets(int H, int K, const float* logits, const float* protos, const int* y, const int* cls,
                               double* state, double update_min, double decay, float* mult, float* tgt, double* loss,
                               hipStream_t st) {
  tune_targets_kernel<<<1, 64, 0, st>>>(H, K, logits, protos, y, cls, state, update_min, decay, mult, tgt, loss);
  return hipGetLastError();
}

}  // namespace pgp
