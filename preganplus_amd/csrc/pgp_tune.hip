// pgp_tune.hip — the semi-supervised tuning step (train.py:42-57): forward with
// checkpoints and backward of the PreGAN+ Transformer (models.py:376-416) over
// a batch of windows.
//
// The encoder layers run as fused per-unit kernels (pgp_tunef.hip: every
// activation of a layer in MFMA registers, weight gradients contracted in
// registers / LDS).  Around them, token-major kernels over the batch's M = B*3H
// tokens ([M][ld] rows, pgp_tune.hpp): the GAT aggregation and its backward
// (one wave per (window, step)), the time encoder's input gradient (a linear
// layer on v_mfma_f32_16x16x4_f32, weights as the A operand staged in LDS,
// 16 token rows per wave as B), the weight-gradient contractions that stay
// tall (in_proj over dQKV, time encoder, GAT fc: partial slabs over
// workgroups), and the decoders, which contract over a window's whole encoder
// output (3H x DP, token layout) as split-K GEMMs on a permuted copy of their
// weights.  Every weight-gradient reduction is deferred to the end of the
// backward and runs in a fixed order (deterministic).
//
// Deviations from the reference's op order are algebraic only: the GAT
// aggregates the raw features (sum_i a_ij x_i, then fc) instead of fc(x_i)
// (dlutils.py:315-342), and the edge scores use u.x_i + v.x_j with u = fc^T a_1
// (dlutils.py:326-329); the result is the same function, rounded once in fp32.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <mutex>

#include <algorithm>

#include "pgp_device.hpp"
#include "pgp_gemm.hpp"
#include "pgp_train.hpp"
#include "pgp_tune.hpp"
#include "pgp_tunedp.hpp"
#include "pgp_tunef.hpp"
#include "pgp_tunetargets.hpp"


namespace pgp {
namespace {

// workgroups of the token-major GEMMs / weight-gradient kernels (grid-stride loops)
constexpr int kLinCap = 512, kDwCap = 512;

enum : int { EPI_STORE = 0 };

// ============================================================================
// Linear layer over all tokens: Y = X . W'^T (+ bias), W' = W (trans 0,
// W[n][k] = W[n*ldw+k]) or W^T (trans 1, W'[n][k] = W[k*ldw+n]).  Used for the
// decoders' input gradient (per token, batched over grid.y) and the time
// encoder's.
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
  // batched launch (grid.y = batch index): offsets of W and Y per batch entry
  long bw, by;
  int frag;  // W points at W' pre-packed as [NP/16][KP/16][64 lanes][4] fragments
};

template <int NP, int KP, int EPI>
__global__ __launch_bounds__(256, 2) void linear_kernel(LinArgs a) {
  static_assert(EPI == EPI_STORE, "store epilogue only");
  constexpr int NT = NP / 16, KB = KP / 16;
  __shared__ f32x4 wl[NT * KB * 64];
  __shared__ float cb[NP];
  float* wf_flat = reinterpret_cast<float*>(wl);
  const float* Wb = a.W + blockIdx.y * a.bw;
  float* Yb = a.Y + blockIdx.y * a.by;
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
  for (int n = threadIdx.x; n < NP; n += 256) cb[n] = (a.bias && n < a.N) ? a.bias[n] : 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, mi = lane & 15;
  const long nrb = (a.M + 15) >> 4;
  // B-operand k-blocks are prefetched PF ahead (a ring of registers), so a
  // wave keeps several HBM loads in flight; wide layers (NT > 4) keep the LDS
  // fragments out of registers with a short unroll.  The next row block's first
  // PF k-blocks are loaded while the current one computes.
  constexpr int PF = NT > 4 ? (KB < 2 ? KB : 2) : (KB < 4 ? KB : 4);
  const long rstep = (long)gridDim.x * 4;
  f32x4 xq[PF];
  // rows past M read row 0 (the address is clamped: a select on the loaded
  // value would wait for the prefetch at once); their columns are not stored
  {
    const long m0 = ((long)blockIdx.x * 4 + wv) * 16 + mi;
#pragma unroll
    for (int j = 0; j < PF; ++j) xq[j] = ld4(a.X + (m0 < a.M ? m0 : 0) * a.ldx + 4 * g + 16 * j);
  }
  for (long rb = (long)blockIdx.x * 4 + wv; rb < nrb; rb += rstep) {
    const long m = rb * 16 + mi;
    const bool ok = m < a.M;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = *reinterpret_cast<const f32x4*>(&cb[16 * t + 4 * g]);
    const float* xr = a.X + (ok ? m : 0) * a.ldx + 4 * g;
    f32x4 xn[PF];
    {
      const long mn = m + rstep * 16;
#pragma unroll
      for (int j = 0; j < PF; ++j) xn[j] = ld4(a.X + (mn < a.M ? mn : 0) * a.ldx + 4 * g + 16 * j);
    }
#pragma unroll 1
    for (int j0 = 0; j0 < KB; j0 += PF) {
#pragma unroll
      for (int jj = 0; jj < PF; ++jj) {
        const int j = j0 + jj;
        if (j < KB) {
          f32x4 xv = xq[jj];
          if (j + PF < KB) xq[jj] = ld4(xr + 16 * (j + PF));
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
    if (ok) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(yr + 16 * t, acc[t]);
    }
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

// rows per staged chunk: 64-row chunks (one barrier pair per 64 rows, twice
// the registers in flight) were slower for every shape (A/B at H = 50: C3
// 1.287 -> 1.307-1.312 ms, in_proj dW 53 -> 85 us; profiles/r04/dw_rows/)
constexpr int dw_rows(int) { return kDwRows; }
// block bx of nbx (the rows split evenly over the blocks), LDS staging ys / xs
template <int NP, int KP>
PGP_DEV void dw_block(const DwArgs& a, int bx, int nbx, float* ys, float* xs) {
  constexpr int NT = NP / 16, KT = KP / 16, NTW = (NT + 3) / 4, ROWS = dw_rows(NP);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  f32x4 acc[NTW][KT];
  float pb[NTW];
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    pb[q] = 0.f;
#pragma unroll
    for (int u = 0; u < KT; ++u) acc[q][u] = zero4();
  }
  const long nch = (a.M + ROWS - 1) / ROWS;
  const long r0 = nch * bx / nbx * ROWS;
  const long r1 = std::min<long>(a.M, nch * (bx + 1) / nbx * ROWS);
  dw_accumulate<NP, KP, NTW, ROWS>(r0, r1, a.Y, a.ldy, a.X, a.ldx, a.relu_x, 0, 4, ys, xs, acc, pb);
  float* P = a.part + (long)bx * (NP * KP + NP);
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
template <int NP, int KP>
__global__ __launch_bounds__(256) void dw_kernel(DwArgs a) {
  constexpr int ROWS = dw_rows(NP);
  __shared__ __attribute__((aligned(16))) float ys[ROWS * lds_stride(NP)];
  __shared__ __attribute__((aligned(16))) float xs[ROWS * lds_stride(KP)];
  dw_block<NP, KP>(a, blockIdx.x, gridDim.x, ys, xs);
}
// Several weight gradients in ONE launch (the backward's without a side
// stream: in_proj of both layers, the time encoder, the GAT fc aggregation):
// segment s takes blocks [s * nbx, (s + 1) * nbx), each block exactly as its
// own dw_kernel launch would run it (same rows, same slab), so the partials
// are bit-identical.  Shapes: kind 0 = <3 DP, DP>, 1 = <DP, DP>, 2 = <DP, XBP>.
constexpr int kMaxDwSeg = 4;
// the decoders' weight gradient (dec_dw_block): windows split over S parts,
// one block per (token, n-half, part)
struct DecDwArgs {
  int B, S;
  const float* dpre;
  const float* X2;
  float* Gd;
  float* part;
  unsigned* counter;
};
template <int H>
PGP_DEV void dec_dw_block(const DecDwArgs& d, int tok, int y, int z, float* ys, float* xs);
struct DwMulti {
  int n, nbx;
  int kind[kMaxDwSeg];
  DwArgs seg[kMaxDwSeg];
  int gat_nb;  // leading blocks running the GAT backward (0: none)
  int dec_nb;  // then blocks running the decoders' weight gradient (0: none)
  DecDwArgs dec;
};

// Deterministic reduction of partial slabs.  Outputs: segment A, rows x cols
// (source i*ldp + j, destination outA[i*ldo + j]) then segment B, nb values
// (source srcb + j, destination outB[j]); each sums part[p*pstride + src] over
// p in [y*pc, (y+1)*pc) of this block's split y — 4 lane groups x 4 independent
// chains, a fixed order — and adds into the destination (one split) or writes
// lvl2[y][o] for a second pass.
// parts per split of one reduction: the step's dW slabs (<= kDwCap = 512) and the
// fused launches' slabs (<= one per CU) reduce in ONE level (one launch of
// reduce_multi_kernel, not two)
constexpr int kRedChunk = 512;
struct RedArgs {
  int nparts, pc;
  long pstride;
  const float* part;
  int rows, cols, ldp, ldo, nb;
  long srcb;
  float* outA;
  float* outB;
  float* lvl2;
  int wt = 0;  // outputs stored write-through (read by the launch's last workgroup)
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
    // 16 loads in flight per lane, then their adds in the same order as the
    // loop below (a part count of hundreds was otherwise ~25 dependent memory
    // rounds of 4 loads: reduce_multi 13 us per C3 step at H = 16)
    for (; p + 60 < p1; p += 64) {
      float v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = sp[(long)(p + 4 * q) * a.pstride];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s0 += v[4 * q];
        s1 += v[4 * q + 1];
        s2 += v[4 * q + 2];
        s3 += v[4 * q + 3];
      }
    }
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
    float* dst;
    if (a.lvl2) {
      dst = a.lvl2 + by * nout + o;
    } else if (o < na) {
      const int i = (int)(o / a.cols), j = (int)(o - (long)i * a.cols);
      dst = a.outA + (long)i * a.ldo + j;
    } else {
      dst = a.outB + (o - na);
    }
    if (a.wt)
      store_wt(dst, t);
    else
      *dst = t;
  }
}
__global__ __launch_bounds__(256) void reduce_kernel(RedArgs a) { reduce_block(a, blockIdx.x, blockIdx.y); }

// Up to kMaxRedSeg reductions in one launch (the backward defers every weight-
// gradient reduction to its end): block x -> (segment, local block) by the
// prefix table, y = split; a segment's blocks run reduce_block exactly as its own
// reduce_kernel launch would, so the sums are bit-identical.
constexpr int kMaxRedSeg = 20;
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
// Each wave forms the fold itself: lane c loads row c of fc and both attn_fc
// weights (one round of loads for the whole wave) and the six sums are wave
// butterflies.  (A serial loop over c issued 50 dependent rounds of loads per
// wave: most of gat_fwd's and gat_bwd's time at H = 50.)  The same function in
// the forward and the backward, so both see the same u, v.
template <int H>
PGP_DEV GatFold<H> gat_fold(const float* P) {
  using G = TGeo<H>;
  static_assert(H <= 64, "one host per lane");
  const int c = threadIdx.x & 63;
  const bool ok = c < H;
  const float a_s = ok ? P[G::W_ATT + c] : 0.f, a_d = ok ? P[G::W_ATT + H + c] : 0.f;
  GatFold<H> f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float fc = ok ? P[G::W_FC + c * 3 + k] : 0.f;
    f.u[k] = wave_sum(a_s * fc);
    f.v[k] = wave_sum(a_d * fc);
  }
  return f;
}

// node factors of the factorised edge exponentials: for source i (s) and
// destination j (t), exp(lrelu(s_i + t_j) - mx) = max(a_i * b_j, an_i * bn_j)
// (exp is monotone and lrelu(e) = max(e, 0.01 e)); with smax = max_i s_i and
// mx = lrelu(smax + tmax) every factor is <= 1, so none overflows and an
// underflow only drops an edge below 1e-38 of the largest.  4 exponentials per
// node instead of H per edge row.
struct GatEdge {
  float a, an, b, bn;
};
PGP_DEV GatEdge gat_edge(float s, float t, float smax, float mx) {
  GatEdge e;
  e.a = expf(s - smax);
  e.an = expf(0.01f * (s - smax));
  e.b = expf(t + smax - mx);
  e.bn = expf(0.01f * (t + smax) - mx);
  return e;
}

struct GatFwdIn {
  int B;
  const float* win;
  float *wcopy, *Gout, *XB, *GS;
};
template <int H>
PGP_DEV void gat_fwd_block(int bx, int B, const float* __restrict__ win, const float* __restrict__ P,
                           float* __restrict__ wcopy, float* __restrict__ Gout, float* __restrict__ XB,
                           float* __restrict__ GS) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  __shared__ float sa[4][64][2], sx[4][64][3], sxb[4][64][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long pw = (long)bx * 4 + wv;  // (window, step)
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
  // the H^2 edge exponentials factorise (as K1's, pgp_gat.hip):
  // exp(lrelu(s_i + t_j) - mx) = max(A_i B_j, A'_i B'_j), every factor <= 1
  const GatEdge ge = gat_edge(s, t, smax, mx);
  sa[wv][j][0] = ge.a;
  sa[wv][j][1] = ge.an;
#pragma unroll
  for (int k = 0; k < 3; ++k) sx[wv][j][k] = x[k];
  __syncthreads();
  float sum = 0.f, xb[3] = {0.f, 0.f, 0.f};
  if (okj)
#pragma unroll 10
    for (int i = 0; i < H; ++i) {
      const float p = fmaxf(sa[wv][i][0] * ge.b, sa[wv][i][1] * ge.bn);  // graph-wise softmax_edges (dlutils.py:335)
      sum += p;
#pragma unroll
      for (int k = 0; k < 3; ++k) xb[k] = fmaf(p, sx[wv][i][k], xb[k]);
    }
  const float Z = wave_sum(sum);
  const float iz = 1.0f / Z;
  const long m0 = b * Q::T + (long)w * H;  // token row of host 0
  if (okj) {
#pragma unroll
    for (int k = 0; k < 3; ++k) xb[k] *= iz;
#pragma unroll
    for (int k = 0; k < 3; ++k) XB[(m0 + j) * Q::XBP + k] = xb[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) sxb[wv][j][k] = xb[k];
  __syncthreads();
  // G rows = fc x-bar, written row-coalesced: lane (rr, q) computes features
  // 4q .. 4q+3 of rows rr, rr+4, ...; the feature pads come out 0 (fc is 0
  // there) and are written too (the fused encoder reads whole DP rows)
  if (okw) {
    const int q = lane & 15, rr = lane >> 4;
    if (4 * q < Q::DP) {
      float fc[4][3];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int k = 0; k < 3; ++k) fc[e][k] = 4 * q + e < H ? P[G::W_FC + (4 * q + e) * 3 + k] : 0.f;
      for (int r = rr; r < H; r += 4) {
        const float x0 = sxb[wv][r][0], x1 = sxb[wv][r][1], x2 = sxb[wv][r][2];
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(fc[e][0], x0, fmaf(fc[e][1], x1, fc[e][2] * x2));
        st4(Gout + (m0 + r) * Q::DP + 4 * q, v);
      }
    }
  }
  if (okw && lane == 0) {
    GS[pw * 4] = mx;
    GS[pw * 4 + 1] = Z;
  }
}

// GAT backward from dX0, the gradient of the time encoder's output: the time
// encoder X0 = G W_TE^T + b is linear, so the gradient of the aggregated raw
// features x-bar_j = fc^T dG_j = fc^T W_TE^T dX0_j = Mt^T dX0_j with
// Mt = W_TE fc ([64][3], formed by the forward's packing launch); no dG round trip.  This
// kernel back-propagates into the edge softmax and writes, per workgroup (its
// 4 (window, step) graphs summed in wave order), Xs = sum_i ds_i x_i and
// Xt = sum_j dt_j x_j (ds, dt: grads of the per-node source / destination
// scores), from which gat_param_body forms the attn_fc and fc grads.
// (fcd, the tokens' dX0 (x) x-bar sum that gat_param_body maps through W_TE
// into the fc gradient, is a weight-gradient reduction of its own.)  Runs as
// the first segment of the backward's multi-segment tail launch.
struct GatBwdArgs {
  int B;
  const float* wcopy;
  const float* P;
  const float* dX0;
  const float* GS;
  const float* Mt;
  float* GSX;
};
// workgroup bx (4 (window, step) graphs) of the GAT backward
template <int H>
PGP_DEV void gat_bwd_block(const GatBwdArgs& ga, int bx) {
  using Q = TuneGeo<H>;
  const int B = ga.B;
  const float* __restrict__ wcopy = ga.wcopy;
  const float* __restrict__ P = ga.P;
  const float* __restrict__ dX0 = ga.dX0;
  const float* __restrict__ GS = ga.GS;
  const float* __restrict__ Mt = ga.Mt;
  float* __restrict__ GSX = ga.GSX;
  __shared__ float ss[4][64], st[4][64], sx[4][64][3], sdx[4][64][3], smt[64][3], sred[4][6], sab[4][64][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long pw = (long)bx * 4 + wv;
  const bool okw = pw < 3L * B;
  const long b = okw ? pw / 3 : 0;
  const int w = okw ? (int)(pw - b * 3) : 0;
  const int j = lane;
  const bool okj = okw && j < H;
  if (threadIdx.x < 64 * 3) smt[threadIdx.x / 3][threadIdx.x % 3] = Mt[threadIdx.x];
  const GatFold<H> fo = gat_fold<H>(P);
  float x[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) x[k] = okj ? wcopy[(b * 3 + w) * 3 * H + 3 * j + k] : 0.f;
  const float s = fo.u[0] * x[0] + fo.u[1] * x[1] + fo.u[2] * x[2];
  const float t = fo.v[0] * x[0] + fo.v[1] * x[1] + fo.v[2] * x[2];
  const float mx = okw ? GS[pw * 4] : 0.f, iz = okw ? 1.0f / GS[pw * 4 + 1] : 0.f;
  const float smax = wave_max(okj ? s : -INFINITY);
  const GatEdge ge = gat_edge(s, t, smax, mx);  // the forward's factorised edge weights (gat_fwd_block)
  ss[wv][j] = s;
  st[wv][j] = t;
  sab[wv][j][0] = ge.a;
  sab[wv][j][1] = ge.an;
  sab[wv][j][2] = ge.b;
  sab[wv][j][3] = ge.bn;
#pragma unroll
  for (int k = 0; k < 3; ++k) sx[wv][j][k] = x[k];
  __syncthreads();
  // grad of x-bar_j = Mt^T dX0_j, the dX0 rows read coalesced: lane (rr, q)
  // takes features 4q .. 4q+3 of rows rr, rr+4, ...; the 16 lanes of a row are summed
  {
    const int q = lane & 15, rr = lane >> 4;
    float mt[4][3];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int k = 0; k < 3; ++k) mt[e][k] = 4 * q + e < Q::DP ? smt[4 * q + e][k] : 0.f;
    const float* g0 = dX0 + (b * Q::T + (long)w * H) * Q::DP + 4 * q;
    // unrolled: the ceil(H/4) row loads are all in flight before the first sum
    // (a rolled loop waited for each load in turn)
#pragma unroll
    for (int r0 = 0; r0 < H; r0 += 4) {  // uniform trip count: the row sums are cross-lane
      const int r = r0 + rr;
      const bool okr = okw && r < H && 4 * q < Q::DP;
      const f32x4 v = okr ? ld4(g0 + (long)r * Q::DP) : zero4();
      float d[3];
#pragma unroll
      for (int k = 0; k < 3; ++k)
        d[k] = row16_sum(fmaf(mt[0][k], v[0], fmaf(mt[1][k], v[1], fmaf(mt[2][k], v[2], mt[3][k] * v[3]))));
      if (okr && q == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) sdx[wv][r][k] = d[k];
      }
    }
  }
  __syncthreads();
  float dxb[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) dxb[k] = okj ? sdx[wv][j][k] : 0.f;
  // softmax backward: da_ij = dxb_j . x_i ; dot = sum_ij a_ij da_ij; with this
  // lane as destination dt = sum_i a_ij (da_ij - dot) lrelu'(pre_ij), gathered
  // in the same pass as sum a da lrelu' - dot * sum a lrelu'
  float part = 0.f, s1 = 0.f, s2 = 0.f;
  if (okj)
#pragma unroll 10
    for (int i = 0; i < H; ++i) {
      const float pre = ss[wv][i] + t;
      const float a = fmaxf(sab[wv][i][0] * ge.b, sab[wv][i][1] * ge.bn) * iz;
      const float da = dxb[0] * sx[wv][i][0] + dxb[1] * sx[wv][i][1] + dxb[2] * sx[wv][i][2];
      const float sl = pre > 0.f ? a : 0.01f * a;
      part = fmaf(a, da, part);
      s1 = fmaf(sl, da, s1);
      s2 += sl;
    }
  const float dot = wave_sum(part);
  float dt = 0.f, ds = 0.f;
  if (okj) {
    dt = fmaf(-dot, s2, s1);
#pragma unroll 10
    for (int jj = 0; jj < H; ++jj) {  // this lane as source
      const float pre = s + st[wv][jj];
      const float a = fmaxf(ge.a * sab[wv][jj][2], ge.an * sab[wv][jj][3]) * iz;
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
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      sred[wv][k] = okw ? xs[k] : 0.f;
      sred[wv][3 + k] = okw ? xt[k] : 0.f;
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int k = threadIdx.x;
    GSX[(long)bx * 8 + k] = (sred[0][k] + sred[1][k]) + (sred[2][k] + sred[3][k]);
  }
}

template <int H>
__global__ __launch_bounds__(256) void gat_bwd_kernel(GatBwdArgs ga) {
  gat_bwd_block<H>(ga, blockIdx.x);
}
// The backward's tail in ONE launch: the GAT backward (leading gat_nb
// blocks, gat_bwd_block) and the weight gradients that do not wait for it
// (segments: each block exactly as its own dw_kernel launch would run it, so
// the partials are bit-identical).  Shapes: kind 0 = <3 DP, DP> (in_proj),
// 1 = <DP, DP> (time encoder), 2 = <DP, XBP> (GAT fc aggregation).
template <int H>
__global__ __launch_bounds__(256) void dw_multi_kernel(DwMulti m, GatBwdArgs ga) {
  using Q = TuneGeo<H>;
  constexpr int DP = Q::DP, XBP = Q::XBP;
  constexpr int ROWS = dw_rows(0);
  constexpr int SY0 = ROWS * lds_stride(3 * DP), SX0 = ROWS * lds_stride(DP > XBP ? DP : XBP);
  constexpr int SYD = kDwRows * lds_stride(Q::NOP), SXD = kDwRows * lds_stride(DP);
  constexpr int SY = SY0 > SYD ? SY0 : SYD, SX = SX0 > SXD ? SX0 : SXD;
  if ((int)blockIdx.x < m.gat_nb) {
    gat_bwd_block<H>(ga, blockIdx.x);
    return;
  }
  __shared__ __attribute__((aligned(16))) float ys[SY];
  __shared__ __attribute__((aligned(16))) float xs[SX];
  if ((int)blockIdx.x < m.gat_nb + m.dec_nb) {  // (token, half, part) = blocks in dec_dw_kernel's grid order
    const int q = blockIdx.x - m.gat_nb, T = Q::T;
    dec_dw_block<H>(m.dec, q % T, (q / T) % 2, q / (2 * T), ys, xs);
    return;
  }
  const int b = blockIdx.x - m.gat_nb - m.dec_nb;
  const int s = b / m.nbx, bx = b - s * m.nbx;
  if (s >= m.n) return;
  switch (m.kind[s]) {
    case 0: dw_block<3 * DP, DP>(m.seg[s], bx, m.nbx, ys, xs); break;
    case 1: dw_block<DP, DP>(m.seg[s], bx, m.nbx, ys, xs); break;
    default: dw_block<DP, XBP>(m.seg[s], bx, m.nbx, ys, xs); break;
  }
}

// attn_fc and the score part of the fc gradient: s_i = a_1 . fc x_i, so
// d a_1 = fc Xs, d fc += a_1 Xs^T (and likewise a_2, Xt), summed over the
// gat_bwd workgroups in a fixed order; plus the aggregation part of the fc
// gradient, sum_tokens dG (x) x-bar = W_TE^T fcd.  Runs after the deferred
// reductions (fcd is one of them).
// (run by the last workgroup of the backward's final reduction, after its
// agent-scope acquire on the launch's counter: fcd, just written by other
// workgroups, is read with plain loads)
template <int H>
PGP_DEV void gat_param_body(int n, const float* __restrict__ GSX, const float* __restrict__ P,
                            const float* __restrict__ fcd, float* __restrict__ Gd) {
  using G = TGeo<H>;
  // the workgroups' partials: strided per thread, a butterfly per wave, the
  // four waves in order (one barrier; the 8-level LDS tree took 9)
  __shared__ float wred[4][6];
  __shared__ float tot[6];
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = threadIdx.x; p < n; p += 256)
#pragma unroll
    for (int k = 0; k < 6; ++k) acc[k] += GSX[(long)p * 8 + k];
#pragma unroll
  for (int k = 0; k < 6; ++k) acc[k] = wave_sum(acc[k]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 6; ++k) wred[threadIdx.x >> 6][k] = acc[k];
  __syncthreads();
  if (threadIdx.x < 6) tot[threadIdx.x] = ((wred[0][threadIdx.x] + wred[1][threadIdx.x]) + wred[2][threadIdx.x]) +
                                         wred[3][threadIdx.x];
  __syncthreads();
  const float* xs = tot;
  const float* xt = tot + 3;
  for (int c = threadIdx.x; c < H; c += 256) {
    const float* fc = P + G::W_FC + c * 3;
    const float a1 = P[G::W_ATT + c], a2 = P[G::W_ATT + H + c];
    float agg[3] = {0.f, 0.f, 0.f};
    for (int r = 0; r < H; ++r) {
      const float wt = P[G::W_TE + r * H + c];
#pragma unroll
      for (int k = 0; k < 3; ++k) agg[k] = fmaf(wt, fcd[r * 3 + k], agg[k]);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) Gd[G::W_FC + c * 3 + k] = agg[k] + (a1 * xs[k] + a2 * xt[k]);
    Gd[G::W_ATT + c] = fc[0] * xs[0] + fc[1] * xs[1] + fc[2] * xs[2];
    Gd[G::W_ATT + H + c] = fc[0] * xt[0] + fc[1] * xt[1] + fc[2] * xt[2];
  }
}
// the backward's last reduction launch with the GAT parameter gradient as its
// tail: the launch's last workgroup (device counter at the workspace head)
// runs gat_param_body once every reduction, fcd's included, is written
struct GatTail {
  int n;
  const float* gsx;
  const float* P;
  const float* fcd;
  float* Gd;
  unsigned* counter;
};
template <int H>
__global__ __launch_bounds__(256) void reduce_multi_gat_kernel(RedTable t, GatTail g) {
  const int bx = blockIdx.x;
  int s = 0;
  while (s + 1 < t.n && bx >= t.bx0[s + 1]) ++s;
  if ((int)blockIdx.y < t.nsplit[s]) reduce_block(t.seg[s], bx - t.bx0[s], blockIdx.y);
  __shared__ int s_last;
  if (!arrive_last(g.counter, gridDim.x * gridDim.y, &s_last)) return;
  gat_param_body<H>(g.n, g.gsx, g.P, g.fcd, g.Gd);
}

// ============================================================================
// Decoders (models.py:359-370, 399) and the loss gradient (train.py:27-40).
// ============================================================================
// Decoder weights permuted to the token layout: Wp[n][k'] with k' = tok*DP + c,
// tok = w*H + h, natural column h*3H + w*H + c (the latent order, models.py:399);
// rows n: anomaly 0..2H-1, prototype 2H..4H-1, zero pads.  WpT holds, per token,
// the transposed slab WpT[tok][c][n] = Wp[n][tok*DP + c] (the decoder backward
// into the encoder output, pgp_dec.hip).
template <int H>
__global__ __launch_bounds__(256) void dec_pack_kernel(const float* __restrict__ P, float* __restrict__ Wp,
                                                       float* __restrict__ WpT) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
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
  WpT[((long)tok * Q::DP + c) * Q::NOP + n] = v;
}

// The step's per-step packing as ONE launch when it all runs on the caller's
// stream (below the side-stream threshold, e.g. C3 at H = 16): blocks
// [0, nb_dec) dec_pack_kernel's elements (none with a side stream), then one block forming Mt,
// then tf_pack_kernel's elements (pgp_tunef.hpp tf_pack_elem).  Each element is
// computed as by its own kernel: the same bits.
template <int H>
__global__ __launch_bounds__(256) void tune_pack_kernel(const float* __restrict__ P, float* __restrict__ Wp,
                                                        float* __restrict__ WpT, float* __restrict__ Mt,
                                                        float* __restrict__ frags, int nb_dec, int nb_tf,
                                                        GatFwdIn g) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  int bx = blockIdx.x;
  // the blocks after the packings: the GAT forward (it reads P and the
  // windows only), one launch fewer on the step's chain
  if (bx >= nb_dec + 1 + nb_tf) {
    gat_fwd_block<H>(bx - (nb_dec + 1 + nb_tf), g.B, g.win, P, g.wcopy, g.Gout, g.XB, g.GS);
    return;
  }
  const int t = threadIdx.x;
  if (bx < nb_dec) {
    const long idx = (long)bx * 256 + t;
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
    WpT[((long)tok * Q::DP + c) * Q::NOP + n] = v;
    return;
  }
  bx -= nb_dec;
  if (bx == 0) {  // Mt[c][k] = sum_f W_TE[c][f] fc[f][k] (rows past H are 0): the time encoder
                  // folded into the GAT backward's first contraction (gat_bwd_kernel)
    const int c = t / 3, k = t - 3 * c;
    if (c >= 64 || !Mt) return;
    float m = 0.f;
    if (c < H)
      for (int f = 0; f < H; ++f) m = fmaf(P[G::W_TE + c * H + f], P[G::W_FC + f * 3 + k], m);
    Mt[t] = m;
    return;
  }
  bx -= 1;
  tf_pack_elem<H>(P, frags, (long)bx * 256 + t);
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
  float* d = dpre + b * NOP;
  dpre_host(logits[2 * idx], logits[2 * idx + 1], y[idx], mult[idx], protos[2 * idx], protos[2 * idx + 1],
            tgt[2 * idx], tgt[2 * idx + 1], d + 2 * h, d + 2 * H + 2 * h);
}

// decoder weight / bias gradients straight into G (natural layout): one
// workgroup per (token, n-half); the contraction runs over the batch's windows
// (rows: dpre[b], X2 row b*T + tok), staged through LDS like dw_kernel.
// Decoder weight gradient: for token tok (grid.x) and output-tile half y,
// sum over windows of dpre[b] (x) X2[b][tok].  The windows are split over
// grid.z = S parts (latency: one part is a short chain of LDS-staged chunks);
// S = 1 writes straight into G, otherwise each part writes its [NOP][DP] slab
// (and tok 0 its bias column) to `part` and the last part of each (token,
// half) adds them into G in part order (a device counter per (token, half) at
// the workspace head).
template <int H>
PGP_DEV void dec_dw_block(const DecDwArgs& d, int tok, int y, int z, float* ys, float* xs) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  constexpr int NP = Q::NOP, KP = Q::DP, NT = NP / 16, NTW = (NT + 7) / 8, KT = KP / 16;
  const int B = d.B, S = d.S;
  const float* __restrict__ dpre = d.dpre;
  const float* __restrict__ X2 = d.X2;
  float* __restrict__ Gd = d.Gd;
  float* __restrict__ part = d.part;
  unsigned* __restrict__ counter = d.counter;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
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
  float sbs[NTW];
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    const int t = 4 * y + wv + 8 * q;
    sbs[q] = 0.f;
    if (t < NT) {
#pragma unroll
      for (int u = 0; u < KT; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * t + 4 * g + r, c = 16 * u + i;
          if (S > 1) {
            store_wt(ps + n * KP + c, acc[q][u][r]);
          } else if (n < 4 * H && c < H) {
            const long col = (long)h * 3 * H + w * H + c;
            Gd[(n < 2 * H ? G::W_AN + (long)n * G::L : G::W_PR + (long)(n - 2 * H) * G::L) + col] = acc[q][u][r];
          }
        }
      if (tok == 0) {
        const float sb = xsum(pb[q], true);
        sbs[q] = sb;
        const int n = 16 * t + i;
        if (S > 1) {
          if (g == 0) store_wt(pbias + n, sb);
        } else if (g == 0 && n < 4 * H) {
          Gd[n < 2 * H ? G::B_AN + n : G::B_PR + n - 2 * H] = sb;
        }
      }
    }
  }
  if (S == 1) return;
  // the last of the S parts of this (token, half) sums them in part order
  // into G (what dec_dw_sum_kernel did: one launch fewer); its own part from
  // registers, the others' with plain loads after the agent-scope acquire
  __shared__ int s_last;
  if (!arrive_last(counter + 2 * tok + y, (unsigned)S, &s_last)) return;
  const long zstride = (long)Q::T * NP * KP;
  const float* p0 = part + (long)tok * NP * KP;
#pragma unroll
  for (int q = 0; q < NTW; ++q) {
    const int t = 4 * y + wv + 8 * q;
    if (t < NT) {
#pragma unroll
      for (int u = 0; u < KT; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * t + 4 * g + r, c = 16 * u + i;
          if (n < 4 * H && c < H) {
            // every part loaded (its own too, stored above; parts past S
            // re-read part S - 1, unused) before the sum: a per-part
            // "register or load" choice would wait once per load
            float pv[kMaxDecDws];
#pragma unroll
            for (int zz = 0; zz < kMaxDecDws; ++zz) pv[zz] = p0[(zz < S ? zz : S - 1) * zstride + n * KP + c];
            float v = 0.f;
#pragma unroll
            for (int zz = 0; zz < kMaxDecDws; ++zz)
              if (zz < S) v += pv[zz];
            const long col = (long)h * 3 * H + w * H + c;
            Gd[(n < 2 * H ? G::W_AN + (long)n * G::L : G::W_PR + (long)(n - 2 * H) * G::L) + col] = v;
          }
        }
      if (tok == 0 && g == 0) {
        const int n = 16 * t + i;
        if (n < 4 * H) {
          const float* pb0 = part + (long)S * Q::T * NP * KP + n;
          float pv[kMaxDecDws];
#pragma unroll
          for (int zz = 0; zz < kMaxDecDws; ++zz) pv[zz] = pb0[(long)(zz < S ? zz : S - 1) * NP];
          float v = 0.f;
#pragma unroll
          for (int zz = 0; zz < kMaxDecDws; ++zz)
            if (zz < S) v += pv[zz];
          Gd[n < 2 * H ? G::B_AN + n : G::B_PR + n - 2 * H] = v;
        }
      }
    }
  }
}
template <int H>
__global__ __launch_bounds__(256) void dec_dw_kernel(DecDwArgs d) {
  using Q = TuneGeo<H>;
  __shared__ __attribute__((aligned(16))) float ys[kDwRows * lds_stride(Q::NOP)];
  __shared__ __attribute__((aligned(16))) float xs[kDwRows * lds_stride(Q::DP)];
  dec_dw_block<H>(d, blockIdx.x, blockIdx.y, blockIdx.z, ys, xs);
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
  // the last registered reduction's final outputs stored write-through (the
  // flush's last workgroup reads them: flush_gat)
  void mark_last_wt() {
    RedArgs& a = l1.seg[l1.n - 1];
    if (a.lvl2)
      l2.seg[l2.n - 1].wt = 1;
    else
      a.wt = 1;
  }
  // the same, the last launch carrying the GAT parameter gradient as its tail
  template <int H>
  hipError_t flush_gat(hipStream_t st, const GatTail& g) {
    if (used > cap) return hipErrorInvalidValue;
    l1.bx0[l1.n] = gx1;
    l2.bx0[l2.n] = gx2;
    if (!l1.n) return hipErrorInvalidValue;  // the backward always has reductions
    if (l2.n) {
      TCK((reduce_multi_kernel<<<dim3(gx1, ny1), 256, 0, st>>>(l1)));
      TCK((reduce_multi_gat_kernel<H><<<gx2, 256, 0, st>>>(l2, g)));
    } else {
      TCK((reduce_multi_gat_kernel<H><<<dim3(gx1, ny1), 256, 0, st>>>(l1, g)));
    }
    return hipSuccess;
  }
  // reduce what is registered so far (on `st`, ordered after its partials) and
  // start new lists; the pool regions already taken stay theirs
  hipError_t flush_now(hipStream_t st) {
    const hipError_t e = flush(st);
    l1.n = l2.n = 0;
    gx1 = gx2 = 0;
    ny1 = 1;
    return e;
  }
};

// dW[N][K] (row stride K) += sum_m Y[m][n] X[m][k];  db[N] += sum_m Y[m][n]
// (partial slabs from the pool; the reduction is deferred to rb.flush)
// (dm != nullptr: the launch is deferred into that multi-segment launch as
// segment kind `kind`, dw_multi_kernel)
template <int NP, int KP>
hipError_t dw(const TunePlan& p, RedBatch& rb, const float* Y, int ldy, const float* X, int ldx, int relu, int N,
              int K, float* gW, float* gb, hipStream_t st, DwMulti* dm = nullptr, int kind = 0) {
  const long pstride = (long)NP * KP + NP;
  float* part = rb.take((long)p.dw_grid * pstride);
  DwArgs a{p.M, Y, ldy, X, ldx, relu, part};
  if (dm) {
    if (dm->n >= kMaxDwSeg) return hipErrorInvalidValue;
    dm->kind[dm->n] = kind;
    dm->seg[dm->n++] = a;
  } else {
    TCK((dw_kernel<NP, KP><<<p.dw_grid, 256, 0, st>>>(a)));
  }
  return rb.add(p.dw_grid, pstride, part, N, K, KP, gW, K, gb ? N : 0, (long)NP * KP, gb) ? hipSuccess
                                                                                          : hipErrorInvalidValue;
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
  long off = kTuneCounters;  // the head: device counters (zero in a fresh workspace, reset by their users)
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
  // buffers the fused encoder kernels write carry a spare row M (pgp_tunef.hpp)
  const long M1 = M + 1;
  for (int i = 0; i < 3; ++i) q.x[i] = take(M1 * Q::DP);
  for (int l = 0; l < 2; ++l) {
    q.xh1[l] = take(M1 * Q::DP);
    q.rs1[l] = take(M1);
  }
  q.da = take(M1 * Q::DP);
  q.db = take(M1 * Q::DP);
  // one dQKV buffer per layer: layer 1's in_proj weight gradient reads its
  // buffer on the side stream while layer 0's attention backward writes the other
  for (int l = 0; l < 2; ++l) q.dq[l] = take(M1 * 3 * Q::DP);
  q.gsx = take(((3L * B + 3) / 4) * 8);
  q.fcd = take(64 * 3);
  q.mt = take(64 * 3);
  q.dpre = take((long)B * Q::NOP);
  q.wp = take((long)Q::NOP * Q::KD);
  q.wpt = take((long)Q::NOP * Q::KD);
  q.tff = take(tf_frag_floats(H));
  q.tf_grid = tf_bwd_grid(H, B);   // this call's backward launches (slabs); sized below for the most
  for (int l = 0; l < 2; ++l)
    for (int k = 0; k < 2; ++k) q.tfs[l][k] = take((long)tf_max_grid() * tf_slab_floats(H, 2 + k));
  const long nrb = (M + 15) / 16;
  q.lin_grid = (int)std::min<long>(kLinCap, std::max<long>(1, (nrb + 3) / 4));
  q.dw_grid = (int)std::min<long>(kDwCap, std::max<long>(1, (nrb + 7) / 8));
  q.dec_s = dec_fwd_splits(H, B);
  // partial slabs; every bound grows with B, so a workspace sized for B_max serves any B <= B_max
  const long np_max = std::max(Q::Q3P, 64);
  long part = (long)kDwCap * (np_max * 64 + np_max);                  // dW slabs
  part = std::max(part, (long)q.dec_s * B * Q::NOP);                    // decoder split-K
  // decoder weight gradient: windows split over up to 4 parts of >= 8 chunks
  q.dec_dws = (int)std::max<long>(1, std::min<long>(kMaxDecDws, (B + kDwRows - 1) / kDwRows / 8));
  if (q.dec_dws > 1) part = std::max(part, (long)q.dec_dws * (Q::T * Q::NOP * Q::DP + Q::NOP));
  q.part = take(part);
  // the backward's deferred reductions (RedBatch): each dW partial region plus
  // its level-2 region, in the order tune_bwd_h takes them (the fused kernels'
  // slabs have regions of their own, tfs)
  {
    long pool = 0;
    auto r64 = [](long n) { return (n + 63) / 64 * 64; };
    auto red = [&](long nparts, long slab, long nout) {
      pool += r64(nparts * slab);
      const long ns = (nparts + kRedChunk - 1) / kRedChunk;
      if (ns > 1) pool += r64(ns * nout);
    };
    auto dwr = [&](long np, long kp, long n, long k, bool bias) { red(q.dw_grid, np * kp + np, n * k + (bias ? n : 0)); };
    const long DPl = Q::DP, Hl = H;
    for (int l = 1; l >= 0; --l) {  // in_proj: one dW launch over [q|k|v] x DP rows, three reductions
      pool += r64((long)q.dw_grid * (3 * DPl * DPl + 3 * DPl));
      const long ns2 = (q.dw_grid + kRedChunk - 1) / kRedChunk;
      if (ns2 > 1) pool += 3 * r64(ns2 * (Hl * Hl + Hl));
    }
    dwr(DPl, DPl, Hl, Hl, true);           // time encoder
    dwr(DPl, Q::XBP, Hl, 3, false);        // GAT fc
    // level-2 regions of the fused slabs (more than 256 workgroups)
    const long ns = (tf_max_grid() + kRedChunk - 1) / kRedChunk;
    if (ns > 1) pool += 2 * ns * r64(tf_slab_floats(H, 2) + tf_slab_floats(H, 3)) * 2;
    q.pool = take(pool);
    q.pool_len = pool;
  }
  q.total = off;
  *out = q;
  return true;
}

// Live timing of the fused encoder launches (pgp_tune_timing): events around
// each of the six per step, [fwd l0, fwd l1, ffn l1, att l1, ffn l0, att l0]
struct TfTiming {
  bool on = false, made = false;
  hipEvent_t ev[12];
  void mark(int k, hipStream_t st) {
    if (on) (void)hipEventRecord(ev[k], st);
  }
};
TfTiming g_tft;

// The backward's second stream: work off the critical path (the decoder's and
// in_proj's weight gradients) runs beside the chain loss -> dX -> fused layer
// backwards -> time encoder -> GAT, on the CUs the fused launches leave idle
// in their last unit round (tf_unit_range packs the waves with an extra unit
// into the first workgroups).  One non-blocking stream per device at low
// priority; fork / join by events.  While the caller's stream is being
// captured into a graph the events become the graph's edges (two branches).
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t ev[8] = {};
  std::atomic<unsigned> next{0};  // event rotation (callers on several host threads)
  bool ok = false;
};
SideStream* side_stream() {
  static SideStream ss[16];
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  SideStream& x = ss[dev];
  if (!x.s) {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);  // lo: the least urgent
    x.ok = hipStreamCreateWithPriority(&x.s, hipStreamNonBlocking, lo) == hipSuccess;
    for (auto& e : x.ev) x.ok = x.ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  }
  return x.ok ? &x : nullptr;
}
// a caller-owned stream to use as the side stream (pgp_tune_set_side_stream),
// per device; null: the library's own
std::atomic<hipStream_t> g_side_override[16];
// Below kSideMinTokens tokens (B * 3H) the side work is a few microseconds per
// launch and the fork / join events cost more than the overlap returns (A/B on
// one box, C3 at 1,030 windows: H = 16 (49 k tokens) 0.362 -> 0.302 ms per step
// without the fork, H = 50 (154 k tokens) 1.297 -> 1.340 ms; profiles/r04/s5/)
constexpr long kSideMinTokens = 65536;
}  // namespace
bool tune_side_active(long tokens) { return tokens >= kSideMinTokens; }
namespace {
struct Fork {
  hipStream_t main, side;
  SideStream* ss = nullptr;
  bool capturing = false;
  Fork(hipStream_t st, long tokens) : main(st), side(st) {
    if (tokens < kSideMinTokens) return;
    // while `st` is being captured into a graph the fork / join events become
    // the graph's edges: the side stream joins the capture at the fork's wait
    // and leaves it at the join, so the graph keeps the two branches (a
    // replayed graph runs independent branches concurrently, measured:
    // profiles/r04/s3/graph_concurrency.txt)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs == hipStreamCaptureStatusInvalidated) return;
    capturing = cs == hipStreamCaptureStatusActive;
    ss = side_stream();
    if (!ss) return;
    int dev = 0;
    const hipStream_t o = (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 16)
                              ? g_side_override[dev].load(std::memory_order_relaxed)
                              : nullptr;
    side = o ? o : ss->s;  // an override equal to `st`: everything on the caller's stream
  }
  // `to` waits for everything issued on `from` so far
  hipError_t order(hipStream_t from, hipStream_t to) {
    if (!ss || from == to) return hipSuccess;
    hipEvent_t e = ss->ev[ss->next.fetch_add(1, std::memory_order_relaxed) % 8];
    hipError_t r = hipEventRecord(e, from);
    return r != hipSuccess ? r : hipStreamWaitEvent(to, e, 0);
  }
  hipError_t fork() { return order(main, side); }
  hipError_t join() { return order(side, main); }
  // An event for the NEXT launch on the main stream to signal at its end
  // (hipExtLaunchKernel's stop event) for a fork right after it: no marker
  // packet on the main stream.  A hipEventRecord costs the recording stream
  // ~4.9 us of device time, a stop event ~1.4 (tools/micro/fork_cost.hip,
  // profiles/r05/fork_cost/).  nullptr (no side stream, or a graph capture:
  // fork_on records as before).
  hipEvent_t launch_event() {
    if (!ss || side == main || capturing) return nullptr;
    return ss->ev[ss->next.fetch_add(1, std::memory_order_relaxed) % 8];
  }
  // fork after the launch that signals `e` (launch_event or the caller's own
  // stop event); e == nullptr: an ordinary fork
  hipError_t fork_on(hipEvent_t e) {
    if (!ss || side == main) return hipSuccess;
    return e ? hipStreamWaitEvent(side, e, 0) : fork();
  }
};

template <int H>
hipError_t tune_fwd_h(const TunePlan& p, const float* win, const float* P, float* ws, float* latent, float* logits,
                      float* protos, hipStream_t st, hipEvent_t post) {
  using Q = TuneGeo<H>;
  const int B = p.B;
  hipError_t e;
  Fork fk(st, p.M);
  TfArgs t{};
  t.B = B;
  t.P = P;
  t.frags = ws + p.tff;
  if (fk.side == st) {  // all on the caller's stream: every packing in ONE launch
    const int nb_dec = (int)((Q::NOP * Q::KD + 255) / 256), nb_tf = (int)((tf_pack_items(H) + 255) / 256);
    // ... and the GAT forward in the same launch
    const GatFwdIn g{B, win, ws + p.win, ws + p.g, ws + p.xb, ws + p.gs};
    TCK((tune_pack_kernel<H><<<nb_dec + 1 + nb_tf + (3 * B + 3) / 4, 256, 0, st>>>(
        P, ws + p.wp, ws + p.wpt, ws + p.mt, ws + p.tff, nb_dec, nb_tf, g)));
  } else {
    // main: the encoder's fragments packed from P and the GAT forward in ONE
    // launch (the packing kernel's tf blocks, then the GAT blocks)
    const int nb_tf = (int)((tf_pack_items(H) + 255) / 256);
    const GatFwdIn g{B, win, ws + p.win, ws + p.g, ws + p.xb, ws + p.gs};
    // (and the GAT's Mt for the backward: its block, not a side-stream
    // launch the forward's join would wait for)
    TCK((tune_pack_kernel<H><<<1 + nb_tf + (3 * B + 3) / 4, 256, 0, st>>>(P, nullptr, nullptr, ws + p.mt, ws + p.tff, 0,
                                                                           nb_tf, g)));
  }
  for (int l = 0; l < 2; ++l) {
    t.layer = l;
    t.in = ws + (l == 0 ? p.g : p.x[1]);
    t.out = ws + p.x[l + 1];
    t.x0 = ws + p.x[0];
    t.xh1 = ws + p.xh1[l];
    t.rs1 = ws + p.rs1[l];
    g_tft.mark(2 * l, st);
    // side: the decoder weights permuted for this step's decoder forward and
    // backward, forked at the end of the layer-0 launch: beside layer 1's forward, not beside layer 0's (which
    // also runs the time encoder / GAT input): C3 at H = 50 1.050 -> 1.043 ms
    // (A/B, profiles/r05/pack_late/)
    const bool pack_here = fk.side != st && l == 0;
    hipEvent_t f0 = (pack_here && !g_tft.on) ? fk.launch_event() : nullptr;
    if ((e = launch_tf(H, 1, t, st, f0)) != hipSuccess) return e;
    g_tft.mark(2 * l + 1, st);
    if (pack_here) {
      if ((e = fk.fork_on(f0)) != hipSuccess) return e;
      TCK((dec_pack_kernel<H><<<(int)((Q::NOP * Q::KD + 255) / 256), 256, 0, fk.side>>>(P, ws + p.wp, ws + p.wpt)));
    }
  }
  if ((e = fk.join()) != hipSuccess) return e;
  if ((e = launch_dec_fwd(H, B, p.dec_s, ws + p.x[2], ws + p.wp, ws + p.part, st)) != hipSuccess) return e;
  const int nfin = (int)(((long)B * 4 * H + 255) / 256);
  if (post && !latent) {  // the forward's last launch signals `post` at its end
    int Bv = B, S = p.dec_s;
    const float* partc = ws + p.part;
    void* args[] = {&Bv, &S, &partc, &P, &logits, &protos};
    TCK((void)hipExtLaunchKernel(reinterpret_cast<const void*>(dec_fin_kernel<H>), dim3(nfin), dim3(256), args, 0, st,
                                 nullptr, post, 0));
  } else {
    TCK((dec_fin_kernel<H><<<nfin, 256, 0, st>>>(B, p.dec_s, ws + p.part, P, logits, protos)));
    if (post) TCK((void)hipEventRecord(post, st));
  }
  if (latent)
    TCK((latent_kernel<H><<<(int)(((long)B * 3 * H * H + 255) / 256), 256, 0, st>>>(B, ws + p.x[2], latent)));
  return hipSuccess;
}

template <int H>
hipError_t tune_bwd_h(const TunePlan& p, const float* P, float* Gd, float* ws, const float* logits,
                      const float* protos, const int* y, const float* mult, const float* tgt, hipStream_t st,
                      bool dpre_ready, hipEvent_t pre) {
  using Q = TuneGeo<H>;
  using G = TGeo<H>;
  constexpr int DP = Q::DP;
  const int B = p.B;
  const long M = p.M;
  hipError_t e;
  RedBatch rb{ws + p.pool, p.pool_len};
  Fork fk(st, p.M);
  const hipStream_t sd = fk.side;
  if (!dpre_ready)  // (pgp_online_step: written by the targets kernel)
    TCK((tune_loss_kernel<<<(int)(((long)B * H + 255) / 256), 256, 0, st>>>(B, H, Q::NOP, logits, protos, y, mult,
                                                                             tgt, ws + p.dpre)));
  // Side work issued as soon as its inputs exist: the decoders' weight
  // gradient early (bit 2: after the first fused launch, dec_late below),
  // layer 1's in_proj weight gradient right after layer 1's attention backward
  // (bit 1).  They run beside the fused launches
  // on the CUs those leave free (tf_grid_for takes the fewest workgroups with
  // the same longest wave): C3 at H = 50 1.171 -> 1.131 ms
  // (profiles/r04/side_early/).  Bit 4: layer 0's in_proj weight gradient on
  // the side stream beside the time encoder / GAT tail, 1.137 -> 1.126 ms;
  // bit 8 (the time encoder's too) measured neutral.
  constexpr int early = 7;  // round 5 A/B (H = 50): 5 1.102, 13 1.118, 15 1.090, 7 1.092 ms (profiles/r05/side_early_ab.txt)
  // Without a side stream the tail's weight gradients that nothing on the
  // chain reads (in_proj of both layers, the time encoder's, the GAT fc
  // aggregation's) join the GAT backward in ONE multi-segment launch before
  // the reductions: their inputs stay untouched until then (per-layer dQKV /
  // X regions; dX0 is read-only after the attention backward).  H = 16:
  // 0.207 -> 0.202 ms.  With a side stream (H = 50) the same merge of the GAT
  // backward and the two main-stream weight gradients ran as long as the
  // three launches in turn (82 vs 85 us: their blocks are throughput-bound)
  // and slowed the side stream's in_proj weight gradient beside it (50 -> 93
  // us): C3 1.080 -> 1.100 ms, so there they stay separate launches.
  const bool defer = sd == st;
  DwMulti dm{};
  dm.nbx = p.dw_grid;
  // side work: the decoders' weight gradients (dpre, encoder output -> G)
  // and each layer's in_proj weight gradient (dQKV [M][3][DP] (x) X -> three
  // [H][H] blocks of L_IN + bias); nothing on the critical path reads them
  auto side_dec = [&]() -> hipError_t {
    const DecDwArgs da{B, p.dec_dws, ws + p.dpre, ws + p.x[2], Gd, ws + p.part, reinterpret_cast<unsigned*>(ws)};
    if (defer) {  // no side stream: its blocks join the tail's multi-segment launch
      dm.dec = da;
      dm.dec_nb = Q::T * 2 * p.dec_dws;
      return hipSuccess;
    }
    TCK((dec_dw_kernel<H><<<dim3(Q::T, 2, p.dec_dws), 256, 0, sd>>>(da)));
    return hipSuccess;
  };
  auto in_proj_dw = [&](int l, hipStream_t ss) -> hipError_t {
    float* Lg = Gd + G::LAY0 + l * G::L_SIZE;
    constexpr int NP = 3 * DP;
    const long pstride = (long)NP * DP + NP;
    float* part = rb.take((long)p.dw_grid * pstride);
    DwArgs a{M, ws + p.dq[l], NP, ws + p.x[l], DP, 0, part};
    if (defer && ss == st) {
      if (dm.n >= kMaxDwSeg) return hipErrorInvalidValue;
      dm.kind[dm.n] = 0;
      dm.seg[dm.n++] = a;
    } else {
      TCK((dw_kernel<NP, DP><<<p.dw_grid, 256, 0, ss>>>(a)));
    }
    for (int q = 0; q < 3; ++q)
      if (!rb.add(p.dw_grid, pstride, part + (long)q * DP * DP, H, H, DP, Lg + G::L_IN + (long)q * H * H, H, H,
                  (long)NP * DP + q * DP - (long)q * DP * DP, Lg + G::L_INB + q * H))
        return hipErrorInvalidValue;
    return hipSuccess;
  };

  // With a side stream the decoders' weight gradient forks at the end of the
  // first fused launch (layer 1's feed-forward backward), so it runs beside
  // layer 1's attention backward, where the side stream was idle, instead of
  // beside that first launch, which the GAN stream already shares: C3 at
  // H = 50 1.067 -> 1.049 ms (A/B, profiles/r05/dec_late/)
  const bool dec_late = (early & 2) && !defer;
  if ((early & 2) && !dec_late) {
    // after the targets (pre: the caller's launch of them signals it; the
    // loss kernel above when dpre was not ready)
    if ((e = fk.fork_on(dpre_ready ? pre : nullptr)) != hipSuccess) return e;
    if ((e = side_dec()) != hipSuccess) return e;
  }
  // grad of the encoder output = dpre . Wp (token layout, pgp_dec.hip)
  if ((e = launch_dec_dx(H, B, ws + p.dpre, ws + p.wpt, ws + p.da, st)) != hipSuccess) return e;
  // the encoder layers, fused per unit (pgp_tunef.hip); their weight-gradient
  // slabs (one per workgroup) join the deferred reductions
  const int ng = p.tf_grid;
  hipEvent_t tail_fork = nullptr;
  for (int l = 1; l >= 0; --l) {
    float* Lg = Gd + G::LAY0 + l * G::L_SIZE;
    TfArgs t{};
    t.layer = l;
    t.B = B;
    t.P = P;
    t.frags = ws + p.tff;
    // feed-forward block: dOut (p.da) -> dR1 (p.db)
    t.in = ws + p.da;
    t.out = ws + p.db;
    t.xh1 = ws + p.xh1[l];
    t.rs1 = ws + p.rs1[l];
    t.part = ws + p.tfs[l][0];
    const int tk = 4 + 4 * (1 - l);
    g_tft.mark(tk, st);
    hipEvent_t ffn_end = (dec_late && l == 1 && !g_tft.on) ? fk.launch_event() : nullptr;
    if ((e = launch_tf(H, 2, t, st, ffn_end)) != hipSuccess) return e;
    g_tft.mark(tk + 1, st);
    if (dec_late && l == 1) {
      if ((e = fk.fork_on(ffn_end)) != hipSuccess) return e;
      if ((e = side_dec()) != hipSuccess) return e;
    }
    {
      const long sl = tf_slab_floats(H, 2);
      const float* s0 = ws + p.tfs[l][0];
      // slab: dW2 [H][64] | db2 [H] | dW1 [64][H] | db1 [64] | g1 | b1 | g2 | b2 (pgp_tunef.hip BffL)
      const long oW1 = (long)H * 64 + H, oG1 = oW1 + 64L * H + 64, oG2 = oG1 + 2L * H;
      bool ok = rb.add(ng, sl, s0, H, 64, 64, Lg + G::L_W2, 64, H, (long)H * 64, Lg + G::L_B2);
      ok = ok && rb.add(ng, sl, s0 + oW1, 64, H, H, Lg + G::L_W1, H, 64, 64L * H, Lg + G::L_B1);
      ok = ok && rb.add(ng, sl, s0 + oG1, 1, H, 0, Lg + G::L_N1W, 0, H, H, Lg + G::L_N1B);
      ok = ok && rb.add(ng, sl, s0 + oG2, 1, H, 0, Lg + G::L_N2W, 0, H, H, Lg + G::L_N2B);
      if (!ok) return hipErrorInvalidValue;
    }
    // attention block: dR1 (p.db), X_l -> dX_l (p.da), dQKV (p.dq[l])
    t.in = ws + p.db;
    t.out = ws + p.da;
    t.x = ws + p.x[l];
    t.dqkv = ws + p.dq[l];
    t.part = ws + p.tfs[l][1];
    g_tft.mark(tk + 2, st);
    // its end forks the side work (layer 1: in_proj dW and the early flush;
    // layer 0: the tail's side work)
    hipEvent_t att_end = g_tft.on ? nullptr : fk.launch_event();
    if ((e = launch_tf(H, 3, t, st, att_end)) != hipSuccess) return e;
    g_tft.mark(tk + 3, st);
    if (!rb.add(ng, tf_slab_floats(H, 3), ws + p.tfs[l][1], H, H, H, Lg + G::L_OUT, H, H, (long)H * H,
                Lg + G::L_OUTB))
      return hipErrorInvalidValue;
    if (l == 0) tail_fork = att_end;
    if (l == 1 && (early & 1)) {
      if ((e = fk.fork_on(att_end)) != hipSuccess) return e;
      if ((e = in_proj_dw(1, sd)) != hipSuccess) return e;
      // layer 1's reductions (its fused slabs, in_proj) on the side stream
      // beside layer 0's backward, not in the final flush
      if (sd != st && (e = rb.flush_now(sd)) != hipSuccess) return e;
    }
  }
  // side, beside the serial tail below (time encoder, GAT), unless issued
  // early: weight gradients nothing on the critical path reads — the
  // decoders' and layer 1's in_proj.  (While the fused launches spread over
  // every CU, side work beside them only slowed them: a long side workgroup on
  // a CU delays the next fused launch's workgroup there; profiles/r03/s3/.)
  if ((e = fk.fork_on(tail_fork)) != hipSuccess) return e;
  if (!(early & 2) && (e = side_dec()) != hipSuccess) return e;
  if (!(early & 1) && (e = in_proj_dw(1, sd)) != hipSuccess) return e;
  // bits 4 / 8: layer 0's in_proj and the time encoder's weight gradients on
  // the side stream too
  if ((early & 4) && (e = in_proj_dw(0, sd)) != hipSuccess) return e;
  // time encoder: p.da = grad of X0 (weight gradient: dX0 (x) G)
  if ((e = dw<DP, DP>(p, rb, ws + p.da, DP, ws + p.g, DP, 0, H, H, Gd + G::W_TE, Gd + G::B_TE,
                      (early & 8) ? sd : st, defer ? &dm : nullptr, 1)) != hipSuccess)
    return e;
  // GAT, straight from dX0 (the time encoder's input gradient folded in,
  // gat_bwd_kernel); the fc gradient's aggregation part: fcd = dX0 (x) x-bar
  const int gat_wg = (3 * B + 3) / 4;
  const GatBwdArgs gba{B, ws + p.win, P, ws + p.da, ws + p.gs, ws + p.mt, ws + p.gsx};
  if (defer)
    dm.gat_nb = gat_wg;
  else
    TCK((gat_bwd_kernel<H><<<gat_wg, 256, 0, st>>>(gba)));
  if ((e = dw<DP, Q::XBP>(p, rb, ws + p.da, DP, ws + p.xb, Q::XBP, 0, H, 3, ws + p.fcd, nullptr, st,
                          defer ? &dm : nullptr, 2)) != hipSuccess)
    return e;
  rb.mark_last_wt();  // fcd: read by the final reduction launch's last workgroup (gat_param_body)
  // without bit 4, layer 0's in_proj weight gradient closes the main stream's share
  if (!(early & 4) && (e = in_proj_dw(0, st)) != hipSuccess) return e;
  if (defer) TCK((dw_multi_kernel<H><<<dm.gat_nb + dm.dec_nb + dm.n * dm.nbx, 256, 0, st>>>(dm, gba)));
  if ((e = fk.join()) != hipSuccess) return e;  // the side stream's partials and G writes
  // every deferred weight-gradient reduction, then (the same launch's last
  // workgroup) the GAT parameter gradient, which needs fcd's reduction
  const GatTail gt{gat_wg, ws + p.gsx, P, ws + p.fcd, Gd, reinterpret_cast<unsigned*>(ws) + kCtrGatTail};
  if ((e = rb.flush_gat<H>(st, gt)) != hipSuccess) return e;
  return hipSuccess;
}

}  // namespace

hipError_t tune_set_side_stream(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return hipErrorInvalidDevice;
  g_side_override[dev].store(s, std::memory_order_relaxed);
  return hipSuccess;
}

hipError_t tune_timing(bool on) {
  if (on && !g_tft.made) {
    for (auto& e : g_tft.ev)
      if (hipEventCreate(&e) != hipSuccess) return hipErrorOutOfMemory;
    g_tft.made = true;
  }
  g_tft.on = on;
  return hipSuccess;
}

hipError_t tune_fused_ms(float* out) {
  if (!g_tft.made) return hipErrorInvalidValue;
  // every event: a forward records its pair twice per C3 step (detect, then tuning)
  for (auto& ev : g_tft.ev) {
    const hipError_t w = hipEventSynchronize(ev);
    if (w != hipSuccess) return w;
  }
  for (int k = 0; k < 6; ++k) {
    const hipError_t e = hipEventElapsedTime(&out[k], g_tft.ev[2 * k], g_tft.ev[2 * k + 1]);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

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

// The plan of a backward over the first B windows of a forward of B_fwd: the
// regions stay where the forward's plan put them (its activations are read in
// place; rows are window-major, so the first B windows are the first B*3H
// rows), the launch geometry is B's.  Every bound that sized a region grows
// with the batch, so B's grids fit B_fwd's regions.  The spare row M of the
// backward's outputs is then a row of window B: the backward only writes
// temporaries (da, db, dQKV) there, never a forward activation.
bool tune_plan_prefix(int H, int B_fwd, int B, TunePlan* p) {
  if (B < 1 || B > B_fwd || !tune_plan(H, B_fwd, p)) return false;
  if (B == B_fwd) return true;
  TunePlan n;
  if (!tune_plan(H, B, &n)) return false;
  p->B = B;
  p->M = n.M;
  p->tf_grid = n.tf_grid;
  p->lin_grid = n.lin_grid;
  p->dw_grid = n.dw_grid;
  p->dec_s = n.dec_s;
  p->dec_dws = n.dec_dws;
  return true;
}

hipError_t launch_tune_forward(const TunePlan& p, const float* windows, const float* P, float* ws, float* latent,
                               float* logits, float* protos, hipStream_t st, hipEvent_t post) {
  switch (p.H) {
#define CASE(h) \
  case h:       \
    return tune_fwd_h<h>(p, windows, P, ws, latent, logits, protos, st, post);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_tune_backward(const TunePlan& p, const float* P, float* G, float* ws, const float* logits,
                                const float* protos, const int* y, const float* mult, const float* tgt,
                                hipStream_t st, bool dpre_ready, hipEvent_t pre) {
  switch (p.H) {
#define CASE(h) \
  case h:       \
    return tune_bwd_h<h>(p, P, G, ws, logits, protos, y, mult, tgt, st, dpre_ready, pre);
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
