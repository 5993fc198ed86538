// pgp_gat.hip — K1: GAT edge softmax + aggregation (dlutils.py:304-348).
//
//   s_i = u.x_i, t_j = v.x_j           (attn_fc split, folded through fc, pre-scaled by
//                                       log2(e) so exp() is one v_exp_f32: pgp_pack.cpp)
//   e_ij = leaky_relu_0.01(s_i + t_j)  (dlutils.py:329)
//   a_ij = exp(e_ij - M) / sum_{i,j} exp(e_ij - M)   graph-wise over all H^2 edges
//                                      (dgl.softmax_edges, dlutils.py:335)
//   agg_j = sum_i a_ij x_i             (update_all src_mul_edge/sum, dlutils.py:338-342,
//                                       taken before the linear fc)
// The H^2 exponentials factorise: exp is monotone, so exp(lrelu(e) - M) =
// max(exp(e - M), exp(0.01 e - M)), and each branch is a product of a source
// factor and a destination factor:
//   exp(s_i + t_j - M)        = A_i  * B_j,   A_i  = exp(s_i - smax),         B_j  = exp(t_j + smax - M)
//   exp(0.01 (s_i + t_j) - M) = A'_i * B'_j,  A'_i = exp(0.01 (s_i - smax)),  B'_j = exp(0.01 (t_j + smax) - M)
// Every factor is <= 1 (M = lrelu(smax + tmax)), so nothing overflows, and the
// edge loop is 2 multiplies and a max instead of an add, lrelu and v_exp_f32
// (4H exponentials per graph instead of H^2).
// Output = the B operand of the encoder's time-encoder MFMA:
//   agg[((blk*H + j)*3 + w)*48 + f*16 + (b & 15)]
#include "pgp_device.hpp"
#include "pgp_gemm.hpp"

namespace pgp {
namespace {

__device__ __forceinline__ float lrelu001(float e) { return fmaxf(e, 0.01f * e); }  // slope 0.01 < 1

// One workgroup per 16-window block: 4 waves over the block's 48 (window, step)
// items, lane = destination host.  For H <= 32 a wave holds P = 64 / S items at
// once, one per S-lane segment (S = the power of two >= H): at H = 16 a
// one-item wave left 3/4 of its lanes idle.  Segment reductions are xor
// butterflies below S (DPP and row swaps, seg_max / seg_sum); the per-item source tables in LDS are padded by one entry per segment
// so the P segments' broadcast reads fall in different banks.  The block's
// aggregation [H][3][48] is assembled in LDS and written out with contiguous
// 16-B stores (scattered 4-B stores amplified the HBM writes 6x:
// profiles/r01/pmc_r01pmc2_summary.txt).
// one-item-per-wave mode (H > 32): load the next item's features one item
// ahead (kGatPf), and the edge loop's independent accumulation chains (kGatChains)
constexpr bool kGatPf = true;
constexpr int kGatChains = 2;
constexpr int seg_lanes(int h) { return h <= 8 ? 8 : h <= 16 ? 16 : h <= 32 ? 32 : 64; }

template <int H>
__global__ __launch_bounds__(256) void gat_agg_kernel(int B, const float* __restrict__ win,
                                                      float* __restrict__ agg, const float* __restrict__ gcp) {
  static_assert(H <= 64, "GAT kernel maps hosts to lanes");
  constexpr int S = seg_lanes(H), P = 64 / S, SS = P > 1 ? S + 1 : S;
  constexpr int BLK = H * 3 * 48;  // floats per 16-window block
  __shared__ __attribute__((aligned(16))) float out_lds[BLK];
  __shared__ f32x4 sx[4][P * SS];                // P == 1: {A_i, A'_i, x_i0, x_i1}; else {A_i, x_i}
  __shared__ f32x2 sy[4][P == 1 ? P * SS : 1];    // P == 1: {x_i2, 1}
  __shared__ float sa[4][P == 1 ? 1 : P * SS];    // P > 1: A'_i
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int seg = lane / S, hl = lane % S;  // item slot, destination host
  const long blk = blockIdx.x;
  const float gu0 = gcp[0], gu1 = gcp[1], gu2 = gcp[2], gv0 = gcp[4], gv1 = gcp[5], gv2 = gcp[6];
  for (int i = threadIdx.x; i < BLK; i += 256) out_lds[i] = 0.f;
  __syncthreads();
  // P == 1 (H > 32): the next item's features are loaded one item ahead, from a
  // clamped address (unconditional loads, zeroed when out of range)
  constexpr bool PF1 = P == 1 && kGatPf;
  auto ldx = [&](int i0, float& x0, float& x1, float& x2) {
    const int it = i0 + seg;
    const long b = blk * 16 + it / 3;
    const bool ok = it < 48 && b < B && hl < H;
    const float* p = win + (ok ? (b * 3 + it % 3) * 3 * H + 3 * hl : 0);
    x0 = p[0];
    x1 = p[1];
    x2 = p[2];
    if (!ok) x0 = x1 = x2 = 0.f;
  };
  float nx0 = 0.f, nx1 = 0.f, nx2 = 0.f;
  if constexpr (PF1) ldx(wv * P, nx0, nx1, nx2);
  for (int i0 = wv * P; i0 < 48; i0 += 4 * P) {
    const int it = i0 + seg;
    const int j = it / 3, w = it % 3;
    const long b = blk * 16 + j;
    const bool active = it < 48 && b < B;
    const bool host = hl < H;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
    if constexpr (PF1) {
      x0 = nx0;
      x1 = nx1;
      x2 = nx2;
      ldx(i0 + 4 * P < 48 ? i0 + 4 * P : i0, nx0, nx1, nx2);
    } else if (active && host) {
      const float* p = win + (b * 3 + w) * 3 * H + 3 * hl;
      x0 = p[0];
      x1 = p[1];
      x2 = p[2];
    }
    const float s = gu0 * x0 + gu1 * x1 + gu2 * x2;
    const float t = gv0 * x0 + gv1 * x1 + gv2 * x2;
    float smax = host ? s : -INFINITY, tmax = host ? t : -INFINITY;
    smax = seg_max<S>(smax);  // DPP / row swaps, no ds_bpermute (pgp_gemm.hpp)
    tmax = seg_max<S>(tmax);
    const float M = lrelu001(smax + tmax);  // = max_ij e_ij (lrelu and rounding are monotone)
    // u,v are pre-scaled by log2(e): the factors are v_exp_f32 (2^x) of the scaled terms
    const float ds = s - smax;
    const int base = seg * SS;
    const float Ap = __builtin_amdgcn_exp2f(ds), An = __builtin_amdgcn_exp2f(0.01f * ds);
    const float Bp = __builtin_amdgcn_exp2f(t + smax - M);
    const float Bn = __builtin_amdgcn_exp2f(0.01f * (t + smax) - M);
    float S_, a0, a1, a2;
    if constexpr (P == 1) {
      // one item per wave (H > 32): the edge loop is latency-bound on its
      // accumulation chains, so packed f32 (one v_pk_mul for both branch
      // products, a max, two v_pk_fma for (a0, a1) and (a2, S)) over kGatChains
      // interleaved chains (source i -> chain i mod NC) summed at the end
      sx[wv][base + hl] = f32x4{Ap, An, x0, x1};
      sy[wv][base + hl] = f32x2{x2, 1.f};
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      const f32x2 Bpn = {Bp, Bn};
      constexpr int NC = kGatChains;
      f32x2 a01[NC], a2s[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) a01[c] = a2s[c] = f32x2{0.f, 0.f};
      auto edge = [&](int i, int c) {
        const f32x4 v = sx[wv][base + i];
        const f32x2 q = f32x2{v.x, v.y} * Bpn;
        const float p = fmaxf(q.x, q.y);  // exp2(lrelu(s_i + t_j) - M)
        const f32x2 pp = {p, p};
        a01[c] = __builtin_elementwise_fma(pp, f32x2{v.z, v.w}, a01[c]);
        a2s[c] = __builtin_elementwise_fma(pp, sy[wv][base + i], a2s[c]);
      };
#pragma unroll 5
      for (int i = 0; i + NC <= H; i += NC)
#pragma unroll
        for (int c = 0; c < NC; ++c) edge(i + c, c);
#pragma unroll
      for (int c = 0; c < H % NC; ++c) edge(H - H % NC + c, c);
      f32x2 s01 = a01[0], s2s = a2s[0];
#pragma unroll
      for (int c = 1; c < NC; ++c) {
        s01 += a01[c];
        s2s += a2s[c];
      }
      S_ = s2s.y;
      a0 = s01.x;
      a1 = s01.y;
      a2 = s2s.x;
    } else {
      // P items per wave already interleave P independent chains
      sx[wv][base + hl] = f32x4{Ap, x0, x1, x2};
      sa[wv][base + hl] = An;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
      __builtin_amdgcn_wave_barrier();
      S_ = a0 = a1 = a2 = 0.f;
      auto edge = [&](int i) {
        const f32x4 v = sx[wv][base + i];
        const float p = fmaxf(v.x * Bp, sa[wv][base + i] * Bn);  // exp2(lrelu(s_i + t_j) - M)
        S_ += p;
        a0 += p * v.y;
        a1 += p * v.z;
        a2 += p * v.w;
      };
#pragma unroll 4
      for (int i = 0; i < H; ++i) edge(i);
    }
    float St = host ? S_ : 0.f;
    St = seg_sum<S>(St);
    if (active && host) {
      const float inv = 1.0f / St;
      float* o = out_lds + (hl * 3 + w) * 48 + j;
      o[0] = a0 * inv;
      o[16] = a1 * inv;
      o[32] = a2 * inv;
    }
    __builtin_amdgcn_wave_barrier();  // sx is reused by this wave's next items
  }
  __syncthreads();
  f32x4* dst = reinterpret_cast<f32x4*>(agg + blk * BLK);
  const f32x4* src = reinterpret_cast<const f32x4*>(out_lds);
  for (int i = threadIdx.x; i < BLK / 4; i += 256) dst[i] = src[i];
}

template <int H>
hipError_t launch(const FwdArgs& a, hipStream_t st) {
  const long nblk = (a.B + 15) / 16;
  gat_agg_kernel<H><<<(int)nblk, 256, 0, st>>>(a.B, a.windows, a.agg, a.gat);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_gat(const FwdArgs& a, hipStream_t st) {
  switch (a.H) {
#define CASE(h) \
  case h:       \
    return launch<h>(a, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
