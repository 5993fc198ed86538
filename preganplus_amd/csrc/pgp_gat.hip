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

namespace pgp {
namespace {

__device__ __forceinline__ float lrelu001(float e) { return fmaxf(e, 0.01f * e); }  // slope 0.01 < 1

// One workgroup per 16-window block: 4 waves x 12 (window, step) items, lane =
// destination host.  The block's aggregation [H][3][48] is assembled in LDS and
// written out with contiguous 16-B stores (scattered 4-B stores amplified the
// HBM writes 6x: profiles/r01/pmc_r01pmc2_summary.txt).
template <int H>
__global__ __launch_bounds__(256) void gat_agg_kernel(int B, const float* __restrict__ win,
                                                      float* __restrict__ agg, GatConst gc) {
  static_assert(H <= 64, "GAT kernel maps hosts to lanes");
  constexpr int BLK = H * 3 * 48;  // floats per 16-window block
  __shared__ __attribute__((aligned(16))) float out_lds[BLK];
  __shared__ f32x4 sx[4][64];  // {A_i, x_i}
  __shared__ float sa[4][64];  // A'_i
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long blk = blockIdx.x;
  for (int i = threadIdx.x; i < BLK; i += 256) out_lds[i] = 0.f;
  __syncthreads();
  for (int it = wv; it < 48; it += 4) {
    const int j = it / 3, w = it % 3;
    const long b = blk * 16 + j;
    const bool active = b < B;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
    if (active && lane < H) {
      const float* p = win + (b * 3 + w) * 3 * H + 3 * lane;
      x0 = p[0];
      x1 = p[1];
      x2 = p[2];
    }
    const float s = gc.u[0] * x0 + gc.u[1] * x1 + gc.u[2] * x2;
    const float t = gc.v[0] * x0 + gc.v[1] * x1 + gc.v[2] * x2;
    float smax = lane < H ? s : -INFINITY, tmax = lane < H ? t : -INFINITY;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      smax = fmaxf(smax, __shfl_xor(smax, off));
      tmax = fmaxf(tmax, __shfl_xor(tmax, off));
    }
    const float M = lrelu001(smax + tmax);  // = max_ij e_ij (lrelu and rounding are monotone)
    // u,v are pre-scaled by log2(e): the factors are v_exp_f32 (2^x) of the scaled terms
    const float ds = s - smax;
    sx[wv][lane] = f32x4{__builtin_amdgcn_exp2f(ds), x0, x1, x2};
    sa[wv][lane] = __builtin_amdgcn_exp2f(0.01f * ds);
    const float Bp = __builtin_amdgcn_exp2f(t + smax - M);
    const float Bn = __builtin_amdgcn_exp2f(0.01f * (t + smax) - M);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    float S = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll 5
    for (int i = 0; i < H; ++i) {
      const f32x4 v = sx[wv][i];
      const float p = fmaxf(v.x * Bp, sa[wv][i] * Bn);  // exp2(lrelu(s_i + t_j) - M)
      S += p;
      a0 += p * v.y;
      a1 += p * v.z;
      a2 += p * v.w;
    }
    float St = lane < H ? S : 0.f;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) St += __shfl_xor(St, off);
    if (active && lane < H) {
      const float inv = 1.0f / St;
      float* o = out_lds + (lane * 3 + w) * 48 + j;
      o[0] = a0 * inv;
      o[16] = a1 * inv;
      o[32] = a2 * inv;
    }
    __builtin_amdgcn_wave_barrier();  // sx is reused by this wave's next item
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
