// pgp_gemm.hpp — device building blocks shared by the batch-major training
// kernels (pgp_tune.hip: tuning step, pgp_gantrain.hip: GAN step).
#pragma once
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"

namespace pgp {

// Cross-lane butterflies without ds_bpermute round trips: xor 1 / 2 as DPP
// quad_perm, xor 8 as DPP row_ror 8, xor 4 as two bank-masked DPP row shifts,
// xor 16 / 32 as the gfx950 row / half swaps (v_permlane16/32_swap).  Each
// step returns own <op> partner exactly as v <op> __shfl_xor(v, o) did, so the
// butterflies keep their association and results are bitwise unchanged.
template <int O>
PGP_DEV float xpartner(float v) {  // the value of lane ^ O, O in {1, 2, 4, 8}
  const int b = __float_as_int(v);
  if constexpr (O == 1) return __int_as_float(__builtin_amdgcn_update_dpp(0, b, 0xB1, 0xF, 0xF, false));
  if constexpr (O == 2) return __int_as_float(__builtin_amdgcn_update_dpp(0, b, 0x4E, 0xF, 0xF, false));
  if constexpr (O == 8) return __int_as_float(__builtin_amdgcn_update_dpp(0, b, 0x128, 0xF, 0xF, false));
  if constexpr (O == 4) {
    const int lo = __builtin_amdgcn_update_dpp(0, b, 0x104, 0xF, 0x5, false);    // row_shl 4 into banks 0, 2
    return __int_as_float(__builtin_amdgcn_update_dpp(lo, b, 0x114, 0xF, 0xA, false));  // row_shr 4 into 1, 3
  }
  static_assert(O == 1 || O == 2 || O == 4 || O == 8, "in-row partner");
  return v;
}
// v + v[lane ^ O] for any O in {1, ..., 32}
template <int O>
PGP_DEV float xadd(float v) {
  if constexpr (O == 16 || O == 32) {
    const unsigned u = __float_as_uint(v);
    const auto r = O == 16 ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                           : __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // own + partner in either order: a+b == b+a
  } else {
    return v + xpartner<O>(v);
  }
}
template <int O>
PGP_DEV float xmax(float v) {
  if constexpr (O == 16 || O == 32) {
    const unsigned u = __float_as_uint(v);
    const auto r = O == 16 ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                           : __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  } else {
    return fmaxf(v, xpartner<O>(v));
  }
}

PGP_DEV float wave_max(float v) {
  v = xmax<32>(v);
  v = xmax<16>(v);
  v = xmax<8>(v);
  v = xmax<4>(v);
  v = xmax<2>(v);
  return xmax<1>(v);
}
PGP_DEV float wave_sum(float v) {
  v = xadd<32>(v);
  v = xadd<16>(v);
  v = xadd<8>(v);
  v = xadd<4>(v);
  v = xadd<2>(v);
  return xadd<1>(v);
}
// sum over the 16 lanes of one lane group (the 16 token rows of a tile)
PGP_DEV float row16_sum(float v) {
  v = xadd<8>(v);
  v = xadd<4>(v);
  v = xadd<2>(v);
  return xadd<1>(v);
}
// sum over 32 lanes (lane ^ 16 ... lane ^ 1)
PGP_DEV float half_sum(float v) {
  v = xadd<16>(v);
  return row16_sum(v);
}
// max / sum over aligned S-lane segments (S a power of two <= 64), offsets S/2 .. 1
template <int S>
PGP_DEV float seg_max(float v) {
  if constexpr (S >= 64) v = xmax<32>(v);
  if constexpr (S >= 32) v = xmax<16>(v);
  if constexpr (S >= 16) v = xmax<8>(v);
  if constexpr (S >= 8) v = xmax<4>(v);
  if constexpr (S >= 4) v = xmax<2>(v);
  if constexpr (S >= 2) v = xmax<1>(v);
  return v;
}
template <int S>
PGP_DEV float seg_sum(float v) {
  if constexpr (S >= 64) v = xadd<32>(v);
  if constexpr (S >= 32) v = xadd<16>(v);
  if constexpr (S >= 16) v = xadd<8>(v);
  if constexpr (S >= 8) v = xadd<4>(v);
  if constexpr (S >= 4) v = xadd<2>(v);
  if constexpr (S >= 2) v = xadd<1>(v);
  return v;
}
PGP_DEV f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
PGP_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
PGP_DEV float lrelu(float x) { return x > 0.f ? x : 0.01f * x; }

// ============================================================================
// Weight gradients: sum over rows of Y[row][n] X[row][k].  Rows are staged 32 at
// a time through LDS with float4 loads; wave wv owns n-tiles tbase + wv +
// tstride*q and every k-tile; the contraction (MFMA k) runs over the rows.
// LDS row strides are = 16 (mod 64) floats so the 4 lane groups (4 rows) of a
// fragment read hit disjoint banks.
// ============================================================================
constexpr int lds_stride(int n) { return n + ((16 - n % 64) % 64 + 64) % 64; }
static __device__ __attribute__((aligned(16))) float dw_zero4[4];  // zero, read by masked-off lanes
constexpr int kDwRows = 32;  // rows per LDS-staged chunk of the weight-gradient contractions

template <int NP, int KP, int NTW, int ROWS = kDwRows>
PGP_DEV void dw_accumulate(long r0, long r1, const float* __restrict__ Y, long ldy, const float* __restrict__ X,
                           long ldx, int relu_x, int tbase, int tstride, float* ys, float* xs,
                           f32x4 (&acc)[NTW][KP / 16], float (&pb)[NTW], int ny = NP, int nx = KP) {
  constexpr int NT = NP / 16, KT = KP / 16, YS = lds_stride(NP), XS = lds_stride(KP);
  constexpr int NY = (ROWS * NP / 4 + 255) / 256, NX = (ROWS * KP / 4 + 255) / 256;  // float4 per thread
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int tq[NTW];  // this wave's n-tiles (clamped; see below)
#pragma unroll
  for (int q = 0; q < NTW; ++q) tq[q] = min(tbase + wv + tstride * q, NT - 1);
  f32x4 ry[NY], rx[NX];
  // software pipeline: chunk c+1 is loaded into registers while chunk c is
  // computed from LDS.  Rows past the range read a zero float4 (the ADDRESS
  // is selected: a select on the loaded value would make the compiler wait for
  // the prefetch at once, before the chunk's MFMAs)
  auto fetch = [&](long c0) {
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int idx = threadIdx.x + 256 * k, row = idx / (NP / 4), c4 = idx - row * (NP / 4);
      const long m = c0 + row;
      ry[k] = ld4((idx < ROWS * NP / 4 && m < r1 && 4 * c4 < ny) ? Y + m * ldy + 4 * c4 : dw_zero4);
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int idx = threadIdx.x + 256 * k, row = idx / (KP / 4), c4 = idx - row * (KP / 4);
      const long m = c0 + row;
      rx[k] = ld4((idx < ROWS * KP / 4 && m < r1 && 4 * c4 < nx) ? X + m * ldx + 4 * c4 : dw_zero4);
    }
  };
  if (r0 < r1) fetch(r0);
  for (long c0 = r0; c0 < r1; c0 += ROWS) {
    __syncthreads();  // the previous chunk has been consumed
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int idx = threadIdx.x + 256 * k, row = idx / (NP / 4), c4 = idx - row * (NP / 4);
      if (idx < ROWS * NP / 4) st4(ys + row * YS + 4 * c4, ry[k]);
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int idx = threadIdx.x + 256 * k, row = idx / (KP / 4), c4 = idx - row * (KP / 4);
      f32x4 v = rx[k];
      if (relu_x) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (idx < ROWS * KP / 4) st4(xs + row * XS + 4 * c4, v);
    }
    __syncthreads();
    if (c0 + ROWS < r1) fetch(c0 + ROWS);
    // the chunk's 8 row groups, fully unrolled and branch-free: a wave whose
    // tile q is past NT computes tile NT - 1 again and never stores it, so the
    // compiler can issue the next group's LDS reads under this group's MFMAs
#pragma unroll
    for (int s = 0; s < ROWS / 4; ++s) {
      const int row = 4 * s + g;
      float bv[KT];
#pragma unroll
      for (int u = 0; u < KT; ++u) bv[u] = xs[row * XS + 16 * u + i];
#pragma unroll
      for (int q = 0; q < NTW; ++q) {
        const float av = ys[row * YS + 16 * tq[q] + i];
        pb[q] += av;
#pragma unroll
        for (int u = 0; u < KT; ++u) acc[q][u] = mfma(av, bv[u], acc[q][u]);
      }
    }
  }
}

}  // namespace pgp
