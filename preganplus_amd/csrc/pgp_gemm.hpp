// pgp_gemm.hpp — device building blocks shared by the batch-major training
// kernels (pgp_tune.hip: tuning step, pgp_gantrain.hip: GAN step).
#pragma once
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"

namespace pgp {

PGP_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
PGP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// sum over the 16 lanes of one lane group (the 16 token rows of a tile)
PGP_DEV float row16_sum(float v) {
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// sum over a 32-lane half wave
PGP_DEV float half_sum(float v) {
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o);
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
#ifndef PGP_DW_ROWS
#define PGP_DW_ROWS 32
#endif
constexpr int kDwRows = PGP_DW_ROWS;  // rows per LDS-staged chunk of the weight-gradient contractions

template <int NP, int KP, int NTW>
PGP_DEV void dw_accumulate(long r0, long r1, const float* __restrict__ Y, long ldy, const float* __restrict__ X,
                           long ldx, int relu_x, int tbase, int tstride, float* ys, float* xs,
                           f32x4 (&acc)[NTW][KP / 16], float (&pb)[NTW], int ny = NP, int nx = KP) {
  constexpr int NT = NP / 16, KT = KP / 16, YS = lds_stride(NP), XS = lds_stride(KP);
  constexpr int NY = (kDwRows * NP / 4 + 255) / 256, NX = (kDwRows * KP / 4 + 255) / 256;  // float4 per thread
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  f32x4 ry[NY], rx[NX];
  // software pipeline: chunk c+1 is loaded into registers while chunk c is computed from LDS
  auto fetch = [&](long c0) {
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int idx = threadIdx.x + 256 * k, row = idx / (NP / 4), c4 = idx - row * (NP / 4);
      const long m = c0 + row;
      ry[k] = (idx < kDwRows * NP / 4 && m < r1 && 4 * c4 < ny) ? ld4(Y + m * ldy + 4 * c4) : zero4();
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int idx = threadIdx.x + 256 * k, row = idx / (KP / 4), c4 = idx - row * (KP / 4);
      const long m = c0 + row;
      rx[k] = (idx < kDwRows * KP / 4 && m < r1 && 4 * c4 < nx) ? ld4(X + m * ldx + 4 * c4) : zero4();
    }
  };
  if (r0 < r1) fetch(r0);
  for (long c0 = r0; c0 < r1; c0 += kDwRows) {
    __syncthreads();  // the previous chunk has been consumed
#pragma unroll
    for (int k = 0; k < NY; ++k) {
      const int idx = threadIdx.x + 256 * k, row = idx / (NP / 4), c4 = idx - row * (NP / 4);
      if (idx < kDwRows * NP / 4) st4(ys + row * YS + 4 * c4, ry[k]);
    }
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int idx = threadIdx.x + 256 * k, row = idx / (KP / 4), c4 = idx - row * (KP / 4);
      f32x4 v = rx[k];
      if (relu_x) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      if (idx < kDwRows * KP / 4) st4(xs + row * XS + 4 * c4, v);
    }
    __syncthreads();
    if (c0 + kDwRows < r1) fetch(c0 + kDwRows);
#pragma unroll 2
    for (int s = 0; s < kDwRows / 4; ++s) {
      const int row = 4 * s + g;
      float bv[KT];
#pragma unroll
      for (int u = 0; u < KT; ++u) bv[u] = xs[row * XS + 16 * u + i];
#pragma unroll
      for (int q = 0; q < NTW; ++q) {
        const int t = tbase + wv + tstride * q;
        if (t < NT) {
          const float av = ys[row * YS + 16 * t + i];
          pb[q] += av;
#pragma unroll
          for (int u = 0; u < KT; ++u) acc[q][u] = mfma(av, bv[u], acc[q][u]);
        }
      }
    }
  }
}

}  // namespace pgp
