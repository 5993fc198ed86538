// pgp_dec.hip — the tuning step's decoder GEMMs (models.py:359-370, 399):
//   forward  pre[b][n]     = sum_k X2[b][k] Wp[n][k]         k = tok*DP + c
//   backward dX2[b][tok][c] = sum_n dpre[b][n] Wp[n][tok*DP + c]
// over the encoder output X2 in token layout ([M][DP], row b*T + tok) and the
// decoder weights permuted to it (pgp_tune.hip dec_pack_kernel: Wp [NOP][KD],
// WpT [T][DP][NOP]).  Both are f32 MFMA (v_mfma_f32_16x16x4_f32) GEMMs whose
// weight operand is shared by a workgroup of 8 waves (2 per SIMD): it is copied
// global -> LDS asynchronously (global_load_lds_dwordx4, one 1-KiB A-fragment
// group per instruction, in the natural row map k = 16q + 4g + e so that one
// ds_read_b128 feeds 4 k-steps) while the previous token computes.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pgp_device.hpp"
#include "pgp_gemm.hpp"
#include "pgp_tune.hpp"

namespace pgp {
namespace {

constexpr int kDecWaves = 8;  // b-tiles (16 windows) per workgroup

PGP_DEV void dma_piece(const float* src, float* dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// Split-K forward: workgroup (x: 8 b-tiles, y: token range s of S) writes
// part[s][b][n].  Per token: 13 A groups x 4 k-blocks of Wp (52 KiB, double
// buffered in LDS); the wave's X2 row block (16 windows x DP) is the B operand,
// loaded one token ahead.  Feature pads: k-steps of the last k-block whose
// columns are all pads (e >= H - 16 (KB - 1); e = 2, 3 at H = 50) are skipped.
template <int H>
__global__ __launch_bounds__(kDecWaves * 64) void dec_fwd2_kernel(int B, int S, const float* __restrict__ X2,
                                                                  const float* __restrict__ Wp,
                                                                  float* __restrict__ part) {
  using Q = TuneGeo<H>;
  constexpr int NT = Q::NOP / 16, KB = Q::DP / 16, PCS = NT * KB;
  // k-steps of the last k-block that touch a real feature: 16(KB-1) + 4g + e < H for some g
  constexpr int ELAST = (H - 16 * (KB - 1)) >= 4 ? 4 : (H - 16 * (KB - 1));
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [2][PCS][256]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const long b = ((long)blockIdx.x * kDecWaves + wv) * 16 + j;
  const bool okb = b < B;
  const int s = blockIdx.y;
  const int tok0 = Q::T * s / S, tok1 = Q::T * (s + 1) / S;
  auto dma = [&](int tok, int buf) {
    for (int pc = wv; pc < PCS; pc += kDecWaves) {
      const int t = pc / KB, kb = pc - t * KB;
      dma_piece(Wp + (long)(16 * t + j) * Q::KD + (long)tok * Q::DP + 16 * kb + 4 * g,
                lds + (buf * PCS + pc) * 256);
    }
  };
  // a lane past the batch reads window 0 (clamped address) into its own
  // column, which is not stored; no select on the loaded value, so the next
  // token's loads are not waited for before this token's MFMAs
  const float* xr = X2 + (okb ? b : 0) * Q::T * Q::DP + 4 * g;
  // (the last k-block reads only its ELAST live features: a dead half of a
  // float4 would let the compiler reuse its registers right after the load,
  // which makes it wait for the prefetch before this token's MFMAs)
  auto xload = [&](int tok, f32x4 (&x)[KB]) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const float* p = xr + (long)tok * Q::DP + 16 * kb;
      if (kb == KB - 1 && ELAST <= 2) {
        const float2 v = *reinterpret_cast<const float2*>(p);
        x[kb] = f32x4{v.x, v.y, 0.f, 0.f};
      } else {
        x[kb] = ld4(p);
      }
    }
  };
  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = zero4();
  f32x4 xc[KB], xn[KB];
  if (tok0 < tok1) {
    dma(tok0, 0);
    xload(tok0, xc);
  }
#pragma unroll 1
  for (int tok = tok0; tok < tok1; ++tok) {
    const int buf = (tok - tok0) & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // token tok landed for every wave; buffer buf ^ 1 is free
    if (tok + 1 < tok1) {
      dma(tok + 1, buf ^ 1);
      xload(tok + 1, xn);
    }
    const float* L = lds + buf * PCS * 256 + lane * 4;
    // k-block outer, output tile inner: consecutive MFMAs go to different
    // accumulators (a tile's 16 MFMAs in a row waited on each other)
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      f32x4 a[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) a[t] = ld4(L + (t * KB + kb) * 256);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (kb < KB - 1 || e < ELAST)
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = mfma(a[t][e], xc[kb][e], acc[t]);
    }
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) xc[kb] = xn[kb];
  }
  if (okb) {
#pragma unroll
    for (int t = 0; t < NT; ++t) st4(part + ((long)s * B + b) * Q::NOP + 16 * t + 4 * g, acc[t]);
  }
}

// Backward into the encoder output: workgroup (x: 8 b-tiles, y: token) computes
// dX2[b][tok][0..DP) = sum_n dpre[b][n] WpT[tok][c][n]; A = WpT[tok] (DP x NOP,
// 52 KiB in LDS), B = the wave's dpre rows (registers).  Pad columns come out 0.
template <int H>
__global__ __launch_bounds__(kDecWaves * 64) void dec_dx_kernel(int B, const float* __restrict__ dpre,
                                                                const float* __restrict__ WpT,
                                                                float* __restrict__ dX) {
  using Q = TuneGeo<H>;
  constexpr int CT = Q::DP / 16, QG = Q::NOP / 16, PCS = CT * QG;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [PCS][256]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int tok = blockIdx.y;
  const long b = ((long)blockIdx.x * kDecWaves + wv) * 16 + j;
  const bool okb = b < B;
  for (int pc = wv; pc < PCS; pc += kDecWaves) {
    const int ct = pc / QG, q = pc - ct * QG;
    dma_piece(WpT + ((long)tok * Q::DP + 16 * ct + j) * Q::NOP + 16 * q + 4 * g, lds + pc * 256);
  }
  f32x4 x[QG];
  const float* dr = dpre + (okb ? b : 0) * Q::NOP + 4 * g;
#pragma unroll
  for (int q = 0; q < QG; ++q) {
    const f32x4 v = ld4(dr + 16 * q);
    x[q] = okb ? v : zero4();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if ((long)((long)blockIdx.x * kDecWaves + wv) * 16 >= B) return;  // a b-tile past the batch (after the barrier)
  f32x4 acc[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) acc[ct] = zero4();
  const float* L = lds + lane * 4;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int q = 0; q < QG; ++q) {
      const f32x4 a = ld4(L + (ct * QG + q) * 256);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[ct] = mfma(a[e], x[q][e], acc[ct]);
    }
  if (okb) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) st4(dX + ((long)b * Q::T + tok) * Q::DP + 16 * ct + 4 * g, acc[ct]);
  }
}

template <int H>
hipError_t dec_fwd_h(int B, int S, const float* X2, const float* Wp, float* part, hipStream_t st) {
  using Q = TuneGeo<H>;
  constexpr int PCS = (Q::NOP / 16) * (Q::DP / 16);
  constexpr size_t lds = 2 * PCS * 1024;
  static_assert(lds <= 160 * 1024, "decoder forward LDS");
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dec_fwd2_kernel<H>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return true;
  }();
  (void)attr;
  const int bg = (B + 16 * kDecWaves - 1) / (16 * kDecWaves);
  dec_fwd2_kernel<H><<<dim3(bg, S), kDecWaves * 64, lds, st>>>(B, S, X2, Wp, part);
  return hipGetLastError();
}

template <int H>
hipError_t dec_dx_h(int B, const float* dpre, const float* WpT, float* dX, hipStream_t st) {
  using Q = TuneGeo<H>;
  constexpr int PCS = (Q::NOP / 16) * (Q::DP / 16);
  constexpr size_t lds = PCS * 1024;
  static_assert(lds <= 160 * 1024, "decoder backward LDS");
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dec_dx_kernel<H>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    return true;
  }();
  (void)attr;
  const int bg = (B + 16 * kDecWaves - 1) / (16 * kDecWaves);
  dec_dx_kernel<H><<<dim3(bg, Q::T), kDecWaves * 64, lds, st>>>(B, dpre, WpT, dX);
  return hipGetLastError();
}

}  // namespace

int dec_fwd_splits(int H, int B) {
  const int bg = (B + 16 * kDecWaves - 1) / (16 * kDecWaves);
  return std::max(1, std::min(3 * H, device_cus() / std::max(1, bg)));
}

hipError_t launch_dec_fwd(int H, int B, int S, const float* X2, const float* Wp, float* part, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return dec_fwd_h<h>(B, S, X2, Wp, part, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_dec_dx(int H, int B, const float* dpre, const float* WpT, float* dX, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return dec_dx_h<h>(B, dpre, WpT, dX, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
