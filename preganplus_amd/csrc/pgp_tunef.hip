// pgp_tunef.hip — the tuning step's Transformer encoder (models.py:344-356,
// 390-396; train.py:42-57) as fused per-unit kernels, windows on lanes.
//
// A unit is 16 (window, host) pairs, p = b*H + h (16u .. 16u+15); lane column
// j = lane & 15 is pair 16u + j and its 3 window steps are 3 column tiles, so
// the 3-step attention is lane-local and every activation of a layer lives in
// v_mfma_f32_16x16x4_f32 accumulators: feature row c = 16t + 4g + r in tile t,
// lane group g = lane >> 4, register r ("N layout", the natural row order of
// the token-major buffers, so a tile row group is one 16-byte load).  Weights
// are A-operand fragments packed from the master P each step (tf_pack_kernel)
// and held in LDS; an activation register is directly the B operand of the
// next GEMM.  Per layer:
//   tf_fwd      X -> q|k|v -> attention -> out_proj + X -> LN1 -> FFN -> LN2,
//               storing only X, LN1's x-hat / rstd and the layer output;
//   tf_bwd_ffn  from dOut (grad of the layer output): recompute the FFN from
//               LN1's x-hat, LN2 / linear2 / linear1 / LN1 backward -> dR1;
//               dW2, dW1 (+ biases) and both LayerNorms' gamma / beta
//               gradients accumulated in registers over the wave's units;
//   tf_bwd_att  from dR1: recompute q|k|v and the attention from X, out_proj /
//               attention / in_proj backward -> dX; dWo (+ bias) in registers;
//               dQKV to HBM for in_proj's weight gradient (tall contraction).
// Weight gradients contract over tokens, which sit on lane columns: each step's
// 16 tokens are staged through a per-wave LDS scratch ([token][row]) and read
// back with the token as the MFMA k index (lane group g <-> tokens 4g..4g+3,
// one k-step per register).  The waves of a workgroup combine their registers
// in a fixed order at the end, one partial slab per workgroup, reduced in a
// fixed order by the tuning step's deferred reduction: deterministic.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "pgp_device.hpp"
#include "pgp_gemm.hpp"
#include "pgp_train.hpp"
#include "pgp_tune.hpp"
#include "pgp_tunef.hpp"

namespace pgp {
namespace {

constexpr int kTfWaves = 4;  // one wave per SIMD (the backward needs > 256 registers)

// Phase attribution (profiling builds only: make variant NAME=st
// VFLAGS=-DPGP_TF_STAMPS, read by tools/tf_stamps.py): each wave adds the
// shader-clock cycles between consecutive TF_ST(k) marks to phase k of its slot
// in tf_stamps[kind][wave] (vector stores by lane 0; one writer per slot).
#ifdef PGP_TF_STAMPS
constexpr int kStPhases = 16, kStWaves = 2048;
__device__ unsigned long long tf_stamps[4][kStWaves][kStPhases];
#define TF_ST_INIT()                                              \
  unsigned long long st_acc[kStPhases];                           \
  for (int _k = 0; _k < kStPhases; ++_k) st_acc[_k] = 0;          \
  unsigned long long st_t = __builtin_amdgcn_s_memtime()
#define TF_ST(k)                                                  \
  do {                                                            \
    __builtin_amdgcn_sched_barrier(0);                            \
    const unsigned long long _n = __builtin_amdgcn_s_memtime();   \
    st_acc[k] += _n - st_t;                                       \
    st_t = _n;                                                    \
    __builtin_amdgcn_sched_barrier(0);                            \
  } while (0)
#define TF_ST_END(kind)                                                                    \
  do {                                                                                     \
    const int _w = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));                 \
    if ((threadIdx.x & 63) == 0 && _w < kStWaves)                                          \
      for (int _k = 0; _k < kStPhases; ++_k) tf_stamps[kind][_w][_k] += st_acc[_k];         \
  } while (0)
#else
#define TF_ST_INIT() \
  do {               \
  } while (0)
#define TF_ST(k) \
  do {           \
  } while (0)
#define TF_ST_END(kind) \
  do {                  \
  } while (0)
#endif

template <int H>
__global__ __launch_bounds__(256) void tf_pack_kernel(const float* __restrict__ P, float* __restrict__ frags) {
  tf_pack_elem<H>(P, frags, (long)blockIdx.x * 256 + threadIdx.x);
}

// ---------------------------------------------------------------------------
// unit addressing: token-major row of pair p at window step w
template <int H>
PGP_DEV long tf_row(long p, int w) {
  const long b = p / H;
  return b * 3 * H + (long)w * H + (p - b * H);
}

// N-layout tiles <-> token-major [M][ld] rows (16-byte row groups).  Loads and
// stores are unconditional (no branches, so the compiler's memory-counter waits
// stay exact and a load issued a unit ahead is not waited for together with the
// stores after it): a lane outside the batch reads a row of zeros (the ADDRESS
// is selected, so the loaded value is not touched until its first use: a select
// on the value made the compiler wait for each prefetch right after issuing it)
// and writes the spare row M of the destination (plan: M + 1 rows).
__device__ __attribute__((aligned(16))) float tf_zero_row[64];  // never written (DP <= 64)
PGP_DEV const float* row_ptr(const float* __restrict__ base, long row, int ld, bool ok) {
  return ok ? base + row * ld : tf_zero_row;
}
template <int NTL>
PGP_DEV void load_tiles(f32x4 (&v)[NTL][3], const float* __restrict__ base, int ld, const long (&row)[3], bool ok,
                        int g) {
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float* p = row_ptr(base, row[w], ld, ok);
#pragma unroll
    for (int t = 0; t < NTL; ++t) v[t][w] = ld4(p + 16 * t + 4 * g);
  }
}
template <int NTL>
PGP_DEV void store_tiles(const f32x4 (&v)[NTL][3], float* __restrict__ base, int ld, const long (&row)[3], bool ok,
                         long spare, int g) {
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const long r = ok ? row[w] : spare;
#pragma unroll
    for (int t = 0; t < NTL; ++t) st4(base + r * ld + 16 * t + 4 * g, v[t][w]);
  }
}

// one tile (c: tile c / 3 of step c % 3) of load_tiles, for tf_gemm_side work
template <int NTL>
PGP_DEV void load_tile(f32x4 (&v)[NTL][3], const float* __restrict__ base, int ld, const long (&row)[3], bool ok,
                       int g, int c) {
  v[c / 3][c % 3] = ld4(row_ptr(base, row[c % 3], ld, ok) + 16 * (c / 3) + 4 * g);
}

// acc[o][w] += A . B over KSn k-steps; A = NO tiles of fragment groups in LDS
// (KG groups per tile), B k-step s for step w = bsrc(s, w).  side(i) runs after
// the i-th of the NO * KG fragment groups (its 12 MFMAs): memory instructions
// placed there are spread over the GEMM instead of bursting between phases
// (every CU reaches a phase at about the same time).
template <int NO, int KSn, class BF, class SIDE>
PGP_DEV void tf_gemm_side(f32x4 (&acc)[NO][3], const float* A, BF bsrc, int lane, SIDE side) {
  constexpr int KGn = (KSn + 3) / 4;
  // the A fragment group of the next 12 MFMAs is read one group ahead, so its
  // LDS latency hides under the current group's MFMAs (one wave per SIMD: no
  // other wave covers it), across output tiles too
  f32x4 an = ld4(A + lane * 4);
#pragma unroll
  for (int o = 0; o < NO; ++o) {
#pragma unroll
    for (int q = 0; q < KGn; ++q) {
      const f32x4 a = an;
      if (o * KGn + q + 1 < NO * KGn) an = ld4(A + ((o * KGn + q + 1) * 64 + lane) * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * q + e < KSn) {
#pragma unroll
          for (int w = 0; w < 3; ++w) acc[o][w] = mfma(a[e], bsrc(4 * q + e, w), acc[o][w]);
        }
      side(o * KGn + q);
    }
    // one output tile at a time: keeps the scheduler from hoisting every tile's
    // LDS fragments (register pressure)
    __builtin_amdgcn_sched_barrier(0);
  }
}
template <int NO, int KSn, class BF>
PGP_DEV void tf_gemm(f32x4 (&acc)[NO][3], const float* A, BF bsrc, int lane) {
  tf_gemm_side<NO, KSn>(acc, A, bsrc, lane, [](int) {});
}

// The same product on split-bf16 planes (TF<H>::SPLIT): A = NO tiles x NB
// 32-k blocks x 3 planes of 1-KiB fragments in LDS (tf_split_item), B's k-step
// s of step w = bsrc(s, w), block b = k-steps 8b..8b+7 (zero past KSn) split in
// registers per step; six v_mfma_f32_16x16x32_bf16 per block and tile
// (mfma_bf6: the fp32 product to within 2^-26 of |w x|, fp32 accumulation).
// Step by step, so only one step's split B operand (NB x 12 registers) is live;
// the NO * KGn side slots are spread over the 3 * NO * NB blocks.
template <int NO, int KSn, bool PF = false, class BF, class SIDE>
PGP_DEV void tf_gemm_split_side(f32x4 (&acc)[NO][3], const float* A, BF bsrc, int lane, SIDE side) {
  constexpr int NB = (KSn + 7) / 8, KGn = (KSn + 3) / 4, NS = NO * KGn, NI = 3 * NO * NB;
  auto planes = [&](int o, int b, u32x4 (&wp)[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) wp[k] = *reinterpret_cast<const u32x4*>(A + ((o * NB + b) * 3 + k) * 256 + lane * 4);
  };
  if constexpr (PF) {
    // as below, with the next (tile, block)'s planes read ahead of this one's
    // MFMAs and pinned there (the forward: 2 waves per SIMD, registers to
    // spare); the same MFMAs in the same order
    constexpr int QN = NO * NB;
    u32x4 wn[3];
    planes(0, 0, wn);
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      u32x4 xs[NB][3];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 8 * b + e < KSn ? bsrc(8 * b + e, w) : 0.f;
        split8(v, xs[b]);
      }
#pragma unroll
      for (int o = 0; o < NO; ++o) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          u32x4 wp[3];
#pragma unroll
          for (int k = 0; k < 3; ++k) wp[k] = wn[k];
          const int q = o * NB + b + 1;  // the next (tile, block), wrapping to the next step's first
          if (q < QN)
            planes(q / NB, q % NB, wn);
          else if (w + 1 < 3)
            planes(0, 0, wn);
          __builtin_amdgcn_sched_barrier(0);
          acc[o][w] = mfma_bf6(wp, xs[b], acc[o][w]);
          const int it = (w * NO + o) * NB + b;
#pragma unroll
          for (int i = it * NS / NI; i < (it + 1) * NS / NI; ++i) side(i);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    return;
  }
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    u32x4 xs[NB][3];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 8 * b + e < KSn ? bsrc(8 * b + e, w) : 0.f;
      split8(v, xs[b]);
    }
#pragma unroll
    for (int o = 0; o < NO; ++o) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        u32x4 wp[3];
#pragma unroll
        for (int k = 0; k < 3; ++k)
          wp[k] = *reinterpret_cast<const u32x4*>(A + ((o * NB + b) * 3 + k) * 256 + lane * 4);
        acc[o][w] = mfma_bf6(wp, xs[b], acc[o][w]);
        const int it = (w * NO + o) * NB + b;
#pragma unroll
        for (int i = it * NS / NI; i < (it + 1) * NS / NI; ++i) side(i);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
template <int NO, int KSn, class BF>
PGP_DEV void tf_gemm_split(f32x4 (&acc)[NO][3], const float* A, BF bsrc, int lane) {
  tf_gemm_split_side<NO, KSn>(acc, A, bsrc, lane, [](int) {});
}
// fp32 or split form by TF<H>::SPLIT (A: the matching LDS image)
template <bool SPL, int NO, int KSn, bool PF = false, class BF, class SIDE>
PGP_DEV void tf_gemm_any(f32x4 (&acc)[NO][3], const float* A, BF bsrc, int lane, SIDE side) {
  if constexpr (SPL)
    tf_gemm_split_side<NO, KSn, PF>(acc, A, bsrc, lane, side);
  else
    tf_gemm_side<NO, KSn>(acc, A, bsrc, lane, side);
}

// accumulators initialised with a per-row bias (LDS, natural rows)
template <int NO>
PGP_DEV void init_bias(f32x4 (&acc)[NO][3], const float* bias, int g) {
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    const f32x4 b = ld4(bias + 16 * o + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[o][w] = b;
  }
}

// LayerNorm (eps 1e-5, biased variance) of each step's feature column, in
// place: v becomes x-hat (pads 0); rs[w] = rstd.  Two-pass, masked (as
// pgp_tune.hip's ln_rows).
template <int H, int NTL>
PGP_DEV void tf_ln(f32x4 (&v)[NTL][3], float (&rs)[3], int g) {
  float s[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int t = 0; t < NTL; ++t) s[w] += (v[t][w][0] + v[t][w][1]) + (v[t][w][2] + v[t][w][3]);
  xsum2(s[0], s[1]);
  s[2] = xsum(s[2], true);
  float q[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float mu = s[w] / (float)H;
#pragma unroll
    for (int t = 0; t < NTL; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dv = (16 * t + 4 * g + r < H) ? v[t][w][r] - mu : 0.f;
        v[t][w][r] = dv;
        q[w] = fmaf(dv, dv, q[w]);
      }
  }
  xsum2(q[0], q[1]);
  q[2] = xsum(q[2], true);
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    rs[w] = 1.0f / sqrtf(q[w] / (float)H + 1e-5f);
#pragma unroll
    for (int t = 0; t < NTL; ++t) v[t][w] = v[t][w] * rs[w];
  }
}

// per-unit token sums of an N-layout quantity, compressed: v[t][r] holds this
// lane's (one token column's) partial for row 16t+4g+r; the sum over the 16
// token lanes is added to acc on lane j = 4t + r, so lane (g, j) accumulates row
// 16(j/4) + 4g + (j%4) (DP <= 64).  One register per gradient vector.
template <int NTL>
PGP_DEV void acc_rows(float& acc, const f32x4 (&v)[NTL], int j) {
  // opaque to the optimiser: otherwise it hoists the loop-invariant lane test
  // out of the unit loop and keeps 16 accumulators per vector instead of one
  asm volatile("" : "+v"(j));
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float sm = row16_sum(v[t][r]);
      acc += (j == 4 * t + r) ? sm : 0.f;
    }
}

// LayerNorm backward in place: dy (grad of the output) -> grad of the input,
// from x-hat xh, rstd rs and gamma (LDS); the gamma / beta gradients of the
// unit's tokens are added to the compressed accumulators ag / ab (acc_rows).
template <int H, int NTL>
PGP_DEV void tf_ln_bwd(f32x4 (&dy)[NTL][3], const f32x4 (&xh)[NTL][3], const float (&rs)[3], const float* gam, int g,
                       int j, float& ag, float& ab) {
  float s1[3] = {0.f, 0.f, 0.f}, s2[3] = {0.f, 0.f, 0.f};
  asm volatile("" : "+v"(j));
#pragma unroll
  for (int t = 0; t < NTL; ++t) {
    const f32x4 ga = ld4(gam + 16 * t + 4 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float pg = 0.f, pb = 0.f;
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        pg = fmaf(dy[t][w][r], xh[t][w][r], pg);
        pb += dy[t][w][r];
        const float d = dy[t][w][r] * ga[r];
        dy[t][w][r] = d;
        s1[w] += d;
        s2[w] = fmaf(d, xh[t][w][r], s2[w]);
      }
      // gamma / beta sums of this row over the unit's tokens (acc_rows)
      pg = row16_sum(pg);
      pb = row16_sum(pb);
      ag += (j == 4 * t + r) ? pg : 0.f;
      ab += (j == 4 * t + r) ? pb : 0.f;
    }
  }
  xsum2(s1[0], s1[1]);
  xsum2(s1[2], s2[0]);
  xsum2(s2[1], s2[2]);
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float m1 = s1[w] / (float)H, m2 = s2[w] / (float)H;
#pragma unroll
    for (int t = 0; t < NTL; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        dy[t][w][r] = (16 * t + 4 * g + r < H) ? rs[w] * (dy[t][w][r] - m1 - xh[t][w][r] * m2) : 0.f;
  }
}

// self-attention over the 3 steps (2 heads, scale 1/sqrt(H/2)); QKV tiles
// [q: 0..NT) [k: NT..2NT) [v: 2NT..3NT); P[head][query w][key w2]
template <int H>
PGP_DEV void tf_attn_fwd(const f32x4 (&Q)[3 * TF<H>::NT][3], float (&P)[2][3][3], f32x4 (&O)[TF<H>::NT][3], int g) {
  using F = TF<H>;
  constexpr int NT = F::NT;
  float s[2][3][3];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) s[hh][w][w2] = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 16 * t + 4 * g + r;
      const bool h0 = c < F::HD, h1 = c >= F::HD && c < H;
#pragma unroll
      for (int w = 0; w < 3; ++w)
#pragma unroll
        for (int w2 = 0; w2 < 3; ++w2) {
          const float pr = Q[t][w][r] * Q[NT + t][w2][r];
          s[0][w][w2] += h0 ? pr : 0.f;
          s[1][w][w2] += h1 ? pr : 0.f;
        }
    }
  float* f = &s[0][0][0];
#pragma unroll
  for (int i = 0; i < 18; i += 2) xsum2(f[i], f[i + 1]);
  const float scale = 1.0f / sqrtf((float)F::HD);
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const float a0 = s[hh][w][0] * scale, a1 = s[hh][w][1] * scale, a2 = s[hh][w][2] * scale;
      const float mx = fmaxf(a0, fmaxf(a1, a2));
      const float e0 = expf(a0 - mx), e1 = expf(a1 - mx), e2 = expf(a2 - mx);
      const float inv = 1.0f / (e0 + e1 + e2);
      P[hh][w][0] = e0 * inv;
      P[hh][w][1] = e1 * inv;
      P[hh][w][2] = e2 * inv;
    }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 16 * t + 4 * g + r;
      const int hh = c < F::HD ? 0 : 1;
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        const float p0 = hh ? P[1][w][0] : P[0][w][0], p1 = hh ? P[1][w][1] : P[0][w][1],
                    p2 = hh ? P[1][w][2] : P[0][w][2];
        O[t][w][r] = fmaf(p0, Q[2 * NT + t][0][r], fmaf(p1, Q[2 * NT + t][1][r], p2 * Q[2 * NT + t][2][r]));
      }
    }
}

// per-wave LDS scratch for the weight-gradient contractions: one step's 16
// tokens of an N-layout operand as [token][row] (pitch PITCH floats)
template <int NTL>
struct Scr {
  static constexpr int PITCH = 16 * NTL + 4;
  static constexpr int SIZE = 16 * PITCH;
};
template <int NTL>
PGP_DEV void stage(const f32x4 (&v)[NTL][3], int w, float* s, int g, int j) {
#pragma unroll
  for (int t = 0; t < NTL; ++t) st4(s + j * Scr<NTL>::PITCH + 16 * t + 4 * g, v[t][w]);
}
// the same for a value computed per tile (fn(t) -> f32x4)
template <int NTL, class FN>
PGP_DEV void stage_fn(FN fn, float* s, int g, int j) {
#pragma unroll
  for (int t = 0; t < NTL; ++t) st4(s + j * Scr<NTL>::PITCH + 16 * t + 4 * g, fn(t));
}
// acc[T][U] += sum over the step's 16 tokens of A[16T+4g+r][tok] B[16U+j][tok]
// (k-step e <-> token 4g + e); bsum[T] += the A values read (its token sum)
template <int NA, int NB>
PGP_DEV void dw_step(f32x4 (&acc)[NA][NB], float (&bsum)[NA], const float* sa, const float* sb, int g, int i) {
  float a[NA][4], b[NB][4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
#pragma unroll
    for (int T = 0; T < NA; ++T) a[T][e] = sa[(4 * g + e) * Scr<NA>::PITCH + 16 * T + i];
#pragma unroll
    for (int U = 0; U < NB; ++U) b[U][e] = sb[(4 * g + e) * Scr<NB>::PITCH + 16 * U + i];
  }
#pragma unroll
  for (int T = 0; T < NA; ++T) bsum[T] += (a[T][0] + a[T][1]) + (a[T][2] + a[T][3]);
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int T = 0; T < NA; ++T)
#pragma unroll
      for (int U = 0; U < NB; ++U) acc[T][U] = mfma(a[T][e], b[U][e], acc[T][U]);
}

// rows of unit u's pairs at the 3 window steps; false for a lane past the
// wave's units or the batch
template <int H>
PGP_DEV bool unit_rows(long u, long u1, long npairs, int j, long (&row)[3]) {
  const long p = u * 16 + j;
  const bool ok = u < u1 && p < npairs;
#pragma unroll
  for (int w = 0; w < 3; ++w) row[w] = ok ? tf_row<H>(p, w) : 0;
  return ok;
}

// unit range of one wave (contiguous, balanced over all waves of the grid):
// floor(nu / waves) units each, and the nu % waves extra units in rank order:
// the first wave of every SIMD of every workgroup, then the second wave of
// every SIMD, ... (waves w and w + 4 of a workgroup share SIMD w % 4), so the
// units per SIMD stay balanced whatever the batch (a small batch gets one unit
// per SIMD, not two on half of them); with one wave per SIMD the extras fill
// the first workgroups, which free the others' CUs a unit round early
PGP_DEV void unit_range(long nu, long& u0, long& u1, int waves = kTfWaves) {
  const long nw = (long)gridDim.x * waves;
  const int w = threadIdx.x >> 6;
  const long rank = (long)(w / 4) * gridDim.x * 4 + (long)blockIdx.x * 4 + (w % 4);
  const long q = nu / nw, r = nu - q * nw;
  u0 = rank * q + (rank < r ? rank : r);
  u1 = u0 + q + (rank < r ? 1 : 0);
}

// LDS parameter block of a layer (natural rows, zero-padded)
template <int H>
struct TfPar {
  using F = TF<H>;
  static constexpr int BIN = 0;                       // [NQ*16] in_proj bias in q|k|v tiles
  static constexpr int BO = BIN + F::NQ * 16;         // [DP]
  static constexpr int N1W = BO + F::DP, N1B = N1W + F::DP;
  static constexpr int B1 = N1B + F::DP;              // [64]
  static constexpr int B2 = B1 + 64;                  // [DP]
  static constexpr int N2W = B2 + F::DP, N2B = N2W + F::DP;
  static constexpr int BTE = N2B + F::DP;             // [3][DP] time-encoder bias + pe[w]
  static constexpr int SIZE = BTE + 3 * F::DP;
};
template <int H>
PGP_DEV void load_params(float* sp, const float* __restrict__ P, int layer) {
  using F = TF<H>;
  using G = TGeo<H>;
  using Q = TfPar<H>;
  const float* L = P + G::LAY0 + (long)layer * G::L_SIZE;
  for (int k = threadIdx.x; k < Q::SIZE; k += blockDim.x) {
    float v = 0.f;
    if (k < Q::BO) {
      const int part = k / F::DP, n = k - part * F::DP;
      v = n < H ? L[G::L_INB + part * H + n] : 0.f;
    } else if (k < Q::BTE) {
      const int sec = k < Q::N1W ? 0 : k < Q::N1B ? 1 : k < Q::B1 ? 2 : k < Q::B2 ? 3 : k < Q::N2W ? 4 : k < Q::N2B ? 5 : 6;
      const int base[7] = {Q::BO, Q::N1W, Q::N1B, Q::B1, Q::B2, Q::N2W, Q::N2B};
      const long src[7] = {G::L_OUTB, G::L_N1W, G::L_N1B, G::L_B1, G::L_B2, G::L_N2W, G::L_N2B};
      const int n = k - base[sec];
      const int lim = sec == 3 ? 64 : H;
      v = n < lim ? L[src[sec] + n] : 0.f;
    } else {
      const int w = (k - Q::BTE) / F::DP, n = (k - Q::BTE) - w * F::DP;
      v = n < H ? P[G::B_TE + n] + P[G::PE + w * H + n] : 0.f;
    }
    sp[k] = v;
  }
}

// ============================================================================
// forward of one layer (layer 0 includes the time encoder + PE)
// ============================================================================
template <int H>
struct FwdL {
  using F = TF<H>;
  // F1 / F2 as fp32 fragments or (SPLIT) split planes (the first P_F1 + P_F2
  // fragments of the layer's plane block)
  static constexpr int N_F1 = F::SPLIT ? F::P_F1 : F::G_F1, N_F2 = F::SPLIT ? F::P_F2 : F::G_F2;
  static constexpr int W_TE = 0, W_IN = W_TE + F::G_TE * 256, W_O = W_IN + F::G_IN * 256,
                       W_F1 = W_O + F::G_O * 256, W_F2 = W_F1 + N_F1 * 256, PAR = W_F2 + N_F2 * 256,
                       TOTAL = PAR + TfPar<H>::SIZE;
};

// attention scores of both heads from the q | k tiles -> probabilities
// P[head][query w][key w2] (softmax over the 3 keys, lane-local)
template <int H>
PGP_DEV void tf_attn_probs(const f32x4 (&QK)[2 * TF<H>::NT][3], float (&P)[2][3][3], int g) {
  using F = TF<H>;
  constexpr int NT = F::NT;
  float s[2][3][3];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) s[hh][w][w2] = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 16 * t + 4 * g + r;
      const bool h0 = c < F::HD, h1 = c >= F::HD && c < H;
#pragma unroll
      for (int w = 0; w < 3; ++w)
#pragma unroll
        for (int w2 = 0; w2 < 3; ++w2) {
          const float pr = QK[t][w][r] * QK[NT + t][w2][r];
          s[0][w][w2] += h0 ? pr : 0.f;
          s[1][w][w2] += h1 ? pr : 0.f;
        }
    }
  float* f = &s[0][0][0];
#pragma unroll
  for (int i = 0; i < 18; i += 2) xsum2(f[i], f[i + 1]);
  const float scale = 1.0f / sqrtf((float)F::HD);
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const float a0 = s[hh][w][0] * scale, a1 = s[hh][w][1] * scale, a2 = s[hh][w][2] * scale;
      const float mx = fmaxf(a0, fmaxf(a1, a2));
      const float e0 = expf(a0 - mx), e1 = expf(a1 - mx), e2 = expf(a2 - mx);
      const float inv = 1.0f / (e0 + e1 + e2);
      P[hh][w][0] = e0 * inv;
      P[hh][w][1] = e1 * inv;
      P[hh][w][2] = e2 * inv;
    }
}

// the forward runs TWO waves per SIMD (8 per workgroup, <= 256 registers per
// wave): each wave's latencies (LDS fragments, the softmax / LayerNorm chains,
// prefetch waits) are covered by the other wave's MFMAs.  q | k and v are
// separate GEMMs (96 + 48 accumulator registers instead of 144 at once).
constexpr int kTfFwdWaves = 8;
// the forward's split GEMMs read each (tile, block)'s planes one ahead (A/B, C3
// H = 50, 4 interleaved rounds: 1.0255 -> 1.0134 ms, profiles/r06/c3/ab_fwd_pf.txt;
// 28 registers spill at the forward's 256, yet it is faster)
#ifndef PGP_TF_FWD_PF
#define PGP_TF_FWD_PF 1
#endif
constexpr bool kTfFwdPF = PGP_TF_FWD_PF != 0;
// the FFN backward's split GEMMs likewise (A/B, C3 H = 50, 5 interleaved rounds:
// 1.0114 -> 1.0019 ms, no spills; profiles/r06/c3/ab_bff_pf.txt)
#ifndef PGP_TF_BFF_PF
#define PGP_TF_BFF_PF 1
#endif
constexpr bool kTfBffPF = PGP_TF_BFF_PF != 0;

template <int H>
__global__ __launch_bounds__(kTfFwdWaves * 64, 1) void tf_fwd_kernel(TfArgs a) {
  using F = TF<H>;
  using L = FwdL<H>;
  using Q = TfPar<H>;
  constexpr int NT = F::NT;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int layer = a.layer;
  const float* fr = a.frags + F::layer_off(layer);
  if (layer == 0) dma_groups(a.frags + F::TE_OFF, sm + L::W_TE, F::G_TE, wv, kTfFwdWaves, lane);
  if constexpr (F::SPLIT) {
    dma_groups(fr + F::OFF_IN, sm + L::W_IN, F::G_IN + F::G_O, wv, kTfFwdWaves, lane);
    dma_groups(a.frags + F::pl_off(layer), sm + L::W_F1, F::P_F1 + F::P_F2, wv, kTfFwdWaves, lane);
  } else {
    dma_groups(fr + F::OFF_IN, sm + L::W_IN, F::G_IN + F::G_O + F::G_F1 + F::G_F2, wv, kTfFwdWaves, lane);
  }
  load_params<H>(sm + L::PAR, a.P, layer);
  TF_ST_INIT();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  TF_ST(0);
  const float* par = sm + L::PAR;
  const long npairs = (long)a.B * H, nu = (npairs + 15) / 16, spare = 3 * npairs;
  long u0, u1;
  unit_range(nu, u0, u1, kTfFwdWaves);
  // the unit's input (layer 0: the GAT output) is loaded one unit ahead during
  // the previous unit's linear2; x0 is stored during q|k, norm1's x-hat / rstd
  // during linear1, the layer output at the end of the unit
  f32x4 Xn[NT][3];
  {
    long rn[3];
    const bool okn = unit_rows<H>(u0, u1, npairs, j, rn);
    load_tiles<NT>(Xn, a.in, F::DP, rn, okn, g);
  }
  auto tile_at = [&](float* base, long r) { return base + r * F::DP + 4 * g; };
#pragma unroll 1
  for (long u = u0; u < u1; ++u) {
    long row[3];
    const bool ok = unit_rows<H>(u, u1, npairs, j, row);
    long srow[3];
#pragma unroll
    for (int w = 0; w < 3; ++w) srow[w] = ok ? row[w] : spare;
    f32x4 X[NT][3];
    if (layer == 0) {  // X0 = Wte g + bte + pe[w]  (models.py:390-393)
      TF_ST(1);
#pragma unroll
      for (int o = 0; o < NT; ++o)
#pragma unroll
        for (int w = 0; w < 3; ++w) X[o][w] = ld4(par + Q::BTE + w * F::DP + 16 * o + 4 * g);
      tf_gemm<NT, F::KS>(X, sm + L::W_TE, [&](int s, int w) { return Xn[s >> 2][w][s & 3]; }, lane);
      TF_ST(2);
    } else {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int w = 0; w < 3; ++w) X[t][w] = Xn[t][w];
      TF_ST(1);
    }
    float Pr[2][3][3];
    {  // q | k (side work: layer 0's x0) -> the attention probabilities
      f32x4 QK[2 * NT][3];
      init_bias<2 * NT>(QK, par + Q::BIN, g);
      constexpr int NS = 3 * NT, NG = 2 * NT * F::KG, PER = (NS + NG - 1) / NG;
      tf_gemm_side<2 * NT, F::KS>(QK, sm + L::W_IN, [&](int s, int w) { return X[s >> 2][w][s & 3]; }, lane,
                                  [&](int i) {
#pragma unroll
                                    for (int k = 0; k < PER; ++k) {
                                      const int c = i * PER + k;
                                      if (c < NS && layer == 0)
                                        st4(tile_at(a.x0, srow[c % 3]) + 16 * (c / 3), X[c / 3][c % 3]);
                                    }
                                  });
      TF_ST(3);
      tf_attn_probs<H>(QK, Pr, g);
    }
    f32x4 O[NT][3];
    {  // v, then O = P . v per head
      f32x4 V[NT][3];
      init_bias<NT>(V, par + Q::BIN + 2 * NT * 16, g);
      tf_gemm<NT, F::KS>(V, sm + L::W_IN + 2 * NT * F::KG * 256, [&](int s, int w) { return X[s >> 2][w][s & 3]; },
                         lane);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int hh = (16 * t + 4 * g + r) < F::HD ? 0 : 1;
#pragma unroll
          for (int w = 0; w < 3; ++w) {
            const float p0 = hh ? Pr[1][w][0] : Pr[0][w][0], p1 = hh ? Pr[1][w][1] : Pr[0][w][1],
                        p2 = hh ? Pr[1][w][2] : Pr[0][w][2];
            O[t][w][r] = fmaf(p0, V[t][0][r], fmaf(p1, V[t][1][r], p2 * V[t][2][r]));
          }
        }
    }
    TF_ST(4);
    f32x4 R[NT][3];
    init_bias<NT>(R, par + Q::BO, g);
    tf_gemm<NT, F::KS>(R, sm + L::W_O, [&](int s, int w) { return O[s >> 2][w][s & 3]; }, lane);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int w = 0; w < 3; ++w) R[t][w] += X[t][w];
    TF_ST(5);
    float rs[3];
    tf_ln<H, NT>(R, rs, g);  // R = x-hat of norm1
    TF_ST(6);
    // y1 = gamma1 x-hat + beta1 (in place of X: the residual of the FFN)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 ga = ld4(par + Q::N1W + 16 * t + 4 * g), be = ld4(par + Q::N1B + 16 * t + 4 * g);
#pragma unroll
      for (int w = 0; w < 3; ++w) X[t][w] = R[t][w] * ga + be;
    }
    f32x4 Fh[4][3];
    init_bias<4>(Fh, par + Q::B1, g);
    {  // side work: norm1's x-hat tiles and rstd (every lane group: the same value)
      constexpr int NS = 3 * NT + 3, NG = 4 * F::KG, PER = (NS + NG - 1) / NG;
      tf_gemm_any<F::SPLIT, 4, F::KS, kTfFwdPF>(Fh, sm + L::W_F1, [&](int s, int w) { return X[s >> 2][w][s & 3]; }, lane,
                             [&](int i) {
#pragma unroll
                               for (int k = 0; k < PER; ++k) {
                                 const int c = i * PER + k;
                                 if (c < 3 * NT)
                                   st4(tile_at(a.xh1, srow[c % 3]) + 16 * (c / 3), R[c / 3][c % 3]);
                                 else if (c < NS)
                                   a.rs1[srow[c - 3 * NT]] = rs[c - 3 * NT];
                               }
                             });
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int w = 0; w < 3; ++w)
#pragma unroll
        for (int r = 0; r < 4; ++r) Fh[t][w][r] = fmaxf(Fh[t][w][r], 0.f);
    TF_ST(7);
    init_bias<NT>(R, par + Q::B2, g);
    {  // side work: the next unit's input
      long rn[3];
      const bool okn = unit_rows<H>(u + 1, u1, npairs, j, rn);
      constexpr int NS = 3 * NT, NG = NT * F::KGF, PER = (NS + NG - 1) / NG;
      tf_gemm_any<F::SPLIT, NT, 16, kTfFwdPF>(R, sm + L::W_F2, [&](int s, int w) { return Fh[s >> 2][w][s & 3]; }, lane,
                           [&](int i) {
#pragma unroll
                             for (int k = 0; k < PER; ++k) {
                               const int c = i * PER + k;
                               if (c < NS)
                                 Xn[c / 3][c % 3] = ld4(row_ptr(a.in, rn[c % 3], F::DP, okn) + 16 * (c / 3) + 4 * g);
                             }
                           });
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int w = 0; w < 3; ++w) R[t][w] += X[t][w];
    TF_ST(8);
    tf_ln<H, NT>(R, rs, g);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const f32x4 ga = ld4(par + Q::N2W + 16 * t + 4 * g), be = ld4(par + Q::N2B + 16 * t + 4 * g);
#pragma unroll
      for (int w = 0; w < 3; ++w) R[t][w] = R[t][w] * ga + be;
    }
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(tile_at(a.out, srow[w]) + 16 * t, R[t][w]);
    TF_ST(9);
  }
  TF_ST(10);
  TF_ST_END(layer);
}

// ============================================================================
// end-of-kernel combination: each wave stores its register partials into a
// region of its own (plain stores, all waves at once), then the workgroup sums
// the regions in wave order (deterministic) straight into its global slab
// ============================================================================
// compressed row accumulator (acc_rows) -> dst[row] for rows < lim
PGP_DEV void put_rows_c(float* dst, float acc, int lim, int g, int j) {
  const int n = 16 * (j >> 2) + 4 * g + (j & 3);
  if (n < lim) dst[n] = acc;
}
// bias sums bsum[T] (per lane: row 16T + i, this lane group's tokens) -> dst
template <int NA>
PGP_DEV void put_bias(float* dst, const float (&b)[NA], int lim, int g, int i) {
#pragma unroll
  for (int T = 0; T < NA; ++T) {
    const float s = xsum(b[T], true);
    const int n = 16 * T + i;
    if (g == 0 && n < lim) dst[n] = s;
  }
}
// dW tile sums acc[T][U] (row 16T+4g+r, column 16U+j) -> dst[row * ld + col]
template <int NA, int NB>
PGP_DEV void put_dw(float* dst, const f32x4 (&acc)[NA][NB], int rows, int cols, int ld, int g, int j) {
#pragma unroll
  for (int T = 0; T < NA; ++T)
#pragma unroll
    for (int U = 0; U < NB; ++U)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * T + 4 * g + r, c = 16 * U + j;
        if (n < rows && c < cols) dst[n * ld + c] = acc[T][U][r];
      }
}
// dst[k] = sum over the kTfWaves regions (pitch `pitch`) in wave order, k < n
PGP_DEV void sum_regions(float* __restrict__ dst, const float* src, int pitch, int n) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    float v = src[k];
#pragma unroll
    for (int w = 1; w < kTfWaves; ++w) v += src[w * pitch + k];
    dst[k] = v;
  }
}

// ============================================================================
// backward of a layer's feed-forward block (models.py:356: norm2(y1 + FFN(y1)),
// y1 = norm1(.)): dOut -> dR1 (grad of norm1's input)
// ============================================================================
template <int H>
struct BffL {
  using F = TF<H>;
  // the four matrices as fp32 fragments or (SPLIT) split planes, in the
  // fragment buffer's order (one DMA)
  static constexpr int N_F1 = F::SPLIT ? F::P_F1 : F::G_F1, N_F2 = F::SPLIT ? F::P_F2 : F::G_F2,
                       N_F2T = F::SPLIT ? F::P_F2T : F::G_F2T, N_F1T = F::SPLIT ? F::P_F1T : F::G_F1T;
  static constexpr int W_F1 = 0, W_F2 = W_F1 + N_F1 * 256, W_F2T = W_F2 + N_F2 * 256,
                       W_F1T = W_F2T + N_F2T * 256, PAR = W_F1T + N_F1T * 256,
                       SCR = PAR + TfPar<H>::SIZE,
                       SCR_A = Scr<4>::SIZE, SCR_B = Scr<4>::SIZE,  // both operands <= 64 rows
                       TOTAL = SCR + kTfWaves * (SCR_A + SCR_B),
                       NTW = F::NT * 4;                           // dW2 [NT][4] (and dW1 [4][NT]) tiles of 256 floats
  static constexpr int S_W2 = 0, S_B2 = S_W2 + H * 64, S_W1 = S_B2 + H, S_B1 = S_W1 + 64 * H,
                       S_G1 = S_B1 + 64, S_BT1 = S_G1 + H, S_G2 = S_BT1 + H, S_BT2 = S_G2 + H,
                       SLAB = S_BT2 + H;
  static constexpr int NV = 5 * H + 64;  // per-wave vector partials in the epilogue
};

// The waves' register tiles d[T][U] summed in wave order into dst (row
// 16T+4g+r, column 16U+j per lane; rows < rows, cols < cols, pitch ld): each
// wave stores its tiles to a region of its own, then wave k sums tiles k, k + W, ...
// over the regions and writes them.  Ends with a barrier (the LDS is reusable).
template <int NA, int NB>
PGP_DEV void sum_tiles(float* dst, const f32x4 (&d)[NA][NB], float* lds, int rows, int cols, int ld, int wv, int g,
                       int j, int lane) {
  constexpr int NTL = NA * NB;
#pragma unroll
  for (int T = 0; T < NA; ++T)
#pragma unroll
    for (int U = 0; U < NB; ++U) st4(lds + ((wv * NTL + T * NB + U) * 64 + lane) * 4, d[T][U]);
  __syncthreads();
  for (int k = wv; k < NTL; k += kTfWaves) {
    f32x4 v = ld4(lds + (k * 64 + lane) * 4);
#pragma unroll
    for (int w = 1; w < kTfWaves; ++w) v += ld4(lds + ((w * NTL + k) * 64 + lane) * 4);
    const int T = k / NB, U = k - T * NB;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * T + 4 * g + r, c = 16 * U + j;
      if (n < rows && c < cols) dst[n * ld + c] = v[r];
    }
  }
  __syncthreads();
}

template <int H>
__global__ __launch_bounds__(kTfWaves * 64, 1) void tf_bwd_ffn_kernel(TfArgs a) {
  using F = TF<H>;
  using L = BffL<H>;
  using Q = TfPar<H>;
  constexpr int NT = F::NT;
  static_assert(kTfWaves * L::NV <= L::SCR, "epilogue partials fit the LDS they reuse");
  static_assert(kTfWaves * L::NTW * 256 <= L::TOTAL, "epilogue dW regions fit the LDS they reuse");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int layer = a.layer;
  if constexpr (F::SPLIT)
    dma_groups(a.frags + F::pl_off(layer), sm + L::W_F1, F::PO_OT, wv, kTfWaves, lane);
  else
    dma_groups(a.frags + F::layer_off(layer) + F::OFF_F1, sm + L::W_F1, F::G_F1 + F::G_F2 + F::G_F2T + F::G_F1T,
               wv, kTfWaves, lane);
  load_params<H>(sm + L::PAR, a.P, layer);
  TF_ST_INIT();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  TF_ST(0);
  float* sa = sm + L::SCR + wv * (L::SCR_A + L::SCR_B);
  float* sb = sa + L::SCR_A;
  // dW2 / dW1 accumulate in registers over all of the wave's units (no
  // per-unit LDS accumulation: the waves run their units without barriers);
  // the waves' sums are combined in wave order at the end
  f32x4 dW2[NT][4], dW1[4][NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int U = 0; U < 4; ++U) dW2[t][U] = dW1[U][t] = zero4();
  float b2s[NT], b1s[4];
  float ag1 = 0.f, ab1 = 0.f, ag2 = 0.f, ab2 = 0.f;  // LayerNorm gamma / beta sums (compressed rows)
#pragma unroll
  for (int t = 0; t < NT; ++t) b2s[t] = 0.f;
#pragma unroll
  for (int U = 0; U < 4; ++U) b1s[U] = 0.f;
  const long npairs = (long)a.B * H, nu = (npairs + 15) / 16, spare = 3 * npairs;
  long u0, u1;
  unit_range(nu, u0, u1);
#pragma unroll 1
  for (long u = u0; u < u1; ++u) {
    // loop-variant view of the LDS base: keeps LICM from hoisting the
    // loop-invariant parameter / weight reads out of the unit loop (hundreds of
    // registers held across it)
    int z = 0;
    asm volatile("" : "+s"(z));
    float* smz = sm + z;
    const float* par = smz + L::PAR;
    // y1 = gamma1 x-hat1 + beta1, tile t of step w
    auto y1 = [&](const f32x4 (&xh)[NT][3], int t, int w) {
      return xh[t][w] * ld4(par + Q::N1W + 16 * t + 4 * g) + ld4(par + Q::N1B + 16 * t + 4 * g);
    };
    long row[3];
    const bool ok = unit_rows<H>(u, u1, npairs, j, row);
    f32x4 dY[NT][3], Fh[4][3];
    float rs1[3], rs2[3];
    {  // recompute the FFN (pre-activation F) and norm2's x-hat
      f32x4 X2[NT][3];
      {
        // LN1's x-hat and rstd of the unit (not prefetched a unit ahead: with
        // the dW accumulators in registers that prefetch spilled)
        f32x4 Y1[NT][3];
        load_tiles<NT>(Y1, a.xh1, F::DP, row, ok, g);
#pragma unroll
        for (int w = 0; w < 3; ++w) {
          const float r = a.rs1[row[w]];
          rs1[w] = ok ? r : 0.f;
        }
        TF_ST(1);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int w = 0; w < 3; ++w) Y1[t][w] = y1(Y1, t, w);
        init_bias<4>(Fh, par + Q::B1, g);
        tf_gemm_any<F::SPLIT, 4, F::KS, kTfBffPF>(Fh, smz + L::W_F1, [&](int s, int w) { return Y1[s >> 2][w][s & 3]; }, lane,
                                        [](int) {});
        init_bias<NT>(X2, par + Q::B2, g);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int w = 0; w < 3; ++w) X2[t][w] += Y1[t][w];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)  // keep relu(F): its sign is F's for the mask (F = 0 -> 0 either way)
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
          for (int r = 0; r < 4; ++r) Fh[t][w][r] = fmaxf(Fh[t][w][r], 0.f);
      TF_ST(2);
      {  // side work: dOut of the unit
        constexpr int NS = 3 * NT, NG = NT * F::KGF, PER = (NS + NG - 1) / NG;
        tf_gemm_any<F::SPLIT, NT, 16, kTfBffPF>(X2, smz + L::W_F2, [&](int s, int w) { return Fh[s >> 2][w][s & 3]; }, lane,
                                      [&](int i) {
#pragma unroll
                                        for (int k = 0; k < PER; ++k)
                                          if (i * PER + k < NS) load_tile<NT>(dY, a.in, F::DP, row, ok, g, i * PER + k);
                                      });
      }
      __builtin_amdgcn_sched_barrier(0);
      TF_ST(3);
      tf_ln<H, NT>(X2, rs2, g);
      tf_ln_bwd<H, NT>(dY, X2, rs2, par + Q::N2W, g, j, ag2, ab2);  // dY <- dR2
    }
    TF_ST(4);
    __builtin_amdgcn_sched_barrier(0);
    {  // dW2 += dR2 (x) relu(F), db2 += sum dR2
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        stage<NT>(dY, w, sa, g, j);
        stage<4>(Fh, w, sb, g, j);
        dw_step<NT, 4>(dW2, b2s, sa, sb, g, j);
      }
      TF_ST(5);
      TF_ST(6);
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 XH1[NT][3];
    // dF = (W2^T dR2) * (F > 0)
    {
      f32x4 dF[4][3];
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int w = 0; w < 3; ++w) dF[t][w] = zero4();
      {  // side work: norm1's x-hat, reloaded (L2): not held through the phases above
        constexpr int NS = 3 * NT, NG = 4 * F::KG, PER = (NS + NG - 1) / NG;
        tf_gemm_any<F::SPLIT, 4, F::KS, kTfBffPF>(dF, smz + L::W_F2T, [&](int s, int w) { return dY[s >> 2][w][s & 3]; }, lane,
                                        [&](int i) {
#pragma unroll
                                          for (int k = 0; k < PER; ++k)
                                            if (i * PER + k < NS)
                                              load_tile<NT>(XH1, a.xh1, F::DP, row, ok, g, i * PER + k);
                                        });
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
          for (int r = 0; r < 4; ++r) dF[t][w][r] = Fh[t][w][r] > 0.f ? dF[t][w][r] : 0.f;
      __builtin_amdgcn_sched_barrier(0);
      TF_ST(7);
      {  // dW1 += dF (x) y1, db1 += sum dF
#pragma unroll
        for (int w = 0; w < 3; ++w) {
          stage<4>(dF, w, sa, g, j);
          stage_fn<NT>([&](int t) { return y1(XH1, t, w); }, sb, g, j);
          dw_step<4, NT>(dW1, b1s, sa, sb, g, j);
        }
        TF_ST(8);
        TF_ST(9);
      }
      __builtin_amdgcn_sched_barrier(0);
      // dy1 = W1^T dF + dR2 (residual)
      tf_gemm_any<F::SPLIT, NT, 16, kTfBffPF>(dY, smz + L::W_F1T, [&](int s, int w) { return dF[s >> 2][w][s & 3]; }, lane,
                                    [](int) {});
    }
    __builtin_amdgcn_sched_barrier(0);
    TF_ST(10);
    tf_ln_bwd<H, NT>(dY, XH1, rs1, par + Q::N1W, g, j, ag1, ab1);  // -> dR1
    store_tiles<NT>(dY, a.out, F::DP, row, ok, spare, g);
    TF_ST(11);
  }
  TF_ST(12);
  // one slab per workgroup: the waves' dW tiles summed in wave order (two
  // passes through the LDS the weights held), then their vector partials
  float* slab = a.part + (long)blockIdx.x * L::SLAB;
  __syncthreads();   // every wave is past its units: the weight area is free
  sum_tiles<NT, 4>(slab + L::S_W2, dW2, sm, H, 64, 64, wv, g, j, lane);
  sum_tiles<4, NT>(slab + L::S_W1, dW1, sm, 64, H, H, wv, g, j, lane);
  float* vr = sm + wv * L::NV;  // this wave's vector partials: b2 | b1 | g1 | bt1 | g2 | bt2
  put_bias<NT>(vr, b2s, H, g, j);
  put_bias<4>(vr + H, b1s, 64, g, j);
  put_rows_c(vr + H + 64, ag1, H, g, j);
  put_rows_c(vr + 2 * H + 64, ab1, H, g, j);
  put_rows_c(vr + 3 * H + 64, ag2, H, g, j);
  put_rows_c(vr + 4 * H + 64, ab2, H, g, j);
  __syncthreads();
  sum_regions(slab + L::S_B2, sm, L::NV, H);
  sum_regions(slab + L::S_B1, sm + H, L::NV, 64);
  sum_regions(slab + L::S_G1, sm + H + 64, L::NV, 4 * H);  // g1 bt1 g2 bt2 are contiguous in the slab too
  TF_ST(13);
  TF_ST_END(2);
}

// ============================================================================
// backward of a layer's attention block (models.py:356: norm1(x + SA(x))):
// dR1 (grad of norm1's input) -> dX (grad of the layer input) and dQKV
// ============================================================================
template <int H>
struct BatL {
  using F = TF<H>;
  static constexpr int N_OT = F::SPLIT ? F::P_OT : F::G_OT;  // Wo^T as fp32 fragments or split planes
  static constexpr int W_IN = 0, W_INT = W_IN + F::G_IN * 256, W_OT = W_INT + F::G_INT * 256,
                       PAR = W_OT + N_OT * 256, SCR = PAR + TfPar<H>::SIZE,
                       SCR_A = Scr<F::NT>::SIZE, SCR_B = Scr<F::NT>::SIZE,
                       TOTAL = SCR + kTfWaves * (SCR_A + SCR_B);
  static constexpr int S_WO = 0, S_BO = H * H, SLAB = S_BO + H;
};

template <int H>
__global__ __launch_bounds__(kTfWaves * 64, 1) void tf_bwd_att_kernel(TfArgs a) {
  using F = TF<H>;
  using L = BatL<H>;
  using Q = TfPar<H>;
  constexpr int NT = F::NT;
  static_assert(kTfWaves * L::SLAB <= L::SCR, "epilogue partials fit the LDS they reuse");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int layer = a.layer;
  const float* fr = a.frags + F::layer_off(layer);
  dma_groups(fr + F::OFF_IN, sm + L::W_IN, F::G_IN, wv, kTfWaves, lane);
  if constexpr (F::SPLIT) {
    dma_groups(fr + F::OFF_INT, sm + L::W_INT, F::G_INT, wv, kTfWaves, lane);
    dma_groups(a.frags + F::pl_off(layer) + F::PO_OT * 256L, sm + L::W_OT, F::P_OT, wv, kTfWaves, lane);
  } else {
    dma_groups(fr + F::OFF_INT, sm + L::W_INT, F::G_INT + F::G_OT, wv, kTfWaves, lane);
  }
  load_params<H>(sm + L::PAR, a.P, layer);
  TF_ST_INIT();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  TF_ST(0);
  const float* par = sm + L::PAR;
  float* sa = sm + L::SCR + wv * (L::SCR_A + L::SCR_B);
  float* sb = sa + L::SCR_A;
  f32x4 dWo[NT][NT];
  float bos[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bos[t] = 0.f;
#pragma unroll
    for (int U = 0; U < NT; ++U) dWo[t][U] = zero4();
  }
  const float scale = 1.0f / sqrtf((float)F::HD);
  const long npairs = (long)a.B * H, nu = (npairs + 15) / 16, spare = 3 * npairs;
  long u0, u1;
  unit_range(nu, u0, u1);
  // the layer input X is loaded one unit ahead (see tf_fwd_kernel), dR1 after
  // the q|k|v GEMM (its latency under the attention)
  f32x4 Xn[NT][3];
  {
    long rn[3];
    const bool okn = unit_rows<H>(u0, u1, npairs, j, rn);
    load_tiles<NT>(Xn, a.x, F::DP, rn, okn, g);
  }
#pragma unroll 1
  for (long u = u0; u < u1; ++u) {
    long row[3];
    const bool ok = unit_rows<H>(u, u1, npairs, j, row);
    f32x4 QKV[F::NQ][3];
    f32x4 O[NT][3], dR1[NT][3];
    TF_ST(1);
    init_bias<F::NQ>(QKV, par + Q::BIN, g);
    tf_gemm<F::NQ, F::KS>(QKV, sm + L::W_IN, [&](int s, int w) { return Xn[s >> 2][w][s & 3]; }, lane);
    TF_ST(2);
    float Pr[2][3][3];
    tf_attn_fwd<H>(QKV, Pr, O, g);
    TF_ST(3);
    load_tiles<NT>(dR1, a.in, F::DP, row, ok, g);
    TF_ST(4);
    // dWo += dR1 (x) attention output, dbo += sum dR1
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      stage<NT>(dR1, w, sa, g, j);
      stage<NT>(O, w, sb, g, j);
      dw_step<NT, NT>(dWo, bos, sa, sb, g, j);
    }
    TF_ST(5);
    // dO = Wo^T dR1
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int w = 0; w < 3; ++w) O[t][w] = zero4();
    tf_gemm_any<F::SPLIT, NT, F::KS>(O, sm + L::W_OT, [&](int s, int w) { return dR1[s >> 2][w][s & 3]; }, lane,
                                     [](int) {});
    TF_ST(6);
    // attention backward (pgp_tune.hip attn_bwd_kernel, per lane)
    float dS[2][3][3];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int w = 0; w < 3; ++w)
#pragma unroll
        for (int w2 = 0; w2 < 3; ++w2) dS[hh][w][w2] = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * t + 4 * g + r;
        const bool h0 = c < F::HD, h1 = c >= F::HD && c < H;
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
          for (int w2 = 0; w2 < 3; ++w2) {
            const float pr = O[t][w][r] * QKV[2 * NT + t][w2][r];  // dO[w] . v[w2]
            dS[0][w][w2] += h0 ? pr : 0.f;
            dS[1][w][w2] += h1 ? pr : 0.f;
          }
      }
    {
      float* f = &dS[0][0][0];
#pragma unroll
      for (int i = 0; i < 18; i += 2) xsum2(f[i], f[i + 1]);
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        const float sd = Pr[hh][w][0] * dS[hh][w][0] + Pr[hh][w][1] * dS[hh][w][1] + Pr[hh][w][2] * dS[hh][w][2];
#pragma unroll
        for (int w2 = 0; w2 < 3; ++w2) dS[hh][w][w2] = Pr[hh][w][w2] * (dS[hh][w][w2] - sd) * scale;
      }
    // dv (in place of v), dq (temporary), dk (in place of k), then q <- dq
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hh = (16 * t + 4 * g + r) < F::HD ? 0 : 1;
        float dq[3], dk[3], dv[3];
#pragma unroll
        for (int w = 0; w < 3; ++w) {
          const float d0 = hh ? dS[1][w][0] : dS[0][w][0], d1 = hh ? dS[1][w][1] : dS[0][w][1],
                      d2 = hh ? dS[1][w][2] : dS[0][w][2];
          dq[w] = d0 * QKV[NT + t][0][r] + d1 * QKV[NT + t][1][r] + d2 * QKV[NT + t][2][r];
          const float e0 = hh ? dS[1][0][w] : dS[0][0][w], e1 = hh ? dS[1][1][w] : dS[0][1][w],
                      e2 = hh ? dS[1][2][w] : dS[0][2][w];
          dk[w] = e0 * QKV[t][0][r] + e1 * QKV[t][1][r] + e2 * QKV[t][2][r];
          const float p0 = hh ? Pr[1][0][w] : Pr[0][0][w], p1 = hh ? Pr[1][1][w] : Pr[0][1][w],
                      p2 = hh ? Pr[1][2][w] : Pr[0][2][w];
          dv[w] = p0 * O[t][0][r] + p1 * O[t][1][r] + p2 * O[t][2][r];
        }
#pragma unroll
        for (int w = 0; w < 3; ++w) {
          QKV[t][w][r] = dq[w];
          QKV[NT + t][w][r] = dk[w];
          QKV[2 * NT + t][w][r] = dv[w];
        }
      }
    TF_ST(7);
    TF_ST(8);
    // dX = Win^T dQKV + dR1 (the residual); the dQKV rows go to HBM ([M + 1][3][DP]:
    // q | k | v, each zero-padded) for in_proj's weight gradient, one tile per
    // fragment group
    // and the next unit's input X is loaded
    long rn[3];
    const bool okn = unit_rows<H>(u + 1, u1, npairs, j, rn);
    constexpr int NS = 3 * F::NQ, NL = 3 * NT, NG = F::NT * F::KGQ, PER = (NS + NL + NG - 1) / NG;
    long srow[3];
#pragma unroll
    for (int w = 0; w < 3; ++w) srow[w] = (ok ? row[w] : spare) * (3 * F::DP) + 4 * g;
    tf_gemm_side<NT, F::KSQ>(dR1, sm + L::W_INT, [&](int s, int w) {
      const int part = s / F::KS, sl = s - part * F::KS;
      return QKV[part * NT + (sl >> 2)][w][sl & 3];
    }, lane, [&](int i) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int c = i * PER + k;
        if (c < NS)
          st4(a.dqkv + srow[c % 3] + 16 * (c / 3), QKV[c / 3][c % 3]);
        else if (c < NS + NL)
          load_tile<NT>(Xn, a.x, F::DP, rn, okn, g, c - NS);
      }
    });
    store_tiles<NT>(dR1, a.out, F::DP, row, ok, spare, g);
    TF_ST(9);
  }
  TF_ST(10);
  __syncthreads();  // every wave is past its units: the weight area is free
  float* reg = sm + wv * L::SLAB;
  put_dw<NT, NT>(reg + L::S_WO, dWo, H, H, H, g, j);
  put_bias<NT>(reg + L::S_BO, bos, H, g, j);
  __syncthreads();
  sum_regions(a.part + (long)blockIdx.x * L::SLAB, sm, L::SLAB, L::SLAB);
  TF_ST(11);
  TF_ST_END(3);
}

template <int H>
constexpr size_t bff_lds() { return (size_t)BffL<H>::TOTAL * 4; }  // the FFN backward's dynamic LDS
template <int H>
hipError_t tf_launch(int kind, const TfArgs& a, int grid, hipStream_t st, hipEvent_t stop) {
  using F = TF<H>;
  if (stop && kind != 0) {  // the fused launches with a stop event (a fork right after them)
    void* args[] = {const_cast<TfArgs*>(&a)};
    const void* fn = kind == 1 ? reinterpret_cast<const void*>(tf_fwd_kernel<H>)
                     : kind == 2 ? reinterpret_cast<const void*>(tf_bwd_ffn_kernel<H>)
                                 : reinterpret_cast<const void*>(tf_bwd_att_kernel<H>);
    const size_t lds = kind == 2 ? bff_lds<H>() : (size_t)(kind == 1 ? FwdL<H>::TOTAL : BatL<H>::TOTAL) * 4;
    const int threads = (kind == 1 ? kTfFwdWaves : kTfWaves) * 64;
    return hipExtLaunchKernel(fn, dim3(grid), dim3(threads), args, lds, st, nullptr, stop, 0);
  }
  switch (kind) {
    case 0: {
      const long n = F::PACK_ITEMS;
      tf_pack_kernel<H><<<(int)((n + 255) / 256), 256, 0, st>>>(a.P, a.frags);
      return hipGetLastError();
    }
    case 1: {
      const size_t lds = (size_t)FwdL<H>::TOTAL * 4;
      tf_fwd_kernel<H><<<grid, kTfFwdWaves * 64, lds, st>>>(a);
      return hipGetLastError();
    }
    case 2: {
      const size_t lds = bff_lds<H>();
      tf_bwd_ffn_kernel<H><<<grid, kTfWaves * 64, lds, st>>>(a);
      return hipGetLastError();
    }
    case 3: {
      const size_t lds = (size_t)BatL<H>::TOTAL * 4;
      tf_bwd_att_kernel<H><<<grid, kTfWaves * 64, lds, st>>>(a);
      return hipGetLastError();
    }
  }
  return hipErrorInvalidValue;
}

template <int H>
bool tf_lds_ok() {
  return FwdL<H>::TOTAL * 4 <= 160 * 1024 && BffL<H>::TOTAL * 4 <= 160 * 1024 && BatL<H>::TOTAL * 4 <= 160 * 1024;
}

}  // namespace

long tf_frag_floats(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return TF<h>::TOTAL_FLOATS;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

long tf_pack_items(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return TF<h>::PACK_ITEMS;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

long tf_slab_floats(int H, int kind) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return kind == 2 ? BffL<h>::SLAB : BatL<h>::SLAB;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

// CUs left to other streams (pgp_tune_reserve_cus): a fused launch holds whole
// CUs (one workgroup per CU, its registers and LDS) and deals its units to the
// waves statically, so one CU taken by a concurrent stream's long workgroup
// (the GAN step beside the tuning step) holds back the whole launch; with a
// few CUs reserved the two streams stop blocking each other
std::atomic<int> g_tf_reserve{0};

// The launch takes the FEWEST workgroups that keep its longest wave as short
// as on the whole budget: units are whole 16-pair tiles, so the kernel lasts
// max-units-per-wave unit rounds, and at H = 50 (3,200 units, 248 workgroups x
// 4 waves) a quarter of the waves carry 4 units and the rest 3 -- 200
// workgroups of 4-unit waves finish in the same 4 rounds and leave 56 CUs to
// the GAN stream and the side work instead of sharing CUs with them.
int tf_grid_for(long nu, int waves) {
  const int cus = device_cus();
  const int r = std::max(0, std::min(g_tf_reserve.load(std::memory_order_relaxed), cus / 2));
  const long gmax = std::max<long>(1, std::min<long>(cus - r, (nu + waves - 1) / waves));
  const long m = (nu + waves * gmax - 1) / (waves * gmax);  // units of the longest wave
  return (int)std::max<long>(1, (nu + waves * m - 1) / (waves * m));
}

int tf_max_grid() { return device_cus(); }

int tf_bwd_grid(int H, int B) { return tf_grid_for(((long)B * H + 15) / 16, kTfWaves); }

void tf_reserve_cus(int n) { g_tf_reserve.store(n < 0 ? 0 : n, std::memory_order_relaxed); }

#ifdef PGP_TF_STAMPS
// profiling builds: copy out (host != null) or clear (host == null) the phase stamps
extern "C" int pgp_debug_tf_stamps(unsigned long long* host) {
  if (!host) {
    static unsigned long long zero[4][kStWaves][kStPhases];
    return hipMemcpyToSymbol(HIP_SYMBOL(tf_stamps), zero, sizeof(zero)) == hipSuccess ? 0 : -3;
  }
  if (hipDeviceSynchronize() != hipSuccess) return -3;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(tf_stamps), sizeof(tf_stamps)) == hipSuccess ? 0 : -3;
}
#endif

hipError_t launch_tf(int H, int kind, const TfArgs& a, hipStream_t st, hipEvent_t stop) {
  const long nu = ((long)a.B * H + 15) / 16;
  const int grid = tf_grid_for(nu, kind == 1 ? kTfFwdWaves : kTfWaves);
  switch (H) {
#define CASE(h)                                                                          \
  case h: {                                                                              \
    static_assert(FwdL<h>::TOTAL * 4 <= 160 * 1024, "forward LDS");                      \
    static_assert(TF<h>::DP <= 64, "tf_zero_row covers a row");                          \
    static_assert(BffL<h>::TOTAL * 4 <= 160 * 1024, "ffn backward LDS");                 \
    static_assert(BatL<h>::TOTAL * 4 <= 160 * 1024, "attention backward LDS");           \
    static bool attr = [] {                                                              \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(tf_fwd_kernel<h>),         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, FwdL<h>::TOTAL * 4); \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(tf_bwd_ffn_kernel<h>),     \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bff_lds<h>()); \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(tf_bwd_att_kernel<h>),     \
                                hipFuncAttributeMaxDynamicSharedMemorySize, BatL<h>::TOTAL * 4); \
      return true;                                                                       \
    }();                                                                                 \
    (void)attr;                                                                          \
    return tf_launch<h>(kind, a, grid, st, stop);                                        \
  }
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
