// pgp_gobi.hip — GOBI, the schedule producer of the decision path (SURVEY §8f
// row f3): scheduler/GOBI.py:19-42 -> scheduler/BaGTI/src/opt.py:17-33 over
// the energy_latency_16 surrogate (scheduler/BaGTI/src/models.py:8-27), for a
// batch of independent environments.
//
// One 512-thread workgroup (8 waves, 2 per SIMD) runs the whole optimisation
// of kNE = 4 environments in-kernel (the reference's loop: up to 200 AdamW
// steps on the input matrix, one-hot projection after each, stop after 31
// unchanged steps); the four share the weight registers and every barrier,
// and the launch lasts as long as its slowest workgroup's iteration chain.
// The MLP (288-128-128-64-2) and its input gradient are VALU dot products
// split over the threads in fixed k-chunks whose association every variant
// keeps (the trajectories are bit-identical to round 2's v7): the 128-output
// layers and the input gradient on DPP rows (a row's chunk inputs spread over
// its 16 lanes and broadcast by v_fmac_f32_dpp row_newbcast, the chunk sums by
// permlane swaps), layer 3 and the head on lane groups (DPP butterflies).
// Layer 1's allocation columns sit in LDS (the forward's one-hot column
// gather); the other weights live in registers.  Once some environments of a
// workgroup have converged, only the active ones' chains run.  Elementwise
// semantics follow torch's CPU kernels (softplus threshold 20, tanhshrink =
// x - tanh x composite, sigmoid backward g(1-y)y, AdamW single-tensor op
// order); per-iteration AdamW scalars (cosine lr) are computed on the host in
// double, as torch does.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/preganplus.h"
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kH = 16, kF = 2 + kH, kIn = kH * kF;  // 16 containers x [cpu, ips, one-hot 16] = 288
constexpr int kN1 = 128, kN2 = 128, kN3 = 64;
constexpr int kMaxIt = 200, kPatience = 30;

struct GobiW {  // device offsets (floats) into one buffer
  static constexpr int W1T = 0;                    // [288][128]
  static constexpr int W1 = W1T + kIn * kN1;       // [128][288]
  static constexpr int B1 = W1 + kN1 * kIn;        // [128]
  static constexpr int W2T = B1 + kN1;             // [128][128]
  static constexpr int W2 = W2T + kN1 * kN2;       // [128][128]
  static constexpr int B2 = W2 + kN2 * kN1;
  static constexpr int W3T = B2 + kN2;             // [128][64]
  static constexpr int W3 = W3T + kN2 * kN3;       // [64][128]
  static constexpr int B3 = W3 + kN3 * kN2;
  static constexpr int W4 = B3 + kN3;              // [2][64]
  static constexpr int B4 = W4 + 2 * kN3;
  static constexpr int ADAM = B4 + 4;              // [200][4]: decay, step size, sqrt(bc2), lr
  static constexpr int SIZE = ADAM + kMaxIt * 4;
};

__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + expf(-x)); }

constexpr int kT = 512;  // threads per workgroup (8 waves, 2 per SIMD: 256 VGPRs for the weight slices)
constexpr int kNE = 4;   // environments per workgroup: they share the weight registers and every barrier

// phase timing study (variant builds only): -DPGP_GOBI_PROF accumulates, in
// workgroup 0, the wall clock of each barrier-delimited phase over the run;
// pgp_gobi_prof_read copies the sums out
#ifdef PGP_GOBI_PROF
constexpr int kProfWG = 256, kProfSlots = 32;
__device__ unsigned long long g_gobi_prof[kProfWG][kProfSlots];
// (summed in the workgroup's LDS, L.prof, and added to g_gobi_prof once at
// the end: a global read-modify-write per mark stalled wave 0 for a memory
// round trip that the next barrier then charged to every phase)
#define GMARK(i)                                                        \
  do {                                                                  \
    if (threadIdx.x == 0) {                                             \
      const unsigned long long now_ = wall_clock64();                   \
      L.prof[i] += now_ - gmark_t_;                                     \
      if ((i) < 7 && act[0] + act[1] + act[2] + act[3] == 1)            \
        L.prof[16 + (i)] += now_ - gmark_t_;                            \
      gmark_t_ = now_;                                                  \
    }                                                                   \
  } while (0)
#else
#define GMARK(i) \
  do {           \
  } while (0)
#endif

constexpr int kA = kH * kH;  // allocation entries
__host__ __device__ constexpr int kp(int k) { return k + (k >> 4); }  // padded k-major row
constexpr int kP1 = kp(kN1), kP3 = kp(kN3);
constexpr int kSA = kA + 1;  // LDS row stride of layer 1's allocation columns (257 = 1 mod 64)

// Layer 1's allocation columns (the forward's one-hot column gather) and the
// per-environment activations; the other weights are in registers.
struct GobiLds {
  float w1a[kN1 * kSA];  // W1[o][c*18 + 2 + h] at [o][c*16 + h]
  float x[kNE][kIn];
  // the dot products' inputs k-major ([k][env]: one 16-byte read gives the
  // four environments' k-th value), one pad row after every 16 (kp(k)) so the
  // lanes' chunks (16 or 32 rows each) start in different banks; the head's
  // and the input gradient's inputs per environment
  alignas(16) float h1[kP1][kNE], h2[kP1][kNE], g2[kP1][kNE], g3[kP3][kNE], g1[kP1][kNE];
  float h3[kNE][kN3], th3[kNE][kN3];
  float o[kNE][4];
  alignas(16) float adam[kMaxIt][4];  // the per-iteration AdamW scalars (GobiW::ADAM), read from LDS in the loop
  int hs[kNE][kH];   // each container's host (the one-hot column of its allocation row)
  int dense[kNE];    // the init's allocation is not one-hot (iteration 0 takes the dense layer 1)
  alignas(16) int flag[2][kNE];  // "some entry changed" of the current / next iteration (one 16-byte read)
#ifdef PGP_GOBI_PROF
  unsigned long long prof[kProfSlots];
#endif
};

// Thread roles (fixed for the whole run; every weight slice is loaded once):
//   128-output layers (1, 2 and the backward's dh2, dh1): wave w, row r, row
//     lane i: o = 16w + i, k-chunk sp = r; the rows' sums (row_sum4: the bits
//     of the 4-lane butterfly) in every lane, and row sp == e owns env e's
//     activation and keeps its pre-activation for the backward;
//   layer 3 (64 outputs): o3 = t >> 3, k-chunk sp3 = t & 7, owner lane 2e;
//   the head: wave e (t < 256), lane = o3;
//   allocation entries: a DPP row of 16 lanes (row r of wave w) is container
//     c = 2w + (r >> 1), lane = host, k-chunk sq = r & 1 of the input gradient
//     (the chunk pair of an entry in lanes l and l ^ 16); the lane owns the
//     entry of envs e = sq, sq + 2 (their AdamW moments).
struct GobiRegs {
  float w2f[32], w2b[32], w3f[16], w3b[16], w1c[64];
  float w1x[8];  // layer 1's cpu / ips weights of this lane's 4 containers
  float b1, b2, b3, w40, w41, b40, b41;
};

__device__ void load_regs(const float* __restrict__ W, GobiRegs& R) {
  const int t = threadIdx.x, o = (t >> 6) * 16 + (t & 15), sp = (t >> 4) & 3, o3 = t >> 3, sp3 = t & 7;
  const int sq = (t >> 4) & 1, xi = ((t >> 6) * 2 + ((t >> 5) & 1)) * kF + 2 + (t & 15);
#pragma unroll
  for (int j = 0; j < 64; ++j) R.w1c[j] = W[GobiW::W1T + xi * kN1 + sq * 64 + j];  // W1[k][xi]
#pragma unroll
  for (int j = 0; j < 32; ++j) R.w2f[j] = W[GobiW::W2 + o * kN1 + sp * 32 + j];   // W2[o][k]
#pragma unroll
  for (int j = 0; j < 32; ++j) R.w2b[j] = W[GobiW::W2T + o * kN2 + sp * 32 + j];  // W2[k][o]
#pragma unroll
  for (int j = 0; j < 16; ++j) R.w3f[j] = W[GobiW::W3 + o3 * kN2 + sp3 * 16 + j];  // W3[o3][k]
#pragma unroll
  for (int j = 0; j < 16; ++j) R.w3b[j] = W[GobiW::W3T + o * kN3 + sp * 16 + j];   // W3[k][o]
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * sp + q;
    R.w1x[2 * q] = W[GobiW::W1 + o * kIn + c * kF];
    R.w1x[2 * q + 1] = W[GobiW::W1 + o * kIn + c * kF + 1];
  }
  R.b1 = W[GobiW::B1 + o];
  R.b2 = W[GobiW::B2 + o];
  R.b3 = W[GobiW::B3 + o3];
  R.w40 = W[GobiW::W4 + (t & 63)];
  R.w41 = W[GobiW::W4 + kN3 + (t & 63)];
  R.b40 = W[GobiW::B4];
  R.b41 = W[GobiW::B4 + 1];
}

// cross-lane moves inside a 16-lane row as DPP operand modifiers (a few cycles)
// instead of ds_bpermute round trips (__shfl_xor): quad_perm [1,0,3,2] = xor 1,
// [2,3,0,1] = xor 2; row_half_mirror (lane i <- 7 - i of its 8) pairs the two
// quads of an 8-lane group; row_ror 8 = xor 8; row_ror 4 rotates the row.  Every
// sum keeps the butterfly's association (bitwise as the shuffles)
constexpr int kDppX1 = 0xB1, kDppX2 = 0x4E, kDppHalfMirror = 0x141, kDppRor4 = 0x124, kDppRor8 = 0x128;
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
// lane i <- lane i ^ 4 (row_shl 4 into banks 0 / 2, row_shr 4 into banks 1 / 3)
__device__ __forceinline__ float dppf_xor4(float v) {
  const int b = __float_as_int(v);
  const int lo = __builtin_amdgcn_update_dpp(0, b, 0x104, 0xF, 0x5, false);  // row_shl:4, banks 0, 2
  return __int_as_float(__builtin_amdgcn_update_dpp(lo, b, 0x114, 0xF, 0xA, false));  // row_shr:4, banks 1, 3
}

// sum over N aligned adjacent lanes (N = 2, 4, 8), the same bits in all of them:
// xor 1, xor 2, then the two 4-lane halves (whose lanes already agree) exchanged
template <int N>
__device__ __forceinline__ float lane_sum(float v) {
  static_assert(N == 2 || N == 4 || N == 8, "lane groups of 2, 4 or 8");
  v += dppf<kDppX1>(v);
  if constexpr (N >= 4) v += dppf<kDppX2>(v);
  if constexpr (N >= 8) v += dppf<kDppHalfMirror>(v);  // == lane i ^ 4's value: the quads already agree
  return v;
}

// the four environments' partial dot products over this lane's N-k chunk:
// w[j] times h[kp(j)][e] (h at the chunk's first row, a multiple of 16), one
// 16-byte LDS read per k feeding four independent fmaf chains (one per
// environment, each in k order as before).  The reads go in groups of 2 k,
// the next group's issued before this group's FMAs; the scheduling barriers
// keep the compiler from hoisting every read of the chunk (it would spill the
// weight registers to hold them)
template <int N>
__device__ __forceinline__ void dot4(const float* w, const float (*h)[kNE], float (&r)[kNE]) {
  constexpr int G = 2;
  static_assert(N % G == 0, "chunk of whole groups");
  auto ld = [&](int j) { return *reinterpret_cast<const float4*>(h[kp(j)]); };
#pragma unroll
  for (int e = 0; e < kNE; ++e) r[e] = 0.f;
  float4 cur[G], nxt[G];
#pragma unroll
  for (int q = 0; q < G; ++q) cur[q] = ld(q);
#pragma unroll
  for (int g = 0; g < N / G; ++g) {
    if (g + 1 < N / G) {
#pragma unroll
      for (int q = 0; q < G; ++q) nxt[q] = ld((g + 1) * G + q);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const float wj = w[g * G + q];
      r[0] = fmaf(wj, cur[q].x, r[0]);
      r[1] = fmaf(wj, cur[q].y, r[1]);
      r[2] = fmaf(wj, cur[q].z, r[2]);
      r[3] = fmaf(wj, cur[q].w, r[3]);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < G; ++q) cur[q] = nxt[q];
  }
}
// the k-chunk dot products of the 128-output layers for the four environments:
// row r of the wave holds chunk sp = r; its N inputs x 4 envs (k-major rows h,
// from the chunk's first) are spread over the row's 16 lanes, P = N / 16
// consecutive k each (P 16-byte reads), and k = J is broadcast from row lane
// J / P (component J % P) into each environment's fmaf chain, in k order as
// dot4's.  All four active: the chains side by side; otherwise only the
// active environments' chains run (the others' sums are left at 0, unused).
// Each multiply-add is one v_fmac_f32 with a row_newbcast source (the builtin
// form costs a separate v_mov_b32_dpp).  A DPP instruction reads its swizzled
// source as of 2 wait states back, and inline asm hides it from the compiler's
// hazard check.  The sources here are LDS loads (no VALU writes them), and
// tools/dpp_hazard_check.py checks the BUILT kernel for any VALU write of a
// DPP source within 2 wait states (tests/test_roofline_isa.py runs it on the
// library, so a compiler-inserted copy fails the CPU suite).  A tied s_nop
// before the chains instead made the loads complete before the first FMA
// (0.731 -> 0.756 ms).
// acc += (row lane L's g) * w
template <int L>
__device__ __forceinline__ void fmac_bcast(float& acc, float g, float w) {
  asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(g), "v"(w), "i"(L));
}
// chain1: one environment's chain (k = J)
template <int P, int E, int J, int N>
__device__ __forceinline__ void chain1(const float4 (&gq)[P], const float* w, float& a) {
  const float4 g = gq[J % P];
  fmac_bcast<J / P>(a, E == 0 ? g.x : E == 1 ? g.y : E == 2 ? g.z : g.w, w[J]);
  if constexpr (J + 1 < N) chain1<P, E, J + 1, N>(gq, w, a);
}
// chain4: the four chains side by side
template <int P, int J, int N>
__device__ __forceinline__ void chain4(const float4 (&gq)[P], const float* w, float (&a)[kNE]) {
  const float4 g = gq[J % P];
  fmac_bcast<J / P>(a[0], g.x, w[J]);
  fmac_bcast<J / P>(a[1], g.y, w[J]);
  fmac_bcast<J / P>(a[2], g.z, w[J]);
  fmac_bcast<J / P>(a[3], g.w, w[J]);
  if constexpr (J + 1 < N) chain4<P, J + 1, N>(gq, w, a);
}
template <int N, int P>
__device__ __forceinline__ void dotb_regs(const float4 (&gq)[P], const float* w, const bool (&act)[kNE],
                                          float (&r)[kNE]) {
  static_assert(P == N / 16, "P inputs per row lane");
#pragma unroll
  for (int e = 0; e < kNE; ++e) r[e] = 0.f;
  if (act[0] && act[1] && act[2] && act[3]) {
    chain4<P, 0, N>(gq, w, r);
  } else {
    if (act[0]) chain1<P, 0, 0, N>(gq, w, r[0]);
    if (act[1]) chain1<P, 1, 0, N>(gq, w, r[1]);
    if (act[2]) chain1<P, 2, 0, N>(gq, w, r[2]);
    if (act[3]) chain1<P, 3, 0, N>(gq, w, r[3]);
  }
}
template <int N>
__device__ __forceinline__ void dotb(const float (*h)[kNE], const float* w, const bool (&act)[kNE], float (&r)[kNE]) {
  constexpr int P = N / 16;
  const int lane = threadIdx.x & 15;
  float4 gq[P];
#pragma unroll
  for (int q = 0; q < P; ++q) gq[q] = *reinterpret_cast<const float4*>(h[kp(P * lane + q)]);
  dotb_regs<N, P>(gq, w, act, r);
}
// sum over the wave's 4 rows (lanes l ^ 16, then l ^ 32) by permlane swaps:
// every lane gets (c0 + c1) + (c2 + c3), the bits of the 4-lane butterfly
__device__ __forceinline__ float row_sum4(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// the row sums of the active environments' partials (all four: side by side,
// no branch); the one of env `mine_e`
__device__ __forceinline__ float sum_rows(float (&r)[kNE], const bool (&act)[kNE], int mine_e) {
  float m = 0.f;
  if (act[0] && act[1] && act[2] && act[3]) {
#pragma unroll
    for (int e = 0; e < kNE; ++e) {
      r[e] = row_sum4(r[e]);
      m = mine_e == e ? r[e] : m;
    }
  } else {
#pragma unroll
    for (int e = 0; e < kNE; ++e) {
      if (!act[e]) continue;
      r[e] = row_sum4(r[e]);
      m = mine_e == e ? r[e] : m;
    }
  }
  return m;
}
// the same for the chunk pair of rows 2m, 2m + 1 (c0 + c1 in both)
__device__ __forceinline__ float pair_sum(float v) {
  const auto pr = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(pr[0]) + __uint_as_float(pr[1]);
}
__device__ __forceinline__ void sum_pairs(float (&r)[kNE], const bool (&act)[kNE]) {
  if (act[0] && act[1] && act[2] && act[3]) {
#pragma unroll
    for (int e = 0; e < kNE; ++e) r[e] = pair_sum(r[e]);
  } else {
#pragma unroll
    for (int e = 0; e < kNE; ++e)
      if (act[e]) r[e] = pair_sum(r[e]);
  }
}
// the lane-group sums of the four environments' partials; the one of env `mine_e`
template <int G>
__device__ __forceinline__ float sum_pick(float (&r)[kNE], int mine_e) {
  float m = 0.f;
#pragma unroll
  for (int e = 0; e < kNE; ++e) {
    r[e] = lane_sum<G>(r[e]);
    m = mine_e == e ? r[e] : m;
  }
  return m;
}

// pre-activations (and their exp) of the activations this lane owns
struct FwdKeep {
  float a1, z1, a2, z2;
};
__device__ __forceinline__ float softplus_keep(float a, float& z) {  // softplus (threshold 20), z = exp(a)
  z = expf(a);
  return a > 20.f ? a : log1pf(z);
}
__device__ __forceinline__ float softplus_grad(float g, float a, float z) {  // torch: g * z / (z + 1)
  return a > 20.f ? g : g * z / (z + 1.f);
}

// forward of the surrogate for the environments in act (all threads);
// z = 0.8 o0 + 0.2 o1 in L.o[e][2]; with grad, g3 = dz/dh3 through Tanhshrink.
// act / dense are wave-uniform (the same in every thread).
__device__ void surrogate_fwd(const float* __restrict__ W, const GobiRegs& R, GobiLds& L, FwdKeep& K, bool grad,
                              const bool (&act)[kNE], const bool (&dense)[kNE], unsigned long long& gmark_t_) {
  (void)gmark_t_;
  const int t = threadIdx.x, o = (t >> 6) * 16 + (t & 15), sp = (t >> 4) & 3, o3 = t >> 3, sp3 = t & 7;
  bool act_sp = false, act_sp3 = false;  // this lane's owned environments (sp; sp3 / 2) are active
#pragma unroll
  for (int e = 0; e < kNE; ++e) {
    act_sp = sp == e ? act[e] : act_sp;
    act_sp3 = (sp3 >> 1) == e ? act[e] : act_sp3;
  }
  float mine = 0.f;
  // layer 1 (288 -> 128)
  float l1[kNE] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < kNE; ++e) {
    if (!act[e]) continue;
    float acc = 0.f;
    if (dense[e]) {  // any allocation: k-chunk sp of 72
      const float* wr = W + GobiW::W1 + o * kIn + sp * 72;
      const float* xr = L.x[e] + sp * 72;
#pragma unroll 8
      for (int k = 0; k < 72; ++k) acc = fmaf(wr[k], xr[k], acc);
    } else {  // one-hot allocation: containers 4sp..4sp+3: cpu, ips FMAs + their host's column (LDS)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 4 * sp + q;
        acc = fmaf(R.w1x[2 * q], L.x[e][c * kF], acc);
        acc = fmaf(R.w1x[2 * q + 1], L.x[e][c * kF + 1], acc);
        acc = acc + L.w1a[o * kSA + c * kH + L.hs[e][c]];  // w * 1.0; the other columns multiply 0
      }
    }
    l1[e] = acc;
  }
  mine = sum_rows(l1, act, sp);
  // the elementwise tail once per lane, for its own environment sp (not once
  // per environment under a quarter of the lanes)
  if (act_sp) {
    const float a = mine + R.b1;
    K.a1 = a;
    L.h1[kp(o)][sp] = softplus_keep(a, K.z1);
  }
  __syncthreads();
  GMARK(0);
  float r[kNE];
  // layer 2 (128 -> 128): W2 row o, k-chunk sp
  dotb<32>(&L.h1[kp(sp * 32)], R.w2f, act, r);
  mine = sum_rows(r, act, sp);
  if (act_sp) {
    const float a = mine + R.b2;
    K.a2 = a;
    L.h2[kp(o)][sp] = softplus_keep(a, K.z2);
  }
  __syncthreads();
  GMARK(1);
  // layer 3 (128 -> 64), Tanhshrink: W3 row o3, k-chunk sp3
  dot4<16>(R.w3f, &L.h2[kp(sp3 * 16)], r);
  mine = sum_pick<8>(r, sp3 >> 1);
  if (act_sp3) {  // lanes 2e and 2e + 1 both hold env e's sum; lane 2e writes
    const float a = mine + R.b3;
    const float th = tanhf(a);
    if (!(sp3 & 1)) {
      L.th3[sp3 >> 1][o3] = th;
      L.h3[sp3 >> 1][o3] = a - th;
    }
  }
  __syncthreads();
  GMARK(2);
  // layer 4 (64 -> 2), sigmoid, z; wave e, lane = o3
  if (t < 64 * kNE) {
    const int e = t >> 6, l = t & 63;
    bool on = false;
#pragma unroll
    for (int q = 0; q < kNE; ++q) on = e == q ? act[q] : on;
    if (on) {
      const float h3 = L.h3[e][l];
      float p0 = R.w40 * h3, p1 = R.w41 * h3;
      // 64-lane xor butterfly, offsets 32, 16, 8, 4, 2, 1 (the same bits in every
      // lane): 32 and 16 by permlane swaps instead of ds_bpermute round trips,
      // 8 = row_ror 8, 4 = two bank-masked row shifts, 2 and 1 = quad_perm.
      // The first step keeps the form the compiler gave the shuffle version:
      // the lane's own product fused into the add, fma(w, h3, partner's
      // rounded product)
      {
        const bool hi = (l & 32) != 0;
        const auto a0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(p0), __float_as_uint(p0), false, false);
        const auto a1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(p1), __float_as_uint(p1), false, false);
        p0 = fmaf(R.w40, h3, __uint_as_float(hi ? a0[0] : a0[1]));
        p1 = fmaf(R.w41, h3, __uint_as_float(hi ? a1[0] : a1[1]));
        p0 = pair_sum(p0);
        p1 = pair_sum(p1);
      }
      p0 += dppf<kDppRor8>(p0);
      p1 += dppf<kDppRor8>(p1);
      p0 += dppf_xor4(p0);
      p1 += dppf_xor4(p1);
      p0 += dppf<kDppX2>(p0);
      p1 += dppf<kDppX2>(p1);
      p0 += dppf<kDppX1>(p0);
      p1 += dppf<kDppX1>(p1);
      const float o0 = sigmoid_f(p0 + R.b40), o1 = sigmoid_f(p1 + R.b41);
      if (l == 0) {
        // the row address recomputed here (the compiler kept it in a scratch
        // slot across the loop and reloaded it every iteration)
        int ee = e;
        asm volatile("" : "+v"(ee));
        L.o[ee][0] = o0;
        L.o[ee][1] = o1;
        L.o[ee][2] = 0.8f * o0 + 0.2f * o1;
      }
      if (grad) {  // dz/do = (0.8, 0.2) through the sigmoids, dh3 = W4^T do, through Tanhshrink
        const float d0 = 0.8f * (1.f - o0) * o0, d1 = 0.2f * (1.f - o1) * o1;
        const float gh = R.w40 * d0 + R.w41 * d1;
        const float th = L.th3[e][l];
        L.g3[kp(l)][e] = gh - gh * (1.f - th * th);
      }
    }
  }
  __syncthreads();
  GMARK(3);
}

__global__ __launch_bounds__(kT) void gobi_kernel(int E, const float* __restrict__ W, const float* __restrict__ init,
                                                  float* __restrict__ result, int* __restrict__ iterations,
                                                  float* __restrict__ fitness, int max_it, float* __restrict__ pre) {
#pragma clang fp contract(off)  // elementwise steps as torch's separate mul/add
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  GobiLds& L = *reinterpret_cast<GobiLds*>(lds_raw);
  unsigned long long gmark_t_ = 0;
#ifdef PGP_GOBI_PROF
  gmark_t_ = wall_clock64();
#endif
  const int t = threadIdx.x, o = (t >> 6) * 16 + (t & 15), sp = (t >> 4) & 3;
  const int c = (t >> 6) * 2 + ((t >> 5) & 1), sq = (t >> 4) & 1, hcol = t & 15, entry = c * kH + hcol;
  const int xi = c * kF + 2 + hcol;  // this thread's allocation entry in the flattened input
  const long e0 = (long)blockIdx.x * kNE;
  for (int k = t; k < kN1 * kA; k += kT) {
    const int oo = k / kA, a = k - oo * kA;
    L.w1a[oo * kSA + a] = W[GobiW::W1 + oo * kIn + (a >> 4) * kF + 2 + (a & 15)];
  }
  for (int k = t; k < kNE * kIn; k += kT) {
    const int e = k / kIn;
    L.x[e][k - e * kIn] = e0 + e < E ? init[e0 * kIn + k] : 0.f;
  }
  for (int k = t; k < kMaxIt * 4; k += kT) (&L.adam[0][0])[k] = W[GobiW::ADAM + k];
  if (t < kNE) {
    L.dense[t] = 0;
    L.flag[0][t] = L.flag[1][t] = 0;
  }
#ifdef PGP_GOBI_PROF
  if (t < kProfSlots) L.prof[t] = 0;
#endif
  GobiRegs R;
  load_regs(W, R);
  __syncthreads();
  if (t < kNE * kH) {  // is the init's allocation one-hot?  (then layer 1 is a column gather)
    const int e = t / kH, cc = t % kH;
    int ones = 0, other = 0, h = 0;
    for (int j = 0; j < kH; ++j) {
      const float xv = L.x[e][cc * kF + 2 + j];
      if (xv == 1.f) {
        ++ones;
        h = j;
      } else if (xv != 0.f) {
        ++other;
      }
    }
    L.hs[e][cc] = h;
    if (ones != 1 || other) L.dense[e] = 1;  // benign race: every writer stores 1
  }
  __syncthreads();
#ifdef PGP_GOBI_PROF
  {
    const bool act[kNE] = {false, false, false, false};  // the prologue's mark
    GMARK(7);
  }
#endif
  float m[kNE / 2], v[kNE / 2];  // AdamW moments of this lane's entries (envs sq, sq + 2)
#pragma unroll
  for (int k = 0; k < kNE / 2; ++k) m[k] = v[k] = 0.f;
  FwdKeep K{0.f, 0.f, 0.f, 0.f};
  bool act[kNE], dense[kNE];
  int equal[kNE], its[kNE];
#pragma unroll
  for (int e = 0; e < kNE; ++e) {
    act[e] = e0 + e < E;
    dense[e] = __builtin_amdgcn_readfirstlane(L.dense[e]) != 0;
    equal[e] = 0;
    its[e] = max_it;
  }
  int it = 0;
  while (it < max_it) {
    bool any = false;
#pragma unroll
    for (int e = 0; e < kNE; ++e) any |= act[e];
    if (!any) break;
#ifdef PGP_GOBI_PROF
    int nact_ = 0;
#pragma unroll
    for (int e = 0; e < kNE; ++e) nact_ += act[e];
    const unsigned long long it_t0_ = wall_clock64();
#endif
    surrogate_fwd(W, R, L, K, true, act, dense, gmark_t_);
    // ---- backward to the input (autograd of z; g3 came with the forward) ----
    bool act_sp = false;
#pragma unroll
    for (int e = 0; e < kNE; ++e) act_sp = sp == e ? act[e] : act_sp;
    float mine = 0.f;
    // dh2 = W3^T g3 through softplus (W3 column o, k-chunk sp)
    float r[kNE];
    dotb<16>(&L.g3[kp(sp * 16)], R.w3b, act, r);
    mine = sum_rows(r, act, sp);
    if (act_sp) L.g2[kp(o)][sp] = softplus_grad(mine, K.a2, K.z2);
    if (t < kNE) L.flag[(it + 1) & 1][t] = 0;  // next iteration's flag; its last readers passed barriers since
    __syncthreads();
    GMARK(4);
    // dh1 = W2^T g2 through softplus (W2 column o, k-chunk sp)
    dotb<32>(&L.g2[kp(sp * 32)], R.w2b, act, r);
    mine = sum_rows(r, act, sp);
    if (act_sp) L.g1[kp(o)][sp] = softplus_grad(mine, K.a1, K.z1);
    __syncthreads();
    GMARK(5);
    // dx for the 256 allocation entries (W1[:, xi] . g1, 2 k-chunks of 64), AdamW, one-hot
    // the row's chunk of g1 (64 k x 4 envs) spread over its 16 lanes (four
    // 16-byte reads instead of 64), every k broadcast into the active
    // environments' chains (dotb), then the chunk pair of rows 2m, 2m + 1
    // (c0 + c1 in both) by a permlane swap
    float gxa[kNE];
    dotb<64>(&L.g1[kp(sq * 64)], R.w1c, act, gxa);
    sum_pairs(gxa, act);
    // this iteration's AdamW scalars, from LDS (scalar loads from memory at the
    // loop top made the first phase's LDS waits wait for them too: one lgkmcnt
    // counts both; 0.714 -> see DESIGN §17)
    const float4 ad = *reinterpret_cast<const float4*>(L.adam[it]);
    const float a0 = ad.x, a1 = ad.y, a2 = ad.z;
    // lane sq owns the entry of envs e = sq + 2k: AdamW and the one-hot once
    // per k with every lane busy (rows sq = 0 and 1 on envs 2k and 2k + 1)
#pragma unroll
    for (int k = 0; k < kNE / 2; ++k) {
      if (!act[2 * k] && !act[2 * k + 1]) continue;
      const int e = sq + 2 * k;
      const bool on = sq ? act[2 * k + 1] : act[2 * k];
      // a lane select of two registers: written as `sq ? gxa[2k+1] : gxa[2k]`
      // the compiler made it an indexed load of gxa[2k + sq], i.e. gxa stored
      // to scratch and read back every iteration (4 stores + 2 loads in the
      // AdamW chain); the opaque copies keep it a v_cndmask
      float ga = gxa[2 * k], gb = gxa[2 * k + 1];
      asm volatile("" : "+v"(ga), "+v"(gb));
      const float gx = sq ? gb : ga;
      // ---- AdamW (torch single-tensor, opt.py:18 defaults) on the entry ----
      const float xold = L.x[e][xi];
      float& mm = m[k];
      float& vv = v[k];
      float xv = xold * a0;
      if (on) {
        mm = mm + 0.1f * (gx - mm);           // exp_avg.lerp_(grad, 1 - beta1)
        vv = vv * 0.999f + 0.001f * gx * gx;  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
      }
      const float denom = sqrtf(vv) / a2 + 1e-8f;
      xv = xv + (-a1) * mm / denom;           // addcdiv_: self + value * t1 / t2 (ATen's order)
      // ---- one-hot of the row's first argmax (opt.py:9-15): the row's lanes of this sq ----
      // (max value, then lowest column) over the row's 16 lanes: xor 1, xor 2,
      // then the quads by rotations of 4 and 8 (each lane then holds the winner)
      float best = xv;
      int bi = hcol;
      auto take = [&](float ov, int oi) {
        const bool b = ov > best || (ov == best && oi < bi);
        best = b ? ov : best;
        bi = b ? oi : bi;
      };
      take(dppf<kDppX1>(best), dppi<kDppX1>(bi));
      take(dppf<kDppX2>(best), dppi<kDppX2>(bi));
      take(dppf<kDppRor4>(best), dppi<kDppRor4>(bi));
      take(dppf<kDppRor8>(best), dppi<kDppRor8>(bi));
      if (on) {
        if (pre) pre[(e0 + e) * kH * kH + entry] = xv;  // test tap: the step's values before the projection
        const float nv = bi == hcol ? 1.f : 0.f;
        if (nv != xold) L.flag[it & 1][e] = 1;  // benign race: every writer stores 1
        L.x[e][xi] = nv;
        if (bi == hcol) L.hs[e][c] = hcol;
      }
    }
    __syncthreads();
    GMARK(6);
    // convergence (opt.py:28-31), per environment, in every thread's registers
    // (the four flags in one 16-byte read)
    const int4 fl = *reinterpret_cast<const int4*>(L.flag[it & 1]);
    const int flv[kNE] = {fl.x, fl.y, fl.z, fl.w};
#pragma unroll
    for (int e = 0; e < kNE; ++e) {
      dense[e] = false;  // one-hot from here on
      if (!act[e]) continue;
      equal[e] = __builtin_amdgcn_readfirstlane(flv[e]) ? 0 : equal[e] + 1;
      if (equal[e] > kPatience) {
        its[e] = it;
        act[e] = false;
      }
    }
#ifdef PGP_GOBI_PROF
    if (blockIdx.x < kProfWG && t == 0) {  // iteration time and count by active environments
      L.prof[7 + nact_] += wall_clock64() - it_t0_;
      L.prof[11 + nact_] += 1;
    }
#endif
    ++it;
  }
  // final fitness of every real environment
#pragma unroll
  for (int e = 0; e < kNE; ++e) act[e] = e0 + e < E;
  surrogate_fwd(W, R, L, K, false, act, dense, gmark_t_);
  for (int k = t; k < kNE * kIn; k += kT) {
    const int e = k / kIn;
    if (e0 + e < E) result[e0 * kIn + k] = L.x[e][k - e * kIn];
  }
  if (t < kNE && e0 + t < E) {
    int n = its[0];
#pragma unroll
    for (int e = 1; e < kNE; ++e) n = t == e ? its[e] : n;  // no dynamic register-array index
    iterations[e0 + t] = n;
    fitness[e0 + t] = L.o[t][2];
  }
#ifdef PGP_GOBI_PROF
  if (blockIdx.x < kProfWG && t == 0) {
    for (int i = 0; i < 31; ++i) g_gobi_prof[blockIdx.x][i] += L.prof[i];
    g_gobi_prof[blockIdx.x][31] = (unsigned long long)it;
  }
#endif
}

}  // namespace
}  // namespace pgp

using namespace pgp;

struct pgp_gobi {
  int H = 0;
  float* d_w = nullptr;
};

namespace {
thread_local std::string g_gerr;
int gfail(int code, const std::string& msg) {
  g_gerr = msg;
  return code;
}
}  // namespace

extern "C" {

size_t pgp_gobi_weight_len(int n_hosts) {
  if (n_hosts != kH) return 0;
  return (size_t)kN1 * kIn + kN1 + kN2 * kN1 + kN2 + kN3 * kN2 + kN3 + 2 * kN3 + 2;
}

int pgp_gobi_create(int n_hosts, const float* weights, size_t len, pgp_gobi** out) {
  if (!out) return gfail(PGP_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (n_hosts != kH) return gfail(PGP_ERR_UNSUPPORTED, "GOBI surrogate: only energy_latency_16 exists (16 hosts)");
  if (!weights || len != pgp_gobi_weight_len(n_hosts)) return gfail(PGP_ERR_ARG, "GOBI weight length mismatch");
  // state-dict order: find.0.weight [128,288], find.0.bias, find.2.weight [128,128], find.2.bias,
  //                   find.4.weight [64,128], find.4.bias, find.6.weight [2,64], find.6.bias
  const float* w1 = weights;
  const float* b1 = w1 + kN1 * kIn;
  const float* w2 = b1 + kN1;
  const float* b2 = w2 + kN2 * kN1;
  const float* w3 = b2 + kN2;
  const float* b3 = w3 + kN3 * kN2;
  const float* w4 = b3 + kN3;
  const float* b4 = w4 + 2 * kN3;
  std::vector<float> h(GobiW::SIZE, 0.f);
  for (int o = 0; o < kN1; ++o)
    for (int k = 0; k < kIn; ++k) {
      h[GobiW::W1 + o * kIn + k] = w1[o * kIn + k];
      h[GobiW::W1T + k * kN1 + o] = w1[o * kIn + k];
    }
  for (int o = 0; o < kN2; ++o)
    for (int k = 0; k < kN1; ++k) {
      h[GobiW::W2 + o * kN1 + k] = w2[o * kN1 + k];
      h[GobiW::W2T + k * kN2 + o] = w2[o * kN1 + k];
    }
  for (int o = 0; o < kN3; ++o)
    for (int k = 0; k < kN2; ++k) {
      h[GobiW::W3 + o * kN2 + k] = w3[o * kN2 + k];
      h[GobiW::W3T + k * kN3 + o] = w3[o * kN2 + k];
    }
  for (int i = 0; i < kN1; ++i) h[GobiW::B1 + i] = b1[i];
  for (int i = 0; i < kN2; ++i) h[GobiW::B2 + i] = b2[i];
  for (int i = 0; i < kN3; ++i) h[GobiW::B3 + i] = b3[i];
  for (int i = 0; i < 2 * kN3; ++i) h[GobiW::W4 + i] = w4[i];
  h[GobiW::B4] = b4[0];
  h[GobiW::B4 + 1] = b4[1];
  // AdamW(lr=0.8, betas (0.9, 0.999), eps 1e-8, weight_decay 1e-2) under
  // CosineAnnealingLR(T_max=10), torch's recursive update, in double as torch does
  const double base = 0.8, wd = 1e-2, T = 10.0;
  double lr = base;
  for (int i = 0; i < kMaxIt; ++i) {
    const int step = i + 1;
    h[GobiW::ADAM + i * 4 + 0] = (float)(1.0 - lr * wd);
    h[GobiW::ADAM + i * 4 + 1] = (float)(lr / (1.0 - std::pow(0.9, step)));
    h[GobiW::ADAM + i * 4 + 2] = (float)std::sqrt(1.0 - std::pow(0.999, step));
    h[GobiW::ADAM + i * 4 + 3] = (float)lr;
    const int ep = i + 1;
    if ((ep - 1 - 10) % 20 == 0)
      lr = lr + base * (1 - std::cos(M_PI / T)) / 2;
    else
      lr = (1 + std::cos(M_PI * ep / T)) / (1 + std::cos(M_PI * (ep - 1) / T)) * lr;
  }
  pgp_gobi* g = new pgp_gobi();
  g->H = n_hosts;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gobi_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)sizeof(GobiLds)) != hipSuccess) {
    delete g;
    return gfail(PGP_ERR_HIP, "GOBI: cannot reserve LDS");
  }
  if (hipMalloc(&g->d_w, h.size() * sizeof(float)) != hipSuccess ||
      hipMemcpy(g->d_w, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
    if (g->d_w) (void)hipFree(g->d_w);
    delete g;
    return gfail(PGP_ERR_HIP, "GOBI weight upload failed");
  }
  *out = g;
  return PGP_OK;
}

int pgp_gobi_destroy(pgp_gobi* g) {
  if (!g) return PGP_OK;
  if (g->d_w) (void)hipFree(g->d_w);
  delete g;
  return PGP_OK;
}

const char* pgp_gobi_last_error(void) { return g_gerr.c_str(); }

#ifdef PGP_GOBI_PROF
int pgp_gobi_prof_read(unsigned long long* out) {  // phase sums of workgroup 0 (timing variant only)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gobi_prof), sizeof(g_gobi_prof)) == hipSuccess ? 0 : -1;
}
int pgp_gobi_prof_reset(void) {
  static const unsigned long long z[kProfWG * kProfSlots] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_gobi_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

int pgp_gobi_optimize(pgp_gobi* g, int n_env, const float* init, float* result, int* iterations, float* fitness,
                      int max_iters, float* pre, void* stream) {
  if (!g) return gfail(PGP_ERR_ARG, "NULL optimiser");
  if (n_env < 0) return gfail(PGP_ERR_ARG, "negative batch");
  if (n_env == 0) return PGP_OK;
  if (!init || !result || !iterations || !fitness) return gfail(PGP_ERR_ARG, "NULL input/output pointer");
  const int mi = (max_iters <= 0 || max_iters > kMaxIt) ? kMaxIt : max_iters;
  gobi_kernel<<<(n_env + kNE - 1) / kNE, kT, sizeof(GobiLds), reinterpret_cast<hipStream_t>(stream)>>>(n_env, g->d_w, init, result,
                                                                                          iterations, fitness, mi, pre);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return gfail(PGP_ERR_HIP, std::string("gobi_kernel: ") + hipGetErrorString(e));
  return PGP_OK;
}

}  // extern "C"
