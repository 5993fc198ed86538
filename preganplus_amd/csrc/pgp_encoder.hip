// pgp_encoder.hip — K2: time encoder + positional encoding + 2 post-norm
// TransformerEncoderLayers (models.py:344-356, 390-396) for all H hosts of 16
// windows per wave.  Output: the encoder activations ("latent",
// models.py:399) as MFMA B-operand tiles for the decoder GEMM (K2b).
//
// Weights live in LDS and are read as A-operand fragments with ds_read_b128
// (lane-linear, conflict-free).  Three modes:
// * tail-resident (H = 50): the groups the path reads (layer 0's FFN, all of
//   layer 1) are loaded once into one 8-wave workgroup per CU; each wave takes
//   an equal contiguous range of the (16-window block, host) units (hosts are
//   independent here) and prefetches the next unit's raw features through a
//   per-wave LDS slot; no barrier in the host loop;
// * resident (H <= 16): both layers' weights in LDS, one 16-window block per
//   wave, host loop without barriers;
// * ring (other H): stages stream through a 2-slot LDS ring by
//   global_load_lds (stage k computed while k + 1 loads), shared by the
//   workgroup's 4 waves; two workgroups per CU let one block's VALU phases
//   overlap the other's MFMA phases.
#include "pgp_device.hpp"

namespace pgp {
namespace {

// Launch geometry (the alternatives were A/B-timed and are recorded in
// DESIGN.md §12; they are not kept as build switches):
//  * tail mode, layer 0: attention scores as bilinear forms of the 3 raw
//    features per step (q, k affine in them; pgp_pack.cpp T_F0S): lane-local
//    FMAs instead of q / k tiles, partial dot products and cross-lane sums;
//  * H <= 16 (weights LDS-resident): kEnc16Waves waves per workgroup share one
//    LDS copy, kEnc16EU waves per SIMD requested from the register allocator,
//    one 16-window block per wave (unit ranges measured slower there).
constexpr int kEncWaves = 4;
constexpr int kEnc16Waves = 4, kEnc16EU = 2;
// Tail mode (H = 50) resident: the weight groups the tail path reads (layer 0's
// stage 2 — its q/k/v and out_proj are folded onto the raw features — and all
// of layer 1: 104 KB at H = 50) stay in LDS for the whole launch, one 8-wave
// workgroup per CU (2 waves per SIMD as before); no ring barriers or DMAs in the
// host loop, and one copy per workgroup instead of one per host
template <int H>
constexpr bool tail_res() { return Geo<H>::TAIL; }
// waves per tail-resident workgroup (one workgroup per CU): 8 = 2 waves per
// SIMD, 12 = 3 (the register allocator then has 168 VGPRs + AGPRs per wave)
constexpr int kEncTailWaves = 8;
template <int H>
constexpr int enc_waves() { return H <= 16 ? kEnc16Waves : tail_res<H>() ? kEncTailWaves : kEncWaves; }
template <int H>
constexpr int NW_STAGE() { return enc_waves<H>(); }

// the split feed-forward's planes read one (block, tile) ahead of their MFMAs
// (A/B, C2 at H = 50, 5 interleaved rounds: K2 3.499 -> 3.370 ms, C2 5.160 ->
// 5.025 ms, profiles/r06/c2/ab_encoder_pipe.txt)
#ifndef PGP_ENC_PIPE
#define PGP_ENC_PIPE 1
#endif
constexpr bool kEncPipe = PGP_ENC_PIPE != 0;
// the fp32 GEMMs' A fragments likewise (A/B switch; measured within noise at
// H = 50 (5.217 vs 5.206 ms) and H = 16 (fleet 1.8669 vs 1.8666 ms), 4
// registers spilled at H = 50: off)
#ifndef PGP_ENC_PIPE_F32
#define PGP_ENC_PIPE_F32 0
#endif
constexpr bool kEncPipeF32 = PGP_ENC_PIPE_F32 != 0;

// Split-bf16 feed-forward (tail-resident mode, H = 50): both layers' linear1
// (K = d) and linear2 (K = 64) run as v_mfma_f32_16x16x32_bf16 over exact
// three-part bf16 splits of both operands (the six products i + j <= 2, as K2b
// and K3: pgp_device.hpp split8 / mfma_bf6), 96 MFMA cycles per 32-k block
// against 256 for the fp32 MFMA; the FFN is 54% of K2's MFMA cycles.  A 32-k
// block pairs two of the fp32 form's 4-k-step groups lane-locally (groups 2b,
// 2b + 1: a lane's 8 values), for the weights (planes derived once per weight
// load, enc_split_kernel) and the activations (split in registers).  The LDS
// image (groups of 1 KiB, EncS): layer 0's FFN planes | layer 1's qk, v, o
// (fp32, as in the stream) | layer 1's FFN planes: 132 KiB (fp32 form: 104).
template <int H>
struct EncS {
  using G = Geo<H>;
  static constexpr int NBD = cdiv(G::KQ_D, 2);  // 32-k blocks over d
  static constexpr int NBF = G::KQ_F / 2;       // 32-k blocks over the hidden 64
  static constexpr int F1S = G::MT_F * NBD * 3;  // linear1 planes [c][blk][plane]
  static constexpr int F2S = G::MT_X * NBF * 3;  // linear2 planes [m][blk][plane]
  static constexpr int FFN = F1S + F2S;
  static constexpr int L0F = 0;                 // layer 0 FFN
  static constexpr int L1A = FFN;               // layer 1 stages 0, 1 (fp32 groups [0, P_F1))
  static constexpr int L1F = L1A + G::P_F1;     // layer 1 FFN
  static constexpr int GROUPS = L1F + FFN;
  static constexpr int STREAM = GROUPS * G::FQ;  // floats
  static constexpr long SIZE = STREAM;           // the device image (floats)
};

// RESIDENT (H <= 16): both layers' weights (24 KB at H = 16) are loaded into LDS
// once per workgroup; the host loop then runs with no ring barriers or DMAs.
// Tail-resident: groups [RES0, 2*LAYER_G) of the stream (see tail_res), or the
// split image (EncS).
template <int H, bool SPLIT = false>
struct EncLds {
  static constexpr bool TRES = tail_res<H>();
  // the tail-resident mode has no barrier in the host loop: waves take
  // (block, host) unit ranges and prefetch through an LDS slot (at H <= 16,
  // also resident, that measured slower: fleet 1.97 -> 2.00 ms)
  static constexpr int RES0 = TRES ? Geo<H>::st_begin(Geo<H>::NST - 1) : 0;  // layer 0 stage 2
  static constexpr int STREAM = SPLIT ? EncS<H>::STREAM : (kLayers * Geo<H>::LAYER_G - RES0) * Geo<H>::FQ;  // floats
  static constexpr bool RESIDENT = TRES || STREAM * 4 <= 32 * 1024;
  static constexpr int SLOT = Geo<H>::SLOT_G * Geo<H>::FQ;
  static constexpr int TAB = Geo<H>::t_size(kMaxProtos);
  static constexpr int TOTAL = (RESIDENT ? STREAM : 2 * SLOT) + TAB;
  static constexpr bool UNITS = TRES;
};

template <int H>
constexpr bool enc_split() {
  return tail_res<H>() && EncLds<H, true>::TOTAL * 4 + enc_waves<H>() * 144 * 4 <= 160 * 1024;
}

// fp32 stream -> the split image: one wave per FFN plane triple or fp32 group
template <int H>
__global__ __launch_bounds__(256) void enc_split_kernel(const float* __restrict__ enc, float* __restrict__ out) {
  using G = Geo<H>;
  using S = EncS<H>;
  constexpr int T1 = G::MT_F * S::NBD, T2 = G::MT_X * S::NBF, TL = T1 + T2;  // triples per layer
  const long f = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (f >= 2 * TL + G::P_F1) return;
  if (f >= 2 * TL) {  // layer 1's attention groups, copied
    const long i = f - 2 * TL;
    *reinterpret_cast<f32x4*>(out + (S::L1A + i) * 256 + lane * 4) = ld4(enc + (G::LAYER_G + i) * 256 + lane * 4);
    return;
  }
  const int l = (int)(f / TL), t = (int)(f % TL);
  const float* src = enc + (long)(l * G::LAYER_G + G::P_F1) * 256;  // the layer's f1 | f2 groups
  long q0, q1, dst;  // the two fp32 groups (-1: zero) and the first destination plane
  const long base = l == 0 ? S::L0F : S::L1F;
  if (t < T1) {  // linear1 tile c, d block b: groups [c][q4]
    const int c = t / S::NBD, b = t % S::NBD;
    q0 = c * G::KQ_D + 2 * b;
    q1 = 2 * b + 1 < G::KQ_D ? q0 + 1 : -1;
    dst = base + (long)t * 3;
  } else {  // linear2 tile m, hidden block b: groups G_F1 + [m][q4]
    const int u = t - T1, m = u / S::NBF, b = u % S::NBF;
    q0 = G::G_F1 + m * G::KQ_F + 2 * b;
    q1 = q0 + 1;
    dst = base + S::F1S + (long)u * 3;
  }
  float v[8];
  const f32x4 x0 = ld4(src + q0 * 256 + lane * 4);
  const f32x4 x1 = q1 >= 0 ? ld4(src + q1 * 256 + lane * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = x0[e];
    v[4 + e] = x1[e];
  }
  u32x4 p[3];
  split8(v, p);
#pragma unroll
  for (int k = 0; k < 3; ++k) *reinterpret_cast<u32x4*>(out + (dst + k) * 256 + lane * 4) = p[k];
}

// the lane's 8 values of 32-k block b of a [NT][3] activation (tiles 2b, 2b + 1
// of step w; a tile past NT is zero)
template <int NT>
PGP_DEV void pair_tiles(const f32x4 (&T)[NT][3], int b, int w, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = 2 * b < NT ? T[2 * b][w][e] : 0.f;
    v[4 + e] = 2 * b + 1 < NT ? T[2 * b + 1][w][e] : 0.f;
  }
}
PGP_DEV void planes_lds(const float* F, int lane, u32x4 (&w)[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) w[k] = *reinterpret_cast<const u32x4*>(F + k * 256 + lane * 4);
}

// ReLU as one integer max on the bit pattern (negative floats have negative
// int patterns): fmaxf on an MFMA result costs a NaN-canonicalising v_max first,
// so 2 VALU ops per element; this is 1 (-0.0 -> +0.0, the same value).  H = 32
// keeps fmaxf: there the integer form scheduled into 16 more VGPRs (one wave
// of occupancy).
template <int H>
PGP_DEV float relu_enc(float x) {
  if constexpr (Geo<H>::P8 || Geo<H>::TAIL)
    return __int_as_float(max(__float_as_int(x), 0));
  else
    return fmaxf(x, 0.f);
}

// MFMA phases run at wave priority 1, VALU phases (softmax, LayerNorm) at 0: the
// co-resident wave of the other workgroup on the SIMD then gets its MFMA issue
// slots ahead of a VALU stream
PGP_DEV void prio_mfma() { __builtin_amdgcn_s_setprio(1); }
PGP_DEV void prio_valu() { __builtin_amdgcn_s_setprio(0); }

// acc[m][w] += A[m] . B for the first NM of NMA accumulator tiles, A = NM tiles
// x KQ groups in LDS, B k-step s = Bx[s/4][w][s%4]
template <int NM, int KQ, int KS, int NB, int NMA = NM>
PGP_DEV void gemm3(f32x4 (&acc)[NMA][3], const float* A, const f32x4 (&Bx)[NB][3], int lane) {
  static_assert(NM <= NMA, "accumulator tiles");
  prio_mfma();
#pragma unroll
  for (int m = 0; m < NM; ++m)
#pragma unroll
    for (int q4 = 0; q4 < KQ; ++q4) {
      const f32x4 a = ld4(A + (m * KQ + q4) * 256 + lane * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * q4 + e < KS) {
#pragma unroll
          for (int w = 0; w < 3; ++w) acc[m][w] = mfma(a[e], Bx[q4][w][e], acc[m][w]);
        }
    }
  prio_valu();
}

// gemm3 with NR VALU rows folded into the first tile's pass: the rows' FMAs
// (same B operands, k-step by k-step) sit between that pass's MFMAs, where
// they issue in the matrix pipe's shadow.  racc must start at zero; the
// cross-group sum is done by rows_finish.
template <int NM, int KQ, int KS, int NB, int NMA, int NR>
PGP_DEV void gemm3_rows(f32x4 (&acc)[NMA][3], const float* A, const f32x4 (&Bx)[NB][3], int lane,
                        float (&racc)[NR][3], const float* RW, int g) {
  static_assert(NM <= NMA, "accumulator tiles");
  prio_mfma();
  // (kEncPipeF32) each A fragment read one (tile, group) ahead of its 12 MFMAs
  f32x4 an = ld4(A + lane * 4);
#pragma unroll
  for (int m = 0; m < NM; ++m)
#pragma unroll
    for (int q4 = 0; q4 < KQ; ++q4) {
      f32x4 a;
      if constexpr (kEncPipeF32) {
        a = an;
        if (m * KQ + q4 + 1 < NM * KQ) an = ld4(A + (m * KQ + q4 + 1) * 256 + lane * 4);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        a = ld4(A + (m * KQ + q4) * 256 + lane * 4);
      }
      f32x4 rw[NR];
      if (m == 0) {
#pragma unroll
        for (int n = 0; n < NR; ++n) rw[n] = ld4(RW + ((n * KQ + q4) * 4 + g) * 4);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * q4 + e < KS) {
#pragma unroll
          for (int w = 0; w < 3; ++w) {
            acc[m][w] = mfma(a[e], Bx[q4][w][e], acc[m][w]);
            if (m == 0) {
#pragma unroll
              for (int n = 0; n < NR; ++n) racc[n][w] = fmaf(rw[n][e], Bx[q4][w][e], racc[n][w]);
            }
          }
        }
    }
  prio_valu();
}

// cross-group sums of all NR x 3 row partials (broadcast), two at a time
template <int NR>
PGP_DEV void rows_finish(float (&r)[NR][3]) {
  float* f = &r[0][0];
#pragma unroll
  for (int i = 0; i + 1 < 3 * NR; i += 2) xsum2(f[i], f[i + 1]);
  if constexpr ((3 * NR) % 2) f[3 * NR - 1] = xsum(f[3 * NR - 1], true);
}

// per-group row sums: lane group n gets the sum of row n for step w (0 in
// groups >= NR): the B-operand slot of d-rows 16*MT_X + n (X tile MT_X,
// register 0) in one transposed reduction
template <int NR>
PGP_DEV float rows_pick(const float (&r)[NR][3], int w) {
  float v[NR];
#pragma unroll
  for (int n = 0; n < NR; ++n) v[n] = r[n][w];
  return xsum_rows<NR>(v);
}

template <int NR>
PGP_DEV void zero_rows(float (&r)[NR][3]) {
#pragma unroll
  for (int n = 0; n < NR; ++n)
#pragma unroll
    for (int w = 0; w < 3; ++w) r[n][w] = 0.f;
}

// AFFINE = false (norm1): X = x-hat; gamma / beta are folded into linear1 and
// linear2's bias by the packer, and the residual is formed as x-hat*gamma + b2'
template <int H, bool AFFINE = true>
PGP_DEV void layer_norm_tiles(f32x4 (&acc)[Geo<H>::MT_D][3], f32x4 (&X)[Geo<H>::MT_D][3], const float* gam,
                              const float* bet, int g) {
  using G = Geo<H>;
  constexpr float invH = 1.0f / (float)H;
  // one pass: sum and sum of squares of each step reduced together (xsum2).
  // Padded feature rows hold exact zeros here, so no mask is needed.
  // var = E[x^2] - mean^2 (LN inputs are a residual stream whose mean is O(std))
  float sum[3], mean[3], var[3];
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    sum[w] = 0.f;
    float sq = 0.f;
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt) {
      sum[w] += (acc[mt][w][0] + acc[mt][w][1]) + (acc[mt][w][2] + acc[mt][w][3]);
#pragma unroll
      for (int r = 0; r < 4; ++r) sq = fmaf(acc[mt][w][r], acc[mt][w][r], sq);
    }
    xsum2(sum[w], sq);
    mean[w] = sum[w] * invH;
    var[w] = fmaxf(fmaf(-mean[w], mean[w], sq * invH), 0.f);  // the variance itself
  }
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float rstd = __builtin_amdgcn_rsqf(var[w] + 1e-5f);  // v_rsq_f32 (1 ulp)
    // (x - mean) * rstd as one fma per element: x * rstd + (-mean * rstd)
    const float nm = -mean[w] * rstd;
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt) {
      f32x4 xn;
#pragma unroll
      for (int r = 0; r < 4; ++r) xn[r] = fmaf(acc[mt][w][r], rstd, nm);
      if constexpr (AFFINE) {
        const f32x4 ga = ld4(gam + 16 * mt + 4 * g), be = ld4(bet + 16 * mt + 4 * g);
        X[mt][w] = xn * ga + be;
      } else {
        X[mt][w] = xn;
      }
    }
  }
}

// Ring state: `cur` holds the stage being computed, `nxt` is being filled.
// Resident mode: `nxt` is the LDS copy of the whole stream and advance() only
// moves `cur` to the next stage.
template <int H, bool SPLIT = false>
struct Ring {
  using G = Geo<H>;
  static constexpr bool RES = EncLds<H, SPLIT>::RESIDENT;
  float* cur;
  float* nxt;
  const float* enc;  // global encoder stream [layer][LAYER_G groups]
  int next;          // global index of the stage being filled into nxt
  int last;          // number of stages in the launch
  int wv, lane;
  PGP_DEV void issue() {
    if constexpr (RES) return;
    if (next < last) {
      const int si = next % (kLayers * G::NST), l = si / G::NST, k = si % G::NST;
      dma_groups(enc + (long)(l * G::LAYER_G + G::st_begin(k)) * G::FQ, nxt, G::st_end(k) - G::st_begin(k), wv,
                 enc_waves<H>(), lane);
    }
  }
  PGP_DEV void advance() {
    if constexpr (RES) {
      const int si = next % (kLayers * G::NST), l = si / G::NST, k = si % G::NST;
      int gi;
      if constexpr (SPLIT)  // the split image (EncS); layer 0's stages 0, 1 are never read
        gi = l == 0 ? EncS<H>::L0F : k == 2 ? EncS<H>::L1F : EncS<H>::L1A + G::st_begin(k);
      else
        gi = l * G::LAYER_G + G::st_begin(k) - EncLds<H>::RES0;  // < 0: a stage tail mode never reads
      cur = nxt + (gi > 0 ? gi : 0) * G::FQ;
      ++next;
      __builtin_amdgcn_sched_barrier(0);  // keep stages apart (no hoisting of later stages' LDS reads)
      return;
    }
    __syncthreads();  // drains this wave's DMAs (vmcnt(0)) and orders all waves
    float* t = cur;
    cur = nxt;
    nxt = t;
    ++next;
    issue();
  }
};

// Scores over the 3 window steps for the head(s) of one pass; q is pre-scaled.
template <int H>
PGP_DEV void attention(const f32x4 (&QKV)[3 * Geo<H>::TP][3], f32x4 (&O)[Geo<H>::TP][3]) {
  using G = Geo<H>;
  float pr[3][3];
  // P8: lane groups {0,1} = head 0, {2,3} = head 1 (half sums), reduced in
  // pairs; otherwise one at a time (pairs cost H = 32 a wave of occupancy)
  float sc9[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int w = i / 3, w2 = i % 3;
    float part = 0.f;
#pragma unroll
    for (int tp = 0; tp < G::TP; ++tp)
#pragma unroll
      for (int r = 0; r < 4; ++r) part += QKV[tp][w][r] * QKV[G::TP + tp][w2][r];
    if constexpr (G::P8)
      sc9[i] = part;
    else
      sc9[i] = xsum(part, true);
  }
  if constexpr (G::P8) {
#pragma unroll
    for (int i = 0; i < 8; i += 2) xsum2_half(sc9[i], sc9[i + 1]);
    sc9[8] = xsum(sc9[8], false);
  }
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float* sc = sc9 + 3 * w;
    const float m = fmaxf(sc[0], fmaxf(sc[1], sc[2]));
    const float e0 = __expf(sc[0] - m), e1 = __expf(sc[1] - m), e2 = __expf(sc[2] - m);  // v_exp_f32
    const float inv = __builtin_amdgcn_rcpf(e0 + e1 + e2);
    pr[w][0] = e0 * inv;
    pr[w][1] = e1 * inv;
    pr[w][2] = e2 * inv;
  }
#pragma unroll
  for (int tp = 0; tp < G::TP; ++tp)
#pragma unroll
    for (int w = 0; w < 3; ++w)
      O[tp][w] = pr[w][0] * QKV[2 * G::TP + tp][0] + pr[w][1] * QKV[2 * G::TP + tp][1] +
                 pr[w][2] * QKV[2 * G::TP + tp][2];
}

template <int H>
PGP_DEV void qkv_gemm(f32x4 (&QKV)[3 * Geo<H>::TP][3], const float* A, const float* tabqkv,
                      const f32x4 (&X)[Geo<H>::MT_D][3], int lane, int g) {
  using G = Geo<H>;
#pragma unroll
  for (int m = 0; m < 3 * G::TP; ++m) {
    const f32x4 bias = ld4(tabqkv + m * 16 + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) QKV[m][w] = bias;
  }
  gemm3<3 * G::TP, G::KQ_D, G::KS_D, G::MT_D>(QKV, A, X, lane);
}

// Layer 0's q/k/v tiles [T0, T0 + n) from the aggregated raw features: X0 is
// affine in them, so each tile is ONE K=4 MFMA (raw feature k = lane group,
// ba[w] zero in group 3) onto its per-step bias (pgp_pack.cpp, T_F0*).
template <int H, int NM>
PGP_DEV void qkv_fold(f32x4 (&acc)[NM][3], int T0, int n, const float* tab, const float (&ba)[3], int lane, int g) {
  using G = Geo<H>;
#pragma unroll
  for (int m = 0; m < NM; ++m)
    if (m < n) {
      const float a = tab[G::T_F0 + (T0 + m) * 64 + lane];
#pragma unroll
      for (int w = 0; w < 3; ++w)
        acc[m][w] = mfma(a, ba[w], ld4(tab + G::T_F0B + (w * 3 * G::NQT + T0 + m) * 16 + 4 * g));
    }
}
// tail-mode VALU rows of layer 0 (q/k/v m, head-1 tail row n), without bias:
// this lane group's term (the caller sums over groups)
template <int H>
PGP_DEV float row_fold_part(int m, int n, int w, const float* tab, const float (&ba)[3], int g) {
  using G = Geo<H>;
  const float t = tab[G::T_F0R + (m * G::SR + n) * 4 + g];  // slot 3 exists ([.][4] rows)
  return (g < 3 ? t : 0.f) * ba[w];
}
template <int H>
PGP_DEV float row_fold_bias(int m, int n, int w, const float* tab) {
  using G = Geo<H>;
  return tab[G::T_F0RB + w * 3 * G::SR + m * G::SR + n];
}

// Tail-mode layer (Geo<H>::TAIL, H = 50): stages [qk] [v o] [f1 f2].
// F0: layer 0, q/k/v from the folded raw-feature product (the ring's q/k/v
// stages are then unused).
template <int H, bool F0, bool SPLIT>
PGP_DEV void encoder_layer_tail(f32x4 (&X)[Geo<H>::MT_D][3], Ring<H, SPLIT>& ring, const float* TL, int lane,
                                const float* tab, const float (&ba)[3], const float (&xv)[3][3]) {
  using G = Geo<H>;
  constexpr int TQ = G::TQ, SR = G::SR, HF = G::HF;
  const int g = lane >> 4;
  // [S0] q and k of both heads
  constexpr bool BIL = F0;  // layer 0's scores as bilinear forms (the q / k fold is not needed)
  f32x4 QK[BIL ? 1 : 2 * TQ][3];
  float qr[SR][3], kr[SR][3];
  if constexpr (BIL) {
  } else {
#pragma unroll
    for (int m = 0; m < 2 * TQ; ++m) {
      const f32x4 bias = ld4(TL + G::TL_QKV + m * 16 + 4 * g);
#pragma unroll
      for (int w = 0; w < 3; ++w) QK[m][w] = bias;
    }
    float qkr[2 * SR][3];
    zero_rows(qkr);
    gemm3_rows<2 * TQ, G::KQ_D, G::KS_D, G::MT_D, 2 * TQ, 2 * SR>(QK, ring.cur, X, lane, qkr, TL + G::TL_RQ, g);
    rows_finish(qkr);
#pragma unroll
    for (int n = 0; n < SR; ++n)
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        qr[n][w] = qkr[n][w] + TL[G::TL_RQB + n];
        kr[n][w] = qkr[SR + n][w] + TL[G::TL_RQB + SR + n];
      }
  }
  ring.advance();
  // scores of both heads; the shared tile's slot 4r+g belongs to head 0 below HT
  float P0[3][3], P1[3][3];
  if constexpr (BIL) {
    // score(w, w2) = x_w^T M x_w2 + x_w . U[:, w2] + V[w] . x_w2 + S[w][w2]
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const float* SB = tab + G::T_F0S + hh * 36;
      float tk[3][3], vk[3][3];  // [key step][f]: M x_w2 + U[:, w2];  [query][key]: V[w] . x_w2
#pragma unroll
      for (int w2 = 0; w2 < 3; ++w2) {
#pragma unroll
        for (int f = 0; f < 3; ++f)
          tk[w2][f] = fmaf(SB[3 * f + 2], xv[w2][2], fmaf(SB[3 * f + 1], xv[w2][1], fmaf(SB[3 * f], xv[w2][0], SB[9 + 3 * f + w2])));
#pragma unroll
        for (int w = 0; w < 3; ++w)
          vk[w][w2] = fmaf(SB[18 + 3 * w + 2], xv[w2][2], fmaf(SB[18 + 3 * w + 1], xv[w2][1], fmaf(SB[18 + 3 * w], xv[w2][0], SB[27 + 3 * w + w2])));
      }
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        float s[3];
#pragma unroll
        for (int w2 = 0; w2 < 3; ++w2)
          s[w2] = fmaf(xv[w][2], tk[w2][2], fmaf(xv[w][1], tk[w2][1], fmaf(xv[w][0], tk[w2][0], vk[w][w2])));
        const float m = fmaxf(s[0], fmaxf(s[1], s[2]));
        const float e0 = __expf(s[0] - m), e1 = __expf(s[1] - m), e2 = __expf(s[2] - m);
        const float iv = __builtin_amdgcn_rcpf(e0 + e1 + e2);
        float(&Pw)[3][3] = hh == 0 ? P0 : P1;
        Pw[w][0] = e0 * iv;
        Pw[w][1] = e1 * iv;
        Pw[w][2] = e2 * iv;
      }
    }
  } else
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    float s0[3], s1[3];
#pragma unroll
    for (int w2 = 0; w2 < 3; ++w2) {
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int t = 0; t < HF; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a0 = fmaf(QK[t][w][r], QK[TQ + t][w2][r], a0);
          a1 = fmaf(QK[HF + t][w][r], QK[TQ + HF + t][w2][r], a1);
        }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pr = QK[2 * HF][w][r] * QK[TQ + 2 * HF][w2][r];
        if (4 * r + g < G::HT)
          a0 += pr;
        else
          a1 += pr;
      }
      xsum2(a0, a1);
      s0[w2] = a0;
      float t1 = a1;
#pragma unroll
      for (int n = 0; n < SR; ++n) t1 = fmaf(qr[n][w], kr[n][w2], t1);
      s1[w2] = t1;
    }
    const float m0 = fmaxf(s0[0], fmaxf(s0[1], s0[2])), m1 = fmaxf(s1[0], fmaxf(s1[1], s1[2]));
    // hardware exp2 / rcp (a few ulp; logits are compared at rtol 1e-4): the softmax is the
    // VALU-heaviest phase beside the MFMAs at 2 waves per SIMD
    const float e00 = __expf(s0[0] - m0), e01 = __expf(s0[1] - m0), e02 = __expf(s0[2] - m0);
    const float e10 = __expf(s1[0] - m1), e11 = __expf(s1[1] - m1), e12 = __expf(s1[2] - m1);
    const float i0 = __builtin_amdgcn_rcpf(e00 + e01 + e02), i1 = __builtin_amdgcn_rcpf(e10 + e11 + e12);
    P0[w][0] = e00 * i0;
    P0[w][1] = e01 * i0;
    P0[w][2] = e02 * i0;
    P1[w][0] = e10 * i1;
    P1[w][1] = e11 * i1;
    P1[w][2] = e12 * i1;
  }
  f32x4 acc[G::MT_D][3];
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt) {
    const f32x4 bo = ld4(TL + G::TL_BO + 16 * mt + 4 * g);
    if constexpr (F0) {
#pragma unroll
      for (int w = 0; w < 3; ++w) acc[mt][w] = bo + X[mt][w];
    } else {  // X = layer 0's norm2 x-hat: residual gamma0 * x-hat + (bo + beta0) (packer)
      const f32x4 g0 = ld4(TL - G::TL_SIZE + G::TL_LN2G + 16 * mt + 4 * g);
#pragma unroll
      for (int w = 0; w < 3; ++w) acc[mt][w] = X[mt][w] * g0 + bo;
    }
  }
  if constexpr (F0) {
    // [S1] layer 0: out_proj through the attention, folded (no v, no P.v):
    // B operands per window, raw-feature / key-step slot g < 3:
    //   y_hh[w] = sum_w' P_hh[w][w'] agg_w'[g],  p_hh[w] = P_hh[w][g]
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const float y0 = P0[w][0] * ba[0] + P0[w][1] * ba[1] + P0[w][2] * ba[2];
      const float y1 = P1[w][0] * ba[0] + P1[w][1] * ba[1] + P1[w][2] * ba[2];
      const float p0 = g == 0 ? P0[w][0] : g == 1 ? P0[w][1] : g == 2 ? P0[w][2] : 0.f;
      const float p1 = g == 0 ? P1[w][0] : g == 1 ? P1[w][1] : g == 2 ? P1[w][2] : 0.f;
      const float bops[4] = {y0, p0, y1, p1};
#pragma unroll
      for (int k = 0; k < 4; ++k)  // tiles alternate: no dependent-accumulator issue stall
#pragma unroll
        for (int mt = 0; mt < G::MT_X; ++mt)
          acc[mt][w] = mfma(tab[G::T_F0O + (k * G::MT_X + mt) * 64 + lane], bops[k], acc[mt][w]);
      float ro[G::XR];
#pragma unroll
      for (int n = 0; n < G::XR; ++n) {
        const float* rw = tab + G::T_F0OR + n * 16;
        ro[n] = g < 3 ? rw[g] * y0 + rw[4 + g] * p0 + rw[8 + g] * y1 + rw[12 + g] * p1 : 0.f;
      }
      acc[G::MT_X][w][0] += xsum_rows<G::XR>(ro);  // row n's sum in lane group n
    }
    layer_norm_tiles<H, false>(acc, X, TL + G::TL_LN1G, TL + G::TL_LN1B, g);
  } else {
  // [S1] v, P.v, out_proj (+ residual), norm1
  f32x4 V[TQ][3];
  float vr[SR][3];  // VALU v rows including their bias
#pragma unroll
  for (int t = 0; t < TQ; ++t) {
    const f32x4 bias = ld4(TL + G::TL_QKV + (2 * TQ + t) * 16 + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) V[t][w] = bias;
  }
  zero_rows(vr);
  gemm3_rows<TQ, G::KQ_D, G::KS_D, G::MT_D, TQ, SR>(V, ring.cur, X, lane, vr, TL + G::TL_RQ + 2 * SR * G::KQ_D * 16,
                                                         g);
  // v row n (+ its bias) in lane group n, 0 in groups >= SR (the bias table is
  // padded to 8 entries, so slot 2*SR + g is in bounds)
  float vd[3];
  {
    const float vb = TL[G::TL_RQB + 2 * SR + g];
#pragma unroll
    for (int w = 0; w < 3; ++w) vd[w] = rows_pick<SR>(vr, w) + (g < SR ? vb : 0.f);
  }
  f32x4 O[TQ + 1][3];
#pragma unroll
  for (int w = 0; w < 3; ++w) {
#pragma unroll
    for (int t = 0; t < 2 * HF; ++t) {
      const float(&Pw)[3][3] = t < HF ? P0 : P1;
      O[t][w] = Pw[w][0] * V[t][0] + Pw[w][1] * V[t][1] + Pw[w][2] * V[t][2];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool h0 = 4 * r + g < G::HT;
      const float c0 = h0 ? P0[w][0] : P1[w][0], c1 = h0 ? P0[w][1] : P1[w][1], c2 = h0 ? P0[w][2] : P1[w][2];
      O[2 * HF][w][r] = c0 * V[2 * HF][0][r] + c1 * V[2 * HF][1][r] + c2 * V[2 * HF][2][r];
    }
    const float o3 = P1[w][0] * vd[0] + P1[w][1] * vd[1] + P1[w][2] * vd[2];  // 0 in groups >= SR
    O[TQ][w] = f32x4{o3, 0.f, 0.f, 0.f};
  }
  {
    float ro[G::XR][3];
    zero_rows(ro);
    gemm3_rows<G::MT_X, G::KQ_OT, G::KS_OT, TQ + 1, G::MT_D, G::XR>(acc, ring.cur + G::G_V * G::FQ, O, lane, ro,
                                                                   TL + G::TL_RO, g);
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[G::MT_X][w][0] += rows_pick<G::XR>(ro, w);
  }
  layer_norm_tiles<H, false>(acc, X, TL + G::TL_LN1G, TL + G::TL_LN1B, g);
  }  // F0
  ring.advance();
  // [S2] relu(W1 x + b1), W2 . h + b2 + x, norm2
  // hidden tile by hidden tile: tile c of relu(W1 x + b1) is k-group c of the
  // W2 contraction, consumed as soon as it is formed (12 hidden-state VGPRs
  // live instead of 48; same accumulation order as the unchunked form)
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt) {
    const f32x4 b2 = ld4(TL + G::TL_B2 + 16 * mt + 4 * g), g1 = ld4(TL + G::TL_LN1G + 16 * mt + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[mt][w] = X[mt][w] * g1 + b2;  // residual gamma*x-hat + beta, + b2
  }
  if constexpr (SPLIT) {
    // step by step: X's two 32-k blocks split (24 VGPRs), the four hidden tiles
    // (4 independent MFMA chains), ReLU, the hidden pairs split, linear2 onto
    // the residual accumulators; linear2's XR VALU rows as in the fp32 form
    using S = EncS<H>;
    static_assert(S::NBF * 2 == G::MT_F, "hidden pairs");
    const float* A1 = ring.cur;
    const float* A2 = ring.cur + S::F1S * G::FQ;
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      f32x4 F[G::MT_F];
#pragma unroll
      for (int c = 0; c < G::MT_F; ++c) F[c] = ld4(TL + G::TL_B1 + 16 * c + 4 * g);
      if constexpr (kEncPipe) {
        // block by block (one block's split X, 12 VGPRs, live at a time), the
        // next (block, tile)'s planes read ahead of this one's MFMAs and pinned
        // there (160 of the kernel's LDS reads were waited for right after
        // issue); each F[c] takes its blocks in the same order as below
        constexpr int QN = S::NBD * G::MT_F;
        u32x4 wn[3];
        planes_lds(A1, lane, wn);
#pragma unroll
        for (int b = 0; b < S::NBD; ++b) {
          u32x4 xb[3];
          {
            float v[8];
            pair_tiles<G::MT_D>(X, b, w, v);
            split8(v, xb);
          }
          prio_mfma();
#pragma unroll
          for (int c = 0; c < G::MT_F; ++c) {
            u32x4 wp[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) wp[k] = wn[k];
            const int q = b * G::MT_F + c + 1;
            if (q < QN) planes_lds(A1 + (((q % G::MT_F) * S::NBD + q / G::MT_F) * 3) * 256, lane, wn);
            __builtin_amdgcn_sched_barrier(0);
            F[c] = mfma_bf6(wp, xb, F[c]);
          }
          prio_valu();
        }
      } else {
        u32x4 xs[S::NBD][3];
#pragma unroll
        for (int b = 0; b < S::NBD; ++b) {
          float v[8];
          pair_tiles<G::MT_D>(X, b, w, v);
          split8(v, xs[b]);
        }
        prio_mfma();
#pragma unroll
        for (int b = 0; b < S::NBD; ++b)
#pragma unroll
          for (int c = 0; c < G::MT_F; ++c) {
            u32x4 wp[3];
            planes_lds(A1 + ((c * S::NBD + b) * 3) * 256, lane, wp);
            F[c] = mfma_bf6(wp, xs[b], F[c]);
          }
        prio_valu();
      }
#pragma unroll
      for (int c = 0; c < G::MT_F; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) F[c][r] = relu_enc<H>(F[c][r]);
      float rf[G::XR];
#pragma unroll
      for (int n = 0; n < G::XR; ++n) rf[n] = 0.f;
#pragma unroll
      for (int c = 0; c < G::MT_F; ++c)
#pragma unroll
        for (int n = 0; n < G::XR; ++n) {
          const f32x4 rw = ld4(TL + G::TL_RF + ((n * G::KQ_F + c) * 4 + g) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) rf[n] = fmaf(rw[e], F[c][e], rf[n]);
        }
      if constexpr (kEncPipe) {
        constexpr int QN = S::NBF * G::MT_X;
        u32x4 wn[3];
        planes_lds(A2, lane, wn);
#pragma unroll
        for (int b = 0; b < S::NBF; ++b) {
          u32x4 hb[3];
          {
            float v[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = F[2 * b][e];
              v[4 + e] = F[2 * b + 1][e];
            }
            split8(v, hb);
          }
          prio_mfma();
#pragma unroll
          for (int m = 0; m < G::MT_X; ++m) {
            u32x4 wp[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) wp[k] = wn[k];
            const int q = b * G::MT_X + m + 1;
            if (q < QN) planes_lds(A2 + (((q % G::MT_X) * S::NBF + q / G::MT_X) * 3) * 256, lane, wn);
            __builtin_amdgcn_sched_barrier(0);
            acc[m][w] = mfma_bf6(wp, hb, acc[m][w]);
          }
          prio_valu();
        }
      } else {
        u32x4 hs[S::NBF][3];
#pragma unroll
        for (int b = 0; b < S::NBF; ++b) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = F[2 * b][e];
            v[4 + e] = F[2 * b + 1][e];
          }
          split8(v, hs[b]);
        }
        prio_mfma();
#pragma unroll
        for (int b = 0; b < S::NBF; ++b)
#pragma unroll
          for (int m = 0; m < G::MT_X; ++m) {
            u32x4 wp[3];
            planes_lds(A2 + ((m * S::NBF + b) * 3) * 256, lane, wp);
            acc[m][w] = mfma_bf6(wp, hs[b], acc[m][w]);
          }
        prio_valu();
      }
      acc[G::MT_X][w][0] += xsum_rows<G::XR>(rf);  // row n's sum in lane group n
    }
  } else {
    static_assert(G::KQ_F == G::MT_F, "hidden tile c = W2 k-group c");
    float rf[G::XR][3];
    zero_rows(rf);
#pragma unroll
    for (int c = 0; c < G::MT_F; ++c) {
      f32x4 Fc[1][3];
      const f32x4 b1 = ld4(TL + G::TL_B1 + 16 * c + 4 * g);
#pragma unroll
      for (int w = 0; w < 3; ++w) Fc[0][w] = b1;
      gemm3<1, G::KQ_D, G::KS_D, G::MT_D>(Fc, ring.cur + c * G::KQ_D * 256, X, lane);
#pragma unroll
      for (int w = 0; w < 3; ++w)
#pragma unroll
        for (int r = 0; r < 4; ++r) Fc[0][w][r] = relu_enc<H>(Fc[0][w][r]);
      const float* A2 = ring.cur + G::G_F1 * G::FQ;
      prio_mfma();
#pragma unroll
      for (int m = 0; m < G::MT_X; ++m) {
        const f32x4 a = ld4(A2 + (m * G::KQ_F + c) * 256 + lane * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int w = 0; w < 3; ++w) acc[m][w] = mfma(a[e], Fc[0][w][e], acc[m][w]);
      }
      prio_valu();
#pragma unroll
      for (int n = 0; n < G::XR; ++n) {
        const f32x4 rw = ld4(TL + G::TL_RF + ((n * G::KQ_F + c) * 4 + g) * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int w = 0; w < 3; ++w) rf[n][w] = fmaf(rw[e], Fc[0][w][e], rf[n][w]);
      }
    }
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[G::MT_X][w][0] += rows_pick<G::XR>(rf, w);
  }
  ring.advance();
  // both norm2s emit x-hat: layer 0's gamma / beta are folded into layer 1's
  // in_proj and residual, the last layer's into the decoders (which are linear
  // in the latent), by the packer
  layer_norm_tiles<H, false>(acc, X, TL + G::TL_LN2G, TL + G::TL_LN2B, g);
}

// One encoder layer; weights arrive stage by stage through the ring.  F0:
// layer 0, q/k/v from the folded raw-feature product.
template <int H, bool F0>
PGP_DEV void encoder_layer(f32x4 (&X)[Geo<H>::MT_D][3], Ring<H>& ring, const float* TL, int lane,
                           const float* tab, const float (&ba)[3]) {
  using G = Geo<H>;
  const int g = lane >> 4;
  f32x4 acc[G::MT_D][3];
  f32x4 QKV[3 * G::TP][3];
  f32x4 O[G::TP][3];
  // [S0] qkv pass 0
  if constexpr (F0)
    qkv_fold<H, 3 * G::TP>(QKV, 0, 3 * G::TP, tab, ba, lane, g);
  else
    qkv_gemm<H>(QKV, ring.cur, TL + G::TL_QKV, X, lane, g);
  ring.advance();
  attention<H>(QKV, O);
  // [S1] out_proj pass 0 (+ qkv pass 1)
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt) {
    const f32x4 bo = ld4(TL + G::TL_BO + 16 * mt + 4 * g);
    if constexpr (F0) {
#pragma unroll
      for (int w = 0; w < 3; ++w) acc[mt][w] = bo + X[mt][w];  // residual folded into the accumulator
    } else {  // X = layer 0's norm2 x-hat: residual gamma0 * x-hat + (bo + beta0) (packer)
      const f32x4 g0 = ld4(TL - G::TL_SIZE + G::TL_LN2G + 16 * mt + 4 * g);
#pragma unroll
      for (int w = 0; w < 3; ++w) acc[mt][w] = X[mt][w] * g0 + bo;
    }
  }
  gemm3<G::MT_D, G::KQ_O, G::KS_O, G::TP>(acc, ring.cur, O, lane);
  if constexpr (G::NPASS == 2) {
    if constexpr (F0)
      qkv_fold<H, 3 * G::TP>(QKV, 3 * G::TP, 3 * G::TP, tab, ba, lane, g);
    else
      qkv_gemm<H>(QKV, ring.cur + G::G_O * G::FQ, TL + G::TL_QKV + 3 * G::TP * 16, X, lane, g);
    ring.advance();
    attention<H>(QKV, O);
    // [S2] out_proj pass 1 (+ f1)
    gemm3<G::MT_D, G::KQ_O, G::KS_O, G::TP>(acc, ring.cur, O, lane);
  }
  // x = norm1(x + sa)
  layer_norm_tiles<H, false>(acc, X, TL + G::TL_LN1G, TL + G::TL_LN1B, g);
  // feed-forward: relu(W1 x + b1) in the same stage as the last out_proj
  f32x4 F1[G::MT_F][3];
#pragma unroll
  for (int mt = 0; mt < G::MT_F; ++mt) {
    const f32x4 b1 = ld4(TL + G::TL_B1 + 16 * mt + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) F1[mt][w] = b1;
  }
  gemm3<G::MT_F, G::KQ_D, G::KS_D, G::MT_D>(F1, ring.cur + G::G_O * G::FQ, X, lane);
#pragma unroll
  for (int mt = 0; mt < G::MT_F; ++mt)
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int r = 0; r < 4; ++r) F1[mt][w][r] = relu_enc<H>(F1[mt][w][r]);
  ring.advance();
  // [S3] W2 . h + b2 + x, norm2
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt) {
    const f32x4 b2 = ld4(TL + G::TL_B2 + 16 * mt + 4 * g), g1 = ld4(TL + G::TL_LN1G + 16 * mt + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[mt][w] = X[mt][w] * g1 + b2;  // residual gamma*x-hat + beta, + b2
  }
  gemm3<G::MT_D, G::KQ_F, 16, G::MT_F>(acc, ring.cur, F1, lane);
  ring.advance();
  layer_norm_tiles<H, false>(acc, X, TL + G::TL_LN2G, TL + G::TL_LN2B, g);  // x-hat: both affines folded (see tail)
}

template <int H, bool SPLIT>
__global__ __launch_bounds__(enc_waves<H>() * 64, H <= 16 ? kEnc16EU : tail_res<H>() ? 1 : 2) void encoder_kernel(
    FwdArgs a) {
  using G = Geo<H>;
  using L = EncLds<H, SPLIT>;
  __shared__ __attribute__((aligned(16))) float smem[L::TOTAL];
  // tail-resident mode: per-wave staging slot of the next unit's raw features
  __shared__ float xstage[L::UNITS ? NW_STAGE<H>() * 144 : 1];
  float* tab = smem + (L::RESIDENT ? L::STREAM : 2 * L::SLOT);
  const int tsz = G::t_size(a.K);
  for (int i = threadIdx.x; i < tsz; i += blockDim.x) tab[i] = a.tab[i];

  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int NW = enc_waves<H>();
  const long nblk = (a.B + 15) / 16;

  Ring<H, SPLIT> ring{smem, smem + L::SLOT, a.frags + G::OFF_ENC, 0, H * kLayers * G::NST, wv, lane};
  if constexpr (SPLIT) {
    dma_groups(a.encb, smem, EncS<H>::GROUPS, wv, NW, lane);
    ring.nxt = smem;
    ring.next = 1;
    __syncthreads();
  } else if constexpr (L::RESIDENT) {
    dma_groups(a.frags + G::OFF_ENC + (long)L::RES0 * G::FQ, smem, kLayers * G::LAYER_G - L::RES0, wv, NW, lane);
    ring.nxt = smem;
    ring.next = 1;
    __syncthreads();
  } else {
    ring.nxt = smem;  // prologue: stage 0 -> slot 0
    ring.issue();
    ring.nxt = smem + L::SLOT;
    ring.next = 1;
    __syncthreads();
    ring.issue();  // stage 1 -> slot 1
  }

  // one (16-window block, host) unit: hosts are independent in the encoder
  // one (16-window block, host) unit: hosts are independent in the encoder.
  // tail-resident mode: pre = the unit's 144 raw-feature floats ([step][feature]
  // [window], the agg layout) staged in LDS by the caller; otherwise loaded here
  auto unit = [&](long blk, int h, bool active, const float* pre) {
    const float* agg = a.agg + (active ? blk : 0) * H * 3 * 48;
    float* lat = a.lat + (active ? blk : 0) * G::LAT_BLK;
    float ba[3];
    // all 3 raw features of every step of this lane's window (layer 0's bilinear scores)
    float xv[3][3];
    if constexpr (L::UNITS) {
#pragma unroll
      for (int w = 0; w < 3; ++w) {
#pragma unroll
        for (int f = 0; f < 3; ++f) xv[w][f] = G::TAIL ? pre[w * 48 + 16 * f + j] : 0.f;
        const float v = pre[w * 48 + (lane < 48 ? lane : 47)];
        ba[w] = g < 3 ? v : 0.f;  // feature g of window j
      }
    } else {
#pragma unroll
      for (int w = 0; w < 3; ++w) ba[w] = (active && g < 3) ? agg[(h * 3 + w) * 48 + lane] : 0.f;
#pragma unroll
      for (int w = 0; w < 3; ++w)
#pragma unroll
        for (int f = 0; f < 3; ++f)
          xv[w][f] = (G::TAIL && active) ? agg[(h * 3 + w) * 48 + 16 * f + j] : 0.f;
    }
    f32x4 X[G::MT_D][3];
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt) {
      const float aw = tab[G::T_TEW + mt * 64 + lane];
#pragma unroll
      for (int w = 0; w < 3; ++w) X[mt][w] = mfma(aw, ba[w], ld4(tab + G::T_TE + w * G::DP + 16 * mt + 4 * g));
    }
    static_assert(kLayers == 2, "layer 0 (folded q/k/v) + layer 1");
    if constexpr (G::TAIL) {
      encoder_layer_tail<H, true, SPLIT>(X, ring, tab + G::T_L0, lane, tab, ba, xv);
      encoder_layer_tail<H, false, SPLIT>(X, ring, tab + G::T_L0 + G::TL_SIZE, lane, tab, ba, xv);
    } else if constexpr (!SPLIT) {
      encoder_layer<H, true>(X, ring, tab + G::T_L0, lane, tab, ba);
      encoder_layer<H, false>(X, ring, tab + G::T_L0 + G::TL_SIZE, lane, tab, ba);
    }

    if (active) {
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        // chunk (h, w): full groups of 4 k-steps as one 16-byte store per lane,
        // the remaining k-steps one dword each (pgp_layout.hpp, LAT_FG)
        float* lc = lat + (long)((h * 3 + w) * G::KS_D) * 64;
#pragma unroll
        for (int q = 0; q < G::LAT_FG; ++q) *reinterpret_cast<f32x4*>(lc + q * 256 + lane * 4) = X[q][w];
        if constexpr (G::KS_D % 4 != 0) {
#pragma unroll
          for (int r = 0; r < G::KS_D % 4; ++r) lc[G::LAT_FG * 256 + r * 64 + lane] = X[G::LAT_FG][w][r];
        }
      }
      if (a.latent != nullptr) {
        const long b = blk * 16 + j;
        if (b < a.B) {
#pragma unroll
          for (int w = 0; w < 3; ++w)
#pragma unroll
            for (int mt = 0; mt < G::MT_D; ++mt)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int c = 16 * mt + 4 * r + g;
                const float* TL1 = tab + G::T_L0 + G::TL_SIZE;  // the latent = gamma * x-hat + beta
                if (c < H)
                  a.latent[b * G::LAT + (long)h * 3 * H + w * H + c] =
                      X[mt][w][r] * TL1[G::TL_LN2G + 16 * mt + 4 * g + r] + TL1[G::TL_LN2B + 16 * mt + 4 * g + r];
              }
        }
      }
    }
  };
  if constexpr (L::UNITS) {
    // no barrier in the host loop: each wave takes an equal contiguous range of
    // the nblk x H units (grid = the workgroups that fit at once: CU count x
    // occupancy), so the launch has no partial last round of workgroups
    const long U = nblk * H, NWT = (long)gridDim.x * NW, gw = (long)blockIdx.x * NW + wv;
    const long u1 = (gw + 1) * U / NWT;
    // unit u's raw features are agg[u * 144 ..] (144 floats).  The next unit's
    // are loaded while this one computes and staged through a per-wave LDS slot
    // after this unit's latent stores: no loop-carried registers, so the wait
    // for them is a counted vmcnt in the body (long satisfied) instead of a
    // vmcnt(0) at the loop head that would also wait for the stores.
    float* slot = xstage + wv * 144;
    const long u0 = gw * U / NWT;
    float pf[3];
    auto load_x = [&](long u) {
#pragma unroll
      for (int k = 0; k < 3; ++k) pf[k] = a.agg[u * 144 + (64 * k + lane < 144 ? 64 * k + lane : 143)];
    };
    auto stage_x = [&]() {
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (64 * k + lane < 144) slot[64 * k + lane] = pf[k];
    };
    if (u0 < u1) {
      load_x(u0);
      stage_x();
    }
#pragma unroll 1
    for (long u = u0; u < u1; ++u) {
      load_x(u + 1 < u1 ? u + 1 : u);
      const long blk = u / H;
      unit(blk, (int)(u - blk * H), true, slot);
      stage_x();
    }
  } else {
    const long blk = (long)blockIdx.x * NW + wv;
    const bool active = blk < nblk;  // inactive waves still take part in the ring and barriers
#pragma unroll 1
    for (int h = 0; h < H; ++h) unit(blk, h, active, nullptr);
  }
}

template <int H, bool SPLIT>
hipError_t launch_form(const FwdArgs& a, hipStream_t st) {
  const long nblk = (a.B + 15) / 16;
  constexpr int NW = enc_waves<H>();
  long grid = (nblk + NW - 1) / NW;
  // A workgroup whose waves' registers cannot be co-resident never starts: the
  // round-2 dual-block variant (256 VGPR + 123 AGPR per wave, 8 waves = 2 per
  // SIMD, i.e. 758 of a SIMD's 512 registers) ended in a launch failure.  Check
  // the built kernel's limit against the launch once per H and fail loudly.
  static std::atomic<int> fits{-1};
  if (fits.load(std::memory_order_relaxed) < 0) {
    hipFuncAttributes fa{};
    const bool ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(encoder_kernel<H, SPLIT>)) == hipSuccess &&
                    fa.maxThreadsPerBlock >= NW * 64;
    fits.store(ok ? 1 : 0, std::memory_order_relaxed);
  }
  if (!fits.load(std::memory_order_relaxed)) return hipErrorLaunchOutOfResources;
  if constexpr (EncLds<H>::UNITS) {
    static std::atomic<int> occ_cache{0};  // workgroups resident per CU (registers / LDS), queried once
    int occ = occ_cache.load(std::memory_order_relaxed);
    if (occ <= 0) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, encoder_kernel<H, SPLIT>, NW * 64, 0) != hipSuccess ||
          occ <= 0)
        occ = 1;
      occ_cache.store(occ, std::memory_order_relaxed);
    }
    grid = std::min<long>((long)device_cus() * occ, (nblk * H + NW - 1) / NW);
  }
  encoder_kernel<H, SPLIT><<<(int)grid, NW * 64, 0, st>>>(a);
  return hipGetLastError();
}

template <int H>
hipError_t launch(const FwdArgs& a, hipStream_t st) {
  if constexpr (enc_split<H>())
    if (a.encb != nullptr) return launch_form<H, true>(a, st);
  return launch_form<H, false>(a, st);
}

template <int H>
hipError_t launch_split(const float* frags, float* encb, hipStream_t st) {
  if constexpr (enc_split<H>()) {
    using G = Geo<H>;
    constexpr long n = 2L * (G::MT_F * EncS<H>::NBD + G::MT_X * EncS<H>::NBF) + G::P_F1;
    enc_split_kernel<H><<<(int)((n + 3) / 4), 256, 0, st>>>(frags + G::OFF_ENC, encb);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_encoder(const FwdArgs& a, hipStream_t st) {
  switch (a.H) {
#define CASE(h) \
  case h:       \
    return launch<h>(a, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

long encoder_split_floats(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return enc_split<h>() ? EncS<h>::SIZE : 0;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

hipError_t launch_encoder_split(int H, const float* frags, float* encb, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return launch_split<h>(frags, encb, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
