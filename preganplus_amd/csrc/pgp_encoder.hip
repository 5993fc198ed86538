// pgp_encoder.hip — K2: time encoder + positional encoding + 2 post-norm
// TransformerEncoderLayers (models.py:344-356, 390-396) for all H hosts of 16
// windows per wave.  Output: the encoder activations ("latent",
// models.py:399) as MFMA B-operand tiles for the decoder GEMM (K2b).
//
// Weights stream through a 2-slot LDS ring, shared by the workgroup's 4 waves:
// while the waves compute stage k from one slot, global_load_lds fills the
// other with stage k+1 (the per-host weight stream is identical for every host,
// so it repeats H times per launch and stays L2-resident).  A-operand fragments
// are read with ds_read_b128 (lane-linear, conflict-free).  Two workgroups per
// CU (__launch_bounds__(256, 2)) let one block's VALU phases (softmax, LayerNorm)
// overlap the other's MFMA phases.
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kEncWaves = 4;

template <int H>
struct EncLds {
  static constexpr int SLOT = Geo<H>::SLOT_G * Geo<H>::FQ;  // floats
  static constexpr int TAB = Geo<H>::t_size(kMaxProtos);
  static constexpr int TOTAL = 2 * SLOT + TAB;
};

// acc[m][w] += A[m] . B, A = NM tiles x KQ groups in LDS, B k-step s = Bx[s/4][w][s%4]
template <int NM, int KQ, int KS, int NB>
PGP_DEV void gemm3(f32x4 (&acc)[NM][3], const float* A, const f32x4 (&Bx)[NB][3], int lane) {
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
}

template <int H>
PGP_DEV void layer_norm_tiles(f32x4 (&acc)[Geo<H>::MT_D][3], f32x4 (&X)[Geo<H>::MT_D][3], const float* gam,
                              const float* bet, int g) {
  using G = Geo<H>;
  constexpr float invH = 1.0f / (float)H;
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    float sum = 0.f;
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt) sum += (acc[mt][w][0] + acc[mt][w][1]) + (acc[mt][w][2] + acc[mt][w][3]);
    sum = xsum(sum, true);
    const float mean = sum * invH;
    float var = 0.f;
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dv = (16 * mt + 4 * r + g < H) ? acc[mt][w][r] - mean : 0.f;
        var += dv * dv;
      }
    var = xsum(var, true);
    const float rstd = 1.0f / sqrtf(var * invH + 1e-5f);
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt) {
      const f32x4 ga = ld4(gam + 16 * mt + 4 * g), be = ld4(bet + 16 * mt + 4 * g);
      X[mt][w] = (acc[mt][w] - mean) * rstd * ga + be;
    }
  }
}

// Ring state: `cur` holds the stage being computed, `nxt` is being filled.
template <int H>
struct Ring {
  using G = Geo<H>;
  float* cur;
  float* nxt;
  const float* enc;  // global encoder stream [layer][LAYER_G groups]
  int next;          // global index of the stage being filled into nxt
  int last;          // number of stages in the launch
  int wv, lane;
  PGP_DEV void issue() {
    if (next < last) {
      const int si = next % (kLayers * G::NST), l = si / G::NST, k = si % G::NST;
      dma_groups(enc + (long)(l * G::LAYER_G + G::st_begin(k)) * G::FQ, nxt, G::st_end(k) - G::st_begin(k), wv,
                 kEncWaves, lane);
    }
  }
  PGP_DEV void advance() {
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
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    float sc[3];
#pragma unroll
    for (int w2 = 0; w2 < 3; ++w2) {
      float part = 0.f;
#pragma unroll
      for (int tp = 0; tp < G::TP; ++tp)
#pragma unroll
        for (int r = 0; r < 4; ++r) part += QKV[tp][w][r] * QKV[G::TP + tp][w2][r];
      sc[w2] = xsum(part, !G::P8);  // P8: lane groups {0,1} = head 0, {2,3} = head 1
    }
    const float m = fmaxf(sc[0], fmaxf(sc[1], sc[2]));
    const float e0 = expf(sc[0] - m), e1 = expf(sc[1] - m), e2 = expf(sc[2] - m);
    const float inv = 1.0f / (e0 + e1 + e2);
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

// One encoder layer; weights arrive stage by stage through the ring.
template <int H>
PGP_DEV void encoder_layer(f32x4 (&X)[Geo<H>::MT_D][3], Ring<H>& ring, const float* TL, int lane) {
  using G = Geo<H>;
  const int g = lane >> 4;
  f32x4 acc[G::MT_D][3];
  f32x4 QKV[3 * G::TP][3];
  f32x4 O[G::TP][3];
  // [S0] qkv pass 0
  qkv_gemm<H>(QKV, ring.cur, TL + G::TL_QKV, X, lane, g);
  ring.advance();
  attention<H>(QKV, O);
  // [S1] out_proj pass 0 (+ qkv pass 1)
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt) {
    const f32x4 bo = ld4(TL + G::TL_BO + 16 * mt + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[mt][w] = bo + X[mt][w];  // residual folded into the accumulator
  }
  gemm3<G::MT_D, G::KQ_O, G::KS_O, G::TP>(acc, ring.cur, O, lane);
  if constexpr (G::NPASS == 2) {
    qkv_gemm<H>(QKV, ring.cur + G::G_O * G::FQ, TL + G::TL_QKV + 3 * G::TP * 16, X, lane, g);
    ring.advance();
    attention<H>(QKV, O);
    // [S2] out_proj pass 1 (+ f1)
    gemm3<G::MT_D, G::KQ_O, G::KS_O, G::TP>(acc, ring.cur, O, lane);
  }
  // x = norm1(x + sa)
  layer_norm_tiles<H>(acc, X, TL + G::TL_LN1G, TL + G::TL_LN1B, g);
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
      for (int r = 0; r < 4; ++r) F1[mt][w][r] = fmaxf(F1[mt][w][r], 0.f);
  ring.advance();
  // [S3] W2 . h + b2 + x, norm2
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt) {
    const f32x4 b2 = ld4(TL + G::TL_B2 + 16 * mt + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[mt][w] = b2 + X[mt][w];
  }
  gemm3<G::MT_D, G::KQ_F, 16, G::MT_F>(acc, ring.cur, F1, lane);
  ring.advance();
  layer_norm_tiles<H>(acc, X, TL + G::TL_LN2G, TL + G::TL_LN2B, g);
}

template <int H>
__global__ __launch_bounds__(kEncWaves * 64, 2) void encoder_kernel(FwdArgs a) {
  using G = Geo<H>;
  using L = EncLds<H>;
  __shared__ __attribute__((aligned(16))) float smem[L::TOTAL];
  float* tab = smem + 2 * L::SLOT;
  const int tsz = G::t_size(a.K);
  for (int i = threadIdx.x; i < tsz; i += blockDim.x) tab[i] = a.tab[i];

  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long blk = (long)blockIdx.x * kEncWaves + wv;
  const long nblk = (a.B + 15) / 16;
  const bool active = blk < nblk;  // inactive waves still take part in the ring and barriers

  Ring<H> ring{smem, smem + L::SLOT, a.frags + G::OFF_ENC, 0, H * kLayers * G::NST, wv, lane};
  ring.nxt = smem;  // prologue: stage 0 -> slot 0
  ring.issue();
  ring.nxt = smem + L::SLOT;
  ring.next = 1;
  __syncthreads();
  ring.issue();  // stage 1 -> slot 1

  const float* agg = a.agg + (active ? blk : 0) * H * 3 * 48;
  float* lat = a.lat + (active ? blk : 0) * G::LAT_BLK;
  for (int h = 0; h < H; ++h) {
    float ba[3];
#pragma unroll
    for (int w = 0; w < 3; ++w) ba[w] = (active && g < 3) ? agg[(h * 3 + w) * 48 + lane] : 0.f;
    f32x4 X[G::MT_D][3];
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt) {
      const float aw = tab[G::T_TEW + mt * 64 + lane];
#pragma unroll
      for (int w = 0; w < 3; ++w) X[mt][w] = mfma(aw, ba[w], ld4(tab + G::T_TE + w * G::DP + 16 * mt + 4 * g));
    }
#pragma unroll 1
    for (int l = 0; l < kLayers; ++l) encoder_layer<H>(X, ring, tab + G::T_L0 + l * G::TL_SIZE, lane);

    if (active) {
#pragma unroll
      for (int w = 0; w < 3; ++w)
#pragma unroll
        for (int s = 0; s < G::KS_D; ++s) lat[((h * 3 + w) * G::KS_D + s) * 64 + lane] = X[s / 4][w][s % 4];
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
                if (c < H) a.latent[b * G::LAT + (long)h * 3 * H + w * H + c] = X[mt][w][r];
              }
        }
      }
    }
  }
}

template <int H>
hipError_t launch(const FwdArgs& a, hipStream_t st) {
  const long nblk = (a.B + 15) / 16;
  const int grid = (int)((nblk + kEncWaves - 1) / kEncWaves);
  encoder_kernel<H><<<grid, kEncWaves * 64, 0, st>>>(a);
  return hipGetLastError();
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

}  // namespace pgp
