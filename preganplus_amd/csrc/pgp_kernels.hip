// pgp_kernels.hip — gfx950 kernels of the PreGAN+ decision model + C-ABI.
//
// Three launches per batch:
//   K1 gat_agg_kernel      GAT edge softmax + aggregation      dlutils.py:304-348
//   K2 encdec_kernel       time encoder + PE + 2 encoder layers + both decoders
//                          + detect/embed/classify             models.py:376-416,
//                          PreGANPlus.py:119-131, utils.py:102-109
//   K3 gan_kernel          Gen + Disc forward + decision argmaxes
//                          models.py:118-151, PreGANPlus.py:84-105, Stats.py:162-166
// All matrix products run on v_mfma_f32_16x16x4_f32 (exact fp32 FMA chains);
// "windows on lanes": one wave = 16 windows, features on accumulator rows
// (pgp_layout.hpp).  No bf16 anywhere: the north-star tolerance (rtol 1e-4 on
// logits, bit-exact decisions) rules it out.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/preganplus.h"
#include "pgp_layout.hpp"
#include "pgp_pack.hpp"

using namespace pgp;

typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kMaxProtos = 64;
constexpr int kNWave = 4;  // waves per workgroup (K2, K3)

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ float xsum(float v, bool both) {
  v += __shfl_xor(v, 16);
  if (both) v += __shfl_xor(v, 32);
  return v;
}
__device__ __forceinline__ float lrelu001(float e) { return e > 0.f ? e : 0.01f * e; }

// =============================================================================
// K1: GAT aggregation.  One wave per (window, step); lane = destination host j.
//   s_i = u.x_i, t_j = v.x_j           (attn_fc split, folded through fc)
//   e_ij = leaky_relu_0.01(s_i + t_j)  (dlutils.py:329)
//   a_ij = exp(e_ij - M) / sum_{i,j} exp(e_ij - M)   graph-wise (dlutils.py:335)
//   agg_j = sum_i a_ij x_i             (dlutils.py:338-342, pulled before fc)
// Output layout (B operand of K2's time-encoder MFMA):
//   agg[((blk*H + j)*3 + w)*48 + f*16 + (b&15)]
// =============================================================================
template <int H>
__global__ __launch_bounds__(256) void gat_agg_kernel(int B, const float* __restrict__ win,
                                                      float* __restrict__ agg, GatConst gc) {
  static_assert(H <= 64, "GAT kernel maps hosts to lanes");
  __shared__ f32x4 sx[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long item = (long)blockIdx.x * 4 + wv;
  const bool active = item < (long)B * 3;
  const long b = active ? item / 3 : 0;
  const int w = active ? (int)(item % 3) : 0;
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
  const float M = lrelu001(smax + tmax);  // = max_ij e_ij (lrelu and rounding monotone)
  sx[wv][lane] = f32x4{s, x0, x1, x2};
  __syncthreads();
  float S = 0.f, a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll 5
  for (int i = 0; i < H; ++i) {
    const f32x4 v = sx[wv][i];
    const float p = expf(lrelu001(v.x + t) - M);
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
    float* o = agg + (((b >> 4) * H + lane) * 3 + w) * 48 + (b & 15);
    o[0] = a0 * inv;
    o[16] = a1 * inv;
    o[32] = a2 * inv;
  }
}

// =============================================================================
// K2 helpers: one TransformerEncoderLayer (post-norm, ReLU, eval) for the 3
// tokens (window steps) of 16 windows at one host.  X[mt][w]: d-space tiles.
// =============================================================================
template <int H>
__device__ __forceinline__ void layer_norm_tiles(f32x4 (&acc)[Geo<H>::MT_D][3], f32x4 (&X)[Geo<H>::MT_D][3],
                                                 const float* gam, const float* bet, int g) {
  using G = Geo<H>;
  constexpr float invH = 1.0f / (float)H;
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    float sum = 0.f;
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt) sum += acc[mt][w][0] + acc[mt][w][1] + acc[mt][w][2] + acc[mt][w][3];
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

template <int H>
__device__ __forceinline__ void encoder_layer(f32x4 (&X)[Geo<H>::MT_D][3], const float* __restrict__ FL,
                                              const float* TL, int lane) {
  using G = Geo<H>;
  const int g = lane >> 4;
  const f32x4* Aqkv = reinterpret_cast<const f32x4*>(FL + G::LO_QKV);
  const f32x4* Ao = reinterpret_cast<const f32x4*>(FL + G::LO_O);
  const f32x4* A1 = reinterpret_cast<const f32x4*>(FL + G::LO_F1);
  const f32x4* A2 = reinterpret_cast<const f32x4*>(FL + G::LO_F2);

  f32x4 acc[G::MT_D][3];
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt) {
    const f32x4 bo = ld4(TL + G::TL_BO + 16 * mt + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[mt][w] = bo;
  }

#pragma unroll
  for (int p = 0; p < G::NPASS; ++p) {
    // ---- Q, K projections ----
    f32x4 Q[G::TP][3], Kt[G::TP][3];
#pragma unroll
    for (int tp = 0; tp < G::TP; ++tp) {
      const f32x4 bq = ld4(TL + G::TL_QKV + (p * 3 + 0) * G::TP * 16 + 16 * tp + 4 * g);
      const f32x4 bk = ld4(TL + G::TL_QKV + (p * 3 + 1) * G::TP * 16 + 16 * tp + 4 * g);
#pragma unroll
      for (int w = 0; w < 3; ++w) {
        Q[tp][w] = bq;
        Kt[tp][w] = bk;
      }
#pragma unroll
      for (int q4 = 0; q4 < G::KQ_D; ++q4) {
        const f32x4 aq = Aqkv[(((p * 3 + 0) * G::TP + tp) * G::KQ_D + q4) * 64 + lane];
        const f32x4 ak = Aqkv[(((p * 3 + 1) * G::TP + tp) * G::KQ_D + q4) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (4 * q4 + e < G::KS_D) {
#pragma unroll
            for (int w = 0; w < 3; ++w) {
              Q[tp][w] = mfma(aq[e], X[q4][w][e], Q[tp][w]);
              Kt[tp][w] = mfma(ak[e], X[q4][w][e], Kt[tp][w]);
            }
          }
        }
      }
    }
    // ---- scores over the 3 window steps, per head (q pre-scaled) ----
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
          for (int r = 0; r < 4; ++r) part += Q[tp][w][r] * Kt[tp][w2][r];
        sc[w2] = xsum(part, !G::P8);  // P8: groups {0,1} = head 0, {2,3} = head 1
      }
      const float m = fmaxf(sc[0], fmaxf(sc[1], sc[2]));
      const float e0 = expf(sc[0] - m), e1 = expf(sc[1] - m), e2 = expf(sc[2] - m);
      const float inv = 1.0f / (e0 + e1 + e2);
      pr[w][0] = e0 * inv;
      pr[w][1] = e1 * inv;
      pr[w][2] = e2 * inv;
    }
    // ---- V projection, P.V ----
    f32x4 O[G::TP][3];
#pragma unroll
    for (int tp = 0; tp < G::TP; ++tp) {
      f32x4 V[3];
      const f32x4 bv = ld4(TL + G::TL_QKV + (p * 3 + 2) * G::TP * 16 + 16 * tp + 4 * g);
#pragma unroll
      for (int w = 0; w < 3; ++w) V[w] = bv;
#pragma unroll
      for (int q4 = 0; q4 < G::KQ_D; ++q4) {
        const f32x4 av = Aqkv[(((p * 3 + 2) * G::TP + tp) * G::KQ_D + q4) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * q4 + e < G::KS_D) {
#pragma unroll
            for (int w = 0; w < 3; ++w) V[w] = mfma(av[e], X[q4][w][e], V[w]);
          }
      }
#pragma unroll
      for (int w = 0; w < 3; ++w) O[tp][w] = pr[w][0] * V[0] + pr[w][1] * V[1] + pr[w][2] * V[2];
    }
    // ---- out_proj (accumulate this pass's heads) ----
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt)
#pragma unroll
      for (int q4 = 0; q4 < G::KQ_O; ++q4) {
        const f32x4 a = Ao[((p * G::MT_D + mt) * G::KQ_O + q4) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * q4 + e < G::KS_O) {
#pragma unroll
            for (int w = 0; w < 3; ++w) acc[mt][w] = mfma(a[e], O[q4][w][e], acc[mt][w]);
          }
      }
  }
  // ---- x = norm1(x + sa) ----
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt)
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[mt][w] += X[mt][w];
  layer_norm_tiles<H>(acc, X, TL + G::TL_LN1G, TL + G::TL_LN1B, g);

  // ---- feed-forward ----
  f32x4 F1[G::MT_F][3];
#pragma unroll
  for (int mt = 0; mt < G::MT_F; ++mt) {
    const f32x4 b1 = ld4(TL + G::TL_B1 + 16 * mt + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) F1[mt][w] = b1;
#pragma unroll
    for (int q4 = 0; q4 < G::KQ_D; ++q4) {
      const f32x4 a = A1[(mt * G::KQ_D + q4) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * q4 + e < G::KS_D) {
#pragma unroll
          for (int w = 0; w < 3; ++w) F1[mt][w] = mfma(a[e], X[q4][w][e], F1[mt][w]);
        }
    }
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int r = 0; r < 4; ++r) F1[mt][w][r] = fmaxf(F1[mt][w][r], 0.f);
  }
#pragma unroll
  for (int mt = 0; mt < G::MT_D; ++mt) {
    const f32x4 b2 = ld4(TL + G::TL_B2 + 16 * mt + 4 * g);
#pragma unroll
    for (int w = 0; w < 3; ++w) acc[mt][w] = b2 + X[mt][w];
#pragma unroll
    for (int q4 = 0; q4 < G::KQ_F; ++q4) {
      const f32x4 a = A2[(mt * G::KQ_F + q4) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int w = 0; w < 3; ++w) acc[mt][w] = mfma(a[e], F1[q4][w][e], acc[mt][w]);
    }
  }
  // ---- x = norm2(x + ff) ----
  layer_norm_tiles<H>(acc, X, TL + G::TL_LN2G, TL + G::TL_LN2B, g);
}

// =============================================================================
// K2: encoder + decoders + classify.  One wave = 16 windows; loop over hosts h;
// the decoders' K = 3H^2 contraction is accumulated on the fly from each
// host's encoder output, so the latent never goes to HBM.
// =============================================================================
template <int H>
__global__ __launch_bounds__(kNWave * 64) void encdec_kernel(
    int B, int K, const float* __restrict__ agg, const float* __restrict__ frags,
    const float* __restrict__ tab_g, float* __restrict__ logits, float* __restrict__ protos,
    int* __restrict__ cls, int* __restrict__ any_anom, float* __restrict__ emb,
    float* __restrict__ latent) {
  using G = Geo<H>;
  __shared__ __attribute__((aligned(16))) float tab[G::t_size(kMaxProtos)];
  const int tsz = G::t_size(K);
  for (int i = threadIdx.x; i < tsz; i += blockDim.x) tab[i] = tab_g[i];
  __syncthreads();

  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const long blk = (long)blockIdx.x * kNWave + (threadIdx.x >> 6);
  const long nblk = (B + 15) / 16;
  if (blk >= nblk) return;

  f32x4 accd[G::MT_O];
#pragma unroll
  for (int mt = 0; mt < G::MT_O; ++mt) accd[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4* Ate = reinterpret_cast<const f32x4*>(frags + G::OFF_TE);
  (void)Ate;

  for (int h = 0; h < H; ++h) {
    const float* ap = agg + ((blk * H + h) * 3) * 48;
    float ba[3];
#pragma unroll
    for (int w = 0; w < 3; ++w) ba[w] = (g < 3) ? ap[w * 48 + lane] : 0.f;
    f32x4 X[G::MT_D][3];
#pragma unroll
    for (int mt = 0; mt < G::MT_D; ++mt) {
      const float a = frags[G::OFF_TE + mt * 64 + lane];
#pragma unroll
      for (int w = 0; w < 3; ++w) X[mt][w] = mfma(a, ba[w], ld4(tab + G::T_TE + w * G::DP + 16 * mt + 4 * g));
    }
#pragma unroll 1
    for (int l = 0; l < kLayers; ++l)
      encoder_layer<H>(X, frags + G::OFF_L0 + (long)l * G::SZ_LAYER, tab + G::T_L0 + l * G::TL_SIZE, lane);

    if (latent != nullptr) {
      const long b = blk * 16 + j;
      if (b < B) {
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
          for (int mt = 0; mt < G::MT_D; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int c = 16 * mt + 4 * r + g;
              if (c < H) latent[b * G::LAT + (long)h * 3 * H + w * H + c] = X[mt][w][r];
            }
      }
    }
    // ---- decoders: accd += Wdec[:, (h, w, :)] . X[:, w] ----
    const f32x4* Ad = reinterpret_cast<const f32x4*>(frags + G::OFF_DEC) + (long)h * 3 * G::MT_O * G::KQ_D * 64;
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int mt = 0; mt < G::MT_O; ++mt)
#pragma unroll
        for (int q4 = 0; q4 < G::KQ_D; ++q4) {
          const f32x4 a = Ad[((w * G::MT_O + mt) * G::KQ_D + q4) * 64 + lane];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (4 * q4 + e < G::KS_D) accd[mt] = mfma(a[e], X[q4][w][e], accd[mt]);
        }
  }

  // ---- epilogue: bias, sigmoid, detect, embed, classify ----
  const long b = blk * 16 + j;
  const bool valid = b < B;
  int anyf = 0;
  const float* P = tab + G::T_PROTO;
#pragma unroll
  for (int mt = 0; mt < G::MT_O; ++mt) {
    const int host = 4 * mt + g;
    const f32x4 v = accd[mt] + ld4(tab + G::T_DEC + 16 * mt + 4 * g);
    if (host < H) {
      const float l0 = v[0], l1 = v[1];
      const float p0 = 1.0f / (1.0f + expf(-v[2])), p1 = 1.0f / (1.0f + expf(-v[3]));
      const bool an = l1 > l0;  // torch.argmax: ties -> index 0
      const float e0 = an ? p0 : 0.f, e1 = an ? p1 : 0.f;
      int c = -1;
      if (!(e0 == 0.f && e1 == 0.f)) {
        float best = INFINITY;
        for (int k = 0; k < K; ++k) {
          const float d0 = e0 - P[2 * k], d1 = e1 - P[2 * k + 1];
          const float dist = (d0 * d0 + d1 * d1) * 0.5f;
          if (dist < best) {
            best = dist;
            c = k;
          }
        }
      }
      anyf |= an ? 1 : 0;
      if (valid) {
        const long o = (b * H + host) * 2;
        logits[o] = l0;
        logits[o + 1] = l1;
        protos[o] = p0;
        protos[o + 1] = p1;
        cls[b * H + host] = c;
        emb[b * G::EP + 2 * host] = e0;
        emb[b * G::EP + 2 * host + 1] = e1;
      }
    }
  }
  anyf |= __shfl_xor(anyf, 16);
  anyf |= __shfl_xor(anyf, 32);
  if (valid && g == 0) any_anom[b] = anyf;
}

// =============================================================================
// K3: generator + discriminator + decisions.  One wave = 16 windows.
//   Gen1 [64 x (2H+H^2)] and the s-half of Disc1 [64 x H^2] share one pass over
//   the schedule; Gen2 is produced one container row at a time and immediately
//   consumed by the ns-half of Disc1, so the new schedule never leaves registers.
// =============================================================================
template <int H>
__global__ __launch_bounds__(kNWave * 64) void gan_kernel(
    int B, const float* __restrict__ emb, const float* __restrict__ sched, const float* __restrict__ frags,
    const float* __restrict__ gt, float* __restrict__ probs, int* __restrict__ keep,
    int* __restrict__ final_t, int* __restrict__ gen_t) {
  using G = Geo<H>;
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const long blk = (long)blockIdx.x * kNWave + (threadIdx.x >> 6);
  const long nblk = (B + 15) / 16;
  if (blk >= nblk) return;
  const long b = blk * 16 + j;
  const bool valid = b < B;
  const float* sw = sched + (valid ? b : 0) * G::H2;
  const float* ew = emb + (valid ? b : 0) * G::EP;

  f32x4 hg[G::MT_G], hd[G::MT_G];
#pragma unroll
  for (int mt = 0; mt < G::MT_G; ++mt) {
    hg[mt] = ld4(gt + G::G_B1 + 16 * mt + 4 * g);
    hd[mt] = ld4(gt + G::G_BD1 + 16 * mt + 4 * g);
  }
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  // ---- Gen1, embedding half ----
  const f32x4* A1e = reinterpret_cast<const f32x4*>(frags + G::OFF_G1E);
#pragma unroll
  for (int q = 0; q < G::EQ; ++q) {
    const f32x4 bv = valid ? ld4(ew + 16 * q + 4 * g) : zero4;
#pragma unroll
    for (int mt = 0; mt < G::MT_G; ++mt) {
      const f32x4 a = A1e[(mt * G::EQ + q) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) hg[mt] = mfma(a[e], bv[e], hg[mt]);
    }
  }
  // ---- Gen1 schedule half + Disc1 schedule half (shared B operand) ----
  const f32x4* A1s = reinterpret_cast<const f32x4*>(frags + G::OFF_G1S);
  const f32x4* Ad1s = reinterpret_cast<const f32x4*>(frags + G::OFF_D1S);
#pragma unroll 2
  for (int q = 0; q < G::SQ; ++q) {
    const int idx = 16 * q + 4 * g;
    const f32x4 bv = (valid && idx < G::H2) ? ld4(sw + idx) : zero4;
#pragma unroll
    for (int mt = 0; mt < G::MT_G; ++mt) {
      const f32x4 a = A1s[(mt * G::SQ + q) * 64 + lane];
      const f32x4 ad = Ad1s[(mt * G::SQ + q) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hg[mt] = mfma(a[e], bv[e], hg[mt]);
        hd[mt] = mfma(ad[e], bv[e], hd[mt]);
      }
    }
  }
  // (LeakyReLU(True) is the identity: hg is the hidden layer as is)
  // ---- per container row: Gen2 -> tanh -> ns -> argmaxes -> Disc1 ns half ----
  const f32x4* A2 = reinterpret_cast<const f32x4*>(frags + G::OFF_G2);
  const f32x4* Ad1n = reinterpret_cast<const f32x4*>(frags + G::OFF_D1N);
  for (int c = 0; c < G::C; ++c) {
    f32x4 ns[G::MT_N];
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t) {
      ns[t] = ld4(gt + G::G_B2 + c * G::MT_N * 16 + 16 * t + 4 * g);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const f32x4 a = A2[(((long)c * G::MT_N + t) * 4 + q4) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) ns[t] = mfma(a[e], hg[q4][e], ns[t]);
      }
    }
    float bn = -INFINITY, bs = -INFINITY;
    int bni = 0, bsi = 0;
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hh = 16 * t + 4 * g + r;
        if (hh < H) {
          const float sv = valid ? sw[c * H + hh] : 0.f;
          const float nv = sv + 4.0f * tanhf(ns[t][r]);
          ns[t][r] = nv;
          if (nv > bn) {
            bn = nv;
            bni = hh;
          }
          if (sv > bs) {
            bs = sv;
            bsi = hh;
          }
        } else {
          ns[t][r] = 0.f;
        }
      }
#pragma unroll
    for (int mt = 0; mt < G::MT_G; ++mt)
#pragma unroll
      for (int q4 = 0; q4 < G::MT_N; ++q4) {
        const f32x4 a = Ad1n[(((long)c * G::MT_G + mt) * G::MT_N + q4) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) hd[mt] = mfma(a[e], ns[q4][e], hd[mt]);
      }
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float ov = __shfl_xor(bn, off), os = __shfl_xor(bs, off);
      const int oi = __shfl_xor(bni, off), osi = __shfl_xor(bsi, off);
      if (ov > bn || (ov == bn && oi < bni)) {
        bn = ov;
        bni = oi;
      }
      if (os > bs || (os == bs && osi < bsi)) {
        bs = os;
        bsi = osi;
      }
    }
    if (valid && g == 0) {
      gen_t[b * G::C + c] = bni;
      final_t[b * G::C + c] = bsi;
    }
  }
  // ---- Disc2 + softmax + gate ----
  float z0 = 0.f, z1 = 0.f;
#pragma unroll
  for (int mt = 0; mt < G::MT_G; ++mt) {
    const f32x4 w0 = ld4(gt + G::G_WD2 + 16 * mt + 4 * g), w1 = ld4(gt + G::G_WD2 + 64 + 16 * mt + 4 * g);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      z0 += hd[mt][r] * w0[r];
      z1 += hd[mt][r] * w1[r];
    }
  }
  z0 = xsum(z0, true) + gt[G::G_BD2];
  z1 = xsum(z1, true) + gt[G::G_BD2 + 1];
  const float m = fmaxf(z0, z1);
  const float e0 = expf(z0 - m), e1 = expf(z1 - m);
  const float inv = 1.0f / (e0 + e1);
  const float p0 = e0 * inv, p1 = e1 * inv;
  if (valid && g == 0) {
    probs[2 * b] = p0;
    probs[2 * b + 1] = p1;
    keep[b] = p0 > p1 ? 1 : 0;
  }
}

}  // namespace

// =============================================================================
// C-ABI
// =============================================================================
struct pgp_model {
  int H = 0, K = 0;
  bool loaded = false;
  float* d_frags = nullptr;
  float* d_tab = nullptr;
  float* d_gtab = nullptr;
  GatConst gat{};
  int cap = 0;  // workspace capacity in windows
  float* d_agg = nullptr;
  float* d_emb = nullptr;
};

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                            \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) return fail(PGP_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

template <int H>
size_t frag_floats() { return Geo<H>::SZ_FRAGS; }

template <int H>
int launch_t(pgp_model* m, int stage, int B, const float* windows, const float* sched, float* logits,
             float* protos, int* cls, int* any_anom, float* probs, int* keep, int* final_t, int* gen_t,
             float* latent, hipStream_t st) {
  using G = Geo<H>;
  const long nblk = (B + 15) / 16;
  const int grid = (int)((nblk + kNWave - 1) / kNWave);
  if (stage < 0 || stage == 0) {
    const long items = (long)B * 3;
    gat_agg_kernel<H><<<(int)((items + 3) / 4), 256, 0, st>>>(B, windows, m->d_agg, m->gat);
    HIPCHK(hipGetLastError());
  }
  if (stage < 0 || stage == 1) {
    encdec_kernel<H><<<grid, kNWave * 64, 0, st>>>(B, m->K, m->d_agg, m->d_frags, m->d_tab, logits, protos, cls,
                                                   any_anom, m->d_emb, latent);
    HIPCHK(hipGetLastError());
  }
  if (stage < 0 || stage == 2) {
    gan_kernel<H><<<grid, kNWave * 64, 0, st>>>(B, m->d_emb, sched, m->d_frags, m->d_gtab, probs, keep, final_t,
                                                gen_t);
    HIPCHK(hipGetLastError());
  }
  return PGP_OK;
}

#define PGP_FOR_EACH_H(X) X(8) X(16) X(32) X(50) X(64)

bool supported(int H) {
  switch (H) {
#define CASE(h) case h:
    PGP_FOR_EACH_H(CASE)
#undef CASE
    return true;
  }
  return false;
}

size_t frags_len(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return Geo<h>::SZ_FRAGS;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}
int ep_len(int H) { return round_up(2 * H, 16); }

int reserve(pgp_model* m, int n) {
  if (n <= m->cap) return PGP_OK;
  if (m->d_agg) HIPCHK(hipFree(m->d_agg));
  if (m->d_emb) HIPCHK(hipFree(m->d_emb));
  m->d_agg = m->d_emb = nullptr;
  m->cap = 0;
  const size_t nblk = (size_t)(n + 15) / 16;
  const size_t agg_f = nblk * m->H * 3 * 48;
  const size_t emb_f = nblk * 16 * ep_len(m->H);
  HIPCHK(hipMalloc(&m->d_agg, agg_f * sizeof(float)));
  HIPCHK(hipMalloc(&m->d_emb, emb_f * sizeof(float)));
  HIPCHK(hipMemset(m->d_agg, 0, agg_f * sizeof(float)));
  HIPCHK(hipMemset(m->d_emb, 0, emb_f * sizeof(float)));
  m->cap = n;
  return PGP_OK;
}
}  // namespace

extern "C" {

int pgp_abi_version(void) { return PGP_ABI_VERSION; }
const char* pgp_last_error(void) { return g_err.c_str(); }

int pgp_supported_hosts(int* out, int cap) {
  static const int hs[] = {8, 16, 32, 50, 64};
  const int n = (int)(sizeof(hs) / sizeof(hs[0]));
  for (int i = 0; i < n && i < cap && out; ++i) out[i] = hs[i];
  return n;
}

size_t pgp_weight_blob_len(int n_hosts, int n_protos) {
  if (!supported(n_hosts) || n_protos < 1) return 0;
  return blob_len(n_hosts, n_protos);
}

int pgp_create(int n_hosts, int n_protos, pgp_model** out) {
  if (!out) return fail(PGP_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (!supported(n_hosts)) return fail(PGP_ERR_UNSUPPORTED, "host count not compiled in: " + std::to_string(n_hosts));
  if (n_protos < 1 || n_protos > kMaxProtos) return fail(PGP_ERR_ARG, "n_protos out of range [1,64]");
  pgp_model* m = new pgp_model();
  m->H = n_hosts;
  m->K = n_protos;
  *out = m;
  return PGP_OK;
}

int pgp_destroy(pgp_model* m) {
  if (!m) return PGP_OK;
  if (m->d_frags) (void)hipFree(m->d_frags);
  if (m->d_tab) (void)hipFree(m->d_tab);
  if (m->d_gtab) (void)hipFree(m->d_gtab);
  if (m->d_agg) (void)hipFree(m->d_agg);
  if (m->d_emb) (void)hipFree(m->d_emb);
  delete m;
  return PGP_OK;
}

int pgp_load_weights(pgp_model* m, const double* blob, size_t len) {
  if (!m || !blob) return fail(PGP_ERR_ARG, "NULL model or blob");
  Packed P;
  const std::string err = pack_weights(m->H, m->K, blob, len, &P);
  if (!err.empty()) return fail(PGP_ERR_ARG, err);
  if (!m->d_frags) HIPCHK(hipMalloc(&m->d_frags, P.frags.size() * sizeof(float)));
  if (!m->d_tab) HIPCHK(hipMalloc(&m->d_tab, P.enc_tab.size() * sizeof(float)));
  if (!m->d_gtab) HIPCHK(hipMalloc(&m->d_gtab, P.gan_tab.size() * sizeof(float)));
  HIPCHK(hipMemcpy(m->d_frags, P.frags.data(), P.frags.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(m->d_tab, P.enc_tab.data(), P.enc_tab.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(m->d_gtab, P.gan_tab.data(), P.gan_tab.size() * sizeof(float), hipMemcpyHostToDevice));
  m->gat = P.gat;
  m->loaded = true;
  return PGP_OK;
}

int pgp_reserve(pgp_model* m, int max_batch) {
  if (!m || max_batch < 0) return fail(PGP_ERR_ARG, "bad reserve arguments");
  return reserve(m, max_batch);
}

int pgp_forward_stage(pgp_model* m, int stage, int batch, const float* windows, const float* sched, float* logits,
                      float* protos, int* cls, int* any_anom, float* probs, int* keep_orig, int* final_target,
                      int* gen_target, float* latent, void* stream) {
  if (!m) return fail(PGP_ERR_ARG, "NULL model");
  if (!m->loaded) return fail(PGP_ERR_STATE, "weights not loaded");
  if (batch < 0) return fail(PGP_ERR_ARG, "negative batch");
  if (batch == 0) return PGP_OK;
  if (stage < -1 || stage > 2) return fail(PGP_ERR_ARG, "bad stage");
  if ((stage <= 0 && !windows) || ((stage == -1 || stage == 1) && (!logits || !protos || !cls || !any_anom)) ||
      ((stage == -1 || stage == 2) && (!sched || !probs || !keep_orig || !final_target || !gen_target)))
    return fail(PGP_ERR_ARG, "NULL input/output pointer");
  if (batch > m->cap) {
    const int rc = reserve(m, batch);
    if (rc) return rc;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (m->H) {
#define CASE(h) \
  case h:       \
    return launch_t<h>(m, stage, batch, windows, sched, logits, protos, cls, any_anom, probs, keep_orig, final_target, gen_target, latent, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return fail(PGP_ERR_UNSUPPORTED, "host count");
}

int pgp_forward(pgp_model* m, int batch, const float* windows, const float* sched, float* logits, float* protos,
                int* cls, int* any_anom, float* probs, int* keep_orig, int* final_target, int* gen_target,
                float* latent, void* stream) {
  return pgp_forward_stage(m, -1, batch, windows, sched, logits, protos, cls, any_anom, probs, keep_orig,
                           final_target, gen_target, latent, stream);
}

}  // extern "C"
