// pgp_gansplit.hip — K3 (generator + discriminator + decision argmaxes,
// models.py:118-151, 258-291; PreGANPlus.py:84-105; Stats.py:162-166) with its
// contractions on split-bf16 MFMAs (v_mfma_f32_16x16x32_bf16), at H = 16 and 50
// (16-wave workgroups from 64 K windows up, 4-wave ones below: every wave
// computes its 16 windows the same way, so the outputs do not depend on the
// batch a window arrives in).
//
// Same phases, ring and outputs as gan_kernel (pgp_gan.hip):
//   1. Gen1, embedding columns        hg  = W1[:, :2H] . vec(emb)
//   2. one pass over the schedule     hg += W1[:, 2H:] . vec(s);  hd = Wd1[:, :H^2] . vec(s)
//   3. per container row c            ns_c = s_c + 4 tanh(W2[c] . hg + b2[c]); both first-argmaxes;
//                                      hd += Wd1[:, H^2 + cH : H^2 + (c+1)H] . ns_c
//   then Disc2 + softmax + gate.
// Every fp32 product w.x is the six bf16 products w_i.x_j, i + j <= 2, of the
// operands' exact three-part splits (pgp_device.hpp split8 / mfma_bf6; the
// dropped terms are below 2^-26 of |w x|, tools/micro/bf16_split.hip): the
// weights' planes are derived once per weight load (gan_split_derive_kernel),
// the B operands are split in registers.  A schedule block whose 32 values per
// lane are all exactly bf16 in every lane of the wave (a one-hot GOBI schedule)
// takes three products: the other three would add exact zeros.
//
// A 16x16x32 B operand is a lane's 8 consecutive k of its lane group; here a
// lane keeps two 16-column k-blocks' 4 values each (the fp32 kernels' lane
// layout), so a 32-k block pairs two of gan_kernel's k-blocks: k-block q holds
// column 16q + 4g + e of lane group g; pair p is blocks 2p, 2p + 1, element
// 4h + e of the lane's 8 <-> block 2p + h, value e.  The weight planes are
// paired the same way from the fp32 fragments (lane-local).
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kSWaves = 16;      // waves per workgroup at large batches
constexpr int kSWavesSmall = 4;  // below kSSmallBlocks blocks of 16 windows (spread over more CUs)
constexpr long kSSmallBlocks = 16L * 256;
constexpr int kSQP = 2;  // schedule pairs per ring chunk
#ifndef PGP_K3_OH
#define PGP_K3_OH 1
#endif
constexpr bool kK3OneHot = PGP_K3_OH != 0;  // phase 3 rebuilds one-hot rows from LDS (A/B: -DPGP_K3_OH=0)
#ifndef PGP_K3_PF
#define PGP_K3_PF 1
#endif
constexpr bool kK3PF = kK3OneHot && PGP_K3_PF != 0;  // one-hot containers: planes read a step ahead (A/B: -DPGP_K3_PF=0)

template <int H>
struct GanS {
  using G = Geo<H>;
  static constexpr int NPE = cdiv(G::EQ, 2);    // embedding pairs
  static constexpr int NPS = cdiv(G::SQ, 2);    // schedule pairs
  static constexpr int NPN = cdiv(G::MT_N, 2);  // new-schedule pairs (Disc1 second half)
  // planes, in 1-KiB fragments of [lane][8 bf16]
  static constexpr int FE = NPE * G::MT_G * 3;                       // [pair][mt][plane]
  static constexpr int FS = 8 * 3;                                   // per schedule pair: [gen mt | disc mt][plane]
  static constexpr int FC2 = G::MT_N * 2 * 3;                        // per container, Gen2: [t][pair of q4][plane]
  static constexpr int FCD = G::MT_G * NPN * 3;                      // per container, Disc1 new half: [mt][pair][plane]
  static constexpr int FC = FC2 + FCD;
  static constexpr long OFF_E = 0, OFF_S = FE, OFF_C = OFF_S + (long)NPS * FS;
  static constexpr long FRAGS = OFF_C + (long)G::C * FC;
  static constexpr long SIZE = FRAGS * 256;  // floats
  static constexpr int NQC = cdiv(NPS, kSQP);
  static constexpr int BIAS_F = G::MT_N * 16;
  static constexpr int CPC = 1;
  static constexpr int NCHUNK = 1 + NQC + G::C / CPC;
  static constexpr int mx(int x, int y) { return x > y ? x : y; }
  static constexpr int SLOT_G = mx(FE, mx(kSQP * FS, CPC * FC + 1));
  static constexpr int SLOT = SLOT_G * G::FQ;
  static constexpr int TGT = 2 * G::C * 16;  // int8 targets per wave
  static constexpr int OH = G::C * 16;       // int8 one-hot row index per (container, window) of a wave
  static constexpr int lds_bytes(int nw) { return 2 * SLOT * 4 + nw * (TGT + OH); }
  static constexpr int LDS_BYTES = lds_bytes(kSWaves);
  PGP_DEV static void chunk(int k, const float* planes, const float** src, int* ng) {
    if (k == 0) {
      *src = planes + OFF_E * 256;
      *ng = FE;
    } else if (k <= NQC) {
      const int p0 = (k - 1) * kSQP;
      *src = planes + (OFF_S + (long)p0 * FS) * 256;
      *ng = (NPS - p0 < kSQP ? NPS - p0 : kSQP) * FS;
    } else {
      *src = planes + (OFF_C + (long)(k - 1 - NQC) * CPC * FC) * 256;
      *ng = CPC * FC;
    }
  }
};

template <int H>
constexpr bool gan_split() {
  return (H == 16 || H == 50) && GanS<H>::LDS_BYTES <= 160 * 1024 && Geo<H>::C < 128;
}

// fp32 fragments -> planes.  One wave per destination fragment triple.
template <int H>
__global__ __launch_bounds__(256) void gan_split_derive_kernel(const float* __restrict__ frags,
                                                               float* __restrict__ out) {
  using G = Geo<H>;
  using S = GanS<H>;
  const long f = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // triple index
  const int lane = threadIdx.x & 63;
  if (f * 3 >= S::FRAGS) return;
  long ga = -1, gb = -1;  // the two fp32 groups (float offsets), -1: a zero group
  const long e3 = f * 3;
  if (e3 < S::OFF_S) {  // embedding: [pair][mt]
    const long t = e3 / 3;
    const int mt = (int)(t % G::MT_G), p = (int)(t / G::MT_G);
    const int q0 = 2 * p, q1 = 2 * p + 1;
    ga = G::OFF_GE + (long)(mt * G::EQ + q0) * 256;
    if (q1 < G::EQ) gb = G::OFF_GE + (long)(mt * G::EQ + q1) * 256;
  } else if (e3 < S::OFF_C) {  // schedule: [pair][k8]
    const long t = (e3 - S::OFF_S) / 3;
    const int k = (int)(t % 8), p = (int)(t / 8);
    const int q0 = 2 * p, q1 = 2 * p + 1;
    ga = G::OFF_GS + (long)(q0 * G::GS_G + k) * 256;
    if (q1 < G::SQ) gb = G::OFF_GS + (long)(q1 * G::GS_G + k) * 256;
  } else {  // container c: Gen2 [t][pair] | Disc1 new half [mt][pair]
    const long r = e3 - S::OFF_C;
    const long c = r / S::FC;
    const int w = (int)(r % S::FC) / 3;
    const long base = G::OFF_GC + c * G::GC_G * 256;
    if (w < G::MT_N * 2) {
      const int t = w / 2, p = w % 2;
      ga = base + (long)(t * 4 + 2 * p) * 256;
      gb = base + (long)(t * 4 + 2 * p + 1) * 256;
    } else {
      const int u = w - G::MT_N * 2;
      const int mt = u / S::NPN, p = u % S::NPN;
      const int q0 = 2 * p, q1 = 2 * p + 1;
      ga = base + (long)(G::GC_G2 + mt * G::MT_N + q0) * 256;
      if (q1 < G::MT_N) gb = base + (long)(G::GC_G2 + mt * G::MT_N + q1) * 256;
    }
  }
  float v[8];
  const f32x4 a = ld4(frags + ga + lane * 4);
  const f32x4 b = gb >= 0 ? ld4(frags + gb + lane * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = a[e];
    v[4 + e] = b[e];
  }
  u32x4 p[3];
  split8(v, p);
#pragma unroll
  for (int k = 0; k < 3; ++k) *reinterpret_cast<u32x4*>(out + (e3 + k) * 256 + lane * 4) = p[k];
}

PGP_DEV void pair8(const f32x4& a, const f32x4& b, float (&v)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = a[e];
    v[4 + e] = b[e];
  }
}
PGP_DEV void planes_at(const float* F, int lane, u32x4 (&w)[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) w[k] = *reinterpret_cast<const u32x4*>(F + k * 256 + lane * 4);
}

// The ring's DMA, issued where the compiler does not see it: a pending
// global_load_lds (a VMEM op that writes) makes the compiler's wait for any
// older load a full drain (vmcnt(0)), so each chunk's first use of its
// schedule values also waited for the DMA and the next chunk's prefetch just
// issued.  Its completion is waited for explicitly before every barrier
// (k3_sync); the compiler's own waits stay correct, only stricter, with these
// ops in flight (loads complete in order).
PGP_DEV void k3_dma(const float* __restrict__ src, float* dst, int ngroups, int wv, int nwaves, int lane) {
  for (int g = wv; g < ngroups; g += nwaves) {
    const float* base = src + (long)g * 256;  // wave-uniform: the SGPR-base form, a 32-bit lane offset
    const unsigned off = (unsigned)lane * 16u;
    const unsigned m = (unsigned)(unsigned long)((__attribute__((address_space(3))) float*)(dst + g * 256));
    asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(base), "s"(m) : "memory", "m0");
  }
}
PGP_DEV void k3_sync() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__device__ __attribute__((aligned(8))) float k3s_zero_pair[2];  // never written
__device__ __attribute__((aligned(16))) float k3s_zero4[4];      // never written

template <int H, int NW>
__global__ __launch_bounds__(NW * 64) void gan_split_kernel(FwdArgs a) {
  using G = Geo<H>;
  using S = GanS<H>;
  extern __shared__ __attribute__((aligned(16))) float smem[];  // ring [2][SLOT] | targets
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long blk = (long)blockIdx.x * NW + wv;
  const long nblk = (a.B + 15) / 16;
  const long b = blk * 16 + j;
  const bool valid = blk < nblk && b < a.B;
  const float* sw = a.sched + (valid ? b : 0) * G::H2;
  const float* ew = a.emb + (valid ? b : 0) * G::EP;
  const float* gt = a.gtab;
  signed char* tg = reinterpret_cast<signed char*>(smem + 2 * S::SLOT) + wv * S::TGT;
  // phase 2 records where each schedule row holds its 1.0 (a GOBI placement is
  // one-hot, opt.py:9-15); phase 3 then rebuilds a row from it instead of
  // reading the 4H-byte row from HBM again (the schedules are 2/3 of the
  // kernel's traffic).  Rows proven one-hot only: per window exactly C nonzero
  // values, all exactly 1.0, and every row recorded; otherwise the wave reads
  // its rows as before.
  signed char* oh = reinterpret_cast<signed char*>(smem + 2 * S::SLOT) + NW * S::TGT + wv * S::OH;
  if (kK3OneHot)
    for (int i = lane; i < S::OH; i += 64) oh[i] = -1;
  int n_one = 0, n_nz = 0;
  bool oh_bad = false;  // wave-uniform

  float* cur = smem;
  float* nxt = smem + S::SLOT;
  int next = 1;
  {
    const float* src;
    int ng;
    S::chunk(0, a.ganb, &src, &ng);
    k3_dma(src, cur, ng, wv, NW, lane);
  }
  auto issue = [&]() {
    if (next < S::NCHUNK) {
      const float* src;
      int ng;
      S::chunk(next, a.ganb, &src, &ng);
      k3_dma(src, nxt, ng, wv, NW, lane);
      if (next > S::NQC)  // a container chunk: its Gen2 biases after its planes
        k3_dma(gt + G::G_B2 + (long)(next - 1 - S::NQC) * S::CPC * S::BIAS_F, nxt + ng * 256, 1,
                   (wv + ng) % NW, NW, lane);
    }
  };
  auto advance = [&]() {
    k3_sync();
    float* t = cur;
    cur = nxt;
    nxt = t;
    ++next;
    issue();
  };

  f32x4 hg[G::MT_G], hd[G::MT_G];
#pragma unroll
  for (int mt = 0; mt < G::MT_G; ++mt) {
    hg[mt] = ld4(gt + G::G_B1 + 16 * mt + 4 * g);
    hd[mt] = ld4(gt + G::G_BD1 + 16 * mt + 4 * g);
  }
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  k3_sync();
  issue();

  // ---- phase 1: Gen1, embedding columns ----
#pragma unroll
  for (int p = 0; p < S::NPE; ++p) {
    float v[8];
    const f32x4 e0 = valid ? ld4(ew + 32 * p + 4 * g) : zero4;
    const f32x4 e1 = (valid && 2 * p + 1 < G::EQ) ? ld4(ew + 32 * p + 16 + 4 * g) : zero4;
    pair8(e0, e1, v);
    u32x4 x[3];
    split8(v, x);
#pragma unroll
    for (int mt = 0; mt < G::MT_G; ++mt) {
      u32x4 w[3];
      planes_at(cur + ((p * G::MT_G + mt) * 3) * 256, lane, w);
      hg[mt] = mfma_bf6(w, x, hg[mt]);
    }
  }

  // ---- phase 2: schedule pass (Gen1 + Disc1 schedule half) ----
  auto load_pair = [&](int p, f32x4 (&q)[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int idx = 16 * (2 * p + h) + 4 * g;
      // unconditional: a lane past the row reads zeros; a load behind a branch
      // made the compiler wait for ALL loads at the next chunk's first use
      // (vmcnt(0): the just-issued prefetch too, one HBM latency per chunk)
      q[h] = ld4((valid && p < S::NPS && idx < G::H2) ? sw + idx : k3s_zero4);
    }
  };
  f32x4 bq[kSQP][2];
#pragma unroll
  for (int i = 0; i < kSQP; ++i) load_pair(i, bq[i]);
  advance();
  for (int qc = 0; qc < S::NQC; ++qc) {
    f32x4 bn[kSQP][2];
#pragma unroll
    for (int i = 0; i < kSQP; ++i) load_pair((qc + 1) * kSQP + i, bn[i]);
#pragma unroll
    for (int i = 0; i < kSQP; ++i) {
      if (qc * kSQP + i < S::NPS) {
        float v[8];
        pair8(bq[i][0], bq[i][1], v);
        // every value exactly a bf16 in every lane (one-hot rows: 0 / 1): the
        // residual planes are zero and x0 is the values' high halves
        unsigned low = 0u;
#pragma unroll
        for (int e = 0; e < 8; ++e) low |= __float_as_uint(v[e]) & 0xFFFFu;
        const bool exact = __builtin_amdgcn_ballot_w64(low != 0u) == 0ull;
        u32x4 x[3];
        if (exact) {
#pragma unroll
          for (int d = 0; d < 4; ++d)
            x[0][d] = (__float_as_uint(v[2 * d]) >> 16) | (__float_as_uint(v[2 * d + 1]) & 0xFFFF0000u);
          if (kK3OneHot) {
            // bf16 halves: nonzero / exactly 1.0 (0x3F80), element e = half e
            unsigned m_nz = 0u, m_one = 0u;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const unsigned hv = (x[0][e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
              m_nz |= ((hv & 0x7FFFu) != 0u ? 1u : 0u) << e;
              m_one |= (hv == 0x3F80u ? 1u : 0u) << e;
            }
            n_nz += __builtin_popcount(m_nz);
            n_one += __builtin_popcount(m_one);
            if (m_one != 0u) {
              // the lane's 8 values span at most two rows: record the lowest and
              // the highest 1.0 (a row holding two is caught by the counts)
              const int base = 32 * (qc * kSQP + i) + 4 * g;
              const int elo = __builtin_ctz(m_one), ehi = 31 - __builtin_clz(m_one);
              const int klo = base + 16 * (elo >> 2) + (elo & 3), khi = base + 16 * (ehi >> 2) + (ehi & 3);
              const int clo = klo / H, chi = khi / H;  // flattened c * H + h
              oh[clo * 16 + j] = (signed char)(klo - clo * H);
              oh[chi * 16 + j] = (signed char)(khi - chi * H);
            }
          }
        } else {
          split8(v, x);
          oh_bad = true;  // not all bf16: not one-hot
        }
        const float* F = cur + i * S::FS * 256;
        if (exact) {
#pragma unroll
          for (int mt = 0; mt < G::MT_G; ++mt) {
            u32x4 wg[3], wd[3];
            planes_at(F + (mt * 3) * 256, lane, wg);
            planes_at(F + ((G::MT_G + mt) * 3) * 256, lane, wd);
            hg[mt] = mfma_bf3(wg, x, hg[mt]);
            hd[mt] = mfma_bf3(wd, x, hd[mt]);
          }
        } else {
#pragma unroll
          for (int mt = 0; mt < G::MT_G; ++mt) {
            u32x4 wg[3], wd[3];
            planes_at(F + (mt * 3) * 256, lane, wg);
            planes_at(F + ((G::MT_G + mt) * 3) * 256, lane, wd);
            hg[mt] = mfma_bf6(wg, x, hg[mt]);
            hd[mt] = mfma_bf6(wd, x, hd[mt]);
          }
        }
      }
    }
    // the next chunk's values are taken here, before the barrier (which drains
    // them anyway), so that the compiler's wait for them precedes the next DMA
#pragma unroll
    for (int i = 0; i < kSQP; ++i) asm volatile("" ::"v"(bn[i][0]), "v"(bn[i][1]));
    advance();
#pragma unroll
    for (int i = 0; i < kSQP; ++i) {
      bq[i][0] = bn[i][0];
      bq[i][1] = bn[i][1];
    }
  }

  // ---- phase 3: per container row ----
  static_assert(H % 2 == 0, "row pairs");
  auto load_row = [&](int c, float (&v)[G::MT_N][4]) {
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const int hh = 16 * t + 4 * g + r;
        const float* src = (valid && hh < H && c < G::C) ? sw + c * H + hh : k3s_zero_pair;
        const float2 p = *reinterpret_cast<const float2*>(src);
        v[t][r] = p.x;
        v[t][r + 1] = p.y;
      }
  };
  // the hidden layer's split planes, shared by every container's Gen2
  u32x4 hx[2][3];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    float v[8];
    pair8(hg[2 * p], hg[2 * p + 1], v);
    split8(v, hx[p]);
  }
  float sv[G::MT_N][4];
  // the wave's rows are one-hot iff every window saw exactly C nonzero values,
  // all 1.0, and every one of its C rows recorded a 1.0 (C ones over C rows,
  // none empty: one per row)
  bool ohw = kK3OneHot;
  if (kK3OneHot) {
    const float t1 = xsum((float)n_one, true), tn = xsum((float)n_nz, true);
    bool bad = oh_bad || (valid && (t1 != (float)G::C || tn != (float)G::C));
    for (int i = lane; i < S::OH; i += 64)
      if (blk < nblk && blk * 16 + (i & 15) < a.B && oh[i] < 0) bad = true;
    ohw = __builtin_amdgcn_ballot_w64(bad) == 0ull;
  }
  // cross-group first-argmaxes of a container row, and its two targets
  auto k3_targets = [&](int c, float bn_v, int bn_i, float bs_v, int bs_i) {
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float ov = __shfl_xor(bn_v, off), os = __shfl_xor(bs_v, off);
      const int oi = __shfl_xor(bn_i, off), osi = __shfl_xor(bs_i, off);
      if (ov > bn_v || (ov == bn_v && oi < bn_i)) {
        bn_v = ov;
        bn_i = oi;
      }
      if (os > bs_v || (os == bs_v && osi < bs_i)) {
        bs_v = os;
        bs_i = osi;
      }
    }
    if (g == 0) {
      tg[c * 16 + j] = (signed char)bn_i;
      tg[(G::C + c) * 16 + j] = (signed char)bs_i;
    }
  };
  // the 2 MT_N Gen2 and MT_G NPN Disc1 plane triples of a container, in use order
  constexpr int NF = 2 * G::MT_N + S::NPN * G::MT_G;
  auto pl_addr = [&](const float* cw, int f) -> const float* {
    if (f < 2 * G::MT_N) return cw + (((f % G::MT_N) * 2 + f / G::MT_N) * 3) * 256;  // Gen2 (pair f / MT_N, tile f % MT_N)
    const int q = f - 2 * G::MT_N;
    return cw + (S::FC2 + ((q % G::MT_G) * S::NPN + q / G::MT_G) * 3) * 256;  // Disc1 (pair q / MT_G, tile q % MT_G)
  };
  for (int c = 0; c < G::C; ++c) {
    const float* cw = cur;  // CPC = 1: this container's planes
    if (kK3PF && ohw) {
      // one-hot rows: the row is its 1.0's position (no registers for it), and
      // each plane triple is read one step ahead of the MFMAs that use it,
      // pinned there (the compiler otherwise reads it right before them and
      // waits: 16 exposed LDS round trips per container)
      const int hc = oh[c * 16 + j];  // -1 for a window past B: a zero row, as load_row gives
      u32x4 wb[2][3];
      planes_at(pl_addr(cw, 0), lane, wb[0]);
      f32x4 ns[G::MT_N];
      const float* bias = cur + S::FC * 256;
#pragma unroll
      for (int t = 0; t < G::MT_N; ++t) ns[t] = ld4(bias + 16 * t + 4 * g);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int t = 0; t < G::MT_N; ++t) {
          const int f = p * G::MT_N + t;
          __builtin_amdgcn_sched_barrier(0);
          planes_ready(wb[f & 1]);
          planes_at(pl_addr(cw, f + 1), lane, wb[(f + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
          ns[t] = mfma_bf6(wb[f & 1], hx[p], ns[t]);
        }
      __builtin_amdgcn_s_setprio(0);
      float bn_v = -INFINITY, bs_v = -INFINITY;
      int bn_i = 0, bs_i = 0;
#pragma unroll
      for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int hh = 16 * t + 4 * g + r;
          if (hh < H) {
            const float s0 = hh == hc ? 1.f : 0.f;
            const float nv = s0 + 4.0f * tanh_fast(ns[t][r]);
            ns[t][r] = nv;
            if (nv > bn_v) {  // strict: first maximum wins (list.index(max(...)))
              bn_v = nv;
              bn_i = hh;
            }
            if (s0 > bs_v) {
              bs_v = s0;
              bs_i = hh;
            }
          } else {
            ns[t][r] = 0.f;
          }
        }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int p = 0; p < S::NPN; ++p) {
        float v[8];
        pair8(ns[2 * p], 2 * p + 1 < G::MT_N ? ns[2 * p + 1] : zero4, v);
        u32x4 x[3];
        split8(v, x);
#pragma unroll
        for (int mt = 0; mt < G::MT_G; ++mt) {
          const int f = 2 * G::MT_N + p * G::MT_G + mt;
          __builtin_amdgcn_sched_barrier(0);
          planes_ready(wb[f & 1]);
          if (f + 1 < NF) planes_at(pl_addr(cw, f + 1), lane, wb[(f + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
          hd[mt] = mfma_bf6(wb[f & 1], x, hd[mt]);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      k3_targets(c, bn_v, bn_i, bs_v, bs_i);
      advance();
      continue;
    }
    // this container's schedule row, requested before Gen2's MFMAs (which
    // cover its latency; a row prefetched a container ahead spilled at the
    // 128-register budget of 4 waves per SIMD)
    if (ohw) {
      const int hc = oh[c * 16 + j];  // -1 for a window past B: a zero row, as load_row gives
#pragma unroll
      for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[t][r] = (16 * t + 4 * g + r == hc) ? 1.f : 0.f;
    } else {
      load_row(c, sv);
    }
    // Gen2: ns = b2[c] + W2[c] . hg
    f32x4 ns[G::MT_N];
    const float* bias = cur + S::FC * 256;
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t) ns[t] = ld4(bias + 16 * t + 4 * g);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int t = 0; t < G::MT_N; ++t) {
        u32x4 w[3];
        planes_at(cw + ((t * 2 + p) * 3) * 256, lane, w);
        ns[t] = mfma_bf6(w, hx[p], ns[t]);
      }
    __builtin_amdgcn_s_setprio(0);
    // tanh / new schedule / lane-local first-argmaxes against the schedule row
    float bn_v = -INFINITY, bs_v = -INFINITY;
    int bn_i = 0, bs_i = 0;
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hh = 16 * t + 4 * g + r;
        if (hh < H) {
          const float s0 = sv[t][r];
          const float nv = s0 + 4.0f * tanh_fast(ns[t][r]);
          ns[t][r] = nv;
          if (nv > bn_v) {  // strict: first maximum wins (list.index(max(...)))
            bn_v = nv;
            bn_i = hh;
          }
          if (s0 > bs_v) {
            bs_v = s0;
            bs_i = hh;
          }
        } else {
          ns[t][r] = 0.f;
        }
      }
    // Disc1's new-schedule half: hd += Wd1[:, H^2 + cH ...] . ns_c
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int p = 0; p < S::NPN; ++p) {
      float v[8];
      pair8(ns[2 * p], 2 * p + 1 < G::MT_N ? ns[2 * p + 1] : zero4, v);
      u32x4 x[3];
      split8(v, x);
#pragma unroll
      for (int mt = 0; mt < G::MT_G; ++mt) {
        u32x4 w[3];
        planes_at(cw + (S::FC2 + (mt * S::NPN + p) * 3) * 256, lane, w);
        hd[mt] = mfma_bf6(w, x, hd[mt]);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    k3_targets(c, bn_v, bn_i, bs_v, bs_i);
    advance();
  }

  // the wave's targets: its windows' rows are contiguous in gen_t / final_t
  {
    const long base = blk * 16 * G::C;
    const long n = (a.B - blk * 16 < 16 ? a.B - blk * 16 : 16) * (long)G::C;
    for (int k = 4 * lane; k < 16 * G::C; k += 256) {
#pragma unroll
      for (int arr = 0; arr < 2; ++arr) {
        int v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int idx = k + e, w = idx / G::C, c = idx - w * G::C;
          v[e] = tg[(arr * G::C + c) * 16 + w];
        }
        int* dst = (arr ? a.final_t : a.gen_t) + base + k;
        if (blk < nblk && k + 3 < n) {
          *reinterpret_cast<int4*>(dst) = make_int4(v[0], v[1], v[2], v[3]);
        } else if (blk < nblk) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (k + e < n) dst[e] = v[e];
        }
      }
    }
  }

  // ---- Disc2 + softmax + gate (PreGANPlus.py:87) ----
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
    a.probs[2 * b] = p0;
    a.probs[2 * b + 1] = p1;
    a.keep[b] = p0 > p1 ? 1 : 0;
  }
}

template <int H, int NW>
hipError_t launch_nw(const FwdArgs& a, hipStream_t st) {
  using S = GanS<H>;
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gan_split_kernel<H, NW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, S::lds_bytes(NW));
    return true;
  }();
  (void)attr;
  const long nblk = (a.B + 15) / 16;
  const int grid = (int)((nblk + NW - 1) / NW);
  gan_split_kernel<H, NW><<<grid, NW * 64, S::lds_bytes(NW), st>>>(a);
  return hipGetLastError();
}
template <int H>
hipError_t launch_t(const FwdArgs& a, hipStream_t st) {
  if constexpr (gan_split<H>()) {
    if ((a.B + 15) / 16 < kSSmallBlocks) return launch_nw<H, kSWavesSmall>(a, st);
    return launch_nw<H, kSWaves>(a, st);
  }
  return hipErrorInvalidValue;
}

template <int H>
hipError_t derive_t(const float* frags, float* planes, hipStream_t st) {
  if constexpr (gan_split<H>()) {
    const long triples = GanS<H>::FRAGS / 3;
    gan_split_derive_kernel<H><<<(int)((triples + 3) / 4), 256, 0, st>>>(frags, planes);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

}  // namespace

long gan_split_floats(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_split<h>() ? GanS<h>::SIZE : 0;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

hipError_t launch_gan_split_derive(int H, const float* frags, float* planes, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return derive_t<h>(frags, planes, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_split(const FwdArgs& a, hipStream_t st) {
  switch (a.H) {
#define CASE(h) \
  case h:       \
    return launch_t<h>(a, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
