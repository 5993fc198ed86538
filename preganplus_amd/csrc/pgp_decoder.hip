// pgp_decoder.hip — K2b: anomaly + prototype decoders (models.py:359-370) as
// one GEMM [B x 3H^2] . [3H^2 x 4H], fused with detect/embed
// (PreGANPlus.py:119-131) and get_classes (utils.py:102-109).
//
// One workgroup = 16 waves = 256 windows (16 per wave, on lanes).  The K loop
// runs over (host, step) chunks of the latent; each chunk's weight fragments
// (MT_O x KQ_D groups) are streamed into a 2-slot LDS ring by global_load_lds
// and shared by all 16 waves; each wave's latent B operands for the next chunk
// are prefetched into registers while the current chunk computes.
// Output rows n = 4*host + {logit0, logit1, proto0, proto1} put a host's four
// values in one lane's accumulator, so the epilogue is lane-local.
#include "pgp_device.hpp"

namespace pgp {
namespace {

constexpr int kDecWaves = 16;

// CPS (host, step) chunks per ring slot: at small H one chunk is only a few
// groups (4 KB, 16 MFMAs per wave at H = 16), so a barrier per chunk dominated;
// chunks are grouped up to 16 groups per slot (CPS divides the chunk count;
// the latent B registers of one slot are prefetched a slot ahead).
template <int H>
constexpr int dec_cps() {
  int best = 1;
  for (int c = 1; c * Geo<H>::DEC_G <= 16; ++c)
    if ((H * kWindow) % c == 0) best = c;
  return best;
}

template <int H>
struct DecLds {
  static constexpr int CPS = dec_cps<H>();
  static constexpr int SLOT = CPS * Geo<H>::DEC_G * Geo<H>::FQ;
  static constexpr int TAB = Geo<H>::t_size(kMaxProtos);
  static constexpr int TOTAL = 2 * SLOT + TAB;
};

template <int H>
__global__ __launch_bounds__(kDecWaves * 64, H <= 16 ? 8 : 1) void decoder_kernel(FwdArgs a) {
  using G = Geo<H>;
  using L = DecLds<H>;
  __shared__ __attribute__((aligned(16))) float smem[L::TOTAL];
  float* tab = smem + 2 * L::SLOT;
  const int tsz = G::t_size(a.K);
  for (int i = threadIdx.x; i < tsz; i += blockDim.x) tab[i] = a.tab[i];

  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long blk = (long)blockIdx.x * kDecWaves + wv;
  const long nblk = (a.B + 15) / 16;
  const bool active = blk < nblk;
  const float* wdec = a.frags + G::OFF_DEC;
  const float* lat = a.lat + (active ? blk : 0) * G::LAT_BLK;
  constexpr int NCH = H * kWindow;

  constexpr int CPS = L::CPS, SG = CPS * G::DEC_G;  // chunks, groups per slot
  float* cur = smem;
  float* nxt = smem + L::SLOT;
  dma_groups(wdec, cur, SG, wv, kDecWaves, lane);
  // latent B operands one slot (CPS chunks) ahead: at small H a single chunk is
  // too little work to cover the HBM latency of the next one
  // chunk c's B operands (the latent layout of pgp_layout.hpp LAT_FG: 16-byte
  // loads for the full groups of 4 k-steps)
  auto load_b = [&](int c, bool ok, float (&v)[G::KS_D]) {
    const float* lc = lat + (long)c * G::KS_D * 64;
#pragma unroll
    for (int q = 0; q < G::LAT_FG; ++q) {
      const f32x4 t = ok ? ld4(lc + q * 256 + lane * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = t[e];
    }
#pragma unroll
    for (int r = 0; r < G::KS_D % 4; ++r) v[4 * G::LAT_FG + r] = ok ? lc[G::LAT_FG * 256 + r * 64 + lane] : 0.f;
  };
  float b[CPS][G::KS_D];
#pragma unroll
  for (int u = 0; u < CPS; ++u) load_b(u, active, b[u]);
  __syncthreads();
  if (CPS < NCH) dma_groups(wdec + (long)SG * G::FQ, nxt, SG, wv, kDecWaves, lane);

  f32x4 acc[G::MT_O];
#pragma unroll
  for (int mt = 0; mt < G::MT_O; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int MTM = G::MT_O;  // output tiles (the VALU tail-row form spilled: DESIGN §12)

#pragma unroll 1
  for (int c0 = 0; c0 < NCH; c0 += CPS) {
    float bn[CPS][G::KS_D];
    const bool pre = active && (c0 + CPS < NCH);
#pragma unroll
    for (int u = 0; u < CPS; ++u) load_b(c0 + CPS + u, pre, bn[u]);
#pragma unroll
    for (int sub = 0; sub < CPS; ++sub) {
      const float* A = cur + sub * G::DEC_G * G::FQ;
      // consecutive MFMAs go to different accumulators (dependent-accumulator
      // latency 40 cyc > 32 cyc issue): A fragments of half the output tiles at a time
      constexpr int AMAX = G::MT_O >= 16 ? 4 : H <= 16 ? 2 : 7;  // A fragments live (VGPR budget)
      constexpr int NGRP = (MTM + AMAX - 1) / AMAX;
      constexpr int MH = (MTM + NGRP - 1) / NGRP;
#pragma unroll
      for (int q4 = 0; q4 < G::KQ_D; ++q4) {
#pragma unroll
        for (int m0 = 0; m0 < MTM; m0 += MH) {
          f32x4 av[MH];
#pragma unroll
          for (int i = 0; i < MH; ++i)
            if (m0 + i < MTM) av[i] = ld4(A + ((m0 + i) * G::KQ_D + q4) * 256 + lane * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (4 * q4 + e < G::KS_D)
#pragma unroll
              for (int i = 0; i < MH; ++i)
                if (m0 + i < MTM) acc[m0 + i] = mfma(av[i][e], b[sub][4 * q4 + e], acc[m0 + i]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < CPS; ++u)
#pragma unroll
      for (int s = 0; s < G::KS_D; ++s) b[u][s] = bn[u][s];
    __syncthreads();
    float* t = cur;
    cur = nxt;
    nxt = t;
    if (c0 + 2 * CPS < NCH) dma_groups(wdec + (long)(c0 + 2 * CPS) * G::DEC_G * G::FQ, nxt, SG, wv, kDecWaves, lane);
  }

  // ---- epilogue: bias, sigmoid, detect, embed, classify ----
  const long bw = blk * 16 + j;
  const bool valid = active && bw < a.B;
  int anyf = 0;
  const float* P = tab + G::T_PROTO;
#pragma unroll
  for (int mt = 0; mt < G::MT_O; ++mt) {
    const int host = 4 * mt + g;
    const f32x4 v = acc[mt] + ld4(tab + G::T_DEC + 16 * mt + 4 * g);
    if (host < H) {
      const float l0 = v[0], l1 = v[1];
      const float p0 = __builtin_amdgcn_rcpf(1.0f + __expf(-v[2])), p1 = __builtin_amdgcn_rcpf(1.0f + __expf(-v[3]));
      const bool an = l1 > l0;  // torch.argmax: ties -> index 0
      const float e0 = an ? p0 : 0.f, e1 = an ? p1 : 0.f;
      int cl = -1;
      if (!(e0 == 0.f && e1 == 0.f)) {
        float best = INFINITY;
        for (int k = 0; k < a.K; ++k) {
          const float d0 = e0 - P[2 * k], d1 = e1 - P[2 * k + 1];
          const float dist = (d0 * d0 + d1 * d1) * 0.5f;  // torch.mean over PROTO_DIM = 2
          if (dist < best) {                              // np.argmin: first minimum
            best = dist;
            cl = k;
          }
        }
      }
      anyf |= an ? 1 : 0;
      if (valid) {
        const long o = (bw * H + host) * 2;
        a.logits[o] = l0;
        a.logits[o + 1] = l1;
        a.protos[o] = p0;
        a.protos[o + 1] = p1;
        a.cls[bw * H + host] = cl;
        a.emb[bw * G::EP + 2 * host] = e0;
        a.emb[bw * G::EP + 2 * host + 1] = e1;
      }
    }
  }
  {  // or over the 4 lane groups (the row swaps of xsum)
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)anyf, (unsigned)anyf, false, false);
    const int a16 = (int)(r[0] | r[1]);
    const auto q = __builtin_amdgcn_permlane32_swap((unsigned)a16, (unsigned)a16, false, false);
    anyf = (int)(q[0] | q[1]);
  }
  if (valid && g == 0) a.any_anom[bw] = anyf;
}

// ---------------------------------------------------------------------------
// Split-bf16 form (H = 32, 50): the same GEMM on v_mfma_f32_16x16x32_bf16.
// Every fp32 operand is split exactly into three bf16 parts, x = x0 + x1 + x2
// (x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1); each residual is
// exact in fp32), and w . x = sum over i + j <= 2 of w_i . x_j: six bf16 MFMAs
// whose products are exact in fp32 and accumulate in fp32; the dropped terms
// are below 2^-26 of |w x| (tools/micro/bf16_split.hip measures the result
// against fp64 beside the fp32 MFMA).  A bf16 MFMA does 16x the fp32 one's
// flops per cycle, so six of them cost 3/8 of the fp32 contraction.
// The weights' three planes are derived once per weight load from the fp32
// fragments (dec_split_kernel, lane-local: a lane's 8 k-steps of a 16x16x32
// fragment are its two fp32 groups of 4); the latent is split in registers as
// it is loaded (VALU, shared by all MT_O output tiles).
template <int H>
struct DecB {
  using G = Geo<H>;
  static constexpr int NB = cdiv(G::KQ_D, 2);    // 8-k-step blocks per (host, step) chunk
  static constexpr int FRC = NB * G::MT_O * 3;   // 1-KiB fragments per chunk: [blk][mt][plane]
  static constexpr long SIZE = (long)H * kWindow * FRC * 256;  // floats (bf16 pairs)
  static constexpr int SLOT = FRC * 256;         // one chunk per LDS slot
  static constexpr int TOTAL = 2 * SLOT + G::MT_O * 16 + 2 * kMaxProtos;
};
template <int H>
constexpr bool dec_split() {
  return H >= 32 && DecB<H>::TOTAL * 4 <= 160 * 1024;
}

// fp32 decoder fragments -> bf16 planes [chunk][blk][mt][plane][lane][8]
template <int H>
__global__ __launch_bounds__(256) void dec_split_kernel(const float* __restrict__ wdec, float* __restrict__ out) {
  using G = Geo<H>;
  using D = DecB<H>;
  const long f = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // over [chunk][blk][mt]
  const int lane = threadIdx.x & 63;
  if (f >= (long)H * kWindow * D::NB * G::MT_O) return;
  const int mt = (int)(f % G::MT_O);
  const long r = f / G::MT_O;
  const int blk = (int)(r % D::NB);
  const long c = r / D::NB;
  float v[8];
#pragma unroll
  for (int hq = 0; hq < 2; ++hq) {
    const int q4 = 2 * blk + hq;
    const f32x4 t = q4 < G::KQ_D ? ld4(wdec + ((c * G::DEC_G) + mt * G::KQ_D + q4) * 256 + lane * 4)
                                 : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * hq + e] = t[e];
  }
  u32x4 p[3];
  split8(v, p);
#pragma unroll
  for (int k = 0; k < 3; ++k) *reinterpret_cast<u32x4*>(out + (f * 3 + k) * 256 + lane * 4) = p[k];
}

// TW window tiles (16 windows each) per wave, 16 / TW waves per workgroup (256
// windows, as decoder_kernel): each weight plane read from LDS feeds TW MFMAs
// (A/B, C2 at H = 50, 5 interleaved rounds: TW = 2 5.90 ms against TW = 1
// 6.14 ms; profiles/r06/c2ab/abdec.txt)
#ifndef PGP_DEC_TW
#define PGP_DEC_TW 2
#endif
constexpr int kDecTW = PGP_DEC_TW;
// latent chunks in flight ahead of the one being contracted (registers)
#ifndef PGP_DEC_PF
#define PGP_DEC_PF 1
#endif
constexpr int kDecPF = PGP_DEC_PF;
// weight planes read PGP_DEC_PIPE (block, tile) steps ahead of their MFMAs
// (0: where the compiler puts them; A/B, C2 at H = 50, 5 interleaved rounds:
// K2b 1.035 -> 0.989 ms at 1, profiles/r06/c2/ab_decoder_pipe.txt)
#ifndef PGP_DEC_PIPE
#define PGP_DEC_PIPE 1
#endif
constexpr int kDecPipe = PGP_DEC_PIPE;

template <int H, int TW>
__global__ __launch_bounds__(kDecWaves / TW * 64, 1) void decoder_split_kernel(FwdArgs a) {
  using G = Geo<H>;
  using D = DecB<H>;
  constexpr int NWD = kDecWaves / TW;
  __shared__ __attribute__((aligned(16))) float smem[D::TOTAL];
  float* tdec = smem + 2 * D::SLOT;  // decoder bias [MT_O * 16]
  float* P = tdec + G::MT_O * 16;    // prototypes [K][2]
  for (int i = threadIdx.x; i < G::MT_O * 16; i += blockDim.x) tdec[i] = a.tab[G::T_DEC + i];
  for (int i = threadIdx.x; i < 2 * a.K; i += blockDim.x) P[i] = a.tab[G::T_PROTO + i];

  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long blk0 = (long)blockIdx.x * kDecWaves + wv * TW;
  const long nblk = (a.B + 15) / 16;
  constexpr int NCH = H * kWindow;
  auto load_b = [&](int t, int c, bool ok, float (&v)[G::KS_D]) {
    const bool act = blk0 + t < nblk;
    const float* lc = a.lat + (act ? blk0 + t : 0) * G::LAT_BLK + (long)c * G::KS_D * 64;
    ok = ok && act;
#pragma unroll
    for (int q = 0; q < G::LAT_FG; ++q) {
      const f32x4 u = ok ? ld4(lc + q * 256 + lane * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = u[e];
    }
#pragma unroll
    for (int r = 0; r < G::KS_D % 4; ++r) v[4 * G::LAT_FG + r] = ok ? lc[G::LAT_FG * 256 + r * 64 + lane] : 0.f;
  };
  float* cur = smem;
  float* nxt = smem + D::SLOT;
  dma_groups(a.decb, cur, D::FRC, wv, NWD, lane);
  float b[TW][G::KS_D], b1[TW][G::KS_D];
#pragma unroll
  for (int t = 0; t < TW; ++t) load_b(t, 0, true, b[t]);
  if constexpr (kDecPF > 1) {
#pragma unroll
    for (int t = 0; t < TW; ++t) load_b(t, 1, NCH > 1, b1[t]);
  }
  __syncthreads();
  if (NCH > 1) dma_groups(a.decb + (long)D::SLOT, nxt, D::FRC, wv, NWD, lane);

  f32x4 acc[TW][G::MT_O];
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int mt = 0; mt < G::MT_O; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    float bn[TW][G::KS_D];
#pragma unroll
    for (int t = 0; t < TW; ++t) load_b(t, c + kDecPF, c + kDecPF < NCH, bn[t]);
    // the planes of the next (block, tile) are read while this one's MFMAs
    // run (kDecPipe; without it the compiler waited for each read: one
    // lgkmcnt(0) per tile)
    auto planes = [&](int kb, int mt, u32x4 (&w)[3]) {
      const float* F = cur + ((kb * G::MT_O + mt) * 3) * 256 + lane * 4;
#pragma unroll
      for (int k = 0; k < 3; ++k) w[k] = *reinterpret_cast<const u32x4*>(F + k * 256);
    };
    constexpr int QN = D::NB * G::MT_O;  // (block, tile) steps of a chunk
    constexpr int PD = kDecPipe > 0 ? kDecPipe : 1;
    u32x4 wq[PD][3];
    if constexpr (kDecPipe > 0) {
#pragma unroll
      for (int q = 0; q < PD; ++q)
        if (q < QN) planes(q / G::MT_O, q % G::MT_O, wq[q]);
    }
#pragma unroll
    for (int kb = 0; kb < D::NB; ++kb) {
      u32x4 x[TW][3];
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 8 * kb + e < G::KS_D ? b[t][8 * kb + e] : 0.f;
        split8(v, x[t]);
      }
#pragma unroll
      for (int mt = 0; mt < G::MT_O; ++mt) {
        u32x4 w[3];
        if constexpr (kDecPipe > 0) {
          const int q = kb * G::MT_O + mt;
#pragma unroll
          for (int k = 0; k < 3; ++k) w[k] = wq[q % PD][k];
          if (q + PD < QN) planes((q + PD) / G::MT_O, (q + PD) % G::MT_O, wq[q % PD]);
          // keep the reads here, ahead of this tile's MFMAs (the scheduler
          // otherwise sinks them next to their use)
          __builtin_amdgcn_sched_barrier(0);
        } else {
          planes(kb, mt, w);
        }
#pragma unroll
        for (int t = 0; t < TW; ++t) acc[t][mt] = mfma_bf6(w, x[t], acc[t][mt]);
      }
    }
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int s = 0; s < G::KS_D; ++s) {
        if constexpr (kDecPF > 1) {
          b[t][s] = b1[t][s];
          b1[t][s] = bn[t][s];
        } else {
          b[t][s] = bn[t][s];
        }
      }
    __syncthreads();
    float* tmp = cur;
    cur = nxt;
    nxt = tmp;
    if (c + 2 < NCH) dma_groups(a.decb + (long)(c + 2) * D::SLOT, nxt, D::FRC, wv, NWD, lane);
  }

  // ---- epilogue: bias, sigmoid, detect, embed, classify (as decoder_kernel) ----
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const long blk = blk0 + t;
    const long bw = blk * 16 + j;
    const bool valid = blk < nblk && bw < a.B;
    int anyf = 0;
#pragma unroll
    for (int mt = 0; mt < G::MT_O; ++mt) {
      const int host = 4 * mt + g;
      const f32x4 v = acc[t][mt] + ld4(tdec + 16 * mt + 4 * g);
      if (host < H) {
        const float l0 = v[0], l1 = v[1];
        const float p0 = __builtin_amdgcn_rcpf(1.0f + __expf(-v[2])), p1 = __builtin_amdgcn_rcpf(1.0f + __expf(-v[3]));
        const bool an = l1 > l0;  // torch.argmax: ties -> index 0
        const float e0 = an ? p0 : 0.f, e1 = an ? p1 : 0.f;
        int cl = -1;
        if (!(e0 == 0.f && e1 == 0.f)) {
          float best = INFINITY;
          for (int k = 0; k < a.K; ++k) {
            const float d0 = e0 - P[2 * k], d1 = e1 - P[2 * k + 1];
            const float dist = (d0 * d0 + d1 * d1) * 0.5f;  // torch.mean over PROTO_DIM = 2
            if (dist < best) {                              // np.argmin: first minimum
              best = dist;
              cl = k;
            }
          }
        }
        anyf |= an ? 1 : 0;
        if (valid) {
          const long o = (bw * H + host) * 2;
          a.logits[o] = l0;
          a.logits[o + 1] = l1;
          a.protos[o] = p0;
          a.protos[o + 1] = p1;
          a.cls[bw * H + host] = cl;
          a.emb[bw * G::EP + 2 * host] = e0;
          a.emb[bw * G::EP + 2 * host + 1] = e1;
        }
      }
    }
    {
      const auto r = __builtin_amdgcn_permlane16_swap((unsigned)anyf, (unsigned)anyf, false, false);
      const int a16 = (int)(r[0] | r[1]);
      const auto q = __builtin_amdgcn_permlane32_swap((unsigned)a16, (unsigned)a16, false, false);
      anyf = (int)(q[0] | q[1]);
    }
    if (valid && g == 0) a.any_anom[bw] = anyf;
  }
}

template <int H>
hipError_t launch(const FwdArgs& a, hipStream_t st) {
  const long nblk = (a.B + 15) / 16;
  const int grid = (int)((nblk + kDecWaves - 1) / kDecWaves);
  if constexpr (dec_split<H>()) {
    if (a.decb != nullptr) {
      decoder_split_kernel<H, kDecTW><<<grid, kDecWaves / kDecTW * 64, 0, st>>>(a);
      return hipGetLastError();
    }
  }
  decoder_kernel<H><<<grid, kDecWaves * 64, 0, st>>>(a);
  return hipGetLastError();
}

template <int H>
hipError_t launch_split(const float* frags, float* decb, hipStream_t st) {
  if constexpr (dec_split<H>()) {
    const long nf = (long)H * kWindow * DecB<H>::NB * Geo<H>::MT_O;
    dec_split_kernel<H><<<(int)((nf + 3) / 4), 256, 0, st>>>(frags + Geo<H>::OFF_DEC, decb);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_decoder(const FwdArgs& a, hipStream_t st) {
  switch (a.H) {
#define CASE(h) \
  case h:       \
    return launch<h>(a, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

long decoder_split_floats(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return dec_split<h>() ? DecB<h>::SIZE : 0;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

hipError_t launch_decoder_split(int H, const float* frags, float* decb, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return launch_split<h>(frags, decb, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
