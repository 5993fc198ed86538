// pgp_gan.hip — K3: generator + discriminator + decision argmaxes
// (models.py:118-151, 258-291; PreGANPlus.py:84-105; stats/Stats.py:162-166).
//
// One workgroup = 16 waves = 256 windows (16 per wave, on lanes).  The weights
// (3 MB at H=50) stream once per workgroup through a 2-slot LDS ring
// (global_load_lds), shared by all 16 waves, in three phases:
//   1. Gen1, embedding columns        hg  = W1[:, :2H] . vec(emb)
//   2. one pass over the schedule     hg += W1[:, 2H:] . vec(s);  hd = Wd1[:, :H^2] . vec(s)
//      (Gen1 and the schedule half of Disc1 share the B operand)
//   3. per container row c            ns_c = s_c + 4 tanh(W2[c] . hg + b2[c])   (Gen2)
//                                      gen_target[c] = first-argmax(ns_c), final_target[c] = first-argmax(s_c)
//                                      hd += Wd1[:, H^2 + cH : H^2 + (c+1)H] . ns_c  (Disc1, new-schedule half)
// so the new schedule never leaves registers.  Then Disc2 + softmax + gate.
// LeakyReLU(True) in Gen/Disc has slope 1.0 (identity), so no activation is applied.
#include <type_traits>

#include "pgp_device.hpp"

namespace pgp {
namespace {

// Geometry and schedule (alternatives A/B-timed in DESIGN.md §12, not kept as
// build switches): 16 waves per workgroup (16 windows each); kQC schedule
// k-blocks (16 columns each) per ring chunk; kChunkG caps a phase-3 ring chunk
// (1-KiB groups), which sets the containers per chunk (one barrier per chunk);
// the per-container MFMA loops run at wave priority 1, the tanh / argmax VALU
// at 0; Disc1's new-schedule half skips the MFMAs whose whole k slice is
// padding rows (at H = 50 the last tile's e = 2, 3 steps: 8 of 128 MFMAs per
// container); a Gen2 last row tile with at most kTailMax real rows runs on
// VALU; with one or two containers per chunk the second half of the waves
// starts each chunk kGanSleep x CPC x 64 cycles late (A/B at H = 50, two
// containers per chunk: 24 / 48 / 96 / 127 units 0.788 / 0.788 / 0.793 /
// 0.798 ms against 0.800 without; profiles/r03/c2ab/k3_stagger2.txt).
constexpr int kGanWaves = 16;  // waves per workgroup at large batches (kGanWavesSmall below)
constexpr int kQC = 8;
constexpr int kChunkG = 65;
constexpr int kTailMax = 2;
constexpr int kGanSleep = 24;
// (A/B on the online interval's 1,024 windows, 1 / 2 / 4 / 8 / 16 waves:
// 1.031 / 1.034 / 1.026 / 1.043 / 1.089 ms, profiles/r05/k3_small/)
constexpr int kGanWavesSmall = 4;
constexpr long kGanSmallBlocks = 16L * 256;  // below 64 K windows (16 x 256 blocks of 16), kGanWavesSmall

template <int P>
__device__ __forceinline__ void gan_prio() {
  __builtin_amdgcn_s_setprio(P);
}

template <int H, int NW = kGanWaves>
struct GanGeo {
  using G = Geo<H>;
  static constexpr int NQC = cdiv(G::SQ, kQC);
  // CPC containers per ring chunk (CPC divides C), their weight groups plus one
  // group holding their Gen2 biases (copied from the GAN table: the bias is the
  // accumulator's initial value, so an LDS read instead of a global load that
  // the first MFMA would wait for, together with the prefetched schedule row)
  static constexpr int BIAS_F = G::MT_N * 16;  // bias floats per container
  static constexpr int mx(int x, int y) { return x > y ? x : y; }
  using TgtT = typename std::conditional<(G::C < 128), signed char, short>::type;
  static constexpr int TGT = 2 * G::C * 16;  // target entries per wave
  static constexpr int lds_bytes(int cpc) {
    return 2 * mx(G::GE_G, mx(kQC * G::GS_G, cpc * G::GC_G + 1)) * G::FQ * 4 + NW * TGT * (int)sizeof(TgtT);
  }
  static constexpr int cpc() {
    int best = 1;
    for (int c = 1; c * G::GC_G + 1 <= kChunkG; ++c)
      if (G::C % c == 0 && c * BIAS_F <= 256 && lds_bytes(c) <= 160 * 1024) best = c;
    return best;
  }
  static constexpr int CPC = cpc();
  static constexpr int NCHUNK = 1 + NQC + G::C / CPC;
  static constexpr int SLOT_G = mx(G::GE_G, mx(kQC * G::GS_G, CPC * G::GC_G + 1));
  static constexpr int SLOT = SLOT_G * G::FQ;
  // per-wave container targets (gen | final) as [2][C][16 windows] of TgtT:
  // int8 (C < 128) or int16, flushed row-contiguous at the end (no scattered
  // 4-byte stores in the loop)
  static constexpr int LDS_BYTES = lds_bytes(CPC);
  // chunk k -> (global source, groups)
  PGP_DEV static void chunk(int k, const float* frags, const float** src, int* ng) {
    if (k == 0) {
      *src = frags + G::OFF_GE;
      *ng = G::GE_G;
    } else if (k <= NQC) {
      const int q0 = (k - 1) * kQC;
      *src = frags + G::OFF_GS + (long)q0 * G::GS_G * G::FQ;
      *ng = (G::SQ - q0 < kQC ? G::SQ - q0 : kQC) * G::GS_G;
    } else {
      *src = frags + G::OFF_GC + (long)(k - 1 - NQC) * CPC * G::GC_G * G::FQ;
      *ng = CPC * G::GC_G;
    }
  }
};

__device__ __attribute__((aligned(8))) float k3_zero_pair[2];  // never written

template <int H, int NW>
__global__ __launch_bounds__(NW * 64) void gan_kernel(FwdArgs a) {
  using G = Geo<H>;
  using GG = GanGeo<H, NW>;
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
  using TgtT = typename GG::TgtT;
  TgtT* tg = reinterpret_cast<TgtT*>(smem + 2 * GG::SLOT) + wv * GG::TGT;  // this wave's targets

  float* cur = smem;
  float* nxt = smem + GG::SLOT;
  int next = 1;
  {
    const float* src;
    int ng;
    GG::chunk(0, a.frags, &src, &ng);
    dma_groups(src, cur, ng, wv, NW, lane);
  }
  auto issue = [&]() {
    if (next < GG::NCHUNK) {
      const float* src;
      int ng;
      GG::chunk(next, a.frags, &src, &ng);
      dma_groups(src, nxt, ng, wv, NW, lane);
      if (next > GG::NQC)  // a container chunk: its biases after its groups (G_SIZE pads the last)
        dma_groups(gt + G::G_B2 + (long)(next - 1 - GG::NQC) * GG::CPC * GG::BIAS_F, nxt + ng * 256, 1,
                   (wv + ng) % NW, NW, lane);
    }
  };
  auto advance = [&]() {
    __syncthreads();
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
  f32x4 be[G::EQ];
#pragma unroll
  for (int q = 0; q < G::EQ; ++q) be[q] = valid ? ld4(ew + 16 * q + 4 * g) : zero4;
  __syncthreads();
  issue();

  // ---- phase 1: Gen1, embedding columns ----
  // (MFMA order: consecutive ones on different accumulators — dependent latency 40 > 32 issue)
#pragma unroll
  for (int q = 0; q < G::EQ; ++q)
#pragma unroll
    for (int m0 = 0; m0 < G::MT_G; m0 += 2) {
      f32x4 w[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) w[i] = ld4(cur + ((m0 + i) * G::EQ + q) * 256 + lane * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i) hg[m0 + i] = mfma(w[i][e], be[q][e], hg[m0 + i]);
    }

  // ---- phase 2: schedule pass (Gen1 + Disc1 schedule half) ----
  f32x4 bq[kQC];
#pragma unroll
  for (int i = 0; i < kQC; ++i) {
    const int idx = 16 * i + 4 * g;
    bq[i] = (valid && idx < G::H2) ? ld4(sw + idx) : zero4;
  }
  advance();
  for (int qc = 0; qc < GG::NQC; ++qc) {
    f32x4 bn[kQC];
#pragma unroll
    for (int i = 0; i < kQC; ++i) {
      const int idx = 16 * ((qc + 1) * kQC + i) + 4 * g;
      bn[i] = (valid && idx < G::H2) ? ld4(sw + idx) : zero4;
    }
#pragma unroll
    for (int i = 0; i < kQC; ++i) {
      if (qc * kQC + i < G::SQ) {
#pragma unroll
        for (int mt = 0; mt < G::MT_G; ++mt) {
          const f32x4 wg = ld4(cur + (i * G::GS_G + mt) * 256 + lane * 4);
          const f32x4 wd = ld4(cur + (i * G::GS_G + G::MT_G + mt) * 256 + lane * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            hg[mt] = mfma(wg[e], bq[i][e], hg[mt]);
            hd[mt] = mfma(wd[e], bq[i][e], hd[mt]);
          }
        }
      }
    }
    advance();
#pragma unroll
    for (int i = 0; i < kQC; ++i) bq[i] = bn[i];
  }

  // ---- phase 3: per container row ----
  // a lane's 4 row values 16t+4g+{0..3} as two 8-byte loads (H even: every pair is
  // aligned and lies wholly inside or wholly past the row)
  static_assert(H % 2 == 0, "row pairs");
  // (branch-free: the address is selected, a zero pair outside the row, so the
  // loaded values are not touched, nor waited for, until the next container)
  auto load_row = [&](int c, float (&v)[G::MT_N][4]) {
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const int hh = 16 * t + 4 * g + r;
        const float* src = (valid && hh < H && c < G::C) ? sw + c * H + hh : k3_zero_pair;
        const float2 p = *reinterpret_cast<const float2*>(src);
        v[t][r] = p.x;
        v[t][r + 1] = p.y;
      }
  };
  // Gen2's last row tile at H = 50 holds 2 real rows of 16: those rows are VALU
  // dot products (k split over the lane groups, summed across them) issued in
  // the shadow of the other tiles' MFMAs, instead of 16 MFMAs per container
  constexpr int NTR = H - 16 * (G::MT_N - 1);
  constexpr bool TAIL = G::MT_N > 1 && NTR <= kTailMax;
  constexpr int MTM = TAIL ? G::MT_N - 1 : G::MT_N;  // Gen2 tiles on MFMA
  float sv[G::MT_N][4];
  load_row(0, sv);
  // Gen2 of container c from its chunk groups cw: ns = b2[c] + W2[c] . hg (the
  // VALU tail rows into racc)
  auto gen2 = [&](int c, const float* cw, const float* chunk, f32x4 (&ns)[G::MT_N], float (&racc)[kTailMax]) {
    const float* bias = chunk + GG::CPC * G::GC_G * G::FQ + (c % GG::CPC) * GG::BIAS_F;
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t) ns[t] = ld4(bias + 16 * t + 4 * g);
#pragma unroll
    for (int r = 0; r < kTailMax; ++r) racc[r] = 0.f;
    gan_prio<1>();
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
#pragma unroll
      for (int t0 = 0; t0 < MTM; t0 += 2) {  // two accumulators alternate: no dependent-issue stall
        f32x4 w[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          if (t0 + i < MTM) w[i] = ld4(cw + ((t0 + i) * 4 + q4) * 256 + lane * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            if (t0 + i < MTM) ns[t0 + i] = mfma(w[i][e], hg[q4][e], ns[t0 + i]);
      }
      if (TAIL) {  // row r of the last tile: its A fragment column sits on lane 16g + r
#pragma unroll
        for (int r = 0; r < NTR; ++r) {
          const f32x4 rw = ld4(cw + (MTM * 4 + q4) * 256 + (16 * g + r) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) racc[r] = fmaf(rw[e], hg[q4][e], racc[r]);
        }
      }
    }
    gan_prio<0>();
  };
  // the rest of container c: tanh / new schedule / both first-argmaxes against
  // the schedule row sv, Disc1's new-schedule half, the targets
  // the rest of container c in three parts: v1 (tanh / new schedule / the
  // lane-local first-argmaxes against the schedule row sv), m2 (Disc1's
  // new-schedule half), v2 (the cross-lane argmaxes and the targets)
  struct Arg {
    float bn_v, bs_v;
    int bn_i, bs_i;
  };
  auto finish_v1 = [&](f32x4 (&ns)[G::MT_N], float (&racc)[kTailMax], const float (&sv)[G::MT_N][4]) {
    if (TAIL) {  // lanes g = 0 hold rows 16 MTM + r; the other groups' rows are >= H
#pragma unroll
      for (int r = 0; r < NTR; ++r) ns[MTM][r] += xsum(racc[r], true);
    }
    Arg x{-INFINITY, -INFINITY, 0, 0};
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int hh = 16 * t + 4 * g + r;
        if (hh < H) {
          const float s0 = sv[t][r];
          const float nv = s0 + 4.0f * tanh_fast(ns[t][r]);
          ns[t][r] = nv;
          if (nv > x.bn_v) {  // strict: first maximum wins (list.index(max(...)))
            x.bn_v = nv;
            x.bn_i = hh;
          }
          if (s0 > x.bs_v) {
            x.bs_v = s0;
            x.bs_i = hh;
          }
        } else {
          ns[t][r] = 0.f;
        }
      }
    return x;
  };
  auto finish_m2 = [&](const float* cw, const f32x4 (&ns)[G::MT_N]) {
    gan_prio<1>();
#pragma unroll
    for (int q4 = 0; q4 < G::MT_N; ++q4)
#pragma unroll
      for (int m0 = 0; m0 < G::MT_G; m0 += 2) {
        f32x4 w[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) w[i] = ld4(cw + (G::GC_G2 + (m0 + i) * G::MT_N + q4) * 256 + lane * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (16 * q4 + e < H)  // k = 16 q4 + 4g + e: all lanes' rows >= H are zero
#pragma unroll
            for (int i = 0; i < 2; ++i) hd[m0 + i] = mfma(w[i][e], ns[q4][e], hd[m0 + i]);
      }
    gan_prio<0>();
  };
  auto finish_v2 = [&](int c, Arg x) {
    float bn_v = x.bn_v, bs_v = x.bs_v;
    int bn_i = x.bn_i, bs_i = x.bs_i;
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
      tg[c * 16 + j] = (TgtT)bn_i;
      tg[(G::C + c) * 16 + j] = (TgtT)bs_i;
    }
  };
  auto copy_row = [&](float (&d)[G::MT_N][4], const float (&sr)[G::MT_N][4]) {
#pragma unroll
    for (int t = 0; t < G::MT_N; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) d[t][r] = sr[t][r];
  };
  f32x4 ns[G::MT_N];
  float racc[kTailMax];
  for (int c = 0; c < G::C; ++c) {
    const float* cw = cur + (c % GG::CPC) * G::GC_G * G::FQ;  // this container's groups
    float svn[G::MT_N][4];
    load_row(c + 1, svn);
    // stagger: the second half of the waves (two per SIMD) starts each chunk
    // interval late, so its tanh / argmax VALU phases meet the first half's
    // MFMAs instead of every wave reaching them together (at most two
    // containers per chunk: with 4-8, at H <= 32, it cost the fleet 0.3 %)
    if (NW > 1 && GG::CPC <= 2 && c % GG::CPC == 0 && wv >= NW / 2) __builtin_amdgcn_s_sleep(kGanSleep * GG::CPC);
    gen2(c, cw, cur, ns, racc);
    const Arg x = finish_v1(ns, racc, sv);
    finish_m2(cw, ns);
    finish_v2(c, x);
    if ((c + 1) % GG::CPC == 0) advance();
    copy_row(sv, svn);
  }

  // the wave's targets: its windows' rows are contiguous in gen_t / final_t
  // ([B][C]), written 4 ints per lane (the wave's own LDS region: no barrier)
  {
    const long base = blk * 16 * G::C;
    const long n = (a.B - blk * 16 < 16 ? a.B - blk * 16 : 16) * (long)G::C;  // valid elements
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
  using GG = GanGeo<H, NW>;
  static_assert(GG::LDS_BYTES <= 160 * 1024, "K3 LDS");
  static_assert(Geo<H>::C < 32768, "int8 / int16 targets");
  static bool attr = [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gan_kernel<H, NW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, GG::LDS_BYTES);
    return true;
  }();
  (void)attr;
  const long nblk = (a.B + 15) / 16;
  const int grid = (int)((nblk + NW - 1) / NW);
  gan_kernel<H, NW><<<grid, NW * 64, GG::LDS_BYTES, st>>>(a);
  return hipGetLastError();
}
// Small batches: 16 waves per workgroup put 256 windows on ONE CU (1,024
// windows: 4 CUs); kGanWavesSmall waves per workgroup spread them over more
// CUs, each workgroup streaming the weights through its own LDS ring.  Every
// wave computes its 16 windows exactly as before (same operands, same MFMA
// order): the outputs are the same bits.
template <int H>
hipError_t launch(const FwdArgs& a, hipStream_t st) {
  const long nblk = (a.B + 15) / 16;
  if (nblk < kGanSmallBlocks) return launch_nw<H, kGanWavesSmall>(a, st);
  return launch_nw<H, kGanWaves>(a, st);
}

}  // namespace

hipError_t launch_gan(const FwdArgs& a, hipStream_t st) {
  // the split form at every batch (its own 4-wave workgroups below 64 K
  // windows): a window's outputs do not depend on the batch it arrives in
  if (a.ganb != nullptr && gan_split_floats(a.H) > 0)
    return launch_gan_split(a, st);
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
