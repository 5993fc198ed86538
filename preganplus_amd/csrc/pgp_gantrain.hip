// pgp_gantrain.hip — the GAN step (PreGANPlus.py:60-81) over a batch of
// environments: Gen + Disc forward (models.py:118-151, 258-291), Disc BCE
// backward, then Gen BCE backward through the updated Disc — in five launches
// (plus the simulator between forward and Disc step, pgp_sim.hip):
//
//   gan_fwd_kernel     per 16-environment block: Gen1 over [e; s] and Disc1's
//                      schedule half in one pass over the input, Gen2 + tanh +
//                      ns = s + 4 tanh tile by tile with Disc1's ns half
//                      accumulated from each tile as it is produced, the head
//                      and softmax;
//   disc_head_kernel   BCE gradient toward the simulated label -> dOut, dDD;
//   outer_kernel       the Disc's weight / bias gradients (sums over the batch
//                      of outer products, written into G);
//   gan_gen_kernel     per block: Disc1 with the UPDATED Disc, head, BCE toward
//                      [0, 1] -> dDD', then tile by tile d ns = Disc1[:, ns]^T dDD',
//                      dY = 4 d ns (1 - tanh^2) and dHg = Gen2^T dY accumulated
//                      from each tile;
//   outer_kernel       the Gen's weight / bias gradients.
//
// A block is 16 environments on the lane columns of v_mfma_f32_16x16x4_f32
// (column j = lane & 15); its 8 waves split the contraction of each product
// (Gen1 / Disc1 chunks of 16 inputs, Gen2 / d ns output tiles of 16 rows) and
// combine their partial accumulators through LDS in wave order (deterministic).
// Accumulator registers feed the next product directly: a Gen2 tile (rows =
// schedule entries n, columns = environments) is the B operand of Disc1's ns
// half, a dY tile that of Gen2^T, so neither ns nor dY is re-read.  Weights are
// A operands read straight from the master P (L2-resident, 2.6 MB at H = 50).
// The weight gradients contract over the environments: each wave owns a 64 x 64
// block of one gradient matrix, one MFMA k-step per 4 environments, written
// once (no zero-fill, no split slabs).
//
// Per-environment scratch rows (TGeo::GS_*, one row of GS_SIZE floats each) keep
// what the later launches read: emb (GS_X), [s; ns] (GS_Z), Hg, tanh, DD, the
// probabilities, dOut, dDD, dY, dHg.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pgp_device.hpp"
#include "pgp_gemm.hpp"
#include "pgp_train.hpp"

namespace pgp {
namespace {

constexpr int kGW = 8;     // waves per block workgroup (2 per SIMD)
constexpr int kHP = 68;    // LDS pitch of a [env][64] hidden array (bank spread)

// masked 16-byte loads select this ADDRESS (never written), so a prefetched
// value is not waited for at the select
__device__ __attribute__((aligned(16))) float gk_zero[16];

template <int H>
struct GanK {
  using G = TGeo<H>;
  static constexpr int HH = H * H, E2 = 2 * H, GIN = G::GIN, DIN = G::DIN;
  static constexpr int KE = (E2 + 15) / 16;   // emb chunks of 16 inputs
  static constexpr int KS = (HH + 15) / 16;   // schedule chunks = Gen2 / d ns output tiles
  static constexpr int KZ = (DIN + 15) / 16;  // [s; ns] chunks
  static_assert(HH % 4 == 0 && E2 % 4 == 0, "16-byte groups never straddle the end of a segment");
};

// the kGW waves' partial accumulators acc[4] (per lane) -> their sum in wave
// order, as out[tile t][lane][r] (row 16t + 4g + r, column lane & 15); red holds
// kGW * 4 * 256 floats; ends with a barrier
PGP_DEV void reduce4(float* red, const f32x4 (&acc)[4], int wv, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
    *reinterpret_cast<f32x4*>(red + ((wv * 4 + t) * 64 + lane) * 4) = acc[t];
  __syncthreads();
  for (int k = threadIdx.x; k < 4 * 256; k += blockDim.x) {
    float v = red[k];
#pragma unroll
    for (int w = 1; w < kGW; ++w) v += red[w * 1024 + k];
    red[k] = v;
  }
  __syncthreads();
}
// sum over the S <= kGanMaxSlices slices' partials p[q * stride] in slice
// order, every load issued before the first add (a loop of load-then-add
// waited one memory latency per slice); slices past S add nothing
PGP_DEV float slice_sum(const float* p, long stride, int S) {
  float t[16];
  // unconditional loads (slices past S re-read slice S - 1, unused): a
  // "load or 0" select per slice would branch around each load and wait once
  // per slice
#pragma unroll
  for (int q = 0; q < 16; ++q) t[q] = p[(q < S ? q : S - 1) * stride];
  float v = t[0];
#pragma unroll
  for (int q = 1; q < 16; ++q)
    if (q < S) v += t[q];
  return v;
}
// element k of reduce4's result -> (hidden row h, column j)
PGP_DEV void red_index(int k, int& h, int& j) {
  const int t = k >> 8, l = (k >> 2) & 63, r = k & 3;
  h = 16 * t + 4 * (l >> 4) + r;
  j = l & 15;
}

// the 2-way Disc head (models.py:146-151: Linear(64, 2), Softmax) of the block's
// 16 environments from DD in LDS (ddl[env][h]); p -> pl[env][2].  Thread-serial
// 64-term dot products.
PGP_DEV void head16(const float* ddl, const float* __restrict__ Pd2, const float* __restrict__ db2, float* zl,
                    float* pl) {
  const int t = threadIdx.x;
  if (t < 32) {
    const int j = t >> 1, o = t & 1;
    float z = 0.f;
    for (int h = 0; h < 64; ++h) z = fmaf(Pd2[o * 64 + h], ddl[j * kHP + h], z);
    zl[t] = z + db2[o];
  }
  __syncthreads();
  if (t < 16) {
    const float z0 = zl[2 * t], z1 = zl[2 * t + 1];
    const float mx = fmaxf(z0, z1), e0 = expf(z0 - mx), e1 = expf(z1 - mx);
    pl[2 * t] = e0 / (e0 + e1);
    pl[2 * t + 1] = e1 / (e0 + e1);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Gen + Disc forward of a block of 16 environments
// ---------------------------------------------------------------------------
// Arguments of the batched forward.  Embedding: `emb` [B][2H] is read, or,
// with `logits` set, run_model's masked embedding (PreGANPlus.py:129, the rule
// of embed_kernel) is formed from the detect forward's logits / protos [B][H][2]
// on the fly and written to `emb` (one launch fewer).  The split form's
// partials live after the rows in the workspace (gan_split_offsets).
struct GanFwdArgs {
  int B;
  const float* emb_in;
  float* emb_out;
  const float* logits;
  const float* protos;
  const float* sched;
  const float* Pg;
  const float* Pd;
  float* rows;
  float* ns_out;
  float* probs;
  float* part1;  // [nblk][S][2][1024]: phase-1 Gen1 | Disc1-schedule partials (PH 1)
  float* part2;  // [nblk][S][1024]: Disc1-ns partials (PH 2)
  float* dsum;   // [nblk][1024]: Disc1's schedule half (PH 2, slice 0)
};

// The forward of a block of 16 environments.  PH 0: the whole forward in one
// workgroup (8 waves splitting each contraction's chunks); PH 1 / PH 2: the
// same two contraction phases split over gridDim.y workgroups ("slices") per
// block, chunk c to wave (c mod S*kGW) of slice (c / kGW mod S), the slices'
// partials summed in slice order by the next launch (phase 1 -> PH 2's start;
// phase 2 -> gan_dd_head_kernel): at C3's 103 environments (7 blocks) one
// workgroup per block left most of the chip idle for the whole GAN step.
template <int H, int PH>
__global__ __launch_bounds__(kGW * 64) void gan_fwd_kernel(GanFwdArgs a) {
  using K = GanK<H>;
  using G = TGeo<H>;
  constexpr int HH = K::HH, E2 = K::E2, GIN = K::GIN, DIN = K::DIN;
  __shared__ __attribute__((aligned(16))) float red[kGW * 4 * 256];
  __shared__ __attribute__((aligned(16))) float hgl[16 * kHP];   // Hg [env][hidden]
  __shared__ __attribute__((aligned(16))) float dsl[16 * kHP];   // Disc1's schedule half, then DD
  __shared__ float zl[32], pl[32];
  const int B = a.B;
  const float* __restrict__ sched = a.sched;
  const float* __restrict__ Pg = a.Pg;
  const float* __restrict__ Pd = a.Pd;
  float* __restrict__ rows = a.rows;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  const int blk = blockIdx.x, sl = blockIdx.y, S = gridDim.y;
  const int c0 = sl * kGW + wv, cs = S * kGW;  // this wave's chunks: c0, c0 + cs, ...
  const long env = (long)blk * 16 + i;
  const bool eok = env < B;
  float* row = rows + (eok ? env : 0) * G::GS_SIZE;
  const float* W1 = Pg + G::G_W1;
  const float* D1 = Pd + G::D_W1;

  f32x4 aG[4], aD[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) aG[t] = aD[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (PH != 2) {
  // 1. Gen1 = W1 [e; s] and Disc1's schedule half D1[:, :HH] s, one pass over
  //    the input chunks (16 inputs each, k-step r <-> input 16c + 4g + r)
  for (int c = c0; c < K::KE; c += cs) {  // embedding chunks
    const int f = 16 * c + 4 * g;
    const bool fok = f < E2;
    f32x4 bv;
    if (a.logits) {  // PreGANPlus.py:129: a host's prototype pair where its logits' argmax is 1
      const f32x4 l = ld4(fok && eok ? a.logits + env * E2 + f : gk_zero);
      const f32x4 pr = ld4(fok && eok ? a.protos + env * E2 + f : gk_zero);
      const bool k0 = l[1] > l[0], k1 = l[3] > l[2];
      bv = f32x4{k0 ? pr[0] : 0.f, k0 ? pr[1] : 0.f, k1 ? pr[2] : 0.f, k1 ? pr[3] : 0.f};
      if (fok && eok) st4(a.emb_out + env * E2 + f, bv);
    } else {
      bv = ld4(fok && eok ? a.emb_in + env * E2 + f : gk_zero);
    }
    f32x4 wa[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) wa[t] = ld4(fok ? W1 + (long)(16 * t + i) * GIN + f : gk_zero);
    if (fok && eok) st4(row + G::GS_X + f, bv);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int t = 0; t < 4; ++t) aG[t] = mfma(wa[t][r], bv[r], aG[t]);
  }
  {  // schedule chunks, software-pipelined: chunk c + cs's operands are loaded
     // before chunk c's MFMAs (one latency per wave, not one per chunk)
    struct Ops {
      f32x4 bv, wa[4], wd[4];
    };
    auto load = [&](int c, Ops& o) {
      const int f = 16 * c + 4 * g;
      const bool fok = f < HH;
      o.bv = ld4(fok && eok ? sched + env * HH + f : gk_zero);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        o.wa[t] = ld4(fok ? W1 + (long)(16 * t + i) * GIN + E2 + f : gk_zero);
        o.wd[t] = ld4(fok ? D1 + (long)(16 * t + i) * DIN + f : gk_zero);
      }
    };
    // ping-pong buffers, no loop-carried copy (a copy would make the compiler
    // wait for the prefetch at once)
    Ops A, B;
    auto step = [&](int c, const Ops& cur) {
      const int f = 16 * c + 4 * g;
      if (f < HH && eok) st4(row + G::GS_Z + f, cur.bv);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          aG[t] = mfma(cur.wa[t][r], cur.bv[r], aG[t]);
          aD[t] = mfma(cur.wd[t][r], cur.bv[r], aD[t]);
        }
    };
    if (c0 < K::KS) load(c0, A);
    for (int c = c0; c < K::KS; c += 2 * cs) {
      load(c + cs < K::KS ? c + cs : c, B);
      step(c, A);
      if (c + cs >= K::KS) break;
      load(c + 2 * cs < K::KS ? c + 2 * cs : c + cs, A);
      step(c + cs, B);
    }
  }
  }
  if constexpr (PH == 1) {  // the slice's partials, in wave order
    float* out = a.part1 + ((long)blk * S + sl) * 2048;
    reduce4(red, aG, wv, lane);
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) out[k] = red[k];
    __syncthreads();  // red is read before the next reduction overwrites it
    reduce4(red, aD, wv, lane);
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) out[1024 + k] = red[k];
    return;
  } else if constexpr (PH == 2) {  // phase 1's slices summed in slice order
    const float* in = a.part1 + (long)blk * S * 2048;
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
      int h, j;
      red_index(k, h, j);
      float v = slice_sum(in + k, 2048, S);
      const float d = slice_sum(in + 1024 + k, 2048, S);
      v += Pg[G::G_B1 + h];
      hgl[j * kHP + h] = v;
      if (sl == 0) {
        if ((long)blk * 16 + j < B) rows[((long)blk * 16 + j) * G::GS_SIZE + G::GS_H + h] = v;
        a.dsum[(long)blk * 1024 + k] = d;
      }
    }
    __syncthreads();
  } else {
  // Hg = W1 [e; s] + b1 (LeakyReLU(True): slope 1, the identity, models.py:127)
  reduce4(red, aG, wv, lane);
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
    int h, j;
    red_index(k, h, j);
    const float v = red[k] + Pg[G::G_B1 + h];
    hgl[j * kHP + h] = v;
    if ((long)blk * 16 + j < B) rows[((long)blk * 16 + j) * G::GS_SIZE + G::GS_H + h] = v;
  }
  __syncthreads();
  reduce4(red, aD, wv, lane);
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
    int h, j;
    red_index(k, h, j);
    dsl[j * kHP + h] = red[k];
  }
  __syncthreads();
  }

  // 2. Gen2 tiles: T = tanh(W2 Hg + b2), ns = s + 4 T (models.py:128-133);
  //    Disc1's ns half accumulated from each tile (the tile is its B operand)
  f32x4 hb[4];  // Hg as the B operand of the 16 hidden k-steps
#pragma unroll
  for (int q = 0; q < 4; ++q) hb[q] = ld4(hgl + i * kHP + 16 * q + 4 * g);
  const float* W2 = Pg + G::G_W2;
#pragma unroll
  for (int t = 0; t < 4; ++t) aD[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {  // software-pipelined as phase 1
    struct Ops {
      f32x4 bias, wa[4], wd[4], s4;
    };
    auto load = [&](int c, Ops& o) {
      const int n0 = 16 * c, n = n0 + 4 * g;  // this lane's output rows n .. n + 3
      const bool nok = n < HH, rok = n0 + i < HH;
      o.bias = ld4(nok ? Pg + G::G_B2 + n : gk_zero);
#pragma unroll
      for (int q = 0; q < 4; ++q) o.wa[q] = ld4(rok ? W2 + (long)(n0 + i) * 64 + 16 * q + 4 * g : gk_zero);
#pragma unroll
      for (int t = 0; t < 4; ++t) o.wd[t] = ld4(nok ? D1 + (long)(16 * t + i) * DIN + HH + n : gk_zero);
      o.s4 = ld4(nok && eok ? sched + env * HH + n : gk_zero);
    };
    // ping-pong buffers, no loop-carried copy (a copy would make the compiler
    // wait for the prefetch at once)
    Ops A, B;
    auto step = [&](int c, const Ops& cur) {
      const int n = 16 * c + 4 * g;
      const bool nok = n < HH;
      f32x4 acc = cur.bias;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = mfma(cur.wa[q][r], hb[q][r], acc);
      f32x4 tv, nv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        tv[r] = tanhf(acc[r]);
        nv[r] = cur.s4[r] + 4.0f * tv[r];
      }
      if (nok && eok) {
        st4(row + G::GS_T + n, tv);
        st4(row + G::GS_Z + HH + n, nv);
        st4(a.ns_out + env * HH + n, nv);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 4; ++t) aD[t] = mfma(cur.wd[t][r], nv[r], aD[t]);
    };
    if (c0 < K::KS) load(c0, A);
    for (int c = c0; c < K::KS; c += 2 * cs) {
      load(c + cs < K::KS ? c + cs : c, B);
      step(c, A);
      if (c + cs >= K::KS) break;
      load(c + 2 * cs < K::KS ? c + 2 * cs : c + cs, A);
      step(c + cs, B);
    }
  }
  if constexpr (PH == 2) {  // the slice's Disc1-ns partial (gan_dd_head_kernel sums the slices)
    float* out = a.part2 + ((long)blk * S + sl) * 1024;
    reduce4(red, aD, wv, lane);
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) out[k] = red[k];
    return;
  } else {
  // DD = Disc1 [s; ns] + db1 (LeakyReLU(True) = identity, models.py:145)
  reduce4(red, aD, wv, lane);
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
    int h, j;
    red_index(k, h, j);
    const float v = (red[k] + dsl[j * kHP + h]) + Pd[G::D_B1 + h];
    dsl[j * kHP + h] = v;
    if ((long)blk * 16 + j < B) rows[((long)blk * 16 + j) * G::GS_SIZE + G::GS_DD + h] = v;
  }
  __syncthreads();
  head16(dsl, Pd + G::D_W2, Pd + G::D_B2, zl, pl);
  if (threadIdx.x < 32) {
    const long e = (long)blk * 16 + (threadIdx.x >> 1);
    if (e < B) {
      rows[e * G::GS_SIZE + G::GS_P + (threadIdx.x & 1)] = pl[threadIdx.x];
      if (a.probs) a.probs[2 * e + (threadIdx.x & 1)] = pl[threadIdx.x];
    }
  }
  }
}

// The split forward's end, per block, after the simulator: DD = the slices'
// Disc1-ns partials (slice order) + Disc1's schedule half + db1 -> rows; the
// head and softmax (head16) -> rows' probabilities (and probs); mode 1: the BCE
// gradient toward the simulated label tgt (PreGANPlus.py:66-67) back through
// the softmax and the head -> dOut, dDD (disc_head_kernel's mode 1).
template <int H>
__global__ __launch_bounds__(256) void gan_dd_head_kernel(int B, int S, int mode, const float* __restrict__ Pd,
                                                          float* __restrict__ rows, const float* __restrict__ part2,
                                                          const float* __restrict__ dsum, const float* __restrict__ tgt,
                                                          float* __restrict__ probs) {
  using G = TGeo<H>;
  __shared__ __attribute__((aligned(16))) float ddl[16 * kHP];
  __shared__ float zl[32], pl[32];
  const int blk = blockIdx.x;
  const float* in = part2 + (long)blk * S * 1024;
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
    int h, j;
    red_index(k, h, j);
    float v = slice_sum(in + k, 1024, S);
    v = (v + dsum[(long)blk * 1024 + k]) + Pd[G::D_B1 + h];
    ddl[j * kHP + h] = v;
    if ((long)blk * 16 + j < B) rows[((long)blk * 16 + j) * G::GS_SIZE + G::GS_DD + h] = v;
  }
  __syncthreads();
  head16(ddl, Pd + G::D_W2, Pd + G::D_B2, zl, pl);
  if (threadIdx.x < 32) {
    const long e = (long)blk * 16 + (threadIdx.x >> 1);
    if (e < B) {
      rows[e * G::GS_SIZE + G::GS_P + (threadIdx.x & 1)] = pl[threadIdx.x];
      if (probs) probs[2 * e + (threadIdx.x & 1)] = pl[threadIdx.x];
    }
  }
  if (mode == 0) return;
  if (threadIdx.x < 16) {  // torch BCE grad (p - t) / max(p (1 - p), 1e-12) / N, through the softmax
    const int j = threadIdx.x;
    const long e = (long)blk * 16 + j;
    const float p0 = pl[2 * j], p1 = pl[2 * j + 1];
    const float t0 = e < B ? tgt[2 * e] : 0.f, t1 = e < B ? tgt[2 * e + 1] : 0.f;
    const float dp0 = (p0 - t0) / fmaxf(p0 * (1.f - p0), 1e-12f) * 0.5f;
    const float dp1 = (p1 - t1) / fmaxf(p1 * (1.f - p1), 1e-12f) * 0.5f;
    const float sd = p0 * dp0 + p1 * dp1;
    zl[2 * j] = p0 * (dp0 - sd);
    zl[2 * j + 1] = p1 * (dp1 - sd);
    if (e < B) {
      rows[e * G::GS_SIZE + G::GS_DO] = zl[2 * j];
      rows[e * G::GS_SIZE + G::GS_DO + 1] = zl[2 * j + 1];
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 16 * 64; k += blockDim.x) {
    const int j = k >> 6, h = k & 63;
    const long e = (long)blk * 16 + j;
    if (e < B) rows[e * G::GS_SIZE + G::GS_DDD + h] = Pd[G::D_W2 + h] * zl[2 * j] + Pd[G::D_W2 + 64 + h] * zl[2 * j + 1];
  }
}

// one wave per environment: the Disc head (models.py:146-151) from DD in the
// row, then (mode >= 1) nn.BCELoss's gradient toward the target (mean over the
// 2 probabilities, PreGANPlus.py:66-67,72-73) back through the softmax and the
// head: dOut (2) and dDD = D2^T dOut (64).  mode 1: target from tgt[b]; mode 2: [0,1].
template <int H>
__global__ __launch_bounds__(256) void disc_head_kernel(int B, int mode, const float* __restrict__ Pd,
                                                        float* __restrict__ scr, const float* __restrict__ tgt,
                                                        float* __restrict__ probs) {
  using G = TGeo<H>;
  const int lane = threadIdx.x & 63;
  const long b = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave
  float* S = scr + b * G::GS_SIZE;
  const float dd = S[G::GS_DD + lane];
  const float z0 = wave_sum(Pd[G::D_W2 + lane] * dd) + Pd[G::D_B2];
  const float z1 = wave_sum(Pd[G::D_W2 + 64 + lane] * dd) + Pd[G::D_B2 + 1];
  const float mx = fmaxf(z0, z1), e0 = expf(z0 - mx), e1 = expf(z1 - mx);
  const float p0 = e0 / (e0 + e1), p1 = e1 / (e0 + e1);
  if (lane == 0) {
    S[G::GS_P] = p0;
    S[G::GS_P + 1] = p1;
    if (probs) {
      probs[2 * b] = p0;
      probs[2 * b + 1] = p1;
    }
  }
  if (mode == 0) return;
  const float t0 = mode == 1 ? tgt[2 * b] : 0.f, t1 = mode == 1 ? tgt[2 * b + 1] : 1.f;
  // torch BCE grad: (p - t) / max(p (1 - p), 1e-12) / N
  const float dp0 = (p0 - t0) / fmaxf(p0 * (1.f - p0), 1e-12f) * 0.5f;
  const float dp1 = (p1 - t1) / fmaxf(p1 * (1.f - p1), 1e-12f) * 0.5f;
  const float sd = p0 * dp0 + p1 * dp1;
  const float do0 = p0 * (dp0 - sd), do1 = p1 * (dp1 - sd);
  if (lane == 0) {
    S[G::GS_DO] = do0;
    S[G::GS_DO + 1] = do1;
  }
  S[G::GS_DDD + lane] = Pd[G::D_W2 + lane] * do0 + Pd[G::D_W2 + 64 + lane] * do1;
}

// ---------------------------------------------------------------------------
// Gen backward of a block through the updated Disc
// ---------------------------------------------------------------------------
// Gen backward of a block.  PH 0: one workgroup per block; PH 1 / PH 2: phase
// 1 (Disc1' over [s; ns]) and phase 3 (the tiles) split over gridDim.y slices
// as the forward: PH 1 writes the slices' DD' partials (part3), PH 2 sums them,
// evaluates the head / BCE / dDD' (every slice; slice 0 writes the rows), runs
// its tiles and writes its dHg partial (part4); the last slice of the block to
// finish (a device-scope counter per block, reset by it) sums the partials in
// slice order into the rows.
struct GanGenArgs {
  int B;
  const float* Pg;
  const float* Pd;
  float* rows;
  float* part3;        // [nblk][S][1024]
  float* part4;        // [nblk][S][1024]
  unsigned* counter;   // [nblk], zero between launches
};
template <int H, int PH>
__global__ __launch_bounds__(kGW * 64) void gan_gen_kernel(GanGenArgs ga) {
  using K = GanK<H>;
  using G = TGeo<H>;
  constexpr int HH = K::HH, DIN = K::DIN;
  __shared__ __attribute__((aligned(16))) float red[kGW * 4 * 256];
  __shared__ __attribute__((aligned(16))) float ddl[16 * kHP];  // DD', then dDD' [env][hidden]
  __shared__ float zl[32], pl[32];
  const int B = ga.B;
  const float* __restrict__ Pg = ga.Pg;
  const float* __restrict__ Pd = ga.Pd;
  float* __restrict__ rows = ga.rows;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, i = lane & 15;
  const int blk = blockIdx.x, sl = blockIdx.y, S = gridDim.y;
  const int c0 = sl * kGW + wv, cs = S * kGW;
  const long env = (long)blk * 16 + i;
  const bool eok = env < B;
  float* row = rows + (eok ? env : 0) * G::GS_SIZE;
  const float* D1 = Pd + G::D_W1;

  // 1. DD' = Disc1' [s; ns] + db1' (the row's Z holds [s; ns] contiguously)
  f32x4 a[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) a[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (PH != 2) {  // software-pipelined: chunk c + cs loaded before chunk c's MFMAs
    struct Ops {
      f32x4 bv, wd[4];
    };
    auto load = [&](int c, Ops& o) {
      const int f = 16 * c + 4 * g;
      const bool fok = f < DIN;
      o.bv = ld4(fok && eok ? row + G::GS_Z + f : gk_zero);
#pragma unroll
      for (int t = 0; t < 4; ++t) o.wd[t] = ld4(fok ? D1 + (long)(16 * t + i) * DIN + f : gk_zero);
    };
    // ping-pong buffers, no loop-carried copy (a copy would make the compiler
    // wait for the prefetch at once)
    Ops A, B;
    auto step = [&](int c, const Ops& cur) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 4; ++t) a[t] = mfma(cur.wd[t][r], cur.bv[r], a[t]);
    };
    if (c0 < K::KZ) load(c0, A);
    for (int c = c0; c < K::KZ; c += 2 * cs) {
      load(c + cs < K::KZ ? c + cs : c, B);
      step(c, A);
      if (c + cs >= K::KZ) break;
      load(c + 2 * cs < K::KZ ? c + 2 * cs : c + cs, A);
      step(c + cs, B);
    }
  }
  if constexpr (PH == 1) {
    float* out = ga.part3 + ((long)blk * S + sl) * 1024;
    reduce4(red, a, wv, lane);
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) out[k] = red[k];
    return;
  } else if constexpr (PH == 2) {
    const float* in = ga.part3 + (long)blk * S * 1024;
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
      int h, j;
      red_index(k, h, j);
      const float v = slice_sum(in + k, 1024, S);
      ddl[j * kHP + h] = v + Pd[G::D_B1 + h];
    }
    __syncthreads();
  } else {
  reduce4(red, a, wv, lane);
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
    int h, j;
    red_index(k, h, j);
    ddl[j * kHP + h] = red[k] + Pd[G::D_B1 + h];
  }
  __syncthreads();
  }
  // 2. head, BCE toward [0, 1] (PreGANPlus.py:69-73) -> dOut', dDD' = D2'^T dOut'
  head16(ddl, Pd + G::D_W2, Pd + G::D_B2, zl, pl);
  if (threadIdx.x < 16) {
    const int j = threadIdx.x;
    const float p0 = pl[2 * j], p1 = pl[2 * j + 1];
    const float dp0 = p0 / fmaxf(p0 * (1.f - p0), 1e-12f) * 0.5f;
    const float dp1 = (p1 - 1.f) / fmaxf(p1 * (1.f - p1), 1e-12f) * 0.5f;
    const float sd = p0 * dp0 + p1 * dp1;
    zl[2 * j] = p0 * (dp0 - sd);
    zl[2 * j + 1] = p1 * (dp1 - sd);
    const long e = (long)blk * 16 + j;
    if (e < B && sl == 0) {
      rows[e * G::GS_SIZE + G::GS_P] = p0;  // gen_loss's probabilities (pgp_gan_probs)
      rows[e * G::GS_SIZE + G::GS_P + 1] = p1;
      rows[e * G::GS_SIZE + G::GS_DO] = zl[2 * j];
      rows[e * G::GS_SIZE + G::GS_DO + 1] = zl[2 * j + 1];
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 16 * 64; k += blockDim.x) {
    const int j = k >> 6, h = k & 63;
    ddl[j * kHP + h] = Pd[G::D_W2 + h] * zl[2 * j] + Pd[G::D_W2 + 64 + h] * zl[2 * j + 1];
  }
  __syncthreads();
  // 3. per tile of 16 schedule entries n: d ns = Disc1'[:, HH + n]^T dDD',
  //    dY = 4 d ns (1 - T^2) (models.py:128-133), dHg += W2[n, :]^T dY
  f32x4 db[4];  // dDD' as the B operand of the 16 hidden k-steps
#pragma unroll
  for (int q = 0; q < 4; ++q) db[q] = ld4(ddl + i * kHP + 16 * q + 4 * g);
  const float* W2 = Pg + G::G_W2;
#pragma unroll
  for (int t = 0; t < 4; ++t) a[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {  // software-pipelined: tile c + kGW's operands loaded before tile c's MFMAs
    struct Ops {
      float da[4][4], wa[4][4];
      f32x4 tv;
    };
    auto load = [&](int c, Ops& o) {
      const int n0 = 16 * c, n = n0 + 4 * g;
      const bool nok = n < HH, rok = n0 + i < HH;
      // A[i][k]: Disc1'[hidden 16q + 4g + r][HH + n0 + i] (k-step (q, r))
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          o.da[q][r] = *(rok ? D1 + (long)(16 * q + 4 * g + r) * DIN + HH + n0 + i : gk_zero);
      // A[i][k]: W2[n0 + 4g + r][16t + i] (k-step r of the dY tile)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) o.wa[t][r] = *(nok ? W2 + (long)(n + r) * 64 + 16 * t + i : gk_zero);
      o.tv = ld4(nok && eok ? row + G::GS_T + n : gk_zero);
    };
    // ping-pong buffers, no loop-carried copy (a copy would make the compiler
    // wait for the prefetch at once)
    Ops A, B;
    auto step = [&](int c, const Ops& cur) {
      const int n = 16 * c + 4 * g;
      const bool nok = n < HH;
      f32x4 dn = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) dn = mfma(cur.da[q][r], db[q][r], dn);
      f32x4 dy;
#pragma unroll
      for (int r = 0; r < 4; ++r) dy[r] = 4.0f * dn[r] * (1.f - cur.tv[r] * cur.tv[r]);
      if (nok && eok) st4(row + G::GS_DY + n, dy);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 4; ++t) a[t] = mfma(cur.wa[t][r], dy[r], a[t]);
    };
    if (c0 < K::KS) load(c0, A);
    for (int c = c0; c < K::KS; c += 2 * cs) {
      load(c + cs < K::KS ? c + cs : c, B);
      step(c, A);
      if (c + cs >= K::KS) break;
      load(c + 2 * cs < K::KS ? c + 2 * cs : c + cs, A);
      step(c + cs, B);
    }
  }
  reduce4(red, a, wv, lane);
  if constexpr (PH == 2) {
    // this slice's dHg partial (stored write-through); the block's last slice
    // sums them in slice order (arrive_last: drain, count, acquire, reset)
    float* base = ga.part4 + (long)blk * S * 1024;
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) store_wt(base + (long)sl * 1024 + k, red[k]);
    __shared__ int s_last;
    if (!arrive_last(ga.counter + blk, (unsigned)S, &s_last)) return;
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
      int h, j;
      red_index(k, h, j);
      const float v = slice_sum(base + k, 1024, S);
      if ((long)blk * 16 + j < B) rows[((long)blk * 16 + j) * G::GS_SIZE + G::GS_DH + h] = v;
    }
  } else {
  for (int k = threadIdx.x; k < 1024; k += blockDim.x) {
    int h, j;
    red_index(k, h, j);
    if ((long)blk * 16 + j < B) rows[((long)blk * 16 + j) * G::GS_SIZE + G::GS_DH + h] = red[k];
  }
  }
}

// ---------------------------------------------------------------------------
// weight gradients: dW[n][k] = sum_b Y[b][n] X[b][k] (= into G), db[n] = sum_b Y[b][n]
// ---------------------------------------------------------------------------
struct OuterProd {
  const float* Y;  // Y[b][n] at Y + b * ld_rows, n < N
  const float* X;  // X[b][k] at X + b * ld_rows, k < K
  float* dW;       // dW[n][k] at dW + n * ldw + k
  float* db;       // optional: db[n]
  int N, K, ldw;
  int nbk;    // 64-column blocks of k
  int first;  // index of this product's first 64 x 64 block
};
struct OuterArgs {
  int B;
  long ld_rows;
  int nprod;
  OuterProd p[4];
  AdamFuse adam;  // the section's AdamW applied as each gradient element is written (P == nullptr: not)
};

// one workgroup per 64 x 64 block of one product: 4 x 4 MFMA tiles, one
// k-step per 4 environments (k = lane group); its kOW waves take contiguous
// eighths of the batch (three steps in flight each) and their partial tiles
// are summed in wave order through LDS (deterministic).  One wave per block
// ran a B/4-step chain: 55 us at the online loop's 1,024 environments.
constexpr int kOW = 8;
__global__ __launch_bounds__(kOW * 64) void outer_kernel(OuterArgs a) {
  __shared__ __attribute__((aligned(16))) float red[kOW * 16 * 256];
  __shared__ float bred[kOW * 4 * 64];
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, wv = threadIdx.x >> 6;
  const int blk = blockIdx.x;
  int pi = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (k < a.nprod && blk >= a.p[k].first) pi = k;
  if (pi < 0) return;  // (workgroup-uniform)
  const OuterProd p = a.p[pi];
  const int lb = blk - p.first;
  const int nb = lb / p.nbk, kb = lb - nb * p.nbk;
  if (nb * 64 >= p.N) return;  // past the product (workgroup-uniform)
  const int n0 = nb * 64, k0 = kb * 64;
  f32x4 acc[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
  bool nok[4], kok[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    nok[t] = n0 + 16 * t + i < p.N;
    kok[t] = k0 + 16 * t + i < p.K;
  }
  const int steps = (a.B + 3) / 4;
  const int s0 = (int)((long)steps * wv / kOW), s1 = (int)((long)steps * (wv + 1) / kOW);
  auto load = [&](int s, float (&y)[4], float (&x)[4]) {
    const long e = 4L * s + g;
    const bool ok = s < s1 && e < a.B;
    const float* yr = p.Y + e * a.ld_rows + n0 + i;
    const float* xr = p.X + e * a.ld_rows + k0 + i;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      y[t] = *(ok && nok[t] ? yr + 16 * t : gk_zero);
      x[t] = *(ok && kok[t] ? xr + 16 * t : gk_zero);
    }
  };
  // three steps in flight: step s + 2's values are loaded before step s's MFMAs
  float y[4], x[4], y1[4], x1[4];
  load(s0, y, x);
  load(s0 + 1, y1, x1);
  for (int s = s0; s < s1; ++s) {
    float yn[4], xn[4];
    load(s + 2, yn, xn);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bs[t] += y[t];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[t][u] = mfma(y[t], x[u], acc[t][u]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      y[t] = y1[t];
      x[t] = x1[t];
      y1[t] = yn[t];
      x1[t] = xn[t];
    }
  }
  // every wave's tiles to LDS, then wave w sums tiles 2w, 2w+1 over the waves
  // in wave order (the same association as one wave accumulating them) and
  // writes them (with the section's AdamW when fused): the epilogue spread over
  // the 8 waves
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int u = 0; u < 4; ++u) st4(red + ((wv * 16 + t * 4 + u) * 64 + lane) * 4, acc[t][u]);
    bred[(wv * 4 + t) * 64 + lane] = bs[t];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int tu = 2 * wv + q, t = tu >> 2, u = tu & 3;
    f32x4 v = ld4(red + ((0 * 16 + tu) * 64 + lane) * 4);
#pragma unroll
    for (int w = 1; w < kOW; ++w) v += ld4(red + ((w * 16 + tu) * 64 + lane) * 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 16 * t + 4 * g + r, k = k0 + 16 * u + i;
      if (n < p.N && k < p.K) {
        float* gp = p.dW + (long)n * p.ldw + k;
        *gp = v[r];
        adamw_fused(a.adam, gp, v[r]);
      }
    }
  }
  if (p.db && kb == 0 && wv < 4) {  // bias tile t = wv
    const int t = wv;
    float b = bred[(0 * 4 + t) * 64 + lane];
#pragma unroll
    for (int w = 1; w < kOW; ++w) b += bred[(w * 4 + t) * 64 + lane];
    const float sum = xsum(b, true);
    if (g == 0 && nok[t]) {
      float* gp = p.db + n0 + 16 * t + i;
      *gp = sum;
      adamw_fused(a.adam, gp, sum);
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
#define GCK(expr)                            \
  do {                                       \
    expr;                                    \
    const hipError_t e_ = hipGetLastError(); \
    if (e_ != hipSuccess) return e_;         \
  } while (0)

hipError_t outer(const OuterArgs& a0, hipStream_t st) {
  OuterArgs a = a0;
  int blocks = 0;
  for (int k = 0; k < a.nprod; ++k) {
    OuterProd& p = a.p[k];
    p.nbk = (p.K + 63) / 64;
    p.first = blocks;
    blocks += ((p.N + 63) / 64) * p.nbk;
  }
  GCK((outer_kernel<<<blocks, kOW * 64, 0, st>>>(a)));
  return hipSuccess;
}

// Slices per 16-environment block: the split form when the blocks alone leave
// the chip mostly idle and each wave still gets a chunk (at C3's 103
// environments, H = 50: 7 blocks -> 7 x 16 workgroups); one workgroup per
// block otherwise (H <= 16: 16 chunks are 2 per wave already; large batches).
constexpr int kGanMaxSlices = 16;
template <int H>
int gan_slices(int B) {
  using K = GanK<H>;
  const int nblk = (B + 15) / 16;
  const int cap = std::min(kGanMaxSlices, K::KS / kGW);
  const int s = std::min(cap, (256 + nblk - 1) / nblk);
  return s >= 4 ? s : 1;  // (2 slices at H = 16: train_gan alone 0.067 -> 0.068 ms, profiles/r05/gan_slices2.txt)
}
// the split form's regions after the rows (floats)
struct GanSplit {
  long part1, part2, dsum, part3, part4, counter, total;
};
template <int H>
GanSplit gan_split_offsets(int B) {
  const long nblk = (B + 15) / 16, S = kGanMaxSlices;
  GanSplit o{};
  o.part1 = (long)B * TGeo<H>::GS_SIZE;
  o.part2 = o.part1 + nblk * S * 2048;
  o.dsum = o.part2 + nblk * S * 1024;
  o.part3 = o.dsum + nblk * 1024;
  o.part4 = o.part3 + nblk * S * 1024;
  o.counter = o.part4 + nblk * S * 1024;
  o.total = o.counter + nblk;
  return o;
}

template <int H>
hipError_t gan_fwd_h(int B, const float* emb, const float* logits, const float* protos, float* emb_out,
                     const float* sched, const float* Pg, const float* Pd, float* ws, float* ns_out, float* probs,
                     hipStream_t st) {
  const int nblk = (B + 15) / 16, S = gan_slices<H>(B);
  const GanSplit o = gan_split_offsets<H>(B);
  GanFwdArgs a{B, emb, emb_out, logits, protos, sched, Pg, Pd, ws, ns_out, probs, ws + o.part1, ws + o.part2,
               ws + o.dsum};
  if (S == 1) {
    GCK((gan_fwd_kernel<H, 0><<<nblk, kGW * 64, 0, st>>>(a)));
    return hipSuccess;
  }
  GCK((gan_fwd_kernel<H, 1><<<dim3(nblk, S), kGW * 64, 0, st>>>(a)));
  GCK((gan_fwd_kernel<H, 2><<<dim3(nblk, S), kGW * 64, 0, st>>>(a)));
  if (probs)  // the forward's Disc probabilities (the Disc step re-evaluates the head itself)
    GCK((gan_dd_head_kernel<H><<<nblk, 256, 0, st>>>(B, S, 0, Pd, ws, ws + o.part2, ws + o.dsum, nullptr, probs)));
  return hipSuccess;
}

template <int H>
hipError_t gan_disc_bwd_h(int B, const float* target, const float* Pd, float* Gdd, float* ws, float* probs,
                          const AdamFuse* af, hipStream_t st) {
  using G = TGeo<H>;
  const int nblk = (B + 15) / 16, S = gan_slices<H>(B);
  if (S == 1) {
    GCK((disc_head_kernel<H><<<(B + 3) / 4, 256, 0, st>>>(B, 1, Pd, ws, target, probs)));
  } else {
    const GanSplit o = gan_split_offsets<H>(B);
    GCK((gan_dd_head_kernel<H><<<nblk, 256, 0, st>>>(B, S, 1, Pd, ws, ws + o.part2, ws + o.dsum, target, probs)));
  }
  OuterArgs a{};
  a.B = B;
  a.ld_rows = G::GS_SIZE;
  a.nprod = 2;
  // Disc1: dD1 = sum_b dDD_b [s; ns]_b^T, db1 = sum_b dDD_b
  a.p[0] = OuterProd{ws + G::GS_DDD, ws + G::GS_Z, Gdd + G::D_W1, Gdd + G::D_B1, 64, G::DIN, G::DIN, 0, 0};
  // head: dD2 = sum_b dOut_b DD_b^T, db2 = sum_b dOut_b
  a.p[1] = OuterProd{ws + G::GS_DO, ws + G::GS_DD, Gdd + G::D_W2, Gdd + G::D_B2, 2, 64, 64, 0, 0};
  if (af) a.adam = *af;
  return outer(a, st);
}

template <int H>
hipError_t gan_gen_bwd_h(int B, const float* Pg, const float* Pd, float* Gdg, float* ws, const AdamFuse* af,
                         hipStream_t st) {
  using G = TGeo<H>;
  constexpr int HH = H * H;
  const int nblk = (B + 15) / 16, S = gan_slices<H>(B);
  const GanSplit o = gan_split_offsets<H>(B);
  GanGenArgs ga{B, Pg, Pd, ws, ws + o.part3, ws + o.part4, reinterpret_cast<unsigned*>(ws + o.counter)};
  if (S == 1) {
    GCK((gan_gen_kernel<H, 0><<<nblk, kGW * 64, 0, st>>>(ga)));
  } else {
    GCK((gan_gen_kernel<H, 1><<<dim3(nblk, S), kGW * 64, 0, st>>>(ga)));
    GCK((gan_gen_kernel<H, 2><<<dim3(nblk, S), kGW * 64, 0, st>>>(ga)));
  }
  OuterArgs a{};
  a.B = B;
  a.ld_rows = G::GS_SIZE;
  a.nprod = 3;
  // Gen2: dW2 = sum_b dY_b Hg_b^T, db2 = sum_b dY_b
  a.p[0] = OuterProd{ws + G::GS_DY, ws + G::GS_H, Gdg + G::G_W2, Gdg + G::G_B2, HH, 64, 64, 0, 0};
  // Gen1 over [e; s]: dW1[:, :2H] = sum_b dHg_b e_b^T (+ db1), dW1[:, 2H:] = sum_b dHg_b s_b^T
  a.p[1] = OuterProd{ws + G::GS_DH, ws + G::GS_X, Gdg + G::G_W1, Gdg + G::G_B1, 64, 2 * H, G::GIN, 0, 0};
  a.p[2] = OuterProd{ws + G::GS_DH, ws + G::GS_Z, Gdg + G::G_W1 + 2 * H, nullptr, 64, HH, G::GIN, 0, 0};
  if (af) a.adam = *af;
  return outer(a, st);
}

// the Disc probabilities the last head evaluation left in the rows (after
// pgp_gan_gen_backward: the updated Disc's, i.e. gen_loss's, PreGANPlus.py:71-73)
template <int H>
__global__ void gan_probs_kernel(int B, const float* __restrict__ scr, float* __restrict__ probs) {
  using G = TGeo<H>;
  const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  probs[2 * b] = scr[b * G::GS_SIZE + G::GS_P];
  probs[2 * b + 1] = scr[b * G::GS_SIZE + G::GS_P + 1];
}

template <int H>
hipError_t gan_probs_h(int B, const float* ws, float* probs, hipStream_t st) {
  GCK((gan_probs_kernel<H><<<(B + 255) / 256, 256, 0, st>>>(B, ws, probs)));
  return hipSuccess;
}

}  // namespace

hipError_t launch_gan_probs(int H, int B, const float* ws, float* probs, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_probs_h<h>(B, ws, probs, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

// one row of GS_SIZE floats per environment, then the split form's partials
// and per-block counters (zero in a fresh workspace; reset after each use)
long gan_workspace_floats(int H, int B) {
  if (B < 1) return 0;
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_split_offsets<h>(B).total;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

hipError_t launch_gan_fwd(int H, int B, const float* emb, const float* sched, const float* Pg, const float* Pd,
                          float* ws, float* ns_out, float* probs, hipStream_t st, const float* logits,
                          const float* protos, float* emb_out) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_fwd_h<h>(B, emb, logits, protos, emb_out, sched, Pg, Pd, ws, ns_out, probs, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_disc_bwd(int H, int B, const float* target, const float* Pd, float* Gdd, float* ws,
                               hipStream_t st, float* probs, const AdamFuse* af) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_disc_bwd_h<h>(B, target, Pd, Gdd, ws, probs, af, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

hipError_t launch_gan_gen_bwd(int H, int B, const float* Pg, const float* Pd, float* Gdg, float* ws,
                              hipStream_t st, const AdamFuse* af) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return gan_gen_bwd_h<h>(B, Pg, Pd, Gdg, ws, af, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
