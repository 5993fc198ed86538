// pgp_gan1.hip — train_gan (PreGANPlus.py:60-81) for ONE window as two
// single-workgroup launches, for the plugin's batch-1 call at 8 / 16 hosts:
//
//   gan1_forward_kernel  Gen + Disc forward (models.py:118-151, 258-291): the new
//                        schedule ns and the Disc probabilities (PreGANPlus.py:62-64)
//   gan1_step_kernel     after the host simulator's label: Disc BCE backward and
//                        its AdamW step, the Gen BCE backward through the updated
//                        Disc (the probabilities it saw: gen_loss) and the Gen
//                        AdamW step, then the updated GAN's forward on the same
//                        inputs (recover_decision's gate, PreGANPlus.py:84-87)
//
// replacing ≈30 batch-tiled launches (pgp_gantrain.hip) whose work at batch 1 is
// a handful of 64-wide matrix-vector products.  Every vector lives in LDS; a
// matrix-vector product over a long contraction is a wave per 4 outputs (lanes
// over k, wave_sum), over the short one (64) a thread per output; the weight
// gradients are outer products written straight into G (the gen / disc
// sections are overwritten, no zeroing needed); AdamW applies pgp_train.hpp's
// per-element update (adamw_elem, the same code as the batched kernel) from the
// device table of per-tensor (active, step_size, bc2_sqrt).  The window's
// activations are also written to the GAN scratch row 0 (the layout
// pgp_gantrain.hip uses, TGeo GS_*), so gan_probs / the eager kernels can follow.
#include <hip/hip_runtime.h>

#include "pgp_device.hpp"
#include "pgp_gemm.hpp"
#include "pgp_train.hpp"

namespace pgp {
namespace {

constexpr int kG1Threads = 1024;
constexpr int kG1Waves = kG1Threads / 64;

template <int H>
struct G1 {
  static constexpr int HH = H * H, GIN = 2 * H + HH, DIN = 2 * HH;
  // LDS layout (floats)
  static constexpr int X = 0;          // [GIN] [emb; s]
  static constexpr int Z = X + GIN;    // [DIN] [s; ns]
  static constexpr int HG = Z + DIN;   // [64]
  static constexpr int T = HG + 64;    // [HH] tanh
  static constexpr int DD = T + HH;    // [64]
  static constexpr int DO = DD + 64;   // [4] d logits (2), probs (2)
  static constexpr int DDD = DO + 4;   // [64]
  static constexpr int DY = DDD + 64;  // [HH]
  static constexpr int DH = DY + HH;   // [64]
  static constexpr int TOTAL = DH + 64;
};

// out[n] = bias[n] + sum_k W[n*ldw + k] v[k], n < N, one wave per 4 outputs
template <int N>
PGP_DEV void mv_long(const float* __restrict__ W, int ldw, const float* __restrict__ bias, const float* v, int K,
                     float* out, int wv, int lane) {
  for (int n = wv; n < N; n += kG1Waves) {
    const float* w = W + (long)n * ldw;
    float acc = 0.f;
    for (int k = lane; k < K; k += 64) acc = fmaf(w[k], v[k], acc);
    acc = wave_sum(acc);
    if (lane == 0) out[n] = acc + (bias ? bias[n] : 0.f);
  }
}

// the Disc head (models.py:146-151, Linear(64,2) + Softmax) on DD, one wave;
// mode 1 / 2: nn.BCELoss's gradient toward tgt / [0,1] (mean over the 2
// probabilities, PreGANPlus.py:66-67, 72-73) back through softmax and head:
// d logits -> s[DO], dDD -> s[DDD]; probabilities -> s[DO + 2]
template <int H>
PGP_DEV void g1_head(float* s, const float* __restrict__ Pd, int mode, float t0, float t1, int lane) {
  using G = TGeo<H>;
  using L = G1<H>;
  const float dd = s[L::DD + lane];
  const float z0 = wave_sum(Pd[G::D_W2 + lane] * dd) + Pd[G::D_B2];
  const float z1 = wave_sum(Pd[G::D_W2 + 64 + lane] * dd) + Pd[G::D_B2 + 1];
  const float mx = fmaxf(z0, z1), e0 = expf(z0 - mx), e1 = expf(z1 - mx);
  const float p0 = e0 / (e0 + e1), p1 = e1 / (e0 + e1);
  if (lane == 0) {
    s[L::DO + 2] = p0;
    s[L::DO + 3] = p1;
  }
  if (mode == 0) return;
  // torch BCE grad: (p - t) / max(p (1 - p), 1e-12) / N
  const float dp0 = (p0 - t0) / fmaxf(p0 * (1.f - p0), 1e-12f) * 0.5f;
  const float dp1 = (p1 - t1) / fmaxf(p1 * (1.f - p1), 1e-12f) * 0.5f;
  const float sd = p0 * dp0 + p1 * dp1;
  const float do0 = p0 * (dp0 - sd), do1 = p1 * (dp1 - sd);
  if (lane == 0) {
    s[L::DO] = do0;
    s[L::DO + 1] = do1;
  }
  s[L::DDD + lane] = Pd[G::D_W2 + lane] * do0 + Pd[G::D_W2 + 64 + lane] * do1;
}

// Gen + Disc forward on s[X] (and s[Z]'s schedule half): Hg, T, ns, DD, head
template <int H>
PGP_DEV void g1_forward(float* s, const float* __restrict__ Pg, const float* __restrict__ Pd, int tid) {
  using G = TGeo<H>;
  using L = G1<H>;
  const int lane = tid & 63, wv = tid >> 6;
  // Gen1 (models.py:124-127): Hg = W1 [emb; s] + b1 (LeakyReLU(True): slope 1)
  mv_long<64>(Pg + G::G_W1, L::GIN, Pg + G::G_B1, s + L::X, L::GIN, s + L::HG, wv, lane);
  __syncthreads();
  // Gen2 (models.py:128-133): ns = s + 4 tanh(W2 Hg + b2)
  for (int c = tid; c < L::HH; c += kG1Threads) {
    const float* w = Pg + G::G_W2 + (long)c * 64;
    float acc = 0.f;
#pragma unroll 16
    for (int n = 0; n < 64; ++n) acc = fmaf(w[n], s[L::HG + n], acc);
    const float t = tanhf(acc + Pg[G::G_B2 + c]);
    s[L::T + c] = t;
    s[L::Z + L::HH + c] = s[L::Z + c] + 4.0f * t;
  }
  __syncthreads();
  // Disc1 (models.py:145): DD = D1 [s; ns] + bd1
  mv_long<64>(Pd + G::D_W1, L::DIN, Pd + G::D_B1, s + L::Z, L::DIN, s + L::DD, wv, lane);
  __syncthreads();
  if (wv == 0) g1_head<H>(s, Pd, 0, 0.f, 0.f, lane);
  __syncthreads();
}

// the window's activations into GAN scratch row 0 (pgp_gantrain.hip layout)
template <int H>
PGP_DEV void g1_store_row(const float* s, float* __restrict__ row, int tid) {
  using G = TGeo<H>;
  using L = G1<H>;
  for (int i = tid; i < L::GIN; i += kG1Threads) row[G::GS_X + i] = s[L::X + i];
  for (int i = tid; i < L::DIN; i += kG1Threads) row[G::GS_Z + i] = s[L::Z + i];
  for (int i = tid; i < L::HH; i += kG1Threads) row[G::GS_T + i] = s[L::T + i];
  if (tid < 64) {
    row[G::GS_H + tid] = s[L::HG + tid];
    row[G::GS_DD + tid] = s[L::DD + tid];
  }
  if (tid < 2) row[G::GS_P + tid] = s[L::DO + 2 + tid];
}

template <int H>
PGP_DEV void g1_load_inputs(float* s, const float* __restrict__ emb, const float* __restrict__ sched, int tid) {
  using L = G1<H>;
  for (int k = tid; k < L::GIN; k += kG1Threads) {
    const float v = k < 2 * H ? emb[k] : sched[k - 2 * H];
    s[L::X + k] = v;
    if (k >= 2 * H) s[L::Z + k - 2 * H] = v;
  }
  __syncthreads();
}

template <int H>
__global__ __launch_bounds__(kG1Threads) void gan1_forward_kernel(const float* __restrict__ emb,
                                                                  const float* __restrict__ sched,
                                                                  const float* __restrict__ Pg,
                                                                  const float* __restrict__ Pd, float* __restrict__ row,
                                                                  float* __restrict__ ns_out,
                                                                  float* __restrict__ probs) {
  using L = G1<H>;
  __shared__ float s[L::TOTAL];
  const int tid = threadIdx.x;
  g1_load_inputs<H>(s, emb, sched, tid);
  g1_forward<H>(s, Pg, Pd, tid);
  g1_store_row<H>(s, row, tid);
  for (int c = tid; c < L::HH; c += kG1Threads) ns_out[c] = s[L::Z + L::HH + c];
  if (tid < 2) probs[tid] = s[L::DO + 2 + tid];
}

// AdamW over a section's tensors (rows of a.sched: active, step_size, bc2_sqrt)
PGP_DEV void g1_adamw(const AdamArgs& a, int tid) {
  for (int t = 0; t < a.ntensors; ++t) {
    const float* r = a.sched + 3 * t;
    if (r[0] == 0.f) continue;
    const float step_size = r[1], bc2_sqrt = r[2];
    for (long i = tid; i < a.t[t].n; i += kG1Threads) adamw_elem(a, a.t[t].off + i, step_size, bc2_sqrt);
  }
}

template <int H>
// Pg / Pd / Gg / Gd alias the AdamW arguments' P and G (no __restrict__)
__global__ __launch_bounds__(kG1Threads) void gan1_step_kernel(const float* __restrict__ target, float* Pg,
                                                               float* Pd, float* Gg, float* Gd, float* row,
                                                               AdamArgs ad, AdamArgs ag, float* __restrict__ probs_gen,
                                                               float* __restrict__ probs_after) {
  using G = TGeo<H>;
  using L = G1<H>;
  __shared__ float s[L::TOTAL];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // the forward's activations (gan1_forward_kernel, same inputs)
  for (int i = tid; i < L::GIN; i += kG1Threads) s[L::X + i] = row[G::GS_X + i];
  for (int i = tid; i < L::DIN; i += kG1Threads) s[L::Z + i] = row[G::GS_Z + i];
  for (int i = tid; i < L::HH; i += kG1Threads) s[L::T + i] = row[G::GS_T + i];
  if (tid < 64) {
    s[L::HG + tid] = row[G::GS_H + tid];
    s[L::DD + tid] = row[G::GS_DD + tid];
  }
  __syncthreads();
  // ---- Disc step (PreGANPlus.py:66-68): BCE(Disc(s, ns), target) ----
  if (wv == 0) g1_head<H>(s, Pd, 1, target[0], target[1], lane);
  __syncthreads();
  for (int i = tid; i < 64 * L::DIN; i += kG1Threads) {  // dD1 = dDD (x) [s; ns]
    const int n = i / L::DIN, k = i - n * L::DIN;
    Gd[G::D_W1 + i] = s[L::DDD + n] * s[L::Z + k];
  }
  if (tid < 64) Gd[G::D_B1 + tid] = s[L::DDD + tid];
  if (tid < 128) Gd[G::D_W2 + tid] = s[L::DO + tid / 64] * s[L::DD + (tid & 63)];
  if (tid < 2) Gd[G::D_B2 + tid] = s[L::DO + tid];
  __syncthreads();
  g1_adamw(ad, tid);
  __syncthreads();
  // ---- Gen step (PreGANPlus.py:69-75): BCE(Disc'(s, ns), [0, 1]) back into Gen ----
  mv_long<64>(Pd + G::D_W1, L::DIN, Pd + G::D_B1, s + L::Z, L::DIN, s + L::DD, wv, lane);
  __syncthreads();
  if (wv == 0) g1_head<H>(s, Pd, 2, 0.f, 1.f, lane);
  __syncthreads();
  if (tid < 2) probs_gen[tid] = s[L::DO + 2 + tid];
  for (int c = tid; c < L::HH; c += kG1Threads) {  // d ns = D1'[:, HH:]^T dDD; dY = 4 dns (1 - T^2)
    float acc = 0.f;
#pragma unroll 16
    for (int n = 0; n < 64; ++n) acc = fmaf(Pd[G::D_W1 + (long)n * L::DIN + L::HH + c], s[L::DDD + n], acc);
    const float t = s[L::T + c];
    s[L::DY + c] = 4.0f * acc * (1.f - t * t);
  }
  __syncthreads();
  for (int i = tid; i < L::HH * 64; i += kG1Threads) {  // dW2 = dY (x) Hg
    const int c = i >> 6, n = i & 63;
    Gg[G::G_W2 + i] = s[L::DY + c] * s[L::HG + n];
  }
  for (int c = tid; c < L::HH; c += kG1Threads) Gg[G::G_B2 + c] = s[L::DY + c];
  for (int n = wv; n < 64; n += kG1Waves) {  // dHg = W2^T dY (Gen not yet stepped)
    float acc = 0.f;
    for (int c = lane; c < L::HH; c += 64) acc = fmaf(Pg[G::G_W2 + (long)c * 64 + n], s[L::DY + c], acc);
    acc = wave_sum(acc);
    if (lane == 0) s[L::DH + n] = acc;
  }
  __syncthreads();
  for (int i = tid; i < 64 * L::GIN; i += kG1Threads) {  // dW1 = dHg (x) [emb; s]
    const int n = i / L::GIN, k = i - n * L::GIN;
    Gg[G::G_W1 + i] = s[L::DH + n] * s[L::X + k];
  }
  if (tid < 64) Gg[G::G_B1 + tid] = s[L::DH + tid];
  __syncthreads();
  g1_adamw(ag, tid);
  __syncthreads();
  // ---- the updated GAN on the same inputs: recover_decision's gate ----
  g1_forward<H>(s, Pg, Pd, tid);
  g1_store_row<H>(s, row, tid);
  if (tid < 2) probs_after[tid] = s[L::DO + 2 + tid];
}

}  // namespace

bool gan1_supported(int H) { return H == 8 || H == 16; }

hipError_t launch_gan1_forward(int H, const float* emb, const float* sched, const float* Pg, const float* Pd,
                               float* row, float* ns, float* probs, hipStream_t st) {
  switch (H) {
    case 8:
      gan1_forward_kernel<8><<<1, kG1Threads, 0, st>>>(emb, sched, Pg, Pd, row, ns, probs);
      break;
    case 16:
      gan1_forward_kernel<16><<<1, kG1Threads, 0, st>>>(emb, sched, Pg, Pd, row, ns, probs);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_gan1_step(int H, const float* target, float* Pg, float* Pd, float* Gg, float* Gd, float* row,
                            const AdamArgs& ad, const AdamArgs& ag, float* probs_gen, float* probs_after,
                            hipStream_t st) {
  switch (H) {
    case 8:
      gan1_step_kernel<8><<<1, kG1Threads, 0, st>>>(target, Pg, Pd, Gg, Gd, row, ad, ag, probs_gen, probs_after);
      break;
    case 16:
      gan1_step_kernel<16><<<1, kG1Threads, 0, st>>>(target, Pg, Pd, Gg, Gd, row, ad, ag, probs_gen, probs_after);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace pgp
