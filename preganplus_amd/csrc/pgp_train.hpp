// pgp_train.hpp — geometry of the training (tuning / GAN) kernels.
//
// Training runs on fp32 master weights in the reference's NATURAL layout (the
// blob order of pgp_load_weights): the inference kernels' packed layouts fold
// several parameters together (GAT fc into the time encoder, the attention
// scale into Wq), so they cannot be trained in place; after an optimizer step
// the packed copies are rebuilt from the master weights.
//
// The tuning step's activation workspace is planned in pgp_tune.hpp.
#pragma once
#include <cstddef>

namespace pgp {

template <int H>
struct TGeo {
  static constexpr int D = H, W = 3, T = 3 * H, FF = 64, HD = H / 2, L = 3 * H * H;
  // natural weight blob offsets (transformer section)
  static constexpr long W_FC = 0;                   // [d][3]
  static constexpr long W_ATT = W_FC + 3 * D;       // [2d]
  static constexpr long W_TE = W_ATT + 2 * D;       // [d][d]
  static constexpr long B_TE = W_TE + D * D;        // [d]
  static constexpr long PE = B_TE + D;              // [3][d]
  static constexpr long LAY0 = PE + 3 * D;
  // within a layer
  static constexpr long L_IN = 0, L_INB = 3 * D * D, L_OUT = L_INB + 3 * D, L_OUTB = L_OUT + D * D,
                        L_W1 = L_OUTB + D, L_B1 = L_W1 + FF * D, L_W2 = L_B1 + FF, L_B2 = L_W2 + D * FF,
                        L_N1W = L_B2 + D, L_N1B = L_N1W + D, L_N2W = L_N1B + D, L_N2B = L_N2W + D,
                        L_SIZE = L_N2B + D;
  static constexpr long W_AN = LAY0 + 2 * L_SIZE;   // [2H][L]
  static constexpr long B_AN = W_AN + 2L * H * L;
  static constexpr long W_PR = B_AN + 2 * H;
  static constexpr long B_PR = W_PR + 2L * H * L;
  static constexpr long TR_SIZE = B_PR + 2 * H;     // transformer section length
  // gen / disc sections (relative to their own start)
  static constexpr int GIN = 2 * H + H * H;
  static constexpr long G_W1 = 0, G_B1 = 64L * GIN, G_W2 = G_B1 + 64, G_B2 = G_W2 + (long)H * H * 64,
                        G_SIZE = G_B2 + H * H;
  static constexpr int DIN = 2 * H * H;
  static constexpr long D_W1 = 0, D_B1 = 64L * DIN, D_W2 = D_B1 + 64, D_B2 = D_W2 + 128, D_SIZE = D_B2 + 2;
  static constexpr long OFF_GEN = TR_SIZE, OFF_DISC = TR_SIZE + G_SIZE, ALL = TR_SIZE + G_SIZE + D_SIZE;

  // ---- GAN scratch per window (floats) ----
  static constexpr long GS_X = 0;                        // [GIN] gen input [emb; s]
  static constexpr long GS_Z = GS_X + GIN;               // [2H^2] disc input [s; ns]
  static constexpr long GS_H = GS_Z + DIN;               // [64] gen hidden
  static constexpr long GS_T = GS_H + 64;                // [H^2] tanh
  static constexpr long GS_DD = GS_T + H * H;            // [64] disc hidden
  static constexpr long GS_P = GS_DD + 64;               // [2] (pad 4) probs
  static constexpr long GS_DO = GS_P + 4;                // [2] (pad 4) d logits
  static constexpr long GS_DDD = GS_DO + 4;              // [64] d disc hidden
  static constexpr long GS_DY = GS_DDD + 64;             // [H^2] d gen pre-tanh
  static constexpr long GS_DH = GS_DY + H * H;           // [64] d gen hidden
  static constexpr long GS_SIZE = GS_DH + 64;
};

// AdamW descriptor: one per parameter tensor in the natural blob
constexpr int kMaxTensors = 48;
constexpr int kAdamFromTable = 2;
struct AdamTensor {
  long off;       // offset in the master buffer (floats)
  int n;          // elements
  int active;     // got a gradient this step (torch skips params whose grad is None); with
                  // kAdamFromTable set, (active, step_size, bc2_sqrt) come from AdamArgs::sched's row
  float step_size;  // lr / (1 - b1^step)
  float bc2_sqrt;   // sqrt(1 - b2^step)
};
struct AdamArgs {
  float* param;
  float* grad;
  float* m;
  float* v;
  float lr_wd;  // lr * weight_decay
  float b1, b2, eps;
  int ntensors;
  const float* sched;  // optional device table [ntensors][3] = (active, step_size, bc2_sqrt), overrides t[]
  AdamTensor t[kMaxTensors];
};

// AdamW, torch single-tensor semantics (torch/optim/adamw.py), element o:
// p *= 1 - lr*wd; m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2;
// p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).  Shared by the batched kernel
// (pgp_train.hip) and the fused batch-1 GAN step (pgp_gan1.hip).
// One section's AdamW fused into the kernel that writes its gradients (the
// batched GAN step's weight-gradient kernel, world size 1: no all-reduce
// between gradient and update): every tensor of the section with the same
// per-step scalars.  P == nullptr: no update.
struct AdamFuse {
  float* P;
  float* m;
  float* v;
  const float* G;  // the gradient buffer the kernel writes (element o of G updates P[o])
  float lr_wd, b1, b2, eps, step_size, bc2_sqrt;
};
#ifdef __HIP__
__device__ __forceinline__ void adamw_update(float* __restrict__ P, float* __restrict__ M, float* __restrict__ V,
                                             long o, float g, float lr_wd, float b1, float b2, float eps,
                                             float step_size, float bc2_sqrt) {
  float p = P[o] * (1.0f - lr_wd);
  const float m = M[o] + (1.0f - b1) * (g - M[o]);
  const float v = b2 * V[o] + (1.0f - b2) * g * g;
  p -= step_size * m / (sqrtf(v) / bc2_sqrt + eps);
  P[o] = p;
  M[o] = m;
  V[o] = v;
}
__device__ __forceinline__ void adamw_elem(const AdamArgs& a, long o, float step_size, float bc2_sqrt) {
  adamw_update(a.param, a.m, a.v, o, a.grad[o], a.lr_wd, a.b1, a.b2, a.eps, step_size, bc2_sqrt);
}
__device__ __forceinline__ void adamw_fused(const AdamFuse& f, const float* g_at, float g) {
  if (f.P) adamw_update(f.P, f.m, f.v, g_at - f.G, g, f.lr_wd, f.b1, f.b2, f.eps, f.step_size, f.bc2_sqrt);
}
#endif

}  // namespace pgp
