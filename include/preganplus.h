/*
 * preganplus.h — C-ABI of the MI355X-native PreGAN+ decision model.
 *
 * The drop-in boundary.  The reference's "FFI" for this path is Python calling
 * torch modules; the binding a maintainer adds is a ctypes stub
 * (INTEGRATION.md).  Plain pointers and sizes only: no torch types.
 *
 * Entry points and the reference interface each replaces (paths relative to
 * the reference repo root):
 *
 *   pgp_create / pgp_load_weights
 *       load_model / load_gan  recovery/PreGANSrc/src/utils.py:60-84
 *       (model construction models.py:314-374, 118-151, 258-291; checkpoint
 *        dict utils.py:53-58).  The blob is the reference's own tensors, fp64,
 *       concatenated in the order documented at pgp_load_weights.
 *   pgp_forward
 *       one batched call of the per-window path of run_model
 *       recovery/PreGANPlus.py:115-136 without its training side effects:
 *         Transformer_16.forward       models.py:376-416  (logits, protos)
 *         detect + embed               PreGANPlus.py:119-131 (any_anom, emb)
 *         get_classes                  utils.py:102-109   (cls)
 *         Gen_*.forward / Disc_*.forward models.py:131-151 (probs)
 *         recover_decision gate+targets PreGANPlus.py:84-105
 *             keep_orig    = probs[0] > probs[1]           (:87)
 *             final_target = first-argmax(sched[c,:])      (:99)
 *         generator proposal (GAN label input)  stats/Stats.py:162-166
 *             gen_target   = first-argmax(new_sched[c,:])
 *   pgp_migrations
 *       recover_decision's container loop PreGANPlus.py:90-105 (PreGAN.py:80-95)
 *   pgp_embedding
 *       run_model's masked prototype embedding PreGANPlus.py:129
 *   pgp_schedule_onehot
 *       result_cache rows from GOBI's one-hot placement (opt.py:9-15), for
 *       streamed fleet chunks
 *   pgp_create_fpe / pgp_forward_fpe
 *       PreGAN: PreGANRecovery.run_encoder + detect/embed/get_classes + the
 *       GAN gate, recovery/PreGAN.py:97-126 over FPE_16.forward models.py:65-115
 *   pgp_tune_* / pgp_gan_* / pgp_adamw / pgp_load_weights_master
 *       online training: tune_model PreGANPlus.py:51-58 (train.py:13-57),
 *       train_gan PreGANPlus.py:60-81 / PreGAN.py:51-71, AdamW utils.py:65
 *   pgp_gobi_*
 *       the schedule producer upstream of the path: GOBIScheduler.run_GOBI's
 *       opt() (scheduler/GOBI.py:19-42, scheduler/BaGTI/src/opt.py:17-33)
 *   pgp_sim_env_len / pgp_simulate
 *       the GAN label: run_simulation (PreGANSrc/src/utils.py:97-100) ->
 *       Stats.runSimulation (stats/Stats.py:154-177), PreGANPlus.py:65-66
 *   pgp_destroy
 *       (object lifetime; no reference counterpart)
 *
 * Conventions: every call returns 0 on success or a negative PGP_ERR_*;
 * pgp_last_error() gives a message (thread-local).  Device pointers, fp32
 * activations, int32 indices, row-major arrays; the stream is a hipStream_t
 * passed as void* (NULL = default stream).  pgp_forward allocates nothing when
 * batch <= the size passed to pgp_reserve (required before graph capture).
 */
#ifndef PREGANPLUS_H
#define PREGANPLUS_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGP_ABI_VERSION 1

#define PGP_OK 0
#define PGP_ERR_ARG (-1)         /* bad argument (null pointer, size, H) */
#define PGP_ERR_UNSUPPORTED (-2) /* host count not compiled in */
#define PGP_ERR_HIP (-3)         /* HIP runtime error */
#define PGP_ERR_STATE (-4)       /* weights not loaded / workspace missing */

typedef struct pgp_model pgp_model;

int pgp_abi_version(void);
const char* pgp_last_error(void);

/* Host counts compiled into this library (H must be even: d_model = H is split
 * over 2 heads, models.py:323-324).  Writes up to cap values; returns count. */
int pgp_supported_hosts(int* out, int cap);

/* A model for H hosts (= C containers, main.py:80) with K prototypes
 * (K = H for PreGAN+, models.py:373-374). */
int pgp_create(int n_hosts, int n_protos, pgp_model** out);
int pgp_destroy(pgp_model* m);

/* Number of doubles pgp_load_weights expects for (H, K). */
size_t pgp_weight_blob_len(int n_hosts, int n_protos);

/* Load the reference's tensors (host memory, fp64), concatenated row-major in
 * this order (names as in the reference state_dicts):
 *   Transformer: gat.layer1.heads.0.fc.weight [H,3], ...attn_fc.weight [1,2H],
 *     time_encoder.weight [H,H], time_encoder.bias [H], pos_encoder.pe [3,1,H],
 *     for layer l in 0,1: self_attn.in_proj_weight [3H,H], in_proj_bias [3H],
 *       out_proj.weight [H,H], out_proj.bias [H], linear1.weight [64,H],
 *       linear1.bias [64], linear2.weight [H,64], linear2.bias [H],
 *       norm1.weight [H], norm1.bias [H], norm2.weight [H], norm2.bias [H],
 *     anomaly_decoder.0.weight [2H,3H^2], .bias [2H],
 *     prototype_decoder.0.weight [2H,3H^2], .bias [2H]
 *   Gen: delta.0.weight [64,2H+H^2], delta.0.bias [64], delta.2.weight [H^2,64],
 *     delta.2.bias [H^2]
 *   Disc: probs.0.weight [64,2H^2], probs.0.bias [64], probs.2.weight [2,64],
 *     probs.2.bias [2]
 *   prototypes [K,2]   (model.prototype list, utils.py:70)
 * Packs them (fp64 host arithmetic, then fp32) into the device layouts and
 * uploads synchronously. */
int pgp_load_weights(pgp_model* m, const double* blob, size_t len);

/* Pre-allocate the device workspace for batches up to max_batch windows. */
int pgp_reserve(pgp_model* m, int max_batch);

/* detect + diagnose + generate for `batch` windows, all pointers on device:
 *   in  windows      [B,3,3H] normalised rows (run_encoder's window,
 *                    PreGANPlus.py:107-112; columns host-major cpu/ram/disk)
 *   in  sched        [B,C,H]  schedule (GOBI result_cache, PreGANPlus.py:117)
 *   out logits       [B,H,2]  anomaly decoder outputs (raw: LeakyReLU(True)=id)
 *   out protos       [B,H,2]  sigmoid prototype embeddings
 *   out cls          [B,H]    diagnosed class, -1 where no anomaly
 *   out any_anom     [B]      1 if any host is anomalous (else run_model
 *                             returns the original decision, :119-127)
 *   out probs        [B,2]    discriminator softmax
 *   out keep_orig    [B]      probs[0] > probs[1]
 *   out final_target [B,C]    first-argmax of sched rows
 *   out gen_target   [B,C]    first-argmax of the generator's rows
 * latent (may be NULL) receives the encoder output [B,3H^2] in the reference's
 * (host, step, channel) order (models.py:399) — a debug/test tap. */
int pgp_forward(pgp_model* m, int batch, const float* windows, const float* sched,
                float* logits, float* protos, int* cls, int* any_anom,
                float* probs, int* keep_orig, int* final_target, int* gen_target,
                float* latent, void* stream);

/* Per-kernel launches of pgp_forward, for profiling and kernel-level tests.
 * stage 0: GAT aggregation (K1), 1: encoder layers (K2), 2: decoders + detect
 * + classify (K2b), 3: GAN + decisions (K3); -1 = all, as pgp_forward.
 * Stages communicate through the model's workspace, so they must run in order
 * on one stream with the same batch. */
int pgp_forward_stage(pgp_model* m, int stage, int batch, const float* windows,
                      const float* sched, float* logits, float* protos, int* cls,
                      int* any_anom, float* probs, int* keep_orig, int* final_target,
                      int* gen_target, float* latent, void* stream);

/* recover_decision's container moves (PreGANPlus.py:87-105, PreGAN.py:77-95)
 * for a batch, from pgp_forward's keep_orig / final_target (device pointers):
 *   in  cur_host  [B,C] current host of container c, -1 = unplaced or None
 *                       (the containerlist filter, PreGANPlus.py:92-95); any
 *                       value outside [0, C) is treated as unplaced
 *   out moves     [B,C] new host where final_target != cur_host and the
 *                       discriminator did not keep the original, else -1
 *   out hosts_from[B,H] 1 for every host a container moves away from
 * C = H (Gen reshapes to H x H, models.py:133).  The decision list is
 * dict(original_decision) with moves[c] >= 0 overriding / appending key c in
 * host-ascending, then container order. */
int pgp_migrations(int n_hosts, int batch, const int* keep_orig, const int* final_target, const int* cur_host,
                   int* moves, int* hosts_from, void* stream);
/* run_model's embedding (PreGANPlus.py:129): emb[b,h,:] = protos[b,h,:] where
 * argmax(logits[b,h,:]) == 1 (ties -> 0), else 0.  fp32 device [B,H,2] each. */
int pgp_embedding(int n_hosts, int batch, const float* logits, const float* protos, float* emb, void* stream);
/* K2b's contraction form.  on = 1 (the default where compiled: H = 32, 50):
 * the decoder GEMM as six split-bf16 MFMAs per fp32 product (every operand
 * split exactly into three bf16 parts; error at the fp32 MFMA's level,
 * tools/micro/bf16_split.hip); on = 0: v_mfma_f32_16x16x4_f32.  Returns
 * PGP_ERR_UNSUPPORTED for on = 1 where the split form is not compiled. */
int pgp_decoder_split(pgp_model* m, int on);
/* K2's feed-forward form, likewise (the default where compiled: H = 50, the
 * tail-resident encoder): both layers' linear1 / linear2 as split-bf16 MFMAs
 * (planes derived on the device at each weight load / repack); on = 0: the
 * fp32 MFMA. */
int pgp_encoder_split(pgp_model* m, int on);
/* K3's contraction form, likewise (the default where compiled: H = 16, 50; also
 * the FPE variant's K3): Gen1, Disc1 and Gen2 as split-bf16 MFMAs, a schedule
 * block exactly representable in bf16 (one-hot GOBI rows) in three products
 * instead of six (the other three add exact zeros). */
int pgp_gan_split(pgp_model* m, int on);
/* The dense schedule pgp_forward reads, from per-container host indices: a
 * GOBI result_cache row is one-hot (scheduler/BaGTI/src/opt.py:9-15), so a
 * streamed fleet chunk (bench.py --config fleet, preganplus_amd/fleet.py)
 * carries one byte per container over PCIe instead of H floats.
 *   in  idx   [B,C] uint8 host of container c; >= n_hosts: an all-zero row
 *   out sched [B,C,H] fp32 device, sched[b,c,h] = (idx[b,c] == h)
 * C = H; n_hosts <= 255. */
int pgp_schedule_onehot(int n_hosts, int batch, const unsigned char* idx, float* sched, void* stream);

/* ------------------------------------------------------------------------
 * PreGAN (FPE) variant — BASELINE config C4, SURVEY.md §8 a14.
 * Replaces PreGANRecovery.run_encoder + the GAN half of run_model
 * (recovery/PreGAN.py:97-126): FPE_16.forward (models.py:65-115), detect
 * (argmax of each host's softmax, :110-111), embedding + get_classes over the
 * K = 3 prototypes (:119-120), Gen_16/Disc_16 (recover_decision, :74-77).
 * ---------------------------------------------------------------------- */
/* A PreGAN model for H hosts (H = 16 only: the reference defines FPE_16 alone). */
int pgp_create_fpe(int n_hosts, pgp_model** out);
/* Doubles pgp_load_weights expects for an FPE model, row-major in this order:
 *   FPE: gru.weight_ih_l0 [9,3H], gru.weight_hh_l0 [9,3], gru.bias_ih_l0 [9],
 *     gru.bias_hh_l0 [9], gat.layer1.heads.0.fc.weight [H,3],
 *     ...attn_fc.weight [1,2H], mha.in_proj_weight [3E,E], mha.in_proj_bias [3E],
 *     mha.out_proj.weight [E,E], mha.out_proj.bias [E] (E = H+3),
 *     encoder.0.weight [10H,3E], encoder.0.bias [10H],
 *     anomaly_decoder.0.weight [2,10], .bias [2],
 *     prototype_decoder.0.weight [2,10], .bias [2]
 *   Gen, Disc: as pgp_load_weights;  prototypes [3,2]. */
size_t pgp_fpe_weight_blob_len(int n_hosts);
/* Device pointers:
 *   in  windows [B,3,3H], h0 [B,3] (the GRU state the reference draws with
 *       torch.randn, models.py:70), sched [B,C,H]
 *   out scores [B,H,2] anomaly softmax, protos [B,H,2], cls [B,H] (-1: none),
 *       any_anom [B], probs [B,2], keep_orig [B], final_target [B,C],
 *       gen_target [B,C]  (as pgp_forward) */
int pgp_forward_fpe(pgp_model* m, int batch, const float* windows, const float* h0, const float* sched,
                    float* scores, float* protos, int* cls, int* any_anom, float* probs, int* keep_orig,
                    int* final_target, int* gen_target, void* stream);
/* Per-kernel launches of pgp_forward_fpe: stage 0 = K4 (FPE encoder, decoders,
 * detect, classify), 1 = K3 (GAN + decisions), -1 = both; in order, one stream. */
int pgp_forward_fpe_stage(pgp_model* m, int stage, int batch, const float* windows, const float* h0,
                          const float* sched, float* scores, float* protos, int* cls, int* any_anom, float* probs,
                          int* keep_orig, int* final_target, int* gen_target, void* stream);

/* ------------------------------------------------------------------------
 * Online training ops (stateless; buffers owned by the caller, device memory).
 * Master weights `P` are fp32 in the NATURAL blob order of pgp_load_weights
 * (transformer | gen | disc, prototypes excluded); grads `G` share the layout.
 * Replace, per window (or summed over a batch of windows):
 *   pgp_tune_forward   Transformer forward in train mode (dropout p=0),
 *                      models.py:376-416, saving activations in `scratch`
 *   pgp_tune_backward  custom_loss / triplet_loss gradients (train.py:13-40;
 *                      the sequential prototype/counter logic stays on the host
 *                      and arrives as y, mult, tgt) + backward into G
 *                      (loss.backward(), train.py:53)
 *   pgp_gan_forward    Gen + Disc forward (PreGANPlus.py:62-63)
 *   pgp_gan_disc_backward  BCE(probs, target) backward; the Disc grads are
 *                      WRITTEN (not accumulated) into G's disc section (:66-67)
 *   pgp_gan_gen_backward   Disc forward with the updated Disc, BCE toward [0,1],
 *                      backward; the Gen grads are written into G's gen section (:69-74)
 *   pgp_adamw          torch.optim.AdamW.step (utils.py:65)
 * ---------------------------------------------------------------------- */
size_t pgp_master_len(int n_hosts);               /* floats in P / G            */
/* floats of tuning workspace for a batch (activations saved by the forward for
 * the backward, token-major, plus split-K / weight-gradient partial slabs).
 * Sizes grow with batch: a workspace for B_max serves every batch <= B_max.
 * Zero-fill it once before its first use: its head holds device counters
 * (last-part finishes of the backward's reductions) that every call leaves at
 * zero. */
size_t pgp_tune_workspace_len(int n_hosts, int batch);
/* floats of GAN-step workspace for a batch (one activation row per
 * environment); grows with batch like the tuning workspace; zero-filled once
 * before first use (per-block counters of the split form, left at zero). */
size_t pgp_gan_workspace_len(int n_hosts, int batch);
size_t pgp_master_offset(int n_hosts, int section); /* 0 transformer, 1 gen, 2 disc */

/* windows [B,3,3H]; outputs logits [B,H,2], protos [B,H,2] (sigmoid) and, if
 * latent != NULL, the encoder output [B,3H^2] in the reference's order;
 * workspace: pgp_tune_workspace_len(H, >= B) floats, kept for the backward. */
int pgp_tune_forward(int n_hosts, int batch, const float* windows, const float* P, float* workspace,
                     float* latent, float* logits, float* protos, void* stream);
/* After pgp_tune_forward with the same batch and workspace: y [B,H] int
 * labels, mult [B,H] CE weights, tgt [B,H,2] positive prototypes (only rows
 * with y>0 used).  WRITES the gradient of the summed per-window losses into
 * the transformer section of G (every trainable entry is written exactly once
 * by the call's reductions: no zeroing needed; the non-trainable positional
 * encoding's entries are left as they are). */
int pgp_tune_backward(int n_hosts, int batch, const float* P, float* G, float* workspace, const float* logits,
                      const float* protos, const int* y, const float* mult, const float* tgt, void* stream);
/* The same backward over the FIRST `batch` windows of a pgp_tune_forward of
 * fwd_batch >= batch windows (same workspace; logits / protos / y / mult / tgt
 * of those windows): a caller that appends inference windows to the tuning
 * batch (the C3 detect: run_encoder's windows, PreGANPlus.py:107-113, read the
 * same step-start weights) runs one forward for both and differentiates only
 * the tuning windows.  pgp_tune_backward(B) == pgp_tune_backward_prefix(B, B). */
int pgp_tune_backward_prefix(int n_hosts, int fwd_batch, int batch, const float* P, float* G, float* workspace,
                             const float* logits, const float* protos, const int* y, const float* mult,
                             const float* tgt, void* stream);
/* Streams: both calls may run part of their work (the decoder weight packing;
 * the decoders' and in_proj's weight gradients) on a library-owned,
 * low-priority stream of the current device, forked from `stream` by an event
 * and joined back into it before the call's last launch, so every result is
 * ordered on `stream` as if all of it ran there.  While `stream` is being
 * captured into a graph the fork / join are captured too (the graph holds the
 * two branches).
 * pgp_tune_set_side_stream(s): use the caller's stream `s` as that side stream
 * on the current device from now on (NULL: the library's own again).  A
 * data-parallel caller that already runs a second stream (the GAN step) and two
 * communicators keeps its streams within the hardware queues this way; `s`
 * equal to the call's own `stream` keeps everything on that one stream. */
int pgp_tune_set_side_stream(void* stream);
/* pgp_tune_reserve_cus(n): the fused encoder launches of pgp_tune_forward /
 * pgp_tune_backward use at most (CUs - n) workgroups (one per CU; at most half
 * the CUs are reserved), leaving n CUs free for a concurrent stream (the GAN
 * step beside the tuning step): a fused launch deals its units to its waves
 * statically, so a CU held by another stream's workgroup would hold back the
 * whole launch.  Within that budget a launch takes the fewest workgroups whose
 * longest wave has as many units as on the whole budget (units are whole
 * 16-pair tiles), so it ends as early and leaves the rest of the CUs to other
 * streams too.  Default 0.  Results do not depend on it beyond fp32 summation
 * grouping of the weight gradients (one slab per workgroup). */
int pgp_tune_reserve_cus(int n);
/* Profiling: with pgp_tune_timing(1), pgp_tune_forward / pgp_tune_backward
 * record HIP events on their stream around each fused encoder launch
 * (pgp_tunef.hip); pgp_tune_fused_ms(ms6) synchronises on them and returns the
 * last forward + backward's six durations [fwd layer 0, fwd layer 1, ffn
 * backward layer 1, attention backward layer 1, ffn backward layer 0,
 * attention backward layer 0] in ms.  Off by default (not graph-capturable). */
int pgp_tune_timing(int on);
int pgp_tune_fused_ms(float* ms6);
/* custom_loss / triplet_loss bookkeeping of ONE window (train.py:13-40,
 * replaces the host loop between `model(...)` and `loss.backward()` in
 * backprop, train.py:47-53), on the stream: reads the batch-1 forward's logits
 * [H,2] / protos [H,2], labels y [H] and classes cls [H] (int32, 0-2 where
 * y>0); updates state [2K+3] fp64 = prototypes [K][2] (model.prototype,
 * K = n_protos >= 3; triplet_loss uses rows 0-2), PROTO_UPDATE_FACTOR,
 * num_zero, num_ones in place in the reference's order; writes mult [H], tgt [H,2] (the inputs of
 * pgp_tune_backward) and loss [2] fp64 = (aloss, tloss).  update_min / decay =
 * constants.py PROTO_UPDATE_MIN / PROTO_FACTOR_DECAY.  Lets a backprop loop of
 * sequential batch-1 steps run without a host round trip. */
int pgp_tune_targets(int n_hosts, int n_protos, const float* logits, const float* protos, const int* y, const int* cls,
                     double* state, double update_min, double decay, float* mult, float* tgt, double* loss,
                     void* stream);
/* ONE whole batch-1 tuning step of backprop (train.py:46-53: model(window),
 * custom_loss, loss.backward()) in a single launch, for n_hosts 8 or 16:
 * pgp_tune_forward + pgp_tune_targets + pgp_tune_backward with batch 1 fused.
 * window [3,3H], y / cls [H] int32, state as pgp_tune_targets (updated in
 * place); writes logits [H,2], protos [H,2], loss [2] fp64 and the whole
 * transformer section of G (overwritten, no zeroing needed; the gen / disc
 * sections are untouched).  The AdamW step stays a separate launch. */
int pgp_tune_step1(int n_hosts, int n_protos, const float* window, const int* y, const int* cls, const float* P,
                   float* G, double* state, double update_min, double decay, float* logits, float* protos,
                   double* loss, void* stream);
/* n independent batch-1 tuning forwards from the master P (n_hosts 8 or 16;
 * one workgroup per window, the forward of pgp_tune_step1): the batched
 * model(windows) that accuracy() scores (train.py:94-109, PreGANPlus.py:56).
 * windows [n,3,3H] fp32; writes logits [n,H,2] and protos [n,H,2] as fp64
 * (the values are the fp32 results, widened).  Replaces pgp_tune_forward for
 * this use at 8 / 16 hosts. */
int pgp_tune_forward_many(int n_hosts, int n_windows, const float* windows, const float* P, double* logits,
                          double* protos, void* stream);
/* run_model's per-interval forward for ONE window (PreGANPlus.py:115-136:
 * run_encoder, detect / embed / get_classes, Gen + Disc, the recover_decision
 * gate and targets), n_hosts 8 or 16, in a single launch, straight from the
 * training master P (natural fp32, as pgp_tune_*) and prototypes [K,2] fp64
 * on the device — no packed weights.  window [3,3H], sched [H,H]; outputs as
 * pgp_forward at batch 1 (logits [H,2], protos [H,2], cls [H], any [1],
 * probs [2], keep [1], final_target [H], gen_target [H]). */
int pgp_forward1(int n_hosts, int n_protos, const float* window, const float* sched, const float* P,
                 const double* prototypes_device, float* logits, float* protos, int* cls, int* any_anom, float* probs,
                 int* keep_orig, int* final_target, int* gen_target, void* stream);
/* ---- data-parallel tuning step on the device ----
 * pgp_tune_dataset replaces load_on_the_fly_dataset (utils.py:40-47) for a
 * batch of E environments: series [E,R,3H] fp64 = each environment's last R
 * rows of stats.time_series (R = LATEST_WINDOW_SIZE = 10, 1 <= R <= 16),
 * train_max [3H] fp64 = np.max(train_time_data, axis=0); normalises
 * (utils.py:94-95), writes the R windows per environment (convert_to_windows,
 * utils.py:7-14) windows [E*R,3,3H] fp32, the labels of form_test_dataset
 * (utils.py:16-24; bit-exact numpy 'linear' 98th percentile) y [E*R,H] and
 * cls [E*R,H] int32, and, if infer != NULL, run_encoder's window of the same
 * rows (PreGANPlus.py:107-112: [R-3, R-3, R-2]) infer [E,3,3H]. */
int pgp_tune_dataset(int n_hosts, int n_env, int n_rows, const double* series, const double* train_max,
                     float* windows, int* y, int* cls, float* infer, void* stream);
/* doubles of workspace pgp_tune_targets_dp needs for a batch (zero-filled
 * once before first use: slot 0 is the finishing counter, left at zero) */
size_t pgp_tune_targets_dp_workspace_len(int batch);
/* custom_loss / triplet_loss (train.py:13-40) for a batch in the data-parallel
 * form (train.loss_targets_dp; replaces its B x H host loop): every window is
 * scored against the step-start state [2K+3] (read only); writes mult [B,H],
 * tgt [B,H,2] (pgp_tune_backward's inputs), loss [B,2] fp64 (aloss, tloss) and
 * the rank's state increments inc [3K+3] fp64 = prototype-EMA deltas [K][2]
 * (f (a - P[c]) per qualifying host, f = factor + update_min), their counts [K],
 * num_zero, num_ones, windows — the buffer the ranks all-reduce (sum). */
int pgp_tune_targets_dp(int n_hosts, int n_protos, int batch, const float* logits, const float* protos, const int* y,
                        const int* cls, const double* state, double update_min, float* mult, float* tgt, double* loss,
                        double* inc, double* workspace, void* stream);
/* train.dp_state_update after the all-reduce, on the device: state [2K+3] +=
 * the summed increments (each prototype moves by the mean of its deltas, the
 * factor decays by decay^windows).  AdamW activity of the n_cond tensors that
 * torch skips when no window of the global batch has a positive label (the
 * prototype decoder, train.py:51-54 -> torch.optim.AdamW): their step counts
 * cond_steps [n_cond] fp64 live on the device; rows cond_rows[i] of the
 * pgp_adamw_table table [T,3] get (active, lr/(1-beta1^step), sqrt(1-beta2^step)). */
int pgp_tune_state_apply(int n_protos, double* state, const double* inc, double decay, int n_cond,
                         const int* cond_rows, double* cond_steps, float* adam_table, double lr, double beta1,
                         double beta2, void* stream);
/* emb [B,2H] (masked prototype embeddings), sched [B,H,H]; outputs the new
 * schedule ns [B,H,H] and probs [B,2]; workspace pgp_gan_workspace_len(H, >= B)
 * floats, shared by the three calls of one step (same batch).  The backward
 * calls accumulate the gradient summed over the batch's windows into G. */
int pgp_gan_forward(int n_hosts, int batch, const float* emb, const float* sched, const float* P, float* workspace,
                    float* ns, float* probs, void* stream);
/* target [B,2]: the BCE label (PreGANPlus.py:65-66) */
int pgp_gan_disc_backward(int n_hosts, int batch, const float* target, const float* P, float* G, float* workspace,
                          void* stream);
int pgp_gan_gen_backward(int n_hosts, int batch, const float* P, float* G, float* workspace, void* stream);
/* probs [B,2] of the last Disc head evaluated in the workspace: after
 * pgp_gan_gen_backward, the updated Disc's probabilities of the generator's
 * schedule, whose BCE toward [0,1] is gen_loss (PreGANPlus.py:69-73; the
 * reference appends (gen_loss, disc_loss) to accuracy_list, :77). */
int pgp_gan_probs(int n_hosts, int batch, const float* workspace, float* probs, void* stream);

typedef struct {
  long long offset;  /* first element of the tensor in P/G/m/v */
  int n;             /* elements */
  int active;        /* 0: the tensor got no gradient (torch skips it) */
  float step_size;   /* lr / (1 - beta1^step) for this tensor's new step */
  float bc2_sqrt;    /* sqrt(1 - beta2^step) */
} pgp_adam_tensor;
int pgp_adamw(float* P, const float* G, float* exp_avg, float* exp_avg_sq, float lr, float weight_decay,
              float beta1, float beta2, float eps, const pgp_adam_tensor* tensors, int ntensors, void* stream);
/* pgp_adamw with the per-step scalars read from the device: sched [ntensors][3]
 * fp32 = (active, step_size, bc2_sqrt) replaces the fields of `tensors` (only
 * offset / n are used from it).  The kernel's arguments then do not change
 * from step to step, so a loop of optimizer steps can be captured once in a
 * HIP graph and replayed with a new table (backprop, train.py:42-57). */
int pgp_adamw_table(float* P, const float* G, float* exp_avg, float* exp_avg_sq, float lr, float weight_decay,
                    float beta1, float beta2, float eps, const pgp_adam_tensor* tensors, int ntensors,
                    const float* sched, void* stream);

/* train_gan (PreGANPlus.py:60-81) for ONE window in two launches, n_hosts 8 or
 * 16 (the plugin's per-interval call), replacing pgp_gan_forward +
 * pgp_gan_disc_backward + pgp_adamw_table(disc) + pgp_gan_gen_backward +
 * pgp_gan_probs + pgp_adamw_table(gen) + pgp_gan_forward at batch 1:
 * pgp_gan_forward1: emb [2H], sched [H,H] -> ns [H,H] (the generator's
 * schedule), probs [2] (Disc on it); saves the window's activations in the GAN
 * workspace (pgp_gan_workspace_len(H, 1) floats).
 * pgp_gan_step1, after the host simulator's label target [2]: the Disc BCE step
 * (gradients written into G's disc section, AdamW over disc_tensors with the
 * device table disc_sched [n_disc,3] as pgp_adamw_table), the Gen step through
 * the updated Disc (probs_gen [2] = the Disc probabilities it saw, gen_loss's
 * input) with its AdamW over gen_tensors / gen_sched, then the updated GAN's
 * Disc probabilities on the same inputs -> probs_after [2] (recover_decision's
 * gate, PreGANPlus.py:84-87).  Tensor offsets index P / G / m / v and must lie
 * in the disc / gen sections. */
int pgp_gan_forward1(int n_hosts, const float* emb, const float* sched, const float* P, float* workspace, float* ns,
                     float* probs, void* stream);
int pgp_gan_step1(int n_hosts, const float* target, float* P, float* G, float* exp_avg, float* exp_avg_sq,
                  float lr_disc, float lr_gen, float weight_decay, float beta1, float beta2, float eps,
                  const pgp_adam_tensor* disc_tensors, int n_disc, const float* disc_sched,
                  const pgp_adam_tensor* gen_tensors, int n_gen, const float* gen_sched, float* workspace,
                  float* probs_gen, float* probs_after, void* stream);

/* ---------------------------------------------------------------------------
 * The whole online training step of run_model in ONE call (BASELINE config
 * C3; replaces, per interval and for a batch of E environments, the sequence
 * PreGANPlus.py:115-136 minus the decision: run_encoder + detect/embed
 * (:107-131), train_gan (:60-81 -> utils.py:97-100 runSimulation), tune_model
 * (:51-58 -> utils.py:40-47 load_on_the_fly_dataset, train.py:42-57 backprop in
 * the data-parallel form of SURVEY §8e), i.e. the composition of
 * pgp_tune_dataset, pgp_tune_forward, pgp_embedding, pgp_gan_forward,
 * pgp_simulate, pgp_gan_disc_backward, pgp_adamw, pgp_gan_gen_backward,
 * pgp_tune_targets_dp, pgp_tune_backward_prefix, pgp_tune_state_apply).
 * pgp_online_create takes every buffer once (caller-owned device memory):
 *   series [E,R,3H] f64, train_max [3H] f64, sched [E,H,H] f32 (the original
 *   schedules), envs [E, pgp_sim_env_len(H)] f64 (simulation records);
 *   P / G / exp_avg / exp_avg_sq: the master (pgp_master_len(H) floats);
 *   tune_ws: pgp_tune_workspace_len(H, E*R + E) floats; logits / protos
 *   [E*R+E, H, 2]; windows [E*R+E, 3, 3H] (the tuning windows, then detect's);
 *   y / cls [E*R, H] int32; state [2K+3] f64 (prototypes, factor, num_zero,
 *   num_ones: updated in place); mult [E*R,H]; tgt [E*R,H,2]; loss [E*R,2] f64;
 *   inc [3K+3] f64; dp_ws pgp_tune_targets_dp_workspace_len(E*R) doubles;
 *   adam_rows [n_tensors of section 0][3] f32 (the conditional rows,
 *   written on the device); cond_steps [n_cond] f64 (their step counts);
 *   gan_ws pgp_gan_workspace_len(H, E) floats; ns [E,H,H]; probs [E,2];
 *   emb [E,H,2]; sim_out [E,4] f64; target [E,2] f32.
 *   tensors: every trainable tensor of the three sections (0 Transformer,
 *   1 Gen, 2 Disc) in blob order, with its AdamW step count so far; `cond`
 *   marks the prototype decoder's (no gradient when the global batch has no
 *   positive label: their activity and step counts live on the device).
 * pgp_online_step issues one step on main_stream (tuning) and gan_stream (the
 * GAN step, beside it; NULL: main_stream), the main stream waiting for the GAN
 * stream at the end.  AdamW's per-step scalars are the host's (double, rounded
 * to fp32 as torch's AdamW computes them per step).  `cb` (NULL at world size
 * 1) performs the data-parallel exchange in place, ordered on `stream`:
 * PGP_COLL_DISC_GRAD / PGP_COLL_GEN_GRAD (the Disc / Gen sections of G, on the
 * GAN stream), PGP_COLL_TUNE_GRAD (the Transformer section of G) and
 * PGP_COLL_TUNE_STATE (inc), on the main stream; the same order on every rank.
 * pgp_online_timing(h, 1) records HIP events in later steps;
 * pgp_online_stage_ms(h, ms[PGP_ONLINE_NSTAGE]) returns the last step's spans:
 * dataset, embedding (folded into the GAN forward's first launch since round 5:
 * an empty span, kept so the array layout is stable), train_gan, tune_model,
 * forward, targets, backward, exchange, state + AdamW, whole main stream.  pgp_online_steps returns the
 * host step counts (in `tensors` order; -1 for the conditional tensors). */
typedef struct {
  long long offset;  /* first element in P/G/m/v */
  int n;
  int section;       /* 0 Transformer, 1 Gen, 2 Disc */
  int cond;          /* prototype decoder (device-side activity) */
  double step;       /* AdamW steps taken so far */
} pgp_online_tensor;
typedef struct {
  int n_hosts, n_env, n_rows, n_protos;
  const double* series;
  const double* train_max;
  const float* sched;
  const double* envs;
  float *P, *G, *exp_avg, *exp_avg_sq;
  float* tune_ws;
  float *logits, *protos, *windows;
  int *y, *cls;
  double* state;
  float *mult, *tgt;
  double *loss, *inc, *dp_ws;
  float* adam_rows;
  double* cond_steps;
  float *gan_ws, *ns, *probs, *emb;
  double* sim_out;
  float* target;
  const pgp_online_tensor* tensors;
  int n_tensors, n_cond;
  double lr[3]; /* per section */
  double weight_decay, beta1, beta2, eps, update_min, decay;
} pgp_online_desc;
typedef struct pgp_online pgp_online;
typedef int (*pgp_collective_fn)(void* user, int which, void* stream);
#define PGP_COLL_DISC_GRAD 0
#define PGP_COLL_GEN_GRAD 1
#define PGP_COLL_TUNE_GRAD 2
#define PGP_COLL_TUNE_STATE 3
#define PGP_ONLINE_NSTAGE 10
int pgp_online_create(const pgp_online_desc* desc, pgp_online** out);
int pgp_online_destroy(pgp_online* h);
int pgp_online_step(pgp_online* h, void* main_stream, void* gan_stream, pgp_collective_fn cb, void* user);
int pgp_online_timing(pgp_online* h, int on);
/* pgp_online_issue_worker(h, on): at world size 1 with two streams, issue the
 * GAN stream's launches from a second host thread of the library while the
 * calling thread issues the tuning backward (default on; 0: one thread issues
 * both, as under a callback or timing). */
int pgp_online_issue_worker(pgp_online* h, int on);
int pgp_online_stage_ms(pgp_online* h, float* ms);
int pgp_online_steps(const pgp_online* h, double* steps, int n);
/* The step's GAN part alone (train_gan, PreGANPlus.py:60-81, for the E
 * environments, from the detect rows of the last step's forward), on `stream`,
 * world size 1: what pgp_online_step runs on its GAN stream (a measurement
 * entry: it advances the GAN's AdamW step counts like a step). */
int pgp_online_gan_step(pgp_online* h, void* stream);

/* ---------------------------------------------------------------------------
 * Offline training of PreGAN's FPE_16 (PreGAN.py:26-27, 39-49: a new FPE is
 * trained when no checkpoint exists, train.py:42-57).  P / G: the FPE's
 * parameters, natural fp32 blob in state_dict order (pgp_fpe_param_len(16) =
 * 11401 floats).
 * pgp_fpe_train_step: one sequential batch-1 step of backprop: FPE forward of
 *   window [3,48] with GRU state h0 [3] (the reference's torch.randn draw,
 *   models.py:70), custom_loss / triplet_loss bookkeeping on state [2K+3]
 *   fp64 (prototypes [K][2], factor, num_zero, num_ones; as pgp_tune_targets),
 *   loss [2] fp64 = (aloss, tloss), and the gradient WRITTEN into G.  The
 *   AdamW step that follows is pgp_adamw / pgp_adamw_table over P, G.
 * pgp_fpe_forward_many: n independent forwards (accuracy(), train.py:94-109):
 *   windows [n,3,48], h0 [n,3] -> probs / protos [n,16,2] fp64. */
size_t pgp_fpe_param_len(int n_hosts);
int pgp_fpe_train_step(int n_hosts, int n_protos, const float* window, const float* h0, const int* y, const int* cls,
                       const float* P, float* G, double* state, double update_min, double decay, double* loss,
                       void* stream);
int pgp_fpe_forward_many(int n_hosts, int n, const float* windows, const float* h0, const float* P, double* probs,
                         double* protos, void* stream);

/* Rebuild the inference layouts from device master weights P (natural fp32)
 * and prototypes [K,2] (host, fp64): the sync after an optimizer step, via the
 * host packer (a device-to-host copy of P, pack, upload; synchronous). */
int pgp_load_weights_master(pgp_model* m, const float* P_device, const double* prototypes);
/* The same rebuild ON THE DEVICE, asynchronous on `stream`: P natural fp32 and
 * prototypes_device [K,2] fp64 (e.g. the head of the tuning state vector) are
 * read by three repack launches that write the model's packed buffers in
 * place — the same bits as pgp_load_weights_master (shared packing code,
 * fp64, no contraction).  Replaces the host round trip after an optimizer step
 * (the reference's AdamW updates the modules in place, utils.py:64-65;
 * PreGANPlus.py:115-136 runs the next interval on the updated model).  The
 * model must have been loaded once (pgp_load_weights). */
int pgp_repack_master(pgp_model* m, const float* P_device, const double* prototypes_device, void* stream);
/* One part of that rebuild: sections bit 0 = the PreGAN+ encoder / decoders
 * (the transformer section of P and the prototypes: three launches), bit 1 =
 * the GAN (Gen / Disc sections: one launch); 3 = pgp_repack_master.  Either
 * part may run as soon as its section of P is final (the online interval
 * repacks the PreGAN+ part after the tuning step while the GAN step runs,
 * then only the GAN part after it); the two write disjoint packed regions. */
int pgp_repack_master_sections(pgp_model* m, const float* P_device, const double* prototypes_device, int sections,
                               void* stream);

/* ------------------------------------------------------------------------
 * GOBI, the schedule producer: replaces
 * GOBIScheduler.run_GOBI's optimiser (scheduler/GOBI.py:19-42) =
 * opt() in scheduler/BaGTI/src/opt.py:17-33 over the energy_latency_16
 * surrogate (scheduler/BaGTI/src/models.py:8-27), for a batch of independent
 * environments.  Its result's allocation columns are run_model's schedule input
 * (env.scheduler.result_cache, PreGANPlus.py:117).
 * ---------------------------------------------------------------------- */
typedef struct pgp_gobi pgp_gobi;
/* floats of the surrogate's state dict (find.0.weight [128,288], find.0.bias,
 * find.2.weight [128,128], find.2.bias, find.4.weight [64,128], find.4.bias,
 * find.6.weight [2,64], find.6.bias), fp32 row-major; 0 if H is not 16 */
size_t pgp_gobi_weight_len(int n_hosts);
int pgp_gobi_create(int n_hosts, const float* weights, size_t len, pgp_gobi** out);
int pgp_gobi_destroy(pgp_gobi* g);
const char* pgp_gobi_last_error(void);
/* device pointers: init / result [E,16,18] (per container: host cpu, container
 * ips, one-hot host), iterations [E] (opt()'s returned count), fitness [E]
 * (surrogate value of the result).  max_iters <= 0: the reference's 200.
 * pre (may be NULL) [E,16,16]: the last step's allocation values before the
 * one-hot projection (a test tap). */
int pgp_gobi_optimize(pgp_gobi* g, int n_env, const float* init, float* result, int* iterations,
                      float* fitness, int max_iters, float* pre, void* stream);

/* ---- GAN-label simulation ----
 * Replaces the two env.stats.runSimulation calls of train_gan
 * (PreGANPlus.py:65 -> utils.py:97-100 -> Stats.py:154-177) for a batch of
 * environments.  Each environment is one fp64 record of pgp_sim_env_len(H) =
 * 2 + 20H doubles (C = H containers; layout in preganplus_amd/simulate.py):
 *   interval time, latency term max(0, mean(avgresponsetime[-5:])),
 *   host[C] (-1: none/unplaced), base_ips[C], ram_size[C], disk_size[C],
 *   apparent_ips[C], ips_available[H], ram_available[H], disk_available[H],
 *   ips_cap[H], power_list[H][11]  (the values the reference's getters return).
 * new_sched / orig_sched [E,C,H] fp32 (generator output, original schedule).
 * out [E,4] fp64 = (energy·interval, 0.8·energy + 0.2·latency) of the new,
 * then of the original schedule, bit-identical to the reference's Python;
 * target [E,2] fp32 = [0,1] if new <= orig else [1,0] (PreGANPlus.py:66), the
 * target argument of pgp_gan_disc_backward.  1 <= H <= 64. */
size_t pgp_sim_env_len(int n_hosts);
int pgp_simulate(int n_hosts, int n_env, const double* envs, const float* new_sched, const float* orig_sched,
                 double* out, float* target, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PREGANPLUS_H */
