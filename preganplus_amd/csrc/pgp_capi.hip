// pgp_capi.hip — the C-ABI of include/preganplus.h: model lifetime, weight
// upload, workspace, and the launch sequence of one forward call:
//   K1 gat (pgp_gat.hip) -> K2 encoder (pgp_encoder.hip) ->
//   K2b decoders+classify (pgp_decoder.hip) -> K3 GAN+decisions (pgp_gan.hip)
// and of the PreGAN (FPE) variant: K4 FPE encoder+classify (pgp_fpe.hip) -> K3
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/preganplus.h"
#include "pgp_device.hpp"
#include "pgp_pack.hpp"
#include "pgp_repack.hpp"
#include "pgp_train.hpp"
#include "pgp_tune.hpp"
#include "pgp_tunef.hpp"
#include "pgp_tunedp.hpp"

#include <vector>

using namespace pgp;

struct pgp_model {
  int H = 0, K = 0;
  bool fpe = false;  // PreGAN FPE_16 variant (pgp_create_fpe)
  bool loaded = false;
  float* d_frags = nullptr;
  float* d_decb = nullptr;   // split-bf16 decoder planes (derived from d_frags on the device)
  float* d_encb = nullptr;   // split-bf16 encoder LDS image (derived likewise)
  bool enc_split = true;     // K2's feed-forward on the split-bf16 planes where compiled (pgp_encoder_split)
  bool dec_split = true;     // K2b on the split-bf16 planes where compiled (pgp_decoder_split)
  float* d_ganb = nullptr;   // split-bf16 GAN planes (derived from d_frags on the device)
  bool gan_split = true;     // K3 on the split-bf16 planes where compiled (pgp_gan_split)
  float* d_tab = nullptr;
  float* d_gtab = nullptr;
  float* d_gat = nullptr;    // GAT constants u[4] | v[4] (K1 reads them on the device)
  double* d_pscr = nullptr;  // device repack scratch (pgp_repack_master)
  int cap = 0;  // workspace capacity in windows
  float* d_agg = nullptr;
  float* d_lat = nullptr;
  float* d_emb = nullptr;
};

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return fail(PGP_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

bool supported(int H) {
  switch (H) {
#define CASE(h) case h:
    PGP_FOR_EACH_H(CASE)
#undef CASE
    return true;
  }
  return false;
}

long lat_blk(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return Geo<h>::LAT_BLK;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

int reserve(pgp_model* m, int n) {
  if (n <= m->cap) return PGP_OK;
  for (float** p : {&m->d_agg, &m->d_lat, &m->d_emb})
    if (*p) {
      HIPCHK(hipFree(*p));
      *p = nullptr;
    }
  m->cap = 0;
  const size_t nblk = (size_t)(n + 15) / 16;
  const size_t agg_f = m->fpe ? 4 : nblk * m->H * 3 * 48;  // the FPE variant needs only emb
  const size_t lat_f = m->fpe ? 4 : nblk * (size_t)lat_blk(m->H);
  const size_t emb_f = nblk * 16 * round_up(2 * m->H, 16);
  HIPCHK(hipMalloc(&m->d_agg, agg_f * sizeof(float)));
  HIPCHK(hipMalloc(&m->d_lat, lat_f * sizeof(float)));
  HIPCHK(hipMalloc(&m->d_emb, emb_f * sizeof(float)));
  HIPCHK(hipMemset(m->d_agg, 0, agg_f * sizeof(float)));
  HIPCHK(hipMemset(m->d_lat, 0, lat_f * sizeof(float)));
  HIPCHK(hipMemset(m->d_emb, 0, emb_f * sizeof(float)));
  m->cap = n;
  return PGP_OK;
}
}  // namespace

int pgp::set_error(int code, const std::string& msg) { return fail(code, msg); }

extern "C" {

int pgp_abi_version(void) { return PGP_ABI_VERSION; }
const char* pgp_last_error(void) { return g_err.c_str(); }

int pgp_supported_hosts(int* out, int cap) {
  int n = 0;
#define CASE(h)                         \
  if (out && n < cap) out[n] = h;       \
  ++n;
  PGP_FOR_EACH_H(CASE)
#undef CASE
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

size_t pgp_fpe_weight_blob_len(int n_hosts) { return fpe_blob_len(n_hosts); }

int pgp_create_fpe(int n_hosts, pgp_model** out) {
  if (!out) return fail(PGP_ERR_ARG, "out is NULL");
  *out = nullptr;
  if (fpe_blob_len(n_hosts) == 0)
    return fail(PGP_ERR_UNSUPPORTED, "FPE variant: host count not compiled in: " + std::to_string(n_hosts));
  pgp_model* m = new pgp_model();
  m->H = n_hosts;
  m->K = 3;
  m->fpe = true;
  *out = m;
  return PGP_OK;
}

int pgp_destroy(pgp_model* m) {
  if (!m) return PGP_OK;
  for (float* p : {m->d_frags, m->d_decb, m->d_encb, m->d_ganb, m->d_tab, m->d_gtab, m->d_agg, m->d_lat, m->d_emb, m->d_gat})
    if (p) (void)hipFree(p);
  if (m->d_pscr) (void)hipFree(m->d_pscr);
  delete m;
  return PGP_OK;
}

int pgp_load_weights(pgp_model* m, const double* blob, size_t len) {
  if (!m || !blob) return fail(PGP_ERR_ARG, "NULL model or blob");
  Packed P;
  const std::string err = m->fpe ? pack_fpe_weights(m->H, blob, len, &P) : pack_weights(m->H, m->K, blob, len, &P);
  if (!err.empty()) return fail(PGP_ERR_ARG, err);
  if (!m->d_frags) HIPCHK(hipMalloc(&m->d_frags, P.frags.size() * sizeof(float)));
  if (!m->d_tab) HIPCHK(hipMalloc(&m->d_tab, P.enc_tab.size() * sizeof(float)));
  if (!m->d_gtab) HIPCHK(hipMalloc(&m->d_gtab, P.gan_tab.size() * sizeof(float)));
  HIPCHK(hipMemcpy(m->d_frags, P.frags.data(), P.frags.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(m->d_tab, P.enc_tab.data(), P.enc_tab.size() * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(m->d_gtab, P.gan_tab.data(), P.gan_tab.size() * sizeof(float), hipMemcpyHostToDevice));
  if (!m->d_gat) HIPCHK(hipMalloc(&m->d_gat, sizeof(GatConst)));
  HIPCHK(hipMemcpy(m->d_gat, &P.gat, sizeof(GatConst), hipMemcpyHostToDevice));
  if (!m->fpe && decoder_split_floats(m->H) > 0) {
    if (!m->d_decb) HIPCHK(hipMalloc(&m->d_decb, decoder_split_floats(m->H) * sizeof(float)));
    HIPCHK(launch_decoder_split(m->H, m->d_frags, m->d_decb, nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));
  }
  if (!m->fpe && encoder_split_floats(m->H) > 0) {
    if (!m->d_encb) HIPCHK(hipMalloc(&m->d_encb, encoder_split_floats(m->H) * sizeof(float)));
    HIPCHK(launch_encoder_split(m->H, m->d_frags, m->d_encb, nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));
  }
  if (gan_split_floats(m->H) > 0) {
    if (!m->d_ganb) HIPCHK(hipMalloc(&m->d_ganb, gan_split_floats(m->H) * sizeof(float)));
    HIPCHK(launch_gan_split_derive(m->H, m->d_frags, m->d_ganb, nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));
  }
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
  if (m->fpe) return fail(PGP_ERR_STATE, "FPE model: use pgp_forward_fpe");
  if (batch < 0) return fail(PGP_ERR_ARG, "negative batch");
  if (stage < -1 || stage > 3) return fail(PGP_ERR_ARG, "bad stage");
  if (batch == 0) return PGP_OK;  // empty batch: nothing to read or write (pointers may be NULL)
  const bool all = stage == -1;
  if (((all || stage == 0) && !windows) ||
      ((all || stage == 2) && (!logits || !protos || !cls || !any_anom)) ||
      ((all || stage == 3) && (!sched || !probs || !keep_orig || !final_target || !gen_target)))
    return fail(PGP_ERR_ARG, "NULL input/output pointer");
  if (batch > m->cap) {
    const int rc = reserve(m, batch);
    if (rc) return rc;
  }
  FwdArgs a{};
  a.B = batch;
  a.H = m->H;
  a.K = m->K;
  a.windows = windows;
  a.sched = sched;
  a.agg = m->d_agg;
  a.lat = m->d_lat;
  a.emb = m->d_emb;
  a.frags = m->d_frags;
  a.decb = m->dec_split ? m->d_decb : nullptr;
  a.encb = m->enc_split ? m->d_encb : nullptr;
  a.ganb = m->gan_split ? m->d_ganb : nullptr;
  a.tab = m->d_tab;
  a.gtab = m->d_gtab;
  a.gat = m->d_gat;
  a.logits = logits;
  a.protos = protos;
  a.cls = cls;
  a.any_anom = any_anom;
  a.probs = probs;
  a.keep = keep_orig;
  a.final_t = final_target;
  a.gen_t = gen_target;
  a.latent = latent;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (all || stage == 0) HIPCHK(launch_gat(a, st));
  if (all || stage == 1) HIPCHK(launch_encoder(a, st));
  if (all || stage == 2) HIPCHK(launch_decoder(a, st));
  if (all || stage == 3) HIPCHK(launch_gan(a, st));
  return PGP_OK;
}

int pgp_forward(pgp_model* m, int batch, const float* windows, const float* sched, float* logits, float* protos,
                int* cls, int* any_anom, float* probs, int* keep_orig, int* final_target, int* gen_target,
                float* latent, void* stream) {
  return pgp_forward_stage(m, -1, batch, windows, sched, logits, protos, cls, any_anom, probs, keep_orig,
                           final_target, gen_target, latent, stream);
}

int pgp_forward_fpe_stage(pgp_model* m, int stage, int batch, const float* windows, const float* h0,
                          const float* sched, float* scores, float* protos, int* cls, int* any_anom, float* probs,
                          int* keep_orig, int* final_target, int* gen_target, void* stream) {
  if (!m) return fail(PGP_ERR_ARG, "NULL model");
  if (!m->loaded) return fail(PGP_ERR_STATE, "weights not loaded");
  if (!m->fpe) return fail(PGP_ERR_STATE, "not an FPE model: use pgp_forward");
  if (batch < 0) return fail(PGP_ERR_ARG, "negative batch");
  if (stage < -1 || stage > 1) return fail(PGP_ERR_ARG, "bad stage");
  if (batch == 0) return PGP_OK;  // empty batch: nothing to read or write (pointers may be NULL)
  const bool all = stage == -1;
  if (((all || stage == 0) && (!windows || !h0 || !scores || !protos || !cls || !any_anom)) ||
      ((all || stage == 1) && (!sched || !probs || !keep_orig || !final_target || !gen_target)))
    return fail(PGP_ERR_ARG, "NULL input/output pointer");
  if (batch > m->cap) {
    const int rc = reserve(m, batch);
    if (rc) return rc;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  FpeArgs f{};
  f.B = batch;
  f.windows = windows;
  f.h0 = h0;
  f.tab = m->d_tab;
  f.scores = scores;
  f.protos = protos;
  f.cls = cls;
  f.any_anom = any_anom;
  f.emb = m->d_emb;
  if (all || stage == 0) HIPCHK(launch_fpe(m->H, f, st));
  FwdArgs a{};
  a.B = batch;
  a.H = m->H;
  a.K = m->K;
  a.sched = sched;
  a.emb = m->d_emb;
  a.frags = m->d_frags;
  a.ganb = m->gan_split ? m->d_ganb : nullptr;
  a.gtab = m->d_gtab;
  a.probs = probs;
  a.keep = keep_orig;
  a.final_t = final_target;
  a.gen_t = gen_target;
  if (all || stage == 1) HIPCHK(launch_gan(a, st));
  return PGP_OK;
}

int pgp_forward_fpe(pgp_model* m, int batch, const float* windows, const float* h0, const float* sched,
                    float* scores, float* protos, int* cls, int* any_anom, float* probs, int* keep_orig,
                    int* final_target, int* gen_target, void* stream) {
  return pgp_forward_fpe_stage(m, -1, batch, windows, h0, sched, scores, protos, cls, any_anom, probs, keep_orig,
                               final_target, gen_target, stream);
}

int pgp_migrations(int n_hosts, int batch, const int* keep_orig, const int* final_target, const int* cur_host,
                   int* moves, int* hosts_from, void* stream) {
  if (n_hosts < 1 || batch < 0) return fail(PGP_ERR_ARG, "bad migrations arguments");
  if (batch == 0) return PGP_OK;
  if (!keep_orig || !final_target || !cur_host || !moves || !hosts_from)
    return fail(PGP_ERR_ARG, "NULL input/output pointer");
  HIPCHK(launch_decide(batch, n_hosts, keep_orig, final_target, cur_host, moves, hosts_from,
                       reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_embedding(int n_hosts, int batch, const float* logits, const float* protos, float* emb, void* stream) {
  if (n_hosts < 1 || batch < 0) return fail(PGP_ERR_ARG, "bad embedding arguments");
  if (batch == 0) return PGP_OK;
  if (!logits || !protos || !emb) return fail(PGP_ERR_ARG, "NULL input/output pointer");
  HIPCHK(launch_embed((long)batch * n_hosts, logits, protos, emb, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_decoder_split(pgp_model* m, int on) {
  if (!m) return fail(PGP_ERR_ARG, "NULL model");
  if (m->fpe || decoder_split_floats(m->H) == 0)
    return on ? fail(PGP_ERR_UNSUPPORTED, "split-bf16 decoder not compiled for this model / host count") : PGP_OK;
  m->dec_split = on != 0;
  return PGP_OK;
}

int pgp_encoder_split(pgp_model* m, int on) {
  if (!m) return fail(PGP_ERR_ARG, "NULL model");
  if (m->fpe || encoder_split_floats(m->H) == 0)
    return on ? fail(PGP_ERR_UNSUPPORTED, "split-bf16 encoder not compiled for this model / host count") : PGP_OK;
  m->enc_split = on != 0;
  return PGP_OK;
}

int pgp_gan_split(pgp_model* m, int on) {
  if (!m) return fail(PGP_ERR_ARG, "NULL model");
  if (gan_split_floats(m->H) == 0)
    return on ? fail(PGP_ERR_UNSUPPORTED, "split-bf16 GAN kernel not compiled for this host count") : PGP_OK;
  m->gan_split = on != 0;
  return PGP_OK;
}

int pgp_schedule_onehot(int n_hosts, int batch, const unsigned char* idx, float* sched, void* stream) {
  if (n_hosts < 1 || n_hosts > 255 || batch < 0) return fail(PGP_ERR_ARG, "bad schedule_onehot arguments");
  if (batch == 0) return PGP_OK;
  if (!idx || !sched) return fail(PGP_ERR_ARG, "NULL input/output pointer");
  HIPCHK(launch_onehot(n_hosts, (long)batch * n_hosts, idx, sched, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

// ---------------------------------------------------------------------------
// training ops
// ---------------------------------------------------------------------------
namespace {
bool master_offsets(int H, long* tr, long* gen, long* disc, long* all) {
  switch (H) {
#define CASE(h)                     \
  case h:                           \
    *tr = 0;                        \
    *gen = TGeo<h>::OFF_GEN;        \
    *disc = TGeo<h>::OFF_DISC;      \
    *all = TGeo<h>::ALL;            \
    return true;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return false;
}
}  // namespace

size_t pgp_master_len(int n_hosts) {
  long a, b, c, d;
  return master_offsets(n_hosts, &a, &b, &c, &d) ? (size_t)d : 0;
}
size_t pgp_master_offset(int n_hosts, int section) {
  long a, b, c, d;
  if (!master_offsets(n_hosts, &a, &b, &c, &d)) return 0;
  return section == 0 ? a : section == 1 ? b : section == 2 ? c : d;
}
size_t pgp_tune_workspace_len(int n_hosts, int batch) {
  TunePlan p;
  return (supported(n_hosts) && tune_plan(n_hosts, batch, &p)) ? (size_t)p.total : 0;
}
size_t pgp_gan_workspace_len(int n_hosts, int batch) {
  return supported(n_hosts) ? (size_t)gan_workspace_floats(n_hosts, batch) : 0;
}

int pgp_tune_forward(int n_hosts, int batch, const float* windows, const float* P, float* workspace, float* latent,
                     float* logits, float* protos, void* stream) {
  if (!supported(n_hosts)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (batch < 0 || (batch > 0 && (!windows || !P || !workspace || !logits || !protos)))
    return fail(PGP_ERR_ARG, "bad tune_forward arguments");
  if (batch == 0) return PGP_OK;
  TunePlan p;
  tune_plan(n_hosts, batch, &p);
  HIPCHK(launch_tune_forward(p, windows, P, workspace, latent, logits, protos, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_tune_backward(int n_hosts, int batch, const float* P, float* G, float* workspace, const float* logits,
                      const float* protos, const int* y, const float* mult, const float* tgt, void* stream) {
  if (!supported(n_hosts)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (batch < 0 || (batch > 0 && (!P || !G || !workspace || !logits || !protos || !y || !mult || !tgt)))
    return fail(PGP_ERR_ARG, "bad tune_backward arguments");
  if (batch == 0) return PGP_OK;
  TunePlan p;
  tune_plan(n_hosts, batch, &p);
  HIPCHK(launch_tune_backward(p, P, G, workspace, logits, protos, y, mult, tgt,
                              reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_tune_backward_prefix(int n_hosts, int fwd_batch, int batch, const float* P, float* G, float* workspace,
                             const float* logits, const float* protos, const int* y, const float* mult,
                             const float* tgt, void* stream) {
  if (!supported(n_hosts)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (batch < 0 || batch > fwd_batch ||
      (batch > 0 && (!P || !G || !workspace || !logits || !protos || !y || !mult || !tgt)))
    return fail(PGP_ERR_ARG, "bad tune_backward_prefix arguments");
  if (batch == 0) return PGP_OK;
  TunePlan p;
  if (!tune_plan_prefix(n_hosts, fwd_batch, batch, &p)) return fail(PGP_ERR_ARG, "tune_backward_prefix plan");
  HIPCHK(launch_tune_backward(p, P, G, workspace, logits, protos, y, mult, tgt,
                              reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

size_t pgp_fpe_param_len(int n_hosts) { return n_hosts == 16 ? (size_t)fpe_param_count() : 0; }

int pgp_fpe_train_step(int n_hosts, int n_protos, const float* window, const float* h0, const int* y, const int* cls,
                       const float* P, float* G, double* state, double update_min, double decay, double* loss,
                       void* stream) {
  if (n_hosts != 16) return fail(PGP_ERR_UNSUPPORTED, "FPE training: n_hosts 16 only (FPE_16)");
  if (n_protos < 3 || n_protos > kMaxProtos) return fail(PGP_ERR_ARG, "n_protos");
  if (!window || !h0 || !y || !cls || !P || !G || !state || !loss) return fail(PGP_ERR_ARG, "NULL argument");
  HIPCHK(launch_fpe_step(window, h0, y, cls, P, G, n_protos, state, update_min, decay, loss,
                         reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_fpe_forward_many(int n_hosts, int n, const float* windows, const float* h0, const float* P, double* probs,
                         double* protos, void* stream) {
  if (n_hosts != 16) return fail(PGP_ERR_UNSUPPORTED, "FPE training: n_hosts 16 only (FPE_16)");
  if (n < 0 || (n > 0 && (!windows || !h0 || !P || !probs || !protos))) return fail(PGP_ERR_ARG, "bad arguments");
  if (n == 0) return PGP_OK;
  HIPCHK(launch_fpe_forward_many(n, windows, h0, P, probs, protos, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_tune_reserve_cus(int n) {
  if (n < 0) return fail(PGP_ERR_ARG, "negative CU count");
  tf_reserve_cus(n);
  return PGP_OK;
}

int pgp_tune_set_side_stream(void* stream) {
  HIPCHK(tune_set_side_stream(reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_tune_timing(int on) {
  HIPCHK(tune_timing(on != 0));
  return PGP_OK;
}

int pgp_tune_fused_ms(float* ms6) {
  if (!ms6) return fail(PGP_ERR_ARG, "NULL output");
  const hipError_t e = tune_fused_ms(ms6);
  if (e == hipErrorInvalidValue) return fail(PGP_ERR_STATE, "pgp_tune_timing(1) was never called");
  HIPCHK(e);
  return PGP_OK;
}

int pgp_tune_targets(int n_hosts, int n_protos, const float* logits, const float* protos, const int* y, const int* cls,
                     double* state, double update_min, double decay, float* mult, float* tgt, double* loss,
                     void* stream) {
  if (n_hosts <= 0 || n_hosts > 64) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (n_protos < 3) return fail(PGP_ERR_ARG, "triplet_loss needs prototypes 0-2");
  if (!logits || !protos || !y || !cls || !state || !mult || !tgt || !loss)
    return fail(PGP_ERR_ARG, "bad tune_targets arguments");
  HIPCHK(launch_tune_targets(n_hosts, n_protos, logits, protos, y, cls, state, update_min, decay, mult, tgt, loss,
                             reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_tune_step1(int n_hosts, int n_protos, const float* window, const int* y, const int* cls, const float* P,
                   float* G, double* state, double update_min, double decay, float* logits, float* protos,
                   double* loss, void* stream) {
  if (!tune1_supported(n_hosts)) return fail(PGP_ERR_UNSUPPORTED, "host count (fused step: 8 or 16)");
  if (n_protos < 3) return fail(PGP_ERR_ARG, "triplet_loss needs prototypes 0-2");
  if (!window || !y || !cls || !P || !G || !state || !logits || !protos || !loss)
    return fail(PGP_ERR_ARG, "bad tune_step1 arguments");
  HIPCHK(launch_tune1(n_hosts, n_protos, window, y, cls, P, G, state, update_min, decay, logits, protos, loss,
                      reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_tune_forward_many(int n_hosts, int n_windows, const float* windows, const float* P, double* logits,
                          double* protos, void* stream) {
  if (!tune1_supported(n_hosts)) return fail(PGP_ERR_UNSUPPORTED, "host count (fused forward: 8 or 16)");
  if (n_windows < 0) return fail(PGP_ERR_ARG, "n_windows >= 0");
  if (n_windows == 0) return PGP_OK;
  if (!windows || !P || !logits || !protos) return fail(PGP_ERR_ARG, "bad tune_forward_many arguments");
  HIPCHK(launch_fwd_many(n_hosts, n_windows, windows, P, logits, protos, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_forward1(int n_hosts, int n_protos, const float* window, const float* sched, const float* P,
                 const double* prototypes_device, float* logits, float* protos, int* cls, int* any_anom, float* probs,
                 int* keep_orig, int* final_target, int* gen_target, void* stream) {
  if (!tune1_supported(n_hosts)) return fail(PGP_ERR_UNSUPPORTED, "host count (batch-1 forward: 8 or 16)");
  if (n_protos < 1 || n_protos > kMaxProtos) return fail(PGP_ERR_ARG, "n_protos out of range");
  if (!window || !sched || !P || !prototypes_device || !logits || !protos || !cls || !any_anom || !probs ||
      !keep_orig || !final_target || !gen_target)
    return fail(PGP_ERR_ARG, "bad forward1 arguments");
  HIPCHK(launch_infer1(n_hosts, n_protos, window, sched, P, prototypes_device, logits, protos, cls, any_anom, probs,
                       keep_orig, final_target, gen_target, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_tune_dataset(int n_hosts, int n_env, int n_rows, const double* series, const double* train_max,
                     float* windows, int* y, int* cls, float* infer, void* stream) {
  if (n_hosts <= 0 || n_hosts > 64) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (n_env < 0 || n_rows < 1 || n_rows > kMaxTuneRows) return fail(PGP_ERR_ARG, "n_env >= 0, 1 <= n_rows <= 16");
  if (n_env == 0) return PGP_OK;
  if (!series || !train_max || !windows || !y || !cls) return fail(PGP_ERR_ARG, "bad tune_dataset arguments");
  HIPCHK(launch_tune_dataset(n_hosts, n_env, n_rows, series, train_max, windows, y, cls, infer,
                             reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

size_t pgp_tune_targets_dp_workspace_len(int batch) {
  return batch > 0 ? (size_t)tune_dp_workspace_doubles(batch) : 0;
}

int pgp_tune_targets_dp(int n_hosts, int n_protos, int batch, const float* logits, const float* protos, const int* y,
                        const int* cls, const double* state, double update_min, float* mult, float* tgt, double* loss,
                        double* inc, double* workspace, void* stream) {
  if (n_hosts <= 0 || n_hosts > 64) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (n_protos < 3 || n_protos > kMaxProtos) return fail(PGP_ERR_ARG, "triplet_loss needs prototypes 0-2");
  if (batch <= 0 || !logits || !protos || !y || !cls || !state || !mult || !tgt || !loss || !inc || !workspace)
    return fail(PGP_ERR_ARG, "bad tune_targets_dp arguments");
  // state is only read here (no fused state update)
  HIPCHK(launch_tune_targets_dp(n_hosts, n_protos, batch, logits, protos, y, cls, const_cast<double*>(state),
                                update_min, mult, tgt, loss, inc, workspace, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_tune_state_apply(int n_protos, double* state, const double* inc, double decay, int n_cond,
                         const int* cond_rows, double* cond_steps, float* adam_table, double lr, double beta1,
                         double beta2, void* stream) {
  if (n_protos < 3 || n_protos > kMaxProtos || !state || !inc) return fail(PGP_ERR_ARG, "bad state arguments");
  if (n_cond < 0 || n_cond > kMaxCond || (n_cond > 0 && (!cond_rows || !cond_steps || !adam_table)))
    return fail(PGP_ERR_ARG, "bad AdamW condition arguments");
  CondRows cr{};
  cr.n = n_cond;
  for (int i = 0; i < n_cond; ++i) {
    if (cond_rows[i] < 0 || cond_rows[i] >= kMaxTensors) return fail(PGP_ERR_ARG, "AdamW table row out of range");
    cr.row[i] = cond_rows[i];
  }
  HIPCHK(launch_tune_state_apply(n_protos, state, inc, decay, cr, cond_steps, adam_table, lr, beta1, beta2,
                                 reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_gan_forward(int n_hosts, int batch, const float* emb, const float* sched, const float* P, float* workspace,
                    float* ns, float* probs, void* stream) {
  long tr, go, dof, all;
  if (!master_offsets(n_hosts, &tr, &go, &dof, &all)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (batch < 0 || (batch > 0 && (!emb || !sched || !P || !workspace || !ns || !probs)))
    return fail(PGP_ERR_ARG, "bad gan_forward arguments");
  if (batch == 0) return PGP_OK;
  HIPCHK(launch_gan_fwd(n_hosts, batch, emb, sched, P + go, P + dof, workspace, ns, probs,
                        reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_gan_disc_backward(int n_hosts, int batch, const float* target, const float* P, float* G, float* workspace,
                          void* stream) {
  long tr, go, dof, all;
  if (!master_offsets(n_hosts, &tr, &go, &dof, &all)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (batch < 0 || (batch > 0 && (!target || !P || !G || !workspace))) return fail(PGP_ERR_ARG, "bad arguments");
  if (batch == 0) return PGP_OK;
  HIPCHK(launch_gan_disc_bwd(n_hosts, batch, target, P + dof, G + dof, workspace,
                             reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_gan_gen_backward(int n_hosts, int batch, const float* P, float* G, float* workspace, void* stream) {
  long tr, go, dof, all;
  if (!master_offsets(n_hosts, &tr, &go, &dof, &all)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (batch < 0 || (batch > 0 && (!P || !G || !workspace))) return fail(PGP_ERR_ARG, "bad arguments");
  if (batch == 0) return PGP_OK;
  HIPCHK(launch_gan_gen_bwd(n_hosts, batch, P + go, P + dof, G + go, workspace,
                            reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_gan_forward1(int n_hosts, const float* emb, const float* sched, const float* P, float* workspace, float* ns,
                     float* probs, void* stream) {
  long tr, go, dof, all;
  if (!gan1_supported(n_hosts) || !master_offsets(n_hosts, &tr, &go, &dof, &all))
    return fail(PGP_ERR_UNSUPPORTED, "host count (fused GAN step: 8 or 16)");
  if (!emb || !sched || !P || !workspace || !ns || !probs) return fail(PGP_ERR_ARG, "bad gan_forward1 arguments");
  HIPCHK(launch_gan1_forward(n_hosts, emb, sched, P + go, P + dof, workspace, ns, probs,
                             reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

static bool adam_args(AdamArgs* a, float* P, float* G, float* m, float* v, float lr, float wd, float b1, float b2,
                      float eps, const pgp_adam_tensor* t, int n, const float* sched, long lo, long hi) {
  if (!t || !sched || n < 0 || n > kMaxTensors) return false;
  *a = AdamArgs{};
  a->param = P;
  a->grad = G;
  a->m = m;
  a->v = v;
  a->lr_wd = lr * wd;
  a->b1 = b1;
  a->b2 = b2;
  a->eps = eps;
  a->ntensors = n;
  a->sched = sched;
  for (int i = 0; i < n; ++i) {
    if (t[i].offset < lo || t[i].n < 0 || (long)t[i].offset + t[i].n > hi) return false;  // inside the section
    a->t[i].off = (long)t[i].offset;
    a->t[i].n = t[i].n;
    a->t[i].active = 1;
  }
  return true;
}

int pgp_gan_step1(int n_hosts, const float* target, float* P, float* G, float* exp_avg, float* exp_avg_sq,
                  float lr_disc, float lr_gen, float weight_decay, float beta1, float beta2, float eps,
                  const pgp_adam_tensor* disc_tensors, int n_disc, const float* disc_sched,
                  const pgp_adam_tensor* gen_tensors, int n_gen, const float* gen_sched, float* workspace,
                  float* probs_gen, float* probs_after, void* stream) {
  long tr, go, dof, all;
  if (!gan1_supported(n_hosts) || !master_offsets(n_hosts, &tr, &go, &dof, &all))
    return fail(PGP_ERR_UNSUPPORTED, "host count (fused GAN step: 8 or 16)");
  if (!target || !P || !G || !exp_avg || !exp_avg_sq || !workspace || !probs_gen || !probs_after)
    return fail(PGP_ERR_ARG, "bad gan_step1 arguments");
  AdamArgs ad, ag;
  if (!adam_args(&ad, P, G, exp_avg, exp_avg_sq, lr_disc, weight_decay, beta1, beta2, eps, disc_tensors, n_disc,
                 disc_sched, dof, all) ||
      !adam_args(&ag, P, G, exp_avg, exp_avg_sq, lr_gen, weight_decay, beta1, beta2, eps, gen_tensors, n_gen,
                 gen_sched, go, dof))
    return fail(PGP_ERR_ARG, "AdamW tensors (disc / gen sections) or tables");
  HIPCHK(launch_gan1_step(n_hosts, target, P + go, P + dof, G + go, G + dof, workspace, ad, ag, probs_gen, probs_after,
                          reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_gan_probs(int n_hosts, int batch, const float* workspace, float* probs, void* stream) {
  if (!supported(n_hosts)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (batch < 0 || (batch > 0 && (!workspace || !probs))) return fail(PGP_ERR_ARG, "bad arguments");
  if (batch == 0) return PGP_OK;
  HIPCHK(launch_gan_probs(n_hosts, batch, workspace, probs, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_adamw(float* P, const float* G, float* exp_avg, float* exp_avg_sq, float lr, float weight_decay,
              float beta1, float beta2, float eps, const pgp_adam_tensor* tensors, int ntensors, void* stream) {
  if (!P || !G || !exp_avg || !exp_avg_sq || !tensors || ntensors < 0 || ntensors > kMaxTensors)
    return fail(PGP_ERR_ARG, "bad adamw arguments");
  if (ntensors == 0) return PGP_OK;
  AdamArgs a{};
  a.param = P;
  a.grad = const_cast<float*>(G);
  a.m = exp_avg;
  a.v = exp_avg_sq;
  a.lr_wd = lr * weight_decay;
  a.b1 = beta1;
  a.b2 = beta2;
  a.eps = eps;
  a.ntensors = ntensors;
  for (int i = 0; i < ntensors; ++i) {
    a.t[i].off = (long)tensors[i].offset;
    a.t[i].n = tensors[i].n;
    a.t[i].active = tensors[i].active;
    a.t[i].step_size = tensors[i].step_size;
    a.t[i].bc2_sqrt = tensors[i].bc2_sqrt;
  }
  HIPCHK(launch_adamw(a, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_adamw_table(float* P, const float* G, float* exp_avg, float* exp_avg_sq, float lr, float weight_decay,
                    float beta1, float beta2, float eps, const pgp_adam_tensor* tensors, int ntensors,
                    const float* sched, void* stream) {
  if (!P || !G || !exp_avg || !exp_avg_sq || !tensors || !sched || ntensors < 0 || ntensors > kMaxTensors)
    return fail(PGP_ERR_ARG, "bad adamw arguments");
  if (ntensors == 0) return PGP_OK;
  AdamArgs a{};
  a.param = P;
  a.grad = const_cast<float*>(G);
  a.m = exp_avg;
  a.v = exp_avg_sq;
  a.lr_wd = lr * weight_decay;
  a.b1 = beta1;
  a.b2 = beta2;
  a.eps = eps;
  a.ntensors = ntensors;
  a.sched = sched;
  for (int i = 0; i < ntensors; ++i) {
    a.t[i].off = (long)tensors[i].offset;
    a.t[i].n = tensors[i].n;
    a.t[i].active = kAdamFromTable;  // every row from the table
    a.t[i].step_size = tensors[i].step_size;
    a.t[i].bc2_sqrt = tensors[i].bc2_sqrt;
  }
  HIPCHK(launch_adamw(a, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_repack_master(pgp_model* m, const float* P_device, const double* prototypes_device, void* stream) {
  return pgp_repack_master_sections(m, P_device, prototypes_device, 3, stream);
}

int pgp_repack_master_sections(pgp_model* m, const float* P_device, const double* prototypes_device, int sections,
                               void* stream) {
  if (!m || !P_device || !prototypes_device) return fail(PGP_ERR_ARG, "NULL argument");
  if (sections < 1 || sections > 3) return fail(PGP_ERR_ARG, "sections: 1 (PreGAN+), 2 (GAN) or 3 (both)");
  if (m->fpe) return fail(PGP_ERR_STATE, "FPE model: master-layout reload covers the PreGAN+ model only");
  if (!m->loaded) return fail(PGP_ERR_STATE, "weights not loaded (the first load packs on the host)");
  long tr, go, dof, all;
  if (!master_offsets(m->H, &tr, &go, &dof, &all)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  if (repack_blob_protos_offset(m->H, m->K) != all) return fail(PGP_ERR_STATE, "master / blob layout mismatch");
  if (!m->d_pscr) HIPCHK(hipMalloc(&m->d_pscr, repack_scratch_len(m->H) * sizeof(double)));
  RepackArgs a{m->K, P_device, all, prototypes_device, m->d_pscr, m->d_frags, m->d_tab, m->d_gtab, m->d_gat, sections};
  HIPCHK(launch_repack(m->H, a, reinterpret_cast<hipStream_t>(stream)));
  if ((sections & 1) && m->d_decb)
    HIPCHK(launch_decoder_split(m->H, m->d_frags, m->d_decb, reinterpret_cast<hipStream_t>(stream)));
  if ((sections & 1) && m->d_encb)
    HIPCHK(launch_encoder_split(m->H, m->d_frags, m->d_encb, reinterpret_cast<hipStream_t>(stream)));
  if ((sections & 2) && m->d_ganb)
    HIPCHK(launch_gan_split_derive(m->H, m->d_frags, m->d_ganb, reinterpret_cast<hipStream_t>(stream)));
  return PGP_OK;
}

int pgp_load_weights_master(pgp_model* m, const float* P_device, const double* prototypes) {
  if (!m || !P_device || !prototypes) return fail(PGP_ERR_ARG, "NULL argument");
  if (m->fpe) return fail(PGP_ERR_STATE, "FPE model: master-layout reload covers the PreGAN+ model only");
  long tr, go, dof, all;
  if (!master_offsets(m->H, &tr, &go, &dof, &all)) return fail(PGP_ERR_UNSUPPORTED, "host count");
  std::vector<float> host((size_t)all);
  HIPCHK(hipMemcpy(host.data(), P_device, host.size() * sizeof(float), hipMemcpyDeviceToHost));
  std::vector<double> blob(host.size() + 2 * (size_t)m->K);
  for (size_t i = 0; i < host.size(); ++i) blob[i] = host[i];
  for (int k = 0; k < 2 * m->K; ++k) blob[host.size() + k] = prototypes[k];
  return pgp_load_weights(m, blob.data(), blob.size());
}

}  // extern "C"
