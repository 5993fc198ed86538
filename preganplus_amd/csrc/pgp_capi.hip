// pgp_capi.hip — the C-ABI of include/preganplus.h: model lifetime, weight
// upload, workspace, and the launch sequence of one forward call:
//   K1 gat (pgp_gat.hip) -> K2 encoder (pgp_encoder.hip) ->
//   K2b decoders+classify (pgp_decoder.hip) -> K3 GAN+decisions (pgp_gan.hip)
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/preganplus.h"
#include "pgp_device.hpp"
#include "pgp_pack.hpp"

using namespace pgp;

struct pgp_model {
  int H = 0, K = 0;
  bool loaded = false;
  float* d_frags = nullptr;
  float* d_tab = nullptr;
  float* d_gtab = nullptr;
  GatConst gat{};
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
  const size_t agg_f = nblk * m->H * 3 * 48;
  const size_t lat_f = nblk * (size_t)lat_blk(m->H);
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

int pgp_destroy(pgp_model* m) {
  if (!m) return PGP_OK;
  for (float* p : {m->d_frags, m->d_tab, m->d_gtab, m->d_agg, m->d_lat, m->d_emb})
    if (p) (void)hipFree(p);
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
  if (stage < -1 || stage > 3) return fail(PGP_ERR_ARG, "bad stage");
  const bool all = stage == -1;
  if (((all || stage == 0) && !windows) ||
      ((all || stage == 2) && (!logits || !protos || !cls || !any_anom)) ||
      ((all || stage == 3) && (!sched || !probs || !keep_orig || !final_target || !gen_target)))
    return fail(PGP_ERR_ARG, "NULL input/output pointer");
  if (batch == 0) return PGP_OK;
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
  a.tab = m->d_tab;
  a.gtab = m->d_gtab;
  a.gat = m->gat;
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

}  // extern "C"
