// pgp_online.hip — run_model's semi-supervised training (PreGANPlus.py:115-136,
// all but the decision; BASELINE config C3) for a batch of environments,
// issued from ONE C-ABI call (pgp_online_step) instead of ~40 host calls:
//
//   main stream  dataset (load_on_the_fly_dataset utils.py:40-47 + run_encoder's
//                window PreGANPlus.py:107-112) -> ONE tuning forward over the
//                R*E tuning windows and the E detect windows (same step-start
//                weights) -> custom_loss / triplet_loss bookkeeping against the
//                step-start state (train.py:13-40, DP form) -> backward over
//                the tuning windows -> [all-reduce grads, state increments] ->
//                state update, AdamW (utils.py:65)
//   GAN stream   (from the forward's end) detect's masked embedding
//                (PreGANPlus.py:129) -> Gen + Disc forward -> both schedules
//                simulated on the device (utils.py:97-100 -> Stats.py:154-177)
//                -> Disc BCE step -> [all-reduce] -> AdamW -> Gen BCE step
//                through the updated Disc -> [all-reduce] -> AdamW
//                (train_gan, PreGANPlus.py:60-81)
//
// The GAN and tuning steps share no data (the GAN reads the embedding and
// writes the Gen / Disc sections; the tuning step writes the Transformer
// section), so they run side by side; the step ends with the main stream
// waiting for the GAN stream.  AdamW's per-step scalars are computed here on
// the host from the step counts this object keeps (lr / (1 - beta1^step),
// sqrt(1 - beta2^step) in double, rounded to fp32: the values the Python
// tables hold) and passed by value; the prototype decoder's rows, whose
// activity depends on the global batch's labels, come from the device table
// pgp_tune_state_apply writes.  The collectives of a data-parallel step are
// the caller's (a callback at the four exchange points, on the stream it
// names): this library has no communicator of its own.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

#include "../../include/preganplus.h"
#include "pgp_device.hpp"
#include "pgp_train.hpp"
#include "pgp_tune.hpp"
#include "pgp_tunedp.hpp"

using namespace pgp;

namespace {

enum Sec { kTr = 0, kGen = 1, kDisc = 2 };
// timing events: main stream 0..6, GAN stream 7..9
enum Ev { kE0, kE1, kE2, kE3, kE4, kE5, kE6, kG0, kG1, kG2, kNumEv };

// A host thread that issues the GAN stream's launches while the calling thread
// issues the tuning backward (world size 1).  Issuing ~20 launches costs the
// host ~0.1 ms; serially, whichever stream is issued second waits for the
// other's issue (H = 16: the main stream sat idle 46 us between the targets and
// the backward while the GAN launches were issued; issuing the backward first
// delays the GAN chain the same amount).  The worker spins a while between
// jobs (back-to-back steps find it awake), then sleeps on a condition
// variable.
class IssueWorker {
 public:
  IssueWorker() : th_([this] { loop(); }) {}
  ~IssueWorker() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    cv_.notify_one();
    th_.join();
  }
  void post(std::function<int()> job) {
    job_ = std::move(job);
    {
      std::lock_guard<std::mutex> lk(m_);
      posted_.store(posted_.load(std::memory_order_relaxed) + 1, std::memory_order_release);
    }
    cv_.notify_one();
  }
  // the posted job's return code (its error message in *err)
  int wait(std::string* err) {
    const unsigned long n = posted_.load(std::memory_order_relaxed);
    while (done_.load(std::memory_order_acquire) != n) __builtin_ia32_pause();
    *err = err_;
    return rc_;
  }

 private:
  void loop() {
    unsigned long seen = 0;
    for (;;) {
      unsigned long n = 0;
      for (long i = 0; i < kSpin && (n = posted_.load(std::memory_order_acquire)) == seen; ++i)
        __builtin_ia32_pause();
      if (n == seen) {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return quit_ || posted_.load(std::memory_order_acquire) != seen; });
        if (quit_) return;
        n = posted_.load(std::memory_order_acquire);
      }
      rc_ = job_();
      err_ = rc_ == PGP_OK ? std::string() : pgp_last_error();
      seen = n;
      done_.store(n, std::memory_order_release);
    }
  }
  static constexpr long kSpin = 200000;  // ~2-5 ms of pause instructions
  std::function<int()> job_;
  int rc_ = PGP_OK;
  std::string err_;
  std::atomic<unsigned long> posted_{0}, done_{0};
  bool quit_ = false;
  std::mutex m_;
  std::condition_variable cv_;
  std::thread th_;
};

}  // namespace

struct pgp_online {
  pgp_online_desc d{};
  int H = 0, E = 0, R = 0, B = 0, K = 0;
  TunePlan fwd{}, bwd{};
  AdamArgs adam[3]{};
  double step[3][kMaxTensors] = {};  // host step counts (the prototype decoder's live on the device)
  bool pending[3] = {false, false, false};  // scalars of step + 1 issued; counted once the step is issued
  int cond_local[kMaxTensors] = {};  // transformer selection index -> cond flag
  CondRows cr{};
  long sec_lo[3] = {0, 0, 0};
  hipEvent_t gate = nullptr, gan_done = nullptr, tgt_end = nullptr;
  bool timing = false, timed = false;
  hipEvent_t tev[kNumEv] = {};
  bool issue_worker = true;  // world size 1, two streams: the GAN launches issued from a second host thread
  IssueWorker* worker = nullptr;
};

namespace {

thread_local std::string g_oerr;
int ofail(int code, const std::string& msg) {
  set_error(code, msg);
  g_oerr = msg;
  return code;
}
#define OCHK(x)                                                                                     \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return ofail(PGP_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define OCALL(x)               \
  do {                         \
    const int r_ = (x);        \
    if (r_ != PGP_OK) return r_; \
  } while (0)

// the next step's AdamW scalars of a section's always-active tensors (step + 1);
// the counts themselves advance in commit_steps, once the whole step is issued
void next_scalars(pgp_online* o, int sec) {
  AdamArgs& a = o->adam[sec];
  const double lr = o->d.lr[sec], b1 = o->d.beta1, b2 = o->d.beta2;
  for (int i = 0; i < a.ntensors; ++i) {
    if (a.t[i].active & kAdamFromTable) continue;
    const double nx = o->step[sec][i] + 1.0;
    const double st = nx > 1.0 ? nx : 1.0;
    a.t[i].step_size = (float)(lr / (1.0 - std::pow(b1, st)));
    a.t[i].bc2_sqrt = (float)std::sqrt(1.0 - std::pow(b2, st));
  }
  o->pending[sec] = true;
}

void commit_steps(pgp_online* o) {
  for (int sec = 0; sec < 3; ++sec) {
    if (!o->pending[sec]) continue;
    const AdamArgs& a = o->adam[sec];
    for (int i = 0; i < a.ntensors; ++i)
      if (!(a.t[i].active & kAdamFromTable)) o->step[sec][i] += 1.0;
    o->pending[sec] = false;
  }
}

// After the GAN stream forks off the main stream, every exit joins it back:
// on an error path the main stream still waits for the GAN work already queued
// (the caller's next use of the weights must not race it).
struct GanJoin {
  pgp_online* o;
  hipStream_t sm, sg;
  bool armed = false;
  ~GanJoin() {
    if (!armed) return;
    (void)hipEventRecord(o->gan_done, sg);
    (void)hipStreamWaitEvent(sm, o->gan_done, 0);
  }
};

void mark(pgp_online* o, int k, hipStream_t s) {
  if (o->timing) (void)hipEventRecord(o->tev[k], s);
}

// A section's AdamW fused into its weight-gradient kernel (world size 1: no
// exchange between gradient and update), when every tensor of the section
// takes the same per-step scalars (all GAN tensors step together); the next
// step's scalars must have been computed (next_scalars).
bool fuse_adam(const pgp_online* o, int sec, AdamFuse* f) {
  const AdamArgs& a = o->adam[sec];
  if (a.ntensors == 0) return false;
  for (int i = 1; i < a.ntensors; ++i)
    if (a.t[i].step_size != a.t[0].step_size || a.t[i].bc2_sqrt != a.t[0].bc2_sqrt ||
        (a.t[i].active & kAdamFromTable))
      return false;
  *f = AdamFuse{a.param, a.m, a.v, a.grad, a.lr_wd, a.b1, a.b2, a.eps, a.t[0].step_size, a.t[0].bc2_sqrt};
  return true;
}

int collective(pgp_collective_fn cb, void* user, int which, hipStream_t s) {
  if (!cb) return PGP_OK;
  const int r = cb(user, which, reinterpret_cast<void*>(s));
  return r == 0 ? PGP_OK : ofail(PGP_ERR_STATE, "collective callback failed (which = " + std::to_string(which) + ")");
}

}  // namespace

namespace {
// train_gan up to the Disc gradient: the embedding (PreGANPlus.py:129, formed
// inside the GAN forward's first launch from detect's logits / protos, the
// forward's last E rows), Gen + Disc forward, the simulated label, the Disc
// BCE gradient (with its AdamW when fused)
int gan_part_a(pgp_online* o, hipStream_t sg, bool fused) {
  const pgp_online_desc& d = o->d;
  const int H = o->H, E = o->E, B = o->B;
  const long go = o->sec_lo[kGen], dof = o->sec_lo[kDisc];
  OCHK(launch_gan_fwd(H, E, nullptr, d.sched, d.P + go, d.P + dof, d.gan_ws, d.ns, nullptr, sg,
                      d.logits + (long)B * H * 2, d.protos + (long)B * H * 2, d.emb));
  OCHK(launch_simulate(H, E, d.envs, d.ns, d.sched, d.sim_out, d.target, sg));
  AdamFuse f{};
  bool fz = false;
  if (fused) {
    next_scalars(o, kDisc);
    fz = fuse_adam(o, kDisc, &f);
  }
  OCHK(launch_gan_disc_bwd(H, E, d.target, d.P + dof, d.G + dof, d.gan_ws, sg, d.probs, fz ? &f : nullptr));
  if (fused && !fz) OCHK(launch_adamw(o->adam[kDisc], sg));
  return PGP_OK;
}
// the rest: [exchange] Disc AdamW, the Gen step through the updated Disc,
// [exchange] Gen AdamW
int gan_part_b(pgp_online* o, hipStream_t sg, bool fused, pgp_collective_fn cb, void* user) {
  const pgp_online_desc& d = o->d;
  const int H = o->H, E = o->E;
  const long go = o->sec_lo[kGen], dof = o->sec_lo[kDisc];
  if (!fused) {
    OCALL(collective(cb, user, PGP_COLL_DISC_GRAD, sg));
    next_scalars(o, kDisc);
    OCHK(launch_adamw(o->adam[kDisc], sg));
  }
  AdamFuse f{};
  bool fz = false;
  if (fused) {
    next_scalars(o, kGen);
    fz = fuse_adam(o, kGen, &f);
  }
  OCHK(launch_gan_gen_bwd(H, E, d.P + go, d.P + dof, d.G + go, d.gan_ws, sg, fz ? &f : nullptr));
  if (!fused) {
    OCALL(collective(cb, user, PGP_COLL_GEN_GRAD, sg));
    next_scalars(o, kGen);
  }
  if (!fz) OCHK(launch_adamw(o->adam[kGen], sg));
  return PGP_OK;
}

}  // namespace

extern "C" {

int pgp_online_create(const pgp_online_desc* desc, pgp_online** out) {
  if (!desc || !out) return ofail(PGP_ERR_ARG, "pgp_online_create: NULL argument");
  *out = nullptr;
  const pgp_online_desc& d = *desc;
  const int H = d.n_hosts, E = d.n_env, R = d.n_rows, K = d.n_protos;
  if (E < 1 || R < 1 || R > kMaxTuneRows) return ofail(PGP_ERR_ARG, "pgp_online_create: 1 <= n_env, 1 <= n_rows <= 16");
  if (K < 3 || K > kMaxProtos) return ofail(PGP_ERR_ARG, "pgp_online_create: n_protos");
  const size_t olen = pgp_master_len(H);
  if (olen == 0) return ofail(PGP_ERR_UNSUPPORTED, "pgp_online_create: host count not compiled in");
  const void* need[] = {d.series, d.train_max, d.sched, d.envs, d.P, d.G, d.exp_avg, d.exp_avg_sq, d.tune_ws,
                        d.logits, d.protos, d.windows, d.y, d.cls, d.state, d.mult, d.tgt, d.loss, d.inc, d.dp_ws,
                        d.adam_rows, d.gan_ws, d.ns, d.probs, d.emb, d.sim_out, d.target, d.tensors};
  for (const void* p : need)
    if (!p) return ofail(PGP_ERR_ARG, "pgp_online_create: NULL buffer in the descriptor");
  if ((d.n_cond > 0 && !d.cond_steps) || d.n_tensors < 1 || d.n_tensors > 3 * kMaxTensors)
    return ofail(PGP_ERR_ARG, "pgp_online_create: tensors / cond_steps");
  auto* o = new pgp_online;
  o->d = d;
  o->H = H;
  o->E = E;
  o->R = R;
  o->B = E * R;
  o->K = K;
  const int B = o->B;
  if (!tune_plan(H, B + E, &o->fwd) || !tune_plan_prefix(H, B + E, B, &o->bwd)) {
    delete o;
    return ofail(PGP_ERR_ARG, "pgp_online_create: tuning plan");
  }
  o->sec_lo[kTr] = (long)pgp_master_offset(H, 0);
  o->sec_lo[kGen] = (long)pgp_master_offset(H, 1);
  o->sec_lo[kDisc] = (long)pgp_master_offset(H, 2);
  const long sec_hi[3] = {o->sec_lo[kGen], o->sec_lo[kDisc], (long)olen};
  for (int s = 0; s < 3; ++s) {
    AdamArgs& a = o->adam[s];
    a.param = d.P;
    a.grad = d.G;
    a.m = d.exp_avg;
    a.v = d.exp_avg_sq;
    a.lr_wd = (float)d.lr[s] * (float)d.weight_decay;  // pgp_adamw_table's (float lr) * (float wd)
    a.b1 = (float)d.beta1;
    a.b2 = (float)d.beta2;
    a.eps = (float)d.eps;
    a.ntensors = 0;
    a.sched = s == kTr ? d.adam_rows : nullptr;
  }
  int ncond = 0;
  for (int i = 0; i < d.n_tensors; ++i) {
    const pgp_online_tensor& t = d.tensors[i];
    if (t.section < 0 || t.section > 2) {
      delete o;
      return ofail(PGP_ERR_ARG, "pgp_online_create: tensor section");
    }
    AdamArgs& a = o->adam[t.section];
    if (a.ntensors >= kMaxTensors || t.offset < o->sec_lo[t.section] || t.n < 0 ||
        (long)t.offset + t.n > sec_hi[t.section] || (t.cond && t.section != kTr)) {
      delete o;
      return ofail(PGP_ERR_ARG, "pgp_online_create: tensor outside its section (or a conditional GAN tensor)");
    }
    const int j = a.ntensors++;
    a.t[j].off = (long)t.offset;
    a.t[j].n = t.n;
    a.t[j].active = t.cond ? kAdamFromTable : 1;
    o->step[t.section][j] = t.step;
    if (t.cond) {
      if (ncond >= kMaxCond) {
        delete o;
        return ofail(PGP_ERR_ARG, "pgp_online_create: too many conditional tensors");
      }
      o->cr.row[ncond++] = j;
    }
  }
  if (ncond != d.n_cond) {
    delete o;
    return ofail(PGP_ERR_ARG, "pgp_online_create: n_cond does not match the tensors flagged cond");
  }
  o->cr.n = ncond;
  if (hipEventCreateWithFlags(&o->gate, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&o->gan_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&o->tgt_end, hipEventDisableTiming) != hipSuccess) {
    delete o;
    return ofail(PGP_ERR_HIP, "pgp_online_create: events");
  }
  *out = o;
  return PGP_OK;
}

int pgp_online_destroy(pgp_online* o) {
  if (!o) return PGP_OK;
  if (o->gate) (void)hipEventDestroy(o->gate);
  if (o->gan_done) (void)hipEventDestroy(o->gan_done);
  if (o->tgt_end) (void)hipEventDestroy(o->tgt_end);
  for (auto& e : o->tev)
    if (e) (void)hipEventDestroy(e);
  delete o->worker;
  delete o;
  return PGP_OK;
}

int pgp_online_step(pgp_online* o, void* main_stream, void* gan_stream, pgp_collective_fn cb, void* user) {
  if (!o) return ofail(PGP_ERR_ARG, "pgp_online_step: NULL handle");
  const pgp_online_desc& d = o->d;
  const int H = o->H, E = o->E, R = o->R, B = o->B, K = o->K;
  const hipStream_t sm = reinterpret_cast<hipStream_t>(main_stream);
  const hipStream_t sg = gan_stream ? reinterpret_cast<hipStream_t>(gan_stream) : sm;
  o->timed = o->timing;
  o->pending[0] = o->pending[1] = o->pending[2] = false;
  // 1. the dataset: R tuning windows per environment, then the E detect windows
  mark(o, kE0, sm);
  float* detect_win = d.windows + (long)B * 9 * H;
  OCHK(launch_tune_dataset(H, E, R, d.series, d.train_max, d.windows, d.y, d.cls, detect_win, sm));
  mark(o, kE1, sm);
  // 2. ONE forward over the B + E windows (step-start weights)
  // its end (the stop event of its last launch) starts the GAN stream: the
  // GAN forward runs beside the targets
  hipEvent_t gate = (sg != sm && !o->timed) ? o->gate : nullptr;
  OCHK(launch_tune_forward(o->fwd, d.windows, d.P, d.tune_ws, nullptr, d.logits, d.protos, sm, gate));
  mark(o, kE2, sm);
  // 3. main: bookkeeping against the step-start state (the decoders' input
  //    gradient dpre written by the same launch), issued before the GAN part so
  //    the main stream has work while the host issues the GAN launches
  //    (H = 16: the main stream sat idle ≈30 µs here); at world size 1 (no
  //    exchange of the increments) the state update by the same launch's last
  //    workgroup.  Its end (the launch's stop event, no marker packet on the
  //    main stream) starts the backward's side work.
  const StateApplyArgs sa{1, d.decay, o->cr, d.cond_steps, d.adam_rows, d.lr[kTr], d.beta1, d.beta2};
  hipEvent_t tgt_end = (!o->timed && tune_side_active(o->bwd.M)) ? o->tgt_end : nullptr;
  OCHK(launch_tune_targets_dp(H, K, B, d.logits, d.protos, d.y, d.cls, d.state, d.update_min, d.mult, d.tgt, d.loss,
                              d.inc, d.dp_ws, sm, d.tune_ws + o->bwd.dpre, o->bwd.NOP, cb ? nullptr : &sa,
                              tgt_end));
  mark(o, kE3, sm);
  // 4. the GAN stream, from the forward's end: Gen + Disc forward (the
  //    embedding formed inside), the simulated label, the Disc gradient
  GanJoin join{o, sm, sg};
  if (sg != sm) {
    if (!gate) OCHK(hipEventRecord(o->gate, sm));
    OCHK(hipStreamWaitEvent(sg, o->gate, 0));
    join.armed = true;
  }
  mark(o, kG0, sg);
  mark(o, kG1, sg);
  const bool fused = cb == nullptr;  // world size 1: each GAN AdamW inside its gradient kernel
  if (fused && sg != sm && !o->timed && o->issue_worker) {
    // the whole GAN chain issued by the worker while this thread issues the
    // backward (both parts: no exchange between them at world size 1)
    if (!o->worker) o->worker = new IssueWorker;
    struct Joined {  // every exit waits for the worker (its job refers to this frame)
      IssueWorker* w;
      bool waited = false;
      int rc = PGP_OK;
      std::string err;
      int wait() {
        if (!waited) {
          rc = w->wait(&err);
          waited = true;
        }
        return rc;
      }
      ~Joined() { wait(); }
    } jw{o->worker};
    o->worker->post([o, sg] {
      OCALL(gan_part_a(o, sg, true));
      return gan_part_b(o, sg, true, nullptr, nullptr);
    });
    OCHK(launch_tune_backward(o->bwd, d.P, d.G, d.tune_ws, d.logits, d.protos, d.y, d.mult, d.tgt, sm, true,
                              tgt_end));
    if (jw.wait() != PGP_OK) return ofail(jw.rc, jw.err);
  } else {
    // (issuing the backward before the GAN part at world size 1 measured the same:
    // 0.1851 vs 0.1853 ms at H = 16, profiles/r06/ab/abb16_bwdfirst.txt)
    OCALL(gan_part_a(o, sg, fused));
    // then the backward
    OCHK(launch_tune_backward(o->bwd, d.P, d.G, d.tune_ws, d.logits, d.protos, d.y, d.mult, d.tgt, sm, true,
                              tgt_end));
    mark(o, kE4, sm);
    // 5. the GAN's updates (its collectives on the GAN stream)
    OCALL(gan_part_b(o, sg, fused, cb, user));
    mark(o, kG2, sg);
  }
  // 6. the tuning step's exchange, state update and AdamW
  OCALL(collective(cb, user, PGP_COLL_TUNE_GRAD, sm));
  OCALL(collective(cb, user, PGP_COLL_TUNE_STATE, sm));
  mark(o, kE5, sm);
  if (cb)
    OCHK(launch_tune_state_apply(K, d.state, d.inc, d.decay, o->cr, d.cond_steps, d.adam_rows, d.lr[kTr], d.beta1,
                                 d.beta2, sm));
  next_scalars(o, kTr);
  OCHK(launch_adamw(o->adam[kTr], sm));
  mark(o, kE6, sm);
  if (sg != sm) {
    join.armed = false;
    OCHK(hipEventRecord(o->gan_done, sg));
    OCHK(hipStreamWaitEvent(sm, o->gan_done, 0));
  }
  commit_steps(o);
  (void)R;
  return PGP_OK;
}

int pgp_online_issue_worker(pgp_online* o, int on) {
  if (!o) return ofail(PGP_ERR_ARG, "pgp_online_issue_worker: NULL handle");
  o->issue_worker = on != 0;
  return PGP_OK;
}

int pgp_online_timing(pgp_online* o, int on) {
  if (!o) return ofail(PGP_ERR_ARG, "pgp_online_timing: NULL handle");
  if (on && !o->tev[0])
    for (auto& e : o->tev) OCHK(hipEventCreate(&e));
  o->timing = on != 0;
  return PGP_OK;
}

int pgp_online_stage_ms(pgp_online* o, float* ms) {
  if (!o || !ms) return ofail(PGP_ERR_ARG, "pgp_online_stage_ms: NULL argument");
  if (!o->timed) return ofail(PGP_ERR_STATE, "pgp_online_stage_ms: the last step was not timed (pgp_online_timing)");
  for (auto& e : o->tev) OCHK(hipEventSynchronize(e));
  const int pairs[PGP_ONLINE_NSTAGE][2] = {{kE0, kE1}, {kG0, kG1}, {kG1, kG2}, {kE1, kE6}, {kE1, kE2},
                                           {kE2, kE3}, {kE3, kE4}, {kE4, kE5}, {kE5, kE6}, {kE0, kE6}};
  for (int k = 0; k < PGP_ONLINE_NSTAGE; ++k) OCHK(hipEventElapsedTime(&ms[k], o->tev[pairs[k][0]], o->tev[pairs[k][1]]));
  return PGP_OK;
}

int pgp_online_gan_step(pgp_online* o, void* stream) {
  if (!o) return ofail(PGP_ERR_ARG, "pgp_online_gan_step: NULL handle");
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  o->pending[0] = o->pending[1] = o->pending[2] = false;
  OCALL(gan_part_a(o, s, true));
  OCALL(gan_part_b(o, s, true, nullptr, nullptr));
  commit_steps(o);
  return PGP_OK;
}

int pgp_online_steps(const pgp_online* o, double* steps, int n) {
  if (!o || !steps || n != o->d.n_tensors) return ofail(PGP_ERR_ARG, "pgp_online_steps: arguments");
  int cnt[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const pgp_online_tensor& t = o->d.tensors[i];
    const int j = cnt[t.section]++;
    steps[i] = t.cond ? -1.0 : o->step[t.section][j];
  }
  return PGP_OK;
}

}  // extern "C"
