// pgp_device.hpp — device helpers shared by the gfx950 kernels, and the host
// launch entry points each kernel file exports (pgp_capi.hip calls them).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <string>

#include "pgp_layout.hpp"

namespace pgp {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int kMaxProtos = 64;

// compute units of the current device (cached per device id): grids of
// one-workgroup-per-CU kernels
inline int device_cus() {
  static std::atomic<int> cached[64];  // zero-initialised (static storage)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cached[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

// Kernel arguments shared by the launches of one forward call.
struct FwdArgs {
  int B, H, K;
  const float* windows;  // [B,3,3H]
  const float* sched;    // [B,H,H]
  float* agg;            // workspace: GAT output, [blk][H][3][48]
  float* lat;            // workspace: encoder output tiles, [blk][H][3][KS_D][64]
  float* emb;            // workspace: masked embeddings [B][EP]
  const float* frags;    // device weight fragments (Geo<H> offsets)
  const float* decb;     // split-bf16 decoder weight planes (pgp_decoder.hip DecB), or nullptr
  const float* ganb;     // split-bf16 GAN weight planes (pgp_gansplit.hip GanS), or nullptr
  const float* encb;     // split-bf16 encoder LDS image (pgp_encoder.hip EncS), or nullptr
  const float* tab;      // encoder/decoder tables (LDS-staged)
  const float* gtab;     // GAN tables
  const float* gat;      // GAT constants u[4] | v[4] (device)
  float* logits;
  float* protos;
  int* cls;
  int* any_anom;
  float* probs;
  int* keep;
  int* final_t;
  int* gen_t;
  float* latent;  // optional debug tap [B, 3H^2] (reference order)
};

// PreGAN FPE encoder + detect/diagnose (pgp_fpe.hip)
struct FpeArgs {
  int B;
  const float* windows;  // [B,3,3H]
  const float* h0;       // [B,3] GRU initial state
  const float* tab;      // FpeGeo<H> table
  float* scores;         // [B,H,2] anomaly softmax
  float* protos;         // [B,H,2]
  int* cls;              // [B,H]
  int* any_anom;         // [B]
  float* emb;            // workspace [B][EP] -> K3
};
hipError_t launch_fpe(int H, const FpeArgs& a, hipStream_t st);
// offline FPE_16 training (pgp_fpetrain.hip): one batch-1 step / n forwards
int fpe_param_count();
hipError_t launch_fpe_step(const float* win, const float* h0, const int* y, const int* cls, const float* P, float* G,
                           int K, double* state, double update_min, double decay, double* loss, hipStream_t st);
hipError_t launch_fpe_forward_many(int n, const float* wins, const float* h0s, const float* P, double* probs,
                                   double* protos, hipStream_t st);

// recover_decision's per-container moves (pgp_decide.hip)
hipError_t launch_decide(int B, int C, const int* keep, const int* target, const int* cur, int* moves,
                         int* hosts_from, hipStream_t st);
// run_model's masked embedding over n (window, host) pairs (pgp_decide.hip)
hipError_t launch_embed(long n, const float* logits, const float* protos, float* emb, hipStream_t st);
// dense one-hot schedule rows [rows][H] from host indices (pgp_decide.hip)
hipError_t launch_onehot(int H, long rows, const unsigned char* idx, float* sched, hipStream_t st);

hipError_t launch_gat(const FwdArgs& a, hipStream_t st);
hipError_t launch_encoder(const FwdArgs& a, hipStream_t st);
hipError_t launch_decoder(const FwdArgs& a, hipStream_t st);
// split-bf16 decoder weights (pgp_decoder.hip): floats of the planes (0: the
// fp32 decoder runs at this H) and their derivation from the fp32 fragments
long decoder_split_floats(int H);
hipError_t launch_decoder_split(int H, const float* frags, float* decb, hipStream_t st);
long encoder_split_floats(int H);  // 0: no split-bf16 encoder at this H
hipError_t launch_encoder_split(int H, const float* frags, float* encb, hipStream_t st);
hipError_t launch_gan(const FwdArgs& a, hipStream_t st);
// K3 on split-bf16 MFMAs (pgp_gansplit.hip): plane floats (0: not compiled at
// this H), their derivation from the fp32 fragments, the launch
long gan_split_floats(int H);
hipError_t launch_gan_split_derive(int H, const float* frags, float* planes, hipStream_t st);
hipError_t launch_gan_split(const FwdArgs& a, hipStream_t st);

// training ops (pgp_train.hip)
struct AdamArgs;
struct AdamFuse;
long gan_workspace_floats(int H, int B);
hipError_t launch_adamw(const AdamArgs& a, hipStream_t st);
// fused batch-1 GAN step (pgp_gan1.hip), H in {8, 16}
bool gan1_supported(int H);
hipError_t launch_gan1_forward(int H, const float* emb, const float* sched, const float* Pg, const float* Pd,
                               float* row, float* ns, float* probs, hipStream_t st);
hipError_t launch_gan1_step(int H, const float* target, float* Pg, float* Pd, float* Gg, float* Gd, float* row,
                            const AdamArgs& ad, const AdamArgs& ag, float* probs_gen, float* probs_after,
                            hipStream_t st);

// GAN step (pgp_gantrain.hip); ws = gan_workspace_floats(H, B) floats
// logits != nullptr: the embedding is run_model's mask of logits / protos
// [B][H][2] (PreGANPlus.py:129), formed in the launch and written to emb_out
// (emb unused); probs may be nullptr (the Disc step evaluates the head itself)
hipError_t launch_gan_fwd(int H, int B, const float* emb, const float* sched, const float* Pg, const float* Pd,
                          float* ws, float* ns_out, float* probs, hipStream_t st, const float* logits = nullptr,
                          const float* protos = nullptr, float* emb_out = nullptr);
// probs (may be nullptr): the Disc probabilities of the step's forward; af
// (may be nullptr): the section's AdamW applied as its gradients are written
hipError_t launch_gan_disc_bwd(int H, int B, const float* target, const float* Pd, float* Gdd, float* ws,
                               hipStream_t st, float* probs = nullptr, const AdamFuse* af = nullptr);
hipError_t launch_gan_gen_bwd(int H, int B, const float* Pg, const float* Pd, float* Gdg, float* ws,
                              hipStream_t st, const AdamFuse* af = nullptr);
hipError_t launch_gan_probs(int H, int B, const float* ws, float* probs, hipStream_t st);
// GAN labels (pgp_sim.hip, pgp_simulate's kernel): 1 <= H <= 64
hipError_t launch_simulate(int H, int E, const double* envs, const float* new_sched, const float* orig_sched,
                           double* out, float* target, hipStream_t st);

#define PGP_DEV __device__ __forceinline__

PGP_DEV f32x4 mfma(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
// ---- split-bf16 contraction (K2b, K3): x = x0 + x1 + x2 exactly, each a bf16 ----
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
PGP_DEV unsigned bf16_bits(float x) {  // round to nearest even (finite inputs)
  const unsigned u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
PGP_DEV float bf16_val(unsigned h) { return __uint_as_float(h << 16); }
// 8 floats -> their three bf16 planes, packed as 4 dwords each (element 2d in
// the low half of dword d, 2d + 1 in the high half): one 16x16x32 operand each.
// Per pair: v_cvt_pk_bf16_f32 (round to nearest even, as bf16_bits), the part
// back as two floats, a packed subtract for the exact residual; 9 VALU per pair
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
PGP_DEV unsigned bf16_pack(f32x2 x) { return __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2)); }
PGP_DEV f32x2 bf16_unpack(unsigned h) { return f32x2{__uint_as_float(h << 16), __uint_as_float(h & 0xFFFF0000u)}; }
PGP_DEV void split8(const float (&v)[8], u32x4 (&p)[3]) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const f32x2 x = {v[2 * d], v[2 * d + 1]};
    const unsigned h0 = bf16_pack(x);
    const f32x2 r1 = x - bf16_unpack(h0);
    const unsigned h1 = bf16_pack(r1);
    const f32x2 r2 = r1 - bf16_unpack(h1);
    p[0][d] = h0;
    p[1][d] = h1;
    p[2][d] = bf16_pack(r2);
  }
}
PGP_DEV f32x4 mfma_bf(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
// w . x over one 32-k block as the six products with i + j <= 2, smallest first
// A plane triple's reads have landed here: the compiler's wait for them goes
// before whatever follows (the next triple's reads), not after it with a
// drain of those too (its LDS waits in these loops are lgkmcnt(0))
PGP_DEV void planes_ready(const u32x4 (&w)[3]) { asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2])); }
PGP_DEV f32x4 mfma_bf6(const u32x4 (&w)[3], const u32x4 (&x)[3], f32x4 c) {
  c = mfma_bf(w[2], x[0], c);
  c = mfma_bf(w[1], x[1], c);
  c = mfma_bf(w[0], x[2], c);
  c = mfma_bf(w[1], x[0], c);
  c = mfma_bf(w[0], x[1], c);
  return mfma_bf(w[0], x[0], c);
}
// the same when x is exactly a bf16 (x1 = x2 = 0, e.g. a one-hot schedule): three
// products, the same sums as mfma_bf6 (its other three add exact zeros)
PGP_DEV f32x4 mfma_bf3(const u32x4 (&w)[3], const u32x4 (&x)[3], f32x4 c) {
  c = mfma_bf(w[2], x[0], c);
  c = mfma_bf(w[1], x[0], c);
  return mfma_bf(w[0], x[0], c);
}

// In-launch last-arriver finish (cdna_hip_programming.md, split-K recipe, the
// write-through form): every partial the other workgroups read was stored
// write-through (__hip_atomic_store relaxed / agent = sc1 stores), so no
// release fence: every wave drains its stores, the workgroup counts itself in
// with ONE relaxed agent-scope add, and the workgroup that came last takes an
// agent-scope acquire (then plain loads of the partials are current) and
// resets the counter for the next launch.  Returns whether this workgroup is
// the last of n (every thread; flag: one __shared__ int of the caller's).
PGP_DEV bool arrive_last(unsigned* ctr, unsigned n, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const bool last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}
// a write-through store (sc1) of a partial another workgroup of the launch reads
PGP_DEV void store_wt(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
PGP_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
// Sum over lane groups: v + v[lane ^ 16] (+ the same across lane ^ 32), with
// the gfx950 half-row swaps instead of ds_bpermute round trips.
// permlane16_swap(v, v) returns (rows 0,0,2,2 | rows 1,1,3,3) of v and
// tanh as 1 - 2 / (exp(2x) + 1) on the hardware exp2 / rcp (5 VALU ops vs ~26
// for tanhf): absolute error ~1e-7 (cancellation near 0), saturates to +-1.
// For inference outputs compared at fp32 tolerance; training kernels keep tanhf.
PGP_DEV float tanh_fast(float x) {
  const float e = __expf(2.f * x);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

// permlane32_swap(v, v) returns (halves 0,0 | 1,1): the element-wise sum of the
// pair is the xor-16 / xor-32 sum, bit-identical to v + shfl_xor (a+b == b+a).
PGP_DEV float xsum(float v, bool both) {
  const unsigned u = __float_as_uint(v);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  if (both) {
    const unsigned u2 = __float_as_uint(v);
    const auto q = __builtin_amdgcn_permlane32_swap(u2, u2, false, false);
    v = __uint_as_float(q[0]) + __uint_as_float(q[1]);
  }
  return v;
}

// Paired / transposed forms of xsum.  v_permlane16_swap(d, s) exchanges the
// odd 16-lane rows of d with the even rows of s; v_permlane32_swap(d, s) the
// upper half of d with the lower half of s.  Two different values in one swap
// reduce both at once; every sum keeps xsum's association
// (v0 + v1) + (v2 + v3) over lane groups, so results are bitwise equal to xsum.
PGP_DEV float pl_sum16(float a, float b) {  // rows [a0+a1, b0+b1, a2+a3, b2+b3]
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
PGP_DEV float pl_sum32(float a, float b) {  // rows [a0+a2, a1+a3, b0+b2, b1+b3]
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// a, b <- xsum(a, true), xsum(b, true): 3 swaps + 2 adds instead of 4 + 4
PGP_DEV void xsum2(float& a, float& b) {
  const float s = pl_sum16(a, b);                       // [a01, b01, a23, b23]
  const unsigned su = __float_as_uint(s);
  const auto q = __builtin_amdgcn_permlane32_swap(su, su, false, false);
  const float t = __uint_as_float(q[0]) + __uint_as_float(q[1]);  // [a, b, a, b]
  const unsigned tu = __float_as_uint(t);
  const auto p = __builtin_amdgcn_permlane16_swap(tu, tu, false, false);
  a = __uint_as_float(p[0]);
  b = __uint_as_float(p[1]);
}
// a, b <- xsum(a, false), xsum(b, false) (sums within lane-group pairs {0,1}, {2,3})
PGP_DEV void xsum2_half(float& a, float& b) {
  const unsigned su = __float_as_uint(pl_sum16(a, b));  // [a01, b01, a23, b23]
  const auto p = __builtin_amdgcn_permlane16_swap(su, su, false, false);
  a = __uint_as_float(p[0]);
  b = __uint_as_float(p[1]);
}
// Transposed reduction of up to 4 values: lane group n gets xsum(v[n], true),
// groups n >= NR get 0 (the per-group row pick of the VALU-row GEMVs).
template <int NR>
PGP_DEV float xsum_rows(const float (&v)[NR]) {
  static_assert(NR >= 1 && NR <= 4, "at most 4 rows");
  const float s01 = pl_sum16(v[0], NR > 1 ? v[1] : 0.f);
  const float s23 = NR > 2 ? pl_sum16(v[2], NR > 3 ? v[3] : 0.f) : 0.f;
  return pl_sum32(s01, s23);
}

// Async copy of `ngroups` 1-KiB fragment groups global -> LDS, spread over the
// workgroup's waves (group g by wave g % nwaves).  LDS destination is the
// wave-uniform base + lane*16 (global_load_lds_dwordx4), so a group's 64
// lane-consecutive float4 land contiguously, exactly as packed.
// The lane's byte offset is re-derived at each use (opaque to the optimiser):
// otherwise the compiler keeps a 64-bit per-lane pointer per call site live
// across the kernel's loops, and in K3 (127 VGPRs at H = 50) it spilled them,
// each reload followed by an s_waitcnt vmcnt(0) that also drained the wave's
// prefetches.  With the offset fresh, the load takes the scalar base and a
// 32-bit vector offset.
PGP_DEV void dma_groups(const float* __restrict__ src, float* dst, int ngroups, int wv, int nwaves, int lane) {
  for (int g = wv; g < ngroups; g += nwaves) {
    unsigned off = (unsigned)lane * 16u;
    asm volatile("" : "+v"(off));
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(reinterpret_cast<const char*>(src + (long)g * 256) + off),
        (__attribute__((address_space(3))) void*)(dst + g * 256), 16, 0, 0);
  }
}

// Record an error for pgp_last_error() (pgp_capi.hip) and return `code`.
int set_error(int code, const std::string& msg);

}  // namespace pgp
