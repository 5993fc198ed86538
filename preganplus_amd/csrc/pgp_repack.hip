// pgp_repack.hip — rebuild the inference kernels' packed weights ON THE DEVICE
// from the training master weights after an optimizer step (the reference's
// AdamW updates the modules in place, utils.py:64-65; the plugin's next
// run_model sees the updated model, PreGANPlus.py:115-136).
//
// The packing code is pgp_packcore.hpp, shared with the host packer
// (pgp_pack.cpp): same loops, fp64 with contraction off, so the device result
// is the host packer's bit for bit.  The source is the master P (fp32, natural
// layout, transformer | gen | disc) followed by the prototypes (fp64 device
// state, [K][2] — the tuning state vector's head), read as fp64 exactly as
// pgp_load_weights_master used to build its host blob.  Three launches (the
// phases of pgp_packcore.hpp), all on the caller's stream; no host round trip,
// no synchronisation.
#include <hip/hip_runtime.h>

#include <cmath>

#include "pgp_packcore.hpp"
#include "pgp_repack.hpp"

namespace pgp {
namespace {

struct DevSrc {
  const float* P;
  long all;
  const double* protos;
  __device__ double operator()(long i) const { return i < all ? (double)P[i] : protos[i - all]; }
};

struct DevEx {
  long tid, nth;
  template <class F>
  __device__ void par(long n, F&& f) const {
    for (long i = tid; i < n; i += nth) f(i);
  }
};

template <int H>
__global__ __launch_bounds__(256) void repack_kernel(int phase, int K, DevSrc src, double scale, double* scr,
                                                     float* F, float* T, float* GT, float* gatc, int sections) {
  const DevEx ex{(long)blockIdx.x * blockDim.x + threadIdx.x, (long)gridDim.x * blockDim.x};
  if (phase == 0)
    packcore::pack_phase0<H>(K, src, ex, scr, gatc);
  else if (phase == 1)
    packcore::pack_phase1<H>(K, src, ex, scale, scr);
  else
    packcore::pack_phase2<H>(K, src, ex, scale, scr, F, T, GT, sections);
}

template <int H>
hipError_t repack_h(const RepackArgs& a, hipStream_t st) {
  using G = Geo<H>;
  const DevSrc src{a.P, a.all, a.protos};
  const double scale = 1.0 / std::sqrt((double)G::HD);
  // the largest loop is the decoders' (H * 3 * DEC_G groups of 256 floats)
  const long big = (long)H * 3 * G::DEC_G * 256;
  const int grid2 = (int)std::min<long>(2048, (big + 255) / 256);
  if (a.sections & 1) {  // phases 0 / 1 feed the encoder / decoder part of phase 2 only
    repack_kernel<H><<<1, 256, 0, st>>>(0, a.K, src, scale, a.scr, a.frags, a.tab, a.gtab, a.gat, a.sections);
    // phase 1 also sums the decoder weights per (row, feature, step): MT_O*16*H*3 items
    const int grid1 = (int)std::min<long>(256, ((long)G::MT_O * 16 * H * 3 + 255) / 256);
    repack_kernel<H><<<grid1, 256, 0, st>>>(1, a.K, src, scale, a.scr, a.frags, a.tab, a.gtab, a.gat, a.sections);
  }
  // the GAN alone: its largest loop is the per-container groups (C * GC_G groups of 256)
  const int gridg = (int)std::min<long>(2048, ((long)G::C * G::GC_G * 256 + 255) / 256);
  repack_kernel<H><<<(a.sections & 1) ? grid2 : gridg, 256, 0, st>>>(2, a.K, src, scale, a.scr, a.frags, a.tab,
                                                                       a.gtab, a.gat, a.sections);
  return hipGetLastError();
}

}  // namespace

long repack_scratch_len(int H) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return packcore::Scratch<h>::SIZE;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return 0;
}

long repack_blob_protos_offset(int H, int K) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return packcore::BlobOff<h>(K).protos;
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return -1;
}

hipError_t launch_repack(int H, const RepackArgs& a, hipStream_t st) {
  switch (H) {
#define CASE(h) \
  case h:       \
    return repack_h<h>(a, st);
    PGP_FOR_EACH_H(CASE)
#undef CASE
  }
  return hipErrorInvalidValue;
}

}  // namespace pgp
