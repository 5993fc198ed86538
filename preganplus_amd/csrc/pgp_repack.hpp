// pgp_repack.hpp — device repack of the inference weights (pgp_repack.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace pgp {

struct RepackArgs {
  int K;               // prototypes
  const float* P;      // training master, natural layout (transformer | gen | disc)
  long all;            // its length (= the blob offset of the prototypes)
  const double* protos;  // [K][2] fp64, device
  double* scr;         // fp64 scratch, repack_scratch_len(H)
  float* frags;        // Geo<H>::SZ_FRAGS
  float* tab;          // Geo<H>::t_size(K)
  float* gtab;         // Geo<H>::G_SIZE
  float* gat;          // [8] GAT constants u[4] | v[4]
  int sections = 3;    // bit 0: the PreGAN+ encoder / decoders (phases 0-2), bit 1: the GAN (pack_gan)
};

long repack_scratch_len(int H);
long repack_blob_protos_offset(int H, int K);
hipError_t launch_repack(int H, const RepackArgs& a, hipStream_t st);

}  // namespace pgp
