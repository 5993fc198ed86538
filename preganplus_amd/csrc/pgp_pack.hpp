// pgp_pack.hpp — host-side packing of the reference's fp64 tensors into the
// fragment / table layouts of pgp_layout.hpp.
#pragma once
#include <cstddef>
#include <string>
#include <vector>

#include "pgp_layout.hpp"

namespace pgp {

struct Packed {
  std::vector<float> frags;    // Geo<H>::SZ_FRAGS
  std::vector<float> enc_tab;  // Geo<H>::t_size(K), or FpeGeo<H>::F_SIZE for the FPE variant
  std::vector<float> gan_tab;  // Geo<H>::G_SIZE
  GatConst gat;
};

// Number of doubles in the C-ABI blob for (H, K).
size_t blob_len(int H, int K);

// Pack; returns "" on success or an error message.
std::string pack_weights(int H, int K, const double* blob, size_t len, Packed* out);

// PreGAN FPE variant (FpeGeo<H>): FPE table in enc_tab, GAN chunks in frags.
size_t fpe_blob_len(int H);
std::string pack_fpe_weights(int H, const double* blob, size_t len, Packed* out);

}  // namespace pgp
