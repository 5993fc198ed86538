// pack_check.cpp — host-only driver of the weight packer (pgp_pack.cpp +
// pgp_packcore.hpp) for sanitizer builds (make asan): packs seeded random
// blobs for every compiled host count and the FPE variant, checks the error
// paths (wrong length), and that packing is deterministic.  Exit code 0 = ok.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../preganplus_amd/csrc/pgp_pack.hpp"

using namespace pgp;

static std::vector<double> blob(size_t n, unsigned seed) {
  std::mt19937_64 g(seed);
  std::normal_distribution<double> nd(0.0, 0.3);
  std::vector<double> b(n);
  for (auto& x : b) x = nd(g);
  return b;
}

static bool same(const Packed& a, const Packed& b) {
  return a.frags == b.frags && a.enc_tab == b.enc_tab && a.gan_tab == b.gan_tab &&
         !std::memcmp(&a.gat, &b.gat, sizeof(a.gat));
}

int main() {
  int bad = 0;
  for (int H : {8, 16, 32, 50, 64}) {
    for (int K : {3, H}) {
      const size_t n = blob_len(H, K);
      const auto b = blob(n, 1000u * H + K);
      Packed p1, p2, p3;
      const std::string e1 = pack_weights(H, K, b.data(), n, &p1);
      const std::string e2 = pack_weights(H, K, b.data(), n, &p2);
      const std::string e3 = pack_weights(H, K, b.data(), n - 1, &p3);
      const bool ok = e1.empty() && e2.empty() && !e3.empty() && same(p1, p2);
      std::printf("H=%d K=%d blob %zu -> frags %zu tab %zu gan %zu: %s\n", H, K, n, p1.frags.size(),
                  p1.enc_tab.size(), p1.gan_tab.size(), ok ? "ok" : "FAIL");
      bad += !ok;
    }
  }
  {
    const size_t n = fpe_blob_len(16);
    const auto b = blob(n, 7);
    Packed p1, p2;
    const bool ok = pack_fpe_weights(16, b.data(), n, &p1).empty() && pack_fpe_weights(16, b.data(), n, &p2).empty() &&
                    same(p1, p2) && !pack_fpe_weights(16, b.data(), n + 1, &p2).empty();
    std::printf("FPE H=16 blob %zu: %s\n", n, ok ? "ok" : "FAIL");
    bad += !ok;
  }
  if (!pack_weights(7, 3, nullptr, 0, nullptr).empty()) std::printf("unsupported H rejected: ok\n");
  return bad;
}
