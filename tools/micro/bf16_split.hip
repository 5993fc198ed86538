// bf16_split.hip — accuracy of an fp32 GEMM evaluated as split-bf16 MFMAs on
// gfx950 (the decoder GEMM of K2b: [windows x 3H^2] x [3H^2 x 4H]).
//
// x = x0 + x1 + x2 with x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)
// (each residual exact in fp32), w likewise.  a.b = sum over i + j <= 2 of
// a_i.b_j (6 v_mfma_f32_16x16x32_bf16, every bf16 x bf16 product exact in
// fp32) drops terms below 2^-26 relative.  Compared with the fp32 MFMA
// (v_mfma_f32_16x16x4_f32, an exact fmaf chain) against an fp64 reference on
// the host, per output: |err| / sum_k |a_k b_k| and |err| / |ref|.
//   variants: f32   16x16x4 fp32 MFMA
//             bf6   6 products into one accumulator
//             bf6s  a0.b0 into one accumulator, the 5 correction products into
//                   a second, summed at the end
//             bf3   2-way split, 3 products (a0b0 + a0b1 + a1b0)
// usage: bf16_split [tiles] [K]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned short bf16_rne(float x) {
  unsigned u = __float_as_uint(x);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf16_f(unsigned short h) { return __uint_as_float((unsigned)h << 16); }

__device__ __forceinline__ void split3(float x, unsigned short& h0, unsigned short& h1, unsigned short& h2) {
  h0 = bf16_rne(x);
  const float r1 = x - bf16_f(h0);
  h1 = bf16_rne(r1);
  const float r2 = r1 - bf16_f(h1);
  h2 = bf16_rne(r2);
}

union V8 {
  bf16x8 v;
  unsigned short s[8];
};

// one wave per 16x16 tile; A [T][16][K] row-major, B [T][K][16] row-major
__global__ void k_f32(int K, const float* A, const float* B, float* C) {
  const int t = blockIdx.x, l = threadIdx.x, i = l % 16, g = l / 16;
  const float* a = A + (long)t * 16 * K;
  const float* b = B + (long)t * K * 16;
  f32x4 acc = {0, 0, 0, 0};
  for (int k = 0; k < K; k += 4)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i * K + k + g], b[(k + g) * 16 + i], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(long)t * 256 + (4 * g + r) * 16 + i] = acc[r];
}

template <int MODE>  // 0 bf6, 1 bf6s, 2 bf3
__global__ void k_bf(int K, const float* A, const float* B, float* C) {
  const int t = blockIdx.x, l = threadIdx.x, i = l % 16, g = l / 16;
  const float* a = A + (long)t * 16 * K;
  const float* b = B + (long)t * K * 16;
  f32x4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
  for (int k = 0; k < K; k += 32) {
    V8 a0, a1, a2, b0, b1, b2;
    for (int e = 0; e < 8; ++e) {
      const float av = a[i * K + k + 8 * g + e];
      const float bv = b[(k + 8 * g + e) * 16 + i];
      if (MODE == 2) {
        a0.s[e] = bf16_rne(av);
        a1.s[e] = bf16_rne(av - bf16_f(a0.s[e]));
        b0.s[e] = bf16_rne(bv);
        b1.s[e] = bf16_rne(bv - bf16_f(b0.s[e]));
      } else {
        split3(av, a0.s[e], a1.s[e], a2.s[e]);
        split3(bv, b0.s[e], b1.s[e], b2.s[e]);
      }
    }
    if (MODE == 0) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2.v, b0.v, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1.v, b1.v, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, b2.v, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1.v, b0.v, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, b1.v, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, b0.v, acc, 0, 0, 0);
    } else if (MODE == 1) {
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2.v, b0.v, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1.v, b1.v, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, b2.v, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1.v, b0.v, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, b1.v, acc2, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, b0.v, acc, 0, 0, 0);
    } else {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1.v, b0.v, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, b1.v, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0.v, b0.v, acc, 0, 0, 0);
    }
  }
  for (int r = 0; r < 4; ++r) C[(long)t * 256 + (4 * g + r) * 16 + i] = acc[r] + acc2[r];
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 128;
  const int K = argc > 2 ? atoi(argv[2]) : 7680;
  if (K % 32) return 2;
  std::mt19937_64 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::uniform_real_distribution<float> ud(-1.f, 1.f);
  const float wb = 1.f / std::sqrt((float)K);
  std::vector<float> A((size_t)T * 16 * K), B((size_t)T * K * 16);
  for (auto& v : A) v = nd(rng);          // post-LayerNorm latent ~ N(0, 1)
  for (auto& v : B) v = ud(rng) * wb;     // Linear default init
  std::vector<double> R((size_t)T * 256), S((size_t)T * 256);
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0, sa = 0;
        for (int k = 0; k < K; ++k) {
          const double p = (double)A[((size_t)t * 16 + i) * K + k] * (double)B[((size_t)t * K + k) * 16 + j];
          s += p;
          sa += std::fabs(p);
        }
        R[(size_t)t * 256 + i * 16 + j] = s;
        S[(size_t)t * 256 + i * 16 + j] = sa;
      }
  float *dA, *dB, *dC;
  CK(hipMalloc(&dA, A.size() * 4));
  CK(hipMalloc(&dB, B.size() * 4));
  CK(hipMalloc(&dC, (size_t)T * 256 * 4));
  CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  std::vector<float> C((size_t)T * 256);
  const char* names[4] = {"f32", "bf6", "bf6s", "bf3"};
  for (int v = 0; v < 4; ++v) {
    if (v == 0) k_f32<<<T, 64>>>(K, dA, dB, dC);
    if (v == 1) k_bf<0><<<T, 64>>>(K, dA, dB, dC);
    if (v == 2) k_bf<1><<<T, 64>>>(K, dA, dB, dC);
    if (v == 3) k_bf<2><<<T, 64>>>(K, dA, dB, dC);
    CK(hipGetLastError());
    CK(hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost));
    double mx = 0, rms = 0, mxr = 0, mxa = 0;
    for (size_t n = 0; n < C.size(); ++n) {
      const double e = std::fabs((double)C[n] - R[n]);
      mx = std::max(mx, e / S[n]);
      rms += (e / S[n]) * (e / S[n]);
      mxa = std::max(mxa, e);
      if (std::fabs(R[n]) > 0.1) mxr = std::max(mxr, e / std::fabs(R[n]));
    }
    printf("%-5s K=%d tiles=%d  max|err|/sum|ab| %.3e  rms %.3e  max|err| %.3e  max rel (|ref|>0.1) %.3e\n", names[v],
           K, T, mx, std::sqrt(rms / C.size()), mxa, mxr);
  }
  return 0;
}
