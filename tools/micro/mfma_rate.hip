// Microbenchmark: f32 MFMA issue rate on gfx950 (v_mfma_f32_16x16x4_f32 and
// v_mfma_f32_32x32x2_f32), measured the way MI355X_MICROARCH.md's F32 row is:
// RANDOM operands (per lane, per accumulator), independent accumulators, one
// or two waves per SIMD on every CU, >= 2 s of back-to-back launches before the
// timed one, and the in-kernel clock reported (delta s_memtime / delta
// s_memrealtime x 100 MHz, median over workgroups; the stamps go to a buffer
// of their own).
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_rate mfma_rate.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
constexpr int NACC = 8;

template <int FORM>
__global__ __launch_bounds__(512) void loop(const float* __restrict__ rnd, float* out, unsigned long long* stamps,
                                            int iters) {
  const int t = threadIdx.x;
  float a[NACC], b[NACC];
  for (int i = 0; i < NACC; ++i) {
    a[i] = rnd[(blockIdx.x * 997 + t * 13 + i * 7919) & 0xFFFF];
    b[i] = rnd[(blockIdx.x * 577 + t * 29 + i * 104729) & 0xFFFF];
  }
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  if constexpr (FORM == 0) {
    f4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f4{a[i], b[i], a[i] * b[i], a[i] - b[i]};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[i], acc[i], 0, 0, 0);
    }
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    f16v acc[NACC / 2];
    for (int i = 0; i < NACC / 2; ++i)
      for (int r = 0; r < 16; ++r) acc[i][r] = a[i] * (r + 1) - b[i];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < NACC / 2; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[i], acc[i], 0, 0, 0);
    }
    for (int i = 0; i < NACC / 2; ++i)
      for (int r = 0; r < 16; ++r) s += acc[i][r];
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + t] = s;
  if (t == 0) {
    stamps[2 * blockIdx.x] = c1 - c0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int FORM>
void run(const char* name, const float* rnd, int threads, int iters) {
  const int blocks = 256;  // one workgroup per CU: 256 threads = 1 wave per SIMD, 512 = 2
  float* out;
  unsigned long long* st;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipMalloc(&st, sizeof(unsigned long long) * 2 * blocks);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // warm the clock: >= 2 s of back-to-back launches
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.0) {
    loop<FORM><<<blocks, threads>>>(rnd, out, st, iters);
    hipDeviceSynchronize();
  }
  hipEventRecord(e0);
  loop<FORM><<<blocks, threads>>>(rnd, out, st, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(2 * blocks);
  hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::vector<double> clk(blocks);
  for (int i = 0; i < blocks; ++i) clk[i] = (double)h[2 * i] / (double)h[2 * i + 1] * 100.0;  // MHz
  std::sort(clk.begin(), clk.end());
  const double macs_per = FORM == 0 ? 1024.0 : 2048.0;  // MACs per MFMA: 16x16x4, 32x32x2
  const int nmfma = FORM == 0 ? NACC : NACC / 2;
  const double waves = (double)blocks * threads / 64;
  const double flops = 2.0 * macs_per * nmfma * iters * waves;
  const double cyc_per_mfma = clk[blocks / 2] * 1e6 * ms * 1e-3 / (nmfma * (double)iters * threads / 256);
  printf("%-9s %d wave/SIMD: %.3f ms  %.1f TFLOP/s  in-kernel clock %.0f MHz (median)  %.1f cyc per MFMA per SIMD\n",
         name, threads / 256, ms, flops / ms / 1e9, clk[blocks / 2], cyc_per_mfma);
  hipFree(out);
  hipFree(st);
}

int main() {
  std::mt19937 g(7);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  std::vector<float> h(1 << 16);
  for (auto& v : h) v = u(g);
  float* rnd;
  hipMalloc(&rnd, h.size() * sizeof(float));
  hipMemcpy(rnd, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
  for (int t : {256, 512}) {
    run<0>("16x16x4", rnd, t, 20000);
    run<1>("32x32x2", rnd, t, 10000);
  }
  return 0;
}
