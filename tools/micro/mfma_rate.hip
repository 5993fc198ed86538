// Microbenchmark: f32 MFMA issue rate on gfx950 for the 16x16x4 and the
// 4x4x1 (16-block) forms, independent accumulators, 1 or 2 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_rate mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int NACC = 8;

template <int FORM>
__global__ __launch_bounds__(256) void loop(float* out, int iters, float a0, float b0) {
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0, 0, 0, 0};
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if constexpr (FORM == 0)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
      else
        acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
    }
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int FORM>
void run(const char* name, int blocks, int threads, int iters) {
  float* out;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  loop<FORM><<<blocks, threads>>>(out, iters, 1.0f, 1.0f);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  loop<FORM><<<blocks, threads>>>(out, iters, 1.0f, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double macs_per = FORM == 0 ? 1024.0 : 256.0;
  const double waves = (double)blocks * threads / 64;
  const double flops = 2.0 * macs_per * NACC * iters * waves;
  printf("%-10s blocks %5d threads %4d: %.3f ms  %.1f TFLOP/s\n", name, blocks, threads, ms, flops / ms / 1e9);
  hipFree(out);
}

int main() {
  // 256 CUs: 256 threads = 1 wave/SIMD, 512 = 2 waves/SIMD
  for (int t : {256, 512}) {
    run<0>("16x16x4", 256, t, 20000);
    run<1>("4x4x1_16b", 256, t, 20000);
  }
  run<0>("16x16x4", 1024, 256, 5000);
  run<1>("4x4x1_16b", 1024, 256, 5000);
  return 0;
}
