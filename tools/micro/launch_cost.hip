// Host cost of one kernel launch on this ROCm (tools/micro): N back-to-back
// launches of an empty kernel, host wall time per launch, for the launch
// forms the library could use.  Build: hipcc --offload-arch=gfx950 -O2 -o
// launch_cost launch_cost.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>

struct Big {
  float v[384];  // 1.5 KB of kernel arguments (AdamArgs / RedTable size)
};
__global__ void k_small(float* p, int n) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) p[0] = 1.f;
}
__global__ void k_big(Big b, float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[7] < -1.f) p[0] = 1.f;
}

template <class F>
double per_launch(F f, int n, hipStream_t s) {
  for (int i = 0; i < 200; ++i) f();
  (void)hipStreamSynchronize(s);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  (void)hipStreamSynchronize(s);
  auto t2 = std::chrono::steady_clock::now();
  double issue = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
  double total = std::chrono::duration<double, std::micro>(t2 - t0).count() / n;
  printf("   issue %.2f us/launch, issue+drain %.2f us/launch\n", issue, total);
  return issue;
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float* d;
  (void)hipMalloc(&d, 1024);
  Big b{};
  const int n = 5000;
  printf("<<<>>> small args, 1 block\n");
  per_launch([&] { k_small<<<1, 64, 0, s>>>(d, n); }, n, s);
  printf("<<<>>> small args, 1024 blocks\n");
  per_launch([&] { k_small<<<1024, 256, 0, s>>>(d, n); }, n, s);
  printf("<<<>>> 1.5 KB args\n");
  per_launch([&] { k_big<<<1, 64, 0, s>>>(b, d); }, n, s);
  printf("<<<>>> + hipGetLastError\n");
  per_launch([&] { k_small<<<1, 64, 0, s>>>(d, n); (void)hipGetLastError(); }, n, s);
  printf("hipLaunchKernel (function pointer)\n");
  void* args[] = {&d, (void*)&n};
  per_launch([&] { (void)hipLaunchKernel((const void*)k_small, dim3(1), dim3(64), args, 0, s); }, n, s);
  printf("hipExtLaunchKernel\n");
  per_launch([&] { (void)hipExtLaunchKernel((const void*)k_small, dim3(1), dim3(64), args, 0, s, nullptr, nullptr, 0); }, n, s);
  hipFunction_t fn = nullptr;
  if (hipGetFuncBySymbol(&fn, (const void*)k_small) == hipSuccess && fn) {
    printf("hipModuleLaunchKernel (hipGetFuncBySymbol)\n");
    per_launch([&] { (void)hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, s, args, nullptr); }, n, s);
  } else {
    printf("hipGetFuncBySymbol unavailable\n");
  }
  hipEvent_t e;
  (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  printf("hipEventRecord\n");
  per_launch([&] { (void)hipEventRecord(e, s); }, n, s);
  hipStream_t s2;
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  printf("record + wait on a second stream + launch there\n");
  per_launch([&] { (void)hipEventRecord(e, s); (void)hipStreamWaitEvent(s2, e, 0); k_small<<<1, 64, 0, s2>>>(d, n); }, n, s2);
  printf("hipMemsetAsync 4 KB\n");
  per_launch([&] { (void)hipMemsetAsync(d, 0, 1024, s); }, n, s);
  // GPU-side: dependent chain of empty kernels, device time per kernel
  hipEvent_t a, z;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&z);
  for (int blocks : {1, 256, 2048}) {
    (void)hipEventRecord(a, s);
    for (int i = 0; i < 2000; ++i) k_small<<<blocks, 256, 0, s>>>(d, n);
    (void)hipEventRecord(z, s);
    (void)hipEventSynchronize(z);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, z);
    printf("device time per back-to-back empty kernel, %d blocks: %.2f us\n", blocks, ms * 1e3 / 2000);
  }
  return 0;
}
