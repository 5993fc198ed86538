// Device-side cost of forking work to a second stream and joining it back
// (tools/micro): a chain of N empty kernels on the main stream, with a fork
// (the main stream's event, the side stream waits, one kernel there) and/or a
// join (the side stream's event, the main stream waits) after every kernel, in
// several forms; prints the main stream's device time per chain link (the
// chain enqueued behind a 60 ms hold kernel, so the host's issue rate is out
// of the measurement).
// Build: hipcc --offload-arch=gfx950 -O2 -o fork_cost fork_cost.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void k_small(float* p, int n) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) p[0] = 1.f;
}
// holds the main stream while the host enqueues a whole chain, so the chain
// then runs at the device's pace (not the host's issue rate)
__global__ void k_hold(long long cycles) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(100);
}

int main() {
  hipStream_t m, s;
  (void)hipStreamCreateWithFlags(&m, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float* d;
  (void)hipMalloc(&d, 1024);
  const int n = 1000;
  std::vector<hipEvent_t> evt(2 * n), evd(2 * n);
  for (auto& e : evt) (void)hipEventCreate(&e);
  for (auto& e : evd) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  hipEvent_t a, z;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&z);
  void* args[] = {&d, (void*)&n};
  auto run = [&](const char* name, auto body) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipDeviceSynchronize();
      k_hold<<<1, 64, 0, m>>>(100LL * 60000);  // 60 ms at the 100 MHz wall clock
      (void)hipEventRecord(a, m);
      for (int i = 0; i < n; ++i) body(i);
      (void)hipEventRecord(z, m);
      (void)hipEventSynchronize(z);
      (void)hipDeviceSynchronize();
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, z);
      if (rep) printf("%-58s %.2f us per link\n", name, ms * 1e3 / n);
    }
  };
  run("main only", [&](int) { k_small<<<256, 256, 0, m>>>(d, n); });
  run("+ record (timing event)", [&](int i) {
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipEventRecord(evt[i], m);
  });
  run("+ record (no-timing event)", [&](int i) {
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipEventRecord(evd[i], m);
  });
  run("+ fork: record, side waits, side kernel", [&](int i) {
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipEventRecord(evd[i], m);
    (void)hipStreamWaitEvent(s, evd[i], 0);
    k_small<<<1, 64, 0, s>>>(d, n);
  });
  run("+ fork via hipExtLaunchKernel stop event", [&](int i) {
    (void)hipExtLaunchKernel((const void*)k_small, dim3(256), dim3(256), args, 0, m, nullptr, evd[i], 0);
    (void)hipStreamWaitEvent(s, evd[i], 0);
    k_small<<<1, 64, 0, s>>>(d, n);
  });
  run("+ fork and join (side done long before)", [&](int i) {
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipEventRecord(evd[i], m);
    (void)hipStreamWaitEvent(s, evd[i], 0);
    k_small<<<1, 64, 0, s>>>(d, n);
    (void)hipEventRecord(evd[n + i], s);
    k_small<<<256, 256, 0, m>>>(d, n);
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipStreamWaitEvent(m, evd[n + i], 0);
  });
  run("+ join only (side kernel, ext stop event; main waits 2 later)", [&](int i) {
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipExtLaunchKernel((const void*)k_small, dim3(1), dim3(64), args, 0, s, nullptr, evd[n + i], 0);
    k_small<<<256, 256, 0, m>>>(d, n);
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipStreamWaitEvent(m, evd[n + i], 0);
  });
  run("+ join only (side kernel + record; main waits 2 later)", [&](int i) {
    k_small<<<256, 256, 0, m>>>(d, n);
    k_small<<<1, 64, 0, s>>>(d, n);
    (void)hipEventRecord(evd[n + i], s);
    k_small<<<256, 256, 0, m>>>(d, n);
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipStreamWaitEvent(m, evd[n + i], 0);
  });
  run("+ join only, timing event", [&](int i) {
    k_small<<<256, 256, 0, m>>>(d, n);
    k_small<<<1, 64, 0, s>>>(d, n);
    (void)hipEventRecord(evt[n + i], s);
    k_small<<<256, 256, 0, m>>>(d, n);
    k_small<<<256, 256, 0, m>>>(d, n);
    (void)hipStreamWaitEvent(m, evt[n + i], 0);
  });
  run("  (its baseline: 3 main kernels per link)", [&](int) {
    for (int q = 0; q < 3; ++q) k_small<<<256, 256, 0, m>>>(d, n);
  });
  return 0;
}
