// Which hardware CU does each bit of hipExtStreamCreateWithCUMask select?
// (tools/micro): for every bit k, a stream masked to that one CU runs one
// workgroup that records its XCC_ID and HW_ID (SE / SH / CU fields); prints
// "bit: xcc.se.cu of each of 16 workgroups".  Build: hipcc --offload-arch=gfx950 -O2 -o cumask_probe cumask_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kWg = 16;  // workgroups per probe launch (two per XCC under round-robin dispatch)
__global__ void probe(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  const int n = prop.multiProcessorCount;
  unsigned* d;
  if (hipMalloc(&d, 2 * kWg * sizeof(unsigned)) != hipSuccess) return 1;
  std::vector<unsigned> mask((n + 31) / 32);
  printf("cus %d\n", n);
  for (int k = 0; k < n; ++k) {
    for (auto& m : mask) m = 0;
    mask[k / 32] = 1u << (k % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (unsigned)mask.size(), mask.data()) != hipSuccess) {
      printf("bit %d: create failed\n", k);
      return 2;
    }
    probe<<<kWg, 64, 0, s>>>(d);
    unsigned h[2 * kWg] = {};
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 4;
    (void)hipStreamDestroy(s);
    // HW_ID (gfx9): wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13
    printf("bit %3d:", k);
    for (int w = 0; w < kWg; ++w)
      printf(" %u.%u.%u", h[2 * w] & 0xf, (h[2 * w + 1] >> 13) & 0x7, (h[2 * w + 1] >> 8) & 0xf);
    printf("\n");
  }
  return 0;
}
