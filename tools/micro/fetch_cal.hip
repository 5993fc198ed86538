// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE per access width on
// gfx950 (tools/micro): each kernel streams a 1 GiB buffer (far past the
// 256 MB Infinity Cache) once, coalesced, with W bytes per lane per
// instruction, W = 4, 8, 12, 16 (12: a kernel's
// bytes are 12 x floor(2^30 / 12)); the read kernels write one float per workgroup,
// the write kernels read nothing.  Run under `rocprofv3 --pmc FETCH_SIZE` and
// `--pmc WRITE_SIZE` (separate passes); bytes / (counter x 1024) is the
// correction factor for that width (tools/pmc_traffic.py).
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_cal fetch_cal.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr long kBytes = 1L << 30;

template <int W>
struct Vec;
template <>
struct Vec<4> {
  using T = float;
  __device__ static float sum(T v) { return v; }
  __device__ static T make(float x) { return x; }
};
template <>
struct Vec<8> {
  using T = float2;
  __device__ static float sum(T v) { return v.x + v.y; }
  __device__ static T make(float x) { return make_float2(x, x); }
};
template <>
struct Vec<12> {
  using T = float3;
  __device__ static float sum(T v) { return v.x + v.y + v.z; }
  __device__ static T make(float x) { return make_float3(x, x, x); }
};
template <>
struct Vec<16> {
  using T = float4;
  __device__ static float sum(T v) { return v.x + v.y + v.z + v.w; }
  __device__ static T make(float x) { return make_float4(x, x, x, x); }
};

template <int W>
__global__ __launch_bounds__(256) void read_w(const typename Vec<W>::T* __restrict__ p, long n, float* out) {
  float acc = 0.f;
  const long stride = (long)gridDim.x * blockDim.x;
#pragma unroll 4
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc += Vec<W>::sum(p[i]);
  __shared__ float red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int k = 0; k < 256; ++k) s += red[k];
    out[blockIdx.x] = s;
  }
}

template <int W>
__global__ __launch_bounds__(256) void write_w(typename Vec<W>::T* __restrict__ p, long n, float x) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = Vec<W>::make(x + (float)i);
}

int main() {
  void* buf;
  float* out;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 4096 * sizeof(float)) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, kBytes);
  const int grid = 2048;
  for (int rep = 0; rep < 3; ++rep) {
    read_w<4><<<grid, 256>>>((const float*)buf, kBytes / 4, out);
    read_w<8><<<grid, 256>>>((const float2*)buf, kBytes / 8, out);
    read_w<12><<<grid, 256>>>((const float3*)buf, kBytes / 12, out);
    read_w<16><<<grid, 256>>>((const float4*)buf, kBytes / 16, out);
    write_w<4><<<grid, 256>>>((float*)buf, kBytes / 4, 1.f);
    write_w<8><<<grid, 256>>>((float2*)buf, kBytes / 8, 1.f);
    write_w<12><<<grid, 256>>>((float3*)buf, kBytes / 12, 1.f);
    write_w<16><<<grid, 256>>>((float4*)buf, kBytes / 16, 1.f);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("fetch_cal: %ld bytes per kernel, widths 4 / 8 / 12 / 16 B per lane, 3 launches each\n", kBytes);
  return 0;
}
