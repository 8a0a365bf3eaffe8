// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the library's kernels use
// (MI355X_MICROARCH.md: the x2 FETCH correction is calibrated for 16 B/lane streaming reads only).
// Streams a 1 GiB buffer (well past the 256 MiB Infinity Cache) with 4 B/lane and 16 B/lane loads
// and stores; prints the algorithmic bytes of every launch.  Profile with
//   rocprofv3 --pmc FETCH_SIZE -- scripts/bin/fetch_calib   (and a separate WRITE_SIZE pass)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void rd1(const float* __restrict__ x, size_t n, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += x[i];
  if (s == 12345.f) out[0] = s;  // keeps the loads, writes nothing in practice
}
__global__ void rd4(const float4* __restrict__ x, size_t n4, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}
__global__ void wr1(float* __restrict__ x, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) x[i] = 1.f;
}
__global__ void wr4(float4* __restrict__ x, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    x[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
  const size_t bytes = (size_t)1 << 30, n = bytes / 4;
  float *x = nullptr, *out = nullptr;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) { printf("alloc failed\n"); return 1; }
  const dim3 g(4096), b(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(wr4, g, b, 0, 0, (float4*)x, n / 4);
    hipLaunchKernelGGL(wr1, g, b, 0, 0, x, n);
    hipLaunchKernelGGL(rd1, g, b, 0, 0, x, n, out);
    hipLaunchKernelGGL(rd4, g, b, 0, 0, (const float4*)x, n / 4, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) { printf("sync failed\n"); return 1; }
  printf("every launch moves %zu bytes (%.1f KiB): wr4, wr1, rd1, rd4 x3\n", bytes, bytes / 1024.0);
  (void)hipFree(x);
  (void)hipFree(out);
  return 0;
}
