// Read-bandwidth microbenchmark: repeated float4 streaming reads of a buffer of
// a given size, to see where the 256 MB Infinity Cache stops helping
// (decides the epoch chunk size of the engine). Not part of the product.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k_read(const float4* __restrict__ x, long long n, float* out) {
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float4 v = x[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}
__global__ void k_copy(const float4* __restrict__ x, float4* __restrict__ y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) y[i] = x[i];
}

int main() {
  const long long sizes_mb[] = {32, 64, 128, 192, 256, 384, 512, 1024, 4096};
  float* buf; float* buf2; float* out;
  hipMalloc(&buf, 4096ll << 20); hipMalloc(&buf2, 4096ll << 20); hipMalloc(&out, 4);
  hipMemset(buf, 0, 4096ll << 20);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (long long mb : sizes_mb) {
    long long n = (mb << 20) / 16;
    int blocks = 256 * 8;
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, 0, (const float4*)buf, n, out);
    int reps = (int)(8192 / mb) + 2;
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, 0, (const float4*)buf, n, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    double gbs = (double)(mb << 20) * reps / (ms * 1e-3) / 1e9;
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, 0, (const float4*)buf, (float4*)buf2, n);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms2; hipEventElapsedTime(&ms2, a, b);
    double gbs2 = 2.0 * (mb << 20) * reps / (ms2 * 1e-3) / 1e9;
    printf("size %5lld MB  read %7.1f GB/s  copy(r+w) %7.1f GB/s  (%d reps, %.3f ms/read pass)\n", mb, gbs, gbs2, reps, ms / reps);
  }
  return 0;
}
