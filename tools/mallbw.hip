// Infinity Cache (MALL) read-rate microbenchmark (not part of the product):
// stream-read a buffer of S MiB again and again (grid-stride float4 loads,
// 8 blocks per CU); once S fits in the 256 MiB Infinity Cache the re-reads are
// served on die. Answers whether a phase that re-reads W shortly after an
// earlier phase read it (a MALL-sized chunk of epochs) can beat HBM.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float fvec4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_read(const fvec4* __restrict__ x, long long n, float* out) {
  fvec4 acc = {0.f, 0.f, 0.f, 0.f};
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    fvec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = acc.x;
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long long maxb = 2048ll << 20;
  fvec4* x;
  float* out;
  if (hipMalloc(&x, maxb) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  (void)hipMemset(x, 0, maxb);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (long long mib : {16, 32, 64, 128, 192, 256, 384, 2048}) {
    const long long n = (mib << 20) / 16;
    for (int u : {1, 4}) {
      auto go = [&] {
        if (u == 1) hipLaunchKernelGGL(k_read<1>, dim3(cus * 8), dim3(256), 0, 0, x, n, out);
        else hipLaunchKernelGGL(k_read<4>, dim3(cus * 8), dim3(256), 0, 0, x, n, out);
      };
      for (int w = 0; w < 3; ++w) go();
      const int reps = (int)(8192 / mib) + 4;
      (void)hipEventRecord(a);
      for (int r = 0; r < reps; ++r) go();
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, a, b);
      printf("read %5lld MiB U%d  %8.4f ms/pass  %7.0f GB/s\n", mib, u, ms / reps,
             (double)(mib << 20) * reps / ms / 1e6);
    }
  }
  return 0;
}
