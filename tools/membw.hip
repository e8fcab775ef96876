// Memory-bandwidth microbenchmark (not part of the product): the ceilings the
// engine's streaming kernels are judged against.
//   read   U float4 loads in flight per thread, grid-stride, summed
//   copy   the same loads, stored plain / non-temporal (the bond scan's shape:
//          read W, write the bond history)
// over buffer sizes from L2-resident (32 MB) through the 256 MB Infinity Cache
// to HBM (4 GB). Usage: membw [blocks_per_cu]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

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
  for (; i < n; i += stride) acc += x[i];
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = acc.x;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const fvec4* __restrict__ x, fvec4* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    fvec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT)
        __builtin_nontemporal_store(v[u], y + i + u * stride);
      else
        y[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) y[i] = x[i];
}

template <typename F>
static float time_ms(int reps, F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 2; ++w) f();
  hipEventRecord(a);
  for (int r = 0; r < reps; ++r) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms / reps;
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int bpc = argc > 1 ? atoi(argv[1]) : 8;
  const int blocks = cus * bpc;
  const long long big = 4096ll << 20;
  fvec4 *buf, *buf2;
  float* out;
  if (hipMalloc(&buf, big) != hipSuccess || hipMalloc(&buf2, big) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  hipMemset(buf, 0, big);
  hipMemset(buf2, 0, big);
  printf("CUs %d, %d blocks x 256 threads\n", cus, blocks);
  const long long sizes_mb[] = {32, 64, 128, 192, 256, 512, 1024, 4096};
  for (long long mb : sizes_mb) {
    const long long n = (mb << 20) / 16;
    const int reps = (int)(16384 / mb) + 3;
    const double B = (double)(mb << 20);
    float r1 = time_ms(reps, [&] { hipLaunchKernelGGL(k_read<1>, dim3(blocks), dim3(256), 0, 0, buf, n, out); });
    float r4 = time_ms(reps, [&] { hipLaunchKernelGGL(k_read<4>, dim3(blocks), dim3(256), 0, 0, buf, n, out); });
    float r8 = time_ms(reps, [&] { hipLaunchKernelGGL(k_read<8>, dim3(blocks), dim3(256), 0, 0, buf, n, out); });
    float c4 = time_ms(reps, [&] {
      hipLaunchKernelGGL((k_copy<4, false>), dim3(blocks), dim3(256), 0, 0, buf, buf2, n);
    });
    float c4n = time_ms(reps, [&] {
      hipLaunchKernelGGL((k_copy<4, true>), dim3(blocks), dim3(256), 0, 0, buf, buf2, n);
    });
    float c8n = time_ms(reps, [&] {
      hipLaunchKernelGGL((k_copy<8, true>), dim3(blocks), dim3(256), 0, 0, buf, buf2, n);
    });
    printf("size %5lld MB  read U1 %6.0f U4 %6.0f U8 %6.0f GB/s | copy(r+w) U4 %6.0f U4nt %6.0f U8nt %6.0f GB/s\n",
           mb, B / r1 / 1e6, B / r4 / 1e6, B / r8 / 1e6, 2 * B / c4 / 1e6, 2 * B / c4n / 1e6,
           2 * B / c8n / 1e6);
  }
  return 0;
}
