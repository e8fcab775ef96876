// Access-pattern microbenchmark for the column-resident kernels (consensus,
// rank): read 1000 slices of 256 x 4096 fp32 (4 GiB) where each wave owns a
// column group of a slice and every lane reads rows rg, rg+RG, ... of its
// column quad. RG row groups x CQ column quads = 64 lanes, so one float4 wave
// instruction touches RG rows x (16*CQ) contiguous bytes. Not part of the
// product; decides the lane layout.
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int V = 256, M = 4096, SL = 1000;

template <int RG, int HOLD>
__global__ __launch_bounds__(256) void k_tile(const float* __restrict__ W, float* out) {
  constexpr int CQ = 64 / RG, CW = 4 * CQ, NR = V / RG;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rg = lane % RG, cq = lane / RG;
  const long long wid = (long long)blockIdx.x * 4 + wave;
  const long long groups = M / CW;
  const long long slice = wid / groups;
  const int g = (int)(wid % groups);
  const float* base = W + slice * (long long)V * M + g * CW + cq * 4;
  float acc = 0.f;
  if (HOLD) {
    // all rows resident in registers before use (what the kernels do)
    float4 v[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) v[i] = *reinterpret_cast<const float4*>(base + (long long)(rg + RG * i) * M);
#pragma unroll
    for (int i = 0; i < NR; ++i) acc += v[i].x + v[i].y + v[i].z + v[i].w;
  } else {
#pragma unroll 16
    for (int i = 0; i < NR; ++i) {
      const float4 v = *reinterpret_cast<const float4*>(base + (long long)(rg + RG * i) * M);
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 1234.5f) out[0] = acc;
}

// LDS-staged: the block loads its 256 x 64 tile with 4 rows x 256 B per wave
// instruction into LDS, then each wave reads its 16 columns back.
__global__ __launch_bounds__(256) void k_lds(const float* __restrict__ W, float* out) {
  __shared__ float4 t[V * 16];  // 64 KB: [row][16 quads]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long tiles = M / 64;
  const long long slice = blockIdx.x / tiles;
  const int tile = (int)(blockIdx.x % tiles);
  const float* base = W + slice * (long long)V * M + tile * 64;
  const int r0 = threadIdx.x >> 4, q = threadIdx.x & 15;
#pragma unroll 16
  for (int i = 0; i < V / 16; ++i) t[(r0 + 16 * i) * 16 + q] = *reinterpret_cast<const float4*>(base + (long long)(r0 + 16 * i) * M + q * 4);
  __syncthreads();
  const int rg = lane & 15, cq = lane >> 4;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float4 v = t[(rg + 16 * i) * 16 + wave * 4 + cq];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

template <typename F>
void timeit(const char* name, F launch, double bytes) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 2; ++w) launch();
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms / reps, bytes * reps / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t n = (size_t)SL * V * M;
  float *W, *out;
  hipMalloc(&W, n * 4);
  hipMalloc(&out, 4);
  hipMemset(W, 0, n * 4);
  const double bytes = (double)n * 4;
#define T(RG, HOLD)                                                                       \
  timeit("rows/instr " #RG " hold " #HOLD, [&] {                                         \
    const long long waves = (long long)SL * (M / (4 * (64 / RG)));                        \
    hipLaunchKernelGGL((k_tile<RG, HOLD>), dim3(waves / 4), dim3(256), 0, 0, W, out);     \
  }, bytes)
  T(16, 1);
  T(16, 0);
  T(8, 1);
  T(8, 0);
  T(4, 0);
  T(2, 0);
  T(1, 0);
  timeit("lds-staged 64-col tile", [&] {
    hipLaunchKernelGGL(k_lds, dim3((long long)SL * (M / 64)), dim3(256), 0, 0, W, out);
  }, bytes);
  return 0;
}
