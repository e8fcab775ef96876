// HBM write-pattern sweep (not part of the product; round 3). tools/hbmbw
// found pure writes at 4.5-5.6 TB/s in the lane-interleaved shape while
// hipMemsetAsync fills the same 4 GiB at 6.4 TB/s; this sweep looks for the
// store shape that reaches the fill rate, and tries it in a copy.
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbmbw2 tools/hbmbw2.hip
//   tools/hbmbw2            (sweep)      tools/hbmbw2 memset (memset only, for a kernel trace)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

typedef float fvec4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(fvec4* p, fvec4 v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// lane-interleaved: instruction u of a wave writes 1 KiB contiguous; the block
// takes chunks of 256*U float4 grid-stride (tools/hbmbw's shape)
template <int U, bool NT>
__global__ void k_w_inter(fvec4* __restrict__ y, long long n, float val) {
  const fvec4 v = {val, val, val, val};
  const long long chunk = (long long)blockDim.x * U;
  for (long long c = (long long)blockIdx.x * chunk; c < n; c += (long long)gridDim.x * chunk)
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(y + c + u * blockDim.x + threadIdx.x, v);
}

// lane-contiguous: each lane writes U consecutive float4 (U*16 B per lane)
template <int U, bool NT>
__global__ void k_w_lane(fvec4* __restrict__ y, long long n, float val) {
  const fvec4 v = {val, val, val, val};
  const long long chunk = (long long)blockDim.x * U;
  for (long long c = (long long)blockIdx.x * chunk; c < n; c += (long long)gridDim.x * chunk)
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(y + c + (long long)threadIdx.x * U + u, v);
}

// blocked: block b owns one contiguous n/grid region, lane-interleaved U deep
template <int U, bool NT>
__global__ void k_w_block(fvec4* __restrict__ y, long long n, float val) {
  const fvec4 v = {val, val, val, val};
  const long long per = n / gridDim.x;
  fvec4* base = y + (long long)blockIdx.x * per;
  for (long long o = 0; o < per; o += (long long)blockDim.x * U)
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(base + o + u * blockDim.x + threadIdx.x, v);
}

// copy, lane-contiguous U float4 per lane (loads then stores)
template <int U, bool NT>
__global__ void k_c_lane(const fvec4* __restrict__ x, fvec4* __restrict__ y, long long n) {
  const long long chunk = (long long)blockDim.x * U;
  for (long long c = (long long)blockIdx.x * chunk; c < n; c += (long long)gridDim.x * chunk) {
    fvec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[c + (long long)threadIdx.x * U + u];
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(y + c + (long long)threadIdx.x * U + u, v[u]);
  }
}

// copy, lane-interleaved (grid-stride chunks)
template <int U, bool NT>
__global__ void k_c_inter(const fvec4* __restrict__ x, fvec4* __restrict__ y, long long n) {
  const long long chunk = (long long)blockDim.x * U;
  for (long long c = (long long)blockIdx.x * chunk; c < n; c += (long long)gridDim.x * chunk) {
    fvec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[c + u * blockDim.x + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(y + c + u * blockDim.x + threadIdx.x, v[u]);
  }
}

// copy, blocked regions
template <int U, bool NT>
__global__ void k_c_block(const fvec4* __restrict__ x, fvec4* __restrict__ y, long long n) {
  const long long per = n / gridDim.x;
  const long long b0 = (long long)blockIdx.x * per;
  for (long long o = 0; o < per; o += (long long)blockDim.x * U) {
    fvec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[b0 + o + u * blockDim.x + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(y + b0 + o + u * blockDim.x + threadIdx.x, v[u]);
  }
}

template <typename F>
static float time_ms(int reps, F f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  f();
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms / reps;
}

static void rep(const char* name, double moved, float ms) {
  printf("%-46s %8.3f ms  %7.0f GB/s\n", name, ms, moved / ms / 1e6);
  fflush(stdout);
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long long bytes = 4096ll << 20;
  const long long n = bytes / 16;
  fvec4 *x, *y;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, bytes) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  (void)hipMemset(x, 0, bytes);
  (void)hipMemset(y, 0, bytes);
  const int reps = 5;
  const double B = (double)bytes;
  if (argc > 1 && strcmp(argv[1], "memset") == 0) {
    rep("hipMemsetAsync", B, time_ms(reps, [&] { (void)hipMemsetAsync(y, 1, bytes, 0); }));
    rep("hipMemsetD32Async", B, time_ms(reps, [&] { (void)hipMemsetD32Async((hipDeviceptr_t)y, 7, bytes / 4, 0); }));
    return 0;
  }
  rep("hipMemsetAsync", B, time_ms(reps, [&] { (void)hipMemsetAsync(y, 1, bytes, 0); }));
  char nm[96];
  for (int bs : {256, 1024}) {
    for (int bpc : {1, 2, 4, 8}) {
      if (bs == 1024 && bpc > 2) continue;
      const int g = cus * bpc;
#define W(K, LBL)                                                                                  \
  snprintf(nm, sizeof nm, "%s bs%d %d/CU", LBL, bs, bpc);                                          \
  rep(nm, B, time_ms(reps, [&] { hipLaunchKernelGGL(K, dim3(g), dim3(bs), 0, 0, y, n, 1.f); }));
      W((k_w_inter<8, false>), "write inter U8")
      W((k_w_inter<4, false>), "write inter U4")
      W((k_w_lane<4, false>), "write lane U4")
      W((k_w_lane<4, true>), "write lane U4 nt")
      W((k_w_lane<8, false>), "write lane U8")
      W((k_w_block<8, false>), "write block U8")
      W((k_w_block<8, true>), "write block U8 nt")
      W((k_w_block<4, false>), "write block U4")
#undef W
#define C(K, LBL)                                                                                  \
  snprintf(nm, sizeof nm, "%s bs%d %d/CU", LBL, bs, bpc);                                          \
  rep(nm, 2 * B, time_ms(reps, [&] { hipLaunchKernelGGL(K, dim3(g), dim3(bs), 0, 0, x, y, n); }));
      C((k_c_inter<4, false>), "copy inter U4")
      C((k_c_lane<4, false>), "copy lane U4")
      C((k_c_lane<4, true>), "copy lane U4 nt")
      C((k_c_block<4, false>), "copy block U4")
      C((k_c_block<8, false>), "copy block U8")
#undef C
    }
  }
  return 0;
}
