// HBM ceiling sweep (not part of the product; round 3):
// what read-only, write-only and copy rates a 4 GiB stream reaches on this
// part, by bytes in flight per CU (waves per CU x float4 per lane in flight)
// and by store flavour (plain, nt, sc1 write-through via buffer stores).
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbmbw tools/hbmbw.hip && tools/hbmbw
// Persistent grid (cus x bpc blocks of 256 threads) walking 16 KiB x U
// chunks: every block takes chunks b, b + grid, ... ; within a chunk lane l
// of wave w moves float4s (w*64 + l) + 256 k, k < U (U wave instructions of
// 1 KiB contiguous each).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float fvec4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

// ST: 0 plain, 1 nt (__builtin_nontemporal_store), 2 sc1 (buffer store aux 16), 3 nt|sc1 (aux 18)
template <int ST>
__device__ __forceinline__ void st4(fvec4* base, long long i, fvec4 v) {
  if (ST == 0) {
    base[i] = v;
  } else if (ST == 1) {
    __builtin_nontemporal_store(v, base + i);
  } else {
    // buffer offsets are 32-bit: rebase per 1 GiB window
    const long long win = i >> 26;  // 2^26 float4 = 1 GiB
    const int off = (int)((i & ((1ll << 26) - 1)) * 16);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                           rsrc(base + (win << 26)), off, 0, ST == 2 ? 16 : 18);
  }
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const fvec4* __restrict__ x, long long chunks, float* out) {
  fvec4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long long c = blockIdx.x; c < chunks; c += gridDim.x) {
    const fvec4* p = x + c * 256 * U + threadIdx.x;
    fvec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = acc.x;
}

template <int U, int ST>
__global__ __launch_bounds__(256) void k_write(fvec4* __restrict__ y, long long chunks, float val) {
  const fvec4 v = {val, val + 1.f, val + 2.f, val + 3.f};
  for (long long c = blockIdx.x; c < chunks; c += gridDim.x) {
    const long long b = c * 256 * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) st4<ST>(y, b + u * 256, v);
  }
}

// copy; PIPE: the next chunk's loads are issued before this chunk's stores
template <int U, int ST, bool PIPE>
__global__ __launch_bounds__(256) void k_copy(const fvec4* __restrict__ x, fvec4* __restrict__ y, long long chunks) {
  long long c = blockIdx.x;
  if (c >= chunks) return;
  fvec4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = x[c * 256 * U + threadIdx.x + u * 256];
  for (; c < chunks; c += gridDim.x) {
    const long long b = c * 256 * U + threadIdx.x;
    const long long cn = c + gridDim.x;
    if (PIPE) {
      fvec4 w[U];
      if (cn < chunks) {
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = x[cn * 256 * U + threadIdx.x + u * 256];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) st4<ST>(y, b + u * 256, v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = w[u];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) st4<ST>(y, b + u * 256, v[u]);
      if (cn < chunks) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = x[cn * 256 * U + threadIdx.x + u * 256];
      }
    }
  }
}

// even blocks read x, odd blocks write y (concurrent independent streams)
template <int U, int ST>
__global__ __launch_bounds__(256) void k_split(const fvec4* __restrict__ x, fvec4* __restrict__ y, long long chunks,
                                               float* out) {
  const int half = gridDim.x / 2;
  const int b = blockIdx.x >> 1;
  if (blockIdx.x & 1) {
    const fvec4 v = {1.f, 2.f, 3.f, 4.f};
    for (long long c = b; c < chunks; c += half) {
      const long long o = c * 256 * U + threadIdx.x;
#pragma unroll
      for (int u = 0; u < U; ++u) st4<ST>(y, o + u * 256, v);
    }
  } else {
    fvec4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long c = b; c < chunks; c += half) {
      const fvec4* p = x + c * 256 * U + threadIdx.x;
      fvec4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p[u * 256];
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = acc.x;
  }
}

template <typename F>
static float time_ms(int reps, F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  f();
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

static void rep(const char* name, double moved, float ms) {
  printf("%-44s %8.3f ms  %7.0f GB/s\n", name, ms, moved / ms / 1e6);
  fflush(stdout);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long long bytes = 4096ll << 20;
  const long long n = bytes / 16;
  fvec4 *x, *y;
  float* out;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  hipMemset(x, 0, bytes);
  hipMemset(y, 0, bytes);
  const int reps = 5;
  const double B = (double)bytes;
  char nm[96];
#define SWEEP_U(KERNEL_EXPR, LABEL, MOVED)                                                         \
  for (int bpc : {2, 4, 8}) {                                                                      \
    const int g = cus * bpc;                                                                       \
    snprintf(nm, sizeof nm, "%s U4 (%d blk/CU)", LABEL, bpc);                                      \
    { constexpr int U = 4; const long long ch = n / (256 * U); rep(nm, MOVED, time_ms(reps, [&] { KERNEL_EXPR; })); } \
    snprintf(nm, sizeof nm, "%s U8 (%d blk/CU)", LABEL, bpc);                                      \
    { constexpr int U = 8; const long long ch = n / (256 * U); rep(nm, MOVED, time_ms(reps, [&] { KERNEL_EXPR; })); } \
    if (bpc <= 4) {                                                                                \
      snprintf(nm, sizeof nm, "%s U16 (%d blk/CU)", LABEL, bpc);                                   \
      { constexpr int U = 16; const long long ch = n / (256 * U); rep(nm, MOVED, time_ms(reps, [&] { KERNEL_EXPR; })); } \
    }                                                                                              \
  }
  SWEEP_U(hipLaunchKernelGGL((k_read<U>), dim3(g), dim3(256), 0, 0, x, ch, out), "read", B)
  SWEEP_U(hipLaunchKernelGGL((k_write<U, 0>), dim3(g), dim3(256), 0, 0, y, ch, 1.f), "write plain", B)
  SWEEP_U(hipLaunchKernelGGL((k_write<U, 1>), dim3(g), dim3(256), 0, 0, y, ch, 1.f), "write nt", B)
  SWEEP_U(hipLaunchKernelGGL((k_write<U, 2>), dim3(g), dim3(256), 0, 0, y, ch, 1.f), "write sc1", B)
  SWEEP_U(hipLaunchKernelGGL((k_write<U, 3>), dim3(g), dim3(256), 0, 0, y, ch, 1.f), "write nt sc1", B)
  SWEEP_U(hipLaunchKernelGGL((k_copy<U, 0, false>), dim3(g), dim3(256), 0, 0, x, y, ch), "copy plain", 2 * B)
  SWEEP_U(hipLaunchKernelGGL((k_copy<U, 1, false>), dim3(g), dim3(256), 0, 0, x, y, ch), "copy nt", 2 * B)
  SWEEP_U(hipLaunchKernelGGL((k_copy<U, 2, false>), dim3(g), dim3(256), 0, 0, x, y, ch), "copy sc1", 2 * B)
  SWEEP_U(hipLaunchKernelGGL((k_copy<U, 0, true>), dim3(g), dim3(256), 0, 0, x, y, ch), "copy plain pipe", 2 * B)
  SWEEP_U(hipLaunchKernelGGL((k_copy<U, 1, true>), dim3(g), dim3(256), 0, 0, x, y, ch), "copy nt pipe", 2 * B)
  SWEEP_U(hipLaunchKernelGGL((k_copy<U, 2, true>), dim3(g), dim3(256), 0, 0, x, y, ch), "copy sc1 pipe", 2 * B)
  SWEEP_U(hipLaunchKernelGGL((k_split<U, 0>), dim3(2 * g), dim3(256), 0, 0, x, y, ch, out), "split r|w plain", 2 * B)
  SWEEP_U(hipLaunchKernelGGL((k_split<U, 1>), dim3(2 * g), dim3(256), 0, 0, x, y, ch, out), "split r|w nt", 2 * B)
  rep("hipMemcpyAsync D2D", 2 * B, time_ms(reps, [&] { hipMemcpyAsync(y, x, bytes, hipMemcpyDeviceToDevice, 0); }));
  rep("hipMemsetAsync", B, time_ms(reps, [&] { hipMemsetAsync(y, 1, bytes, 0); }));
  return 0;
}
