// Read+write ceiling microbenchmark (not part of the product): how fast can
// MI355X stream B bytes in AND B different bytes out of HBM, in the shapes the
// bond scan could use. Every variant moves a 4 GiB source into a 4 GiB
// destination (far beyond the 256 MB Infinity Cache).
//   gridstride  U float4 per thread per trip, grid-stride (tools/membw)
//   blocked     each block copies one contiguous chunk, U loads then U stores
//   write-only  stores only (a fill)
//   read-only   loads only
//   scan        the bond scan's walk: 1000 steps, each reading one 4 MiB slice
//               and writing another, a block owning the same rows every step
//   hipMemcpy   the runtime's device-to-device copy
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float fvec4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_grid(const fvec4* __restrict__ x, fvec4* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i + (U - 1) * stride < n; i += U * stride) {
    fvec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], y + i + u * stride);
      else y[i + u * stride] = v[u];
    }
  }
}

// block b copies [b*chunk, (b+1)*chunk), U float4 per thread per trip, lanes contiguous
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_blocked(const fvec4* __restrict__ x, fvec4* __restrict__ y, long long chunk) {
  const long long base = (long long)blockIdx.x * chunk;
  for (long long o = 0; o < chunk; o += 256 * U) {
    fvec4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[base + o + u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], y + base + o + u * 256 + threadIdx.x);
      else y[base + o + u * 256 + threadIdx.x] = v[u];
    }
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_fill(fvec4* __restrict__ y, long long n, float val) {
  const long long stride = (long long)gridDim.x * 256;
  const fvec4 v = {val, val, val, val};
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    if (NT) __builtin_nontemporal_store(v, y + i);
    else y[i] = v;
  }
}

__global__ __launch_bounds__(256) void k_read(const fvec4* __restrict__ x, long long n, float* out) {
  fvec4 acc = {0.f, 0.f, 0.f, 0.f};
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) acc += x[i];
  if (acc.x + acc.y + acc.z + acc.w == 1234.5f) out[0] = acc.x;
}

// the bond scan's shape: slice t of x ([steps][V][M], 4 MiB) -> slice t of y;
// block (rb, tile) owns rows rb*16.. +16, miners tile*64 .. +64 in every slice;
// P slices of loads in flight (register ring)
template <int P, bool NT>
__global__ __launch_bounds__(256) void k_scan(const fvec4* __restrict__ x, fvec4* __restrict__ y, int steps, int V,
                                              int M) {
  const int tiles = M / 64;
  const int tile = blockIdx.x % tiles, rb = blockIdx.x / tiles;
  const int row = rb * 16 + (threadIdx.x >> 4), c4 = threadIdx.x & 15;
  const long long m4 = (long long)M / 4;
  const long long off = (long long)row * m4 + tile * 16 + c4;
  const long long sl = (long long)V * m4;
  fvec4 ring[P];
  fvec4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < P; ++k) ring[k] = x[k * sl + off];
  for (int t0 = 0; t0 < steps; t0 += P) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int t = t0 + k;
      if (t >= steps) break;
      acc = acc * 0.5f + ring[k];
      if (NT) __builtin_nontemporal_store(acc, y + t * sl + off);
      else y[t * sl + off] = acc;
      if (t + P < steps) ring[k] = x[(t + P) * sl + off];
    }
  }
}

// the scan with R rows per thread (a block owns 16 R rows of the tile)
template <int P, int R, bool NT>
__global__ __launch_bounds__(256) void k_scan_r(const fvec4* __restrict__ x, fvec4* __restrict__ y, int steps, int V,
                                                int M) {
  const int tiles = M / 64;
  const int tile = blockIdx.x % tiles, rb = blockIdx.x / tiles;
  const int c4 = threadIdx.x & 15;
  const long long m4 = (long long)M / 4;
  const long long sl = (long long)V * m4;
  long long off[R];
#pragma unroll
  for (int i = 0; i < R; ++i) off[i] = (long long)(rb * 16 * R + (threadIdx.x >> 4) + 16 * i) * m4 + tile * 16 + c4;
  fvec4 ring[P][R];
  fvec4 acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = fvec4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < P; ++k)
#pragma unroll
    for (int i = 0; i < R; ++i) ring[k][i] = x[k * sl + off[i]];
  for (int t0 = 0; t0 < steps; t0 += P) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int t = t0 + k;
      if (t >= steps) break;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        acc[i] = acc[i] * 0.5f + ring[k][i];
        if (NT) __builtin_nontemporal_store(acc[i], y + t * sl + off[i]);
        else y[t * sl + off[i]] = acc[i];
        if (t + P < steps) ring[k][i] = x[(t + P) * sl + off[i]];
      }
    }
  }
}

// the fused rank + bond scan's shape: a 1024-thread block owns all V = 256
// rows of a 16-miner strip (thread = 1 row x 4 miners, a wave = 16 rows x
// 64 B); per step a column sum over the rows (wave butterfly -> LDS -> one
// barrier every G steps) models the in-block rank reduction
template <int P, int G, bool RED>
__global__ __launch_bounds__(1024) void k_scan16(const fvec4* __restrict__ x, fvec4* __restrict__ y, int steps,
                                                 int V, int M, float* __restrict__ out) {
  __shared__ fvec4 part[G][16][4];
  const int strips = M / 16;
  int blk = blockIdx.x;
  if ((gridDim.x & 7) == 0) blk = (blk & 7) * (gridDim.x >> 3) + (blk >> 3);  // neighbours share an XCD
  const int strip = blk % strips;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane & 3;
  const int row = wave * 16 + (lane >> 2);
  const long long m4 = (long long)M / 4;
  const long long off = (long long)row * m4 + strip * 4 + q;
  const long long sl = (long long)V * m4;
  fvec4 ring[P];
  fvec4 acc = {0.f, 0.f, 0.f, 0.f}, tot = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < P; ++k) ring[k] = x[k * sl + off];
  for (int t0 = 0; t0 < steps; t0 += G) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int t = t0 + g;
      const int k = g % P;
      acc = acc * 0.5f + ring[k];
      __builtin_nontemporal_store(acc, y + t * sl + off);
      if (t + P < steps) ring[k] = x[(t + P) * sl + off];
      if (RED) {
        fvec4 r = acc;
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) {
          r.x += __shfl_xor(r.x, o, 64);
          r.y += __shfl_xor(r.y, o, 64);
          r.z += __shfl_xor(r.z, o, 64);
          r.w += __shfl_xor(r.w, o, 64);
        }
        if (lane < 4) part[g][wave][q] = r;
      }
    }
    if (RED) {
      __syncthreads();
      if (lane < 16 && wave < G) {
        float s = 0.f;
        for (int w = 0; w < 16; ++w) s += part[wave][w][lane >> 2][lane & 3];
        tot.x += s;
      }
      __syncthreads();
    }
  }
  if (tot.x == 1234.5f) out[0] = tot.x;
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
  auto rep = [&](const char* name, double moved, float ms) {
    printf("%-34s %8.3f ms  %7.0f GB/s\n", name, ms, moved / ms / 1e6);
  };
  for (int bpc : {4, 8}) {
    const int g = cus * bpc;
    char nm[64];
    snprintf(nm, sizeof nm, "gridstride U1 (%d/CU)", bpc);
    rep(nm, 2 * B, time_ms(reps, [&] { hipLaunchKernelGGL((k_grid<1, false>), dim3(g), dim3(256), 0, 0, x, y, n); }));
    snprintf(nm, sizeof nm, "gridstride U2 nt (%d/CU)", bpc);
    rep(nm, 2 * B, time_ms(reps, [&] { hipLaunchKernelGGL((k_grid<2, true>), dim3(g), dim3(256), 0, 0, x, y, n); }));
  }
  for (int nb : {1024, 4096, 16384}) {
    const long long chunk = n / nb;
    char nm[64];
    snprintf(nm, sizeof nm, "blocked U4 (%d blocks)", nb);
    rep(nm, 2 * B, time_ms(reps, [&] { hipLaunchKernelGGL((k_blocked<4, false>), dim3(nb), dim3(256), 0, 0, x, y, chunk); }));
    snprintf(nm, sizeof nm, "blocked U4 nt (%d blocks)", nb);
    rep(nm, 2 * B, time_ms(reps, [&] { hipLaunchKernelGGL((k_blocked<4, true>), dim3(nb), dim3(256), 0, 0, x, y, chunk); }));
    snprintf(nm, sizeof nm, "blocked U8 nt (%d blocks)", nb);
    rep(nm, 2 * B, time_ms(reps, [&] { hipLaunchKernelGGL((k_blocked<8, true>), dim3(nb), dim3(256), 0, 0, x, y, chunk); }));
  }
  rep("write-only", B, time_ms(reps, [&] { hipLaunchKernelGGL((k_fill<false>), dim3(cus * 8), dim3(256), 0, 0, y, n, 1.f); }));
  rep("write-only nt", B, time_ms(reps, [&] { hipLaunchKernelGGL((k_fill<true>), dim3(cus * 8), dim3(256), 0, 0, y, n, 1.f); }));
  rep("read-only", B, time_ms(reps, [&] { hipLaunchKernelGGL(k_read, dim3(cus * 8), dim3(256), 0, 0, x, n, out); }));
  rep("hipMemcpyAsync D2D", 2 * B, time_ms(reps, [&] { hipMemcpyAsync(y, x, bytes, hipMemcpyDeviceToDevice, 0); }));
  {
    const int V = 256, M = 4096, steps = 1000;  // 4 MiB slices, 1000 steps = 4 GiB
    const int g = (M / 64) * (V / 16);
    rep("scan P4", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan<4, false>), dim3(g), dim3(256), 0, 0, x, y, steps, V, M); }));
    rep("scan P4 nt", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan<4, true>), dim3(g), dim3(256), 0, 0, x, y, steps, V, M); }));
    rep("scan P8 nt", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan<8, true>), dim3(g), dim3(256), 0, 0, x, y, steps, V, M); }));
    rep("scan P16 nt", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan<16, true>), dim3(g), dim3(256), 0, 0, x, y, steps, V, M); }));
    rep("scan R2 P4", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan_r<4, 2, false>), dim3(g / 2), dim3(256), 0, 0, x, y, steps, V, M); }));
    rep("scan R2 P4 nt", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan_r<4, 2, true>), dim3(g / 2), dim3(256), 0, 0, x, y, steps, V, M); }));
    rep("scan R2 P8 nt", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan_r<8, 2, true>), dim3(g / 2), dim3(256), 0, 0, x, y, steps, V, M); }));
    rep("scan R4 P4 nt", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan_r<4, 4, true>), dim3(g / 4), dim3(256), 0, 0, x, y, steps, V, M); }));
    rep("scan16 P4 (strip, no reduce)", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan16<4, 4, false>), dim3(M / 16), dim3(1024), 0, 0, x, y, steps, V, M, out); }));
    rep("scan16 P4 G8 reduce", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan16<4, 8, true>), dim3(M / 16), dim3(1024), 0, 0, x, y, steps, V, M, out); }));
    rep("scan16 P2 G8 reduce", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan16<2, 8, true>), dim3(M / 16), dim3(1024), 0, 0, x, y, steps, V, M, out); }));
    rep("scan16 P8 G8 reduce", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan16<8, 8, true>), dim3(M / 16), dim3(1024), 0, 0, x, y, steps, V, M, out); }));
    rep("scan R1 P8", 2 * B * 1000 / 1024, time_ms(reps, [&] { hipLaunchKernelGGL((k_scan_r<8, 1, false>), dim3(g), dim3(256), 0, 0, x, y, steps, V, M); }));
  }
  return 0;
}
