// Bond-scan shape sweep (not part of the product; round 3). The bond scan
// (k_bonds_elem) walks 1000 epochs; each block reads its rows x columns of
// W[t] (4 MiB slice, 256 x 4096 fp32) and writes the same footprint of the
// bond history B_hist[t]. tools/hbmbw2 found 1024-thread blocks at one per CU
// copying at 5.7 TB/s against 5.3 for 256-thread blocks; this sweep tries the
// scan's footprint shapes: block size BS, tile width CB columns (CB/4 lanes
// per row), R rows per thread, P epochs of loads in flight, plain / nt stores.
//   hipcc --offload-arch=gfx950 -O3 -o tools/scanbw tools/scanbw.hip && tools/scanbw
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float fvec4 __attribute__((ext_vector_type(4)));

// DP: per-epoch dividend partials like the scan's: one fp32 per (row, 64-column
// sub-tile) from the 16 lanes of the sub-tile; 0 none, 1 stored [tile][V]
// (the engine's dpart layout), 2 stored [V][tile], 5 [column block][V][epoch]
// [sub-tile], 6 [epoch][column block][V][sub-tile]
template <int BS, int CB, int R, int P, bool NT, int DP = 0>
__global__ __launch_bounds__(BS) void k_scan(const fvec4* __restrict__ x, fvec4* __restrict__ y, int steps,
                                             int V, int M, float* out) {
  constexpr int LPR = CB / 4, G = BS / LPR;
  const int tiles = M / CB;
  int tile = blockIdx.x % tiles, rb = blockIdx.x / tiles;
  if (DP == 3 || DP == 4) {  // XCD-grouped: XCD x (= block % 8) owns a contiguous band of rows, every column block
    const int x = blockIdx.x & 7, k = blockIdx.x >> 3, per = gridDim.x >> 3;
    const int band = per / tiles;  // row blocks per XCD
    tile = k / band;
    rb = x * band + k % band;
  }
  const int c = threadIdx.x % LPR, g = threadIdx.x / LPR;
  const long long m4 = M / 4, sl = (long long)V * m4;
  long long off[R];
#pragma unroll
  for (int i = 0; i < R; ++i) off[i] = (long long)(rb * G * R + g + G * i) * m4 + tile * LPR + c;
  fvec4 ring[P][R], acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = fvec4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < P; ++k)
#pragma unroll
    for (int i = 0; i < R; ++i) ring[k][i] = x[k * sl + off[i]];
  float d = 0.f;
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
        d += acc[i].x;
        if (DP) {
          float p = acc[i].x + acc[i].y + acc[i].z + acc[i].w;
          for (int o = 1; o < 16; o <<= 1) p += __shfl_xor(p, o, 64);
          const int row = rb * G * R + g + G * i, st = (tile * CB + c * 4) / 64, tl = M / 64;
          if ((threadIdx.x & 15) == 0) {
            if (DP == 1 || DP == 3) out[1 + ((long long)t * tl + st) * V + row] = p;
            else if (DP == 5) {  // [column block][V][epoch][sub-tiles of the block]
              constexpr int TPB = CB / 64;
              out[1 + (((long long)tile * V + row) * steps + t) * TPB + (st % TPB)] = p;
            } else if (DP == 6) {  // [epoch][column block][V][sub-tiles of the block]
              constexpr int TPB = CB / 64;
              out[1 + (((long long)t * tiles + tile) * V + row) * TPB + (st % TPB)] = p;
            } else out[1 + ((long long)t * V + row) * tl + st] = p;
          }
        }
        if (t + P < steps) ring[k][i] = x[(t + P) * sl + off[i]];
      }
    }
  }
  if (d == 1234.5f) out[0] = d;
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

int main() {
  const int V = 256, M = 4096, steps = 1000;
  const long long bytes = 4096ll << 20;  // 1024 slices of 4 MiB
  fvec4 *x, *y;
  float* out;  // [0] sink, then dividend partials [1000][64][256]
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, bytes) != hipSuccess ||
      hipMalloc(&out, 4 + 4ll * 1000 * 64 * 256) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  (void)hipMemset(x, 0, bytes);
  (void)hipMemset(y, 0, bytes);
  const double moved = 2.0 * steps * (double)V * M * 4;
  const int reps = 5;
#define RUN(BS, CB, R, P, NT, DP)                                                                             \
  {                                                                                                           \
    constexpr int G = BS / (CB / 4);                                                                          \
    const int blocks = (V / (G * R)) * (M / CB);                                                              \
    const float ms = time_ms(reps, [&] {                                                                      \
      hipLaunchKernelGGL((k_scan<BS, CB, R, P, NT, DP>), dim3(blocks), dim3(BS), 0, 0, x, y, steps, V, M, out); \
    });                                                                                                       \
    printf("scan BS%-5d CB%-5d R%d P%d %-3s dp%d %5d blocks (%2d rows x %4d B)  %7.3f ms  %6.0f GB/s\n", BS, CB, R, \
           P, NT ? "nt" : "", DP, blocks, G * R, CB * 4, ms, moved / ms / 1e6);                               \
    fflush(stdout);                                                                                           \
  }
  for (int rep2 = 0; rep2 < 3; ++rep2) {
    RUN(512, 1024, 2, 2, true, 0)  // no partials
    RUN(512, 1024, 2, 2, true, 2)  // [epoch][V][sub-tile]: the engine's wide scan (round 3)
    RUN(512, 1024, 2, 2, true, 5)
    RUN(512, 1024, 2, 2, true, 6)
  }
  return 0;
}
