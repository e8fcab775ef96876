// Read-only bond-scan shape sweep at the wide subnet's size (not part of the
// product; round 4). The history-less scan (k_bonds_elem R = 1, P = 4 on
// 64-miner tiles; c4: 256 x 65536 fp32 slices of 64 MiB, 100 epochs) reads
// W[t] once and writes only the per-(row, 64-miner tile) dividend partials.
// This walks the same footprints with a trivial recurrence to find the
// access pattern's own ceiling: block size BS, tile width CB columns (CB/4
// lanes per row), R rows per thread, P epochs of loads in flight, block order
// (0 column-block minor, 1 row-block minor), loads plain / non-temporal,
// partials none (dp0) / [t][tile][V] (dp1, the engine's DP_TV) / [tile][V][t]
// with 16 epochs gathered per 16-lane row before one 64-B store (dp7), 32
// epochs per two stores (dp8), the partials reduced but never stored (dp10),
// stored to an L2-resident 1 MiB buffer overwritten every epoch (dp11);
// RED 0 shuffle butterfly, 1 DPP row butterfly. dp12 / dp13: four 64-miner
// tiles summed per wave (CB = 256: one row per wave) and stored per epoch
// [t][quad][V] / gathered over 16 epochs [quad][V][t].
//   hipcc --offload-arch=gfx950 -O3 -o tools/scanrd tools/scanrd.hip && tools/scanrd
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float fvec4 __attribute__((ext_vector_type(4)));

template <int BS, int CB, int R, int P, bool NTL, int ORDER, int DP, int RED = 0>
__global__ __launch_bounds__(BS) void k_scanrd(const fvec4* __restrict__ x, int steps, int V, int M,
                                               float* out) {
  constexpr int LPR = CB / 4, G = BS / LPR;
  const int tiles = M / CB, rbs = V / (G * R);
  const int tile = ORDER == 0 ? blockIdx.x % tiles : blockIdx.x / rbs;
  const int rb = ORDER == 0 ? blockIdx.x / tiles : blockIdx.x % rbs;
  const int c = threadIdx.x % LPR, g = threadIdx.x / LPR;
  const long long m4 = M / 4, sl = (long long)V * m4;
  long long off[R];
#pragma unroll
  for (int i = 0; i < R; ++i) off[i] = (long long)(rb * G * R + g + G * i) * m4 + tile * LPR + c;
  auto ld = [&](long long o) { return NTL ? __builtin_nontemporal_load(x + o) : x[o]; };
  fvec4 ring[P][R], acc[R];
  float gath[R], gath2[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = fvec4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < P; ++k)
#pragma unroll
    for (int i = 0; i < R; ++i) ring[k][i] = ld(k * sl + off[i]);
  const int ep = (steps + 31) & ~31;
  for (int t0 = 0; t0 < steps; t0 += P) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int t = t0 + k;
      if (t >= steps) break;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        acc[i] = acc[i] * 0.5f + ring[k][i];
        if (DP) {
          float p = acc[i].x + acc[i].y + acc[i].z + acc[i].w;
          if (RED == 0) {
            for (int o = 1; o < 16; o <<= 1) p += __shfl_xor(p, o, 64);
          } else {
            p += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, p), 0xB1, 0xF, 0xF, false));
            p += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, p), 0x4E, 0xF, 0xF, false));
            p += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, p), 0x141, 0xF, 0xF, false));
            p += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, p), 0x140, 0xF, 0xF, false));
          }
          const int row = rb * G * R + g + G * i, st = (tile * CB + c * 4) / 64, tl = M / 64;
          if (DP == 1) {
            if ((threadIdx.x & 15) == 0) out[1 + ((long long)t * tl + st) * V + row] = p;
          } else if (DP == 7) {
            const int j = threadIdx.x & 15;
            if (j == (t & 15)) gath[i] = p;
            if ((t & 15) == 15 || t == steps - 1) {
              const int te = (t & ~15) + j;
              if (te <= t) out[32 + ((long long)st * V + row) * ep + te] = gath[i];
            }
          } else if (DP == 8) {
            const int j = threadIdx.x & 15;
            if (j == (t & 15)) {
              if (t & 16) gath2[i] = p;
              else gath[i] = p;
            }
            if ((t & 31) == 31 || t == steps - 1) {
              const int te = (t & ~31) + j;
              float* o = out + 32 + ((long long)st * V + row) * ep;
              if (te <= t) o[te] = gath[i];
              if (te + 16 <= t) o[te + 16] = gath2[i];
            }
          } else if (DP == 12 || DP == 13) {
            float q = p + __shfl_xor(p, 16, 64);
            q = q + __shfl_xor(q, 32, 64);
            const int quad = (tile * CB) / 256, nq = M / 256;
            if (DP == 12) {
              if ((threadIdx.x & 63) == 0) out[1 + ((long long)t * nq + quad) * V + row] = q;
            } else {
              const int j = threadIdx.x & 63;
              if (j == (t & 15)) gath[i] = q;
              if ((t & 15) == 15 || t == steps - 1) {
                const int te = (t & ~15) + j;
                if (j < 16 && te <= t) out[32 + ((long long)quad * V + row) * ep + te] = gath[i];
              }
            }
          } else if (DP == 10) {
            if ((threadIdx.x & 15) == 0 && p == 1234.5f) out[1 + ((long long)t * tl + st) * V + row] = p;
          } else if (DP == 11) {
            if ((threadIdx.x & 15) == 0) out[1 + ((long long)(st & 1023)) * V + row] = p;
          }
        }
        if (t + P < steps) ring[k][i] = ld((t + P) * sl + off[i]);
      }
    }
  }
  float d = 0.f;
#pragma unroll
  for (int i = 0; i < R; ++i) d += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
  if (d == 1234.5f) out[0] = d;
}

// the rowsum-like walk for comparison: one block per (epoch, row), the row
// read contiguously (no recurrence across epochs)
template <bool NTL>
__global__ __launch_bounds__(256) void k_rows(const fvec4* __restrict__ x, int M, float* out) {
  const long long base = (long long)blockIdx.x * (M / 4);
  float s = 0.f;
  for (int j = threadIdx.x; j < M / 4; j += 256) {
    const fvec4 v = NTL ? __builtin_nontemporal_load(x + base + j) : x[base + j];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;
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
  const int V = 256, M = 65536, steps = 100;
  const long long bytes = (long long)steps * V * M * 4;  // 100 slices of 64 MiB
  fvec4* x;
  float* out;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&out, 128 + 4ll * ((steps + 31) & ~31) * (M / 64) * V) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  (void)hipMemset(x, 0, bytes);
  const double moved = (double)bytes;
  const int reps = 5;
#define RUN(BS, CB, R, P, NTL, ORDER, DP, RED)                                                                         \
  {                                                                                                             \
    constexpr int G = BS / (CB / 4);                                                                            \
    const int blocks = (V / (G * R)) * (M / CB);                                                                \
    const float ms = time_ms(reps, [&] {                                                                        \
      hipLaunchKernelGGL((k_scanrd<BS, CB, R, P, NTL, ORDER, DP, RED>), dim3(blocks), dim3(BS), 0, 0, x, steps, V, M, \
                         out);                                                                                  \
    });                                                                                                         \
    printf("scanrd BS%-5d CB%-5d R%d P%d %-3s order%d dp%-2d red%d %6d blocks (%3d rows x %5d B)  %7.3f ms  %6.0f GB/s\n", \
           BS, CB, R, P, NTL ? "ntl" : "", ORDER, DP, RED, blocks, G * R, CB * 4, ms, moved / ms / 1e6);              \
    fflush(stdout);                                                                                             \
  }
  for (int rep2 = 0; rep2 < 2; ++rep2) {
    for (int ntl = 0; ntl < 2; ++ntl) {
      const float ms = time_ms(reps, [&] {
        if (ntl) hipLaunchKernelGGL(k_rows<true>, dim3(steps * V), dim3(256), 0, 0, x, M, out);
        else hipLaunchKernelGGL(k_rows<false>, dim3(steps * V), dim3(256), 0, 0, x, M, out);
      });
      printf("rows   one block per (epoch, row) %-3s                      %7.3f ms  %6.0f GB/s\n", ntl ? "ntl" : "", ms,
             moved / ms / 1e6);
    }
    RUN(256, 64, 1, 4, true, 0, 0, 1)
    RUN(256, 64, 1, 4, true, 0, 7, 1)   // the engine's DP_TE
    RUN(256, 256, 1, 4, true, 0, 0, 1)
    RUN(256, 256, 1, 4, true, 0, 10, 1)
    RUN(256, 256, 1, 4, true, 0, 12, 1)
    RUN(256, 256, 1, 4, true, 0, 13, 1)
    RUN(256, 256, 2, 4, true, 0, 13, 1)
    RUN(256, 256, 1, 6, true, 0, 13, 1)
    RUN(512, 256, 1, 4, true, 0, 13, 1)
  }
  return 0;
}
