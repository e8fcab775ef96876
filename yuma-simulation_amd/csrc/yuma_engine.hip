// yuma_engine.hip — MI355X (gfx950) engine for the Yuma consensus epoch step.
//
// What it computes: the epoch step of the reference's five variants
// (src/yuma_simulation/_internal/yumas.py:61 YumaRust, :175 Yuma, :285 Yuma2,
// :399 Yuma3, :494 Yuma4) and the epoch loop of run_simulation
// (src/yuma_simulation/_internal/simulation_utils.py:26-112).
//
// How (DESIGN.md has the long form):
//  * Fact 1 of the survey: inside one epoch everything except the bond
//    recurrence is a pure function of (W_t, S_t). So phase 1 runs over ALL
//    epochs of a chunk at once (one slice = one (epoch, scenario) matrix):
//      k_rowsum     row sums of W + stake normalisation          (HBM pass 1)
//      k_consensus  per 64-miner tile: normalise, prerank, the
//                   kappa-bisection per column (LDS column reduce) (HBM pass 2)
//      k_quantise   per slice: sum C, int32 quantisation, liquid-alpha
//                   quantiles by integer histogram select, bond_alpha[m]
//      k_rank       per tile: clip, rank R, sum-R partials       (HBM pass 3)
//      k_incentive  per slice: I = nan_to_num(R / sum R)
//  * Phase 2 (k_bonds*) walks the epochs of the chunk per bond tile with the
//    bond state held in registers (fact 2: the recurrence is column-local),
//    reading W_t once more (HBM pass 4) and writing per-tile dividend partials.
//  * k_finalize turns the partials into D and D_normalized per slice.
// No float atomics, no data-dependent reduction order: every sum is a fixed
// tree, so results are bitwise reproducible run to run.
//
// Numerics follow the reference op by op in fp32 (torch CPU semantics): Python
// scalars are rounded to fp32 before they meet a tensor, `py / t` is
// reciprocal(t) * py, math.e ** t is pow(fp32(e), t), torch.quantile's lerp
// uses an FMA, torch.min / clamp propagate NaN, nan_to_num maps +-inf to
// +-FLT_MAX. Built with -ffp-contract=off and IEEE division so that no
// product is fused unless the reference fuses it.
#include <hip/hip_runtime.h>

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "yuma_hip.h"

#define YUMA_VERSION_STRING "yuma_hip 0.1.0 gfx950"
// the source identity the build stamps in (-DYUMA_BUILD_ID=...; yuma_build_id)
#ifndef YUMA_BUILD_ID
#define YUMA_BUILD_ID "unstamped"
#endif

// Kernel variants are A/B-tested from patched copies of this file
// (tools/ab_build.py), so the product source carries no build switches.

namespace yk {

constexpr int kTileM = 64;
// validators whose column a workgroup holds in registers / stages in LDS;
// above, the streaming paths (k_consensus_big, k_rank_sw<BIGV>, ...)
constexpr int kRegRows = YUMA_REG_VALIDATORS;
typedef float fvec4 __attribute__((ext_vector_type(4)));       // miner columns per tile: 16 lanes x float4
constexpr int kMaxTiles = 1 << 20;

// ---------------------------------------------------------------------------
// torch-CPU-faithful scalar helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float qnan() { return __builtin_nanf(""); }

// torch.minimum / torch.min(a, b) / clamp(max=b): NaN in -> NaN out.
__device__ __forceinline__ float tmin(float a, float b) {
  if (a != a || b != b) return qnan();
  return b < a ? b : a;
}
// torch.maximum / clamp(min=b): NaN in -> NaN out.
__device__ __forceinline__ float tmax(float a, float b) {
  if (a != a || b != b) return qnan();
  return b > a ? b : a;
}
// torch.minimum / torch.maximum in one instruction (gfx950 v_minimum3_f32 /
// v_maximum3_f32, NaN-propagating); unlike tmin/tmax they order -0 < +0,
// which no sum, product or comparison downstream can tell apart
__device__ __forceinline__ float vmin(float a, float b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ float vmax(float a, float b) { return __builtin_elementwise_maximum(a, b); }
// torch.nan_to_num(x, nan=nan_v): +-inf -> +-FLT_MAX.
__device__ __forceinline__ float nan_to_num(float x, float nan_v = 0.0f) {
  if (x != x) return nan_v;
  if (x == INFINITY) return FLT_MAX;
  if (x == -INFINITY) return -FLT_MAX;
  return x;
}

// Correctly rounded a / d for a per-row divisor d with its reciprocal r =
// RN(1/d) precomputed (one IEEE division per row instead of per element):
// q = RN(a r); e = fma(-d, q, a) (exact); q' = RN(q + e r) is RN(a/d)
// (Markstein) as long as nothing underflows or overflows. Guard: |d| and |a|
// in [2^-60, 2^60] (or a = +-0, where q already carries the right sign); any
// other operand takes the IEEE division. Checked bitwise against IEEE fp32
// division on 7.9e8 random pairs (tools/README: divtest).
struct RowDiv {
  float d, r;
  bool ok;
};
__device__ __forceinline__ RowDiv row_div(float d) {
  const float ad = fabsf(d);
  return {d, 1.0f / d, ad >= 0x1p-60f && ad <= 0x1p60f};
}
// Fast path only; `slow` is raised when an operand is outside the guard. The
// caller redoes the whole tile with IEEE division behind a wave-uniform
// branch (__any(slow)) so the rare path is never if-converted into the hot one.
__device__ __forceinline__ float div_fast(float a, const RowDiv& rd, bool& slow) {
  const float q = a * rd.r;
  const float e = fmaf(-rd.d, q, a);
  const float q1 = fmaf(e, rd.r, q);
  const float aa = fabsf(a);
  slow |= !(rd.ok && ((aa >= 0x1p-60f && aa <= 0x1p60f) || a == 0.0f));
  return a == 0.0f ? q : q1;
}
// div_fast without the signed-zero fix-up: a = -0 yields +0 instead of -0.
// For the consensus search and the rank sums only (a comparison with a
// positive grid point, min with C >= 0 times S, added to a +0-seeded sum
// cannot tell the two apart); saves a compare and a select per element.
__device__ __forceinline__ float div_fast_nz(float a, const RowDiv& rd, bool& slow) {
  const float q = a * rd.r;
  const float e = fmaf(-rd.d, q, a);
  const float aa = fabsf(a);
  slow |= !(rd.ok && ((aa >= 0x1p-60f && aa <= 0x1p60f) || a == 0.0f));
  return fmaf(e, rd.r, q);
}
// a / d exactly as IEEE: fast path, IEEE if outside the guard (used where a
// per-element branch is cheap: the rare paths themselves)
__device__ __forceinline__ float div_rn(float a, const RowDiv& rd) {
  bool slow = false;
  const float q = div_fast(a, rd, slow);
  return slow ? a / rd.d : q;
}

// Block barrier for an LDS hand-off only: waits for this wave's LDS traffic,
// not for its global loads (__syncthreads()' workgroup fence would wait for
// vmcnt(0), i.e. drain the loads in flight at every barrier).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// a quantised consensus level as C (yumas.py:211 `.int() / 65_535`)
__device__ __forceinline__ float level_value(int q) { return (float)q / 65535.0f; }

// Input slice of a slice (epoch t, scenario n) = t N + n: the slice itself,
// or epoch t when every scenario reads the same input trajectory (wsh: a
// parameter sweep over one subnet, yuma_run_shared).
__device__ __forceinline__ long long in_slice(long long slice, int N, int wsh) {
  return wsh ? slice / N : slice;
}

// Consensus classes of a shared-input run: with one input trajectory, the
// consensus, its quantisation and the rank of scenario n depend only on the
// parameters the search reads (κ, the bisection trip count, the histogram
// switch), so crep[n] = the first scenario with the same ones; the others
// take its results (bitwise the same computation). Every other parameter
// (bond α, liquid α, resets, ...) stays per scenario.
constexpr int kClassKeys = 4096;  // scenarios whose class keys fit in LDS (64 KiB)
// with_penalty: the key also holds bond_penalty (Yuma's rank pass forms the
// bond column sums Σ_v S·W_b, which depend on it)
__global__ __launch_bounds__(256) void k_classes(const yuma_params_t* __restrict__ prm, int N,
                                                 int* __restrict__ crep, int with_penalty) {
  if (N <= kClassKeys) {
    // the keys staged once per block: the first-match walk then reads LDS,
    // not one dependent 3-field global load per scenario (c3: 69 us per run)
    __shared__ uint4 key[kClassKeys];
    for (int j = threadIdx.x; j < N; j += 256) {
      const yuma_params_t& b = prm[j];
      key[j] = make_uint4(__float_as_uint(b.kappa), (unsigned)b.bisect_iters,
                          b.flags & YUMA_FLAG_NO_HIST, with_penalty ? __float_as_uint(b.bond_penalty) : 0u);
    }
    __syncthreads();
    for (int n = blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
      const uint4 a = key[n];
      int r = n;
      for (int j = 0; j < n; ++j) {
        const uint4 b = key[j];
        if (b.x == a.x && b.y == a.y && b.z == a.z && b.w == a.w) {
          r = j;
          break;
        }
      }
      crep[n] = r;
    }
    return;
  }
  for (int n = blockIdx.x * 256 + threadIdx.x; n < N; n += gridDim.x * 256) {
    const yuma_params_t& a = prm[n];
    const unsigned ka = __float_as_uint(a.kappa), ha = a.flags & YUMA_FLAG_NO_HIST;
    int r = n;
    for (int j = 0; j < n; ++j) {
      const yuma_params_t& b = prm[j];
      if (__float_as_uint(b.kappa) == ka && b.bisect_iters == a.bisect_iters &&
          (b.flags & YUMA_FLAG_NO_HIST) == ha &&
          (!with_penalty || __float_as_uint(b.bond_penalty) == __float_as_uint(a.bond_penalty))) {
        r = j;
        break;
      }
    }
    crep[n] = r;
  }
}
// The representatives of k_classes' classes in scenario order, compacted:
// clist[0] = the class count, clist[1 + j] = the j-th representative (one
// block; the multi-class consensus of a sweep walks this list)
__global__ __launch_bounds__(256) void k_class_list(const int* __restrict__ crep, int N, int* __restrict__ clist) {
  __shared__ int wc[4];
  __shared__ int base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  for (int n0 = 0; n0 < N; n0 += 256) {
    const int n = n0 + (int)threadIdx.x;
    const bool rep = n < N && crep[n] == n;
    const unsigned long long b = __ballot(rep);
    if (lane == 0) wc[wave] = __popcll(b);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wc[w];
    if (rep) clist[1 + off + __popcll(b & ((1ull << lane) - 1ull))] = n;
    __syncthreads();
    if (threadIdx.x == 0) base += wc[0] + wc[1] + wc[2] + wc[3];
    __syncthreads();
  }
  if (threadIdx.x == 0) clist[0] = base;
}
// is slice (t, n) computed by another scenario's block (crep[n] != n)?
__device__ __forceinline__ bool dup_slice(const int* crep, long long slice, int N) {
  if (crep == nullptr) return false;
  const int n = (int)(slice % N);
  return crep[n] != n;
}
// the slice whose consensus / rank results slice (t, n) takes
__device__ __forceinline__ long long rep_slice(const int* crep, long long slice, int N) {
  if (crep == nullptr) return slice;
  const int n = (int)(slice % N);
  return slice - n + crep[n];
}

// thread -> (row group g, column quad c4). A wave covers 4 row groups x 64
// columns, so one float4 load instruction moves 4 x 256 contiguous bytes.
struct Lay {
  int g, c4, lane, wave;
};
__device__ __forceinline__ Lay lay() {
  Lay L;
  L.lane = threadIdx.x & 63;
  L.wave = threadIdx.x >> 6;
  L.g = L.wave * 4 + (L.lane >> 4);
  L.c4 = L.lane & 15;
  return L;
}

// Sum over the 4 lanes of a wave that share a column quad (l, l^16, l^32,
// l^48). IEEE addition is commutative, so every lane ends with the same bits.
__device__ __forceinline__ float sum_rowgroups(float x) {
  x = x + __shfl_xor(x, 16, 64);
  x = x + __shfl_xor(x, 32, 64);
  return x;
}
// Sum over the 16 lanes of one row (the 64 columns of a tile row).
__device__ __forceinline__ float sum_row16(float x) {
  x = x + __shfl_xor(x, 1, 64);
  x = x + __shfl_xor(x, 2, 64);
  x = x + __shfl_xor(x, 4, 64);
  x = x + __shfl_xor(x, 8, 64);
  return x;
}
__device__ __forceinline__ float wave_sum(float x) {
  for (int o = 1; o < 64; o <<= 1) x = x + __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ double wave_sum_d(double x) {
  for (int o = 1; o < 64; o <<= 1) x = x + __shfl_xor(x, o, 64);
  return x;
}

// Column sums of a [rows x 64] tile: v holds this thread's partial sums for
// its 4 columns; on return every thread holds the full column sums. Order:
// thread-sequential rows, lane butterfly, then waves 0..NW-1 in order.
template <int NW>
__device__ __forceinline__ void col_reduce4(float (&v)[4], float4* red /*[NW*16]*/,
                                            const Lay& L) {
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = sum_rowgroups(v[c]);
  if (L.lane < 16) red[L.wave * 16 + L.c4] = make_float4(v[0], v[1], v[2], v[3]);
  __syncthreads();
  float4 a = red[L.c4];
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    const float4 b = red[w * 16 + L.c4];
    a.x = a.x + b.x;
    a.y = a.y + b.y;
    a.z = a.z + b.z;
    a.w = a.w + b.w;
  }
  v[0] = a.x;
  v[1] = a.y;
  v[2] = a.z;
  v[3] = a.w;
}

// Column max / min of a [rows x 64] tile (NaN-ignoring), same structure as col_reduce4.
template <int NW, bool MAX>
__device__ __forceinline__ void col_reduce4_ext(float (&v)[4], float4* red, const Lay& L) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float w = __shfl_xor(v[c], o, 64);
      v[c] = MAX ? (w > v[c] ? w : v[c]) : (w < v[c] ? w : v[c]);
    }
  }
  if (L.lane < 16) red[L.wave * 16 + L.c4] = make_float4(v[0], v[1], v[2], v[3]);
  __syncthreads();
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const float4 b = red[w * 16 + L.c4];
    const float bb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = MAX ? (bb[c] > v[c] ? bb[c] : v[c]) : (bb[c] < v[c] ? bb[c] : v[c]);
  }
}
template <int NW>
__device__ __forceinline__ void col_reduce4_max(float (&v)[4], float4* red, const Lay& L) {
  col_reduce4_ext<NW, true>(v, red, L);
}
template <int NW>
__device__ __forceinline__ void col_reduce4_min(float (&v)[4], float4* red, const Lay& L) {
  col_reduce4_ext<NW, false>(v, red, L);
}

template <bool VEC>
__device__ __forceinline__ void load4(const float* __restrict__ row, int m, int M, float (&x)[4]) {
  if (VEC) {
    if (m < M) {
      const float4 t = *reinterpret_cast<const float4*>(row + m);
      x[0] = t.x;
      x[1] = t.y;
      x[2] = t.z;
      x[3] = t.w;
    } else {
      x[0] = x[1] = x[2] = x[3] = 0.0f;
    }
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = (m + c < M) ? row[m + c] : 0.0f;
  }
}
// Branch-free loads: out-of-range rows / columns read a clamped in-range
// address and are zeroed afterwards, so a thread's loads issue back to back
// instead of one HBM round trip per (divergent) row. NTL: non-temporal loads
// (streaming reads of data no later access in the launch re-reads).
template <bool VEC, bool NTL = false>
__device__ __forceinline__ void load4c(const float* __restrict__ base, int row, int V, int m,
                                       int M, float (&x)[4]) {
  const int rr = row < V ? row : V - 1;
  const float* r = base + (long long)rr * M;
  if (VEC) {
    const int mm = m < M ? m : M - 4;
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 t = NTL ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(r + mm))
                     : *reinterpret_cast<const f4*>(r + mm);
    x[0] = t.x;
    x[1] = t.y;
    x[2] = t.z;
    x[3] = t.w;
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = NTL ? __builtin_nontemporal_load(r + min(m + c, M - 1)) : r[min(m + c, M - 1)];
  }
}
__device__ __forceinline__ void mask4(int row, int V, int m, int M, float (&x)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (row >= V || m + c >= M) x[c] = 0.0f;
}
__device__ __forceinline__ void vec4raw(const float* __restrict__ v, int m, int M, float (&x)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) x[c] = v[min(m + c, M - 1)];
}
__device__ __forceinline__ void vec4c(const float* __restrict__ v, int m, int M, float (&x)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float t = v[min(m + c, M - 1)];
    x[c] = m + c < M ? t : 0.0f;
  }
}

template <bool VEC>
__device__ __forceinline__ void store4(float* __restrict__ row, int m, int M, const float (&x)[4]) {
  if (VEC) {
    if (m < M) *reinterpret_cast<float4*>(row + m) = make_float4(x[0], x[1], x[2], x[3]);
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) row[m + c] = x[c];
  }
}
__device__ __forceinline__ void load4_vec(const float* __restrict__ v, int m, int M, float (&x)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) x[c] = (m + c < M) ? v[m + c] : 0.0f;
}

// ---------------------------------------------------------------------------
// Phase 1a: row sums (yumas.py:186 `W.sum(dim=1) + 1e-6`) and S / S.sum()
// (yumas.py:189). One wave per row. Block x: (slice, 4-row block).
// Summation order:
// the row is cut into 256-miner chunks; a chunk's partial is the balanced
// binary tree over its 64 column quads of the sequential quad sums
// ((x0+x1)+x2)+x3 (lane l holds quad l: the 64-lane butterfly); the chunk
// partials are added in chunk order. W is read with non-temporal loads: no
// later access in the launch re-reads it (c2 0.687 -> 0.636 ms, c4 1.09 ->
// 0.96, same box; the same loads in the consensus kernel lose, 0.87 -> 1.02:
// there the two halves of a 128-byte line go to neighbouring waves).
// ---------------------------------------------------------------------------
// WIDE (rows of >= kWideChunks chunks, e.g. a 65536-miner subnet): block =
// ONE row, its chunks dealt to the 4 waves, the chunk partials parked in LDS
// and added in chunk order by one lane — the same bits, and 4x the blocks
// (one long wave per row leaves the last of ~3 dispatch rounds mostly idle).
constexpr int kWideChunks = 64, kMaxWideChunks = 4096;
// RN(1 / rs) when div_fast of every weight of the row by rs takes its fast
// path (|rs| and every nonzero |w| in [2^-60, 2^60]; bmax / bmin1: the row's
// max |w| and min nonzero |w| - 1 as bit patterns), else NaN: the sweep
// scan then divides without a per-row reciprocal or a per-element guard
// (k_bonds_grp; the memory-bound scans lost with it, k_bonds_elem). k_rowsum
// stores it per INPUT slice and row as rq4 = {row sum, this, normalised stake,
// 1 if some weight of the row is negative else 0}.
__device__ __forceinline__ bool screen_ok(unsigned bmax, unsigned bmin1) {
  return bmax <= __float_as_uint(0x1p60f) && (bmin1 == 0xFFFFFFFFu || bmin1 + 1u >= __float_as_uint(0x1p-60f));
}
__device__ __forceinline__ float fast_row_rcp(float rs, unsigned bmax, unsigned bmin1) {
  const float ad = fabsf(rs);
  return ad >= 0x1p-60f && ad <= 0x1p60f && screen_ok(bmax, bmin1) ? 1.0f / rs : qnan();
}

template <bool VEC, bool WIDE = false>
__global__ __launch_bounds__(256) void k_rowsum(const float* __restrict__ W,
                                                const float* __restrict__ S, int V, int M,
                                                long long islice0, int rowblocks,
                                                float* __restrict__ rsd, float* __restrict__ sn,
                                                int partial, int* __restrict__ sx, int fan,
                                                float4* __restrict__ rq4) {
  // Block = 4 rows (WIDE: one row) of input slice wsl. Its row sums and
  // normalised stakes belong to output slices wsl·fan .. wsl·fan + fan - 1:
  // fan = 1, or N with shared inputs (they do not depend on the scenario:
  // computed once, stored for every scenario).
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long wsl = islice0 + blockIdx.x / rowblocks;
  const int rb = blockIdx.x % rowblocks;
  // the fast-division screen of the row (rq4): max |w| and min nonzero |w|
  // as bit patterns (|w| = 0 wraps to the maximum of bmin1)
  // bneg: some weight of the row is below -0 (sign bit set, not -0; a
  // negative-signed NaN counts), rq4.w = 1: the sweep scan's bounded Yuma 4
  // update needs non-negative weights (k_bonds_grp)
  unsigned bmax = 0u, bmin1 = 0xFFFFFFFFu, bneg = 0u;
  auto screen = [&](const float (&x)[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned b = __float_as_uint(x[c]) & 0x7FFFFFFFu;
      bmax = b > bmax ? b : bmax;
      bmin1 = b - 1u < bmin1 ? b - 1u : bmin1;
      bneg |= __float_as_uint(x[c]) > 0x80000000u ? 1u : 0u;
    }
  };
  if constexpr (WIDE) {
    __shared__ float qs[kMaxWideChunks];
    __shared__ unsigned qb[3][4];
    const int nc = (M + 255) / 256;
    const float* r = W + (wsl * V + rb) * (long long)M;
#pragma unroll 4
    for (int k = wave; k < nc; k += 4) {
      const int m = k * 256 + lane * 4;
      float x[4];
      if (VEC) {
        if (m < M) {
          const fvec4 t = __builtin_nontemporal_load(reinterpret_cast<const fvec4*>(r + m));
          x[0] = t.x;
          x[1] = t.y;
          x[2] = t.z;
          x[3] = t.w;
        } else {
          x[0] = x[1] = x[2] = x[3] = 0.0f;
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) x[c] = m + c < M ? r[m + c] : 0.0f;
      }
      const float q = wave_sum(((x[0] + x[1]) + x[2]) + x[3]);
      if (lane == 0) qs[k] = q;
      screen(x);
    }
    for (int o = 1; o < 64; o <<= 1) {
      bmax = max(bmax, (unsigned)__shfl_xor((int)bmax, o, 64));
      bmin1 = min(bmin1, (unsigned)__shfl_xor((int)bmin1, o, 64));
      bneg |= (unsigned)__shfl_xor((int)bneg, o, 64);
    }
    if (lane == 0) {
      qb[0][wave] = bmax;
      qb[1][wave] = bmin1;
      qb[2][wave] = bneg;
    }
    __syncthreads();
    if (wave == 0) {
      float acc = 0.0f;
      if (lane == 0)
        for (int k = 0; k < nc; ++k) acc = acc + qs[k];
      acc = __shfl(acc, 0, 64);
      const float rs = partial ? acc : acc + 1e-6f;
      for (int f = lane; f < fan; f += 64) rsd[(wsl * fan + f) * V + rb] = rs;
      if (rq4 != nullptr && lane == 0) {
        unsigned bx = qb[0][0], bn = qb[1][0], ng = qb[2][0];
        for (int w = 1; w < 4; ++w) {
          bx = max(bx, qb[0][w]);
          bn = min(bn, qb[1][w]);
          ng |= qb[2][w];
        }
        *reinterpret_cast<float2*>(&rq4[wsl * V + rb]) = make_float2(rs, fast_row_rcp(rs, bx, bn));
        reinterpret_cast<float*>(&rq4[wsl * V + rb])[3] = ng ? 1.0f : 0.0f;
      }
    }
  }
  const int row = rb * 4 + wave;
  if (!WIDE && row < V) {
    const float* r = W + (wsl * V + row) * (long long)M;
    float acc = 0.0f;
#pragma unroll 4
    for (int m0 = 0; m0 < M; m0 += 256) {
      const int m = m0 + lane * 4;
      float x[4];
      if (VEC) {
        if (m < M) {
          const fvec4 t = __builtin_nontemporal_load(reinterpret_cast<const fvec4*>(r + m));
          x[0] = t.x;
          x[1] = t.y;
          x[2] = t.z;
          x[3] = t.w;
        } else {
          x[0] = x[1] = x[2] = x[3] = 0.0f;
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) x[c] = m + c < M ? r[m + c] : 0.0f;
      }
      float q = ((x[0] + x[1]) + x[2]) + x[3];
      q = wave_sum(q);  // the balanced tree over the chunk's 64 quads
      acc = acc + q;
      screen(x);
    }
    // partial (column shard): the caller sums the shards, then k_add_eps
    const float rs = partial ? acc : acc + 1e-6f;
    for (int f = lane; f < fan; f += 64) rsd[(wsl * fan + f) * V + row] = rs;
    if (rq4 != nullptr) {
      for (int o = 1; o < 64; o <<= 1) {
        bmax = max(bmax, (unsigned)__shfl_xor((int)bmax, o, 64));
        bmin1 = min(bmin1, (unsigned)__shfl_xor((int)bmin1, o, 64));
        bneg |= (unsigned)__shfl_xor((int)bneg, o, 64);
      }
      if (lane == 0) {
        *reinterpret_cast<float2*>(&rq4[wsl * V + row]) = make_float2(rs, fast_row_rcp(rs, bmax, bmin1));
        reinterpret_cast<float*>(&rq4[wsl * V + row])[3] = bneg ? 1.0f : 0.0f;
      }
    }
  }
  // the stake normalisation: output slices f = rb, rb + rowblocks, ... of
  // the fan (block 0 alone when fan = 1)
  if (rb < fan && wave == 0) {
    const float* s = S + wsl * V;
    float acc = 0.0f;
    for (int v = lane; v < V; v += 64) acc = acc + s[v];
    acc = wave_sum(acc);
    // sx[slice]: the normalised stakes in units of 2^-24 when every one is
    // such a multiple and they total <= 1 (subset sums exact in fp32: the
    // consensus search's histogram finish), else -1
    int units = 0;
    bool exact = true;
    for (int v = lane; v < V; v += 64) {
      const float q = s[v] / acc;
      for (int f = rb; f < fan; f += rowblocks) sn[(wsl * fan + f) * V + v] = q;
      if (rq4 != nullptr && rb == 0) reinterpret_cast<float*>(&rq4[wsl * V + v])[2] = q;
      const float f = q * 16777216.0f;
      exact &= f >= 0.0f && f <= 16777216.0f && __builtin_amdgcn_fractf(f) == 0.0f;
      units += exact ? (int)f : 0;
    }
    for (int o = 1; o < 64; o <<= 1) units += __shfl_xor(units, o, 64);
    exact = __all(exact) && units <= (1 << 24);
    if (lane == 0)
      for (int f = rb; f < fan; f += rowblocks) sx[wsl * fan + f] = exact ? units : -1;
  }
}

// ---------------------------------------------------------------------------
// Phase 1b: consensus bisection (yumas.py:195-209, YumaRust :81-95) + prerank
// P = sum_v S W (yumas.py:192). Block = one 64-miner tile of one slice, the
// whole validator column resident in registers (R rows per thread).
// Per iteration: mid in double exactly as the reference, compared as fp32
// (torch casts the python scalar), masked stake sums reduced in a fixed tree.
// ---------------------------------------------------------------------------
template <int NT, int R, bool VEC>
__global__ __launch_bounds__(NT) void k_consensus(const float* __restrict__ W,
                                                  const float* __restrict__ rsd,
                                                  const float* __restrict__ sn,
                                                  const yuma_params_t* __restrict__ prm, int N,
                                                  int V, int M, long long slice0, int tiles,
                                                  double* __restrict__ craw,
                                                  float* __restrict__ Pout, int wsh,
                                                  const int* __restrict__ crep) {
  constexpr int NW = NT / 64, G = NT / 16;
  __shared__ float4 red[2][NW * 16];
  const Lay L = lay();
  const long long slice = slice0 + blockIdx.x / tiles;
  const int tile = blockIdx.x % tiles;
  const int n = (int)(slice % N);
  if (dup_slice(crep, slice, N)) return;  // block-uniform
  const int m = tile * kTileM + L.c4 * 4;
  const float* Ws = W + in_slice(slice, N, wsh) * (long long)V * M;

  float wn[R][4], s[R], d[R];
#pragma unroll
  for (int i = 0; i < R; ++i) load4c<VEC>(Ws, L.g + G * i, V, m, M, wn[i]);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int rr = min(L.g + G * i, V - 1);
    d[i] = rsd[slice * V + rr];
    s[i] = sn[slice * V + rr];
  }
  {
    bool slow = false;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const RowDiv rdv = row_div(d[i]);
#pragma unroll
      for (int c = 0; c < 4; ++c) wn[i][c] = div_fast(wn[i][c], rdv, slow);
    }
    if (__any(slow)) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        load4c<VEC>(Ws, L.g + G * i, V, m, M, wn[i]);
#pragma unroll
        for (int c = 0; c < 4; ++c) wn[i][c] = wn[i][c] / d[i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    mask4(L.g + G * i, V, m, M, wn[i]);
    if (L.g + G * i >= V) s[i] = 0.0f;
  }

  if (Pout != nullptr) {
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = acc[c] + s[i] * wn[i][c];
    col_reduce4<NW>(acc, red[1], L);
    if (L.g == 0)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (m + c < M) Pout[slice * M + m + c] = acc[c];
    __syncthreads();
  }

  const float kappa = prm[n].kappa;
  const int iters = prm[n].bisect_iters;  // host guarantees <= 30
  // The reference bisection (yumas.py:201-207) on the grid k 2^-n: mid is
  // (hi + lo) / 2 in double, i.e. the integer midpoint (L + H) / 2, compared
  // as fp32 (float)(mid) = (float)k * 2^-n. F(k) = sum_v float(W > mid) * S.
  // When every stake is finite and >= 0 (and kappa >= 0), F is monotone in k
  // and the result is k* = min{k in [1, 2^n] : F(k) <= kappa} (2^n if none), so
  // the search may start from a per-column bracket instead of [0, 2^n]:
  //   F(k) = 0 <= kappa      for k >= gmax = ceil(max Wn 2^n)
  //   F(k) = sum S (all set) for k <  gmin = ceil(min Wn 2^n)
  // Both searches keep (L == 0 or F(L) > kappa) && (H == 2^n or F(H) <= kappa),
  // so they end at the same k*; every F uses the same fixed-order reduction.
  bool odd_stake = false;
#pragma unroll
  for (int i = 0; i < R; ++i) odd_stake |= !(s[i] >= 0.0f) || s[i] == INFINITY;
  const bool bracket = !__syncthreads_or(odd_stake) && kappa >= 0.0f;
  const int top = 1 << iters;
  const float scale = (float)top, inv_scale = 1.0f / scale;
  int lo_k[4], hi_k[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    lo_k[c] = 0;
    hi_k[c] = top;
  }
  if (bracket) {
    float vmax[4], vmin[4], stot[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      vmax[c] = -INFINITY;
      vmin[c] = INFINITY;
      stot[c] = 0.0f;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (L.g + G * i >= V) continue;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float x = wn[i][c];
        vmax[c] = x > vmax[c] ? x : vmax[c];  // a NaN weight is never counted
        const float xm = x == x ? x : 0.0f;   // ... so it acts like a zero weight
        vmin[c] = xm < vmin[c] ? xm : vmin[c];
        stot[c] = stot[c] + s[i];
      }
    }
    col_reduce4_max<NW>(vmax, red[0], L);
    __syncthreads();
    col_reduce4_min<NW>(vmin, red[1], L);
    __syncthreads();
    col_reduce4<NW>(stot, red[0], L);  // == F(k) with every mask set
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int gmax = vmax[c] > 0.0f ? (int)fminf(ceilf(vmax[c] * scale), scale) : 0;
      const int gmin = vmin[c] > 0.0f ? (int)fminf(ceilf(vmin[c] * scale), scale + 1.0f) : 0;
      int lo_c = gmin >= 2 ? gmin - 1 : 0;
      int hi_c = gmax < 1 ? 1 : gmax;
      if (lo_c > 0 && !(stot[c] > kappa)) {  // F <= kappa everywhere: k* = 1
        lo_c = 0;
        hi_c = 1;
      }
      if (lo_c >= top) {  // all weights above 1: F(k) = sum S > kappa for every k < 2^n
        lo_c = top - 1;
        hi_c = top;
      }
      if (hi_c <= lo_c) hi_c = lo_c + 1;  // unreachable guard
      lo_k[c] = lo_c;
      hi_k[c] = hi_c;
    }
  }
  for (int it = 0;; ++it) {
    bool active = false;
#pragma unroll
    for (int c = 0; c < 4; ++c) active |= (hi_k[c] - lo_k[c]) > 1;
    if (!__syncthreads_or(active)) break;
    float part[4];
    int mid[4];
    float midf[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      mid[c] = (lo_k[c] + hi_k[c]) >> 1;
      midf[c] = (float)mid[c] * inv_scale;
      part[c] = 0.0f;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float zs = 0.0f * s[i];
#pragma unroll
      for (int c = 0; c < 4; ++c) part[c] = part[c] + ((wn[i][c] > midf[c]) ? s[i] : zs);
    }
    col_reduce4<NW>(part, red[it & 1], L);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (hi_k[c] - lo_k[c] > 1) {
        if (part[c] > kappa)
          lo_k[c] = mid[c];
        else
          hi_k[c] = mid[c];
      }
    }
  }
  double hi[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) hi[c] = (double)hi_k[c] / (double)top;
  if (L.g == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) craw[slice * M + m + c] = hi[c];
}

// Consensus above YUMA_REG_VALIDATORS validators: the column no longer fits a
// workgroup's registers, so every pass of the search streams the 64-miner
// tile's rows from memory (the normalised weights recomputed per pass with
// IEEE division, as k_consensus). Pass 0: prerank, bracket (k_consensus'
// rules); then the bisection on the grid k 2^-iters. Order of every sum:
// thread-sequential rows g + 16 i, the 4 row groups of a wave, waves in order.
template <bool VEC>
__global__ __launch_bounds__(256) void k_consensus_big(const float* __restrict__ W,
                                                      const float* __restrict__ rsd,
                                                      const float* __restrict__ sn,
                                                      const yuma_params_t* __restrict__ prm, int N,
                                                      int V, int M, long long slice0, int tiles,
                                                      double* __restrict__ craw,
                                                      float* __restrict__ Pout, int wsh,
                                                      const int* __restrict__ crep) {
  constexpr int NW = 4, G = 16;
  __shared__ float4 red[2][NW * 16];
  const Lay L = lay();
  const long long slice = slice0 + blockIdx.x / tiles;
  const int tile = blockIdx.x % tiles;
  const int n = (int)(slice % N);
  if (dup_slice(crep, slice, N)) return;  // block-uniform
  const int m = tile * kTileM + L.c4 * 4;
  const float* Ws = W + in_slice(slice, N, wsh) * (long long)V * M;
  const float* rs = rsd + slice * V;
  const float* ss = sn + slice * V;
  // row `row`'s normalised weights of this lane's 4 columns (0 outside) and stake
  auto row_w = [&](int row, float (&x)[4]) -> float {
    load4c<VEC>(Ws, row, V, m, M, x);
    const int rr = row < V ? row : V - 1;
    const RowDiv rdv = row_div(rs[rr]);
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = div_rn(x[c], rdv);
    mask4(row, V, m, M, x);
    return row < V ? ss[rr] : 0.0f;
  };
  const float kappa = prm[n].kappa;
  const int iters = prm[n].bisect_iters;
  const int top = 1 << iters;
  const float scale = (float)top, inv_scale = 1.0f / scale;
  float pacc[4] = {0.0f, 0.0f, 0.0f, 0.0f}, vmax[4], vmin[4], stot[4];
  bool odd_stake = false;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    vmax[c] = -INFINITY;
    vmin[c] = INFINITY;
    stot[c] = 0.0f;
  }
  for (int row = L.g; row < V; row += G) {
    float x[4];
    const float s = row_w(row, x);
    odd_stake |= !(s >= 0.0f) || s == INFINITY;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      pacc[c] = pacc[c] + s * x[c];
      vmax[c] = x[c] > vmax[c] ? x[c] : vmax[c];  // a NaN weight is never counted
      const float xm = x[c] == x[c] ? x[c] : 0.0f;
      vmin[c] = xm < vmin[c] ? xm : vmin[c];
      stot[c] = stot[c] + s;
    }
  }
  if (Pout != nullptr) {
    col_reduce4<NW>(pacc, red[1], L);
    if (L.g == 0)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (m + c < M) Pout[slice * M + m + c] = pacc[c];
    __syncthreads();
  }
  const bool bracket = !__syncthreads_or(odd_stake) && kappa >= 0.0f;
  int lo_k[4], hi_k[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    lo_k[c] = 0;
    hi_k[c] = top;
  }
  if (bracket) {
    col_reduce4_max<NW>(vmax, red[0], L);
    __syncthreads();
    col_reduce4_min<NW>(vmin, red[1], L);
    __syncthreads();
    col_reduce4<NW>(stot, red[0], L);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int gmax = vmax[c] > 0.0f ? (int)fminf(ceilf(vmax[c] * scale), scale) : 0;
      const int gmin = vmin[c] > 0.0f ? (int)fminf(ceilf(vmin[c] * scale), scale + 1.0f) : 0;
      int lo_c = gmin >= 2 ? gmin - 1 : 0;
      int hi_c = gmax < 1 ? 1 : gmax;
      if (lo_c > 0 && !(stot[c] > kappa)) {
        lo_c = 0;
        hi_c = 1;
      }
      if (lo_c >= top) {
        lo_c = top - 1;
        hi_c = top;
      }
      if (hi_c <= lo_c) hi_c = lo_c + 1;
      lo_k[c] = lo_c;
      hi_k[c] = hi_c;
    }
  }
  for (int it = 0;; ++it) {
    bool active = false;
#pragma unroll
    for (int c = 0; c < 4; ++c) active |= (hi_k[c] - lo_k[c]) > 1;
    if (!__syncthreads_or(active)) break;
    float part[4], midf[4];
    int mid[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      mid[c] = (lo_k[c] + hi_k[c]) >> 1;
      midf[c] = (float)mid[c] * inv_scale;
      part[c] = 0.0f;
    }
    for (int row = L.g; row < V; row += G) {
      float x[4];
      const float s = row_w(row, x);
      const float zs = 0.0f * s;
#pragma unroll
      for (int c = 0; c < 4; ++c) part[c] = part[c] + ((x[c] > midf[c]) ? s : zs);
    }
    col_reduce4<NW>(part, red[it & 1], L);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (hi_k[c] - lo_k[c] > 1) {
        if (part[c] > kappa)
          lo_k[c] = mid[c];
        else
          hi_k[c] = mid[c];
      }
    }
  }
  if (L.g == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) craw[slice * M + m + c] = (double)hi_k[c] / (double)top;
}

// ---------------------------------------------------------------------------
// Wave-owned columns: a 64-miner tile per block, 16 miners per wave, every
// validator row of those miners in the wave's registers. Lane l owns the row
// group rg = l & 15 (rows rg + 16 i) and the column quad cq = l >> 4, so the
// 16 row groups of a column quad are the 16 lanes of one DPP row: column
// reductions are 4 DPP-modified adds (no LDS, no barriers), and each wave runs
// its own search loop.
// ---------------------------------------------------------------------------
struct WLay {
  int lane, wave, cq, rg;
};
__device__ __forceinline__ WLay wlay() {
  WLay L;
  L.lane = threadIdx.x & 63;
  L.wave = threadIdx.x >> 6;
  L.cq = L.lane >> 4;
  L.rg = L.lane & 15;
  return L;
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
// Reduction over the 16 lanes of a DPP row by pairwise exchanges (quad_perm
// [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror): every step
// pairs lane i with a partner that pairs back, and a + b == b + a bitwise, so
// all 16 lanes end with identical bits.
__device__ __forceinline__ float wsum16(float x) {
  x = x + dpp_f<0xB1>(x);
  x = x + dpp_f<0x4E>(x);
  x = x + dpp_f<0x141>(x);
  x = x + dpp_f<0x140>(x);
  return x;
}
// NaN-free inputs only (callers exclude NaN before reducing)
__device__ __forceinline__ float wmax16(float x) {
  x = fmaxf(x, dpp_f<0xB1>(x));
  x = fmaxf(x, dpp_f<0x4E>(x));
  x = fmaxf(x, dpp_f<0x141>(x));
  x = fmaxf(x, dpp_f<0x140>(x));
  return x;
}
__device__ __forceinline__ float wmin16(float x) {
  x = fminf(x, dpp_f<0xB1>(x));
  x = fminf(x, dpp_f<0x4E>(x));
  x = fminf(x, dpp_f<0x141>(x));
  x = fminf(x, dpp_f<0x140>(x));
  return x;
}
// Integer sum over the 16 lanes of a DPP row (exact, so any order).
__device__ __forceinline__ int iwsum16(int x) {
  x = x + __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);
  x = x + __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);
  x = x + __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false);
  x = x + __builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, false);
  return x;
}
__device__ __forceinline__ int iwmax16(int x) {
  x = max(x, __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, false));
  return x;
}
__device__ __forceinline__ int iwmin16(int x) {
  x = min(x, __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, false));
  return x;
}
// Exclusive prefix sum over the 16 lanes of a DPP row (row_shr:1,2,4,8 with
// bound_ctrl: lanes shifted in from outside the row read 0).
__device__ __forceinline__ int iscan16_excl(int x) {
  int y = x;
  y = y + __builtin_amdgcn_update_dpp(0, y, 0x111, 0xF, 0xF, true);
  y = y + __builtin_amdgcn_update_dpp(0, y, 0x112, 0xF, 0xF, true);
  y = y + __builtin_amdgcn_update_dpp(0, y, 0x114, 0xF, 0xF, true);
  y = y + __builtin_amdgcn_update_dpp(0, y, 0x118, 0xF, 0xF, true);
  return y - x;
}
// sum over the 4 column quads of a wave (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float qsum4(float x) {
  x = x + __shfl_xor(x, 16, 64);
  x = x + __shfl_xor(x, 32, 64);
  return x;
}

// Load + normalise this lane's R rows x 4 miners of a slice (branch-free).
template <int R, bool VEC>
__device__ __forceinline__ void load_norm_w(const float* __restrict__ Ws, const float* rsd_s,
                                            const float* sn_s, int V, int M, int m, int rg,
                                            float (&wn)[R][4], float (&s)[R]) {
  float d[R];
  // padding rows / columns exist only in edge tiles (wave-uniform test)
  const bool full = rg + 16 * (R - 1) < V && m + 3 < M;
  const bool allfull = VEC && __all(full) && (long long)V * M < (1ll << 30);
  if (allfull) {
    // 32-bit element offsets from the uniform slice base (saddr + voffset
    // loads, one add per row instead of a 64-bit address per row)
    const unsigned o0 = (unsigned)rg * (unsigned)M + (unsigned)m, st = 16u * (unsigned)M;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float4 t = *reinterpret_cast<const float4*>(Ws + (o0 + (unsigned)i * st));
      wn[i][0] = t.x;
      wn[i][1] = t.y;
      wn[i][2] = t.z;
      wn[i][3] = t.w;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      d[i] = rsd_s[rg + 16 * i];
      s[i] = sn_s[rg + 16 * i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) load4c<VEC>(Ws, rg + 16 * i, V, m, M, wn[i]);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int rr = min(rg + 16 * i, V - 1);
      d[i] = rsd_s[rr];
      s[i] = sn_s[rr];
    }
  }
  bool slow = false;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const RowDiv rdv = row_div(d[i]);
#pragma unroll
    for (int c = 0; c < 4; ++c) wn[i][c] = div_fast(wn[i][c], rdv, slow);
  }
  if (__any(slow)) {  // rare: some operand outside the fast-division guard
#pragma unroll
    for (int i = 0; i < R; ++i) {
      load4c<VEC>(Ws, rg + 16 * i, V, m, M, wn[i]);
#pragma unroll
      for (int c = 0; c < 4; ++c) wn[i][c] = wn[i][c] / d[i];
    }
  }
  if (!__all(full)) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      mask4(rg + 16 * i, V, m, M, wn[i]);
      if (rg + 16 * i >= V) s[i] = 0.0f;
    }
  }
}

// The consensus kernel's load + normalise. The wave's row sums, stakes and row
// reciprocals are staged in a wave-private LDS copy `rl` ([16 R] row sums,
// [16 R] stakes with 0 on padding rows, [16 R] RN(1 / row sum)) instead of
// 2 x R VGPRs per lane (166 -> 127 VGPRs, 4 waves / SIMD): the row-sum / stake
// loads go out first, the W loads behind them, and the copy is written while
// W is in flight. Each IEEE reciprocal is computed once per wave (by the lane
// that stages the row) instead of once per column quad.
// Division: div_fast_nz's sequence (q = a·r, e = fma(-d, q, a), q + e·r) on
// packed pairs (v_pk_mul / v_pk_fma: two lanes' worth of fp32 per
// instruction), with the operand guard reduced to a lane-wide max |a| (NaN-
// ignoring: the fast path returns the same quiet NaN as IEEE division) and a
// min over nonzero |a| taken on 2·bits(|a|) - 1 (zeros wrap to the maximum),
// instead of three compares per element; no signed-zero fix-up (consensus
// only compares normalised weights against grid points >= 0).
template <int R, bool VEC>
__device__ __forceinline__ void load_norm_w_lds(const float* __restrict__ Ws, const float* rsd_s,
                                                const float* sn_s, float* rl, int V, int M, int m,
                                                int rg, int lane, float (&wn)[R][4]) {
  constexpr int NR = 16 * R, PL = (NR + 63) / 64;
  float dv[PL], sv[PL];
#pragma unroll
  for (int k = 0; k < PL; ++k) {
    const int jj = min(lane + 64 * k, V - 1);
    dv[k] = rsd_s[jj];
    sv[k] = sn_s[jj];
  }
  const bool full = rg + 16 * (R - 1) < V && m + 3 < M;
  const bool allfull = VEC && __all(full) && (long long)V * M < (1ll << 30);
  if (allfull) {
    const unsigned o0 = (unsigned)rg * (unsigned)M + (unsigned)m, st = 16u * (unsigned)M;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float4 t = *reinterpret_cast<const float4*>(Ws + (o0 + (unsigned)i * st));
      wn[i][0] = t.x;
      wn[i][1] = t.y;
      wn[i][2] = t.z;
      wn[i][3] = t.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) load4c<VEC>(Ws, rg + 16 * i, V, m, M, wn[i]);
  }
  // the division guard's row-sum part over the staged rows (the guard is
  // wave-wide: __any below)
  float amax = 0.0f, dmin = INFINITY;
#pragma unroll
  for (int k = 0; k < PL; ++k) {
    const int j = lane + 64 * k;
    amax = fmaxf(amax, fabsf(dv[k]));
    dmin = fminf(dmin, fabsf(dv[k]));
    if (j < NR) {
      rl[j] = dv[k];
      rl[NR + j] = j < V ? sv[k] : 0.0f;
      rl[2 * NR + j] = 1.0f / dv[k];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // packed division, row sums and reciprocals from LDS
  typedef float f2 __attribute__((ext_vector_type(2)));
  unsigned ymin = 0xFFFFFFFFu;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const float d = rl[rg + 16 * i];
    const float r = rl[2 * NR + rg + 16 * i];
    const f2 r2 = {r, r}, nd2 = {-d, -d};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f2 a2 = {wn[i][2 * h], wn[i][2 * h + 1]};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        amax = fmaxf(amax, fabsf(a2[c]));
        const unsigned y = (__float_as_uint(a2[c]) << 1) - 1u;
        ymin = y < ymin ? y : ymin;
      }
      const f2 q = a2 * r2;
      const f2 e = __builtin_elementwise_fma(nd2, q, a2);
      const f2 q1 = __builtin_elementwise_fma(e, r2, q);
      wn[i][2 * h] = q1[0];
      wn[i][2 * h + 1] = q1[1];
    }
  }
  const bool slow = !(dmin >= 0x1p-60f && amax <= 0x1p60f &&
                      (ymin == 0xFFFFFFFFu || ymin + 1u >= (__float_as_uint(0x1p-60f) << 1)));
  if (__any(slow)) {  // rare: some operand outside the fast-division guard
#pragma unroll
    for (int i = 0; i < R; ++i) {
      load4c<VEC>(Ws, rg + 16 * i, V, m, M, wn[i]);
      const float d = rl[rg + 16 * i];
#pragma unroll
      for (int c = 0; c < 4; ++c) wn[i][c] = wn[i][c] / d;
    }
  }
  if (!__all(full)) {
#pragma unroll
    for (int i = 0; i < R; ++i) mask4(rg + 16 * i, V, m, M, wn[i]);
  }
}

// P = sum_v S·Wn (yumas.py:192) for this lane's 4 columns: product rounded,
// then summed (no FMA), two columns per packed v_pk_mul / v_pk_add; row
// order rg + 16 i per lane, then the 16-lane DPP tree.
// Stakes of a lane's rows rg + 16 i read from a wave-private LDS copy on
// every use instead of 16 VGPRs (k_consensus_w). `off` goes through an empty
// asm at each pass (`fresh`), so the compiler cannot hoist the reads out of
// the search loops back into registers.
struct LdsRows {
  const float* base;  // a __shared__ array
  int off;
  __device__ __forceinline__ float operator[](int i) const { return base[off + 16 * i]; }
};
__device__ __forceinline__ LdsRows fresh(LdsRows s) {
  asm volatile("" : "+v"(s.off));
  return s;
}

template <int R, typename SV>
__device__ __forceinline__ void prerank_store(const float (&wn)[R][4], const SV& s,
                                              const WLay& L, int m, int M, float* __restrict__ Pout) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a01 = {0.0f, 0.0f}, a23 = {0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const f2 s2 = {s[i], s[i]};
    const f2 w01 = {wn[i][0], wn[i][1]}, w23 = {wn[i][2], wn[i][3]};
    a01 = a01 + s2 * w01;
    a23 = a23 + s2 * w23;
  }
  float acc[4] = {a01[0], a01[1], a23[0], a23[1]};
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = wsum16(acc[c]);
  if (L.rg == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) Pout[m + c] = acc[c];
}

// Consensus (see k_consensus for the search argument), wave-owned columns.
// HIST: exact-stake histogram finish (below); kHB grid points per column,
// kHS words per column in LDS (16-B aligned, 4-bank skew between columns).
constexpr int kHB = 64, kHS = 68, kHistMinW = 8;
constexpr int kHistWords = 4 * 16 * kHS;  // one block: 4 waves x 16 columns

// The consensus search of this lane's 4 columns over the wave's normalised
// validator rows (wn, s: rows rg + 16 i, padding rows hold wn = 0, s = 0).
// `ut`: the slice's stakes in units of 2^-24 when they are exact (k_rowsum /
// its shard-stage twin), else -1. `hb`: this wave's 16 x kHS histogram words.
// Returns k* per column (C_raw = k* 2^-iters), identical in the 16 lanes of a
// column quad.
// Reductions over the LPC lanes that share a column quad (LPC = 16: one DPP
// row; LPC = 32: two adjacent DPP rows, joined by a lane swap xor 16). Every
// step pairs lanes that pair back and a + b == b + a bitwise, so all lanes
// of the group end with identical bits.
template <int LPC>
__device__ __forceinline__ float red_sum(float x) {
  x = wsum16(x);
  if constexpr (LPC == 32) x = x + __shfl_xor(x, 16, 64);
  return x;
}
template <int LPC>
__device__ __forceinline__ int red_isum(int x) {
  x = iwsum16(x);
  if constexpr (LPC == 32) x = x + __shfl_xor(x, 16, 64);
  return x;
}
template <int LPC>
__device__ __forceinline__ int red_imax(int x) {
  x = iwmax16(x);
  if constexpr (LPC == 32) x = max(x, __shfl_xor(x, 16, 64));
  return x;
}
template <int LPC>
__device__ __forceinline__ int red_imin(int x) {
  x = iwmin16(x);
  if constexpr (LPC == 32) x = min(x, __shfl_xor(x, 16, 64));
  return x;
}
// exclusive prefix sum over the LPC lanes of a group (lane index rg in it)
template <int LPC>
__device__ __forceinline__ int red_iscan_excl(int x, int rg) {
  int e = iscan16_excl(x);
  if constexpr (LPC == 32) {
    const int lower = __shfl_xor(iwsum16(x), 16, 64);  // the other row's total
    e += rg >= 16 ? lower : 0;
  }
  return e;
}

// LPC lanes per column quad: lane (cq, rg) holds rows rg + LPC i of columns
// 4 cq .. 4 cq + 3 of the wave's 256 / LPC columns.
template <int R, int LPC, typename SV>
__device__ __forceinline__ void consensus_search(const float (&wn)[R][4], const SV& s,
                                                 float kappa, int iters, int ut, unsigned* hb,
                                                 int lane, int cq, int rg, int (&hi_k)[4]) {
  constexpr int NCOL = 256 / LPC;  // columns per wave
  constexpr int BPL = 64 / LPC;    // histogram bins per lane in the scan
  bool odd_stake = false;
#pragma unroll
  for (int i = 0; i < R; ++i) odd_stake |= !(s[i] >= 0.0f) || s[i] == INFINITY;
  // every wave of the slice sees the same stakes, so this is slice-uniform
  const bool bracket = !__any(odd_stake) && kappa >= 0.0f;
  const int top = 1 << iters;
  const float scale = (float)top, inv_scale = 1.0f / scale;
  int lo_k[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    lo_k[c] = 0;
    hi_k[c] = top;
  }
  if (bracket) {
    // Column max / min on the fp32 bit patterns as signed integers (the
    // order of non-negative floats; negatives, -0 and negative NaNs compare
    // below +0): v_max3_i32 / v_min3_i32 with no NaN canonicalisation. A
    // positive NaN shows up as a max above +inf and drops that column's
    // bracket (the search then starts from [0, 2^iters]); clamping the min
    // at +0 afterwards equals the min of max(wn, 0). Padding rows hold
    // wn = 0, s = 0 (only lowers the min: a wider, still valid bracket).
    int imax[4], imin[4];
    float stot = 0.0f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      imax[c] = INT_MIN;
      imin[c] = INT_MAX;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      stot = stot + s[i];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int b = __float_as_int(wn[i][c]);
        imax[c] = b > imax[c] ? b : imax[c];
        imin[c] = b < imin[c] ? b : imin[c];
      }
    }
    // F(k) with every mask set, in exactly the order every F below uses
    stot = red_sum<LPC>(stot);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      imax[c] = red_imax<LPC>(imax[c]);
      imin[c] = red_imin<LPC>(imin[c]);
      const bool nanc = imax[c] > 0x7f800000;
      const float vmx = __int_as_float(imax[c]);
      const float vmn = imin[c] > 0 ? __int_as_float(imin[c]) : 0.0f;
      const int gmax = vmx > 0.0f ? (int)fminf(ceilf(vmx * scale), scale) : 0;
      const int gmin = vmn > 0.0f ? (int)fminf(ceilf(vmn * scale), scale + 1.0f) : 0;
      int lo_c = gmin >= 2 ? gmin - 1 : 0;
      int hi_c = gmax < 1 ? 1 : gmax;
      if (lo_c > 0 && !(stot > kappa)) {
        lo_c = 0;
        hi_c = 1;
      }
      if (lo_c >= top) {
        lo_c = top - 1;
        hi_c = top;
      }
      if (hi_c <= lo_c) hi_c = lo_c + 1;
      lo_k[c] = nanc ? 0 : lo_c;
      hi_k[c] = nanc ? top : hi_c;
    }
  }
  // Exact-stake finish (HIST): when every normalised stake is a multiple of
  // 2^-24 and they total <= 1, every subset sum of stakes is exact in fp32,
  // so F(k) = sum_v S[v]·[Wn[v,m] > k/2^iters] does not depend on summation
  // order and equals the reference's fp32 sum. Then one stake histogram over
  // the bracket's grid points (integer stake units, LDS integer atomics ->
  // deterministic) answers the whole remaining search at once: the result of
  // the bisection over [lo, hi] is lo + 1 + #{b in [1, w-1] : F(lo+b) > κ}
  // (F is non-increasing). Brackets wider than kHB-1 grid points are first
  // narrowed by ordinary bisection passes. Any other input (generic float
  // stakes, non-finite or > 2 weights) takes the bisection unchanged.
  int lim = 1;
  bool hist = false;
  int thr = 0;
  hist = bracket && ut >= 0;  // slice-uniform
  if (hist) {
    lim = kHB - 1;
    const double kd = floor((double)kappa * 16777216.0);
    thr = ut - (kd > 33554432.0 ? 33554432 : (int)kd);
  }
  for (;;) {
    for (;;) {
      bool active = false;
#pragma unroll
      for (int c = 0; c < 4; ++c) active |= (hi_k[c] - lo_k[c]) > lim;
      if (!__any(active)) break;
      float part[4], midf[4];
      int mid[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        mid[c] = (lo_k[c] + hi_k[c]) >> 1;
        midf[c] = (float)mid[c] * inv_scale;
        part[c] = 0.0f;
      }
      const auto& sp = fresh(s);
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const float si = sp[i];
        const float zs = 0.0f * si;
#pragma unroll
        for (int c = 0; c < 4; ++c) part[c] = part[c] + ((wn[i][c] > midf[c]) ? si : zs);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        part[c] = red_sum<LPC>(part[c]);
        const bool act = hi_k[c] - lo_k[c] > lim, up = part[c] > kappa;
        lo_k[c] = (act && up) ? mid[c] : lo_k[c];
        hi_k[c] = (act && !up) ? mid[c] : hi_k[c];
      }
    }
    // Brackets of at most kHistMinW grid points (a wide subnet's tiny
    // normalised weights: c4) put every row of a column into a few bins, and
    // the histogram's LDS atomics to one address serialise; such waves finish
    // with <= 3 more bisection passes instead (the same result: the
    // histogram finish equals the bisection, test_consensus_hist.py)
    if (!hist) break;
    bool wide = false;
#pragma unroll
    for (int c = 0; c < 4; ++c) wide |= (hi_k[c] - lo_k[c]) > kHistMinW;
    if (__any(wide)) break;
    hist = false;
    lim = 1;
  }
  {
    if (hist) {
      unsigned* wb = hb;  // this wave's NCOL columns
      uint4* wb4 = reinterpret_cast<uint4*>(wb);
      for (int j = lane; j < NCOL * kHS / 4; j += 64) wb4[j] = make_uint4(0u, 0u, 0u, 0u);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      float nlo[4];
      unsigned w[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        nlo[c] = -(float)lo_k[c];
        w[c] = (unsigned)(hi_k[c] - lo_k[c]);
      }
      const auto& sp = fresh(s);
      // rows outer: one stake conversion per row (integer atomics: any order)
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const unsigned su = (unsigned)(sp[i] * 16777216.0f);  // stake in 2^-24 units (exact, checked above)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          // bin = clamp(ceil(wn·2^iters) - lo, 0, w). wn·2^iters is exact,
          // and so is its difference with the integer lo whenever it is
          // >= 0 (both are multiples of ulp(wn·2^iters)); anything that
          // rounds is negative and lands in bin 0 either way. The u32
          // convert saturates (negatives and -inf -> 0, +inf -> max) and
          // maps NaN to 0, i.e. never above a grid point, as `>` does.
          const unsigned k = (unsigned)ceilf(fmaf(wn[i][c], scale, nlo[c]));
          atomicAdd(wb + (cq * 4 + c) * kHS + (k < w[c] ? k : w[c]), su);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        int p[BPL];
        const unsigned* hc = wb + (cq * 4 + c) * kHS + BPL * rg;
        if constexpr (BPL == 4) {
          const uint4 h = *reinterpret_cast<const uint4*>(hc);
          p[0] = (int)h.x;
          p[1] = p[0] + (int)h.y;
          p[2] = p[1] + (int)h.z;
          p[3] = p[2] + (int)h.w;
        } else {
          const uint2 h = *reinterpret_cast<const uint2*>(hc);
          p[0] = (int)h.x;
          p[1] = p[0] + (int)h.y;
        }
        // P(b) is non-decreasing, so {b : P(b) < thr} is a prefix [0, B);
        // bins b >= w hold P = total >= thr (κ >= 0), so B <= w and the
        // count over [1, w-1] is max(B - 1, 0) without per-bin range tests
        const int t = thr - red_iscan_excl<LPC>(p[BPL - 1], rg);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < BPL; ++j) cnt += p[j] < t ? 1 : 0;
        hi_k[c] = lo_k[c] + max(red_isum<LPC>(cnt), 1);
      }
    }
  }
}

template <int R, bool VEC>
__global__ __launch_bounds__(256, 4) void k_consensus_w(const float* __restrict__ W,
                                                     const float* __restrict__ rsd,
                                                     const float* __restrict__ sn,
                                                     const int* __restrict__ sx,
                                                     const yuma_params_t* __restrict__ prm, int N,
                                                     int V, int M, long long slice0, int tiles,
                                                     double* __restrict__ craw,
                                                     float* __restrict__ Pout, int wsh,
                                                     const int* __restrict__ crep) {
  __shared__ __attribute__((aligned(16))) unsigned hb[kHistWords];
  const WLay L = wlay();
  const long long slice = slice0 + blockIdx.x / tiles;
  const int tile = blockIdx.x % tiles;
  const int n = (int)(slice % N);
  if (dup_slice(crep, slice, N)) return;  // block-uniform
  const int m = tile * kTileM + L.wave * 16 + L.cq * 4;
  if (tile * kTileM + L.wave * 16 >= M) return;  // whole wave past the last miner
  __shared__ __attribute__((aligned(16))) float rl[4][48 * R];
  float wn[R][4];
  load_norm_w_lds<R, VEC>(W + in_slice(slice, N, wsh) * (long long)V * M, rsd + slice * V,
                          sn + slice * V, rl[L.wave], V, M, m, L.rg, L.lane, wn);
  const LdsRows s{&rl[0][0], L.wave * 48 * R + 16 * R + L.rg};
  if (Pout != nullptr) prerank_store<R>(wn, s, L, m, M, Pout + slice * M);
  int hi_k[4];
  const yuma_params_t& p = prm[n];
  const bool hist_ok = !(p.flags & YUMA_FLAG_NO_HIST);
  consensus_search<R, 16>(wn, s, p.kappa, p.bisect_iters, hist_ok ? sx[slice] : -1,
                          hb + L.wave * 16 * kHS, L.lane, L.cq, L.rg, hi_k);
  const int top = 1 << p.bisect_iters;
  if (L.rg == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) craw[slice * M + m + c] = (double)hi_k[c] / (double)top;
}

// Shared-input sweeps (c3): every consensus class of an epoch searches the
// same normalised tile, so a block loads and divides the epoch's 64-miner
// tile once and runs the search of classes g, g + G, ... of the compacted
// class list (k_class_list) on it -- the same search, the same bits as
// k_consensus_w's per-slice blocks. Grid: epochs x tiles x G. (k_consensus_w
// launches a block for every (slice, tile) and lets the duplicate scenarios'
// blocks exit: at c3 31 of 32 of its 1M blocks, each class re-reading the
// tile from the caches.)
template <int R, bool VEC>
__global__ __launch_bounds__(256, 4) void k_consensus_mc(const float* __restrict__ W,
                                                      const float* __restrict__ rsd,
                                                      const float* __restrict__ sn,
                                                      const int* __restrict__ sx,
                                                      const yuma_params_t* __restrict__ prm, int N,
                                                      int V, int M, long long t0, int tiles,
                                                      double* __restrict__ craw,
                                                      const int* __restrict__ clist, int G) {
  __shared__ __attribute__((aligned(16))) unsigned hb[kHistWords];
  const WLay L = wlay();
  const int tile = blockIdx.x % tiles;
  const int g = (blockIdx.x / tiles) % G;
  const long long t = t0 + blockIdx.x / (tiles * G);
  const int nc = clist[0];
  if (g >= nc) return;  // block-uniform
  const int m = tile * kTileM + L.wave * 16 + L.cq * 4;
  if (tile * kTileM + L.wave * 16 >= M) return;  // whole wave past the last miner
  // the epoch's row sums and stakes: stored for every scenario (k_rowsum fan)
  const long long s0 = t * N + clist[1 + g];
  __shared__ __attribute__((aligned(16))) float rl[4][48 * R];
  float wn[R][4];
  load_norm_w_lds<R, VEC>(W + t * (long long)V * M, rsd + s0 * V, sn + s0 * V, rl[L.wave], V, M, m, L.rg,
                          L.lane, wn);
  const LdsRows s{&rl[0][0], L.wave * 48 * R + 16 * R + L.rg};
  for (int j = g; j < nc; j += G) {
    const int n = clist[1 + j];
    const long long slice = t * N + n;
    const yuma_params_t& p = prm[n];
    const bool hist_ok = !(p.flags & YUMA_FLAG_NO_HIST);
    int hi_k[4];
    consensus_search<R, 16>(wn, s, p.kappa, p.bisect_iters, hist_ok ? sx[slice] : -1,
                            hb + L.wave * 16 * kHS, L.lane, L.cq, L.rg, hi_k);
    const int top = 1 << p.bisect_iters;
    if (L.rg == 0)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (m + c < M) craw[slice * M + m + c] = (double)hi_k[c] / (double)top;
  }
}
constexpr int kMcGroups = 4;  // k_consensus_mc: blocks per (epoch, tile), each a quarter of the classes

// ---------------------------------------------------------------------------
// Consensus with 128-byte row segments (round 4). Same
// block / tile as k_consensus_w (one 64-miner tile of one slice), but two
// waves share each 32-miner column group: pair p = wave / 2 owns miners
// 32p .. 32p+31 of the tile, half h = wave % 2 the rows 128h + rg + 8i, and
// lane (cq, rg) = (lane / 8, lane % 8) holds rows rg + 8i of the columns
// 4cq .. 4cq+3. A wave load moves 8 rows x 128 B -- whole lines -- instead of
// k_consensus_w's 16 rows x 64 B, whose line halves land in two waves.
// Column reductions: the 8-lane DPP butterfly inside the wave, then the two
// halves of the pair through LDS, always added h0 + h1, so both waves of a
// pair hold the same bits. Every exchange is one block barrier, so the search
// steps are block-uniform: every wave reads all four waves' bracket data from
// the bracket exchange, derives the block's widest bracket and from it the
// pass count and the histogram-or-bisection finish. The histogram
// is shared by the pair (integer atomics: any order), zeroed ahead of the
// bracket barrier. W loads are non-temporal (whole lines per wave now; in
// k_consensus_w, whose line halves go to two waves, they lost). Not used for
// shared-input sweeps (launch_consensus). 3 waves /
// SIMD: at 4 (128 VGPRs) 3 VGPRs spilled, consensus 0.95 ms against 0.86.
// Measured at c2 (profiles/r04/ab_round6.txt): 0.852-0.853 ms against
// 0.869 for k_consensus_w. V in (64, 256].
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wsum8(float x) {
  x = x + dpp_f<0xB1>(x);   // quad_perm [1,0,3,2]
  x = x + dpp_f<0x4E>(x);   // quad_perm [2,3,0,1]
  x = x + dpp_f<0x141>(x);  // row_half_mirror: lane i <-> 7 - i of each 8-lane half
  return x;
}
__device__ __forceinline__ int iwsum8(int x) {
  x = x + __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);
  x = x + __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);
  x = x + __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false);
  return x;
}
__device__ __forceinline__ int iwmax8(int x) {
  x = max(x, __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));
  x = max(x, __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false));
  return x;
}
__device__ __forceinline__ int iwmin8(int x) {
  x = min(x, __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false));
  return x;
}
// exclusive prefix sum over the 8 lanes of a half row (row_shr with
// bound_ctrl; shifts that cross into the other half are masked)
__device__ __forceinline__ int iscan8_excl(int x, int r8) {
  int y = x;
  int t = __builtin_amdgcn_update_dpp(0, y, 0x111, 0xF, 0xF, true);
  y = y + (r8 >= 1 ? t : 0);
  t = __builtin_amdgcn_update_dpp(0, y, 0x112, 0xF, 0xF, true);
  y = y + (r8 >= 2 ? t : 0);
  t = __builtin_amdgcn_update_dpp(0, y, 0x114, 0xF, 0xF, true);
  y = y + (r8 >= 4 ? t : 0);
  return y - x;
}

// NP: wave pairs per block (2: a 64-miner tile per 4-wave block; 1: a
// 32-miner group per 2-wave block, so a block barrier waits for the pair only)
constexpr int kConsPairs = 2;
template <bool VEC, int NP = 2>
__global__ __launch_bounds__(128 * NP, 3) void k_consensus_p(const float* __restrict__ W,
                                                     const float* __restrict__ rsd,
                                                     const float* __restrict__ sn,
                                                     const int* __restrict__ sx,
                                                     const yuma_params_t* __restrict__ prm, int N,
                                                     int V, int M, long long slice0, int tiles,
                                                     double* __restrict__ craw,
                                                     float* __restrict__ Pout, int wsh,
                                                     const int* __restrict__ crep,
                                                     const float4* __restrict__ rq4) {
  constexpr int R = 16, HR = 8 * R;  // rows per lane, rows per half
  constexpr int NWV = 2 * NP;         // waves per block
  __shared__ __attribute__((aligned(16))) unsigned hb[NP * 32 * kHS];  // per pair: 32 columns
  __shared__ __attribute__((aligned(16))) float rl[NWV][3 * HR];        // per wave: sums, stakes, 1 / sums
  __shared__ float xf[2][NWV][32];  // float exchange, double-buffered
  __shared__ int xi[2][NWV][32];    // bracket max / min bit patterns
  __shared__ unsigned xflag[2][NWV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int pair = wave >> 1, h = wave & 1, pw = wave ^ 1;
  const int cq = lane >> 3, rg = lane & 7;
  const int ctiles = NP == 2 ? tiles : (M + 31) / 32;  // column groups of 32 NP miners per slice
  const long long slice = slice0 + blockIdx.x / ctiles;
  const int tile = blockIdx.x % ctiles;
  const int n = (int)(slice % N);
  if (dup_slice(crep, slice, N)) return;  // block-uniform
  const int m = tile * (32 * NP) + pair * 32 + cq * 4;
  const int r0 = h * HR + rg;  // this lane's rows r0 + 8 i
  const float* Ws = W + in_slice(slice, N, wsh) * (long long)V * M;
  const float* rsd_s = rsd + slice * V;
  const float* sn_s = sn + slice * V;
  float* rw = rl[wave];

  // load + normalise (load_norm_w_lds over the half's rows). With k_rowsum's
  // screened reciprocals (rq4: {row sum, RN(1 / row sum) or NaN, stake}) a
  // wave whose rows all passed the screen divides without the per-element
  // guard; a NaN anywhere sends the wave to IEEE division (the same values)
  float dv[2], sv[2], rv[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int jj = min(h * HR + lane + 64 * k, V - 1);
    if (rq4 != nullptr) {
      const float4 q = rq4[slice * V + jj];
      dv[k] = q.x;
      rv[k] = q.y;
      sv[k] = q.z;
    } else {
      dv[k] = rsd_s[jj];
      sv[k] = sn_s[jj];
      rv[k] = 1.0f / dv[k];
    }
  }
  float wn[R][4];
  const bool full = r0 + 8 * (R - 1) < V && m + 3 < M;
  const bool allfull = VEC && __all(full) && (long long)V * M < (1ll << 30);
  if (allfull) {
    const unsigned o0 = (unsigned)r0 * (unsigned)M + (unsigned)m, st = 8u * (unsigned)M;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const fvec4 t = __builtin_nontemporal_load(reinterpret_cast<const fvec4*>(Ws + (o0 + (unsigned)i * st)));
      wn[i][0] = t.x;
      wn[i][1] = t.y;
      wn[i][2] = t.z;
      wn[i][3] = t.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) load4c<VEC>(Ws, r0 + 8 * i, V, m, M, wn[i]);
  }
  float amax = 0.0f, dmin = INFINITY;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int j = lane + 64 * k;
    amax = fmaxf(amax, fabsf(dv[k]));
    dmin = fminf(dmin, fabsf(dv[k]));
    rw[j] = dv[k];
    rw[HR + j] = h * HR + j < V ? sv[k] : 0.0f;
    rw[2 * HR + j] = rv[k];
  }
  const bool screened = rq4 != nullptr && __all(rv[0] == rv[0] && rv[1] == rv[1]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (screened) {
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float d = rw[rg + 8 * i];
      const float r = rw[2 * HR + rg + 8 * i];
      const f2 r2 = {r, r}, nd2 = {-d, -d};
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const f2 a2 = {wn[i][2 * hh], wn[i][2 * hh + 1]};
        const f2 q = a2 * r2;
        const f2 e = __builtin_elementwise_fma(nd2, q, a2);
        const f2 q1 = __builtin_elementwise_fma(e, r2, q);
        wn[i][2 * hh] = q1[0];
        wn[i][2 * hh + 1] = q1[1];
      }
    }
    if (!__all(full)) {
#pragma unroll
      for (int i = 0; i < R; ++i) mask4(r0 + 8 * i, V, m, M, wn[i]);
    }
  } else if (rq4 != nullptr) {  // some row failed the screen: IEEE division
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float d = rw[rg + 8 * i];
#pragma unroll
      for (int c = 0; c < 4; ++c) wn[i][c] = wn[i][c] / d;
    }
    if (!__all(full)) {
#pragma unroll
      for (int i = 0; i < R; ++i) mask4(r0 + 8 * i, V, m, M, wn[i]);
    }
  } else {
    typedef float f2 __attribute__((ext_vector_type(2)));
    unsigned ymin = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float d = rw[rg + 8 * i];
      const float r = rw[2 * HR + rg + 8 * i];
      const f2 r2 = {r, r}, nd2 = {-d, -d};
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const f2 a2 = {wn[i][2 * hh], wn[i][2 * hh + 1]};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          amax = fmaxf(amax, fabsf(a2[c]));
          const unsigned y = (__float_as_uint(a2[c]) << 1) - 1u;
          ymin = y < ymin ? y : ymin;
        }
        const f2 q = a2 * r2;
        const f2 e = __builtin_elementwise_fma(nd2, q, a2);
        const f2 q1 = __builtin_elementwise_fma(e, r2, q);
        wn[i][2 * hh] = q1[0];
        wn[i][2 * hh + 1] = q1[1];
      }
    }
    const bool slow = !(dmin >= 0x1p-60f && amax <= 0x1p60f &&
                        (ymin == 0xFFFFFFFFu || ymin + 1u >= (__float_as_uint(0x1p-60f) << 1)));
    if (__any(slow)) {  // rare: some operand outside the fast-division guard
#pragma unroll
      for (int i = 0; i < R; ++i) {
        load4c<VEC>(Ws, r0 + 8 * i, V, m, M, wn[i]);
        const float d = rw[rg + 8 * i];
#pragma unroll
        for (int c = 0; c < 4; ++c) wn[i][c] = wn[i][c] / d;
      }
    }
    if (!__all(full)) {
#pragma unroll
      for (int i = 0; i < R; ++i) mask4(r0 + 8 * i, V, m, M, wn[i]);
    }
  }
  const int col = cq * 4;  // this lane's first column within the pair's 32
  // stakes are read from LDS at every use (an empty asm on the offset keeps
  // the compiler from hoisting the 16 reads into registers)
  auto stake_off = [&]() {
    int off = HR + rg;
    asm volatile("" : "+v"(off));
    return off;
  };

  if (Pout != nullptr) {  // P = sum_v S·Wn (yumas.py:192)
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const int so = stake_off();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float si = rw[so + 8 * i];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = acc[c] + si * wn[i][c];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = wsum8(acc[c]);
    if (rg == 0)
#pragma unroll
      for (int c = 0; c < 4; ++c) xf[1][wave][col + c] = acc[c];
    lds_barrier();
    if (h == 0 && rg == 0)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (m + c < M) Pout[slice * M + m + c] = xf[1][wave][col + c] + xf[1][pw][col + c];
    lds_barrier();
  }

  const yuma_params_t& p = prm[n];
  const float kappa = p.kappa;
  const int top = 1 << p.bisect_iters;
  const float scale = (float)top, inv_scale = 1.0f / scale;
  // bracket (consensus_search): column max / min of the bit patterns, stake total
  int lo_k[4], hi_k[4];
  {
    bool odd = false;
    float stot = 0.0f;
    int imax[4], imin[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      imax[c] = INT_MIN;
      imin[c] = INT_MAX;
    }
    const int so = stake_off();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float si = rw[so + 8 * i];
      odd |= !(si >= 0.0f) || si == INFINITY;
      stot = stot + si;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int b = __float_as_int(wn[i][c]);
        imax[c] = b > imax[c] ? b : imax[c];
        imin[c] = b < imin[c] ? b : imin[c];
      }
    }
    stot = wsum8(stot);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      imax[c] = iwmax8(imax[c]);
      imin[c] = iwmin8(imin[c]);
    }
    const bool odd_w = __any(odd);
    {  // zero the pair's histogram ahead of the bracket barrier (used only after it)
      uint4* hz = reinterpret_cast<uint4*>(hb + pair * 32 * kHS);
      constexpr int NW4 = 32 * kHS / 4;
      for (int j = h * (NW4 / 2) + lane; j < (h + 1) * (NW4 / 2); j += 64) hz[j] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (rg == 0)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        xi[0][wave][col + c] = imax[c];
        xi[1][wave][col + c] = imin[c];
      }
    if (lane == 0) {
      xf[0][wave][0] = stot;
      xflag[0][wave] = odd_w ? 1u : 0u;
    }
    lds_barrier();
    // both pairs hold the same rows: block-uniform
    const bool bracket = !(xflag[0][wave] | xflag[0][pw]) && kappa >= 0.0f;
    // a column's bracket from the block's exchanged max / min bit patterns
    // and its pair's stake total (consensus_search's rules)
    auto bracket_of = [&](int mx, int mn, float st, int& lo, int& hi) {
      lo = 0;
      hi = top;
      if (!bracket) return;
      const bool nanc = mx > 0x7f800000;
      const float vmx = __int_as_float(mx);
      const float vmn = mn > 0 ? __int_as_float(mn) : 0.0f;
      const int gmax = vmx > 0.0f ? (int)fminf(ceilf(vmx * scale), scale) : 0;
      const int gmin = vmn > 0.0f ? (int)fminf(ceilf(vmn * scale), scale + 1.0f) : 0;
      int lo_c = gmin >= 2 ? gmin - 1 : 0;
      int hi_c = gmax < 1 ? 1 : gmax;
      if (lo_c > 0 && !(st > kappa)) {
        lo_c = 0;
        hi_c = 1;
      }
      if (lo_c >= top) {
        lo_c = top - 1;
        hi_c = top;
      }
      if (hi_c <= lo_c) hi_c = lo_c + 1;
      lo = nanc ? 0 : lo_c;
      hi = nanc ? top : hi_c;
    };
    const float stot_p = xf[0][pair * 2][0] + xf[0][pair * 2 + 1][0];
#pragma unroll
    for (int c = 0; c < 4; ++c)
      bracket_of(max(xi[0][wave][col + c], xi[0][pw][col + c]), min(xi[1][wave][col + c], xi[1][pw][col + c]),
                 stot_p, lo_k[c], hi_k[c]);
    // the widest bracket of the BLOCK, from the same exchange (lane l forms
    // column l's bracket): every wave derives the same pass schedule, so the
    // search needs no activity flags and no closing all-idle pass
    int wmax;
    {
      const int pl = NP == 2 ? lane >> 5 : 0, cl = lane & 31;
      int lo, hi;
      bracket_of(max(xi[0][2 * pl][cl], xi[0][2 * pl + 1][cl]), min(xi[1][2 * pl][cl], xi[1][2 * pl + 1][cl]),
                 xf[0][2 * pl][0] + xf[0][2 * pl + 1][0], lo, hi);
      wmax = iwmax16(hi - lo);
      wmax = max(wmax, __shfl_xor(wmax, 16, 64));
      wmax = max(wmax, __shfl_xor(wmax, 32, 64));
    }
    // passes (each halves every active bracket to at most ceil(w / 2)):
    // exact stakes and some bracket wider than kHistMinW -> narrow to
    // <= kHB - 1 grid points, then the histogram; otherwise bisect to width 1
    // (the histogram finish equals the bisection, so deciding on the block's
    // widest initial bracket gives the same result)
    bool hist = bracket && (p.flags & YUMA_FLAG_NO_HIST) == 0 && sx[slice] >= 0 && wmax > kHistMinW;
    const int lim = hist ? kHB - 1 : 1;
    int npass = 0;
    for (int w = wmax; w > lim; w = (w + 1) >> 1) ++npass;
    int buf = 1;
    for (int ps = 0; ps < npass; ++ps) {
      bool active = false;
      float part[4], midf[4];
      int mid[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        active |= (hi_k[c] - lo_k[c]) > lim;
        mid[c] = (lo_k[c] + hi_k[c]) >> 1;
        midf[c] = (float)mid[c] * inv_scale;
        part[c] = 0.0f;
      }
      // the pair's two waves hold the same brackets: a wave with no active
      // column (and its partner) skips the sums, never the barrier
      const bool wact = __any(active);
      if (wact) {
        const int so2 = stake_off();
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const float si = rw[so2 + 8 * i];
          const float zs = 0.0f * si;
#pragma unroll
          for (int c = 0; c < 4; ++c) part[c] = part[c] + ((wn[i][c] > midf[c]) ? si : zs);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) part[c] = wsum8(part[c]);
        if (rg == 0)
#pragma unroll
          for (int c = 0; c < 4; ++c) xf[buf][wave][col + c] = part[c];
      }
      lds_barrier();
      if (wact) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float f = xf[buf][pair * 2][col + c] + xf[buf][pair * 2 + 1][col + c];
          const bool act = hi_k[c] - lo_k[c] > lim, up = f > kappa;
          lo_k[c] = (act && up) ? mid[c] : lo_k[c];
          hi_k[c] = (act && !up) ? mid[c] : hi_k[c];
        }
      }
      buf ^= 1;
    }
    if (hist) {
      // exact-stake histogram finish (consensus_search), shared by the pair
      const double kd = floor((double)kappa * 16777216.0);
      const int thr = sx[slice] - (kd > 33554432.0 ? 33554432 : (int)kd);
      unsigned* hp = hb + pair * 32 * kHS;  // zeroed before the bracket barrier
      float nlo[4];
      unsigned w[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        nlo[c] = -(float)lo_k[c];
        w[c] = (unsigned)(hi_k[c] - lo_k[c]);
      }
      const int so = stake_off();
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const unsigned su = (unsigned)(rw[so + 8 * i] * 16777216.0f);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const unsigned k = (unsigned)ceilf(fmaf(wn[i][c], scale, nlo[c]));
          atomicAdd(hp + (col + c) * kHS + (k < w[c] ? k : w[c]), su);
        }
      }
      lds_barrier();
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const unsigned* hc = hp + (col + c) * kHS + 8 * rg;
        const uint4 a = *reinterpret_cast<const uint4*>(hc);
        const uint4 b = *reinterpret_cast<const uint4*>(hc + 4);
        int q[8];
        q[0] = (int)a.x;
        q[1] = q[0] + (int)a.y;
        q[2] = q[1] + (int)a.z;
        q[3] = q[2] + (int)a.w;
        q[4] = q[3] + (int)b.x;
        q[5] = q[4] + (int)b.y;
        q[6] = q[5] + (int)b.z;
        q[7] = q[6] + (int)b.w;
        const int t = thr - iscan8_excl(q[7], rg);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) cnt += q[j] < t ? 1 : 0;
        hi_k[c] = lo_k[c] + max(iwsum8(cnt), 1);
      }
    }
  }
  if (h == 0 && rg == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) craw[slice * M + m + c] = (double)hi_k[c] / (double)top;
}

// Clip + rank (yumas.py:214-217; Yuma2 clips W_prev :328), wave-owned columns.
// rpart[slice][tile] = sum over the tile's 64 miners (wave sums, waves in order).
template <int R, bool VEC, bool YUMA2, bool FULL>
__global__ __launch_bounds__(256) void k_rank_w(
    const float* __restrict__ W, const float* __restrict__ rsd, const float* __restrict__ sn,
    const float* __restrict__ C, const float* __restrict__ Wprev_init, int yuma2_unused, int N, int V,
    int M, long long slice0, int tiles, float* __restrict__ Rout, float* __restrict__ rpart,
    float* __restrict__ Wn_out, float* __restrict__ Wc_out, float* __restrict__ tvc,
    float* __restrict__ tvn, int wsh) {
  __shared__ float wsums[4];
  const WLay L = wlay();
  const long long slice = slice0 + blockIdx.x / tiles;
  const int tile = blockIdx.x % tiles;
  const int n = (int)(slice % N);
  const long long t = slice / N;
  const long long VM = (long long)V * M;
  const int m = tile * kTileM + L.wave * 16 + L.cq * 4;
  float wn[R][4], s[R];
  load_norm_w<R, VEC>(W + in_slice(slice, N, wsh) * VM, rsd + slice * V, sn + slice * V, V, M, m, L.rg,
                      wn, s);
  float Cc[4];
  vec4c(C + slice * M, m, M, Cc);
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  // source of the clip: W (or Yuma2's previous normalised W), per row
  auto source = [&](int i, float (&src)[4]) {
    const int row = L.rg + 16 * i;
    if (YUMA2) {
      if (t == 0) {
        if (Wprev_init != nullptr) {
          load4c<VEC>(Wprev_init + n * VM, row, V, m, M, src);
          mask4(row, V, m, M, src);
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) src[c] = wn[i][c];
        }
      } else {
        load4c<VEC>(W + in_slice(slice - N, N, wsh) * VM, row, V, m, M, src);
        const RowDiv rdp = row_div(rsd[(slice - N) * V + min(row, V - 1)]);
#pragma unroll
        for (int c = 0; c < 4; ++c) src[c] = div_rn(src[c], rdp);
        mask4(row, V, m, M, src);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) src[c] = wn[i][c];
    }
  };
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = L.rg + 16 * i;
    float src[4], wc[4];
    source(i, src);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      wc[c] = vmin(src[c], Cc[c]);
      acc[c] = acc[c] + s[i] * wc[c];
    }
    if (FULL && row < V) {
      if (Wn_out != nullptr) store4<VEC>(Wn_out + slice * VM + (long long)row * M, m, M, wn[i]);
      if (Wc_out != nullptr) store4<VEC>(Wc_out + slice * VM + (long long)row * M, m, M, wc);
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = wsum16(acc[c]);
  if (L.rg == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) Rout[slice * M + m + c] = acc[c];
  // wave sum of its 16 miners (quads in order 0..3), then waves in order
  float ws = 0.0f;
#pragma unroll
  for (int c = 0; c < 4; ++c) ws = ws + acc[c];
  ws = qsum4(ws);
  if (L.lane == 0) wsums[L.wave] = ws;
  if (FULL && tvc != nullptr) {
    // full-output mode only: validator-trust partials over this tile's 64
    // miners (quads xor 1, 2; then waves in order via LDS); V <= 256 here
    __shared__ float tvs[2][4][256];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = L.rg + 16 * i;
      float src[4];
      source(i, src);
      float a = 0.0f, b = 0.0f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (m + c < M) {
          a = a + vmin(src[c], Cc[c]);
          b = b + wn[i][c];
        }
      a = qsum4(a);
      b = qsum4(b);
      if (L.cq == 0 && row < 256) {
        tvs[0][L.wave][row] = a;
        tvs[1][L.wave][row] = b;
      }
    }
    __syncthreads();
    for (int row = threadIdx.x; row < V && row < 256; row += 256) {
      float a = tvs[0][0][row], b = tvs[1][0][row];
      for (int w = 1; w < 4; ++w) {
        a = a + tvs[0][w][row];
        b = b + tvs[1][w][row];
      }
      tvc[(slice * tiles + tile) * V + row] = a;
      tvn[(slice * tiles + tile) * V + row] = b;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = wsums[0];
    for (int w = 1; w < 4; ++w) r = r + wsums[w];
    rpart[slice * tiles + tile] = r;
  }
}

// Clip + rank, streaming form for run outputs (no Wn / Wc / T_v):
// R[m] = sum_v S[v] min(W[v,m], C[m]) (yumas.py:439-442). Nothing is held
// across rows, so the block takes the bond kernel's wide layout (a wave
// instruction moves 4 rows x 256 contiguous bytes instead of 16 x 64) and
// streams its rows in batches of 8 loads per lane. Order: rows g, g+16, ...
// sequentially per lane, then the 4 row groups of a wave (xor 16, 32), then
// the 4 waves in order. YUMA2 clips the previous epoch's normalised weights
// instead (yumas.py:299-300, 328-331: W_prev, at the first epoch the caller's
// W_prev or W itself) with this epoch's stakes: the previous slice divided by
// its own row sums — only W_prev is read, not W.
// BCS (Yuma / Yuma2): the same pass also forms the column sums of the
// instantaneous bond numerator, csb[m] = Σ_v S·W_b with W_b = (1-β)·src +
// β·min(src, C) (yumas.py:227-228, :341-342; src = W, Yuma2's W_prev). They
// depend on the epoch's inputs only, so the bond scan then runs element-wise
// (k_bonds_elem) instead of reducing every column over all validators each
// epoch. Same summation order as R. Beside csb it stores csr[m] = RN(1 / csb)
// when the column passes the fast-division screen (csb and every nonzero
// |S·W_b| of the column in [2^-60, 2^60], as RowDiv's guard), else NaN: the
// scan then divides by Markstein's correction with no per-element guard, and
// its quotients are finite, so nan_to_num is the identity there.
// Shared-input sweeps (c3): the rank of every consensus class of an epoch
// from one block per (epoch, tile, class group) -- k_class_list's classes g,
// g + G, ... in chunks of KC, each chunk one walk over the tile's rows (the
// normalised rows are formed once per walk for KC classes' clips) -- the same
// operations and orders as k_rank_s (Yuma 3 / 4: no bond column sums), so the
// same bits. k_rank_s launches a block for every (slice, tile) and lets the
// duplicate scenarios' blocks exit.
template <bool VEC, int KC>
__global__ __launch_bounds__(256, 1) void k_rank_mc(const float* __restrict__ W,
                                                 const float* __restrict__ rsd,
                                                 const float* __restrict__ sn,
                                                 const float* __restrict__ C, int N, int V, int M,
                                                 long long t0, int tiles,
                                                 float* __restrict__ Rout,
                                                 float* __restrict__ rpart,
                                                 const int* __restrict__ clist, int G) {
  __shared__ float4 red[KC][4][16];
  const Lay L = lay();
  const int tile = blockIdx.x % tiles;
  const int g = (blockIdx.x / tiles) % G;
  const long long t = t0 + blockIdx.x / (tiles * G);
  const int nc = clist[0];
  if (g >= nc) return;  // block-uniform
  const long long VM = (long long)V * M;
  const int m = tile * kTileM + L.c4 * 4;
  const float* Ws = W + t * VM;
  const long long s0 = t * N + clist[1 + g];  // the epoch's row sums and stakes (every scenario's)
  __shared__ float rows_d[kRegRows], rows_r[kRegRows], rows_s[kRegRows];
  for (int j = threadIdx.x; j < V; j += 256) {
    const float dj = rsd[s0 * V + j];
    rows_d[j] = dj;
    rows_r[j] = 1.0f / dj;
    rows_s[j] = sn[s0 * V + j];
  }
  __syncthreads();
  for (int j0 = g; j0 < nc; j0 += G * KC) {
    float Cc[KC][4], acc[KC][4];
    long long sl[KC];
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      const int j = j0 + G * q;
      sl[q] = t * N + clist[1 + (j < nc ? j : g)];
      load4c<VEC>(C + sl[q] * M, 0, 1, m, M, Cc[q]);
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[q][c] = 0.0f;
    }
    constexpr int B = 8;
    for (int r0 = L.g; r0 < V; r0 += 16 * B) {
      float w[B][4], d[B], s[B];
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const int rr = min(r0 + 16 * i, V - 1);
        load4c<VEC>(Ws, rr, V, m, M, w[i]);
        d[i] = rows_d[rr];
        s[i] = rows_s[rr];
      }
      bool slow = false;
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const int rr = min(r0 + 16 * i, V - 1);
        const float ad = fabsf(d[i]);
        const RowDiv rdv{d[i], rows_r[rr], ad >= 0x1p-60f && ad <= 0x1p60f};
#pragma unroll
        for (int c = 0; c < 4; ++c) w[i][c] = div_fast_nz(w[i][c], rdv, slow);
      }
      if (__any(slow)) {  // rare: redo the batch with IEEE division (wave-uniform)
#pragma unroll
        for (int i = 0; i < B; ++i) {
          const int rr = min(r0 + 16 * i, V - 1);
          float x[4];
          load4c<VEC>(Ws, rr, V, m, M, x);
#pragma unroll
          for (int c = 0; c < 4; ++c) w[i][c] = x[c] / d[i];
        }
      }
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const bool live = r0 + 16 * i < V;
#pragma unroll
        for (int q = 0; q < KC; ++q)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float x = s[i] * vmin(w[i][c], Cc[q][c]);
            acc[q][c] = live ? acc[q][c] + x : acc[q][c];
          }
      }
    }
#pragma unroll
    for (int q = 0; q < KC; ++q) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[q][c] = sum_rowgroups(acc[q][c]);
      if (L.lane < 16) red[q][L.wave][L.c4] = make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      if (L.wave != q % 4 || j0 + G * q >= nc) continue;  // wave q % 4 writes class q
      const float* rf = reinterpret_cast<const float*>(&red[q][0][0]);
      float r = rf[L.lane];
#pragma unroll
      for (int w = 1; w < 4; ++w) r = r + rf[w * 64 + L.lane];
      const int mg = tile * kTileM + L.lane;
      if (mg < M) Rout[sl[q] * M + mg] = r;
      float tt = mg < M ? r : 0.0f;
      tt = wave_sum(tt);
      if (L.lane == 0) rpart[sl[q] * tiles + tile] = tt;
    }
    __syncthreads();  // red[] reuse
  }
}

template <bool VEC, bool YUMA2 = false, bool BCS = false>
__global__ __launch_bounds__(256, 1) void k_rank_s(const float* __restrict__ W,
                                                const float* __restrict__ rsd,
                                                const float* __restrict__ sn,
                                                const float* __restrict__ C, int N, int V, int M,
                                                long long slice0, int tiles,
                                                float* __restrict__ Rout,
                                                float* __restrict__ rpart, int wsh,
                                                const int* __restrict__ crep,
                                                const float* __restrict__ Wprev_init,
                                                float* __restrict__ csb,
                                                float* __restrict__ csr,
                                                const yuma_params_t* __restrict__ prm) {
  __shared__ float4 red[4][16];
  __shared__ float4 red2[BCS ? 4 : 1][16];
  __shared__ unsigned smx[BCS ? 4 : 1][64], smn[BCS ? 4 : 1][64];
  const Lay L = lay();
  const long long slice = slice0 + blockIdx.x / tiles;
  const int tile = blockIdx.x % tiles;
  if (dup_slice(crep, slice, N)) return;  // block-uniform
  float p_pen = 0.0f, p_ompen = 0.0f;
  if (BCS) {
    const yuma_params_t& pg = prm[slice % N];
    p_pen = pg.bond_penalty;
    p_ompen = pg.one_minus_bond_penalty;
  }
  const long long VM = (long long)V * M;
  const int m = tile * kTileM + L.c4 * 4;
  // the clipped matrix and the row sums that normalise it (block-uniform)
  long long wsl = slice;
  bool divide = true;
  const float* Ws = W + in_slice(slice, N, wsh) * VM;
  if (YUMA2) {
    if (slice >= N) {
      wsl = slice - N;
      Ws = W + in_slice(wsl, N, wsh) * VM;
    } else if (Wprev_init != nullptr) {
      Ws = Wprev_init + (slice % N) * VM;  // already normalised
      divide = false;
    }
  }
  float Cc[4];
  load4c<VEC>(C + slice * M, 0, 1, m, M, Cc);
  // the slice's row sums, their IEEE reciprocals and the stakes staged in LDS
  // once per block (coalesced), instead of two per-lane scalar loads per row
  // and a reciprocal per row in every lane
  __shared__ float rows_d[kRegRows], rows_r[kRegRows], rows_s[kRegRows];
  for (int j = threadIdx.x; j < V; j += 256) {
    const float dj = rsd[wsl * V + j];
    rows_d[j] = dj;
    rows_r[j] = 1.0f / dj;
    rows_s[j] = sn[slice * V + j];
  }
  __syncthreads();
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float acb[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  // BCS screen: max of |y| and min of nonzero |y| as bit patterns (<< 1 drops
  // the sign; - 1 sends a zero to the top of the min)
  unsigned ymx[4] = {0u, 0u, 0u, 0u}, ymn[4] = {~0u, ~0u, ~0u, ~0u};
  constexpr int B = 8;
  for (int r0 = L.g; r0 < V; r0 += 16 * B) {
    float w[B][4], d[B], s[B];
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int rr = min(r0 + 16 * i, V - 1);
      load4c<VEC>(Ws, rr, V, m, M, w[i]);
      d[i] = rows_d[rr];
      s[i] = rows_s[rr];
    }
    if (!YUMA2 || divide) {
      bool slow = false;
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const int rr = min(r0 + 16 * i, V - 1);
        const float ad = fabsf(d[i]);
        const RowDiv rdv{d[i], rows_r[rr], ad >= 0x1p-60f && ad <= 0x1p60f};
#pragma unroll
        for (int c = 0; c < 4; ++c) w[i][c] = div_fast_nz(w[i][c], rdv, slow);
      }
      if (__any(slow)) {  // rare: redo the batch with IEEE division (wave-uniform)
#pragma unroll
        for (int i = 0; i < B; ++i) {
          const int rr = min(r0 + 16 * i, V - 1);
          float x[4];
          load4c<VEC>(Ws, rr, V, m, M, x);
#pragma unroll
          for (int c = 0; c < 4; ++c) w[i][c] = x[c] / d[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const bool live = r0 + 16 * i < V;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float wc = vmin(w[i][c], Cc[c]);
        const float x = s[i] * wc;
        acc[c] = live ? acc[c] + x : acc[c];
        if (BCS) {
          const float y = s[i] * (p_ompen * w[i][c] + p_pen * wc);
          acb[c] = live ? acb[c] + y : acb[c];
          // (a padding row repeats row V - 1: no mask needed for max / min)
          const unsigned yb = __float_as_uint(y) << 1;
          ymx[c] = max(ymx[c], yb);
          ymn[c] = min(ymn[c], yb - 1u);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = sum_rowgroups(acc[c]);
  if (L.lane < 16) red[L.wave][L.c4] = make_float4(acc[0], acc[1], acc[2], acc[3]);
  if (BCS) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      acb[c] = sum_rowgroups(acb[c]);
#pragma unroll
      for (int o = 16; o <= 32; o <<= 1) {
        ymx[c] = max(ymx[c], (unsigned)__shfl_xor((int)ymx[c], o, 64));
        ymn[c] = min(ymn[c], (unsigned)__shfl_xor((int)ymn[c], o, 64));
      }
    }
    if (L.lane < 16) {
      red2[L.wave][L.c4] = make_float4(acb[0], acb[1], acb[2], acb[3]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        smx[L.wave][L.c4 * 4 + c] = ymx[c];
        smn[L.wave][L.c4 * 4 + c] = ymn[c];
      }
    }
  }
  __syncthreads();
  if (L.wave == 0) {
    // lane l: miner tile*64 + l
    const float* rf = reinterpret_cast<const float*>(&red[0][0]);
    float r = rf[L.lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) r = r + rf[w * 64 + L.lane];
    const int mg = tile * kTileM + L.lane;
    if (mg < M) Rout[slice * M + mg] = r;
    float t = mg < M ? r : 0.0f;
    t = wave_sum(t);
    if (L.lane == 0) rpart[slice * tiles + tile] = t;
  } else if (BCS && L.wave == 1) {
    const float* rf = reinterpret_cast<const float*>(&red2[0][0]);
    float r = rf[L.lane];
    unsigned mx = smx[0][L.lane], mn = smn[0][L.lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      r = r + rf[w * 64 + L.lane];
      mx = max(mx, smx[w][L.lane]);
      mn = min(mn, smn[w][L.lane]);
    }
    const int mg = tile * kTileM + L.lane;
    const float ar = fabsf(r);
    const bool ok = ar >= 0x1p-60f && ar <= 0x1p60f && mx <= (__float_as_uint(0x1p60f) << 1) &&
                    (mn == ~0u || mn + 1u >= (__float_as_uint(0x1p-60f) << 1));
    if (mg < M) {
      csb[slice * M + mg] = r;
      csr[slice * M + mg] = ok ? 1.0f / r : qnan();
    }
  }
}

// k_rank_s on wide column blocks: a block owns 256 miners (four tiles) of
// every row, a wave instruction moves one row's 1 KiB (the bond scan's and
// the row sums' footprint, tools/scanbw), wave w streams rows w, w + 4, ...
// in batches of 8 loads per lane. Order: rows sequentially per lane, then the
// 4 waves in order (LDS); tile partials as k_rank_s (the 64 miners of a tile
// by the wave butterfly). Same outputs and options as k_rank_s. Launched for
// the ranks that also form Yuma / Yuma2's bond column sums (BCS): there it
// takes 0.75 ms at c2 against 0.79 for k_rank_s; and for wide subnets (c4
// 1.10 against 1.15). c2's plain rank is a tie (0.70-0.72 against 0.70,
// profiles/r05/ab_rank_wide.txt), so k_rank_s stays there.
// BIGV (above kRegRows validators): the row sums, reciprocals and stakes are
// read per row from memory instead of the LDS staging.
constexpr int kRankWide = 1;  // launch the wide form (0: k_rank_s everywhere)
template <bool VEC, bool YUMA2 = false, bool BCS = false, bool BIGV = false>
__global__ __launch_bounds__(256, 1) void k_rank_sw(const float* __restrict__ W,
                                                 const float* __restrict__ rsd,
                                                 const float* __restrict__ sn,
                                                 const float* __restrict__ C, int N, int V, int M,
                                                 long long slice0, int tiles,
                                                 float* __restrict__ Rout,
                                                 float* __restrict__ rpart, int wsh,
                                                 const int* __restrict__ crep,
                                                 const float* __restrict__ Wprev_init,
                                                 float* __restrict__ csb,
                                                 float* __restrict__ csr,
                                                 const yuma_params_t* __restrict__ prm) {
  constexpr int CB = 256;
  __shared__ float red[4][CB];
  __shared__ float red2[BCS ? 4 : 1][CB];
  __shared__ unsigned smx[BCS ? 4 : 1][CB], smn[BCS ? 4 : 1][CB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cblocks = (M + CB - 1) / CB;
  const long long slice = slice0 + blockIdx.x / cblocks;
  const int cb = blockIdx.x % cblocks;
  if (dup_slice(crep, slice, N)) return;  // block-uniform
  float p_pen = 0.0f, p_ompen = 0.0f;
  if (BCS) {
    const yuma_params_t& pg = prm[slice % N];
    p_pen = pg.bond_penalty;
    p_ompen = pg.one_minus_bond_penalty;
  }
  const long long VM = (long long)V * M;
  const int m = cb * CB + lane * 4;
  long long wsl = slice;
  bool divide = true;
  const float* Ws = W + in_slice(slice, N, wsh) * VM;
  if (YUMA2) {
    if (slice >= N) {
      wsl = slice - N;
      Ws = W + in_slice(wsl, N, wsh) * VM;
    } else if (Wprev_init != nullptr) {
      Ws = Wprev_init + (slice % N) * VM;  // already normalised
      divide = false;
    }
  }
  float Cc[4];
  load4c<VEC>(C + slice * M, 0, 1, m, M, Cc);
  __shared__ float rows_d[BIGV ? 1 : kRegRows], rows_r[BIGV ? 1 : kRegRows], rows_s[BIGV ? 1 : kRegRows];
  if constexpr (!BIGV) {
    for (int j = threadIdx.x; j < V; j += 256) {
      const float dj = rsd[wsl * V + j];
      rows_d[j] = dj;
      rows_r[j] = 1.0f / dj;
      rows_s[j] = sn[slice * V + j];
    }
    __syncthreads();
  }
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float acb[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  unsigned ymx[4] = {0u, 0u, 0u, 0u}, ymn[4] = {~0u, ~0u, ~0u, ~0u};
  constexpr int B = 8;
  for (int r0 = wave; r0 < V; r0 += 4 * B) {
    float w[B][4], d[B], s[B], rcp[B];
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int rr = min(r0 + 4 * i, V - 1);
      load4c<VEC>(Ws, rr, V, m, M, w[i]);
      if constexpr (BIGV) {
        d[i] = rsd[wsl * V + rr];
        s[i] = sn[slice * V + rr];
        rcp[i] = 1.0f / d[i];
      } else {
        d[i] = rows_d[rr];
        s[i] = rows_s[rr];
        rcp[i] = rows_r[rr];
      }
    }
    if (!YUMA2 || divide) {
      bool slow = false;
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const float ad = fabsf(d[i]);
        const RowDiv rdv{d[i], rcp[i], ad >= 0x1p-60f && ad <= 0x1p60f};
#pragma unroll
        for (int c = 0; c < 4; ++c) w[i][c] = div_fast_nz(w[i][c], rdv, slow);
      }
      if (__any(slow)) {  // rare: redo the batch with IEEE division (wave-uniform)
#pragma unroll
        for (int i = 0; i < B; ++i) {
          const int rr = min(r0 + 4 * i, V - 1);
          float x[4];
          load4c<VEC>(Ws, rr, V, m, M, x);
#pragma unroll
          for (int c = 0; c < 4; ++c) w[i][c] = x[c] / d[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const bool live = r0 + 4 * i < V;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float wc = vmin(w[i][c], Cc[c]);
        const float x = s[i] * wc;
        acc[c] = live ? acc[c] + x : acc[c];
        if (BCS) {
          const float y = s[i] * (p_ompen * w[i][c] + p_pen * wc);
          acb[c] = live ? acb[c] + y : acb[c];
          // (a padding row repeats row V - 1: no mask needed for max / min)
          const unsigned yb = __float_as_uint(y) << 1;
          ymx[c] = max(ymx[c], yb);
          ymn[c] = min(ymn[c], yb - 1u);
        }
      }
    }
  }
  *reinterpret_cast<float4*>(&red[wave][lane * 4]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  if (BCS) {
    *reinterpret_cast<float4*>(&red2[wave][lane * 4]) = make_float4(acb[0], acb[1], acb[2], acb[3]);
    *reinterpret_cast<uint4*>(&smx[wave][lane * 4]) = make_uint4(ymx[0], ymx[1], ymx[2], ymx[3]);
    *reinterpret_cast<uint4*>(&smn[wave][lane * 4]) = make_uint4(ymn[0], ymn[1], ymn[2], ymn[3]);
  }
  __syncthreads();
  // wave w: tile 4 cb + w, lane l its miner l
  const int j = wave * 64 + lane, mg = cb * CB + j, tile = cb * 4 + wave;
  float r = red[0][j];
#pragma unroll
  for (int w = 1; w < 4; ++w) r = r + red[w][j];
  if (mg < M) Rout[slice * M + mg] = r;
  float t = mg < M ? r : 0.0f;
  t = wave_sum(t);
  if (lane == 0 && tile < tiles) rpart[slice * tiles + tile] = t;
  if (BCS) {
    float b = red2[0][j];
    unsigned mx = smx[0][j], mn = smn[0][j];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      b = b + red2[w][j];
      mx = max(mx, smx[w][j]);
      mn = min(mn, smn[w][j]);
    }
    const float ab = fabsf(b);
    const bool ok = ab >= 0x1p-60f && ab <= 0x1p60f && mx <= (__float_as_uint(0x1p60f) << 1) &&
                    (mn == ~0u || mn + 1u >= (__float_as_uint(0x1p-60f) << 1));
    if (mg < M) {
      csb[slice * M + mg] = b;
      csr[slice * M + mg] = ok ? 1.0f / b : qnan();
    }
  }
}

// The full outputs of the clip above kRegRows validators (the register-
// resident k_rank_w / k_rank form them at or below): the normalised weights
// Wn (yumas.py:186), the clipped weights Wc = min(src, C) (:214; Yuma2 clips
// W_prev, :328) and the per-tile row sums of Wc and Wn that validator_trust
// T_v = sum Wc / sum Wn divides (:224; k_finalize adds the tiles in order).
// Block = one 64-miner tile of a slice, rows g + 16 i per thread; every
// division IEEE-exact (div_rn).
template <bool VEC, bool YUMA2>
__global__ __launch_bounds__(256) void k_full_big(const float* __restrict__ W,
                                                 const float* __restrict__ rsd,
                                                 const float* __restrict__ C, int N, int V, int M,
                                                 long long slice0, int tiles, int wsh,
                                                 const float* __restrict__ Wprev_init,
                                                 float* __restrict__ Wn_out, float* __restrict__ Wc_out,
                                                 float* __restrict__ tvc, float* __restrict__ tvn) {
  const Lay L = lay();
  const long long slice = slice0 + blockIdx.x / tiles;
  const int tile = blockIdx.x % tiles;
  const int m = tile * kTileM + L.c4 * 4;
  const long long VM = (long long)V * M;
  const float* Ws = W + in_slice(slice, N, wsh) * VM;
  // Yuma2's clipped source: the previous slice's normalised weights (the
  // caller's W_prev at the first epoch, or W itself without one)
  const float* Wp = Ws;
  long long psl = slice;
  bool pdiv = true;
  if (YUMA2) {
    if (slice >= N) {
      psl = slice - N;
      Wp = W + in_slice(psl, N, wsh) * VM;
    } else if (Wprev_init != nullptr) {
      Wp = Wprev_init + (slice % N) * VM;
      pdiv = false;
    }
  }
  float Cc[4];
  load4c<VEC>(C + slice * M, 0, 1, m, M, Cc);
  for (int row = L.g; row < V; row += 16) {
    float x[4], src[4];
    load4c<VEC>(Ws, row, V, m, M, x);
    const RowDiv rdv = row_div(rsd[slice * V + min(row, V - 1)]);
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = div_rn(x[c], rdv);
    if (YUMA2) {
      load4c<VEC>(Wp, row, V, m, M, src);
      if (pdiv) {
        const RowDiv pdv = row_div(rsd[psl * V + min(row, V - 1)]);
#pragma unroll
        for (int c = 0; c < 4; ++c) src[c] = div_rn(src[c], pdv);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) src[c] = x[c];
    }
    float wc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) wc[c] = tmin(src[c], Cc[c]);
    if (row < V) {
      if (Wn_out != nullptr) store4<VEC>(Wn_out + slice * VM + (long long)row * M, m, M, x);
      if (Wc_out != nullptr) store4<VEC>(Wc_out + slice * VM + (long long)row * M, m, M, wc);
    }
    if (tvc != nullptr) {
      float a = 0.0f, b = 0.0f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (m + c < M) {
          a = a + wc[c];
          b = b + x[c];
        }
      a = sum_row16(a);
      b = sum_row16(b);
      if (L.c4 == 0 && row < V) {
        tvc[(slice * tiles + tile) * (long long)V + row] = a;
        tvn[(slice * tiles + tile) * (long long)V + row] = b;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Block-wide reductions with a fixed order (thread-sequential, wave butterfly,
// waves in order).
// ---------------------------------------------------------------------------
template <int NT>
__device__ float block_sum(float x, float* red) {
  constexpr int NW = NT / 64;
  x = wave_sum(x);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  float t = red[0];
  for (int w = 1; w < NW; ++w) t = t + red[w];
  return t;
}
template <int NT>
__device__ double block_sum_d(double x, double* red) {
  constexpr int NW = NT / 64;
  x = wave_sum_d(x);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  double t = red[0];
  for (int w = 1; w < NW; ++w) t = t + red[w];
  return t;
}

// h[key] += 1 for every active lane. The lanes holding the first active
// lane's key add once, by their count: the levels of a slice crowd into a few
// bins (M = 4096 puts every level of a uniform consensus in high byte 0), and
// same-address LDS atomics serialise lane by lane. Counts are integers, so the
// histogram does not depend on how the adds are grouped.
__device__ inline void hist_add(int* h, int key) {
  const int k0 = __builtin_amdgcn_readfirstlane(key);
  const unsigned long long same = __ballot(key == k0);
  if (key == k0) {
    if ((int)__lane_id() == __ffsll((long long)same) - 1) atomicAdd(&h[k0], (int)__popcll(same));
  } else {
    atomicAdd(&h[key], 1);
  }
}

// high-byte histogram of the levels (four loads in flight per thread)
template <int NT>
__device__ void hist_high(const int* __restrict__ q, int M, int* hist1) {
  int j = threadIdx.x;
  for (; j + 3 * NT < M; j += 4 * NT) {
    int v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = min(max(q[j + u * NT], 0), 65535);
#pragma unroll
    for (int u = 0; u < 4; ++u) hist_add(hist1, v[u] >> 8);
  }
  for (; j < M; j += NT) hist_add(hist1, min(max(q[j], 0), 65535) >> 8);
}

// Bin of the k-th smallest entry of a 256-bin count histogram h: the first bin
// b with sum(h[0..b]) > k, and k minus the counts below it. One wave (all 64
// lanes, four bins each, an inclusive shuffle scan) replaces the serial walk
// of 256 dependent LDS reads; b = 256 when k >= sum(h), as the walk gives.
__device__ void find_bin(const int* h, int k, int* dst) {
  const int l = threadIdx.x & 63;
  const int c0 = h[4 * l], c1 = h[4 * l + 1], c2 = h[4 * l + 2], c3 = h[4 * l + 3];
  const int s = c0 + c1 + c2 + c3;
  int incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (l >= o) incl += y;
  }
  const int excl = incl - s;
  if (excl <= k && k < incl) {
    int cum = excl, i = 0;
    if (cum + c0 <= k) {
      cum += c0;
      ++i;
      if (cum + c1 <= k) {
        cum += c1;
        ++i;
        if (cum + c2 <= k) {
          cum += c2;
          ++i;
        }
      }
    }
    dst[0] = 4 * l + i;
    dst[1] = k - cum;
  } else if (l == 63 && k >= incl) {
    dst[0] = 256;
    dst[1] = k - incl;
  }
}

// low-byte histogram of the levels whose high byte is b (four in flight)
template <int NT>
__device__ void hist_low(const int* __restrict__ q, int M, int b, int* hist2) {
  int j = threadIdx.x;
  for (; j + 3 * NT < M; j += 4 * NT) {
    int v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = min(max(q[j + u * NT], 0), 65535);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if ((v[u] >> 8) == b) hist_add(hist2, v[u] & 255);
  }
  for (; j < M; j += NT) {
    const int v = min(max(q[j], 0), 65535);
    if ((v >> 8) == b) hist_add(hist2, v & 255);
  }
}

// The k0-th and k1-th smallest quantisation levels (0-based) by a two-level
// 256-bin integer histogram select. Integer counts are order independent, so
// the selection is exact and deterministic. hist1 must already hold the
// high-byte histogram; bc holds 8 ints. The two ranks of one quantile share
// the low-byte pass when they share a high byte (the usual case).
template <int NT>
__device__ int2 select_levels(const int* __restrict__ q, int M, int k0, int k1, const int* hist1,
                              int* hist2, int* bc) {
  if (threadIdx.x < 64) {
    find_bin(hist1, k0, bc);
    find_bin(hist1, k1, bc + 2);
  }
  for (int j = threadIdx.x; j < 256; j += NT) hist2[j] = 0;
  __syncthreads();
  const int b0 = bc[0], r0 = bc[1], b1 = bc[2], r1 = bc[3];
  hist_low<NT>(q, M, b0, hist2);
  __syncthreads();
  if (threadIdx.x < 64) {
    find_bin(hist2, r0, bc + 4);
    if (b1 == b0) find_bin(hist2, r1, bc + 6);
  }
  __syncthreads();
  int2 lev;
  lev.x = (b0 << 8) | bc[4];
  if (b1 != b0) {
    for (int j = threadIdx.x; j < 256; j += NT) hist2[j] = 0;
    __syncthreads();
    hist_low<NT>(q, M, b1, hist2);
    __syncthreads();
    if (threadIdx.x < 64) find_bin(hist2, r1, bc + 6);
    __syncthreads();
  }
  lev.y = (b1 << 8) | bc[6];
  __syncthreads();
  return lev;
}


// torch.quantile(C, qf) on levels (Sorting.cpp: rank = q*(n-1) in fp32,
// weight = rank - floor, lerp in the FMA form of the vectorised lerp kernel).
template <int NT>
__device__ float quantile_of(const int* q, int M, float qf, const int* hist1, int* hist2,
                             int* bc) {
  const float rank = qf * (float)(M - 1);
  const int lo_i = (int)rank;
  const int hi_i = (int)ceilf(rank);
  const float w = rank - (float)lo_i;
  const int2 lv = select_levels<NT>(q, M, lo_i, hi_i, hist1, hist2, bc);
  const float a = level_value(lv.x);
  const float b = level_value(lv.y);
  const float diff = b - a;
  if (fabsf(w) < 0.5f) return fmaf(w, diff, a);
  return fmaf(-diff, 1.0f - w, b);
}

// ---------------------------------------------------------------------------
// Phase 1c, one block per slice: C = int32(C / C.sum() * 65535) / 65535
// (yumas.py:211; YumaRust :97 in fp64) and the liquid-alpha block
// (yumas.py:231-253): quantiles -> a, b -> bond_alpha[m].
// scal[slice] = {sum C, a, b, consensus_high, consensus_low, -, -, -}.
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void k_quantise(const double* __restrict__ craw,
                                                 const yuma_params_t* __restrict__ prm,
                                                 int variant, int N, int M, long long slice0,
                                                 float* __restrict__ C, int* __restrict__ qlev,
                                                 float* __restrict__ ba,
                                                 float* __restrict__ scal,
                                                 const float* __restrict__ ext_sumf,
                                                 const double* __restrict__ ext_sumd,
                                                 int no_liquid, const int* __restrict__ crep) {
  __shared__ float redf[NT / 64];
  __shared__ double redd[NT / 64];
  __shared__ int hist1[256], hist2[256], bc[8];
  const long long slice = slice0 + blockIdx.x;
  const yuma_params_t& p = prm[slice % N];
  const double* cr = craw + rep_slice(crep, slice, N) * M;
  int* q = qlev + slice * M;
  float* Cs = C + slice * M;

  float sumf = 0.0f;
  double sumd = 0.0;
  if (ext_sumf != nullptr || ext_sumd != nullptr) {
    // miner-column shard: sum C over every shard, reduced by the caller
    if (variant == YUMA_VARIANT_RUST) {
      sumd = ext_sumd[slice];
      sumf = (float)sumd;
    } else {
      sumf = ext_sumf[slice];
    }
  } else if (variant == YUMA_VARIANT_RUST) {
    double acc = 0.0;
    int m = threadIdx.x;
    for (; m + 7 * NT < M; m += 8 * NT) {  // loads in flight, same summation order
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = cr[m + u * NT];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = acc + x[u];
    }
    for (; m < M; m += NT) acc = acc + cr[m];
    sumd = block_sum_d<NT>(acc, redd);
    sumf = (float)sumd;
  } else {
    float acc = 0.0f;
    int m = threadIdx.x;
    for (; m + 7 * NT < M; m += 8 * NT) {  // loads in flight, same summation order
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = cr[m + u * NT];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = acc + (float)x[u];
    }
    for (; m < M; m += NT) acc = acc + (float)cr[m];
    sumf = block_sum<NT>(acc, redf);
  }
  // the levels are kept only for the quantile select here or a shard's
  // k_liquid later; every other slice needs C alone
  const bool keep_q = no_liquid || p.liquid_mode == YUMA_LIQUID_QUANTILE;
  auto level_of = [&](double c) {
    if (variant == YUMA_VARIANT_RUST) return (int)(c / sumd * 65535.0);
    return (int)((float)c / sumf * 65535.0f);
  };
  {
    int m = threadIdx.x;
    for (; m + 7 * NT < M; m += 8 * NT) {  // a wide subnet: 65536 levels per slice
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = cr[m + u * NT];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int lev = level_of(x[u]);
        if (keep_q) q[m + u * NT] = lev;
        Cs[m + u * NT] = level_value(lev);
      }
    }
    for (; m < M; m += NT) {
      const int lev = level_of(cr[m]);
      if (keep_q) q[m] = lev;
      Cs[m] = level_value(lev);
    }
  }
  float a32 = qnan(), b32 = qnan(), ch = qnan(), cl = qnan();
  // no_liquid: the quantiles need every shard's levels (k_liquid, later stage)
  if (p.liquid_mode != YUMA_LIQUID_OFF && !no_liquid) {
    if (p.liquid_mode == YUMA_LIQUID_CONST_AB) {
      a32 = p.const_a;
      b32 = p.const_b;
      ch = (float)p.override_high;
      cl = (float)p.override_low;
    } else {
      for (int j = threadIdx.x; j < 256; j += NT) hist1[j] = 0;
      __syncthreads();
      hist_high<NT>(q, M, hist1);
      __syncthreads();
      const bool H = p.override_flags & YUMA_OVR_HIGH, Lw = p.override_flags & YUMA_OVR_LOW;
      ch = H ? (float)p.override_high : quantile_of<NT>(q, M, 0.75f, hist1, hist2, bc);
      cl = Lw ? (float)p.override_low : quantile_of<NT>(q, M, 0.25f, hist1, hist2, bc);
      // both overrides: the host decided the (double) equality; otherwise fp32 compare
      const bool eq = (H && Lw) ? (p.override_flags & YUMA_OVR_FORCE_Q99) != 0 : (ch == cl);
      if (eq) ch = quantile_of<NT>(q, M, 0.99f, hist1, hist2, bc);
      const float d = cl - ch;
      const float inv = 1.0f / d;
      a32 = inv * (float)p.ln_num;
      b32 = (float)p.ln_low + a32 * cl;
    }
    const float e32 = 2.71828182845904523536f;
    for (int m = threadIdx.x; m < M; m += NT) {
      const float x = (-a32) * Cs[m];
      const float y = x + b32;
      const float pw = powf(e32, y);
      const float den = 1.0f + pw;
      const float alpha = 1.0f / den;
      const float clamped = tmin(tmax(alpha, p.alpha_low), p.alpha_high);
      ba[slice * M + m] = 1.0f - clamped;
    }
  }
  if (threadIdx.x == 0) {
    float* sc = scal + slice * 8;
    sc[0] = sumf;
    sc[1] = a32;
    sc[2] = b32;
    sc[3] = ch;
    sc[4] = cl;
  }
}

// ---------------------------------------------------------------------------
// Phase 1d: clip + rank (yumas.py:214-217; Yuma2 clips W_prev :328) and the
// full-output extras (weight, clipped weight, validator-trust partials).
// rpart[slice][tile] = sum over the tile's 64 columns of R.
// ---------------------------------------------------------------------------
template <int NT, int R, bool VEC>
__global__ __launch_bounds__(NT) void k_rank(
    const float* __restrict__ W, const float* __restrict__ rsd, const float* __restrict__ sn,
    const float* __restrict__ C, const float* __restrict__ Wprev_init, int yuma2, int N, int V,
    int M, long long slice0, int tiles, float* __restrict__ Rout, float* __restrict__ rpart,
    float* __restrict__ Wn_out, float* __restrict__ Wc_out, float* __restrict__ tvc,
    float* __restrict__ tvn, int wsh) {
  constexpr int NW = NT / 64, G = NT / 16;
  __shared__ float4 red[NW * 16];
  const Lay L = lay();
  const long long slice = slice0 + blockIdx.x / tiles;
  const int tile = blockIdx.x % tiles;
  const int n = (int)(slice % N);
  const long long t = slice / N;
  const int m = tile * kTileM + L.c4 * 4;
  const long long VM = (long long)V * M;
  const float* Ws = W + in_slice(slice, N, wsh) * VM;
  float Cc[4];
  load4_vec(C + slice * M, m, M, Cc);

  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  float xw[R][4], dv[R], sv[R];
#pragma unroll
  for (int i = 0; i < R; ++i) load4c<VEC>(Ws, L.g + G * i, V, m, M, xw[i]);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int rr = min(L.g + G * i, V - 1);
    dv[i] = rsd[slice * V + rr];
    sv[i] = sn[slice * V + rr];
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = L.g + G * i;
    if (row >= V) continue;
    float wn[4], src[4], wc[4];
    const RowDiv rdv = row_div(dv[i]);
#pragma unroll
    for (int c = 0; c < 4; ++c) wn[c] = div_rn(xw[i][c], rdv);
    if (yuma2) {
      if (t == 0) {
        if (Wprev_init != nullptr) {
          load4<VEC>(Wprev_init + n * VM + (long long)row * M, m, M, src);
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) src[c] = wn[c];
        }
      } else {
        float xp[4];
        load4<VEC>(W + in_slice(slice - N, N, wsh) * VM + (long long)row * M, m, M, xp);
        const RowDiv rdp = row_div(rsd[(slice - N) * V + row]);
#pragma unroll
        for (int c = 0; c < 4; ++c) src[c] = div_rn(xp[c], rdp);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) src[c] = wn[c];
    }
    const float s = sv[i];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      wc[c] = tmin(src[c], Cc[c]);
      acc[c] = acc[c] + s * wc[c];
    }
    if (Wn_out != nullptr) store4<VEC>(Wn_out + slice * VM + (long long)row * M, m, M, wn);
    if (Wc_out != nullptr) store4<VEC>(Wc_out + slice * VM + (long long)row * M, m, M, wc);
    if (tvc != nullptr) {
      float a = 0.0f, b = 0.0f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (m + c < M) {
          a = a + wc[c];
          b = b + wn[c];
        }
      a = sum_row16(a);
      b = sum_row16(b);
      if (L.c4 == 0) {
        tvc[(slice * tiles + tile) * V + row] = a;
        tvn[(slice * tiles + tile) * V + row] = b;
      }
    }
  }
  col_reduce4<NW>(acc, red, L);
  if (L.g == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) Rout[slice * M + m + c] = acc[c];
  // tile sum of R in a fixed order: quad sums, lane butterfly over 16 quads
  float ts = 0.0f;
#pragma unroll
  for (int c = 0; c < 4; ++c) ts = ts + acc[c];
  ts = sum_row16(ts);
  if (threadIdx.x == 0) rpart[slice * tiles + tile] = ts;
}

// Liquid alpha only (a miner-column-sharded run quantised C per shard): quantiles of
// the levels and bond_alpha[m] (yumas.py:231-253). One block per slice.
template <int NT>
__global__ __launch_bounds__(NT) void k_liquid(const yuma_params_t* __restrict__ prm, int N, int M,
                                               long long slice0, const float* __restrict__ C,
                                               const int* __restrict__ qlev, int Mq,
                                               float* __restrict__ ba, float* __restrict__ scal,
                                               const float* __restrict__ sumc_f,
                                               const double* __restrict__ sumc_d, int rust) {
  __shared__ int hist1[256], hist2[256], bc[8];
  const long long slice = slice0 + blockIdx.x;
  const yuma_params_t& p = prm[slice % N];
  const int* q = qlev + slice * Mq;
  float a32 = qnan(), b32 = qnan(), ch = qnan(), cl = qnan();
  if (p.liquid_mode != YUMA_LIQUID_OFF) {
    if (p.liquid_mode == YUMA_LIQUID_CONST_AB) {
      a32 = p.const_a;
      b32 = p.const_b;
      ch = (float)p.override_high;
      cl = (float)p.override_low;
    } else if (qlev != nullptr) {  // (a shard caller that omits the levels gets NaN alphas)
      for (int j = threadIdx.x; j < 256; j += NT) hist1[j] = 0;
      __syncthreads();
      hist_high<NT>(q, Mq, hist1);
      __syncthreads();
      const bool H = p.override_flags & YUMA_OVR_HIGH, Lw = p.override_flags & YUMA_OVR_LOW;
      ch = H ? (float)p.override_high : quantile_of<NT>(q, Mq, 0.75f, hist1, hist2, bc);
      cl = Lw ? (float)p.override_low : quantile_of<NT>(q, Mq, 0.25f, hist1, hist2, bc);
      const bool eq = (H && Lw) ? (p.override_flags & YUMA_OVR_FORCE_Q99) != 0 : (ch == cl);
      if (eq) ch = quantile_of<NT>(q, Mq, 0.99f, hist1, hist2, bc);
      const float d = cl - ch;
      const float inv = 1.0f / d;
      a32 = inv * (float)p.ln_num;
      b32 = (float)p.ln_low + a32 * cl;
    }
    const float e32 = 2.71828182845904523536f;
    for (int mm = threadIdx.x; mm < M; mm += NT) {
      const float xx = (-a32) * C[slice * M + mm];
      const float y = xx + b32;
      const float pw = powf(e32, y);
      const float den = 1.0f + pw;
      const float alpha = 1.0f / den;
      const float clamped = tmin(tmax(alpha, p.alpha_low), p.alpha_high);
      ba[slice * M + mm] = 1.0f - clamped;
    }
  }
  if (threadIdx.x == 0) {
    float* sc = scal + slice * 8;
    sc[0] = rust ? (float)sumc_d[slice - slice0] : sumc_f[slice - slice0];
    sc[1] = a32;
    sc[2] = b32;
    sc[3] = ch;
    sc[4] = cl;
  }
}

// ---------------------------------------------------------------------------
// Phase 1e, one block per slice: I = nan_to_num(R / R.sum(), 0) and the
// server trust T = nan_to_num(R / P) (yumas.py:220-223).
// ---------------------------------------------------------------------------
constexpr int kIncCols = 4096;
__global__ __launch_bounds__(256) void k_incentive(float* __restrict__ Rio,
                                                   const float* __restrict__ rpart,
                                                   const float* __restrict__ Pin, int M,
                                                   long long slice0, int tiles,
                                                   float* __restrict__ I, float* __restrict__ T,
                                                   float* __restrict__ scal,
                                                   const float* __restrict__ ext_rsum,
                                                   const int* __restrict__ crep, int N,
                                                   int nchunk, int v4, int copyr) {
  // block = (slice, chunk of kIncCols miners): every block of a slice forms
  // the same ΣR (same order, same bits), then scales its own chunk
  constexpr int kStage = 4096;
  __shared__ float tot;
  __shared__ float rp[kStage];
  const long long slice = slice0 + blockIdx.x / nchunk;
  const int ch = blockIdx.x % nchunk;
  // rank computed by the class representative (crep): R copied into this
  // slice when someone reads it (the caller's R output; YumaRust's bond scan)
  const long long rs = rep_slice(crep, slice, N);
  const bool cp = copyr && rs != slice;
  float s = 0.0f;
  if (ext_rsum != nullptr) {  // miner-column shard: sum over every shard
    s = ext_rsum[slice];
  } else {
    // the tile partials staged through LDS by the whole block (a wide subnet
    // has 1024 per slice), summed in tile order by one thread
    for (int k0 = 0; k0 < tiles; k0 += kStage) {
      const int nk = tiles - k0 < kStage ? tiles - k0 : kStage;
      for (int k = threadIdx.x; k < nk; k += 256) rp[k] = rpart[rs * tiles + k0 + k];
      __syncthreads();
      if (threadIdx.x == 0)
        for (int k = 0; k < nk; ++k) s = s + rp[k];
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    tot = s;
    if (ch == 0) scal[slice * 8 + 5] = s;
  }
  __syncthreads();
  const float sr = tot;
  const int m1 = min(M, (ch + 1) * kIncCols);
  if (v4) {  // M % 4 == 0, 16-byte aligned rows: one float4 per lane (c3 writes R and I of 16384 slices)
    const float4* r4 = reinterpret_cast<const float4*>(Rio + rs * M);
    float4* d4 = reinterpret_cast<float4*>(Rio + slice * M);
    float4* i4 = reinterpret_cast<float4*>(I + slice * M);
    for (int j = ch * (kIncCols / 4) + threadIdx.x; j < m1 / 4; j += 256) {
      const float4 r = r4[j];
      if (cp) d4[j] = r;
      i4[j] = make_float4(nan_to_num(r.x / sr, 0.0f), nan_to_num(r.y / sr, 0.0f),
                          nan_to_num(r.z / sr, 0.0f), nan_to_num(r.w / sr, 0.0f));
      if (T != nullptr) {
        const float4 pv = reinterpret_cast<const float4*>(Pin + slice * M)[j];
        reinterpret_cast<float4*>(T + slice * M)[j] =
            make_float4(nan_to_num(r.x / pv.x, 0.0f), nan_to_num(r.y / pv.y, 0.0f),
                        nan_to_num(r.z / pv.z, 0.0f), nan_to_num(r.w / pv.w, 0.0f));
      }
    }
    return;
  }
  for (int m = ch * kIncCols + threadIdx.x; m < m1; m += 256) {
    const float r = Rio[rs * M + m];
    if (cp) Rio[slice * M + m] = r;
    I[slice * M + m] = nan_to_num(r / sr, 0.0f);
    if (T != nullptr) T[slice * M + m] = nan_to_num(r / Pin[slice * M + m], 0.0f);
  }
}

// ---------------------------------------------------------------------------
// Phase 2: bond recurrence over the epochs [t0, t1) of a chunk, one block per
// (scenario, row block, 64-miner tile); the bond tile stays in registers.
//   VARIANT 3 (yumas.py:452-472) and 4 (:570-586) are element-wise, so a block
//   owns R*G rows of the tile. VARIANT 0/1/2 normalise bond columns over all
//   validators (yumas.py:113-116,147-149; :228; :342), so a block owns the
//   whole column (single row block).
// dpart[slice][tile][v] = sum over the tile's columns of B_state * I.
// ---------------------------------------------------------------------------
struct BondArgs {
  const float* W;
  const float* rsd;
  const float* sn;
  const float* C;
  const float* I;
  const float* ba;  // liquid bond_alpha [slice][M] (read for liquid scenarios)
  const yuma_params_t* prm;
  const float* B_init;
  const float* Wprev_init;
  float* Bstate;  // [N][V][M]
  float* B_hist;
  float* Wb_out;
  float* Binst_out;
  float* dpart;
  const float4* rq4;  // per input slice and row {row sum, RN(1 / row sum) or NaN, stake, 0} (k_rowsum)
  const float* csb;   // Yuma / Yuma2: [slice][M] Σ_v S·W_b (k_rank_s), or null
  const float* csr;   // ... RN(1 / csb) or NaN (the column fails the division screen)
  const float* R;     // [slice][M] rank R = Σ_v S·Wc (YumaRust's first bond column sum)
  const int* csrep;   // shared inputs: per scenario, the rank class representative whose
                      // rank pass formed csb / csr (k_classes with bond_penalty), or null
  float* cpart;       // YumaRust above kRegRows validators: [N][row block][M] column partials
  int N, V, M, tiles, rowblocks, t0, t1;
  int wsh;      // every scenario reads input slice t (yuma_run_shared)
  int cblocks;  // k_bonds_elem: column blocks of CB miners per row block
  int ep;       // DP_QTE: epoch stride of a (scenario, quad, row) series (multiple of 16)
};

// Dividend partials. Each bond scan forms p_k = sum over tile k's columns of
// B·I per (slice, validator) -- k a 64-miner tile, or the column-normalised
// strip scan's 16-miner strip -- and D[v] of a slice is their canonical sum
// (dp_quad / dp_canon): quads Q_b = (p_4b + p_4b+1) + (p_4b+2 + p_4b+3)
// (absent tiles 0), S_g = sequential sum over the quads b = g (mod 4), then
// D = ((S_0 + S_1) + S_2) + S_3. Every layout gives the same bits:
//   DP_TV  [slice][tile][V]  per tile (k_bonds, k_bonds_cn, k_bonds_grp,
//          k_bonds_elem on 64-miner tiles)
//   DP_VQ  [slice][V][quad]  the wide history scan: a wave holds one quad of a
//          row and stores Q_b (a quarter of the partial bytes)
//   DP_QTE [scenario][quad][V][epoch]  the one-row history-less scan: Q_b of 16
//          epochs gathered in one 16-lane row and stored as one 64-byte run
//          (partial stores into HBM cost a read stream far more than their
//          bytes: tools/scanrd, profiles/r04/scanrd*.txt)
//   DP_PRE [slice][V]        D itself (k_dte_sum)
enum DpLayout { DP_TV = 0, DP_VQ = 1, DP_QTE = 2, DP_PRE = 3 };
__host__ __device__ __forceinline__ int dp_quads(int tiles) { return (tiles + 3) >> 2; }
// Q_b of validator v from per-tile partials pv[k * stride]
__device__ __forceinline__ float dp_quad(const float* __restrict__ pv, long long stride, int b, int tiles) {
  float x[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) x[j] = 4 * b + j < tiles ? pv[(4 * b + j) * stride] : 0.0f;
  return (x[0] + x[1]) + (x[2] + x[3]);
}
__device__ __forceinline__ long long dp_index(long long slice, int tile, int v, int tiles, int V) {
  return (slice * tiles + tile) * (long long)V + v;
}
// YUMA_RESET_IF_ZERO_CONSENSUS (simulation_utils.py:62-88): is C of the epoch
// before the reset epoch zero at the reset column? (false when the reset
// epoch is outside this launch's epochs or the mode does not test C)
__device__ __forceinline__ bool reset_c_zero(const BondArgs& A, int n, int mode, bool all, int epoch,
                                             int index) {
  if (mode != YUMA_RESET_IF_ZERO_CONSENSUS || all || epoch < 1 || epoch < A.t0 || epoch >= A.t1 ||
      index < 0 || index >= A.M)
    return false;
  return A.C[((long long)(epoch - 1) * A.N + n) * A.M + index] == 0.0f;
}

template <int VARIANT, int NT, int R, bool VEC>
__global__ __launch_bounds__(NT) void k_bonds(BondArgs A) {
  constexpr int NW = NT / 64, G = NT / 16;
  constexpr bool COLNORM = (VARIANT == YUMA_VARIANT_RUST || VARIANT == YUMA_VARIANT_YUMA1 ||
                            VARIANT == YUMA_VARIANT_YUMA2);
  __shared__ float4 red[2][NW * 16];
  const Lay L = lay();
  const int tile = blockIdx.x % A.tiles;
  const int rb = (blockIdx.x / A.tiles) % A.rowblocks;
  const int n = blockIdx.x / (A.tiles * A.rowblocks);
  const int N = A.N, V = A.V, M = A.M;
  const long long VM = (long long)V * M;
  const int m = tile * kTileM + L.c4 * 4;
  const yuma_params_t& p = A.prm[n];
  const int row0 = rb * G * R + L.g;

  float B[R][4];
  float Wp[R][4];  // Yuma2: previous epoch's normalised W
  bool has_old;
  if (A.t0 == 0) {
    has_old = A.B_init != nullptr;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = row0 + G * i;
      if (has_old && row < V)
        load4<VEC>(A.B_init + n * VM + (long long)row * M, m, M, B[i]);
      else
#pragma unroll
        for (int c = 0; c < 4; ++c) B[i][c] = 0.0f;
    }
  } else {
    has_old = true;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = row0 + G * i;
      if (row < V)
        load4<VEC>(A.Bstate + n * VM + (long long)row * M, m, M, B[i]);
      else
#pragma unroll
        for (int c = 0; c < 4; ++c) B[i][c] = 0.0f;
    }
  }
  bool have_wp = false;
  if (VARIANT == YUMA_VARIANT_YUMA2) {
    if (A.t0 == 0) {
      if (A.Wprev_init != nullptr) {
        have_wp = true;
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const int row = row0 + G * i;
          if (row < V)
            load4<VEC>(A.Wprev_init + n * VM + (long long)row * M, m, M, Wp[i]);
          else
#pragma unroll
            for (int c = 0; c < 4; ++c) Wp[i][c] = 0.0f;
        }
      }
    } else {
      have_wp = true;
      const long long ps = (long long)(A.t0 - 1) * N + n;
      const long long pw = A.wsh ? (long long)(A.t0 - 1) : ps;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = row0 + G * i;
        if (row < V) {
          float x[4];
          load4<VEC>(A.W + pw * VM + (long long)row * M, m, M, x);
          const float d = A.rsd[ps * V + row];
#pragma unroll
          for (int c = 0; c < 4; ++c) Wp[i][c] = x[c] / d;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) Wp[i][c] = 0.0f;
        }
      }
    }
  }

  for (int t = A.t0; t < A.t1; ++t) {
    const long long slice = (long long)t * N + n;
    // bond resets of run_simulation (simulation_utils.py:62-88), applied to
    // the state before this epoch's update
    const bool reset_all = (p.flags & YUMA_FLAG_RESET_ALL_COLUMNS) != 0;
    if ((VARIANT == YUMA_VARIANT_YUMA3 || VARIANT == YUMA_VARIANT_YUMA4) && has_old &&
        p.reset_mode != YUMA_RESET_NONE && t == p.reset_epoch &&
        (reset_all || (p.reset_index >= 0 && p.reset_index < M))) {
      bool fire = p.reset_mode == YUMA_RESET_ALWAYS;
      if (p.reset_mode == YUMA_RESET_IF_ZERO_CONSENSUS && t >= 1 && !reset_all)
        fire = A.C[(slice - N) * M + p.reset_index] == 0.0f;
      const int c = p.reset_index - m;
      if (fire && (reset_all || (c >= 0 && c < 4)))
#pragma unroll
        for (int i = 0; i < R; ++i) {
#pragma unroll
          for (int cc = 0; cc < 4; ++cc)
            if (reset_all || cc == c) B[i][cc] = 0.0f;
        }
    }
    float Ic[4], Cc[4], bac[4], omba[4];
    load4_vec(A.I + slice * M, m, M, Ic);
    if (COLNORM) load4_vec(A.C + slice * M, m, M, Cc);
    if (p.liquid_mode != YUMA_LIQUID_OFF) {
      load4_vec(A.ba + slice * M, m, M, bac);
#pragma unroll
      for (int c = 0; c < 4; ++c) omba[c] = 1.0f - bac[c];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bac[c] = p.bond_alpha;
        omba[c] = p.one_minus_bond_alpha;
      }
    }

    float wn[R][4], s[R], dd[R];
    const long long wsl = A.wsh ? (long long)t : slice;
#pragma unroll
    for (int i = 0; i < R; ++i) load4c<VEC>(A.W + wsl * VM, row0 + G * i, V, m, M, wn[i]);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int rr = min(row0 + G * i, V - 1);
      dd[i] = A.rsd[slice * V + rr];
      s[i] = A.sn[slice * V + rr];
    }
    {
      bool slow = false;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const RowDiv rdv = row_div(dd[i]);
#pragma unroll
        for (int c = 0; c < 4; ++c) wn[i][c] = div_fast(wn[i][c], rdv, slow);
      }
      if (__syncthreads_or(slow)) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
          load4c<VEC>(A.W + wsl * VM, row0 + G * i, V, m, M, wn[i]);
#pragma unroll
          for (int c = 0; c < 4; ++c) wn[i][c] = wn[i][c] / dd[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      mask4(row0 + G * i, V, m, M, wn[i]);
      if (row0 + G * i >= V) s[i] = 0.0f;
    }

    if (VARIANT == YUMA_VARIANT_YUMA3) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const float cap = s[i] * p.maxint;
        const float ca = p.capacity_alpha * cap;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float rem = tmax(cap - B[i][c], 0.0f);
          const float pc = tmin(ca, rem);
          const float purchase = pc * wn[i][c];
          const float nb = p.decay_keep * B[i][c] + purchase;
          B[i][c] = tmin(nb, cap);
        }
      }
    } else if (VARIANT == YUMA_VARIANT_YUMA4) {
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float bd = B[i][c] * omba[c];
          const float rem = tmax(1.0f - bd, 0.0f);
          const float pi = bac[c] * wn[i][c];
          const float nb = bd + tmin(pi, rem);
          B[i][c] = tmin(nb, 1.0f);
        }
    } else {
      // column-normalised variants
      float num[R][4];
      float colsum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = row0 + G * i;
        float src[4], wc[4], wb[4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
          src[c] = (VARIANT == YUMA_VARIANT_YUMA2 && have_wp) ? Wp[i][c] : wn[i][c];
#pragma unroll
        for (int c = 0; c < 4; ++c) wc[c] = tmin(src[c], Cc[c]);
        if (VARIANT == YUMA_VARIANT_RUST) {
#pragma unroll
          for (int c = 0; c < 4; ++c) num[i][c] = s[i] * wc[c];
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            wb[c] = p.one_minus_bond_penalty * src[c] + p.bond_penalty * wc[c];
            num[i][c] = s[i] * wb[c];
          }
          if (A.Wb_out != nullptr && row < V)
            store4<VEC>(A.Wb_out + slice * VM + (long long)row * M, m, M, wb);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) colsum[c] = colsum[c] + num[i][c];
      }
      col_reduce4<NW>(colsum, red[0], L);
      float den[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        den[c] = (VARIANT == YUMA_VARIANT_RUST) ? colsum[c] + 1e-6f : colsum[c];
      float ema_sum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = row0 + G * i;
        float binst[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float b = num[i][c] / den[c];
          binst[c] = (VARIANT == YUMA_VARIANT_RUST) ? nan_to_num(b, 0.0f) : nan_to_num(b, 0.0f);
        }
        if (A.Binst_out != nullptr && row < V)
          store4<VEC>(A.Binst_out + slice * VM + (long long)row * M, m, M, binst);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float e = binst[c];
          if (has_old) e = bac[c] * binst[c] + omba[c] * B[i][c];
          if (row >= V) e = 0.0f;
          B[i][c] = e;
          ema_sum[c] = ema_sum[c] + e;
        }
      }
      if (VARIANT == YUMA_VARIANT_RUST) {
        col_reduce4<NW>(ema_sum, red[1], L);
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c) B[i][c] = nan_to_num(B[i][c] / (ema_sum[c] + 1e-6f), 0.0f);
      }
      if (VARIANT == YUMA_VARIANT_YUMA2) {
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c) Wp[i][c] = wn[i][c];
        have_wp = true;
      }
    }
    has_old = true;

    // state history + dividend partials
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = row0 + G * i;
      if (A.B_hist != nullptr && row < V)
        store4<VEC>(A.B_hist + slice * VM + (long long)row * M, m, M, B[i]);
      float d = 0.0f;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (m + c < M) d = d + B[i][c] * Ic[c];
      d = sum_row16(d);
      if (L.c4 == 0 && row < V) A.dpart[(slice * A.tiles + tile) * V + row] = d;
    }
    if (COLNORM) __syncthreads();  // red[] reuse across epochs
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = row0 + G * i;
    if (row < V) store4<VEC>(A.Bstate + n * VM + (long long)row * M, m, M, B[i]);
  }
}

// ---------------------------------------------------------------------------
// Phase 2, column-normalised variants for run outputs (YumaRust yumas.py:
// 113-116 + 142-149, Yuma :227-258, Yuma2 :341-372): the bond matrix is
// normalised over every validator of a miner column each epoch, so a block
// owns whole columns — all V rows of a 16-miner strip (one block per strip
// and scenario: 256 blocks at 4096 miners, where k_bonds' 64-miner columns
// give 64) — and walks the epochs with the strip's bond state in registers
// and the inputs of the next P epochs in flight, like k_bonds_elem.
// Layout: 512 threads; lane (cq, rr) = (lane >> 4, lane & 15) of wave w owns
// miners 4 cq .. 4 cq + 3 of rows rr + 16 w + 128 i (i < R), so the 16 rows of
// a column quad are one DPP row. Column sums (Σ_v S·W_b, and YumaRust's
// Σ_v B_ema): per-thread rows in order, the DPP row tree (wsum16), then the
// 8 waves in order through LDS; every lane ends with the same bits. The LDS
// hand-off waits for LDS traffic only (lds_barrier), so the epoch prefetch
// ring stays in flight across it. Dividend partials per (row, 16-miner
// strip): [slice][strip][V], k_finalize adds the strips.
// ---------------------------------------------------------------------------
constexpr int kCnStrip = 16;  // miners per column-normalised block
constexpr int kCnDB = 32;     // k_bonds_cn: epochs of dividend partials parked in LDS per flush


// Sum over the NW waves (in order) of per-wave column partials: wave w's DPP
// row tree result for the 16 strip columns sits in red[w][0..15].
template <int NW>
__device__ __forceinline__ void cn_wave_sums(float (&x)[4], float (*red)[kCnStrip], int cq, int rr,
                                             int wave) {
#pragma unroll
  for (int c = 0; c < 4; ++c) x[c] = wsum16(x[c]);
  if constexpr (NW == 1) return;  // one wave holds the whole column
  if (rr == 0) *reinterpret_cast<float4*>(&red[wave][cq * 4]) = make_float4(x[0], x[1], x[2], x[3]);
  lds_barrier();
  float4 a = *reinterpret_cast<const float4*>(&red[0][cq * 4]);
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    const float4 b = *reinterpret_cast<const float4*>(&red[w][cq * 4]);
    a.x = a.x + b.x;
    a.y = a.y + b.y;
    a.z = a.z + b.z;
    a.w = a.w + b.w;
  }
  x[0] = a.x;
  x[1] = a.y;
  x[2] = a.z;
  x[3] = a.w;
}

template <int VARIANT, int R, int P, int NW = 8, bool RQ = false>
__global__ __launch_bounds__(64 * NW, 1) void k_bonds_cn(BondArgs A) {
  constexpr bool RUST = VARIANT == YUMA_VARIANT_RUST, YUMA2 = VARIANT == YUMA_VARIANT_YUMA2;
  constexpr int RS = 16 * NW;  // row stride between a lane's rows
  __shared__ __attribute__((aligned(16))) float red[2][NW][kCnStrip];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cq = lane >> 4, rr = lane & 15;
  // Strips 2k and 2k + 1 read the two halves of every 128-byte line of their
  // rows, and blocks b, b + 8 run on one XCD (round-robin dispatch): pair
  // them there, or each XCD's L2 fetches the whole line for its half (PMC:
  // 8.5 GB read per c2 launch for 4.2 GB of W)
  int strip = blockIdx.x % A.cblocks;
  if (strip < (A.cblocks & ~15)) strip = (strip & ~15) | ((strip & 7) << 1) | ((strip >> 3) & 1);
  const int n = blockIdx.x / A.cblocks;
  const int N = A.N, V = A.V, M = A.M;
  const long long VM = (long long)V * M;
  const int m = strip * kCnStrip + cq * 4;
  const bool colok = m < M;  // M % 4 == 0: a column quad is wholly in or out
  const int mc = colok ? m : M - 4;
  const int row0 = rr + 16 * wave;
  // every parameter read once into registers (a load inside the epoch loop
  // would wait on the prefetch ring)
  const yuma_params_t& pg = A.prm[n];
  const bool liquid = pg.liquid_mode != YUMA_LIQUID_OFF;
  const float p_ba = pg.bond_alpha, p_omba = pg.one_minus_bond_alpha;
  const float p_pen = pg.bond_penalty, p_ompen = pg.one_minus_bond_penalty;

  float B[R][4];
  bool has_old;
  {
    const float* src = A.t0 == 0 ? A.B_init : A.Bstate;
    has_old = src != nullptr;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = row0 + RS * i;
      if (has_old && row < V && colok)
        load4<true>(src + n * VM + (long long)row * M, m, M, B[i]);
      else
#pragma unroll
        for (int c = 0; c < 4; ++c) B[i][c] = 0.0f;
    }
  }
  // Yuma2: the previous epoch's normalised weights (yumas.py:299-300, 328)
  float Wp[R][4];
  bool have_wp = false;
  if constexpr (YUMA2) {
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) Wp[i][c] = 0.0f;
    if (A.t0 == 0) {
      if (A.Wprev_init != nullptr) {
        have_wp = true;
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const int row = row0 + RS * i;
          if (row < V && colok) load4<true>(A.Wprev_init + n * VM + (long long)row * M, m, M, Wp[i]);
        }
      }
    } else {
      have_wp = true;
      const long long ps = (long long)(A.t0 - 1) * N + n;
      const long long pw = A.wsh ? (long long)(A.t0 - 1) : ps;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = row0 + RS * i;
        if (row < V && colok) {
          float x[4];
          load4<true>(A.W + pw * VM + (long long)row * M, m, M, x);
          const float d = A.rsd[ps * V + row];
#pragma unroll
          for (int c = 0; c < 4; ++c) Wp[i][c] = x[c] / d;
        }
      }
    }
  }

  // the inputs of the next P epochs in flight: W rows, row sums, k_rowsum's
  // screened RN(1 / row sum) (RQ), stakes, and the strip's consensus,
  // incentive and (liquid) bond_alpha; YumaRust also its rank R, which is its
  // first bond column sum: B_sum = Σ_v S·Wc (yumas.py:113-114) is R's
  // expression (:103), formed once by the rank pass
  float rw[P][R][4], rd[P][R], rq[P][R], rsn[P][R], rcc[P][4], ri[P][4], rba[P][4], rrk[P][4];
  auto fetch = [&](int k, int t) {
    const long long slice = (long long)t * N + n;
    const long long isl = A.wsh ? (long long)t : slice;
    const float* Wt = A.W + isl * VM;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int rr_ = min(row0 + RS * i, V - 1);
      const float4 x = *reinterpret_cast<const float4*>(Wt + (long long)rr_ * M + mc);
      rw[k][i][0] = x.x;
      rw[k][i][1] = x.y;
      rw[k][i][2] = x.z;
      rw[k][i][3] = x.w;
      rd[k][i] = A.rsd[slice * V + rr_];
      rsn[k][i] = A.sn[slice * V + rr_];
      // the reciprocal alone (rq4.y): a 16-byte rq4 load made the compiler
      // copy it out of the tuple right after the load (k_bonds_elem RQ)
      if constexpr (RQ) rq[k][i] = reinterpret_cast<const float*>(A.rq4)[(isl * V + rr_) * 4 + 1];
    }
    load4c<true>(A.C + slice * M, 0, 1, m, M, rcc[k]);
    load4c<true>(A.I + slice * M, 0, 1, m, M, ri[k]);
    if (liquid) load4c<true>(A.ba + slice * M, 0, 1, m, M, rba[k]);
    if (RUST) load4c<true>(A.R + slice * M, 0, 1, m, M, rrk[k]);
  };
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (A.t0 + k < A.t1) fetch(k, A.t0 + k);

  // RN(1 / d[c]) of the lane's four column divisors (the column sums; every
  // lane of a column quad holds the same bits): lane c of each lane quad
  // divides once and the quad takes the four results by DPP broadcast, one
  // IEEE division per lane instead of four
  const int qsel = lane & 3;
  auto col_rcp = [&](const float (&d)[4], RowDiv (&cd)[4]) {
    const float dm = qsel == 0 ? d[0] : qsel == 1 ? d[1] : qsel == 2 ? d[2] : d[3];
    const float rm = 1.0f / dm;
    const float r0 = dpp_f<0x00>(rm), r1 = dpp_f<0x55>(rm), r2 = dpp_f<0xAA>(rm), r3 = dpp_f<0xFF>(rm);
    const float r[4] = {r0, r1, r2, r3};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float ad = fabsf(d[c]);
      cd[c] = {d[c], r[c], ad >= 0x1p-60f && ad <= 0x1p60f};
    }
  };

  // Dividend partials parked per wave in LDS (DB epochs x R row sets x the
  // wave's 16 rows) and written as 64-byte row runs when the buffer fills or
  // the launch ends: no global store of a 4-byte partial inside the epoch loop
  // (the history-less scan's LDS parking: c4 bonds 1.50 -> 1.41 ms)
  constexpr int DB = R <= 2 ? kCnDB : 2 * kCnDB / R;  // 32 KiB per block
  __shared__ __attribute__((aligned(16))) float dpark[NW * DB * R * 16];
  float* dpb = dpark + wave * (DB * R * 16);
  int tq = A.t0;  // first epoch held in the wave's buffer
  auto flush_d = [&](int t) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int ne = (t - tq + 1) * R * 4;  // 16-byte pieces: (epoch, row set, row quad)
    for (int j = lane; j < ne; j += 64) {
      const int q4 = j & 3, i = (j >> 2) % R, e = (j >> 2) / R;
      const int r = 16 * wave + RS * i + 4 * q4;
      float* dst = A.dpart + (((long long)(tq + e) * N + n) * A.cblocks + strip) * V + r;
      const float* src = dpb + j * 4;
      if ((V & 3) == 0 && r + 3 < V) {
        *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
      } else {
        for (int q = 0; q < 4; ++q)
          if (r + q < V) dst[q] = src[q];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    tq = t + 1;
  };

  int par = 0;  // LDS buffer of this epoch's first column sum
  for (int tb = A.t0; tb < A.t1; tb += P) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int t = tb + k;
      if (t >= A.t1) break;
      const long long slice = (long long)t * N + n;
      float bac[4], omba[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bac[c] = liquid ? rba[k][c] : p_ba;
        omba[c] = liquid ? 1.0f - rba[k][c] : p_omba;
      }
      // normalised weights (yumas.py:186), padding rows / columns zero. RQ:
      // Markstein's correction from k_rowsum's screened reciprocal (the
      // screen covers the row's every weight: no per-element guard; a NaN
      // sends the wave to IEEE division, the same values)
      float wn[R][4], s[R];
      {
        bool slow = false;
#pragma unroll
        for (int i = 0; i < R; ++i) {
          if constexpr (RQ) {
            const float d = rd[k][i], r = rq[k][i];
            slow |= r != r;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float x = rw[k][i][c];
              const float q = x * r;
              const float e = fmaf(-d, q, x);
              const float q1 = fmaf(e, r, q);
              wn[i][c] = x == 0.0f ? q : q1;
            }
          } else {
            const RowDiv rdv = row_div(rd[k][i]);
#pragma unroll
            for (int c = 0; c < 4; ++c) wn[i][c] = div_fast(rw[k][i][c], rdv, slow);
          }
        }
        if (__any(slow)) {
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) wn[i][c] = rw[k][i][c] / rd[k][i];
        }
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const bool live = row0 + RS * i < V;
        s[i] = live ? rsn[k][i] : 0.0f;
#pragma unroll
        for (int c = 0; c < 4; ++c) wn[i][c] = (live && colok) ? wn[i][c] : 0.0f;
      }
      // instantaneous bonds: S·W_b (Yuma, Yuma2: W_b = (1-β) W + β Wc;
      // YumaRust: S·Wc) over their column sums. The clip by v_minimum: C is a
      // quantised level >= +0, so its -0 < +0 order gives torch.min's bits
      float num[R][4], csum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float src = (YUMA2 && have_wp) ? Wp[i][c] : wn[i][c];
          const float wc = vmin(src, rcc[k][c]);
          const float wb = RUST ? wc : p_ompen * src + p_pen * wc;
          num[i][c] = s[i] * wb;
          csum[c] = csum[c] + num[i][c];
        }
      if constexpr (YUMA2) {
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c) Wp[i][c] = wn[i][c];
        have_wp = true;
      }
      float ic[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) ic[c] = ri[k][c];
      if constexpr (RUST) {
#pragma unroll
        for (int c = 0; c < 4; ++c) csum[c] = rrk[k][c] + 1e-6f;  // B / (B.sum(0) + 1e-6)
      }
      if (t + P < A.t1) fetch(k, t + P);  // slot k consumed: refill it
      if constexpr (!RUST) {
        cn_wave_sums<NW>(csum, red[par], cq, rr, wave);
        par ^= 1;
      }
      float ema[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      {
        RowDiv cd[4];
        col_rcp(csum, cd);
        float bi[R][4];
        bool slow = false;
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c) bi[i][c] = div_fast(num[i][c], cd[c], slow);
        // the fast path's quotients are finite (operands inside the guard):
        // nan_to_num is the identity there
        if (__any(slow)) {
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) bi[i][c] = nan_to_num(num[i][c] / cd[c].d, 0.0f);
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const bool live = row0 + RS * i < V;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float b = bi[i][c];
            float e = has_old ? bac[c] * b + omba[c] * B[i][c] : b;
            e = (live && colok) ? e : 0.0f;
            B[i][c] = e;
            ema[c] = ema[c] + e;
          }
        }
      }
      if constexpr (RUST) {  // B_ema / (Σ_v B_ema + 1e-6), nan_to_num (yumas.py:147-149)
        cn_wave_sums<NW>(ema, red[par], cq, rr, wave);
        par ^= 1;
#pragma unroll
        for (int c = 0; c < 4; ++c) ema[c] = ema[c] + 1e-6f;
        RowDiv cd[4];
        col_rcp(ema, cd);
        float q[R][4];
        bool slow = false;
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c) q[i][c] = div_fast(B[i][c], cd[c], slow);
        if (__any(slow)) {
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) q[i][c] = nan_to_num(B[i][c] / cd[c].d, 0.0f);
        }
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c) B[i][c] = q[i][c];
      }
      has_old = true;
      // bond history and the dividend partials Σ_{m in strip} B·I (the four
      // column quads of a row: lanes l, l^16, l^32, l^48)
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = row0 + RS * i;
        if (A.B_hist != nullptr && row < V && colok)
          // plain (write-back) stores: the L2 of the XCD merges the paired
          // strips' 64-byte halves of each line (non-temporal stores wrote
          // 1.26x the history: PMC 5.65 -> 4.46 GB per c2 launch, same time)
          *reinterpret_cast<fvec4*>(A.B_hist + slice * VM + (long long)row * M + m) =
              fvec4{B[i][0], B[i][1], B[i][2], B[i][3]};
        float d = 0.0f;
#pragma unroll
        for (int c = 0; c < 4; ++c) d = d + B[i][c] * ic[c];
        d = colok ? d : 0.0f;
        d = qsum4(d);
        if (cq == 0) dpb[((t - tq) * R + i) * 16 + rr] = d;
      }
      if (t - tq == DB - 1 || t == A.t1 - 1) flush_d(t);  // block-uniform
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = row0 + RS * i;
    if (row < V && colok) store4<true>(A.Bstate + n * VM + (long long)row * M, m, M, B[i]);
  }
}

// ---------------------------------------------------------------------------
// YumaRust above kRegRows validators: the bond column normalisation of an
// epoch (yumas.py:147-149) needs the column sums over every validator, which
// no workgroup holds, so each epoch is two launches over (scenario, 64-row
// block, 64-miner tile) blocks:
//   k_rust_big_ema   B = nan_to_num(S·Wc / (R + 1e-6)) (:113-116; the
//                    column sum B_sum is R's expression, :103), the EMA
//                    α·B + (1-α)·B_old or B (:142-145) into the bond state,
//                    and the block's column partial sums of it;
//   k_rust_big_norm  Z = the partials in row-block order + 1e-6, B_ema / Z
//                    with nan_to_num, the bond history, and the per-tile
//                    dividend partials Σ B·I ([slice][tile][V], k_finalize).
// ---------------------------------------------------------------------------
constexpr int kRustBigRows = 64;  // rows per block: 16 row groups x 4
template <bool VEC>
__global__ __launch_bounds__(256) void k_rust_big_ema(BondArgs A, int t, float* __restrict__ cpart) {
  __shared__ float4 red[4 * 16];
  const Lay L = lay();
  const int tile = blockIdx.x % A.tiles;
  const int rb = (blockIdx.x / A.tiles) % A.rowblocks;
  const int n = blockIdx.x / (A.tiles * A.rowblocks);
  const int N = A.N, V = A.V, M = A.M;
  const long long VM = (long long)V * M;
  const long long slice = (long long)t * N + n;
  const int m = tile * kTileM + L.c4 * 4;
  const yuma_params_t& pg = A.prm[n];
  const bool liquid = pg.liquid_mode != YUMA_LIQUID_OFF;
  // the bond state before this epoch: the caller's B_init (or none) at epoch 0
  const float* Bsrc = (t == 0) ? A.B_init : A.Bstate;
  const bool has_old = Bsrc != nullptr;
  float Cc[4], Rc[4], bac[4], omba[4];
  load4c<VEC>(A.C + slice * M, 0, 1, m, M, Cc);
  load4c<VEC>(A.R + slice * M, 0, 1, m, M, Rc);
  if (liquid) {
    load4c<VEC>(A.ba + slice * M, 0, 1, m, M, bac);
#pragma unroll
    for (int c = 0; c < 4; ++c) omba[c] = 1.0f - bac[c];
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      bac[c] = pg.bond_alpha;
      omba[c] = pg.one_minus_bond_alpha;
    }
  }
  const float* Wt = A.W + (A.wsh ? (long long)t : slice) * VM;
  float csum[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int i = 0; i < kRustBigRows / 16; ++i) {
    const int row = rb * kRustBigRows + L.g + 16 * i;
    float x[4], e[4];
    load4c<VEC>(Wt, row, V, m, M, x);
    const int rr = row < V ? row : V - 1;
    const RowDiv rdv = row_div(A.rsd[slice * V + rr]);
    const float sv = A.sn[slice * V + rr];
    float bo[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (has_old && row < V) load4<VEC>(Bsrc + n * VM + (long long)row * M, m, M, bo);
    float bi[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float wn = div_rn(x[c], rdv);
      const float wc = tmin(wn, Cc[c]);
      bi[c] = nan_to_num((sv * wc) / (Rc[c] + 1e-6f), 0.0f);
      e[c] = has_old ? bac[c] * bi[c] + omba[c] * bo[c] : bi[c];
      e[c] = (row < V && m + c < M) ? e[c] : 0.0f;
      csum[c] = csum[c] + e[c];
    }
    if (row < V) {
      if (A.Binst_out != nullptr) store4<VEC>(A.Binst_out + slice * VM + (long long)row * M, m, M, bi);
      store4<VEC>(A.Bstate + n * VM + (long long)row * M, m, M, e);
    }
  }
  col_reduce4<4>(csum, red, L);
  if (L.g == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) cpart[((long long)n * A.rowblocks + rb) * M + m + c] = csum[c];
}

template <bool VEC>
__global__ __launch_bounds__(256) void k_rust_big_norm(BondArgs A, int t, const float* __restrict__ cpart) {
  const Lay L = lay();
  const int tile = blockIdx.x % A.tiles;
  const int rb = (blockIdx.x / A.tiles) % A.rowblocks;
  const int n = blockIdx.x / (A.tiles * A.rowblocks);
  const int N = A.N, V = A.V, M = A.M;
  const long long VM = (long long)V * M;
  const long long slice = (long long)t * N + n;
  const int m = tile * kTileM + L.c4 * 4;
  float Z[4], Ic[4];
  load4c<VEC>(A.I + slice * M, 0, 1, m, M, Ic);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int mc = min(m + c, M - 1);
    float z = 0.0f;
    for (int b = 0; b < A.rowblocks; ++b) z = z + cpart[((long long)n * A.rowblocks + b) * M + mc];
    Z[c] = z + 1e-6f;
  }
#pragma unroll
  for (int i = 0; i < kRustBigRows / 16; ++i) {
    const int row = rb * kRustBigRows + L.g + 16 * i;
    float e[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (row < V) load4<VEC>(A.Bstate + n * VM + (long long)row * M, m, M, e);
#pragma unroll
    for (int c = 0; c < 4; ++c) e[c] = nan_to_num(e[c] / Z[c], 0.0f);
    if (row < V) {
      store4<VEC>(A.Bstate + n * VM + (long long)row * M, m, M, e);
      if (A.B_hist != nullptr) store4<VEC>(A.B_hist + slice * VM + (long long)row * M, m, M, e);
    }
    float d = 0.0f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m + c < M) d = d + e[c] * Ic[c];
    d = sum_row16(d);
    if (L.c4 == 0 && row < V) A.dpart[dp_index(slice, tile, row, A.tiles, V)] = d;
  }
}

// ---------------------------------------------------------------------------
// Phase 2, element-wise variants (Yuma3 yumas.py:452-472, Yuma4 :570-586):
// a software-pipelined scan. Each thread owns R rows x 4 miners of the bond
// tile in registers and keeps the inputs of the next P epochs in flight
// (a register ring refilled as each epoch is consumed), so the per-epoch HBM
// latency is hidden behind P-1 epochs of work.
// Yuma / Yuma2 (yumas.py:227-258, :341-372) run here too once the rank pass
// has formed their bond column sums csb = Σ_v S·W_b (k_rank_s BCS): then
// B = nan_to_num(S·W_b / csb) and the EMA are element-wise, and the scan
// reads each miner's C and csb beside its incentive (Yuma2 keeps the
// previous epoch's normalised W in registers as its W_prev).
// ---------------------------------------------------------------------------
// Block shape: BS threads over CB miners x (G = BS / (CB/4)) rows per pass,
// R passes, i.e. a block owns G R rows x CB miners of the bond state; lane
// quads run along a row (CB/4 lanes per row), so a wave instruction moves
// 4 rows x 256 B (CB = 64) or 1 row x 1 KiB (CB >= 256). The dividend partial
// of each 64-miner tile is the 16-lane DPP sum of one DPP row in every shape.
template <int VARIANT, int R, bool VEC, int P, bool VECI, bool NT = false, int BS = 256, int CB = 64,
          int DPL = DP_TV, bool RQ = false>
__global__ __launch_bounds__(BS, 1) void k_bonds_elem(BondArgs A) {
  constexpr int LPR = CB / 4, G = BS / LPR;
  static_assert(CB % 64 == 0 && BS % LPR == 0, "a 16-lane DPP row must cover one 64-miner tile");
  const int cq = threadIdx.x % LPR, lane = threadIdx.x & 63;
  const int cb = blockIdx.x % A.cblocks;
  const int rb = (blockIdx.x / A.cblocks) % A.rowblocks;
  const int n = blockIdx.x / (A.cblocks * A.rowblocks);
  const int N = A.N, V = A.V, M = A.M;
  const long long VM = (long long)V * M;
  const int m = cb * CB + cq * 4;
  const int tile = m >> 6;  // this lane's 64-miner tile (dividend partials)
  const int g = threadIdx.x / LPR;
  // every parameter is read once into registers: a global load inside the
  // epoch loop would make the compiler drain the prefetch ring (vmcnt(0))
  const yuma_params_t& pg = A.prm[n];
  const bool liquid = pg.liquid_mode != YUMA_LIQUID_OFF;
  const int reset_mode = pg.reset_mode, reset_epoch = pg.reset_epoch, reset_index = pg.reset_index;
  const bool reset_all = (pg.flags & YUMA_FLAG_RESET_ALL_COLUMNS) != 0;
  const float p_bond_alpha = pg.bond_alpha, p_omba = pg.one_minus_bond_alpha;
  const float p_maxint = pg.maxint, p_capacity_alpha = pg.capacity_alpha, p_decay_keep = pg.decay_keep;
  const float p_pen = pg.bond_penalty, p_ompen = pg.one_minus_bond_penalty;
  constexpr bool COLNORM = VARIANT == YUMA_VARIANT_YUMA1 || VARIANT == YUMA_VARIANT_YUMA2;
  constexpr bool YUMA2 = VARIANT == YUMA_VARIANT_YUMA2;
  static_assert(VARIANT != YUMA_VARIANT_RUST, "YumaRust renormalises B_ema over every validator (k_bonds_cn)");
  const int row0 = rb * G * R + g;
  // the conditional reset's test (C of the previous epoch at the reset
  // column), read before the epoch loop: a load in the loop's rare reset
  // branch made the waitcnt pass drain the whole prefetch ring (vmcnt(0))
  // at every epoch, stores included. Resets are Yuma 3.x / 4 only.
  const bool zero_c = !COLNORM && reset_c_zero(A, n, reset_mode, reset_all, reset_epoch, reset_index);

  float B[R][4];
  bool has_old;
  {
    const float* src = A.t0 == 0 ? A.B_init : A.Bstate;
    has_old = src != nullptr;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = row0 + G * i;
      if (has_old && row < V)
        load4<VEC>(src + n * VM + (long long)row * M, m, M, B[i]);
      else
#pragma unroll
        for (int c = 0; c < 4; ++c) B[i][c] = 0.0f;
    }
  }
  // Yuma2: the previous epoch's normalised weights (yumas.py:299-300, 328):
  // the caller's W_prev at epoch 0 (none: W itself), else W[t0 - 1] / its row sums
  float Wp[COLNORM ? R : 1][4];
  bool have_wp = false;
  if constexpr (YUMA2) {
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) Wp[i][c] = 0.0f;
    if (A.t0 == 0) {
      if (A.Wprev_init != nullptr) {
        have_wp = true;
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const int row = row0 + G * i;
          if (row < V) load4<VEC>(A.Wprev_init + n * VM + (long long)row * M, m, M, Wp[i]);
        }
      }
    } else {
      have_wp = true;
      const long long ps = (long long)(A.t0 - 1) * N + n;
      const long long pw = A.wsh ? (long long)(A.t0 - 1) : ps;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = row0 + G * i;
        if (row < V) {
          float x[4];
          load4<VEC>(A.W + pw * VM + (long long)row * M, m, M, x);
          const float d = A.rsd[ps * V + row];
#pragma unroll
          for (int c = 0; c < 4; ++c) Wp[i][c] = x[c] / d;
        }
      }
    }
  }

  float rw[P][R][4], rd[P][R], rsn[P][R], ri[P][4], rba[P][4];
  float rcc[COLNORM ? P : 1][4], rcs[COLNORM ? P : 1][4], rcr[COLNORM ? P : 1][4];  // Yuma / Yuma2: C, csb, csr
  float rrq[RQ ? P : 1][RQ ? R : 1];  // RQ: k_rowsum's screened RN(1 / row sum) (rq4.y)
  // DP_QTE: the quad partials of up to kQBuf epochs parked in LDS (one float
  // per wave row and epoch) and written out as contiguous runs when the
  // buffer fills or the launch ends: no global store inside the epoch loop
  // (partial stores cost the read stream far more than their bytes:
  // [slice][tile][V] stores 0.24 ms at c4, 16-epoch 64-byte runs still 0.16)
  constexpr int kQBuf = 256, NWB = BS / 64;
  __shared__ float qbuf[DPL == DP_QTE ? NWB * R * kQBuf : 1];
  int tq = A.t0;  // first epoch held in qbuf
  // a duplicate scenario of a rank class reads its representative's column sums
  // (the rank pass skips duplicate slices; k_incentive copies R, not csb / csr)
  const int ncs = (COLNORM && A.csrep != nullptr) ? A.csrep[n] : n;
  auto fetch = [&](int k, int t) {
    const long long slice = (long long)t * N + n;
    const long long cslice = (long long)t * N + ncs;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int rr = min(row0 + G * i, V - 1);
      // the one-row history-less scan streams each W slice exactly once
      // (rowsum / consensus / rank read it in their own launches): non-
      // temporal loads (c4 bonds 1.63 -> 1.50 ms, same box)
      load4c<VEC, DPL == DP_QTE>(A.W + (A.wsh ? (long long)t : slice) * VM, rr, V, m, M, rw[k][i]);
      rd[k][i] = A.rsd[slice * V + rr];
      rsn[k][i] = A.sn[slice * V + rr];
      // RQ: the screened reciprocal alone (rq4.y). (One 16-byte rq4 load for
      // all three made the compiler copy the reciprocal out of the load's
      // register tuple right after the load, waiting vmcnt(0) at every
      // epoch: c4 bonds 1.25 -> 1.58 ms.)
      if constexpr (RQ) rrq[k][i] = reinterpret_cast<const float*>(A.rq4)[((A.wsh ? (long long)t : slice) * V + rr) * 4 + 1];
    }
    // columns >= M never reach an output
    if (VECI) {
      load4c<true>(A.I + slice * M, 0, 1, m, M, ri[k]);
      if (liquid) load4c<true>(A.ba + slice * M, 0, 1, m, M, rba[k]);
      if constexpr (COLNORM) {
        load4c<true>(A.C + slice * M, 0, 1, m, M, rcc[k]);
        load4c<true>(A.csb + cslice * M, 0, 1, m, M, rcs[k]);
        load4c<true>(A.csr + cslice * M, 0, 1, m, M, rcr[k]);
      }
    } else {
      vec4raw(A.I + slice * M, m, M, ri[k]);
      if (liquid) vec4raw(A.ba + slice * M, m, M, rba[k]);
      if constexpr (COLNORM) {
        vec4raw(A.C + slice * M, m, M, rcc[k]);
        vec4raw(A.csb + cslice * M, m, M, rcs[k]);
        vec4raw(A.csr + cslice * M, m, M, rcr[k]);
      }
    }
  };
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (A.t0 + k < A.t1) fetch(k, A.t0 + k);

  for (int tb = A.t0; tb < A.t1; tb += P) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int t = tb + k;
      if (t >= A.t1) break;
      const long long slice = (long long)t * N + n;
      if (!COLNORM && has_old && reset_mode != YUMA_RESET_NONE && t == reset_epoch &&
          (reset_all || (reset_index >= 0 && reset_index < M))) {
        bool fire = reset_mode == YUMA_RESET_ALWAYS;
        if (reset_mode == YUMA_RESET_IF_ZERO_CONSENSUS && t >= 1 && !reset_all) fire = zero_c;
        const int c = reset_index - m;
        if (fire && (reset_all || (c >= 0 && c < 4)))
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
              if (reset_all || cc == c) B[i][cc] = 0.0f;
      }
      float bac[4], omba[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        bac[c] = liquid ? rba[k][c] : p_bond_alpha;
        omba[c] = liquid ? 1.0f - rba[k][c] : p_omba;
      }
      // Yuma / Yuma2: every column of the wave passed the rank pass's
      // division screen (csr not NaN): Markstein division, finite quotients
      bool cfast = false;
      if constexpr (COLNORM) {
        bool ok = true;
#pragma unroll
        for (int c = 0; c < 4; ++c) ok &= rcr[k][c] == rcr[k][c];
        cfast = __all(ok);
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = row0 + G * i;
        // Signed zeros cannot show here: W = -0 gives wn = +0 instead of
        // -0 (div_fast_nz), and v_minimum / v_maximum order -0 < +0, but the
        // bond state starts at +0 and every -0 candidate (a purchase term of
        // -0, a clamp at 0) is added to a non-negative decayed bond or
        // clamped by a cap that is +0 or positive (the Yuma3 cap clamp keeps
        // tmin: a -0 stake makes cap = -0), so B and its history keep the
        // bits of the torch-order tmin / tmax / IEEE-division form.
        // (Yuma4 with the history stream keeps the compare/select forms:
        // same-box A/B, its scan ran 1.70 -> 1.81 ms with the short ones,
        // while Yuma3 gained 0.05 ms and the history-less c3 sweep 20 %.)
        // (Yuma / Yuma2 keep the sign-exact division and clip: there a
        // -0 weight can reach the bond state as S·W_b = -0.)
        constexpr bool SHORT = !COLNORM && !(VARIANT == YUMA_VARIANT_YUMA4 && NT);
        auto mn = [](float a, float b) { return SHORT ? vmin(a, b) : tmin(a, b); };
        auto mx = [](float a, float b) { return SHORT ? vmax(a, b) : tmax(a, b); };
        // (k_rowsum's screened reciprocal instead of the per-row one and the
        // per-element guard: c2 wide history scan 1.58 -> 1.70 ms, c4 1.63 ->
        // 1.73, same box; kept only in the issue-bound sweep scan k_bonds_grp)
        float wn[4];
        if constexpr (RQ) {
          // RN(w / rs) from k_rowsum's screened RN(1 / rs) with RowDiv's
          // correction and no per-element guard; a row that failed the
          // screen (NaN reciprocal) sends the wave to IEEE division
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float a = rw[k][i][c];
            const float q = a * rrq[k][i];
            const float e = fmaf(-rd[k][i], q, a);
            const float q1 = fmaf(e, rrq[k][i], q);
            wn[c] = SHORT ? q1 : (a == 0.0f ? q : q1);
          }
          if (__any(rrq[k][i] != rrq[k][i])) {
#pragma unroll
            for (int c = 0; c < 4; ++c) wn[c] = rw[k][i][c] / rd[k][i];
          }
        } else {
          const RowDiv rdv = row_div(rd[k][i]);
          bool slow = false;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            wn[c] = SHORT ? div_fast_nz(rw[k][i][c], rdv, slow) : div_fast(rw[k][i][c], rdv, slow);
          if (__any(slow)) {
#pragma unroll
            for (int c = 0; c < 4; ++c) wn[c] = rw[k][i][c] / rd[k][i];
          }
        }
        if constexpr (COLNORM) {
          // B = nan_to_num(S·W_b / Σ_v S·W_b), W_b = (1-β)·src + β·min(src, C)
          // (yumas.py:227-229; Yuma2 src = W_prev :341-343), then the EMA
          // α·B + (1-α)·B_old, or B itself without a bond state (:255-258)
          // (min: C is a quantised level >= +0, so v_minimum's -0 < +0 order
          // gives torch.min's bits)
          float num[4], b[4], wbv[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float src = (YUMA2 && have_wp) ? Wp[i][c] : wn[c];
            const float wc = vmin(src, rcc[k][c]);
            wbv[c] = p_ompen * src + p_pen * wc;
            num[c] = rsn[k][i] * wbv[c];
          }
          if (cfast) {
            // RN(num / csb) from RN(1 / csb) (RowDiv's correction; the screen
            // bounds every operand), a zero numerator keeping its sign
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float q = num[c] * rcr[k][c];
              const float e = fmaf(-rcs[k][c], q, num[c]);
              b[c] = num[c] == 0.0f ? q : fmaf(e, rcr[k][c], q);
            }
          } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) b[c] = nan_to_num(num[c] / rcs[k][c], 0.0f);
          }
          // the full outputs weight_for_bond / validator_bond (yumas.py:274-275)
          if (A.Wb_out != nullptr && row < V) store4<VEC>(A.Wb_out + slice * VM + (long long)row * M, m, M, wbv);
          if (A.Binst_out != nullptr && row < V) store4<VEC>(A.Binst_out + slice * VM + (long long)row * M, m, M, b);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            B[i][c] = has_old ? bac[c] * b[c] + omba[c] * B[i][c] : b[c];
            if (YUMA2) Wp[i][c] = wn[c];
          }
        } else if (VARIANT == YUMA_VARIANT_YUMA3) {
          const float cap = rsn[k][i] * p_maxint;
          const float ca = p_capacity_alpha * cap;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float rem = mx(cap - B[i][c], 0.0f);
            const float pc = mn(ca, rem);
            const float nb = p_decay_keep * B[i][c] + pc * wn[c];
            B[i][c] = tmin(nb, cap);  // cap = -0 (a -0 stake) must keep nb = +0
          }
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float bd = B[i][c] * omba[c];
            const float rem = mx(1.0f - bd, 0.0f);
            const float nb = bd + mn(bac[c] * wn[c], rem);
            B[i][c] = mn(nb, 1.0f);
          }
        }
        if (A.B_hist != nullptr && row < V) {
          float* hp = A.B_hist + slice * VM + (long long)row * M;
          if (NT && VEC) {  // write-once history: non-temporal stores
            if (m < M)
              __builtin_nontemporal_store(fvec4{B[i][0], B[i][1], B[i][2], B[i][3]},
                                          reinterpret_cast<fvec4*>(hp + m));
          } else {
            store4<VEC>(hp, m, M, B[i]);
          }
        }
        float d = 0.0f;
        // M % 4 == 0: a column quad is wholly in or out. (Not with the
        // history stream: there the lane branch cost the c2 scan 1.65 ->
        // 2.71 ms, same box.)
        if (VEC && !NT) {
          if (m < M)
#pragma unroll
            for (int c = 0; c < 4; ++c) d = d + B[i][c] * ri[k][c];
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (m + c < M) d = d + B[i][c] * ri[k][c];
        }
        d = wsum16(d);  // sum_row16's xor-butterfly tree, on DPP
        if constexpr (DPL == DP_QTE || DPL == DP_VQ) {
          // the wave holds one quad of this row (CB >= 256, LPR >= 64):
          // Q = (p0 + p1) + (p2 + p3) in every lane (xor butterflies pair
          // back, a + b == b + a)
          static_assert(LPR >= 64, "a quad partial needs one row per wave");
          float q = d + __shfl_xor(d, 16, 64);
          q = q + __shfl_xor(q, 32, 64);
          const int quad = m >> 8, nq = dp_quads(A.tiles);
          if constexpr (DPL == DP_QTE) {
            float* qb = qbuf + ((threadIdx.x >> 6) * R + i) * kQBuf;
            if (lane == 0) qb[t - tq] = q;
            if (t - tq == kQBuf - 1 || t == A.t1 - 1) {  // wave-uniform
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              float* dq = A.dpart + ((long long)(n * nq + quad) * V + row) * A.ep + tq;
              if (row < V && quad < nq)
                for (int e = lane; e <= t - tq; e += 64) dq[e] = qb[e];
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              if (i == R - 1) tq = t + 1;
            }
          } else if (lane == 0 && row < V && quad < nq) {
            A.dpart[(slice * V + row) * (long long)nq + quad] = q;
          }
        } else if ((lane & 15) == 0 && row < V && tile < A.tiles) {
          A.dpart[dp_index(slice, tile, row, A.tiles, V)] = d;
        }
      }
      has_old = true;
      if (YUMA2) have_wp = true;
      if (t + P < A.t1) fetch(k, t + P);
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = row0 + G * i;
    if (row < V) store4<VEC>(A.Bstate + n * VM + (long long)row * M, m, M, B[i]);
  }
}

// ---------------------------------------------------------------------------
// Phase 2 for parameter sweeps over ONE input trajectory (shared inputs,
// config c3), element-wise variants: a block runs the scan of K scenarios
// side by side over one 16 R-row x 64-miner tile of W. Every scenario of the
// sweep reads the same W[t]; W[t], the row sums and the normalised weights
// are loaded and divided once per K scenarios; each scenario keeps its own
// bond tile in registers and its own parameters, resets, liquid bond_alpha
// and dividend partials — the same operations in the same order as
// k_bonds_elem, so the same bits. The scan is bound by instruction issue,
// not by HBM (W is re-read from the caches; profiles/r03/c3sq), so the
// per-element work is cut to the bond update itself:
//  * the row division takes k_rowsum's RN(1/row sum) (rq4), NaN when some
//    weight or the row sum leaves the fast division's range: no per-row IEEE
//    reciprocal and no per-element guard (a wave whose rows are not all in
//    range divides in IEEE, same bits);
//  * blocks whose scenarios all use a fixed bond_alpha (LIQ = false) take
//    bond_alpha / 1 - bond_alpha as block-uniform operands; liquid (or mixed)
//    blocks the per-miner operands with the exact one_minus_bond_alpha
//    correction for their fixed-alpha scenarios (p_corr);
// History: round 3 K = 2 beat 1 / 3 / 4 / 8 (profiles/r03/ab/
// c3_scan_group_k.txt); packed-pair f32 math and an XCD-grouped block order
// lost. Round 4 also: the dividend partials parked in LDS (32 epochs per
// block, written by the block after a barrier) took it 6.73-6.78 -> 7.09-7.10 ms
// (profiles/r04/ab_round8.txt). Round 4 (rq4, R = 2, liquid split): K = 4 at 3 waves / SIMD (144 /
// 168 VGPRs, 6 VGPRs spilled for Yuma 4) 6.90-6.97 ms against 7.03-7.22 for
// K = 2 at 4 waves; K = 4 at 2 waves 8.96, K = 4 with R = 1 9.36; the
// scenario groups of one W slab in consecutive blocks 7.15-7.17
// (profiles/r04/ab_round3.txt, ab_round4.txt).
// ---------------------------------------------------------------------------
constexpr int kGrpWaves = 3;  // minimum waves per SIMD of the sweep scan
constexpr bool kGrpPark = true;  // dividend partials parked per wave in LDS
constexpr int kGrpDB = 32;       // ... epochs per flush
// LQ: 0 = every scenario of the block has a fixed bond_alpha (block-uniform
// operands), 2 = every one is liquid (per-miner bond_alpha), 1 = mixed.
// BND (Yuma 4): the wave's bond state starts in [0, 1] (or NaN), every
// scenario's bond_alpha and 1 - bond_alpha lie in [0, 1] and no weight of the
// wave's rows is negative over the launch (k_bonds_grp decides it per wave).
// Then Bd = B (1 - a) is in [0, 1], so 1 - Bd >= +0 and the clamp(min = 0)
// of the remaining capacity is the identity; and Bd + min(a W, RN(1 - Bd))
// rounds to at most 1 (1 - Bd is exact for Bd >= 1/2, otherwise within
// 2^-25 of it, below the half-ulp of 1 above 1), so the clamp(max = 1) is the
// identity too and B stays in [0, 1]: the update drops both clamps with the
// same bits (yumas.py:574-586). NaN operands propagate alike in both forms.
template <int VARIANT, int K, int R, int P, int LQ, bool HIST, bool BND = false>
__device__ __forceinline__ void grp_scan(const BondArgs& A, unsigned liquid_mask, float* dpark) {
  constexpr bool LIQ = LQ != 0;
  constexpr int G = 16;
  const Lay L = lay();
  const int tile = blockIdx.x % A.tiles;
  const int rb = (blockIdx.x / A.tiles) % A.rowblocks;
  const int n0 = (blockIdx.x / (A.tiles * A.rowblocks)) * K;
  const int N = A.N, V = A.V, M = A.M;
  const long long VM = (long long)V * M;
  const int m = tile * kTileM + L.c4 * 4;
  const int row0 = rb * G * R + L.g;
  const int nk = N - n0 < K ? N - n0 : K;  // scenarios of this block (block-uniform)

  // every parameter read once into registers (a load inside the epoch loop
  // would wait on the prefetches, see k_bonds_elem)
  float p_ba[K], p_omba[K], p_maxint[K], p_ca[K], p_dk[K];
  // bond resets (simulation_utils.py:62-88) decided before the epoch loop:
  // p_repoch[k] = the epoch whose update starts from the reset state, or -1
  // when scenario k's reset never fires in this launch (mode, index range,
  // the conditional test on the previous epoch's C: reset_c_zero); rcols =
  // the columns of this lane it zeroes, 4 bits per scenario
  int p_repoch[K];
  unsigned rcols = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const yuma_params_t& pg = A.prm[min(n0 + k, N - 1)];
    p_ba[k] = pg.bond_alpha;
    p_omba[k] = pg.one_minus_bond_alpha;
    p_maxint[k] = pg.maxint;
    p_ca[k] = pg.capacity_alpha;
    p_dk[k] = pg.decay_keep;
    const int mode = pg.reset_mode, index = pg.reset_index;
    const bool all = (pg.flags & YUMA_FLAG_RESET_ALL_COLUMNS) != 0;
    bool fire = k < nk && mode != YUMA_RESET_NONE && (all || (index >= 0 && index < M));
    if (mode == YUMA_RESET_IF_ZERO_CONSENSUS && pg.reset_epoch >= 1 && !all)
      fire = fire && reset_c_zero(A, n0 + k, mode, all, pg.reset_epoch, index);
    else if (mode != YUMA_RESET_ALWAYS)
      fire = false;
    p_repoch[k] = fire ? pg.reset_epoch : -1;
    const int c = index - m;
    if (fire) rcols |= (all ? 0xFu : (c >= 0 && c < 4 ? 1u << c : 0u)) << (4 * k);
  }

  float B[K][R][4];
  bool has_old;
  {
    const float* src = A.t0 == 0 ? A.B_init : A.Bstate;
    has_old = src != nullptr;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const int row = row0 + G * i;
        if (has_old && k < nk && row < V)
          load4<true>(src + (n0 + k) * VM + (long long)row * M, m, M, B[k][i]);
        else
#pragma unroll
          for (int c = 0; c < 4; ++c) B[k][i][c] = 0.0f;
      }
  }

  // Addressing: per-lane pointers (load4c's clamped row and column folded
  // in) advanced by a constant stride per epoch (one v_lshl_add_u64 each);
  // block-uniform bases instead keep ~12 64-bit pointers live in SGPRs and
  // spill them (k_bonds_grp<4,2,1,2>: 148 SGPR spills, 507 v_readlane /
  // v_writelane against 88).
  const int mc = m < M ? m : M - 4;
  const long long sM = (long long)N * M, sD = (long long)N * A.tiles * V;

  // the shared inputs of the next P epochs in flight: W rows and their
  // {row sum, reciprocal, stake} (k_rowsum's rq4, per input epoch)
  float rw[P][R][4], rd[P][R], rq[P][R], rsn[P][R];
  const float* fW[R];  // next epoch to fetch
  const float4* fQ[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int rr = min(row0 + G * i, V - 1);
    fW[i] = A.W + (long long)A.t0 * VM + (long long)rr * M + mc;
    fQ[i] = A.rq4 + (long long)A.t0 * V + rr;
  }
  // (the record's three fields as three 4-byte loads, the reciprocal with the
  // non-temporal hint so that they are not merged into one: from one 16-byte
  // load the compiler copied the fields out of the load's register tuple
  // right after issuing it and waited vmcnt(0) there, every epoch)
  // (Unconditional refills from clamped addresses instead of the skipped
  // loads past the last epoch: 149-168 VGPRs and spills, the latch's drain
  // stayed.)
  // Every ring load is unconditional: the pointers hold the next epoch to
  // fetch, clamped at the last one (a fetch past the end re-reads it), and
  // advance only while epochs remain (`more`, block-uniform). (Loads skipped
  // on some path left the waitcnt pass no count for the older ones but
  // vmcnt(0).)
  auto fetch = [&](int kk, bool more) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float4 x = *reinterpret_cast<const float4*>(fW[i]);
      rw[kk][i][0] = x.x;
      rw[kk][i][1] = x.y;
      rw[kk][i][2] = x.z;
      rw[kk][i][3] = x.w;
      const float* q = reinterpret_cast<const float*>(fQ[i]);
      rd[kk][i] = q[0];
      rq[kk][i] = __builtin_nontemporal_load(q + 1);
      rsn[kk][i] = q[2];
      fW[i] += more ? VM : 0;
      fQ[i] += more ? V : 0;
    }
  };
  // per scenario: incentive (and liquid bond_alpha) of the epoch in use, each
  // refilled with the next epoch's as soon as it is consumed
  float ri[K][4], rba[K][4];
  const float* fI[K];
  const float* fB[K];
  float* pD[K];  // this epoch's dividend partials
  float* pH[K];  // this epoch's bond history, if stored
  constexpr bool hist = HIST;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const long long s0 = (long long)A.t0 * N + min(n0 + k, N - 1);
    fI[k] = A.I + s0 * M + mc;
    fB[k] = A.ba + s0 * M + mc;
    pD[k] = A.dpart + (s0 * A.tiles + tile) * V + row0;
    pH[k] = hist ? A.B_hist + s0 * VM + (long long)row0 * M + m : nullptr;
  }
  auto fetch_s = [&](int k, bool more) {  // as fetch: unconditional, clamped
    const float4 x = *reinterpret_cast<const float4*>(fI[k]);
    ri[k][0] = x.x;
    ri[k][1] = x.y;
    ri[k][2] = x.z;
    ri[k][3] = x.w;
    if (LQ == 2 || (LQ == 1 && ((liquid_mask >> k) & 1u))) {
      const float4 y = *reinterpret_cast<const float4*>(fB[k]);
      rba[k][0] = y.x;
      rba[k][1] = y.y;
      rba[k][2] = y.z;
      rba[k][3] = y.w;
    }
    fI[k] += more ? sM : 0;
    fB[k] += more ? sM : 0;
  };
#pragma unroll
  for (int kk = 0; kk < P; ++kk) fetch(kk, A.t0 + kk + 1 < A.t1);
#pragma unroll
  for (int k = 0; k < K; ++k) fetch_s(k, A.t0 + 1 < A.t1);
  // Liquid blocks: a fixed-alpha scenario keeps bond_alpha in rba for the
  // whole scan, and one_minus_bond_alpha = (1 - bond_alpha) + p_corr. Both
  // terms of p_corr are fp32 roundings of 1 - bond_alpha within 2^-25 of each
  // other, so their difference is exact (Sterbenz, or one of them is 0) and
  // adding it back to 1 - bond_alpha gives one_minus_bond_alpha bit for bit
  // (tests/test_host.py::test_grp_one_minus_alpha_correction).
  float p_corr[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    p_corr[k] = 0.0f;
    if (LIQ && !((liquid_mask >> k) & 1u)) {
      p_corr[k] = p_omba[k] - (1.0f - p_ba[k]);
      if (p_corr[k] != p_corr[k]) p_corr[k] = 0.0f;  // bond_alpha = +-inf: -+inf + 0
#pragma unroll
      for (int c = 0; c < 4; ++c) rba[k][c] = p_ba[k];
    }
  }

  // Dividend partials parked per wave in LDS (kGrpDB epochs x K scenarios x R
  // rows x the wave's 4 row groups) and written out as 16-byte row runs when
  // the buffer fills or the launch ends: no global store in the epoch loop
  // and no block barrier (a block-wide version lost in round 4)
  float* dpb = dpark + (kGrpPark ? L.wave * (kGrpDB * K * R * 4) : 0);
  int tq = A.t0;  // first epoch held in the wave's buffer
  auto flush_d = [&](int t) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int rw0 = rb * G * R + L.wave * 4;  // this wave's first row of row-set i = 0
    const int ne = (t - tq + 1) * K * R;
    for (int j = L.lane; j < ne; j += 64) {
      const int i = j % R, k = (j / R) % K, e = j / (R * K);
      if (k >= nk) continue;
      const int r = rw0 + G * i;
      float* dst = A.dpart + (((long long)(tq + e) * N + n0 + k) * A.tiles + tile) * V + r;
      const float* src = dpb + j * 4;
      if ((V & 3) == 0 && r + 3 < V) {
        *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
      } else {
        for (int q = 0; q < 4; ++q)
          if (r + q < V) dst[q] = src[q];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    tq = t + 1;
  };
  for (int tb = A.t0; tb < A.t1; tb += P) {
#pragma unroll
    for (int kk = 0; kk < P; ++kk) {
      const int t = tb + kk;
      if (t >= A.t1) break;
      // normalised weights, once for the K scenarios: div_fast_nz's result
      // from the stored reciprocal when every row of the wave is in range,
      // else IEEE division (the same values up to the sign of a zero)
      float wn[R][4];
      bool slow = false;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        slow |= rq[kk][i] != rq[kk][i];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float a = rw[kk][i][c];
          const float q = a * rq[kk][i];
          const float e = fmaf(-rd[kk][i], q, a);
          wn[i][c] = fmaf(e, rq[kk][i], q);
        }
      }
      if (__any(slow)) {  // (tested after the division: a test ahead of it drained the ring)
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int c = 0; c < 4; ++c) wn[i][c] = rw[kk][i][c] / rd[kk][i];
      }
      float sv[R];
#pragma unroll
      for (int i = 0; i < R; ++i) sv[i] = rsn[kk][i];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (k >= nk) break;
        if (__builtin_expect(t == p_repoch[k] && has_old, 0)) {
          const unsigned cols = rcols >> (4 * k);
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int cc = 0; cc < 4; ++cc)
              if ((cols >> cc) & 1u) B[k][i][cc] = 0.0f;
        }
        // this epoch's incentive / bond_alpha are used in place; the next
        // epoch's are fetched after the update (no register copies)
        float bac[4], omba[4];
        const float* ic = ri[k];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (LQ == 2) {  // every scenario liquid: omba = 1 - bond_alpha (yumas.py:256)
            bac[c] = rba[k][c];
            omba[c] = 1.0f - rba[k][c];
          } else if (LQ == 1) {
            // rba holds bond_alpha for a fixed-alpha scenario; p_corr turns
            // 1 - rba into its (double-derived) one_minus_bond_alpha exactly
            // and is +0 for a liquid one (see the set-up above)
            bac[c] = rba[k][c];
            omba[c] = (1.0f - rba[k][c]) + p_corr[k];
          } else {
            bac[c] = p_ba[k];
            omba[c] = p_omba[k];
          }
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const int row = row0 + G * i;
          // k_bonds_elem's short clamp forms (signed zeros cannot show, see there)
          if (VARIANT == YUMA_VARIANT_YUMA3) {
            const float cap = sv[i] * p_maxint[k];
            const float ca = p_ca[k] * cap;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float rem = vmax(cap - B[k][i][c], 0.0f);
              const float pc = vmin(ca, rem);
              const float nb = p_dk[k] * B[k][i][c] + pc * wn[i][c];
              B[k][i][c] = tmin(nb, cap);
            }
          } else if (BND) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float bd = B[k][i][c] * omba[c];
              B[k][i][c] = bd + vmin(bac[c] * wn[i][c], 1.0f - bd);
            }
          } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float bd = B[k][i][c] * omba[c];
              const float rem = vmax(1.0f - bd, 0.0f);
              const float nb = bd + vmin(bac[c] * wn[i][c], rem);
              B[k][i][c] = vmin(nb, 1.0f);
            }
          }
          if (hist && row < V && m < M)
            *reinterpret_cast<float4*>(pH[k] + (long long)G * i * M) =
                make_float4(B[k][i][0], B[k][i][1], B[k][i][2], B[k][i][3]);
          // (a select, not a lane branch: the branch made the compiler wait
          // vmcnt(0) inside it, draining the W ring)
          float d = 0.0f;
#pragma unroll
          for (int c = 0; c < 4; ++c) d = d + B[k][i][c] * ic[c];
          d = m < M ? d : 0.0f;
          d = wsum16(d);
          if constexpr (kGrpPark) {
            if (L.c4 == 0) dpb[(((t - tq) * K + k) * R + i) * 4 + (L.lane >> 4)] = d;
          } else {
            if (L.c4 == 0 && row < V) pD[k][G * i] = d;
          }
        }
        fetch_s(k, t + 2 < A.t1);
        pD[k] += sD;
        if (hist) pH[k] += sM * V;
      }
      // the W ring refill after this epoch's per-scenario incentive loads:
      // vmcnt drains in issue order, so waiting for the next epoch's
      // incentive does not wait for the rows two epochs ahead (c3 bonds
      // 6.69-6.73 -> 6.61-6.62 ms, profiles/r05/ab_grp.txt)
      fetch(kk, t + P + 1 < A.t1);
      if constexpr (kGrpPark) {
        if (t - tq == kGrpDB - 1 || t == A.t1 - 1) flush_d(t);  // wave-uniform
      }
      has_old = true;
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (k >= nk) break;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = row0 + G * i;
      if (row < V) store4<true>(A.Bstate + (n0 + k) * VM + (long long)row * M, m, M, B[k][i]);
    }
  }
}

template <int VARIANT, int K, int R, int P, bool HIST>
__global__ __launch_bounds__(256, kGrpWaves) void k_bonds_grp(BondArgs A) {
  __shared__ float dpark[kGrpPark ? 4 * kGrpDB * K * R * 4 : 1];
  const int n0 = (blockIdx.x / (A.tiles * A.rowblocks)) * K;
  unsigned liquid_mask = 0;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (n0 + k < A.N && A.prm[n0 + k].liquid_mode != YUMA_LIQUID_OFF) liquid_mask |= 1u << k;
  const int nk = A.N - n0 < K ? A.N - n0 : K;
  if constexpr (VARIANT == YUMA_VARIANT_YUMA4) {
    // the bounded update (grp_scan BND), decided per wave (the scan has no
    // block barrier): parameters, the wave's starting bond state and its
    // rows' weights over the launch (k_rowsum's negative-weight flag rq4.w)
    bool ok = A.rq4 != nullptr;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (k >= nk) break;
      const yuma_params_t& pg = A.prm[n0 + k];
      if ((liquid_mask >> k) & 1u)  // bond_alpha = 1 - clamp(alpha, alpha_low, alpha_high)
        ok = ok && pg.alpha_low >= 0.0f && pg.alpha_low <= 1.0f && pg.alpha_high >= 0.0f && pg.alpha_high <= 1.0f;
      else
        ok = ok && pg.bond_alpha >= 0.0f && pg.bond_alpha <= 1.0f && pg.one_minus_bond_alpha >= 0.0f &&
             pg.one_minus_bond_alpha <= 1.0f;
    }
    const Lay L = lay();
    const int tile = blockIdx.x % A.tiles, rb = (blockIdx.x / A.tiles) % A.rowblocks;
    const int m = tile * kTileM + L.c4 * 4, row0 = rb * 16 * R + L.g;
    const float* src = A.t0 == 0 ? A.B_init : A.Bstate;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int row = row0 + 16 * i;
      if (row >= A.V) continue;
      if (src != nullptr && m < A.M)
#pragma unroll
        for (int k = 0; k < K; ++k) {
          if (k >= nk) break;
          float b[4];
          load4<true>(src + (long long)(n0 + k) * A.V * A.M + (long long)row * A.M, m, A.M, b);
#pragma unroll
          for (int c = 0; c < 4; ++c) ok &= (b[c] >= 0.0f && b[c] <= 1.0f) || b[c] != b[c];
        }
      if (A.rq4 != nullptr) {  // independent loads (no short-circuit chain of load latencies)
        float neg = 0.0f;
        const float* fw = reinterpret_cast<const float*>(A.rq4 + (long long)A.t0 * A.V + row) + 3;
#pragma unroll 8
        for (int t = A.t0; t < A.t1; ++t, fw += 4 * A.V) neg = fmaxf(neg, *fw);
        ok &= neg == 0.0f;
      }
    }
    if (__all(ok)) {
      if (liquid_mask == (1u << nk) - 1u)
        grp_scan<VARIANT, K, R, P, 2, HIST, true>(A, liquid_mask, dpark);
      else if (liquid_mask != 0)
        grp_scan<VARIANT, K, R, P, 1, HIST, true>(A, liquid_mask, dpark);
      else
        grp_scan<VARIANT, K, R, P, 0, HIST, true>(A, 0u, dpark);
      return;
    }
  }
  if (VARIANT == YUMA_VARIANT_YUMA4 && liquid_mask == (1u << nk) - 1u)  // block-uniform; Yuma3 has no bond_alpha
    grp_scan<VARIANT, K, R, P, 2, HIST>(A, liquid_mask, dpark);
  else if (VARIANT == YUMA_VARIANT_YUMA4 && liquid_mask != 0)
    grp_scan<VARIANT, K, R, P, 1, HIST>(A, liquid_mask, dpark);
  else
    grp_scan<VARIANT, K, R, P, 0, HIST>(A, 0u, dpark);
}

// ---------------------------------------------------------------------------
// Finalize, one block per slice: D = sum over tiles of the partials (Yuma4:
// D = S * that, yumas.py:590), D_normalized = D / (D.sum() + 1e-6), and
// validator trust T_v = sum Wc / sum W (yumas.py:224).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_finalize(const float* __restrict__ dpart,
                                                  const float* __restrict__ sn, int variant,
                                                  int V, long long slice0, int tiles,
                                                  const float* __restrict__ tvc,
                                                  const float* __restrict__ tvn,
                                                  float* __restrict__ Dn, float* __restrict__ D,
                                                  float* __restrict__ Tv, int dpl, int ttiles) {
  // thread (tg, vq): quad group tg = tid / 64 sums the quads tg, tg+4, ...;
  // vq owns validators 4vq..4vq+3 of the current 256-validator window. The
  // canonical order (dp_quad): per-group sequential, then groups 0..3.
  __shared__ float part[4][256];
  __shared__ float red[4];
  __shared__ float dsh[kRegRows];
  const long long slice = slice0 + blockIdx.x;
  const int tg = threadIdx.x >> 6, vq = threadIdx.x & 63;
  const int nq = dp_quads(tiles);
  if (dpl == DP_PRE) {  // D already formed (k_dte_sum, same order)
    for (int v = threadIdx.x; v < V; v += 256) {
      float d = dpart[slice * V + v];
      if (variant == YUMA_VARIANT_YUMA4) d = sn[slice * V + v] * d;
      dsh[v] = d;
    }
    __syncthreads();
  }
  if (dpl == DP_VQ) {
    // [V][quad]: one thread per validator walks its contiguous quads, keeping
    // the four group sums apart (quad b goes to group b % 4)
    const float* dq = dpart + slice * (long long)nq * V;
    for (int v = threadIdx.x; v < V; v += 256) {
      const float* pv = dq + (long long)v * nq;
      float pg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      int b = 0;
      if ((nq & 3) == 0) {
#pragma unroll 4
        for (; b < nq; b += 4) {
          const float4 x = *reinterpret_cast<const float4*>(pv + b);
          pg[0] = pg[0] + x.x;
          pg[1] = pg[1] + x.y;
          pg[2] = pg[2] + x.z;
          pg[3] = pg[3] + x.w;
        }
      } else {
        for (; b < nq; ++b) pg[b & 3] = pg[b & 3] + pv[b];
      }
      float d = pg[0];
      d = d + pg[1];
      d = d + pg[2];
      d = d + pg[3];
      if (variant == YUMA_VARIANT_YUMA4) d = sn[slice * V + v] * d;
      dsh[v] = d;
    }
    __syncthreads();
  }
  const float* dp = dpart + slice * (long long)tiles * V;
  for (int v0 = 0; v0 < V && dpl == DP_TV; v0 += 256) {
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const int vb = v0 + vq * 4;
    if ((V & 3) == 0 && vb < V) {
      // whole validator quads: float4 loads of a quad's four tiles, one quad
      // at a time (c3 0.229 -> 0.221 ms against two in flight, 0.247 with four)
#pragma unroll 1
      for (int b = tg; b < nq; b += 4) {
        float4 x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          x[j] = 4 * b + j < tiles ? *reinterpret_cast<const float4*>(dp + (long long)(4 * b + j) * V + vb)
                                   : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        acc[0] = acc[0] + ((x[0].x + x[1].x) + (x[2].x + x[3].x));
        acc[1] = acc[1] + ((x[0].y + x[1].y) + (x[2].y + x[3].y));
        acc[2] = acc[2] + ((x[0].z + x[1].z) + (x[2].z + x[3].z));
        acc[3] = acc[3] + ((x[0].w + x[1].w) + (x[2].w + x[3].w));
      }
    } else {
      for (int b = tg; b < nq; b += 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int v = vb + j;
          if (v < V) acc[j] = acc[j] + dp_quad(dp + v, V, b, tiles);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) part[tg][vq * 4 + j] = acc[j];
    __syncthreads();
    for (int j = threadIdx.x; j < 256; j += 256) {
      const int v = v0 + j;
      if (v < V) {
        float d = part[0][j];
        d = d + part[1][j];
        d = d + part[2][j];
        d = d + part[3][j];
        if (variant == YUMA_VARIANT_YUMA4) d = sn[slice * V + v] * d;
        dsh[v] = d;
      }
    }
    __syncthreads();
  }
  float local = 0.0f;
  for (int v = threadIdx.x; v < V; v += 256) local = local + dsh[v];
  const float tot = block_sum<256>(local, red);
  const float den = tot + 1e-6f;
  for (int v = threadIdx.x; v < V; v += 256) {
    if (Dn != nullptr) Dn[slice * V + v] = dsh[v] / den;
    if (D != nullptr) D[slice * V + v] = dsh[v];
    if (Tv != nullptr) {
      float a = 0.0f, b = 0.0f;
      for (int k = 0; k < ttiles; ++k) {
        a = a + tvc[(slice * ttiles + k) * V + v];
        b = b + tvn[(slice * ttiles + k) * V + v];
      }
      Tv[slice * V + v] = a / b;
    }
  }
}

// k_finalize above kRegRows validators (no LDS copy of D): one thread per
// validator forms D[v] in the canonical order of the same layouts, parks it in
// dtmp, and a second pass divides by the block's total (the same
// thread-sequential + block_sum order as k_finalize).
__global__ __launch_bounds__(256) void k_finalize_big(const float* __restrict__ dpart,
                                                      const float* __restrict__ sn, int variant,
                                                      int V, long long slice0, int tiles,
                                                      const float* __restrict__ tvc,
                                                      const float* __restrict__ tvn,
                                                      float* __restrict__ Dn, float* __restrict__ D,
                                                      float* __restrict__ Tv, int dpl, int ttiles,
                                                      float* __restrict__ dtmp) {
  __shared__ float red[4];
  const long long slice = slice0 + blockIdx.x;
  const int nq = dp_quads(tiles);
  float local = 0.0f;
  for (int v = threadIdx.x; v < V; v += 256) {
    float d;
    if (dpl == DP_PRE) {
      d = dpart[slice * V + v];
    } else {
      float pg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (dpl == DP_VQ) {
        const float* pv = dpart + (slice * V + v) * (long long)nq;
        for (int b = 0; b < nq; ++b) pg[b & 3] = pg[b & 3] + pv[b];
      } else {
        const float* dp = dpart + slice * (long long)tiles * V + v;
        for (int b = 0; b < nq; ++b) pg[b & 3] = pg[b & 3] + dp_quad(dp, V, b, tiles);
      }
      d = pg[0];
      d = d + pg[1];
      d = d + pg[2];
      d = d + pg[3];
    }
    if (variant == YUMA_VARIANT_YUMA4) d = sn[slice * V + v] * d;
    dtmp[slice * V + v] = d;
    local = local + d;
  }
  const float tot = block_sum<256>(local, red);
  const float den = tot + 1e-6f;
  for (int v = threadIdx.x; v < V; v += 256) {
    const float d = dtmp[slice * V + v];
    if (Dn != nullptr) Dn[slice * V + v] = d / den;
    if (D != nullptr) D[slice * V + v] = d;
    if (Tv != nullptr) {
      float a = 0.0f, b = 0.0f;
      for (int k = 0; k < ttiles; ++k) {
        a = a + tvc[(slice * ttiles + k) * (long long)V + v];
        b = b + tvn[(slice * ttiles + k) * (long long)V + v];
      }
      Tv[slice * V + v] = a / b;
    }
  }
}

// DP_QTE quad partials -> D (DP_PRE) for the epochs [t0, t1): out[slice][v]
// in the canonical order (one wave per quad group g = b % 4, summed
// sequentially, the groups joined in order through LDS). Block: 16 epochs x
// 4 validators per wave (a wave load = four 64-byte epoch runs), grid
// (scenario, 16-epoch group, validator quad).
__global__ __launch_bounds__(256) void k_dte_sum(const float* __restrict__ dpart, int N, int V, int tiles,
                                                 int ep, int t0, int t1, float* __restrict__ out) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nq = dp_quads(tiles);
  const int vgroups = (V + 3) / 4;
  const int tgroups = (t1 - (t0 & ~15) + 15) / 16;
  const int vg = blockIdx.x % vgroups;
  const int tg = (blockIdx.x / vgroups) % tgroups;
  const int n = blockIdx.x / (vgroups * tgroups);
  const int t = (t0 & ~15) + tg * 16 + (lane & 15);
  const int v = vg * 4 + (lane >> 4);
  const bool ok = t >= t0 && t < t1 && v < V;
  const float* p = dpart + ((long long)n * nq * V + (ok ? v : 0)) * ep + (ok ? t : 0);
  const long long bstride = (long long)V * ep;
  float acc = 0.0f;
#pragma unroll 8
  for (int b = wave; b < nq; b += 4) acc = acc + p[b * bstride];
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && ok) {
    float d = part[0][lane];
    d = d + part[1][lane];
    d = d + part[2][lane];
    d = d + part[3][lane];
    out[((long long)t * N + n) * V + v] = d;
  }
}

// ---------------------------------------------------------------------------
// Miner-column shards: the per-shard partial sums a
// caller reduces across shards between stages, and the hand-back of the
// reduced values. Each partial is a fixed-order sum over this shard's columns.
// ---------------------------------------------------------------------------
// rsd = (sum of the shards' row sums) + 1e-6 (yumas.py:186)
__global__ __launch_bounds__(256) void k_add_eps(const float* __restrict__ rowsum, long long n,
                                                 float* __restrict__ rsd) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    rsd[i] = rowsum[i] + 1e-6f;
}
// per slice: sum over this shard's columns of C_raw (fp32; YumaRust fp64)
__global__ __launch_bounds__(256) void k_csum(const double* __restrict__ craw, int rust, int M,
                                              float* __restrict__ csum_f,
                                              double* __restrict__ csum_d) {
  __shared__ float redf[4];
  __shared__ double redd[4];
  const long long slice = blockIdx.x;
  const double* cr = craw + slice * M;
  if (rust) {
    double acc = 0.0;
    for (int m = threadIdx.x; m < M; m += 256) acc = acc + cr[m];
    acc = block_sum_d<256>(acc, redd);
    if (threadIdx.x == 0) csum_d[slice] = acc;
  } else {
    float acc = 0.0f;
    for (int m = threadIdx.x; m < M; m += 256) acc = acc + (float)cr[m];
    acc = block_sum<256>(acc, redf);
    if (threadIdx.x == 0) csum_f[slice] = acc;
  }
}
// per slice: sum over this shard's tiles of the rank partials
__global__ __launch_bounds__(64) void k_rsum(const float* __restrict__ rpart, int tiles,
                                             float* __restrict__ out) {
  const long long slice = blockIdx.x;
  if (threadIdx.x == 0) {
    float s = 0.0f;
    for (int k = 0; k < tiles; ++k) s = s + rpart[slice * tiles + k];
    out[slice] = s;
  }
}
// per slice and validator: sum over this shard's tiles of [slice][tile][V]
// partials (validator-trust numerators / denominators), sequentially
__global__ __launch_bounds__(256) void k_dsum(const float* __restrict__ dpart, int V, int tiles,
                                              float* __restrict__ out) {
  const long long slice = blockIdx.x;
  for (int v = threadIdx.x; v < V; v += 256) {
    float d = 0.0f;
    for (int k = 0; k < tiles; ++k) d = d + dpart[dp_index(slice, k, v, tiles, V)];
    out[slice * V + v] = d;
  }
}
// per slice and validator: this shard's dividend partials (DP_TV / DP_VQ) in
// the canonical order (k_finalize)
__global__ __launch_bounds__(256) void k_dsum_canon(const float* __restrict__ dpart, int V, int tiles,
                                                    float* __restrict__ out, int dpl) {
  const long long slice = blockIdx.x;
  const int nq = dp_quads(tiles);
  for (int v = threadIdx.x; v < V; v += 256) {
    float pg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int b = 0; b < nq; ++b) {
      const float q = dpl == DP_VQ ? dpart[(slice * V + v) * nq + b]
                                   : dp_quad(dpart + slice * (long long)tiles * V + v, V, b, tiles);
      pg[b & 3] = pg[b & 3] + q;
    }
    float d = pg[0];
    d = d + pg[1];
    d = d + pg[2];
    d = d + pg[3];
    out[slice * V + v] = d;
  }
}

// ---------------------------------------------------------------------------
// Synthetic weights, integer-only so numpy and HIP agree bit for
// bit: see yuma_simulation/_internal/synth.py for the reference definition.
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t hash3(uint64_t seed, uint64_t a, uint64_t b,
                                                   uint64_t c) {
  return splitmix64(splitmix64(splitmix64(seed ^ a) ^ b) ^ c);
}
constexpr uint64_t kTagWeight = 1ull << 63, kTagZero = 1ull << 62, kTagQuality = 1ull << 61;

__global__ void k_synth(uint64_t seed, int E, int N, int V, int M, int t0, float* __restrict__ W) {
  const long long total = (long long)E * N * V * M;
  const uint64_t wmax = (uint64_t)((16777215ull) / (uint64_t)M);
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(idx % M);
    const int v = (int)((idx / M) % V);
    const long long sl = idx / ((long long)V * M);
    const int n = (int)(sl % N);
    const int t = (int)(sl / N) + t0;
    const uint64_t sd = seed + 0x1000003ull * (uint64_t)n;
    const uint64_t qa = hash3(sd, kTagQuality, 0, (uint64_t)m) >> 40;
    const uint64_t Q = (1ull << 22) + ((3ull * qa) >> 2);
    const uint64_t ua = hash3(sd, kTagWeight | (uint64_t)t, (uint64_t)v, (uint64_t)m) >> 40;
    const uint64_t F = (3ull * (1ull << 24) + 4ull * ua) / 5ull;
    uint64_t w = (Q * F) >> 24;
    if (w > (1ull << 24)) w = 1ull << 24;
    uint64_t val = (w * wmax) >> 24;
    const uint64_t z = hash3(sd, kTagZero | (uint64_t)t, (uint64_t)v, (uint64_t)m) >> 40;
    if (z < 1677722ull) val = 0;
    W[idx] = (float)val;
  }
}

}  // namespace yk

// ===========================================================================
// Host side: workspace carving, dispatch, C-ABI
// ===========================================================================
namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct Workspace {
  float* rsd;
  float4* rq4;  // per input slice and row: {row sum, RN(1 / row sum) or NaN, stake, 0} (k_rowsum)
  int* sx;  // per slice: exact stake units or -1 (k_rowsum)
  float* sn;
  double* craw;
  int* qlev;
  float* C;
  float* R;
  float* I;
  float* ba;
  float* rpart;
  float* dpart;
  float* dsum;  // DP_PRE: D of DP_QTE partials [slice][V]
  float* scal;
  float* tvc;
  float* tvn;
  float* Bstate;
  float* sumc_f;
  double* sumc_d;
  int* crep;  // per scenario: consensus class representative (k_classes)
  int* clist;  // [1 + N]: class count, then the representatives (k_class_list)
  int* rcrep;  // per scenario: rank class representative (Yuma: + bond_penalty)
  float* csb;  // Yuma / Yuma2: [slice][M] Σ_v S·W_b (k_rank_s)
  float* csr;  // ... and RN(1 / csb) where the column passes the division screen, else NaN
  float* cpart;  // YumaRust above kRegRows validators: [N][row block][M]
  size_t bytes;
};

// dividend-partial granularity of the bond scan: 64-miner tiles, or the
// column-normalised scan's 16-miner strips (k_bonds_cn)
size_t partial_tiles(int variant, int M) {
  return variant <= YUMA_VARIANT_YUMA2 ? (size_t)(M + yk::kCnStrip - 1) / yk::kCnStrip
                                       : (size_t)(M + yk::kTileM - 1) / yk::kTileM;
}

int dte_stride(int E) { return (E + 15) & ~15; }

Workspace carve(char* base, int variant, int N, int E, int V, int M, int full) {
  Workspace w{};
  const size_t S = (size_t)E * N;
  const size_t tiles = (size_t)(M + yk::kTileM - 1) / yk::kTileM;
  size_t off = 0;
  auto take = [&](size_t bytes) -> char* {
    char* p = base ? base + off : nullptr;
    off += align256(bytes);
    return p;
  };
  w.rsd = (float*)take(S * V * 4);
  w.rq4 = (float4*)take(S * V * 16);
  w.sx = (int*)take(S * 4);
  w.sn = (float*)take(S * V * 4);
  w.craw = (double*)take(S * M * 8);
  w.qlev = (int*)take(S * M * 4);
  w.C = (float*)take(S * M * 4);
  w.R = (float*)take(S * M * 4);
  w.I = (float*)take(S * M * 4);
  w.ba = (float*)take(S * M * 4);
  w.rpart = (float*)take(S * tiles * 4);
  // DP_QTE pads each (scenario, quad, row) epoch series to a multiple of 16
  const size_t dp_te = (size_t)N * yk::dp_quads((int)tiles) * V * (size_t)dte_stride(E);
  w.dpart = (float*)take(std::max(S * partial_tiles(variant, M) * V, dp_te) * 4);
  w.dsum = (float*)take(S * V * 4);
  w.scal = (float*)take(S * 8 * 4);
  w.tvc = full ? (float*)take(S * tiles * V * 4) : nullptr;
  w.tvn = full ? (float*)take(S * tiles * V * 4) : nullptr;
  w.Bstate = (float*)take((size_t)N * V * M * 4);
  w.sumc_f = (float*)take(S * 4);
  w.sumc_d = (double*)take(S * 8);
  w.crep = (int*)take((size_t)N * 4);
  w.clist = (int*)take((size_t)(N + 1) * 4);
  w.rcrep = (int*)take((size_t)N * 4);
  const bool cn = variant == YUMA_VARIANT_YUMA1 || variant == YUMA_VARIANT_YUMA2;
  w.csb = cn ? (float*)take(S * M * 4) : nullptr;
  w.csr = cn ? (float*)take(S * M * 4) : nullptr;
  w.cpart = (variant == YUMA_VARIANT_RUST && V > yk::kRegRows)
                ? (float*)take((size_t)N * ((V + yk::kRustBigRows - 1) / yk::kRustBigRows) * M * 4)
                : nullptr;
  w.bytes = off;
  return w;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// k_incentive's float4 rows: M % 4 == 0 and every row buffer it touches
// 16-byte aligned (R, I, and T / P when the trust is requested); a caller's
// output tensor may be a view at any 4-byte offset
int incentive_v4(int M, const float* R, const float* I, const yuma_outputs_t* out) {
  if ((M & 3) != 0 || !aligned16(R) || !aligned16(I)) return 0;
  if (out->P != nullptr && (!aligned16(out->P) || (out->T != nullptr && !aligned16(out->T)))) return 0;
  return 1;
}

// Row-configuration of the column-resident kernels: NT threads, R rows each.
enum RowCfg { RC_256_1, RC_256_4, RC_256_16, RC_1024_16 };
RowCfg row_cfg(int V) {
  if (V <= 16) return RC_256_1;
  if (V <= 64) return RC_256_4;
  if (V <= 256) return RC_256_16;
  return RC_1024_16;
}

#define YK_LAUNCH(kernel, grid, block, stream, ...) \
  hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, (hipStream_t)(stream), __VA_ARGS__)

template <int R, bool VEC>
void launch_consensus_w(long long nblocks, hipStream_t st, const float* W, const float* rsd,
                        const float* sn, const int* sx, const yuma_params_t* prm, int N, int V,
                        int M, long long slice0, int tiles, double* craw, float* P, int wsh,
                        const int* crep) {
  YK_LAUNCH((yk::k_consensus_w<R, VEC>), nblocks, 256, st, W, rsd, sn, sx, prm, N, V, M, slice0,
            tiles, craw, P, wsh, crep);
}

template <bool VEC>
void launch_consensus_mc(RowCfg rc, long long nblocks, hipStream_t st, const float* W, const float* rsd,
                         const float* sn, const int* sx, const yuma_params_t* prm, int N, int V, int M,
                         long long t0, int tiles, double* craw, const int* clist, int G) {
  switch (rc) {
    case RC_256_1:
      YK_LAUNCH((yk::k_consensus_mc<1, VEC>), nblocks, 256, st, W, rsd, sn, sx, prm, N, V, M, t0, tiles, craw,
                clist, G);
      return;
    case RC_256_4:
      YK_LAUNCH((yk::k_consensus_mc<4, VEC>), nblocks, 256, st, W, rsd, sn, sx, prm, N, V, M, t0, tiles, craw,
                clist, G);
      return;
    default:
      YK_LAUNCH((yk::k_consensus_mc<16, VEC>), nblocks, 256, st, W, rsd, sn, sx, prm, N, V, M, t0, tiles, craw,
                clist, G);
      return;
  }
}

template <bool VEC>
void launch_consensus(RowCfg rc, long long nblocks, hipStream_t st, const float* W,
                      const float* rsd, const float* sn, const int* sx,
                      const yuma_params_t* prm, int N, int V, int M, long long slice0, int tiles,
                      double* craw, float* P, int wsh, const int* crep,
                      const float4* rq4 = nullptr) {
  if (V > yk::kRegRows) {  // the column streamed per search pass
    YK_LAUNCH(yk::k_consensus_big<VEC>, nblocks, 256, st, W, rsd, sn, prm, N, V, M, slice0, tiles, craw, P,
              wsh, crep);
    return;
  }
  switch (rc) {  // wave-owned columns up to 256 validators
    case RC_256_1:
      launch_consensus_w<1, VEC>(nblocks, st, W, rsd, sn, sx, prm, N, V, M, slice0, tiles, craw,
                                  P, wsh, crep);
      return;
    case RC_256_4:
      launch_consensus_w<4, VEC>(nblocks, st, W, rsd, sn, sx, prm, N, V, M, slice0, tiles, craw,
                                  P, wsh, crep);
      return;
    case RC_256_16:  // 65-256 validators: 128-byte row segments, wave pairs (float4 rows)
      // shared-input sweeps keep the wave-owned kernel: there the consensus
      // classes re-read each slice from the Infinity Cache and the pairs'
      // barriers are what shows (c3 0.70 ms against 0.85-0.86 with or
      // without the non-temporal loads). So do runs that ask for the prerank
      // P (full outputs): its sum order is the wave-owned kernel's, the same
      // bits in a sweep and in the replicated run. C does not depend on the
      // kernel for exact-stake inputs (the histogram / bisection sums are
      // exact); for generic float stakes the two kernels' F sums may differ
      // in the last bit at a tie, inside the tie window the tests allow.
      if (VEC && !wsh && P == nullptr) {
        constexpr int NP = yk::kConsPairs;
        const long long nb = NP == 2 ? nblocks : nblocks / tiles * ((M + 31) / 32);
        YK_LAUNCH((yk::k_consensus_p<true, NP>), nb, 128 * NP, st, W, rsd, sn, sx, prm, N, V, M, slice0, tiles,
                  craw, P, wsh, crep, rq4);
      }
      else
        launch_consensus_w<16, VEC>(nblocks, st, W, rsd, sn, sx, prm, N, V, M, slice0, tiles, craw, P, wsh,
                                    crep);
      return;
    default:
      break;
  }
  switch (rc) {
    case RC_256_1:
      YK_LAUNCH((yk::k_consensus<256, 1, VEC>), nblocks, 256, st, W, rsd, sn, prm, N, V, M,
                slice0, tiles, craw, P, wsh, crep);
      break;
    case RC_256_4:
      YK_LAUNCH((yk::k_consensus<256, 4, VEC>), nblocks, 256, st, W, rsd, sn, prm, N, V, M,
                slice0, tiles, craw, P, wsh, crep);
      break;
    case RC_256_16:
      YK_LAUNCH((yk::k_consensus<256, 16, VEC>), nblocks, 256, st, W, rsd, sn, prm, N, V, M,
                slice0, tiles, craw, P, wsh, crep);
      break;
    case RC_1024_16:
      YK_LAUNCH((yk::k_consensus<1024, 16, VEC>), nblocks, 1024, st, W, rsd, sn, prm, N, V, M,
                slice0, tiles, craw, P, wsh, crep);
      break;
  }
}

// csb (streaming rank only, Yuma / Yuma2): also form the bond column sums
// Σ_v S·W_b per slice and miner (k_rank_s BCS) for the element-wise bond scan
template <bool VEC>
void launch_rank(RowCfg rc, long long nblocks, hipStream_t st, const float* W, const float* rsd,
                 const float* sn, const float* C, const float* Wprev_init, int yuma2, int N,
                 int V, int M, long long slice0, int tiles, float* R, float* rpart, float* Wn,
                 float* Wc, float* tvc, float* tvn, int wsh, const int* crep = nullptr,
                 float* csb = nullptr, float* csr = nullptr, const yuma_params_t* prm = nullptr,
                 const int* clist = nullptr) {
  const bool full = Wn != nullptr || Wc != nullptr || tvc != nullptr;
  if (V > yk::kRegRows) {  // streamed rows: the wide rank with per-row loads, plus the full outputs
    const long long nb = nblocks / tiles * ((M + 255) / 256);
    if (yuma2 && csb)
      YK_LAUNCH((yk::k_rank_sw<VEC, true, true, true>), nb, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles,
                R, rpart, wsh, nullptr, Wprev_init, csb, csr, prm);
    else if (yuma2)
      YK_LAUNCH((yk::k_rank_sw<VEC, true, false, true>), nb, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles,
                R, rpart, wsh, nullptr, Wprev_init, nullptr, nullptr, prm);
    else if (csb)
      YK_LAUNCH((yk::k_rank_sw<VEC, false, true, true>), nb, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles,
                R, rpart, wsh, full ? nullptr : crep, nullptr, csb, csr, prm);
    else
      YK_LAUNCH((yk::k_rank_sw<VEC, false, false, true>), nb, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles,
                R, rpart, wsh, full ? nullptr : crep, nullptr, nullptr, nullptr, prm);
    if (full) {
      if (yuma2)
        YK_LAUNCH((yk::k_full_big<VEC, true>), nblocks, 256, st, W, rsd, C, N, V, M, slice0, tiles, wsh,
                  Wprev_init, Wn, Wc, tvc, tvn);
      else
        YK_LAUNCH((yk::k_full_big<VEC, false>), nblocks, 256, st, W, rsd, C, N, V, M, slice0, tiles, wsh,
                  Wprev_init, Wn, Wc, tvc, tvn);
    }
    return;
  }
  // the wide form for the ranks that also form bond column sums, and for wide
  // subnets (c4 rank 1.15 -> 1.10 ms; c2's plain rank is a tie, 0.70 both,
  // profiles/r05/ab_rank_wide.txt, ab_c4_rank.txt)
  if (!full && (csb || M >= 16384) && yk::kRankWide) {  // streaming rank on 256-miner column blocks
    const long long nb = nblocks / tiles * ((M + 255) / 256);
    if (yuma2 && csb)
      YK_LAUNCH((yk::k_rank_sw<VEC, true, true>), nb, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles,
                R, rpart, wsh, nullptr, Wprev_init, csb, csr, prm);
    else if (yuma2)
      YK_LAUNCH((yk::k_rank_sw<VEC, true>), nb, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles, R,
                rpart, wsh, nullptr, Wprev_init, nullptr, nullptr, prm);
    else if (csb)
      YK_LAUNCH((yk::k_rank_sw<VEC, false, true>), nb, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles,
                R, rpart, wsh, crep, nullptr, csb, csr, prm);
    else
      YK_LAUNCH((yk::k_rank_sw<VEC, false>), nb, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles, R,
                rpart, wsh, crep, nullptr, nullptr, nullptr, prm);
    return;
  }
  if (!full && clist != nullptr && !yuma2 && !csb) {  // shared-input sweep: every class per block
    const int G = N < yk::kMcGroups ? N : yk::kMcGroups;
    YK_LAUNCH((yk::k_rank_mc<VEC, 4>), nblocks / N * G, 256, st, W, rsd, sn, C, N, V, M, slice0 / N, tiles, R,
              rpart, clist, G);
    return;
  }
  if (!full) {  // streaming rank; k_rank_w also materialises Wn / Wc / T_v
    if (yuma2 && csb)  // per scenario: W_prev (the caller's) is not shared by a consensus class
      YK_LAUNCH((yk::k_rank_s<VEC, true, true>), nblocks, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles,
                R, rpart, wsh, nullptr, Wprev_init, csb, csr, prm);
    else if (yuma2)
      YK_LAUNCH((yk::k_rank_s<VEC, true>), nblocks, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles, R,
                rpart, wsh, nullptr, Wprev_init, nullptr, nullptr, prm);
    else if (csb)
      YK_LAUNCH((yk::k_rank_s<VEC, false, true>), nblocks, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles,
                R, rpart, wsh, crep, nullptr, csb, csr, prm);
    else
      YK_LAUNCH((yk::k_rank_s<VEC, false>), nblocks, 256, st, W, rsd, sn, C, N, V, M, slice0, tiles, R,
                rpart, wsh, crep, nullptr, nullptr, nullptr, prm);
    return;
  }
  auto go = [&](auto kern) {
    YK_LAUNCH(kern, nblocks, 256, st, W, rsd, sn, C, Wprev_init, yuma2, N, V, M, slice0, tiles, R,
              rpart, Wn, Wc, tvc, tvn, wsh);
  };
#define YK_RANKW(RR)                                                   \
  if (yuma2) {                                                         \
    if (full) go(yk::k_rank_w<RR, VEC, true, true>);                   \
    else go(yk::k_rank_w<RR, VEC, true, false>);                       \
  } else {                                                             \
    if (full) go(yk::k_rank_w<RR, VEC, false, true>);                  \
    else go(yk::k_rank_w<RR, VEC, false, false>);                      \
  }                                                                    \
  return;
  switch (rc) {  // wave-owned columns up to 256 validators
    case RC_256_1:
      YK_RANKW(1)
    case RC_256_4:
      YK_RANKW(4)
    case RC_256_16:
      YK_RANKW(16)
    default:
      break;
  }
  switch (rc) {
    case RC_256_1:
      YK_LAUNCH((yk::k_rank<256, 1, VEC>), nblocks, 256, st, W, rsd, sn, C, Wprev_init, yuma2,
                N, V, M, slice0, tiles, R, rpart, Wn, Wc, tvc, tvn, wsh);
      break;
    case RC_256_4:
      YK_LAUNCH((yk::k_rank<256, 4, VEC>), nblocks, 256, st, W, rsd, sn, C, Wprev_init, yuma2,
                N, V, M, slice0, tiles, R, rpart, Wn, Wc, tvc, tvn, wsh);
      break;
    case RC_256_16:
      YK_LAUNCH((yk::k_rank<256, 16, VEC>), nblocks, 256, st, W, rsd, sn, C, Wprev_init, yuma2,
                N, V, M, slice0, tiles, R, rpart, Wn, Wc, tvc, tvn, wsh);
      break;
    case RC_1024_16:
      YK_LAUNCH((yk::k_rank<1024, 16, VEC>), nblocks, 1024, st, W, rsd, sn, C, Wprev_init,
                yuma2, N, V, M, slice0, tiles, R, rpart, Wn, Wc, tvc, tvn, wsh);
      break;
  }
}

// Column-normalised variants (Rust / Yuma1 / Yuma2): one block owns whole
// columns (single row block). Run outputs of subnets above 64 validators take
// the strip scan k_bonds_cn (16-miner strips, 8 waves, epochs in flight);
// small subnets and the full-output epoch (W_b / instantaneous bonds stored)
// k_bonds on 64-miner tiles. Returns the dividend-partial layout and sets
// *ptiles to the partials per (slice, validator).
template <int VARIANT, int R, int NW = 8>
int launch_cn(hipStream_t st, yk::BondArgs& A, int* ptiles) {
  A.rowblocks = 1;
  A.cblocks = (A.M + yk::kCnStrip - 1) / yk::kCnStrip;
  *ptiles = A.cblocks;
  const long long nblocks = (long long)A.N * A.cblocks;
  constexpr int P = NW == 8 ? (R <= 2 ? 4 : (R == 4 ? 2 : 1)) : (R <= 4 ? 3 : 2);
  if (A.rq4 != nullptr)  // k_rowsum's screened reciprocals (run_impl; not the shard stages)
    YK_LAUNCH((yk::k_bonds_cn<VARIANT, R, P, NW, true>), nblocks, 64 * NW, st, A);
  else
    YK_LAUNCH((yk::k_bonds_cn<VARIANT, R, P, NW, false>), nblocks, 64 * NW, st, A);
  return yk::DP_TV;
}
// YumaRust's strip scan: 8 waves per 16-miner strip. Fewer waves with more
// rows per lane (a cheaper per-epoch column reduction) lose: c2 YumaRust
// bonds 3.50 -> 5.11 ms with 4 waves, 9.12 with 2 (profiles/r05/ab_cn_waves.txt)
template <int VARIANT>
int launch_cn_rows(hipStream_t st, yk::BondArgs& A, int* ptiles) {
  const int V = A.V;
  if (V <= 128) return launch_cn<VARIANT, 1>(st, A, ptiles);
  if (V <= 256) return launch_cn<VARIANT, 2>(st, A, ptiles);
  if (V <= 512) return launch_cn<VARIANT, 4>(st, A, ptiles);
  return launch_cn<VARIANT, 8>(st, A, ptiles);
}
template <int VARIANT, bool VEC>
int launch_bonds_elem(hipStream_t st, yk::BondArgs& A);
template <int VARIANT, bool VEC>
int launch_bonds_colnorm(RowCfg rc, hipStream_t st, yk::BondArgs& A, int* ptiles) {
  if (A.V > yk::kRegRows) {  // no workgroup holds a column: streaming forms
    *ptiles = A.tiles;
    if constexpr (VARIANT == YUMA_VARIANT_RUST) {
      A.rowblocks = (A.V + yk::kRustBigRows - 1) / yk::kRustBigRows;
      A.cblocks = A.tiles;
      const long long nb = (long long)A.N * A.rowblocks * A.tiles;
      for (int t = A.t0; t < A.t1; ++t) {
        YK_LAUNCH((yk::k_rust_big_ema<VEC>), nb, 256, st, A, t, A.cpart);
        YK_LAUNCH((yk::k_rust_big_norm<VEC>), nb, 256, st, A, t, A.cpart);
      }
      return yk::DP_TV;
    } else {
      return launch_bonds_elem<VARIANT, VEC>(st, A);  // the rank pass formed csb
    }
  }
  if constexpr (VARIANT != YUMA_VARIANT_RUST) {
    // the rank pass formed the bond column sums: element-wise scan
    if (A.csb != nullptr && A.Wb_out == nullptr && A.Binst_out == nullptr) {
      *ptiles = A.tiles;
      return launch_bonds_elem<VARIANT, VEC>(st, A);
    }
  }
  if constexpr (VEC) {
    if (A.V > 64 && A.Wb_out == nullptr && A.Binst_out == nullptr) return launch_cn_rows<VARIANT>(st, A, ptiles);
  }
  *ptiles = A.tiles;
  A.rowblocks = 1;
  A.cblocks = A.tiles;
  const long long nblocks = (long long)A.N * A.tiles;
  switch (rc) {
    case RC_256_1:
      YK_LAUNCH((yk::k_bonds<VARIANT, 256, 1, VEC>), nblocks, 256, st, A);
      break;
    case RC_256_4:
      YK_LAUNCH((yk::k_bonds<VARIANT, 256, 4, VEC>), nblocks, 256, st, A);
      break;
    case RC_256_16:
      YK_LAUNCH((yk::k_bonds<VARIANT, 256, 16, VEC>), nblocks, 256, st, A);
      break;
    case RC_1024_16:
      YK_LAUNCH((yk::k_bonds<VARIANT, 1024, 16, VEC>), nblocks, 1024, st, A);
      break;
  }
  return yk::DP_TV;
}

// Element-wise variants (Yuma3 / Yuma4): R rows x 4 miners per thread, the
// inputs of the next P epochs in flight, float4 incentive / bond_alpha loads.
// Measured on MI355X at c2 (tools/ab_bonds.sh): without
// the history, R = 1, P = 4 on 64-miner tiles (1.13 ms vs 1.36 for R = 2);
// shared-input sweeps (W reads served by the caches) R = 2, P = 2.
// Writing the bond history (the c2 line): wide column blocks, one row per
// wave instruction (tools/scanbw: a 4-row x 4 KiB block footprint streams
// the 4 GB in + 4 GB out at 5.6-5.9 TB/s against 5.0 for 32 rows x 256 B;
// in the engine c2 Yuma 3 bonds 1.66-1.72 -> 1.54-1.58 ms). Without the
// history the same shapes lose (c2 1.05 -> 1.07-1.69 ms, c4 1.63 -> 1.63-1.84,
// the c3 sweep 10.2 -> 10.6-14.7 ms: profiles/r03/ab/scan_shapes_nohist.txt).
// Sweeps over one shared input trajectory run k_bonds_grp with K = 4
// scenarios per block (k_bonds_grp's history).
constexpr int kWideP = 2;      // epochs in flight of the wide history scan
constexpr int kWidePCn = 2;    // ... for Yuma / Yuma2 (more work per epoch)
// epochs in flight of the two-row history-less scan (c4 bonds 1.37-1.39 ->
// 1.33 ms with 3 against 2 with the guarded division, profiles/r05/ab_c4_scan.txt;
// with the screened reciprocal 2: 1.25-1.27 against 1.32-1.36 at 3)
constexpr int kNoHistP2 = 2;
constexpr int kScanGroup = 4;  // scenarios per block of the shared-input scan
// the scans that divide W by k_rowsum's screened reciprocal (rq4) instead of
// a per-row IEEE reciprocal and a per-element guard: the Yuma / Yuma2 wide
// history scan (Yuma 1 bonds 1.84 -> 1.73 ms, same box) and the history-less
// forms (c4 1.32-1.33 -> 1.25-1.27 with 2 epochs in flight, c2 --no-history
// 0.985-0.997 -> 0.916-0.923; profiles/r05/ab_elem_rq.txt)
constexpr bool kElemRq(int variant, bool hist) { return hist ? variant <= YUMA_VARIANT_YUMA2 : true; }
int bonds_rows(bool vec, bool hist, bool wsh) { return vec && (hist || wsh) ? 2 : 1; }
template <int VARIANT, int R, bool VEC, int P, bool VECI, bool NT, int BS, int CB, int DPL, bool RQ = false>
int launch_elem_shape(hipStream_t st, yk::BondArgs& A) {
  constexpr int G = BS / (CB / 4);
  A.rowblocks = (A.V + G * R - 1) / (G * R);
  A.cblocks = (A.M + CB - 1) / CB;
  const long long nblocks = (long long)A.N * A.rowblocks * A.cblocks;
  YK_LAUNCH((yk::k_bonds_elem<VARIANT, R, VEC, P, VECI, NT, BS, CB, DPL, RQ>), nblocks, BS, st, A);
  return DPL;
}
template <int VARIANT, bool VEC>
int launch_bonds_elem(hipStream_t st, yk::BondArgs& A) {
  const bool hist = A.B_hist != nullptr;
  if constexpr (VEC) {
    if (hist && A.M >= 1024) {
      constexpr int P = VARIANT <= YUMA_VARIANT_YUMA2 ? kWidePCn : kWideP;
      if constexpr (kElemRq(VARIANT, true)) {
        if (A.rq4 != nullptr) return launch_elem_shape<VARIANT, 2, true, P, true, true, 512, 1024, yk::DP_VQ, true>(st, A);
      }
      return launch_elem_shape<VARIANT, 2, true, P, true, true, 512, 1024, yk::DP_VQ>(st, A);
    }
  }
  if constexpr (VEC && VARIANT >= YUMA_VARIANT_YUMA3) {
    if (A.wsh && A.N >= 2 && A.rq4 != nullptr) {  // a sweep over one input trajectory
      constexpr int K = kScanGroup, R = 2;
      A.rowblocks = (A.V + 16 * R - 1) / (16 * R);
      A.cblocks = A.tiles;
      const long long nblocks = (long long)((A.N + K - 1) / K) * A.rowblocks * A.tiles;
      if (hist)
        YK_LAUNCH((yk::k_bonds_grp<VARIANT, K, R, 2, true>), nblocks, 256, st, A);
      else
        YK_LAUNCH((yk::k_bonds_grp<VARIANT, K, R, 2, false>), nblocks, 256, st, A);
      return yk::DP_TV;
    }
  }
  if (bonds_rows(VEC, hist, A.wsh != 0) != 2) {
    // two rows per lane (one incentive load per two rows, 2 epochs in
    // flight) once the grid has blocks to spare: c4 1.41 -> 1.38 ms; with
    // c2's 512 such blocks 0.99 -> 1.31, so one row per lane there
    const long long blocks_r2 = (long long)A.N * ((A.V + 7) / 8) * ((A.M + 255) / 256);
    if constexpr (VEC && kElemRq(VARIANT, false)) {
      if (A.rq4 != nullptr) {
        if (blocks_r2 >= 4096)
          return launch_elem_shape<VARIANT, 2, VEC, kNoHistP2, VEC, false, 256, 256, yk::DP_QTE, true>(st, A);
        return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 256, yk::DP_QTE, true>(st, A);
      }
    }
    if (blocks_r2 >= 4096)
      return launch_elem_shape<VARIANT, 2, VEC, kNoHistP2, VEC, false, 256, 256, yk::DP_QTE>(st, A);
    return launch_elem_shape<VARIANT, 1, VEC, 4, VEC, false, 256, 256, yk::DP_QTE>(st, A);
  }
  if (hist) return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, true, 256, 64, yk::DP_TV>(st, A);
  return launch_elem_shape<VARIANT, 2, VEC, 2, VEC, false, 256, 64, yk::DP_TV>(st, A);
}

// Launch the bond scan for A.N scenarios over epochs [A.t0, A.t1); returns
// the layout of the dividend partials it wrote (k_finalize / k_dsum read it).
template <bool VEC>
int launch_bonds(int variant, RowCfg rc, hipStream_t st, yk::BondArgs& A, int* ptiles) {
  *ptiles = A.tiles;
  switch (variant) {
    case YUMA_VARIANT_RUST:
      return launch_bonds_colnorm<YUMA_VARIANT_RUST, VEC>(rc, st, A, ptiles);
    case YUMA_VARIANT_YUMA1:
      return launch_bonds_colnorm<YUMA_VARIANT_YUMA1, VEC>(rc, st, A, ptiles);
    case YUMA_VARIANT_YUMA2:
      return launch_bonds_colnorm<YUMA_VARIANT_YUMA2, VEC>(rc, st, A, ptiles);
    case YUMA_VARIANT_YUMA3:
      return launch_bonds_elem<YUMA_VARIANT_YUMA3, VEC>(st, A);
    default:
      return launch_bonds_elem<YUMA_VARIANT_YUMA4, VEC>(st, A);
  }
}

// Optional per-phase timing (bench / roofline): a HIP event is recorded on the
// launch stream at every phase boundary, labelled with the phase that starts
// there; each segment's elapsed time goes to its label.
struct PhaseTimer {
  float* ms;  // [YUMA_NUM_PHASES] accumulated milliseconds, or nullptr
  hipStream_t st;
  std::vector<hipEvent_t> ev;
  std::vector<int> label;
  int ok = 1;
  void mark(int phase) {
    if (!ms || !ok) return;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) {
      ok = 0;
      return;
    }
    (void)hipEventRecord(e, st);
    ev.push_back(e);
    label.push_back(phase);
  }
};

int run_impl(int variant, const yuma_params_t* prm, int N, int E, int V, int M, const float* W,
             const float* S, const float* B_init, const float* Wprev_init,
             const yuma_outputs_t* out, void* workspace, size_t ws_bytes, int chunk,
             void* stream, float* phase_ms = nullptr, int wsh = 0) {
  if (variant < 0 || variant > 4) return fail(YUMA_EINVAL, "unknown variant %d", variant);
  if (N < 1 || E < 1 || V < 1 || M < 1)
    return fail(YUMA_EINVAL, "sizes must be positive (N=%d E=%d V=%d M=%d)", N, E, V, M);
  if (V > YUMA_MAX_VALIDATORS)
    return fail(YUMA_EUNSUPPORTED, "V=%d exceeds YUMA_MAX_VALIDATORS=%d", V,
                YUMA_MAX_VALIDATORS);
  if ((M + yk::kTileM - 1) / yk::kTileM > yk::kMaxTiles) return fail(YUMA_EINVAL, "M too large");
  if (!prm || !W || !S || !out || !workspace)
    return fail(YUMA_EINVAL, "null params/W/S/outputs/workspace");
  const int full = out->Tv != nullptr;
  // bisection trip counts above 30 (consensus_precision > 2^30) are not supported;
  // params live in device memory, so the Python marshaller enforces it.
  Workspace ws = carve((char*)workspace, variant, N, E, V, M, full);
  if (ws.bytes > ws_bytes)
    return fail(YUMA_EWORKSPACE, "workspace %zu < required %zu bytes (full_outputs=%d)",
                ws_bytes, ws.bytes, full);
  hipStream_t st = (hipStream_t)stream;
  const int tiles = (M + yk::kTileM - 1) / yk::kTileM;
  const RowCfg rc = row_cfg(V);

  bool vec = (M % 4) == 0 && aligned16(W);
  const float* mats[] = {B_init, Wprev_init, out->Wn, out->Wc, out->Wb, out->B_inst,
                         out->B_hist, out->B_final};
  for (const float* p : mats)
    if (p != nullptr && !aligned16(p)) vec = false;

  float* C = out->C ? out->C : ws.C;
  float* I = out->I ? out->I : ws.I;
  float* Rr = out->R ? out->R : ws.R;
  float* Bstate = out->B_final ? out->B_final : ws.Bstate;
  // liquid bond_alpha lives in the caller's buffer when requested; scenarios
  // with liquid_mode OFF neither write nor read it
  float* ba_buf = out->bond_alpha ? out->bond_alpha : ws.ba;

  // one chunk by default: phase 1 of every epoch, then one bond scan
  if (chunk <= 0 || chunk > E) chunk = E;


  // Shared inputs: scenarios with the same consensus parameters take one
  // representative's consensus, quantisation input and (streaming) rank
  // (k_classes). Off when the prerank P is requested (the consensus pass
  // writes it for every slice) and for the materialising / Yuma2 rank.
  const int* crep = nullptr;
  const long long ncb = (N + 255) / 256 < 64 ? (N + 255) / 256 : 64;
  if (wsh && N > 1 && out->P == nullptr) {
    YK_LAUNCH(yk::k_classes, ncb, 256, st, prm, N, ws.crep, 0);
    crep = ws.crep;
  }
  // ... and one block per (epoch, tile, class group) searching every class on
  // one load of the tile (k_consensus_mc; wave-owned columns, <= 256 validators)
  const bool mc = crep != nullptr && V <= 256;
  if (mc) YK_LAUNCH(yk::k_class_list, 1, 256, st, ws.crep, N, ws.clist);
  // Yuma / Yuma2 run outputs above 64 validators: the streaming rank also
  // forms the bond column sums Σ_v S·W_b and the bond scan is element-wise
  const bool streaming = out->Wn == nullptr && out->Wc == nullptr && ws.tvc == nullptr;
  // (above kRegRows validators always: the element-wise scan is the only
  // Yuma / Yuma2 bond scan there, and it writes W_b / B_inst itself)
  float* csb = (ws.csb != nullptr &&
                (V > yk::kRegRows || (streaming && V > 64 && out->Wb == nullptr && out->B_inst == nullptr)))
                   ? ws.csb : nullptr;
  const bool rank_stream = streaming && variant != YUMA_VARIANT_YUMA2;  // Yuma2's W_prev: rank per scenario
  const int* rcrep = rank_stream ? crep : nullptr;
  if (rcrep != nullptr && csb != nullptr) {  // the column sums depend on bond_penalty too
    YK_LAUNCH(yk::k_classes, ncb, 256, st, prm, N, ws.rcrep, 1);
    rcrep = ws.rcrep;
  }

  PhaseTimer tm{};
  tm.ms = phase_ms;
  tm.st = st;

  for (int c0 = 0; c0 < E; c0 += chunk) {
    const int c1 = c0 + chunk < E ? c0 + chunk : E;
    const long long s0 = (long long)c0 * N;
    const long long ns = (long long)(c1 - c0) * N;
    {
      const int rowblocks4 = (V + 3) / 4;
      // shared inputs: one row-sum pass per input epoch, stored for all N
      const long long rs_in = wsh ? c1 - c0 : ns, rs_s0 = wsh ? c0 : s0;
      const int fan = wsh ? N : 1;
      const int nchunks = (M + 255) / 256;
      const bool wide = nchunks >= yk::kWideChunks && nchunks <= yk::kMaxWideChunks;
      tm.mark(YUMA_PHASE_ROWSUM);
      if (wide && vec)
        YK_LAUNCH((yk::k_rowsum<true, true>), rs_in * V, 256, st, W, S, V, M, rs_s0, V, ws.rsd,
                  ws.sn, 0, ws.sx, fan, ws.rq4);
      else if (wide)
        YK_LAUNCH((yk::k_rowsum<false, true>), rs_in * V, 256, st, W, S, V, M, rs_s0, V, ws.rsd,
                  ws.sn, 0, ws.sx, fan, ws.rq4);
      else if (vec)
        YK_LAUNCH(yk::k_rowsum<true>, rs_in * rowblocks4, 256, st, W, S, V, M, rs_s0, rowblocks4,
                  ws.rsd, ws.sn, 0, ws.sx, fan, ws.rq4);
      else
        YK_LAUNCH(yk::k_rowsum<false>, rs_in * rowblocks4, 256, st, W, S, V, M, rs_s0,
                  rowblocks4, ws.rsd, ws.sn, 0, ws.sx, fan, ws.rq4);
      tm.mark(YUMA_PHASE_CONSENSUS);
      if (mc) {
        const int G = N < yk::kMcGroups ? N : yk::kMcGroups;
        const long long nb = (long long)(c1 - c0) * tiles * G;
        if (vec)
          launch_consensus_mc<true>(rc, nb, st, W, ws.rsd, ws.sn, ws.sx, prm, N, V, M, c0, tiles, ws.craw,
                                    ws.clist, G);
        else
          launch_consensus_mc<false>(rc, nb, st, W, ws.rsd, ws.sn, ws.sx, prm, N, V, M, c0, tiles, ws.craw,
                                     ws.clist, G);
      } else if (vec)
        launch_consensus<true>(rc, ns * tiles, st, W, ws.rsd, ws.sn, ws.sx, prm, N, V, M, s0, tiles,
                               ws.craw, out->P, wsh, crep, ws.rq4);
      else
        launch_consensus<false>(rc, ns * tiles, st, W, ws.rsd, ws.sn, ws.sx, prm, N, V, M, s0,
                                tiles, ws.craw, out->P, wsh, crep);
      tm.mark(YUMA_PHASE_QUANTISE);
      YK_LAUNCH(yk::k_quantise<256>, ns, 256, st, ws.craw, prm, variant, N, M, s0, C, ws.qlev,
                ba_buf, ws.scal, nullptr, nullptr, 0, crep);
      tm.mark(YUMA_PHASE_RANK);
      // the multi-class rank walks the consensus classes' list: only when the
      // rank classes are those classes (no bond column sums) and the streaming
      // rank of <= 1024 validators on 64-miner tiles would run
      const int* rlist = (mc && rcrep == crep && csb == nullptr && M < 16384) ? ws.clist : nullptr;
      if (vec)
        launch_rank<true>(rc, ns * tiles, st, W, ws.rsd, ws.sn, C, Wprev_init,
                          variant == YUMA_VARIANT_YUMA2, N, V, M, s0, tiles, Rr, ws.rpart, out->Wn,
                          out->Wc, ws.tvc, ws.tvn, wsh, rcrep, csb, ws.csr, prm, rlist);
      else
        launch_rank<false>(rc, ns * tiles, st, W, ws.rsd, ws.sn, C, Wprev_init,
                           variant == YUMA_VARIANT_YUMA2, N, V, M, s0, tiles, Rr, ws.rpart,
                           out->Wn, out->Wc, ws.tvc, ws.tvn, wsh, rcrep, csb, ws.csr, prm, rlist);
    }
    tm.mark(YUMA_PHASE_INCENTIVE);
    const int ich = (M + yk::kIncCols - 1) / yk::kIncCols;
    YK_LAUNCH(yk::k_incentive, ns * ich, 256, st, Rr, ws.rpart, out->P, M, s0, tiles, I,
              out->P ? out->T : nullptr, ws.scal, nullptr, rcrep, N, ich, incentive_v4(M, Rr, I, out),
              (out->R != nullptr || variant == YUMA_VARIANT_RUST) ? 1 : 0);

    yk::BondArgs A{};
    A.W = W;
    A.rsd = ws.rsd;
    A.sn = ws.sn;
    A.C = C;
    A.I = I;
    A.ba = ba_buf;
    A.prm = prm;
    A.B_init = B_init;
    A.Wprev_init = Wprev_init;
    A.Bstate = Bstate;
    A.B_hist = out->B_hist;
    A.Wb_out = out->Wb;
    A.Binst_out = out->B_inst;
    A.dpart = ws.dpart;
    A.rq4 = ws.rq4;
    A.csb = csb;
    A.csr = ws.csr;
    A.csrep = csb != nullptr ? rcrep : nullptr;
    A.R = Rr;
    A.cpart = ws.cpart;
    A.N = N;
    A.V = V;
    A.M = M;
    A.tiles = tiles;
    A.t0 = c0;
    A.t1 = c1;
    A.wsh = wsh;
    A.ep = dte_stride(E);
    tm.mark(YUMA_PHASE_BONDS);
    int ptiles = tiles;
    int dpl = vec ? launch_bonds<true>(variant, rc, st, A, &ptiles)
                  : launch_bonds<false>(variant, rc, st, A, &ptiles);
    tm.mark(YUMA_PHASE_FINALIZE);
    const float* dsrc = ws.dpart;
    if (dpl == yk::DP_QTE) {
      YK_LAUNCH(yk::k_dte_sum, (long long)N * ((c1 - (c0 & ~15) + 15) / 16) * ((V + 3) / 4), 256, st,
                ws.dpart, N, V, ptiles, A.ep, c0, c1, ws.dsum);
      dsrc = ws.dsum;
      dpl = yk::DP_PRE;
    }
    if (V > yk::kRegRows)
      YK_LAUNCH(yk::k_finalize_big, ns, 256, st, dsrc, ws.sn, variant, V, s0, ptiles, ws.tvc, ws.tvn, out->Dn,
                out->D, out->Tv, dpl, tiles, ws.dsum);
    else
      YK_LAUNCH(yk::k_finalize, ns, 256, st, dsrc, ws.sn, variant, V, s0, ptiles, ws.tvc,
                ws.tvn, out->Dn, out->D, out->Tv, dpl, tiles);
    if (out->Sn != nullptr)
      (void)hipMemcpyAsync(out->Sn + s0 * V, ws.sn + s0 * V, (size_t)ns * V * 4,
                           hipMemcpyDeviceToDevice, st);
    if (out->alpha_ab != nullptr)
      (void)hipMemcpy2DAsync(out->alpha_ab + s0 * 2, 2 * sizeof(float), ws.scal + s0 * 8 + 1,
                             8 * sizeof(float), 2 * sizeof(float), (size_t)ns,
                             hipMemcpyDeviceToDevice, st);
    tm.mark(-1);  // end of chunk
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(YUMA_EHIP, "HIP launch failed: %s", hipGetErrorString(e));
  if (phase_ms != nullptr) {
    // bench-only path: waits for the stream, then sums per-phase elapsed times
    for (int ph = 0; ph < YUMA_NUM_PHASES; ++ph) phase_ms[ph] = 0.0f;
    if (!tm.ok || tm.ev.empty()) return fail(YUMA_EHIP, "event recording failed");
    if (hipEventSynchronize(tm.ev.back()) != hipSuccess)
      return fail(YUMA_EHIP, "hipEventSynchronize failed");
    for (size_t i = 0; i + 1 < tm.ev.size(); ++i) {
      float t = 0.0f;
      (void)hipEventElapsedTime(&t, tm.ev[i], tm.ev[i + 1]);
      if (tm.label[i] >= 0 && tm.label[i] < YUMA_NUM_PHASES) phase_ms[tm.label[i]] += t;
    }
    for (auto& ev : tm.ev) (void)hipEventDestroy(ev);
  }
  return YUMA_OK;
}

// One stage of a miner-column-sharded run (yuma_hip.h, yuma_shard_stage): the
// multi-pass path of run_impl cut at its four cross-miner reductions, over all
// E epochs at once (one chunk), with the reductions supplied by the caller.
int shard_stage_impl(int stage, int variant, const yuma_params_t* prm, int N, int E, int V, int M,
                     const float* W, const float* S, const float* B_init,
                     const float* Wprev_init, const yuma_shard_io_t* io,
                     const yuma_outputs_t* out, void* workspace, size_t ws_bytes, void* stream) {
  if (variant < 0 || variant > 4) return fail(YUMA_EINVAL, "unknown variant %d", variant);
  if (stage < 1 || stage > 5) return fail(YUMA_EINVAL, "unknown shard stage %d", stage);
  if (N < 1 || E < 1 || V < 1 || M < 1)
    return fail(YUMA_EINVAL, "sizes must be positive (N=%d E=%d V=%d M=%d)", N, E, V, M);
  if (V > YUMA_MAX_VALIDATORS)
    return fail(YUMA_EUNSUPPORTED, "V=%d exceeds YUMA_MAX_VALIDATORS=%d", V,
                YUMA_MAX_VALIDATORS);
  if (!prm || !W || !S || !out || !io || !workspace)
    return fail(YUMA_EINVAL, "null params/W/S/io/outputs/workspace");
  if (io->M_total < M || io->col0 < 0 || io->col0 + M > io->M_total)
    return fail(YUMA_EINVAL, "shard [%d, %d) outside M_total=%d", io->col0, io->col0 + M,
                io->M_total);
  // validator_trust (yumas.py:224): stage 3 sums sum(Wc) and sum(Wn) over
  // the local columns (per-tile partials, tiles in order), stage 5 divides
  // the shard-ordered totals the caller hands back
  const int full = out->Tv != nullptr;
  Workspace ws = carve((char*)workspace, variant, N, E, V, M, full);
  if (ws.bytes > ws_bytes)
    return fail(YUMA_EWORKSPACE, "workspace %zu < required %zu bytes", ws_bytes, ws.bytes);
  hipStream_t st = (hipStream_t)stream;
  const int tiles = (M + yk::kTileM - 1) / yk::kTileM;
  const RowCfg rc = row_cfg(V);
  const bool rust = variant == YUMA_VARIANT_RUST;
  bool vec = (M % 4) == 0 && aligned16(W);
  const float* mats[] = {B_init, Wprev_init, out->Wn, out->Wc, out->Wb, out->B_inst,
                         out->B_hist, out->B_final};
  for (const float* p : mats)
    if (p != nullptr && !aligned16(p)) vec = false;
  float* C = out->C ? out->C : ws.C;
  float* I = out->I ? out->I : ws.I;
  float* R = out->R ? out->R : ws.R;
  float* Bstate = out->B_final ? out->B_final : ws.Bstate;
  float* ba_buf = out->bond_alpha ? out->bond_alpha : ws.ba;
  int* qlev = io->levels ? io->levels : ws.qlev;
  const long long ns = (long long)E * N;
  // Yuma / Yuma2: the bond column sums are sums over validators, local to
  // the shard's columns: formed by stage 3's rank pass, read by stage 4's scan
  float* shard_csb = (ws.csb != nullptr &&
                      (V > yk::kRegRows || (!full && V > 64 && out->Wn == nullptr && out->Wc == nullptr &&
                                            out->Wb == nullptr && out->B_inst == nullptr)))
                         ? ws.csb : nullptr;
  switch (stage) {
    case 1: {
      if (!io->rowsum_part) return fail(YUMA_EINVAL, "stage 1 needs io->rowsum_part");
      const int rb4 = (V + 3) / 4;
      if (vec)
        YK_LAUNCH(yk::k_rowsum<true>, ns * rb4, 256, st, W, S, V, M, 0LL, rb4, io->rowsum_part,
                  ws.sn, 1, ws.sx, 1, (float4*)nullptr);
      else
        YK_LAUNCH(yk::k_rowsum<false>, ns * rb4, 256, st, W, S, V, M, 0LL, rb4, io->rowsum_part,
                  ws.sn, 1, ws.sx, 1, (float4*)nullptr);
      break;
    }
    case 2: {
      if (!io->rowsum || (rust ? !io->csum_part_d : !io->csum_part))
        return fail(YUMA_EINVAL, "stage 2 needs io->rowsum and io->csum_part%s", rust ? "_d" : "");
      long long nb = (ns * V + 255) / 256;
      if (nb > 4096) nb = 4096;
      YK_LAUNCH(yk::k_add_eps, nb, 256, st, io->rowsum, ns * V, ws.rsd);
      if (vec)
        launch_consensus<true>(rc, ns * tiles, st, W, ws.rsd, ws.sn, ws.sx, prm, N, V, M, 0LL, tiles,
                               ws.craw, out->P, 0, nullptr);
      else
        launch_consensus<false>(rc, ns * tiles, st, W, ws.rsd, ws.sn, ws.sx, prm, N, V, M, 0LL, tiles,
                                ws.craw, out->P, 0, nullptr);
      YK_LAUNCH(yk::k_csum, ns, 256, st, ws.craw, rust ? 1 : 0, M, io->csum_part, io->csum_part_d);
      break;
    }
    case 3: {
      if ((rust ? !io->csum_d : !io->csum) || !io->rsum_part)
        return fail(YUMA_EINVAL, "stage 3 needs io->csum%s and io->rsum_part", rust ? "_d" : "");
      if (full && !io->tv_part) return fail(YUMA_EINVAL, "stage 3 with out->Tv needs io->tv_part");
      YK_LAUNCH(yk::k_quantise<256>, ns, 256, st, ws.craw, prm, variant, N, M, 0LL, C, qlev,
                ba_buf, ws.scal, rust ? nullptr : io->csum, rust ? io->csum_d : nullptr, 1, nullptr);
      if (vec)
        launch_rank<true>(rc, ns * tiles, st, W, ws.rsd, ws.sn, C, Wprev_init,
                          variant == YUMA_VARIANT_YUMA2, N, V, M, 0LL, tiles, R, ws.rpart,
                          out->Wn, out->Wc, ws.tvc, ws.tvn, 0, nullptr, shard_csb, ws.csr, prm);
      else
        launch_rank<false>(rc, ns * tiles, st, W, ws.rsd, ws.sn, C, Wprev_init,
                           variant == YUMA_VARIANT_YUMA2, N, V, M, 0LL, tiles, R, ws.rpart,
                           out->Wn, out->Wc, ws.tvc, ws.tvn, 0, nullptr, shard_csb, ws.csr, prm);
      YK_LAUNCH(yk::k_rsum, ns, 64, st, ws.rpart, tiles, io->rsum_part);
      if (full) {
        YK_LAUNCH(yk::k_dsum, ns, 256, st, ws.tvc, V, tiles, io->tv_part);
        YK_LAUNCH(yk::k_dsum, ns, 256, st, ws.tvn, V, tiles, io->tv_part + ns * V);
      }
      break;
    }
    case 4: {
      if (!io->rsum || !io->dsum_part || (rust ? !io->csum_d : !io->csum))
        return fail(YUMA_EINVAL, "stage 4 needs io->rsum, io->csum%s and io->dsum_part",
                    rust ? "_d" : "");
      // liquid quantiles over every shard's levels; bond_alpha of local columns
      YK_LAUNCH(yk::k_liquid<256>, ns, 256, st, prm, N, M, 0LL, C, io->levels_all, io->M_total,
                ba_buf, ws.scal, rust ? nullptr : io->csum, rust ? io->csum_d : nullptr,
                rust ? 1 : 0);
      const int ich = (M + yk::kIncCols - 1) / yk::kIncCols;
      YK_LAUNCH(yk::k_incentive, ns * ich, 256, st, R, ws.rpart, out->P, M, 0LL, tiles, I,
                out->P ? out->T : nullptr, ws.scal, io->rsum, nullptr, N, ich, incentive_v4(M, R, I, out), 1);
      yk::BondArgs A{};
      A.W = W;
      A.rsd = ws.rsd;
      A.sn = ws.sn;
      A.C = C;
      A.I = I;
      A.ba = ba_buf;
      A.prm = prm;
      A.B_init = B_init;
      A.Wprev_init = Wprev_init;
      A.Bstate = Bstate;
      A.B_hist = out->B_hist;
      A.Wb_out = out->Wb;
      A.Binst_out = out->B_inst;
      A.dpart = ws.dpart;
      A.csb = shard_csb;
      A.csr = ws.csr;
      A.R = R;
      A.cpart = ws.cpart;
      A.N = N;
      A.V = V;
      A.M = M;
      A.tiles = tiles;
      A.t0 = 0;
      A.t1 = E;
      A.ep = dte_stride(E);
      int ptiles = tiles;
      const int dpl = vec ? launch_bonds<true>(variant, rc, st, A, &ptiles)
                          : launch_bonds<false>(variant, rc, st, A, &ptiles);
      if (dpl == yk::DP_QTE)
        YK_LAUNCH(yk::k_dte_sum, (long long)N * ((E + 15) / 16) * ((V + 3) / 4), 256, st, ws.dpart, N, V,
                  ptiles, A.ep, 0, E, io->dsum_part);
      else
        YK_LAUNCH(yk::k_dsum_canon, ns, 256, st, ws.dpart, V, ptiles, io->dsum_part, dpl);
      break;
    }
    case 5: {
      if (!io->dsum) return fail(YUMA_EINVAL, "stage 5 needs io->dsum");
      if (full && !io->tv) return fail(YUMA_EINVAL, "stage 5 with out->Tv needs io->tv");
      if (V > yk::kRegRows)
        YK_LAUNCH(yk::k_finalize_big, ns, 256, st, io->dsum, ws.sn, variant, V, 0LL, 1,
                  full ? io->tv : nullptr, full ? io->tv + ns * V : nullptr, out->Dn, out->D, out->Tv,
                  (int)yk::DP_TV, 1, ws.dsum);
      else
        YK_LAUNCH(yk::k_finalize, ns, 256, st, io->dsum, ws.sn, variant, V, 0LL, 1,
                  full ? io->tv : nullptr, full ? io->tv + ns * V : nullptr, out->Dn, out->D,
                  out->Tv, (int)yk::DP_TV, 1);
      if (out->Sn != nullptr)
        (void)hipMemcpyAsync(out->Sn, ws.sn, (size_t)ns * V * 4, hipMemcpyDeviceToDevice, st);
      if (out->alpha_ab != nullptr)
        (void)hipMemcpy2DAsync(out->alpha_ab, 2 * sizeof(float), ws.scal + 1, 8 * sizeof(float),
                               2 * sizeof(float), (size_t)ns, hipMemcpyDeviceToDevice, st);
      break;
    }
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(YUMA_EHIP, "HIP launch failed: %s", hipGetErrorString(e));
  return YUMA_OK;
}

}  // namespace

struct yuma_graph {
  hipGraph_t graph;
  hipGraphExec_t exec;
};

extern "C" {

size_t yuma_workspace_bytes(int variant, int N, int E, int V, int M, int full_outputs) {
  if (N < 1 || E < 1 || V < 1 || M < 1) return 0;
  return carve(nullptr, variant, N, E, V, M, full_outputs).bytes;
}

int yuma_run(int variant, const yuma_params_t* params_dev, int N, int E, int V, int M,
             const float* W, const float* S, const float* B_init, const float* Wprev_init,
             const yuma_outputs_t* out, void* workspace, size_t workspace_bytes,
             int chunk_epochs, void* stream) {
  return run_impl(variant, params_dev, N, E, V, M, W, S, B_init, Wprev_init, out, workspace,
                  workspace_bytes, chunk_epochs, stream);
}

int yuma_run_ex(int variant, const yuma_params_t* params_dev, int N, int E, int V, int M,
                const float* W, const float* S, const float* B_init, const float* Wprev_init,
                const yuma_outputs_t* out, void* workspace, size_t workspace_bytes,
                int chunk_epochs, int flags, void* stream, float* phase_ms) {
  if (flags & ~YUMA_RUN_SHARED_INPUTS) return fail(YUMA_EINVAL, "unknown run flags 0x%x", flags);
  return run_impl(variant, params_dev, N, E, V, M, W, S, B_init, Wprev_init, out, workspace,
                  workspace_bytes, chunk_epochs, stream, phase_ms,
                  (flags & YUMA_RUN_SHARED_INPUTS) ? 1 : 0);
}

int yuma_run_profiled(int variant, const yuma_params_t* params_dev, int N, int E, int V, int M,
                      const float* W, const float* S, const float* B_init,
                      const float* Wprev_init, const yuma_outputs_t* out, void* workspace,
                      size_t workspace_bytes, int chunk_epochs, void* stream, float* phase_ms) {
  if (phase_ms == nullptr) return fail(YUMA_EINVAL, "phase_ms is required");
  return run_impl(variant, params_dev, N, E, V, M, W, S, B_init, Wprev_init, out, workspace,
                  workspace_bytes, chunk_epochs, stream, phase_ms);
}

int yuma_epoch(int variant, const yuma_params_t* params_dev, int N, int V, int M,
               const float* W, const float* W_prev, const float* S, const float* B_old,
               const yuma_outputs_t* out, void* workspace, size_t workspace_bytes,
               void* stream) {
  return run_impl(variant, params_dev, N, 1, V, M, W, S, B_old, W_prev, out, workspace,
                  workspace_bytes, 1, stream);
}

int yuma_synth_weights(uint64_t seed, int E, int N, int V, int M, int t0, float* W,
                       void* stream) {
  if (E < 1 || N < 1 || V < 1 || M < 1 || !W) return fail(YUMA_EINVAL, "bad synth args");
  if (M > 16777215) return fail(YUMA_EINVAL, "M too large for exact synthetic weights");
  const long long total = (long long)E * N * V * M;
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  YK_LAUNCH(yk::k_synth, blocks, 256, stream, seed, E, N, V, M, t0, W);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(YUMA_EHIP, "HIP launch failed: %s", hipGetErrorString(e));
  return YUMA_OK;
}

int yuma_shard_stage(int stage, int variant, const yuma_params_t* params_dev, int N, int E,
                     int V, int M, const float* W, const float* S, const float* B_init,
                     const float* Wprev_init, const yuma_shard_io_t* io,
                     const yuma_outputs_t* out, void* workspace, size_t workspace_bytes,
                     void* stream) {
  return shard_stage_impl(stage, variant, params_dev, N, E, V, M, W, S, B_init, Wprev_init, io,
                          out, workspace, workspace_bytes, stream);
}

int yuma_graph_create_ex(yuma_graph_t* graph, int variant, const yuma_params_t* params_dev, int N,
                         int E, int V, int M, const float* W, const float* S,
                         const float* B_init, const float* Wprev_init, const yuma_outputs_t* out,
                         void* workspace, size_t workspace_bytes, int chunk_epochs, int flags) {
  if (flags & ~YUMA_RUN_SHARED_INPUTS) return fail(YUMA_EINVAL, "unknown run flags 0x%x", flags);
  if (graph == nullptr) return fail(YUMA_EINVAL, "graph handle pointer is NULL");
  *graph = nullptr;
  hipStream_t cs = nullptr;
  if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess)
    return fail(YUMA_EHIP, "capture stream creation failed");
  if (hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed) != hipSuccess) {
    (void)hipStreamDestroy(cs);
    return fail(YUMA_EHIP, "hipStreamBeginCapture failed");
  }
  const int rc = run_impl(variant, params_dev, N, E, V, M, W, S, B_init, Wprev_init, out,
                          workspace, workspace_bytes, chunk_epochs, cs, nullptr,
                          (flags & YUMA_RUN_SHARED_INPUTS) ? 1 : 0);
  hipGraph_t g = nullptr;
  const hipError_t ec = hipStreamEndCapture(cs, &g);
  (void)hipStreamDestroy(cs);
  if (rc != YUMA_OK) {
    if (g) (void)hipGraphDestroy(g);
    return rc;  // run_impl's message stands
  }
  if (ec != hipSuccess || g == nullptr)
    return fail(YUMA_EHIP, "hipStreamEndCapture failed: %s", hipGetErrorString(ec));
  hipGraphExec_t x = nullptr;
  if (hipGraphInstantiate(&x, g, nullptr, nullptr, 0) != hipSuccess) {
    (void)hipGraphDestroy(g);
    return fail(YUMA_EHIP, "hipGraphInstantiate failed");
  }
  *graph = new yuma_graph{g, x};
  return YUMA_OK;
}

int yuma_graph_create(yuma_graph_t* graph, int variant, const yuma_params_t* params_dev, int N,
                      int E, int V, int M, const float* W, const float* S,
                      const float* B_init, const float* Wprev_init, const yuma_outputs_t* out,
                      void* workspace, size_t workspace_bytes, int chunk_epochs) {
  return yuma_graph_create_ex(graph, variant, params_dev, N, E, V, M, W, S, B_init, Wprev_init, out,
                              workspace, workspace_bytes, chunk_epochs, 0);
}

int yuma_graph_launch(yuma_graph_t graph, void* stream) {
  if (graph == nullptr) return fail(YUMA_EINVAL, "NULL graph");
  const hipError_t e = hipGraphLaunch(graph->exec, (hipStream_t)stream);
  if (e != hipSuccess) return fail(YUMA_EHIP, "hipGraphLaunch failed: %s", hipGetErrorString(e));
  return YUMA_OK;
}

int yuma_graph_nodes(yuma_graph_t graph) {
  if (graph == nullptr) return fail(YUMA_EINVAL, "NULL graph");
  size_t n = 0;
  if (hipGraphGetNodes(graph->graph, nullptr, &n) != hipSuccess)
    return fail(YUMA_EHIP, "hipGraphGetNodes failed");
  return (int)n;
}

int yuma_graph_destroy(yuma_graph_t graph) {
  if (graph == nullptr) return YUMA_OK;
  (void)hipGraphExecDestroy(graph->exec);
  (void)hipGraphDestroy(graph->graph);
  delete graph;
  return YUMA_OK;
}

const char* yuma_last_error(void) { return g_err; }
const char* yuma_version(void) { return YUMA_VERSION_STRING; }
const char* yuma_build_id(void) { return YUMA_BUILD_ID; }

}  // extern "C"
