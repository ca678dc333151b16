// Device-side helpers shared by the gfx950 kernels (wave64 everywhere).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pr {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ unsigned long long lanemask_lt() {
  const int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Inclusive prefix sum over the 64 lanes of a wave.
template <class T>
__device__ __forceinline__ T wave_inclusive_scan(T x) {
  const int l = lane_id();
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    T y = __shfl_up(x, off, kWave);
    if (l >= off) x += y;
  }
  return x;
}

// Fixed-order (deterministic) wave reduction; result valid in every lane.
__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) x += __shfl_xor(x, off, kWave);
  return x;
}

// Exclusive block scan for blockDim.x == NT (multiple of 64).  `scratch` holds NT/64 values.
// Returns the exclusive prefix; *total gets the block total.  Contains __syncthreads().
template <int NT, class T>
__device__ __forceinline__ T block_exclusive_scan(T x, T *scratch, T *total) {
  constexpr int NW = NT / kWave;
  T inc = wave_inclusive_scan(x);
  if (lane_id() == kWave - 1) scratch[wave_id()] = inc;
  __syncthreads();
  T base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    T v = scratch[w];
    if (w < wave_id()) base += v;
    tot += v;
  }
  __syncthreads();
  *total = tot;
  return base + inc - x;
}

// Deterministic block sum of doubles (fixed tree); result valid in every thread.
template <int NT>
__device__ __forceinline__ double block_sum(double x, double *scratch) {
  constexpr int NW = NT / kWave;
  x = wave_sum(x);
  if (lane_id() == 0) scratch[wave_id()] = x;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < NW; ++w) t += scratch[w];
  __syncthreads();
  return t;
}

// Deterministic block sum of two doubles at once (one barrier pair).
template <int NT>
__device__ __forceinline__ double2 block_sum2(double2 x, double2 *scratch) {
  constexpr int NW = NT / kWave;
  x.x = wave_sum(x.x);
  x.y = wave_sum(x.y);
  if (lane_id() == 0) scratch[wave_id()] = x;
  __syncthreads();
  double2 t = make_double2(0.0, 0.0);
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    t.x += scratch[w].x;
    t.y += scratch[w].y;
  }
  __syncthreads();
  return t;
}

}  // namespace pr
