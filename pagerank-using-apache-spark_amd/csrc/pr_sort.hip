// Hand-written stable LSD radix sort of u64 keys for gfx950 (K1 in SURVEY.md §2.1).
//
// Replaces the hash shuffles of `distinct().groupByKey()` (Sparky.java:124): the graph build
// sorts packed (dst << b | src) keys, after which duplicates are adjacent and every row of the
// in-link CSR is a contiguous run.
//
// One pass per 8-bit digit, three launches per pass:
//   k_digit_hist    per-workgroup digit histogram of a contiguous chunk of tiles
//   k_scan_hist     exclusive scan of the [digit][workgroup] histogram (one workgroup)
//   k_scatter       per tile: wave64 match-any ranking (8 ballots), tile-local counting sort
//                   in LDS, then runs of equal digits are written out contiguously.
// Workgroup w owns a contiguous chunk, so global order = (digit, workgroup, tile, index):
// the sort is stable.  No inter-workgroup communication inside a launch.
#include <vector>

#include "pr_device.h"
#include "pr_internal.h"

namespace pr {
namespace {

constexpr int kSortThreads = 256;
constexpr int kSortKPT = 8;
constexpr int kTile = kSortThreads * kSortKPT;  // 2048 keys
constexpr int kMaxSortWG = 2048;

__global__ __launch_bounds__(kSortThreads) void k_digit_hist(const uint64_t *__restrict__ keys,
                                                             int64_t n, int64_t tiles_per_wg,
                                                             int shift, uint32_t mask,
                                                             uint32_t *__restrict__ hist, int nwg) {
  __shared__ uint32_t h[4 * 256];
  for (int i = threadIdx.x; i < 4 * 256; i += kSortThreads) h[i] = 0;
  __syncthreads();
  const int64_t begin = (int64_t)blockIdx.x * tiles_per_wg * kTile;
  int64_t end = begin + tiles_per_wg * kTile;
  if (end > n) end = n;
  uint32_t *hw = h + wave_id() * 256;
  for (int64_t i = begin + threadIdx.x; i < end; i += kSortThreads) {
    const uint32_t d = (uint32_t)(keys[i] >> shift) & mask;
    atomicAdd(&hw[d], 1u);
  }
  __syncthreads();
  const int t = threadIdx.x;
  hist[(size_t)t * nwg + blockIdx.x] = h[t] + h[256 + t] + h[512 + t] + h[768 + t];
}

// Exclusive scan of m uint32 values in place with one 1024-thread workgroup.
__global__ __launch_bounds__(1024) void k_scan_hist(uint32_t *__restrict__ a, int64_t m) {
  __shared__ uint32_t scratch[16];
  const int64_t per = (m + 1023) / 1024;
  const int64_t b = threadIdx.x * per;
  int64_t e = b + per;
  if (e > m) e = m;
  uint32_t s = 0;
  for (int64_t i = b; i < e; ++i) s += a[i];
  uint32_t tot;
  uint32_t run = block_exclusive_scan<1024>(s, scratch, &tot);
  for (int64_t i = b; i < e; ++i) {
    uint32_t v = a[i];
    a[i] = run;
    run += v;
  }
}

__global__ __launch_bounds__(kSortThreads) void k_scatter(const uint64_t *__restrict__ in,
                                                          uint64_t *__restrict__ out, int64_t n,
                                                          int64_t tiles_per_wg, int shift,
                                                          int nbits,
                                                          const uint32_t *__restrict__ hist,
                                                          int nwg) {
  __shared__ uint32_t run_off[256];
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t tile_off[256];
  __shared__ uint32_t dig_tot[256];
  __shared__ uint32_t scratch[4];
  __shared__ uint64_t sorted[kTile];

  const int t = threadIdx.x, w = wave_id(), lane = lane_id();
  const uint32_t mask = (nbits >= 32) ? 0xFFFFFFFFu : ((1u << nbits) - 1u);
  run_off[t] = hist[(size_t)t * nwg + blockIdx.x];
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_wg;
  const int64_t ntiles = (n + kTile - 1) / kTile;
  int64_t t1 = t0 + tiles_per_wg;
  if (t1 > ntiles) t1 = ntiles;
  const unsigned long long lt = lanemask_lt();

  for (int64_t tile = t0; tile < t1; ++tile) {
    const int64_t base = tile * kTile;
    uint64_t k[kSortKPT];
    uint32_t d[kSortKPT];
    uint32_t rank[kSortKPT];
    bool valid[kSortKPT];
#pragma unroll
    for (int j = 0; j < kSortKPT; ++j) {
      const int64_t idx = base + w * (kSortKPT * kWave) + j * kWave + lane;
      valid[j] = idx < n;
      k[j] = valid[j] ? in[idx] : 0ull;
      d[j] = (uint32_t)(k[j] >> shift) & mask;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) wcnt[w][lane * 4 + q] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSortKPT; ++j) {
      unsigned long long peers = __ballot(valid[j]);
      for (int b = 0; b < nbits; ++b) {
        const bool bit = (d[j] >> b) & 1u;
        const unsigned long long m = __ballot(bit);
        peers &= bit ? m : ~m;
      }
      const uint32_t below = __popcll(peers & lt);
      const uint32_t cnt = __popcll(peers);
      uint32_t basev = 0;
      if (valid[j]) basev = wcnt[w][d[j]];
      __builtin_amdgcn_wave_barrier();
      if (valid[j] && below == 0) wcnt[w][d[j]] = basev + cnt;
      __builtin_amdgcn_wave_barrier();
      rank[j] = basev + below;
    }
    __syncthreads();
    {
      const uint32_t c0 = wcnt[0][t], c1 = wcnt[1][t], c2 = wcnt[2][t], c3 = wcnt[3][t];
      wcnt[0][t] = 0;
      wcnt[1][t] = c0;
      wcnt[2][t] = c0 + c1;
      wcnt[3][t] = c0 + c1 + c2;
      const uint32_t tot = c0 + c1 + c2 + c3;
      dig_tot[t] = tot;
      uint32_t all;
      tile_off[t] = block_exclusive_scan<kSortThreads>(tot, scratch, &all);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSortKPT; ++j)
      if (valid[j]) sorted[tile_off[d[j]] + wcnt[w][d[j]] + rank[j]] = k[j];
    __syncthreads();
    int64_t rem = n - base;
    const int tile_n = rem < kTile ? (int)rem : kTile;
#pragma unroll
    for (int q = 0; q < kSortKPT; ++q) {
      const int j = q * kSortThreads + t;
      if (j < tile_n) {
        const uint64_t key = sorted[j];
        const uint32_t dd = (uint32_t)(key >> shift) & mask;
        out[(size_t)run_off[dd] + (uint32_t)(j - (int)tile_off[dd])] = key;
      }
    }
    __syncthreads();
    run_off[t] += dig_tot[t];
    __syncthreads();
  }
}

}  // namespace

int radix_sort_u64(uint64_t *keys, uint64_t *tmp, int64_t n, int begin_bit, int end_bit,
                   hipStream_t s) {
  if (n <= 1 || end_bit <= begin_bit) return PR_OK;
  if (n >= (int64_t(1) << 32)) return fail(PR_ERR_INVALID, "radix_sort_u64: n >= 2^32");
  const int64_t ntiles = (n + kTile - 1) / kTile;
  int nwg = (int)(ntiles < kMaxSortWG ? ntiles : kMaxSortWG);
  const int64_t tpw = (ntiles + nwg - 1) / nwg;
  nwg = (int)((ntiles + tpw - 1) / tpw);
  DevBuf hist;
  PR_TRY(hist.alloc(sizeof(uint32_t) * 256 * (size_t)nwg));
  uint64_t *src = keys, *dst = tmp;
  for (int shift = begin_bit; shift < end_bit; shift += 8) {
    int nbits = end_bit - shift;
    if (nbits > 8) nbits = 8;
    const uint32_t mask = (1u << nbits) - 1u;
    hipLaunchKernelGGL(k_digit_hist, dim3(nwg), dim3(kSortThreads), 0, s, src, n, tpw, shift,
                       mask, hist.as<uint32_t>(), nwg);
    hipLaunchKernelGGL(k_scan_hist, dim3(1), dim3(1024), 0, s, hist.as<uint32_t>(),
                       (int64_t)256 * nwg);
    hipLaunchKernelGGL(k_scatter, dim3(nwg), dim3(kSortThreads), 0, s, src, dst, n, tpw, shift,
                       nbits, hist.as<uint32_t>(), nwg);
    PR_HIP(hipGetLastError());
    uint64_t *x = src;
    src = dst;
    dst = x;
  }
  if (src != keys) PR_HIP(hipMemcpyAsync(keys, src, sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, s));
  PR_HIP(hipStreamSynchronize(s));  // `hist` is freed on return
  return PR_OK;
}

}  // namespace pr
