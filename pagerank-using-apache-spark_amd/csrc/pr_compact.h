// Stable stream compaction over an index domain [0, n): out[k] = xf(i) for the k-th i with
// pred(i).  Used by the graph build (dedupe of sorted keys, per-part edge filter) and by the
// device interner.  Two launches (count, write) with a host prefix over <= 2048 workgroup
// counts in between; build-time only, so the host round trip is acceptable.
#pragma once

#include <vector>

#include "pr_device.h"
#include "pr_internal.h"

namespace pr {

constexpr int kCompactThreads = 256;
constexpr int kCompactIPT = 8;
constexpr int kCompactTile = kCompactThreads * kCompactIPT;

template <class Pred>
__global__ __launch_bounds__(kCompactThreads) void k_compact_count(int64_t n, int64_t tiles_per_wg,
                                                                   Pred pred,
                                                                   uint32_t *__restrict__ counts) {
  __shared__ uint32_t scratch[kCompactThreads / kWave];
  const int64_t begin = (int64_t)blockIdx.x * tiles_per_wg * kCompactTile;
  int64_t end = begin + tiles_per_wg * kCompactTile;
  if (end > n) end = n;
  uint32_t c = 0;
  for (int64_t i = begin + threadIdx.x; i < end; i += kCompactThreads) c += pred(i) ? 1u : 0u;
  uint32_t tot;
  (void)block_exclusive_scan<kCompactThreads>(c, scratch, &tot);
  if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

template <class Pred, class Xform, class OutT>
__global__ __launch_bounds__(kCompactThreads) void k_compact_write(int64_t n, int64_t tiles_per_wg,
                                                                   Pred pred, Xform xf,
                                                                   const int64_t *__restrict__ offs,
                                                                   OutT *__restrict__ out) {
  __shared__ uint32_t scratch[kCompactThreads / kWave];
  const int64_t t0 = (int64_t)blockIdx.x * tiles_per_wg;
  int64_t run = offs[blockIdx.x];
  for (int64_t tile = t0; tile < t0 + tiles_per_wg; ++tile) {
    const int64_t base = tile * kCompactTile + (int64_t)threadIdx.x * kCompactIPT;
    if (tile * kCompactTile >= n) break;
    bool p[kCompactIPT];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kCompactIPT; ++j) {
      p[j] = (base + j < n) && pred(base + j);
      c += p[j] ? 1u : 0u;
    }
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan<kCompactThreads>(c, scratch, &tot);
    int64_t pos = run + ex;
#pragma unroll
    for (int j = 0; j < kCompactIPT; ++j)
      if (p[j]) out[pos++] = xf(base + j);
    run += tot;
  }
}

// Returns the number of selected items in *count (host).  `out` must have room for them;
// out == nullptr only counts.
template <class Pred, class Xform, class OutT>
int compact_index(int64_t n, Pred pred, Xform xf, OutT *out, int64_t *count, hipStream_t s) {
  *count = 0;
  if (n <= 0) return PR_OK;
  const int64_t ntiles = (n + kCompactTile - 1) / kCompactTile;
  int nwg = (int)(ntiles < 2048 ? ntiles : 2048);
  const int64_t tpw = (ntiles + nwg - 1) / nwg;
  nwg = (int)((ntiles + tpw - 1) / tpw);
  DevBuf counts, offs;
  PR_TRY(counts.alloc(sizeof(uint32_t) * nwg));
  PR_TRY(offs.alloc(sizeof(int64_t) * nwg));
  hipLaunchKernelGGL(k_compact_count<Pred>, dim3(nwg), dim3(kCompactThreads), 0, s, n, tpw, pred,
                     counts.as<uint32_t>());
  PR_HIP(hipGetLastError());
  std::vector<uint32_t> hc(nwg);
  std::vector<int64_t> ho(nwg);
  PR_HIP(hipMemcpyAsync(hc.data(), counts.p, sizeof(uint32_t) * nwg, hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  int64_t acc = 0;
  for (int w = 0; w < nwg; ++w) { ho[w] = acc; acc += hc[w]; }
  if (out == nullptr) {  // count only
    *count = acc;
    return PR_OK;
  }
  PR_HIP(hipMemcpyAsync(offs.p, ho.data(), sizeof(int64_t) * nwg, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL((k_compact_write<Pred, Xform, OutT>), dim3(nwg), dim3(kCompactThreads), 0, s,
                     n, tpw, pred, xf, offs.as<int64_t>(), out);
  PR_HIP(hipGetLastError());
  PR_HIP(hipStreamSynchronize(s));
  *count = acc;
  return PR_OK;
}

}  // namespace pr
