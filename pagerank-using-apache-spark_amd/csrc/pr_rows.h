// The row-block ("rows") layout's SpMV pass (Sparky.java:192-235) on gfx950: for graphs whose
// in-links the LDS hot sets of the split layout barely serve (uniform degrees, e.g. Erdos-Renyi:
// ~11 % of the in-links, against 74 % at R-MAT s26), so every in-link is a gather-space load
// anyway and the split layout's (row, class) partial slots -- nearly one per in-link there -- are
// pure overhead (237.5 M slots for 268.4 M in-links at ER s24).
//
// Layout (pr_graph.h, built in pr_build.hip):
//   tile        kRowsTile consecutive local rows, owned by ONE wave for a whole pass; the wave keeps
//               the tile's row sums in LDS (8 KiB), so no partial sum ever leaves the CU.
//   stream      the tile's in-links sorted by (region, row, gather position), region = gather
//               position >> kRowsRegionShift (1 MiB of contributions): all waves of a pass start
//               at region 0 and sweep the gather space in order, so an XCD's L2 holds the few
//               regions its waves are in, not the whole (Infinity-Cache-sized) space.
//   units       the stream cut into kWaveUnit-entry units (8 per lane), padded per tile; per entry a
//               32-bit code (byte offset of the contribution | end mark in bit 0) and the u16 row
//               within the tile.  A segment = a run of one row inside one region, also cut at unit
//               ends; its sum is added to the row's LDS accumulator (ds_add_f64: a row can recur
//               in a later region of the same unit), in stream order -- a fixed order, so results
//               are bitwise reproducible.
//   pass        one launch: wave w of the grid takes tile pass * n_waves + w, zeroes its
//               accumulators, sweeps its units, then runs the update for its rows (the in-degree-0
//               quirk, r' = 0.15 + 0.85 (S + dc/N) without FMA, c' = r'/d, the dangling and L1
//               partials) -- the epilogue is fused, there is no second kernel.
#pragma once

#include "pr_spmv.h"

namespace pr {

struct RowsUnitData {
  WaveCodes w;
  uint32_t row[kWavePT / 2];  // 8 u16 rows, two per word
};

// Unit k of the tile (descriptors over the tile's units): lane l's 8 codes (two 16-byte loads)
// and 8 rows (one 16-byte load); past the tile both read zeros (range check).
__device__ __forceinline__ void rows_unit_load(__amdgpu_buffer_rsrc_t cs, __amdgpu_buffer_rsrc_t rs, int k,
                                               RowsUnitData &d) {
  const int lane = lane_id();
  const uint32_t cb = (uint32_t)k * (kWaveUnit * 4) + (uint32_t)lane * kWavePT * 4;
#pragma unroll
  for (int q = 0; q < kWavePT / 4; ++q) {
    const pr_v4i x = __builtin_bit_cast(pr_v4i, __builtin_amdgcn_raw_buffer_load_b128(cs, cb + 16 * q, 0, 2));
    d.w.c[4 * q + 0] = (uint32_t)x.x;
    d.w.c[4 * q + 1] = (uint32_t)x.y;
    d.w.c[4 * q + 2] = (uint32_t)x.z;
    d.w.c[4 * q + 3] = (uint32_t)x.w;
  }
  const uint32_t rb = (uint32_t)k * (kWaveUnit * 2) + (uint32_t)lane * kWavePT * 2;
  const pr_v4i y = __builtin_bit_cast(pr_v4i, __builtin_amdgcn_raw_buffer_load_b128(rs, rb, 0, 2));
  d.row[0] = (uint32_t)y.x;
  d.row[1] = (uint32_t)y.y;
  d.row[2] = (uint32_t)y.z;
  d.row[3] = (uint32_t)y.w;
}

// Every entry is a gather-space load (no hot set): the code's byte offset, bit 0 masked.
__device__ __forceinline__ void rows_unit_gather(const WaveCodes &w, __amdgpu_buffer_rsrc_t crs, double (&v)[kWavePT]) {
#pragma unroll
  for (int j = 0; j < kWavePT; ++j)
    v[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(crs, w.c[j] & ~1u, 0, 0));
}

// The unit's segment sums into the tile's LDS accumulators.
__device__ __forceinline__ void rows_unit_reduce(const RowsUnitData &d, const double (&v)[kWavePT], double *acc) {
  const uint32_t meta = derive_meta(d.w);
  double sv[kWavePT], carry;
  wave_segmented_sums(meta, v, sv, &carry);
  const uint32_t endm = meta & 0xFFu;
  bool first = true;
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    if ((endm >> j) & 1u) {
      const uint32_t row = (d.row[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
      atomicAdd(acc + row, first ? __dadd_rn(carry, sv[j]) : sv[j]);  // ds_add_f64
      first = false;
    }
  }
}

// One pass of the row-block layout.  tile_u[t]: first unit of tile t (tile_u[n_tiles] = all
// units); rows of tile t: [t * kRowsTile, min(+kRowsTile, n_rows)).
__global__ __launch_bounds__(kRowsThreads) void k_spmv_rows(
    int pass, int64_t n_tiles, const int64_t *__restrict__ tile_u, const uint32_t *__restrict__ codes,
    const uint16_t *__restrict__ rows, const double *__restrict__ cin, uint32_t cin_bytes,
    double *__restrict__ cout, double *__restrict__ r, const uint32_t *__restrict__ rowinfo, int64_t n_rows,
    SlotPos sp, double n_vertices, double teleport, double damping, double2 *__restrict__ ep_part) {
  extern __shared__ double acc_all[];  // kRowsWaves tiles of kRowsTile row sums, then the block sum
  double2 *red2 = reinterpret_cast<double2 *>(acc_all + kRowsWaves * kRowsTile);
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(wave_id());
  double *acc = acc_all + wv * kRowsTile;
  const int64_t t = (int64_t)pass * gridDim.x * kRowsWaves + (int64_t)blockIdx.x * kRowsWaves + wv;
  double dcp = 0.0, l1p = 0.0;
  if (t < n_tiles) {
    for (int i = lane; i < kRowsTile; i += kWave) acc[i] = 0.0;
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc((void *)cin, 0, cin_bytes, 0x00020000);
    const int64_t u0 = tile_u[t];
    const int nu = (int)(tile_u[t + 1] - u0);  // nu * 2 KiB < 4 GiB: 32-bit descriptor offsets
    // per-tile descriptors: offsets stay 32-bit whatever the stream's size
    const __amdgpu_buffer_rsrc_t cs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(codes + u0 * kWaveUnit), 0, (uint32_t)nu * kWaveUnit * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(rows + u0 * kWaveUnit), 0, (uint32_t)nu * kWaveUnit * 2, 0x00020000);
    // ring of three units as in k_spmv_hot: codes of i+2 in flight while unit i is reduced, then
    // unit i+1's gathers (units past the tile read zeros)
    RowsUnitData d[3];
    double v[3][kWavePT];
    if (nu > 0) {
      rows_unit_load(cs, rs, 0, d[0]);
      rows_unit_load(cs, rs, 1, d[1]);
      rows_unit_gather(d[0].w, crs, v[0]);
      for (int k = 0; k < nu;) {
#pragma unroll
        for (int sl = 0; sl < 3; ++sl) {
          const int s1 = (sl + 1) % 3, s2 = (sl + 2) % 3;
          rows_unit_load(cs, rs, k + 2, d[s2]);
          rows_unit_reduce(d[sl], v[sl], acc);
          rows_unit_gather(d[s1].w, crs, v[s1]);
          if (++k >= nu) break;
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0);  // this wave's LDS adds have landed (no other wave touches acc)
    const double tdc = dc_from_slots(cin, sp) / n_vertices;
    const int64_t r0 = t * kRowsTile;
    const int nr = (int)min((int64_t)kRowsTile, n_rows - r0);
    for (int i = lane; i < nr; i += kWave) {
      const int64_t L = r0 + i;
      const uint32_t info = rowinfo[L];
      if (info & kRowHole) continue;
      const double rold = r[L];
      // no in-link: subtractByKey + union keeps the old rank (Sparky.java:224-225)
      const double S = (info & kRowIndeg0) ? rold : acc[i];
      const double rn = affine(S, tdc, teleport, damping);
      r[L] = rn;
      const uint32_t deg = info & kRowDegMask;
      if (deg > 0) cout[L] = __ddiv_rn(rn, (double)deg);
      else if (info & kRowSink) dcp = __dadd_rn(dcp, rn);
      l1p = __dadd_rn(l1p, fabs(rn - rold));
    }
  }
  const double2 part = block_sum2<kRowsThreads>(make_double2(dcp, l1p), red2);
  if (threadIdx.x == 0) ep_part[(int64_t)pass * gridDim.x + blockIdx.x] = part;
}

}  // namespace pr
