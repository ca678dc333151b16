// k_spmv_units: the fused PageRank SpMV pass (Sparky.java:192-235), gfx950.
//
// One 256-thread workgroup per work unit (pr_internal.h).  Thread t owns the PT consecutive
// in-links [PT*t, PT*t + PT) of its unit: it loads their gather positions with 16-byte vector
// loads from the padded column array (every unit starts 32-byte aligned, so a wave reads one
// contiguous 64*PT*4-byte run) and issues PT independent 8-byte gathers of the contributions
// c[u] = r(u)/d(u) into registers.  No LDS staging of values.
//
//   STREAM unit (whole rows): every thread sums its values along row boundaries (unit-local row
//     pointers in LDS); rows that cross threads are completed by a wave64 segmented scan plus a
//     carry across the 4 waves; completed row sums go to LDS.  The epilogue then walks the unit's
//     rows (coalesced) and fuses the in-degree-0 quirk, r' = 0.15 + 0.85 (S + dc/N) without FMA,
//     c' = r'/d, the partial sum of r' over sink rows and the partial L1 norm.
//   PIECE unit (PT*256 in-links of one long row): one fixed-order block sum -> piece_part.
//
// All sums have a fixed order: results are bitwise reproducible.  Template knobs (used by the
// diagnostics library to A/B variants on the same graph): PT in-links per thread, NT = non-
// temporal column loads (streamed once per iteration), MASK_GATHER = diagnostic only.
#pragma once

#include <climits>

#include "pr_device.h"
#include "pr_internal.h"

namespace pr {

__device__ __forceinline__ double dc_from_slots(const double *cin, int P, int64_t S_pad) {
  double dc = 0.0;
  for (int p = 0; p < P; ++p) dc = __dadd_rn(dc, cin[(int64_t)p * S_pad + S_pad - 2]);
  return dc;
}

// r' = teleport + damping * (S + tdc), evaluated exactly as Sparky.java:233 (no contraction).
__device__ __forceinline__ double affine(double S, double tdc, double teleport, double damping) {
  return __dadd_rn(teleport, __dmul_rn(damping, __dadd_rn(S, tdc)));
}

typedef int pr_v4i __attribute__((ext_vector_type(4)));

template <int PT, bool NT>
__device__ __forceinline__ void load_cols(const int32_t *__restrict__ p, int32_t (&ci)[PT]) {
  static_assert(PT % 4 == 0, "PT must be a multiple of 4");
  const pr_v4i *q = reinterpret_cast<const pr_v4i *>(p);
#pragma unroll
  for (int k = 0; k < PT / 4; ++k) {
    pr_v4i x;
    if constexpr (NT) x = __builtin_nontemporal_load(q + k);
    else x = q[k];
    ci[4 * k + 0] = x.x;
    ci[4 * k + 1] = x.y;
    ci[4 * k + 2] = x.z;
    ci[4 * k + 3] = x.w;
  }
}

// Gather flavours (GM): 0 = plain global_load (product), 1 = nontemporal, 2 = agent-scope
// relaxed atomic load (sc1: bypasses L1), 3 = 4-byte gathers (diagnostics only: wrong values).
template <int GM>
__device__ __forceinline__ double gather(const double *__restrict__ cin, int32_t c) {
  if constexpr (GM == 1) return __builtin_nontemporal_load(cin + c);
  else if constexpr (GM == 2)
    return __longlong_as_double((long long)__hip_atomic_load(
        reinterpret_cast<const unsigned long long *>(cin + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  else if constexpr (GM == 3) return (double)reinterpret_cast<const float *>(cin)[c];
  else return cin[c];
}

template <int PT, bool NT, bool MASK_GATHER = false, int GM = 0, int XCLASS = 0>
__global__ __launch_bounds__(kThreads) void k_spmv_units(
    const Unit *__restrict__ units, const int64_t *__restrict__ rowptr,
    const int32_t *__restrict__ colp, const double *__restrict__ cin, double *__restrict__ cout,
    double *__restrict__ r, const uint32_t *__restrict__ rowinfo, double *__restrict__ piece_part,
    double2 *__restrict__ unit_part, int P, int64_t S_pad, double n_vertices, double teleport,
    double damping, uint32_t gather_mask) {
  __shared__ double rowsum[kUnitRows];
  __shared__ int32_t lrp[kUnitRows + 1];
  __shared__ double red[kThreads / kWave];
  __shared__ double2 red2[kThreads / kWave];
  __shared__ int32_t wrow_first[kThreads / kWave], wrow_last[kThreads / kWave];
  __shared__ double wval_last[kThreads / kWave];

  const int t = threadIdx.x, lane = lane_id(), w = wave_id();
  const Unit u = units[blockIdx.x];
  const int n = unit_n(u);
  const int i0 = t * PT;
  const bool stream = u.meta >= 0;
  const int nr = stream ? u.meta : 0;
  const int32_t r0 = u.r0;

  // Issue every load that does not depend on the gathers first, so a unit costs two dependent
  // memory round trips (columns -> gathers), not four: gather positions, the unit's row
  // pointers, and the first epilogue row's old rank and out-degree.
  int32_t ci[PT];
  if (i0 < n) {
    load_cols<PT, NT>(colp + (int64_t)u.p8 * 8 + i0, ci);
  } else {
#pragma unroll
    for (int j = 0; j < PT; ++j) ci[j] = 0;
  }
  int64_t rp_t = 0;
  double rold0 = 0.0;
  uint32_t info0 = 0;
  if (stream) {
    if (t <= nr) rp_t = rowptr[r0 + t];
    if (t < nr) {
      rold0 = r[(int64_t)r0 + t];
      info0 = rowinfo[(int64_t)r0 + t];
    }
  }

  // gather this thread's PT contributions (registers)
  double v[PT];
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    int32_t c = ci[j];
    if constexpr (MASK_GATHER) c = (int32_t)((uint32_t)c & gather_mask);
    if constexpr (XCLASS > 1)  // diagnostics only: emulate XCLASS column-line classes per XCD
      c = (c & ~((XCLASS - 1) << 4)) | (int32_t)((blockIdx.x & (XCLASS - 1)) << 4);
    if constexpr (XCLASS < 0) {  // diagnostics only: contiguous class regions by XCC id
      constexpr int C = -XCLASS, SH = (C == 8) ? 3 : ((C == 4) ? 2 : 1);
      uint32_t xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      c = (int32_t)((xcc & (C - 1)) * (uint32_t)(S_pad >> SH) + ((uint32_t)c >> SH));
    }
    v[j] = (i0 + j < n) ? gather<GM>(cin, c) : 0.0;
  }

  if (!stream) {  // ---- PIECE of a long row: fixed-order block sum ----
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < PT; ++j) acc = __dadd_rn(acc, v[j]);
    acc = block_sum<kThreads>(acc, red);
    if (t == 0) {
      piece_part[-u.meta - 1] = acc;
      unit_part[blockIdx.x] = make_double2(0.0, 0.0);
    }
    return;
  }

  // ---- STREAM unit ----
  const int64_t e0 = rowptr[r0];
  if (t <= nr) lrp[t] = (int32_t)(rp_t - e0);
  for (int k = t + kThreads; k <= nr; k += kThreads) lrp[k] = (int32_t)(rowptr[r0 + k] - e0);
  const double tdc = dc_from_slots(cin, P, S_pad) / n_vertices;
  __syncthreads();

  int carry_row = -1, first_row = -1;
  double carry_val = 0.0, first_sum = 0.0;
  if (i0 < n) {
    int lo = 0, hi = nr + 1;  // first k with lrp[k] > i0
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (lrp[mid] <= i0) lo = mid + 1;
      else hi = mid;
    }
    int cur = lo - 1;
    const int kstart = cur;
    const bool started_before = lrp[cur] < i0;
    int next_end = lrp[cur + 1];
    double acc = 0.0;
    bool open = false;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      if (i0 + j < n) {
        acc = __dadd_rn(acc, v[j]);
        open = true;
        if (i0 + j + 1 == next_end) {
          if (cur == kstart && started_before) {
            first_row = cur;
            first_sum = acc;
          } else {
            rowsum[cur] = acc;
          }
          acc = 0.0;
          open = false;
          ++cur;
          while (cur < nr && lrp[cur + 1] == lrp[cur]) ++cur;  // skip in-degree-0 rows
          next_end = (cur < nr) ? lrp[cur + 1] : INT_MAX;
        }
      }
    }
    if (open) {
      carry_row = cur;
      carry_val = acc;
    }
  }

  // Segmented inclusive scan of (carry_row, carry_val) over threads.  Equal rows are
  // contiguous in thread order, so a Hillis-Steele step may add the partner's value when the
  // partner carries the same row.
  int srow = carry_row;
  double sval = carry_val;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int prow = __shfl_up(srow, off, kWave);
    const double pval = __shfl_up(sval, off, kWave);
    if (lane >= off && srow >= 0 && prow == srow) sval = __dadd_rn(pval, sval);
  }
  const int lane0_row = __shfl(carry_row, 0, kWave);
  if (lane == kWave - 1) {
    wrow_last[w] = srow;
    wval_last[w] = sval;
    wrow_first[w] = lane0_row;
  }
  __syncthreads();
  int prow_in = -1;  // carry-in from earlier waves (identical in every lane)
  double pval_in = 0.0;
  for (int ww = 0; ww < w; ++ww) {
    const int rl = wrow_last[ww];
    const bool full = (rl >= 0) && (wrow_first[ww] == rl);
    if (full && prow_in == rl) {
      pval_in = __dadd_rn(pval_in, wval_last[ww]);
    } else {
      prow_in = rl;
      pval_in = (rl >= 0) ? wval_last[ww] : 0.0;
    }
  }
  if (srow >= 0 && srow == prow_in && lane0_row == srow) sval = __dadd_rn(pval_in, sval);
  int erow = __shfl_up(srow, 1, kWave);  // exclusive = inclusive of thread t-1
  double eval = __shfl_up(sval, 1, kWave);
  if (lane == 0) {
    erow = prow_in;
    eval = pval_in;
  }
  if (first_row >= 0) rowsum[first_row] = (erow == first_row) ? __dadd_rn(eval, first_sum) : first_sum;
  __syncthreads();

  // Epilogue over the unit's rows (coalesced).
  double dcp = 0.0, l1p = 0.0;
  for (int k = t; k < nr; k += kThreads) {
    const int64_t vtx = (int64_t)r0 + k;
    const double rold = (k == t) ? rold0 : r[vtx];
    const uint32_t info = (k == t) ? info0 : rowinfo[vtx];
    if (info & (kRowHole | kRowHeavy)) continue;
    const double S = (lrp[k + 1] > lrp[k]) ? rowsum[k] : rold;
    const double rn = affine(S, tdc, teleport, damping);
    r[vtx] = rn;
    const uint32_t d = info & kRowDegMask;
    if (d > 0) cout[vtx] = __ddiv_rn(rn, (double)d);
    else if (info & kRowSink) dcp = __dadd_rn(dcp, rn);
    l1p = __dadd_rn(l1p, fabs(rn - rold));
  }
  const double2 part = block_sum2<kThreads>(make_double2(dcp, l1p), red2);
  if (t == 0) unit_part[blockIdx.x] = part;
}

// ============================================================================================
// Split layout (C column classes, pr_graph.h): per-class row sums, then one epilogue pass.
// ============================================================================================

// Walk + segmented scan shared by both STREAM paths: every thread sums its PT values along the
// unit's row boundaries (lrp in LDS); completed row sums land in rowsum[] (LDS).
template <int PT>
__device__ __forceinline__ void stream_row_sums(const double (&v)[PT], int n, int nr, const int32_t *lrp,
                                                double *rowsum, int32_t *wrow_first, int32_t *wrow_last,
                                                double *wval_last) {
  const int t = threadIdx.x, lane = lane_id(), w = wave_id();
  const int i0 = t * PT;
  int carry_row = -1, first_row = -1;
  double carry_val = 0.0, first_sum = 0.0;
  if (i0 < n) {
    int lo = 0, hi = nr + 1;  // first k with lrp[k] > i0
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (lrp[mid] <= i0) lo = mid + 1;
      else hi = mid;
    }
    int cur = lo - 1;
    const int kstart = cur;
    const bool started_before = lrp[cur] < i0;
    int next_end = lrp[cur + 1];
    double acc = 0.0;
    bool open = false;
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      if (i0 + j < n) {
        acc = __dadd_rn(acc, v[j]);
        open = true;
        if (i0 + j + 1 == next_end) {
          if (cur == kstart && started_before) {
            first_row = cur;
            first_sum = acc;
          } else {
            rowsum[cur] = acc;
          }
          acc = 0.0;
          open = false;
          ++cur;
          while (cur < nr && lrp[cur + 1] == lrp[cur]) ++cur;
          next_end = (cur < nr) ? lrp[cur + 1] : INT_MAX;
        }
      }
    }
    if (open) {
      carry_row = cur;
      carry_val = acc;
    }
  }
  int srow = carry_row;
  double sval = carry_val;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int prow = __shfl_up(srow, off, kWave);
    const double pval = __shfl_up(sval, off, kWave);
    if (lane >= off && srow >= 0 && prow == srow) sval = __dadd_rn(pval, sval);
  }
  const int lane0_row = __shfl(carry_row, 0, kWave);
  if (lane == kWave - 1) {
    wrow_last[w] = srow;
    wval_last[w] = sval;
    wrow_first[w] = lane0_row;
  }
  __syncthreads();
  int prow_in = -1;
  double pval_in = 0.0;
  for (int ww = 0; ww < w; ++ww) {
    const int rl = wrow_last[ww];
    const bool full = (rl >= 0) && (wrow_first[ww] == rl);
    if (full && prow_in == rl) {
      pval_in = __dadd_rn(pval_in, wval_last[ww]);
    } else {
      prow_in = rl;
      pval_in = (rl >= 0) ? wval_last[ww] : 0.0;
    }
  }
  if (srow >= 0 && srow == prow_in && lane0_row == srow) sval = __dadd_rn(pval_in, sval);
  int erow = __shfl_up(srow, 1, kWave);
  double eval = __shfl_up(sval, 1, kWave);
  if (lane == 0) {
    erow = prow_in;
    eval = pval_in;
  }
  if (first_row >= 0) rowsum[first_row] = (erow == first_row) ? __dadd_rn(eval, first_sum) : first_sum;
  __syncthreads();
}

// Class-x work unit (launched at blockIdx % 8 == x): gathers only class-x contributions and
// writes partial[x][row] for every row of the unit (0 for rows without class-x in-links).
template <int PT, bool NT, bool MASK_GATHER = false>
__global__ __launch_bounds__(kThreads) void k_spmv_split(
    const Unit *__restrict__ units, const uint16_t *__restrict__ lens, const int32_t *__restrict__ colp,
    const double *__restrict__ cin, double *__restrict__ partial, double *__restrict__ piece_part,
    int64_t R, uint32_t gather_mask = 0xFFFFFFFFu) {
  static_assert(kUnitRows <= 4 * kThreads, "lens scan covers 4 rows per thread");
  __shared__ double rowsum[kUnitRows];
  __shared__ int32_t lrp[kUnitRows + 1];
  __shared__ double red[kThreads / kWave];
  __shared__ int32_t wrow_first[kThreads / kWave], wrow_last[kThreads / kWave];
  __shared__ double wval_last[kThreads / kWave];
  __shared__ uint32_t scan_scratch[kThreads / kWave];

  const int t = threadIdx.x;
  const Unit u = units[blockIdx.x];
  const int n = unit_n(u), x = unit_cls(u);
  if (u.meta == 0) return;  // empty padding unit (or a unit of zero rows)
  const int i0 = t * PT;
  const bool stream = u.meta > 0;
  const int nr = stream ? u.meta : 0;
  const int32_t r0 = u.r0;

  int32_t ci[PT];
  if (i0 < n) {
    load_cols<PT, NT>(colp + (int64_t)u.p8 * 8 + i0, ci);
  } else {
#pragma unroll
    for (int j = 0; j < PT; ++j) ci[j] = 0;
  }
  uint32_t l4[4] = {0, 0, 0, 0};
  if (stream) {  // streamed once per iteration: non-temporal, keep the L2 for contributions
    const uint16_t *lx = lens + (int64_t)x * (R + 1) + r0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * t + q < nr) l4[q] = __builtin_nontemporal_load(lx + 4 * t + q);
  }
  double v[PT];
#pragma unroll
  for (int j = 0; j < PT; ++j) {
    int32_t c = ci[j];
    if constexpr (MASK_GATHER) c = (int32_t)((uint32_t)c & gather_mask);  // diagnostics only
    v[j] = (i0 + j < n) ? cin[c] : 0.0;
  }

  if (!stream) {  // PIECE of a long (row, class) segment
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < PT; ++j) acc = __dadd_rn(acc, v[j]);
    acc = block_sum<kThreads>(acc, red);
    if (t == 0) piece_part[-u.meta - 1] = acc;
    return;
  }

  // unit-local row pointers from the class's uint16 row lengths
  uint32_t tot;
  const uint32_t base = block_exclusive_scan<kThreads>(l4[0] + l4[1] + l4[2] + l4[3], scan_scratch, &tot);
  {
    uint32_t acc = base;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (4 * t + q < nr) lrp[4 * t + q] = (int32_t)acc;
      acc += l4[q];
    }
    if (t == 0) lrp[nr] = (int32_t)tot;
  }
  __syncthreads();
  stream_row_sums<PT>(v, n, nr, lrp, rowsum, wrow_first, wrow_last, wval_last);
  double *px = partial + (int64_t)x * R + r0;
  for (int k = t; k < nr; k += kThreads)
    __builtin_nontemporal_store((lrp[k + 1] > lrp[k]) ? rowsum[k] : 0.0, px + k);
}

// Persistent form of k_spmv_split: gridDim (a multiple of 8) workgroups walk the unit list with
// stride gridDim, so unit k still runs at blockIdx % 8 == k % 8 (its class's XCD).  While one
// unit is reduced, the next unit's gather positions are already in flight (descriptor two units
// ahead), hiding the HBM latency that bounds a one-unit-per-workgroup launch.
template <int PT, bool NT>
__device__ __forceinline__ void split_unit(const Unit &u, const int32_t (&ci)[PT], const uint16_t *__restrict__ lens,
                                           const double *__restrict__ cin, double *__restrict__ partial,
                                           double *__restrict__ piece_part, int64_t R, double *rowsum,
                                           int32_t *lrp, double *red, int32_t *wrow_first, int32_t *wrow_last,
                                           double *wval_last, uint32_t *scan_scratch) {
  const int t = threadIdx.x;
  const int n = unit_n(u), x = unit_cls(u);
  const int i0 = t * PT;
  const bool stream = u.meta > 0;
  const int nr = stream ? u.meta : 0;
  const int32_t r0 = u.r0;
  uint32_t l4[4] = {0, 0, 0, 0};
  if (stream) {
    const uint16_t *lx = lens + (int64_t)x * (R + 1) + r0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * t + q < nr) l4[q] = __builtin_nontemporal_load(lx + 4 * t + q);
  }
  double v[PT];
#pragma unroll
  for (int j = 0; j < PT; ++j) v[j] = (i0 + j < n) ? cin[ci[j]] : 0.0;
  if (!stream) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < PT; ++j) acc = __dadd_rn(acc, v[j]);
    acc = block_sum<kThreads>(acc, red);
    if (t == 0) piece_part[-u.meta - 1] = acc;
    return;
  }
  uint32_t tot;
  const uint32_t base = block_exclusive_scan<kThreads>(l4[0] + l4[1] + l4[2] + l4[3], scan_scratch, &tot);
  {
    uint32_t acc = base;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (4 * t + q < nr) lrp[4 * t + q] = (int32_t)acc;
      acc += l4[q];
    }
    if (t == 0) lrp[nr] = (int32_t)tot;
  }
  __syncthreads();
  stream_row_sums<PT>(v, n, nr, lrp, rowsum, wrow_first, wrow_last, wval_last);
  double *px = partial + (int64_t)x * R + r0;
  for (int k = t; k < nr; k += kThreads)
    __builtin_nontemporal_store((lrp[k + 1] > lrp[k]) ? rowsum[k] : 0.0, px + k);
  __syncthreads();  // rowsum / lrp are reused by the next unit
}

template <int PT, bool NT, int MINW = 1>
__global__ __launch_bounds__(kThreads, MINW) void k_spmv_split_persist(
    const Unit *__restrict__ units, int64_t n_units, const uint16_t *__restrict__ lens,
    const int32_t *__restrict__ colp, const double *__restrict__ cin, double *__restrict__ partial,
    double *__restrict__ piece_part, int64_t R) {
  __shared__ double rowsum[kUnitRows];
  __shared__ int32_t lrp[kUnitRows + 1];
  __shared__ double red[kThreads / kWave];
  __shared__ int32_t wrow_first[kThreads / kWave], wrow_last[kThreads / kWave];
  __shared__ double wval_last[kThreads / kWave];
  __shared__ uint32_t scan_scratch[kThreads / kWave];
  const int64_t stride = gridDim.x;
  int64_t k = blockIdx.x;
  if (k >= n_units) return;
  const int i0 = threadIdx.x * PT;
  const Unit empty{0, 0, 0, 0};
  Unit u = units[k];
  Unit un = (k + stride < n_units) ? units[k + stride] : empty;
  int32_t ci[PT];
  if (i0 < unit_n(u)) load_cols<PT, NT>(colp + (int64_t)u.p8 * 8 + i0, ci);
  else {
#pragma unroll
    for (int j = 0; j < PT; ++j) ci[j] = 0;
  }
  while (true) {
    const int64_t k1 = k + stride, k2 = k1 + stride;
    int32_t ci1[PT];
    if (k1 < n_units && i0 < unit_n(un)) load_cols<PT, NT>(colp + (int64_t)un.p8 * 8 + i0, ci1);
    else {
#pragma unroll
      for (int j = 0; j < PT; ++j) ci1[j] = 0;
    }
    const Unit unn = (k2 < n_units) ? units[k2] : empty;
    if (u.meta != 0)
      split_unit<PT, NT>(u, ci, lens, cin, partial, piece_part, R, rowsum, lrp, red, wrow_first, wrow_last,
                         wval_last, scan_scratch);
    if (k1 >= n_units) break;
    u = un;
    un = unn;
#pragma unroll
    for (int j = 0; j < PT; ++j) ci[j] = ci1[j];
    k = k1;
  }
}

// Long (row, class) segments: the sum of their pieces in piece order -> partial[x][row].
__global__ __launch_bounds__(kThreads) void k_seg_reduce(int64_t n_seg, const int32_t *__restrict__ seg_row,
                                                         const int32_t *__restrict__ seg_cls,
                                                         const int32_t *__restrict__ seg_p0,
                                                         const double *__restrict__ piece_part,
                                                         double *__restrict__ partial, int64_t R) {
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * (kThreads / kWave);
  for (int64_t q = (int64_t)blockIdx.x * (kThreads / kWave) + wave_id(); q < n_seg; q += nw) {
    const int32_t p0 = seg_p0[q], np = seg_p0[q + 1] - p0;
    double acc = 0.0;
    for (int k = lane; k < np; k += kWave) acc = __dadd_rn(acc, piece_part[p0 + k]);
    acc = wave_sum(acc);
    if (lane == 0) partial[(int64_t)seg_cls[q] * R + seg_row[q]] = acc;
  }
}

// Epilogue of the split layout over the heavy rows h: S = sum of the C class partials in class
// order (heavy rows always have in-links), then the fused update of k_spmv_units.
template <int C>
__global__ __launch_bounds__(kThreads) void k_epilogue(int64_t H, ClassGeom geo, const double *__restrict__ partial,
                                                       const uint32_t *__restrict__ rowinfo,
                                                       double *__restrict__ r, double *__restrict__ cout,
                                                       const double *__restrict__ cin, int P,
                                                       double n_vertices, double teleport, double damping,
                                                       double2 *__restrict__ ep_part) {
  __shared__ double2 red2[kThreads / kWave];
  const double tdc = dc_from_slots(cin, P, geo.S_pad) / n_vertices;
  double dcp = 0.0, l1p = 0.0;
  for (int64_t h = (int64_t)blockIdx.x * kThreads + threadIdx.x; h < H; h += (int64_t)gridDim.x * kThreads) {
    const int64_t L = geo.heavy_to_row(h);
    const uint32_t info = rowinfo[L];
    const double rold = r[L];
    double S = __builtin_nontemporal_load(partial + h);
#pragma unroll
    for (int x = 1; x < C; ++x) S = __dadd_rn(S, __builtin_nontemporal_load(partial + (int64_t)x * H + h));
    if (info & kRowIndeg0) S = rold;
    const double rn = affine(S, tdc, teleport, damping);
    r[L] = rn;
    const uint32_t d = info & kRowDegMask;
    if (d > 0) cout[L] = __ddiv_rn(rn, (double)d);
    else if (info & kRowSink) dcp = __dadd_rn(dcp, rn);
    l1p = __dadd_rn(l1p, fabs(rn - rold));
  }
  const double2 part = block_sum2<kThreads>(make_double2(dcp, l1p), red2);
  if (threadIdx.x == 0) ep_part[blockIdx.x] = part;
}

}  // namespace pr
