// The PageRank SpMV pass (Sparky.java:192-235) on gfx950: the product kernels only.
//
//   k_spmv_units    fused layout (small graphs): one 256-thread workgroup per work unit, the
//                   update fused into the same kernel
//   k_spmv_hot      split layout: the (row, column class) segment sums into partial slots, one
//                   1024-thread workgroup per CU holding the class's LDS hot set, an XCD's
//                   classes one after another (phases)
//   k_seg_reduce    split layout: long segments summed from their pieces in piece order
//   k_epilogue_grp  split layout: per row its segment sums in class order, then the update
//
// Every sum has a fixed order: results are bitwise reproducible.  A/B variants of these kernels
// are built as separate libraries (PR_LIB_PATH), never compiled into the product.
#pragma once

#include <climits>

#include "pr_device.h"
#include "pr_internal.h"

namespace pr {

// dc = the parts' dangling partials added in part order (identical on every part)
__device__ __forceinline__ double dc_from_slots(const double *cin, const SlotPos &sp) {
  double dc = 0.0;
  for (int p = 0; p < sp.n; ++p) dc = __dadd_rn(dc, cin[sp.pos[p]]);
  return dc;
}

// r' = teleport + damping * (S + tdc), evaluated exactly as Sparky.java:233 (no contraction).
__device__ __forceinline__ double affine(double S, double tdc, double teleport, double damping) {
  return __dadd_rn(teleport, __dmul_rn(damping, __dadd_rn(S, tdc)));
}

typedef int pr_v4i __attribute__((ext_vector_type(4)));
typedef int pr_v2i __attribute__((ext_vector_type(2)));
// LDS windows are written as doubles and read back as 16-byte int vectors (or written as u32
// offsets and then as doubles, wave_unit_gather_compact): these access types alias anything, so
// type-based alias analysis can never reorder such accesses of one window against each other.
typedef pr_v4i pr_v4i_alias __attribute__((may_alias));
typedef uint32_t pr_u32_alias __attribute__((may_alias));
typedef double pr_f64_alias __attribute__((may_alias));

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

// ============================================================================================
// Fused layout: k_spmv_units
// ============================================================================================
// Thread t owns the PT consecutive in-links [PT*t, PT*t + PT) of its unit: it loads their
// gather positions with 16-byte vector loads from the padded column array (every unit starts
// 32-byte aligned, so a wave reads one contiguous 64*PT*4-byte run) and issues PT independent
// 8-byte gathers of the contributions c[u] = r(u)/d(u) into registers.
//   STREAM unit (whole rows): every thread sums its values along row boundaries (unit-local row
//     pointers in LDS); rows that cross threads are completed by a wave64 segmented scan plus a
//     carry across the 4 waves; completed row sums go to LDS.  The epilogue then walks the unit's
//     rows (coalesced) and fuses the in-degree-0 quirk, r' = 0.15 + 0.85 (S + dc/N) without FMA,
//     c' = r'/d, the partial sum of r' over sink rows and the partial L1 norm.
//   PIECE unit (PT*256 in-links of one long row): one fixed-order block sum -> piece_part.
template <int PT, bool NT>
__global__ __launch_bounds__(kThreads) void k_spmv_units(
    const Unit *__restrict__ units, const int64_t *__restrict__ rowptr,
    const int32_t *__restrict__ colp, const double *__restrict__ cin, double *__restrict__ cout,
    double *__restrict__ r, const uint32_t *__restrict__ rowinfo, double *__restrict__ piece_part,
    double2 *__restrict__ unit_part, SlotPos sp, int64_t S_pad, double n_vertices, double teleport,
    double damping) {
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
  for (int j = 0; j < PT; ++j) v[j] = (i0 + j < n) ? cin[ci[j]] : 0.0;

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
  const double tdc = dc_from_slots(cin, sp) / n_vertices;
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
    if (info & kRowHole) continue;
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
// Split layout (C column classes, pr_graph.h): per-class segment sums, then one epilogue pass.
// ============================================================================================
// (row, class) segments are cut into wave units (pr_internal.h): one wavefront per unit, no
// workgroup barriers.  k_spmv_hot runs one 1024-thread workgroup per CU (its LDS holds the
// class's hot set, so only one fits).  Round-robin dispatch puts workgroup b on XCD b % 8; XCD k
// owns classes k, k + 8, ... and runs them one after another (one phase per class), so its L2
// only ever caches one class region of the gather space; the hot set is restaged per class.
//
// Per unit, lane l owns entries [8l, 8l + 8): two 16-byte buffer loads of entry codes (a wave
// reads 2 KiB contiguous; lanes past the unit read 0 through the descriptor's range check).
// Each entry costs one LDS read (hot codes: the most-gathered contributions, top out-degree
// first; every other lane reads slot 0 = 0.0) and one buffer load of the gather space (hot codes
// turn into offsets >= 2^31: range-checked away, no memory request), summed -- one of the two is
// an exact zero.  No branches, so the waits stay exact.  The loop is software-pipelined over a
// ring of three units: the codes of unit i+2 are in flight while unit i is reduced (its partial
// stores go out), then the gathers of unit i+1 are issued.
//
// STREAM reduction: each lane sums its values along its segment ends; segments that cross lanes
// are completed by a wave64 segmented scan in DPP (row_shr 1/2/4/8, row_bcast 15/31) whose
// per-step "add the partner" predicates are derived from where the ends are (derive_meta).
// Segment s of the unit is slot r0 + s, written through the wave's LDS staging window as
// coalesced 16-byte non-temporal stores.  PIECE: wave sum.

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const pr_v2i v = __builtin_bit_cast(pr_v2i, x);
  pr_v2i r;
  r.x = __builtin_amdgcn_update_dpp(0, v.x, CTRL, 0xF, 0xF, true);
  r.y = __builtin_amdgcn_update_dpp(0, v.y, CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, r);
}

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true);
}

// Inclusive wave64 scan of an int (row_shr 1/2/4/8, then row_bcast 15/31).
__device__ __forceinline__ int wave_incl_scan_i32(int x) {
  const int row = lane_id() >> 4;
  x += dpp_i32<0x111>(x);
  x += dpp_i32<0x112>(x);
  x += dpp_i32<0x114>(x);
  x += dpp_i32<0x118>(x);
  int p = dpp_i32<0x142>(x);
  if (row == 1 || row == 3) x += p;
  p = dpp_i32<0x143>(x);
  if (row >= 2) x += p;
  return x;
}

// Inclusive wave64 max-scan of a non-negative int (0 is neutral: what bound_ctrl reads).
__device__ __forceinline__ int wave_incl_max_i32(int x) {
  const int row = lane_id() >> 4;
  x = max(x, dpp_i32<0x111>(x));
  x = max(x, dpp_i32<0x112>(x));
  x = max(x, dpp_i32<0x114>(x));
  x = max(x, dpp_i32<0x118>(x));
  int p = dpp_i32<0x142>(x);
  if (row == 1 || row == 3) x = max(x, p);
  p = dpp_i32<0x143>(x);
  if (row >= 2) x = max(x, p);
  return x;
}

struct WaveCodes {
  uint32_t c[kWavePT];
};

// The unit's entry codes, lane l's entries [8l, 8l + 8) (two 16-byte loads; the descriptor's
// base and size are wave-uniform: u lives in SGPRs).
__device__ __forceinline__ void wave_unit_codes(const Unit &u, const uint32_t *__restrict__ colh, WaveCodes &w) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)(colh + (int64_t)u.p8 * 8), 0, u.n * 4, 0x00020000);
  const int base = lane_id() * kWavePT * 4;
#pragma unroll
  for (int q = 0; q < kWavePT / 4; ++q) {
    const pr_v4i x = __builtin_bit_cast(pr_v4i, __builtin_amdgcn_raw_buffer_load_b128(rs, base + 16 * q, 0, 2));
    w.c[4 * q + 0] = (uint32_t)x.x;
    w.c[4 * q + 1] = (uint32_t)x.y;
    w.c[4 * q + 2] = (uint32_t)x.z;
    w.c[4 * q + 3] = (uint32_t)x.w;
  }
}

// Compact codes (pr_internal.h kCodeC20): lane l's 8 low-index halves (one 16-byte load) and its
// side word of end marks and high bits (one 4-byte load); lanes past the unit read 0 (padding).
struct WaveCodesC20 {
  uint32_t w[kWavePT / 2];
  uint32_t s;
};
__device__ __forceinline__ void wave_unit_codes(const Unit &u, const uint16_t *__restrict__ code16,
                                                const uint32_t *__restrict__ cside, WaveCodesC20 &w) {
  const __amdgpu_buffer_rsrc_t rm =
      __builtin_amdgcn_make_buffer_rsrc((void *)(code16 + (int64_t)u.p8 * 8), 0, u.n * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsd =
      __builtin_amdgcn_make_buffer_rsrc((void *)(cside + (int64_t)u.p8), 0, u.n / 2, 0x00020000);
  const pr_v4i x = __builtin_bit_cast(pr_v4i, __builtin_amdgcn_raw_buffer_load_b128(rm, lane_id() * 16, 0, 2));
  w.w[0] = (uint32_t)x.x;
  w.w[1] = (uint32_t)x.y;
  w.w[2] = (uint32_t)x.z;
  w.w[3] = (uint32_t)x.w;
  w.s = __builtin_amdgcn_raw_buffer_load_b32(rsd, lane_id() * 4, 0, 2);
}

// 3-byte codes (kCodeC24, class regions up to 2^20 rows): the same low halves and a u64 side word
// (8 end marks, 4 high bits per entry; one 8-byte load).
struct WaveCodesC24 {
  uint32_t w[kWavePT / 2];
  uint64_t s;
};
__device__ __forceinline__ void wave_unit_codes(const Unit &u, const uint16_t *__restrict__ code16,
                                                const uint64_t *__restrict__ cside, WaveCodesC24 &w) {
  const __amdgpu_buffer_rsrc_t rm =
      __builtin_amdgcn_make_buffer_rsrc((void *)(code16 + (int64_t)u.p8 * 8), 0, u.n * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsd =
      __builtin_amdgcn_make_buffer_rsrc((void *)(cside + (int64_t)u.p8), 0, u.n, 0x00020000);
  const pr_v4i x = __builtin_bit_cast(pr_v4i, __builtin_amdgcn_raw_buffer_load_b128(rm, lane_id() * 16, 0, 2));
  w.w[0] = (uint32_t)x.x;
  w.w[1] = (uint32_t)x.y;
  w.w[2] = (uint32_t)x.z;
  w.w[3] = (uint32_t)x.w;
  w.s = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rsd, lane_id() * 8, 0, 2));
}

// Which of the lane's entries end a segment (bit j: entry j).
__device__ __forceinline__ uint32_t end_marks(const WaveCodes &w) {
  uint32_t endm = 0;
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) endm |= (w.c[j] & 1u) << j;
  return endm;
}
__device__ __forceinline__ uint32_t end_marks(const WaveCodesC20 &w) { return w.s & 0xFFu; }
__device__ __forceinline__ uint32_t end_marks(const WaveCodesC24 &w) { return (uint32_t)w.s & 0xFFu; }

// The lane metadata of a STREAM unit from the end marks of its entries: which of the lane's
// entries end a segment, the index (within the unit) of the lane's first segment end (an
// exclusive scan of the per-lane end counts), and the six "add the partner" predicates of the
// wave's segmented scan (step k: no segment end in the lanes from the partner + 1 to this one).
// The predicates come from one max-scan: d = distance to the last lane at or before this one
// that holds an end (t + 1 if none); the row_shr k step needs d >= k (and the partner in the
// row), row_bcast 15 d > r, row_bcast 31 d > t - 32.  About half the VALU of testing the end
// ballot per step.
struct LaneMeta {
  uint32_t endm;
  int excl;
  bool c[6];
};
__device__ __forceinline__ LaneMeta derive_meta(uint32_t endm) {
  LaneMeta m;
  m.endm = endm;
  const int t = lane_id(), r = t & 15, row = t >> 4;
  const int last1 = wave_incl_max_i32(endm ? t + 1 : 0);  // last lane <= t with an end, + 1 (0: none)
  const int d = t + 1 - last1;
  const int dr = min(d, r);
#pragma unroll
  for (int s = 0; s < 4; ++s) m.c[s] = dr >= (1 << s);
  m.c[4] = (row & 1) && d > r;
  m.c[5] = row >= 2 && d > t - 32;
  const int cnt = __builtin_popcount(endm);
  m.excl = wave_incl_scan_i32(cnt) - cnt;
  return m;
}

// The gather-space side of a class: 32-bit codes hold byte offsets into the whole gather space;
// compact codes hold region indices, so class x's descriptor starts past its hot positions
// (go = 8 idx - hb: hot and padding entries wrap to >= 2^31, out of range) and a cold entry's LDS
// read is clamped to the 0.0 slot at zb = 8 slots().
struct ClassSrc {
  __amdgpu_buffer_rsrc_t crs;
  uint32_t zb, hb;
  const uint32_t *tbl;  // piece codes: the class's piece table in LDS (pr_internal.h kCodeC20P)
};

// Byte offset of a compact code's cold source: past the class's hot positions (hot and padding
// entries wrap to >= 2^31: out of range); piece codes add their virtual block's delta (hot entries
// read the 0 sentinel and stay out of range).
template <bool PIECE>
__device__ __forceinline__ uint32_t cold_offset(uint32_t b8, const ClassSrc &cs) {
  if constexpr (PIECE) return piece_cold_offset(b8, cs.hb, cs.tbl);  // pr_pieces.h
  else return b8 - cs.hb;
}

// Cache policy of the cold gathers (aux bits of the buffer load); A/B builds only.
#ifndef PR_GATHER_AUX
#define PR_GATHER_AUX 0
#endif
// Attribution ladder of k_spmv_hot (A/B builds only, compact codes; 0 = the product):
//   1 every gather out of range (no cold gather; same instructions)   [wrong ranks]
//   2 no gather instructions at all (values from LDS only)           [wrong ranks]
//   3 one extra all-out-of-range gather per entry (TA cost of an idle gather instruction)
//   4 no partial-slot stores (the reduce still runs)                  [wrong ranks]
//   5 the hot set is loaded in the first phase only (stale values after) [wrong ranks]
//   6 = 2 + 4: no gather instructions and no partial-slot stores          [wrong ranks]
//   7 64 extra VALU instructions per unit (same results): is VALU on the critical path?
// (profiles/r06/README.md: the measured ladder, and the variants measured and removed)
#ifndef PR_HOT_DIAG
#define PR_HOT_DIAG 0
#endif

// The unit's values: per entry an LDS read (hot) and a range-checked gather-space load (cold),
// one of them an exact 0.
template <bool PIECE>
__device__ __forceinline__ void wave_unit_gather(const WaveCodes &w, const double *hot, const ClassSrc &cs,
                                                 double (&v)[kWavePT]) {
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    const uint32_t c = w.c[j] & ~1u;  // bit 0: segment end mark (end_marks)
    const uint32_t la = (int32_t)c < 0 ? 0u : c;
    const double a = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(hot) + la);
    const uint32_t go = c ^ kEntGlobal;  // LDS codes become offsets >= 2^31: out of range, no request
    const double b = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, go, 0, PR_GATHER_AUX));
    v[j] = __dadd_rn(a, b);
  }
}
template <bool PIECE>
__device__ __forceinline__ void wave_unit_gather(const WaveCodesC20 &w, const double *hot, const ClassSrc &cs,
                                                 double (&v)[kWavePT]) {
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    const uint32_t lo = (j & 1) ? (w.w[j >> 1] >> 16) : (w.w[j >> 1] & 0xFFFFu);
    const uint32_t idx = lo | (((w.s >> (8 + 3 * j)) & 7u) << 16);
    const uint32_t b8 = idx << 3;
    const uint32_t la = min(b8, cs.zb);  // hot: its slot; cold: the 0.0 slot
    const double a = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(hot) + la);
#if PR_HOT_DIAG == 1
    const double b = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, cold_offset<PIECE>(b8, cs) | kEntGlobal, 0, PR_GATHER_AUX));
#elif PR_HOT_DIAG == 2 || PR_HOT_DIAG == 6
    const double b = 0.0;
#elif PR_HOT_DIAG == 3
    const uint32_t off = cold_offset<PIECE>(b8, cs);
    const double b = __dadd_rn(__builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, off, 0, PR_GATHER_AUX)),
                               __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, off | kEntGlobal, 0, PR_GATHER_AUX)));
#else
    const double b = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, cold_offset<PIECE>(b8, cs), 0, PR_GATHER_AUX));
#endif
    v[j] = __dadd_rn(a, b);
  }
}

// Entry j of a lane: its LDS hot-set byte address (cold entries: the 0.0 slot) and its gather-space
// byte offset (hot and padding entries: >= 2^31, out of range).
template <bool PIECE>
__device__ __forceinline__ void entry_addr(const WaveCodes &w, int j, const ClassSrc &, uint32_t &la, uint32_t &go) {
  const uint32_t c = w.c[j] & ~1u;  // bit 0: segment end mark
  la = (int32_t)c < 0 ? 0u : c;
  go = c ^ kEntGlobal;
}
template <bool PIECE>
__device__ __forceinline__ void entry_addr(const WaveCodesC20 &w, int j, const ClassSrc &cs, uint32_t &la, uint32_t &go) {
  const uint32_t lo = (j & 1) ? (w.w[j >> 1] >> 16) : (w.w[j >> 1] & 0xFFFFu);
  const uint32_t b8 = (lo | (((w.s >> (8 + 3 * j)) & 7u) << 16)) << 3;
  la = min(b8, cs.zb);
  go = cold_offset<PIECE>(b8, cs);
}
template <bool PIECE>
__device__ __forceinline__ void entry_addr(const WaveCodesC24 &w, int j, const ClassSrc &cs, uint32_t &la, uint32_t &go) {
  const uint32_t lo = (j & 1) ? (w.w[j >> 1] >> 16) : (w.w[j >> 1] & 0xFFFFu);
  const uint32_t b8 = (lo | ((uint32_t)(w.s >> (8 + 4 * j)) & 15u) << 16) << 3;
  la = min(b8, cs.zb);
  go = cold_offset<PIECE>(b8, cs);
}

// The product's gathers (round 6): a unit's cold entries are gathered by dense instructions.  Every
// lane finds its cold entries' ranks (a wave scan of the per-lane counts), their offsets go
// through the wave's LDS window (256 at a time), each buffer load takes 64 of them, and the values
// come back through the window to the lanes that own them: ceil(cold / 64) gather instructions per
// unit instead of one per entry position (8), whose hot lanes were out of range -- an idle gather
// instruction costs ~24 us per pass at R-MAT s26 (profiles/r06/README.md §1).  R-MAT s26 -2.5 %
// per pass, Twitter shape -1.0 %, ER s24 -0.5 %, LiveJournal shape +0.7 %, s26 P = 8 parts
// unchanged (profiles/r06/README.md §6).  v[j] is bitwise the per-position a + b (one of them an
// exact zero).  The ladder builds (PR_HOT_DIAG) keep the per-position gathers above.
static_assert(kStageSlots >= 2 * kWave, "the compact gather window holds 128 values (256 offsets)");
template <bool PIECE, class WC>
__device__ __forceinline__ void wave_unit_gather_compact(const WC &w, const double *hot, const ClassSrc &cs,
                                                         double (&v)[kWavePT], double *win) {
  uint32_t off[kWavePT], la[kWavePT];
  uint32_t coldm = 0u;
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    entry_addr<PIECE>(w, j, cs, la[j], off[j]);
    coldm |= ((int32_t)off[j] >= 0 ? 1u : 0u) << j;
  }
  // the hot-set reads first: issued after the first round's gathers instead they cost +4.5 % (the
  // round's value write-back then queues behind them, profiles/r06/README.md §6)
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) v[j] = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(hot) + la[j]);
  const int cnt = __builtin_popcount(coldm);
  const int incl = wave_incl_scan_i32(cnt);
  const int excl = incl - cnt, total = __builtin_amdgcn_readlane(incl, kWave - 1);
  const int lane = lane_id();
  pr_u32_alias *win32 = reinterpret_cast<pr_u32_alias *>(win);
  pr_f64_alias *winf = reinterpret_cast<pr_f64_alias *>(win);
  // rounds of 256 cold entries (one round for most units at R-MAT s26): the window holds 256 u32 offsets,
  // so up to four gather instructions are in flight at once, and their values come back through it
  // in two halves of 128 (-0.8 % at s26 against rounds of 128 with two loads each, ER s24 the same:
  // profiles/r06/dense/r6_wide/)
  for (int base = 0; base < total; base += 4 * kWave) {
    int rk = excl - base;
#pragma unroll
    for (int j = 0; j < kWavePT; ++j) {
      const bool c = (coldm >> j) & 1u;
      if (c && (uint32_t)rk < (uint32_t)(4 * kWave)) win32[rk] = off[j];
      rk += c ? 1 : 0;
    }
    const int n = min(4 * kWave, total - base);
    const uint32_t a0 = lane < n ? win32[lane] : kEntGlobal;
    const uint32_t a1 = lane + kWave < n ? win32[lane + kWave] : kEntGlobal;
    const uint32_t a2 = lane + 2 * kWave < n ? win32[lane + 2 * kWave] : kEntGlobal;
    const uint32_t a3 = lane + 3 * kWave < n ? win32[lane + 3 * kWave] : kEntGlobal;
    const double g0 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, a0, 0, PR_GATHER_AUX));
    double g1 = 0.0, g2 = 0.0, g3 = 0.0;  // a further instruction only for each further 64 entries
    if (n > kWave) g1 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, a1, 0, PR_GATHER_AUX));
    if (n > 2 * kWave) g2 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, a2, 0, PR_GATHER_AUX));
    if (n > 3 * kWave) g3 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, a3, 0, PR_GATHER_AUX));
    winf[lane] = g0;  // the offsets are in a0..a3 already (the wave's LDS accesses run in order)
    if (n > kWave) winf[lane + kWave] = g1;
    rk = excl - base;
#pragma unroll
    for (int j = 0; j < kWavePT; ++j) {
      const bool c = (coldm >> j) & 1u;
      if (c && (uint32_t)rk < (uint32_t)(2 * kWave)) v[j] = winf[rk];
      rk += c ? 1 : 0;
    }
    if (n > 2 * kWave) {  // the second half, after the first half's reads (in order, as above)
      winf[lane] = g2;
      if (n > 3 * kWave) winf[lane + kWave] = g3;
      rk = excl - base - 2 * kWave;
#pragma unroll
      for (int j = 0; j < kWavePT; ++j) {
        const bool c = (coldm >> j) & 1u;
        if (c && (uint32_t)rk < (uint32_t)(2 * kWave)) v[j] = winf[rk];
        rk += c ? 1 : 0;
      }
    }
  }
}

template <bool PIECE>
__device__ __forceinline__ void wave_unit_gather(const WaveCodesC24 &w, const double *hot, const ClassSrc &cs,
                                                 double (&v)[kWavePT]) {
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    const uint32_t lo = (j & 1) ? (w.w[j >> 1] >> 16) : (w.w[j >> 1] & 0xFFFFu);
    const uint32_t idx = lo | ((uint32_t)(w.s >> (8 + 4 * j)) & 15u) << 16;
    const uint32_t b8 = idx << 3;
    const uint32_t la = min(b8, cs.zb);  // hot: its slot; cold: the 0.0 slot
    const double a = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(hot) + la);
    const double b = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(cs.crs, cold_offset<PIECE>(b8, cs), 0, PR_GATHER_AUX));
    v[j] = __dadd_rn(a, b);
  }
}

// Per-lane sums along the segment ends, then the wave's segmented scan; on return sv[j] is the
// lane's running sum at entry j (restarted after every end) and *carry the sum flowing into the
// lane's first segment from earlier lanes.
__device__ __forceinline__ void wave_segmented_sums(const LaneMeta &m, const double (&v)[kWavePT],
                                                    double (&sv)[kWavePT], double *carry) {
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    acc = __dadd_rn(acc, v[j]);
    sv[j] = acc;
    if (m.endm & (1u << j)) acc = 0.0;
  }
  // segmented inclusive scan of the lane tails
  double a = acc, p;
  p = dpp_f64<0x111>(a);  // row_shr:1
  if (m.c[0]) a = __dadd_rn(p, a);
  p = dpp_f64<0x112>(a);  // row_shr:2
  if (m.c[1]) a = __dadd_rn(p, a);
  p = dpp_f64<0x114>(a);  // row_shr:4
  if (m.c[2]) a = __dadd_rn(p, a);
  p = dpp_f64<0x118>(a);  // row_shr:8
  if (m.c[3]) a = __dadd_rn(p, a);
  p = dpp_f64<0x142>(a);  // row_bcast:15
  if (m.c[4]) a = __dadd_rn(p, a);
  p = dpp_f64<0x143>(a);  // row_bcast:31
  if (m.c[5]) a = __dadd_rn(p, a);
  *carry = dpp_f64<0x138>(a);  // wave_shr:1 (lane 0 reads 0)
}

// Segment sums of staged pass [base, base + kStageSlots) into the wave's LDS window; the lane's
// first segment end then gets the carry added in place (carry + its sum: the same add as before
// staging, one add per lane instead of a speculative one per entry).
__device__ __forceinline__ void stage_segment_sums(const LaneMeta &m, const double (&sv)[kWavePT], double carry,
                                                   int base, double *stage) {
  int e = m.excl - base;
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    const bool end = (m.endm >> j) & 1u;
    if (end && e >= 0 && e < kStageSlots) stage[e] = sv[j];
    e += end ? 1 : 0;
  }
  const int e0 = m.excl - base;
  if (m.endm != 0u && e0 >= 0 && e0 < kStageSlots) stage[e0] = __dadd_rn(carry, stage[e0]);
}


// A STREAM unit's segment sums, held in registers until they are stored (wave_unit_store).
struct UnitSums {
  LaneMeta m;
  double sv[kWavePT];
  double carry;
};

// The sums of one unit: a PIECE is summed and written here (false); a STREAM unit's segment sums go
// to `r` (true).
template <class WC>
__device__ __forceinline__ bool wave_unit_sums(const Unit &u, const WC &w, const double (&v)[kWavePT],
                                               double *__restrict__ piece_part, UnitSums &r) {
  if (u.meta < 0) {  // PIECE of a long segment
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < kWavePT; ++j) acc = __dadd_rn(acc, v[j]);
    acc = wave_sum(acc);
    if (lane_id() == 0) piece_part[-u.meta - 1] = acc;
    return false;
  }
  r.m = derive_meta(end_marks(w));
  wave_segmented_sums(r.m, v, r.sv, &r.carry);
  return true;
}

// The sums are staged in the wave's LDS window (kStageSlots at a time) and leave as coalesced
// stores: two slots per lane in one 16-byte non-temporal store (dword alignment is enough; half
// the store instructions of one 8-byte store per slot: -1.7 % at s26, profiles/r02/store_walk/),
// through a descriptor of the unit's own slots, so an odd last slot rides a 16-byte store whose
// second half the range check drops (it checks per dword; one store instruction per pass instead
// of a 16-byte and an 8-byte one: -0.6 % at s26, profiles/r06/README.md §6).  Non-temporal: the
// partials are read back by the epilogue only after every class has run, so they should not evict
// the class region from L2.
__device__ __forceinline__ void wave_unit_store(const Unit &u, const UnitSums &r, double *pcls, double *stage) {
  const int nseg = u.meta;
  static_assert(kStageSlots <= 2 * kWave, "one b128 pass");
  const __amdgpu_buffer_rsrc_t urs =
      __builtin_amdgcn_make_buffer_rsrc((void *)(pcls + u.r0), 0, (uint32_t)nseg * 8u, 0x00020000);
  for (int base = 0; base < nseg; base += kStageSlots) {
    stage_segment_sums(r.m, r.sv, r.carry, base, stage);
    const int n = min(kStageSlots, nseg - base);
    const int i2 = 2 * lane_id();
#if PR_HOT_DIAG == 4 || PR_HOT_DIAG == 6
    if (u.r0 != 0x7FFFFFFF) continue;  // never false: the stores are skipped, the reduce is kept
#endif
    if (i2 < n)
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const pr_v4i_alias *>(stage + i2), urs,
                                             (uint32_t)(base + i2) * 8u, 0, 2);
  }
}

// The code streams of a part (pr_internal.h): 32-bit codes, or compact low halves + side words
// (u32 per 8 entries for kCodeC20, u64 for kCodeC24).
struct CodeSrc {
  const void *codes;
  const uint32_t *side;
};
template <int CODE>
struct CodeOf {
  using T = WaveCodes;
};
template <>
struct CodeOf<kCodeC20> {
  using T = WaveCodesC20;
};
template <>
struct CodeOf<kCodeC24> {
  using T = WaveCodesC24;
};
template <>
struct CodeOf<kCodeC20P> {
  using T = WaveCodesC20;
};
template <>
struct CodeOf<kCodeC24P> {
  using T = WaveCodesC24;
};
template <int CODE>
__device__ __forceinline__ void unit_codes(const Unit &u, const CodeSrc &cd, typename CodeOf<CODE>::T &w) {
  if constexpr (CODE == kCodeC20 || CODE == kCodeC20P)
    wave_unit_codes(u, static_cast<const uint16_t *>(cd.codes), cd.side, w);
  else if constexpr (CODE == kCodeC24 || CODE == kCodeC24P)
    wave_unit_codes(u, static_cast<const uint16_t *>(cd.codes), reinterpret_cast<const uint64_t *>(cd.side), w);
  else wave_unit_codes(u, static_cast<const uint32_t *>(cd.codes), w);
}

// A unit's values: dense cold gathers (DENSE: many units per CU), or one gather instruction per
// entry position (small passes, where a unit's chain latency matters more than its instruction
// count: R-MAT s20 +11 % with dense gathers, LiveJournal shape +0.7 %; and the ladder builds,
// PR_HOT_DIAG, as measured in profiles/r06/README.md §1).
template <int CODE, bool DENSE>
__device__ __forceinline__ void unit_gather(const typename CodeOf<CODE>::T &w, const double *hot, const ClassSrc &cs,
                                            double (&v)[kWavePT], double *win) {
  if constexpr (DENSE && (!PR_HOT_DIAG || PR_HOT_DIAG == 7)) {
    wave_unit_gather_compact<code_is_piece(CODE)>(w, hot, cs, v, win);
  } else {
    (void)win;
    wave_unit_gather<code_is_piece(CODE)>(w, hot, cs, v);
  }
}

// One class's wave units with the class's hot set already in LDS.  The class's unit list is
// dealt to the XCD's `nteams` workgroups in slices of kWaves consecutive units every
// nteams * kWaves (this one is `team`; the slice rotates with the phase, so a workgroup on a
// slower CU does not take the same slice of every class: -0.6 % at s26), and a workgroup's waves
// take its units in order from a counter in a spare LDS word (zeroed before the class), so a slow
// wave takes fewer and the waves reach the class's end together (-3.5 % at s26 against a static
// interleave, profiles/r02/assign_lds_ab/).
template <int CODE, bool DENSE>
__device__ __forceinline__ void hot_class_units(int x, int team, int nteams, const Unit *__restrict__ units,
                                                const int64_t *__restrict__ ucum, const HotGeom &hg,
                                                const CodeSrc &cd, const double *hot, const ClassSrc &cs,
                                                double *__restrict__ partial, const int64_t *__restrict__ poff,
                                                double *__restrict__ piece_part, double *stage) {
  const int64_t p0 = poff[x];
  const int64_t beg = ucum[x], end = ucum[x + 1];
  constexpr int kWaves = kHotThreads / kWave;
  team = (team + 5 * (x / kXcds)) % nteams;
  const int64_t stride = (int64_t)nteams * kWaves;
  uint32_t *ctr = reinterpret_cast<uint32_t *>(const_cast<double *>(hot) + hg.ctr_slot());
  const int lane = lane_id();
  auto counter = [&]() -> uint32_t {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(ctr, 1u);
    return (uint32_t)__builtin_amdgcn_readlane((int)t, 0);
  };
  auto take = [&]() -> int64_t {
    const uint32_t t = counter();
    return beg + (int64_t)team * kWaves + (int64_t)(t % kWaves) + (int64_t)(t / kWaves) * stride;
  };
  int64_t k = take();
  if (k >= end) return;
  // unit descriptors through the scalar cache; index n_units (= ucum[kMaxClasses]) is an empty unit
  const __attribute__((address_space(4))) pr_v4i *cu = (const __attribute__((address_space(4))) pr_v4i *)units;
  auto unit_at = [&](int64_t i) -> Unit {
    const pr_v4i q = cu[i];
    return Unit{(uint32_t)q.x, q.y, q.z, q.w};
  };
  const int64_t none_k = ucum[kMaxClasses];
  // ring of three units: codes of i+2 in flight while unit i is reduced, then unit i+1's gathers
  Unit u[3];
  typename CodeOf<CODE>::T wc[3];
  double v[3][kWavePT];
  int64_t k1 = take();
  u[0] = unit_at(k);
  unit_codes<CODE>(u[0], cd, wc[0]);
  u[1] = unit_at(k1 < end ? k1 : none_k);
  unit_codes<CODE>(u[1], cd, wc[1]);
  unit_gather<CODE, DENSE>(wc[0], hot, cs, v[0], stage);
  while (true) {
#pragma unroll
    for (int sl = 0; sl < 3; ++sl) {
      const int s1 = (sl + 1) % 3, s2 = (sl + 2) % 3;
      const int64_t k2 = take();
      u[s2] = unit_at(k2 < end ? k2 : none_k);
      unit_codes<CODE>(u[s2], cd, wc[s2]);
      // reduce first: a gather issue stalled by a busy address unit cannot hold it up (ORDER 1:
      // -3.7 % at s26, profiles/r02/order_ab/; with the dense gathers, issuing unit i+1's first
      // round before unit i's sums and stores spilled 53 VGPRs at 4 waves per SIMD, between the
      // sums and the stores 51: not kept)
#if PR_HOT_DIAG == 7
      {  // ladder 7: 64 extra dependent VALU instructions per unit (is VALU on the critical path?)
        uint32_t d = (uint32_t)lane;
#pragma unroll
        for (int q = 0; q < 64; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(d) : "v"((uint32_t)q));
        if (d == 0xFFFFFFFFu) piece_part[0] = 0.0;  // never (keeps the chain)
      }
#endif
      UnitSums us;
      const bool stream = wave_unit_sums(u[sl], wc[sl], v[sl], piece_part, us);
      if (stream) wave_unit_store(u[sl], us, partial + p0, stage);
      // piece codes look their table delta up here; reading them before the reduce instead
      // measured the same (s26 P = 8 part 375 vs 371 us, profiles/r03/piece_codes/hoist_ab/)
      // (unit i+2's codes issued after unit i+1's first gathers instead: +2..7 % at s26, the codes
      // arrive later than the next decode needs them; profiles/r06/dense/r6_late/)
      unit_gather<CODE, DENSE>(wc[s1], hot, cs, v[s1], stage);
      k = k1;
      k1 = k2;
      if (k >= end) return;
    }
  }
}

// Stage class x's hot contributions (the previous iteration's, final before this launch) into LDS
// slots 1..nh, the 0.0 slots and the workgroup's unit counter (all 1024 threads; the caller's
// barrier follows): every position load, then every gather in flight before the first LDS write --
// a rolled loop pays two dependent memory latencies per element, 18 times per phase (-2.7 % at s26).
// CONTIG (one part, compact codes): the hot set is the first q_load positions of class x's region
// (pr_build.hip k_hot_tables), so it is read straight from there, one coalesced load per element
// and no dependent position load.
template <bool PIECE, bool CONTIG = false>
__device__ __forceinline__ void stage_hot_set(const HotGeom &hg, int x, const int32_t *__restrict__ hpos,
                                              const int32_t *__restrict__ ptab, const double *__restrict__ cin,
                                              double *hot, uint32_t *tblw) {
  const int nh = hg.P * hg.Kp;
  const int32_t *hp = hpos + (int64_t)x * nh;
  const double *reg = cin + (int64_t)x * hg.Q_pad;
  // ladder 5: only the first phase loads its hot set (the rest keep stale values)
  const bool load = PR_HOT_DIAG != 5 || x < kXcds;
  constexpr int kSB = 6;  // elements per thread in flight (3 batches cover 18429 slots)
  for (int b0 = 0; load && b0 < nh; b0 += kSB * kHotThreads) {
    int32_t pos[kSB];
    double val[kSB];
    if constexpr (CONTIG) {
#pragma unroll
      for (int j = 0; j < kSB; ++j) {
        const int i = b0 + (int)threadIdx.x + j * kHotThreads;
        val[j] = i < hg.q_load ? reg[i] : 0.0;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kSB; ++j) {
        const int i = b0 + (int)threadIdx.x + j * kHotThreads;
        pos[j] = i < nh ? hp[i] : -1;
      }
#pragma unroll
      for (int j = 0; j < kSB; ++j) val[j] = pos[j] >= 0 ? cin[pos[j]] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < kSB; ++j) {
      const int i = b0 + (int)threadIdx.x + j * kHotThreads;
      if (i < nh) hot[1 + i] = val[j];
    }
  }
  if constexpr (PIECE)
    for (int i = (int)threadIdx.x; i < kPieceTblWords; i += kHotThreads)
      tblw[i] = (uint32_t)ptab[(int64_t)x * kPieceTblWords + i];
  if (threadIdx.x == 0) {
    hot[0] = 0.0;
    hot[hg.slots()] = 0.0;
    *reinterpret_cast<uint32_t *>(hot + hg.ctr_slot()) = 0u;  // the workgroup's unit counter
  }
}

// The class units of the split layout, one 1024-thread workgroup per CU (a grid that is a
// multiple of the XCD count).  All of an XCD's workgroups run its classes one after another
// (phases [ph0, ph1): one launch per phase when the exchange overlaps), restaging the hot set
// per class.  CODE: the entry code format (pr_internal.h); compact codes address class x's
// region of the gather space [x*Q_pad, (x+1)*Q_pad) (P = 1 only).
template <int CODE, bool DENSE>
__global__ __launch_bounds__(kHotThreads) void k_spmv_hot(const Unit *__restrict__ units,
                                                          const int64_t *__restrict__ ucum, HotGeom hg,
                                                          CodeSrc cd, const double *__restrict__ cin,
                                                          uint32_t cin_bytes, double *__restrict__ partial,
                                                          const int64_t *__restrict__ poff,
                                                          double *__restrict__ piece_part,
                                                          const int32_t *__restrict__ hpos,
                                                          const int32_t *__restrict__ ptab, int ph0, int ph1) {
  __shared__ double hot[kHotLdsBytes / sizeof(double)];  // static: LDS addresses fold into the instructions
  constexpr bool kPiece = code_is_piece(CODE);
  ClassSrc cs;
  cs.zb = (uint32_t)hg.slots() * 8u;
  cs.hb = kPiece ? cs.zb : (uint32_t)(hg.q_load + 1) * 8u;  // piece codes: cold idx = nh + 1 + k
  uint32_t *tblw = reinterpret_cast<uint32_t *>(hot + hg.tbl_off());
  cs.tbl = tblw;
  if constexpr (CODE == kCodeU32 || kPiece)
    cs.crs = __builtin_amdgcn_make_buffer_rsrc((void *)cin, 0, cin_bytes, 0x00020000);
  const int wv = __builtin_amdgcn_readfirstlane(wave_id());
  double *stage = hot + hg.stage_off() + wv * kStageSlots;  // this wave's staging window
  const int team = (int)(blockIdx.x / kXcds), nteams = (int)(gridDim.x / kXcds);
  for (int ph = ph0; ph < ph1; ++ph) {
    const int x = (int)(blockIdx.x % kXcds) + kXcds * ph;
    if constexpr (CODE == kCodeC20 || CODE == kCodeC24) {  // region index q_load + 1 + k -> x*Q_pad + q_load + k
      const int64_t first = (int64_t)x * hg.Q_pad + hg.q_load;
      cs.crs = __builtin_amdgcn_make_buffer_rsrc((void *)(cin + first), 0,
                                                 (uint32_t)((hg.Q_pad - hg.q_load) * 8), 0x00020000);
    }
    if (ph > ph0) __syncthreads();  // every wave is done with the previous class's hot set
    stage_hot_set<kPiece, CODE == kCodeC20 || CODE == kCodeC24>(hg, x, hpos, ptab, cin, hot, tblw);
    __syncthreads();
    hot_class_units<CODE, DENSE>(x, team, nteams, units, ucum, hg, cd, hot, cs, partial, poff, piece_part, stage);
  }
}

// Long segments: the sum of their pieces in piece order -> partial[seg_slot[q]].
__global__ __launch_bounds__(kThreads) void k_seg_reduce(int64_t n_seg, const int64_t *__restrict__ seg_slot,
                                                         const int32_t *__restrict__ seg_p0,
                                                         const double *__restrict__ piece_part,
                                                         double *__restrict__ partial) {
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * (kThreads / kWave);
  for (int64_t q = (int64_t)blockIdx.x * (kThreads / kWave) + wave_id(); q < n_seg; q += nw) {
    const int32_t p0 = seg_p0[q], np = seg_p0[q + 1] - p0;
    double acc = 0.0;
    for (int k = lane; k < np; k += kWave) acc = __dadd_rn(acc, piece_part[p0 + k]);
    acc = wave_sum(acc);
    if (lane == 0) partial[seg_slot[q]] = acc;
  }
}

// One class of a group in k_epilogue_grp: per block, one ballot of the rows with in-links of
// the class (bit `bit` of their mask word) puts each such row at window slot run + (its rank among
// them), counted straight into the mbcnt accumulator; the other rows read the window's zero slot.
// All G reads are in flight before the first add; returns run past the group's slots.
template <int G>
__device__ __forceinline__ int epi_class_add(const uint32_t (&mw)[G], uint32_t bit, int run, const double *win,
                                             int zslot, double (&S)[G]) {
  double v[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bool has = (mw[g] & bit) != 0u;
    const unsigned long long bal = __ballot(has);
    const int idx = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)bal, (uint32_t)run));
    v[g] = win[has ? idx : zslot];
    run += __popcll(bal);
  }
#pragma unroll
  for (int g = 0; g < G; ++g) S[g] = __dadd_rn(S[g], v[g]);  // absent: + (+0), exact since S >= +0
  return run;
}

// The walk's batches (k_epilogue_grp WALK, k_epi_walk_plan): from class x0, the longest run of
// classes whose staged runs plus their slots' u16 positions (in 16-byte lanes) fit the window.
// Lane y holds class y's run prefix (incl, pre) and slot-count prefix (sincl, spre).  One class
// always fits: at most 64 G + 2 staged slots and 64 G positions (<= 8 G + 2 more slots) <= W.
template <int C, int W>
__device__ __forceinline__ int walk_batch_end(int x0, int incl, int pre, int sincl, int spre) {
  static_assert(W >= 64 * kEpiGroup + 2 + 2 * 8 * kEpiGroup, "one class and its positions fit the window");
  const int lane = lane_id();
  const int base = __builtin_amdgcn_readlane(pre, x0), sbase = __builtin_amdgcn_readlane(spre, x0);
  const int need = (incl - base) + 2 * ((sincl - sbase + 7) >> 3);
  const unsigned long long over = __ballot(lane >= x0 && lane < C && need > W);
  return over ? (int)__builtin_ctzll(over) : C;
}
// bits [x0, x1) of a 64-bit class mask
__device__ __forceinline__ uint64_t class_range_mask(int x0, int x1) {
  const uint64_t hi = x1 >= 64 ? ~0ull : ((1ull << x1) - 1ull);
  return hi & ~((1ull << x0) - 1ull);
}

// Grouped epilogue: a wave takes G = kEpiGroup consecutive 64-row blocks.  For every class their
// slots are ONE contiguous run, [cbase[b0][x], cbase[b0 + G][x]) (class x's segments are
// numbered in row order; cbase carries a sentinel row), so the wave copies whole runs into its
// LDS window by LDS-DMA (`global_load_lds`, 16 bytes per lane, 128 slots per instruction), as
// many classes at a time as the window holds; classes without slots in the group are skipped.
// Lane y holds class y's staged length; one wave scan gives every run's window position and one
// ballot per window load ends the batch.  Then, per class in class order and block, one ballot
// gives the row's position in the staged run and the row adds it from LDS (epi_class_add).  Runs
// start at even slots (16-byte alignment): slot s of a run staged at window offset f sits at
// f + s - (s & ~1).  Each wave's window is W slots plus a zero slot (and one of padding).  At 128
// classes (four mask words) the runs are staged by a per-class loop.
//
// WALK (per-row walk): a group whose class runs and slot positions fit one window load
// (eoff[group] >= 0, k_epi_walk_plan) stages the runs followed by the u16 window positions of
// its slots (epos, row-major: block, row, class).  Each row then adds only its own slots, in
// class order -- as many steps per block as its busiest row has classes, instead of one per class
// -- and the sums are bitwise those of the class loop (whose absent classes add an exact +0).
// (at least 4 waves per SIMD: the LDS of four four-wave workgroups per CU)

// The arguments of the grouped epilogue (k_epilogue_grp); the fused-pack target
// (an array indexed by peer) stays a kernel argument, passed on by reference (a local copy of it
// would be indexed in scratch).
struct EpiArgs {
  int64_t nblk;
  const double *partial;
  const void *rmask;
  const int32_t *cbase;
  const uint32_t *rowinfo;
  double *r, *cout;
  double teleport, damping;
  const int64_t *eoff;
  const uint16_t *epos;
  const uint8_t *pmask;
  const int32_t *sbase;
};

// Cache policy of the epilogue's LDS-DMA of the partial runs (aux bits); A/B builds only.
#ifndef PR_EPI_DMA_AUX
#define PR_EPI_DMA_AUX 0
#endif
#ifndef PR_EPI_LATE_ROW
#define PR_EPI_LATE_ROW 0  // 1: k_epilogue_grp loads rowinfo / r after the class loop (A/B builds)
#endif

// One group gi (kEpiGroup consecutive 64-row blocks) of the grouped epilogue, by one wave with its
// LDS window win (kEpiWin slots + the zero slot win[kEpiWin]).  The group's dangling and L1
// partials go to ep_part[gi] (a fixed-order wave sum), so k_finalize adds the same values in the
// same order whichever wave, workgroup or launch ran the group: every epilogue schedule and grid
// shape is bitwise the same (round 4's overlapped-epilogue schedules relied on it; they were
// measured slower and removed, profiles/r04/README.md).  The body of k_epilogue_grp (below).
template <int C, bool WALK>
__device__ __forceinline__ void epi_group(const EpiArgs &a, const PackDst &pd, int64_t gi, double tdc, double *win,
                                          double2 *__restrict__ ep_part) {
  double dcp = 0.0, l1p = 0.0;
  constexpr int G = kEpiGroup, W = kEpiWin;
  constexpr int MW = mask_words<C>();  // 32-bit mask words per row
  static_assert(MW == 1 || MW == 2 || MW == 4, "mask words");
  static_assert(W >= 64 * G + 2, "one class run of a group must fit the window");
  static_assert(!WALK || C <= kWave, "the per-row walk needs at most 64 classes");
  const int lane = lane_id();
  const int64_t b0 = gi * G;
  const int nb = (int)min((int64_t)G, a.nblk - b0);
  uint32_t mw[MW][G], info[G];
  double rold[G], S[G];
  double cnv[G];    // c' per block, for the fused pack
  uint32_t pmv[G];  // the peers that read the row, per block
#pragma unroll
  for (int g = 0; g < G; ++g) pmv[g] = (pd.P > 1 && g < nb) ? a.pmask[(b0 + g) * kWave + lane] : 0u;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t L = (b0 + g) * kWave + lane;
    const bool ok = g < nb;
    if constexpr (MW == 4) {
      const uint4 q = ok ? static_cast<const uint4 *>(a.rmask)[L] : make_uint4(0u, 0u, 0u, 0u);
      mw[0][g] = q.x, mw[1][g] = q.y, mw[2][g] = q.z, mw[3][g] = q.w;
    } else if constexpr (MW == 2) {
      const uint2 q = ok ? static_cast<const uint2 *>(a.rmask)[L] : make_uint2(0u, 0u);
      mw[0][g] = q.x, mw[1][g] = q.y;
    } else {
      mw[0][g] = ok ? static_cast<const uint32_t *>(a.rmask)[L] : 0u;
    }
#if !PR_EPI_LATE_ROW
    info[g] = ok ? a.rowinfo[L] : kRowHole;
    rold[g] = ok ? a.r[L] : 0.0;
#endif
    S[g] = 0.0;
  }
  // lane x holds class x's run [cs, ce) (and class 64 + x's in cs1/ce1 at C = 128), read back
  // per class with v_readlane
  const int cs = lane < C ? a.cbase[b0 * C + lane] : 0;
  const int ce = lane < C ? a.cbase[(b0 + nb) * C + lane] : 0;
  if constexpr (C <= kWave) {
    // lane y: class y's run start rounded down to 16 bytes (sa), its staged length n2 (0: no
    // slots in this group) and its window position, the exclusive prefix of n2 over the
    // classes.  A batch is the longest sequence of classes from x0 whose staged runs fit the
    // window (one ballot), so the per-class work is a readlane or two and the DMA itself.
    const int sa = cs & ~1;
    const int n2 = (lane < C && ce > cs) ? (((ce + 1) & ~1) - sa) : 0;
    const int incl = wave_incl_scan_i32(n2);
    const int pre = incl - n2;
    const int roff = incl - n2 + (cs - sa);  // window position of the run's first slot
    bool walked = false;
    if constexpr (WALK) {
      const int64_t eo = a.eoff[gi];
      if (eo >= 0) {  // one batch: every class's run and every slot's position fit the window
        const int nsl = lane < C ? ce - cs : 0;  // class y's slots in this group
        const int sincl = wave_incl_scan_i32(nsl);
        for (int y = 0; y < C; ++y) {
          const int n = __builtin_amdgcn_readlane(n2, y);
          if (n == 0) continue;
          const double *src = a.partial + __builtin_amdgcn_readlane(sa, y);
          double *dst = win + __builtin_amdgcn_readlane(pre, y);
          for (int o = 0; o < n; o += 2 * kWave)
            if (o + 2 * lane < n) __builtin_amdgcn_global_load_lds(src + o + 2 * lane, dst + o, 16, 0, PR_EPI_DMA_AUX);
        }
        const int Tb = __builtin_amdgcn_readlane(incl, C - 1);  // staged slots (even)
        const int nl = (__builtin_amdgcn_readlane(sincl, C - 1) + 7) >> 3;  // 16-byte lanes of positions
        const double *esrc = reinterpret_cast<const double *>(a.epos + eo);
        for (int o = 0; o < nl; o += kWave)
          if (o + lane < nl) __builtin_amdgcn_global_load_lds(esrc + 2 * (o + lane), win + Tb + 2 * o, 16, 0, PR_EPI_DMA_AUX);
        __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed
        const uint16_t *ep = reinterpret_cast<const uint16_t *>(win + Tb);
        int acc = 0;  // index of block g's first position
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const uint64_t m = (uint64_t)(MW > 1 ? mw[MW > 1 ? 1 : 0][g] : 0u) << 32 | mw[0][g];
          const int cnt = __popcll(m);
          const int inc = wave_incl_scan_i32(cnt);
          const uint16_t *e = ep + acc + inc - cnt;  // this row's positions, in class order
          acc += __builtin_amdgcn_readlane(inc, kWave - 1);
          for (int k = 0; __ballot(k < cnt) != 0ull; ++k)
            if (k < cnt) S[g] = __dadd_rn(S[g], win[e[k]]);
        }
        __builtin_amdgcn_s_waitcnt(0);  // the window's reads are done before the next group's DMA
        walked = true;
      }
    }
    for (int x0 = 0; x0 < C && !walked;) {
      const int base = __builtin_amdgcn_readlane(pre, x0);
      const unsigned long long over = __ballot(lane >= x0 && lane < C && incl - base > W);
      const int x1 = over ? (int)__builtin_ctzll(over) : C;  // > x0: one run always fits
      for (int y = x0; y < x1; ++y) {
        const int n = __builtin_amdgcn_readlane(n2, y);
        if (n == 0) continue;
        const double *src = a.partial + __builtin_amdgcn_readlane(sa, y);
        double *dst = win + (__builtin_amdgcn_readlane(pre, y) - base);
        for (int o = 0; o < n; o += 2 * kWave)
          if (o + 2 * lane < n) __builtin_amdgcn_global_load_lds(src + o + 2 * lane, dst + o, 16, 0, PR_EPI_DMA_AUX);
      }
      __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed (vmcnt = lgkmcnt = 0)
      for (int y = x0; y < x1; ++y) {
        if (__builtin_amdgcn_readlane(n2, y) == 0) continue;
        const uint32_t bit = 1u << (y & 31);
        const int run = __builtin_amdgcn_readlane(roff, y) - base;
        if (MW == 1 || y < 32) epi_class_add<G>(mw[0], bit, run, win, W, S);
        else epi_class_add<G>(mw[MW > 1 ? 1 : 0], bit, run, win, W, S);
      }
      __builtin_amdgcn_s_waitcnt(0);  // the window's reads are done before the next DMA rewrites it
      x0 = x1;
    }
  } else {  // 128 classes: lanes 64..127's class runs come from a second register
    const int cs1 = lane + kWave < C ? a.cbase[b0 * C + kWave + lane] : 0;
    const int ce1 = lane + kWave < C ? a.cbase[(b0 + nb) * C + kWave + lane] : 0;
    auto run_start = [&](int y) {
      return y < kWave ? __builtin_amdgcn_readlane(cs, y) : __builtin_amdgcn_readlane(cs1, y - kWave);
    };
    auto run_end = [&](int y) {
      return y < kWave ? __builtin_amdgcn_readlane(ce, y) : __builtin_amdgcn_readlane(ce1, y - kWave);
    };
    for (int x = 0; x < C;) {
      // stage the runs of classes [x, xe) that fit the window (at least one always does)
      int fill = 0, xe = x;
      for (; xe < C; ++xe) {
        const int s = run_start(xe), e = run_end(xe);
        if (e == s) continue;  // no slots in this group
        const int sa = s & ~1, n2 = ((e + 1) & ~1) - sa;
        if (xe > x && fill + n2 > W) break;
        const double *src = a.partial + sa;
        for (int o = 0; o < n2; o += 2 * kWave)
          if (o + 2 * lane < n2) __builtin_amdgcn_global_load_lds(src + o + 2 * lane, win + fill + o, 16, 0, PR_EPI_DMA_AUX);
        fill += n2;
      }
      __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed (vmcnt = lgkmcnt = 0)
      fill = 0;
      for (int y = x; y < xe; ++y) {
        const int s = run_start(y), e = run_end(y);
        if (e == s) continue;
        const int sa = s & ~1;
        const uint32_t bit = 1u << (y & 31);
        const int run = fill + (s - sa);
        // static word index (a runtime index into mw would put it in scratch)
        if (y < 32) epi_class_add<G>(mw[0], bit, run, win, W, S);
        else if (y < 64) epi_class_add<G>(mw[MW > 1 ? 1 : 0], bit, run, win, W, S);
        else if (y < 96) epi_class_add<G>(mw[MW > 2 ? 2 : 0], bit, run, win, W, S);
        else epi_class_add<G>(mw[MW > 3 ? 3 : 0], bit, run, win, W, S);
        fill += ((e + 1) & ~1) - sa;
      }
      __builtin_amdgcn_s_waitcnt(0);  // the window's reads are done before the next DMA rewrites it
      x = xe;
    }
  }
#if PR_EPI_LATE_ROW
  // the row data is loaded after the sums (fewer live registers through the class loop)
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t L = (b0 + g) * kWave + lane;
    const bool ok = g < nb;
    info[g] = ok ? a.rowinfo[L] : kRowHole;
    rold[g] = ok ? a.r[L] : 0.0;
  }
#endif
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t L = (b0 + g) * kWave + lane;
    double Sv = S[g];
    uint32_t any = 0u;
#pragma unroll
    for (int w = 0; w < MW; ++w) any |= mw[w][g];
    if (any == 0u) Sv = rold[g];  // no in-link: subtractByKey + union keeps the old rank (Sparky.java:224-225)
    const double rn = affine(Sv, tdc, a.teleport, a.damping);
    double cn = 0.0;
    if (!(info[g] & kRowHole)) {
      a.r[L] = rn;
      const uint32_t d = info[g] & kRowDegMask;
      if (d > 0) {
        cn = __ddiv_rn(rn, (double)d);
        a.cout[L] = cn;
      } else if (info[g] & kRowSink) {
        dcp = __dadd_rn(dcp, rn);
      }
      l1p = __dadd_rn(l1p, fabs(rn - rold[g]));
    }
    cnv[g] = cn;
  }
  // fused pack (P = 2...8): per peer q the group's rows that q reads form ONE run of its send buffer
  // (consecutive from sbase[b0][q]); their c' are gathered in the (now free) LDS window in run order
  // and leave as 16-byte stores through a descriptor ending at the run's end (the range check drops
  // an odd last half) -- a few full-width stores per peer instead of one ballot store per block and
  // peer (s26 P = 8 part: epilogue 109 -> 100 us, profiles/r06/README.md)
  static_assert(G * kWave <= W, "a group's run for one peer fits the window");
  if (pd.P > 1) {
    const int64_t sb0 = b0 * pd.P;
    for (int q = 0; q < pd.P; ++q) {
      int run = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const bool has = (pmv[g] >> q) & 1u;
        const unsigned long long bal = __ballot(has);
        const int k = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, (uint32_t)run));
        if (has) win[k] = cnv[g];
        run += __popcll(bal);
      }
      if (run == 0) continue;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(pd.sbuf + pd.soff[q] + a.sbase[sb0 + q]), 0, (uint32_t)run * 8u, 0x00020000);
      for (int o = 0; o < run; o += 2 * kWave) {
        const int i = o + 2 * lane;
        if (i < run)
          __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const pr_v4i_alias *>(win + i), rs, (uint32_t)i * 8u, 0, 0);
      }
    }
  }
  dcp = wave_sum(dcp);
  l1p = wave_sum(l1p);
  if (lane == 0) ep_part[gi] = make_double2(dcp, l1p);
}

//
// Dispatch positions [g_lo, g_hi) of the pass (all of them in the product).
#ifndef PR_EPI_WAVES
#define PR_EPI_WAVES 0  // > 0: amdgpu_waves_per_eu floor of k_epilogue_grp (A/B builds)
#endif
#if PR_EPI_WAVES > 0
#define PR_EPI_BOUNDS(NT) __attribute__((amdgpu_flat_work_group_size(NT, NT), amdgpu_waves_per_eu(PR_EPI_WAVES)))
#else
#define PR_EPI_BOUNDS(NT) __launch_bounds__(NT, 4)
#endif
template <int C, bool WALK, int NT>
__global__ PR_EPI_BOUNDS(NT) void k_epilogue_grp(
    int64_t nblk, int64_t g_lo, int64_t g_hi, const double *__restrict__ partial, const void *__restrict__ rmask_v,
    const int32_t *__restrict__ cbase, const uint32_t *__restrict__ rowinfo, double *__restrict__ r,
    double *__restrict__ cout, const double *__restrict__ cin, SlotPos sp, double n_vertices, double teleport,
    double damping, double2 *__restrict__ ep_part /* [group] */, const int64_t *__restrict__ eoff,
    const uint16_t *__restrict__ epos, const uint8_t *__restrict__ pmask, const int32_t *__restrict__ sbase,
    const int32_t *__restrict__ order, PackDst pd) {
  constexpr int W = kEpiWin;
  constexpr int NW = NT / kWave;
  extern __shared__ double epi_lds[];  // NW windows of W + 2 slots
  const EpiArgs a{nblk, partial, rmask_v, cbase, rowinfo, r, cout, teleport, damping, eoff, epos, pmask, sbase};
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(wave_id());
  double *win = epi_lds + wv * (W + 2);
  if (lane == 0) win[W] = 0.0;  // the zero slot (never a DMA target: fill <= W)
  const double tdc = dc_from_slots(cin, sp) / n_vertices;
  const int64_t nw = (int64_t)gridDim.x * NW;
  // order: the group of each dispatch position (heaviest first, plan_epi_order); the group's
  // partials go to its own ep_part slot, so the order changes no sum
  for (int64_t k = g_lo + (int64_t)blockIdx.x * NW + wv; k < g_hi; k += nw)
    epi_group<C, WALK>(a, pd, order ? (int64_t)order[k] : k, tdc, win, ep_part);
}

// Build-time plan of the per-row walk (WALK above), one wave per group of G 64-row blocks.
// COUNT: eoff[group] = the group's position entries (padded to 8) if its class runs and the u16
// positions of its slots fit one window load (the sparse tail of R-MAT), else -1.  !COUNT: for
// every group with eoff >= 0, the window position of each slot (the index epi_class_add would
// compute) at epos[eoff + ...], row-major (block, row, class).
template <int C, bool COUNT>
__global__ __launch_bounds__(kEpiThreads) void k_epi_walk_plan(int64_t nblk, const void *__restrict__ rmask_v,
                                                               const int32_t *__restrict__ cbase,
                                                               int64_t *__restrict__ eoff,
                                                               uint16_t *__restrict__ epos) {
  static_assert(C <= kWave, "per-row walk: at most 64 classes");
  constexpr int G = kEpiGroup, W = kEpiWin;
  constexpr int MW = mask_words<C>();
  const int lane = lane_id();
  const int64_t ngrp = (nblk + G - 1) / G;
  const int64_t nw = (int64_t)gridDim.x * (kEpiThreads / kWave);
  for (int64_t gi = (int64_t)blockIdx.x * (kEpiThreads / kWave) + wave_id(); gi < ngrp; gi += nw) {
    int64_t ebase = 0;
    if constexpr (!COUNT) {
      ebase = eoff[gi];
      if (ebase < 0) continue;
    }
    const int64_t b0 = gi * G;
    const int nb = (int)min((int64_t)G, nblk - b0);
    uint64_t m[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t L = (b0 + g) * kWave + lane;
      if (g >= nb) m[g] = 0;
      else if constexpr (MW == 2) m[g] = static_cast<const uint64_t *>(rmask_v)[L];
      else m[g] = static_cast<const uint32_t *>(rmask_v)[L];
    }
    const int cs = lane < C ? cbase[b0 * C + lane] : 0;
    const int ce = lane < C ? cbase[(b0 + nb) * C + lane] : 0;
    const int sa = cs & ~1;
    const int n2 = (lane < C && ce > cs) ? (((ce + 1) & ~1) - sa) : 0;
    const int incl = wave_incl_scan_i32(n2);
    const int pre = incl - n2;
    const int roff = pre + (cs - sa);
    const int nsl = lane < C ? ce - cs : 0;
    const int sincl = wave_incl_scan_i32(nsl);
    const int spre = sincl - nsl;
    const int x1 = walk_batch_end<C, W>(0, incl, pre, sincl, spre);
    const int nl = (__builtin_amdgcn_readlane(sincl, x1 - 1) + 7) >> 3;
    if constexpr (COUNT) {
      if (lane == 0) eoff[gi] = x1 == C ? 8 * (int64_t)nl : -1;
    } else {
      int pref[G], acc = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int cnt = __popcll(m[g]);
        const int inc = wave_incl_scan_i32(cnt);
        pref[g] = acc + inc - cnt;
        acc += __builtin_amdgcn_readlane(inc, kWave - 1);
      }
      for (int x = 0; x < C; ++x) {
        int run = __builtin_amdgcn_readlane(roff, x);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const bool has = (m[g] >> x) & 1ull;
          const unsigned long long bal = __ballot(has);
          if (has) {
            const int k = __popcll(m[g] & ((1ull << x) - 1ull));  // the row's classes before x
            epos[ebase + pref[g] + k] = (uint16_t)__builtin_amdgcn_mbcnt_hi(
                (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, (uint32_t)run));
          }
          run += __popcll(bal);
        }
      }
    }
  }
}

// k_epilogue_grp instantiations: walk (<= 64 classes), one-wave (narrow, <= 64 classes) or
// four-wave workgroups
using EpiGrpFn = void (*)(int64_t, int64_t, int64_t, const double *, const void *, const int32_t *, const uint32_t *, double *,
                          double *, const double *, SlotPos, double, double, double, double2 *, const int64_t *,
                          const uint16_t *, const uint8_t *, const int32_t *, const int32_t *, PackDst);
template <int C>
inline EpiGrpFn epi_grp_kernel_c(bool walk, bool narrow) {
  if constexpr (C <= kWave) {
    if (narrow) return walk ? k_epilogue_grp<C, true, kEpiThreadsNarrow> : k_epilogue_grp<C, false, kEpiThreadsNarrow>;
    if (walk) return k_epilogue_grp<C, true, kEpiThreads>;
  }
  return k_epilogue_grp<C, false, kEpiThreads>;
}
inline EpiGrpFn epi_grp_kernel(int C, bool walk, bool narrow) {
  switch (C) {
    case 8: return epi_grp_kernel_c<8>(walk, narrow);
    case 16: return epi_grp_kernel_c<16>(walk, narrow);
    case 32: return epi_grp_kernel_c<32>(walk, narrow);
    case 64: return epi_grp_kernel_c<64>(walk, narrow);
    default: return epi_grp_kernel_c<128>(false, false);
  }
}

}  // namespace pr
