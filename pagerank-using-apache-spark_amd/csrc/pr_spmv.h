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

// Diagnostics only (tools/diag, DIAG 24): per workgroup of k_spmv_hot the realtime clock at its
// start and after every class phase ([b * 17 + 0] start, [b * 17 + 1 + ph] phase ph done).
extern __device__ unsigned long long pr_diag_clock[];

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
    double2 *__restrict__ unit_part, SlotPos sp, int64_t S_pad, double n_vertices, double teleport,
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
// Split layout (C column classes, pr_graph.h): per-class row sums, then one epilogue pass.
// ============================================================================================
// Heavy (row, class) segments are cut into wave units (pr_internal.h): one wavefront per unit,
// no workgroup barriers.  k_spmv_hot runs one 1024-thread workgroup per CU (its LDS holds the
// class's hot set, so only one fits); workgroup b serves class x = b % 8 -- under the observed
// round-robin dispatch one XCD per class, so that XCD's L2 caches only class-x contributions --
// and its 16 waves walk the class's unit list with a stride of (gridDim/8)*16 units.
//
// Per unit, lane l owns entries [8l, 8l + 8): two 16-byte buffer loads of entry codes (a wave
// reads 2 KiB contiguous; lanes past the unit read 0 through the descriptor's range check) and
// one 4-byte load of the lane's static metadata.  Each entry costs one LDS read (hot codes: the
// most-gathered contributions, top out-degree first; every other lane reads slot 0 = 0.0) and
// one buffer load of the gather space (hot codes turn into offsets >= 2^31: range-checked away,
// no memory request), summed -- one of the two is an exact zero.  No branches, so the waits stay exact.
// The loop is software-pipelined over a ring of three units: the codes of unit i+2 and the
// values of unit i+1 are in flight while unit i is reduced.
//
// STREAM reduction: each lane sums its values along its segment ends; segments that cross lanes
// are completed by a wave64 segmented scan in DPP (row_shr 1/2/4/8, row_bcast 15/31) whose
// per-step "add the partner" predicates are static (a function of where the ends are) and come
// precomputed in the metadata.  Segment s of the unit is row r0 + s, written to partial[x][row]
// through the wave's LDS staging window as coalesced stores.  PIECE: wave sum.  Every sum has a fixed order: results are bitwise reproducible.
typedef int pr_v2i __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const pr_v2i v = __builtin_bit_cast(pr_v2i, x);
  pr_v2i r;
  r.x = __builtin_amdgcn_update_dpp(0, v.x, CTRL, 0xF, 0xF, true);
  r.y = __builtin_amdgcn_update_dpp(0, v.y, CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, r);
}

struct WaveCodes {
  uint32_t c[kWavePT];
  uint32_t meta;  // only with MIK = 0 (precomputed hmeta words)
};

// MIK (meta in kernel, the default): the lane metadata is derived from the segment-end marks
// the codes carry in bit 0 (derive_meta) instead of a precomputed word per lane (hmeta,
// 4 B per lane and unit: 0.53 GB per pass at R-MAT s26).
template <bool MIK>
__device__ __forceinline__ void wave_unit_codes(const Unit &u, const uint32_t *__restrict__ colh,
                                                const uint32_t *__restrict__ hmeta, int64_t k, WaveCodes &w) {
  // per-unit descriptor: base and size are wave-uniform (u lives in SGPRs)
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
  if constexpr (!MIK) {
    const __amdgpu_buffer_rsrc_t ms =
        __builtin_amdgcn_make_buffer_rsrc((void *)(hmeta + k * kWave), 0, u.n > 0 ? kWave * 4 : 0, 0x00020000);
    w.meta = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(ms, lane_id() * 4, 0, 2);
  } else {
    w.meta = 0;
  }
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

// The lane metadata of a STREAM unit (pr_internal.h) from the end marks in bit 0 of its codes:
// which of the lane's entries end a segment, the six "add the partner" predicates of the wave's
// segmented scan (the partner lanes up to this one hold no segment end), and the index of the
// lane's first segment end within the unit (an exclusive scan of the per-lane end counts).
__device__ __forceinline__ uint32_t derive_meta(const WaveCodes &w) {
  uint32_t endm = 0;
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) endm |= (w.c[j] & 1u) << j;
  const int t = lane_id(), r = t & 15, row = t >> 4;
  const uint64_t F = __ballot(endm != 0u);
  const uint64_t upto = (t == 63) ? ~0ull : ((1ull << (t + 1)) - 1);  // lanes [0, t]
  auto clear = [&](int lo) { return (F & upto & ~((1ull << lo) - 1)) == 0ull; };  // no end in [lo, t]
  uint32_t cond = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 1 << s;
    if (r >= k && clear(t - k + 1)) cond |= 1u << s;
  }
  if ((row == 1 || row == 3) && clear(row * 16)) cond |= 1u << 4;
  if (row >= 2 && clear(32)) cond |= 1u << 5;
  // inclusive wave scan of the end counts (row_shr 1/2/4/8, then row_bcast 15/31)
  const int cnt = __builtin_popcount(endm);
  int x = cnt;
  x += dpp_i32<0x111>(x);
  x += dpp_i32<0x112>(x);
  x += dpp_i32<0x114>(x);
  x += dpp_i32<0x118>(x);
  int p = dpp_i32<0x142>(x);
  if (row == 1 || row == 3) x += p;
  p = dpp_i32<0x143>(x);
  if (row >= 2) x += p;
  const uint32_t excl = (uint32_t)(x - cnt);
  return endm | (cond * kMetaStep0) | (excl << kMetaExclShift);
}

// DIAG (diagnostics library only; results wrong when != 0): 1 = every value from LDS (no
// gather-space loads), 2 = no partial stores, 3 = temporal (default-policy) partial stores, 4 / 5 = every
// gather-space load folded into the first 4 / 32 MiB (L2- / Infinity-Cache-resident), 6 =
// exec-masked gathers, 8 = every gather instruction reads 512 contiguous bytes, 13 = every value
// from LDS plus an out-of-range buffer load per entry, 14 = no LDS reads (gathers only), 30 = every
// partial store folded into one 256 KiB window (wave_unit_reduce), 31 = the product (was: 16-byte
// partial stores before they became the product's), 32 / 33 = carry through the staging window,
// 34 = one 8-byte partial store per slot (the product until round 3).
template <int DIAG>
__device__ __forceinline__ void wave_unit_gather(const WaveCodes &w, const double *hot, __amdgpu_buffer_rsrc_t crs,
                                                 double (&v)[kWavePT]) {
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    const uint32_t c = w.c[j] & ~1u;  // bit 0: segment end mark (derive_meta)
    const bool glob = (int32_t)c < 0;
    uint32_t la = glob ? 0u : c;
    if constexpr (DIAG == 1 || DIAG == 13) la = c & 0xFFF8u;
    double a = 0.0;
    if constexpr (DIAG != 14) a = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(hot) + la);
    double b = 0.0;
    uint32_t go = c ^ kEntGlobal;  // LDS codes become offsets >= 2^31: out of range, no request
    if constexpr (DIAG == 13) go = 0xFFFFFFF8u;  // every buffer load out of range (cost of the instruction)
    if constexpr (DIAG == 4) go = glob ? (go & 0x3FFFF8u) : go;   // every gather within 4 MiB
    if constexpr (DIAG == 5) go = glob ? (go & 0x1FFFFF8u) : go;  // every gather within 32 MiB
    if constexpr (DIAG == 8)  // every wave-instruction reads 512 contiguous bytes
      go = glob ? ((__builtin_amdgcn_readfirstlane(go) & 0x3FF000u) + (uint32_t)lane_id() * 8u) : go;
    if constexpr (DIAG == 6) {  // exec-masked instead of range-checked
      if (glob) b = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(crs, go, 0, 0));
    } else if constexpr (DIAG != 1) {
      // DIAG 9..12: cache-policy bits of the gather (nt, sc1, sc0|sc1, sc0)
      constexpr int AUX = DIAG == 9 ? 2 : (DIAG == 10 ? 16 : (DIAG == 11 ? 17 : (DIAG == 12 ? 1 : 0)));
      b = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(crs, go, 0, AUX));
    }
    v[j] = __dadd_rn(a, b);
  }
}

// ORDER 4: the gather-space half of every entry's value (range-checked buffer loads) is issued a
// step ahead and nothing waits for it then; the LDS half is read and added when the unit is
// reduced (wave_unit_add_hot).
__device__ __forceinline__ void wave_unit_gather_glob(const WaveCodes &w, __amdgpu_buffer_rsrc_t crs,
                                                      double (&b)[kWavePT]) {
#pragma unroll
  for (int j = 0; j < kWavePT; ++j)
    b[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(crs, (w.c[j] & ~1u) ^ kEntGlobal, 0, 0));
}
__device__ __forceinline__ void wave_unit_add_hot(const WaveCodes &w, const double *hot, const double (&b)[kWavePT],
                                                  double (&v)[kWavePT]) {
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    const uint32_t c = w.c[j] & ~1u;
    const double a = *reinterpret_cast<const double *>(reinterpret_cast<const char *>(hot) + ((int32_t)c < 0 ? 0u : c));
    v[j] = __dadd_rn(a, b[j]);
  }
}

// The stores of one staged pass: slots [base, base + n) of the unit from the wave's window.
template <int DIAG>
__device__ __forceinline__ void store_staged(const Unit &u, __amdgpu_buffer_rsrc_t prs, const double *stage, int base,
                                             int n) {
  for (int i = lane_id(); i < n; i += kWave) {
    const uint32_t o = (uint32_t)(u.r0 + base + i) * 8u;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(pr_v2i, stage[i]), prs, o, 0, 2);
  }
}

// DEFER (diagnostics, ORDER 3): the last staged pass is not stored here; *dbase / *dn say which
// slots the caller stores later (store_staged) -- after the next unit's gathers are issued.
template <int DIAG, bool MIK, bool DEFER = false>
__device__ __forceinline__ void wave_unit_reduce(const Unit &u, const WaveCodes &w, const double (&v)[kWavePT],
                                                 __amdgpu_buffer_rsrc_t prs, double *__restrict__ piece_part,
                                                 double *stage, int *dbase = nullptr, int *dn = nullptr) {
  if constexpr (DEFER) *dn = 0;
  if (u.meta < 0) {  // PIECE of a long segment
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < kWavePT; ++j) acc = __dadd_rn(acc, v[j]);
    acc = wave_sum(acc);
    if (lane_id() == 0) piece_part[-u.meta - 1] = acc;
    return;
  }
  // DIAG 37: when every lane holds a segment end (short segments), the carry into a lane is the
  // previous lane's tail alone, so the segmented scan and its predicates are skipped (same sums)
  uint32_t meta;
  bool all_ends = false;
  if constexpr (DIAG == 37 && MIK) {
    uint32_t em = 0;
#pragma unroll
    for (int j = 0; j < kWavePT; ++j) em |= (w.c[j] & 1u) << j;
    all_ends = __ballot(em != 0u) == ~0ull;
    meta = all_ends ? (em | ((uint32_t)(wave_incl_scan_i32(__builtin_popcount(em)) - __builtin_popcount(em))
                             << kMetaExclShift))
                    : derive_meta(w);
  } else {
    meta = MIK ? derive_meta(w) : w.meta;
  }
  const uint32_t endm = meta & 0xFFu;
  double sv[kWavePT];
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < kWavePT; ++j) {
    acc = __dadd_rn(acc, v[j]);
    sv[j] = acc;
    if (endm & (1u << j)) acc = 0.0;
  }
  // segmented inclusive scan of the lane tails; partner-add predicates precomputed
  double a = acc, p;
  if (all_ends) goto scanned;
  p = dpp_f64<0x111>(a);  // row_shr:1
  if (meta & kMetaStep0) a = __dadd_rn(p, a);
  p = dpp_f64<0x112>(a);  // row_shr:2
  if (meta & (kMetaStep0 << 1)) a = __dadd_rn(p, a);
  p = dpp_f64<0x114>(a);  // row_shr:4
  if (meta & (kMetaStep0 << 2)) a = __dadd_rn(p, a);
  p = dpp_f64<0x118>(a);  // row_shr:8
  if (meta & (kMetaStep0 << 3)) a = __dadd_rn(p, a);
  p = dpp_f64<0x142>(a);  // row_bcast:15
  if (meta & (kMetaStep0 << 4)) a = __dadd_rn(p, a);
  p = dpp_f64<0x143>(a);  // row_bcast:31
  if (meta & (kMetaStep0 << 5)) a = __dadd_rn(p, a);
scanned:
  const double carry = dpp_f64<0x138>(a);  // wave_shr:1 (lane 0 reads 0)
  // lane's first segment end gets the carry; segment s of the unit is row r0 + s.  The sums are
  // staged in the wave's LDS window (kStageSlots at a time) and leave as coalesced 512-byte
  // stores instead of eight scattered store instructions.
  const int e0 = (int)(meta >> kMetaExclShift), nseg = u.meta;
  if constexpr (DIAG == 23) {
    // every unit issues the same number of store instructions (all kWaveUnit / kStageSlots
    // passes; the unused ones out of range), so the compiler can count them in the vmcnt waits
    // for the next unit's gathers instead of waiting for these stores to complete
#pragma unroll
    for (int pass = 0; pass < kWaveUnit / kStageSlots; ++pass) {
      const int base = pass * kStageSlots;
      int e = e0 - base;
      bool first = true;
#pragma unroll
      for (int j = 0; j < kWavePT; ++j) {
        const bool end = (endm >> j) & 1u;
        if (end && e >= 0 && e < kStageSlots) stage[e] = first ? __dadd_rn(carry, sv[j]) : sv[j];
        if (end) first = false;
        e += end ? 1 : 0;
      }
#pragma unroll
      for (int h = 0; h < kStageSlots / kWave; ++h) {
        const int i = h * kWave + lane_id();
        const bool live = base + i < nseg;
        const uint32_t o = live ? (uint32_t)(u.r0 + base + i) * 8u : 0xFFFFFFF8u;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(pr_v2i, stage[i]), prs, o, 0, 2);
      }
    }
    return;
  }
  // DIAG 32: the carry is added to the lane's first end through the window (one add instead of
  // one per entry); DIAG 33: the same with unconditional window writes (non-ends to a spare slot)
  constexpr int kCap = DIAG == 33 ? kStageSlots - 1 : kStageSlots;
  for (int base = 0; base < nseg; base += kCap) {
    int e = e0 - base;
    if constexpr (DIAG == 32 || DIAG == 33) {
#pragma unroll
      for (int j = 0; j < kWavePT; ++j) {
        const bool end = (endm >> j) & 1u;
        if constexpr (DIAG == 33) {
          stage[(end && e >= 0 && e < kCap) ? e : kCap] = sv[j];
        } else {
          if (end && e >= 0 && e < kCap) stage[e] = sv[j];
        }
        e += end ? 1 : 0;
      }
      const int f = e0 - base;
      if (endm != 0u && f >= 0 && f < kCap) stage[f] = __dadd_rn(carry, stage[f]);
    } else {
    bool first = true;
#pragma unroll
    for (int j = 0; j < kWavePT; ++j) {
      const bool end = (endm >> j) & 1u;
      if (end && e >= 0 && e < kStageSlots) stage[e] = first ? __dadd_rn(carry, sv[j]) : sv[j];
      if (end) first = false;
      e += end ? 1 : 0;
    }
    }
    const int n = min(kCap, nseg - base);
    if constexpr (DEFER) {
      if (base + kCap >= nseg) {  // the last pass: stored by the caller
        *dbase = base;
        *dn = n;
        continue;
      }
    }
    // two slots per lane in one 16-byte non-temporal store (dword alignment is enough), an odd
    // last slot alone: half the store instructions of one 8-byte store per slot (-1.7 % at s26,
    // profiles/r02/store_walk/; DIAG 34 keeps the 8-byte stores for A/B)
    if constexpr (!(DIAG == 2 || DIAG == 3 || DIAG == 30 || DIAG == 34)) {
      static_assert(kStageSlots <= 2 * kWave, "one b128 pass");
      const int i2 = 2 * lane_id();
      const uint32_t o = (uint32_t)(u.r0 + base + i2) * 8u;
      if (i2 + 1 < n) {
        const pr_v4i q = *reinterpret_cast<const pr_v4i *>(stage + i2);
        __builtin_amdgcn_raw_buffer_store_b128(q, prs, o, 0, 2);
      } else if (i2 < n) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(pr_v2i, stage[i2]), prs, o, 0, 2);
      }
      continue;
    }
    for (int i = lane_id(); i < n; i += kWave) {
      uint32_t o = (uint32_t)(u.r0 + base + i) * 8u;
      if constexpr (DIAG == 30) o &= 0x3FFF8u;  // every partial store into one 256 KiB (L2-resident) window
      // non-temporal (nt): the partials are read back by the epilogue only after every class
      // has run, so they should not evict the class region from L2 (5 % of the kernel at s26;
      // DIAG 3 = the temporal stores of round 1, profiles/r02/experiments.md)
      if constexpr (DIAG != 2)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(pr_v2i, stage[i]), prs, o, 0, DIAG == 3 ? 0 : 2);
    }
  }
}

// One class's wave units, strided over `nteams` workgroups (this one is `team`), with the
// class's hot set already in LDS.
template <int ORDER, int DIAG, bool MIK>
__device__ __forceinline__ void hot_class_units(int x, int team, int nteams, const Unit *__restrict__ units,
                                                const int64_t *__restrict__ ucum, const HotGeom &hg,
                                                const uint32_t *__restrict__ colh,
                                                const uint32_t *__restrict__ hmeta, const double *hot,
                                                __amdgpu_buffer_rsrc_t crs, double *__restrict__ partial,
                                                const int64_t *__restrict__ poff, double *__restrict__ piece_part,
                                                double *stage, int wv) {
  const int64_t p0 = poff[x];
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void *)(partial + p0), 0, (uint32_t)((poff[x + 1] - p0) * 8), 0x00020000);
  const int64_t beg = ucum[x];
  int64_t end = ucum[x + 1];
  constexpr int kWaves = kHotThreads / kWave;
  // mode 3: the workgroup's slice of the class rotates with the phase, so a workgroup on a slower
  // CU does not take the same slice of every class (-0.6 % at s26, -1.8 % per part at P = 8)
  if (hg.assign == 3) team = (team + 5 * (x / kXcds)) % nteams;
  int64_t stride = (int64_t)nteams * kWaves;
  int64_t k = beg + (int64_t)team * kWaves + wv;
  if (hg.assign == 1) {  // a contiguous run of units per wave
    const int64_t per = (end - beg + stride - 1) / stride;
    k = beg + ((int64_t)team * kWaves + wv) * per;
    end = k + per < end ? k + per : end;
    stride = 1;
  } else if (hg.assign == 2) {  // a contiguous run per workgroup, its waves interleaved
    const int64_t per = (end - beg + nteams - 1) / nteams;
    const int64_t t0 = beg + (int64_t)team * per;
    end = t0 + per < end ? t0 + per : end;
    k = t0 + wv;
    stride = kWaves;
  }
  // mode 3: the workgroup's units of mode 0 (every stride, kWaves consecutive ones) in the order
  // its waves take them from the LDS counter hot[slots()] (zeroed before the class): a slow wave
  // takes fewer units, so the waves reach the class's end together
  const bool dyn = hg.assign == 3;
  uint32_t *ctr = reinterpret_cast<uint32_t *>(const_cast<double *>(hot) + hg.slots());
  const int lane = lane_id();
  auto take = [&]() -> int64_t {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(ctr, 1u);
    t = (uint32_t)__builtin_amdgcn_readlane((int)t, 0);
    return beg + (int64_t)team * kWaves + (int64_t)(t % kWaves) + (int64_t)(t / kWaves) * stride;
  };
  if (dyn) k = take();
  if (k >= end) return;
  // unit descriptors through the scalar cache; index n_units (= ucum[kMaxClasses]) is an empty unit
  const __attribute__((address_space(4))) pr_v4i *cu = (const __attribute__((address_space(4))) pr_v4i *)units;
  auto unit_at = [&](int64_t i) -> Unit {
    const pr_v4i q = cu[i];
    return Unit{(uint32_t)q.x, q.y, q.z, q.w};
  };
  const int64_t none_k = ucum[kMaxClasses];
  // ring of three units: codes of i+2 and values of i+1 in flight while unit i is reduced
  Unit u[3];
  WaveCodes wc[3];
  double v[3][kWavePT];
  int64_t k1 = dyn ? take() : k + stride;
  u[0] = unit_at(k);
  wave_unit_codes<MIK>(u[0], colh, hmeta, k, wc[0]);
  u[1] = unit_at(k1 < end ? k1 : none_k);
  wave_unit_codes<MIK>(u[1], colh, hmeta, k1, wc[1]);
  if constexpr (ORDER == 4) {
    // the gathers of unit i + 1 stay in flight while unit i is reduced: their values are added
    // (LDS half + buffer half) only when that unit is reduced, one step later
    double vb[3][kWavePT];
    wave_unit_gather_glob(wc[0], crs, vb[0]);
    while (true) {
#pragma unroll
      for (int sl = 0; sl < 3; ++sl) {
        const int s1 = (sl + 1) % 3, s2 = (sl + 2) % 3;
        const int64_t k2 = dyn ? take() : k1 + stride;
        u[s2] = unit_at(k2 < end ? k2 : none_k);
        wave_unit_codes<MIK>(u[s2], colh, hmeta, k2, wc[s2]);
        wave_unit_gather_glob(wc[s1], crs, vb[s1]);
        double vv[kWavePT];
        wave_unit_add_hot(wc[sl], hot, vb[sl], vv);
        wave_unit_reduce<DIAG, MIK>(u[sl], wc[sl], vv, prs, piece_part, stage);
        k = k1;
        k1 = k2;
        if (k >= end) return;
      }
    }
  }
  wave_unit_gather<DIAG>(wc[0], hot, crs, v[0]);
  while (true) {
#pragma unroll
    for (int sl = 0; sl < 3; ++sl) {
      const int s1 = (sl + 1) % 3, s2 = (sl + 2) % 3;
      const int64_t k2 = dyn ? take() : k1 + stride;
      u[s2] = unit_at(k2 < end ? k2 : none_k);
      wave_unit_codes<MIK>(u[s2], colh, hmeta, k2, wc[s2]);
      if constexpr (ORDER == 0) {
        wave_unit_gather<DIAG>(wc[s1], hot, crs, v[s1]);
        wave_unit_reduce<DIAG, MIK>(u[sl], wc[sl], v[sl], prs, piece_part, stage);
      } else if constexpr (ORDER == 3) {  // diagnostics: the last staged stores after the next gathers
        int db = 0, dn = 0;
        wave_unit_reduce<DIAG, MIK, true>(u[sl], wc[sl], v[sl], prs, piece_part, stage, &db, &dn);
        wave_unit_gather<DIAG>(wc[s1], hot, crs, v[s1]);
        store_staged<DIAG>(u[sl], prs, stage, db, dn);
      } else {  // reduce first: a gather issue stalled by a busy address unit cannot hold it up
        wave_unit_reduce<DIAG, MIK>(u[sl], wc[sl], v[sl], prs, piece_part, stage);
        wave_unit_gather<DIAG>(wc[s1], hot, crs, v[s1]);
      }
      k = k1;
      k1 = k2;
      if (k >= end) return;
    }
  }
}

// The class units of the split layout, one 1024-thread workgroup per CU.  Round-robin dispatch
// puts workgroup b on XCD b % 8; XCD k owns classes k, k + 8, ...  PHASED = 0: the XCD's
// workgroups are split between its classes, all running at once.  PHASED = 1: all of the XCD's
// workgroups run its classes one after another, so its L2 holds one class's sources at a time
// (1/C of the gather space instead of 8/C); the hot set is restaged per class.  MIK: lane
// metadata derived in the kernel (default) or read from hmeta (A/B, PR_HOT_META=1).
template <int ORDER = 0, int DIAG = 0, int PHASED = 0, bool MIK = true>
__global__ __launch_bounds__(kHotThreads) void k_spmv_hot(const Unit *__restrict__ units,
                                                          const int64_t *__restrict__ ucum, HotGeom hg,
                                                          const uint32_t *__restrict__ colh,
                                                          const uint32_t *__restrict__ hmeta,
                                                          const double *__restrict__ cin, uint32_t cin_bytes,
                                                          double *__restrict__ partial,
                                                          const int64_t *__restrict__ poff,
                                                          double *__restrict__ piece_part,
                                                          const int32_t *__restrict__ hpos, int ph0, int ph1) {
  extern __shared__ double hot[];
  const int nh = hg.P * hg.Kp;
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc((void *)cin, 0, cin_bytes, 0x00020000);
  const int wv = __builtin_amdgcn_readfirstlane(wave_id());
  double *stage = hot + hg.stage_off() + wv * kStageSlots;  // this wave's staging window
  // PHASED: phases [ph0, ph1) of this launch (one launch per phase when the exchange overlaps)
  const int p_lo = PHASED ? ph0 : 0, p_hi = PHASED ? ph1 : 1;
  if constexpr (DIAG == 24)
    if (threadIdx.x == 0) pr_diag_clock[blockIdx.x * 17] = wall_clock64();
  for (int ph = p_lo; ph < p_hi; ++ph) {
    int x, team, nteams;
    if constexpr (PHASED) {
      x = (int)(blockIdx.x % kXcds) + kXcds * ph;
      team = (int)(blockIdx.x / kXcds);
      nteams = (int)(gridDim.x / kXcds);
      if (ph > p_lo) __syncthreads();  // every wave is done with the previous class's hot set
    } else {
      x = (int)(blockIdx.x % kXcds) + kXcds * (int)((blockIdx.x / kXcds) % (hg.C / kXcds));
      team = (int)(blockIdx.x / hg.C);
      nteams = (int)(gridDim.x / hg.C);
    }
    // stage the class's hot contributions (the previous iteration's, final before this launch):
    // every position load, then every gather in flight before the first LDS write -- a rolled
    // loop pays two dependent memory latencies per element, 18 times per phase
    const int32_t *hp = hpos + (int64_t)x * nh;
    constexpr int kSB = 6;  // elements per thread in flight (3 batches cover 18430 slots)
    // DIAG 35 (timing only, wrong values): the hot set is staged for the first phase only.
    // DIAG 36: at P = 1 the class's hot set is rows [x Q_pad, + q_load) of the slice, contiguous:
    // staged by 4-byte LDS-DMA instead of position loads and gathers through registers.
    bool staged = DIAG == 35 && ph > p_lo;
    if constexpr (DIAG == 36) {
      if (hg.P == 1) {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(cin + (int64_t)x * hg.Q_pad);
        uint32_t *dst = reinterpret_cast<uint32_t *>(hot + 1);
        const int nd = 2 * hg.q_load, ln = lane_id();
        for (int b = wv * kWave; b < nd; b += kHotThreads)
          if (b + ln < nd) __builtin_amdgcn_global_load_lds(src + b + ln, dst + b, 4, 0, 0);
        __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed before the barrier
        staged = true;
      }
    }
    for (int b0 = 0; b0 < nh && !staged; b0 += kSB * kHotThreads) {
      int32_t pos[kSB];
      double val[kSB];
#pragma unroll
      for (int j = 0; j < kSB; ++j) {
        const int i = b0 + (int)threadIdx.x + j * kHotThreads;
        pos[j] = i < nh ? hp[i] : -1;
      }
#pragma unroll
      for (int j = 0; j < kSB; ++j) val[j] = pos[j] >= 0 ? cin[pos[j]] : 0.0;
#pragma unroll
      for (int j = 0; j < kSB; ++j) {
        const int i = b0 + (int)threadIdx.x + j * kHotThreads;
        if (i < nh) hot[1 + i] = val[j];
      }
    }
    if (threadIdx.x == 0) {
      hot[0] = 0.0;
      *reinterpret_cast<uint32_t *>(hot + hg.slots()) = 0u;  // unit counter (PR_HOT_ASSIGN=3)
    }
    __syncthreads();
    hot_class_units<ORDER, DIAG, MIK>(x, team, nteams, units, ucum, hg, colh, hmeta, hot, crs, partial, poff,
                                 piece_part, stage, wv);
    if constexpr (DIAG == 24) {  // phase done by every wave of this workgroup
      __syncthreads();
      if (threadIdx.x == 0) pr_diag_clock[blockIdx.x * 17 + 1 + ph] = wall_clock64();
    }
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

// Epilogue of the split layout, one wave per 64 consecutive rows: S = the row's class partial
// sums in class order (row L's class-x slot = cbase[blk][x] + rows of the block before L that
// have class-x in-links: one ballot), the in-degree-0 quirk, then the fused update of
// k_spmv_units (r' without FMA, c' = r'/d, dangling and L1 partials).
// ABS: cbase holds absolute slot indices (all classes' partials < 2^29 slots): one buffer
// resource over the whole partial array instead of one per class (which spills SGPRs).
template <int C, bool ABS = false>
__global__ __launch_bounds__(kThreads) void k_epilogue(int64_t nblk, PartOff po, const double *__restrict__ partial,
                                                       const uint32_t *__restrict__ rmask,
                                                       const int32_t *__restrict__ cbase,
                                                       const uint32_t *__restrict__ rowinfo,
                                                       double *__restrict__ r, double *__restrict__ cout,
                                                       const double *__restrict__ cin, SlotPos sp,
                                                       double n_vertices, double teleport, double damping,
                                                       double2 *__restrict__ ep_part) {
  typedef int cb_t __attribute__((ext_vector_type(C)));
  __shared__ double2 red2[kThreads / kWave];
  const double tdc = dc_from_slots(cin, sp) / n_vertices;
  const int lane = lane_id();
  double dcp = 0.0, l1p = 0.0;
  const int64_t nw = (int64_t)gridDim.x * (kThreads / kWave);
  const int wv = __builtin_amdgcn_readfirstlane(wave_id());
  for (int64_t blk = (int64_t)blockIdx.x * (kThreads / kWave) + wv; blk < nblk; blk += nw) {
    const int64_t L = blk * kWave + lane;  // rows come in whole blocks (holes flagged)
    const uint32_t m = rmask[L];
    const uint32_t info = rowinfo[L];
    const double rold = r[L];
    // the block's C first-slot indices in one scalar load (cbase is [blk][C])
    const cb_t cb = *(const __attribute__((address_space(4))) cb_t *)(cbase + blk * C);
    // every class's partial load in flight before the first add (absent: out of range, no request)
    double v[C];
#pragma unroll
    for (int x = 0; x < C; ++x) {
      const bool has = (m >> x) & 1u;
      const unsigned long long bal = __ballot(has);
      const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      const uint32_t off = has ? ((uint32_t)cb[x] + (uint32_t)pre) * 8u : 0xFFFFFFF8u;
      if constexpr (ABS) {
        const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)partial, 0, (uint32_t)(po.o[C] * 8), 0x00020000);
        v[x] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(prs, off, 0, 2));
      } else {
        const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(partial + po.o[x]), 0, (uint32_t)((po.o[x + 1] - po.o[x]) * 8), 0x00020000);
        v[x] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(prs, off, 0, 2));
      }
    }
    double S = 0.0;
#pragma unroll
    for (int x = 0; x < C; ++x) S = __dadd_rn(S, v[x]);  // absent classes add an exact 0
    if (m == 0) S = rold;  // no in-link: subtractByKey + union keeps the old rank (Sparky.java:224-225)
    const double rn = affine(S, tdc, teleport, damping);
    if (!(info & kRowHole)) {
      r[L] = rn;
      const uint32_t d = info & kRowDegMask;
      if (d > 0) cout[L] = __ddiv_rn(rn, (double)d);
      else if (info & kRowSink) dcp = __dadd_rn(dcp, rn);
      l1p = __dadd_rn(l1p, fabs(rn - rold));
    }
  }
  const double2 part = block_sum2<kThreads>(make_double2(dcp, l1p), red2);
  if (threadIdx.x == 0) ep_part[blockIdx.x] = part;
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

// Grouped epilogue (row sums bitwise those of k_epilogue): the address unit charges per load
// instruction, and k_epilogue spends C + 3 of them per 64-row block although a block's class-x
// slots are only ~12 consecutive partials.  Here a wave takes G = kEpiGroup consecutive blocks.
// For every class their slots are ONE contiguous run, [cbase[b0][x], cbase[b0 + G][x]) (class x's
// segments are numbered in row order; cbase carries a sentinel row), so the wave copies whole
// runs into its LDS window by LDS-DMA, 16 bytes per lane (128 slots per instruction: ~4 per
// block instead of 35 at C = 32), as many classes at a time as the window holds; classes without
// slots in the group are skipped.  Then, per class in class order and block, one ballot gives the
// row's position in the staged run and the row adds it from LDS (epi_class_add).  Runs start at
// even slots (16-byte alignment): slot s of a run staged at window offset f sits at
// f + s - (s & ~1).  Each wave's window is W slots plus a zero slot (and one of padding).
//
// WALK (per-row walk, PR_EPI_WALK): for a group the build chose (eoff[group] >= 0: where the
// walk is the cheaper of the two), each batch of classes holds the staged runs followed in the
// window by the u16 window positions of the batch's slots (epos, row-major: block, row, class),
// batched so that both fit (walk_batch_end).  Each row then adds only its own slots, in class
// order -- as many steps per batch and block as its busiest row has classes there, instead of
// one per class -- and the sums are bitwise those of the class loop (whose absent classes add an
// exact +0).  k_epi_walk_plan plans the positions with the same staging and batching rules.
// (at least 4 waves per SIMD: the LDS of four four-wave workgroups per CU; the register budget
// keeps the walk there.  PR_EPI_MINWAVES: A/B builds only)
#ifndef PR_EPI_MINWAVES
#define PR_EPI_MINWAVES 4
#endif
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

// EDIAG (diagnostics library only; results wrong when != 0): 1 = no partial-run DMA (the window
// is read as it is), 2 = DMA but no per-class adds, 3 = neither (row data, masks, writes only).
template <int C, int G = kEpiGroup, int W = kEpiWin, bool LEGACY = false, bool WALK = false, int EDIAG = 0,
          int NT = kEpiThreads>
__global__ __launch_bounds__(NT, PR_EPI_MINWAVES) void k_epilogue_grp(
    int64_t nblk, const double *__restrict__ partial, const void *__restrict__ rmask_v,
    const int32_t *__restrict__ cbase, const uint32_t *__restrict__ rowinfo, double *__restrict__ r,
    double *__restrict__ cout, const double *__restrict__ cin, SlotPos sp, double n_vertices, double teleport,
    double damping, double2 *__restrict__ ep_part, const int64_t *__restrict__ eoff,
    const uint16_t *__restrict__ epos) {
  constexpr int NW = NT / kWave;
  constexpr int MW = mask_words<C>();  // 32-bit mask words per row
  static_assert(MW == 1 || MW == 2 || MW == 4, "mask words");
  static_assert(W >= 64 * G + 2, "one class run of a group must fit the window");
  extern __shared__ double epi_lds[];  // NW windows of W + 2 slots, then NW double2 for the block sum
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(wave_id());
  double *win = epi_lds + wv * (W + 2);
  if (lane == 0) win[W] = 0.0;  // the zero slot (never a DMA target: fill <= W)
  const double tdc = dc_from_slots(cin, sp) / n_vertices;
  double dcp = 0.0, l1p = 0.0;
  const int64_t ngrp = (nblk + G - 1) / G;
  const int64_t nw = (int64_t)gridDim.x * NW;
  for (int64_t gi = (int64_t)blockIdx.x * NW + wv; gi < ngrp; gi += nw) {
    const int64_t b0 = gi * G;
    const int nb = (int)min((int64_t)G, nblk - b0);
    uint32_t mw[MW][G], info[G];
    double rold[G], S[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t L = (b0 + g) * kWave + lane;
      const bool ok = g < nb;
      if constexpr (MW == 4) {
        const uint4 q = ok ? static_cast<const uint4 *>(rmask_v)[L] : make_uint4(0u, 0u, 0u, 0u);
        mw[0][g] = q.x, mw[1][g] = q.y, mw[2][g] = q.z, mw[3][g] = q.w;
      } else if constexpr (MW == 2) {
        const uint2 q = ok ? static_cast<const uint2 *>(rmask_v)[L] : make_uint2(0u, 0u);
        mw[0][g] = q.x, mw[1][g] = q.y;
      } else {
        mw[0][g] = ok ? static_cast<const uint32_t *>(rmask_v)[L] : 0u;
      }
      info[g] = ok ? rowinfo[L] : kRowHole;
      rold[g] = ok ? r[L] : 0.0;
      S[g] = 0.0;
    }
    // lane x holds class x's run [cs, ce) (and class 64 + x's in cs1/ce1 at C = 128), read back
    // per class with v_readlane
    const int cs = lane < C ? cbase[b0 * C + lane] : 0;
    const int ce = lane < C ? cbase[(b0 + nb) * C + lane] : 0;
    const int cs1 = (C > kWave && lane + kWave < C) ? cbase[b0 * C + kWave + lane] : 0;
    const int ce1 = (C > kWave && lane + kWave < C) ? cbase[(b0 + nb) * C + kWave + lane] : 0;
    auto run_start = [&](int y) {
      return (C <= kWave || y < kWave) ? __builtin_amdgcn_readlane(cs, y) : __builtin_amdgcn_readlane(cs1, y - kWave);
    };
    auto run_end = [&](int y) {
      return (C <= kWave || y < kWave) ? __builtin_amdgcn_readlane(ce, y) : __builtin_amdgcn_readlane(ce1, y - kWave);
    };
    if constexpr (C <= kWave && !LEGACY) {
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
        const int64_t eo = eoff[gi];
        if (eo >= 0) {
          const int nsl = lane < C ? ce - cs : 0;  // class y's slots in this group
          const int sincl = wave_incl_scan_i32(nsl);
          const int spre = sincl - nsl;
          int64_t ebase = eo;  // the batch's first position entry (16-byte aligned)
          for (int x0 = 0; x0 < C;) {
            const int x1 = walk_batch_end<C, W>(x0, incl, pre, sincl, spre);
            const int base = __builtin_amdgcn_readlane(pre, x0);
            const int sbase = __builtin_amdgcn_readlane(spre, x0);
            for (int y = x0; y < x1; ++y) {
              const int n = __builtin_amdgcn_readlane(n2, y);
              if (n == 0) continue;
              const double *src = partial + __builtin_amdgcn_readlane(sa, y);
              double *dst = win + (__builtin_amdgcn_readlane(pre, y) - base);
              for (int o = 0; o < n; o += 2 * kWave)
                if (o + 2 * lane < n) __builtin_amdgcn_global_load_lds(src + o + 2 * lane, dst + o, 16, 0, 0);
            }
            const int Tb = __builtin_amdgcn_readlane(incl, x1 - 1) - base;  // staged slots (even)
            const int nl = (__builtin_amdgcn_readlane(sincl, x1 - 1) - sbase + 7) >> 3;  // 16-byte lanes
            const double *esrc = reinterpret_cast<const double *>(epos + ebase);
            for (int o = 0; o < nl; o += kWave)
              if (o + lane < nl) __builtin_amdgcn_global_load_lds(esrc + 2 * (o + lane), win + Tb + 2 * o, 16, 0, 0);
            ebase += 8 * nl;
            __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed
            const uint16_t *ep = reinterpret_cast<const uint16_t *>(win + Tb);
            const uint64_t bm = class_range_mask(x0, x1);
            int acc = 0;  // index of block g's first position in the batch
#pragma unroll
            for (int g = 0; g < G; ++g) {
              const uint64_t m = ((uint64_t)(MW > 1 ? mw[MW > 1 ? 1 : 0][g] : 0u) << 32 | mw[0][g]) & bm;
              const int cnt = __popcll(m);
              const int inc = wave_incl_scan_i32(cnt);
              const uint16_t *e = ep + acc + inc - cnt;  // this row's positions, in class order
              acc += __builtin_amdgcn_readlane(inc, kWave - 1);
              for (int k = 0; __ballot(k < cnt) != 0ull; ++k)
                if (k < cnt) S[g] = __dadd_rn(S[g], win[e[k]]);
            }
            __builtin_amdgcn_s_waitcnt(0);  // the window's reads are done before the next DMA rewrites it
            x0 = x1;
          }
          walked = true;
        }
      }
      for (int x0 = 0; x0 < C && !walked;) {
        const int base = __builtin_amdgcn_readlane(pre, x0);
        const unsigned long long over = __ballot(lane >= x0 && lane < C && incl - base > W);
        const int x1 = over ? (int)__builtin_ctzll(over) : C;  // > x0: one run always fits
        for (int y = x0; y < x1 && EDIAG != 1 && EDIAG != 3; ++y) {
          const int n = __builtin_amdgcn_readlane(n2, y);
          if (n == 0) continue;
          const double *src = partial + __builtin_amdgcn_readlane(sa, y);
          double *dst = win + (__builtin_amdgcn_readlane(pre, y) - base);
          for (int o = 0; o < n; o += 2 * kWave)
            if (o + 2 * lane < n) __builtin_amdgcn_global_load_lds(src + o + 2 * lane, dst + o, 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA has landed (vmcnt = lgkmcnt = 0)
        for (int y = x0; y < x1 && EDIAG < 2; ++y) {
          if (__builtin_amdgcn_readlane(n2, y) == 0) continue;
          const uint32_t bit = 1u << (y & 31);
          const int run = __builtin_amdgcn_readlane(roff, y) - base;
          if (MW == 1 || y < 32) epi_class_add<G>(mw[0], bit, run, win, W, S);
          else epi_class_add<G>(mw[MW > 1 ? 1 : 0], bit, run, win, W, S);
        }
        __builtin_amdgcn_s_waitcnt(0);  // the window's reads are done before the next DMA rewrites it
        x0 = x1;
      }
    } else {
    for (int x = 0; x < C;) {
      // stage the runs of classes [x, xe) that fit the window (at least one always does)
      int fill = 0, xe = x;
      for (; xe < C; ++xe) {
        const int s = run_start(xe), e = run_end(xe);
        if (e == s) continue;  // no slots in this group
        const int sa = s & ~1, n2 = ((e + 1) & ~1) - sa;
        if (xe > x && fill + n2 > W) break;
        const double *src = partial + sa;
        for (int o = 0; o < n2; o += 2 * kWave)
          if (o + 2 * lane < n2) __builtin_amdgcn_global_load_lds(src + o + 2 * lane, win + fill + o, 16, 0, 0);
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
        if (MW == 1 || y < 32) epi_class_add<G>(mw[0], bit, run, win, W, S);
        else if (MW == 2 || y < 64) epi_class_add<G>(mw[MW > 1 ? 1 : 0], bit, run, win, W, S);
        else if (y < 96) epi_class_add<G>(mw[MW > 2 ? 2 : 0], bit, run, win, W, S);
        else epi_class_add<G>(mw[MW > 3 ? 3 : 0], bit, run, win, W, S);
        fill += ((e + 1) & ~1) - sa;
      }
      __builtin_amdgcn_s_waitcnt(0);  // the window's reads are done before the next DMA rewrites it
      x = xe;
    }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t L = (b0 + g) * kWave + lane;
      double Sv = S[g];
      uint32_t any = 0u;
#pragma unroll
      for (int w = 0; w < MW; ++w) any |= mw[w][g];
      if (any == 0u) Sv = rold[g];  // no in-link: subtractByKey + union keeps the old rank (Sparky.java:224-225)
      const double rn = affine(Sv, tdc, teleport, damping);
      if (!(info[g] & kRowHole)) {
        r[L] = rn;
        const uint32_t d = info[g] & kRowDegMask;
        if (d > 0) cout[L] = __ddiv_rn(rn, (double)d);
        else if (info[g] & kRowSink) dcp = __dadd_rn(dcp, rn);
        l1p = __dadd_rn(l1p, fabs(rn - rold[g]));
      }
    }
  }
  double2 *red2 = reinterpret_cast<double2 *>(epi_lds + NW * (W + 2));
  const double2 part = block_sum2<NT>(make_double2(dcp, l1p), red2);
  if (threadIdx.x == 0) ep_part[blockIdx.x] = part;
}

// Build-time plan of the per-row walk (WALK above), one wave per group of G 64-row blocks, with
// k_epilogue_grp's staging and the walk's batching.  COUNT: eoff[group] = the group's position
// entries (16-byte padded per batch) if it walks, else -1.  Rule (PR_EPI_WALK): 1 (default) = the
// group fits one batch (runs and positions in one window load: the sparse tail of R-MAT); 2 = any
// group whose walk takes at most 3/4 of the class loop's steps (per batch and block the busiest
// row's classes, against one per class with slots) -- slower in practice (R-MAT s26 +3 %, ER s24
// +18 %: a walk step costs more than a loop step, and the positions add 2 B per slot).  !COUNT:
// for every group with eoff >= 0, the window position of each slot (the index epi_class_add would
// compute) at epos[eoff + ...].
template <int C, int G, int W, bool COUNT>
__global__ __launch_bounds__(kEpiThreads) void k_epi_walk_plan(int64_t nblk, const void *__restrict__ rmask_v,
                                                               const int32_t *__restrict__ cbase,
                                                               int64_t *__restrict__ eoff,
                                                               uint16_t *__restrict__ epos, int rule) {
  static_assert(C <= kWave, "per-row walk: at most 64 classes");
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
    int64_t loop_steps = 0, walk_steps = 0, total = 0;
    int batches = 0;
    for (int x0 = 0; x0 < C;) {
      const int x1 = walk_batch_end<C, W>(x0, incl, pre, sincl, spre);
      const int base = __builtin_amdgcn_readlane(pre, x0), sbase = __builtin_amdgcn_readlane(spre, x0);
      const int nl = (__builtin_amdgcn_readlane(sincl, x1 - 1) - sbase + 7) >> 3;
      const uint64_t bm = class_range_mask(x0, x1);
      if constexpr (COUNT) {
        loop_steps += (int64_t)G * __popcll(__ballot(lane >= x0 && lane < x1 && n2 > 0));
#pragma unroll
        for (int g = 0; g < G; ++g) {
          int c = __popcll(m[g] & bm);
          for (int off = kWave / 2; off > 0; off >>= 1) c = max(c, __shfl_xor(c, off, kWave));
          walk_steps += c;
        }
        total += 8 * nl;
        ++batches;
      } else {
        int pref[G], acc = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int cnt = __popcll(m[g] & bm);
          const int inc = wave_incl_scan_i32(cnt);
          pref[g] = acc + inc - cnt;
          acc += __builtin_amdgcn_readlane(inc, kWave - 1);
        }
        for (int x = x0; x < x1; ++x) {
          int run = __builtin_amdgcn_readlane(roff, x) - base;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const bool has = (m[g] >> x) & 1ull;
            const unsigned long long bal = __ballot(has);
            if (has) {
              const int k = __popcll(m[g] & bm & ((1ull << x) - 1ull));  // the row's classes before x in the batch
              epos[ebase + pref[g] + k] = (uint16_t)__builtin_amdgcn_mbcnt_hi(
                  (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, (uint32_t)run));
            }
            run += __popcll(bal);
          }
        }
        ebase += 8 * nl;
      }
      x0 = x1;
    }
    if constexpr (COUNT)
      if (lane == 0) {
        const bool walk = rule == 1 ? batches == 1 : walk_steps * 4 <= loop_steps * 3;
        eoff[gi] = walk ? total : -1;
      }
  }
}

// k_epilogue_grp instantiations by variant (pr_internal.h kEpiVariants); walk: the per-row walk
// of sparse groups (variants 0 and 7, at most 64 classes)
using EpiGrpFn = void (*)(int64_t, const double *, const void *, const int32_t *, const uint32_t *, double *,
                          double *, const double *, SlotPos, double, double, double, double2 *, const int64_t *,
                          const uint16_t *);
inline bool epi_walk_variant(int C, int var) { return C <= kWave && (var == 0 || var == 7); }
template <int C>
inline EpiGrpFn epi_grp_kernel_c(int var, bool walk, bool narrow) {
  if (narrow && var == 0) {  // one-wave workgroups (variant 0 only)
    if constexpr (C <= kWave)
      if (walk) return k_epilogue_grp<C, kEpiGroup, kEpiWin, false, true, 0, kEpiThreadsNarrow>;
    return k_epilogue_grp<C, kEpiGroup, kEpiWin, false, false, 0, kEpiThreadsNarrow>;
  }
  if constexpr (C <= kWave) {
    if (walk && var == 7) return k_epilogue_grp<C, kEpiVariants[7].G, kEpiVariants[7].W, false, true>;
    if (walk && var == 0) return k_epilogue_grp<C, kEpiVariants[0].G, kEpiVariants[0].W, false, true>;
  }
  switch (var) {
    case 7: return k_epilogue_grp<C, kEpiVariants[7].G, kEpiVariants[7].W>;
    case 1: return k_epilogue_grp<C, kEpiVariants[1].G, kEpiVariants[1].W>;
    case 2: return k_epilogue_grp<C, kEpiVariants[2].G, kEpiVariants[2].W>;
    case 3: return k_epilogue_grp<C, kEpiVariants[3].G, kEpiVariants[3].W>;
    case 4: return k_epilogue_grp<C, kEpiVariants[4].G, kEpiVariants[4].W>;
    case 5: return k_epilogue_grp<C, kEpiVariants[5].G, kEpiVariants[5].W>;
    case 6: return k_epilogue_grp<C, kEpiVariants[6].G, kEpiVariants[6].W, kEpiVariants[6].legacy>;
    default: return k_epilogue_grp<C, kEpiVariants[0].G, kEpiVariants[0].W>;
  }
}
inline EpiGrpFn epi_grp_kernel(int C, int var, bool walk = false, bool narrow = false) {
  if (C == 128) return epi_grp_kernel_c<128>(var, false, false);
  return C == 64 ? epi_grp_kernel_c<64>(var, walk, narrow)
                 : (C == 32 ? epi_grp_kernel_c<32>(var, walk, narrow)
                            : (C == 16 ? epi_grp_kernel_c<16>(var, walk, narrow) : epi_grp_kernel_c<8>(var, walk, narrow)));
}
inline size_t epi_grp_lds(int var, bool narrow = false) {
  return sizeof(double) * (size_t)(epi_grp_threads(var, narrow) / kWave) * (kEpiVariants[var].W + 4);
}

}  // namespace pr
