// The PageRank power iteration on gfx950 (K3/K4 in SURVEY.md §2.1): the hot path.
//
// One iteration of Sparky.java:189-235 on one part (pr_graph.h layouts):
//
//   split layout (C > 1 column classes; every graph whose gather space passes 4 MiB):
//     k_spmv_hot     per class, the wave units of consecutive (row, class) segments: codes
//                    address the class's LDS hot set or the gather space; per-lane sums and a
//                    wave64 DPP segmented scan give one partial sum per segment
//                    (join + flatMapToPair + the map side of reduceByKey, Sparky.java:192-216, :229)
//     k_seg_reduce   long segments: their pieces summed in piece order
//     k_epilogue_grp per row, its segment sums in class order (reduceByKey(Sum), :27-32, :229),
//                    then the update fused:
//                      in-degree-0 quirk: S = r_old             (subtractByKey + union, :224-225)
//                      r' = 0.15 + 0.85 * (S + dc / N)          (:233, no FMA contraction)
//                      c' = r' / d for the next iteration       (:207, a true division)
//                      block partials of sum r' over sink rows  (danglingContrib, :219-222)
//                      block partials of |r' - r|               (L1 convergence norm; reported only)
//   fused layout (C = 1, small graphs): k_spmv_units does all of that in one launch per unit.
//   k_finalize       long rows of the fused layout, then a deterministic reduction of all block
//                    partials into the part's two slots {dc partial, L1 partial} at the end of
//                    its gather slice (last-arriving workgroup, agent-scope protocol of
//                    cdna_hip_programming.md Guideline 16).
//   P > 1: the exchange (pr_exchange.hip) sends every peer the contributions its in-links read.
//
// Every sum has a fixed order, so results are bitwise reproducible run to run.
#include <algorithm>
#include <climits>
#include <vector>

#include "pr_device.h"
#include "pr_graph.h"
#include "pr_ipc_protocol.h"
#include "pr_spmv.h"

namespace pr {
namespace {

__device__ __forceinline__ void store_sc1(double *p, double x) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), (unsigned long long)__double_as_longlong(x),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double *p) {
  return __longlong_as_double((long long)__hip_atomic_load(
      reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__global__ __launch_bounds__(kThreads) void k_finalize(
    int64_t n_long, const int32_t *__restrict__ lr_row, const int32_t *__restrict__ lr_p0,
    const double *__restrict__ piece_part, const double2 *__restrict__ parts, int64_t n_parts,
    double *__restrict__ r, const uint32_t *__restrict__ rowinfo, const double *__restrict__ cin,
    double *__restrict__ cout, SlotPos sp, double n_vertices, double teleport,
    double damping, double *__restrict__ fin_part, unsigned *__restrict__ counter,
    double *__restrict__ slot_out, PackSlots ps) {
  __shared__ double red[kThreads / kWave];
  __shared__ int is_last;
  const int t = threadIdx.x, lane = lane_id();
  double dcp = 0.0, l1p = 0.0;
  if (n_long > 0) {
    const double tdc = dc_from_slots(cin, sp) / n_vertices;
    const int64_t nw = (int64_t)gridDim.x * (kThreads / kWave);
    for (int64_t q = (int64_t)blockIdx.x * (kThreads / kWave) + wave_id(); q < n_long; q += nw) {
      const int32_t p0 = lr_p0[q], np = lr_p0[q + 1] - p0;
      double acc = 0.0;
      for (int k = lane; k < np; k += kWave) acc = __dadd_rn(acc, piece_part[p0 + k]);
      acc = wave_sum(acc);
      if (lane == 0) {
        const int32_t v = lr_row[q];
        const double rold = r[v];
        const double rn = affine(acc, tdc, teleport, damping);
        r[v] = rn;
        const uint32_t info = rowinfo[v];
        const uint32_t d = info & kRowDegMask;
        if (d > 0) cout[v] = __ddiv_rn(rn, (double)d);
        else if (info & kRowSink) dcp = __dadd_rn(dcp, rn);
        l1p = __dadd_rn(l1p, fabs(rn - rold));
      }
    }
  }
  for (int64_t i = (int64_t)blockIdx.x * kThreads + t; i < n_parts; i += (int64_t)gridDim.x * kThreads) {
    const double2 pv = parts[i];
    dcp = __dadd_rn(dcp, pv.x);
    l1p = __dadd_rn(l1p, pv.y);
  }
  dcp = block_sum<kThreads>(dcp, red);
  l1p = block_sum<kThreads>(l1p, red);
  if (t == 0) {
    store_sc1(&fin_part[2 * blockIdx.x], dcp);
    store_sc1(&fin_part[2 * blockIdx.x + 1], l1p);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (prev == gridDim.x - 1) ? 1 : 0;
  }
  __syncthreads();
  if (!is_last) return;
  double a = 0.0, b = 0.0;
  for (int i = t; i < (int)gridDim.x; i += kThreads) {
    a = __dadd_rn(a, load_sc1(&fin_part[2 * i]));
    b = __dadd_rn(b, load_sc1(&fin_part[2 * i + 1]));
  }
  a = block_sum<kThreads>(a, red);
  b = block_sum<kThreads>(b, red);
  if (t == 0) {
    slot_out[0] = a;
    slot_out[1] = b;
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (t < ps.n) {  // fused pack: the two slots close every peer's send run
    ps.sbuf[ps.off[t]] = a;
    ps.sbuf[ps.off[t] + 1] = b;
  }
}

__global__ __launch_bounds__(kThreads) void k_reset(int64_t n_rows, const double *__restrict__ init,
                                                    double *__restrict__ r,
                                                    const uint32_t *__restrict__ rowinfo,
                                                    double *__restrict__ cout,
                                                    double2 *__restrict__ parts) {
  __shared__ double red[kThreads / kWave];
  double dcp = 0.0;
  for (int64_t j = (int64_t)blockIdx.x * kThreads + threadIdx.x; j < n_rows;
       j += (int64_t)gridDim.x * kThreads) {
    const uint32_t info = rowinfo[j];
    if (info & kRowHole) {
      r[j] = 0.0;
      continue;
    }
    const double x = init ? init[j] : 1.0;  // Sparky.java:165-170
    r[j] = x;
    const uint32_t d = info & kRowDegMask;
    if (d > 0) cout[j] = __ddiv_rn(x, (double)d);
    else if (info & kRowSink) dcp = __dadd_rn(dcp, x);
  }
  dcp = block_sum<kThreads>(dcp, red);
  if (threadIdx.x == 0) parts[blockIdx.x] = make_double2(dcp, 0.0);
}

int launch_finalize(pr_graph *g, int64_t n_long, const double2 *parts, int64_t n_parts, int in_buf,
                    int out_buf, hipStream_t stream) {
  double *cout = g->cbuf[out_buf].as<double>() + g->own_off;
  PackSlots ps{};
  if (g->x_fused) {  // the slots of every peer's run (its last two entries)
    ps.sbuf = send_runs(g, out_buf);
    for (int q = 0; q < g->nparts; ++q)
      if (q != g->part) ps.off[ps.n++] = g->x_soff[q + 1] - 2;
  }
  hipLaunchKernelGGL(k_finalize, dim3(g->fin_blocks), dim3(kThreads), 0, stream, n_long,
                     g->lr_row.as<int32_t>(), g->lr_p0.as<int32_t>(), g->piece_part.as<double>(),
                     parts, n_parts, g->r.as<double>(), g->rowinfo.as<uint32_t>(),
                     g->cbuf[in_buf].as<double>(), cout, g->slots, (double)g->V,
                     g->teleport, g->damping, g->fin_part.as<double>(), g->fin_counter.as<unsigned>(),
                     cout + g->S_pad - 2, ps);
  PR_HIP(hipGetLastError());
  return PR_OK;
}

}  // namespace

hipEvent_t next_event(pr_graph *g) {
  if (g->ev_next >= g->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    g->ev_pool.push_back(e);
  }
  return g->ev_pool[g->ev_next++];
}

int time_mark(pr_graph *g, hipStream_t s, int *index) {
  hipEvent_t e = next_event(g);
  if (!e) return fail(PR_ERR_HIP, "hipEventCreate failed");
  PR_HIP(hipEventRecord(e, s));
  *index = (int)g->ev_next - 1;
  return PR_OK;
}

int prepare_hot_kernel() {
  for (int c : {8, 16, 32, 64, 128})
    for (bool walk : {false, true})
      for (bool narrow : {false, true}) {
        if ((walk || narrow) && c > kWave) continue;  // walk and one-wave workgroups: <= 64 classes
        PR_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(epi_grp_kernel(c, walk, narrow)),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)epi_grp_lds(narrow)));
      }
  // k_spmv_hot holds its LDS statically (kHotLdsBytes): no dynamic-LDS attribute to raise
  return PR_OK;
}

// The per-row walk of the grouped epilogue (pr_spmv.h k_epilogue_grp WALK): on by default
// (PR_BOPT_EPI_WALK) at <= 64 classes for the groups whose runs and slot positions fit one window
// load.  Plans which groups walk (k_epi_walk_plan COUNT), places their positions (host prefix over
// the groups) and writes them.
int plan_epi_walk(pr_graph *g) {
  g->epi_walk = false;
  g->n_walk_groups = 0;
  if (!g->opts.epi_walk || g->C > kWave || g->nblk <= 0) return PR_OK;
  const int64_t ngrp = (g->nblk + kEpiGroup - 1) / kEpiGroup;
  using PlanFn = void (*)(int64_t, const void *, const int32_t *, int64_t *, uint16_t *);
  PlanFn count = nullptr, write = nullptr;
  switch (g->C) {
    case 8: count = k_epi_walk_plan<8, true>, write = k_epi_walk_plan<8, false>; break;
    case 16: count = k_epi_walk_plan<16, true>, write = k_epi_walk_plan<16, false>; break;
    case 32: count = k_epi_walk_plan<32, true>, write = k_epi_walk_plan<32, false>; break;
    case 64: count = k_epi_walk_plan<64, true>, write = k_epi_walk_plan<64, false>; break;
    default: return PR_OK;
  }
  PR_TRY(g->eoff.alloc(sizeof(int64_t) * (size_t)ngrp));
  const unsigned blocks = grid_for(ngrp, kEpiThreads / kWave, 8192);
  hipLaunchKernelGGL(count, dim3(blocks), dim3(kEpiThreads), 0, g->stream, g->nblk, g->rmask.p, g->cbase.as<int32_t>(),
                     g->eoff.as<int64_t>(), nullptr);
  PR_HIP(hipGetLastError());
  std::vector<int64_t> off((size_t)ngrp);
  PR_HIP(hipMemcpyAsync(off.data(), g->eoff.p, sizeof(int64_t) * (size_t)ngrp, hipMemcpyDeviceToHost, g->stream));
  PR_HIP(hipStreamSynchronize(g->stream));
  int64_t total = 0;
  for (auto &o : off) {
    if (o < 0) continue;
    const int64_t n = o;
    o = total;  // a multiple of 8 positions: every group's run of positions is padded to 16 bytes
    total += n;
    ++g->n_walk_groups;
  }
  PR_TRY(g->epos.alloc(sizeof(uint16_t) * (size_t)(total > 0 ? total : 8)));
  PR_HIP(hipMemcpyAsync(g->eoff.p, off.data(), sizeof(int64_t) * (size_t)ngrp, hipMemcpyHostToDevice, g->stream));
  if (total > 0)
    hipLaunchKernelGGL(write, dim3(blocks), dim3(kEpiThreads), 0, g->stream, g->nblk, g->rmask.p,
                       g->cbase.as<int32_t>(), g->eoff.as<int64_t>(), g->epos.as<uint16_t>());
  PR_HIP(hipGetLastError());
  PR_HIP(hipStreamSynchronize(g->stream));
  g->epi_walk = true;
  return PR_OK;
}

namespace {
// partial slots of every epilogue group: its class runs [cbase[b0][x], cbase[b0 + nb][x]) summed
__global__ __launch_bounds__(kThreads) void k_epi_cost(int64_t nblk, int C, const int32_t *__restrict__ cbase,
                                                       int32_t *__restrict__ cost) {
  const int64_t ngrp = (nblk + kEpiGroup - 1) / kEpiGroup;
  const int64_t gi = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (gi >= ngrp) return;
  const int64_t b0 = gi * kEpiGroup, b1 = min(nblk, b0 + kEpiGroup);
  int64_t n = 0;
  for (int x = 0; x < C; ++x) n += (int64_t)cbase[b1 * C + x] - cbase[b0 * C + x];
  cost[gi] = (int32_t)min(n, (int64_t)INT32_MAX);
}
}  // namespace

// Dispatch order of the epilogue groups (PR_BOPT_EPI_ORDER; auto: heaviest first for the parts of a
// row partition, row order for one part -- VERDICT r5 item 3).  A group's wave
// stages its class runs batch after batch, so a group holding the first (highest in-degree) rows
// of a class region runs far longer than most; in row order those groups sit at the start of
// every class region and the last regions' ones are dispatched (blockIdx order) last.  Options 1
// and 2 sort the dispatch by slots, heaviest first: runs of kEpiOrderRun consecutive groups (1) or
// single groups (2).  Measured: an s26 P = 8 part's epilogue -8 %, the one-GPU
// pass +2.5 % (every light group then runs at the end), so row order stays for one part.  The
// per-chunk launches of PR_OPT_XCHG_IPC = 2 take positions [lo, hi) of chunk ranges: their order
// is sorted within each.
constexpr int64_t kEpiOrderRun = 8;
int plan_epi_order(pr_graph *g) {
  g->epi_ord.reset();
  const int order = g->opts.epi_order >= 0 ? g->opts.epi_order : (g->nparts > 1 ? 2 : 0);
  if (order == 0 || g->C <= 1 || g->nblk <= 0) return PR_OK;
  const int64_t ngrp = (g->nblk + kEpiGroup - 1) / kEpiGroup;
  DevBuf dcost;
  PR_TRY(dcost.alloc(sizeof(int32_t) * (size_t)ngrp));
  hipLaunchKernelGGL(k_epi_cost, dim3((unsigned)((ngrp + kThreads - 1) / kThreads)), dim3(kThreads), 0, g->stream,
                     g->nblk, g->C, g->cbase.as<int32_t>(), dcost.as<int32_t>());
  PR_HIP(hipGetLastError());
  std::vector<int32_t> cost((size_t)ngrp), ord(2 * (size_t)ngrp);
  PR_HIP(hipMemcpyAsync(cost.data(), dcost.p, sizeof(int32_t) * (size_t)ngrp, hipMemcpyDeviceToHost, g->stream));
  PR_HIP(hipStreamSynchronize(g->stream));
  const int64_t run = order == 1 ? kEpiOrderRun : 1;
  // [lo, hi) in runs of `run` groups from lo, runs by their slots descending, groups in a run in order
  auto sort_range = [&](int32_t *o, int64_t lo, int64_t hi) {
    std::vector<std::pair<int64_t, int64_t>> runs;  // (-slots, first group)
    for (int64_t a = lo; a < hi; a += run) {
      int64_t n = 0;
      for (int64_t k = a; k < std::min(hi, a + run); ++k) n += cost[k];
      runs.emplace_back(-n, a);
    }
    std::sort(runs.begin(), runs.end());
    int64_t w = lo;
    for (const auto &r : runs)
      for (int64_t k = r.second; k < std::min(hi, r.second + run); ++k) o[w++] = (int32_t)k;
  };
  sort_range(ord.data(), 0, ngrp);
  const int nxc = std::max(1, g->C / kXcds);  // the exchange chunks (pr_exchange.hip n_xc)
  const int64_t rows_per_grp = (int64_t)kEpiGroup * kWave, chunk_rows = (int64_t)kXcds * g->Q_pad;
  int64_t lo = 0;
  for (int c = 0; c < nxc; ++c) {
    const int64_t hi = std::max(lo, ipc_epi_chunk_end(ngrp, c, nxc, chunk_rows, rows_per_grp));
    sort_range(ord.data() + ngrp, lo, hi);
    lo = hi;
  }
  if (lo < ngrp) sort_range(ord.data() + ngrp, lo, ngrp);
  PR_TRY(g->epi_ord.alloc(sizeof(int32_t) * ord.size()));
  PR_HIP(hipMemcpyAsync(g->epi_ord.p, ord.data(), sizeof(int32_t) * ord.size(), hipMemcpyHostToDevice, g->stream));
  PR_HIP(hipStreamSynchronize(g->stream));
  return PR_OK;
}

int n_hot_phases(const pr_graph *g) { return g->C > 1 ? std::max(1, g->C / kXcds) : 1; }

int set_hot_reserve(pr_graph *g, int per_xcd) {
  if (per_xcd == 0 || g->C <= 1) {
    g->hot_grid = g->hot_grid_full;
    return PR_OK;
  }
  const int grid = g->hot_grid_full - kXcds * per_xcd;  // still a multiple of kXcds
  if (per_xcd < 0 || grid < kXcds) return fail(PR_ERR_INVALID, "bad CU reserve");
  g->hot_grid = grid;
  return PR_OK;
}

// Dense cold gathers (pr_spmv.h unit_gather) once a pass has this many wave units per CU: R-MAT s26
// (8.8 K per CU) -2.5 %, ER s24 (2 K) -0.5 %; below it a unit's latency chain matters more than its
// gather instructions (R-MAT s20, 0.12 K: +11 %; LiveJournal shape, 0.5 K: +0.7 %; with the rounds of
// 256 still +15 % / +0.4 %, profiles/r06/dense/r6_dense0/).
constexpr int64_t kDenseUnitsPerCU = 1024;
template <bool DENSE>
void *hot_kernel(int code) {
  return code == kCodeC20    ? reinterpret_cast<void *>(k_spmv_hot<kCodeC20, DENSE>)
         : code == kCodeC24  ? reinterpret_cast<void *>(k_spmv_hot<kCodeC24, DENSE>)
         : code == kCodeC20P ? reinterpret_cast<void *>(k_spmv_hot<kCodeC20P, DENSE>)
         : code == kCodeC24P ? reinterpret_cast<void *>(k_spmv_hot<kCodeC24P, DENSE>)
                             : reinterpret_cast<void *>(k_spmv_hot<kCodeU32, DENSE>);
}

int launch_hot(pr_graph *g, int in, int ph0, int ph1) {
  if (ph1 < 0) ph1 = n_hot_phases(g);
  const CodeSrc cd{g->colh.p, g->cside.as<uint32_t>()};
  const bool dense = g->n_hunits >= kDenseUnitsPerCU * (int64_t)g->hot_grid_full;
  auto kern = reinterpret_cast<decltype(&k_spmv_hot<kCodeU32, false>)>(dense ? hot_kernel<true>(g->code)
                                                                              : hot_kernel<false>(g->code));
  if (g->hot.lds_bytes() > (size_t)kHotLdsBytes) return fail(PR_ERR_STATE, "hot set exceeds the LDS");
  hipLaunchKernelGGL(kern, dim3((unsigned)g->hot_grid), dim3(kHotThreads), 0, g->stream,
                     g->hunits.as<Unit>(), g->hucum.as<int64_t>(), g->hot, cd, g->cbuf[in].as<double>(),
                     (uint32_t)(sizeof(double) * g->gsize), g->partial.as<double>(), g->poff.as<int64_t>(),
                     g->piece_part.as<double>(), g->hpos.as<int32_t>(), g->ptab.as<int32_t>(), ph0, ph1);
  PR_HIP(hipGetLastError());
  return PR_OK;
}

void set_exchange_chunking(pr_graph *g) { g->x_chunked = g->opts.xchg_chunks && g->n_xc > 1; }

int join_exchange(pr_graph *g) {
  if (!g->x_pending) return PR_OK;
  PR_HIP(hipStreamWaitEvent(g->stream, g->x_ev.back(), 0));  // chunks are recorded in order
  g->x_pending = false;
  return PR_OK;
}

int iter_reset(pr_graph *g, const double *init_host) {
  hipStream_t s = g->stream;
  PR_TRY(join_exchange(g));  // a previous run's exchange may still be on xstream
  DevBuf dinit;
  if (init_host && g->n_rows > 0) {
    std::vector<double> loc((size_t)g->n_rows, 0.0);
    for (int64_t L = 0; L < g->n_rows; ++L)
      if (g->orig_of_local[L] >= 0) loc[L] = init_host[g->orig_of_local[L]];
    PR_TRY(dinit.alloc(sizeof(double) * g->n_rows));
    PR_HIP(hipMemcpyAsync(dinit.p, loc.data(), sizeof(double) * g->n_rows, hipMemcpyHostToDevice, s));
    PR_HIP(hipStreamSynchronize(s));
  }
  g->cur = 0;
  g->x_packed = -1;
  if (g->x_free_ev) PR_HIP(hipEventRecord(g->x_free_ev, s));  // the exchange below fills buffer 0
  PR_TRY(ipc_send_runs_free(g, 0));  // k_finalize below writes the slots of the runs of buffer 0
  const int64_t own = g->own_off;
  hipLaunchKernelGGL(k_reset, dim3(g->reset_blocks), dim3(kThreads), 0, s, g->n_rows,
                     dinit.p ? dinit.as<double>() : nullptr, g->r.as<double>(), g->rowinfo.as<uint32_t>(),
                     g->cbuf[0].as<double>() + own, g->reset_part.as<double2>());
  PR_HIP(hipGetLastError());
  PR_TRY(launch_finalize(g, 0, g->reset_part.as<double2>(), g->reset_blocks, 0, 0, s));
  if (!g->grouped) {
    PR_TRY(exchange(g, 0));
    PR_TRY(join_exchange(g));
  }
  PR_HIP(hipStreamSynchronize(s));
  g->iters_done = 0;
  g->ready = true;
  g->ev_next = 0;
  g->spmv_ev.clear();
  g->spmv_passes = 0;
  g->iter_timed = 0;
  g->iter_ev.clear();
  g->xchg_ev.clear();
  return PR_OK;
}

namespace {
int64_t epi_groups(const pr_graph *g) { return (g->nblk + kEpiGroup - 1) / kEpiGroup; }
}  // namespace

int iter_compute(pr_graph *g) {
  hipStream_t s = g->stream;
  const int64_t own = g->own_off;
  const int in = g->cur, out = g->cur ^ 1;
  // timing (spmv_ms_mean): the pass's kernels only.  Every start event is recorded after the
  // stream's wait for the exchange, so a transfer still in flight is never counted as SpMV time;
  // the overlapped exchange contributes one interval per hot phase.
  int open_ev = -1;  // ev_pool index of the running interval's start
  const int hint = g->ev_start_hint;
  g->ev_start_hint = -1;
  bool enqueued = false;  // anything on the stream since the hint's record
  auto mark_start = [&]() -> int {
    if (!g->timing) return PR_OK;
    if (hint >= 0 && !enqueued) {  // the iteration's start event is the pass's start too
      open_ev = hint;
      enqueued = true;  // once
      return PR_OK;
    }
    hipEvent_t e = next_event(g);
    if (!e) return fail(PR_ERR_HIP, "hipEventCreate failed");
    PR_HIP(hipEventRecord(e, s));
    open_ev = (int)g->ev_next - 1;
    return PR_OK;
  };
  auto mark_end = [&]() -> int {
    if (!g->timing) return PR_OK;
    hipEvent_t e = next_event(g);
    if (!e) return fail(PR_ERR_HIP, "hipEventCreate failed");
    PR_HIP(hipEventRecord(e, s));
    g->spmv_ev.push_back({open_ev, (int)g->ev_next - 1});
    open_ev = (int)g->ev_next - 1;  // a following interval may start where this one ended
    return PR_OK;
  };
  // the gather buffer this iteration's exchange fills (`out`) was last read by the previous pass
  if (g->x_free_ev) PR_HIP(hipEventRecord(g->x_free_ev, s));
  PR_TRY(ipc_send_runs_free(g, out));  // the epilogue and k_finalize write the runs of `out`
  const int nph = g->C > 1 ? n_hot_phases(g) : 1;
  const bool phased_wait = g->C > 1 && g->n_hunits > 0 && g->x_pending && g->x_chunked && g->n_xc == nph && nph > 1;
  // one part: nothing above enqueued anything (no exchange, no IPC buffers)
  enqueued = g->nparts > 1 || g->x_free_ev != nullptr || g->x_pending;
  if (!phased_wait) PR_TRY(join_exchange(g));
  else PR_HIP(hipStreamWaitEvent(s, g->x_ev[0], 0));  // phase 0's chunk
  PR_TRY(mark_start());
  // light rows (all rows when C == 1): fused single pass
  if (g->n_units > 0)
    hipLaunchKernelGGL((k_spmv_units<kPerThread, true>), dim3((unsigned)g->n_units), dim3(kThreads), 0, s,
                       g->units.as<Unit>(), g->rowptr.as<int64_t>(), g->colp.as<int32_t>(),
                       g->cbuf[in].as<double>(), g->cbuf[out].as<double>() + own, g->r.as<double>(),
                       g->rowinfo.as<uint32_t>(), g->piece_part.as<double>(), g->unit_part.as<double2>(),
                       g->slots, g->S_pad, (double)g->V, g->teleport, g->damping);
  int64_t n_parts = g->n_units;
  if (g->C > 1) {  // split layout: class units, long segments, then the epilogue over all rows
    if (phased_wait) {
      // overlapped exchange: hot phase c needs only chunk c of the runs received from every peer
      for (int c = 0; c < nph; ++c) {
        if (c > 0) {
          PR_TRY(mark_end());
          PR_HIP(hipStreamWaitEvent(s, g->x_ev[c], 0));
          PR_TRY(mark_start());
        }
        PR_TRY(launch_hot(g, in, c, c + 1));
      }
      g->x_pending = false;
    } else if (g->n_hunits > 0) {
      PR_TRY(launch_hot(g, in));
    }
    if (g->n_segs > 0)
      hipLaunchKernelGGL(k_seg_reduce, dim3(grid_for(g->n_segs, kThreads / kWave, 4096)), dim3(kThreads), 0, s,
                         g->n_segs, g->seg_slot.as<int64_t>(), g->seg_p0.as<int32_t>(), g->piece_part.as<double>(),
                         g->partial.as<double>());
    const EpiGrpFn epi = epi_grp_kernel(g->C, g->epi_walk, g->epi_narrow);
    PackDst pd{};  // fused pack: c' straight into the send runs paired with buffer `out`
    if (g->x_fused) {
      pd.sbuf = send_runs(g, out);
      pd.P = g->nparts;
      pd.self = g->part;
      for (int q = 0; q < g->nparts; ++q) pd.soff[q] = g->x_soff[q];
    }
    const int64_t ngrp = epi_groups(g);
    // dispatch order (plan_epi_order): the whole pass, or sorted within each chunk's range
    const int32_t *ord = g->epi_ord.p ? g->epi_ord.as<int32_t>() + (ipc_early(g) ? ngrp : 0) : nullptr;
    auto epilogue = [&](int64_t g_lo, int64_t g_hi, unsigned grid) -> int {
      hipLaunchKernelGGL(epi, dim3(grid), dim3(epi_grp_threads(g->epi_narrow)), epi_grp_lds(g->epi_narrow), s,
                         g->nblk, g_lo, g_hi, g->partial.as<double>(), g->rmask.p, g->cbase.as<int32_t>(),
                         g->rowinfo.as<uint32_t>(), g->r.as<double>(), g->cbuf[out].as<double>() + own,
                         g->cbuf[in].as<double>(), g->slots, (double)g->V, g->teleport, g->damping,
                         g->unit_part.as<double2>() + g->n_units, g->eoff.as<int64_t>(), g->epos.as<uint16_t>(),
                         g->x_pmask.as<uint8_t>(), g->x_sbase.as<int32_t>(), ord, pd);
      PR_HIP(hipGetLastError());
      return PR_OK;
    };
    if (!ipc_early(g)) {
      PR_TRY(epilogue(0, ngrp, (unsigned)g->ep_blocks));
    } else {
      // PR_OPT_XCHG_IPC = 2: chunk c of the send runs holds the rows of class regions [8c, 8c + 8),
      // local rows [8c Q_pad, (8c + 8) Q_pad): the epilogue runs over the groups that end them, and
      // the chunk is published as soon as it is written (its peers' pulls then overlap the rest of
      // the epilogue); the last chunk carries the slots k_finalize writes and goes with the exchange
      const int64_t rows_per_grp = (int64_t)kEpiGroup * kWave, chunk_rows = (int64_t)kXcds * g->Q_pad;
      const int wpb = epi_grp_threads(g->epi_narrow) / kWave;
      int64_t g_lo = 0;
      for (int c = 0; c < g->n_xc; ++c) {
        const int64_t g_hi = ipc_epi_chunk_end(ngrp, c, g->n_xc, chunk_rows, rows_per_grp);
        if (g_hi > g_lo) PR_TRY(epilogue(g_lo, g_hi, grid_for(g_hi - g_lo, wpb, 1u << 20)));
        g_lo = std::max(g_lo, g_hi);
        if (c < g->n_xc - 1) PR_TRY(ipc_chunk_sent(g, out, c));
      }
    }
    n_parts += epi_groups(g);
  }
  PR_HIP(hipGetLastError());
  PR_TRY(mark_end());
  if (g->timing) ++g->spmv_passes;
  PR_TRY(launch_finalize(g, g->n_long, g->unit_part.as<double2>(), n_parts, in, out, s));
  g->x_packed = (g->x_fused && g->C > 1) ? out : -1;  // the exchange then skips k_pack
  g->cur = out;
  ++g->iters_done;
  return PR_OK;
}

int iter_step(pr_graph *g, int32_t iterations) {
  if (!g->ready) return fail(PR_ERR_STATE, "pr_step before pr_reset");
  if (g->grouped) return fail(PR_ERR_STATE, "graph belongs to a group: use pr_group_step");
  if (g->timing && g->nparts == 1 && iterations > 0) {
    // one part (no exchange): the call's iterations are one interval, its kernels back to back --
    // every event recorded between two kernels is a marker packet of ~5 us (R-MAT s20: 2 of them
    // were 18 % of an iteration), so the pass here is the whole iteration, k_finalize included
    hipEvent_t e0 = next_event(g);
    if (!e0) return fail(PR_ERR_HIP, "hipEventCreate failed");
    PR_HIP(hipEventRecord(e0, g->stream));
    const int i0 = (int)g->ev_next - 1;
    g->timing = false;
    int rc = PR_OK;
    for (int32_t it = 0; it < iterations && rc == PR_OK; ++it) {
      rc = iter_compute(g);
      if (rc == PR_OK) rc = exchange(g, g->cur);
    }
    g->timing = true;
    PR_TRY(rc);
    hipEvent_t e1 = next_event(g);
    if (!e1) return fail(PR_ERR_HIP, "hipEventCreate failed");
    PR_HIP(hipEventRecord(e1, g->stream));
    const int i1 = (int)g->ev_next - 1;
    g->spmv_ev.push_back({i0, i1});
    g->spmv_passes += iterations;
    g->iter_ev.push_back({i0, i1});
    g->iter_timed += iterations;
    return PR_OK;
  }
  int carry = -1;  // the previous iteration's end event: nothing was enqueued after it
  for (int32_t it = 0; it < iterations; ++it) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int i0 = carry;
    if (g->timing && i0 < 0) {
      e0 = next_event(g);
      if (!e0) return fail(PR_ERR_HIP, "hipEventCreate failed");
      PR_HIP(hipEventRecord(e0, g->stream));
      i0 = (int)g->ev_next - 1;
    }
    g->ev_start_hint = g->timing ? i0 : -1;
    PR_TRY(iter_compute(g));
    hipEvent_t xa = nullptr, xb = nullptr;
    if (g->timing && g->nparts > 1) {
      xa = next_event(g);
      xb = next_event(g);
      if (!xa || !xb) return fail(PR_ERR_HIP, "hipEventCreate failed");
      const int ia = (int)g->ev_next - 2;
      g->xchg_ev.push_back({ia, ia + 1});  // pack done -> last chunk received (xstream)
    }
    PR_TRY(exchange(g, g->cur, xa, xb));
    if (g->timing) {
      e1 = next_event(g);
      if (!e1) return fail(PR_ERR_HIP, "hipEventCreate failed");
      PR_HIP(hipEventRecord(e1, g->stream));  // compute stream: the iteration's kernels + the pack
      const int i1 = (int)g->ev_next - 1;
      g->iter_ev.push_back({i0, i1});
      ++g->iter_timed;
      carry = i1;  // the next iteration starts where this one ended (same stream, nothing between)
    }
  }
  return PR_OK;
}

int read_slots(pr_graph *g, int buf, double *dc, double *l1) {
  PR_TRY(join_exchange(g));  // the peers' slots arrive with the exchange
  std::vector<double> h(2 * (size_t)g->nparts);
  for (int p = 0; p < g->nparts; ++p)
    PR_HIP(hipMemcpyAsync(&h[2 * p], g->cbuf[buf].as<double>() + g->slots.pos[p], 2 * sizeof(double),
                          hipMemcpyDeviceToHost, g->stream));
  PR_HIP(hipStreamSynchronize(g->stream));
  double a = 0.0, b = 0.0;
  for (int p = 0; p < g->nparts; ++p) {
    a += h[2 * p];
    b += h[2 * p + 1];
  }
  *dc = a;
  *l1 = b;
  return PR_OK;
}

}  // namespace pr
