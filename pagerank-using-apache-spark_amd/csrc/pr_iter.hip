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
#include <climits>

#include "pr_device.h"
#include "pr_graph.h"
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
    double *__restrict__ slot_out) {
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

hipEvent_t next_event(pr_graph *g) {
  if (g->ev_next >= g->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    g->ev_pool.push_back(e);
  }
  return g->ev_pool[g->ev_next++];
}

int launch_finalize(pr_graph *g, int64_t n_long, const double2 *parts, int64_t n_parts, int in_buf,
                    int out_buf) {
  double *cout = g->cbuf[out_buf].as<double>() + g->own_off;
  hipLaunchKernelGGL(k_finalize, dim3(g->fin_blocks), dim3(kThreads), 0, g->stream, n_long,
                     g->lr_row.as<int32_t>(), g->lr_p0.as<int32_t>(), g->piece_part.as<double>(),
                     parts, n_parts, g->r.as<double>(), g->rowinfo.as<uint32_t>(),
                     g->cbuf[in_buf].as<double>(), cout, g->slots, (double)g->V,
                     g->teleport, g->damping, g->fin_part.as<double>(), g->fin_counter.as<unsigned>(),
                     cout + g->S_pad - 2);
  PR_HIP(hipGetLastError());
  return PR_OK;
}

}  // namespace

int prepare_hot_kernel() {
  for (int v = 0; v < kNumEpiVariants; ++v)
    for (int c : {8, 16, 32, 64, 128})
      for (bool walk : {false, true})
        for (bool narrow : {false, true})
          PR_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(epi_grp_kernel(c, v, walk, narrow)),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)epi_grp_lds(v, narrow)));
  for (const void *k : {reinterpret_cast<const void *>(&k_spmv_hot<0, 0, 0, true>),
                        reinterpret_cast<const void *>(&k_spmv_hot<1, 0, 1, true>),
                        reinterpret_cast<const void *>(&k_spmv_hot<0, 0, 0, false>),
                        reinterpret_cast<const void *>(&k_spmv_hot<1, 0, 1, false>)})
    PR_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  return PR_OK;
}

// The per-row walk of the grouped epilogue (pr_spmv.h k_epilogue_grp WALK): on by default for its
// variants 0 and 7 at <= 64 classes for the groups that fit one window load (PR_EPI_WALK=1);
// 0 keeps the class loop everywhere, 2 walks by the step estimate (A/B, k_epi_walk_plan).  Plans
// which groups walk (k_epi_walk_plan COUNT), places their positions (host prefix over the groups)
// and writes them.
int plan_epi_walk(pr_graph *g) {
  g->epi_walk = false;
  g->n_walk_groups = 0;
  int rule = 1;
  if (const char *e = getenv("PR_EPI_WALK")) rule = std::min(std::max(atoi(e), 0), 2);
  if (rule == 0 || !g->epi_grp || !epi_walk_variant(g->C, g->epi_var) || g->nblk <= 0) return PR_OK;
  const int G = kEpiVariants[g->epi_var].G;
  const int64_t ngrp = (g->nblk + G - 1) / G;
  using PlanFn = void (*)(int64_t, const void *, const int32_t *, int64_t *, uint16_t *, int);
  PlanFn count = nullptr, write = nullptr;
  constexpr int G7 = kEpiVariants[7].G, W7 = kEpiVariants[7].W;
  static_assert(kEpiVariants[0].G == kEpiGroup && kEpiVariants[0].W == kEpiWin, "variant 0 is the default");
  const bool wide = g->epi_var == 7;
#define PR_WALK_PLAN(CC)                                                                                   \
  count = wide ? k_epi_walk_plan<CC, G7, W7, true> : k_epi_walk_plan<CC, kEpiGroup, kEpiWin, true>;        \
  write = wide ? k_epi_walk_plan<CC, G7, W7, false> : k_epi_walk_plan<CC, kEpiGroup, kEpiWin, false>;
  switch (g->C) {
    case 8: PR_WALK_PLAN(8) break;
    case 16: PR_WALK_PLAN(16) break;
    case 32: PR_WALK_PLAN(32) break;
    case 64: PR_WALK_PLAN(64) break;
    default: return PR_OK;
  }
#undef PR_WALK_PLAN
  PR_TRY(g->eoff.alloc(sizeof(int64_t) * (size_t)ngrp));
  const unsigned blocks = grid_for(ngrp, kEpiThreads / kWave, 8192);
  hipLaunchKernelGGL(count, dim3(blocks), dim3(kEpiThreads), 0, g->stream, g->nblk, g->rmask.p, g->cbase.as<int32_t>(),
                     g->eoff.as<int64_t>(), nullptr, rule);
  PR_HIP(hipGetLastError());
  std::vector<int64_t> off((size_t)ngrp);
  PR_HIP(hipMemcpyAsync(off.data(), g->eoff.p, sizeof(int64_t) * (size_t)ngrp, hipMemcpyDeviceToHost, g->stream));
  PR_HIP(hipStreamSynchronize(g->stream));
  int64_t total = 0;
  for (auto &o : off) {
    if (o < 0) continue;
    const int64_t n = o;
    o = total;  // a multiple of 8 positions: every batch's run of positions is padded to 16 bytes
    total += n;
    ++g->n_walk_groups;
  }
  PR_TRY(g->epos.alloc(sizeof(uint16_t) * (size_t)(total > 0 ? total : 8)));
  PR_HIP(hipMemcpyAsync(g->eoff.p, off.data(), sizeof(int64_t) * (size_t)ngrp, hipMemcpyHostToDevice, g->stream));
  if (total > 0)
    hipLaunchKernelGGL(write, dim3(blocks), dim3(kEpiThreads), 0, g->stream, g->nblk, g->rmask.p,
                       g->cbase.as<int32_t>(), g->eoff.as<int64_t>(), g->epos.as<uint16_t>(), rule);
  PR_HIP(hipGetLastError());
  PR_HIP(hipStreamSynchronize(g->stream));
  g->epi_walk = true;
  return PR_OK;
}

int n_hot_phases(const pr_graph *g) { return g->hot_phased ? std::max(1, g->C / kXcds) : 1; }

int set_hot_reserve(pr_graph *g, int per_xcd) {
  if (per_xcd == 0) {
    g->hot_grid = g->hot_grid_full;
    return PR_OK;
  }
  if (!g->hot_phased) return fail(PR_ERR_INVALID, "reserving CUs needs the phased k_spmv_hot schedule");
  const int grid = g->hot_grid_full - kXcds * per_xcd;  // still a multiple of kXcds
  if (per_xcd < 0 || grid < kXcds) return fail(PR_ERR_INVALID, "bad CU reserve");
  g->hot_grid = grid;
  return PR_OK;
}

int launch_hot(pr_graph *g, int in, int ph0, int ph1) {
  const size_t lds = g->hot.lds_bytes();
  // phased: ORDER 1, each unit reduced before the next unit's gathers are issued (-3.7 % at s26,
  // -6.6 % for a P = 8 part, -3.6 % ER s24: profiles/r02/order_ab/)
  auto *kern = g->hot_meta ? (g->hot_phased ? &k_spmv_hot<1, 0, 1, false> : &k_spmv_hot<0, 0, 0, false>)
                           : (g->hot_phased ? &k_spmv_hot<1, 0, 1, true> : &k_spmv_hot<0, 0, 0, true>);
  if (ph1 < 0) ph1 = n_hot_phases(g);
  hipLaunchKernelGGL(kern, dim3((unsigned)g->hot_grid), dim3(kHotThreads), lds, g->stream,
                     g->hunits.as<Unit>(), g->hucum.as<int64_t>(), g->hot, g->colh.as<uint32_t>(),
                     g->hmeta.as<uint32_t>(), g->cbuf[in].as<double>(),
                     (uint32_t)(sizeof(double) * g->gsize), g->partial.as<double>(),
                     g->poff.as<int64_t>(), g->piece_part.as<double>(), g->hpos.as<int32_t>(), ph0, ph1);
  PR_HIP(hipGetLastError());
  return PR_OK;
}

void set_exchange_chunking(pr_graph *g) {
  bool on = false;
  if (const char *e = getenv("PR_XCHG_CHUNKS")) on = atoi(e) != 0;
  g->x_chunked = on && g->n_xc > 1;
}

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
  const int64_t own = g->own_off;
  hipLaunchKernelGGL(k_reset, dim3(g->reset_blocks), dim3(kThreads), 0, s, g->n_rows,
                     dinit.p ? dinit.as<double>() : nullptr, g->r.as<double>(), g->rowinfo.as<uint32_t>(),
                     g->cbuf[0].as<double>() + own, g->reset_part.as<double2>());
  PR_HIP(hipGetLastError());
  PR_TRY(launch_finalize(g, 0, g->reset_part.as<double2>(), g->reset_blocks, 0, 0));
  if (!g->grouped) {
    PR_TRY(exchange(g, 0));
    PR_TRY(join_exchange(g));
  }
  PR_HIP(hipStreamSynchronize(s));
  g->iters_done = 0;
  g->ready = true;
  g->ev_next = 0;
  g->spmv_ev.clear();
  g->iter_ev.clear();
  g->xchg_ev.clear();
  return PR_OK;
}

int iter_compute(pr_graph *g) {
  hipStream_t s = g->stream;
  const int64_t own = g->own_off;
  const int in = g->cur, out = g->cur ^ 1;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (g->timing) {
    e0 = next_event(g);
    e1 = next_event(g);
    if (!e0 || !e1) return fail(PR_ERR_HIP, "hipEventCreate failed");
    PR_HIP(hipEventRecord(e0, s));
  }
  // light rows (all rows when C == 1): fused single pass
  if (g->C == 1) PR_TRY(join_exchange(g));
  if (g->n_units > 0)
    hipLaunchKernelGGL((k_spmv_units<kPerThread, true>), dim3((unsigned)g->n_units), dim3(kThreads), 0, s,
                       g->units.as<Unit>(), g->rowptr.as<int64_t>(), g->colp.as<int32_t>(),
                       g->cbuf[in].as<double>(), g->cbuf[out].as<double>() + own, g->r.as<double>(),
                       g->rowinfo.as<uint32_t>(), g->piece_part.as<double>(), g->unit_part.as<double2>(),
                       g->slots, g->S_pad, (double)g->V, g->teleport, g->damping, 0xFFFFFFFFu);
  int64_t n_parts = g->n_units;
  if (g->C > 1) {  // split layout: class units, long segments, then the epilogue over all rows
    const int nph = n_hot_phases(g);
    if (g->n_hunits > 0 && g->x_pending && g->x_chunked && g->n_xc == nph && nph > 1) {
      // overlapped exchange: hot phase c needs only chunk c of the runs received from every peer
      for (int c = 0; c < nph; ++c) {
        PR_HIP(hipStreamWaitEvent(s, g->x_ev[c], 0));
        PR_TRY(launch_hot(g, in, c, c + 1));
      }
      g->x_pending = false;
    } else {
      PR_TRY(join_exchange(g));
      if (g->n_hunits > 0) PR_TRY(launch_hot(g, in));
    }
    if (g->n_segs > 0)
      hipLaunchKernelGGL(k_seg_reduce, dim3(grid_for(g->n_segs, kThreads / kWave, 4096)), dim3(kThreads), 0, s,
                         g->n_segs, g->seg_slot.as<int64_t>(), g->seg_p0.as<int32_t>(), g->piece_part.as<double>(),
                         g->partial.as<double>());
    if (g->epi_grp) {
      const EpiGrpFn epi = epi_grp_kernel(g->C, g->epi_var, g->epi_walk, g->epi_narrow);
      const size_t lds = epi_grp_lds(g->epi_var, g->epi_narrow);
      hipLaunchKernelGGL(epi, dim3(g->ep_blocks), dim3(epi_grp_threads(g->epi_var, g->epi_narrow)), lds, s, g->nblk, g->partial.as<double>(),
                         g->rmask.p, g->cbase.as<int32_t>(), g->rowinfo.as<uint32_t>(),
                         g->r.as<double>(), g->cbuf[out].as<double>() + own, g->cbuf[in].as<double>(), g->slots,
                         (double)g->V, g->teleport, g->damping, g->unit_part.as<double2>() + g->n_units,
                         g->eoff.as<int64_t>(), g->epos.as<uint16_t>());
    } else {
    auto *epi = g->epi_abs ? (g->C == 32 ? k_epilogue<32, true> : (g->C == 16 ? k_epilogue<16, true> : k_epilogue<8, true>))
                           : (g->C == 32 ? k_epilogue<32> : (g->C == 16 ? k_epilogue<16> : k_epilogue<8>));
    hipLaunchKernelGGL(epi, dim3(g->ep_blocks),
                       dim3(kThreads), 0, s, g->nblk, g->part_off, g->partial.as<double>(),
                       g->rmask.as<uint32_t>(), g->cbase.as<int32_t>(),
                       g->rowinfo.as<uint32_t>(), g->r.as<double>(), g->cbuf[out].as<double>() + own,
                       g->cbuf[in].as<double>(), g->slots, (double)g->V, g->teleport, g->damping,
                       g->unit_part.as<double2>() + g->n_units);
    }
    n_parts += g->ep_blocks;
  }
  PR_HIP(hipGetLastError());
  if (g->timing) {
    PR_HIP(hipEventRecord(e1, s));
    const int base = (int)g->ev_next - 2;
    g->spmv_ev.push_back({base, base + 1});
  }
  PR_TRY(launch_finalize(g, g->n_long, g->unit_part.as<double2>(), n_parts, in, out));
  g->cur = out;
  ++g->iters_done;
  return PR_OK;
}

int iter_step(pr_graph *g, int32_t iterations) {
  if (!g->ready) return fail(PR_ERR_STATE, "pr_step before pr_reset");
  if (g->grouped) return fail(PR_ERR_STATE, "graph belongs to a group: use pr_group_step");
  for (int32_t it = 0; it < iterations; ++it) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (g->timing) {
      e0 = next_event(g);
      if (!e0) return fail(PR_ERR_HIP, "hipEventCreate failed");
      PR_HIP(hipEventRecord(e0, g->stream));
    }
    const int i0 = (int)g->ev_next - 1;
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
