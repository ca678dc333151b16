// C ABI of libpagerank_hip (include/pagerank_hip.h): handle management, error reporting,
// the run loop with its per-iteration callback, export, and the RCCL exchange.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "pr_graph.h"
#include "pr_xcheck.h"

namespace pr {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }
int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

int DevBuf::alloc(size_t n) {
  reset();
  if (n == 0) n = 1;
  hipError_t e = hipMalloc(&p, n);
  if (e != hipSuccess) {
    p = nullptr;
    (void)hipGetLastError();
    return fail(PR_ERR_OOM, "hipMalloc(" + std::to_string(n) + " bytes) failed: " + hipGetErrorString(e));
  }
  bytes = n;
  return PR_OK;
}

void DevBuf::reset() {
  if (p) (void)hipFree(p);
  p = nullptr;
  bytes = 0;
}

}  // namespace pr

size_t pr_graph::device_bytes() const {
  size_t b = canon_rowptr.bytes + canon_col.bytes + canon_deg.bytes + canon_vflags.bytes;
  b += rowptr.bytes + col.bytes + colp.bytes + rowinfo.bytes + colh.bytes + hunits.bytes + partial.bytes + poff.bytes + rmask.bytes + cbase.bytes + seg_slot.bytes + seg_p0.bytes + r.bytes + cbuf[0].bytes + cbuf[1].bytes + eoff.bytes + epos.bytes;
  b += units.bytes + unit_part.bytes + lr_row.bytes + lr_p0.bytes + piece_part.bytes;
  b += fin_part.bytes + fin_counter.bytes + reset_part.bytes + x_send.bytes + x_sbuf.bytes + hpos.bytes + cside.bytes;
  return b;
}

using pr::fail;

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int check_device(int32_t device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return fail(PR_ERR_NODEVICE, "no HIP device available");
  }
  if (device < 0 || device >= n) return fail(PR_ERR_INVALID, "device index out of range");
  return PR_OK;
}

// (key, value) build options -> g->opts (PR_BOPT_*); an unknown key or a value out of range fails
int parse_options(const int64_t *options, int32_t n, pr_build_opts *o) {
  if (n < 0 || (n > 0 && !options)) return fail(PR_ERR_INVALID, "options is NULL");
  for (int32_t i = 0; i < n; ++i) {
    const int64_t k = options[2 * i], v = options[2 * i + 1];
    switch (k) {
      case PR_BOPT_CLASSES:
        if (v != 0 && v != 8 && v != 16 && v != 32 && v != 64 && v != 128)
          return fail(PR_ERR_INVALID, "PR_BOPT_CLASSES: 0 (policy), 8, 16, 32, 64 or 128");
        o->classes = (int)v;
        break;
      case PR_BOPT_HOT_SLOTS:
        if (v < -1 || v > pr::kHotSlotsMax) return fail(PR_ERR_INVALID, "PR_BOPT_HOT_SLOTS: -1 (default) or 0..18429");
        o->hot_slots = (int)v;
        break;
      case PR_BOPT_EXCHANGE:
        if (v != 0 && v != 1) return fail(PR_ERR_INVALID, "PR_BOPT_EXCHANGE: 0 (runs) or 1 (all-gather)");
        o->allgather = v == 1;
        break;
      case PR_BOPT_XCHG_CHUNKS:
        if (v != 0 && v != 1) return fail(PR_ERR_INVALID, "PR_BOPT_XCHG_CHUNKS: 0 (whole runs) or 1 (overlapped)");
        o->xchg_chunks = v == 1;
        break;
      case PR_BOPT_HOT_RESERVE:
        if (v < 0 || v > 3) return fail(PR_ERR_INVALID, "PR_BOPT_HOT_RESERVE: 0..3 CUs per XCD");
        o->hot_reserve = (int)v;
        break;
      case PR_BOPT_EPI_WALK:
        if (v != 0 && v != 1) return fail(PR_ERR_INVALID, "PR_BOPT_EPI_WALK: 0 (class loop) or 1 (per-row walk)");
        o->epi_walk = v == 1;
        break;
      case PR_BOPT_EPI_NARROW:
        if (v < -1 || v > 1) return fail(PR_ERR_INVALID, "PR_BOPT_EPI_NARROW: -1 (auto), 0 or 1");
        o->epi_narrow = (int)v;
        break;
      case PR_BOPT_CODES:
        if (v != -1 && v != 0) return fail(PR_ERR_INVALID, "PR_BOPT_CODES: -1 (compact where they fit) or 0 (32-bit)");
        o->codes = (int)v;
        break;
      case PR_BOPT_PACK_FUSED:
        if (v != 0 && v != 1) return fail(PR_ERR_INVALID, "PR_BOPT_PACK_FUSED: 0 (pack kernel) or 1 (in the epilogue)");
        o->pack_fused = v == 1;
        break;
      case PR_BOPT_XCHG_SDMA:
        if (v != 0 && v != 1) return fail(PR_ERR_INVALID, "PR_BOPT_XCHG_SDMA: 0 (device copies) or 1 (copy engines)");
        o->xchg_sdma = v == 1;
        break;
      case PR_BOPT_EPI_ORDER:
        if (v < -1 || v > 2)
          return fail(PR_ERR_INVALID, "PR_BOPT_EPI_ORDER: -1 (auto), 0 (row order), 1 (runs of 8 groups heaviest first), "
                                      "2 (groups heaviest first)");
        o->epi_order = (int)v;
        break;
      default:
        return fail(PR_ERR_INVALID, "unknown build option " + std::to_string(k));
    }
  }
  return PR_OK;
}

int create_common(int32_t device, int32_t part, int32_t n_parts, int32_t n_vertices, int64_t n_edges,
                  const int32_t *src, const int32_t *dst, uint32_t flags, const int64_t *options,
                  int32_t n_options, pr_graph **out) {
  if (!out) return fail(PR_ERR_INVALID, "out is NULL");
  *out = nullptr;
  if (n_parts < 1 || part < 0 || part >= n_parts) return fail(PR_ERR_INVALID, "bad part / n_parts");
  if (n_parts > pr::kMaxParts) return fail(PR_ERR_INVALID, "n_parts above 64 is not supported");
  if (n_vertices < 0 || n_edges < 0) return fail(PR_ERR_INVALID, "negative size");
  if (n_edges > 0 && (!src || !dst)) return fail(PR_ERR_INVALID, "src/dst is NULL");
  if (flags & ~(PR_DANGLING_NONE | PR_INPUT_DEVICE | PR_NO_CANONICAL | PR_LAYOUT_FUSED | PR_LAYOUT_SPLIT))
    return fail(PR_ERR_INVALID, "unknown flag bits");
  if ((flags & PR_LAYOUT_FUSED) && (flags & PR_LAYOUT_SPLIT)) return fail(PR_ERR_INVALID, "PR_LAYOUT_FUSED and PR_LAYOUT_SPLIT are exclusive");
  pr_build_opts opts;
  PR_TRY(parse_options(options, n_options, &opts));
  PR_TRY(check_device(device));
  DeviceGuard dg(device);
  pr_graph *g = new (std::nothrow) pr_graph();
  if (!g) return fail(PR_ERR_OOM, "host allocation failed");
  g->opts = opts;
  g->device = device;
  g->flags = flags;
  g->V = n_vertices;
  g->part = part;
  g->nparts = n_parts;
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
    delete g;
    return fail(PR_ERR_HIP, "hipStreamCreate failed");
  }
  int rc = pr::build_graph(g, n_edges, src, dst);
  if (rc != PR_OK) {
    std::string msg = pr_last_error();
    pr_graph_destroy(g);
    pr::set_error(msg);
    return rc;
  }
  *out = g;
  return PR_OK;
}

}  // namespace

extern "C" {

int pr_abi_version(void) { return PR_ABI_VERSION; }

const char *pr_last_error(void) { return pr::g_last_error.c_str(); }

int pr_device_count(int32_t *out) {
  if (!out) return fail(PR_ERR_INVALID, "out is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  *out = n;
  return PR_OK;
}

int pr_graph_create(int32_t device, int32_t n_vertices, int64_t n_edges, const int32_t *src,
                    const int32_t *dst, uint32_t flags, pr_graph **out) {
  return create_common(device, 0, 1, n_vertices, n_edges, src, dst, flags, nullptr, 0, out);
}

int pr_graph_create_part(int32_t device, int32_t part, int32_t n_parts, int32_t n_vertices,
                         int64_t n_edges, const int32_t *src, const int32_t *dst, uint32_t flags,
                         pr_graph **out) {
  return create_common(device, part, n_parts, n_vertices, n_edges, src, dst, flags, nullptr, 0, out);
}

int pr_graph_create_ex(int32_t device, int32_t part, int32_t n_parts, int32_t n_vertices, int64_t n_edges,
                       const int32_t *src, const int32_t *dst, uint32_t flags, const int64_t *options,
                       int32_t n_options, pr_graph **out) {
  return create_common(device, part, n_parts, n_vertices, n_edges, src, dst, flags, options, n_options, out);
}

// doubles moved per iteration by this part: the packed runs, or whole slices (PR_BOPT_EXCHANGE = 1)
static int64_t xchg_volume(const pr_graph *g, bool send) {
  if (g->nparts <= 1) return 0;
  if (g->x_allgather) return (send ? 1 : g->nparts - 1) * g->S_pad;
  const std::vector<int64_t> &o = send ? g->x_soff : g->x_roff;
  return o.empty() ? 0 : o.back();
}

int pr_graph_info(const pr_graph *g, int64_t *info, int32_t n_info) {
  if (!g || !info) return fail(PR_ERR_INVALID, "NULL argument");
  const int64_t v[PR_INFO_COUNT] = {g->V,        g->E_dedup,  g->n_sink,    g->n_nolink, g->n_indeg0,
                                    g->max_indeg, g->n_local,  g->local_nnz, g->part,     g->nparts,
                                    g->n_units + g->n_hunits, g->n_long + g->n_segs,
                                    (int64_t)g->device_bytes(), g->C,
                                    xchg_volume(g, true), xchg_volume(g, false), g->n_slots,
                                    g->C > 1 ? (int64_t)g->hot.P * g->hot.Kp : 0,
                                    g->C == 1 ? 0 : 3, g->gather_est, g->n_walk_groups, g->layout,
                                    g->hot_cover_ppm, g->C > 1 ? (g->code == pr::kCodeC20 || g->code == pr::kCodeC20P ? 20 : g->code == pr::kCodeC24 || g->code == pr::kCodeC24P ? 24 : 32) : 0};
  for (int32_t i = 0; i < n_info && i < PR_INFO_COUNT; ++i) info[i] = v[i];
  return PR_OK;
}

int pr_graph_export_csr(const pr_graph *g, int64_t *row_ptr, int32_t *col_idx, int32_t *out_deg,
                        uint8_t *vflags) {
  if (!g) return fail(PR_ERR_INVALID, "NULL graph");
  if (!g->has_canonical) return fail(PR_ERR_STATE, "canonical CSR was dropped (PR_NO_CANONICAL)");
  DeviceGuard dg(g->device);
  hipStream_t s = g->stream;
  if (row_ptr)
    PR_HIP(hipMemcpyAsync(row_ptr, g->canon_rowptr.p, sizeof(int64_t) * ((size_t)g->V + 1), hipMemcpyDeviceToHost, s));
  if (col_idx && g->E_dedup > 0)
    PR_HIP(hipMemcpyAsync(col_idx, g->canon_col.p, sizeof(int32_t) * g->E_dedup, hipMemcpyDeviceToHost, s));
  if (out_deg && g->V > 0)
    PR_HIP(hipMemcpyAsync(out_deg, g->canon_deg.p, sizeof(int32_t) * g->V, hipMemcpyDeviceToHost, s));
  if (vflags && g->V > 0)
    PR_HIP(hipMemcpyAsync(vflags, g->canon_vflags.p, (size_t)g->V, hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  return PR_OK;
}

int pr_reset(pr_graph *g, double teleport, double damping, const double *init_ranks) {
  if (!g) return fail(PR_ERR_INVALID, "NULL graph");
  DeviceGuard dg(g->device);
  g->teleport = teleport;
  g->damping = damping;
  return pr::iter_reset(g, init_ranks);
}

int pr_step(pr_graph *g, int32_t iterations) {
  if (!g || iterations < 0) return fail(PR_ERR_INVALID, "bad argument");
  DeviceGuard dg(g->device);
  return pr::iter_step(g, iterations);
}

int pr_sync(pr_graph *g) {
  if (!g) return fail(PR_ERR_INVALID, "NULL graph");
  DeviceGuard dg(g->device);
  PR_TRY(pr::join_exchange(g));  // an overlapped exchange still on xstream
  PR_HIP(hipStreamSynchronize(g->stream));
  return PR_OK;
}

int pr_get_ranks(pr_graph *g, double *ranks_out) {
  if (!g || !ranks_out) return fail(PR_ERR_INVALID, "NULL argument");
  if (!g->ready) return fail(PR_ERR_STATE, "pr_get_ranks before pr_reset");
  DeviceGuard dg(g->device);
  std::vector<double> loc((size_t)g->n_rows);
  if (g->n_rows > 0)
    PR_HIP(hipMemcpyAsync(loc.data(), g->r.p, sizeof(double) * g->n_rows, hipMemcpyDeviceToHost, g->stream));
  PR_HIP(hipStreamSynchronize(g->stream));
  for (int64_t L = 0; L < g->n_rows; ++L)
    if (g->orig_of_local[L] >= 0) ranks_out[g->orig_of_local[L]] = loc[L];
  return PR_OK;
}

int pr_set_timing(pr_graph *g, int32_t enable) {
  if (!g) return fail(PR_ERR_INVALID, "NULL graph");
  g->timing = enable != 0;
  return PR_OK;
}

int pr_set_option(pr_graph *g, int32_t option, int64_t value) {
  if (!g) return fail(PR_ERR_INVALID, "NULL graph");
  DeviceGuard dg(g->device);
  if (option == PR_OPT_HOT_RESERVE) {
    if (value < 0 || value > 3) return fail(PR_ERR_INVALID, "PR_OPT_HOT_RESERVE: 0..3 CUs per XCD");
    if (g->C > 1) PR_TRY(pr::set_hot_reserve(g, (int)value));
    return PR_OK;
  }
  if (option == PR_OPT_XCHG_IPC_BLIT) {
    if (value != 0 && value != 1) return fail(PR_ERR_INVALID, "PR_OPT_XCHG_IPC_BLIT: 0 (copy engines) or 1 (blit kernel)");
    PR_TRY(pr::join_exchange(g));  // a pending exchange finishes with the old mover
    g->x_ipc_blit = value == 1;
    return PR_OK;
  }
  if (option == PR_OPT_XCHG_IPC) {
    if (value < 0 || value > 2)
      return fail(PR_ERR_INVALID, "PR_OPT_XCHG_IPC: 0 (RCCL), 1 (IPC copy engines) or 2 (IPC, per-chunk publication)");
    return pr::set_exchange_ipc(g, (int)value);
  }
  if (option != PR_OPT_XCHG_CHUNKS) return fail(PR_ERR_INVALID, "unknown option");
  PR_TRY(pr::join_exchange(g));  // a pending overlapped exchange finishes under the old setting
  g->x_chunked = value != 0 && g->n_xc > 1;
  if (g->comm && g->comm_size > 1) PR_TRY(pr::verify_exchange(g));  // collective: ranks must agree
  return PR_OK;
}

int pr_get_stats(pr_graph *g, double *stats, int32_t n_stats) {
  if (!g || !stats) return fail(PR_ERR_INVALID, "NULL argument");
  DeviceGuard dg(g->device);
  PR_TRY(pr::join_exchange(g));
  PR_HIP(hipStreamSynchronize(g->stream));
  auto mean_ms = [&](const std::vector<std::pair<int, int>> &ev, double *out) -> int {
    double acc = 0.0;
    for (auto &pr_ : ev) {
      float ms = 0.f;
      PR_HIP(hipEventElapsedTime(&ms, g->ev_pool[pr_.first], g->ev_pool[pr_.second]));
      acc += ms;
    }
    *out = ev.empty() ? 0.0 : acc / (double)ev.size();
    return PR_OK;
  };
  double v[PR_STAT_COUNT] = {0};
  v[PR_STAT_ITERS] = (double)g->iters_done;
  if (g->ready) {
    PR_TRY(pr::read_slots(g, g->cur, &v[PR_STAT_LAST_DC], &v[PR_STAT_LAST_L1]));
    // the dc *used* by the last iteration lives in the previous buffer
    if (g->iters_done > 0) {
      double dc_prev = 0, l1_prev = 0;
      PR_TRY(pr::read_slots(g, g->cur ^ 1, &dc_prev, &l1_prev));
      v[PR_STAT_LAST_DC] = dc_prev;
    } else {
      v[PR_STAT_LAST_L1] = 0.0;
    }
  }
  PR_TRY(mean_ms(g->spmv_ev, &v[PR_STAT_SPMV_MS_MEAN]));  // per interval: scaled to per pass below
  if (g->spmv_passes > 0) v[PR_STAT_SPMV_MS_MEAN] *= (double)g->spmv_ev.size() / (double)g->spmv_passes;
  v[PR_STAT_SPMV_LAUNCHES] = (double)g->spmv_passes;
  // an iteration ends when both its kernels (compute stream) and its exchange (xstream, P > 1)
  // are done: per iteration the later of the two ends, measured from the iteration's start
  // (the transfer runs on xstream since round 2)
  if (g->xchg_ev.size() == g->iter_ev.size() && !g->xchg_ev.empty()) {
    double acc = 0.0;
    for (size_t i = 0; i < g->iter_ev.size(); ++i) {
      float a = 0.f, b = 0.f;
      PR_HIP(hipEventElapsedTime(&a, g->ev_pool[g->iter_ev[i].first], g->ev_pool[g->iter_ev[i].second]));
      PR_HIP(hipEventElapsedTime(&b, g->ev_pool[g->iter_ev[i].first], g->ev_pool[g->xchg_ev[i].second]));
      acc += a > b ? a : b;
    }
    v[PR_STAT_ITER_MS_MEAN] = acc / (double)g->iter_ev.size();
  } else {  // per interval: scaled to per iteration (one part: one interval per pr_step call)
    PR_TRY(mean_ms(g->iter_ev, &v[PR_STAT_ITER_MS_MEAN]));
    if (g->iter_timed > 0) v[PR_STAT_ITER_MS_MEAN] *= (double)g->iter_ev.size() / (double)g->iter_timed;
  }
  v[PR_STAT_BUILD_MS] = g->build_ms;
  PR_TRY(mean_ms(g->xchg_ev, &v[PR_STAT_EXCHANGE_MS_MEAN]));
  for (int32_t i = 0; i < n_stats && i < PR_STAT_COUNT; ++i) stats[i] = v[i];
  return PR_OK;
}

int pr_run(pr_graph *g, int32_t iterations, double teleport, double damping,
           const double *init_ranks, double *ranks_out, pr_iter_cb cb, uint32_t cb_flags,
           void *user) {
  if (!g || iterations < 0) return fail(PR_ERR_INVALID, "bad argument");
  DeviceGuard dg(g->device);
  g->teleport = teleport;
  g->damping = damping;
  PR_TRY(pr::iter_reset(g, init_ranks));
  std::vector<double> cb_ranks;
  if (cb && (cb_flags & PR_CB_RANKS)) {
    cb_ranks.assign((size_t)g->V, 0.0);
    if (init_ranks) std::memcpy(cb_ranks.data(), init_ranks, sizeof(double) * g->V);
  }
  for (int32_t it = 0; it < iterations; ++it) {
    if (!cb) {
      PR_TRY(pr::iter_step(g, iterations));
      break;
    }
    auto t0 = std::chrono::steady_clock::now();
    double dc = 0, l1 = 0, dummy = 0;
    PR_TRY(pr::read_slots(g, g->cur, &dc, &dummy));  // dc used by this iteration
    PR_TRY(pr::iter_step(g, 1));
    PR_HIP(hipStreamSynchronize(g->stream));
    PR_TRY(pr::read_slots(g, g->cur, &dummy, &l1));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const double *rp = nullptr;
    if (cb_flags & PR_CB_RANKS) {
      PR_TRY(pr_get_ranks(g, cb_ranks.data()));
      rp = cb_ranks.data();
    }
    cb(it, rp, dc, l1, ms, user);
  }
  PR_HIP(hipStreamSynchronize(g->stream));
  if (ranks_out) PR_TRY(pr_get_ranks(g, ranks_out));
  return PR_OK;
}

int pr_comm_unique_id(uint8_t *id_out) {
  if (!id_out) return fail(PR_ERR_INVALID, "NULL argument");
  static_assert(sizeof(ncclUniqueId) == PR_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  ncclResult_t rc = ncclGetUniqueId(&id);
  if (rc != ncclSuccess) return fail(PR_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(rc));
  std::memcpy(id_out, &id, sizeof(id));
  return PR_OK;
}

int pr_graph_attach_comm(pr_graph *g, int32_t rank, int32_t n_ranks, const uint8_t *id) {
  if (!g || !id) return fail(PR_ERR_INVALID, "NULL argument");
  if (n_ranks != g->nparts || rank != g->part)
    return fail(PR_ERR_INVALID, "rank/n_ranks must equal the graph's part/n_parts");
  if (g->comm) return fail(PR_ERR_STATE, "communicator already attached");
  DeviceGuard dg(g->device);
  if (!g->comm_scratch.p) {  // the IPC set-up's records and the exchange agreement records
    const size_t xrec = sizeof(int64_t) * (size_t)pr::xrec_width(n_ranks) * (size_t)(n_ranks + 1);
    PR_TRY(g->comm_scratch.alloc(std::max(pr::kCommScratchBytes, xrec)));
  }
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclResult_t rc = ncclCommInitRank(&g->comm, n_ranks, uid, rank);
  if (rc != ncclSuccess) {
    g->comm = nullptr;
    return fail(PR_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(rc));
  }
  g->comm_rank = rank;
  g->comm_size = n_ranks;
  if (n_ranks > 1) {
    const int rv = pr::verify_exchange(g);
    if (rv != PR_OK) {
      ncclCommDestroy(g->comm);
      g->comm = nullptr;
      return rv;
    }
  }
  return PR_OK;
}

static int check_group(pr_graph *const *parts, int32_t n) {
  if (!parts || n < 1) return fail(PR_ERR_INVALID, "bad group");
  for (int32_t p = 0; p < n; ++p) {
    const pr_graph *g = parts[p];
    if (!g) return fail(PR_ERR_INVALID, "NULL part in group");
    if (g->nparts != n || g->part != p) return fail(PR_ERR_INVALID, "parts[p] must be part p of n_parts");
    if (g->V != parts[0]->V || g->S_pad != parts[0]->S_pad) return fail(PR_ERR_INVALID, "parts of different graphs");
    if (g->comm) return fail(PR_ERR_STATE, "a part with an RCCL communicator cannot join a group");
    if (g->x_allgather != parts[0]->x_allgather) return fail(PR_ERR_INVALID, "parts built with different PR_BOPT_EXCHANGE");
  }
  return PR_OK;
}

int pr_group_reset(pr_graph *const *parts, int32_t n_parts, double teleport, double damping,
                   const double *init_ranks) {
  PR_TRY(check_group(parts, n_parts));
  for (int32_t p = 0; p < n_parts; ++p) {
    pr_graph *g = parts[p];
    PR_HIP(hipSetDevice(g->device));
    if (!g->xev) PR_HIP(hipEventCreateWithFlags(&g->xev, hipEventDisableTiming));
    for (int32_t q = 0; q < n_parts; ++q) {  // peer access for xGMI copies between GPUs
      if (parts[q]->device == g->device) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, g->device, parts[q]->device) == hipSuccess && can) {
        hipError_t e = hipDeviceEnablePeerAccess(parts[q]->device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) PR_HIP(e);
        (void)hipGetLastError();
      }
    }
    g->grouped = true;
    g->teleport = teleport;
    g->damping = damping;
    PR_TRY(pr::iter_reset(g, init_ranks));
  }
  PR_TRY(pr::group_exchange(parts, n_parts, 0));
  for (int32_t p = 0; p < n_parts; ++p) {
    PR_HIP(hipSetDevice(parts[p]->device));
    PR_TRY(pr::join_exchange(parts[p]));
    PR_HIP(hipStreamSynchronize(parts[p]->stream));
    parts[p]->xchg_ev.clear();  // the reset's exchange is not an iteration's
  }
  return PR_OK;
}

int pr_group_step(pr_graph *const *parts, int32_t n_parts, int32_t iterations) {
  PR_TRY(check_group(parts, n_parts));
  if (iterations < 0) return fail(PR_ERR_INVALID, "iterations < 0");
  for (int32_t p = 0; p < n_parts; ++p)
    if (!parts[p]->grouped || !parts[p]->ready) return fail(PR_ERR_STATE, "pr_group_step before pr_group_reset");
  std::vector<int> i0((size_t)n_parts, -1);
  for (int32_t it = 0; it < iterations; ++it) {
    for (int32_t p = 0; p < n_parts; ++p) {
      PR_HIP(hipSetDevice(parts[p]->device));
      if (parts[p]->timing) PR_TRY(pr::time_mark(parts[p], parts[p]->stream, &i0[p]));
      PR_TRY(pr::iter_compute(parts[p]));
    }
    PR_TRY(pr::group_exchange(parts, n_parts, parts[0]->cur));
    for (int32_t p = 0; p < n_parts; ++p) {  // per part: its kernels and its pack (the copies: xchg_ev)
      if (!parts[p]->timing) continue;
      PR_HIP(hipSetDevice(parts[p]->device));
      int i1 = -1;
      PR_TRY(pr::time_mark(parts[p], parts[p]->stream, &i1));
      parts[p]->iter_ev.push_back({i0[p], i1});
      ++parts[p]->iter_timed;
    }
  }
  return PR_OK;
}

int pr_group_sync(pr_graph *const *parts, int32_t n_parts) {
  PR_TRY(check_group(parts, n_parts));
  for (int32_t p = 0; p < n_parts; ++p) {
    PR_HIP(hipSetDevice(parts[p]->device));
    PR_TRY(pr::join_exchange(parts[p]));
    PR_HIP(hipStreamSynchronize(parts[p]->stream));
  }
  return PR_OK;
}

void pr_graph_destroy(pr_graph *g) {
  if (!g) return;
  DeviceGuard dg(g->device);
  if (g->ipc) {
    // IPC transport: the compute stream may hold a wait on a peer's copied[] event and
    // the transfer stream one on a peer's sent[] event; if that peer died they never fire.  Poll with
    // a deadline instead of an unbounded synchronize; on expiry the handle and its device memory are
    // leaked (freeing memory a wedged stream may still touch is worse), and the error says so.
    const bool idle = pr::stream_idle_within(g->stream, 30.0) && pr::stream_idle_within(g->xstream, 30.0);
    if (!idle) {
      pr::set_error("pr_graph_destroy: a stream did not drain within 30 s (a peer of the IPC exchange died?); "
                    "the handle is leaked");
      return;
    }
  }
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  if (g->xstream) (void)hipStreamSynchronize(g->xstream);
  pr::ipc_destroy(g);  // after the peers' last copies out of this part's send runs
  if (g->comm) (void)ncclCommDestroy(g->comm);
  for (hipEvent_t e : g->ev_pool) (void)hipEventDestroy(e);
  if (g->xev) (void)hipEventDestroy(g->xev);
  for (hipEvent_t e : g->x_ev) (void)hipEventDestroy(e);
  if (g->x_pack_ev) (void)hipEventDestroy(g->x_pack_ev);
  if (g->x_free_ev) (void)hipEventDestroy(g->x_free_ev);
  if (g->xstream) (void)hipStreamDestroy(g->xstream);
  g->ev_pool.clear();
  hipStream_t s = g->stream;
  g->stream = nullptr;
  delete g;  // DevBufs free their memory
  if (s) (void)hipStreamDestroy(s);
}

}  // extern "C"
