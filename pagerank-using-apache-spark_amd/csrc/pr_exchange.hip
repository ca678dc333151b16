// The exchange of the row-partitioned iteration: after its epilogue every part
// has fresh contributions c' = r'/d for its own rows (its slice) and the two slots {dangling
// partial, L1 partial}.  Part q only ever reads the contributions of the sources of its own
// in-links, so part p sends q exactly those positions of its slice (plus the two slots), packed
// densely, and q receives them straight into its gather space: q's gather space is its own slice
// followed by the runs it receives, peer by peer (the compacted layout; pr_graph.h).  q's
// column codes and hot-set table point into that space, so nothing is unpacked.
//
// Both ends derive the p -> q position list from the same edge list with the same rules, so they
// agree on every count without communicating (verify_exchange checks it once at attach time).
// At R-MAT s26 with 8 parts each rank receives 39 % of what an all-gather of whole slices moves.
//
// Transport: RCCL grouped ncclSend / ncclRecv (one process per GPU), or device-to-device copies
// (pr_group_*: one process, several parts).  PR_BOPT_EXCHANGE = 1 restores whole slices in an
// uncompacted gather space of P slices (A/B, diagnostics).
#include <cstdlib>
#include <cstring>

#include "pr_compact.h"
#include "pr_device.h"
#include "pr_graph.h"
#include "pr_xcheck.h"

namespace pr {
namespace {

// edge (u -> v) of the deduped, sorted edge keys: ((v << b) | u)
struct XPred {
  const uint64_t *k;
  const int32_t *rank_of;
  int b, P, part;
  uint64_t mask;
  bool send;  // send: u owned here, v elsewhere; receive: v owned here, u elsewhere
  __device__ bool operator()(int64_t i) const {
    const uint64_t key = k[i];
    const int pu = rank_of[(int32_t)(key & mask)] % P, pv = rank_of[(int32_t)(key >> b)] % P;
    return send ? (pu == part && pv != part) : (pv == part && pu != part);
  }
};
// (peer << 32) | position of u inside its owner's slice
struct XKey {
  const uint64_t *k;
  const int32_t *rank_of, *gpos;
  int b, P;
  uint64_t mask;
  int64_t S_pad;
  bool send;
  __device__ uint64_t operator()(int64_t i) const {
    const uint64_t key = k[i];
    const int32_t u = (int32_t)(key & mask), v = (int32_t)(key >> b);
    const int64_t gu = gpos[u];
    const int pu = rank_of[u] % P, pv = rank_of[v] % P;
    const uint64_t peer = (uint64_t)(send ? pv : pu);
    return (peer << 32) | (uint64_t)(gu - (int64_t)pu * S_pad);
  }
};
struct XUnique {
  const uint64_t *k;
  __device__ bool operator()(int64_t i) const { return i == 0 || k[i] != k[i - 1]; }
};
struct XIdent {
  const uint64_t *k;
  __device__ uint64_t operator()(int64_t i) const { return k[i]; }
};

// Sorted unique (peer, pos) keys -> positions grouped by peer (peer order), each peer's run
// followed by its two slot positions: out[k + 2 * peer_ordinal] for key k.  Send lists hold
// positions in this part's slice, receive lists global positions (peer * S_pad + pos).
__global__ void k_xlist(int64_t n, const uint64_t *__restrict__ keys, const int64_t *__restrict__ first,
                        int P, int self, int64_t S_pad, bool send, uint32_t *__restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(keys[i] >> 32);
    const int ord = q - (q > self ? 1 : 0);
    const int64_t base = send ? 0 : (int64_t)q * S_pad;  // send: own slice; receive: global position
    out[i + 2 * ord] = (uint32_t)(base + (int64_t)(keys[i] & 0xFFFFFFFFull));
  }
  if (blockIdx.x == 0 && threadIdx.x < P) {  // the slots close every peer's run
    const int q = threadIdx.x;
    if (q != self) {
      const int ord = q - (q > self ? 1 : 0);
      const int64_t base = send ? 0 : (int64_t)q * S_pad;
      const int64_t end = first[q + 1] + 2 * ord;  // run end of peer q
      out[end] = (uint32_t)(base + S_pad - 2);
      out[end + 1] = (uint32_t)(base + S_pad - 1);
    }
  }
}

// first[q] = first key of peer >= q (keys sorted by peer)
__global__ void k_peer_bounds(const uint64_t *__restrict__ keys, int64_t m, int P, int64_t *__restrict__ first) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= m; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t qc = (i < m) ? (int64_t)(keys[i] >> 32) : P;
    const int64_t qp = (i > 0) ? (int64_t)(keys[i - 1] >> 32) : -1;
    for (int64_t q = qp + 1; q <= qc; ++q) first[q] = i;
  }
}

// Four positions per thread (one 16-byte load of the list): the gather/scatter side is the
// cost, so keep every lane's four loads in flight at once.
__global__ __launch_bounds__(256) void k_pack(int64_t n, const uint32_t *__restrict__ pos,
                                              const double *__restrict__ cbuf, double *__restrict__ out) {
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 p = reinterpret_cast<const uint4 *>(pos)[i];
    const double a = cbuf[p.x], b = cbuf[p.y], c = cbuf[p.z], d = cbuf[p.w];
    reinterpret_cast<double2 *>(out)[2 * i] = make_double2(a, b);
    reinterpret_cast<double2 *>(out)[2 * i + 1] = make_double2(c, d);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    out[i] = cbuf[pos[i]];
  }
}

// Fused pack (pr_graph.h x_fused): pmask[row] bit q = peer q reads the row (its send run lists
// it); sbase[blk * P + q] = entries of peer q's run (slots excluded) at rows < 64 blk, so the
// epilogue stores lane L's c' at run q + sbase + (lanes below L with bit q).  One launch per peer:
// a peer's positions are unique, so the byte updates of one launch never collide.
__global__ void k_pmask(int64_t n, const uint32_t *__restrict__ pos, uint8_t bit, uint8_t *__restrict__ pmask) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    pmask[pos[i]] |= bit;
}
__global__ void k_sbase(int64_t nblk, int P, int self, const uint32_t *__restrict__ send,
                        const int64_t *__restrict__ soff, int32_t *__restrict__ sbase) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nblk * P; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = t / P;
    const int q = (int)(t - blk * P);
    int64_t r = 0;
    if (q != self) {
      const int64_t b = soff[q], e = soff[q + 1] - 2;  // the run without its two slots
      const uint32_t target = (uint32_t)(blk * kWave);
      int64_t lo = b, hi = e;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (send[mid] < target) lo = mid + 1;
        else hi = mid;
      }
      r = lo - b;
    }
    sbase[t] = (int32_t)r;
  }
}

// Compacted gather space: global position -> this part's position (-1: never read here).
__global__ void k_cmap_own(int64_t S_pad, int part, int32_t *__restrict__ cmap) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < S_pad; j += (int64_t)gridDim.x * blockDim.x)
    cmap[(int64_t)part * S_pad + j] = (int32_t)j;
}
__global__ void k_cmap_recv(int64_t n, const uint32_t *__restrict__ recv, int64_t S_pad, int32_t *__restrict__ cmap) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    cmap[recv[k]] = (int32_t)(S_pad + k);
}

// Chunk starts of every peer's run (overlapped exchange): out[q * (nc + 1) + c] = index within
// peer q's run [off[q], off[q + 1]) of its first position at or past the class regions of hot
// phases < c (slice row 8 c Q_pad); out[q * (nc + 1) + nc] = the run length (the two slots, the
// largest positions of a run, fall in the last chunk).  Receive lists hold global positions.
__global__ void k_chunk_bounds(const uint32_t *__restrict__ list, const int64_t *__restrict__ off, int P, int self,
                               int nc, int64_t row_stride, int64_t S_pad, bool send, int64_t *__restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= P * (nc + 1)) return;
  const int q = t / (nc + 1), c = t - q * (nc + 1);
  const int64_t b = off[q], e = off[q + 1];
  int64_t r = 0;
  if (q != self) {
    if (c == nc) {
      r = e - b;
    } else if (c > 0) {
      const int64_t base = send ? 0 : (int64_t)q * S_pad, target = (int64_t)c * row_stride;
      int64_t lo = b, hi = e;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)list[mid] - base < target) lo = mid + 1;
        else hi = mid;
      }
      r = lo - b;
    }
  }
  out[t] = r;
}

int chunk_bounds(pr_graph *g, const uint32_t *list, const std::vector<int64_t> &off, bool send,
                 std::vector<int64_t> *out) {
  const int P = g->nparts, nc = g->n_xc;
  hipStream_t s = g->stream;
  DevBuf doff, dout;
  PR_TRY(doff.alloc(sizeof(int64_t) * (P + 1)));
  PR_TRY(dout.alloc(sizeof(int64_t) * P * (nc + 1)));
  PR_HIP(hipMemcpyAsync(doff.p, off.data(), sizeof(int64_t) * (P + 1), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_chunk_bounds, dim3((P * (nc + 1) + 255) / 256), dim3(256), 0, s, list, doff.as<int64_t>(), P,
                     g->part, nc, (int64_t)kXcds * g->Q_pad, g->S_pad, send, dout.as<int64_t>());
  PR_HIP(hipGetLastError());
  out->assign((size_t)P * (nc + 1), 0);
  PR_HIP(hipMemcpyAsync(out->data(), dout.p, sizeof(int64_t) * P * (nc + 1), hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  return PR_OK;
}

// One direction's list (send or receive) of part g->part.
int build_list(pr_graph *g, const uint64_t *ukeys, int64_t m, int b, uint64_t mask, const int32_t *rank_of,
               const int32_t *gpos, bool send, DevBuf *list, std::vector<int64_t> *off) {
  hipStream_t s = g->stream;
  const int P = g->nparts, self = g->part;
  const XPred pred{ukeys, rank_of, b, P, self, mask, send};
  int64_t n = 0;
  PR_TRY(compact_index(m, pred, XIdent{ukeys}, (uint64_t *)nullptr, &n, s));  // count only
  DevBuf keys, tmp, uk, first;
  PR_TRY(keys.alloc(sizeof(uint64_t) * (n > 0 ? n : 1)));
  PR_TRY(tmp.alloc(sizeof(uint64_t) * (n > 0 ? n : 1)));
  int64_t n2 = 0;
  PR_TRY(compact_index(m, pred, XKey{ukeys, rank_of, gpos, b, P, mask, g->S_pad, send}, keys.as<uint64_t>(), &n2, s));
  PR_TRY(radix_sort_u64(keys.as<uint64_t>(), tmp.as<uint64_t>(), n2, 0, 32 + bits_for((uint64_t)P), s));
  int64_t nu = 0;
  PR_TRY(compact_index(n2, XUnique{keys.as<uint64_t>()}, XIdent{keys.as<uint64_t>()}, tmp.as<uint64_t>(), &nu, s));
  PR_TRY(first.alloc(sizeof(int64_t) * (P + 1)));
  hipLaunchKernelGGL(k_peer_bounds, dim3(grid_for(nu + 1, 256, 65536)), dim3(256), 0, s, tmp.as<uint64_t>(), nu, P,
                     first.as<int64_t>());
  std::vector<int64_t> hf(P + 1);
  PR_HIP(hipMemcpyAsync(hf.data(), first.p, sizeof(int64_t) * (P + 1), hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  const int64_t total = nu + 2 * (P - 1);
  PR_TRY(list->alloc(sizeof(uint32_t) * (size_t)total));
  hipLaunchKernelGGL(k_xlist, dim3(grid_for(nu > 0 ? nu : 1, 256, 65536)), dim3(256), 0, s, nu, tmp.as<uint64_t>(),
                     first.as<int64_t>(), P, self, g->S_pad, send, list->as<uint32_t>());
  PR_HIP(hipGetLastError());
  PR_HIP(hipStreamSynchronize(s));
  off->assign(P + 1, 0);  // offsets of every peer's run (self: empty)
  for (int q = 0; q < P; ++q) (*off)[q + 1] = (*off)[q] + (q == self ? 0 : (hf[q + 1] - hf[q]) + 2);
  return PR_OK;
}

int build_fused_pack(pr_graph *g) {
  const int P = g->nparts;
  hipStream_t s = g->stream;
  const int64_t nblk = (g->n_rows + kWave - 1) / kWave;  // the epilogue's 64-row blocks (g->nblk)
  const int64_t rows = nblk * kWave;
  DevBuf doff;
  PR_TRY(doff.alloc(sizeof(int64_t) * (P + 1)));
  PR_TRY(g->x_pmask.alloc((size_t)rows));
  PR_TRY(g->x_sbase.alloc(sizeof(int32_t) * (size_t)(nblk * P)));
  PR_HIP(hipMemcpyAsync(doff.p, g->x_soff.data(), sizeof(int64_t) * (P + 1), hipMemcpyHostToDevice, s));
  PR_HIP(hipMemsetAsync(g->x_pmask.p, 0, (size_t)rows, s));
  for (int q = 0; q < P; ++q) {
    const int64_t n = g->x_soff[q + 1] - 2 - g->x_soff[q];
    if (q == g->part || n <= 0) continue;
    hipLaunchKernelGGL(k_pmask, dim3(grid_for(n, 256, 65536)), dim3(256), 0, s, n,
                       g->x_send.as<uint32_t>() + g->x_soff[q], (uint8_t)(1u << q), g->x_pmask.as<uint8_t>());
  }
  hipLaunchKernelGGL(k_sbase, dim3(grid_for(nblk * P, 256, 65536)), dim3(256), 0, s, nblk, P, g->part,
                     g->x_send.as<uint32_t>(), doff.as<int64_t>(), g->x_sbase.as<int32_t>());
  PR_HIP(hipGetLastError());
  PR_HIP(hipStreamSynchronize(s));
  g->x_fused = true;
  return PR_OK;
}

}  // namespace

// doubles per send buffer, even so that the second buffer stays 16-byte aligned (k_pack)
int64_t send_stride(const pr_graph *g) {
  const int64_t n = g->x_soff[g->nparts];
  return (n + 1) & ~int64_t(1);
}

double *send_runs(const pr_graph *g, int buf) {
  return g->x_sbuf.as<double>() + (buf & 1) * send_stride(g);
}

int build_exchange(pr_graph *g, const uint64_t *ukeys, int64_t m, int b, uint64_t mask, const int32_t *rank_of,
                   const int32_t *gpos, DevBuf *cmap) {
  const int P = g->nparts, self = g->part;
  g->x_allgather = P > 1 && g->opts.allgather;
  g->slots.n = P;
  if (P <= 1 || g->x_allgather) {  // P slices side by side
    g->gsize = (int64_t)P * g->S_pad;
    g->own_off = (int64_t)self * g->S_pad;
    for (int q = 0; q < P; ++q) g->slots.pos[q] = (int32_t)((int64_t)q * g->S_pad + g->S_pad - 2);
    return PR_OK;
  }
  DevBuf recv;
  PR_TRY(build_list(g, ukeys, m, b, mask, rank_of, gpos, true, &g->x_send, &g->x_soff));
  PR_TRY(build_list(g, ukeys, m, b, mask, rank_of, gpos, false, &recv, &g->x_roff));
  const int64_t R = g->x_roff[P];
  g->gsize = g->S_pad + R;
  g->own_off = 0;
  for (int q = 0; q < P; ++q)
    g->slots.pos[q] = (int32_t)(q == self ? g->S_pad - 2 : g->S_pad + g->x_roff[q + 1] - 2);
  hipStream_t s = g->stream;
  const int64_t G = (int64_t)P * g->S_pad;
  PR_TRY(cmap->alloc(sizeof(int32_t) * (size_t)G));
  PR_HIP(hipMemsetAsync(cmap->p, 0xFF, sizeof(int32_t) * (size_t)G, s));
  hipLaunchKernelGGL(k_cmap_own, dim3(grid_for(g->S_pad, 256, 65536)), dim3(256), 0, s, g->S_pad, self,
                     cmap->as<int32_t>());
  if (R > 0)
    hipLaunchKernelGGL(k_cmap_recv, dim3(grid_for(R, 256, 65536)), dim3(256), 0, s, R, recv.as<uint32_t>(), g->S_pad,
                       cmap->as<int32_t>());
  PR_HIP(hipGetLastError());
  // two send buffers, one per gather-space buffer: in the group path a peer's copy out of the
  // runs of iteration k may still be pending when this part packs iteration k + 1
  PR_TRY(g->x_sbuf.alloc(sizeof(double) * 2 * (size_t)(send_stride(g) > 0 ? send_stride(g) : 1)));
  PR_HIP(hipStreamSynchronize(s));
  // chunk bounds of the overlapped exchange: one chunk per hot phase (whether the chunks travel
  // separately: x_chunked, PR_BOPT_XCHG_CHUNKS / pr_set_option(PR_OPT_XCHG_CHUNKS))
  g->n_xc = g->C > 1 ? std::max(1, g->C / kXcds) : 1;
  set_exchange_chunking(g);
  PR_TRY(chunk_bounds(g, g->x_send.as<uint32_t>(), g->x_soff, true, &g->x_sch));
  PR_TRY(chunk_bounds(g, recv.as<uint32_t>(), g->x_roff, false, &g->x_rch));
  PR_HIP(hipStreamCreateWithFlags(&g->xstream, hipStreamNonBlocking));
  g->x_ev.assign(g->n_xc, nullptr);
  for (auto &e : g->x_ev) PR_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  PR_HIP(hipEventCreateWithFlags(&g->x_pack_ev, hipEventDisableTiming));
  PR_HIP(hipEventCreateWithFlags(&g->x_free_ev, hipEventDisableTiming));
  // fused pack: the split epilogue writes the runs itself (P <= 8: the row mask is one byte)
  g->x_fused = false;
  if (g->opts.pack_fused && g->C > 1 && P <= kMaxPackParts && g->x_soff[P] > 0) PR_TRY(build_fused_pack(g));
  return PR_OK;
}

int exchange_pack(pr_graph *g, int buf) {
  const int64_t n = g->x_soff[g->nparts];
  if (n > 0)
    hipLaunchKernelGGL(k_pack, dim3(grid_for((n + 3) / 4, 256, 8192)), dim3(256), 0, g->stream, n, g->x_send.as<uint32_t>(),
                       g->cbuf[buf].as<double>(), send_runs(g, buf));
  PR_HIP(hipGetLastError());
  return PR_OK;
}

// After ncclCommInitRank: every rank publishes its exchange record (pr_xcheck.h) and checks every
// peer's against what it expects to receive, chunk by chunk; a mismatch fails loudly at attach
// time (or at pr_set_option) instead of desynchronising the send/receive pairs.
int verify_exchange(pr_graph *g) {
  const int P = g->nparts, nc = g->n_xc;
  const int W = xrec_width(P);
  std::vector<int64_t> mine(W, 0);
  if (!xrec_fill(g->V, g->S_pad, g->x_allgather, nc, g->x_chunked, P, g->x_soff.data(), g->x_sch.data(), mine.data()))
    return fail(PR_ERR_INVALID, "too many exchange chunks");
  // through the scratch allocated with the communicator (sized for this record), so no rank can fail
  // an allocation here and leave its peers waiting in the all-gather
  if (g->comm_scratch.bytes < sizeof(int64_t) * (size_t)W * (P + 1))
    return fail(PR_ERR_STATE, "communicator scratch too small for the exchange records");
  int64_t *d = static_cast<int64_t *>(g->comm_scratch.p);
  PR_HIP(hipMemcpyAsync(d, mine.data(), sizeof(int64_t) * W, hipMemcpyHostToDevice, g->stream));
  ncclResult_t rc = ncclAllGather(d, d + W, (size_t)W, ncclInt64, g->comm, g->stream);
  if (rc != ncclSuccess) return fail(PR_ERR_COMM, std::string("ncclAllGather: ") + ncclGetErrorString(rc));
  std::vector<int64_t> all((size_t)W * P);
  PR_HIP(hipMemcpyAsync(all.data(), d + W, sizeof(int64_t) * W * P, hipMemcpyDeviceToHost, g->stream));
  PR_HIP(hipStreamSynchronize(g->stream));
  const char *why = "";
  const int rv = xrec_check(all.data(), P, g->part, mine.data(), g->x_roff.data(), g->x_rch.data(), nc, &why);
  return rv == PR_OK ? PR_OK : fail(rv, why);
}

// One process per GPU (RCCL).  Whole slices: one in-place ncclAllGather on the compute stream.
// Runs: the pack runs on the compute stream; the n_xc chunks of every peer's run go out as
// grouped ncclSend / ncclRecv on xstream, x_ev[c] after chunk c (the next iteration's hot phase c
// waits for it: iter_compute).  ev_a / ev_b (may be null): timing events around the transfer.
int exchange(pr_graph *g, int buf, hipEvent_t ev_a, hipEvent_t ev_b) {
  if (g->nparts <= 1) return PR_OK;
  if (!g->comm) return fail(PR_ERR_STATE, "graph part has no communicator (pr_graph_attach_comm)");
  double *base = g->cbuf[buf].as<double>();
  if (g->x_allgather) {  // whole slices, in place
    if (ev_a) PR_HIP(hipEventRecord(ev_a, g->stream));
    ncclResult_t rc = ncclAllGather(base + (int64_t)g->part * g->S_pad, base, (size_t)g->S_pad, ncclDouble, g->comm,
                                    g->stream);
    if (rc != ncclSuccess) return fail(PR_ERR_COMM, std::string("ncclAllGather: ") + ncclGetErrorString(rc));
    if (ev_b) PR_HIP(hipEventRecord(ev_b, g->stream));
    return PR_OK;
  }
  if (g->x_ipc) return exchange_ipc(g, buf, ev_a, ev_b);  // copy engines out of the peers' runs
  if (g->x_packed != buf) PR_TRY(exchange_pack(g, buf));  // else the epilogue wrote the runs
  g->x_packed = -1;
  PR_HIP(hipEventRecord(g->x_pack_ev, g->stream));
  PR_HIP(hipStreamWaitEvent(g->xstream, g->x_pack_ev, 0));
  if (ev_a) PR_HIP(hipEventRecord(ev_a, g->xstream));
  const int nc = g->n_xc, steps = g->x_chunked ? nc : 1;
  const double *sruns = send_runs(g, buf);
  for (int c = 0; c < steps; ++c) {
    const int lo = g->x_chunked ? c : 0, hi = g->x_chunked ? c + 1 : nc;  // unchunked: whole runs
    ncclResult_t rc = ncclGroupStart();
    for (int q = 0; q < g->nparts && rc == ncclSuccess; ++q) {
      if (q == g->part) continue;
      const int64_t s0 = g->x_sch[(size_t)q * (nc + 1) + lo], s1 = g->x_sch[(size_t)q * (nc + 1) + hi];
      const int64_t r0 = g->x_rch[(size_t)q * (nc + 1) + lo], r1 = g->x_rch[(size_t)q * (nc + 1) + hi];
      // both ends derive the chunk sizes from the same positions: a zero-size pair is skipped on both
      if (s1 > s0) rc = ncclSend(sruns + g->x_soff[q] + s0, (size_t)(s1 - s0), ncclDouble, q, g->comm, g->xstream);
      if (rc == ncclSuccess && r1 > r0)
        rc = ncclRecv(base + g->S_pad + g->x_roff[q] + r0, (size_t)(r1 - r0), ncclDouble, q, g->comm, g->xstream);
    }
    const ncclResult_t rc2 = ncclGroupEnd();
    if (rc != ncclSuccess) return fail(PR_ERR_COMM, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(rc));
    if (rc2 != ncclSuccess) return fail(PR_ERR_COMM, std::string("ncclGroupEnd: ") + ncclGetErrorString(rc2));
    PR_HIP(hipEventRecord(g->x_ev[hi - 1], g->xstream));
  }
  if (ev_b) PR_HIP(hipEventRecord(ev_b, g->xstream));
  g->x_pending = true;
  return PR_OK;
}

// One process, several parts: the same packed runs, chunk by chunk, moved by device copies (peer
// copies over xGMI when the parts live on different GPUs) on the receiver's xstream after every
// part's pack (its own included: the copies overwrite gather space its previous iteration read).
// p's next pack goes to its other send buffer; the one after that is ordered behind q's copies:
// q's next iteration waits for them before its pack, and p waits for q's pack.
int group_exchange(pr_graph *const *parts, int n, int buf) {
  if (n <= 1) return PR_OK;
  const bool whole = parts[0]->x_allgather;
  for (int p = 0; p < n; ++p) {
    PR_HIP(hipSetDevice(parts[p]->device));
    if (!whole && parts[p]->x_packed != buf) PR_TRY(exchange_pack(parts[p], buf));
    parts[p]->x_packed = -1;
    PR_HIP(hipEventRecord(whole ? parts[p]->xev : parts[p]->x_pack_ev, parts[p]->stream));
  }
  for (int q = 0; q < n; ++q) {
    pr_graph *g = parts[q];
    PR_HIP(hipSetDevice(g->device));
    if (whole) {  // whole slices on the compute stream (the A/B reference)
      int ta = -1, tb = -1;
      for (int p = 0; p < n; ++p) {
        if (p == q) continue;
        PR_HIP(hipStreamWaitEvent(g->stream, parts[p]->xev, 0));
      }
      if (g->timing) PR_TRY(time_mark(g, g->stream, &ta));
      for (int p = 0; p < n; ++p) {
        if (p == q) continue;
        const int64_t off = (int64_t)p * g->S_pad;
        PR_HIP(hipMemcpyAsync(g->cbuf[buf].as<double>() + off, parts[p]->cbuf[buf].as<double>() + off,
                              sizeof(double) * g->S_pad, hipMemcpyDeviceToDevice, g->stream));
      }
      if (g->timing) {
        PR_TRY(time_mark(g, g->stream, &tb));
        g->xchg_ev.push_back({ta, tb});
      }
      continue;
    }
    for (int p = 0; p < n; ++p) PR_HIP(hipStreamWaitEvent(g->xstream, parts[p]->x_pack_ev, 0));
    int ta = -1, tb = -1;  // every pack done -> the last copy into this part
    if (g->timing) PR_TRY(time_mark(g, g->xstream, &ta));
    const int nc = g->n_xc, steps = g->x_chunked ? nc : 1;
    // copy engines (PR_BOPT_XCHG_SDMA): no CU is taken from the receiver's k_spmv_hot phases
    const hipMemcpyKind kind = g->opts.xchg_sdma ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
    for (int c = 0; c < steps; ++c) {
      const int lo = g->x_chunked ? c : 0, hi = g->x_chunked ? c + 1 : nc;  // unchunked: whole runs
      for (int p = 0; p < n; ++p) {
        if (p == q) continue;
        const pr_graph *src = parts[p];
        const int64_t r0 = g->x_rch[(size_t)p * (nc + 1) + lo], r1 = g->x_rch[(size_t)p * (nc + 1) + hi];
        const int64_t s0 = src->x_sch[(size_t)q * (nc + 1) + lo], s1 = src->x_sch[(size_t)q * (nc + 1) + hi];
        if (r1 - r0 != s1 - s0) return fail(PR_ERR_STATE, "exchange lists disagree");
        if (r1 > r0)
          PR_HIP(hipMemcpyAsync(g->cbuf[buf].as<double>() + g->S_pad + g->x_roff[p] + r0,
                                send_runs(src, buf) + src->x_soff[q] + s0, sizeof(double) * (r1 - r0), kind,
                                g->xstream));
      }
      PR_HIP(hipEventRecord(g->x_ev[hi - 1], g->xstream));
    }
    if (g->timing) {
      PR_TRY(time_mark(g, g->xstream, &tb));
      g->xchg_ev.push_back({ta, tb});
    }
    g->x_pending = true;
  }
  return PR_OK;
}

}  // namespace pr
