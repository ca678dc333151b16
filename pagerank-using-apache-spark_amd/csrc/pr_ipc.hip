// CU-free exchange for the RCCL path (PR_OPT_XCHG_IPC): one process per GPU on
// one node, every rank pulls the runs its in-links read straight out of its peers' send buffers
// with the copy engines, so no transfer kernel competes with k_spmv_hot for a CU.
//
// Replaces the same per-iteration re-shuffle as exchange() (Sparky.java:192's join of the links
// with the ranks), with the same runs, chunks and gather-space positions; only the transport and
// its completion signals differ:
//   memory   every rank's double-buffered send runs (x_sbuf) are mapped into every peer
//            (hipIpcGetMemHandle / hipIpcOpenMemHandle); a receiver copies run q -> its gather space
//            with hipMemcpyDeviceToDeviceNoCU on a copy stream of its own per peer (the peers' runs
//            move at once, over their own links), chunk by chunk; the transfer stream (xstream)
//            joins every peer's chunk c before it records x_ev[c], as the RCCL exchange does.
//   device   interprocess events per buffer b and rank: `sent[b][c]` per exchange chunk c
//            (recorded on the owner's compute stream once chunk c of the runs of b is written: with
//            PR_OPT_XCHG_IPC = 2 right after the epilogue chunk that wrote it, otherwise all at the
//            end of the pass -- fused epilogue + k_finalize, or k_pack) and `copied[b]` (recorded
//            on the owner's xstream after its copies out of every peer's runs of b).  A receiver's
//            copy stream waits for a peer's sent[b][c] before copying chunk c (whole runs: the last
//            chunk's record, which implies the others); an owner's compute stream waits for every
//            peer's copied[b] of the previous exchange of b before it writes the runs of b again
//            (the reuse hazard of the double buffer).
//   host     a wait on an interprocess event binds to the latest record *enqueued so far*, so the
//            waiter's host must not enqueue it before the owner's host has enqueued the record it
//            means.  Every rank publishes, in a small shared-memory page of its own, how many
//            sent[b] / copied[b] records it has enqueued; a waiter spins on its host until the
//            owner's count reaches the exchange it needs, then enqueues the stream wait.  No device
//            work ever waits for a record that is not already enqueued, and the hosts stay at most
//            one exchange apart per buffer, so a later record of the same event cannot be taken for
//            the one meant (its owner would first have had to pass a wait on this rank).  A host
//            spin that exceeds kSpinLimit fails with PR_ERR_COMM instead of hanging.
//   events   the HIP runtime's interprocess events take at most 32 records each (their
//            shared-memory ring of signals; measured: the 33rd record's wait fails with "invalid
//            argument" and the event stays broken, profiles/r05/ipc_events/), so every event here is
//            recorded at most kRecordsPerEvent times and then replaced by a fresh one: its owner
//            writes the new handle into one of three slots per event of its shared-memory page,
//            stamped with the first exchange it serves, before it publishes that exchange; a waiter
//            that needs exchange k picks the newest slot whose range holds k and opens that handle
//            once.  An event is replaced three generations after it was last meant, long after
//            every wait on it (the hosts stay within one exchange per buffer of each other).
// Set-up and switching are collective (pr_set_option on every rank): the memory handle, run offsets
// and page names travel by ncclAllGather over the attached communicator, and every rank agrees on
// success with an ncclAllReduce before the mode is used.
#include <fcntl.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "pagerank_hip.h"
#include "pr_graph.h"
#include "pr_ipc_gens.h"
#include "pr_ipc_protocol.h"

namespace pr {

int exchange_pack(pr_graph *g, int buf);  // pr_exchange.hip
int64_t send_stride(const pr_graph *g);   // pr_exchange.hip

namespace {

constexpr double kSpinLimit = 120.0;  // seconds a host waits for a peer's record before failing
constexpr int kIpcMaxChunks = 16;     // sent events per buffer: one per exchange chunk (C / 8 <= 16)

constexpr int64_t kRecordsPerEvent = kIpcRecordsPerEvent;  // pr_ipc_gens.h (see "events" above)
constexpr int kGens = kIpcGens;                            // handle slots per event in the page
// A host may run at most 2 * kLeadEvery exchanges ahead of its own device (bound_lead).  An event
// generation is destroyed (own) or closed (opened) only when an exchange at least
// (kGens - 1) * kRecordsPerEvent past its last record or wait is enqueued, and the hosts stay within
// one exchange of each other; so with this bound every record and wait on it has executed on every
// device by then (without it, one long pr_step let a host destroy an event its device
// had not reached).
constexpr int64_t kLeadEvery = 8;
static_assert(2 * kLeadEvery + 2 < (kGens - 1) * kRecordsPerEvent, "the lead bound must stay below an event's reuse");

// one generation of one event: the exchanges [first_k, first_k + kRecordsPerEvent) it serves
struct IpcSlot {
  std::atomic<int64_t> id;       // generation id (0: empty), stored last (release)
  std::atomic<int64_t> first_k;
  hipIpcEventHandle_t h;
};

// one rank's shared-memory page: how many sent[b] / copied[b] records it has enqueued, and the
// handles of its events, per (kind, buffer, chunk) three generations
struct alignas(64) IpcCounters {
  std::atomic<int64_t> sent[2];
  std::atomic<int64_t> copied[2];
  IpcSlot slot[2][2][kIpcMaxChunks][kGens];  // [kind][b][c][generation % kGens]
};
static_assert(std::atomic<int64_t>::is_always_lock_free, "cross-process counters must be lock-free");

// what every rank publishes at set-up (ncclAllGather of bytes)
struct IpcRecord {
  hipIpcMemHandle_t mem;         // its x_sbuf
  char page[64];                 // its counter page (shm_open name)
  int64_t stride;                // doubles per send buffer (send_stride)
  int64_t soff[kMaxParts + 1];   // its send-run offsets
  int32_t ok;                    // its local set-up succeeded
  int32_t pad;
};

}  // namespace

struct HipIpcOps;

struct IpcState {
  int P = 0, self = 0;
  char page[64] = {0};
  IpcCounters *mine = nullptr;
  std::vector<IpcCounters *> peer;    // mapped counter pages (nullptr: self / not opened)
  std::vector<void *> peer_sbuf;      // mapped send buffers
  std::vector<int64_t> peer_stride;   // doubles per peer send buffer
  std::vector<int64_t> peer_soff_me;  // start of the peer's run for this rank
  // own events per (kind, b, c) and generation slot, with the slot's id / first exchange; the
  // current slot per (kind, b, c) (-1: none yet); the next generation id
  struct Own {
    hipEvent_t ev[kGens] = {nullptr, nullptr, nullptr};
    IpcGenOwner gen;  // pr_ipc_gens.h
  };
  std::vector<Own> own;  // [(kind * 2 + b) * nc + c]
  int64_t next_id = 1;
  int64_t epoch = 0;  // bumped at every enable: the exchange counts restart, so do the generations
  // the peers' events as opened here, per (q, kind, b, c) and slot: the generation id it holds
  struct Opened {
    hipEvent_t ev[kGens] = {nullptr, nullptr, nullptr};
    int64_t id[kGens] = {0, 0, 0};
  };
  std::vector<Opened> opened;  // [((q * 2 + kind) * 2 + b) * nc + c]
  // one copy stream per peer, so the runs of different peers move at once (on their own copy
  // engines / xGMI links), and per (peer, chunk) the event the transfer stream joins on
  std::vector<hipStream_t> cstream;
  std::vector<hipEvent_t> cev;  // [q * nc + c]
  int nc = 0;
  IpcProtocol<HipIpcOps> proto;  // the host-side ordering (pr_ipc_protocol.h)
  // the host's lead over its own device, bounded (bound_lead): a local event recorded on the compute
  // stream every kLeadEvery exchanges, alternating between two; the host waits for an event's
  // previous record before recording it again
  hipEvent_t lead_ev[2] = {nullptr, nullptr};
  bool lead_rec[2] = {false, false};
  int64_t n_exch = 0;
};

namespace {

void unmap_page(IpcCounters *c) {
  if (c) munmap(c, sizeof(IpcCounters));
}

IpcCounters *map_page(const char *name, bool create) {
  const int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) return nullptr;
  if (create && ftruncate(fd, sizeof(IpcCounters)) != 0) {
    close(fd);
    shm_unlink(name);
    return nullptr;
  }
  void *p = mmap(nullptr, sizeof(IpcCounters), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (create) shm_unlink(name);
    return nullptr;
  }
  IpcCounters *c = static_cast<IpcCounters *>(p);
  if (create) new (c) IpcCounters{};
  return c;
}

void free_state(IpcState *s) {
  if (!s) return;
  for (hipStream_t st : s->cstream)
    if (st) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
    }
  for (hipEvent_t e : s->cev)
    if (e) (void)hipEventDestroy(e);
  for (size_t q = 0; q < s->peer_sbuf.size(); ++q)
    if (s->peer_sbuf[q]) (void)hipIpcCloseMemHandle(s->peer_sbuf[q]);
  for (auto &o : s->opened)
    for (hipEvent_t e : o.ev)
      if (e) (void)hipEventDestroy(e);
  for (auto &o : s->own)
    for (hipEvent_t e : o.ev)
      if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : s->lead_ev)
    if (e) (void)hipEventDestroy(e);
  for (IpcCounters *c : s->peer) unmap_page(c);
  if (s->mine) {
    unmap_page(s->mine);
    if (s->page[0]) shm_unlink(s->page);  // normally unlinked at set-up already
  }
  (void)hipGetLastError();
  delete s;
}

// host wait until `c` reaches v (a peer's enqueued records); PR_ERR_COMM after kSpinLimit
int spin_until(const std::atomic<int64_t> &c, int64_t v, const char *what, int peer, double limit = kSpinLimit) {
  if (c.load(std::memory_order_acquire) >= v) return PR_OK;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; c.load(std::memory_order_acquire) < v; ++i) {
    if (i < 256) {
      std::this_thread::yield();
      continue;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    if ((i & 1023) == 0 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit)
      return fail(PR_ERR_COMM, std::string("IPC exchange: peer ") + std::to_string(peer) + " never enqueued its " +
                                   what + " record (did every rank make the same calls?)");
  }
  return PR_OK;
}

// every rank's streams are idle and every rank got here (tiny all-reduce on the compute stream,
// through the scratch allocated with the communicator: no allocation can fail here on one rank only)
int comm_barrier(pr_graph *g, int32_t *flag_inout) {
  if (!g->comm_scratch.p) return fail(PR_ERR_STATE, "no communicator scratch (pr_graph_attach_comm)");
  void *d = g->comm_scratch.p;
  PR_HIP(hipMemcpyAsync(d, flag_inout, sizeof(int32_t), hipMemcpyHostToDevice, g->stream));
  const ncclResult_t rc = ncclAllReduce(d, d, 1, ncclInt32, ncclMin, g->comm, g->stream);
  if (rc != ncclSuccess) return fail(PR_ERR_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(rc));
  PR_HIP(hipMemcpyAsync(flag_inout, d, sizeof(int32_t), hipMemcpyDeviceToHost, g->stream));
  PR_HIP(hipStreamSynchronize(g->stream));
  return PR_OK;
}

int quiesce(pr_graph *g) {
  PR_TRY(join_exchange(g));
  PR_HIP(hipStreamSynchronize(g->stream));
  if (g->xstream) PR_HIP(hipStreamSynchronize(g->xstream));
  return PR_OK;
}

// the IPC state of a set-up in progress: freed (events, mappings, the counter page and its name)
// on every return that does not hand it to the graph
struct IpcStateGuard {
  IpcState *s;
  ~IpcStateGuard() { free_state(s); }
  IpcState *release() {
    IpcState *t = s;
    s = nullptr;
    return t;
  }
};

static_assert(sizeof(IpcRecord) * (kMaxParts + 1) <= kCommScratchBytes, "IPC records exceed the comm scratch");

// collective: map every peer's send buffers, events and counter page.  Every local failure goes
// through rec.ok, so every rank reaches the record all-gather and the agreement all-reduce whatever
// failed where; only a failing collective itself returns early.
int ipc_setup(pr_graph *g) {
  const int P = g->nparts, self = g->part;
  if (!g->comm_scratch.p) return fail(PR_ERR_STATE, "no communicator scratch (pr_graph_attach_comm)");
  IpcState *s0 = new (std::nothrow) IpcState();
  IpcStateGuard guard{s0};
  std::string why;
  IpcRecord rec;
  std::memset(&rec, 0, sizeof(rec));
  rec.ok = 1;
  auto local = [&](bool cond, const char *what) {
    if (!cond && rec.ok) {
      rec.ok = 0;
      why = what;
    }
    (void)hipGetLastError();
  };
  local(s0 != nullptr, "host allocation failed");
  IpcState dummy;  // stands in for a failed allocation so the collectives below still run
  IpcState *s = s0 ? s0 : &dummy;
  s->P = P;
  s->self = self;
  s->proto.P = P;
  s->proto.self = self;
  s->peer.assign(P, nullptr);
  s->peer_sbuf.assign(P, nullptr);
  s->peer_stride.assign(P, 0);
  s->peer_soff_me.assign(P, 0);
  s->nc = g->n_xc;
  s->proto.nc = s->nc;
  s->own.assign(4 * (size_t)s->nc, IpcState::Own{});
  s->opened.assign(4 * (size_t)P * s->nc, IpcState::Opened{});
  s->cstream.assign(P, nullptr);
  s->cev.assign((size_t)P * s->nc, nullptr);
  local(s->nc >= 1 && s->nc <= kIpcMaxChunks, "exchange chunk count out of range");
  if (rec.ok) {
    std::snprintf(s->page, sizeof(s->page), "/pr_xipc_%d_%d_%llx", (int)getpid(), self,
                  (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count());
    s->mine = map_page(s->page, true);
    local(s->mine != nullptr, "shm_open of the counter page failed");
    std::memcpy(rec.page, s->page, sizeof(rec.page));
  }
  if (rec.ok) local(hipIpcGetMemHandle(&rec.mem, g->x_sbuf.p) == hipSuccess, "hipIpcGetMemHandle failed");
  rec.stride = send_stride(g);
  for (int q = 0; q <= P; ++q) rec.soff[q] = g->x_soff[q];
  // publish (the scratch holds P + 1 records: this rank's, then everyone's)
  std::vector<IpcRecord> all((size_t)P);
  {
    const size_t W = sizeof(IpcRecord);
    uint8_t *d = static_cast<uint8_t *>(g->comm_scratch.p);
    PR_HIP(hipMemcpyAsync(d, &rec, W, hipMemcpyHostToDevice, g->stream));
    const ncclResult_t rc = ncclAllGather(d, d + W, W, ncclUint8, g->comm, g->stream);
    if (rc != ncclSuccess) return fail(PR_ERR_COMM, std::string("ncclAllGather: ") + ncclGetErrorString(rc));
    PR_HIP(hipMemcpyAsync(all.data(), d + W, W * (size_t)P, hipMemcpyDeviceToHost, g->stream));
    PR_HIP(hipStreamSynchronize(g->stream));
  }
  int32_t ok = 1;
  for (int q = 0; q < P; ++q) ok &= all[q].ok;
  if (!rec.ok) ok = 0;
  // open the peers' resources (only if every rank's set-up succeeded)
  for (int q = 0; q < P && ok; ++q) {
    if (q == self) continue;
    const IpcRecord &r = all[q];
    char name[64];
    std::memcpy(name, r.page, sizeof(name));
    name[63] = 0;
    s->peer[q] = map_page(name, false);
    if (!s->peer[q]) {
      ok = 0;
      why = "shm_open of a peer's counter page failed";
      break;
    }
    if (hipIpcOpenMemHandle(&s->peer_sbuf[q], r.mem, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      (void)hipGetLastError();
      s->peer_sbuf[q] = nullptr;
      ok = 0;
      why = "hipIpcOpenMemHandle failed";
      break;
    }
    if (ok && hipStreamCreateWithFlags(&s->cstream[q], hipStreamNonBlocking) != hipSuccess) {
      (void)hipGetLastError();
      s->cstream[q] = nullptr;
      ok = 0;
      why = "hipStreamCreate failed";
    }
    for (int c = 0; c < s->nc && ok; ++c)
      if (hipEventCreateWithFlags(&s->cev[(size_t)q * s->nc + c], hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        ok = 0;
        why = "hipEventCreate failed";
      }
    s->peer_stride[q] = r.stride;
    s->peer_soff_me[q] = r.soff[self];
    // the peer's run for this rank must be exactly what this rank receives from it
    if (r.soff[self + 1] - r.soff[self] != g->x_roff[q + 1] - g->x_roff[q]) {
      ok = 0;
      why = "a peer's send run disagrees with the receive run";
    }
  }
  // every rank has opened every page: the names can go
  int32_t agreed = ok;
  const int rv = comm_barrier(g, &agreed);
  if (s->mine) {
    shm_unlink(s->page);
    s->page[0] = 0;
  }
  if (s == &dummy) {  // nothing of the stand-in may outlive this call (it holds no resources)
    guard.s = nullptr;
    return rv != PR_OK ? rv : fail(PR_ERR_OOM, "IPC exchange set-up failed on this rank: host allocation failed");
  }
  if (rv != PR_OK) return rv;
  if (!agreed)
    return fail(PR_ERR_COMM, "IPC exchange set-up failed on " + std::string(ok ? "a peer" : "this rank") +
                                 (why.empty() ? std::string() : ": " + why));
  g->ipc = guard.release();
  return PR_OK;
}

}  // namespace

int set_exchange_ipc(pr_graph *g, int mode) {
  const bool on = mode != 0;
  if (!on && !g->x_ipc) return PR_OK;  // off and staying off
  if (on) {
    if (!g->comm || g->comm_size <= 1) return fail(PR_ERR_STATE, "PR_OPT_XCHG_IPC needs an attached communicator (P > 1)");
    if (g->x_allgather) return fail(PR_ERR_STATE, "PR_OPT_XCHG_IPC needs the per-peer runs (PR_BOPT_EXCHANGE = 0)");
  }
  PR_TRY(quiesce(g));
  // every rank asks for the same mode: a receiver waits for per-chunk records only if
  // its peers make them (mode 2), so a 1 <-> 2 switch on some ranks only would bind a wait to a
  // stale generation or fail later; min over the ranks of mode and of -mode must agree
  int32_t lo = mode, nhi = -mode;
  PR_TRY(comm_barrier(g, &lo));
  PR_TRY(comm_barrier(g, &nhi));
  if (lo != -nhi) return fail(PR_ERR_STATE, "PR_OPT_XCHG_IPC: the ranks asked for different modes (" + std::to_string(lo) +
                                                " .. " + std::to_string(-nhi) + "); nothing changed");
  if (on == g->x_ipc) {
    g->x_ipc_early = mode == 2;  // per-chunk publication: every rank idle, every rank switches
    return PR_OK;
  }
  if (on && !g->ipc) PR_TRY(ipc_setup(g));
  // every rank idle (so no copy out of another's buffers is pending) before the mode changes
  int32_t one = 1;
  if (on) {
    IpcState *s = g->ipc;
    for (int b = 0; b < 2; ++b) {
      s->mine->sent[b].store(0, std::memory_order_release);
      s->mine->copied[b].store(0, std::memory_order_release);
    }
    s->proto.reset();
    ++s->epoch;  // the counts restart at 1: every event starts a fresh generation
  }
  PR_TRY(comm_barrier(g, &one));
  g->x_ipc = on;
  g->x_ipc_early = mode == 2;
  return PR_OK;
}

bool ipc_early(const pr_graph *g) { return g->x_ipc && g->x_ipc_early && g->ipc && g->x_fused && g->n_xc > 1; }

// The HIP side of the protocol's steps: interprocess events, the counter pages, the copy streams.
struct HipIpcOps {
  pr_graph *g;
  IpcState *s;
  hipEvent_t ev_a;  // timing: recorded on the transfer stream before the copies (may be null)

  int spin(int q, int kind, int b, int64_t v) {
    const std::atomic<int64_t> &c = kind == kIpcSent ? s->peer[q]->sent[b] : s->peer[q]->copied[b];
    return spin_until(c, v, kind == kIpcSent ? "sent" : "copied", q);
  }
  // peer q's event of (kind, b, c) that holds its record of exchange k: the newest page slot whose
  // range holds k (written before k was published), opened here once per generation
  int peer_event(int q, int kind, int b, int c, int64_t k, hipEvent_t *out) {
    IpcState::Opened &o = s->opened[(((size_t)q * 2 + kind) * 2 + b) * s->nc + c];
    int64_t ids[kGens], firsts[kGens];
    for (int i = 0; i < kGens; ++i) {
      const IpcSlot &sl = s->peer[q]->slot[kind][b][c][i];
      ids[i] = sl.id.load(std::memory_order_acquire);
      firsts[i] = sl.first_k.load(std::memory_order_acquire);
    }
    const int best = ipc_gen_pick(ids, firsts, k);
    const int64_t best_id = best >= 0 ? ids[best] : 0;
    if (best < 0)
      return pr::fail(PR_ERR_COMM, "IPC exchange: peer " + std::to_string(q) + " published exchange " + std::to_string(k) +
                                       " without an event for it");
    if (o.id[best] != best_id) {
      if (o.ev[best]) (void)hipEventDestroy(o.ev[best]);
      o.ev[best] = nullptr;
      o.id[best] = 0;
      hipIpcEventHandle_t h;
      std::memcpy(&h, &s->peer[q]->slot[kind][b][c][best].h, sizeof(h));
      PR_HIP(hipIpcOpenEventHandle(&o.ev[best], h));
      o.id[best] = best_id;
    }
    *out = o.ev[best];
    return PR_OK;
  }
  int wait_compute(int q, int kind, int b, int, int64_t v) {
    if (kind != kIpcCopied) return fail("IPC exchange: the compute stream only waits for copied records");
    hipEvent_t e = nullptr;
    PR_TRY(peer_event(q, kIpcCopied, b, 0, v, &e));
    PR_HIP(hipStreamWaitEvent(g->stream, e, 0));
    return PR_OK;
  }
  int wait_copy(int q, int kind, int b, int c, int64_t v) {
    if (kind != kIpcSent) return fail("IPC exchange: a copy stream only waits for sent records");
    hipEvent_t e = nullptr;
    PR_TRY(peer_event(q, kIpcSent, b, c, v, &e));
    if (!s->cstream[q]) return fail("IPC exchange: a copy stream is missing");
    const hipError_t rc = hipStreamWaitEvent(s->cstream[q], e, 0);
    if (rc != hipSuccess) {
      (void)hipGetLastError();
      return pr::fail(PR_ERR_HIP, std::string("IPC exchange: wait for peer ") + std::to_string(q) + "'s sent[" +
                                      std::to_string(b) + "] chunk " + std::to_string(c) + " of " + std::to_string(s->nc) +
                                      " (record " + std::to_string(v) + ", early " + std::to_string(g->x_ipc_early) +
                                      ", chunked " + std::to_string(g->x_chunked) + "): " + hipGetErrorString(rc));
    }
    return PR_OK;
  }
  // this rank's event of (kind, b, c) for its record of exchange k: a fresh generation once the
  // current one has served kRecordsPerEvent exchanges (or the counts restarted), its handle written
  // to the page slot before k is published
  int own_event(int kind, int b, int c, int64_t k, hipEvent_t *out) {
    IpcState::Own &o = s->own[((size_t)kind * 2 + b) * s->nc + c];
    const int i = ipc_gen_rotate(o.gen, k, s->epoch);
    if (i >= 0) {
      IpcSlot &sl = s->mine->slot[kind][b][c][i];
      sl.id.store(0, std::memory_order_release);  // the slot's previous generation (three back) is over
      if (o.ev[i]) (void)hipEventDestroy(o.ev[i]);
      o.ev[i] = nullptr;
      PR_HIP(hipEventCreateWithFlags(&o.ev[i], hipEventInterprocess | hipEventDisableTiming));
      hipIpcEventHandle_t h;
      PR_HIP(hipIpcGetEventHandle(&h, o.ev[i]));
      std::memcpy(&sl.h, &h, sizeof(h));
      sl.first_k.store(k, std::memory_order_release);
      sl.id.store(s->next_id++, std::memory_order_release);
      ipc_gen_started(o.gen, i, k, s->epoch);
    }
    *out = o.ev[o.gen.cur];
    return PR_OK;
  }
  int record(int kind, int b, int c, int64_t k) {
    hipEvent_t e = nullptr;
    PR_TRY(own_event(kind, b, c, k, &e));
    if (kind == kIpcSent) {  // chunk c of the runs of b is written (compute stream)
      if (c == s->nc - 1) PR_HIP(hipEventRecord(g->x_pack_ev, g->stream));  // the whole pass (+ pack) is done
      PR_HIP(hipEventRecord(e, g->stream));
    } else {  // the transfer stream has joined every copy of b
      PR_HIP(hipEventRecord(e, g->xstream));
    }
    return PR_OK;
  }
  int publish(int kind, int b, int64_t k) {
    (kind == kIpcSent ? s->mine->sent[b] : s->mine->copied[b]).store(k, std::memory_order_release);
    return PR_OK;
  }
  int pack(int b) { return exchange_pack(g, b); }
  int fail(const char *msg) { return pr::fail(PR_ERR_STATE, msg); }

  int copy_steps() const { return g->x_chunked ? s->nc : 1; }
  bool per_chunk() const { return g->x_ipc_early; }
  // the transfer stream joins this rank's pass (timing: pack done -> last chunk in); every copy
  // stream waits only until this rank no longer reads gather buffer b (x_free_ev, recorded before
  // the pass), so a peer's chunk can land while this rank's own epilogue still runs
  int copy_begin(int) {
    if (g->n_xc != s->nc) return fail("IPC exchange: chunk count changed");
    PR_HIP(hipStreamWaitEvent(g->xstream, g->x_pack_ev, 0));
    if (ev_a) PR_HIP(hipEventRecord(ev_a, g->xstream));
    for (int q = 0; q < s->P; ++q)
      if (q != s->self) PR_HIP(hipStreamWaitEvent(s->cstream[q], g->x_free_ev, 0));
    return PR_OK;
  }
  int copy(int q, int b, int lo, int hi) {
    const int nc = s->nc;
    const int64_t r0 = g->x_rch[(size_t)q * (nc + 1) + lo], r1 = g->x_rch[(size_t)q * (nc + 1) + hi];
    if (r1 > r0) {
      const double *src = static_cast<const double *>(s->peer_sbuf[q]) + (int64_t)(b & 1) * s->peer_stride[q] +
                          s->peer_soff_me[q] + r0;
      PR_HIP(hipMemcpyAsync(g->cbuf[b].as<double>() + g->S_pad + g->x_roff[q] + r0, src,
                            sizeof(double) * (size_t)(r1 - r0),
                            g->x_ipc_blit ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToDeviceNoCU, s->cstream[q]));
    }
    hipEvent_t e = s->cev[(size_t)q * nc + (hi - 1)];
    PR_HIP(hipEventRecord(e, s->cstream[q]));
    PR_HIP(hipStreamWaitEvent(g->xstream, e, 0));  // chunk hi - 1 of every peer -> x_ev[hi - 1]
    return PR_OK;
  }
  int step_done(int, int hi) {
    PR_HIP(hipEventRecord(g->x_ev[hi - 1], g->xstream));
    return PR_OK;
  }
};

bool stream_idle_within(hipStream_t st, double seconds) {
  if (!st) return true;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(st);
    if (e != hipErrorNotReady) {
      (void)hipGetLastError();
      return true;  // idle (or an error: nothing left to wait for)
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}

// Before the compute stream writes the send runs of `buf` for the next exchange: order the writes
// after every peer's copies of the previous exchange of `buf`.
int ipc_send_runs_free(pr_graph *g, int buf) {
  if (!g->x_ipc) return PR_OK;
  HipIpcOps o{g, g->ipc, nullptr};
  return g->ipc->proto.send_runs_free(o, buf);
}

int ipc_chunk_sent(pr_graph *g, int buf, int c) {
  HipIpcOps o{g, g->ipc, nullptr};
  return g->ipc->proto.chunk_sent(o, buf, c);
}

// Every kLeadEvery exchanges: wait (bounded) until the device has passed the compute-stream marker
// recorded 2 * kLeadEvery exchanges ago, then record it again.  The compute stream waits for the
// transfers each pass reads, so its progress bounds the copy streams' too.
static int bound_lead(pr_graph *g, IpcState *s) {
  if (++s->n_exch % kLeadEvery != 0) return PR_OK;
  const int j = (int)((s->n_exch / kLeadEvery) & 1);
  if (!s->lead_ev[j]) PR_HIP(hipEventCreateWithFlags(&s->lead_ev[j], hipEventDisableTiming));
  if (s->lead_rec[j]) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipEventQuery(s->lead_ev[j]);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) PR_HIP(e);
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kSpinLimit)
        return fail(PR_ERR_COMM, "IPC exchange: the device did not reach an exchange enqueued " +
                                     std::to_string(2 * kLeadEvery) + " exchanges ago (a peer stalled?)");
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  PR_HIP(hipEventRecord(s->lead_ev[j], g->stream));
  s->lead_rec[j] = true;
  return PR_OK;
}

int exchange_ipc(pr_graph *g, int buf, hipEvent_t ev_a, hipEvent_t ev_b) {
  HipIpcOps o{g, g->ipc, ev_a};
  const bool packed = g->x_packed == buf;
  g->x_packed = -1;
  PR_TRY(g->ipc->proto.exchange(o, buf, packed));
  if (ev_b) PR_HIP(hipEventRecord(ev_b, g->xstream));
  g->x_pending = true;
  return bound_lead(g, g->ipc);
}

// Destroy: the peers may still be copying out of this rank's send buffers; wait for the copies of
// every exchange this rank published, then unmap everything.  Host polls only, each bounded: a peer
// that died mid-run must not hang this process's teardown.
void ipc_destroy(pr_graph *g) {
  IpcState *s = g->ipc;
  if (!s) return;
  g->ipc = nullptr;
  g->x_ipc = false;
  const std::string err = pr_last_error();  // the bounded waits below must not replace a real error
  for (int q = 0; q < s->P; ++q) {
    if (q == s->self || !s->peer[q]) continue;
    for (int b = 0; b < 2; ++b) {
      const int64_t k = s->mine->sent[b].load(std::memory_order_acquire);
      if (k <= 0) continue;
      if (spin_until(s->peer[q]->copied[b], k, "copied", q, 10.0) != PR_OK) break;  // peer gone
      // then its copies of exchange k (the event it recorded after them), polled with a deadline
      hipEvent_t e = nullptr;
      HipIpcOps o{g, s, nullptr};
      if (o.peer_event(q, kIpcCopied, b, 0, k, &e) != PR_OK) break;
      const auto t0 = std::chrono::steady_clock::now();
      while (hipEventQuery(e) == hipErrorNotReady &&
             std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 10.0)
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  set_error(err);
  free_state(s);
}

}  // namespace pr
