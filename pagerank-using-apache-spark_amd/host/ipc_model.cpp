// CPU model checker of the IPC exchange's host-side ordering (csrc/pr_ipc_protocol.h), the same
// template the library runs (csrc/pr_ipc.hip).  One thread per rank runs a seeded sequence of
// resets and iterations -- the same sequence on every rank, as the library requires -- with random
// delays; interprocess events are modelled as "the exchange of the latest record enqueued so far"
// per (rank, kind, buffer, chunk), and the record counters as atomics.  Every stream wait checks that the latest
// record of the peer's event at that moment is exactly the record the protocol means (so the
// device wait would bind to it), and the run ends without deadlock.  Used by
// tests/test_ipc_protocol_cpu.py through ipc_model_run().
//
// Generations (csrc/pr_ipc_gens.h, the helper the library uses): every event is modelled
// as its page slots, each with a generation id, the first exchange it serves, its record count and
// its latest record.  An owner rotates to a fresh generation exactly as the library does, a record
// past the runtime's 32 per event fails, and a waiter picks its slot with the library's rule: the
// picked generation's latest record must be the record meant.  Optional re-enables (every rank
// idle, the counts restart, a new epoch) exercise the rotation at the restart.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "pr_ipc_gens.h"
#include "pr_ipc_protocol.h"

namespace {

constexpr int kMaxChunks = 16;
constexpr int64_t kRuntimeRecordLimit = 32;  // records one interprocess event takes (the runtime's ring)

// one page slot of one event: generation id (0: empty), first exchange, records, latest record
struct GenSlot {
  std::atomic<int64_t> id{0}, first_k{0}, count{0}, latest{0};
};

struct World {
  int P, nc;
  // per (rank, kind, buffer, chunk): records enqueued ("latest record"); per (rank, kind, buffer):
  // the published counter
  std::vector<std::atomic<int64_t>> enq, pub;
  std::vector<GenSlot> gens;  // [ex(r, kind, b, c) * kIpcGens + slot]
  std::atomic<int64_t> bar_count{0}, bar_gen{0};  // re-enable barrier
  std::mutex mu;
  std::string err;
  std::atomic<bool> failed{false};
  std::atomic<int64_t> waits{0};
  World(int p, int c) : P(p), nc(c), enq(4 * (size_t)p * kMaxChunks), pub(4 * (size_t)p),
                       gens(4 * (size_t)p * kMaxChunks * pr::kIpcGens) {
    for (auto &a : enq) a.store(0);
    for (auto &a : pub) a.store(0);
  }
  size_t ix(int r, int kind, int b) const { return (size_t)r * 4 + (size_t)kind * 2 + (size_t)b; }
  size_t ex(int r, int kind, int b, int c) const { return ix(r, kind, b) * kMaxChunks + (size_t)c; }
  int fail(const std::string &m) {
    std::lock_guard<std::mutex> g(mu);
    if (err.empty()) err = m;
    failed.store(true);
    return -1;
  }
  // every rank arrives before any leaves (false: a rank failed meanwhile)
  bool barrier() {
    const int64_t gen = bar_gen.load();
    if (bar_count.fetch_add(1) + 1 == P) {
      bar_count.store(0);
      bar_gen.fetch_add(1);
      return true;
    }
    while (bar_gen.load() == gen) {
      if (failed.load()) return false;
      std::this_thread::yield();
    }
    return true;
  }
};

struct ModelOps {
  World *w;
  int self;
  std::mt19937_64 rng;
  int max_delay_us;
  bool broken;     // checker self-test: no host spin before the sent waits
  int steps = 1;   // copy steps of the current exchange (1: whole runs; nc: per chunk)
  bool pc = false;  // per-chunk publication (every chunk its own record)
  int64_t epoch = 0;  // bumped at every re-enable (the library's IpcState::epoch)
  int64_t next_id = 1;
  std::vector<pr::IpcGenOwner> own = std::vector<pr::IpcGenOwner>(4 * (size_t)kMaxChunks);

  void delay() {
    if (max_delay_us <= 0) return;
    const int d = (int)(rng() % (uint64_t)(max_delay_us + 1));
    if (d > 0) std::this_thread::sleep_for(std::chrono::microseconds(d));
    else std::this_thread::yield();
  }
  int spin(int q, int kind, int b, int64_t v) {
    if (broken && kind == pr::kIpcSent) {
      delay();
      return 0;
    }
    const auto t0 = std::chrono::steady_clock::now();
    while (w->pub[w->ix(q, kind, b)].load(std::memory_order_acquire) < v) {
      if (w->failed.load()) return -1;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20))
        return w->fail("deadlock: rank " + std::to_string(self) + " never saw record " + std::to_string(v) +
                       " of rank " + std::to_string(q));
      std::this_thread::yield();
    }
    delay();
    return 0;
  }
  int wait_any(int q, int kind, int b, int c, int64_t v) {
    const int64_t latest = w->enq[w->ex(q, kind, b, c)].load(std::memory_order_acquire);
    w->waits.fetch_add(1);
    const std::string what = "rank " + std::to_string(self) + " waits on rank " + std::to_string(q) + "'s " +
                             (kind == pr::kIpcSent ? "sent" : "copied") + "[" + std::to_string(b) + "] chunk " +
                             std::to_string(c) + " meaning record " + std::to_string(v);
    if (latest != v) return w->fail(what + " but its latest record is " + std::to_string(latest));
    // the generation the library would open (pr_ipc.hip peer_event) must hold that record as its latest
    int64_t ids[pr::kIpcGens], firsts[pr::kIpcGens];
    GenSlot *sl = &w->gens[w->ex(q, kind, b, c) * pr::kIpcGens];
    for (int i = 0; i < pr::kIpcGens; ++i) {
      ids[i] = sl[i].id.load(std::memory_order_acquire);
      firsts[i] = sl[i].first_k.load(std::memory_order_acquire);
    }
    const int pick = pr::ipc_gen_pick(ids, firsts, v);
    if (pick < 0) return w->fail(what + " but no generation of it holds that record");
    const int64_t gl = sl[pick].latest.load(std::memory_order_acquire);
    if (gl != v)
      return w->fail(what + " but the generation it picks (slot " + std::to_string(pick) + ") has latest record " +
                     std::to_string(gl));
    delay();
    return 0;
  }
  int wait_compute(int q, int kind, int b, int c, int64_t v) { return wait_any(q, kind, b, c, v); }
  int wait_copy(int q, int kind, int b, int c, int64_t v) { return wait_any(q, kind, b, c, v); }
  int record(int kind, int b, int c, int64_t k) {
    // the event's latest record is now exchange k's (a chunk may skip exchanges whose sender
    // published whole runs, so the value is the exchange number, not a count)
    // the library's own_event: a fresh generation in the next slot when the current one is used up
    // or the counts restarted; its slot is stamped (id last) before the record, as in the page
    pr::IpcGenOwner &o = own[(size_t)(kind * 2 + b) * kMaxChunks + c];
    GenSlot *sl = &w->gens[w->ex(self, kind, b, c) * pr::kIpcGens];
    const int i = pr::ipc_gen_rotate(o, k, epoch);
    if (i >= 0) {
      sl[i].id.store(0, std::memory_order_release);
      sl[i].count.store(0);
      sl[i].latest.store(0);
      sl[i].first_k.store(k, std::memory_order_release);
      sl[i].id.store(next_id++, std::memory_order_release);
      pr::ipc_gen_started(o, i, k, epoch);
    }
    GenSlot &cur = sl[o.cur];
    if (cur.count.fetch_add(1) + 1 > kRuntimeRecordLimit)
      return w->fail("rank " + std::to_string(self) + " recorded one event more than " +
                     std::to_string(kRuntimeRecordLimit) + " times");
    cur.latest.store(k, std::memory_order_release);
    const int64_t prev = w->enq[w->ex(self, kind, b, c)].exchange(k);
    if (prev >= k)
      return w->fail("rank " + std::to_string(self) + " recorded chunk " + std::to_string(c) + " for exchange " +
                     std::to_string(k) + " after exchange " + std::to_string(prev));
    delay();
    return 0;
  }
  // pr_ipc.hip set_exchange_ipc off -> on: every rank idle; the counters restart, a new epoch
  bool reenable(pr::IpcProtocol<ModelOps> &proto) {
    if (!w->barrier()) return false;
    for (int kind = 0; kind < 2; ++kind)
      for (int b = 0; b < 2; ++b) {
        w->pub[w->ix(self, kind, b)].store(0);
        for (int c = 0; c < kMaxChunks; ++c) w->enq[w->ex(self, kind, b, c)].store(0);
      }
    proto.reset();
    ++epoch;
    return w->barrier();
  }
  int publish(int kind, int b, int64_t k) {
    const int n = kind == pr::kIpcSent ? w->nc : 1;
    for (int c = (kind == pr::kIpcSent && !pc) ? n - 1 : 0; c < n; ++c)  // record k enqueued before k is published
      if (w->enq[w->ex(self, kind, b, c)].load() != k)
        return w->fail("rank " + std::to_string(self) + " published " + std::to_string(k) + " before chunk " +
                       std::to_string(c) + "'s record");
    w->pub[w->ix(self, kind, b)].store(k, std::memory_order_release);
    delay();
    return 0;
  }
  int pack(int) {
    delay();
    return 0;
  }
  int copy_steps() const { return steps; }
  bool per_chunk() const { return pc; }
  int copy_begin(int) { return 0; }
  int copy(int, int, int, int) {
    delay();
    return 0;
  }
  int step_done(int, int) { return 0; }
  int fail(const char *m) { return w->fail(m); }
};

}  // namespace

extern "C" {

// pr_ipc_protocol.h ipc_epi_chunk_end, for tests/test_ipc_protocol_cpu.py
int64_t ipc_model_chunk_end(int64_t ngrp, int c, int nxc, int64_t chunk_rows, int64_t rows_per_grp) {
  return pr::ipc_epi_chunk_end(ngrp, c, nxc, chunk_rows, rows_per_grp);
}

// P ranks, nc sent chunks per buffer, run n_ops steps each (seeded, the same sequence on every
// rank: 0 = reset, which writes and exchanges buffer 0 with the pack kernel; otherwise an
// iteration whose pass writes the runs of the other buffer -- unfused (pack kernel), fused, or
// fused with its chunks recorded one by one during the pass -- and whose copies go whole or per
// chunk); returns the number of stream waits checked, or -1 with the first violation in err.
// max_delay_us < 0: the checker's self-test -- the same run with the sent spins left out.
// reenable_one_in > 0: about one op in that many is a re-enable (op 8) instead.
int64_t ipc_model_run2(int P, int nc, int n_ops, uint64_t seed, int max_delay_us, int reenable_one_in, char *err,
                       int errlen) {
  if (P < 2 || P > 64 || nc < 1 || nc > kMaxChunks || n_ops < 0) return -1;
  std::mt19937_64 ops_rng(seed);
  std::vector<int> ops((size_t)n_ops), steps((size_t)n_ops);
  for (size_t i = 0; i < ops.size(); ++i) {
    ops[i] = (int)(ops_rng() % 8);  // 0: reset, 1: unfused pack, 2..4: fused, 5..7: fused + early chunks
    steps[i] = (ops_rng() & 1) ? nc : 1;
    if (reenable_one_in > 0 && ops_rng() % (uint64_t)reenable_one_in == 0) ops[i] = 8;
  }
  World w(P, nc);
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r)
    th.emplace_back([&, r]() {
      ModelOps o{&w, r, std::mt19937_64(seed * 1315423911ull + (uint64_t)r + 1), max_delay_us < 0 ? -max_delay_us : max_delay_us,
                 max_delay_us < 0};
      pr::IpcProtocol<ModelOps> proto;
      proto.P = P;
      proto.self = r;
      proto.nc = nc;
      int cur = 0;
      for (size_t i = 0; i < ops.size(); ++i) {
        const int op = ops[i];
        o.steps = steps[i];
        // per-chunk publication is a mode (PR_OPT_XCHG_IPC = 2): the same on every rank; a reset
        // exchanges with the pack kernel either way
        o.pc = op == 0 ? (steps[i] & 1) != 0 : op >= 5;
        if (w.failed.load()) return;
        int rv;
        if (op == 8) {  // re-enable, then the reset that every enable is followed by
          if (!o.reenable(proto)) return;
          cur = 0;
          rv = proto.send_runs_free(o, 0);
          if (rv == 0) rv = proto.exchange(o, 0, false);
        } else if (op == 0) {  // pr_reset: k_finalize writes the slots of buffer 0's runs, then exchange(0)
          cur = 0;
          rv = proto.send_runs_free(o, 0);
          if (rv == 0) rv = proto.exchange(o, 0, false);
        } else {  // an iteration: the pass writes the runs of `out` (fused) unless op == 1
          const int out = cur ^ 1;
          rv = proto.send_runs_free(o, out);
          for (int c = 0; rv == 0 && op >= 5 && c < nc - 1; ++c) {  // epilogue chunk c done
            o.delay();
            rv = proto.chunk_sent(o, out, c);
          }
          if (rv == 0) rv = proto.exchange(o, out, op != 1);
          cur = out;
        }
        if (rv != 0) {
          w.fail("rank " + std::to_string(r) + ": protocol step failed");
          return;
        }
      }
    });
  for (auto &t : th) t.join();
  if (w.failed.load()) {
    if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", w.err.c_str());
    return -1;
  }
  return w.waits.load();
}

int64_t ipc_model_run(int P, int nc, int n_ops, uint64_t seed, int max_delay_us, char *err, int errlen) {
  return ipc_model_run2(P, nc, n_ops, seed, max_delay_us, 0, err, errlen);
}

}  // extern "C"
