// Host-side ordering protocol of the IPC exchange (PR_OPT_XCHG_IPC, pr_ipc.hip), written against an
// abstract Ops so that the library (HIP interprocess events + shared-memory record counters) and a
// CPU model checker (host/ipc_model.cpp, tests/test_ipc_protocol_cpu.py: one thread per rank,
// random delays, events modelled as "latest record enqueued") run the same sequence of steps.
// Plain C++, no HIP.
//
// Per rank and buffer b two interprocess events: sent[b] (its runs of b are written) and copied[b]
// (it has copied every peer's runs of b).  A wait on such an event binds to the latest record
// enqueued when the wait is enqueued, so before every wait the waiter's host spins until the
// owner has *published* (after enqueueing) the record it means: exchange k of b waits for the
// peers' sent[b] record k, and the writes of the runs of b for exchange k wait for the peers'
// copied[b] record k - 1.  A peer cannot enqueue the next record of the same event (k + 1, or k for
// copied) before it has passed a wait on this rank that comes after this rank's wait, so every
// wait binds to exactly the record meant -- the property the model checker asserts.
//
// Ops (all return 0 or a negative error code):
//   spin(q, kind, b, v)         host: until peer q has published >= v records of kind[b]
//   wait_compute(q, kind, b, v) the compute stream waits on peer q's kind[b] (meaning record v)
//   wait_copy(q, kind, b, v)    peer q's copy stream waits on peer q's kind[b] (record v)
//   record(kind, b, k)          enqueue this rank's k-th record of kind[b] (sent: compute stream,
//                               copied: transfer stream), then publish k
//   pack(b)                     write the runs of b (when the pass did not: pack kernel)
//   copies(b)                   the copy-stream waits for this rank's own pass, then the copies
//   fail(msg)                   an error code with a message
#pragma once

#include <stdint.h>

namespace pr {

enum IpcKind { kIpcSent = 0, kIpcCopied = 1 };

template <class Ops>
struct IpcProtocol {
  int P = 0, self = 0;
  int64_t n[2] = {0, 0};      // exchanges of buffer b since the mode was (re)enabled
  int64_t freed[2] = {0, 0};  // exchange of b whose run writes are already ordered after the copies

  void reset() { n[0] = n[1] = freed[0] = freed[1] = 0; }

  // Before the compute stream writes the runs of b for the next exchange of b.
  int send_runs_free(Ops &o, int b) {
    const int64_t k = n[b] + 1;
    if (freed[b] >= k) return 0;
    if (k > 1)
      for (int q = 0; q < P; ++q) {
        if (q == self) continue;
        int rv = o.spin(q, kIpcCopied, b, k - 1);
        if (rv == 0) rv = o.wait_compute(q, kIpcCopied, b, k - 1);
        if (rv != 0) return rv;
      }
    freed[b] = k;
    return 0;
  }

  // The exchange of buffer b; packed: the pass already wrote the runs (fused pack).
  int exchange(Ops &o, int b, bool packed) {
    int rv = 0;
    if (!packed) {
      if ((rv = send_runs_free(o, b)) != 0) return rv;
      if ((rv = o.pack(b)) != 0) return rv;
    }
    const int64_t k = ++n[b];
    if (freed[b] < k) return o.fail("IPC exchange: send runs written without the reuse wait");
    if ((rv = o.record(kIpcSent, b, k)) != 0) return rv;
    for (int q = 0; q < P; ++q) {
      if (q == self) continue;
      rv = o.spin(q, kIpcSent, b, k);
      if (rv == 0) rv = o.wait_copy(q, kIpcSent, b, k);
      if (rv != 0) return rv;
    }
    if ((rv = o.copies(b)) != 0) return rv;
    return o.record(kIpcCopied, b, k);
  }
};

}  // namespace pr
