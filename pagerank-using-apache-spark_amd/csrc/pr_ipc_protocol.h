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
// Per-chunk sent records (round 5): sent[b] is nc events, one per exchange chunk
// (chunk c = the sources of hot phase c).  With the fused pack the pass may record chunk c as soon
// as the epilogue has written that chunk's runs (chunk_sent, during the pass); exchange() records
// the chunks the pass did not (all of them after an unfused pack) and then publishes k once.  A
// receiver's copy of chunks [lo, hi) waits for the peer's chunk hi - 1 record only: the owner
// records its chunks in order on one stream.  Publishing once per exchange, after the last chunk's
// record, keeps the binding argument above unchanged: a waiter that saw k published finds record k
// as the latest of every chunk, and the owner records chunk c of exchange k + 1 of b only after it
// has passed its reuse wait on this rank's copied[b] record k.
//
// Ops (all return 0 or a negative error code):
//   spin(q, kind, b, v)            host: until peer q has published >= v records of kind[b]
//   wait_compute(q, kind, b, c, v) the compute stream waits on peer q's kind[b] (chunk c; copied: c
//                                  = 0), meaning record v
//   wait_copy(q, kind, b, c, v)    peer q's copy stream waits on peer q's kind[b] chunk c (record v)
//   record(kind, b, c, k)          enqueue this rank's k-th record of kind[b] chunk c (sent: compute
//                                  stream, copied: transfer stream)
//   publish(kind, b, k)            make this rank's k-th records of kind[b] visible to the peers
//   pack(b)                        write the runs of b (when the pass did not: pack kernel)
//   per_chunk()                    the pass publishes chunk by chunk (PR_OPT_XCHG_IPC = 2): every
//                                  chunk has its own record; otherwise only the last chunk's event is
//                                  recorded and every copy waits for it (one record per exchange, the
//                                  round-4 transport)
//   copy_steps()                   how many steps the copies take (1: whole runs; nc: per chunk)
//   copy_begin(b)                  the copy streams wait until this rank's gather buffer b is free
//   copy(q, b, lo, hi)             copy chunks [lo, hi) of peer q's run of b
//   step_done(lo, hi)              every peer's chunks [lo, hi) are in: the transfer stream records
//   fail(msg)                      an error code with a message
#pragma once

#include <stdint.h>

namespace pr {

enum IpcKind { kIpcSent = 0, kIpcCopied = 1 };

// Per-chunk publication: the epilogue groups (of rows_per_grp local rows) launched before chunk c's
// record.  Chunk c of the send runs holds the sources at local rows below (c + 1) * chunk_rows (the
// class regions of hot phase c); launch c covers groups [end(c - 1), end(c)), so every row of chunk
// c is written before its record and the launches partition [0, ngrp).
inline int64_t ipc_epi_chunk_end(int64_t ngrp, int c, int nxc, int64_t chunk_rows, int64_t rows_per_grp) {
  if (c >= nxc - 1) return ngrp;
  const int64_t e = ((int64_t)(c + 1) * chunk_rows + rows_per_grp - 1) / rows_per_grp;
  return e < ngrp ? e : ngrp;
}

template <class Ops>
struct IpcProtocol {
  int P = 0, self = 0;
  int nc = 1;                 // sent chunks per buffer
  int64_t n[2] = {0, 0};      // exchanges of buffer b since the mode was (re)enabled
  int64_t freed[2] = {0, 0};  // exchange of b whose run writes are already ordered after the copies
  int rec_c[2] = {0, 0};      // chunks of the next exchange of b already recorded by the pass

  void reset() {
    n[0] = n[1] = freed[0] = freed[1] = 0;
    rec_c[0] = rec_c[1] = 0;
  }

  // Before the compute stream writes the runs of b for the next exchange of b.
  int send_runs_free(Ops &o, int b) {
    const int64_t k = n[b] + 1;
    if (freed[b] >= k) return 0;
    if (k > 1)
      for (int q = 0; q < P; ++q) {
        if (q == self) continue;
        int rv = o.spin(q, kIpcCopied, b, k - 1);
        if (rv == 0) rv = o.wait_compute(q, kIpcCopied, b, 0, k - 1);
        if (rv != 0) return rv;
      }
    freed[b] = k;
    return 0;
  }

  // During the pass (fused pack): the runs of chunk c of b are written; chunks in order, c < nc - 1
  // (the last chunk carries the two slots k_finalize writes, recorded by exchange()).
  int chunk_sent(Ops &o, int b, int c) {
    if (!o.per_chunk()) return o.fail("IPC exchange: chunk records without per-chunk publication");
    const int64_t k = n[b] + 1;
    if (freed[b] < k) return o.fail("IPC exchange: chunk recorded before the reuse wait");
    if (c != rec_c[b] || c >= nc - 1) return o.fail("IPC exchange: chunk records out of order");
    const int rv = o.record(kIpcSent, b, c, k);
    if (rv == 0) rec_c[b] = c + 1;
    return rv;
  }

  // The exchange of buffer b; packed: the pass already wrote the runs (fused pack).
  int exchange(Ops &o, int b, bool packed) {
    int rv = 0;
    if (!packed) {
      if (rec_c[b] != 0) return o.fail("IPC exchange: chunks recorded without the fused pack");
      if ((rv = send_runs_free(o, b)) != 0) return rv;
      if ((rv = o.pack(b)) != 0) return rv;
    }
    const int64_t k = ++n[b];
    if (freed[b] < k) return o.fail("IPC exchange: send runs written without the reuse wait");
    const bool pc = o.per_chunk();
    for (int c = pc ? rec_c[b] : nc - 1; c < nc; ++c)
      if ((rv = o.record(kIpcSent, b, c, k)) != 0) return rv;
    rec_c[b] = 0;
    if ((rv = o.publish(kIpcSent, b, k)) != 0) return rv;
    for (int q = 0; q < P; ++q) {
      if (q == self) continue;
      if ((rv = o.spin(q, kIpcSent, b, k)) != 0) return rv;
    }
    if ((rv = o.copy_begin(b)) != 0) return rv;
    const int steps = o.copy_steps();
    if (steps != 1 && steps != nc) return o.fail("IPC exchange: copy steps must be 1 or the chunk count");
    for (int s = 0; s < steps; ++s) {
      const int lo = steps == 1 ? 0 : s, hi = steps == 1 ? nc : s + 1;
      for (int q = 0; q < P; ++q) {
        if (q == self) continue;
        // per chunk: wait for that chunk's record; otherwise one wait per exchange and peer, for the
        // only record there is, before the first copy (each record is waited on once per peer)
        if (pc || s == 0)
          if ((rv = o.wait_copy(q, kIpcSent, b, pc ? hi - 1 : nc - 1, k)) != 0) return rv;
        if ((rv = o.copy(q, b, lo, hi)) != 0) return rv;
      }
      if ((rv = o.step_done(lo, hi)) != 0) return rv;
    }
    if ((rv = o.record(kIpcCopied, b, 0, k)) != 0) return rv;
    return o.publish(kIpcCopied, b, k);
  }
};

}  // namespace pr
