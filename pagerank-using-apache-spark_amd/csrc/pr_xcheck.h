// The attach-time agreement check of the row-partitioned exchange (pr_exchange.hip
// verify_exchange), host-only so that it is unit-tested on the CPU (tests/test_xcheck.py through
// host/xcheck_shim.cpp).  Every rank publishes one fixed-width record (all-gathered over RCCL):
//   [0] V   [1] S_pad   [2] whole-slice all-gather (0/1)
//   [3 + q]            doubles this rank sends peer q per iteration (its run length)
//   [P + 3]            2 * chunks + (chunked ? 1 : 0): how the runs travel
//   [P + 4 + q * kXMaxChunks + c]  the size of chunk c of the run to peer q
// and checks every other rank's record against what it expects to receive, chunk by chunk, so a
// mismatch (different inputs, different exchange options per rank) fails loudly at attach time
// instead of desynchronising the grouped ncclSend / ncclRecv pairs.  Replaces the ordering that
// Sparky.java:192's join shuffle enforced implicitly.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "pagerank_hip.h"

namespace pr {

constexpr int kXMaxChunks = 16;  // kMaxClasses / kXcds

inline int xrec_width(int P) { return P + 4 + P * kXMaxChunks; }

// This rank's record.  soff: P + 1 run offsets of what it sends; sch: P * (nc + 1) chunk starts
// within every run (pr_graph.h x_sch).  Returns false when nc exceeds kXMaxChunks.
inline bool xrec_fill(int64_t V, int64_t S_pad, bool allgather, int nc, bool chunked, int P, const int64_t *soff,
                      const int64_t *sch, int64_t *rec) {
  if (nc < 1 || nc > kXMaxChunks) return false;
  const int CH = P + 4, W = xrec_width(P);
  for (int i = 0; i < W; ++i) rec[i] = 0;
  rec[0] = V;
  rec[1] = S_pad;
  rec[2] = allgather ? 1 : 0;
  rec[P + 3] = 2 * (int64_t)nc + (chunked ? 1 : 0);
  if (!allgather)
    for (int q = 0; q < P; ++q) {
      rec[3 + q] = soff[q + 1] - soff[q];
      for (int c = 0; c < nc; ++c)
        rec[CH + q * kXMaxChunks + c] = sch[(size_t)q * (nc + 1) + c + 1] - sch[(size_t)q * (nc + 1) + c];
    }
  return true;
}

// Rank `me`'s check of all P records (`all`, P * width) against its own record and what it
// receives (roff: P + 1 run offsets, rch: P * (nc + 1) chunk starts).  Returns PR_OK, or
// PR_ERR_INVALID (the ranks were built differently) / PR_ERR_STATE (the lists disagree) with the
// reason in *why.
inline int xrec_check(const int64_t *all, int P, int me, const int64_t *mine, const int64_t *roff, const int64_t *rch,
                      int nc, const char **why) {
  const int CH = P + 4, W = xrec_width(P);
  const bool allgather = mine[2] != 0;
  for (int q = 0; q < P; ++q) {
    const int64_t *o = all + (size_t)q * W;
    if (o[0] != mine[0] || o[1] != mine[1]) return *why = "ranks hold parts of different graphs", PR_ERR_INVALID;
    if (o[2] != mine[2]) return *why = "ranks disagree on PR_BOPT_EXCHANGE", PR_ERR_INVALID;
    if (o[P + 3] != mine[P + 3]) return *why = "ranks disagree on the exchange chunking", PR_ERR_INVALID;
    if (q == me || allgather) continue;
    if (o[3 + me] != roff[q + 1] - roff[q]) return *why = "exchange lists disagree between ranks", PR_ERR_STATE;
    for (int c = 0; c < nc; ++c)
      if (o[CH + me * kXMaxChunks + c] != rch[(size_t)q * (nc + 1) + c + 1] - rch[(size_t)q * (nc + 1) + c])
        return *why = "exchange chunks disagree between ranks", PR_ERR_STATE;
  }
  return PR_OK;
}

}  // namespace pr
