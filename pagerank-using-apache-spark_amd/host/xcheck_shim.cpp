// Test shim (not product code): exposes the exchange agreement check of pr_xcheck.h -- the host
// logic verify_exchange runs after ncclCommInitRank -- to tests/test_xcheck.py on the CPU.
#include "pr_xcheck.h"

extern "C" {
int prx_width(int P) { return pr::xrec_width(P); }
int prx_fill(int64_t V, int64_t S_pad, int allgather, int nc, int chunked, int P, const int64_t *soff,
             const int64_t *sch, int64_t *rec) {
  return pr::xrec_fill(V, S_pad, allgather != 0, nc, chunked != 0, P, soff, sch, rec) ? 0 : -1;
}
int prx_check(const int64_t *all, int P, int me, const int64_t *mine, const int64_t *roff, const int64_t *rch, int nc,
              char *why, int why_len) {
  const char *w = "";
  const int rc = pr::xrec_check(all, P, me, mine, roff, rch, nc, &w);
  int i = 0;
  for (; w[i] && i + 1 < why_len; ++i) why[i] = w[i];
  if (why_len > 0) why[i] = 0;
  return rc;
}
}
