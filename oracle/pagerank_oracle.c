/*
 * Oracle #2 -- plain-C (OpenMP) restatement of Sparky.java's PageRank on the canonical CSR.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker for libpagerank_hip and the CPU
 * baseline ("kind": "port") of bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it.  The product library never links or calls it.
 *
 * Parity status: the reference (Sparky.java, a Spark 1.x job) cannot run in this image (no
 * JDK, no Spark) and holds no tests or golden vectors, so the oracle is
 * "parity unpinned" against a run of the reference.  It is pinned to the hand-derived
 * known-answer test of SURVEY.md §4 and cross-checked against the literal RDD emulator
 * oracle/sparky_rdd.py (tests/test_oracle.py, tests/golden/).
 *
 * Semantics restated:
 *   A1  edge set E' = distinct (src,dst) pairs, self-loops kept    Sparky.java:98-110, :124
 *   A2  V = every interned ID (keys U targets), N = |V|            Sparky.java:127-162
 *   A3  d(u) = number of distinct targets of u                     Sparky.java:196-207
 *   A4  D = sink-only vertices (never a record/src) in local mode  Sparky.java:114-118, :146-149, :172-184
 *   A5  r0 = 1.0                                                   Sparky.java:164-170
 *   A6  c(u) = r(u) / d(u), one fp64 division                      Sparky.java:207
 *   A7  dc = sum_{v in D} r(v)                                     Sparky.java:219-222
 *   A8  in-degree-0 vertices use their OLD rank as the sum         Sparky.java:224-225
 *   A9  S(v) = sum of c(u) over in-links                           Sparky.java:27-32, :229
 *   A10 r' = 0.15 + 0.85 * (S + dc / (double)N), no FMA            Sparky.java:233
 *
 * Input convention (same as the C ABI): interned IDs in [0, V); dst[i] == -1 marks a
 * record without 'a' links (Sparky.java:114-118).  Row sums use Neumaier compensated
 * summation so that the oracle is closer to the exactly rounded value than any Spark order.
 *
 * Build: see oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* vertex flag bits -- must equal PR_VF_* in include/pagerank_hip.h (checked by a test) */
#define ORC_VF_KEY 1u    /* appeared as a record / src          (Sparky.java:127)      */
#define ORC_VF_SINK 2u   /* target that is never a record       (Sparky.java:146-149)  */
#define ORC_VF_NOLINK 4u /* record whose list holds only null   (Sparky.java:114-118)  */
#define ORC_VF_INDEG0 8u /* receives no contribution            (Sparky.java:224)      */

static void radix_sort_u64(uint64_t *a, uint64_t *tmp, int64_t n, int bits) {
  /* LSD radix sort, 16-bit digits, only the low `bits` bits are significant. */
  for (int shift = 0; shift < bits; shift += 16) {
    int64_t *cnt = (int64_t *)calloc(65537, sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i) cnt[((a[i] >> shift) & 0xFFFF) + 1]++;
    for (int d = 0; d < 65536; ++d) cnt[d + 1] += cnt[d];
    for (int64_t i = 0; i < n; ++i) tmp[cnt[(a[i] >> shift) & 0xFFFF]++] = a[i];
    memcpy(a, tmp, (size_t)n * sizeof(uint64_t));
    free(cnt);
  }
}

static int bits_for(int64_t v) {
  int b = 1;
  while (b < 63 && ((int64_t)1 << b) < v) ++b;
  return b;
}

/* Canonical CSR of in-links (rows = dst, columns = src ascending, deduplicated).
 * row_ptr: V+1, col: capacity >= E, out_deg: V, vflags: V.  Returns 0, or -1 on bad input
 * (an ID out of range, or an ID in [0,V) that appears nowhere). */
int orc_build(int32_t V, int64_t E, const int32_t *src, const int32_t *dst, int64_t *row_ptr,
              int32_t *col, int32_t *out_deg, uint8_t *vflags, int64_t *n_dedup) {
  if (V < 0 || E < 0) return -1;
  uint8_t *seen = (uint8_t *)calloc((size_t)V + 1, 1);
  int64_t m = 0;
  for (int64_t i = 0; i < E; ++i) {
    if (src[i] < 0 || src[i] >= V || dst[i] < -1 || dst[i] >= V) { free(seen); return -1; }
    seen[src[i]] = 1;
    if (dst[i] >= 0) { seen[dst[i]] = 1; ++m; }
  }
  for (int32_t v = 0; v < V; ++v)
    if (!seen[v]) { free(seen); return -1; }
  free(seen);
  int b = bits_for(V);
  uint64_t *keys = (uint64_t *)malloc((size_t)(m ? m : 1) * sizeof(uint64_t));
  uint64_t *tmp = (uint64_t *)malloc((size_t)(m ? m : 1) * sizeof(uint64_t));
  int64_t k = 0;
  memset(vflags, 0, (size_t)V);
  for (int64_t i = 0; i < E; ++i) {
    vflags[src[i]] |= ORC_VF_KEY;
    if (dst[i] >= 0) keys[k++] = ((uint64_t)(uint32_t)dst[i] << b) | (uint32_t)src[i];
  }
  radix_sort_u64(keys, tmp, m, 2 * b);
  int64_t u = 0;
  for (int64_t i = 0; i < m; ++i)
    if (i == 0 || keys[i] != keys[i - 1]) keys[u++] = keys[i];
  memset(out_deg, 0, (size_t)V * sizeof(int32_t));
  for (int64_t v = 0; v <= V; ++v) row_ptr[v] = 0;
  uint64_t mask = ((uint64_t)1 << b) - 1;
  for (int64_t i = 0; i < u; ++i) {
    int32_t d = (int32_t)(keys[i] >> b), s = (int32_t)(keys[i] & mask);
    row_ptr[d + 1]++;
    col[i] = s;
    out_deg[s]++;
  }
  for (int64_t v = 0; v < V; ++v) row_ptr[v + 1] += row_ptr[v];
  for (int32_t v = 0; v < V; ++v) {
    if (!(vflags[v] & ORC_VF_KEY)) vflags[v] |= ORC_VF_SINK;
    else if (out_deg[v] == 0) vflags[v] |= ORC_VF_NOLINK;
    if (row_ptr[v + 1] == row_ptr[v]) vflags[v] |= ORC_VF_INDEG0;
  }
  free(keys);
  free(tmp);
  *n_dedup = u;
  return 0;
}

static inline void neumaier_add(double *s, double *c, double x) {
  double t = *s + x;
  if (fabs(*s) >= fabs(x)) *c += (*s - t) + x;
  else *c += (x - t) + *s;
  *s = t;
}

/* Power iteration of Sparky.java:187-236.  `ranks` holds r0 on entry (or is filled with
 * 1.0 when init == NULL) and r_iters on exit.  dc_out[i] / l1_out[i] (may be NULL) get the
 * dangling sum used by iteration i and sum |r_{i+1} - r_i|.  dangling_none != 0 gives the
 * cluster-mode semantics (dc == 0).  history (may be NULL) gets V doubles per
 * iteration.  nthreads <= 0 uses the OpenMP default. */
int orc_run(int32_t V, const int64_t *row_ptr, const int32_t *col, const int32_t *out_deg,
            const uint8_t *vflags, int32_t iters, int32_t dangling_none, double teleport,
            double damping, const double *init, double *ranks, double *dc_out, double *l1_out,
            double *history, int32_t nthreads) {
  if (nthreads > 0) omp_set_num_threads(nthreads);
  double *c = (double *)malloc((size_t)(V ? V : 1) * sizeof(double));
  double *rn = (double *)malloc((size_t)(V ? V : 1) * sizeof(double));
  for (int32_t v = 0; v < V; ++v) ranks[v] = init ? init[v] : 1.0;
  const double n = (double)V;
  for (int32_t it = 0; it < iters; ++it) {
    double dc = 0.0, dcc = 0.0;
    if (!dangling_none)
      for (int32_t v = 0; v < V; ++v)
        if (vflags[v] & ORC_VF_SINK) neumaier_add(&dc, &dcc, ranks[v]);
    dc += dcc;
#pragma omp parallel for schedule(static)
    for (int32_t u = 0; u < V; ++u) c[u] = out_deg[u] > 0 ? ranks[u] / (double)out_deg[u] : 0.0;
    const double t = dc / n;
#pragma omp parallel for schedule(dynamic, 4096)
    for (int32_t v = 0; v < V; ++v) {
      double s;
      if (row_ptr[v + 1] == row_ptr[v]) {
        s = ranks[v]; /* Sparky.java:224-225 */
      } else {
        double acc = 0.0, comp = 0.0;
        for (int64_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) neumaier_add(&acc, &comp, c[col[e]]);
        s = acc + comp;
      }
      double x = s + t;
      double y = damping * x;
      rn[v] = teleport + y;
    }
    double l1 = 0.0, l1c = 0.0;
    for (int32_t v = 0; v < V; ++v) neumaier_add(&l1, &l1c, fabs(rn[v] - ranks[v]));
    memcpy(ranks, rn, (size_t)V * sizeof(double));
    if (dc_out) dc_out[it] = dc;
    if (l1_out) l1_out[it] = l1 + l1c;
    if (history) memcpy(history + (size_t)it * V, ranks, (size_t)V * sizeof(double));
  }
  free(c);
  free(rn);
  return 0;
}

/* Flag constants, exported so a test can check they equal the ABI's PR_VF_*. */
uint32_t orc_flag_bits(void) {
  return ORC_VF_KEY | (ORC_VF_SINK << 8) | (ORC_VF_NOLINK << 16) | (ORC_VF_INDEG0 << 24);
}
