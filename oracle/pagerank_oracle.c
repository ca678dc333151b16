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

/* Parallel LSD radix sort (OpenMP): per-thread digit histograms over contiguous chunks, then a
 * stable scatter.  Only the low `bits` bits are significant.  The result ends in `a`. */
static void radix_sort_u64(uint64_t *a, uint64_t *tmp, int64_t n, int bits) {
  if (n <= 1 || bits <= 0) return;
  const int npass = (bits + 10) / 11;
  const int dbits = (bits + npass - 1) / npass;
  const int64_t nd = (int64_t)1 << dbits;
  const int T = omp_get_max_threads();
  int64_t *cnt = (int64_t *)calloc((size_t)(nd * T), sizeof(int64_t));
  uint64_t *src = a, *dst = tmp;
  for (int pass = 0; pass < npass; ++pass) {
    const int shift = pass * dbits;
    const uint64_t dmask = (uint64_t)nd - 1;
#pragma omp parallel num_threads(T)
    {
      const int t = omp_get_thread_num(), nt = omp_get_num_threads();
      const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
      int64_t *c = cnt + (int64_t)t * nd;
      memset(c, 0, (size_t)nd * sizeof(int64_t));
      for (int64_t i = lo; i < hi; ++i) c[(src[i] >> shift) & dmask]++;
#pragma omp barrier
#pragma omp single
      {
        int64_t run = 0; /* digit-major, thread-minor: stable */
        for (int64_t d = 0; d < nd; ++d)
          for (int tt = 0; tt < nt; ++tt) {
            const int64_t x = cnt[(int64_t)tt * nd + d];
            cnt[(int64_t)tt * nd + d] = run;
            run += x;
          }
      }
      for (int64_t i = lo; i < hi; ++i) dst[c[(src[i] >> shift) & dmask]++] = src[i];
    }
    uint64_t *x = src;
    src = dst;
    dst = x;
  }
  if (src != a) memcpy(a, src, (size_t)n * sizeof(uint64_t));
  free(cnt);
}

static int bits_for(int64_t v) {
  int b = 1;
  while (b < 63 && ((int64_t)1 << b) < v) ++b;
  return b;
}

/* Canonical CSR of in-links (rows = dst, columns = src ascending, deduplicated).
 * row_ptr: V+1, col: capacity >= E, out_deg: V, vflags: V.  Returns 0, or -1 on bad input
 * (an ID out of range, or an ID in [0,V) that appears nowhere).  Every step is a parallel
 * loop whose result does not depend on the thread count (the sort is stable). */
int orc_build(int32_t V, int64_t E, const int32_t *src, const int32_t *dst, int64_t *row_ptr,
              int32_t *col, int32_t *out_deg, uint8_t *vflags, int64_t *n_dedup) {
  if (V < 0 || E < 0) return -1;
  uint8_t *seen = (uint8_t *)calloc((size_t)V + 1, 1);
  int64_t m = 0;
  int bad = 0;
  memset(vflags, 0, (size_t)V);
#pragma omp parallel for reduction(+ : m) reduction(| : bad) schedule(static)
  for (int64_t i = 0; i < E; ++i) {
    const int32_t s = src[i], d = dst[i];
    if (s < 0 || s >= V || d < -1 || d >= V) { bad = 1; continue; }
    __atomic_store_n(&seen[s], 1, __ATOMIC_RELAXED);
    __atomic_store_n(&vflags[s], ORC_VF_KEY, __ATOMIC_RELAXED); /* Sparky.java:127 key set */
    if (d >= 0) { __atomic_store_n(&seen[d], 1, __ATOMIC_RELAXED); ++m; }
  }
  if (!bad) {
#pragma omp parallel for reduction(| : bad) schedule(static)
    for (int32_t v = 0; v < V; ++v)
      if (!seen[v]) bad = 1;
  }
  free(seen);
  if (bad) return -1;
  const int b = bits_for(V);
  uint64_t *keys = (uint64_t *)malloc((size_t)(m ? m : 1) * sizeof(uint64_t));
  uint64_t *tmp = (uint64_t *)malloc((size_t)(m ? m : 1) * sizeof(uint64_t));
  /* keys in input order: per-thread counts, then each thread writes its chunk's edges */
  const int T = omp_get_max_threads();
  int64_t *off = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const int64_t lo = E * t / nt, hi = E * (t + 1) / nt;
    int64_t c = 0;
    for (int64_t i = lo; i < hi; ++i) c += dst[i] >= 0;
    off[t + 1] = c;
#pragma omp barrier
#pragma omp single
    for (int tt = 0; tt < nt; ++tt) off[tt + 1] += off[tt];
    int64_t k = off[t];
    for (int64_t i = lo; i < hi; ++i)
      if (dst[i] >= 0) keys[k++] = ((uint64_t)(uint32_t)dst[i] << b) | (uint32_t)src[i];
  }
  radix_sort_u64(keys, tmp, m, 2 * b); /* Sparky.java:124 distinct + groupByKey */
  /* adjacent unique into tmp (chunk counts, prefix, write) */
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const int64_t lo = m * t / nt, hi = m * (t + 1) / nt;
    int64_t c = 0;
    for (int64_t i = lo; i < hi; ++i) c += (i == 0 || keys[i] != keys[i - 1]);
    off[t + 1] = c;
#pragma omp barrier
#pragma omp single
    {
      off[0] = 0;
      for (int tt = 0; tt < nt; ++tt) off[tt + 1] += off[tt];
    }
    int64_t k = off[t];
    for (int64_t i = lo; i < hi; ++i)
      if (i == 0 || keys[i] != keys[i - 1]) tmp[k++] = keys[i];
  }
  const int64_t u = off[T];
  free(off);
  free(keys);
  keys = tmp;
  const uint64_t mask = ((uint64_t)1 << b) - 1;
#pragma omp parallel for schedule(static)
  for (int32_t v = 0; v < V; ++v) out_deg[v] = 0;
  /* row_ptr[v] = first edge whose row >= v (every v written once) */
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i <= u; ++i) {
    const int64_t rc = (i < u) ? (int64_t)(keys[i] >> b) : (int64_t)V;
    const int64_t rp = (i > 0) ? (int64_t)(keys[i - 1] >> b) : -1;
    for (int64_t v = rp + 1; v <= rc; ++v) row_ptr[v] = i;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < u; ++i) {
    const int32_t s = (int32_t)(keys[i] & mask);
    col[i] = s;
    __atomic_fetch_add(&out_deg[s], 1, __ATOMIC_RELAXED); /* Sparky.java:196-207 */
  }
#pragma omp parallel for schedule(static)
  for (int32_t v = 0; v < V; ++v) {
    uint8_t f = vflags[v];
    if (!(f & ORC_VF_KEY)) f |= ORC_VF_SINK;            /* Sparky.java:146-149 */
    else if (out_deg[v] == 0) f |= ORC_VF_NOLINK;       /* Sparky.java:114-118 */
    if (row_ptr[v + 1] == row_ptr[v]) f |= ORC_VF_INDEG0; /* Sparky.java:224 */
    vflags[v] = f;
  }
  free(keys);
  *n_dedup = u;
  return 0;
}

static inline void neumaier_add(double *s, double *c, double x) {
  double t = *s + x;
  if (fabs(*s) >= fabs(x)) *c += (*s - t) + x;
  else *c += (x - t) + *s;
  *s = t;
}

/* Neumaier-compensated sum of x[i] over i in [0, n) with flt(i) true, in parallel: per-thread
 * compensated partials over static chunks, combined in thread order (deterministic for a given
 * thread count). */
static double par_sum(int64_t n, const double *x, const double *y, const uint8_t *flags, uint8_t bit) {
  const int T = omp_get_max_threads();
  double *ps = (double *)calloc((size_t)T, sizeof(double));
  double *pc = (double *)calloc((size_t)T, sizeof(double));
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    double s = 0.0, c = 0.0;
    for (int64_t i = lo; i < hi; ++i) {
      if (flags && !(flags[i] & bit)) continue;
      neumaier_add(&s, &c, y ? fabs(x[i] - y[i]) : x[i]);
    }
    ps[t] = s;
    pc[t] = c;
  }
  double s = 0.0, c = 0.0;
  for (int t = 0; t < T; ++t) {
    neumaier_add(&s, &c, ps[t]);
    neumaier_add(&s, &c, pc[t]);
  }
  free(ps);
  free(pc);
  return s + c;
}

/* Power iteration of Sparky.java:187-236.  `ranks` holds r0 on entry (or is filled with
 * 1.0 when init == NULL) and r_iters on exit.  dc_out[i] / l1_out[i] (may be NULL) get the
 * dangling sum used by iteration i and sum |r_{i+1} - r_i|; iter_ms[i] (may be NULL) the wall
 * time of iteration i.  dangling_none != 0 gives the cluster-mode semantics (dc == 0, SURVEY.md
 * A4).  history (may be NULL) gets V doubles per iteration.  nthreads <= 0 uses the OpenMP
 * default. */
int orc_run(int32_t V, const int64_t *row_ptr, const int32_t *col, const int32_t *out_deg,
            const uint8_t *vflags, int32_t iters, int32_t dangling_none, double teleport,
            double damping, const double *init, double *ranks, double *dc_out, double *l1_out,
            double *history, int32_t nthreads, double *iter_ms) {
  if (nthreads > 0) omp_set_num_threads(nthreads);
  double *c = (double *)malloc((size_t)(V ? V : 1) * sizeof(double));
  double *rn = (double *)malloc((size_t)(V ? V : 1) * sizeof(double));
  double *r = (double *)malloc((size_t)(V ? V : 1) * sizeof(double));
#pragma omp parallel for schedule(static)
  for (int32_t v = 0; v < V; ++v) r[v] = init ? init[v] : 1.0; /* Sparky.java:165-170 */
  const double n = (double)V;
  for (int32_t it = 0; it < iters; ++it) {
    const double t0 = omp_get_wtime();
    /* Sparky.java:219-222: dc = sum of the previous ranks over the sink-only set D */
    const double dc = dangling_none ? 0.0 : par_sum(V, r, NULL, vflags, ORC_VF_SINK);
#pragma omp parallel for schedule(static)
    for (int32_t u = 0; u < V; ++u) c[u] = out_deg[u] > 0 ? r[u] / (double)out_deg[u] : 0.0; /* :207 */
    const double t = dc / n;
#pragma omp parallel for schedule(dynamic, 4096)
    for (int32_t v = 0; v < V; ++v) {
      double s;
      if (row_ptr[v + 1] == row_ptr[v]) {
        s = r[v]; /* Sparky.java:224-225 */
      } else {
        double acc = 0.0, comp = 0.0;
        for (int64_t e = row_ptr[v]; e < row_ptr[v + 1]; ++e) neumaier_add(&acc, &comp, c[col[e]]);
        s = acc + comp;
      }
      double x = s + t; /* Sparky.java:233, evaluated in Java's order without FMA */
      double y = damping * x;
      rn[v] = teleport + y;
    }
    const double l1 = par_sum(V, rn, r, NULL, 0);
    double *sw = r;
    r = rn;
    rn = sw;
    if (iter_ms) iter_ms[it] = (omp_get_wtime() - t0) * 1e3;
    if (dc_out) dc_out[it] = dc;
    if (l1_out) l1_out[it] = l1;
    if (history) memcpy(history + (size_t)it * V, r, (size_t)V * sizeof(double));
  }
  memcpy(ranks, r, (size_t)V * sizeof(double));
  free(c);
  free(rn);
  free(r);
  return 0;
}

/* Flag constants, exported so a test can check they equal the ABI's PR_VF_*. */
uint32_t orc_flag_bits(void) {
  return ORC_VF_KEY | (ORC_VF_SINK << 8) | (ORC_VF_NOLINK << 16) | (ORC_VF_INDEG0 << 24);
}
