/*
 * libpagerank_hip -- C ABI of the MI355X (gfx950) PageRank engine that replaces the power
 * iteration of Sparky.java (mayursharma/PageRank-using-Apache-Spark).
 *
 * The reference has no plugin/FFI interface: its hot path is inline Spark transformations in
 * main() (Sparky.java:124-238).  This header is the drop-in boundary a JVM host binds through
 * Panama FFM or JNI.  Each entry point names the reference code it
 * replaces.  Plain pointers and sizes only; every function returns PR_OK (0) or a negative
 * PR_ERR_* code with a thread-local message in pr_last_error(); nothing throws across the ABI.
 *
 * Ownership: pointer inputs are caller-owned and borrowed only for the duration of the call.
 * Device memory is owned by the library and released by pr_graph_destroy().  Outputs are
 * caller-allocated.  A pr_graph handle is not re-entrant; distinct handles may be used from
 * distinct threads.
 *
 * Vertex IDs are dense int32 IDs produced by the host's URL interner (first appearance,
 * src before dst).  Every ID in [0, n_vertices) must appear in the edge list.  dst[i] == -1
 * marks a record without any type=="a" link (Sparky.java:114-118: "(url, null)").
 */
#ifndef PAGERANK_HIP_H
#define PAGERANK_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PR_ABI_VERSION 2

/* ---- status codes ------------------------------------------------------------------- */
#define PR_OK 0
#define PR_ERR_INVALID (-1)  /* bad argument / malformed edge list                        */
#define PR_ERR_HIP (-2)      /* HIP runtime failure                                        */
#define PR_ERR_OOM (-3)      /* device or host allocation failed                           */
#define PR_ERR_COMM (-4)     /* RCCL failure                                               */
#define PR_ERR_STATE (-5)    /* call not valid in the handle's current state               */
#define PR_ERR_NODEVICE (-6) /* no usable GPU                                              */

/* ---- graph creation flags ------------------------------------------------------------ */
#define PR_DANGLING_LOCAL 0u /* Spark local[N] semantics: D = sink-only vertices (default) */
#define PR_DANGLING_NONE 1u  /* cluster-mode semantics: dangUrls empty on the driver, dc=0 */
#define PR_INPUT_DEVICE 2u   /* src/dst are device pointers on `device` (not host)        */
#define PR_NO_CANONICAL 4u   /* drop the canonical CSR after the build (no export)        */
#define PR_LAYOUT_FUSED 8u   /* force the single-pass layout (default: chosen by size)    */
#define PR_LAYOUT_SPLIT 16u  /* force the per-XCD column-class layout                     */

/* ---- vertex flag bits (pr_graph_export_csr vflags) ---------------------------------- */
#define PR_VF_KEY 1u    /* vertex is a record key / src          Sparky.java:127-135      */
#define PR_VF_SINK 2u   /* target never seen as a record         Sparky.java:146-149      */
#define PR_VF_NOLINK 4u /* record whose only value is null       Sparky.java:114-118      */
#define PR_VF_INDEG0 8u /* no in-link: keeps its old rank as sum Sparky.java:224-225      */

/* ---- pr_graph_info indices ------------------------------------------------------------ */
#define PR_INFO_N_VERTICES 0   /* N = totalUrlCount (Sparky.java:162)                       */
#define PR_INFO_N_EDGES 1      /* E' = distinct edges (Sparky.java:124)                      */
#define PR_INFO_N_SINK 2       /* |D| in local mode (Sparky.java:172-184)                    */
#define PR_INFO_N_NOLINK 3     /* keys without links (their mass leaks)                     */
#define PR_INFO_N_INDEG0 4     /* vertices hit by the subtractByKey quirk                   */
#define PR_INFO_MAX_INDEG 5
#define PR_INFO_LOCAL_ROWS 6   /* rows owned by this part                                   */
#define PR_INFO_LOCAL_EDGES 7  /* in-links owned by this part                               */
#define PR_INFO_PART 8
#define PR_INFO_N_PARTS 9
#define PR_INFO_N_UNITS 10     /* work units of the SpMV launch                             */
#define PR_INFO_N_LONG_ROWS 11 /* rows split across several units                          */
#define PR_INFO_DEVICE_BYTES 12
#define PR_INFO_CLASSES 13     /* column classes of the layout (1 = fused single pass)     */
#define PR_INFO_XCHG_SEND 14   /* doubles this part sends per iteration (P > 1)           */
#define PR_INFO_XCHG_RECV 15   /* doubles this part receives per iteration (P > 1)        */
#define PR_INFO_PARTIAL_SLOTS 16 /* (row, column class) segment sums of the split layout     */
#define PR_INFO_HOT_SLOTS 17   /* LDS hot-set contributions per class (split layout)        */
#define PR_INFO_EPILOGUE 18    /* 0 fused units, 3 grouped (split)                           */
#define PR_INFO_GATHER_EST 19  /* bytes of the part's expected gather space (class policy)   */
#define PR_INFO_WALK_GROUPS 20 /* epilogue groups (8 x 64 rows) that walk their rows' own slots */
#define PR_INFO_LAYOUT 21      /* 0 fused, 1 split (column classes + partial slots)          */
#define PR_INFO_HOT_COVER 22   /* in-links read from the LDS hot sets, parts per million      */
#define PR_INFO_CODE_BITS 23   /* bits per in-link of the split layout's entry codes: 20 / 24 compact, 32 */
#define PR_INFO_COUNT 24

/* ---- pr_get_stats indices ------------------------------------------------------------- */
#define PR_STAT_ITERS 0          /* iterations run since the last reset                     */
#define PR_STAT_LAST_DC 1        /* danglingContrib used by the last iteration              */
#define PR_STAT_LAST_L1 2        /* sum |r_k - r_{k-1}| of the last iteration                */
#define PR_STAT_SPMV_MS_MEAN 3   /* mean HIP-event time of one SpMV pass, kernels only: exchange waits excluded (timing on);
                                    one part: the whole iteration (k_finalize included), one
                                    interval per pr_step call with no event between kernels */
#define PR_STAT_SPMV_LAUNCHES 4  /* SpMV passes timed */
#define PR_STAT_ITER_MS_MEAN 5   /* mean HIP-event time of a whole iteration, its exchange
                                    included (timing on)                                    */
#define PR_STAT_BUILD_MS 6       /* wall time of the graph build                            */
#define PR_STAT_EXCHANGE_MS_MEAN 7 /* mean time of the RCCL exchange (parts > 1)            */
#define PR_STAT_COUNT 8

typedef struct pr_graph pr_graph;

/* Per-iteration callback (runs on the calling thread between iterations).
 * ranks_or_null: V doubles in original-ID order when PR_CB_RANKS is set (else NULL);
 * for a part, only the part's own vertices are written, the rest hold the previous content. */
typedef void (*pr_iter_cb)(int32_t iter, const double *ranks_or_null, double dangling_sum,
                           double l1_delta, double ms, void *user);
#define PR_CB_RANKS 1u

int pr_abi_version(void);
const char *pr_last_error(void);
int pr_device_count(int32_t *out);

/* Graph construction: replaces Sparky.java:124-184 (distinct/groupByKey, key broadcast,
 * sink completion, union/count, dangling fixup).  Builds the canonical in-link CSR on the
 * GPU (radix sort + dedupe) and the internal degree-ordered layout used by the iteration.
 * src/dst: n_edges raw interned edges (duplicates and self-loops allowed, dst = -1 for a
 * record without links).  Host pointers unless PR_INPUT_DEVICE. */
int pr_graph_create(int32_t device, int32_t n_vertices, int64_t n_edges, const int32_t *src,
                    const int32_t *dst, uint32_t flags, pr_graph **out);

/* The same, keeping only the rows of `part` out of `n_parts` (1D row partition for one
 * process per GPU; 1 <= n_parts <= 64).  Every part must be created from the same edge list;
 * the part also derives which contributions it exchanges with every peer. */
int pr_graph_create_part(int32_t device, int32_t part, int32_t n_parts, int32_t n_vertices,
                         int64_t n_edges, const int32_t *src, const int32_t *dst, uint32_t flags,
                         pr_graph **out);

/* The same with build options: n_options (key, value) pairs of int64 in `options` (may be NULL
 * when n_options is 0).  They tune the layout (A/B, tests); results do not depend on them beyond
 * summation order.  An unknown key or an out-of-range value fails with PR_ERR_INVALID.  The library
 * reads no environment variables: every choice is an explicit option. */
#define PR_BOPT_CLASSES 1     /* column classes of the split layout: 0 (size policy), 8, 16, 32, 64, 128 */
#define PR_BOPT_HOT_SLOTS 2   /* LDS hot-set slots per class: -1 (default 18429) or 0..18429            */
#define PR_BOPT_EXCHANGE 3    /* P > 1: 0 per-peer runs (default), 1 whole-slice all-gather (all parts alike) */
#define PR_BOPT_XCHG_CHUNKS 4 /* P > 1: 1 = the overlapped exchange from the start (PR_OPT_XCHG_CHUNKS) */
#define PR_BOPT_HOT_RESERVE 5 /* CUs per XCD the heavy SpMV kernel leaves free, 0..3 (PR_OPT_HOT_RESERVE) */
#define PR_BOPT_EPI_WALK 6    /* split layout: 1 (default) per-row walk of sparse epilogue groups, 0 never */
#define PR_BOPT_EPI_NARROW 7  /* split layout: -1 auto (default), 0 four-wave, 1 one-wave epilogue workgroups */
#define PR_BOPT_CODES 8       /* split layout: -1 (default) compact entry codes where they fit (P = 1: 2.5 bytes
                                 for class regions < 2^19 positions, 3 bytes < 2^20; P = 2..8: piece codes,
                                 2.5 / 3 bytes when hot slots + a class's pieces < 2^19 / 2^20), 0 always
                                 4-byte codes; same sums either way (PR_INFO code_bits: 20 / 24 / 32) */
#define PR_BOPT_PACK_FUSED 9  /* P > 1 (per-peer runs, split layout): 1 (default) the epilogue writes the
                                 contributions every peer reads straight into the send runs, 0 a separate
                                 pack kernel gathers them after the pass; same values either way */
#define PR_BOPT_XCHG_SDMA 10  /* group path (pr_group_*, P > 1 per-peer runs): 0 (default) the runs move by
                                 device copies (ROCclr blit kernels on the CUs), 1 by the copy engines
                                 (hipMemcpyDeviceToDeviceNoCU), which leave k_spmv_hot every CU */
#define PR_BOPT_EPI_ORDER 11  /* split layout: the epilogue's dispatch order, -1 (default) auto: 2 for a
                                 part of a row partition (n_parts > 1), 0 for one part; 0 row order, 1 runs
                                 of 8 consecutive groups heaviest first (most partial slots; within each
                                 exchange chunk when the epilogue runs chunk by chunk), 2 single groups
                                 heaviest first; same sums either way */
int pr_graph_create_ex(int32_t device, int32_t part, int32_t n_parts, int32_t n_vertices, int64_t n_edges,
                       const int32_t *src, const int32_t *dst, uint32_t flags, const int64_t *options,
                       int32_t n_options, pr_graph **out);

/* info[i] for i < min(n_info, PR_INFO_COUNT). */
int pr_graph_info(const pr_graph *g, int64_t *info, int32_t n_info);

/* Canonical CSR (rows = dst, columns = src ascending, deduplicated) in original IDs, for
 * bit-exact tests.  row_ptr[V+1], col_idx[E'], out_deg[V], vflags[V]; any may be NULL. */
int pr_graph_export_csr(const pr_graph *g, int64_t *row_ptr, int32_t *col_idx, int32_t *out_deg,
                        uint8_t *vflags);

/* Whole job: replaces Sparky.java:164-238.  Resets ranks to init_ranks (NULL = 1.0 for every
 * vertex, Sparky.java:165-170), runs `iterations` steps of
 * r' = teleport + damping * (S + dc / N) and copies the final ranks (original-ID order, V
 * doubles) to ranks_out (may be NULL).  cb (may be NULL) is called after every iteration. */
int pr_run(pr_graph *g, int32_t iterations, double teleport, double damping,
           const double *init_ranks, double *ranks_out, pr_iter_cb cb, uint32_t cb_flags,
           void *user);

/* Lower-level stepping (resume from saved ranks, benchmarking).  pr_step enqueues work on
 * the library's stream and returns; pr_sync waits for it.  init_ranks (pr_run, pr_reset,
 * pr_group_reset): NULL (every rank 1.0, Sparky.java:165-170) or V doubles in original-ID
 * order; the library reads exactly V of them. */
int pr_reset(pr_graph *g, double teleport, double damping, const double *init_ranks);
int pr_step(pr_graph *g, int32_t iterations);
int pr_sync(pr_graph *g);
int pr_get_ranks(pr_graph *g, double *ranks_out);
int pr_set_timing(pr_graph *g, int32_t enable);
int pr_get_stats(pr_graph *g, double *stats, int32_t n_stats);

/* Execution options (no effect on results; A/B and tuning).  PR_OPT_XCHG_CHUNKS: 1 = the
 * exchange of a part with peers travels in one chunk per SpMV phase and the next iteration's
 * phase c waits only for chunk c (overlap), 0 = whole runs (the default; PR_BOPT_XCHG_CHUNKS sets
 * it at build).  With RCCL every rank must make the same call (it is collective: the ranks check
 * that they agree, so a mismatch fails instead of hanging); in a group, set every part alike. */
#define PR_OPT_XCHG_CHUNKS 1
/* PR_OPT_HOT_RESERVE: CUs per XCD that the heavy SpMV kernel leaves free (0..3, default 0), for
 * the overlapped exchange's transfer kernels, which cannot share a CU with it (LDS, registers). */
#define PR_OPT_HOT_RESERVE 2
/* PR_OPT_XCHG_IPC (RCCL path, ranks on one node): 1 = every rank pulls the runs it reads straight
 * out of its peers' send buffers (IPC-mapped) with the copy engines, ordered by interprocess
 * events, so no transfer kernel takes a CU from the SpMV; 0 = RCCL send/recv (the default);
 * 2 = as 1, and the epilogue runs chunk by chunk, publishing each chunk's runs as soon as they are
 * written, so (with PR_OPT_XCHG_CHUNKS) a peer's pull of chunk c overlaps this rank's epilogue of
 * the later chunks (the split layout's fused pack with several chunks; otherwise as 1).
 * Collective like PR_OPT_XCHG_CHUNKS (which it combines with): every rank must pass the same value
 * (ranks that disagree all fail with PR_ERR_STATE, nothing changed); the first enable maps the
 * peers' buffers and fails with PR_ERR_COMM on every rank if any rank cannot. */
#define PR_OPT_XCHG_IPC 3
/* PR_OPT_XCHG_IPC_BLIT: how this rank's IPC pulls move the bytes: 0 = the copy engines
 * (hipMemcpyDeviceToDeviceNoCU, the default: no CU taken from the SpMV, but ~60 GB/s per engine),
 * 1 = the runtime's blit kernel on the CUs (link speed; it competes with the SpMV for CUs).  Local
 * to the rank (not collective); no effect on results. */
#define PR_OPT_XCHG_IPC_BLIT 4
int pr_set_option(pr_graph *g, int32_t option, int64_t value);

/* Multi-process (one process per GPU): rank 0 creates an id, the host ships the 128 bytes
 * to every rank (any channel), every rank attaches it to its part.  Once per iteration each
 * part sends every peer exactly the contributions (and the two dangling/L1 slots) that the
 * peer's in-links read, with grouped RCCL ncclSend/ncclRecv over xGMI (PR_BOPT_EXCHANGE = 1:
 * one ncclAllGather of whole slices instead).  Attach cross-checks the per-peer run lengths. */
#define PR_COMM_ID_BYTES 128
int pr_comm_unique_id(uint8_t *id_out);
int pr_graph_attach_comm(pr_graph *g, int32_t rank, int32_t n_ranks, const uint8_t *id);

/* Single process, one host thread, n_parts parts (one per GPU -- or several on one GPU): the
 * parts exchange contributions by device-to-device copies (peer copies over xGMI between GPUs)
 * instead of RCCL.  parts[p] must be part p of n_parts, created from the same edge list.
 * Ranks: pr_get_ranks on every part (each fills its own vertices). */
int pr_group_reset(pr_graph *const *parts, int32_t n_parts, double teleport, double damping,
                   const double *init_ranks);
int pr_group_step(pr_graph *const *parts, int32_t n_parts, int32_t iterations);
int pr_group_sync(pr_graph *const *parts, int32_t n_parts);

void pr_graph_destroy(pr_graph *g);

/* ---- synthetic inputs and device-side interning (benchmark front-end) ----------------- */
/* R-MAT (Graph500 parameters a,b,c, d = 1-a-b-c), n_edges edges over 2^scale labels, labels
 * scrambled by a seeded bijection.  d_src/d_dst: device arrays of n_edges int32. */
int pr_gen_rmat(int32_t device, int32_t scale, int64_t n_edges, double a, double b, double c,
                uint64_t seed, int32_t *d_src, int32_t *d_dst);
/* Uniform Erdos-Renyi G(n, m): src, dst uniform over 2^scale labels. */
int pr_gen_er(int32_t device, int32_t scale, int64_t n_edges, uint64_t seed, int32_t *d_src,
              int32_t *d_dst);
/* Chung-Lu graph with power-law weights (the LiveJournal- and Twitter-shaped
 * configs): n_edges edges whose source rank follows w(r) ~ (r + v0_out)^(-1/(gamma_out-1)) over
 * ranks [0, src_frac * n_labels) and whose target rank follows the same law with gamma_in, v0_in
 * over [0, n_labels); then n_nolink records (label, -1) for the ranks just past the source range
 * (keys without links).  Ranks map to labels by a seeded bijection of [0, n_labels).
 * d_src/d_dst: device arrays of n_edges + n_nolink int32. */
int pr_gen_chunglu(int32_t device, int32_t n_labels, int64_t n_edges, double gamma_out, double v0_out,
                   double gamma_in, double v0_in, double src_frac, int64_t n_nolink, uint64_t seed,
                   int32_t *d_src, int32_t *d_dst);
/* Relabel raw labels in [0, label_bound) to dense IDs in first-appearance order (src before
 * dst, edge by edge) -- the same mapping the host URL interner produces -- in place.
 * dst == -1 entries are kept.  *n_vertices_out = number of distinct labels. */
int pr_intern_device(int32_t device, int64_t n_edges, int32_t label_bound, int32_t *d_src,
                     int32_t *d_dst, int32_t *n_vertices_out);

#ifdef __cplusplus
}
#endif

#endif /* PAGERANK_HIP_H */
