// The pr_graph handle: device-resident graph of one part plus iteration state.
//
// HBM layout of one part (DESIGN.md "Data layout"):
//   internal vertex order   vertices sorted by (out-degree desc, original ID asc); sorted index
//                           i is owned by part i % P as local rank j = i / P.  Hot sources (high
//                           out-degree = most-gathered contributions) sit together at the front.
//   slice                   S_pad doubles per part: the contributions c = r/d of its rows, then
//                           two slots {dangling partial, L1 partial}.
//   gather space (cbuf)     what this part's in-links read: P slices side by side (P = 1,
//                           PR_BOPT_EXCHANGE = 1), or - the default for P > 1 - this part's
//                           slice followed by the runs it receives from every peer (only the
//                           sources of its own in-links; pr_exchange.hip).  Double-buffered.
//   rowinfo uint32[R]         out-degree | kRowSink (in D) | kRowIndeg0 | kRowHole
//   r       fp64[R]           ranks, updated in place
//
// Column classes (C = 8..64 once the whole gather space passes 4 MiB -- the fewest whose class
// region of the part's expected gather space is <= 4 MB -- else C = 1): local rank j -> class x = j % C, row
// L = x*Q_pad + j/C (also its position in the slice).  Split layout (C > 1): every row's in-links
// are split by the class of their source; each non-empty (row, class) pair is a segment with one
// slot of a class-dense partial array.  Class-x wave units run on XCD x % 8, one class after
// another (phased), so its L2 caches only class-x sources; they address either the gather space
// or the class's LDS hot set (the first Kp rows of every part's class-x region; pr_internal.h
// HotGeom, positions from the hpos table).  k_epilogue_grp adds a row's segment sums in class
// order.  Fused layout (C = 1, small graphs): rowptr/colp CSR with 256-thread units and the
// update fused into the same kernel (pr_spmv.h k_spmv_units).
#pragma once

#include <rccl/rccl.h>

#include <vector>

#include "pr_internal.h"

namespace pr {
struct IpcState;  // pr_ipc.hip
}

// Build options (include/pagerank_hip.h PR_BOPT_*): the library reads no environment variables.
struct pr_build_opts {
  int classes = 0;       // 0: the size policy
  int hot_slots = -1;    // -1: kHotSlotsDefault
  bool allgather = false;
  bool xchg_chunks = false;
  int hot_reserve = 0;
  bool epi_walk = true;
  int epi_narrow = -1;   // -1: by the share of walking groups
  int codes = -1;        // -1: compact codes where they fit (P = 1), 0: 32-bit codes
  bool pack_fused = true;  // P > 1: the epilogue writes the send runs (no pack kernel)
  bool xchg_sdma = false;  // group path: runs move on the copy engines (hipMemcpyDeviceToDeviceNoCU)
  int epi_order = -1;      // epilogue dispatch order (PR_BOPT_EPI_ORDER): -1 auto, 0 rows, 1 runs of 8 groups, 2 groups
};

struct pr_graph {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t flags = 0;
  pr_build_opts opts;

  int32_t V = 0;          // N = totalUrlCount
  int64_t E_dedup = 0;    // E'
  int part = 0, nparts = 1;
  int64_t n_local = 0;      // rows owned (without holes)
  int64_t n_rows = 0;       // C * Q_pad local rows (with holes)
  int layout = 0;           // pr::kLayoutFused / kLayoutSplit
  int C = 1;                // column classes (split layout; 1 otherwise)
  int64_t gather_est = 0;   // expected gather-space bytes the class count was chosen from
  int64_t Q_pad = 0;        // rows per class region
  int64_t n_local_max = 0;  // ceil(V / P)
  int64_t S_pad = 0;        // doubles per gather slice
  int64_t local_nnz = 0;

  int64_t n_sink = 0, n_nolink = 0, n_indeg0 = 0, max_indeg = 0;
  int64_t n_units = 0, n_long = 0, n_pieces = 0;
  double build_ms = 0.0;

  // canonical CSR in original IDs (kept unless PR_NO_CANONICAL)
  pr::DevBuf canon_rowptr, canon_col, canon_deg, canon_vflags;
  bool has_canonical = false;

  // part layout
  pr::DevBuf rowptr, col, colp, rowinfo, r;
  // split layout (C > 1): wave units per class (hunits[hucum[x], hucum[x+1])), their entry codes
  // and lane metadata; per class x the partial sums of its segments at partial[poff[x] + slot];
  // per row the mask of classes with in-links (rmask) and per class the slot of the first
  // segment of every 64-row block (cbase[blk][x]); long segments: pieces reduced in order into
  // partial[seg_slot[q]]; hpos[x * P*Kp + i]: gather position of LDS hot slot 1 + i of class x
  pr::DevBuf colh, hunits, hucum, poff, partial, rmask, cbase, seg_slot, seg_p0, hpos;
  // entry code format (pr_internal.h): kCodeU32 (colh = u32 codes), kCodeC24 (as C20 with a u64
  // side word and 4 high bits per entry) or kCodeC20 (colh = u16 low
  // index bits, cside = one u32 of end marks and high bits per 8 entries); kCodeC20P / kCodeC24P
  // at P > 1 (the same streams, indices into a class's pieces; ptab maps them back)
  int code = pr::kCodeU32;
  pr::DevBuf cside;
  pr::DevBuf ptab;  // piece codes (kCodeC20P / kCodeC24P): per class kPieceTblWords gather deltas
  int ep_blocks = 0;
  pr::ClassGeom geo{};
  pr::HotGeom hot{};
  int hot_grid = 0;       // workgroups of k_spmv_hot (a multiple of C: one per CU)
  int hot_grid_full = 0;  // the same without reserved CUs (PR_OPT_HOT_RESERVE)
  // per-row walk in k_epilogue_grp (PR_BOPT_EPI_WALK): per group the first of its u16 slot
  // positions in epos, or -1 for the class loop (eoff, i64)
  bool epi_walk = false;
  bool epi_narrow = false;  // one-wave epilogue workgroups (PR_BOPT_EPI_NARROW; default: many walking groups)
  int64_t n_walk_groups = 0;
  pr::DevBuf eoff, epos;
  // dispatch order of the epilogue groups (PR_BOPT_EPI_ORDER): epi_ord[k] = the group the k-th
  // wave takes, heaviest first; [0, ngrp) for the whole pass, [ngrp, 2 ngrp) sorted within each
  // exchange chunk's group range (the per-chunk epilogue of PR_OPT_XCHG_IPC = 2)
  pr::DevBuf epi_ord;
  int64_t n_hunits = 0, n_segs = 0, nblk = 0, n_slots = 0;
  int64_t hot_cover_ppm = 0;  // in-links whose source is in a class's hot set (layout policy input)
  pr::DevBuf cbuf[2];
  pr::DevBuf units, unit_part;
  pr::DevBuf lr_row, lr_p0, piece_part;
  pr::DevBuf fin_part, fin_counter;
  pr::DevBuf reset_part;
  int fin_blocks = 0;
  int reset_blocks = 0;
  std::vector<int32_t> orig_of_local;  // host copy: local row -> original ID

  // run state
  double teleport = 0.15, damping = 0.85;
  int cur = 0;  // cbuf[cur] holds the contributions of the current ranks
  int64_t iters_done = 0;
  bool ready = false;  // pr_reset was called

  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  // indices into ev_pool; spmv_ev holds one interval per pass, or one per hot phase (+ the rest of
  // the pass) when the overlapped exchange gates the phases, or (one part) one per pr_step call
  // covering all its iterations: spmv_passes passes in all; iter_ev's intervals cover iter_timed
  // iterations
  std::vector<std::pair<int, int>> spmv_ev, iter_ev, xchg_ev;
  int64_t spmv_passes = 0, iter_timed = 0;
  size_t ev_next = 0;
  // ev_pool index of an event recorded on `stream` with nothing enqueued after it yet, which the
  // next interval may start from instead of recording its own (-1: none); every record is a
  // marker packet of ~5 us between kernels (R-MAT s20: 4 per iteration were 28 % of it)
  int ev_start_hint = -1;

  // gather space (doubles per cbuf): P slices side by side (P = 1, PR_BOPT_EXCHANGE = 1), or
  // compacted: this part's slice, then the runs received from every peer in peer order
  int64_t gsize = 0;
  int64_t own_off = 0;  // this part's slice in the gather space
  pr::SlotPos slots{};  // every part's slot pair in the gather space
  // exchange (P > 1, pr_exchange.hip): positions of this part's slice sent to every peer (runs
  // in peer order, each closed by the two slots), run offsets of what it sends / receives
  // (received runs land at S_pad + x_roff[p]), and the double-buffered packed send runs
  pr::DevBuf x_send, x_sbuf;
  std::vector<int64_t> x_soff, x_roff;
  bool x_allgather = false;  // PR_BOPT_EXCHANGE = 1: whole slices instead
  // Overlapped exchange (P > 1, split layout, phased k_spmv_hot): every peer's run is sent in
  // n_xc chunks on xstream, chunk c = its positions in the class regions of hot phase c (classes
  // [8c, 8c + 8)), the last chunk also carrying the two slots (a run is sorted by position, so
  // the chunks are consecutive pieces of it).  x_sch / x_rch[peer * (n_xc + 1) + c]: chunk starts
  // within the peer's send / receive run.  x_ev[c] is recorded after chunk c; while x_pending,
  // the next iteration's phase c waits for x_ev[c] only (pr_iter.hip), so the transfer of the
  // later classes overlaps the SpMV of the earlier ones.
  int n_xc = 1;
  // whether the chunks travel separately (PR_BOPT_XCHG_CHUNKS at build, pr_set_option later);
  // otherwise whole runs, and the next iteration waits for all of them
  bool x_chunked = false;
  std::vector<int64_t> x_sch, x_rch;
  hipStream_t xstream = nullptr;
  std::vector<hipEvent_t> x_ev;
  hipEvent_t x_pack_ev = nullptr;
  bool x_pending = false;
  // Fused pack (PR_BOPT_PACK_FUSED, split layout, per-peer runs, P <= 8): per local row the peers
  // that read it (x_pmask, bit q), per 64-row block and peer the index of the block's first entry
  // in that peer's send run (x_sbase[blk * P + q]); the epilogue stores c' there directly and
  // k_finalize writes the two slots at every run's end.  x_packed: the gather buffer whose send
  // runs the last epilogue already wrote (-1: none; the exchange then runs k_pack).
  bool x_fused = false;
  pr::DevBuf x_pmask, x_sbase;
  int x_packed = -1;

  // CU-free transport of the RCCL path (PR_OPT_XCHG_IPC, pr_ipc.hip): every rank pulls its runs out
  // of its peers' IPC-mapped send buffers with the copy engines
  pr::IpcState *ipc = nullptr;  // mapped on first use, kept until destroy
  bool x_ipc = false;           // exchanges use it
  // PR_OPT_XCHG_IPC = 2: the epilogue runs chunk by chunk and publishes each chunk's send runs as
  // soon as they are written (per-chunk sent records, pr_ipc_protocol.h), so the peers' pulls of
  // chunk c overlap this rank's epilogue of the later chunks
  bool x_ipc_early = false;
  // PR_OPT_XCHG_IPC_BLIT: the pulls run as the runtime's blit kernel (CUs, link speed) instead of
  // on the copy engines (no CU, ~60 GB/s per engine, profiles/r05/copy_engines.log)
  bool x_ipc_blit = false;
  // recorded on the compute stream when the gather buffer the next exchange fills is no longer read
  // (the start of an iteration / reset): the IPC copy streams wait for it, not for the whole pass
  hipEvent_t x_free_ev = nullptr;

  // RCCL (one process per GPU)
  ncclComm_t comm = nullptr;
  int comm_rank = 0, comm_size = 1;
  // device scratch of the library's small collectives (the IPC set-up's record all-gather, the
  // agreement all-reduces), allocated before the communicator: no rank can fail to take part in a
  // collective for want of a buffer
  pr::DevBuf comm_scratch;
  // single-process group (pr_group_*): the group performs the exchange by device copies
  bool grouped = false;
  hipEvent_t xev = nullptr;

  size_t device_bytes() const;
};

namespace pr {
constexpr size_t kCommScratchBytes = 256 << 10;
int build_graph(pr_graph *g, int64_t n_edges, const int32_t *src, const int32_t *dst);
int iter_reset(pr_graph *g, const double *init_ranks_host);
int plan_epi_walk(pr_graph *g);  // per-row walk of sparse epilogue groups (after rmask/cbase)
int plan_epi_order(pr_graph *g);  // dispatch order of the epilogue groups (after cbase)
int prepare_hot_kernel();  // lets k_spmv_hot use up to 160 KiB of dynamic LDS (current device)
// the heavy-row pass (k_spmv_hot) on g's stream, hot phases [ph0, ph1) (-1: all)
int launch_hot(pr_graph *g, int in_buf, int ph0 = 0, int ph1 = -1);
int join_exchange(pr_graph *g);  // g's stream waits for a pending overlapped exchange
// x_chunked from the build option (1: the overlapped exchange; 0: whole runs, the next iteration
// waits for all of them).  Off by default: the transfers are kernels (RCCL, blit copies) that
// compete with k_spmv_hot for CUs -- k_spmv_hot takes a CU's whole LDS, so the two cannot share
// one -- and on one GPU the chunked group ran 8 % slower.
void set_exchange_chunking(pr_graph *g);
int n_hot_phases(const pr_graph *g);
// k_spmv_hot leaves `per_xcd` CUs of every XCD free (phased schedule only: its grid need only be
// a multiple of the XCD count)
int set_hot_reserve(pr_graph *g, int per_xcd);
int iter_step(pr_graph *g, int32_t iterations);
int iter_compute(pr_graph *g);  // one iteration without the exchange; flips g->cur
// timing (every part's g->timing): per receiving part one xchg_ev interval, its copies on xstream
int group_exchange(pr_graph *const *parts, int n, int buf);
// Exchange lists and the gather-space geometry (gsize, own_off, slots); *cmap receives the
// global -> compacted position map (-1: not read by this part) when the space is compacted.
int build_exchange(pr_graph *g, const uint64_t *ukeys, int64_t m, int b, uint64_t mask, const int32_t *rank_of,
                   const int32_t *gpos, DevBuf *cmap);
int exchange(pr_graph *g, int buf, hipEvent_t ev_a = nullptr, hipEvent_t ev_b = nullptr);
double *send_runs(const pr_graph *g, int buf);  // the packed send runs paired with gather buffer buf
int verify_exchange(pr_graph *g);  // after ncclCommInitRank
int read_slots(pr_graph *g, int buf, double *dc, double *l1);
// IPC transport (pr_ipc.hip): collective switch; the reuse wait before the send runs of buf are
// written (no-op unless x_ipc); the exchange itself; unmapping at destroy
int set_exchange_ipc(pr_graph *g, int mode);  // 0: RCCL, 1: IPC, 2: IPC with per-chunk publication
int ipc_send_runs_free(pr_graph *g, int buf);
bool ipc_early(const pr_graph *g);               // the epilogue publishes chunk by chunk
int ipc_chunk_sent(pr_graph *g, int buf, int c);  // the epilogue wrote the runs of chunk c of buf
int exchange_ipc(pr_graph *g, int buf, hipEvent_t ev_a, hipEvent_t ev_b);
void ipc_destroy(pr_graph *g);
bool stream_idle_within(hipStream_t s, double seconds);  // host poll of hipStreamQuery with a deadline
hipEvent_t next_event(pr_graph *g);  // the next timing event of g's pool (nullptr: creation failed)
int time_mark(pr_graph *g, hipStream_t s, int *index);  // records one on s; *index into ev_pool
}  // namespace pr
