// Internal declarations shared by the libpagerank_hip translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <type_traits>
#include <vector>

#include "pagerank_hip.h"
#include "pr_pieces.h"

namespace pr {

// ---- error plumbing ---------------------------------------------------------------------
void set_error(const std::string &msg);
struct Status {
  int code = PR_OK;
  bool ok() const { return code == PR_OK; }
};
int fail(int code, const std::string &msg);

#define PR_HIP(call)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (call);                                                                   \
    if (e_ != hipSuccess)                                                                     \
      return ::pr::fail(e_ == hipErrorOutOfMemory ? PR_ERR_OOM : PR_ERR_HIP,                  \
                        std::string(#call) + ": " + hipGetErrorString(e_));                   \
  } while (0)

#define PR_TRY(expr)                                                                          \
  do {                                                                                        \
    int rc_ = (expr);                                                                         \
    if (rc_ != PR_OK) return rc_;                                                             \
  } while (0)

// ---- device buffer (owning) ---------------------------------------------------------------
struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  DevBuf(DevBuf &&o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  DevBuf &operator=(DevBuf &&o) noexcept {
    if (this != &o) { reset(); p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0; }
    return *this;
  }
  ~DevBuf() { reset(); }
  int alloc(size_t n);  // frees any previous allocation
  void reset();
  template <class T> T *as() const { return static_cast<T *>(p); }
};

// ---- primitives (pr_sort.hip) ---------------------------------------------------------------
// Stable LSD radix sort of n u64 keys on bits [begin_bit, end_bit).  `tmp` must hold n keys.
// The sorted result is left in `keys`.
int radix_sort_u64(uint64_t *keys, uint64_t *tmp, int64_t n, int begin_bit, int end_bit,
                   hipStream_t s);

// Number of bits needed so that every value in [0, v] fits (v >= 0).
inline int bits_for(uint64_t v) {
  int b = 1;
  while (b < 64 && (uint64_t(1) << b) <= v) ++b;
  return b;
}

inline unsigned grid_for(int64_t n, int threads, unsigned cap = 1u << 20) {
  int64_t g = (n + threads - 1) / threads;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// ---- layouts (pr_graph.h) -----------------------------------------------------------------------
constexpr int kLayoutFused = 0;  // one class, k_spmv_units (gather space <= 4 MiB)
constexpr int kLayoutSplit = 1;  // column classes, LDS hot sets, partial slots (k_spmv_hot + k_epilogue_grp)

// ---- SpMV work plan ------------------------------------------------------------------------
// A unit is one workgroup of the SpMV launch.  STREAM: whole rows [r0, r0+meta) whose in-links
// total n <= kUnitNnz.  PIECE: n <= kUnitNnz in-links of one long row r0; meta = -(piece+1).
// Each unit's gather positions start at colp[8 * p8] (units padded to 32-byte boundaries).
constexpr int kThreads = 256;       // workgroup size of the SpMV kernels (4 waves)
constexpr int kPerThread = 8;       // in-links gathered per thread per unit
constexpr int kUnitNnz = kThreads * kPerThread;  // 2048
constexpr int kUnitRows = 1024;     // max rows per STREAM unit (LDS bound)

struct Unit {
  uint32_t p8;   // padded column offset / 8
  int32_t r0;    // first row (STREAM) or the long row (PIECE)
  int32_t meta;  // rows (>= 0) or -(piece index + 1)
  int32_t n;     // in-links in the unit (low 16 bits) | column class << 16
};
static_assert(sizeof(Unit) == 16, "Unit must stay 16 bytes");
__host__ __device__ inline int unit_n(const Unit &u) { return u.n & 0xFFFF; }
__host__ __device__ inline int unit_cls(const Unit &u) { return u.n >> 16; }

// ---- column classes (pr_graph.h "split" layout) -----------------------------------------------
constexpr int kXcds = 8;                             // XCDs of the MI355X (one L2 each)
constexpr int64_t kL2BytesPerXcd = 4ll << 20;        // class count: a class region should fit one L2
constexpr int kMaxClasses = 128;                     // 8, 16, 32, 64 or 128 (PR_BOPT_CLASSES)
constexpr int kAutoMaxClasses = 64;                  // the most the size policy picks by itself
// per-row class mask (rmask): ceil(C / 32) 32-bit words per row, class x in bit x % 32 of word
// x / 32 (at 64 classes the two words are one little-endian u64)
template <int C> constexpr int mask_words() { return (C + 31) / 32; }
// split once the gather space passes 4 MiB: R-MAT s20 (5.2 MB, L2-resident either way) runs the
// split layout at 8 classes in 0.09 ms/iter against 0.18 ms fused (profiles/r01/configs_ab/s20_*)
constexpr int64_t kSplitMinSliceBytes = 4ll << 20;
// Grouped epilogue (k_epilogue_grp): a wave takes kEpiGroup consecutive 64-row blocks and stages
// their partial sums in an LDS window of kEpiWin slots, class runs a few at a time.
constexpr int kEpiGroup = 8;
#ifndef PR_EPI_WIN
#define PR_EPI_WIN 1024
#endif
constexpr int kEpiWin = PR_EPI_WIN;  // 8 KiB per wave; >= 64 * kEpiGroup + 2 (one class run always fits)
constexpr int kEpiThreads = 256;  // 4 waves, 32.1 KiB of LDS: four workgroups per CU
// narrow grouped epilogue: one-wave workgroups (8.2 KiB of LDS each), so a wave that finishes a
// cheap group frees its window at once -- chosen when a graph has many walking (sparse) groups
constexpr int kEpiThreadsNarrow = 64;  // one wave64
inline bool epi_narrow_ok(int C) { return C <= 64; }  // one-wave workgroups: at most 64 classes
inline int epi_grp_threads(bool narrow) { return narrow ? kEpiThreadsNarrow : kEpiThreads; }
// dynamic LDS of k_epilogue_grp: per wave its window of kEpiWin slots + the zero slot and padding,
// then per wave a double2 for the block sum
inline size_t epi_grp_lds(bool narrow) {
  return sizeof(double) * (size_t)(epi_grp_threads(narrow) / 64) * (kEpiWin + 4);
}

// per-row info word: out-degree | flags
constexpr uint32_t kRowDegMask = (1u << 28) - 1;
constexpr uint32_t kRowSink = 1u << 28;    // in the dangling set D (contributes to dc)
constexpr uint32_t kRowIndeg0 = 1u << 29;  // no in-link: the old rank is the sum
constexpr uint32_t kRowHole = 1u << 30;    // padding row of the class layout

// ---- heavy rows: wave units with an LDS-resident hot set (pr_spmv.h k_spmv_hot) -------------
// A wave unit is one wavefront's work: kWavePT in-link entries per lane, kWaveUnit entries in
// all.  STREAM: whole (row, class) segments of consecutive rows (only non-empty (row, class)
// pairs are segments); PIECE: kWaveUnit entries of one long segment.  Entries are 32-bit codes:
//   bit 31 set    kEntGlobal | byte offset of the contribution in the gather space (< 2 GiB)
//   bit 31 clear  LDS byte address of a hot-set slot; slot 0 (address 0) holds 0.0
//   bit 0         set on the last entry of a segment (both kinds are multiples of 8 otherwise)
// Padding entries are 0 -- also what a range-checked load past the unit returns.  k_spmv_hot
// derives each lane's scan metadata from the end marks (pr_spmv.h derive_meta).
constexpr int kWavePT = 8;
constexpr int kWaveUnit = 64 * kWavePT;  // 512 (wave64)
constexpr int kHotThreads = 1024;        // 16 waves per CU: one workgroup per CU
constexpr uint32_t kEntGlobal = 1u << 31;
constexpr uint32_t kEntZero = 0u;  // LDS slot 0
// Compact entry codes (one part, P = 1; round 3): the codes above cost 4 B per in-link, the
// largest stream of the pass (4.3 GB at R-MAT s26).  At P = 1 every source of a class-x in-link
// lies in the class's region of the slice, [x*Q_pad, (x+1)*Q_pad), and its hot set is the first
// q_load positions of that region, so an entry needs only its region index idx = offset + 1
// (0 = padding, read as 0.0; hot iff idx <= q_load, LDS slot idx).  Per lane group of 8 entries:
//   code16[8]  u16: the low 16 bits of idx (one 16-byte load per lane)
//   side       u32: bits 0-7 the segment-end marks of the 8 entries, bits 8 + 3j .. 10 + 3j the
//              high 3 bits of entry j's idx (one 4-byte load per lane)
// -> 2.5 B per in-link, idx < 2^19 (R-MAT s26: Q_pad = 512640).  Class regions up to 2^20 rows
// (the Twitter shape: Q_pad = 650816) take the 3-byte variant kCodeC24: a u64 side word per lane,
// bits 0-7 the end marks, bits 8 + 4j .. 11 + 4j the high 4 bits of idx (one 8-byte load).  Larger
// class regions keep the 32-bit codes.
//
// Parts of a row partition (P > 1): a class's sources are its region of the own slice plus, for
// every peer, the sub-run of that peer's received run holding the peer's class-x sources (a run is
// sorted by the peer's slice position, so that sub-run is contiguous in the gather space).  The
// *piece* codes kCodeC20P / kCodeC24P (same streams as kCodeC20 / kCodeC24) index a per-class
// virtual space: idx 1..P*Kp = LDS hot slot (as the 32-bit codes' hot entries), idx = P*Kp + 1 + k
// a cold source at virtual index k, where the class's pieces (in part order) start at multiples of
// kPieceAlign.  Gather position = k + tbl[x][k / kPieceAlign]: a per-class table of kPieceTbl
// deltas (plus a 0 sentinel that keeps hot entries' loads out of range), restaged into LDS with
// the hot set.  The hot set gives up kPieceTblSlots slots for it.
constexpr int kCodeU32 = 0;
constexpr int kCodeC20 = 1;
constexpr int kCodeC24 = 2;
constexpr int kCodeC20P = 3;
constexpr int kCodeC24P = 4;
// kC20IdxBits, kC24IdxBits and the piece-table constants: pr_pieces.h
constexpr __host__ __device__ bool code_is_piece(int code) { return code >= kCodeC20P; }
// LDS of k_spmv_hot: the hot set (slot 0 = 0.0, then the hot contributions of every part), one
// more 0.0 slot (where compact cold entries point their LDS read), the workgroup's unit counter,
// then one staging window of kStageSlots segment sums per wave (16 KiB in all; 128 beat 256 by
// ~0.5 % and 64 by ~0.8 % at R-MAT s26, profiles/r01/stage_ab/).
#ifndef PR_STAGE_SLOTS  // A/B builds only (tools/ab_build.sh): the library reads no environment
#define PR_STAGE_SLOTS 128
#endif
constexpr int kStageSlots = PR_STAGE_SLOTS;
constexpr int kHotLdsBytes = 160 * 1024;
constexpr int kHotSlotsMax = (kHotLdsBytes - (kHotThreads / 64) * kStageSlots * 8) / 8 - 3;
constexpr int kHotSlotsDefault = kHotSlotsMax;  // 18429 hot contributions (144 KiB)

// Geometry of the split layout of one part, passed to kernels by value.
struct ClassGeom {
  int C;
  int64_t Q_pad, S_pad;
};

// Gather positions of every part's {dangling partial, L1 partial} slot pair (the dangling one;
// L1 follows), in part order.  Passed by value: the kernels read them as scalars.
constexpr int kMaxParts = 64;
struct SlotPos {
  int n;
  int32_t pos[kMaxParts];
};
// Fused pack (pr_graph.h x_fused): where the epilogue stores the contributions the peers read (the
// send runs of the buffer it writes, peer q's run at soff[q]; P = 0: no fused pack), and where
// k_finalize stores the two slots that close every peer's run.
constexpr int kMaxPackParts = 8;
struct PackDst {
  double *sbuf;
  int P, self;
  int64_t soff[kMaxPackParts];
};
struct PackSlots {
  double *sbuf;
  int n;
  int64_t off[kMaxPackParts];
};

// A class's hot set: for every part p, rows [x*Q_pad, + q_load) of p's slice go to LDS slots
// 1 + [p*Kp, p*Kp + q_load); slot 0 holds 0.0.  Their gather positions come from a table (the
// part's gather space is compacted when only some remote positions are received).
struct HotGeom {
  int C, P, Kp, q_load;
  int64_t S_pad, Q_pad;
  int tbl;  // 1: piece codes, the class's piece table follows the staging windows (kPieceTblSlots)
  __host__ __device__ int slots() const { return P * Kp + 1; }
  // slot `slots()` holds 0.0 (compact codes' cold entries read it), slot `slots() + 1` is a
  // control word (the workgroup's unit counter, pr_spmv.h hot_class_units); the staging windows
  // start 16-byte aligned after it
  __host__ __device__ int ctr_slot() const { return slots() + 1; }
  __host__ __device__ int stage_off() const { return (slots() + 3) & ~1; }
  __host__ __device__ int tbl_off() const { return stage_off() + (kHotThreads / 64) * kStageSlots; }
  __host__ __device__ size_t lds_bytes() const {
    return sizeof(double) * ((size_t)tbl_off() + (tbl ? (size_t)kPieceTblSlots : 0));
  }
};

// Host plan over a part's row_ptr: units, their source offsets in the unpadded column array,
// long rows (split into pieces) and the padded column length.
struct UnitPlan {
  std::vector<Unit> units;
  std::vector<int64_t> src_off;  // per unit: first in-link in the unpadded CSR
  std::vector<int32_t> lr_row, lr_p0;
  int64_t n_pieces = 0;
  int64_t padded_len = 0;
};
// Plans rows [row_begin, row_end) (default: all rows); appends to *plan when append is true.
void plan_units(const std::vector<int64_t> &rp, int unit_nnz, int unit_rows, UnitPlan *plan,
                int64_t row_begin = 0, int64_t row_end = -1, bool append = false);
// colp[8*p8 + i] = col[src_off + i] for every unit (padding entries are 0).
int build_padded_cols(const UnitPlan &plan, const int32_t *col, int32_t *colp, hipStream_t s);

}  // namespace pr
