// GPU work planner of the split layout (pr_plan.hip).
#pragma once

#include <vector>

#include "pr_internal.h"

namespace pr {

// Usage: segments() -> (caller reads cseg, picks the epilogue) -> block_bases() -> units_plan().
struct SplitPlanner {
  // after segments(): slot boundaries per class (cseg[x] = first slot of class x = poff[x]),
  // and the per-row class masks (ceil(C / 32) words per row)
  std::vector<int64_t> cseg;
  DevBuf rmask;
  // after block_bases(): cbase[(nblk + 1) * C], absolute or class-local first slots
  DevBuf cbase;
  // after units_plan(): wave units (+ one empty unit), their first column entry and real size,
  // per class the first unit (ucum, kMaxClasses + 1 entries), long segments (absolute slot,
  // first piece; seg_p0[n_long] = n_pieces), and the padded entry count
  DevBuf units, src_off, n_real, seg_slot, seg_p0;
  std::vector<int64_t> ucum;
  int64_t n_units = 0, n_pieces = 0, n_long = 0, entries = 0;

  // Segments of the keys sorted by (class << (brow + bg)) | (row << bg) | gather position;
  // marks every segment's last entry in col (bit 31).
  int segments(const uint64_t *keys, int64_t lm, int bg, int brow, int C, int64_t R, int32_t *col, hipStream_t s);
  int block_bases(bool absolute, hipStream_t s);
  int units_plan(hipStream_t s);
  int64_t n_segments() const { return nseg_; }

 private:
  int C_ = 1;
  int64_t nblk_ = 0, nseg_ = 0;
  DevBuf seg_beg_, seg_row_, cseg_dev_;
};

}  // namespace pr
