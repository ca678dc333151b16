// Work plan of the split layout, built on the GPU (pr_graph.h).
//
// Input: the part's in-link keys sorted by (column class, local row, gather position) and the
// matching column array.  A *segment* is a run of keys with the same (class, row): one partial
// sum slot, numbered in key order, so the slot of segment k is k itself (class x's slots are
// [cseg[x], cseg[x+1]) and cseg doubles as the partial offsets poff).  From the segments:
//   rmask   per row, bit x when the row has a class-x segment;
//   cbase   per 64-row block and class, the first slot of the class at or after the block (one
//           sentinel block row at the end holds every class's end slot);
//   units   the wave units of k_spmv_hot: consecutive segments of one class while they fit
//           kWaveUnit entries (STREAM), or kWaveUnit-entry pieces of one longer segment (PIECE,
//           summed in piece order by k_seg_reduce).  Packing is greedy over chunks of kPlanChunk
//           segments, one thread per chunk (a unit never crosses a chunk), in two passes: count,
//           host prefix over the chunks, emit.
// Everything but the per-chunk counts and the C + 1 class boundaries stays on the device; the
// previous host planner copied C row-pointer arrays (17 GB at R-MAT s26) to the host.
// Replaces the grouping of Sparky.java:124 (groupByKey) as the kernels consume it.
#include <vector>

#include "pr_compact.h"
#include "pr_device.h"
#include "pr_graph.h"
#include "pr_plan.h"

namespace pr {
namespace {

constexpr int kPlanChunk = 2048;  // segments per greedy chunk

struct SegStart {
  const uint64_t *k;
  int shift;  // (class, row) = key >> shift
  __device__ bool operator()(int64_t i) const { return i == 0 || (k[i] >> shift) != (k[i - 1] >> shift); }
};
struct Index64 {
  __device__ int64_t operator()(int64_t i) const { return i; }
};

// Per segment: its row, the end mark on its last column entry, the row's class bit; the class
// boundaries cseg[x] = first segment of class >= x (cseg[C] = nseg); seg_beg[nseg] = lm.
__global__ void k_seg_info(int64_t nseg, int64_t lm, const uint64_t *__restrict__ keys, int64_t *__restrict__ seg_beg,
                           int bg, int brow, int C, int nw, int32_t *__restrict__ seg_row,
                           int32_t *__restrict__ col, uint32_t *__restrict__ rmask, int64_t *__restrict__ cseg) {
  const uint64_t rowm = (uint64_t(1) << brow) - 1;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k <= nseg; k += (int64_t)gridDim.x * blockDim.x) {
    const int xc = k < nseg ? (int)(keys[seg_beg[k]] >> (bg + brow)) : C;
    const int xp = k > 0 ? (int)(keys[seg_beg[k - 1]] >> (bg + brow)) : -1;
    for (int x = xp + 1; x <= xc; ++x) cseg[x] = k;
    if (k == nseg) {
      seg_beg[nseg] = lm;
      continue;
    }
    const int32_t row = (int32_t)((keys[seg_beg[k]] >> bg) & rowm);
    seg_row[k] = row;
    atomicOr(&rmask[(int64_t)row * nw + (xc >> 5)], 1u << (xc & 31));
    const int64_t last = (k + 1 < nseg ? seg_beg[k + 1] : lm) - 1;  // seg_beg[nseg] may not be written yet
    col[last] |= (int32_t)0x80000000u;  // segment end (moved into the lane metadata by k_unit_meta)
  }
}

// cbase[blk][x] = first slot of class x whose row is >= 64 blk (blk = nblk: the class's end).
__global__ void k_cbase(int64_t nblk, int C, const int64_t *__restrict__ cseg, const int32_t *__restrict__ seg_row,
                        bool absolute, int32_t *__restrict__ cbase) {
  const int64_t n = (nblk + 1) * C;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t blk = t / C;
    const int x = (int)(t - blk * C);
    int64_t lo = cseg[x], hi = cseg[x + 1];
    const int64_t base = lo;
    const int64_t target = blk * kWave;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (seg_row[mid] < target) lo = mid + 1;
      else hi = mid;
    }
    cbase[t] = (int32_t)(absolute ? lo : lo - base);
  }
}

struct Chunk {
  int64_t beg, end;  // segments [beg, end) of one class
  int64_t cls_base;  // cseg[class]: class-local slot = k - cls_base
};
struct ChunkCount {
  int64_t units, pieces, longs, entries;  // entries: padded to kWavePT per unit
};

// The greedy of one chunk (shared by the count and the emit pass).
template <bool EMIT>
__device__ void plan_chunk(const Chunk &ch, const int64_t *__restrict__ seg_beg, ChunkCount *cnt, ChunkCount off,
                           Unit *__restrict__ units, int64_t *__restrict__ src_off, int32_t *__restrict__ n_real,
                           int64_t *__restrict__ seg_slot, int32_t *__restrict__ seg_p0) {
  const int64_t cap = kWaveUnit;
  ChunkCount c{0, 0, 0, 0};
  auto push = [&](int64_t src, int64_t r0, int64_t meta, int64_t n) {
    const int64_t np = (n + kWavePT - 1) / kWavePT * kWavePT;
    if constexpr (EMIT) {
      const int64_t u = off.units + c.units;
      units[u] = Unit{(uint32_t)((off.entries + c.entries) / 8), (int32_t)r0, (int32_t)meta, (int32_t)np};
      src_off[u] = src;
      n_real[u] = (int32_t)n;
    }
    ++c.units;
    c.entries += np;
  };
  int64_t u_r0 = 0, u_src = 0, u_n = 0, u_seg = 0;
  for (int64_t k = ch.beg; k < ch.end; ++k) {
    const int64_t b = seg_beg[k], len = seg_beg[k + 1] - b, slot = k - ch.cls_base;
    if (len > cap) {  // long segment: pieces in order, summed by k_seg_reduce into slot k
      if (u_seg > 0) push(u_src, u_r0, u_seg, u_n);
      u_seg = u_n = 0;
      const int64_t np = (len + cap - 1) / cap;
      const int64_t p0 = off.pieces + c.pieces;
      if constexpr (EMIT) {
        seg_slot[off.longs + c.longs] = k;
        seg_p0[off.longs + c.longs] = (int32_t)p0;
      }
      ++c.longs;
      for (int64_t q = 0; q < np; ++q) push(b + q * cap, slot, -(p0 + q) - 1, min(cap, len - q * cap));
      c.pieces += np;
      continue;
    }
    if (u_seg > 0 && u_n + len > cap) {
      push(u_src, u_r0, u_seg, u_n);
      u_seg = u_n = 0;
    }
    if (u_seg == 0) {
      u_r0 = slot;
      u_src = b;
    }
    u_n += len;
    ++u_seg;
  }
  if (u_seg > 0) push(u_src, u_r0, u_seg, u_n);
  if constexpr (!EMIT) *cnt = c;
}

__global__ void k_plan_count(int64_t n_chunks, const Chunk *__restrict__ chunks, const int64_t *__restrict__ seg_beg,
                             ChunkCount *__restrict__ counts) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n_chunks; q += (int64_t)gridDim.x * blockDim.x)
    plan_chunk<false>(chunks[q], seg_beg, counts + q, ChunkCount{}, nullptr, nullptr, nullptr, nullptr, nullptr);
}

__global__ void k_plan_emit(int64_t n_chunks, const Chunk *__restrict__ chunks, const int64_t *__restrict__ seg_beg,
                            const ChunkCount *__restrict__ offs, Unit *__restrict__ units, int64_t *__restrict__ src_off,
                            int32_t *__restrict__ n_real, int64_t *__restrict__ seg_slot, int32_t *__restrict__ seg_p0) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n_chunks; q += (int64_t)gridDim.x * blockDim.x)
    plan_chunk<true>(chunks[q], seg_beg, nullptr, offs[q], units, src_off, n_real, seg_slot, seg_p0);
}

}  // namespace

int SplitPlanner::segments(const uint64_t *keys, int64_t lm, int bg, int brow, int C, int64_t R, int32_t *col,
                           hipStream_t s) {
  C_ = C;
  nblk_ = (R + kWave - 1) / kWave;
  const int nw = (C + 31) / 32;
  PR_TRY(compact_index(lm, SegStart{keys, bg}, Index64{}, (int64_t *)nullptr, &nseg_, s));
  PR_TRY(seg_beg_.alloc(sizeof(int64_t) * (size_t)(nseg_ + 1)));
  int64_t n2 = 0;
  PR_TRY(compact_index(lm, SegStart{keys, bg}, Index64{}, seg_beg_.as<int64_t>(), &n2, s));
  if (n2 != nseg_) return fail(PR_ERR_STATE, "segment count changed between passes");
  PR_TRY(seg_row_.alloc(sizeof(int32_t) * (size_t)(nseg_ + 1)));
  PR_TRY(rmask.alloc(sizeof(uint32_t) * (size_t)nw * ((size_t)R + 1)));
  PR_HIP(hipMemsetAsync(rmask.p, 0, sizeof(uint32_t) * (size_t)nw * ((size_t)R + 1), s));
  DevBuf dcseg;
  PR_TRY(dcseg.alloc(sizeof(int64_t) * (C + 1)));
  hipLaunchKernelGGL(k_seg_info, dim3(grid_for(nseg_ + 1, 256, 65536)), dim3(256), 0, s, nseg_, lm, keys,
                     seg_beg_.as<int64_t>(), bg, brow, C, nw, seg_row_.as<int32_t>(), col, rmask.as<uint32_t>(),
                     dcseg.as<int64_t>());
  PR_HIP(hipGetLastError());
  cseg.assign(C + 1, 0);
  PR_HIP(hipMemcpyAsync(cseg.data(), dcseg.p, sizeof(int64_t) * (C + 1), hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  cseg_dev_ = std::move(dcseg);
  return PR_OK;
}

int SplitPlanner::block_bases(bool absolute, hipStream_t s) {
  const int64_t n = (nblk_ + 1) * C_;
  PR_TRY(cbase.alloc(sizeof(int32_t) * (size_t)(n + 1)));
  hipLaunchKernelGGL(k_cbase, dim3(grid_for(n, 256, 65536)), dim3(256), 0, s, nblk_, C_, cseg_dev_.as<int64_t>(),
                     seg_row_.as<int32_t>(), absolute, cbase.as<int32_t>());
  PR_HIP(hipGetLastError());
  PR_HIP(hipStreamSynchronize(s));
  seg_row_.reset();
  return PR_OK;
}

int SplitPlanner::units_plan(hipStream_t s) {
  // chunks: kPlanChunk consecutive segments of one class
  std::vector<Chunk> ch;
  std::vector<int64_t> first_chunk(C_ + 1, 0);
  for (int x = 0; x < C_; ++x) {
    first_chunk[x] = (int64_t)ch.size();
    for (int64_t b = cseg[x]; b < cseg[x + 1]; b += kPlanChunk)
      ch.push_back(Chunk{b, std::min<int64_t>(b + kPlanChunk, cseg[x + 1]), cseg[x]});
  }
  first_chunk[C_] = (int64_t)ch.size();
  const int64_t nq = (int64_t)ch.size();
  ucum.assign(kMaxClasses + 1, 0);
  n_units = n_pieces = n_long = entries = 0;
  DevBuf dch, dcnt;
  PR_TRY(dch.alloc(sizeof(Chunk) * (size_t)(nq + 1)));
  PR_TRY(dcnt.alloc(sizeof(ChunkCount) * (size_t)(nq + 1)));
  std::vector<ChunkCount> cnt((size_t)nq), off((size_t)nq);
  if (nq > 0) {
    PR_HIP(hipMemcpyAsync(dch.p, ch.data(), sizeof(Chunk) * nq, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_plan_count, dim3(grid_for(nq, 64, 65536)), dim3(64), 0, s, nq, dch.as<Chunk>(),
                       seg_beg_.as<int64_t>(), dcnt.as<ChunkCount>());
    PR_HIP(hipGetLastError());
    PR_HIP(hipMemcpyAsync(cnt.data(), dcnt.p, sizeof(ChunkCount) * nq, hipMemcpyDeviceToHost, s));
    PR_HIP(hipStreamSynchronize(s));
  }
  ChunkCount acc{0, 0, 0, 0};
  for (int64_t q = 0; q < nq; ++q) {
    off[q] = acc;
    acc.units += cnt[q].units;
    acc.pieces += cnt[q].pieces;
    acc.longs += cnt[q].longs;
    acc.entries += cnt[q].entries;
  }
  for (int x = 0; x <= kMaxClasses; ++x) {
    const int64_t q = first_chunk[std::min(x, C_)];
    ucum[x] = q < nq ? off[q].units : acc.units;
  }
  n_units = acc.units;
  n_pieces = acc.pieces;
  n_long = acc.longs;
  entries = acc.entries;
  PR_TRY(units.alloc(sizeof(Unit) * (size_t)(n_units + 1)));
  PR_HIP(hipMemsetAsync(units.p, 0, sizeof(Unit) * (size_t)(n_units + 1), s));  // unit n_units: the empty unit
  PR_TRY(src_off.alloc(sizeof(int64_t) * (size_t)(n_units + 1)));
  PR_TRY(n_real.alloc(sizeof(int32_t) * (size_t)(n_units + 1)));
  PR_TRY(seg_slot.alloc(sizeof(int64_t) * (size_t)(n_long + 1)));
  PR_TRY(seg_p0.alloc(sizeof(int32_t) * (size_t)(n_long + 1)));
  const int32_t p_end = (int32_t)n_pieces;
  PR_HIP(hipMemcpyAsync(seg_p0.as<int32_t>() + n_long, &p_end, sizeof(int32_t), hipMemcpyHostToDevice, s));
  if (nq > 0) {
    PR_HIP(hipMemcpyAsync(dcnt.p, off.data(), sizeof(ChunkCount) * nq, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_plan_emit, dim3(grid_for(nq, 64, 65536)), dim3(64), 0, s, nq, dch.as<Chunk>(),
                       seg_beg_.as<int64_t>(), dcnt.as<ChunkCount>(), units.as<Unit>(), src_off.as<int64_t>(),
                       n_real.as<int32_t>(), seg_slot.as<int64_t>(), seg_p0.as<int32_t>());
    PR_HIP(hipGetLastError());
  }
  PR_HIP(hipStreamSynchronize(s));
  seg_beg_.reset();
  return PR_OK;
}

}  // namespace pr
