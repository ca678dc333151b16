// Piece codes of a row partition's parts (pr_internal.h kCodeC20P / kCodeC24P): the address
// arithmetic shared by the build (pr_build.hip plan_pieces, k_fill_piece), the hot kernel
// (pr_spmv.h cold_offset) and the CPU test shim (host/pieces_shim.cpp, tests/test_piece_codes_cpu.py).
// Plain C++ with PR_HD qualifiers, so a host compiler builds it without the HIP runtime.
//
// A part's class-x sources are its own class region plus, per peer, the sub-run of that peer's
// received run holding the peer's class-x sources (a *piece*, a contiguous range [g0, g1) of the
// gather space).  The pieces of a class are laid out in part order at kPieceAlign-aligned starts
// of a virtual index space; an entry's code is its LDS hot slot (1 .. nh) or nh + 1 + its virtual
// index, and k_spmv_hot maps a cold code back to a byte offset with one table lookup per
// kPieceAlign-entry block: go = 8 idx - 8 (nh + 1); go += tbl[min(go >> 15, kPieceTbl)].  Hot and
// padding codes wrap to >= 2^31 (the table's sentinel entry is 0), out of range of any gather space,
// so their range-checked loads cost no memory request.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <vector>

#if defined(__HIPCC__)
#define PR_HD __host__ __device__
#else
#define PR_HD
#endif

namespace pr {

constexpr int kC20IdxBits = 19;
constexpr int kC24IdxBits = 20;
constexpr int kPieceShift = 12;
constexpr int kPieceAlign = 1 << kPieceShift;
constexpr int kPieceTbl = (1 << kC24IdxBits) >> kPieceShift;  // 256 blocks cover any 20-bit index
constexpr int kPieceTblWords = kPieceTbl + 2;                 // + the sentinel, rounded to 8 bytes
constexpr int kPieceTblSlots = kPieceTblWords / 2;            // in doubles

// Per class x and part p the piece [lohi[x*P + p], lohi[C*P + x*P + p]) of the gather space ->
// pc[3 (x P + p) + {0, 1, 2}] = {g0, g1, virtual start} (all 0 for an empty piece, which matches
// no position), tbl[x kPieceTblWords + t] = the u32 byte delta of virtual block t (0 beyond the
// class's pieces, the sentinel included), and the largest virtual extent over the classes.
inline int64_t piece_tables(const int32_t *lohi, int C, int P, std::vector<int32_t> *pc, std::vector<int32_t> *tbl) {
  const int64_t np = (int64_t)C * P;
  pc->assign((size_t)(3 * np), 0);
  tbl->assign((size_t)C * kPieceTblWords, 0);
  int64_t vmax = 0;
  for (int x = 0; x < C; ++x) {
    int64_t v = 0;
    for (int p = 0; p < P; ++p) {
      const int64_t i = (int64_t)x * P + p;
      const int32_t g0 = lohi[i], g1 = lohi[np + i];
      int32_t *e = &(*pc)[(size_t)(3 * i)];
      if (g1 <= g0) continue;  // empty piece: matches nothing
      v = (v + kPieceAlign - 1) / kPieceAlign * kPieceAlign;
      e[0] = g0;
      e[1] = g1;
      e[2] = (int32_t)std::min<int64_t>(v, INT32_MAX);
      for (int64_t t = v >> kPieceShift; t <= (v + (g1 - g0) - 1) >> kPieceShift && t < kPieceTbl; ++t)
        (*tbl)[(size_t)(x * kPieceTblWords + t)] = (int32_t)(uint32_t)(8u * (uint32_t)(g0 - (int32_t)v));
      v += g1 - g0;
    }
    vmax = std::max(vmax, v);
  }
  return vmax;
}

// k_fill_piece: the code of the entry whose source sits at gather position `pos` in class x
// (px = pc + 3 x P): its hot slot when it has one, else nh + 1 + its virtual index; *bad is set
// (and 0 returned) when no piece of the class holds pos.
PR_HD inline uint32_t piece_encode(int32_t pos, int32_t hot_slot, const int32_t *px, int P, int nh, bool *bad) {
  if (hot_slot) return (uint32_t)hot_slot;
  int p = 0;
  while (p < P && !(pos >= px[3 * p] && pos < px[3 * p + 1])) ++p;
  if (p == P) {
    *bad = true;
    return 0u;
  }
  return (uint32_t)(nh + 1 + px[3 * p + 2] + (pos - px[3 * p]));
}

// k_spmv_hot: byte offset of a piece code's source, b8 = 8 idx, hb = 8 (nh + 1), tbl = the class's
// table (LDS in the kernel); hot and padding codes come out >= 2^31 (u32 arithmetic).
PR_HD inline uint32_t piece_cold_offset(uint32_t b8, uint32_t hb, const uint32_t *tbl) {
  const uint32_t go = b8 - hb;
  const uint32_t t = go >> (kPieceShift + 3);
  return go + tbl[t < (uint32_t)kPieceTbl ? t : (uint32_t)kPieceTbl];
}

}  // namespace pr
