// Test shim (not product code): exposes the piece-code arithmetic of csrc/pr_pieces.h -- the
// table plan of the build, the encoder of k_fill_piece and the decoder of k_spmv_hot -- to
// tests/test_piece_codes_cpu.py on the CPU.
#include "pr_pieces.h"

#include <cstring>

extern "C" {
int prp_tbl_words(void) { return pr::kPieceTblWords; }
// lohi: 2 C P ints (lo block, then hi block); pc: 3 C P ints; tbl: C kPieceTblWords ints.
int64_t prp_tables(const int32_t *lohi, int C, int P, int32_t *pc, int32_t *tbl) {
  std::vector<int32_t> vpc, vtbl;
  const int64_t vmax = pr::piece_tables(lohi, C, P, &vpc, &vtbl);
  std::memcpy(pc, vpc.data(), sizeof(int32_t) * vpc.size());
  std::memcpy(tbl, vtbl.data(), sizeof(int32_t) * vtbl.size());
  return vmax;
}
// the code of n positions of class x (hot: their hot slots, 0 = cold); bad[i] = 1 when no piece holds it
void prp_encode(const int32_t *pos, const int32_t *hot, int64_t n, const int32_t *px, int P, int nh, uint32_t *idx,
                uint8_t *bad) {
  for (int64_t i = 0; i < n; ++i) {
    bool b = false;
    idx[i] = pr::piece_encode(pos[i], hot[i], px, P, nh, &b);
    bad[i] = b ? 1 : 0;
  }
}
// byte offsets of n codes of one class (its table)
void prp_cold_offset(const uint32_t *idx, int64_t n, int nh, const uint32_t *tbl, uint32_t *off) {
  for (int64_t i = 0; i < n; ++i) off[i] = pr::piece_cold_offset(8u * idx[i], 8u * (uint32_t)(nh + 1), tbl);
}
}
