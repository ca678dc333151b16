"""CPU check of the piece-code address arithmetic (pr_internal.h kCodeC20P / kCodeC24P).

The build (pr_build.hip plan_pieces / k_fill_piece) lays every class's pieces -- the own region and
one sub-run of each peer's received run -- out in part order at kPieceAlign-aligned starts of a
virtual index space and writes, per class, a table of byte deltas per 4096-entry block plus a 0
sentinel; k_spmv_hot (pr_spmv.h cold_offset) turns an entry's index back into a byte offset with
u32 arithmetic: go = 8*idx - 8*(nh+1); go += tbl[min(go >> 15, 256)].  This restates both sides in
numpy and checks, for random piece layouts, that every cold source decodes to its own gather
position and that hot and padding entries decode to offsets >= 2^31 (out of range of any gather
space, so the range-checked load returns 0 and costs no memory request).  Host logic only: the
GPU tests (tests/test_gpu_parity.py::test_piece_codes_bitwise) run the kernels themselves.
"""
import numpy as np
import pytest

PIECE_SHIFT = 12
PIECE_ALIGN = 1 << PIECE_SHIFT
PIECE_TBL = (1 << 20) >> PIECE_SHIFT  # 256
TBL_WORDS = PIECE_TBL + 2


def plan_pieces(lo, hi):
    """lo/hi[x, p] -> pc[x, p] = (g0, g1, v0), tbl[x, TBL_WORDS] (u32 byte deltas), vmax."""
    C, P = lo.shape
    pc = np.zeros((C, P, 3), np.int64)
    tbl = np.zeros((C, TBL_WORDS), np.uint32)
    vmax = 0
    for x in range(C):
        v = 0
        for p in range(P):
            g0, g1 = int(lo[x, p]), int(hi[x, p])
            if g1 <= g0:
                continue
            v = (v + PIECE_ALIGN - 1) // PIECE_ALIGN * PIECE_ALIGN
            pc[x, p] = (g0, g1, v)
            for t in range(v >> PIECE_SHIFT, min(((v + g1 - g0 - 1) >> PIECE_SHIFT) + 1, PIECE_TBL)):
                tbl[x, t] = np.uint32((8 * (g0 - v)) & 0xFFFFFFFF)
            v += g1 - g0
        vmax = max(vmax, v)
    return pc, tbl, vmax


def encode(pos, hot_slot, x, pc, nh):
    """k_fill_piece: the hot slot, or nh + 1 + the virtual index; -1 when no piece holds pos."""
    if hot_slot:
        return hot_slot
    for g0, g1, v0 in pc[x]:
        if g0 <= pos < g1:
            return nh + 1 + v0 + (pos - g0)
    return -1


def cold_offset(idx, x, tbl, nh):
    """pr_spmv.h cold_offset<true> in u32 arithmetic."""
    go = (8 * int(idx) - 8 * (nh + 1)) & 0xFFFFFFFF
    t = min(int(go) >> (PIECE_SHIFT + 3), PIECE_TBL)
    return (int(go) + int(tbl[x, t])) & 0xFFFFFFFF


@pytest.mark.parametrize("P,C,seed", [(2, 16, 0), (3, 32, 1), (8, 32, 2), (8, 64, 3), (4, 8, 4)])
def test_piece_codes_round_trip(P, C, seed):
    rng = np.random.default_rng(seed)
    Q = int(rng.integers(2000, 40000))  # class region rows of a slice
    S = C * Q + 2
    # gather space: own slice [0, S), then per peer a run sorted by the peer's slice position
    self_part = int(rng.integers(0, P))
    lo = np.zeros((C, P), np.int64)
    hi = np.zeros((C, P), np.int64)
    members = {}
    base = S
    for p in range(P):
        for x in range(C):
            if p == self_part:
                lo[x, p], hi[x, p] = x * Q, (x + 1) * Q
                members[(x, p)] = np.arange(x * Q, (x + 1) * Q)
            else:
                n = int(rng.integers(0, Q // 2))  # some (class, peer) pieces are empty
                lo[x, p], hi[x, p] = base, base + n
                members[(x, p)] = np.arange(base, base + n)
                base += n
        if p != self_part:
            base += 2  # the run's two slots (no class's sources)
    pc, tbl, vmax = plan_pieces(lo, hi)
    nh = 18299 // P * P
    assert nh + vmax < (1 << 20)
    gather_bytes = 8 * base
    for x in range(C):
        for p in range(P):
            m = members[(x, p)]
            if len(m) == 0:
                continue
            for pos in rng.choice(m, size=min(64, len(m)), replace=False).tolist() + [int(m[0]), int(m[-1])]:
                idx = encode(pos, 0, x, pc, nh)
                assert nh < idx < (1 << 20)
                assert cold_offset(idx, x, tbl, nh) == 8 * pos
        # hot slots and padding (idx 0) stay out of range, and their LDS read is the slot itself
        for idx in [0, 1, nh // 2, nh]:
            off = cold_offset(idx, x, tbl, nh)
            assert off >= (1 << 31) and off >= gather_bytes
            assert min(8 * idx, 8 * (nh + 1)) == 8 * idx
        # a cold entry's LDS read is clamped to the zero slot
        assert min(8 * (nh + 1 + 5), 8 * (nh + 1)) == 8 * (nh + 1)


def test_piece_plan_alignment_and_table_ownership():
    lo = np.array([[0, 100000, 0], [5000, 200000, 300000]], np.int64)
    hi = np.array([[4097, 100001, 0], [9000, 200000, 309999]], np.int64)
    pc, tbl, vmax = plan_pieces(lo, hi)
    # class 0: pieces at virtual 0 (4097 long -> blocks 0, 1) and 8192 (1 long); part 2 empty
    assert pc[0, 0].tolist() == [0, 4097, 0] and pc[0, 1].tolist() == [100000, 100001, 8192]
    assert vmax == 4096 + 9999  # class 1: 4000 rows, then 9999 from the next boundary
    assert pc[0, 2].tolist() == [0, 0, 0]
    # every block of a piece maps to that piece; the sentinel stays 0
    assert all(tbl[x, PIECE_TBL] == 0 for x in range(2))
    assert int(tbl[0, 0]) == 0 and int(tbl[0, 1]) == 0 and int(tbl[0, 2]) == (8 * (100000 - 8192)) & 0xFFFFFFFF
    # class 1: part 1's piece is empty, part 2's starts at the next 4096 boundary after 4000
    assert pc[1, 0].tolist() == [5000, 9000, 0] and pc[1, 2].tolist() == [300000, 309999, 4096]
