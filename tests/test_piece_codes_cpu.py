"""CPU check of the piece-code address arithmetic (pr_internal.h kCodeC20P / kCodeC24P).

The build (pr_build.hip plan_pieces / k_fill_piece) lays every class's pieces -- the own region and
one sub-run of each peer's received run -- out in part order at kPieceAlign-aligned starts of a
virtual index space and writes, per class, a table of byte deltas per 4096-entry block plus a 0
sentinel; k_spmv_hot (pr_spmv.h cold_offset) turns an entry's index back into a byte offset with
u32 arithmetic: go = 8*idx - 8*(nh+1); go += tbl[min(go >> 15, 256)].  All three live in
csrc/pr_pieces.h, which the library and this test's shim (host/pieces_shim.cpp) compile alike, so
the test runs the product's own code: for random piece layouts every cold source
decodes to its own gather position, and hot and padding entries decode to offsets >= 2^31 (out of
range of any gather space, so the range-checked load returns 0 and costs no memory request).  The
GPU tests (tests/test_gpu_parity.py::test_piece_codes_bitwise) run the kernels themselves.
"""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpr_pieces_shim.so")
PIECE_TBL = 256


@pytest.fixture(scope="module")
def shim():
    import subprocess

    # always: make's dependency on pr_pieces.h rebuilds a stale shim after an edit
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "pagerank-using-apache-spark_amd", "host")], check=True)
    lib = ctypes.CDLL(SHIM)
    P_ = ctypes.c_void_p
    lib.prp_tbl_words.restype = ctypes.c_int
    lib.prp_tables.argtypes = [P_, ctypes.c_int, ctypes.c_int, P_, P_]
    lib.prp_tables.restype = ctypes.c_int64
    lib.prp_encode.argtypes = [P_, P_, ctypes.c_int64, P_, ctypes.c_int, ctypes.c_int, P_, P_]
    lib.prp_cold_offset.argtypes = [P_, ctypes.c_int64, ctypes.c_int, P_, P_]
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def plan_pieces(shim, lo, hi):
    """lo/hi[x, p] -> pc[x, p] = (g0, g1, v0), tbl[x, words] (u32 byte deltas), vmax -- the build's plan."""
    C, P = lo.shape
    lohi = np.concatenate([lo.reshape(-1), hi.reshape(-1)]).astype(np.int32)
    pc = np.zeros(3 * C * P, np.int32)
    W = shim.prp_tbl_words()
    tbl = np.zeros(C * W, np.int32)
    vmax = shim.prp_tables(_p(lohi), C, P, _p(pc), _p(tbl))
    return pc.reshape(C, P, 3).astype(np.int64), tbl.view(np.uint32).reshape(C, W), int(vmax)


def encode(shim, pos, hot_slot, x, pc, nh):
    """k_fill_piece: the hot slot, or nh + 1 + the virtual index; -1 when no piece holds pos."""
    P = pc.shape[1]
    px = np.ascontiguousarray(pc[x].reshape(-1), np.int32)
    a_pos, a_hot = np.array([pos], np.int32), np.array([hot_slot], np.int32)
    idx, bad = np.zeros(1, np.uint32), np.zeros(1, np.uint8)
    shim.prp_encode(_p(a_pos), _p(a_hot), 1, _p(px), P, nh, _p(idx), _p(bad))
    return -1 if bad[0] else int(idx[0])


def cold_offset(shim, idx, x, tbl, nh):
    """pr_spmv.h cold_offset<true> (pr_pieces.h piece_cold_offset) in u32 arithmetic."""
    a, out = np.array([idx], np.uint32), np.zeros(1, np.uint32)
    t = np.ascontiguousarray(tbl[x])
    shim.prp_cold_offset(_p(a), 1, nh, _p(t), _p(out))
    return int(out[0])


@pytest.mark.parametrize("P,C,seed", [(2, 16, 0), (3, 32, 1), (8, 32, 2), (8, 64, 3), (4, 8, 4)])
def test_piece_codes_round_trip(shim, P, C, seed):
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
    pc, tbl, vmax = plan_pieces(shim, lo, hi)
    nh = 18299 // P * P
    assert nh + vmax < (1 << 20)
    gather_bytes = 8 * base
    for x in range(C):
        for p in range(P):
            m = members[(x, p)]
            if len(m) == 0:
                continue
            for pos in rng.choice(m, size=min(64, len(m)), replace=False).tolist() + [int(m[0]), int(m[-1])]:
                idx = encode(shim, pos, 0, x, pc, nh)
                assert nh < idx < (1 << 20)
                assert cold_offset(shim, idx, x, tbl, nh) == 8 * pos
        # hot slots and padding (idx 0) stay out of range, and their LDS read is the slot itself
        for idx in [0, 1, nh // 2, nh]:
            off = cold_offset(shim, idx, x, tbl, nh)
            assert off >= (1 << 31) and off >= gather_bytes
            assert min(8 * idx, 8 * (nh + 1)) == 8 * idx
        # a cold entry's LDS read is clamped to the zero slot
        assert min(8 * (nh + 1 + 5), 8 * (nh + 1)) == 8 * (nh + 1)


def test_piece_plan_alignment_and_table_ownership(shim):
    lo = np.array([[0, 100000, 0], [5000, 200000, 300000]], np.int64)
    hi = np.array([[4097, 100001, 0], [9000, 200000, 309999]], np.int64)
    pc, tbl, vmax = plan_pieces(shim, lo, hi)
    # class 0: pieces at virtual 0 (4097 long -> blocks 0, 1) and 8192 (1 long); part 2 empty
    assert pc[0, 0].tolist() == [0, 4097, 0] and pc[0, 1].tolist() == [100000, 100001, 8192]
    assert vmax == 4096 + 9999  # class 1: 4000 rows, then 9999 from the next boundary
    assert pc[0, 2].tolist() == [0, 0, 0]
    # every block of a piece maps to that piece; the sentinel stays 0
    assert all(tbl[x, PIECE_TBL] == 0 for x in range(2))
    assert int(tbl[0, 0]) == 0 and int(tbl[0, 1]) == 0 and int(tbl[0, 2]) == (8 * (100000 - 8192)) & 0xFFFFFFFF
    # class 1: part 1's piece is empty, part 2's starts at the next 4096 boundary after 4000
    assert pc[1, 0].tolist() == [5000, 9000, 0] and pc[1, 2].tolist() == [300000, 309999, 4096]
