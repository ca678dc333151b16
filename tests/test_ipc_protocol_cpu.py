"""CPU model check of the IPC exchange's host-side ordering (PR_OPT_XCHG_IPC).

The library's CU-free transport (csrc/pr_ipc.hip) orders its copy-engine pulls with interprocess
events, and a wait on such an event binds to the latest record enqueued when the wait is enqueued.
Its hosts therefore publish record counts and spin before every wait (csrc/pr_ipc_protocol.h).  The
same protocol template runs here in host/ipc_model.cpp with one thread per rank, random delays
between every step and events modelled as "records enqueued so far": every wait must find exactly
the record it means as the peer's latest (never an older one -- the device would not wait for the
data -- nor a newer one -- it would wait for the wrong iteration), and no rank may deadlock, over
seeded sequences of resets, fused-pack and pack-kernel iterations (buffer reuse every other
iteration; a reset exchanges buffer 0 again).  The GPU tests (tests/test_gpu_rccl.py) run the
transport itself and check its ranks bitwise against RCCL's.
"""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pagerank-using-apache-spark_amd", "build", "libpr_ipc_model.so")


@pytest.fixture(scope="module")
def model():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "pagerank-using-apache-spark_amd", "host")], check=True)
    lib = ctypes.CDLL(LIB)
    lib.ipc_model_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                  ctypes.c_char_p, ctypes.c_int]
    lib.ipc_model_run.restype = ctypes.c_int64
    lib.ipc_model_run2.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_char_p, ctypes.c_int]
    lib.ipc_model_run2.restype = ctypes.c_int64
    lib.ipc_model_chunk_end.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
    lib.ipc_model_chunk_end.restype = ctypes.c_int64
    return lib


def _run(model, P, n_ops, seed, delay_us, nc=8):
    err = ctypes.create_string_buffer(512)
    waits = model.ipc_model_run(P, nc, n_ops, seed, delay_us, err, len(err))
    assert waits >= 0, err.value.decode()
    return waits


@pytest.mark.parametrize("P,nc,n_ops,seed,delay_us", [(2, 1, 400, 1, 0), (2, 8, 200, 2, 30), (3, 4, 200, 3, 20),
                                                      (4, 8, 150, 4, 20), (5, 2, 100, 7, 15), (6, 8, 100, 8, 10),
                                                      (7, 4, 90, 9, 10), (8, 8, 80, 5, 10), (8, 1, 150, 6, 0)])
def test_every_wait_binds_to_the_record_it_means(model, P, nc, n_ops, seed, delay_us):
    """Per-chunk sent records: the pass records chunk c of its runs as soon as the
    epilogue has written it, a receiver's per-chunk copy waits for exactly that chunk's record."""
    waits = _run(model, P, n_ops, seed, delay_us, nc=nc)
    # every exchange waits on each peer's sent record, and every reuse of a buffer on each peer's
    # copied record of its previous exchange
    assert waits >= n_ops * (P - 1)


@pytest.mark.parametrize("P,nc,n_ops,seed,delay_us,reenable", [(2, 8, 700, 21, 0, 0), (3, 4, 500, 22, 5, 0),
                                                               (2, 8, 600, 23, 5, 25), (4, 8, 400, 24, 5, 15),
                                                               (8, 2, 300, 25, 3, 20)])
def test_event_generations_past_the_runtime_limit(model, P, nc, n_ops, seed, delay_us, reenable):
    """the event generations (csrc/pr_ipc_gens.h, the helper pr_ipc.hip uses) under the
    checker -- runs far past 3 x 30 exchanges per buffer, optionally with re-enables (the counts
    restart, a new epoch): no event takes more than the runtime's 32 records, and every wait picks,
    by the library's rule, the generation whose latest record is the one meant."""
    err = ctypes.create_string_buffer(512)
    waits = model.ipc_model_run2(P, nc, n_ops, seed, delay_us, reenable, err, len(err))
    assert waits >= 0, err.value.decode()
    assert waits >= n_ops * (P - 1)


def test_the_model_catches_a_broken_order(model):
    """Sanity of the checker itself: a protocol that skips the host spin before the sent wait must be
    caught -- with delays, some rank enqueues its wait before the peer has recorded that exchange.
    (ipc_model_run with a negative delay runs that broken variant.)"""
    err = ctypes.create_string_buffer(512)
    caught = any(model.ipc_model_run(4, 8, 200, s, -30, err, len(err)) < 0 for s in range(1, 6))
    assert caught and b"latest record" in err.value


@pytest.mark.parametrize("C,Q_pad", [(16, 4096), (32, 5120), (64, 512 * 1024 + 64), (64, 64), (128, 1 << 20), (64, 8000)])
def test_epilogue_chunk_launches_cover_each_chunk_before_its_record(model, C, Q_pad):
    """PR_OPT_XCHG_IPC = 2 (pr_iter.hip): the epilogue launch before chunk c's record covers every
    group holding a row of chunks <= c (local rows below (c + 1) * 8 * Q_pad), and the launches
    partition the groups (each row's update runs exactly once)."""
    import numpy as np

    nxc, rows_per_grp = C // 8, 8 * 64
    n_rows = C * Q_pad
    ngrp = (n_rows + rows_per_grp - 1) // rows_per_grp
    ends = [model.ipc_model_chunk_end(ngrp, c, nxc, 8 * Q_pad, rows_per_grp) for c in range(nxc)]
    assert ends[-1] == ngrp and all(a <= b for a, b in zip(ends, ends[1:]))
    covered = np.zeros(ngrp, np.int32)
    lo = 0
    for c, hi in enumerate(ends):
        covered[lo:hi] += 1
        last_row_of_chunk = min((c + 1) * 8 * Q_pad, n_rows) - 1
        assert last_row_of_chunk // rows_per_grp < hi  # its group ran before the record
        lo = max(lo, hi)
    assert (covered == 1).all()
