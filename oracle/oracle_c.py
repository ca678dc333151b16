"""ctypes binding of oracle/pagerank_oracle.c (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module;
it is the checker / CPU baseline, never the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

VF_KEY, VF_SINK, VF_NOLINK, VF_INDEG0 = 1, 2, 4, 8


def build() -> str:
    """Compile the C restatement with the committed Makefile (gcc, no reference sources)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.orc_build.argtypes = [ctypes.c_int32, ctypes.c_int64, P, P, P, P, P, P, P]
        L.orc_build.restype = ctypes.c_int
        L.orc_run.argtypes = [ctypes.c_int32, P, P, P, P, ctypes.c_int32, ctypes.c_int32,
                              ctypes.c_double, ctypes.c_double, P, P, P, P, P, ctypes.c_int32, P]
        L.orc_run.restype = ctypes.c_int
        L.orc_flag_bits.restype = ctypes.c_uint32
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class CSR:
    n_vertices: int
    row_ptr: np.ndarray  # int64[V+1]
    col_idx: np.ndarray  # int32[E']
    out_deg: np.ndarray  # int32[V]
    vflags: np.ndarray  # uint8[V]

    @property
    def n_edges(self) -> int:
        return int(self.col_idx.shape[0])


def build_csr(n_vertices: int, src: np.ndarray, dst: np.ndarray) -> CSR:
    src = np.ascontiguousarray(src, dtype=np.int32)
    dst = np.ascontiguousarray(dst, dtype=np.int32)
    E = src.shape[0]
    row_ptr = np.zeros(n_vertices + 1, np.int64)
    col = np.zeros(max(E, 1), np.int32)
    deg = np.zeros(max(n_vertices, 1), np.int32)
    vf = np.zeros(max(n_vertices, 1), np.uint8)
    nd = ctypes.c_int64(0)
    rc = lib().orc_build(n_vertices, E, _p(src), _p(dst), _p(row_ptr), _p(col), _p(deg), _p(vf),
                         ctypes.byref(nd))
    if rc != 0:
        raise ValueError("oracle: invalid edge list (ID out of range or an ID that never appears)")
    return CSR(n_vertices, row_ptr, col[: nd.value].copy(), deg[:n_vertices], vf[:n_vertices])


def run(csr: CSR, iterations: int, dangling_none: bool = False, teleport: float = 0.15,
        damping: float = 0.85, init=None, keep_history: bool = False, nthreads: int = 0):
    """Returns dict(ranks, dc[iters], l1[iters], iter_ms[iters], history[iters, V] or None)."""
    V = csr.n_vertices
    ranks = np.zeros(max(V, 1), np.float64)
    dc = np.zeros(max(iterations, 1), np.float64)
    l1 = np.zeros(max(iterations, 1), np.float64)
    ms = np.zeros(max(iterations, 1), np.float64)
    hist = np.zeros((iterations, V), np.float64) if keep_history else None
    init_a = None if init is None else np.ascontiguousarray(init, dtype=np.float64)
    lib().orc_run(V, _p(csr.row_ptr), _p(csr.col_idx), _p(csr.out_deg), _p(csr.vflags), iterations,
                  1 if dangling_none else 0, teleport, damping, _p(init_a), _p(ranks), _p(dc), _p(l1),
                  _p(hist), nthreads, _p(ms))
    return {"ranks": ranks[:V], "dc": dc[:iterations], "l1": l1[:iterations], "iter_ms": ms[:iterations],
            "history": hist}
