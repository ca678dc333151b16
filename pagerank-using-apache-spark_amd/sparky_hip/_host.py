"""ctypes binding of libpagerank_host (include/pagerank_host.h): native input front-ends
(edge list, Common Crawl ``url<TAB>json`` records), URL interning and the output writers."""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional

import numpy as np

from ._lib import BUILD_DIR

HOST_LIB_PATH = os.path.join(BUILD_DIR, "libpagerank_host.so")
FORMAT_EDGES = 0
FORMAT_CCJSON = 1
FORMATS = {"edges": FORMAT_EDGES, "ccjson": FORMAT_CCJSON}

_hl = None


class HostError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    global _hl
    if _hl is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise FileNotFoundError(f"{HOST_LIB_PATH} is missing: make -C pagerank-using-apache-spark_amd/host")
        L = ctypes.CDLL(HOST_LIB_PATH)
        P = ctypes.c_void_p
        L.prh_last_error.restype = ctypes.c_char_p
        L.prh_read.argtypes = [ctypes.c_char_p, ctypes.c_int32, P]
        L.prh_parse.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int32, P]
        L.prh_n_edges.argtypes = [P]
        L.prh_n_edges.restype = ctypes.c_int64
        L.prh_n_vertices.argtypes = [P]
        L.prh_n_vertices.restype = ctypes.c_int32
        L.prh_src.argtypes = [P]
        L.prh_src.restype = ctypes.POINTER(ctypes.c_int32)
        L.prh_dst.argtypes = [P]
        L.prh_dst.restype = ctypes.POINTER(ctypes.c_int32)
        L.prh_name.argtypes = [P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
        L.prh_name.restype = ctypes.c_void_p
        L.prh_java_double.argtypes = [ctypes.c_double, ctypes.c_char_p]
        L.prh_java_double.restype = ctypes.c_int32
        L.prh_write_part.argtypes = [P, ctypes.c_char_p, ctypes.c_int32, P]
        L.prh_write_has_rank.argtypes = [P, ctypes.c_char_p, P]
        L.prh_read_ranks.argtypes = [P, ctypes.c_char_p, P]
        L.prh_free.argtypes = [P]
        L.prh_free.restype = None
        L.prh_set_read_threads.argtypes = [ctypes.c_int32]
        L.prh_set_read_threads.restype = None
        _hl = L
    return _hl


def set_read_threads(n: int) -> None:
    """Threads of the native edge-list reader (0: automatic); the IDs do not depend on it."""
    load().prh_set_read_threads(int(n))


def _check(rc):
    if rc != 0:
        raise HostError(load().prh_last_error().decode(errors="replace"))


class HostEdges:
    """Interned edge list held by libpagerank_host (names stay in native memory)."""

    def __init__(self, handle: ctypes.c_void_p):
        self._h = handle
        L = load()
        self.n_edges = int(L.prh_n_edges(self._h))
        self.n_vertices = int(L.prh_n_vertices(self._h))
        if self.n_edges > 0:
            self.src = np.ctypeslib.as_array(L.prh_src(self._h), shape=(self.n_edges,))
            self.dst = np.ctypeslib.as_array(L.prh_dst(self._h), shape=(self.n_edges,))
        else:
            self.src = np.zeros(0, np.int32)
            self.dst = np.zeros(0, np.int32)

    @classmethod
    def read(cls, path: str, fmt: str = "edges") -> "HostEdges":
        h = ctypes.c_void_p()
        _check(load().prh_read(path.encode(), FORMATS[fmt], ctypes.byref(h)))
        return cls(h)

    @classmethod
    def parse(cls, data: bytes, fmt: str = "edges") -> "HostEdges":
        h = ctypes.c_void_p()
        _check(load().prh_parse(data, len(data), FORMATS[fmt], ctypes.byref(h)))
        return cls(h)

    def name(self, i: int) -> bytes:
        n = ctypes.c_int64()
        p = load().prh_name(self._h, i, ctypes.byref(n))
        return ctypes.string_at(p, n.value)

    def names(self) -> List[str]:
        return [self.name(i).decode("utf-8", errors="surrogateescape") for i in range(self.n_vertices)]

    def write_part(self, out_dir: str, iteration: int, ranks: np.ndarray) -> None:
        r = np.ascontiguousarray(ranks, dtype=np.float64)
        _check(load().prh_write_part(self._h, out_dir.encode(), iteration, r.ctypes.data_as(ctypes.c_void_p)))

    def write_has_rank(self, path: Optional[str], ranks: np.ndarray) -> None:
        r = np.ascontiguousarray(ranks, dtype=np.float64)
        _check(load().prh_write_has_rank(self._h, path.encode() if path else None,
                                         r.ctypes.data_as(ctypes.c_void_p)))

    def read_ranks(self, directory: str) -> np.ndarray:
        """Resume input: the saved ``(url,rank)`` lines of ``directory/part-*`` in ID order."""
        r = np.zeros(max(self.n_vertices, 1), np.float64)
        _check(load().prh_read_ranks(self._h, directory.encode(), r.ctypes.data_as(ctypes.c_void_p)))
        return r[: self.n_vertices]

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            load().prh_free(self._h)
            self._h = ctypes.c_void_p()
            self.src = self.dst = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def java_double_native(x: float) -> str:
    buf = ctypes.create_string_buffer(64)
    n = load().prh_java_double(x, buf)
    return buf.raw[:n].decode()
