"""sparky_hip -- Python host of the MI355X PageRank engine (drop-in for Sparky.java's hot path).

The compute path is libpagerank_hip (HIP, gfx950); this package binds its C ABI and mirrors the
reference job's I/O (edge list in, ``(url,rank)`` / ``<url> has rank: <r>.`` out).
"""
from ._host import HostEdges, HostError, java_double_native
from ._lib import LIB_PATH, PageRankError, load
from .driver import java_double_to_string, main, read_edge_list, write_has_rank, write_part_file
from .graph import (CHUNGLU_PRESETS, CanonicalCSR, IterationStats, PageRankGraph, PartGroup, comm_unique_id,
                    device_count, gen_chunglu, gen_er, gen_rmat, intern_device)

__all__ = [
    "HostEdges", "HostError", "java_double_native",
    "LIB_PATH", "PageRankError", "load", "java_double_to_string", "main", "read_edge_list",
    "write_has_rank", "write_part_file", "CanonicalCSR", "IterationStats", "PageRankGraph", "PartGroup",
    "comm_unique_id", "device_count", "gen_chunglu", "gen_er", "gen_rmat", "intern_device", "CHUNGLU_PRESETS",
]
