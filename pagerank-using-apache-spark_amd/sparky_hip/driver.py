"""Process-level drop-in for the Spark job (Python host; the C++ CLI ``pagerank`` is the same).

CLI: ``python -m sparky_hip <input-path> [iterations=10] [--format edges|ccjson]
[--out DIR] [--save-every-iter] [--dangling=local|none] [--device N] [--quiet]
[--resume DIR/PageRank<i>]``

* input: text edge list, ``src dst`` per line; a single-token line ``src`` is a record without
  ``a`` links (Sparky.java:114-118).  Tokens (URLs) are taken verbatim and interned to dense
  int32 IDs in first-appearance order, src before dst.
* stdout: ``Starting iter<i>`` before every iteration (Sparky.java:188), then
  ``<url> has rank: <r>.`` for every URL after the last iteration (north_star contract).
* ``--out DIR``: ``DIR/PageRank<i>/part-00000`` with ``(url,rank)`` lines -- Scala
  ``Tuple2.toString`` of ``(String, Double)`` with Java ``Double.toString`` -- plus an empty
  ``_SUCCESS`` (Sparky.java:237 ``saveAsTextFile``); only the last iteration unless
  ``--save-every-iter``.
* ``--resume DIR/PageRank<i>``: start from the ranks saved there (instead of 1.0,
  Sparky.java:165-170) and continue the same loop with iterations i+1 .. N-1 (a directory not
  named ``PageRank<i>`` starts the loop at 0).  Same rules as the C++ CLI.
"""
from __future__ import annotations

import argparse
import math
import os
import sys
from typing import Dict, Iterable, List, Sequence, TextIO, Tuple

import numpy as np

from .graph import PageRankGraph, PartGroup


def java_double_to_string(x: float) -> str:
    """``Double.toString`` (shortest-uniquely-distinguishing digits, JDK 19+ algorithm).

    Layout per the JDK spec: decimal notation for 1e-3 <= |x| < 1e7 with at least one digit
    after the point; otherwise ``d.dddE<exp>``.  JDK <= 18 (Spark 1.x era) emits a longer,
    non-shortest digit string for a few values (JDK-4511638); parity tests therefore compare
    parsed numbers, never strings.
    """
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    ax = abs(x)
    r = repr(ax)  # shortest round-trip digits
    if "e" in r or "E" in r:
        mant, exp = r.lower().split("e")
        e10 = int(exp)
    else:
        mant, e10 = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # position of the decimal point relative to the first significant digit
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    point = len(ip) - lead_zeros + e10  # value = 0.digits * 10^point
    digits = digits.rstrip("0") or "0"
    if len(digits) == 1:
        # JDK 19+ renders at least two significant digits and picks the 2-digit decimal
        # closest to the value when the 1-digit shortest is not (e.g. 4.9E-324, not 5.0E-324).
        m2, e2 = f"{ax:.1e}".split("e")
        d2 = m2.replace(".", "").rstrip("0") or "0"
        digits, point = d2, int(e2) + 1
    if 1e-3 <= ax < 1e7:
        if point <= 0:
            s = "0." + "0" * (-point) + digits
        elif point >= len(digits):
            s = digits + "0" * (point - len(digits)) + ".0"
        else:
            s = digits[:point] + "." + digits[point:]
        return sign + s
    frac = digits[1:] or "0"
    return f"{sign}{digits[0]}.{frac}E{point - 1}"


def read_edge_list(lines: Iterable[str]) -> Tuple[List[str], np.ndarray, np.ndarray]:
    """Tokenise and intern (first appearance, src before dst).  Returns (urls, src, dst)."""
    ids: Dict[str, int] = {}
    urls: List[str] = []
    src: List[int] = []
    dst: List[int] = []
    for ln, line in enumerate(lines):
        toks = line.split()
        if not toks:
            continue
        if len(toks) > 2:
            raise ValueError(f"line {ln + 1}: expected 'src [dst]', got {len(toks)} tokens")
        u = toks[0]
        iu = ids.get(u)
        if iu is None:
            iu = ids[u] = len(urls)
            urls.append(u)
        src.append(iu)
        if len(toks) == 1:
            dst.append(-1)
        else:
            v = toks[1]
            iv = ids.get(v)
            if iv is None:
                iv = ids[v] = len(urls)
                urls.append(v)
            dst.append(iv)
    return urls, np.asarray(src, np.int32), np.asarray(dst, np.int32)


def write_part_file(out_dir: str, iteration: int, urls: Sequence[str], ranks: np.ndarray) -> str:
    """``ranks.saveAsTextFile(out_dir + "/PageRank" + iter + "/")`` (Sparky.java:237)."""
    d = os.path.join(out_dir, f"PageRank{iteration}")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "part-00000"), "w") as f:
        for u, r in zip(urls, ranks.tolist()):
            f.write(f"({u},{java_double_to_string(r)})\n")
    open(os.path.join(d, "_SUCCESS"), "w").close()
    return d


def write_has_rank(stream: TextIO, urls: Sequence[str], ranks: np.ndarray) -> None:
    for u, r in zip(urls, ranks.tolist()):
        stream.write(f"{u} has rank: {java_double_to_string(r)}.\n")


def saved_iteration(path: str) -> int:
    """i of a ``.../PageRank<i>`` directory, or -1."""
    base = os.path.basename(os.path.normpath(path))
    if base.startswith("PageRank") and base[8:].isdigit():
        return int(base[8:])
    return -1


def _run_group(edges, devices, dangling, n_run, init, cb, want_ranks):
    """--devices: one part per listed device, one process (pr_group_*); the callback gets the
    merged ranks of every part after each iteration, as with PageRankGraph.run."""
    P = len(devices)
    parts = []
    try:
        for p, d in enumerate(devices):
            parts.append(PageRankGraph(edges.n_vertices, edges.src, edges.dst, device=d, dangling=dangling,
                                       keep_canonical=False, part=p, n_parts=P))
        grp = PartGroup(parts)
        grp.reset(init_ranks=init)
        for it in range(n_run):
            grp.step(1)
            grp.sync()
            cb(it, grp.ranks() if want_ranks else None, None)
        return grp.ranks()
    finally:
        for g in parts:
            g.close()


def main(argv=None) -> int:
    from ._host import HostEdges

    ap = argparse.ArgumentParser(prog="sparky_hip", description=__doc__.splitlines()[0])
    ap.add_argument("edge_list")
    ap.add_argument("iterations", nargs="?", type=int, default=10)  # Sparky.java:187
    ap.add_argument("--format", choices=["edges", "ccjson"], default="edges")
    ap.add_argument("--out", default=None)
    ap.add_argument("--save-every-iter", action="store_true")
    ap.add_argument("--dangling", choices=["local", "none"], default="local")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--quiet", action="store_true", help="omit the '<url> has rank' lines")
    ap.add_argument("--resume", default=None, metavar="DIR", help="start from saved (url,rank) part files")
    ap.add_argument("--devices", default=None, metavar="D0,D1,...",
                    help="one row part per listed GPU (a device may repeat), one process (pr_group_*)")
    a = ap.parse_args(argv)
    devices = [a.device]
    if a.devices is not None:
        try:
            devices = [int(t) for t in a.devices.split(",")]
        except ValueError:
            ap.error("--devices takes a comma-separated list of device numbers")
    edges = HostEdges.read(a.edge_list, a.format)  # native front-end + first-appearance interning
    out = sys.stdout
    init, start = None, 0
    if a.resume:
        init = edges.read_ranks(a.resume)
        start = saved_iteration(a.resume) + 1
    n_run = max(a.iterations - start, 0)
    # Sparky prints "Starting iter<i>" before each iteration (Sparky.java:188); the library
    # calls back after iteration i, so the host prints the next line there.
    def cb(it_run, ranks, _st):
        it = start + it_run
        if a.out and (a.save_every_iter or it == a.iterations - 1):
            edges.write_part(a.out, it, ranks)
        if it + 1 < a.iterations:
            out.write(f"Starting iter{it + 1}\n")

    if n_run > 0:
        out.write(f"Starting iter{start}\n")
    if len(devices) == 1:
        with PageRankGraph(edges.n_vertices, edges.src, edges.dst, device=devices[0], dangling=a.dangling,
                           keep_canonical=False) as g:
            ranks, _ = g.run(n_run, callback=cb, want_ranks_in_callback=bool(a.out), init_ranks=init)
    else:
        ranks = _run_group(edges, devices, a.dangling, n_run, init, cb, bool(a.out))
    out.flush()
    if not a.quiet:
        edges.write_has_rank(None, ranks)
    edges.close()
    return 0
