"""Generate the committed golden fixtures in tests/golden/*.json.

The reference (Sparky.java, Spark 1.x) cannot run in this image (no JDK / Spark) and ships no
test vectors, so the fixtures are produced by oracle/sparky_rdd.py -- the literal RDD-level
restatement of Sparky.java:78-237 -- and pinned by the hand-derived KAT of SURVEY.md §4
(``kat_survey``).  Each fixture holds the edge-list text, the first-appearance URL order,
N, the dangling set size and the ranks + danglingContrib of every iteration.

Usage:  python tests/golden/make_golden.py      (rewrites the fixtures deterministically)
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import sparky_rdd  # noqa: E402


def case(name, lines, iterations=10, dangling="local"):
    pairs = sparky_rdd.pairs_from_edge_lines(lines)
    names, _src, _dst = sparky_rdd.intern_first_appearance(pairs)
    g, hist, dcs = sparky_rdd.run(pairs, iterations, dangling)
    return {
        "name": name,
        "source": "oracle/sparky_rdd.py (literal restatement of Sparky.java:78-237)",
        "lines": list(lines),
        "iterations": iterations,
        "dangling": dangling,
        "urls": names,
        "N": g.total_url_count,
        "n_dangling": len(g.dang_urls),
        "ranks": [[h[u] for u in names] for h in hist],
        "dc": dcs,
    }


def rand_graph(seed, n_urls, n_lines, p_single=0.1, p_dup=0.1, p_self=0.05):
    rng = random.Random(seed)
    urls = [f"http://site{rng.randrange(10**6)}.example/p{i}" for i in range(n_urls)]
    lines = []
    for _ in range(n_lines):
        u = rng.choice(urls)
        r = rng.random()
        if r < p_single:
            lines.append(u)
        elif r < p_single + p_self:
            lines.append(f"{u} {u}")
        else:
            v = rng.choice(urls)
            lines.append(f"{u} {v}")
            if rng.random() < p_dup:
                lines.append(f"{u} {v}")
    return lines


def rmat_lines(seed, scale, edge_factor, a=0.57, b=0.19, c=0.19):
    rng = random.Random(seed)
    lines = []
    for _ in range(edge_factor << scale):
        s = d = 0
        for lvl in range(scale):
            x = rng.random()
            sb = 1 if x >= a + b else 0
            db = 1 if (a <= x < a + b) or x >= a + b + c else 0
            s |= sb << lvl
            d |= db << lvl
        lines.append(f"v{s} v{d}")
    return lines


def main():
    cases = [
        # SURVEY.md §4 worked example: dedupe, self-loop, no-link key, in-degree-0, sink-only.
        case("kat_survey", ["A B", "A C", "A B", "B C", "C A", "C C", "D", "E A", "E F"], 3),
        case("kat_survey_10", ["A B", "A C", "A B", "B C", "C A", "C C", "D", "E A", "E F"], 10),
        case("kat_survey_cluster", ["A B", "A C", "A B", "B C", "C A", "C C", "D", "E A", "E F"],
             5, "none"),
        case("single_self_loop", ["x x"], 4),
        case("single_nolink", ["x"], 3),
        case("chain_sink", ["a b", "b c", "c d"], 6),
        case("star_in", [f"s{i} hub" for i in range(40)], 5),
        case("star_out", [f"hub t{i}" for i in range(40)], 5),
        case("mixed_key", ["m", "m n", "n m", "z"], 5),
        case("all_duplicates", ["p q"] * 7 + ["q p"] * 3, 5),
        case("two_components", ["a b", "b a", "c d", "d c", "e"], 5),
        case("random_small", rand_graph(7, 30, 120), 10),
        case("random_medium", rand_graph(11, 300, 2000, p_single=0.05), 10),
        case("random_medium_cluster", rand_graph(13, 200, 1500), 10, "none"),
        case("rmat_s8", rmat_lines(1, 8, 8), 10),
    ]
    for c in cases:
        with open(os.path.join(HERE, f"{c['name']}.json"), "w") as f:
            json.dump(c, f, separators=(",", ":"))
    print(f"wrote {len(cases)} fixtures to {HERE}")


if __name__ == "__main__":
    main()
