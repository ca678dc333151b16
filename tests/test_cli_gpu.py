"""End-to-end drop-in on the GPU: the C++ `pagerank` CLI and `python -m sparky_hip` on edge-list
and Common Crawl JSON inputs; stdout lines and (url,rank) part files against the oracle."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import sparky_rdd
from conftest import PKG_DIR

pytestmark = pytest.mark.gpu
CLI = os.path.join(PKG_DIR, "build", "pagerank")
KAT = ["A B", "A C", "A B", "B C", "C A", "C C", "D", "E A", "E F"]


def parse_has_rank(text):
    out = {}
    for line in text.splitlines():
        if " has rank: " in line:
            u, r = line.rsplit(" has rank: ", 1)
            assert r.endswith(".")
            out[u] = float(r[:-1])
    return out


def parse_part(path):
    out = {}
    for line in open(path):
        assert line.startswith("(") and line.endswith(")\n")
        u, r = line[1:-2].rsplit(",", 1)
        out[u] = float(r)
    return out


def oracle(pairs, iters):
    g, hist, _ = sparky_rdd.run(pairs, iters)
    return hist


@pytest.mark.parametrize("runner", ["cpp", "python"])
def test_cli_edge_list(tmp_path, runner):
    inp = tmp_path / "edges.txt"
    inp.write_text("\n".join(KAT) + "\n")
    out_dir = tmp_path / "out"
    if runner == "cpp":
        cmd = [CLI, str(inp), "3", "--out", str(out_dir), "--save-every-iter"]
    else:
        cmd = [sys.executable, "-m", "sparky_hip", str(inp), "3", "--out", str(out_dir), "--save-every-iter"]
    env = dict(os.environ, PYTHONPATH=PKG_DIR)
    res = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=120)
    assert res.returncode == 0, res.stderr
    lines = res.stdout.splitlines()
    assert lines[:3] == ["Starting iter0", "Starting iter1", "Starting iter2"]
    hist = oracle(sparky_rdd.pairs_from_edge_lines(KAT), 3)
    got = parse_has_rank(res.stdout)
    assert got.keys() == hist[-1].keys()
    for u, v in hist[-1].items():
        assert abs(got[u] - v) <= 1e-9 * v
    for it in range(3):
        part = parse_part(out_dir / f"PageRank{it}" / "part-00000")
        assert (out_dir / f"PageRank{it}" / "_SUCCESS").exists()
        for u, v in hist[it].items():
            assert abs(part[u] - v) <= 1e-9 * v


def test_cli_writes_only_the_last_part_and_reports_the_job(tmp_path):
    """Without --save-every-iter only PageRank<N-1> is written (Sparky.java:237 for the last
    iteration; its ranks are the ones pr_run returns, no per-iteration copy), and --stats reports
    the job's phases as one JSON object on stderr."""
    inp = tmp_path / "edges.txt"
    inp.write_text("\n".join(KAT) + "\n")
    out_dir = tmp_path / "out"
    res = subprocess.run([CLI, str(inp), "4", "--out", str(out_dir), "--stats"], capture_output=True, text=True,
                         timeout=120)
    assert res.returncode == 0, res.stderr
    assert sorted(os.listdir(out_dir)) == ["PageRank3"]
    hist = oracle(sparky_rdd.pairs_from_edge_lines(KAT), 4)
    part = parse_part(out_dir / "PageRank3" / "part-00000")
    assert part.keys() == hist[-1].keys()
    for u, v in hist[-1].items():
        assert abs(part[u] - v) <= 1e-9 * v
    assert parse_has_rank(res.stdout) == part
    job = json.loads([l for l in res.stderr.splitlines() if l.startswith('{"job"')][-1])["job"]
    assert job["urls"] == len(hist[-1]) and job["edge_records"] == len(KAT) and job["iterations"] == 4
    assert all(job[k] >= 0 for k in ("read_intern_ms", "build_ms", "run_ms", "has_rank_out_ms", "total_ms"))


def test_cli_ccjson(tmp_path):
    rng = np.random.default_rng(2)
    recs = []
    for i in range(400):
        links = [{"href": f"http://s{int(rng.integers(0, 300))}.org/", "type": "a" if rng.random() < 0.9 else "img"}
                 for _ in range(int(rng.integers(0, 7)))]
        recs.append(f"http://s{i % 250}.org/\t" + json.dumps({"url": "x", "content": {"links": links}}))
    inp = tmp_path / "cc.tsv"
    inp.write_text("\n".join(recs) + "\n")
    res = subprocess.run([CLI, str(inp), "10", "--format=ccjson"], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    hist = oracle(sparky_rdd.pairs_from_ccjson_lines(recs), 10)
    got = parse_has_rank(res.stdout)
    assert got.keys() == hist[-1].keys()
    err = max(abs(got[u] - v) / v for u, v in hist[-1].items())
    assert err <= 1e-9


def test_cli_rejects_bad_input(tmp_path):
    inp = tmp_path / "bad.txt"
    inp.write_text("a b c\n")
    res = subprocess.run([CLI, str(inp)], capture_output=True, text=True, timeout=60)
    assert res.returncode != 0 and "tokens" in res.stderr


@pytest.mark.parametrize("runner", ["cpp", "python"])
def test_cli_resume_from_saved_iteration(tmp_path, runner, oracle_c):
    """--resume DIR/PageRank4 continues the same 10-iteration loop (iterations 5..9): the saved
    Double.toString digits restore the ranks exactly, so PageRank9 matches the uninterrupted run
    (to rounding: the resumed dc is summed by k_reset's blocks, not the epilogue's) and the
    continued ranks match the oracle started from the saved ranks (oracle_c.run(..., init=...)).
    Reference: Sparky.java:165-170 (init) and :237 (the saves)."""
    rng = np.random.default_rng(12)
    lines = [f"u{int(s)} u{int(d)}" for s, d in zip(rng.integers(0, 400, 3000), rng.integers(0, 500, 3000))]
    lines += [f"u{i}" for i in range(400, 420)]  # records without links
    inp = tmp_path / "edges.txt"
    inp.write_text("\n".join(lines) + "\n")
    env = dict(os.environ, PYTHONPATH=PKG_DIR)
    base = [CLI] if runner == "cpp" else [sys.executable, "-m", "sparky_hip"]
    full, part = tmp_path / "full", tmp_path / "cont"
    r1 = subprocess.run(base + [str(inp), "10", "--out", str(full), "--save-every-iter", "--quiet"],
                        capture_output=True, text=True, env=env, timeout=120)
    assert r1.returncode == 0, r1.stderr
    r2 = subprocess.run(base + [str(inp), "10", "--out", str(part), "--save-every-iter", "--quiet",
                                "--resume", str(full / "PageRank4")], capture_output=True, text=True, env=env,
                        timeout=120)
    assert r2.returncode == 0, r2.stderr
    assert r2.stdout.splitlines() == [f"Starting iter{i}" for i in range(5, 10)]
    assert not (part / "PageRank4").exists() and (part / "PageRank5" / "_SUCCESS").exists()
    a9, b9 = parse_part(part / "PageRank9" / "part-00000"), parse_part(full / "PageRank9" / "part-00000")
    assert a9.keys() == b9.keys() and max(abs(a9[u] - b9[u]) / b9[u] for u in a9) <= 1e-13
    # oracle: 5 iterations from the saved PageRank4 ranks
    from sparky_hip import read_edge_list

    urls, src, dst = read_edge_list(lines)
    saved = parse_part(full / "PageRank4" / "part-00000")
    init = np.array([saved[u] for u in urls])
    ref = oracle_c.run(oracle_c.build_csr(len(urls), src, dst), 5, init=init)
    got = parse_part(part / "PageRank9" / "part-00000")
    err = max(abs(got[u] - ref["ranks"][i]) / ref["ranks"][i] for i, u in enumerate(urls))
    assert err <= 1e-9


@pytest.mark.parametrize("runner", ["cpp", "python"])
def test_cli_unwritable_out_fails(tmp_path, runner):
    """A failed saveAsTextFile (here: --out below a regular file) must end the job with a non-zero
    status, from the C++ CLI and from the Python host (whose writer runs inside a ctypes callback)."""
    inp = tmp_path / "edges.txt"
    inp.write_text("\n".join(KAT) + "\n")
    blocker = tmp_path / "file"
    blocker.write_text("x")
    env = dict(os.environ, PYTHONPATH=PKG_DIR)
    base = [CLI] if runner == "cpp" else [sys.executable, "-m", "sparky_hip"]
    res = subprocess.run(base + [str(inp), "3", "--out", str(blocker / "out")], capture_output=True, text=True,
                         env=env, timeout=120)
    assert res.returncode != 0


@pytest.mark.parametrize("runner", ["cpp", "python"])
def test_cli_devices_group(tmp_path, runner, oracle_c):
    """--devices 0,0,0: three row parts driven as one group (pr_group_*; on a multi-GPU box each
    entry is its own GPU) produce the same outputs as one part -- Starting iter lines, every
    saved PageRank<i>, the has-rank lines -- within the oracle bar, also when resumed."""
    rng = np.random.default_rng(21)
    lines = [f"u{int(s)} u{int(d)}" for s, d in zip(rng.integers(0, 600, 5000), rng.integers(0, 700, 5000))]
    lines += [f"u{i}" for i in range(600, 630)]  # records without links
    inp = tmp_path / "edges.txt"
    inp.write_text("\n".join(lines) + "\n")
    env = dict(os.environ, PYTHONPATH=PKG_DIR)
    base = [CLI] if runner == "cpp" else [sys.executable, "-m", "sparky_hip"]
    out = tmp_path / "grp"
    res = subprocess.run(base + [str(inp), "6", "--out", str(out), "--save-every-iter", "--devices", "0,0,0"],
                         capture_output=True, text=True, env=env, timeout=120)
    assert res.returncode == 0, res.stderr
    assert [ln for ln in res.stdout.splitlines() if ln.startswith("Starting")] == [f"Starting iter{i}" for i in range(6)]
    from sparky_hip import read_edge_list

    urls, src, dst = read_edge_list(lines)
    csr = oracle_c.build_csr(len(urls), src, dst)
    for it in range(6):
        ref = oracle_c.run(csr, it + 1)["ranks"]
        got = parse_part(out / f"PageRank{it}" / "part-00000")
        assert max(abs(got[u] - ref[i]) / ref[i] for i, u in enumerate(urls)) <= 1e-9
    final = parse_has_rank(res.stdout)
    ref = oracle_c.run(csr, 6)["ranks"]
    assert max(abs(final[u] - ref[i]) / ref[i] for i, u in enumerate(urls)) <= 1e-9
    # resumed on two parts from the group's own save
    cont = tmp_path / "cont"
    r2 = subprocess.run(base + [str(inp), "6", "--out", str(cont), "--quiet", "--devices", "0,0",
                                "--resume", str(out / "PageRank3")], capture_output=True, text=True, env=env, timeout=120)
    assert r2.returncode == 0, r2.stderr
    assert r2.stdout.splitlines() == ["Starting iter4", "Starting iter5"]
    a5, b5 = parse_part(cont / "PageRank5" / "part-00000"), parse_part(out / "PageRank5" / "part-00000")
    assert a5.keys() == b5.keys() and max(abs(a5[u] - b5[u]) / b5[u] for u in a5) <= 1e-13


def test_cli_devices_rejects_bad_list(tmp_path):
    inp = tmp_path / "edges.txt"
    inp.write_text("\n".join(KAT) + "\n")
    for bad in ["", "0,,1", "a", "0,-1"]:
        res = subprocess.run([CLI, str(inp), "3", "--devices", bad], capture_output=True, text=True, timeout=60)
        assert res.returncode == 2 and "--devices" in res.stderr
