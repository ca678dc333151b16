"""Host-side logic on CPU: tokeniser/interner, Java Double.toString, output writers."""
import io
import os
import random
import struct

import numpy as np
import pytest

import sparky_rdd
from sparky_hip import java_double_to_string, read_edge_list, write_has_rank, write_part_file


@pytest.mark.parametrize("x,s", [
    (1.1416666666666666, "1.1416666666666666"), (0.15, "0.15"), (1.0, "1.0"), (100.0, "100.0"),
    (1e7, "1.0E7"), (9999999.0, "9999999.0"), (0.001, "0.001"), (9.99e-4, "9.99E-4"),
    (12345678.9, "1.23456789E7"), (2e-5, "2.0E-5"), (1.2345e16, "1.2345E16"), (0.0, "0.0"),
    (-0.0, "-0.0"), (-1.5, "-1.5"), (float("inf"), "Infinity"), (float("nan"), "NaN"),
    (1e-300, "1.0E-300"), (123.456, "123.456"), (5e-324, "4.9E-324"),
])
def test_java_double_to_string(x, s):
    assert java_double_to_string(x) == s


def test_java_double_round_trips():
    rng = random.Random(5)
    for _ in range(2000):
        x = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(63)))[0]
        if x != x or x in (float("inf"),):
            continue
        s = java_double_to_string(x)
        assert float(s.replace("E", "e")) == x


def test_reader_matches_oracle_interning(golden_cases):
    for c in golden_cases:
        urls, src, dst = read_edge_list(c["lines"])
        names, osrc, odst = sparky_rdd.intern_first_appearance(sparky_rdd.pairs_from_edge_lines(c["lines"]))
        assert urls == names == c["urls"]
        assert src.tolist() == osrc and dst.tolist() == odst


def test_reader_rejects_three_tokens():
    with pytest.raises(ValueError):
        read_edge_list(["a b c"])


def test_reader_skips_blank_lines_and_keeps_tokens_verbatim():
    urls, src, dst = read_edge_list(["", "http://a.b/?q=1 HTTP://A.B", "   ", "x"])
    assert urls == ["http://a.b/?q=1", "HTTP://A.B", "x"]
    assert src.tolist() == [0, 2] and dst.tolist() == [1, -1]


def _read_with_threads(data: bytes, threads: int):
    from sparky_hip import _host

    _host.set_read_threads(threads)
    try:
        e = _host.HostEdges.parse(data)
        out = (e.names(), e.src.tolist(), e.dst.tolist())
        e.close()
        return out
    finally:
        _host.set_read_threads(0)


@pytest.mark.parametrize("threads", [2, 3, 7, 16])
def test_chunked_reader_gives_the_sequential_ids(threads):
    """The multi-threaded edge-list reader (chunks interned locally, merged in chunk order) gives
    exactly the first-appearance IDs of one thread: blank and CRLF lines, link-less records,
    names repeated across chunk boundaries, a last line without a newline."""
    rng = random.Random(threads)
    lines = []
    for i in range(3000):
        r = rng.random()
        if r < 0.05:
            lines.append(rng.choice(["", "   ", "\t"]))
        elif r < 0.15:
            lines.append(f"u{rng.randrange(400)}")
        else:
            a, b = rng.randrange(400), int(rng.paretovariate(1.2)) % 900
            lines.append(f"u{a}{rng.choice([' ', '  ', chr(9)])}u{b}" + ("\r" if rng.random() < 0.1 else ""))
    data = "\n".join(lines).encode()  # no trailing newline
    seq = _read_with_threads(data, 1)
    assert _read_with_threads(data, threads) == seq
    names, src, dst = seq
    ref_names, ref_src, ref_dst = sparky_rdd.intern_first_appearance(
        sparky_rdd.pairs_from_edge_lines([l.rstrip("\r") for l in lines]))
    assert names == ref_names and src == ref_src and dst == ref_dst


def test_chunked_reader_reports_the_global_line_number():
    from sparky_hip import _host

    data = ("a b\n" * 500 + "a b c\n" + "c d\n" * 500).encode()
    for t in (1, 4):
        _host.set_read_threads(t)
        try:
            with pytest.raises(_host.HostError, match="line 501: expected 'src \\[dst\\]', got 3 tokens"):
                _host.HostEdges.parse(data)
        finally:
            _host.set_read_threads(0)


def test_part_file_format(tmp_path):
    d = write_part_file(str(tmp_path), 3, ["u1", "u2"], np.array([1.0, 0.7166666666666667]))
    assert os.path.basename(d) == "PageRank3"
    assert open(os.path.join(d, "part-00000")).read() == "(u1,1.0)\n(u2,0.7166666666666667)\n"
    assert os.path.exists(os.path.join(d, "_SUCCESS"))


def test_has_rank_format():
    buf = io.StringIO()
    write_has_rank(buf, ["a"], np.array([0.15]))
    assert buf.getvalue() == "a has rank: 0.15.\n"


def test_cpp_formatter_matches_python():
    """The C++ CLI's Double.toString (host/javafmt.h) == the Python host's, bit pattern by bit pattern."""
    import subprocess

    from conftest import PKG_DIR

    exe = os.path.join(PKG_DIR, "build", "javafmt_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(PKG_DIR, "host"), exe], check=True)
    rng = random.Random(11)
    vals = [1.1416666666666666, 0.15, 1e7, 9999999.999999998, 1e-3, 9.99e-4, 5e-324, 2e-5, 1.0, 100.0,
            123456.789, 1.7976931348623157e308, 0.0, -0.0, -2.5]
    vals += [struct.unpack("<d", struct.pack("<Q", rng.getrandbits(63)))[0] for _ in range(3000)]
    vals += [rng.uniform(0.15, 50.0) for _ in range(3000)]
    vals = [v for v in vals if v == v]
    inp = "".join(f"{struct.unpack('<Q', struct.pack('<d', v))[0]:x}\n" for v in vals)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
    for v, s in zip(vals, out):
        assert s == java_double_to_string(v), (v, s)


# ---- resume input: saved (url,rank) part files back to ranks in ID order ----
def _edges(lines):
    from sparky_hip._host import HostEdges

    return HostEdges.parse("\n".join(lines).encode())


def test_read_ranks_round_trips_saved_part_files_exactly(tmp_path):
    rng = random.Random(3)
    lines = [f"http://s{i}.org/a,b?x={i} http://s{(i * 7) % 60}.org/" for i in range(60)] + ["lonely"]
    e = _edges(lines)
    ranks = np.array([rng.uniform(0.15, 40.0) for _ in range(e.n_vertices)])
    ranks[3] = 1e-5  # exponent form "1.0E-5"
    e.write_part(str(tmp_path), 4, ranks)
    got = e.read_ranks(str(tmp_path / "PageRank4"))
    assert np.array_equal(got, ranks)  # Double.toString digits restore the double exactly
    e.close()


def test_read_ranks_reads_every_part_file_and_any_line_order(tmp_path):
    e = _edges(["a b", "b c", "c a"])
    d = tmp_path / "PageRank0"
    d.mkdir()
    (d / "part-00000").write_text("(c,0.5)\n")
    (d / "part-00001").write_text("(b,2.0E-3)\r\n\n(a,1.25)\n")
    (d / "_SUCCESS").write_text("")
    assert e.read_ranks(str(d)).tolist() == [1.25, 0.002, 0.5]
    e.close()


@pytest.mark.parametrize("content,msg", [
    ("(a,1.0)\n(b,1.0)\n", "no saved rank"),              # c missing
    ("(a,1.0)\n(b,1.0)\n(c,1.0)\n(zz,1.0)\n", "not in the edge list"),
    ("(a,1.0)\n(a,1.0)\n(b,1.0)\n(c,1.0)\n", "twice"),
    ("a,1.0\n", "expected"),
    ("(a,one)\n", "bad rank"),
])
def test_read_ranks_rejects_inconsistent_saves(tmp_path, content, msg):
    from sparky_hip._host import HostError

    e = _edges(["a b", "b c", "c a"])
    d = tmp_path / "PageRank1"
    d.mkdir()
    (d / "part-00000").write_text(content)
    with pytest.raises(HostError) as ei:
        e.read_ranks(str(d))
    assert msg in str(ei.value)
    with pytest.raises(HostError):
        e.read_ranks(str(tmp_path / "missing"))
    e.close()


def test_saved_iteration_numbering():
    from sparky_hip.driver import saved_iteration

    assert saved_iteration("/x/out/PageRank4") == 4
    assert saved_iteration("/x/out/PageRank12/") == 12
    assert saved_iteration("/x/out/PageRank") == -1
    assert saved_iteration("/x/out/ranks") == -1


def test_init_ranks_length_is_checked():
    from sparky_hip.graph import _init_array

    assert _init_array(None, 3) is None
    assert _init_array([1, 2, 3], 3).dtype == np.float64
    with pytest.raises(ValueError):
        _init_array(np.ones(2), 3)
