"""Common Crawl JSON front-end (Sparky.java:78-123) on CPU: the native
libpagerank_host parser against the oracle restatement (oracle/sparky_rdd.py), including the
Gson JsonElement.toString() quirks the reference's `aLink.replace("\"", "")` relies on."""
import json
import random

import pytest

import sparky_rdd
from sparky_hip import HostEdges, HostError

RECORDS = [
    ("http://a.com/", {"content": {"links": [{"href": "http://b.com/", "type": "a"},
                                             {"href": "http://c.com/", "type": "link"},
                                             {"href": "http://b.com/", "type": "a"}]}}),
    ("http://b.com/", {"content": {"links": []}}),  # empty links: dangling record
    ("http://c.com/", {"content": {}}),  # no links
    ("http://d.com/", {"other": 1}),  # no content
    ("http://e.com/", {"content": {"links": [{"href": "q\"uote\\back", "type": "a"}]}}),
    ("http://f.com/", {"content": {"links": [{"href": "tab\there\nnl\u0001ctl ls", "type": "a"}]}}),
    ("http://g.com/", {"content": {"links": [{"href": "üñí©ødé/路径", "type": "a"}]}}),
    ("http://h.com/", {"content": {"links": [{"href": 12.50, "type": "a"}, {"href": True, "type": "a"},
                                             {"href": None, "type": "a"},
                                             {"href": {"k": "v", "n": [1, "x"]}, "type": "a"}]}}),
    ("http://i.com/", {"content": {"links": [{"href": "http://a.com/", "type": "A"},
                                             {"href": "http://a.com/", "type": ["a"]}]}}),
    ("http://j.com/", {"content": {"links": [{"href": "http://j.com/", "type": "a"}]}}),  # self loop
]


def lines():
    return [f"{u}\t{json.dumps(j, ensure_ascii=False)}" for u, j in RECORDS]


def native(text: str, fmt="ccjson"):
    e = HostEdges.parse(text.encode("utf-8"), fmt)
    names = e.names()
    out = [(names[s], None if d < 0 else names[d]) for s, d in zip(e.src.tolist(), e.dst.tolist())]
    e.close()
    return out, names


def test_ccjson_matches_oracle():
    want = sparky_rdd.pairs_from_ccjson_lines(lines())
    got, names = native("\n".join(lines()) + "\n")
    assert got == want
    wnames, _, _ = sparky_rdd.intern_first_appearance(want)
    assert names == wnames
    d = dict((u, v) for u, v in want if u == "http://e.com/")
    assert d["http://e.com/"] == "q\\uote\\\\back"  # escaped quote keeps its backslash
    hrefs = [v for u, v in want if u == "http://h.com/"]
    assert hrefs == ["12.5", "true", "null", "{k:v,n:[1,x]}"]  # numbers keep their source text
    assert ("http://i.com/", None) in want  # "A" / ["a"] are not type "a"


def test_ccjson_number_source_text_kept():
    text = 'u\t{"content":{"links":[{"href":1.50e+2,"type":"a"}]}}'
    assert native(text)[0] == sparky_rdd.pairs_from_ccjson_lines([text]) == [("u", "1.50e+2")]


def test_ccjson_duplicate_keys_last_wins():
    text = 'u\t{"content":{"links":[{"href":"x","type":"a","href":"y"}]}}'
    want = sparky_rdd.pairs_from_ccjson_lines([text])
    got, _ = native(text)
    assert got == want == [("u", "y")]


@pytest.mark.parametrize("bad", [
    'u\t[1,2]',  # not an object (IllegalStateException)
    'u\t{"content":[1]}',  # content not an object
    'u\t{"content":null}',  # JsonNull -> ClassCastException
    'u\t{"content":{"links":{"a":1}}}',  # links not an array
    'u\t{"content":{"links":[{"type":"a"}]}}',  # missing href -> NPE
    'u\t{"content":{"links":[{"href":"x"}]}}',  # missing type -> NPE
    'u\t{"content":{"links":[3]}}',  # link not an object
    'u\t{"content": {',  # malformed JSON
    'no tab here',
])
def test_ccjson_errors_like_reference(bad):
    with pytest.raises(ValueError):
        sparky_rdd.pairs_from_ccjson_lines([bad])
    with pytest.raises(HostError):
        native(bad)


def test_ccjson_random_records():
    rng = random.Random(3)
    alphabet = ["a", "b", "/", "\"", "\\", "\t", "é", " ", " ", "?", "="]
    recs = []
    for i in range(300):
        links = []
        for _ in range(rng.randrange(0, 6)):
            href = "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 8)))
            links.append({"href": href, "type": rng.choice(["a", "a", "img", "link"])})
        rec = {"content": {"links": links}} if rng.random() < 0.9 else {}
        recs.append(f"u{rng.randrange(100)}\t{json.dumps(rec, ensure_ascii=rng.random() < 0.5)}")
    want = sparky_rdd.pairs_from_ccjson_lines(recs)
    got, _ = native("\n".join(recs))
    assert got == want


def test_native_edge_list_matches_python_reader(golden_cases):
    import sparky_hip

    for c in golden_cases:
        got, names = native("\n".join(c["lines"]) + "\n", "edges")
        urls, src, dst = sparky_hip.read_edge_list(c["lines"])
        assert names == urls
        assert got == [(urls[s], None if d < 0 else urls[d]) for s, d in zip(src.tolist(), dst.tolist())]


# Gson's lenient reader (Sparky.java:87 `new JsonParser().parse(String)`): records a strict
# RFC 8259 parser would reject.  Native front-end against the oracle restatement; both restate
# Gson's published lenient rules, and no reference run pins them (parity unpinned).
LENIENT = [
    "http://l1.com/\t{'content': {'links': [{'href': 'http://x.com/', 'type': 'a'}]}}",  # single quotes
    "http://l2.com/\t{content: {links: [{href: y.com?q, type: a}]}}",  # unquoted names/strings (no : / in them)
    "http://l3.com/\t{\"content\" = {\"links\" => [{\"href\": \"http://z.com/\"; \"type\": \"a\"}]}}",  # = => ;
    "http://l4.com/\t{\"content\": {\"links\": [{\"href\": \"http://x.com/\", \"type\": \"a\"}], \"o\": [1,,2,]}}",  # nulls
    "http://l5.com/\t// lead comment\n",  # placeholder replaced below (comments need one line)
    "http://l6.com/\t{\"content\": {\"links\": [{\"href\": NaN, \"type\": a}, {\"href\": 01, \"type\": a},"
    " {\"href\": -0, \"type\": a}, {\"href\": TRUE, \"type\": a}, {\"href\": nulL, \"type\": a}]}}",
    "http://l7.com/\t)]}'\n",  # placeholder (prefix)
]
LENIENT[4] = "http://l5.com/\t/* c */ {\"content\": /* in */ {\"links\": []}} # trailing comment"
LENIENT[6] = "http://l7.com/\t{\"content\": {\"links\": [{\"href\": \"u\\'q\", \"type\": 'a'}]}} /* tail */"


def test_ccjson_lenient_records_match_oracle():
    want = sparky_rdd.pairs_from_ccjson_lines(LENIENT)
    got, _ = native("\n".join(LENIENT) + "\n")
    assert got == want
    d = {}
    for u, v in want:
        d.setdefault(u, []).append(v)
    assert d["http://l1.com/"] == ["http://x.com/"] and d["http://l2.com/"] == ["y.com?q"]
    assert d["http://l3.com/"] == ["http://z.com/"] and d["http://l4.com/"] == ["http://x.com/"]
    assert d["http://l5.com/"] == [None]  # no links: a record without links
    # unquoted NaN / 01 are strings, -0 a number, TRUE / nulL keywords (Gson's peekKeyword)
    assert d["http://l6.com/"] == ["NaN", "01", "-0", "true", "null"]


@pytest.mark.parametrize("bad", ["{\"content\": {\"a\": 1,}}", "{content: {links: [{href: http://x.com/}]}}", "{\"content\": 1} {\"x\": 2}", "{'a': 'open}",
                                 "{/* unterminated : 1}", "{\"a\" 1}",
                                 "{\"content\": {\"links\": [{\"href\": \"h\", \"type\": \"a\"},,]}}"])
def test_ccjson_lenient_still_rejects(bad):
    with pytest.raises(HostError):
        native(f"http://bad.com/\t{bad}\n")
    with pytest.raises(ValueError):
        sparky_rdd.pairs_from_ccjson_lines([f"http://bad.com/\t{bad}"])


def test_nonexecute_prefix_after_leading_whitespace():
    """Gson's consumeNonExecutePrefix skips leading whitespace and (lenient) comments before it
    looks for ")]}'\\n" (ADVICE r2); the native parser (pr_host.cpp JParser::parse) applies the same
    rule.  A line-framed record cannot hold the prefix's newline, so this is checked on the
    restatement's parser directly."""
    for text in (")]}'\n{\"a\": 1}", "  )]}'\n{\"a\": 1}", "\t/* c */ )]}'\n {\"a\": 1}"):
        assert sparky_rdd._parse_json(text) == ("obj", [("a", sparky_rdd._Num("1"))])
    with pytest.raises(ValueError):
        sparky_rdd._parse_json("x )]}'\n{\"a\": 1}")


@pytest.mark.parametrize("threads", [2, 5])
def test_ccjson_chunked_reader_matches_one_thread(threads):
    """The Common Crawl front-end on several threads (chunks of whole records, merged in chunk
    order): the same (url, href) pairs, IDs and names as one thread, and errors at the file's line."""
    from sparky_hip import _host

    rng = random.Random(threads)
    recs = []
    for i in range(2000):
        links = [{"href": f"h{rng.randrange(300)}" + ("\"" if rng.random() < 0.1 else ""),
                  "type": rng.choice(["a", "a", "img"])} for _ in range(rng.randrange(0, 5))]
        rec = {"content": {"links": links}} if rng.random() < 0.9 else {}
        recs.append(f"u{rng.randrange(500)}\t{json.dumps(rec)}")
        if rng.random() < 0.02:
            recs.append("")
    data = "\n".join(recs).encode()

    def read(t, d):
        _host.set_read_threads(t)
        try:
            e = _host.HostEdges.parse(d, "ccjson")
            out = (e.names(), e.src.tolist(), e.dst.tolist())
            e.close()
            return out
        finally:
            _host.set_read_threads(0)

    assert read(threads, data) == read(1, data)
    names, src, dst = read(threads, data)
    assert [(names[s], None if d < 0 else names[d]) for s, d in zip(src, dst)] == \
        sparky_rdd.pairs_from_ccjson_lines(recs)
    bad = data + b"\nu1\t{\"content\": 3}\n"
    for t in (1, threads):
        _host.set_read_threads(t)
        try:
            with pytest.raises(HostError, match=f"line {len(recs) + 1}: 'content' is not an object"):
                _host.HostEdges.parse(bad, "ccjson")
        finally:
            _host.set_read_threads(0)
