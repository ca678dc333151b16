"""Oracle #1 -- literal RDD-level restatement of Sparky.java's PageRank (TEST INFRASTRUCTURE).

This module is a *checker*, not product code.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  The product path
(``libpagerank_hip``) never routes through it.

It emulates, on Python dicts/sets, the Spark operators Sparky.java applies, line by line,
so that every quirk of the reference survives:

* ``pairs`` is the output of the link-extraction ``flatMapToPair`` (Sparky.java:78-123):
  ``(url, href)`` for each ``type=="a"`` link (:107) and ``(url, None)`` for a record with
  no ``a`` link (:114-118, which also does ``dangUrls.add(url)``).  The edge-list
  front-end maps a line ``u v`` to ``(u, v)`` and a single-token line ``u`` to ``(u, None)``.
* ``distinct().groupByKey()`` (:124), key collect/broadcast (:127-135), sink completion
  (:137-159), ``union`` (:161), ``count`` (:162), rank init to 1.0 (:165-170), the
  dangling-set fixup with ``lookup`` (:172-184), and the 10-iteration loop (:187-238):
  join/flatMap contributions (:192-216), dangling sum (:219-222), ``subtractByKey`` +
  ``union`` in-degree-0 quirk (:224-225), ``reduceByKey(Sum)`` + affine update (:229-235).

Parity status: **unpinned against a run of the reference** -- the reference cannot run here
(no JDK/Spark in the image) and ships no tests or golden vectors.  The
emulator is pinned to the hand-derived known-answer test of SURVEY.md §4 (see
``tests/test_oracle.py``) and cross-checked against the C restatement ``pagerank_oracle.c``.

Summation order: Spark's ``reduceByKey`` and the driver's HashSet iteration order are
unspecified (Sparky.java:219-222, :229); this oracle uses exactly rounded sums
(``math.fsum``), the order-independent ideal that any Spark order approximates to ~1 ulp·n.
"""
from __future__ import annotations

import math
import re
from collections import OrderedDict
from typing import Dict, Hashable, Iterable, List, Optional, Sequence, Tuple

TELEPORT = 0.15  # Sparky.java:233
DAMPING = 0.85  # Sparky.java:233


def pairs_from_edge_lines(lines: Iterable[str]) -> List[Tuple[str, Optional[str]]]:
    """Edge-list front-end: ``u v`` -> (u, v); ``u`` -> (u, None) (Sparky.java:107, :116).

    Tokens are taken verbatim (whitespace separated).  Blank lines are ignored.  Extra
    tokens beyond the second are an error (the product reader rejects them too).
    """
    out: List[Tuple[str, Optional[str]]] = []
    for ln, line in enumerate(lines):
        toks = line.split()
        if not toks:
            continue
        if len(toks) == 1:
            out.append((toks[0], None))
        elif len(toks) == 2:
            out.append((toks[0], toks[1]))
        else:
            raise ValueError(f"line {ln + 1}: expected 1 or 2 tokens, got {len(toks)}")
    return out


def intern_first_appearance(pairs: Sequence[Tuple[str, Optional[str]]]):
    """Canonical ID mapping: first appearance, ``src`` before ``dst``.

    Returns ``(names, src_ids, dst_ids)`` with ``dst_ids[i] == -1`` for a no-link record.
    """
    ids: Dict[str, int] = {}
    names: List[str] = []
    src_ids: List[int] = []
    dst_ids: List[int] = []
    for u, v in pairs:
        if u not in ids:
            ids[u] = len(names)
            names.append(u)
        src_ids.append(ids[u])
        if v is None:
            dst_ids.append(-1)
        else:
            if v not in ids:
                ids[v] = len(names)
                names.append(v)
            dst_ids.append(ids[v])
    return names, src_ids, dst_ids


class SparkyRDD:
    """Graph construction of Sparky.java:124-184, kept as dict-shaped 'RDDs'."""

    def __init__(self, pairs: Sequence[Tuple[Hashable, Optional[Hashable]]], dangling: str = "local"):
        if dangling not in ("local", "none"):
            raise ValueError("dangling must be 'local' or 'none'")
        self.dangling = dangling
        # Sparky.java:117 -- dangUrls.add(url) for records without 'a' links.  In cluster mode
        # the executor-side static never reaches the driver: D stays empty.
        dang_urls = set()
        if dangling == "local":
            dang_urls.update(u for u, t in pairs if t is None)
        # Sparky.java:124 -- .distinct().groupByKey(); insertion order is irrelevant.
        links: "OrderedDict[Hashable, List[Optional[Hashable]]]" = OrderedDict()
        for u, t in OrderedDict.fromkeys(pairs):
            links.setdefault(u, []).append(t)
        # Sparky.java:127-135 -- key set broadcast.
        key_set = set(links)
        # Sparky.java:137-159 -- sink completion: (url, null) for every target not a key.
        sinks: "OrderedDict[Hashable, None]" = OrderedDict()
        for _k, lst in links.items():
            # arg._2 is never null after groupByKey, so the else-branch (:152-155) is dead.
            for url in lst:
                if url not in key_set and url is not None:
                    if dangling == "local":
                        dang_urls.add(url)  # :148
                    sinks[url] = None
        # Sparky.java:161 -- union; keys are disjoint by construction.
        self.all_urls: "OrderedDict[Hashable, Optional[List[Optional[Hashable]]]]" = OrderedDict(links)
        for s in sinks:
            self.all_urls[s] = None
        # Sparky.java:162 -- totalUrlCount.
        self.total_url_count = len(self.all_urls)
        # Sparky.java:172-184 -- fixup: keep s only if lookup(s) is [null].
        not_dangling = set()
        for s in dang_urls:
            look = [self.all_urls[s]] if s in self.all_urls else []
            if not (look is None or len(look) == 0 or (len(look) == 1 and look[0] is None)):
                not_dangling.add(s)
        self.dang_urls = dang_urls - not_dangling

    def initial_ranks(self) -> Dict[Hashable, float]:
        """Sparky.java:165-170 -- every URL starts at rank 1.0 (no 1/N normalisation)."""
        return {u: 1.0 for u in self.all_urls}

    def iterate(self, ranks: Dict[Hashable, float]) -> Tuple[Dict[Hashable, float], float]:
        """One pass of Sparky.java:189-235. Returns (new_ranks, danglingContrib)."""
        # :192-216 -- contributions.
        contribs: Dict[Hashable, List[float]] = {}
        for u, lst in self.all_urls.items():
            if lst is None:
                continue  # sink-only vertex: null Iterable, emits nothing (:198)
            url_count = len(lst)  # Iterables.size counts nulls (:199)
            for s in lst:
                if s is None:
                    url_count -= 1  # :200-205
            if url_count == 0:
                continue  # r/0 = +Inf in Java (:207) but nothing is emitted (:208-211)
            page_rank = ranks[u] / url_count  # one fp64 division (:207)
            for s in lst:
                if s is not None:
                    contribs.setdefault(s, []).append(page_rank)
        # :219-222 -- danglingContrib over the fixed-up dangUrls (sink-only vertices).
        dc = math.fsum(ranks[u] for u in self.dang_urls)
        # :224-225 -- vertices without a contribution re-use their OLD rank as the "sum".
        for u in ranks:
            if u not in contribs:
                contribs[u] = [ranks[u]]
        # :229-235 -- reduceByKey(Sum) then 0.15 + 0.85 * (sum + dc / N).
        n = float(self.total_url_count)
        new_ranks = {}
        for u in ranks:
            s = math.fsum(contribs[u])
            new_ranks[u] = TELEPORT + DAMPING * (s + dc / n)
        return new_ranks, dc


def run(pairs, iterations: int = 10, dangling: str = "local", init: Optional[Dict] = None):
    """Run the whole job; returns (graph, list of per-iteration rank dicts, list of dc)."""
    g = SparkyRDD(pairs, dangling=dangling)
    ranks = dict(init) if init is not None else g.initial_ranks()
    history, dcs = [], []
    for _ in range(iterations):  # Sparky.java:187
        ranks, dc = g.iterate(ranks)
        history.append(ranks)
        dcs.append(dc)
    return g, history, dcs


# ---- Common Crawl JSON front-end (Sparky.java:84-118), restated with Python's json -----------
class _Num(str):
    """A JSON number kept as its source text (Gson's LazilyParsedNumber prints it verbatim)."""


def _gson_str(s: str) -> str:
    """JsonWriter.value(String) with htmlSafe = false (JsonElement.toString())."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\t":
            out.append("\\t")
        elif ch == "\b":
            out.append("\\b")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\f":
            out.append("\\f")
        elif o < 0x20:
            out.append(f"\\u{o:04x}")
        elif o in (0x2028, 0x2029):
            out.append(f"\\u{o:04x}")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def gson_to_string(v) -> str:
    """JsonElement.toString() of a value parsed by _parse_json."""
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, _Num):
        return str.__str__(v)
    if isinstance(v, str):
        return _gson_str(v)
    if isinstance(v, list):
        return "[" + ",".join(gson_to_string(x) for x in v) + "]"
    # object: list of (key, value) pairs; LinkedTreeMap keeps first position, last value
    pairs = v[1]
    last = {}
    for k, x in pairs:
        last[k] = x
    seen, parts = set(), []
    for k, _ in pairs:
        if k in seen:
            continue
        seen.add(k)
        parts.append(_gson_str(k) + ":" + gson_to_string(last[k]))
    return "{" + ",".join(parts) + "}"


_NOT_LITERAL = set("/\\;#={}[]:, \t\f\r\n")
_ESCAPES = {'"': '"', "'": "'", "\\": "\\", "/": "/", "b": "\b", "f": "\f", "n": "\n", "r": "\r", "t": "\t",
            "\n": "\n"}
_NUMBER = re.compile(r"-?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?\Z")


def _parse_json(text: str):
    """Gson's lenient JsonReader as Sparky.java:87 `new JsonParser().parse(String)` runs it:
    comments (//, # to the end of the line; /* */), single-quoted and unquoted names and strings,
    '=' / '=>' for ':', ';' for ',', an omitted array element read as null, the ")]}'\n"
    prefix, one top-level value.  Unquoted literal: keyword (true/false/null, each letter in
    either case) / JSON number (no leading zeros) / else string.  Restated from Gson's published
    JsonReader rules (version unpinned): lenient inputs are parity-unpinned.
    Objects: ("obj", [(key, value), ...]); numbers: _Num (source text)."""
    n = len(text)
    pos = [0]

    def fail(msg):
        raise ValueError(f"JSON: {msg} at {pos[0]}")

    def ws():
        i = pos[0]
        while i < n:
            c = text[i]
            if c in " \t\n\r":
                i += 1
            elif c == "#" or text.startswith("//", i):
                while i < n and text[i] != "\n":
                    i += 1
            elif text.startswith("/*", i):
                j = text.find("*/", i + 2)
                if j < 0:
                    pos[0] = i
                    fail("unterminated comment")
                i = j + 2
            else:
                break
        pos[0] = i

    def string(quote):
        i = pos[0] + 1
        out = []
        while True:
            if i >= n:
                fail("unterminated string")
            c = text[i]
            i += 1
            if c == quote:
                pos[0] = i
                return "".join(out)
            if c != "\\":
                out.append(c)
                continue
            if i >= n:
                fail("bad escape")
            x = text[i]
            i += 1
            if x == "u":
                h = text[i:i + 4]
                if len(h) < 4 or any(ch not in "0123456789abcdefABCDEF" for ch in h):
                    fail("bad \\u escape")
                v = int(h, 16)
                i += 4
                if 0xD800 <= v < 0xDC00 and text.startswith("\\u", i):
                    h2 = text[i + 2:i + 6]
                    if len(h2) == 4 and all(ch in "0123456789abcdefABCDEF" for ch in h2) and 0xDC00 <= int(h2, 16) < 0xE000:
                        v = 0x10000 + ((v - 0xD800) << 10) + (int(h2, 16) - 0xDC00)
                        i += 6
                out.append(chr(v))
            elif x in _ESCAPES:
                out.append(_ESCAPES[x])
            else:
                fail("bad escape")

    def unquoted():
        i = j = pos[0]
        while j < n and text[j] not in _NOT_LITERAL:
            j += 1
        if j == i:
            fail("expected value")
        pos[0] = j
        return text[i:j]

    def keyword(s, word):
        return len(s) == len(word) and all(a in (b, b.upper()) for a, b in zip(s, word))

    def value(depth):
        if depth > 512:
            fail("nesting too deep")
        ws()
        if pos[0] >= n:
            fail("unexpected end")
        c = text[pos[0]]
        if c == "{":
            pos[0] += 1
            pairs = []
            ws()
            if pos[0] < n and text[pos[0]] == "}":
                pos[0] += 1
                return ("obj", pairs)
            while True:
                ws()
                if pos[0] >= n or text[pos[0]] == "}":
                    fail("expected name")
                k = string(text[pos[0]]) if text[pos[0]] in "\"'" else unquoted()
                ws()
                if pos[0] < n and text[pos[0]] == ":":
                    pos[0] += 1
                elif pos[0] < n and text[pos[0]] == "=":
                    pos[0] += 2 if text.startswith("=>", pos[0]) else 1
                else:
                    fail("expected ':'")
                pairs.append((k, value(depth + 1)))
                ws()
                if pos[0] < n and text[pos[0]] in ",;":
                    pos[0] += 1
                    continue
                if pos[0] < n and text[pos[0]] == "}":
                    pos[0] += 1
                    return ("obj", pairs)
                fail("expected ',' or '}'")
        if c == "[":
            pos[0] += 1
            arr = []
            ws()
            if pos[0] < n and text[pos[0]] == "]":
                pos[0] += 1
                return arr
            while True:
                ws()
                if pos[0] < n and text[pos[0]] in ",;]":
                    arr.append(None)  # an omitted element is null (lenient)
                else:
                    arr.append(value(depth + 1))
                ws()
                if pos[0] < n and text[pos[0]] in ",;":
                    pos[0] += 1
                    continue
                if pos[0] < n and text[pos[0]] == "]":
                    pos[0] += 1
                    return arr
                fail("expected ',' or ']'")
        if c in "\"'":
            return string(c)
        lit = unquoted()
        if keyword(lit, "true"):
            return True
        if keyword(lit, "false"):
            return False
        if keyword(lit, "null"):
            return None
        return _Num(lit) if _NUMBER.match(lit) else lit

    # consumeNonExecutePrefix: leading whitespace (and, lenient, comments) is skipped first,
    # then a ")]}'\n" prefix is dropped
    ws()
    if text.startswith(")]}'\n", pos[0]):
        pos[0] += 5
    v = value(0)
    ws()
    if pos[0] != n:
        fail("trailing characters")
    return v


def _get(obj, key):
    """JsonObject.get(name): last duplicate wins; None when absent."""
    r = None
    for k, x in obj[1]:
        if k == key:
            r = x
    return r


def _is_obj(v):
    return isinstance(v, tuple) and len(v) == 2 and v[0] == "obj"


def pairs_from_ccjson_lines(lines: Iterable[str]) -> List[Tuple[str, Optional[str]]]:
    """'url<TAB>json' records -> the flatMapToPair output of Sparky.java:78-123.

    Raises ValueError where the reference's executor would throw (malformed JSON,
    ClassCastException / IllegalStateException on wrong types, NullPointerException on a link
    without "href" or "type")."""
    out: List[Tuple[str, Optional[str]]] = []
    for ln, line in enumerate(lines):
        line = line.rstrip("\n").rstrip("\r")
        if not line:
            continue
        if "\t" not in line:
            raise ValueError(f"line {ln + 1}: expected url<TAB>json")
        url, text = line.split("\t", 1)
        root = _parse_json(text)  # Sparky.java:87
        if not _is_obj(root):  # :88
            raise ValueError(f"line {ln + 1}: record is not a JSON object")
        dangling = True  # :90
        content = _get(root, "content")  # :89
        if content is not None or any(k == "content" for k, _ in root[1]):
            if not _is_obj(content):  # JsonNull / non-object -> ClassCastException
                raise ValueError(f"line {ln + 1}: 'content' is not an object")
            links = _get(content, "links")  # :93
            if links is not None or any(k == "links" for k, _ in content[1]):
                if not isinstance(links, list):
                    raise ValueError(f"line {ln + 1}: 'links' is not an array")
                for el in links:  # :98-110
                    if not _is_obj(el):
                        raise ValueError(f"line {ln + 1}: link is not an object")
                    href, typ = _get(el, "href"), _get(el, "type")
                    has_h = any(k == "href" for k, _ in el[1])
                    has_t = any(k == "type" for k, _ in el[1])
                    if not has_h or not has_t:
                        raise ValueError(f"line {ln + 1}: link without href/type (NPE)")
                    if gson_to_string(typ) != '"a"':  # :103
                        continue
                    out.append((url, gson_to_string(href).replace('"', "")))  # :101, :105, :107
                    dangling = False
        if dangling:
            out.append((url, None))  # :114-118
    return out
