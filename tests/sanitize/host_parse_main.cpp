// Seeded mutation fuzzing of libpagerank_host's front-ends (pr_host.cpp prh_parse: the edge list
// and the Common Crawl JSON records of Sparky.java:61-123) for the sanitizer builds of
// tests/test_sanitizers_cpu.py.  A small corpus of valid inputs is mutated (byte flips, inserted
// structural bytes, truncation, splices); every input must either parse or fail with an error
// message, and a parsed one is walked end to end (every name, the Java Double.toString writer).
// argv[1]: iterations; argv[2]: reader threads (the edge-list reader's parallel chunking).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "pagerank_host.h"

namespace {

const char *kEdges[] = {
    "a b\nb c\nc a\n",
    "1 2\n2 3\n3\n4 4\n\n5 1\r\n",
    "http://x.com/ http://y.com/\nhttp://y.com/\nhttp://z.com/ http://x.com/\n",
    "  lead  trail  \n\t tab\tsep\nsolo\n",
};
const char *kCc[] = {
    "http://a.com/\t{\"content\": {\"links\": [{\"href\": \"http://b.com/\", \"type\": \"a\"}, "
    "{\"href\": \"http://c.com/\", \"type\": \"link\"}]}}\n",
    "http://b.com/\t{\"content\": {\"links\": []}}\nhttp://c.com/\t{\"content\": {}}\n",
    "http://e.com/\t{\"content\": {\"links\": [{\"href\": \"q\\\"uote\\\\back\", \"type\": \"a\"}]}}\n",
    "http://h.com/\t{\"content\": {\"links\": [{\"href\": 12.50, \"type\": \"a\"}, {\"href\": true, \"type\": \"a\"}, "
    "{\"href\": null, \"type\": \"a\"}, {\"href\": {\"k\": \"v\", \"n\": [1, \"x\"]}, \"type\": \"a\"}]}}\n",
    "http://g.com/\t{\"content\": {\"links\": [{\"href\": \"\\u00fc\\u8def/\xc3\xa9\", \"type\": \"a\"}]}}\n",
    "http://i.com/\t)]}'\n{\"content\": {\"links\": [{'href': 'x', type: a}]}}\n",
};
const char kStruct[] = "{}[]\":,\\\t\n \r'u0123456789.-+eE/";

std::string mutate(std::string s, std::mt19937_64 &rng) {
  const int n = 1 + (int)(rng() % 6);
  for (int k = 0; k < n; ++k) {
    const size_t len = s.size();
    switch (rng() % 6) {
      case 0:  // flip a byte
        if (len) s[rng() % len] = (char)(rng() & 0xff);
        break;
      case 1:  // insert a structural byte
        s.insert(len ? rng() % (len + 1) : 0, 1, kStruct[rng() % (sizeof kStruct - 1)]);
        break;
      case 2:  // truncate
        if (len) s.resize(rng() % len);
        break;
      case 3:  // delete a span
        if (len > 1) {
          const size_t a = rng() % len;
          s.erase(a, 1 + rng() % std::min<size_t>(16, len - a));
        }
        break;
      case 4:  // duplicate a span (deep nesting, repeated keys)
        if (len > 1) {
          const size_t a = rng() % len, b = 1 + rng() % std::min<size_t>(32, len - a);
          s.insert(rng() % (s.size() + 1), s.substr(a, b));
        }
        break;
      default:  // a NUL or high byte
        s.insert(len ? rng() % (len + 1) : 0, 1, (rng() & 1) ? '\0' : (char)0xff);
    }
  }
  return s;
}

volatile int64_t sink;

int walk(const prh_edges *e) {
  const int64_t ne = prh_n_edges(e);
  const int32_t nv = prh_n_vertices(e);
  const int32_t *src = prh_src(e), *dst = prh_dst(e);
  int64_t acc = 0;
  for (int64_t i = 0; i < ne; ++i) {
    if (src[i] < 0 || src[i] >= nv || dst[i] < -1 || dst[i] >= nv) return 1;
    acc += src[i] + dst[i];
  }
  for (int32_t v = 0; v < nv; ++v) {
    int64_t len = -1;
    const char *p = prh_name(e, v, &len);
    if (!p || len < 0) return 1;
    for (int64_t k = 0; k < len; ++k) acc += (unsigned char)p[k];
  }
  sink = acc;  // keeps the walk
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  prh_set_read_threads(argc > 2 ? std::atoi(argv[2]) : 1);
  std::mt19937_64 rng(12345);
  int parsed = 0, rejected = 0, bad = 0;
  for (int it = 0; it < iters; ++it) {
    const bool cc = (it & 1) != 0;
    std::string in;
    const int parts = 1 + (int)(rng() % 3);
    for (int p = 0; p < parts; ++p)
      in += cc ? kCc[rng() % (sizeof kCc / sizeof *kCc)] : kEdges[rng() % (sizeof kEdges / sizeof *kEdges)];
    if (it % 4 != 0) in = mutate(in, rng);
    prh_edges *e = nullptr;
    const int rc = prh_parse(in.data(), (int64_t)in.size(), cc ? PRH_FORMAT_CCJSON : PRH_FORMAT_EDGES, &e);
    if (rc == 0) {
      ++parsed;
      if (!e || walk(e)) ++bad;
      prh_free(e);
    } else {
      ++rejected;
      const char *m = prh_last_error();
      if (e || !m || !*m) ++bad;
    }
  }
  // the Java Double.toString writer over awkward values
  char buf[64];
  const double xs[] = {0.0, -0.0, 1.0, 0.15, 1e-300, 5e-324, 1.7976931348623157e308, 1e7, 9999999.999, 1e-3,
                       0.001, 123456789012345678.0, 0.1 + 0.2};
  for (double x : xs)
    if (prh_java_double(x, buf) <= 0) ++bad;
  for (int k = 0; k < 20000; ++k) {
    uint64_t b = rng();
    double x;
    static_assert(sizeof x == sizeof b, "");
    __builtin_memcpy(&x, &b, sizeof x);
    if (x != x) continue;  // NaN is never a rank
    if (prh_java_double(x, buf) <= 0) ++bad;
  }
  std::printf("parsed %d rejected %d bad %d\n", parsed, rejected, bad);
  return bad != 0;
}
