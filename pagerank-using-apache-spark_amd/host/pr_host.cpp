// libpagerank_host: native input front-ends, URL interning and output writers (CPU).
// See include/pagerank_host.h.  Everything before the GPU build and after the iteration.
#include "pagerank_host.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <dirent.h>

#include <sched.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "javafmt.h"

namespace {

thread_local std::string g_err;
int fail(const std::string &m) {
  g_err = m;
  return -1;
}

// ---- first-appearance interner over string_views (storage owned elsewhere) ----------------
class Interner {
 public:
  // expect: a guess of the distinct names; the table starts at most 2^17 slots and doubles as it
  // fills (a table sized for the input bytes would be mostly empty and miss the caches / TLB on
  // every probe: an edge list names each URL many times)
  explicit Interner(size_t expect) { rehash(next_pow2(std::min<size_t>(std::max<size_t>(expect * 2, 2048), 1 << 17))); }
  int32_t intern(std::string_view s) { return intern_hashed(s, hash(s)); }
  int32_t intern_hashed(std::string_view s, uint64_t h) {
    size_t i = h & mask_;
    while (true) {
      Slot &sl = slots_[i];
      if (sl.id < 0) {
        sl.id = (int32_t)names_.size();
        sl.hash = h;
        sl.p = s.data();
        sl.len = (uint32_t)s.size();
        names_.push_back(s);
        hashes_.push_back(h);
        if (names_.size() * 2 > slots_.size()) rehash(slots_.size() * 2);
        return (int32_t)names_.size() - 1;
      }
      if (sl.hash == h && sl.len == s.size() && std::memcmp(sl.p, s.data(), s.size()) == 0) return sl.id;
      i = (i + 1) & mask_;
    }
  }
  // software prefetch of a probe's first slot, then of the name it holds (batched readers)
  void prefetch_slot(uint64_t h) const { __builtin_prefetch(&slots_[h & mask_]); }
  void prefetch_name(uint64_t h) const {
    const Slot &sl = slots_[h & mask_];
    if (sl.id >= 0) __builtin_prefetch(sl.p);
  }
  std::vector<std::string_view> &names() { return names_; }
  const std::vector<uint64_t> &hashes() const { return hashes_; }
  // 8 bytes per step (multiply-xorshift), the tail bytes packed into one word, murmur finaliser
  static uint64_t hash(std::string_view s) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)s.size();
    const char *p = s.data();
    size_t n = s.size();
    for (; n >= 8; n -= 8, p += 8) {
      uint64_t w;
      std::memcpy(&w, p, 8);
      h = (h ^ w) * 0xff51afd7ed558ccdull;
      h ^= h >> 29;
    }
    uint64_t t = 0;
    for (size_t k = 0; k < n; ++k) t |= (uint64_t)(unsigned char)p[k] << (8 * k);
    h = (h ^ t) * 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    return h ^ (h >> 33);
  }

 private:
  struct Slot {  // the name's bytes are compared in place (one memory access per hit)
    uint64_t hash;
    const char *p;
    uint32_t len;
    int32_t id;
  };
  static size_t next_pow2(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
  }
  void rehash(size_t n) {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(n, Slot{0, nullptr, 0, -1});
    mask_ = n - 1;
    for (const Slot &sl : old) {
      if (sl.id < 0) continue;
      size_t i = sl.hash & mask_;
      while (slots_[i].id >= 0) i = (i + 1) & mask_;
      slots_[i] = sl;
    }
  }
  std::vector<Slot> slots_;
  std::vector<std::string_view> names_;
  std::vector<uint64_t> hashes_;
  size_t mask_ = 0;
};

// ---- minimal JSON DOM (RFC 8259) with Gson JsonElement.toString() re-serialisation ----------
struct JVal {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  std::string s;  // NUM: source text; STR: decoded UTF-8
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;  // insertion order, duplicate keys: last wins
  const JVal *get(std::string_view k) const {
    const JVal *r = nullptr;
    for (auto &kv : obj)
      if (kv.first == k) r = &kv.second;
    return r;
  }
};

// Gson's lenient JsonReader (Sparky.java:87 `new JsonParser().parse(String)` parses leniently):
// comments (// and # to the end of the line, /* */), 'single-quoted' and unquoted names and
// strings, '=' or '=>' for ':', ';' for ',', a missing array element read as null ("[1,,2]",
// "[1,]"), the ")]}'\n" non-execute prefix; one top-level value.  An unquoted literal is a
// keyword (true/false/null, each letter in either case), a JSON number (no leading zeros), or
// else a string.  Restated from Gson's published JsonReader documentation and behaviour; the
// reference's Gson version is unpinned, so lenient inputs are parity-unpinned.
class JParser {
 public:
  JParser(const char *p, const char *e) : p_(p), e_(e) {}
  bool parse(JVal &out) {
    // Gson's consumeNonExecutePrefix skips leading whitespace (and, lenient, comments) first
    static const char kPrefix[] = ")]}'\n";
    if (!ws()) return false;
    if ((size_t)(e_ - p_) >= 5 && std::memcmp(p_, kPrefix, 5) == 0) p_ += 5;
    if (!value(out, 0)) return false;
    if (!ws()) return false;
    if (p_ != e_) return err("trailing characters");
    return true;
  }
  std::string error;

 private:
  const char *p_, *e_;
  bool err(const char *m) {
    if (error.empty()) error = m;
    return false;
  }
  bool ws() {  // whitespace and comments
    while (p_ < e_) {
      const char c = *p_;
      if (c == ' ' || c == '\t' || c == '\n' || c == '\r') {
        ++p_;
      } else if (c == '#' || (c == '/' && p_ + 1 < e_ && p_[1] == '/')) {
        while (p_ < e_ && *p_ != '\n') ++p_;
      } else if (c == '/' && p_ + 1 < e_ && p_[1] == '*') {
        const char *q = p_ + 2;
        while (q + 1 < e_ && !(q[0] == '*' && q[1] == '/')) ++q;
        if (q + 1 >= e_) return err("unterminated comment");
        p_ = q + 2;
      } else {
        break;
      }
    }
    return true;
  }
  static bool literal_char(char c) {  // Gson JsonReader.isLiteral
    switch (c) {
      case '/': case '\\': case ';': case '#': case '=': case '{': case '}': case '[': case ']':
      case ':': case ',': case ' ': case '\t': case '\f': case '\r': case '\n':
        return false;
      default:
        return true;
    }
  }
  static void put_utf8(std::string &o, uint32_t cp) {
    if (cp < 0x80) o.push_back((char)cp);
    else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (cp >> 18)));
      o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(uint32_t &v) {
    if (e_ - p_ < 4) return err("short \\u escape");
    v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else return err("bad \\u escape");
    }
    return true;
  }
  bool string(std::string &o, char quote) {
    ++p_;  // opening quote
    while (true) {
      if (p_ >= e_) return err("unterminated string");
      char c = *p_++;
      if (c == quote) return true;
      if (c != '\\') { o.push_back(c); continue; }
      if (p_ >= e_) return err("bad escape");
      char x = *p_++;
      switch (x) {
        case '"': o.push_back('"'); break;
        case '\'': o.push_back('\''); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case '\n': o.push_back('\n'); break;  // Gson: an escaped line break is the line break
        case 'u': {
          uint32_t v;
          if (!hex4(v)) return false;
          if (v >= 0xD800 && v < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            const char *save = p_;
            p_ += 2;
            uint32_t lo;
            if (!hex4(lo)) return false;
            if (lo >= 0xDC00 && lo < 0xE000) v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
            else p_ = save;  // unpaired: keep as is
          }
          put_utf8(o, v);
          break;
        }
        default: return err("bad escape");
      }
    }
  }
  // an unquoted literal: the longest run of literal characters
  bool unquoted(std::string &o) {
    const char *b = p_;
    while (p_ < e_ && literal_char(*p_)) ++p_;
    if (p_ == b) return err("expected value");
    o.assign(b, p_);
    return true;
  }
  static bool keyword(const std::string &s, const char *lower) {
    const size_t n = std::strlen(lower);
    if (s.size() != n) return false;
    for (size_t i = 0; i < n; ++i)
      if (s[i] != lower[i] && s[i] != lower[i] - 32) return false;
    return true;
  }
  static bool json_number(const std::string &s) {  // -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?
    size_t i = 0, n = s.size();
    if (i < n && s[i] == '-') ++i;
    if (i >= n) return false;
    if (s[i] == '0') ++i;
    else if (s[i] >= '1' && s[i] <= '9') while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
    else return false;
    if (i < n && s[i] == '.') {
      ++i;
      if (i >= n || s[i] < '0' || s[i] > '9') return false;
      while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
    }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
      ++i;
      if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
      if (i >= n || s[i] < '0' || s[i] > '9') return false;
      while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
    }
    return i == n;
  }
  bool name(std::string &k) {
    if (*p_ == '"' || *p_ == '\'') return string(k, *p_);
    return unquoted(k);
  }
  bool value(JVal &o, int depth) {
    if (depth > 512) return err("nesting too deep");
    if (!ws()) return false;
    if (p_ >= e_) return err("unexpected end");
    char c = *p_;
    if (c == '{') {
      ++p_;
      o.kind = JVal::OBJ;
      if (!ws()) return false;
      if (p_ < e_ && *p_ == '}') { ++p_; return true; }
      while (true) {
        if (!ws()) return false;
        if (p_ >= e_ || *p_ == '}') return err("expected name");
        std::string k;
        if (!name(k)) return false;
        if (!ws()) return false;
        if (p_ < e_ && *p_ == ':') ++p_;
        else if (p_ < e_ && *p_ == '=') { ++p_; if (p_ < e_ && *p_ == '>') ++p_; }
        else return err("expected ':'");
        JVal v;
        if (!value(v, depth + 1)) return false;
        o.obj.emplace_back(std::move(k), std::move(v));
        if (!ws()) return false;
        if (p_ < e_ && (*p_ == ',' || *p_ == ';')) { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; return true; }
        return err("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p_;
      o.kind = JVal::ARR;
      if (!ws()) return false;
      if (p_ < e_ && *p_ == ']') { ++p_; return true; }
      while (true) {
        if (!ws()) return false;
        if (p_ < e_ && (*p_ == ',' || *p_ == ';' || *p_ == ']')) {
          o.arr.emplace_back();  // an omitted element is null (lenient)
        } else {
          JVal v;
          if (!value(v, depth + 1)) return false;
          o.arr.push_back(std::move(v));
        }
        if (!ws()) return false;
        if (p_ < e_ && (*p_ == ',' || *p_ == ';')) { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; return true; }
        return err("expected ',' or ']'");
      }
    }
    if (c == '"' || c == '\'') {
      o.kind = JVal::STR;
      return string(o.s, c);
    }
    std::string lit;
    if (!unquoted(lit)) return false;
    if (keyword(lit, "true") || keyword(lit, "false")) {
      o.kind = JVal::BOOL;
      o.b = (lit[0] == 't' || lit[0] == 'T');
    } else if (keyword(lit, "null")) {
      o.kind = JVal::NUL;
    } else if (json_number(lit)) {
      o.kind = JVal::NUM;
      o.s = lit;
    } else {
      o.kind = JVal::STR;
      o.s = lit;
    }
    return true;
  }
};

// Gson JsonWriter string escaping (htmlSafe = false, the JsonElement.toString() writer).
void gson_string(std::string &o, const std::string &s) {
  static const char *hex = "0123456789abcdef";
  o.push_back('"');
  for (size_t i = 0; i < s.size(); ++i) {
    unsigned char c = (unsigned char)s[i];
    switch (c) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\t': o += "\\t"; continue;
      case '\b': o += "\\b"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\f': o += "\\f"; continue;
      default: break;
    }
    if (c < 0x20) {
      o += "\\u00";
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
      continue;
    }
    // U+2028 / U+2029 (E2 80 A8 / E2 80 A9 in UTF-8)
    if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
        ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      o += ((unsigned char)s[i + 2] == 0xA8) ? "\\u2028" : "\\u2029";
      i += 2;
      continue;
    }
    o.push_back((char)c);
  }
  o.push_back('"');
}

void gson_to_string(std::string &o, const JVal &v) {
  switch (v.kind) {
    case JVal::NUL: o += "null"; break;
    case JVal::BOOL: o += v.b ? "true" : "false"; break;
    case JVal::NUM: o += v.s; break;
    case JVal::STR: gson_string(o, v.s); break;
    case JVal::ARR:
      o.push_back('[');
      for (size_t i = 0; i < v.arr.size(); ++i) {
        if (i) o.push_back(',');
        gson_to_string(o, v.arr[i]);
      }
      o.push_back(']');
      break;
    case JVal::OBJ: {
      // LinkedTreeMap: a repeated key keeps its first position and its last value
      o.push_back('{');
      bool first = true;
      for (size_t i = 0; i < v.obj.size(); ++i) {
        bool seen = false;
        for (size_t j = 0; j < i; ++j)
          if (v.obj[j].first == v.obj[i].first) seen = true;
        if (seen) continue;
        if (!first) o.push_back(',');
        first = false;
        gson_string(o, v.obj[i].first);
        o.push_back(':');
        gson_to_string(o, *v.get(v.obj[i].first));
      }
      o.push_back('}');
      break;
    }
  }
}

}  // namespace

struct prh_edges {
  std::shared_ptr<void> mapping;     // mmap'd file or copied buffer backing the name views
  std::deque<std::string> arena;     // names created by the JSON front-end
  std::vector<std::deque<std::string>> chunk_arenas;  // the same, of the parallel reader's chunks
  std::vector<std::string_view> names;
  std::vector<int32_t> src, dst;
};

namespace {

struct Mapping {
  void *p = nullptr;
  size_t n = 0;
  ~Mapping() {
    if (p && n) munmap(p, n);
  }
};

// Sparky.java:84-118 for one record: (url, href) per type=="a" link, or (url, null).
int extract_links(std::string_view url, const char *jb, const char *je, prh_edges *E, Interner &in,
                  size_t lineno) {
  JVal root;
  JParser jp(jb, je);
  if (!jp.parse(root))
    return fail("line " + std::to_string(lineno) + ": JSON: " + jp.error);
  if (root.kind != JVal::OBJ)  // getAsJsonObject() on a non-object (Sparky.java:88)
    return fail("line " + std::to_string(lineno) + ": record is not a JSON object");
  const int32_t su = in.intern(url);
  bool dangling = true;  // Sparky.java:90
  const JVal *content = root.get("content");  // :89
  if (content) {
    if (content->kind != JVal::OBJ)
      return fail("line " + std::to_string(lineno) + ": 'content' is not an object (ClassCastException in the reference)");
    const JVal *links = content->get("links");  // :93
    if (links) {
      if (links->kind != JVal::ARR)
        return fail("line " + std::to_string(lineno) + ": 'links' is not an array");
      for (const JVal &el : links->arr) {  // :98
        if (el.kind != JVal::OBJ)
          return fail("line " + std::to_string(lineno) + ": link is not an object");
        const JVal *href = el.get("href"), *type = el.get("type");
        if (!href || !type)  // temp.get(...).toString() on null: NPE (:101-102)
          return fail("line " + std::to_string(lineno) + ": link without 'href' or 'type' (NullPointerException in the reference)");
        std::string ts;
        gson_to_string(ts, *type);
        if (ts != "\"a\"") continue;  // :103
        std::string hs;
        gson_to_string(hs, *href);  // :101
        std::string stripped;
        stripped.reserve(hs.size());
        for (char ch : hs)
          if (ch != '"') stripped.push_back(ch);  // aLink.replace("\"", "") (:105)
        dangling = false;
        E->arena.push_back(std::move(stripped));
        E->src.push_back(su);
        E->dst.push_back(in.intern(E->arena.back()));
      }
    }
  }
  if (dangling) {  // (url, null) (:114-118)
    E->src.push_back(su);
    E->dst.push_back(-1);
  }
  return 0;
}

// Tokens of one edge-list line [b, e) (space / tab separated): returns how many there are, the
// first two in tok.
int edge_tokens(const char *data, size_t b, size_t e, std::string_view (&tok)[2]) {
  int nt = 0;
  size_t j = b;
  while (j < e) {
    while (j < e && (data[j] == ' ' || data[j] == '\t')) ++j;
    if (j >= e) break;
    const size_t tb = j;
    while (j < e && data[j] != ' ' && data[j] != '\t') ++j;
    if (nt < 2) tok[nt] = std::string_view(data + tb, j - tb);
    ++nt;
  }
  return nt;
}

int g_read_threads = 0;  // prh_set_read_threads; 0: automatic

// Host threads for the edge-list reader: the affinity mask, capped by the cgroup CPU quota (a GPU
// box shows the whole machine but grants a share of it) and 64.
int host_threads() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
  if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0)
      n = std::min(n, (int)std::max(1LL, (std::atoll(q) + period - 1) / period));
    std::fclose(f);
  }
  return std::max(1, std::min(n, 64));
}

// One chunk of an edge list (whole lines) interned on its own: local IDs in first-appearance order
// within the chunk.
struct EdgeChunk {
  size_t b = 0, e = 0;
  size_t lines = 0;      // records seen ('\n'-terminated, and a last unterminated one)
  size_t bad_line = 0;   // 1-based line (within the chunk) of the first malformed record, 0: none
  std::string err;       // its message, without the "line N: " prefix
  std::vector<int32_t> &src, &dst;
  prh_edges le;          // the chunk's local IDs (src, dst) and JSON-made names (arena)
  std::unique_ptr<Interner> in;
  EdgeChunk() : src(le.src), dst(le.dst) {}
  // src / dst refer into this object's own le: a copy or a move would leave them pointing at the
  // source object's vectors, so a chunk never moves
  EdgeChunk(const EdgeChunk &) = delete;
  EdgeChunk &operator=(const EdgeChunk &) = delete;
  EdgeChunk(EdgeChunk &&) = delete;
  EdgeChunk &operator=(EdgeChunk &&) = delete;
};

void parse_edge_chunk(const char *data, EdgeChunk &c) {
  c.in.reset(new Interner((c.e - c.b) / 32));
  Interner &in = *c.in;
  // lines in batches: tokenize and hash a batch, prefetch every token's first slot and then the
  // name it holds, then intern in line order (the same IDs as one token at a time)
  constexpr int kB = 32;
  std::string_view tok[kB][2];
  uint64_t h[kB][2];
  int nt[kB];
  size_t i = c.b;
  while (i < c.e) {
    int nb = 0;
    while (nb < kB && i < c.e) {
      ++c.lines;
      const size_t b = i;
      const char *nl = static_cast<const char *>(std::memchr(data + i, '\n', c.e - i));
      size_t e = nl ? (size_t)(nl - data) : c.e;
      i = e + 1;
      if (e > b && data[e - 1] == '\r') --e;
      const int n = edge_tokens(data, b, e, tok[nb]);
      if (n == 0) continue;
        if (n > 2) {  // the lines before it in this batch are still interned, as sequentially
        c.bad_line = c.lines;
        c.err = "expected 'src [dst]', got " + std::to_string(n) + " tokens";
        break;
      }
      nt[nb++] = n;
    }
    for (int k = 0; k < nb; ++k)
      for (int j = 0; j < nt[k]; ++j) in.prefetch_slot(h[k][j] = Interner::hash(tok[k][j]));
    for (int k = 0; k < nb; ++k)
      for (int j = 0; j < nt[k]; ++j) in.prefetch_name(h[k][j]);
    for (int k = 0; k < nb; ++k) {
      c.src.push_back(in.intern_hashed(tok[k][0], h[k][0]));
      c.dst.push_back(nt[k] == 2 ? in.intern_hashed(tok[k][1], h[k][1]) : -1);
    }
    if (c.bad_line) return;
  }
}

// Common Crawl "url<TAB>json" records of one chunk (Sparky.java:84-118 per record, extract_links)
void parse_ccjson_chunk(const char *data, EdgeChunk &c) {
  c.in.reset(new Interner((c.e - c.b) / 256));
  size_t i = c.b;
  while (i < c.e) {
    ++c.lines;
    const size_t b = i;
    const char *nl = static_cast<const char *>(std::memchr(data + i, '\n', c.e - i));
    size_t e = nl ? (size_t)(nl - data) : c.e;
    i = e + 1;
    if (e > b && data[e - 1] == '\r') --e;
    if (e == b) continue;
    const char *tab = static_cast<const char *>(std::memchr(data + b, '\t', e - b));
    int rc = 0;
    if (!tab) rc = fail("line 0: expected 'url<TAB>json'");
    else rc = extract_links(std::string_view(data + b, (size_t)(tab - (data + b))), tab + 1, data + e, &c.le, *c.in, 0);
    if (rc != 0) {  // messages are "line <n>: ..."; the chunk's caller puts the file's line number back
      const std::string &m = g_err;  // this thread's
      const size_t k = m.find(": ");
      c.err = (m.rfind("line ", 0) == 0 && k != std::string::npos) ? m.substr(k + 2) : m;
      c.bad_line = c.lines;
      return;
    }
  }
}

// Edge list on T threads, IDs exactly those of the sequential reader (first appearance in file
// order, src before dst): every chunk interns its lines locally in parallel; then the chunks' local
// name lists are merged in chunk order into the global interner (a name new to chunk c gets its ID
// in c's local order, which is file order), and the local IDs are translated in parallel.
int parse_parallel(const char *data, size_t n, int32_t format, int T, prh_edges *E) {
  std::vector<size_t> starts{0};
  for (int t = 1; t < T; ++t) {
    const size_t p = n * (size_t)t / (size_t)T;
    if (p == 0) continue;
    const char *nl = static_cast<const char *>(std::memchr(data + p - 1, '\n', n - (p - 1)));
    const size_t st = nl ? (size_t)(nl - data) + 1 : n;
    if (st < n && st > starts.back()) starts.push_back(st);
  }
  const size_t C = starts.size();
  std::vector<EdgeChunk> ch(C);
  for (size_t c = 0; c < C; ++c) {
    ch[c].b = starts[c];
    ch[c].e = c + 1 < C ? starts[c + 1] : n;
  }
  {
    std::vector<std::thread> th;
    for (size_t c = 0; c < C; ++c)
      th.emplace_back(format == PRH_FORMAT_CCJSON ? parse_ccjson_chunk : parse_edge_chunk, data, std::ref(ch[c]));
    for (auto &t : th) t.join();
  }
  size_t line0 = 0, total = 0, local_names = 0;
  for (size_t c = 0; c < C; ++c) {
    if (ch[c].bad_line) return fail("line " + std::to_string(line0 + ch[c].bad_line) + ": " + ch[c].err);
    line0 += ch[c].lines;
    total += ch[c].src.size();
    local_names += ch[c].in->names().size();
  }
  for (size_t c = 0; c < C; ++c)  // JSON-made names: moving a deque keeps its elements in place
    if (!ch[c].le.arena.empty()) E->chunk_arenas.push_back(std::move(ch[c].le.arena));
  if (C == 1) {  // one chunk: its local IDs are the IDs
    E->src.swap(ch[0].src);
    E->dst.swap(ch[0].dst);
    E->names.swap(ch[0].in->names());
    if (E->names.size() > (size_t)INT32_MAX) return fail("more than 2^31-1 distinct URLs");
    return 0;
  }
  // Merge, sharded by hash over C threads.  Shard s walks every chunk's local names in chunk order
  // and keeps those whose hash it owns: the first time it sees a name, (c, k) is that name's first
  // appearance in the file (chunk order, then local order); otherwise it records where the name
  // first appeared.  A name new at (c, k) then gets ID base[c] + (the names new in c before k),
  // base[c] = the names new in chunks < c: exactly the sequential first-appearance numbering.
  const size_t S = C;
  std::vector<std::vector<uint8_t>> isnew(C);
  std::vector<std::vector<uint64_t>> first(C);  // (c0 << 32) | k0 of the name's first appearance
  for (size_t c = 0; c < C; ++c) {
    isnew[c].assign(ch[c].in->names().size(), 0);
    first[c].resize(ch[c].in->names().size());
  }
  {
    std::vector<std::thread> th;
    for (size_t sh = 0; sh < S; ++sh)
      th.emplace_back([&, sh]() {
        Interner g(std::max(local_names / (2 * S), (size_t)1024));
        std::vector<uint64_t> where;  // per shard-local ID: its first (c, k)
        for (size_t c = 0; c < C; ++c) {
          const auto &nm = ch[c].in->names();
          const auto &hs = ch[c].in->hashes();
          for (size_t k = 0; k < nm.size(); ++k) {
            if ((hs[k] >> 40) % S != sh) continue;
            const size_t before = g.names().size();
            const int32_t id = g.intern_hashed(nm[k], hs[k]);
            if ((size_t)id == before) {  // new: its first appearance
              where.push_back((uint64_t)c << 32 | k);
              isnew[c][k] = 1;
            }
            first[c][k] = where[(size_t)id];
          }
        }
      });
    for (auto &t : th) t.join();
  }
  std::vector<size_t> base(C + 1, 0);
  std::vector<std::vector<int32_t>> to_global(C);
  for (size_t c = 0; c < C; ++c) {
    size_t cnt = 0;
    for (uint8_t f : isnew[c]) cnt += f;
    base[c + 1] = base[c] + cnt;
  }
  if (base[C] > (size_t)INT32_MAX) return fail("more than 2^31-1 distinct URLs");
  E->names.resize(base[C]);
  {
    std::vector<std::thread> th;  // IDs of the names new in each chunk
    for (size_t c = 0; c < C; ++c)
      th.emplace_back([&, c]() {
        const auto &nm = ch[c].in->names();
        to_global[c].assign(nm.size(), -1);
        int32_t id = (int32_t)base[c];
        for (size_t k = 0; k < nm.size(); ++k)
          if (isnew[c][k]) {
            E->names[(size_t)id] = nm[k];
            to_global[c][k] = id++;
          }
      });
    for (auto &t : th) t.join();
  }
  {
    std::vector<std::thread> th;  // the others: the ID of their first appearance
    for (size_t c = 0; c < C; ++c)
      th.emplace_back([&, c]() {
        for (size_t k = 0; k < to_global[c].size(); ++k)
          if (!isnew[c][k]) to_global[c][k] = to_global[first[c][k] >> 32][first[c][k] & 0xFFFFFFFFull];
      });
    for (auto &t : th) t.join();
  }
  for (size_t c = 0; c < C; ++c) ch[c].in.reset();  // the views stay valid: they point into the input
  E->src.resize(total);
  E->dst.resize(total);
  {
    std::vector<std::thread> th;
    size_t off = 0;
    for (size_t c = 0; c < C; ++c) {
      th.emplace_back([&E, &ch, &to_global, c, off]() {
        const std::vector<int32_t> &m = to_global[c];
        const EdgeChunk &k = ch[c];
        for (size_t i = 0; i < k.src.size(); ++i) {
          E->src[off + i] = m[k.src[i]];
          E->dst[off + i] = k.dst[i] < 0 ? -1 : m[k.dst[i]];
        }
      });
      off += ch[c].src.size();
    }
    for (auto &t : th) t.join();
  }
  return 0;
}

int parse_into(const char *data, size_t n, int32_t format, prh_edges *E) {
  // large inputs (or an explicit thread count) on several threads; the same IDs either way
  const int T = g_read_threads > 0 ? g_read_threads : (n >= ((size_t)16 << 20) ? host_threads() : 1);
  return parse_parallel(data, n, format, T, E);
}

bool mkdirs(const std::string &p) {
  std::string cur;
  for (size_t i = 0; i <= p.size(); ++i) {
    if (i == p.size() || p[i] == '/') {
      if (!cur.empty() && mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
    }
    if (i < p.size()) cur.push_back(p[i]);
  }
  return true;
}

template <class Line>
int write_lines(FILE *f, const prh_edges *e, const double *ranks, Line line) {
  std::string buf;
  buf.reserve(1 << 20);
  for (size_t v = 0; v < e->names.size(); ++v) {
    line(buf, e->names[v], ranks[v]);
    if (buf.size() > (1 << 20) - 8192) {
      if (std::fwrite(buf.data(), 1, buf.size(), f) != buf.size()) return fail("write failed");
      buf.clear();
    }
  }
  if (std::fwrite(buf.data(), 1, buf.size(), f) != buf.size()) return fail("write failed");
  return 0;
}

}  // namespace

extern "C" {

const char *prh_last_error(void) { return g_err.c_str(); }

void prh_set_read_threads(int32_t n) { g_read_threads = n > 0 ? n : 0; }

int prh_read(const char *path, int32_t format, prh_edges **out) {
  if (!path || !out) return fail("NULL argument");
  if (format != PRH_FORMAT_EDGES && format != PRH_FORMAT_CCJSON) return fail("unknown format");
  *out = nullptr;
  int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(std::string("cannot open ") + path + ": " + std::strerror(errno));
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return fail("fstat failed");
  }
  auto m = std::make_shared<Mapping>();
  m->n = (size_t)st.st_size;
  if (m->n > 0) {
    m->p = mmap(nullptr, m->n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m->p == MAP_FAILED) {
      m->p = nullptr;
      close(fd);
      return fail("mmap failed");
    }
    madvise(m->p, m->n, MADV_SEQUENTIAL);
  }
  close(fd);
  std::unique_ptr<prh_edges> e(new prh_edges());
  e->mapping = m;
  if (parse_into(static_cast<const char *>(m->p ? m->p : (void *)""), m->n, format, e.get()) != 0) return -1;
  *out = e.release();
  return 0;
}

int prh_parse(const char *data, int64_t len, int32_t format, prh_edges **out) {
  if ((!data && len > 0) || !out || len < 0) return fail("bad argument");
  if (format != PRH_FORMAT_EDGES && format != PRH_FORMAT_CCJSON) return fail("unknown format");
  *out = nullptr;
  auto buf = std::make_shared<std::string>(data ? std::string(data, (size_t)len) : std::string());
  std::unique_ptr<prh_edges> e(new prh_edges());
  e->mapping = buf;
  if (parse_into(buf->data(), buf->size(), format, e.get()) != 0) return -1;
  *out = e.release();
  return 0;
}

int64_t prh_n_edges(const prh_edges *e) { return e ? (int64_t)e->src.size() : -1; }
int32_t prh_n_vertices(const prh_edges *e) { return e ? (int32_t)e->names.size() : -1; }
const int32_t *prh_src(const prh_edges *e) { return e ? e->src.data() : nullptr; }
const int32_t *prh_dst(const prh_edges *e) { return e ? e->dst.data() : nullptr; }

const char *prh_name(const prh_edges *e, int32_t id, int64_t *len) {
  if (!e || id < 0 || (size_t)id >= e->names.size()) return nullptr;
  if (len) *len = (int64_t)e->names[id].size();
  return e->names[id].data();
}

int32_t prh_java_double(double x, char *buf) { return (int32_t)pr_host::java_double_to_string(x, buf); }

int prh_write_part(const prh_edges *e, const char *dir, int32_t iter, const double *ranks) {
  if (!e || !dir || !ranks) return fail("NULL argument");
  const std::string d = std::string(dir) + "/PageRank" + std::to_string(iter);
  if (!mkdirs(d)) return fail("cannot create " + d);
  FILE *f = std::fopen((d + "/part-00000").c_str(), "w");
  if (!f) return fail("cannot write " + d + "/part-00000");
  char num[64];
  int rc = write_lines(f, e, ranks, [&](std::string &b, std::string_view u, double r) {
    b.push_back('(');
    b.append(u);
    b.push_back(',');
    b.append(num, pr_host::java_double_to_string(r, num));
    b.append(")\n");
  });
  std::fclose(f);
  if (rc) return rc;
  FILE *s = std::fopen((d + "/_SUCCESS").c_str(), "w");
  if (!s) return fail("cannot write _SUCCESS");
  std::fclose(s);
  return 0;
}

int prh_write_has_rank(const prh_edges *e, const char *path, const double *ranks) {
  if (!e || !ranks) return fail("NULL argument");
  FILE *f = path ? std::fopen(path, "w") : stdout;
  if (!f) return fail(std::string("cannot write ") + path);
  char num[64];
  int rc = write_lines(f, e, ranks, [&](std::string &b, std::string_view u, double r) {
    b.append(u);
    b.append(" has rank: ");
    b.append(num, pr_host::java_double_to_string(r, num));
    b.append(".\n");
  });
  if (path) std::fclose(f);
  else std::fflush(f);
  return rc;
}

// Resume: the "(url,rank)" lines of every part-* file of a saveAsTextFile
// directory (Sparky.java:237), mapped through the interned names.  Every URL of the edge list
// must appear exactly once and no other URL may; the rank is the text Double.toString wrote
// (shortest round-trip digits), so strtod restores the saved double exactly.
int prh_read_ranks(const prh_edges *e, const char *dir, double *ranks) {
  if (!e || !dir || !ranks) return fail("NULL argument");
  DIR *d = opendir(dir);
  if (!d) return fail(std::string("cannot open directory ") + dir + ": " + std::strerror(errno));
  std::vector<std::string> parts;
  while (struct dirent *de = readdir(d)) {
    const std::string n = de->d_name;
    if (n.rfind("part-", 0) == 0) parts.push_back(n);
  }
  closedir(d);
  if (parts.empty()) return fail(std::string("no part-* files in ") + dir);
  std::sort(parts.begin(), parts.end());
  std::unordered_map<std::string_view, int32_t> id;
  id.reserve(e->names.size() * 2);
  for (size_t v = 0; v < e->names.size(); ++v) id.emplace(e->names[v], (int32_t)v);
  std::vector<uint8_t> seen(e->names.size(), 0);
  size_t n_seen = 0;
  for (const std::string &pn : parts) {
    const std::string path = std::string(dir) + "/" + pn;
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return fail("cannot open " + path);
    std::string data;
    char buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, k);
    std::fclose(f);
    size_t i = 0, lineno = 0;
    while (i < data.size()) {
      ++lineno;
      size_t b = i;
      while (i < data.size() && data[i] != '\n') ++i;
      size_t t = i++;
      if (t > b && data[t - 1] == '\r') --t;
      if (t == b) continue;
      const std::string where = path + ":" + std::to_string(lineno);
      if (data[b] != '(' || data[t - 1] != ')') return fail(where + ": expected '(url,rank)'");
      const std::string_view body(data.data() + b + 1, t - b - 2);
      const size_t c = body.rfind(',');  // URLs may hold commas; the rank never does
      if (c == std::string_view::npos) return fail(where + ": expected '(url,rank)'");
      const std::string num(body.substr(c + 1));
      char *endp = nullptr;
      const double r = std::strtod(num.c_str(), &endp);
      if (num.empty() || *endp != '\0') return fail(where + ": bad rank '" + num + "'");
      auto it = id.find(body.substr(0, c));
      if (it == id.end()) return fail(where + ": URL not in the edge list");
      if (seen[it->second]) return fail(where + ": URL listed twice");
      seen[it->second] = 1;
      ++n_seen;
      ranks[it->second] = r;
    }
  }
  if (n_seen != e->names.size())
    return fail(std::string(dir) + ": " + std::to_string(e->names.size() - n_seen) + " URL(s) of the edge list have no saved rank");
  return 0;
}

void prh_free(prh_edges *e) { delete e; }

}  // extern "C"
