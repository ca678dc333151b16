// pagerank -- process-level drop-in for the Sparky.java Spark job (C++ host over libpagerank_hip).
//
//   pagerank <edge-list-path> [iterations=10] [--out DIR] [--save-every-iter]
//            [--dangling=local|none] [--device N] [--quiet] [--stats]
//
// Input: text edge list, "src dst" per line; a single-token line "src" is a record without
// type=="a" links (Sparky.java:114-118).  Tokens are interned verbatim to dense int32 IDs in
// first-appearance order (src before dst) -- the canonical ID mapping of the C ABI.
// Output (stdout): "Starting iter<i>" before each iteration (Sparky.java:188), then one
// "<url> has rank: <r>." line per URL (north_star contract).  With --out DIR, the
// reference-faithful files DIR/PageRank<i>/part-00000 with "(url,rank)" lines and _SUCCESS
// (Sparky.java:237 saveAsTextFile; Tuple2.toString + Java Double.toString), for the last
// iteration or every iteration with --save-every-iter.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "javafmt.h"
#include "pagerank_hip.h"

namespace {

// ---- first-appearance interner: open addressing over string_views into the mapped file ----
class Interner {
 public:
  explicit Interner(size_t expect) { rehash(expect < 1024 ? 2048 : next_pow2(expect * 2)); }
  int32_t intern(std::string_view s) {
    const uint64_t h = hash(s);
    size_t i = h & mask_;
    while (true) {
      Slot &sl = slots_[i];
      if (sl.id < 0) {
        sl.id = (int32_t)names_.size();
        sl.hash = h;
        names_.push_back(s);
        if (names_.size() * 2 > slots_.size()) rehash(slots_.size() * 2);
        return (int32_t)names_.size() - 1;
      }
      if (sl.hash == h && names_[sl.id] == s) return sl.id;
      i = (i + 1) & mask_;
    }
  }
  const std::vector<std::string_view> &names() const { return names_; }

 private:
  struct Slot {
    uint64_t hash;
    int32_t id;
  };
  static size_t next_pow2(size_t x) {
    size_t p = 1;
    while (p < x) p <<= 1;
    return p;
  }
  static uint64_t hash(std::string_view s) {  // FNV-1a 64 + avalanche
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    return h ^ (h >> 33);
  }
  void rehash(size_t n) {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.assign(n, Slot{0, -1});
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
  size_t mask_ = 0;
};

struct Options {
  std::string path, out;
  int iterations = 10;  // Sparky.java:187
  bool save_every = false, quiet = false, stats = false;
  uint32_t flags = PR_DANGLING_LOCAL;
  int device = 0;
};

[[noreturn]] void usage(const char *msg) {
  if (msg) std::fprintf(stderr, "pagerank: %s\n", msg);
  std::fprintf(stderr,
               "usage: pagerank <edge-list-path> [iterations=10] [--out DIR] [--save-every-iter]\n"
               "                [--dangling=local|none] [--device N] [--quiet] [--stats]\n");
  std::exit(2);
}

Options parse(int argc, char **argv) {
  Options o;
  int pos = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--out" && i + 1 < argc) o.out = argv[++i];
    else if (a.rfind("--out=", 0) == 0) o.out = a.substr(6);
    else if (a == "--save-every-iter") o.save_every = true;
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--stats") o.stats = true;
    else if (a == "--dangling=local") o.flags = PR_DANGLING_LOCAL;
    else if (a == "--dangling=none") o.flags = PR_DANGLING_NONE;
    else if (a == "--device" && i + 1 < argc) o.device = std::atoi(argv[++i]);
    else if (a == "-h" || a == "--help") usage(nullptr);
    else if (!a.empty() && a[0] == '-') usage(("unknown option " + a).c_str());
    else if (pos == 0) { o.path = a; ++pos; }
    else if (pos == 1) { o.iterations = std::atoi(a.c_str()); ++pos; }
    else usage("too many positional arguments");
  }
  if (o.path.empty()) usage("missing edge-list path");
  if (o.iterations < 0) usage("iterations must be >= 0");
  return o;
}

struct Job {
  const Options *opt;
  const std::vector<std::string_view> *names;
  std::string line;
};

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

void write_part(const Options &o, const std::vector<std::string_view> &names, int iter, const double *r) {
  const std::string dir = o.out + "/PageRank" + std::to_string(iter);
  if (!mkdirs(dir)) {
    std::fprintf(stderr, "pagerank: cannot create %s\n", dir.c_str());
    std::exit(1);
  }
  FILE *f = std::fopen((dir + "/part-00000").c_str(), "w");
  if (!f) {
    std::fprintf(stderr, "pagerank: cannot write %s/part-00000\n", dir.c_str());
    std::exit(1);
  }
  std::string buf;
  buf.reserve(1 << 20);
  char num[64];
  for (size_t v = 0; v < names.size(); ++v) {
    buf.push_back('(');
    buf.append(names[v]);
    buf.push_back(',');
    buf.append(num, pr_host::java_double_to_string(r[v], num));
    buf.append(")\n");
    if (buf.size() > (1 << 20) - 4096) {
      std::fwrite(buf.data(), 1, buf.size(), f);
      buf.clear();
    }
  }
  std::fwrite(buf.data(), 1, buf.size(), f);
  std::fclose(f);
  FILE *s = std::fopen((dir + "/_SUCCESS").c_str(), "w");
  if (s) std::fclose(s);
}

void on_iter(int32_t it, const double *ranks, double dc, double l1, double ms, void *user) {
  Job *job = static_cast<Job *>(user);
  const Options &o = *job->opt;
  if (!o.out.empty() && ranks && (o.save_every || it == o.iterations - 1))
    write_part(o, *job->names, it, ranks);
  if (o.stats)
    std::fprintf(stderr, "iter %d: dangling_sum=%.17g l1_delta=%.17g ms=%.3f\n", it, dc, l1, ms);
  if (it + 1 < o.iterations) std::printf("Starting iter%d\n", it + 1);
}

}  // namespace

int main(int argc, char **argv) {
  const Options o = parse(argc, argv);
  int fd = open(o.path.c_str(), O_RDONLY);
  if (fd < 0) {
    std::fprintf(stderr, "pagerank: cannot open %s: %s\n", o.path.c_str(), std::strerror(errno));
    return 1;
  }
  struct stat st;
  fstat(fd, &st);
  const size_t n = (size_t)st.st_size;
  const char *data = "";
  if (n > 0) {
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      std::fprintf(stderr, "pagerank: mmap failed\n");
      return 1;
    }
    data = static_cast<const char *>(m);
  }
  Interner in(n / 32);
  std::vector<int32_t> src, dst;
  src.reserve(n / 24);
  dst.reserve(n / 24);
  size_t i = 0, lineno = 0;
  while (i < n) {
    ++lineno;
    std::string_view tok[3];
    int nt = 0;
    while (i < n && data[i] != '\n') {
      while (i < n && (data[i] == ' ' || data[i] == '\t' || data[i] == '\r')) ++i;
      if (i >= n || data[i] == '\n') break;
      const size_t b = i;
      while (i < n && data[i] != ' ' && data[i] != '\t' && data[i] != '\r' && data[i] != '\n') ++i;
      if (nt < 3) tok[nt] = std::string_view(data + b, i - b);
      ++nt;
    }
    ++i;  // newline
    if (nt == 0) continue;
    if (nt > 2) {
      std::fprintf(stderr, "pagerank: line %zu: expected 'src [dst]', got %d tokens\n", lineno, nt);
      return 1;
    }
    src.push_back(in.intern(tok[0]));
    dst.push_back(nt == 2 ? in.intern(tok[1]) : -1);
  }
  const auto &names = in.names();
  if (names.size() > (size_t)INT32_MAX) {
    std::fprintf(stderr, "pagerank: more than 2^31-1 distinct URLs\n");
    return 1;
  }
  pr_graph *g = nullptr;
  int rc = pr_graph_create(o.device, (int32_t)names.size(), (int64_t)src.size(), src.data(), dst.data(),
                           o.flags | PR_NO_CANONICAL, &g);
  if (rc != PR_OK) {
    std::fprintf(stderr, "pagerank: graph build failed (%d): %s\n", rc, pr_last_error());
    return 1;
  }
  std::vector<int32_t>().swap(src);
  std::vector<int32_t>().swap(dst);
  Job job{&o, &names, {}};
  std::vector<double> ranks(names.size() + 1);
  if (o.iterations > 0) std::printf("Starting iter0\n");
  rc = pr_run(g, o.iterations, 0.15, 0.85, nullptr, ranks.data(), on_iter,
              o.out.empty() ? 0u : PR_CB_RANKS, &job);
  if (rc != PR_OK) {
    std::fprintf(stderr, "pagerank: run failed (%d): %s\n", rc, pr_last_error());
    pr_graph_destroy(g);
    return 1;
  }
  pr_graph_destroy(g);
  if (!o.quiet) {
    std::string buf;
    buf.reserve(1 << 20);
    char num[64];
    for (size_t v = 0; v < names.size(); ++v) {
      buf.append(names[v]);
      buf.append(" has rank: ");
      buf.append(num, pr_host::java_double_to_string(ranks[v], num));
      buf.append(".\n");
      if (buf.size() > (1 << 20) - 4096) {
        std::fwrite(buf.data(), 1, buf.size(), stdout);
        buf.clear();
      }
    }
    std::fwrite(buf.data(), 1, buf.size(), stdout);
  }
  std::fflush(stdout);
  return 0;
}
