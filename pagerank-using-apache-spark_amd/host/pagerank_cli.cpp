// pagerank -- process-level drop-in for the Sparky.java Spark job (C++ host).
//
//   pagerank <input-path> [iterations=10] [--format=edges|ccjson] [--out DIR]
//            [--save-every-iter] [--dangling=local|none] [--device N] [--quiet] [--stats]
//            [--resume DIR/PageRank<i>] [--devices D0,D1,...]
//
// Input (libpagerank_host): "src dst" edge list ("src" alone = record without links), or
// --format=ccjson "url<TAB>json" Common Crawl metadata records (Sparky.java:61-123).  URLs are
// interned to dense int32 IDs in first-appearance order, then libpagerank_hip builds the graph
// (Sparky.java:124-184) and runs the iteration (Sparky.java:164-238) on the GPU.
// Output: "Starting iter<i>" before each iteration (Sparky.java:188), then one
// "<url> has rank: <r>." line per URL (north_star); --out DIR writes DIR/PageRank<i>/part-00000
// "(url,rank)" + _SUCCESS (Sparky.java:237) for the last (or every) iteration.
// --resume DIR/PageRank<i>: start from the ranks a previous run (or Sparky.java:237) saved there
// instead of 1.0 (Sparky.java:165-170) and continue the same loop: iterations i+1 .. N-1, with
// the same "Starting iter" lines and PageRank<iter> numbering.  A directory not named
// PageRank<i> starts the loop at 0.
// --devices D0,D1,...: one row part per listed GPU (a device may repeat), driven from this one
// process by the pr_group_* API; the parts exchange contributions by device copies (xGMI peer
// copies between GPUs).  Same outputs as one GPU.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "pagerank_hip.h"
#include "pagerank_host.h"

namespace {

struct Options {
  std::string path, out, resume;
  int iterations = 10;  // Sparky.java:187
  int format = PRH_FORMAT_EDGES;
  bool save_every = false, quiet = false, stats = false;
  uint32_t flags = PR_DANGLING_LOCAL;
  int device = 0;
  std::vector<int> devices;  // --devices: one part per entry (empty: one part on `device`)
};

std::vector<int> parse_devices(const std::string &s) {
  std::vector<int> d;
  size_t i = 0;
  while (i <= s.size()) {
    const size_t j = s.find(',', i);
    const std::string t = s.substr(i, j == std::string::npos ? std::string::npos : j - i);
    if (t.empty() || t.find_first_not_of("0123456789") != std::string::npos) return {};
    d.push_back(std::atoi(t.c_str()));
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return d;
}

[[noreturn]] void usage(const char *msg) {
  if (msg) std::fprintf(stderr, "pagerank: %s\n", msg);
  std::fprintf(stderr,
               "usage: pagerank <input-path> [iterations=10] [--format=edges|ccjson] [--out DIR]\n"
               "                [--save-every-iter] [--dangling=local|none] [--device N] [--quiet] [--stats]\n"
               "                [--resume DIR/PageRank<i>] [--devices D0,D1,...]\n");
  std::exit(2);
}

Options parse(int argc, char **argv) {
  Options o;
  int pos = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--out" && i + 1 < argc) o.out = argv[++i];
    else if (a.rfind("--out=", 0) == 0) o.out = a.substr(6);
    else if (a == "--format=edges") o.format = PRH_FORMAT_EDGES;
    else if (a == "--format=ccjson") o.format = PRH_FORMAT_CCJSON;
    else if (a == "--save-every-iter") o.save_every = true;
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--stats") o.stats = true;
    else if (a == "--dangling=local") o.flags = PR_DANGLING_LOCAL;
    else if (a == "--dangling=none") o.flags = PR_DANGLING_NONE;
    else if (a == "--device" && i + 1 < argc) o.device = std::atoi(argv[++i]);
    else if (a == "--resume" && i + 1 < argc) o.resume = argv[++i];
    else if (a.rfind("--resume=", 0) == 0) o.resume = a.substr(9);
    else if ((a == "--devices" && i + 1 < argc) || a.rfind("--devices=", 0) == 0) {
      o.devices = parse_devices(a == "--devices" ? std::string(argv[++i]) : a.substr(10));
      if (o.devices.empty()) usage("--devices takes a comma-separated list of device numbers");
    }
    else if (a == "-h" || a == "--help") usage(nullptr);
    else if (!a.empty() && a[0] == '-') usage(("unknown option " + a).c_str());
    else if (pos == 0) { o.path = a; ++pos; }
    else if (pos == 1) { o.iterations = std::atoi(a.c_str()); ++pos; }
    else usage("too many positional arguments");
  }
  if (o.path.empty()) usage("missing input path");
  if (o.iterations < 0) usage("iterations must be >= 0");
  return o;
}

struct Job {
  const Options *opt;
  const prh_edges *edges;
  int start = 0;  // global index of the run's first iteration (--resume)
  int error = 0;
};

// i of a ".../PageRank<i>" directory (trailing '/' allowed), or -1
int saved_iteration(std::string d) {
  while (d.size() > 1 && d.back() == '/') d.pop_back();
  const size_t slash = d.rfind('/');
  const std::string base = slash == std::string::npos ? d : d.substr(slash + 1);
  if (base.rfind("PageRank", 0) != 0 || base.size() == 8) return -1;
  for (size_t k = 8; k < base.size(); ++k)
    if (base[k] < '0' || base[k] > '9') return -1;
  return std::atoi(base.c_str() + 8);
}

void on_iter(int32_t it_run, const double *ranks, double dc, double l1, double ms, void *user) {
  Job *job = static_cast<Job *>(user);
  const Options &o = *job->opt;
  const int32_t it = job->start + it_run;
  if (!o.out.empty() && ranks && (o.save_every || it == o.iterations - 1)) {
    if (prh_write_part(job->edges, o.out.c_str(), it, ranks) != 0) {
      std::fprintf(stderr, "pagerank: %s\n", prh_last_error());
      job->error = 1;
    }
  }
  if (o.stats)
    std::fprintf(stderr, "iter %d: dangling_sum=%.17g l1_delta=%.17g ms=%.3f\n", it, dc, l1, ms);
  if (it + 1 < o.iterations) std::printf("Starting iter%d\n", it + 1);
}

// --devices: build one part per device, then run the iterations as a single-process group with
// the same callback protocol as pr_run (ranks merged from every part, dc / L1 from part 0's
// stats, which sum every part's slots).
int run_group(const Options &o, const prh_edges *edges, const double *init, int n_run, Job *job,
              std::vector<double> *ranks) {
  const int P = (int)o.devices.size();
  const int32_t V = prh_n_vertices(edges);
  std::vector<pr_graph *> parts(P, nullptr);
  int rc = PR_OK;
  for (int p = 0; p < P && rc == PR_OK; ++p)
    rc = pr_graph_create_part(o.devices[p], p, P, V, prh_n_edges(edges), prh_src(edges), prh_dst(edges),
                              o.flags | PR_NO_CANONICAL, &parts[p]);
  const bool want = !o.out.empty();
  if (rc == PR_OK) rc = pr_group_reset(parts.data(), P, 0.15, 0.85, init);
  for (int it = 0; it < n_run && rc == PR_OK; ++it) {
    const auto t0 = std::chrono::steady_clock::now();
    rc = pr_group_step(parts.data(), P, 1);
    if (rc == PR_OK) rc = pr_group_sync(parts.data(), P);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    double st[PR_STAT_COUNT] = {0};
    if (rc == PR_OK) rc = pr_get_stats(parts[0], st, PR_STAT_COUNT);
    // ranks to the host only for a part file that is written (every iteration, or the last)
    const bool fetch = want && (o.save_every || job->start + it == o.iterations - 1);
    for (int p = 0; p < P && rc == PR_OK && fetch; ++p) rc = pr_get_ranks(parts[p], ranks->data());
    if (rc == PR_OK) on_iter(it, fetch ? ranks->data() : nullptr, st[PR_STAT_LAST_DC], st[PR_STAT_LAST_L1], ms, job);
  }
  for (int p = 0; p < P && rc == PR_OK; ++p) rc = pr_get_ranks(parts[p], ranks->data());
  const std::string err = rc == PR_OK ? std::string() : std::string(pr_last_error());
  for (pr_graph *g : parts)
    if (g) pr_graph_destroy(g);
  if (rc != PR_OK) std::fprintf(stderr, "pagerank: multi-GPU run failed (%d): %s\n", rc, err.c_str());
  return rc;
}

}  // namespace

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

int main(int argc, char **argv) {
  const Options o = parse(argc, argv);
  const auto t_job = Clock::now();
  prh_edges *edges = nullptr;
  if (prh_read(o.path.c_str(), o.format, &edges) != 0) {
    std::fprintf(stderr, "pagerank: %s\n", prh_last_error());
    return 1;
  }
  const int32_t V = prh_n_vertices(edges);
  const double ms_read = ms_since(t_job);  // parse + first-appearance interning (host)
  double ms_build = 0.0, ms_run = 0.0;
  Job job{&o, edges};
  std::vector<double> ranks((size_t)V + 1), init;
  if (!o.resume.empty()) {
    init.assign((size_t)V + 1, 0.0);
    if (prh_read_ranks(edges, o.resume.c_str(), init.data()) != 0) {
      std::fprintf(stderr, "pagerank: --resume: %s\n", prh_last_error());
      prh_free(edges);
      return 1;
    }
    job.start = saved_iteration(o.resume) + 1;  // 0 when the directory is not PageRank<i>
  }
  const int n_run = o.iterations > job.start ? o.iterations - job.start : 0;
  const double *init_p = init.empty() ? nullptr : init.data();
  if (o.devices.size() > 1) {
    if (n_run > 0) std::printf("Starting iter%d\n", job.start);
    const auto t0 = Clock::now();
    if (run_group(o, edges, init_p, n_run, &job, &ranks) != PR_OK) {
      prh_free(edges);
      return 1;
    }
    ms_run = ms_since(t0);  // group: build + iterations
  } else {
    const int dev = o.devices.empty() ? o.device : o.devices[0];
    pr_graph *g = nullptr;
    auto t0 = Clock::now();
    int rc = pr_graph_create(dev, V, prh_n_edges(edges), prh_src(edges), prh_dst(edges), o.flags | PR_NO_CANONICAL, &g);
    ms_build = ms_since(t0);
    if (rc != PR_OK) {
      std::fprintf(stderr, "pagerank: graph build failed (%d): %s\n", rc, pr_last_error());
      prh_free(edges);
      return 1;
    }
    if (n_run > 0) std::printf("Starting iter%d\n", job.start);
    t0 = Clock::now();
    // ranks cross PCIe only for the part files that are written: every iteration's with
    // --save-every-iter, else only the last one's, which pr_run returns in `ranks` anyway
    const bool every = !o.out.empty() && o.save_every;
    rc = pr_run(g, n_run, 0.15, 0.85, init_p, ranks.data(), on_iter, every ? PR_CB_RANKS : 0u, &job);
    if (rc == PR_OK && !o.out.empty() && !every && n_run > 0 &&
        prh_write_part(edges, o.out.c_str(), o.iterations - 1, ranks.data()) != 0) {
      std::fprintf(stderr, "pagerank: %s\n", prh_last_error());
      job.error = 1;
    }
    ms_run = ms_since(t0);  // iterations, with the per-iteration callback and the part-file writes
    pr_graph_destroy(g);
    if (rc != PR_OK) {
      std::fprintf(stderr, "pagerank: run failed (%d): %s\n", rc, pr_last_error());
      prh_free(edges);
      return 1;
    }
  }
  std::fflush(stdout);
  const auto t_out = Clock::now();
  if (!o.quiet && prh_write_has_rank(edges, nullptr, ranks.data()) != 0) {
    std::fprintf(stderr, "pagerank: %s\n", prh_last_error());
    job.error = 1;
  }
  std::fflush(stdout);
  const double ms_out = ms_since(t_out);
  if (o.stats)  // the job's phases (wall clock); one JSON object on stderr
    std::fprintf(stderr,
                 "{\"job\": {\"urls\": %d, \"edge_records\": %lld, \"read_intern_ms\": %.1f, \"build_ms\": %.1f, "
                 "\"iterations\": %d, \"run_ms\": %.1f, \"has_rank_out_ms\": %.1f, \"total_ms\": %.1f}}\n",
                 V, (long long)prh_n_edges(edges), ms_read, ms_build, n_run, ms_run, ms_out, ms_since(t_job));
  prh_free(edges);
  return job.error;
}
