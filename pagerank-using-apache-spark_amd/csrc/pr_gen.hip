// Synthetic inputs for the benchmark configs (BASELINE.json) and device-side interning.
//
// The reference reads Common Crawl metadata (Sparky.java:42-123); the drop-in reads an edge
// list and interns URL tokens on the host.  For the 1-billion-edge configs the bench keeps the
// whole front-end on the GPU: a counter-based R-MAT / Erdos-Renyi generator writes raw labels,
// and pr_intern_device relabels them in first-appearance order -- the exact mapping the host
// interner would produce for the same edge list written as text.
#include <cmath>

#include "pr_compact.h"
#include "pr_device.h"
#include "pr_internal.h"

namespace pr {
namespace {

inline uint64_t splitmix64_host(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t edge_hash(uint64_t seed, uint64_t i, uint64_t k) {
  return splitmix64(seed * 0xD1B54A32D192ED03ull ^ splitmix64(i * 0x9E3779B97F4A7C15ull + k));
}

// Seeded bijection on [0, 2^scale): odd multiplies and xorshifts modulo 2^scale.
__device__ __forceinline__ uint32_t scramble(uint32_t v, int scale, uint64_t seed) {
  const uint64_t mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1);
  const uint64_t m1 = (splitmix64(seed + 11) | 1ull), m2 = (splitmix64(seed + 13) | 1ull);
  const uint64_t a1 = splitmix64(seed + 17), a2 = splitmix64(seed + 19);
  uint64_t x = v;
  x = (x * m1 + a1) & mask;
  x ^= x >> ((scale + 1) / 2);
  x = (x * m2 + a2) & mask;
  x ^= x >> ((scale + 2) / 3);
  x = (x * m1) & mask;
  return (uint32_t)x;
}

__global__ void k_gen_rmat(int scale, int64_t E, uint32_t ta, uint32_t tab, uint32_t tabc,
                           uint64_t seed, int32_t *__restrict__ src, int32_t *__restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t s = 0, d = 0;
    for (int l = 0; l < scale; l += 2) {
      const uint64_t h = edge_hash(seed, (uint64_t)i, (uint64_t)(l >> 1));
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (l + q >= scale) break;
        const uint32_t u = (uint32_t)(h >> (32 * q));
        const uint32_t sb = u >= tab ? 1u : 0u;
        const uint32_t db = (u >= ta && u < tab) || u >= tabc ? 1u : 0u;
        s |= sb << (l + q);
        d |= db << (l + q);
      }
    }
    src[i] = (int32_t)scramble(s, scale, seed);
    dst[i] = (int32_t)scramble(d, scale, seed);
  }
}

__global__ void k_gen_er(int scale, int64_t E, uint64_t seed, int32_t *__restrict__ src,
                         int32_t *__restrict__ dst) {
  const uint32_t mask = (uint32_t)((1ull << scale) - 1);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = edge_hash(seed, (uint64_t)i, 0);
    src[i] = (int32_t)((uint32_t)h & mask);
    dst[i] = (int32_t)((uint32_t)(h >> 32) & mask);
  }
}

// Chung-Lu: endpoint ranks drawn from a truncated continuous power law w(r) ~ (r + v0)^-beta by
// inverse transform, then labels = (rank * mul + add) mod n_labels (a bijection: gcd(mul, n) = 1).
// Sources use ranks [0, n_src), so ranks >= n_src never send a link (sink-only vertices); records
// E .. E + n_nolink - 1 are "(url, null)" lines for ranks n_src .. n_src + n_nolink - 1 (keys
// without links, Sparky.java:114-118).
struct PowerLaw {
  double a, lo, span, v0;  // a = 1 - beta; lo = v0^a; span = (n + v0)^a - v0^a
  int64_t n;
};

__device__ __forceinline__ int64_t power_rank(const PowerLaw &pl, uint64_t h) {
  const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  const double x = pow(pl.lo + u * pl.span, 1.0 / pl.a) - pl.v0;
  int64_t r = (int64_t)x;
  r = r < 0 ? 0 : r;
  return r >= pl.n ? pl.n - 1 : r;
}

__global__ void k_gen_chunglu(int64_t E, int64_t n_nolink, int64_t n_labels, PowerLaw out, PowerLaw in,
                              uint64_t mul, uint64_t add, uint64_t seed, int32_t *__restrict__ src,
                              int32_t *__restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E + n_nolink;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t rs, rd = -1;
    if (i < E) {
      rs = power_rank(out, edge_hash(seed, (uint64_t)i, 0));
      rd = power_rank(in, edge_hash(seed, (uint64_t)i, 1));
    } else {
      rs = out.n + (i - E);
    }
    src[i] = (int32_t)(((uint64_t)rs * mul + add) % (uint64_t)n_labels);
    dst[i] = rd < 0 ? -1 : (int32_t)(((uint64_t)rd * mul + add) % (uint64_t)n_labels);
  }
}

__global__ void k_first_pos(int64_t E, int32_t bound, const int32_t *__restrict__ src,
                            const int32_t *__restrict__ dst, uint32_t *__restrict__ first,
                            unsigned *__restrict__ err) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = src[i], d = dst[i];
    if (s < 0 || s >= bound || d < -1 || d >= bound) {
      atomicOr(err, 1u);
      continue;
    }
    const uint32_t ps = (uint32_t)(2 * i), pd = (uint32_t)(2 * i + 1);
    if (first[s] > ps) atomicMin(&first[s], ps);
    if (d >= 0 && first[d] > pd) atomicMin(&first[d], pd);
  }
}

struct AppearPred {
  const uint32_t *first;
  __device__ bool operator()(int64_t l) const { return first[l] != 0xFFFFFFFFu; }
};
struct FirstKey {
  const uint32_t *first;
  __device__ uint64_t operator()(int64_t l) const {
    return ((uint64_t)first[l] << 32) | (uint64_t)l;
  }
};

__global__ void k_new_ids(int64_t n, const uint64_t *__restrict__ keys, int32_t *__restrict__ newid) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x)
    newid[(uint32_t)keys[k]] = (int32_t)k;
}

__global__ void k_apply_ids(int64_t E, const int32_t *__restrict__ newid, int32_t *__restrict__ src,
                            int32_t *__restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
       i += (int64_t)gridDim.x * blockDim.x) {
    src[i] = newid[src[i]];
    const int32_t d = dst[i];
    if (d >= 0) dst[i] = newid[d];
  }
}

struct DevScope {
  int prev = -1;
  explicit DevScope(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(d);
  }
  ~DevScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int gen_check(int32_t device, int32_t scale, int64_t E, int32_t *s, int32_t *d) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return fail(PR_ERR_NODEVICE, "no HIP device available");
  }
  if (device < 0 || device >= n) return fail(PR_ERR_INVALID, "device index out of range");
  if (scale < 1 || scale > 31) return fail(PR_ERR_INVALID, "scale must be in [1, 31]");
  if (E < 0 || (E > 0 && (!s || !d))) return fail(PR_ERR_INVALID, "bad edge arrays");
  return PR_OK;
}

}  // namespace
}  // namespace pr

using namespace pr;

extern "C" {

int pr_gen_rmat(int32_t device, int32_t scale, int64_t n_edges, double a, double b, double c,
                uint64_t seed, int32_t *d_src, int32_t *d_dst) {
  PR_TRY(gen_check(device, scale, n_edges, d_src, d_dst));
  if (!(a >= 0 && b >= 0 && c >= 0 && a + b + c <= 1.0)) return fail(PR_ERR_INVALID, "bad R-MAT probabilities");
  DevScope ds(device);
  auto thr = [](double p) -> uint32_t {
    const double x = p * 4294967296.0;
    return x >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)x;
  };
  const uint32_t ta = thr(a), tab = thr(a + b), tabc = thr(a + b + c);
  if (n_edges > 0)
    hipLaunchKernelGGL(k_gen_rmat, dim3(grid_for(n_edges, 256, 65536)), dim3(256), 0, 0, scale,
                       n_edges, ta, tab, tabc, seed, d_src, d_dst);
  PR_HIP(hipGetLastError());
  PR_HIP(hipDeviceSynchronize());
  return PR_OK;
}

int pr_gen_er(int32_t device, int32_t scale, int64_t n_edges, uint64_t seed, int32_t *d_src,
              int32_t *d_dst) {
  PR_TRY(gen_check(device, scale, n_edges, d_src, d_dst));
  DevScope ds(device);
  if (n_edges > 0)
    hipLaunchKernelGGL(k_gen_er, dim3(grid_for(n_edges, 256, 65536)), dim3(256), 0, 0, scale,
                       n_edges, seed, d_src, d_dst);
  PR_HIP(hipGetLastError());
  PR_HIP(hipDeviceSynchronize());
  return PR_OK;
}

int pr_gen_chunglu(int32_t device, int32_t n_labels, int64_t n_edges, double gamma_out, double v0_out,
                   double gamma_in, double v0_in, double src_frac, int64_t n_nolink, uint64_t seed,
                   int32_t *d_src, int32_t *d_dst) {
  PR_TRY(gen_check(device, 1, n_edges + n_nolink, d_src, d_dst));
  if (n_labels < 1) return fail(PR_ERR_INVALID, "n_labels must be >= 1");
  if (!(gamma_out > 1.0 && gamma_in > 1.0 && gamma_out != 2.0 && gamma_in != 2.0))
    return fail(PR_ERR_INVALID, "power-law exponents must be > 1 and != 2");
  if (!(v0_out > 0.0 && v0_in > 0.0)) return fail(PR_ERR_INVALID, "v0 must be > 0");
  const int64_t n_src = (int64_t)(src_frac * (double)n_labels);
  if (n_src < 1 || n_nolink < 0 || n_src + n_nolink > n_labels)
    return fail(PR_ERR_INVALID, "src_frac * n_labels + n_nolink must fit in [1, n_labels]");
  auto law = [](double gamma, double v0, int64_t n) {
    PowerLaw p{};
    p.a = 1.0 - 1.0 / (gamma - 1.0);
    p.v0 = v0;
    p.lo = std::pow(v0, p.a);
    p.span = std::pow((double)n + v0, p.a) - p.lo;
    p.n = n;
    return p;
  };
  const PowerLaw out = law(gamma_out, v0_out, n_src), in = law(gamma_in, v0_in, n_labels);
  auto gcd = [](uint64_t x, uint64_t y) {
    while (y) { const uint64_t t = x % y; x = y; y = t; }
    return x;
  };
  uint64_t mul = (splitmix64_host(seed + 23) % (uint64_t)n_labels) | 1u, add = splitmix64_host(seed + 29) % (uint64_t)n_labels;
  while (gcd(mul, (uint64_t)n_labels) != 1) mul += 2;
  DevScope ds(device);
  if (n_edges + n_nolink > 0)
    hipLaunchKernelGGL(k_gen_chunglu, dim3(grid_for(n_edges + n_nolink, 256, 65536)), dim3(256), 0, 0, n_edges,
                       n_nolink, (int64_t)n_labels, out, in, mul, add, seed, d_src, d_dst);
  PR_HIP(hipGetLastError());
  PR_HIP(hipDeviceSynchronize());
  return PR_OK;
}

int pr_intern_device(int32_t device, int64_t n_edges, int32_t label_bound, int32_t *d_src,
                     int32_t *d_dst, int32_t *n_vertices_out) {
  if (!n_vertices_out) return fail(PR_ERR_INVALID, "n_vertices_out is NULL");
  if (label_bound < 1) return fail(PR_ERR_INVALID, "label_bound must be >= 1");
  if (n_edges >= (int64_t(1) << 31)) return fail(PR_ERR_INVALID, "n_edges must be < 2^31");
  PR_TRY(gen_check(device, 1, n_edges, d_src, d_dst));
  DevScope dsc(device);
  hipStream_t s = 0;
  DevBuf first, err, keys, tmp, newid;
  PR_TRY(first.alloc(sizeof(uint32_t) * (size_t)label_bound));
  PR_TRY(err.alloc(sizeof(unsigned)));
  PR_HIP(hipMemsetAsync(first.p, 0xFF, sizeof(uint32_t) * (size_t)label_bound, s));
  PR_HIP(hipMemsetAsync(err.p, 0, sizeof(unsigned), s));
  if (n_edges > 0)
    hipLaunchKernelGGL(k_first_pos, dim3(grid_for(n_edges, 256, 65536)), dim3(256), 0, s, n_edges,
                       label_bound, d_src, d_dst, first.as<uint32_t>(), err.as<unsigned>());
  PR_HIP(hipGetLastError());
  unsigned herr = 0;
  PR_HIP(hipMemcpyAsync(&herr, err.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  if (herr) return fail(PR_ERR_INVALID, "label outside [0, label_bound)");
  PR_TRY(keys.alloc(sizeof(uint64_t) * (size_t)label_bound));
  int64_t nv = 0;
  PR_TRY(compact_index((int64_t)label_bound, AppearPred{first.as<uint32_t>()},
                       FirstKey{first.as<uint32_t>()}, keys.as<uint64_t>(), &nv, s));
  first.reset();
  PR_TRY(tmp.alloc(sizeof(uint64_t) * (size_t)(nv > 0 ? nv : 1)));
  const int pos_bits = bits_for((uint64_t)(2 * n_edges + 1));
  PR_TRY(radix_sort_u64(keys.as<uint64_t>(), tmp.as<uint64_t>(), nv, 32, 32 + pos_bits, s));
  tmp.reset();
  PR_TRY(newid.alloc(sizeof(int32_t) * (size_t)label_bound));
  if (nv > 0)
    hipLaunchKernelGGL(k_new_ids, dim3(grid_for(nv, 256, 65536)), dim3(256), 0, s, nv,
                       keys.as<uint64_t>(), newid.as<int32_t>());
  if (n_edges > 0)
    hipLaunchKernelGGL(k_apply_ids, dim3(grid_for(n_edges, 256, 65536)), dim3(256), 0, s, n_edges,
                       newid.as<int32_t>(), d_src, d_dst);
  PR_HIP(hipGetLastError());
  PR_HIP(hipStreamSynchronize(s));
  *n_vertices_out = (int32_t)nv;
  return PR_OK;
}

}  // extern "C"
