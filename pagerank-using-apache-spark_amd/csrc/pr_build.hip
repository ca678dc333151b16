// Graph construction on the GPU (K1/K2 in SURVEY.md §2.1).
//
// Replaces Sparky.java:124-184:
//   distinct().groupByKey()  (:124)      -> radix sort of (dst << b | src) keys + adjacent unique
//   keys().collect/broadcast (:127-135)  -> PR_VF_KEY flag from the src column
//   sink completion + union  (:137-161)  -> PR_VF_SINK = !KEY; every vertex is a row
//   count()                  (:162)      -> N = n_vertices (all interned IDs must appear)
//   dangUrls fixup           (:172-184)  -> D = sink-only vertices, resolved here once
// then lays the part's rows out for the iteration (pr_graph.h) and plans the SpMV work units.
#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <vector>

#include "pr_compact.h"
#include "pr_device.h"
#include "pr_graph.h"
#include "pr_plan.h"

namespace pr {
namespace {

constexpr uint64_t kSentinel = ~0ull;

// ---- validation + key packing ----------------------------------------------------------
__global__ void k_pack_edges(int64_t E, int32_t V, int b, const int32_t *__restrict__ src,
                             const int32_t *__restrict__ dst, uint64_t *__restrict__ keys,
                             uint8_t *__restrict__ appear, uint8_t *__restrict__ is_key,
                             unsigned *__restrict__ err) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = src[i], d = dst[i];
    if (s < 0 || s >= V || d < -1 || d >= V) {
      atomicOr(err, 1u);
      keys[i] = kSentinel;
      continue;
    }
    appear[s] = 1;
    is_key[s] = 1;
    if (d >= 0) {
      appear[d] = 1;
      keys[i] = ((uint64_t)(uint32_t)d << b) | (uint32_t)s;
    } else {
      keys[i] = kSentinel;  // record without links: no edge (Sparky.java:114-118)
    }
  }
}

__global__ void k_check_appear(int32_t V, const uint8_t *__restrict__ appear, unsigned *err) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < V;
       v += (int64_t)gridDim.x * blockDim.x)
    if (!appear[v]) atomicOr(err, 2u);
}

struct UniquePred {
  const uint64_t *k;
  __device__ bool operator()(int64_t i) const {
    const uint64_t x = k[i];
    return x != kSentinel && (i == 0 || x != k[i - 1]);
  }
};
struct IdentityU64 {
  const uint64_t *k;
  __device__ uint64_t operator()(int64_t i) const { return k[i]; }
};

// row_ptr[v] = first position whose row (key >> shift) is >= v; rows [0, R).
__global__ void k_row_ptr(const uint64_t *__restrict__ keys, int64_t m, int shift, int64_t R,
                          int64_t *__restrict__ row_ptr) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rc = (i < m) ? (int64_t)(keys[i] >> shift) : R;
    const int64_t rp = (i > 0) ? (int64_t)(keys[i - 1] >> shift) : -1;
    for (int64_t v = rp + 1; v <= rc; ++v) row_ptr[v] = i;
  }
}

__global__ void k_canon_col_deg(const uint64_t *__restrict__ keys, int64_t m, uint64_t mask,
                                int32_t *__restrict__ col, int32_t *__restrict__ deg) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = (int32_t)(keys[i] & mask);
    col[i] = s;
    atomicAdd(&deg[s], 1);
  }
}

// vflags + global counters {n_sink, n_nolink, n_indeg0, max_indeg, max_outdeg}
__global__ void k_vflags(int32_t V, const uint8_t *__restrict__ is_key,
                         const int32_t *__restrict__ deg, const int64_t *__restrict__ row_ptr,
                         uint8_t *__restrict__ vflags, unsigned long long *__restrict__ cnt) {
  unsigned long long ns = 0, nn = 0, ni = 0;
  unsigned long long mi = 0, mo = 0;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < V;
       v += (int64_t)gridDim.x * blockDim.x) {
    uint8_t f = 0;
    if (is_key[v]) {
      f |= PR_VF_KEY;
      if (deg[v] == 0) { f |= PR_VF_NOLINK; ++nn; }
    } else {
      f |= PR_VF_SINK;
      ++ns;
    }
    const int64_t indeg = row_ptr[v + 1] - row_ptr[v];
    if (indeg == 0) { f |= PR_VF_INDEG0; ++ni; }
    vflags[v] = f;
    mi = mi > (unsigned long long)indeg ? mi : (unsigned long long)indeg;
    mo = mo > (unsigned long long)deg[v] ? mo : (unsigned long long)deg[v];
  }
  atomicAdd(&cnt[0], ns);
  atomicAdd(&cnt[1], nn);
  atomicAdd(&cnt[2], ni);
  atomicMax(&cnt[3], mi);
  atomicMax(&cnt[4], mo);
}

// Expected number of peers' sources a part reads (class policy at P > 1): a source with d
// out-links is read by a given other part with probability 1 - (1 - 1/P)^d (its out-links land
// in random parts: parts own every P-th vertex of the degree order).  Summed in fixed point
// (2^-20) with integer atomics, so every part computes the same value.
__global__ void k_reader_est(int32_t V, int P, const int32_t *__restrict__ deg, unsigned long long *__restrict__ sum) {
  const double q = 1.0 - 1.0 / (double)P;
  unsigned long long acc = 0;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < V; v += (int64_t)gridDim.x * blockDim.x) {
    const int d = deg[v];
    if (d > 0) acc += (unsigned long long)((1.0 - pow(q, (double)d)) * 1048576.0);
  }
  atomicAdd(sum, acc);
}

// Internal order key: out-degree descending, original ID ascending (hot contributions first).
__global__ void k_order_keys(int32_t V, int b, uint64_t maxd, const int32_t *__restrict__ deg,
                             uint64_t *__restrict__ vk) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < V;
       v += (int64_t)gridDim.x * blockDim.x)
    vk[v] = ((maxd - (uint64_t)deg[v]) << b) | (uint64_t)v;
}

// rank_of[v] = sorted index; gpos[v] = gather position of v's contribution.  Sorted index i
// -> part i % P, local rank j = i / P -> class x = j % C, q = j / C -> local row L = x*Q_pad + q.
__global__ void k_rank_gpos(int32_t V, uint64_t mask, int P, int C, int64_t Q_pad, int64_t S_pad,
                            const uint64_t *__restrict__ sorted_vk, int32_t *__restrict__ rank_of,
                            int32_t *__restrict__ gpos) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t v = (int32_t)(sorted_vk[i] & mask);
    rank_of[v] = (int32_t)i;
    const int64_t j = i / P;
    gpos[v] = (int32_t)((i % P) * S_pad + (j % C) * Q_pad + j / C);
  }
}

struct PartPred {
  const uint64_t *k;
  const int32_t *rank_of;
  int b, P, part;
  __device__ bool operator()(int64_t i) const {
    const int32_t d = (int32_t)(k[i] >> b);
    return rank_of[d] % P == part;
  }
};
// local key = (segment << (brow + bg)) | (row << bg) | gather position of src, where the
// segment is the column class of the source (0 in the fused layout) and row the local row L.
struct PartXform {
  const uint64_t *k;
  const int32_t *gpos;
  int b, bg, brow;
  uint64_t mask;
  ClassGeom geo;
  __device__ uint64_t operator()(int64_t i) const {
    const uint64_t key = k[i];
    const int32_t d = (int32_t)(key >> b), s = (int32_t)(key & mask);
    const int64_t gs = gpos[s];
    const uint64_t row = (uint64_t)(gpos[d] % geo.S_pad);
    const uint64_t seg = geo.C > 1 ? (uint64_t)((gs % geo.S_pad) / geo.Q_pad) : 0ull;
    return (seg << (brow + bg)) | (row << bg) | (uint64_t)gs;
  }
};

// row_ptr over rows [0, R) of keys[lo, hi) whose row is (key >> shift) & rmask.
__global__ void k_row_ptr_seg(const uint64_t *__restrict__ keys, int64_t lo, int64_t hi, int shift,
                              uint64_t rmask, int64_t R, int64_t *__restrict__ row_ptr) {
  const int64_t m = hi - lo;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= m;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rc = (i < m) ? (int64_t)((keys[lo + i] >> shift) & rmask) : R;
    const int64_t rp = (i > 0) ? (int64_t)((keys[lo + i - 1] >> shift) & rmask) : -1;
    for (int64_t v = rp + 1; v <= rc; ++v) row_ptr[v] = i;
  }
}

__global__ void k_local_col(const uint64_t *__restrict__ keys, int64_t m, uint64_t mask,
                            int32_t *__restrict__ col) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    col[i] = (int32_t)(keys[i] & mask);
}

// Per local row L: rowinfo (out-degree | RI_* flags) and the original ID (-1 for holes).
__global__ void k_local_rows(int64_t R, int64_t n_local, int P, int part, ClassGeom geo,
                             uint64_t mask, bool dangling_none, const uint64_t *__restrict__ sorted_vk,
                             const int32_t *__restrict__ deg, const uint8_t *__restrict__ vflags,
                             uint32_t *__restrict__ rowinfo, int32_t *__restrict__ orig) {
  for (int64_t L = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; L < R;
       L += (int64_t)gridDim.x * blockDim.x) {
    const int C = geo.C;
    const int64_t x = L / geo.Q_pad, q = L % geo.Q_pad, j = q * C + x;
    if (j >= n_local) {
      rowinfo[L] = kRowHole;
      orig[L] = -1;
      continue;
    }
    const int32_t v = (int32_t)(sorted_vk[j * P + part] & mask);
    orig[L] = v;
    uint32_t info = (uint32_t)deg[v];
    if (deg[v] == 0 && (vflags[v] & PR_VF_SINK) && !dangling_none) info |= kRowSink;
    if (vflags[v] & PR_VF_INDEG0) info |= kRowIndeg0;
    rowinfo[L] = info;
  }
}


}  // namespace

// Greedy work plan over the part's row_ptr (host; linear, deterministic).
void plan_units(const std::vector<int64_t> &rp, int unit_nnz, int unit_rows, UnitPlan *plan,
                int64_t row_begin, int64_t row_end, bool append) {
  const int64_t R = row_end < 0 ? (int64_t)rp.size() - 1 : row_end;
  if (!append) {
    plan->units.clear();
    plan->src_off.clear();
    plan->lr_row.clear();
    plan->lr_p0.clear();
    plan->n_pieces = 0;
    plan->padded_len = 0;
  } else if (!plan->lr_p0.empty()) {
    plan->lr_p0.pop_back();  // re-appended at the end
  }
  int64_t pieces = plan->n_pieces, pad = plan->padded_len, v = row_begin;
  auto push = [&](int64_t src, int32_t r0, int32_t meta, int32_t n) {
    plan->units.push_back(Unit{(uint32_t)(pad / 8), r0, meta, n});
    plan->src_off.push_back(src);
    pad += ((int64_t)n + 7) / 8 * 8;
  };
  while (v < R) {
    const int64_t len = rp[v + 1] - rp[v];
    if (len > unit_nnz) {
      const int64_t np = (len + unit_nnz - 1) / unit_nnz;
      plan->lr_row.push_back((int32_t)v);
      plan->lr_p0.push_back((int32_t)pieces);
      for (int64_t q = 0; q < np; ++q) {
        const int64_t n = std::min<int64_t>(unit_nnz, len - q * unit_nnz);
        push(rp[v] + q * unit_nnz, (int32_t)v, (int32_t)(-(pieces + q) - 1), (int32_t)n);
      }
      pieces += np;
      ++v;
      continue;
    }
    const int64_t start = v;
    int64_t nnz = 0;
    while (v < R && v - start < unit_rows) {
      const int64_t l = rp[v + 1] - rp[v];
      if (l > unit_nnz || nnz + l > unit_nnz) break;
      nnz += l;
      ++v;
    }
    push(rp[start], (int32_t)start, (int32_t)(v - start), (int32_t)nnz);
  }
  plan->lr_p0.push_back((int32_t)pieces);
  plan->n_pieces = pieces;
  plan->padded_len = pad;
}

namespace {
__global__ void k_pad_cols(const Unit *__restrict__ units, const int64_t *__restrict__ src_off,
                           const int32_t *__restrict__ col, int32_t *__restrict__ colp) {
  const Unit u = units[blockIdx.x];
  const int64_t s = src_off[blockIdx.x], d = (int64_t)u.p8 * 8;
  const int n = unit_n(u);
  for (int i = threadIdx.x; i < n; i += blockDim.x) colp[d + i] = col[s + i];
}
}  // namespace

int build_padded_cols(const UnitPlan &plan, const int32_t *col, int32_t *colp, hipStream_t s) {
  const size_t nu = plan.units.size();
  PR_HIP(hipMemsetAsync(colp, 0, sizeof(int32_t) * (plan.padded_len > 0 ? plan.padded_len : 1), s));
  if (nu == 0) return PR_OK;
  DevBuf du, ds;
  PR_TRY(du.alloc(sizeof(Unit) * nu));
  PR_TRY(ds.alloc(sizeof(int64_t) * nu));
  PR_HIP(hipMemcpyAsync(du.p, plan.units.data(), sizeof(Unit) * nu, hipMemcpyHostToDevice, s));
  PR_HIP(hipMemcpyAsync(ds.p, plan.src_off.data(), sizeof(int64_t) * nu, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_pad_cols, dim3((unsigned)nu), dim3(256), 0, s, du.as<Unit>(), ds.as<int64_t>(),
                     col, colp);
  PR_HIP(hipGetLastError());
  PR_HIP(hipStreamSynchronize(s));
  return PR_OK;
}

// ---- split layout: entry codes (pr_internal.h, pr_spmv.h k_spmv_hot) -----------------------
// Entry code (pr_internal.h); a segment end is marked in bit 0 (codes are byte offsets /
// addresses, multiples of 8), from which k_spmv_hot derives its lane metadata.
// hpos[x * P*Kp + p*Kp + q] = gather position of row x*Q_pad + q of part p (0 when q >= q_load or
// the part never reads it: the slot is then never addressed); hotidx[pos] = its LDS slot.
__global__ void k_hot_tables(HotGeom hg, const int32_t *__restrict__ cmap, int32_t *__restrict__ hpos,
                             int32_t *__restrict__ hotidx) {
  const int64_t nh = (int64_t)hg.P * hg.Kp;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < (int64_t)hg.C * nh;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = t / nh, i = t - x * nh, p = i / hg.Kp, q = i - p * hg.Kp;
    int32_t pos = -1;
    if (q < hg.q_load) {
      const int64_t a = p * hg.S_pad + x * hg.Q_pad + q;
      pos = cmap ? cmap[a] : (int32_t)a;
    }
    hpos[t] = pos < 0 ? 0 : pos;
    if (pos >= 0) hotidx[pos] = (int32_t)(1 + i);
  }
}

// Entry code of a gather position: its LDS byte address when hot (pr_internal.h kEntGlobal).
__device__ __forceinline__ uint32_t hot_code(int32_t pos, const int32_t *__restrict__ hotidx, bool end) {
  const int32_t h = hotidx[pos];
  const uint32_t c = h ? (uint32_t)(8 * h) : (kEntGlobal | ((uint32_t)pos * 8u));
  return end ? (c | 1u) : c;
}

// Columns -> compacted gather positions; counts sources the exchange lists miss (a bug).
__global__ void k_map_cols(int64_t n, const int32_t *__restrict__ cmap, int32_t *__restrict__ col,
                           unsigned long long *__restrict__ bad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = cmap[col[i]];
    if (c < 0) atomicAdd(bad, 1ull);
    col[i] = c < 0 ? 0 : c;
  }
}

// One workgroup per wave unit: its entry codes (end marks in bit 0, padding 0); *n_hot counts the
// entries that read the LDS hot set.
__global__ __launch_bounds__(256) void k_fill_hot(int64_t n_units, const Unit *__restrict__ units,
                                                  const int64_t *__restrict__ src_off,
                                                  const int32_t *__restrict__ n_real,
                                                  const int32_t *__restrict__ col,
                                                  const int32_t *__restrict__ hotidx,
                                                  uint32_t *__restrict__ colh, unsigned long long *n_hot) {
  unsigned long long nh = 0;
  for (int64_t b = blockIdx.x; b < n_units; b += gridDim.x) {
    const Unit u = units[b];
    uint32_t *dst = colh + (int64_t)u.p8 * 8;
    const int64_t s0 = src_off[b];
    const int n = n_real[b];
    for (int i = threadIdx.x; i < u.n; i += 256) {
      uint32_t c = 0;
      if (i < n) {
        const int32_t v = col[s0 + i];
        c = hot_code(v & 0x7FFFFFFF, hotidx, u.meta >= 0 && v < 0);
        nh += (c & kEntGlobal) ? 0 : 1;
      }
      dst[i] = c;
    }
  }
  atomicAdd(n_hot, nh);
}

// Compact entry codes (pr_internal.h kCodeC20 / kCodeC24, P = 1): one thread per 8-entry lane
// group of a wave unit writes the group's 8 u16 low index halves and its side word (end marks,
// HB high bits per entry: u32 for 3, u64 for 4).  A source at region offset o of class x (gather
// position x*Q_pad + o) has index o + 1; padding 0.  *n_hot counts the entries that read the LDS
// hot set; *bad the sources outside the unit's region band (none by construction: the codes would
// then read another class's values).
template <int HB, class SideT>
__global__ __launch_bounds__(64) void k_fill_compact(int64_t n_units, const Unit *__restrict__ units,
                                                     const int64_t *__restrict__ src_off,
                                                     const int32_t *__restrict__ n_real,
                                                     const int32_t *__restrict__ col, int64_t Q_pad, int q_load,
                                                     uint16_t *__restrict__ code16, SideT *__restrict__ cside,
                                                     unsigned long long *n_hot, unsigned long long *bad) {
  unsigned long long nh = 0, nb = 0;
  for (int64_t b = blockIdx.x; b < n_units; b += gridDim.x) {
    const Unit u = units[b];
    const int64_t s0 = src_off[b];
    const int n = n_real[b];
    int64_t x0 = -1;  // the unit's class: the region of its first source
    if (n > 0) x0 = (int64_t)(col[s0] & 0x7FFFFFFF) / Q_pad;
    for (int grp = threadIdx.x; grp < u.n / 8; grp += 64) {
      SideT side = 0;
      uint32_t lo[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * grp + j;
        uint32_t idx = 0;
        if (i < n) {
          const int32_t v = col[s0 + i];
          const int64_t pos = v & 0x7FFFFFFF;
          const int64_t x = pos / Q_pad;
          nb += x != x0 ? 1 : 0;
          idx = (uint32_t)(pos - x * Q_pad + 1);
          nh += idx <= (uint32_t)q_load ? 1 : 0;
          if (u.meta >= 0 && v < 0) side |= (SideT)1 << j;  // segment end (STREAM units)
        }
        lo[j] = idx & 0xFFFFu;
        side |= (SideT)((idx >> 16) & ((1u << HB) - 1u)) << (8 + HB * j);
      }
      uint4 q;
      q.x = lo[0] | lo[1] << 16;
      q.y = lo[2] | lo[3] << 16;
      q.z = lo[4] | lo[5] << 16;
      q.w = lo[6] | lo[7] << 16;
      *reinterpret_cast<uint4 *>(code16 + (int64_t)u.p8 * 8 + 8 * grp) = q;
      cside[(int64_t)u.p8 + grp] = side;
    }
  }
  atomicAdd(n_hot, nh);
  atomicAdd(bad, nb);
}

// Piece codes (pr_internal.h kCodeC20P / kCodeC24P, P > 1): the gather-space range of every
// (class x, part p) piece -- the positions of part p's class-x sources in this part's gather space
// (the own region, or the sub-run of p's received run).  lo/hi[x * P + p], hi = 0 when empty.
__global__ __launch_bounds__(256) void k_piece_bounds(int64_t S_pad, int64_t Q_pad, int C, int P,
                                                      const int32_t *__restrict__ cmap, int32_t *__restrict__ lo,
                                                      int32_t *__restrict__ hi) {
  // one workgroup per (class x, part p) region of the global slices: min / max + 1 of its mapped
  // positions (a plain reduction: atomics on P*C addresses serialise, 31 ms per s26 part)
  const int x = (int)(blockIdx.x / P), p = (int)(blockIdx.x % P);
  const int64_t a0 = (int64_t)p * S_pad + (int64_t)x * Q_pad;
  int32_t mn = INT32_MAX, mx = 0;
  for (int64_t o = threadIdx.x; o < Q_pad; o += blockDim.x) {
    const int64_t a = a0 + o;
    const int32_t pos = cmap ? cmap[a] : (int32_t)a;
    if (pos >= 0) {
      mn = min(mn, pos);
      mx = max(mx, pos + 1);
    }
  }
  __shared__ int32_t smn[256], smx[256];
  smn[threadIdx.x] = mn;
  smx[threadIdx.x] = mx;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      smn[threadIdx.x] = min(smn[threadIdx.x], smn[threadIdx.x + w]);
      smx[threadIdx.x] = max(smx[threadIdx.x], smx[threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    lo[blockIdx.x] = smn[0];
    hi[blockIdx.x] = smx[0];
  }
}

// Piece codes: as k_fill_compact, with idx = the hot slot (hotidx) or nh + 1 + the source's index
// in its class's virtual space (piece table pc[(x * P + p) * 3] = {g0, g1, v0}).  *bad counts the
// sources outside every piece of the unit's class (none by construction).
template <int HB, class SideT>
__global__ __launch_bounds__(64) void k_fill_piece(int64_t n_units, const Unit *__restrict__ units,
                                                   const int64_t *__restrict__ src_off,
                                                   const int32_t *__restrict__ n_real,
                                                   const int32_t *__restrict__ col, const int64_t *__restrict__ ucum,
                                                   int C, int P, const int32_t *__restrict__ pc,
                                                   const int32_t *__restrict__ hotidx, int nh,
                                                   uint16_t *__restrict__ code16, SideT *__restrict__ cside,
                                                   unsigned long long *n_hot, unsigned long long *bad) {
  unsigned long long nhot = 0, nb = 0;
  for (int64_t b = blockIdx.x; b < n_units; b += gridDim.x) {
    const Unit u = units[b];
    const int64_t s0 = src_off[b];
    const int n = n_real[b];
    int x = 0;
    while (x + 1 < C && ucum[x + 1] <= b) ++x;  // the unit's class
    const int32_t *px = pc + (int64_t)x * P * 3;
    for (int grp = threadIdx.x; grp < u.n / 8; grp += 64) {
      SideT side = 0;
      uint32_t lo[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * grp + j;
        uint32_t idx = 0;
        if (i < n) {
          const int32_t v = col[s0 + i];
          const int32_t pos = v & 0x7FFFFFFF;
          const int32_t h = hotidx[pos];
          bool miss = false;
          idx = piece_encode(pos, h, px, P, nh, &miss);  // pr_pieces.h
          nhot += h ? 1 : 0;
          nb += miss ? 1 : 0;
          if (u.meta >= 0 && v < 0) side |= (SideT)1 << j;  // segment end (STREAM units)
        }
        lo[j] = idx & 0xFFFFu;
        side |= (SideT)((idx >> 16) & ((1u << HB) - 1u)) << (8 + HB * j);
      }
      uint4 q;
      q.x = lo[0] | lo[1] << 16;
      q.y = lo[2] | lo[3] << 16;
      q.z = lo[4] | lo[5] << 16;
      q.w = lo[6] | lo[7] << 16;
      *reinterpret_cast<uint4 *>(code16 + (int64_t)u.p8 * 8 + 8 * grp) = q;
      cside[(int64_t)u.p8 + grp] = side;
    }
  }
  atomicAdd(n_hot, nhot);
  atomicAdd(bad, nb);
}

// Host plan of the piece codes: per class the pieces in part order at kPieceAlign-aligned virtual
// starts; pc = {g0, g1, v0} per (class, part), tbl[x * kPieceTblWords + t] = byte delta
// 8 * (g0 - v0) of the piece holding virtual block t (0 elsewhere and in the sentinel word
// kPieceTbl).  vmax = the largest class's virtual extent.
struct PiecePlan {
  std::vector<int32_t> pc, tbl;
  int64_t vmax = 0;
};
static int plan_pieces(const pr_graph *g, const int32_t *cmap, int C, int P, PiecePlan *pp, hipStream_t s) {
  DevBuf lohi;
  const int64_t np = (int64_t)C * P;
  PR_TRY(lohi.alloc(sizeof(int32_t) * 2 * (size_t)np));
  hipLaunchKernelGGL(k_piece_bounds, dim3((unsigned)np), dim3(256), 0, s, g->S_pad, g->Q_pad, C, P, cmap,
                     lohi.as<int32_t>(), lohi.as<int32_t>() + np);
  PR_HIP(hipGetLastError());
  std::vector<int32_t> h((size_t)(2 * np));
  PR_HIP(hipMemcpyAsync(h.data(), lohi.p, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  pp->vmax = piece_tables(h.data(), C, P, &pp->pc, &pp->tbl);  // pr_pieces.h
  return PR_OK;
}

// Column classes of the split layout: the fewest (8, 16, 32, 64) whose class region of the part's
// gather space (its slice plus the expected received runs at P > 1) fits one XCD's 4 MiB L2 (the
// phased schedule runs one class per XCD at a time), capped at kAutoMaxClasses; PR_BOPT_CLASSES
// overrides.  More classes keep more gathers in L2 and the LDS hot sets but cost epilogue work per
// (row, class): R-MAT s26 (262 MB) -> 64 at P = 1, 2, 4 and 32 for an 8-way part (121 MB: 8 % less
// per iteration than 64); the Twitter shape stays at 64 at P = 8 (6 % better than 32); ER s24
// (134 MB) -> 64, LiveJournal (39 MB) -> 16 (profiles/r02/class_policy/).
constexpr int64_t kClassRegionBytes = 4000000;  // just under the 4 MiB L2: ER s24 (4.19 MB at 32) stays at 64
static int class_setting(const pr_build_opts &o, int64_t gather_bytes) {
  if (o.classes) return o.classes;
  for (int c = kXcds; c < kAutoMaxClasses; c *= 2)
    if (gather_bytes <= (int64_t)c * kClassRegionBytes) return c;
  return kAutoMaxClasses;
}

static int hot_slots_setting(const pr_build_opts &o) {
  const int k = o.hot_slots < 0 ? kHotSlotsDefault : o.hot_slots;
  return std::max(0, std::min(k, kHotSlotsMax));
}

int build_graph(pr_graph *g, int64_t E, const int32_t *src_in, const int32_t *dst_in) {
  static_assert(kMaxClasses == 16 * kXcds, "class counts");
  auto t_start = std::chrono::steady_clock::now();
  hipStream_t s = g->stream;
  const int32_t V = g->V;
  const int P = g->nparts, part = g->part;
  if (V < 0 || E < 0) return fail(PR_ERR_INVALID, "negative n_vertices or n_edges");
  if (E >= (int64_t(1) << 32) - 1) return fail(PR_ERR_INVALID, "n_edges must be < 2^32 - 1");
  const int b = bits_for((uint64_t)V);  // every ID < 2^b - 1: sentinel sorts last
  const unsigned T = 256;

  // ---- inputs on the device ----
  DevBuf dsrc, ddst;
  const int32_t *src = src_in, *dst = dst_in;
  if (!(g->flags & PR_INPUT_DEVICE) && E > 0) {
    PR_TRY(dsrc.alloc(sizeof(int32_t) * E));
    PR_TRY(ddst.alloc(sizeof(int32_t) * E));
    PR_HIP(hipMemcpyAsync(dsrc.p, src_in, sizeof(int32_t) * E, hipMemcpyHostToDevice, s));
    PR_HIP(hipMemcpyAsync(ddst.p, dst_in, sizeof(int32_t) * E, hipMemcpyHostToDevice, s));
    src = dsrc.as<int32_t>();
    dst = ddst.as<int32_t>();
  }

  DevBuf keys, tmp, appear, is_key, err, cnt;
  const int64_t Ealloc = E > 0 ? E : 1;
  PR_TRY(keys.alloc(sizeof(uint64_t) * Ealloc));
  PR_TRY(tmp.alloc(sizeof(uint64_t) * Ealloc));
  PR_TRY(appear.alloc((size_t)V + 1));
  PR_TRY(is_key.alloc((size_t)V + 1));
  PR_TRY(err.alloc(sizeof(unsigned)));
  PR_TRY(cnt.alloc(sizeof(unsigned long long) * 8));
  PR_HIP(hipMemsetAsync(appear.p, 0, (size_t)V + 1, s));
  PR_HIP(hipMemsetAsync(is_key.p, 0, (size_t)V + 1, s));
  PR_HIP(hipMemsetAsync(err.p, 0, sizeof(unsigned), s));
  PR_HIP(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long) * 8, s));
  if (E > 0)
    hipLaunchKernelGGL(k_pack_edges, dim3(grid_for(E, T, 65536)), dim3(T), 0, s, E, V, b, src, dst,
                       keys.as<uint64_t>(), appear.as<uint8_t>(), is_key.as<uint8_t>(),
                       err.as<unsigned>());
  if (V > 0)
    hipLaunchKernelGGL(k_check_appear, dim3(grid_for(V, T, 65536)), dim3(T), 0, s, V,
                       appear.as<uint8_t>(), err.as<unsigned>());
  PR_HIP(hipGetLastError());
  unsigned herr = 0;
  PR_HIP(hipMemcpyAsync(&herr, err.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  dsrc.reset();
  ddst.reset();
  appear.reset();
  if (herr & 1u) return fail(PR_ERR_INVALID, "edge list holds an ID outside [0, n_vertices) (dst may be -1)");
  if (herr & 2u) return fail(PR_ERR_INVALID, "an ID in [0, n_vertices) never appears in the edge list");

  // ---- A1: sort + dedupe (Sparky.java:124) ----
  PR_TRY(radix_sort_u64(keys.as<uint64_t>(), tmp.as<uint64_t>(), E, 0, 2 * b, s));
  int64_t m = 0;
  PR_TRY(compact_index(E, UniquePred{keys.as<uint64_t>()}, IdentityU64{keys.as<uint64_t>()},
                       tmp.as<uint64_t>(), &m, s));
  g->E_dedup = m;
  uint64_t *ukeys = tmp.as<uint64_t>();
  const uint64_t maskb = (uint64_t(1) << b) - 1;

  // ---- canonical CSR, degrees, flags ----
  DevBuf c_rowptr, c_col, c_deg, c_vflags;
  PR_TRY(c_rowptr.alloc(sizeof(int64_t) * ((size_t)V + 1)));
  PR_TRY(c_col.alloc(sizeof(int32_t) * (m > 0 ? m : 1)));
  PR_TRY(c_deg.alloc(sizeof(int32_t) * ((size_t)V + 1)));
  PR_TRY(c_vflags.alloc((size_t)V + 1));
  PR_HIP(hipMemsetAsync(c_deg.p, 0, sizeof(int32_t) * ((size_t)V + 1), s));
  hipLaunchKernelGGL(k_row_ptr, dim3(grid_for(m + 1, T, 65536)), dim3(T), 0, s, ukeys, m, b,
                     (int64_t)V, c_rowptr.as<int64_t>());
  if (m > 0)
    hipLaunchKernelGGL(k_canon_col_deg, dim3(grid_for(m, T, 65536)), dim3(T), 0, s, ukeys, m, maskb,
                       c_col.as<int32_t>(), c_deg.as<int32_t>());
  if (V > 0)
    hipLaunchKernelGGL(k_vflags, dim3(grid_for(V, T, 4096)), dim3(T), 0, s, V, is_key.as<uint8_t>(),
                       c_deg.as<int32_t>(), c_rowptr.as<int64_t>(), c_vflags.as<uint8_t>(),
                       cnt.as<unsigned long long>());
  PR_HIP(hipGetLastError());
  unsigned long long hc[8] = {0};
  PR_HIP(hipMemcpyAsync(hc, cnt.p, sizeof(hc), hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));
  is_key.reset();
  g->n_sink = (int64_t)hc[0];
  g->n_nolink = (int64_t)hc[1];
  g->n_indeg0 = (int64_t)hc[2];
  g->max_indeg = (int64_t)hc[3];
  const uint64_t max_outdeg = hc[4];

  // ---- internal order: out-degree desc, ID asc (hot contributions first) ----
  g->n_local_max = (V + P - 1) / P;
  g->n_local = V > part ? (V - part + P - 1) / P : 0;
  if (max_outdeg > kRowDegMask) return fail(PR_ERR_INVALID, "out-degree above 2^28-1 is not supported");
  // Column classes when the gather space (every part's slice: the columns a part reads) outgrows
  // the L2s (pr_graph.h); their count from the part's expected compacted gather space.
  int64_t gather_est = g->n_local_max * 8;
  if (P > 1 && V > 0) {
    PR_HIP(hipMemsetAsync(cnt.p, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_reader_est, dim3(grid_for(V, T, 1024)), dim3(T), 0, s, V, P, c_deg.as<int32_t>(),
                       cnt.as<unsigned long long>());
    PR_HIP(hipGetLastError());
    unsigned long long est = 0;
    PR_HIP(hipMemcpyAsync(&est, cnt.p, sizeof(est), hipMemcpyDeviceToHost, s));
    PR_HIP(hipStreamSynchronize(s));
    gather_est += (int64_t)((double)est / 1048576.0 * (double)(P - 1) / (double)P) * 8;
  }
  g->gather_est = gather_est;
  const int bd = bits_for(max_outdeg);
  const uint64_t maxd = (uint64_t(1) << bd) - 1;
  DevBuf vk, vtmp, rank_of, gpos;
  PR_TRY(vk.alloc(sizeof(uint64_t) * ((size_t)V + 1)));
  PR_TRY(vtmp.alloc(sizeof(uint64_t) * ((size_t)V + 1)));
  PR_TRY(rank_of.alloc(sizeof(int32_t) * ((size_t)V + 1)));
  PR_TRY(gpos.alloc(sizeof(int32_t) * ((size_t)V + 1)));
  if (V > 0) {
    hipLaunchKernelGGL(k_order_keys, dim3(grid_for(V, T, 4096)), dim3(T), 0, s, V, b, maxd, c_deg.as<int32_t>(),
                       vk.as<uint64_t>());
    PR_TRY(radix_sort_u64(vk.as<uint64_t>(), vtmp.as<uint64_t>(), V, 0, b + bd, s));
  }
  vtmp.reset();
  // Layout policy: the fused layout while the gather space fits the L2s, the split layout beyond
  // (profiles/r03/rows_layout/: a row-block layout with LDS row sums and no partial slots ran 2x
  // slower at ER s24 and far slower on skewed graphs, and was removed)
  const int c_split = class_setting(g->opts, gather_est);
  const bool big = (int64_t)P * g->n_local_max * 8 > kSplitMinSliceBytes;
  int layout = big ? kLayoutSplit : kLayoutFused;
  if (g->flags & PR_LAYOUT_FUSED) layout = kLayoutFused;
  if (g->flags & PR_LAYOUT_SPLIT) layout = kLayoutSplit;
  // split-layout entry codes are byte offsets below 2^31 (pr_internal.h)
  if ((int64_t)P * (g->n_local_max + 64 + kMaxClasses) * 8 >= (1ll << 31) - (1ll << 20)) layout = kLayoutFused;
  int C = layout == kLayoutSplit ? c_split : 1;
  g->layout = layout;
  g->C = C;
  g->Q_pad = (g->n_local_max + C - 1) / C;
  g->Q_pad = (g->Q_pad + 63) / 64 * 64;  // rows come in whole 64-row blocks (k_epilogue_grp)
  g->n_rows = (int64_t)C * g->Q_pad;
  g->S_pad = ((g->n_rows + 2 + 63) / 64) * 64;
  if ((int64_t)P * g->S_pad >= (int64_t(1) << 31)) return fail(PR_ERR_INVALID, "gather space exceeds 2^31 entries");
  if (V > 0) {
    hipLaunchKernelGGL(k_rank_gpos, dim3(grid_for(V, T, 65536)), dim3(T), 0, s, V, maskb, P, C,
                       g->Q_pad, g->S_pad, vk.as<uint64_t>(), rank_of.as<int32_t>(), gpos.as<int32_t>());
    PR_HIP(hipGetLastError());
  }
  ClassGeom geo{};
  geo.C = C;
  geo.Q_pad = g->Q_pad;
  geo.S_pad = g->S_pad;
  g->geo = geo;

  // ---- exchange lists (P > 1): which of this part's contributions every peer reads ----
  DevBuf cmap;  // global -> compacted gather position (P > 1, sparse exchange)
  PR_TRY(build_exchange(g, ukeys, m, b, maskb, rank_of.as<int32_t>(), gpos.as<int32_t>(), &cmap));

  // ---- the part's in-link CSRs: one per column class (one in the fused layout) ----
  const int64_t R = g->n_rows;
  const int bg = bits_for((uint64_t)P * g->S_pad);
  const int brow = bits_for((uint64_t)R);
  const int bseg = bits_for((uint64_t)C);
  const uint64_t maskg = (uint64_t(1) << bg) - 1;
  int64_t lm = 0;
  PR_TRY(compact_index(m, PartPred{ukeys, rank_of.as<int32_t>(), b, P, part},
                       PartXform{ukeys, gpos.as<int32_t>(), b, bg, brow, maskb, geo},
                       keys.as<uint64_t>(), &lm, s));
  g->local_nnz = lm;
  PR_TRY(radix_sort_u64(keys.as<uint64_t>(), tmp.as<uint64_t>(), lm, 0, bg + brow + bseg, s));
  PR_TRY(g->col.alloc(sizeof(int32_t) * (lm > 0 ? lm : 1)));
  if (lm > 0)
    hipLaunchKernelGGL(k_local_col, dim3(grid_for(lm, T, 65536)), dim3(T), 0, s,
                       keys.as<uint64_t>(), lm, maskg, g->col.as<int32_t>());
  if (cmap.p && lm > 0) {  // columns -> the compacted gather space (order within rows kept)
    DevBuf bad;
    PR_TRY(bad.alloc(sizeof(unsigned long long)));
    PR_HIP(hipMemsetAsync(bad.p, 0, sizeof(unsigned long long), s));
    hipLaunchKernelGGL(k_map_cols, dim3(grid_for(lm, T, 65536)), dim3(T), 0, s, lm, cmap.as<int32_t>(),
                       g->col.as<int32_t>(), bad.as<unsigned long long>());
    unsigned long long hb = 0;
    PR_HIP(hipMemcpyAsync(&hb, bad.p, sizeof(hb), hipMemcpyDeviceToHost, s));
    PR_HIP(hipStreamSynchronize(s));
    if (hb) return fail(PR_ERR_STATE, "exchange lists miss a source of this part's in-links");
  }
  PR_TRY(g->rowinfo.alloc(sizeof(uint32_t) * ((size_t)R + 1)));
  DevBuf orig;
  PR_TRY(orig.alloc(sizeof(int32_t) * ((size_t)R + 1)));
  hipLaunchKernelGGL(k_local_rows, dim3(grid_for(R, T, 65536)), dim3(T), 0, s, R, g->n_local, P, part,
                     geo, maskb, (g->flags & PR_DANGLING_NONE) != 0, vk.as<uint64_t>(),
                     c_deg.as<int32_t>(), c_vflags.as<uint8_t>(), g->rowinfo.as<uint32_t>(),
                     orig.as<int32_t>());
  PR_HIP(hipGetLastError());
  vk.reset();
  rank_of.reset();
  gpos.reset();

  // ---- work plans (fused: host greedy over the row pointers; split: pr_plan.hip on the GPU) ----
  const uint64_t rmask = (uint64_t(1) << brow) - 1;
  std::vector<int64_t> rp;
  std::vector<int32_t> seg_p0;
  std::vector<int32_t> lr_row, lr_p0;
  std::vector<Unit> light_units;
  int64_t pieces = 0;
  g->nblk = (R + 63) / 64;
  std::vector<int64_t> poff(kMaxClasses + 1, 0);
  if (C == 1) {
    // fused layout: one CSR over all rows, 256-thread units with the fused epilogue
    DevBuf rp_dev;
    PR_TRY(rp_dev.alloc(sizeof(int64_t) * ((size_t)R + 1)));
    hipLaunchKernelGGL(k_row_ptr_seg, dim3(grid_for(lm + 1, T, 65536)), dim3(T), 0, s, keys.as<uint64_t>(),
                       (int64_t)0, lm, bg, rmask, R, rp_dev.as<int64_t>());
    PR_HIP(hipGetLastError());
    rp.assign((size_t)R + 1, 0);
    PR_HIP(hipMemcpyAsync(rp.data(), rp_dev.p, sizeof(int64_t) * rp.size(), hipMemcpyDeviceToHost, s));
    PR_HIP(hipStreamSynchronize(s));
    keys.reset();
    tmp.reset();
    UnitPlan px;
    plan_units(rp, kUnitNnz, kUnitRows, &px);
    g->rowptr = std::move(rp_dev);
    lr_row = px.lr_row;
    lr_p0 = px.lr_p0;
    light_units = px.units;
    pieces = px.n_pieces;
    if (px.padded_len / 8 >= (int64_t(1) << 32)) return fail(PR_ERR_INVALID, "graph part too large for 32-bit unit offsets");
    PR_TRY(g->colp.alloc(sizeof(int32_t) * (px.padded_len > 0 ? px.padded_len : 8)));
    PR_TRY(build_padded_cols(px, g->col.as<int32_t>(), g->colp.as<int32_t>(), s));
    seg_p0.push_back(0);
  } else {
    // split layout: segments (row, class), class masks, block bases and wave units, planned on
    // the GPU (pr_plan.hip); the slot of segment k is k, so the class boundaries are poff
    SplitPlanner sp;
    PR_TRY(sp.segments(keys.as<uint64_t>(), lm, bg, brow, C, R, g->col.as<int32_t>(), s));
    keys.reset();
    tmp.reset();
    for (int x = 0; x <= C; ++x) poff[x] = sp.cseg[x];
    for (int x = C; x < kMaxClasses; ++x) poff[x + 1] = poff[x];
    for (int x = 0; x < C; ++x)
      if (poff[x + 1] - poff[x] >= (int64_t(1) << 29)) return fail(PR_ERR_INVALID, "a column class exceeds 2^29 segments");
    // k_epilogue_grp addresses partials through int32 absolute slot indices (< 2^31 slots: R-MAT
    // s26 has ~2^28.1, the Twitter shape ~2^29; a graph several times their size still fits)
    if (poff[C] >= (int64_t(1) << 31) - 4) return fail(PR_ERR_INVALID, "more than 2^31 - 4 partial slots");
    // per-block first slots (absolute), plus the sentinel block row of every class's end slot
    PR_TRY(sp.block_bases(true, s));
    PR_TRY(sp.units_plan(s));
    g->rmask = std::move(sp.rmask);
    g->cbase = std::move(sp.cbase);
    PR_TRY(plan_epi_walk(g));
    pieces = sp.n_pieces;
    if (sp.entries / 8 >= (int64_t(1) << 32)) return fail(PR_ERR_INVALID, "graph part too large for 32-bit unit offsets");
    // LDS hot set per class, then the entry codes
    // entry codes: compact when every region index fits (P = 1: a class's sources are its region
    // of the one slice; 2.5 bytes per entry below 2^19 region rows, 3 below 2^20); a part of a row
    // partition takes the piece codes when its classes' virtual spaces fit (the hot set then gives
    // its last kPieceTblSlots slots to the piece table), else 32-bit codes
    int slots = hot_slots_setting(g->opts);
    const bool compact = g->opts.codes != 0 && P == 1 && g->gsize == g->S_pad;
    g->code = compact && g->Q_pad < (int64_t(1) << kC20IdxBits)   ? kCodeC20
              : compact && g->Q_pad < (int64_t(1) << kC24IdxBits) ? kCodeC24
                                                                   : kCodeU32;
    PiecePlan pplan;
    if (g->opts.codes != 0 && P > 1 && P <= kMaxPackParts) {
      PR_TRY(plan_pieces(g, cmap.p ? cmap.as<int32_t>() : nullptr, C, P, &pplan, s));
      HotGeom t{};
      t.P = P;
      t.tbl = 1;
      int ps = slots;
      for (;; --ps) {  // the largest hot set that leaves LDS room for the table
        t.Kp = ps / P;
        if (t.lds_bytes() <= (size_t)kHotLdsBytes) break;
      }
      const int64_t top = (int64_t)P * (ps / P) + pplan.vmax;  // largest idx + 1
      g->code = top < (int64_t(1) << kC20IdxBits)   ? kCodeC20P
                : top < (int64_t(1) << kC24IdxBits) ? kCodeC24P
                                                     : kCodeU32;
      if (code_is_piece(g->code)) slots = ps;
    }
    HotGeom hg{};
    hg.C = C;
    hg.P = P;
    hg.Kp = slots / P;
    hg.q_load = (int)std::min<int64_t>(hg.Kp, g->Q_pad);
    hg.S_pad = g->S_pad;
    hg.Q_pad = g->Q_pad;
    hg.tbl = code_is_piece(g->code) ? 1 : 0;
    g->hot = hg;
    // hot-set gather positions per class, and the LDS slot of every hot gather position
    DevBuf hotidx;
    const int64_t nh = (int64_t)P * hg.Kp;
    PR_TRY(g->hpos.alloc(sizeof(int32_t) * (size_t)(C * nh > 0 ? C * nh : 1)));
    PR_TRY(hotidx.alloc(sizeof(int32_t) * (size_t)g->gsize));
    PR_HIP(hipMemsetAsync(hotidx.p, 0, sizeof(int32_t) * (size_t)g->gsize, s));
    if (C * nh > 0)
      hipLaunchKernelGGL(k_hot_tables, dim3(grid_for(C * nh, T, 65536)), dim3(T), 0, s, hg,
                         cmap.p ? cmap.as<int32_t>() : nullptr, g->hpos.as<int32_t>(), hotidx.as<int32_t>());
    PR_HIP(hipGetLastError());
    int n_cu = 0;
    PR_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, g->device));
    g->hot_grid = std::max(C, n_cu / C * C);  // C | grid: every class gets the same CUs
    g->hot_grid_full = g->hot_grid;
    PR_TRY(set_hot_reserve(g, g->opts.hot_reserve));

    PR_TRY(prepare_hot_kernel());
    const int64_t nu = sp.n_units;
    g->n_hunits = nu;
    g->hunits = std::move(sp.units);  // + the empty unit nu
    PR_TRY(g->hucum.alloc(sizeof(int64_t) * (kMaxClasses + 1)));
    PR_TRY(g->poff.alloc(sizeof(int64_t) * (kMaxClasses + 1)));
    const bool c20 = g->code == kCodeC20 || g->code == kCodeC20P, c24 = g->code == kCodeC24 || g->code == kCodeC24P;
    const bool piece = code_is_piece(g->code);
    if (piece) {
      PR_TRY(g->ptab.alloc(sizeof(int32_t) * pplan.tbl.size()));
      PR_HIP(hipMemcpyAsync(g->ptab.p, pplan.tbl.data(), sizeof(int32_t) * pplan.tbl.size(), hipMemcpyHostToDevice, s));
    }
    DevBuf pcd;
    if (piece) {
      PR_TRY(pcd.alloc(sizeof(int32_t) * pplan.pc.size()));
      PR_HIP(hipMemcpyAsync(pcd.p, pplan.pc.data(), sizeof(int32_t) * pplan.pc.size(), hipMemcpyHostToDevice, s));
    }
    if (c20 || c24) {
      PR_TRY(g->colh.alloc(sizeof(uint16_t) * (sp.entries > 0 ? sp.entries : 8)));
      PR_TRY(g->cside.alloc((c24 ? sizeof(uint64_t) : sizeof(uint32_t)) * (sp.entries > 0 ? sp.entries / 8 : 1)));
    } else {
      PR_TRY(g->colh.alloc(sizeof(uint32_t) * (sp.entries > 0 ? sp.entries : 8)));
      PR_TRY(g->cside.alloc(sizeof(uint32_t)));
    }
    // + 2 slots: the grouped epilogue stages class runs in 16-byte pairs (one slot past the end)
    PR_TRY(g->partial.alloc(sizeof(double) * (size_t)(poff[C] + 2)));
    g->n_slots = poff[C];
    PR_HIP(hipMemcpyAsync(g->hucum.p, sp.ucum.data(), sizeof(int64_t) * (kMaxClasses + 1), hipMemcpyHostToDevice, s));
    PR_HIP(hipMemcpyAsync(g->poff.p, poff.data(), sizeof(int64_t) * (kMaxClasses + 1), hipMemcpyHostToDevice, s));
    if (nu > 0) {
      PR_HIP(hipMemsetAsync(cnt.p, 0, 2 * sizeof(unsigned long long), s));
      const unsigned fgrid = (unsigned)std::min<int64_t>(nu, 65536);
      const int nhs = P * hg.Kp;
      if (piece && c20)
        hipLaunchKernelGGL((k_fill_piece<3, uint32_t>), dim3(fgrid), dim3(64), 0, s, nu, g->hunits.as<Unit>(),
                           sp.src_off.as<int64_t>(), sp.n_real.as<int32_t>(), g->col.as<int32_t>(),
                           g->hucum.as<int64_t>(), C, P, pcd.as<int32_t>(), hotidx.as<int32_t>(), nhs,
                           g->colh.as<uint16_t>(), g->cside.as<uint32_t>(), cnt.as<unsigned long long>(),
                           cnt.as<unsigned long long>() + 1);
      else if (piece)
        hipLaunchKernelGGL((k_fill_piece<4, uint64_t>), dim3(fgrid), dim3(64), 0, s, nu, g->hunits.as<Unit>(),
                           sp.src_off.as<int64_t>(), sp.n_real.as<int32_t>(), g->col.as<int32_t>(),
                           g->hucum.as<int64_t>(), C, P, pcd.as<int32_t>(), hotidx.as<int32_t>(), nhs,
                           g->colh.as<uint16_t>(), g->cside.as<uint64_t>(), cnt.as<unsigned long long>(),
                           cnt.as<unsigned long long>() + 1);
      else if (c20)
        hipLaunchKernelGGL((k_fill_compact<3, uint32_t>), dim3((unsigned)std::min<int64_t>(nu, 65536)), dim3(64), 0, s,
                           nu, g->hunits.as<Unit>(), sp.src_off.as<int64_t>(), sp.n_real.as<int32_t>(),
                           g->col.as<int32_t>(), g->Q_pad, hg.q_load, g->colh.as<uint16_t>(),
                           g->cside.as<uint32_t>(), cnt.as<unsigned long long>(), cnt.as<unsigned long long>() + 1);
      else if (c24)
        hipLaunchKernelGGL((k_fill_compact<4, uint64_t>), dim3((unsigned)std::min<int64_t>(nu, 65536)), dim3(64), 0, s,
                           nu, g->hunits.as<Unit>(), sp.src_off.as<int64_t>(), sp.n_real.as<int32_t>(),
                           g->col.as<int32_t>(), g->Q_pad, hg.q_load, g->colh.as<uint16_t>(),
                           g->cside.as<uint64_t>(), cnt.as<unsigned long long>(), cnt.as<unsigned long long>() + 1);
      else
        hipLaunchKernelGGL(k_fill_hot, dim3((unsigned)std::min<int64_t>(nu, 65536)), dim3(256), 0, s, nu,
                           g->hunits.as<Unit>(), sp.src_off.as<int64_t>(), sp.n_real.as<int32_t>(),
                           g->col.as<int32_t>(), hotidx.as<int32_t>(), g->colh.as<uint32_t>(),
                           cnt.as<unsigned long long>());
      PR_HIP(hipGetLastError());
      unsigned long long n_hot[2] = {0, 0};
      PR_HIP(hipMemcpyAsync(n_hot, cnt.p, sizeof(n_hot), hipMemcpyDeviceToHost, s));
      PR_HIP(hipStreamSynchronize(s));
      if (n_hot[1]) return fail(PR_ERR_STATE, "compact codes: a unit reads outside its class region / pieces");
      g->hot_cover_ppm = lm > 0 ? (int64_t)((double)n_hot[0] * 1e6 / (double)lm) : 0;
    }
    g->n_segs = sp.n_long;
    g->seg_slot = std::move(sp.seg_slot);
    g->seg_p0 = std::move(sp.seg_p0);
  }
  g->col.reset();
  if (lr_p0.empty()) lr_p0.push_back((int32_t)pieces);
  g->n_units = (int64_t)light_units.size();
  g->n_long = (int64_t)lr_row.size();
  g->n_pieces = pieces;
  PR_TRY(g->units.alloc(sizeof(Unit) * (light_units.size() + 1)));
  PR_TRY(g->lr_row.alloc(sizeof(int32_t) * (lr_row.size() + 1)));
  PR_TRY(g->lr_p0.alloc(sizeof(int32_t) * (lr_p0.size() + 1)));
  if (C == 1) {  // no long segments (the split planner filled these)
    g->n_segs = 0;
    PR_TRY(g->seg_slot.alloc(sizeof(int64_t)));
    PR_TRY(g->seg_p0.alloc(sizeof(int32_t) * (seg_p0.size() + 1)));
    PR_HIP(hipMemcpyAsync(g->seg_p0.p, seg_p0.data(), sizeof(int32_t) * seg_p0.size(), hipMemcpyHostToDevice, s));
  }
  PR_TRY(g->piece_part.alloc(sizeof(double) * ((size_t)g->n_pieces + 1)));
  if (!light_units.empty())
    PR_HIP(hipMemcpyAsync(g->units.p, light_units.data(), sizeof(Unit) * light_units.size(), hipMemcpyHostToDevice, s));
  if (!lr_row.empty())
    PR_HIP(hipMemcpyAsync(g->lr_row.p, lr_row.data(), sizeof(int32_t) * lr_row.size(), hipMemcpyHostToDevice, s));
  PR_HIP(hipMemcpyAsync(g->lr_p0.p, lr_p0.data(), sizeof(int32_t) * lr_p0.size(), hipMemcpyHostToDevice, s));
  g->orig_of_local.resize((size_t)R);
  if (R > 0)
    PR_HIP(hipMemcpyAsync(g->orig_of_local.data(), orig.p, sizeof(int32_t) * R, hipMemcpyDeviceToHost, s));
  PR_HIP(hipStreamSynchronize(s));

  // ---- iteration state ----
  PR_TRY(g->r.alloc(sizeof(double) * ((size_t)g->n_rows + 1)));
  for (int k = 0; k < 2; ++k) {
    PR_TRY(g->cbuf[k].alloc(sizeof(double) * (size_t)g->gsize));
    PR_HIP(hipMemsetAsync(g->cbuf[k].p, 0, sizeof(double) * (size_t)g->gsize, s));
  }
  // k_finalize: one wave per long row, at least 16 workgroups (4096 threads for the block
  // partials), at most 512
  g->fin_blocks = (int)std::min<int64_t>(512, std::max<int64_t>(16, (g->n_long + kThreads / kWave - 1) / (kThreads / kWave)));
  PR_TRY(g->fin_part.alloc(sizeof(double) * 2 * g->fin_blocks));
  PR_TRY(g->fin_counter.alloc(sizeof(unsigned) * 4));
  PR_HIP(hipMemsetAsync(g->fin_counter.p, 0, sizeof(unsigned) * 4, s));
  g->reset_blocks = (int)grid_for(g->n_rows > 0 ? g->n_rows : 1, 256, 2048);
  if (C > 1) {
    // one wave per group, no grid cap: the whole grid in one dispatch lets the workgroups of the
    // last round finish together (R-MAT s26: 16 K workgroups, -1.8 % per step against a 2048 cap
    // whose waves stride over 8 groups; profiles/r02/experiments.md).  One-wave workgroups pay off
    // when many groups walk (a cheap group's wave frees its LDS window at once: R-MAT s26 -0.8 %),
    // four-wave ones on uniform graphs (ER s24 +1.3 % narrow); at most 64 classes
    const int64_t ngrp = (g->nblk + kEpiGroup - 1) / kEpiGroup;
    const bool auto_narrow = g->n_walk_groups * 10 >= ngrp;
    g->epi_narrow = epi_narrow_ok(C) && (g->opts.epi_narrow < 0 ? auto_narrow : g->opts.epi_narrow != 0);
    g->ep_blocks = (int)grid_for(ngrp, epi_grp_threads(g->epi_narrow) / kWave, 1u << 20);
    PR_TRY(plan_epi_order(g));
  }
  // the split epilogue writes one {dangling, L1} partial per group (pr_spmv.h epi_group)
  const int64_t ep_parts = C > 1 ? (g->nblk + kEpiGroup - 1) / kEpiGroup : 0;
  // finalize input: fused-unit partials (C = 1) or the split epilogue's group partials (C > 1)
  PR_TRY(g->unit_part.alloc(sizeof(double) * 2 * ((size_t)g->n_units + ep_parts + 1)));
  PR_TRY(g->reset_part.alloc(sizeof(double) * 2 * g->reset_blocks));

  if (g->flags & PR_NO_CANONICAL) {
    c_rowptr.reset();
    c_col.reset();
    c_deg.reset();
    c_vflags.reset();
    g->has_canonical = false;
  } else {
    g->canon_rowptr = std::move(c_rowptr);
    g->canon_col = std::move(c_col);
    g->canon_deg = std::move(c_deg);
    g->canon_vflags = std::move(c_vflags);
    g->has_canonical = true;
  }
  PR_HIP(hipStreamSynchronize(s));
  g->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  return PR_OK;
}

}  // namespace pr
