// Diagnostics library (NOT product code): A/B timing of k_spmv_units variants on a graph that
// libpagerank_hip built, in one process (cdna_hip_programming.md §5.4 rule 24).  It reuses the
// product's kernel template (pr_spmv.h) and plan code; the variants overwrite the graph's rank
// and contribution buffers, so callers must pr_reset() before using the graph again.
#include <map>
#include <memory>
#include <vector>

#include "pr_graph.h"
#include "pr_spmv.h"

using namespace pr;

// k_spmv_hot's DIAG 24 clock record (pr_spmv.h)
__device__ unsigned long long pr::pr_diag_clock[4096 * 17];

namespace {

struct Layout {  // a work plan + padded columns for a given unit size
  DevBuf units, colp, unit_part, piece_part;
  int64_t n_units = 0;
};

std::map<std::pair<pr_graph *, int>, std::unique_ptr<Layout>> g_layouts;

__global__ void k_unpad(const Unit *__restrict__ units, const int64_t *__restrict__ src_off,
                        const int32_t *__restrict__ colp, int32_t *__restrict__ col) {
  const Unit u = units[blockIdx.x];
  for (int i = threadIdx.x; i < unit_n(u); i += blockDim.x) col[src_off[blockIdx.x] + i] = colp[(int64_t)u.p8 * 8 + i];
}

int layout_for(pr_graph *g, int pt, Layout **out) {
  auto key = std::make_pair(g, pt);
  auto it = g_layouts.find(key);
  if (it != g_layouts.end()) { *out = it->second.get(); return PR_OK; }
  hipStream_t s = g->stream;
  if (g->C != 1) return fail(PR_ERR_STATE, "diag variants need the fused layout (PR_LAYOUT_FUSED)");
  std::vector<int64_t> rp((size_t)g->n_rows + 1);
  PR_HIP(hipMemcpy(rp.data(), g->rowptr.p, sizeof(int64_t) * rp.size(), hipMemcpyDeviceToHost));
  UnitPlan prod;
  plan_units(rp, kUnitNnz, kUnitRows, &prod);  // the product's plan: recover unpadded columns
  DevBuf col, du, ds;
  PR_TRY(col.alloc(sizeof(int32_t) * (g->local_nnz + 1)));
  PR_TRY(du.alloc(sizeof(Unit) * (prod.units.size() + 1)));
  PR_TRY(ds.alloc(sizeof(int64_t) * (prod.units.size() + 1)));
  PR_HIP(hipMemcpy(du.p, prod.units.data(), sizeof(Unit) * prod.units.size(), hipMemcpyHostToDevice));
  PR_HIP(hipMemcpy(ds.p, prod.src_off.data(), sizeof(int64_t) * prod.units.size(), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_unpad, dim3((unsigned)prod.units.size()), dim3(256), 0, s, du.as<Unit>(),
                     ds.as<int64_t>(), g->colp.as<int32_t>(), col.as<int32_t>());
  PR_HIP(hipStreamSynchronize(s));
  auto L = std::make_unique<Layout>();
  UnitPlan plan;
  plan_units(rp, kThreads * pt, kUnitRows, &plan);
  PR_TRY(L->colp.alloc(sizeof(int32_t) * (plan.padded_len + 8)));
  PR_TRY(build_padded_cols(plan, col.as<int32_t>(), L->colp.as<int32_t>(), s));
  PR_TRY(L->units.alloc(sizeof(Unit) * (plan.units.size() + 1)));
  PR_HIP(hipMemcpy(L->units.p, plan.units.data(), sizeof(Unit) * plan.units.size(), hipMemcpyHostToDevice));
  PR_TRY(L->unit_part.alloc(sizeof(double) * 2 * (plan.units.size() + 1)));
  PR_TRY(L->piece_part.alloc(sizeof(double) * (plan.n_pieces + 1)));
  L->n_units = (int64_t)plan.units.size();
  *out = L.get();
  g_layouts[key] = std::move(L);
  return PR_OK;
}

template <int PT, bool NT, bool MASK, int GM = 0, int XC = 0>
void launch(pr_graph *g, Layout *L, uint32_t mask) {
  const int64_t own = g->own_off;
  hipLaunchKernelGGL((k_spmv_units<PT, NT, MASK, GM, XC>), dim3((unsigned)L->n_units), dim3(kThreads), 0,
                     g->stream, L->units.as<Unit>(), g->rowptr.as<int64_t>(), L->colp.as<int32_t>(),
                     g->cbuf[0].as<double>(), g->cbuf[1].as<double>() + own, g->r.as<double>(),
                     g->rowinfo.as<uint32_t>(), L->piece_part.as<double>(), L->unit_part.as<double2>(),
                     g->slots, g->S_pad, (double)g->V, 0.15, 0.85, mask);
}

}  // namespace


// ---- gather microbenchmark (diagnostics): uniform random 8-byte loads from a table ----------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int AUX>
__global__ __launch_bounds__(256) void k_gather_bench(const double *__restrict__ table, uint32_t n_words,
                                                      int64_t n_threads, uint32_t seed, double *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_threads) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, n_words * 8u, 0x00020000);
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t w = mix32((uint32_t)t * 8u + j + seed) % n_words;
    acc += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, w * 8u, 0, AUX));
  }
  if (acc == 12345.0) out[t] = acc;
}

// TA-cost probe: every thread issues 8 random 8-byte loads from a table; lane l is active in
// load j when ((l * 8 + j) * 2654435761u >> 16) % 64 < active (OOB offset otherwise, or
// exec-masked when MASKED).  Time per instruction vs active lanes separates per-lane from
// per-instruction address-processing cost.
template <bool MASKED>
__global__ __launch_bounds__(256) void k_ta_probe(const double *__restrict__ table, uint32_t n_words, int64_t n_threads,
                                                  uint32_t seed, int active, double *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_threads) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, n_words * 8u, 0x00020000);
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t w = mix32((uint32_t)t * 8u + j + seed) % n_words;
    const bool on = (int)((((uint32_t)(lane * 8 + j) * 2654435761u) >> 16) % 64u) < active;
    if constexpr (MASKED) {
      if (on) acc += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, w * 8u, 0, 0));
    } else {
      acc += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, on ? w * 8u : 0xFFFFFFF8u, 0, 0));
    }
  }
  if (acc == 12345.0) out[t] = acc;
}

extern "C" {

// variant: 0 = PT 8 + nt cols (product), 1 = PT 8 plain cols, 2 = PT 16 + nt, 3 = PT 4 + nt,
//          4/5/6 = PT 8/16/4 + nt with gathers masked by `mask` (diagnostic: results are wrong).
int prd_time_spmv(pr_graph *g, int variant, uint32_t mask, int iters, double *ms_out) {
  const int pt = (variant == 2 || variant == 5) ? 16 : ((variant == 3 || variant == 6) ? 4 : 8);
  Layout *L = nullptr;
  PR_HIP(hipSetDevice(g->device));
  PR_TRY(layout_for(g, pt, &L));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  PR_HIP(hipEventRecord(a, g->stream));
  for (int i = 0; i < iters; ++i) {
    switch (variant) {
      case 0: launch<8, true, false>(g, L, mask); break;
      case 1: launch<8, false, false>(g, L, mask); break;
      case 2: launch<16, true, false>(g, L, mask); break;
      case 3: launch<4, true, false>(g, L, mask); break;
      case 4: launch<8, true, true>(g, L, mask); break;
      case 5: launch<16, true, true>(g, L, mask); break;
      case 6: launch<4, true, true>(g, L, mask); break;
      case 7: launch<8, true, false, 1>(g, L, mask); break;
      case 8: launch<8, true, false, 2>(g, L, mask); break;
      case 9: launch<8, true, false, 3>(g, L, mask); break;
      case 10: launch<8, true, true, 2>(g, L, mask); break;
      case 11: launch<8, true, true, 3>(g, L, mask); break;
      case 12: launch<8, true, false, 0, 8>(g, L, mask); break;
      case 13: launch<8, true, false, 3, 8>(g, L, mask); break;
      case 14: launch<8, true, false, 0, 2>(g, L, mask); break;
      case 15: launch<8, true, false, 0, 4>(g, L, mask); break;
      case 16: launch<8, true, false, 0, -8>(g, L, mask); break;
      case 17: launch<8, true, false, 0, -4>(g, L, mask); break;
      case 18: launch<8, true, false, 0, -2>(g, L, mask); break;
      default: return fail(PR_ERR_INVALID, "unknown variant");
    }
  }
  PR_HIP(hipGetLastError());
  PR_HIP(hipEventRecord(b, g->stream));
  PR_HIP(hipEventSynchronize(b));
  float ms = 0;
  PR_HIP(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *ms_out = ms / iters;
  return PR_OK;
}

// Split layout: time the heavy-row kernel k_spmv_hot<0, DIAG> on the graph's own layout.
// variant = DIAG: 0 = product, 1 = all values from LDS, 2 = no partial stores, 3 = non-temporal
// partial stores, 4 / 5 = gathers folded into 4 / 32 MiB (1, 2, 4, 5: diagnostics, results wrong);
// 13 / 14 / 15 = variants 0 / 1 / 4 with the reduce of unit i before the gathers of i+1;
// 16..19 = phased schedule (the product's): product, all-LDS, all-LDS + an out-of-range buffer
// load per entry, gathers without LDS reads; 20..22 = phased: no partial stores, temporal
// partial stores, every gather folded into the first 4 MiB; 23 = phased, the same number of
// partial-store instructions for every unit (out-of-range ones for unused passes); 24 = the
// phased kernel (ORDER 0) recording per-workgroup phase clocks (prd_clock_read); 25 = phased
// with the gathers of unit i + 1 issued before the reduce of unit i (ORDER 0, the product until
// round 2; 16 is the product, ORDER 1; 17..24 keep ORDER 0); ORDER 1 + phased: 26 = no partial
// stores, 27 = every partial store into one 256 KiB window, 28 = every value from LDS, 29 = partial
// stores of two slots per lane (16 bytes), 30 = ORDER 3 (the unit's last staged stores issued after
// the next unit's gathers), 31 / 32 = the carry added through the staging window (one add per
// lane instead of one per entry; 32 with unconditional window writes); 29 = the product since the
// 16-byte partial stores (round 2), 33 = the 8-byte partial stores before them, 34 = ORDER 4
// (the gathers of unit i + 1 in flight while unit i is reduced; adds deferred to the reduce), 35 =
// the hot set staged for the first phase only (the cost of restaging), 36 = P = 1 hot sets staged
// by LDS-DMA, 37 = no segmented scan in units where every lane holds a segment end; ORDER 1 +
// phased with DIAG 6 / 10 / 12: 38 = exec-masked gathers, 39 = sc1 gathers, 40 = sc0 gathers.
// variant + 100 * (a + 1): with the unit assignment PR_HOT_ASSIGN = a.  The hot-set size is a build setting
// (PR_HOT_SLOTS): A/B it with separate graph builds.
// Copies n workgroups' clocks of the last DIAG 24 launch (17 per workgroup, 100 MHz ticks).
int prd_clock_read(unsigned long long *out, int n) {
  if (n < 0 || n > 4096) return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(pr_diag_clock), sizeof(unsigned long long) * 17 * (size_t)n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}

// The grouped epilogue k_epilogue_grp<C, variant> alone, iters launches (rewrites r and the next
// contribution buffer from the current one, like an iteration's epilogue; pr_reset afterwards).
int prd_time_epi(pr_graph *g, int variant, int iters, double *ms_out) {
  if (g->C == 1 || !g->epi_grp) return fail(PR_ERR_STATE, "graph has no grouped epilogue");
  PR_HIP(hipSetDevice(g->device));
  const int edv = variant >= 200 ? variant / 100 - 1 : 0;
  if (edv > 0) variant = 0;
  // variant + 100: the same variant with the per-row walk of sparse groups, planned here for it
  const bool walk = variant >= 100;
  variant %= 100;
  if (variant < 0 || variant >= kNumEpiVariants) return fail(PR_ERR_INVALID, "unknown epilogue variant");
  if (walk) {
    const int keep = g->epi_var;
    g->epi_var = variant;
    const int rc = plan_epi_walk(g);
    g->epi_var = keep;
    if (rc != PR_OK) return rc;
    if (!g->epi_walk) return fail(PR_ERR_INVALID, "no per-row walk for this variant / class count");
  }
  EpiGrpFn epi = epi_grp_kernel(g->C, variant, walk);
  // variant 200 / 300 / 400 (64 classes): variant 0 with k_epilogue_grp EDIAG 1 / 2 / 3
  if (edv > 0) {
    if (g->C != 64) return fail(PR_ERR_INVALID, "EDIAG variants need 64 classes");
    epi = edv == 1 ? k_epilogue_grp<64, kEpiGroup, kEpiWin, false, false, 1>
                   : (edv == 2 ? k_epilogue_grp<64, kEpiGroup, kEpiWin, false, false, 2>
                               : k_epilogue_grp<64, kEpiGroup, kEpiWin, false, false, 3>);
    PR_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(epi), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)epi_grp_lds(0)));
  }
  const size_t lds = epi_grp_lds(variant);
  PR_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(epi), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int G = kEpiVariants[variant].G;
  const int blocks = (int)grid_for((g->nblk + G - 1) / G, kEpiThreads / kWave, 1 << 20);
  DevBuf part;
  PR_TRY(part.alloc(sizeof(double2) * (size_t)blocks));
  const int in = g->cur, out = g->cur ^ 1;
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  PR_HIP(hipEventRecord(a, g->stream));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL(epi, dim3(blocks), dim3(kEpiThreads), lds, g->stream, g->nblk, g->partial.as<double>(),
                       g->rmask.p, g->cbase.as<int32_t>(), g->rowinfo.as<uint32_t>(), g->r.as<double>(),
                       g->cbuf[out].as<double>() + g->own_off, g->cbuf[in].as<double>(), g->slots, (double)g->V,
                       g->teleport, g->damping, part.as<double2>(), g->eoff.as<int64_t>(), g->epos.as<uint16_t>());
  PR_HIP(hipGetLastError());
  PR_HIP(hipEventRecord(b, g->stream));
  PR_HIP(hipEventSynchronize(b));
  float ms = 0;
  PR_HIP(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *ms_out = ms / iters;
  return PR_OK;
}

int prd_time_split(pr_graph *g, int variant, uint32_t mask, int iters, double *ms_out) {
  (void)mask;
  if (g->C == 1) return fail(PR_ERR_STATE, "graph has the fused layout");
  static const void *tab[41] ={reinterpret_cast<const void *>(&k_spmv_hot<0, 0>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 2>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 3>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 4>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 5>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 6>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 0, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 8>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 9>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 10>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 11>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 12>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 0>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 4>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 0, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 1, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 13, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 14, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 2, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 3, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 4, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 23, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 24, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<0, 0, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 2, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 30, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 1, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 31, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<3, 0, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 32, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 33, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 34, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<4, 0, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 35, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 36, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 37, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 6, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 10, 1>),
                               reinterpret_cast<const void *>(&k_spmv_hot<1, 12, 1>)};
  // variant + 100 * (a + 1): the same kernel with the unit assignment PR_HOT_ASSIGN = a
  // (HotGeom.assign); a plain variant keeps the graph's own
  const int assign = variant / 100 - 1;
  variant %= 100;
  if (variant < 0 || variant > 40 || assign > 3) return fail(PR_ERR_INVALID, "unknown variant");
  PR_HIP(hipSetDevice(g->device));
  const void *kern = tab[variant];
  PR_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const uint32_t cin_bytes = (uint32_t)(sizeof(double) * g->gsize);
  Unit *units = g->hunits.as<Unit>();
  int64_t *ucum = g->hucum.as<int64_t>();
  HotGeom hg = g->hot;
  if (assign >= 0) hg.assign = assign;
  uint32_t *colh = g->colh.as<uint32_t>(), *hmeta = g->hmeta.as<uint32_t>();
  double *cin = g->cbuf[0].as<double>(), *partial = g->partial.as<double>(), *pp = g->piece_part.as<double>();
  int64_t *poff = g->poff.as<int64_t>();
  int32_t *hpos = g->hpos.as<int32_t>();
  // must match k_spmv_hot's parameter list exactly
  int ph0 = 0, ph1 = g->C / kXcds;
  void *args[] = {&units, &ucum, &hg, &colh, &hmeta, &cin, (void *)&cin_bytes, &partial, &poff, &pp, &hpos, &ph0, &ph1};
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  PR_HIP(hipEventRecord(a, g->stream));
  for (int i = 0; i < iters; ++i)
    PR_HIP(hipLaunchKernel(kern, dim3((unsigned)g->hot_grid), dim3(kHotThreads), args,
                           g->hot.lds_bytes(), g->stream));
  PR_HIP(hipGetLastError());
  PR_HIP(hipEventRecord(b, g->stream));
  PR_HIP(hipEventSynchronize(b));
  float ms = 0;
  PR_HIP(hipEventElapsedTime(&ms, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *ms_out = ms / iters;
  return PR_OK;
}


// mode: 0 hipMalloc + plain loads, 1 nt, 2 sc1, 3 sc0|sc1, 4 uncached memory (hipDeviceMallocUncached),
// 5 fine-grained memory (hipDeviceMallocFinegrained).  8 loads per thread.
int prd_gather_bench(int device, int64_t table_bytes, int64_t n_loads, int mode, int iters, double *ms_out) {
  PR_HIP(hipSetDevice(device));
  void *tab = nullptr, *out = nullptr;
  const unsigned flags = mode == 4 ? hipDeviceMallocUncached : (mode == 5 ? hipDeviceMallocFinegrained : 0u);
  if (flags) PR_HIP(hipExtMallocWithFlags(&tab, (size_t)table_bytes, flags));
  else PR_HIP(hipMalloc(&tab, (size_t)table_bytes));
  PR_HIP(hipMemset(tab, 0, (size_t)table_bytes));
  PR_HIP(hipMalloc(&out, 8));
  const int64_t nt = n_loads / 8;
  const uint32_t nw = (uint32_t)(table_bytes / 8);
  const dim3 grid((unsigned)((nt + 255) / 256));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms
    PR_HIP(hipEventRecord(a, 0));
    for (int i = 0; i < (rep ? iters : 1); ++i) {
      const uint32_t seed = 977u * (uint32_t)i;
      switch (mode) {
        case 1: hipLaunchKernelGGL(k_gather_bench<2>, grid, dim3(256), 0, 0, (const double *)tab, nw, nt, seed, (double *)out); break;
        case 2: hipLaunchKernelGGL(k_gather_bench<16>, grid, dim3(256), 0, 0, (const double *)tab, nw, nt, seed, (double *)out); break;
        case 3: hipLaunchKernelGGL(k_gather_bench<17>, grid, dim3(256), 0, 0, (const double *)tab, nw, nt, seed, (double *)out); break;
        default: hipLaunchKernelGGL(k_gather_bench<0>, grid, dim3(256), 0, 0, (const double *)tab, nw, nt, seed, (double *)out); break;
      }
    }
    PR_HIP(hipGetLastError());
    PR_HIP(hipEventRecord(b, 0));
    PR_HIP(hipEventSynchronize(b));
  }
  float ms = 0;
  PR_HIP(hipEventElapsedTime(&ms, a, b));
  *ms_out = ms / iters;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(tab);
  (void)hipFree(out);
  return PR_OK;
}


// TA probe (see k_ta_probe): n_loads = 8 * threads; returns ms per launch.
int prd_ta_probe(int device, int64_t table_bytes, int64_t n_loads, int active, int masked, int iters, double *ms_out) {
  PR_HIP(hipSetDevice(device));
  void *tab = nullptr, *out = nullptr;
  PR_HIP(hipMalloc(&tab, (size_t)table_bytes));
  PR_HIP(hipMemset(tab, 0, (size_t)table_bytes));
  PR_HIP(hipMalloc(&out, 8));
  const int64_t nt = n_loads / 8;
  const uint32_t nw = (uint32_t)(table_bytes / 8);
  const dim3 grid((unsigned)((nt + 255) / 256));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {
    PR_HIP(hipEventRecord(a, 0));
    for (int i = 0; i < (rep ? iters : 1); ++i) {
      if (masked) hipLaunchKernelGGL(k_ta_probe<true>, grid, dim3(256), 0, 0, (const double *)tab, nw, nt, 977u * i, active, (double *)out);
      else hipLaunchKernelGGL(k_ta_probe<false>, grid, dim3(256), 0, 0, (const double *)tab, nw, nt, 977u * i, active, (double *)out);
    }
    PR_HIP(hipGetLastError());
    PR_HIP(hipEventRecord(b, 0));
    PR_HIP(hipEventSynchronize(b));
  }
  float ms = 0;
  PR_HIP(hipEventElapsedTime(&ms, a, b));
  *ms_out = ms / iters;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(tab);
  (void)hipFree(out);
  return PR_OK;
}

void prd_release(void) { g_layouts.clear(); }

}  // extern "C"
