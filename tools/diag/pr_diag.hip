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
  const int64_t own = (int64_t)g->part * g->S_pad;
  hipLaunchKernelGGL((k_spmv_units<PT, NT, MASK, GM, XC>), dim3((unsigned)L->n_units), dim3(kThreads), 0,
                     g->stream, L->units.as<Unit>(), g->rowptr.as<int64_t>(), L->colp.as<int32_t>(),
                     g->cbuf[0].as<double>(), g->cbuf[1].as<double>() + own, g->r.as<double>(),
                     g->rowinfo.as<uint32_t>(), L->piece_part.as<double>(), L->unit_part.as<double2>(),
                     g->nparts, g->S_pad, (double)g->V, 0.15, 0.85, mask);
}

}  // namespace

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

// Split layout variants on the graph's own layout: 0 = product kernel, 1 = gathers masked by
// `mask` (diagnostics: results wrong).
int prd_time_split(pr_graph *g, int variant, uint32_t mask, int iters, double *ms_out) {
  if (g->C == 1) return fail(PR_ERR_STATE, "graph has the fused layout");
  PR_HIP(hipSetDevice(g->device));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  PR_HIP(hipEventRecord(a, g->stream));
  for (int i = 0; i < iters; ++i) {
    if (variant == 4)
      hipLaunchKernelGGL((k_spmv_split_persist<kPerThread, true, 8>), dim3(2048), dim3(kThreads), 0,
                         g->stream, g->sunits.as<Unit>(), g->n_sunits, g->lens.as<uint16_t>(), g->colp.as<int32_t>(),
                         g->cbuf[0].as<double>(), g->partial.as<double>(), g->piece_part.as<double>(),
                         g->n_heavy);
    else if (variant == 2 || variant == 3)
      hipLaunchKernelGGL((k_spmv_split_persist<kPerThread, true>), dim3(variant == 2 ? 1536 : 1024), dim3(kThreads), 0,
                         g->stream, g->sunits.as<Unit>(), g->n_sunits, g->lens.as<uint16_t>(), g->colp.as<int32_t>(),
                         g->cbuf[0].as<double>(), g->partial.as<double>(), g->piece_part.as<double>(),
                         g->n_heavy);
    else if (variant == 0)
      hipLaunchKernelGGL((k_spmv_split<kPerThread, true, false>), dim3((unsigned)g->n_sunits), dim3(kThreads), 0,
                         g->stream, g->sunits.as<Unit>(), g->lens.as<uint16_t>(), g->colp.as<int32_t>(),
                         g->cbuf[0].as<double>(), g->partial.as<double>(), g->piece_part.as<double>(),
                         g->n_heavy, mask);
    else
      hipLaunchKernelGGL((k_spmv_split<kPerThread, true, true>), dim3((unsigned)g->n_sunits), dim3(kThreads), 0,
                         g->stream, g->sunits.as<Unit>(), g->lens.as<uint16_t>(), g->colp.as<int32_t>(),
                         g->cbuf[0].as<double>(), g->partial.as<double>(), g->piece_part.as<double>(),
                         g->n_heavy, mask);
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

void prd_release(void) { g_layouts.clear(); }

}  // extern "C"
