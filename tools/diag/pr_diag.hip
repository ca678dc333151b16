// Microbenchmarks of the memory path the SpMV kernels are bound by (diagnostics, NOT product
// code; tools/diag_gather.py, tools/diag_ta.py): random 8-byte gathers by cache policy and memory
// type, and the address unit's cost per active lane.  Self-contained: no product kernels here (A/B
// variants of those are separate builds of libpagerank_hip, PR_LIB_PATH).
#include <chrono>
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PR_HIP(call)                          \
  do {                                        \
    if ((call) != hipSuccess) return -2;      \
  } while (0)

namespace {
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
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
// Mixed probe: every thread issues 8 random vector gathers per round (all lanes active) and every
// wave S random scalar loads (wave-uniform addresses: s_load through the scalar cache) in the same
// round.  If the time stays that of S = 0 as S grows, the scalar path adds gather capacity beside
// the vector path (the cold gathers of k_spmv_hot are bound by the vector path's misses in flight).
template <int S>
__global__ __launch_bounds__(256) void k_mixed_probe(const double *__restrict__ table, uint32_t n_words, int64_t n_threads,
                                                     int rounds, uint32_t seed, double *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_threads) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, n_words * 8u, 0x00020000);
  const __attribute__((address_space(4))) double *ct = (const __attribute__((address_space(4))) double *)table;
  const uint32_t wu = (uint32_t)__builtin_amdgcn_readfirstlane((int)(t >> 6));
  double acc = 0.0, sacc = 0.0;
  for (int r = 0; r < rounds; ++r) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t w = mix32((uint32_t)t * 8u + j + seed + (uint32_t)r * 7919u) % n_words;
      v[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, w * 8u, 0, 0));
    }
    if constexpr (S > 0) {
      double sv[S];
#pragma unroll
      for (int k = 0; k < S; ++k) sv[k] = ct[mix32(wu * 4099u + (uint32_t)(r * S + k) + seed) % n_words];
#pragma unroll
      for (int k = 0; k < S; ++k) sacc += sv[k];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  if (acc + sacc == 12345.0) out[t] = acc;
}
// Line-sharing probe: random 8-byte loads where several accesses hit the same 128-byte line.
//   MODE 0: g consecutive lanes of one instruction read g different words of one line
//   MODE 1: each lane's g consecutive instructions read g different words of one line (the
//           line is an L2 hit the first time, then a vector-L1 hit while it stays there)
// Cost per instruction vs g says whether k_spmv_hot's cold gathers would get cheaper if the sources
// a segment reads sat side by side in the gather space (the TA/TCP cost is per distinct line?).
template <int MODE>
__global__ __launch_bounds__(256) void k_line_probe(const double *__restrict__ table, uint32_t n_lines, int64_t n_threads,
                                                    uint32_t seed, int g, double *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_threads) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, n_lines * 128u, 0x00020000);
  const int lane = threadIdx.x & 63;
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t w;
    if constexpr (MODE == 0) {
      const uint32_t grp = (uint32_t)(t - lane) + (uint32_t)(lane / g);
      w = (mix32(grp * 8u + j + seed) % n_lines) * 16u + (uint32_t)(lane % g);
    } else {
      w = (mix32((uint32_t)t * 8u + (uint32_t)(j / g) + seed) % n_lines) * 16u + (uint32_t)(j % g);
    }
    acc += __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, w * 8u, 0, 0));
  }
  if (acc == 12345.0) out[t] = acc;
}
// Stream probe: every thread issues 8 coalesced buffer loads (or stores) of W bytes per lane; a
// wave's lanes cover one contiguous 64 W-byte run per instruction, the table wrapping (2 MiB: L2
// resident; 1 GiB: HBM).  Lanes >= active are exec-masked.  Time per instruction vs W and active
// lanes gives the vector-memory path's cost of the code loads and partial-slot stores of
// k_spmv_hot (one b128 + one b32 load and ~1 b128 store per wave unit).
typedef unsigned int prd_u32x2 __attribute__((__vector_size__(8)));
typedef unsigned int prd_u32x4 __attribute__((__vector_size__(16)));
template <int W, bool STORE>
__global__ __launch_bounds__(256) void k_stream_probe(char *__restrict__ table, uint32_t table_bytes, int64_t n_threads,
                                                      int active, double *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_threads) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, table_bytes, 0x00020000);
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)(t >> 6);
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t off = (uint32_t)((((wave * 8 + j) * 64 + lane) * W) % table_bytes);
    if (lane < active) {
      if constexpr (STORE) {
        if constexpr (W == 4) __builtin_amdgcn_raw_buffer_store_b32(lane + j, rs, off, 0, 0);
        else if constexpr (W == 8) __builtin_amdgcn_raw_buffer_store_b64(prd_u32x2{(unsigned)lane, (unsigned)j}, rs, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b128(prd_u32x4{(unsigned)lane, (unsigned)j, 1u, 2u}, rs, off, 0, 0);
      } else {
        if constexpr (W == 4) acc ^= __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
        else if constexpr (W == 8) { const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0); acc ^= v[0] ^ v[1]; }
        else { const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0); acc ^= v[0] ^ v[1] ^ v[2] ^ v[3]; }
      }
    }
  }
  if (acc == 12345u) out[t] = acc;
}
// Scalar-path probe: every wave issues `per_wave` random 8-byte loads from uniform (wave-wide)
// addresses, which the compiler turns into s_load_dwordx2 through the scalar data cache (not the
// vector memory path the gathers of k_spmv_hot saturate).  Loads per second say whether the
// scalar path could carry a share of the cold gathers.
template <int UNROLL>
__global__ __launch_bounds__(256) void k_scalar_probe(const double *__restrict__ table, uint32_t n_words,
                                                      int64_t n_waves, int per_wave, uint32_t seed,
                                                      double *__restrict__ out) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n_waves) return;
  const __attribute__((address_space(4))) double *ct = (const __attribute__((address_space(4))) double *)table;
  const uint32_t wu = (uint32_t)__builtin_amdgcn_readfirstlane((int)w);
  double acc = 0.0;
  for (int j0 = 0; j0 < per_wave; j0 += UNROLL) {
    double v[UNROLL];
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) v[k] = ct[mix32(wu * 4099u + (uint32_t)(j0 + k) + seed) % n_words];
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) acc += v[k];
  }
  if (acc == 12345.0 && (threadIdx.x & 63) == 0) out[w] = acc;
}
// LDS probe: one 1024-thread workgroup per CU holds a `slots`-double table in LDS (the size of
// k_spmv_hot's hot set) and every thread reads `per_thread` random slots, 8 independent reads in
// flight -- the LDS side of the SpMV's gathers (roofline.gather in bench.py).
__global__ __launch_bounds__(1024) void k_lds_probe(int slots, int per_thread, uint32_t seed, double *__restrict__ out) {
  extern __shared__ double tab[];
  for (int i = threadIdx.x; i < slots; i += 1024) tab[i] = (double)i;
  __syncthreads();
  const uint32_t t = blockIdx.x * 1024u + threadIdx.x;
  double acc = 0.0;
  for (int j0 = 0; j0 < per_thread; j0 += 8) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = tab[mix32(t * 8191u + (uint32_t)(j0 + k) + seed) % (uint32_t)slots];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  if (acc == 12345.0) out[t] = acc;
}
// CU-mask probe: every workgroup (one wave) records its XCC id and raw HW_ID register (CU, SH, SE
// fields), so a stream's CU-mask bits can be mapped to physical CUs and XCDs.
__global__ void k_cu_probe(uint32_t *__restrict__ out) {
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}
}  // namespace

extern "C" {

// Launch nblocks one-wave workgroups on a stream created with the CU mask (nwords 32-bit words);
// out: 2 words per workgroup (XCC id, HW_ID).
int prd_cu_probe(int device, const uint32_t *mask, int nwords, int nblocks, uint32_t *out) {
  PR_HIP(hipSetDevice(device));
  hipStream_t st;
  PR_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)nwords, mask));
  uint32_t *d = nullptr;
  PR_HIP(hipMalloc(&d, sizeof(uint32_t) * 2 * nblocks));
  hipLaunchKernelGGL(k_cu_probe, dim3(nblocks), dim3(64), 0, st, d);
  PR_HIP(hipGetLastError());
  PR_HIP(hipMemcpyAsync(out, d, sizeof(uint32_t) * 2 * nblocks, hipMemcpyDeviceToHost, st));
  PR_HIP(hipStreamSynchronize(st));
  (void)hipFree(d);
  (void)hipStreamDestroy(st);
  return 0;
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
  return 0;
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
  return 0;
}

// Line-sharing probe (see k_line_probe): n_loads = 8 * threads; returns ms per launch.
int prd_line_probe(int device, int64_t table_bytes, int64_t n_loads, int mode, int g, int iters, double *ms_out) {
  PR_HIP(hipSetDevice(device));
  if (g < 1 || g > 16 || (mode == 1 && g > 8)) return -1;
  void *tab = nullptr, *out = nullptr;
  PR_HIP(hipMalloc(&tab, (size_t)table_bytes));
  PR_HIP(hipMemset(tab, 0, (size_t)table_bytes));
  PR_HIP(hipMalloc(&out, 8));
  const int64_t nt = n_loads / 8;
  const uint32_t nl = (uint32_t)(table_bytes / 128);
  const dim3 grid((unsigned)((nt + 255) / 256));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {
    PR_HIP(hipEventRecord(a, 0));
    for (int i = 0; i < (rep ? iters : 1); ++i) {
      if (mode == 0) hipLaunchKernelGGL(k_line_probe<0>, grid, dim3(256), 0, 0, (const double *)tab, nl, nt, 977u * i, g, (double *)out);
      else hipLaunchKernelGGL(k_line_probe<1>, grid, dim3(256), 0, 0, (const double *)tab, nl, nt, 977u * i, g, (double *)out);
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
  return 0;
}

// Stream probe (see k_stream_probe): width 4 / 8 / 16 bytes per lane, store 0/1; n_instr = 8 *
// threads / 64 wave instructions; returns ms per launch.
int prd_stream_probe(int device, int64_t table_bytes, int64_t n_loads, int width, int store, int active, int iters,
                     double *ms_out) {
  PR_HIP(hipSetDevice(device));
  void *tab = nullptr, *out = nullptr;
  PR_HIP(hipMalloc(&tab, (size_t)table_bytes));
  PR_HIP(hipMemset(tab, 0, (size_t)table_bytes));
  PR_HIP(hipMalloc(&out, 8));
  const int64_t nt = n_loads / 8;
  const dim3 grid((unsigned)((nt + 255) / 256));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {
    PR_HIP(hipEventRecord(a, 0));
    for (int i = 0; i < (rep ? iters : 1); ++i) {
      char *T = (char *)tab;
      const uint32_t tb = (uint32_t)table_bytes;
      double *O = (double *)out;
      if (store) {
        if (width == 4) hipLaunchKernelGGL((k_stream_probe<4, true>), grid, dim3(256), 0, 0, T, tb, nt, active, O);
        else if (width == 8) hipLaunchKernelGGL((k_stream_probe<8, true>), grid, dim3(256), 0, 0, T, tb, nt, active, O);
        else hipLaunchKernelGGL((k_stream_probe<16, true>), grid, dim3(256), 0, 0, T, tb, nt, active, O);
      } else {
        if (width == 4) hipLaunchKernelGGL((k_stream_probe<4, false>), grid, dim3(256), 0, 0, T, tb, nt, active, O);
        else if (width == 8) hipLaunchKernelGGL((k_stream_probe<8, false>), grid, dim3(256), 0, 0, T, tb, nt, active, O);
        else hipLaunchKernelGGL((k_stream_probe<16, false>), grid, dim3(256), 0, 0, T, tb, nt, active, O);
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
  return 0;
}

// LDS probe (see k_lds_probe): blocks x 1024 threads x per_thread random 8-byte LDS reads; ms per launch.
int prd_lds_probe(int device, int blocks, int slots, int per_thread, int iters, double *ms_out) {
  PR_HIP(hipSetDevice(device));
  const size_t lds = sizeof(double) * (size_t)slots;
  PR_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_lds_probe), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds));
  void *out = nullptr;
  PR_HIP(hipMalloc(&out, sizeof(double) * 1024 * (size_t)blocks));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {
    PR_HIP(hipEventRecord(a, 0));
    for (int i = 0; i < (rep ? iters : 1); ++i)
      hipLaunchKernelGGL(k_lds_probe, dim3(blocks), dim3(1024), lds, 0, slots, per_thread, 977u * (uint32_t)i,
                         (double *)out);
    PR_HIP(hipGetLastError());
    PR_HIP(hipEventRecord(b, 0));
    PR_HIP(hipEventSynchronize(b));
  }
  float ms = 0;
  PR_HIP(hipEventElapsedTime(&ms, a, b));
  *ms_out = ms / iters;
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(out);
  return 0;
}

// Scalar-path probe (see k_scalar_probe): n_loads uniform random loads in total; returns ms.
int prd_scalar_probe(int device, int64_t table_bytes, int64_t n_loads, int per_wave, int iters, double *ms_out) {
  PR_HIP(hipSetDevice(device));
  void *tab = nullptr, *out = nullptr;
  PR_HIP(hipMalloc(&tab, (size_t)table_bytes));
  PR_HIP(hipMemset(tab, 0, (size_t)table_bytes));
  PR_HIP(hipMalloc(&out, 8 * 1024 * 1024));
  const int64_t nw = n_loads / per_wave;
  const uint32_t nwords = (uint32_t)(table_bytes / 8);
  const dim3 grid((unsigned)((nw + 3) / 4));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {
    PR_HIP(hipEventRecord(a, 0));
    for (int i = 0; i < (rep ? iters : 1); ++i)
      hipLaunchKernelGGL(k_scalar_probe<8>, grid, dim3(256), 0, 0, (const double *)tab, nwords, nw, per_wave,
                         977u * (uint32_t)i, (double *)out);
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
  return 0;
}


// Copy probe: `nstreams` streams each copy `bytes` device to device, all at once, `iters` times;
// nocu = 1: hipMemcpyDeviceToDeviceNoCU (the copy engines, what the IPC exchange uses), 0: the
// runtime's default (a blit kernel on the CUs).  Returns ms per round (all streams' copies).
int prd_copy_probe(int device, int64_t bytes, int nstreams, int nocu, int iters, double *ms_out) {
  PR_HIP(hipSetDevice(device));
  if (nstreams < 1 || nstreams > 16) return -1;
  std::vector<void *> src(nstreams, nullptr), dst(nstreams, nullptr);
  std::vector<hipStream_t> st(nstreams, nullptr);
  for (int i = 0; i < nstreams; ++i) {
    PR_HIP(hipMalloc(&src[i], (size_t)bytes));
    PR_HIP(hipMalloc(&dst[i], (size_t)bytes));
    PR_HIP(hipMemset(src[i], 1, (size_t)bytes));
    PR_HIP(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  }
  PR_HIP(hipDeviceSynchronize());
  const hipMemcpyKind kind = nocu ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToDevice;
  double best = 1e30;
  for (int rep = 0; rep < iters + 1; ++rep) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < nstreams; ++i) PR_HIP(hipMemcpyAsync(dst[i], src[i], (size_t)bytes, kind, st[i]));
    for (int i = 0; i < nstreams; ++i) PR_HIP(hipStreamSynchronize(st[i]));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rep > 0 && ms < best) best = ms;
  }
  *ms_out = best;
  for (int i = 0; i < nstreams; ++i) {
    (void)hipStreamDestroy(st[i]);
    (void)hipFree(src[i]);
    (void)hipFree(dst[i]);
  }
  return 0;
}

// Mixed probe (see k_mixed_probe): n_threads threads x rounds x 8 vector gathers, plus S scalar
// loads per wave per round; returns ms per launch.
int prd_mixed_probe(int device, int64_t table_bytes, int64_t n_threads, int rounds, int S, int iters, double *ms_out) {
  PR_HIP(hipSetDevice(device));
  void *tab = nullptr, *out = nullptr;
  PR_HIP(hipMalloc(&tab, (size_t)table_bytes));
  PR_HIP(hipMemset(tab, 0, (size_t)table_bytes));
  PR_HIP(hipMalloc(&out, 8 * (size_t)n_threads));
  const uint32_t nw = (uint32_t)(table_bytes / 8);
  const dim3 grid((unsigned)((n_threads + 255) / 256));
  hipEvent_t a, b;
  PR_HIP(hipEventCreate(&a));
  PR_HIP(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {
    PR_HIP(hipEventRecord(a, 0));
    for (int i = 0; i < (rep ? iters : 1); ++i) {
      const double *T = (const double *)tab;
      double *O = (double *)out;
      switch (S) {
        case 0: hipLaunchKernelGGL(k_mixed_probe<0>, grid, dim3(256), 0, 0, T, nw, n_threads, rounds, 977u * i, O); break;
        case 1: hipLaunchKernelGGL(k_mixed_probe<1>, grid, dim3(256), 0, 0, T, nw, n_threads, rounds, 977u * i, O); break;
        case 2: hipLaunchKernelGGL(k_mixed_probe<2>, grid, dim3(256), 0, 0, T, nw, n_threads, rounds, 977u * i, O); break;
        case 4: hipLaunchKernelGGL(k_mixed_probe<4>, grid, dim3(256), 0, 0, T, nw, n_threads, rounds, 977u * i, O); break;
        case 8: hipLaunchKernelGGL(k_mixed_probe<8>, grid, dim3(256), 0, 0, T, nw, n_threads, rounds, 977u * i, O); break;
        case 16: hipLaunchKernelGGL(k_mixed_probe<16>, grid, dim3(256), 0, 0, T, nw, n_threads, rounds, 977u * i, O); break;
        case 32: hipLaunchKernelGGL(k_mixed_probe<32>, grid, dim3(256), 0, 0, T, nw, n_threads, rounds, 977u * i, O); break;
        case 64: hipLaunchKernelGGL(k_mixed_probe<64>, grid, dim3(256), 0, 0, T, nw, n_threads, rounds, 977u * i, O); break;
        default: return -1;
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
  return 0;
}

}  // extern "C"
