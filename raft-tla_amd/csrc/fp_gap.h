// raftmc — TLC's second fingerprint-collision estimate, "based on the actual fingerprints":
// 1 / (the minimum distance between two fingerprints in the seen-set) [ext: TLC's FPSet
// checkFPs, as recalled; TLC is not runnable offline, SURVEY.md §8c].  Computed on request
// after a run (mc_collision_observed), never inside the BFS: the occupied entries of the
// seen-set are compacted, sorted (rocPRIM radix sort) and scanned for the smallest gap.
#pragma once
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <string>

#include "common.h"

namespace rmc {
namespace fpgap {

constexpr int GBS = 256, GPER = 16;

// fingerprints of the occupied entries (stride u64 words per entry, fingerprint first): a
// counting pass (WRITE = false), then the compaction
template <bool WRITE>
static __global__ void __launch_bounds__(GBS) compact(const u64* table, u64 slots, int stride, u64* out, unsigned long long* n) {
  const u64 tile = (u64)blockIdx.x * (GBS * GPER);
  const int lane = __lane_id();
#pragma unroll 1
  for (int j = 0; j < GPER; ++j) {
    const u64 i = tile + (u64)j * GBS + threadIdx.x;
    const u64 fp = i < slots ? table[i * (u64)stride] : 0ull;
    const u64 m = __ballot(fp != 0ull);
    if (!m) continue;
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(n, (unsigned long long)__popcll(m));
    if (!WRITE) continue;
    base = __shfl(base, leader);
    if (fp) out[base + __popcll(m & ((1ull << lane) - 1ull))] = fp;
  }
}

static __global__ void __launch_bounds__(GBS) min_gap(const u64* sorted, u64 n, unsigned long long* gap) {
  const u64 i = (u64)blockIdx.x * GBS + threadIdx.x;
  u64 g = ~0ull;
  if (i + 1 < n) g = sorted[i + 1] - sorted[i];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const u64 o = __shfl_xor(g, d);
    g = o < g ? o : g;
  }
  if (__lane_id() == 0 && g != ~0ull) atomicMin(gap, (unsigned long long)g);
}

// val = 1 / min gap (0 when fewer than two fingerprints); returns 0 or MC_E_* with err set
inline int observed(const u64* table, u64 slots, int stride, hipStream_t s, double& val, std::string& err) {
  auto chk = [&](hipError_t e, const char* what) {
    if (e != hipSuccess) { err = std::string(what) + ": " + hipGetErrorString(e); return false; }
    return true;
  };
  unsigned long long* ctr = nullptr;
  if (!chk(hipMalloc(&ctr, 24), "hipMalloc")) return -5;
  const unsigned long long init[3] = {0ull, ~0ull, 0ull};
  u64* a = nullptr; u64* b = nullptr; void* tmp = nullptr;
  int rc = 0;
  do {
    if (!chk(hipMemcpy(ctr, init, 24, hipMemcpyHostToDevice), "hipMemcpy")) { rc = -5; break; }
    const unsigned grid = (unsigned)((slots + GBS * GPER - 1) / (GBS * GPER));
    u64 n = 0;
    hipLaunchKernelGGL(compact<false>, dim3(grid), dim3(GBS), 0, s, table, slots, stride, (u64*)nullptr, ctr + 2);
    if (!chk(hipGetLastError(), "compact")) { rc = -5; break; }
    if (!chk(hipMemcpyAsync(&n, ctr + 2, 8, hipMemcpyDeviceToHost, s), "hipMemcpyAsync")) { rc = -5; break; }
    if (!chk(hipStreamSynchronize(s), "hipStreamSynchronize")) { rc = -5; break; }
    if (n < 2) { val = 0.0; break; }
    if (!chk(hipMalloc(&a, n * 8), "hipMalloc")) { rc = -6; break; }
    if (!chk(hipMalloc(&b, n * 8), "hipMalloc")) { rc = -6; break; }
    hipLaunchKernelGGL(compact<true>, dim3(grid), dim3(GBS), 0, s, table, slots, stride, a, ctr);
    if (!chk(hipGetLastError(), "compact")) { rc = -5; break; }
    size_t tb = 0;
    if (!chk(rocprim::radix_sort_keys(nullptr, tb, (const u64*)a, b, (size_t)n, 0, 64, s), "radix_sort_keys")) { rc = -5; break; }
    if (!chk(hipMalloc(&tmp, tb > 16 ? tb : 16), "hipMalloc")) { rc = -6; break; }
    if (!chk(rocprim::radix_sort_keys(tmp, tb, (const u64*)a, b, (size_t)n, 0, 64, s), "radix_sort_keys")) { rc = -5; break; }
    hipLaunchKernelGGL(min_gap, dim3((unsigned)((n + GBS - 1) / GBS)), dim3(GBS), 0, s, (const u64*)b, n, ctr + 1);
    if (!chk(hipGetLastError(), "min_gap")) { rc = -5; break; }
    unsigned long long g = 0;
    if (!chk(hipMemcpyAsync(&g, ctr + 1, 8, hipMemcpyDeviceToHost, s), "hipMemcpyAsync")) { rc = -5; break; }
    if (!chk(hipStreamSynchronize(s), "hipStreamSynchronize")) { rc = -5; break; }
    val = g == 0 || g == ~0ull ? 0.0 : 1.0 / (double)g;
  } while (false);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  if (tmp) (void)hipFree(tmp);
  (void)hipFree(ctr);
  return rc;
}

}  // namespace fpgap
}  // namespace rmc
