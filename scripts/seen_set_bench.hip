// Seen-set microbenchmark, a development tool: random 8-B probes and
// insert-if-absent CAS over a u64 open-addressing table on one MI355X, by table size, to
// see where the probe rate is set (HBM, Infinity Cache, L2).
//
//   hipcc -O3 --offload-arch=gfx950 -o seen_set_bench scripts/seen_set_bench.hip
//   ./seen_set_bench                -> one JSON line per (table MiB, mode)
//   ./seen_set_bench calib          -> the 4 GiB table, probe mode only (2^28 probes per launch):
//                                      the known probe count that calibrates rocprofv3's
//                                      FETCH_SIZE for 8-B random loads (scripts/fetch_calib.sh)
//
// Keys: splitmix64 from seed 0x9E3779B97F4A7C15.  Modes: "probe" = a load of
// the home slot per key (the seen-set lookup of a duplicate successor); "insert" = the
// lookup plus atomicCAS of empty home slots (load factor grows to keys/slots over the run).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned long long u64;
constexpr int BS = 256, PER = 16;

__device__ inline u64 splitmix(u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <bool INSERT>
__global__ void __launch_bounds__(BS) probe(u64* table, u64 mask, u64 n, u64 salt, unsigned long long* out) {
  const u64 tile = (u64)blockIdx.x * (BS * PER);
  u64 k[PER], c[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const u64 i = tile + (u64)j * BS + threadIdx.x;
    k[j] = i < n ? (splitmix(i ^ salt) | 1ull) : 0ull;
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) c[j] = k[j] ? table[k[j] & mask] : 0ull;
  u64 acc = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (INSERT && k[j] && c[j] == 0ull) c[j] = atomicCAS(&table[k[j] & mask], 0ull, k[j]);
    acc += c[j] == k[j];
  }
  for (int j = 0; j < PER; ++j) acc ^= c[j];
  if (acc == salt + 1) out[0] = acc;   // keep the loads live (never true: salt + 1 is even, acc's keys are odd)
}

int main(int argc, char** argv) {
  const bool calib = argc > 1 && !std::strcmp(argv[1], "calib");
  const std::vector<u64> mib = calib ? std::vector<u64>{4096} : std::vector<u64>{4, 16, 64, 256, 1024, 4096};
  const u64 n = 1ull << 28;   // 268M probes per launch
  for (u64 m : mib) {
    const u64 slots = m << 17;   // MiB -> 8-B slots
    u64* t = nullptr;
    unsigned long long* out = nullptr;
    if (hipMalloc(&t, slots * 8) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
    hipMemset(t, 0, slots * 8);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const unsigned grid = (unsigned)((n + BS * PER - 1) / (BS * PER));
    for (int mode = 0; mode < (calib ? 1 : 2); ++mode) {
      // warm-up launch, then 3 timed launches with fresh keys
      if (mode) hipLaunchKernelGGL(probe<true>, dim3(grid), dim3(BS), 0, 0, t, slots - 1, n, 0ull, out);
      else hipLaunchKernelGGL(probe<false>, dim3(grid), dim3(BS), 0, 0, t, slots - 1, n, 0ull, out);
      hipEventRecord(a);
      for (int r = 1; r <= 3; ++r) {
        if (mode) hipLaunchKernelGGL(probe<true>, dim3(grid), dim3(BS), 0, 0, t, slots - 1, n, (u64)r << 40, out);
        else hipLaunchKernelGGL(probe<false>, dim3(grid), dim3(BS), 0, 0, t, slots - 1, n, (u64)r << 40, out);
      }
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double probes = 3.0 * (double)n, sec = ms / 1e3;
      std::printf("{\"table_mib\": %llu, \"mode\": \"%s\", \"gprobes_per_s\": %.2f, \"ns_per_probe\": %.4f, "
                  "\"line_GBps\": %.0f}\n",
                  m, mode ? "insert" : "probe", probes / sec / 1e9, sec * 1e9 / probes, probes * 64 / sec / 1e9);
      std::fflush(stdout);
    }
    hipFree(t); hipFree(out);
  }
  return 0;
}
