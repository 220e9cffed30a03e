// TEST HARNESS ONLY.  Device-vs-host probe of the TLC-mode history-rank refinement
// (memb_spec.h tlc_refine) on the successors of Init and of their successors: variant 0 is the
// product's apply(); variants 1-3 are local restatements of the refinement loop written in
// different shapes, to find which form the device compiler gets right.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../raft-tla_amd/csrc/memb_text.h"

using namespace rmc;
using S = Memb<3, 2, 18>;
using W = S::Work;
constexpr int NV = 4;

struct R { int act; u64 hr0[NV], hr1[NV]; };

template <int V>
__host__ __device__ void refine(const W& s, W& t, const S::Delta& d, u32 cfgt) {
  (void)s;
  u64 x[2], y[2];
  const int n = S::appended_entries(d, x[0], y[0], x[1], y[1]);
  for (int e = 0; e < n && !(t.hr1 & S::HR_DISCRETE); ++e) {
    const u64 xe = e ? x[1] : x[0], ye = e ? y[1] : y[0];
    u64 w0 = 0, w1 = 0;
    bool distinct = true;
    if (V == 1) {   // same as the product, loops as written
#pragma unroll 1
      for (int p = 0; p < S::NPERM; ++p) {
        const u32 rp = S::hrank(t, p);
        const u64 kp = S::entry_key(xe, ye, S::perm_of(p), cfgt);
        u32 r = 0;
#pragma unroll 1
        for (int q = 0; q < S::NPERM; ++q) {
          const u32 rq = S::hrank(t, q);
          if (rq > rp) continue;
          const u64 kq = S::entry_key(xe, ye, S::perm_of(q), cfgt);
          r += (rq < rp || kq < kp) ? 1u : 0u;
          distinct &= q == p || rq != rp || kq != kp;
        }
        if (p < S::RPW) w0 |= (u64)r << (S::RKB * p); else w1 |= (u64)r << (S::RKB * (p - S::RPW));
      }
    } else if (V == 2) {   // no early continue: one lexicographic comparison
#pragma unroll 1
      for (int p = 0; p < S::NPERM; ++p) {
        const u32 rp = S::hrank(t, p);
        const u64 kp = S::entry_key(xe, ye, S::perm_of(p), cfgt);
        u32 r = 0;
#pragma unroll 1
        for (int q = 0; q < S::NPERM; ++q) {
          const u32 rq = S::hrank(t, q);
          const u64 kq = S::entry_key(xe, ye, S::perm_of(q), cfgt);
          r += (rq < rp || (rq == rp && kq < kp)) ? 1u : 0u;
          distinct = distinct && (q == p || rq != rp || kq != kp);
        }
        if (p < S::RPW) w0 |= (u64)r << (S::RKB * p); else w1 |= (u64)r << (S::RKB * (p - S::RPW));
      }
    } else {   // V == 3: ranks and keys in unrolled arrays
      u32 rk[S::NPERM]; u64 ky[S::NPERM];
#pragma unroll
      for (int p = 0; p < S::NPERM; ++p) { rk[p] = S::hrank(t, p); ky[p] = S::entry_key(xe, ye, S::perm_of(p), cfgt); }
#pragma unroll
      for (int p = 0; p < S::NPERM; ++p) {
        u32 r = 0;
#pragma unroll
        for (int q = 0; q < S::NPERM; ++q) {
          r += (rk[q] < rk[p] || (rk[q] == rk[p] && ky[q] < ky[p])) ? 1u : 0u;
          if (q != p) distinct = distinct && (rk[q] != rk[p] || ky[q] != ky[p]);
        }
        if (p < S::RPW) w0 |= (u64)r << (S::RKB * p); else w1 |= (u64)r << (S::RKB * (p - S::RPW));
#if defined(__HIP_DEVICE_COMPILE__)
        if (xe == 0xb)
          printf("V3 p %d rk %u ky %llx r %u | rk0 %u rk1 %u ky0 %llx ky1 %llx hr0 %llx hr1 %llx RKB %d RPW %d NPERM %d\n", p, rk[p],
                 (unsigned long long)ky[p], r, rk[0], rk[1], (unsigned long long)ky[0], (unsigned long long)ky[1],
                 (unsigned long long)t.hr0, (unsigned long long)t.hr1, S::RKB, S::RPW, S::NPERM);
#endif
      }
    }
    t.hr0 = w0; t.hr1 = w1 | (distinct ? S::HR_DISCRETE : 0ull);
  }
}

__host__ __device__ R eval(const W& s, int slot, const MembRuntime& rt) {
  int k, sub; S::inst_of_slot(slot, k, sub);
  u32 err = 0;
  R r{};
  W t;
  r.act = S::group_enabled(k, rt.next) ? S::apply(s, k, sub, t, err, rt) : -1;
  if (r.act < 0) return r;
  r.hr0[0] = t.hr0; r.hr1[0] = t.hr1;
  W t1 = s; S::Delta d{0, 0, S::HK_NONE, false, false};
  S::apply_inner(s, k, sub, t1, d, err, rt);
  W a = t1, b = t1, c = t1;
  refine<1>(s, a, d, rt.cfg_type); refine<2>(s, b, d, rt.cfg_type); refine<3>(s, c, d, rt.cfg_type);
  r.hr0[1] = a.hr0; r.hr1[1] = a.hr1; r.hr0[2] = b.hr0; r.hr1[2] = b.hr1; r.hr0[3] = c.hr0; r.hr1[3] = c.hr1;
  return r;
}

__global__ void probe(const W* states, int n, R* out, MembRuntime rt) {
  const int i = threadIdx.x + blockIdx.x * blockDim.x;
  if (i >= n * S::NSLOT) return;
  out[i] = eval(states[i / S::NSLOT], i % S::NSLOT, rt);
}

int main(int argc, char** argv) {
  CfgFile cfg = parse_cfg_text(read_text_file(argv[1]));
  MembModel m = resolve_memb_model(cfg);
  MembRuntime rt = m.rt;
  rt.sym_tlc = 1;
  // Init and its successors (two levels of parents, history ranks not yet discrete)
  std::vector<W> st(1);
  S::init(st[0]);
  for (int slot = 0; slot < S::NSLOT; ++slot) {
    int k, sub; S::inst_of_slot(slot, k, sub); u32 err = 0; W t;
    if (S::group_enabled(k, rt.next) && S::apply(st[0], k, sub, t, err, rt) >= 0) st.push_back(t);
  }
  const int n = (int)st.size();
  W* ds; R* d;
  (void)hipMalloc(&ds, n * sizeof(W)); (void)hipMalloc(&d, n * S::NSLOT * sizeof(R));
  (void)hipMemcpy(ds, st.data(), n * sizeof(W), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3((n * S::NSLOT + 127) / 128), dim3(128), 0, 0, ds, n, d, rt);
  if (hipDeviceSynchronize() != hipSuccess) { std::printf("kernel failed\n"); return 1; }
  std::vector<R> h(n * S::NSLOT);
  (void)hipMemcpy(h.data(), d, h.size() * sizeof(R), hipMemcpyDeviceToHost);
  int bad[NV] = {0}, hostbad[NV] = {0}, pairs = 0;
  for (int i = 0; i < n * S::NSLOT; ++i) {
    const R want = eval(st[i / S::NSLOT], i % S::NSLOT, rt);
    if (want.act < 0 && h[i].act < 0) continue;
    ++pairs;
    for (int v = 0; v < NV; ++v) {
      bad[v] += want.act != h[i].act || want.hr0[0] != h[i].hr0[v] || want.hr1[0] != h[i].hr1[v];
      hostbad[v] += want.hr0[0] != want.hr0[v] || want.hr1[0] != want.hr1[v];
    }
  }
  std::printf("pairs %d\n", pairs);
  for (int v = 0; v < NV; ++v) std::printf("variant %d: device mismatches %d, host self-mismatches %d\n", v, bad[v], hostbad[v]);
  return 0;
}
