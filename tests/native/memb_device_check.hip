// TEST HARNESS ONLY (never part of the product).  Device-vs-host equivalence of
// the packed tlc_membership spec (raft-tla_amd/csrc/memb_spec.h): the host runs a
// FIFO BFS to collect the states of the first levels, then every (state, slot)
// pair is evaluated by one GPU thread and by the host — successor action, packed
// successor words, constraint verdict, invariant verdict and the symmetric FP64
// must agree bit for bit.
//   memb_device_check CFG DEPTH   -> JSON {"pairs": n, "mismatches": m, "first": "..."}
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../raft-tla_amd/csrc/memb_backend.hip"

using namespace rmc;
using S = Memb<SHAPE_N, SHAPE_NV, 2 * SHAPE_N * SHAPE_N>;
using W = S::Work;

struct Out {
  int act, inm;
  u32 inv, err;
  u64 fp;
  u32 w[S::NW];
};

__global__ void eval_pairs(const u32* states, u64 nstates, Out* out, MembRuntime rt, u64 seed) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstates * S::NSLOT) return;
  const u64 st = i / S::NSLOT;
  const int slot = (int)(i % S::NSLOT);
  u32 w[S::NW];
  for (int q = 0; q < S::NW; ++q) w[q] = states[st * S::NW + q];
  W s, t;
  S::unpack(w, s);
  int k, sub;
  S::inst_of_slot(slot, k, sub);
  Out o{};
  o.act = S::group_enabled(k, rt.next) ? S::apply(s, k, sub, t, o.err, rt) : -1;
  if (o.act >= 0) {
    o.inm = S::in_model(t, s, rt);
    o.inv = S::check_invariants(t, rt);
    o.fp = o.inm ? S::fingerprint(t, seed, rt) : 0;
    S::pack(t, o.w);
  }
  out[i] = o;
}

int main(int argc, char** argv) {
  CfgFile cfg = parse_cfg_text(read_text_file(argv[1]));
  MembModel m = resolve_memb_model(cfg);
  const int depth = std::atoi(argv[2]);
  MembRuntime rt = m.rt;
  if (std::getenv("SYM_TLC") && rt.symmetry) rt.sym_tlc = 1;   // MC_COMPAT_SYM_TLC
  const u64 seed = 0x5EED5EED2024ull;
  std::vector<W> all, fr(1);
  S::init(fr[0]);
  std::unordered_set<u64> seen{S::fingerprint(fr[0], seed, rt)};
  u32 err = 0;
  for (int d = 1; d <= depth && !fr.empty(); ++d) {
    std::vector<W> nx;
    for (auto& s : fr) {
      all.push_back(s);
      for (int slot = 0; slot < S::NSLOT; ++slot) {
        int k, sub; S::inst_of_slot(slot, k, sub);
        if (!S::group_enabled(k, rt.next)) continue;
        W t; if (S::apply(s, k, sub, t, err, rt) < 0 || !S::in_model(t, s, rt)) continue;
        if (seen.insert(S::fingerprint(t, seed, rt)).second) nx.push_back(t);
      }
    }
    fr.swap(nx);
  }
  const u64 n = all.size(), np = n * S::NSLOT;
  std::vector<u32> hs(n * S::NW);
  for (u64 q = 0; q < n; ++q) { u32 w[S::NW]; S::pack(all[q], w); for (int j = 0; j < S::NW; ++j) hs[q * S::NW + j] = w[j]; }
  u32* ds; Out* dout;
  if (hipMalloc(&ds, hs.size() * 4) != hipSuccess || hipMalloc(&dout, np * sizeof(Out)) != hipSuccess) { std::printf("{\"error\": \"alloc\"}\n"); return 1; }
  (void)hipMemcpy(ds, hs.data(), hs.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(eval_pairs, dim3((unsigned)((np + 127) / 128)), dim3(128), 0, 0, ds, n, dout, rt, seed);
  if (hipDeviceSynchronize() != hipSuccess) { std::printf("{\"error\": \"kernel\"}\n"); return 1; }
  std::vector<Out> dev(np);
  (void)hipMemcpy(dev.data(), dout, np * sizeof(Out), hipMemcpyDeviceToHost);
  MembText<S> text(m);
  u64 bad = 0; std::string first;
  for (u64 i = 0; i < np; ++i) {
    const W& s = all[i / S::NSLOT];
    const int slot = (int)(i % S::NSLOT);
    int k, sub; S::inst_of_slot(slot, k, sub);
    Out h{}; W t;
    h.act = S::group_enabled(k, rt.next) ? S::apply(s, k, sub, t, h.err, rt) : -1;
    if (h.act >= 0) { h.inm = S::in_model(t, s, rt); h.inv = S::check_invariants(t, rt); h.fp = h.inm ? S::fingerprint(t, seed, rt) : 0; S::pack(t, h.w); }
    const Out& d = dev[i];
    bool same = h.act == d.act && (h.act < 0 || (h.inm == d.inm && h.inv == d.inv && h.fp == d.fp && h.err == d.err));
    if (same && h.act >= 0) for (int j = 0; j < S::NW; ++j) same &= h.w[j] == d.w[j];
    if (!same) {
      if (!bad) {
        char buf[512];
        std::snprintf(buf, sizeof buf, "state %llu slot %d: host act %d inm %d inv %u fp %016llx err %u | dev act %d inm %d inv %u fp %016llx err %u",
                      (unsigned long long)(i / S::NSLOT), slot, h.act, h.inm, h.inv, (unsigned long long)h.fp, h.err, d.act, d.inm, d.inv,
                      (unsigned long long)d.fp, d.err);
        first = buf;
        for (int j = 0; j < S::NW; ++j) if (h.act >= 0 && h.w[j] != d.w[j]) { std::snprintf(buf, sizeof buf, "; word %d host %08x dev %08x", j, h.w[j], d.w[j]); first += buf; break; }
        first += " ; parent " + text.text(s, false).substr(0, 300);
      }
      ++bad;
    }
  }
  // the product's generate kernel over the same states (one chunk): its fingerprint slots must
  // equal the host's fingerprint of every in-model successor (0 elsewhere)
  u64 gbad = 0;
  {
    u64 *dcand, *dctr; unsigned short* dns;
    (void)hipMalloc(&dcand, np * 8); (void)hipMalloc(&dns, n * 2); (void)hipMalloc(&dctr, 64 * 8);
    (void)hipMemset(dctr, 0, 64 * 8);
    u32* dst4;
    (void)hipMalloc(&dst4, n * S::NWP * 4);
    std::vector<u32> h4(n * S::NWP, 0);
    for (u64 q = 0; q < n; ++q) for (int j = 0; j < S::NW; ++j) h4[q * S::NWP + j] = hs[q * S::NW + j];
    (void)hipMemcpy(dst4, h4.data(), h4.size() * 4, hipMemcpyHostToDevice);
    MGenArgs g{};
    const u64 nblk = (n + 255) / 256;
    u32 *dcells, *dcells_oom, *dcount;
    (void)hipMalloc(&dcells, nblk * 256 * S::NSLOT * 4);
    (void)hipMalloc(&dcells_oom, nblk * 256 * S::NSLOT * 4);
    (void)hipMalloc(&dcount, nblk * 8 * 4);
    g.states = dst4; g.chunk_begin = 0; g.chunk_count = n; g.rank0 = 0; g.cand = dcand; g.cells = dcells; g.cells_oom = dcells_oom;
    g.cell_count = dcount; g.nsucc = dns; g.seed = seed; g.rt = rt; g.inv_oom = 1; g.deadlock = 0; g.ctr = (unsigned long long*)dctr;
    hipLaunchKernelGGL((memb_expand<S>), dim3((unsigned)nblk), dim3(256), 0, 0, g);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("{\"error\": \"expand kernel\"}\n"); return 1; }
    // validate every workgroup's two cell lists on the host before any kernel dereferences them
    {
      std::vector<u32> cnts(nblk * 8);   // per workgroup: in-model cells of waves 0-3, out-of-model cells of waves 0-3
      (void)hipMemcpy(cnts.data(), dcount, nblk * 8 * 4, hipMemcpyDeviceToHost);
      u64 nbad = 0, nwant_in = 0, nwant_oom = 0, ncells = 0, noom = 0;
      std::vector<char> seen_cell(np, 0);
      auto check = [&](u32 c, bool want_in, u64 blk) {
        const u64 sl = c / n, st = c - sl * n;
        bool ok = c < np && sl < (u64)S::NSLOT && !seen_cell[c] && st / 256 == blk;
        if (ok) {
          seen_cell[c] = 1;
          int k, sub; S::inst_of_slot((int)sl, k, sub);
          W t; u32 e = 0;
          ok = S::group_enabled(k, rt.next) && S::apply(all[st], k, sub, t, e, rt) >= 0 && S::in_model(t, all[st], rt) == want_in;
        }
        if (!ok) { if (!nbad) std::fprintf(stderr, "bad cell %08x (in-model list: %d)\n", c, (int)want_in); ++nbad; }
      };
      for (u64 b = 0; b < nblk; ++b) {
        std::vector<u32> cl, co;
        for (int w = 0; w < 4; ++w) {
          const u32 ci = cnts[8 * b + w], coo = cnts[8 * b + 4 + w];
          if (ci > 64u * S::NSLOT || coo > 64u * S::NSLOT) { std::printf("{\"error\": \"cell count out of range\"}\n"); return 4; }
          std::vector<u32> x(ci), y(coo);
          const u64 reg = b * 256 * S::NSLOT + (u64)w * 64 * S::NSLOT;
          if (ci) (void)hipMemcpy(x.data(), dcells + reg, ci * 4, hipMemcpyDeviceToHost);
          if (coo) (void)hipMemcpy(y.data(), dcells_oom + reg, coo * 4, hipMemcpyDeviceToHost);
          cl.insert(cl.end(), x.begin(), x.end());
          co.insert(co.end(), y.begin(), y.end());
        }
        for (u32 c : cl) check(c, true, b);
        for (u32 c : co) check(c, false, b);
        ncells += cl.size(); noom += co.size();
      }
      for (u64 i = 0; i < np; ++i) {
        const u64 st = i / S::NSLOT; const int sl = (int)(i % S::NSLOT);
        int k, sub; S::inst_of_slot(sl, k, sub);
        W t; u32 e = 0;
        if (S::group_enabled(k, rt.next) && S::apply(all[st], k, sub, t, e, rt) >= 0) (S::in_model(t, all[st], rt) ? nwant_in : nwant_oom)++;
      }
      std::printf("{\"cells\": %llu, \"oom_cells\": %llu, \"expected\": [%llu, %llu], \"bad_cells\": %llu}\n", (unsigned long long)ncells,
                  (unsigned long long)noom, (unsigned long long)nwant_in, (unsigned long long)nwant_oom, (unsigned long long)nbad);
      if (nbad || ncells != nwant_in || noom != nwant_oom) {
        std::printf("{\"error\": \"expand produced invalid cells; later kernels not launched\"}\n");
        return 4;
      }
    }
    if (rt.sym_tlc) hipLaunchKernelGGL((memb_fingerprint<S, true>), dim3((unsigned)nblk), dim3(256), 0, 0, g);
    else hipLaunchKernelGGL((memb_fingerprint<S, false>), dim3((unsigned)nblk), dim3(256), 0, 0, g);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("{\"error\": \"fingerprint kernel\"}\n"); return 1; }
    hipLaunchKernelGGL((memb_oom_check<S>), dim3((unsigned)nblk), dim3(256), 0, 0, g);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("{\"error\": \"oom check kernel\"}\n"); return 1; }
    std::vector<u64> cand(np);
    (void)hipMemcpy(cand.data(), dcand, np * 8, hipMemcpyDeviceToHost);
    for (u64 i = 0; i < np; ++i) {
      const u64 st = i / S::NSLOT; const int slot = (int)(i % S::NSLOT);
      int k, sub; S::inst_of_slot(slot, k, sub);
      W t; u32 e = 0; u64 want = 0;
      if (S::group_enabled(k, rt.next) && S::apply(all[st], k, sub, t, e, rt) >= 0 && S::in_model(t, all[st], rt)) want = S::fingerprint(t, seed, rt);
      const u64 got = cand[(u64)slot * n + st];
      if (got != want) {
        if (!gbad) std::fprintf(stderr, "generate mismatch: state %llu slot %d want %016llx got %016llx\n", (unsigned long long)st, slot,
                                (unsigned long long)want, (unsigned long long)got);
        ++gbad;
      }
    }
  }
  std::printf("{\"generate_mismatches\": %llu}\n", (unsigned long long)gbad);
  bad += gbad;
  std::printf("{\"states\": %llu, \"pairs\": %llu, \"mismatches\": %llu}\n", (unsigned long long)n,
              (unsigned long long)np, (unsigned long long)bad);
  if (bad) std::fprintf(stderr, "first mismatch: %s\n", first.c_str());
  return bad ? 3 : 0;
}
