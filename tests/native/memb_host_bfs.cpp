// TEST HARNESS ONLY (never part of the product).  Runs a single-worker FIFO BFS
// on the host with the product's packed tlc_membership successor function,
// constraints, invariants and symmetric fingerprint (raft-tla_amd/csrc/
// memb_spec.h, the same header the gfx950 kernels compile), so its semantics
// can be checked against the oracle on CPU before a GPU run.
// Shape: -DSHAPE_N=.. -DSHAPE_NV=..
//   memb_host_bfs CFG MAX_DEPTH [DUMP|-] [--prefix CONSTRAINT TRACE_FILE]...
//     -> JSON {generated, distinct, depth, left_on_queue, verdict, actions}
// SYM_TLC=1 (environment): TLC-mode symmetry (the oracle's --sym tlc), as MC_COMPAT_SYM_TLC.
// SYMCHECK=1 (environment): for every distinct state of the search (run it on a cfg WITHOUT
// SYMMETRY, so symmetric copies are all kept), compare the product's refined symmetric fingerprint
// (S::fingerprint with symmetry on: min over the signature-respecting permutations only) with the
// brute-force one (min over all N! permuted views): the two must induce the same partition of the
// states into orbits ("symcheck": [states, refined classes, brute classes, disagreements]).
#include <cstdio>
#include <string>
#include <cstdlib>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../raft-tla_amd/csrc/memb_prefix.h"
#include "../../raft-tla_amd/csrc/memb_text.h"

#ifdef RMC_FP_STATS   // work counts of the TLC-mode canonical-permutation search (memb_spec.h RMC_FPS), on stderr
long long rmc_fp_stats[32];
#endif
using namespace rmc;
using S = Memb<SHAPE_N, SHAPE_NV, 2 * SHAPE_N * SHAPE_N>;
using W = S::Work;

int main(int argc, char** argv) {
  CfgFile cfg = parse_cfg_text(read_text_file(argv[1]));
  MembModel m = resolve_memb_model(cfg);
  const long long max_depth = argc > 2 ? std::atoll(argv[2]) : 0;
  FILE* dump = argc > 3 && std::string(argv[3]) != "-" ? std::fopen(argv[3], "w") : nullptr;
  MembText<S> text(m);
  MembRuntime rt = m.rt;
  if (std::getenv("SYM_TLC") && rt.symmetry) rt.sym_tlc = 1;   // MC_COMPAT_SYM_TLC
  // punctuated-search prefixes, laid out as the GPU backend does (memb_backend.hip prepare_prefixes)
  std::vector<u64> tabs[2];
  u32 off = S::H_PREFIX;
  for (int a = 4; a + 2 < argc; a += 3) {
    const std::string con = argv[a + 1];
    const int r = con == kMembConNames[kPrefixCon[0]] ? 0 : 1;
    tabs[r] = encode_prefix_table<S>(m, trace_global(parse_tla_value(read_text_file(argv[a + 2]))));
    const u32 len = (u32)(tabs[r].size() / 2 / (S::NB ? S::NB : 1));
    if (r == 0) { rt.ptab0 = tabs[0].data(); rt.plen0 = len; }
    else { rt.ptab1 = tabs[1].data(); rt.plen1 = len; }
  }
  for (int r = 0; r < 2; ++r)
    if ((rt.constraints >> kPrefixCon[r]) & 1u) { if (r == 1) rt.preg1_off = off; off += S::NB; }
  const u64 seed = 0x5EED5EED2024ull;
  std::unordered_set<u64> seen;
  std::vector<W> frontier(1);
  std::vector<W> all;   // SYMCHECK: every distinct state
  const bool keep_all = std::getenv("SYMCHECK") != nullptr;
  S::init(frontier[0]);
  if (keep_all) all.push_back(frontier[0]);
  seen.insert(S::fingerprint(frontier[0], seed, rt));
  if (dump) std::fprintf(dump, "%s\n", text.text(frontier[0], false).c_str());
  long long generated = 1, gen_act[MA_NACT] = {0}, dist_act[MA_NACT] = {0}, left = 0;
  int depth = 1;
  u32 err = 0;
  std::string verdict = "OK", violated;
  while (!frontier.empty()) {
    if (max_depth && depth >= max_depth) { left = (long long)frontier.size(); break; }
    std::vector<W> next;
    for (size_t fi = 0; fi < frontier.size() && verdict == "OK"; ++fi) {
      const W& s = frontier[fi];
      { u32 a[S::NW]; S::pack(s, a); W b; S::unpack(a, b); u32 c[S::NW]; S::pack(b, c);
        for (int q = 0; q < S::NW; ++q) if (a[q] != c[q]) { std::printf("{\"error\": \"pack/unpack mismatch\"}\n"); return 1; } }
      // TLC (oracle) counts a state's whole successor list before checking any of them
      for (int k = 0; k < S::NI; ++k) {
        if (!S::group_enabled(k, rt.next)) continue;
        for (int sub = 0; sub < S::nsub(k); ++sub) { W t; if (S::apply(s, k, sub, t, err, rt) >= 0) generated += S::tlc_copies(s, k, sub, rt); }
      }
      for (int k = 0; k < S::NI && verdict == "OK"; ++k) {
        if (!S::group_enabled(k, rt.next)) continue;
        for (int sub = 0; sub < S::nsub(k); ++sub) {
          W t;
          const int act = S::apply(s, k, sub, t, err, rt);
          if (act < 0) continue;
          gen_act[act]++;
          const bool im = S::in_model(t, s, rt);
          bool isnew = false;
          if (im) {
            isnew = seen.insert(S::fingerprint(t, seed, rt)).second;
            if (isnew) {
              dist_act[act]++; next.push_back(t);
              if (keep_all) all.push_back(t);
              if (dump) std::fprintf(dump, "%s\n", text.text(t, false).c_str());
            }
          }
          if (isnew || !im) {
            const u32 r = S::check_invariants(t, rt);
            if (r) {
              verdict = (r >> 8) == IV_BAD ? "INVARIANT_VIOLATION" : "EVAL_ERROR";
              violated = kMembInvNames[r & 255];
              left = (long long)(frontier.size() - fi - 1 + next.size());
              depth++;
              break;
            }
          }
          gen_act[act] += S::tlc_copies(s, k, sub, rt) - 1;   // TLC's copies of it (they follow it in the list)
        }
      }
    }
    if (verdict != "OK") break;
    if (!next.empty()) depth++;
    frontier.swap(next);
  }
  if (dump) std::fclose(dump);
  if (std::getenv("SYMCHECK")) {
    MembRuntime rs = rt; rs.symmetry = 1;
    std::unordered_map<u64, u64> r2b, b2r;
    long long bad = 0;
    for (const W& t : all) {
      const u64 fr = S::fingerprint(t, seed, rs);
      const bool ce = S::has_config_entries(t, rs.cfg_type);
      u64 best = ~0ull;
      for (int p = 0; p < S::NPERM; ++p) {
        const u64 h = ce ? S::template view_hash1<true>(t, S::perm_of(p), seed, rs.cfg_type)
                         : S::template view_hash1<false>(t, S::perm_of(p), seed, rs.cfg_type);
        best = h < best ? h : best;
      }
      const u64 fb0 = S::fmix(best ^ seed), fb = fb0 ? fb0 : 1ull;
      auto a = r2b.emplace(fr, fb), b = b2r.emplace(fb, fr);
      bad += (a.first->second != fb) + (b.first->second != fr);
    }
    std::printf("{\"symcheck\": [%zu, %zu, %zu, %lld]}\n", all.size(), r2b.size(), b2r.size(), bad);
    return 0;
  }
  std::printf("{\"generated\": %lld, \"distinct\": %zu, \"depth\": %d, \"left_on_queue\": %lld, \"err\": %u, \"verdict\": \"%s\", "
              "\"violated\": \"%s\", \"actions\": {",
              generated, seen.size(), depth, left, err, verdict.c_str(), violated.c_str());
  for (int k = 0; k < MA_NACT; ++k) std::printf("%s\"%s\": [%lld, %lld]", k ? ", " : "", kMembActNames[k], gen_act[k], dist_act[k]);
  std::printf("}}\n");
#ifdef RMC_FP_STATS
  std::fprintf(stderr, "fp_stats");
  for (int i = 0; i < 32; ++i) std::fprintf(stderr, " %d:%lld", i, rmc_fp_stats[i]);
  std::fprintf(stderr, "\n");
#endif
  return 0;
}
