// TEST HARNESS ONLY (never part of the product).  Runs a host-side BFS with the
// product's packed raft_original successor function (raft-tla_amd/csrc/orig_spec.h)
// so its semantics can be checked against the oracle on CPU before a GPU run.
// Shape comes from -DSHAPE_N=.. -DSHAPE_NV=.. -DSHAPE_MT=.. -DSHAPE_ML=.. -DSHAPE_MK=..
//   orig_host_bfs CFG [DUMP|-] [FP_SEED]   -> prints JSON {generated, distinct, depth, actions}
// With FP_SEED the seen-set holds the product's 64-bit fingerprints (fp64 with that seed),
// exactly what the GPU seen-set holds, instead of the full packed states.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../raft-tla_amd/csrc/orig_text.h"

using namespace rmc;
using S = Orig<SHAPE_N, SHAPE_NV, SHAPE_MT, SHAPE_ML, SHAPE_MK>;
using W = S::Work;

struct Key { std::vector<u32> w; bool operator==(const Key& o) const { return w == o.w; } };
struct KH { size_t operator()(const Key& k) const { u32 a[S::NW]; for (int q = 0; q < S::NW; ++q) a[q] = k.w[q]; return (size_t)fp64(a, 1); } };

int main(int argc, char** argv) {
  CfgFile cfg = parse_cfg_text(read_text_file(argv[1]));
  OrigModel m = resolve_orig_model(cfg);
  FILE* dump = argc > 2 && std::string(argv[2]) != "-" ? std::fopen(argv[2], "w") : nullptr;
  const bool by_fp = argc > 3;
  const u64 fp_seed = by_fp ? std::strtoull(argv[3], nullptr, 0) : 0;
  std::unordered_set<Key, KH> seen;
  std::unordered_set<u64> seen_fp;
  std::vector<W> frontier(1);
  S::init(frontier[0]);
  auto key = [](const W& s) { u32 a[S::NW]; S::pack(s, a); Key k; k.w.assign(a, a + S::NW); return k; };
  auto fpk = [&](const W& s) { u32 a[S::NW]; S::pack(s, a); return fp64(a, fp_seed); };
  if (by_fp) seen_fp.insert(fpk(frontier[0])); else seen.insert(key(frontier[0]));
  if (dump) std::fprintf(dump, "%s\n", orig_state_text<S>(m, frontier[0], false).c_str());
  long long generated = 1, gen_act[OA_NACT] = {0}, dist_act[OA_NACT] = {0};
  int depth = 1; u32 err = 0;
  while (!frontier.empty()) {
    std::vector<W> next;
    for (auto& s : frontier) {
      u64 al[S::AW]; S::all_logs_next(s, al);
      // round-trip check of the canonical packing
      { u32 a[S::NW]; S::pack(s, a); W b; S::unpack(a, b); u32 c[S::NW]; S::pack(b, c);
        for (int q = 0; q < S::NW; ++q) if (a[q] != c[q]) { std::printf("{\"error\": \"pack/unpack mismatch\"}\n"); return 1; } }
      for (int k = 0; k < S::NI; ++k) {
        W t; int act = S::apply(s, k, t, err);
        if (act < 0) continue;
        for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
        generated++; gen_act[act]++;
        if (!S::in_model(t, m.rt)) continue;
        if (by_fp ? seen_fp.insert(fpk(t)).second : seen.insert(key(t)).second) {
          dist_act[act]++; next.push_back(t);
          if (dump) std::fprintf(dump, "%s\n", orig_state_text<S>(m, t, false).c_str());
        }
      }
    }
    if (!next.empty()) depth++;
    frontier.swap(next);
  }
  if (dump) std::fclose(dump);
  std::printf("{\"generated\": %lld, \"distinct\": %zu, \"depth\": %d, \"err\": %u, \"actions\": {", generated, by_fp ? seen_fp.size() : seen.size(), depth, err);
  for (int k = 0; k < OA_NACT; ++k) std::printf("%s\"%s\": [%lld, %lld]", k ? ", " : "", kOrigActNames[k], gen_act[k], dist_act[k]);
  std::printf("}}\n");
  return 0;
}
