// TEST HARNESS ONLY (never part of the product).  Seeded random walks over the product's packed
// raft_original successor function (raft-tla_amd/csrc/orig_spec.h) that stop at the first state
// meeting a goal, printing the walk as one canonical state per line — the input of the oracle's
// `check-trace`, which replays it through the literal restatement of raft_original.tla.  Used for
// states the oracle's BFS cannot reach in a test's time: goal 1 asks for an election record and a
// log entry with the second value, goal 2 also for a non-empty log in the record's evoterLog —
// the compact election records of 5 servers with 2 values (orig_spec.h ECOMPACT) at work.
// Every step also checks that pack/unpack is the identity on the state.
// Shape: -DSHAPE_N=.. -DSHAPE_NV=.. -DSHAPE_MT=.. -DSHAPE_ML=.. -DSHAPE_MK=..
//   orig_walk CFG SEED [MAX_WALKS] [GOAL] -> the walk on stdout (one state per line), or exit 2
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../raft-tla_amd/csrc/orig_text.h"

using namespace rmc;
using S = Orig<SHAPE_N, SHAPE_NV, SHAPE_MT, SHAPE_ML, SHAPE_MK>;
using W = S::Work;

static int g_goal = 1;   // 1: an election record and a second-value entry; 2: also a non-empty voterLog cell
static bool goal(const W& t) {
  bool rec = false, any = false, v2 = false;
  for (int k = 0; k < S::EMAX; ++k) {
    if (t.el[k] == S::EMPTY) continue;
    const u64 e = t.el[k];
    any = true;
    const u32 ev = (u32)((e >> (S::ETB + S::SB + S::LIB)) & lomask(S::N));
    const u64 row = S::evoter_row(e >> (S::ETB + S::SB + S::LIB + S::N), ev);
    for (int j = 0; j < S::N; ++j)
      if (((row >> (j * S::VLB)) & 1ull) && ((row >> (j * S::VLB + 1)) & lomask(S::LIB)) != 0) rec = true;
  }
  for (int i = 0; i < S::N; ++i) {
    const u32 li = t.log.v[i];
    for (int p = 0; p < S::llen(li); ++p) v2 |= S::NV > 1 && S::evalue(S::lent(li, p)) == 1;
  }
  return g_goal == 0 ? any : (g_goal == 2 ? rec : any) && v2;
}

int main(int argc, char** argv) {
  CfgFile cfg = parse_cfg_text(read_text_file(argv[1]));
  OrigModel m = resolve_orig_model(cfg);
  std::mt19937_64 rng(std::strtoull(argv[2], nullptr, 0));
  const long long walks = argc > 3 ? std::atoll(argv[3]) : 2000000;
  if (argc > 4) g_goal = std::atoi(argv[4]);
  for (long long w = 0; w < walks; ++w) {
    std::vector<W> path(1);
    S::init(path[0]);
    for (int step = 0; step < 48; ++step) {
      const W& s = path.back();
      std::vector<std::pair<double, W>> succ;
      double tot = 0;
      for (int k = 0; k < S::NI; ++k) {
        W t; u32 err = 0;
        const int act = S::apply(s, k, t, err);
        if (act < 0 || err) continue;
        S::all_logs_next(s, t.allLogs);
        if (!S::in_model(t, m.rt)) continue;
        // restarts, drops and duplicates rarely help reach an election
        const double wgt = act == OA_Restart ? 0.02 : (act == OA_DropMessage || act == OA_DuplicateMessage) ? 0.05 : 1.0;
        succ.push_back({wgt, t});
        tot += wgt;
      }
      if (succ.empty()) break;
      double x = std::uniform_real_distribution<double>(0, tot)(rng);
      size_t pick = 0;
      while (pick + 1 < succ.size() && x >= succ[pick].first) { x -= succ[pick].first; ++pick; }
      const W& t = succ[pick].second;
      u32 a[S::NW], b[S::NW]; W r;
      S::pack(t, a); S::unpack(a, r); S::pack(r, b);
      for (int q = 0; q < S::NW; ++q) if (a[q] != b[q]) { std::fprintf(stderr, "pack/unpack mismatch\n"); return 3; }
      path.push_back(r);
      if (goal(r)) {
        for (const W& st : path) std::printf("%s\n", orig_state_text<S>(m, st, false).c_str());
        std::fprintf(stderr, "walk %lld, %zu states\n", w, path.size());
        return 0;
      }
    }
  }
  return 2;
}
