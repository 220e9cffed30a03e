// ============================================================================
// TEST INFRASTRUCTURE ONLY (see oracle/tla.h header).
// raft_oracle — CLI over the oracle restatements.
//
//   raft_oracle bfs    --tla F.tla --cfg F.cfg [--max-depth D] [--max-states N]
//                      [--dump states.txt] [--sym tlc|view] [--no-inv-oom]
//                      [--deadlock] [--golden-cwcl F] [--golden-morc F] [--trace]
//                      [--workers T] [--lean [--progress]]   (lean: engine.h bfs_lean, no trace)
//   raft_oracle replay --tla F.tla --cfg F.cfg --golden F [--max-steps N]
//   raft_oracle check-trace --tla F.tla --cfg F.cfg --golden TRACE.txt   (one state per line)
//
// Output: one JSON object on stdout.
// ============================================================================
#include <iostream>

#include "raft_apalache.h"
#include "raft_dricketts.h"
#include "raft_membership.h"
#include "raft_original.h"
#include "tla_parse.h"

using namespace oracle;

static std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += c; }
    else if (c == '\n') o += "\\n";
    else if ((unsigned char)c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
    else o += c;
  }
  return o + "\"";
}

// Spec family from the module text: the reference files themselves, or an MC
// wrapper carrying a `raftmc-base:` pragma (configs/*.tla).
static std::string detect_spec(const std::string& text) {
  if (text.find("raftmc-base: thirdparty/raft_original.tla") != std::string::npos) return "original";
  if (text.find("raftmc-base: tlc_membership/raft.tla") != std::string::npos) return "membership";
  if (text.find("raftmc-base: thirdparty/raft_dricketts.tla") != std::string::npos) return "ricketts";
  if (text.find("raftmc-base: apalache_no_membership/raft.tla") != std::string::npos) return "apalache";
  if (text.find("WrapMsg(m) ==") != std::string::npos && text.find("hadAtLeastOneLeader") != std::string::npos) return "apalache";
  if (text.find("VARIABLE elections") != std::string::npos && text.find("VARIABLE allLogs") != std::string::npos) return "original";
  if (text.find("NextAsyncCrash") != std::string::npos) return "membership";
  throw EvalError("unrecognised spec module");
}

static std::vector<V> load_golden_global(const std::string& path) {
  V g = parse_value(read_file(path));
  if (g->k == K::Seq) return g->a;
  return ap(g, "global")->a;
}

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: raft_oracle bfs|replay ...\n"); return 2; }
  std::string mode = argv[1], tla, cfgp, dump, golden, gc, gm;
  Options o; bool want_trace = false; int64_t max_steps = 64;
  for (int a = 2; a < argc; ++a) {
    std::string k = argv[a];
    auto nxt = [&]() -> std::string { if (a + 1 >= argc) throw EvalError("missing value for " + k); return argv[++a]; };
    if (k == "--tla") tla = nxt();
    else if (k == "--cfg") cfgp = nxt();
    else if (k == "--max-depth") o.max_depth = std::stoll(nxt());
    else if (k == "--max-states") o.max_states = std::stoll(nxt());
    else if (k == "--workers") o.workers = std::max(1, std::stoi(nxt()));
    else if (k == "--dump") o.dump_states = nxt();
    else if (k == "--sym") o.sym_mode = nxt();
    else if (k == "--no-inv-oom") o.inv_out_of_model = false;
    else if (k == "--no-disjunct-copies") o.disjunct_copies = false;
    else if (k == "--deadlock") o.check_deadlock = true;
    else if (k == "--golden") golden = nxt();
    else if (k == "--golden-cwcl") gc = nxt();
    else if (k == "--golden-morc") gm = nxt();
    else if (k == "--trace") want_trace = true;
    else if (k == "--lean") o.lean = true;
    else if (k == "--progress") o.progress = true;
    else if (k == "--max-steps") max_steps = std::stoll(nxt());
    else { std::fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
  }
  try {
    std::string family = detect_spec(read_file(tla));
    Cfg cfg = parse_cfg(read_file(cfgp));
    std::unique_ptr<Spec> sp;
    if (family == "original") sp.reset(new RaftOriginal(cfg));
    else if (family == "ricketts") sp.reset(new RaftRicketts(cfg));
    else if (family == "apalache") sp.reset(new RaftApalache(cfg));
    else {
      auto* m = new RaftMembership(cfg);
      m->disjunct_copies = o.disjunct_copies;
      if (!gc.empty()) m->golden_cwcl = load_golden_global(gc);
      if (!gm.empty()) m->golden_morc = load_golden_global(gm);
      sp.reset(m);
    }
    if (mode == "bfs") {
      Result r = o.lean ? bfs_lean(*sp, cfg, o) : bfs(*sp, cfg, o);
      auto an = sp->action_names();
      std::string js = "{";
      js += "\"spec\": " + json_str(family) + ", \"verdict\": " + json_str(r.verdict);
      js += ", \"violated\": " + json_str(r.violated) + ", \"error\": " + json_str(r.error);
      js += ", \"generated\": " + std::to_string(r.generated) + ", \"distinct\": " + std::to_string(r.distinct);
      js += ", \"left_on_queue\": " + std::to_string(r.left_on_queue) + ", \"depth\": " + std::to_string(r.depth);
      js += ", \"seconds\": " + std::to_string(r.seconds);
      js += ", \"levels\": [";
      for (size_t q = 0; q < r.level_sizes.size(); ++q) js += (q ? ", " : "") + std::to_string(r.level_sizes[q]);
      js += "], \"actions\": {";
      for (size_t q = 0; q < an.size(); ++q)
        js += (q ? ", " : "") + json_str(an[q]) + ": [" + std::to_string(r.act_generated[q]) + ", " + std::to_string(r.act_distinct[q]) + "]";
      js += "}, \"trace_len\": " + std::to_string(r.trace.size());
      if (want_trace) {
        js += ", \"trace\": [";
        for (size_t q = 0; q < r.trace.size(); ++q)
          js += (q ? ", " : "") + std::string("{\"action\": ") + json_str(r.trace[q].first < 0 ? "Init" : an[r.trace[q].first]) +
                ", \"state\": " + json_str(sp->dump_line(r.trace[q].second)) + "}";
        js += "]";
      }
      js += "}";
      std::cout << js << std::endl;
      return 0;
    }
    if (mode == "replay") {
      // Guided search for a behaviour whose history["global"] equals the
      // golden TLC trace (raft.tla:1201 / :1231), the golden's s1,s2,s3 bound
      // to distinct servers (the \E s1, s2, s3 \in Server of the constraint).
      auto* mem = dynamic_cast<RaftMembership*>(sp.get());
      if (!mem) throw EvalError("replay needs the membership spec");
      V gold = parse_value(read_file(golden));
      std::vector<V> gg = ap(gold, "global")->a;
      auto& S = mem->Server->a;
      int id1 = Names::get().intern_mv("s1"), id2 = Names::get().intern_mv("s2"), id3 = Names::get().intern_mv("s3");
      int64_t best = -1; std::string best_state, best_actions; int nbind = 0;
      for (size_t a = 0; a < S.size(); ++a) for (size_t b = 0; b < S.size(); ++b) for (size_t c = 0; c < S.size(); ++c) {
        if (a == b || b == c || a == c) continue;
        std::vector<int> perm(Names::get().mv.size() + 8, -1);
        perm[id1] = (int)S[a]->i; perm[id2] = (int)S[b]->i; perm[id3] = (int)S[c]->i;
        std::vector<V> want; for (auto& x : gg) want.push_back(permute(x, perm));
        auto ok_prefix = [&](const State& s) {
          V g = ap(s[RaftMembership::history], "global");
          if (g->a.size() > want.size()) return false;
          for (size_t q = 0; q < g->a.size(); ++q) if (!eq(g->a[q], want[q])) return false;
          return true;
        };
        std::vector<State> frontier = sp->init();
        std::vector<std::vector<int>> acts(1);
        std::unordered_set<std::string> seen;
        std::vector<Succ> succ;
        for (int64_t step = 0; step <= max_steps && !frontier.empty(); ++step) {
          bool done = false;
          for (size_t q = 0; q < frontier.size(); ++q) {
            if (ap(frontier[q][RaftMembership::history], "global")->a.size() == want.size()) {
              if (best < 0 || step < best) {
                best = step; best_state = state_text(*sp, frontier[q]);
                best_actions.clear();
                for (int x : acts[q]) best_actions += (best_actions.empty() ? "" : ",") + sp->action_names()[x];
              }
              nbind++; done = true; break;
            }
          }
          if (done) break;
          std::vector<State> nf; std::vector<std::vector<int>> na;
          for (size_t q = 0; q < frontier.size(); ++q) {
            succ.clear(); sp->next(frontier[q], succ);
            for (auto& su : succ) {
              bool im = true; for (auto& cn : cfg.constraints) if (!sp->constraint(cn, su.s)) { im = false; break; }
              if (!im || !ok_prefix(su.s)) continue;
              std::string k = state_text(*sp, su.s);
              if (!seen.insert(k).second) continue;
              nf.push_back(su.s); auto av = acts[q]; av.push_back(su.action); na.push_back(av);
            }
          }
          frontier.swap(nf); acts.swap(na);
        }
      }
      std::string js = "{\"found\": " + std::string(best >= 0 ? "true" : "false") + ", \"transitions\": " + std::to_string(best) +
                       ", \"bindings_matched\": " + std::to_string(nbind) + ", \"golden_len\": " + std::to_string(gg.size()) +
                       ", \"actions\": " + json_str(best_actions) + ", \"state\": " + json_str(best_state) + "}";
      std::cout << js << std::endl;
      return 0;
    }
    if (mode == "check-trace") {
      // Independent validation of a counterexample found elsewhere (e.g. by the GPU at a
      // depth the oracle's BFS cannot reach): the trace file holds one state per line in
      // dump_line text.  Line 1 must be an initial state; every next line must be the text
      // of an in-model successor (oracle Next, constraints, action constraints) of the
      // current state; no earlier state may violate an invariant; the last must.
      std::ifstream f(golden);
      if (!f) throw EvalError("cannot open trace file " + golden);
      std::vector<std::string> lines;
      for (std::string l; std::getline(f, l);) if (!l.empty()) lines.push_back(l);
      // an invariant whose evaluation raises a TLC evaluation error (e.g. Committed(i) out of range,
      // tlc_membership/raft.tla:969) counts as the trace's stop: TLC reports the error on that state
      std::string eval_error;
      auto check_inv = [&](const State& st) -> std::string {
        for (auto& inv : cfg.invariants) {
          try {
            if (!sp->invariant(inv, st)) return inv;
          } catch (const EvalError& e) {
            eval_error = e.what();
            return inv;
          }
        }
        return "";
      };
      auto in_model = [&](const State& a, const State& b) {
        for (auto& c : cfg.constraints) if (!sp->constraint(c, b)) return false;
        for (auto& c : cfg.action_constraints) if (!sp->action_constraint(c, a, b)) return false;
        return true;
      };
      int64_t bad_step = -1; std::string violated, actions;
      State cur;
      bool ok = false;
      for (auto& s0 : sp->init()) if (sp->dump_line(s0) == lines.at(0)) { cur = s0; ok = true; break; }
      if (!ok) bad_step = 0;
      std::vector<Succ> succ;
      for (size_t k = 1; ok && k < lines.size(); ++k) {
        std::string early = check_inv(cur);
        if (!early.empty()) { ok = false; bad_step = (int64_t)k - 1; violated = early; break; }
        succ.clear(); sp->next(cur, succ);
        bool found = false;
        for (auto& su : succ)
          if (sp->dump_line(su.s) == lines[k] && in_model(cur, su.s)) {
            cur = su.s; found = true; actions += (actions.empty() ? "" : ",") + sp->action_names()[su.action]; break;
          }
        if (!found) { ok = false; bad_step = (int64_t)k; }
      }
      if (ok) violated = check_inv(cur);
      if (ok && violated.empty()) {   // or: computing the last state's successors raises the error
        try { succ.clear(); sp->next(cur, succ); }
        catch (const EvalError& e) { eval_error = e.what(); violated = "<next-state relation>"; }
      }
      std::cout << "{\"valid\": " << ((ok && !violated.empty()) ? "true" : "false") << ", \"length\": " << lines.size()
                << ", \"violated\": " << json_str(violated) << ", \"eval_error\": " << json_str(eval_error)
                << ", \"bad_step\": " << bad_step
                << ", \"actions\": " << json_str(actions) << "}" << std::endl;
      return 0;
    }
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  } catch (const std::exception& e) {
    std::cout << "{\"verdict\": \"ERROR\", \"error\": " << json_str(e.what()) << "}" << std::endl;
    return 1;
  }
}
