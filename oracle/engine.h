// ============================================================================
// TEST INFRASTRUCTURE ONLY (see oracle/tla.h header).
//
// engine.h — the oracle's restatement of TLC's breadth-first search contract
// and of the TLC .cfg format.  TLC (tla2tools.jar) is not vendored in the
// reference and cannot run here, so every TLC-side choice is
// an explicit, named switch (SURVEY.md §7 build plan item 1, [ext] items):
//   inv_out_of_model   (ii)  check invariants on !seen successors that fail a
//                            state constraint (TLC ModelChecker.doNext) [ext]
//   generated counts   (iii) every successor, duplicates and out-of-model
//                            ones included, plus the initial states  [ext]
//   symmetry mode      (iv)  "tlc": min over perms of the FULL variable tuple,
//                            then VIEW; "view": min over perms of the VIEW
//   FIFO order         (v)   single worker, level order, TLC action order
// ============================================================================
#pragma once
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <chrono>
#include <thread>
#include <fstream>
#include <sstream>
#include <unordered_map>
#include <unordered_set>

#include "tla.h"

namespace oracle {
using namespace tla;

using State = std::vector<V>;

struct Succ {
  State s;
  int action;          // index into Spec::action_names()
};

// ----------------------------------------------------------------- cfg model
struct Cfg {
  std::vector<std::pair<std::string, V>> constants;
  std::vector<std::pair<std::string, std::string>> overrides;  // name <- op
  std::string init = "Init", next = "Next", symmetry, view;
  std::vector<std::string> constraints, action_constraints, invariants, properties;
  V get(const std::string& n) const {
    for (auto& c : constants) if (c.first == n) return c.second;
    throw EvalError("constant not assigned in cfg: " + n);
  }
  bool has(const std::string& n) const {
    for (auto& c : constants) if (c.first == n) return true;
    return false;
  }
};

// Tokeniser for the TLC cfg language subset used by the reference's raft.cfg
// (tlc_membership/raft.cfg:1-87): comments \* and (* *), CONSTANT(S) with
// `=` and `<-`, SYMMETRY, VIEW, INIT, NEXT, CONSTRAINT(S),
// ACTION_CONSTRAINT(S), INVARIANT(S), PROPERTY/PROPERTIES.
inline std::vector<std::string> cfg_tokens(const std::string& text) {
  std::vector<std::string> toks; size_t i = 0, n = text.size();
  while (i < n) {
    char c = text[i];
    if (isspace((unsigned char)c)) { ++i; continue; }
    if (c == '\\' && i + 1 < n && text[i + 1] == '*') { while (i < n && text[i] != '\n') ++i; continue; }
    if (c == '(' && i + 1 < n && text[i + 1] == '*') {
      int depth = 1; i += 2;
      while (i < n && depth) {
        if (text[i] == '(' && i + 1 < n && text[i + 1] == '*') { depth++; i += 2; }
        else if (text[i] == '*' && i + 1 < n && text[i + 1] == ')') { depth--; i += 2; }
        else ++i;
      }
      continue;
    }
    if (c == '"') { size_t j = i + 1; while (j < n && text[j] != '"') ++j; toks.push_back(text.substr(i, j - i + 1)); i = j + 1; continue; }
    if (c == '<' && i + 1 < n && text[i + 1] == '-') { toks.push_back("<-"); i += 2; continue; }
    if (c == '{' || c == '}' || c == ',' || c == '=' || c == '-') { toks.push_back(std::string(1, c)); ++i; continue; }
    size_t j = i;
    while (j < n && (isalnum((unsigned char)text[j]) || text[j] == '_' || text[j] == '!' || text[j] == '@')) ++j;
    if (j == i) throw EvalError(std::string("cfg: unexpected character '") + c + "'");
    toks.push_back(text.substr(i, j - i)); i = j;
  }
  return toks;
}

inline bool is_cfg_keyword(const std::string& t) {
  static const char* kw[] = {"CONSTANT", "CONSTANTS", "SYMMETRY", "VIEW", "INIT", "NEXT", "SPECIFICATION",
                             "CONSTRAINT", "CONSTRAINTS", "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS",
                             "INVARIANT", "INVARIANTS", "PROPERTY", "PROPERTIES", "CHECK_DEADLOCK", "ALIAS", "POSTCONDITION"};
  for (auto k : kw) if (t == k) return true;
  return false;
}

inline V cfg_value(const std::vector<std::string>& tk, size_t& p) {
  if (p >= tk.size()) throw EvalError("cfg: value expected");
  const std::string& t = tk[p];
  if (t == "{") {
    ++p; std::vector<V> xs;
    while (p < tk.size() && tk[p] != "}") { xs.push_back(cfg_value(tk, p)); if (tk[p] == ",") ++p; }
    ++p; return set(xs);
  }
  if (t == "-") { ++p; return Int(-std::stoll(tk[p++])); }
  if (t[0] == '"') { ++p; return Str(t.substr(1, t.size() - 2)); }
  if (isdigit((unsigned char)t[0])) { ++p; return Int(std::stoll(t)); }
  if (t == "TRUE") { ++p; return Bool(true); }
  if (t == "FALSE") { ++p; return Bool(false); }
  ++p; return MV(t);   // identifiers on the right-hand side are TLC model values
}

inline Cfg parse_cfg(const std::string& text) {
  Cfg c; auto tk = cfg_tokens(text); size_t p = 0; std::string sec;
  while (p < tk.size()) {
    const std::string& t = tk[p];
    if (is_cfg_keyword(t)) { sec = t; ++p; continue; }
    if (sec == "CONSTANT" || sec == "CONSTANTS") {
      std::string name = tk[p++];
      if (p < tk.size() && tk[p] == "=") { ++p; V v = cfg_value(tk, p); c.constants.push_back({name, v}); }
      else if (p < tk.size() && tk[p] == "<-") { ++p; c.overrides.push_back({name, tk[p++]}); }
      else c.constants.push_back({name, MV(name)});
    } else if (sec == "SYMMETRY") { c.symmetry = tk[p++]; }
    else if (sec == "VIEW") { c.view = tk[p++]; }
    else if (sec == "INIT") { c.init = tk[p++]; }
    else if (sec == "NEXT") { c.next = tk[p++]; }
    else if (sec == "CONSTRAINT" || sec == "CONSTRAINTS") { c.constraints.push_back(tk[p++]); }
    else if (sec == "ACTION_CONSTRAINT" || sec == "ACTION_CONSTRAINTS") { c.action_constraints.push_back(tk[p++]); }
    else if (sec == "INVARIANT" || sec == "INVARIANTS") { c.invariants.push_back(tk[p++]); }
    else if (sec == "PROPERTY" || sec == "PROPERTIES") { c.properties.push_back(tk[p++]); }
    else throw EvalError("cfg: token outside any section: " + t);
  }
  return c;
}

inline std::string read_file(const std::string& path) {
  std::ifstream f(path); if (!f) throw EvalError("cannot open " + path);
  std::stringstream ss; ss << f.rdbuf(); return ss.str();
}

// ----------------------------------------------------------------- spec interface
struct Spec {
  virtual ~Spec() {}
  virtual const std::vector<std::string>& var_names() const = 0;
  virtual std::vector<std::string> action_names() const = 0;
  virtual std::vector<State> init() const = 0;
  virtual void next(const State& s, std::vector<Succ>& out) const = 0;
  virtual bool constraint(const std::string& name, const State& s) const = 0;
  virtual bool action_constraint(const std::string& name, const State& s, const State& t) const {
    (void)s; (void)t; throw EvalError("unknown action constraint " + name);
  }
  virtual bool invariant(const std::string& name, const State& s) const = 0;
  // VIEW: which variables participate (empty => all)
  virtual std::vector<int> view_vars(const std::string& view) const { (void)view; return {}; }
  // SYMMETRY: permutations of model values (each a full mv-id map), empty => none
  virtual std::vector<std::vector<int>> symmetry_perms(const std::string& sym) const { (void)sym; return {}; }
  // the text written by --dump and in traces (default: every variable, see state_text)
  virtual std::string dump_line(const State& s) const;
};

// ----------------------------------------------------------------- BFS
struct Options {
  bool inv_out_of_model = true;     // [ext] switch (ii)
  std::string sym_mode = "tlc";     // [ext] switch (iv): "tlc" | "view"
  bool disjunct_copies = true;      // [ext] switch (vi): a successor is generated once per true disjunct
                                    // of a disjunctive guard inside an action (TLC's getNextStates;
                                    // tlc_membership/raft.tla:783-789, :796); false: once
  int64_t max_depth = 0;            // 0 = unbounded; depth counts init as 1
  int64_t max_states = 0;           // stop after this many distinct (sample mode)
  bool check_deadlock = false;
  std::string dump_states;          // write canonical text of every distinct state
  bool lean = false;                // bfs_lean: 128-bit key hashes, only two levels of states kept
  bool progress = false;            // bfs_lean: a progress line per parent block on stderr
  int workers = 1;                  // >1: successors, constraints, keys and invariants of a batch
                                    // of parents are computed by this many threads, merged in
                                    // frontier order (results identical to workers = 1)
};

struct Result {
  int64_t generated = 0, distinct = 0, left_on_queue = 0, depth = 0;
  std::vector<int64_t> act_generated, act_distinct;
  std::vector<int64_t> level_sizes;
  std::string verdict = "OK";        // OK | INVARIANT_VIOLATION | EVAL_ERROR | DEADLOCK | SAMPLE_LIMIT
  std::string violated, error;
  std::vector<std::pair<int, State>> trace;   // (action that produced it, state); first = init (action -1)
  double seconds = 0;
};

struct Node { int64_t parent; int action; int32_t depth; };

inline std::string state_text(const Spec& sp, const State& s) {
  std::string t = "/\\ ";
  const auto& vn = sp.var_names();
  for (size_t q = 0; q < s.size(); ++q) { if (q) t += " /\\ "; t += vn[q] + " = " + show(s[q]); }
  return t;
}
inline std::string Spec::dump_line(const State& s) const { return state_text(*this, s); }

// Canonical key of a state under SYMMETRY/VIEW (the text replaces TLC's FP64).
inline std::string canon_key(const Spec& sp, const Cfg& cfg, const Options& o, const State& s,
                             const std::vector<std::vector<int>>& perms, const std::vector<int>& vv) {
  auto view_of = [&](const State& x) {
    std::string k;
    if (vv.empty()) { for (auto& v : x) { k += show(v); k += '\x1f'; } }
    else for (int q : vv) { k += show(x[q]); k += '\x1f'; }
    return k;
  };
  (void)cfg;
  if (perms.empty()) return view_of(s);
  if (o.sym_mode == "view") {
    std::string best;
    for (size_t p = 0; p < perms.size(); ++p) {
      State y; for (auto& v : s) y.push_back(permute(v, perms[p]));
      std::string k = view_of(y);
      if (p == 0 || k < best) best = k;
    }
    return best;
  }
  // "tlc": choose the permutation minimising the full variable tuple (in
  // declaration order, lexicographic on values), then apply VIEW  [ext]
  State best;
  for (size_t p = 0; p < perms.size(); ++p) {
    State y; for (auto& v : s) y.push_back(permute(v, perms[p]));
    if (p == 0) { best = y; continue; }
    int c = 0;
    for (size_t q = 0; q < y.size() && !c; ++q) c = cmp(y[q], best[q]);
    if (c < 0) best = y;
  }
  return view_of(best);
}

inline Result bfs(const Spec& sp, const Cfg& cfg, const Options& o) {
  auto t0 = std::chrono::steady_clock::now();
  Result r;
  auto an = sp.action_names();
  r.act_generated.assign(an.size(), 0); r.act_distinct.assign(an.size(), 0);
  auto perms = cfg.symmetry.empty() ? std::vector<std::vector<int>>{} : sp.symmetry_perms(cfg.symmetry);
  auto vv = cfg.view.empty() ? std::vector<int>{} : sp.view_vars(cfg.view);

  std::unordered_set<std::string> seen;
  std::vector<State> store; std::vector<Node> nodes;
  std::FILE* dump = o.dump_states.empty() ? nullptr : std::fopen(o.dump_states.c_str(), "w");

  auto in_model = [&](const State& s) {
    for (auto& c : cfg.constraints) if (!sp.constraint(c, s)) return false;
    return true;
  };
  auto in_actions = [&](const State& s, const State& t) {
    for (auto& c : cfg.action_constraints) if (!sp.action_constraint(c, s, t)) return false;
    return true;
  };
  auto check_inv = [&](const State& s) -> std::string {
    for (auto& inv : cfg.invariants) if (!sp.invariant(inv, s)) return inv;
    return "";
  };
  auto build_trace = [&](int64_t idx, int last_action, const State* last) {
    std::vector<std::pair<int, State>> tr;
    if (last) tr.push_back({last_action, *last});
    while (idx >= 0) { tr.push_back({nodes[idx].action, store[idx]}); idx = nodes[idx].parent; }
    std::reverse(tr.begin(), tr.end());
    r.trace = tr;
  };

  try {
    // ---- initial states (TLC: generated counts them; constraint + invariants checked)
    std::vector<int64_t> frontier;
    for (auto& s : sp.init()) {
      r.generated++;
      bool im = in_model(s);
      bool isnew = false;
      if (im) {
        auto k = canon_key(sp, cfg, o, s, perms, vv);
        isnew = seen.insert(k).second;
        if (isnew) {
          store.push_back(s); nodes.push_back({-1, -1, 1});
          frontier.push_back((int64_t)store.size() - 1);
          if (dump) std::fprintf(dump, "%s\n", sp.dump_line(s).c_str());
        }
      }
      if (isnew || (!im && o.inv_out_of_model)) {
        auto bad = check_inv(s);
        if (!bad.empty()) {
          r.verdict = "INVARIANT_VIOLATION"; r.violated = bad;
          if (isnew) build_trace((int64_t)store.size() - 1, -1, nullptr); else build_trace(-1, -1, &s);
          r.distinct = (int64_t)seen.size(); r.depth = 1;
          goto done;
        }
      }
    }
    r.level_sizes.push_back((int64_t)frontier.size());
    r.depth = frontier.empty() ? 0 : 1;
    std::vector<Succ> succs;
    int32_t level = 1;
    const int succ_debug = std::getenv("ORACLE_SUCC_DEBUG") ? std::atoi(std::getenv("ORACLE_SUCC_DEBUG")) : 0;
    while (!frontier.empty()) {
      if (o.max_depth && level >= o.max_depth) { r.left_on_queue = (int64_t)frontier.size(); break; }
      std::vector<int64_t> nextf;
      if (o.workers > 1) {
        // ---- parallel expansion, sequential merge in frontier order (the FIFO order of the
        // single-worker search, so every count, kept representative and trace is the same)
        struct SRec { int action; bool im; std::string key, bad, bad_err; State s; };
        struct PRec { std::vector<SRec> succ; bool err = false; std::string errmsg; };
        const size_t B = 4096;
        for (size_t b0 = 0; b0 < frontier.size(); b0 += B) {
          const size_t b1 = std::min(frontier.size(), b0 + B);
          std::vector<PRec> recs(b1 - b0);
          std::atomic<size_t> next_i{b0};
          auto work = [&]() {
            std::vector<Succ> ss;
            for (size_t i; (i = next_i.fetch_add(1)) < b1;) {
              PRec& pr = recs[i - b0];
              const State& cur = store[frontier[i]];
              try {
                ss.clear();
                sp.next(cur, ss);
                for (auto& su : ss) {
                  SRec sr;
                  sr.action = su.action;
                  sr.im = in_model(su.s) && in_actions(cur, su.s);
                  if (sr.im) sr.key = canon_key(sp, cfg, o, su.s, perms, vv);
                  if (sr.im || o.inv_out_of_model) {
                    try { sr.bad = check_inv(su.s); } catch (const EvalError& e) { sr.bad_err = e.what(); }
                  }
                  sr.s = su.s;
                  pr.succ.push_back(std::move(sr));
                }
              } catch (const EvalError& e) { pr.err = true; pr.errmsg = e.what(); }
            }
          };
          std::vector<std::thread> th;
          for (int t = 1; t < o.workers; ++t) th.emplace_back(work);
          work();
          for (auto& t : th) t.join();
          for (size_t fi = b0; fi < b1; ++fi) {
            PRec& pr = recs[fi - b0];
            const int64_t idx = frontier[fi];
            if (pr.err) {
              r.verdict = "EVAL_ERROR"; r.error = pr.errmsg; build_trace(idx, -1, nullptr);
              r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
              goto finish;
            }
            r.generated += (int64_t)pr.succ.size();
            if (pr.succ.empty() && o.check_deadlock) {
              r.verdict = "DEADLOCK"; build_trace(idx, -1, nullptr);
              r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
              goto finish;
            }
            for (auto& su : pr.succ) {
              r.act_generated[su.action]++;
              bool isnew = false;
              if (su.im) {
                isnew = seen.insert(su.key).second;
                if (isnew) {
                  store.push_back(su.s); nodes.push_back({idx, su.action, level + 1});
                  nextf.push_back((int64_t)store.size() - 1);
                  r.act_distinct[su.action]++;
                  if (dump) std::fprintf(dump, "%s\n", sp.dump_line(su.s).c_str());
                }
              }
              if (isnew || (!su.im && o.inv_out_of_model)) {
                if (!su.bad_err.empty()) {
                  r.verdict = "EVAL_ERROR"; r.error = su.bad_err;
                  if (isnew) build_trace((int64_t)store.size() - 1, -1, nullptr);
                  else build_trace(idx, su.action, &su.s);
                  r.depth = level + 1;
                  r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
                  goto finish;
                }
                if (!su.bad.empty()) {
                  r.verdict = "INVARIANT_VIOLATION"; r.violated = su.bad;
                  if (isnew) build_trace((int64_t)store.size() - 1, -1, nullptr);
                  else build_trace(idx, su.action, &su.s);
                  r.depth = level + 1;
                  r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
                  goto finish;
                }
              }
              if (o.max_states && (int64_t)seen.size() >= o.max_states) {
                r.verdict = "SAMPLE_LIMIT"; r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
                goto finish;
              }
            }
          }
        }
        if (!nextf.empty()) { level++; r.depth = level; r.level_sizes.push_back((int64_t)nextf.size()); }
        frontier.swap(nextf);
        continue;
      }
      for (size_t fi = 0; fi < frontier.size(); ++fi) {
        int64_t idx = frontier[fi];
        State cur = store[idx];
        succs.clear();
        // TLC evaluation error while computing the successors: the search stops at this parent,
        // with the behaviour up to it as the trace ([ext]: TLC prints "The behavior up to this
        // point is:" and the summary lines)
        try { sp.next(cur, succs); } catch (const EvalError& e) {
          r.verdict = "EVAL_ERROR"; r.error = e.what(); build_trace(idx, -1, nullptr);
          r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
          goto finish;
        }
        r.generated += (int64_t)succs.size();
        if (succ_debug && level >= succ_debug)   // (debugging aid: every parent and its successor count, stderr)
          std::fprintf(stderr, "P\t%d\t%s\t%zu\n", (int)level, state_text(sp, cur).c_str(), succs.size());
        if (succs.empty() && o.check_deadlock) {
          r.verdict = "DEADLOCK"; build_trace(idx, -1, nullptr);
          r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
          goto finish;
        }
        for (auto& su : succs) {
          r.act_generated[su.action]++;
          bool im = in_model(su.s) && in_actions(cur, su.s);
          bool isnew = false;
          if (im) {
            auto k = canon_key(sp, cfg, o, su.s, perms, vv);
            isnew = seen.insert(k).second;
            if (isnew) {
              store.push_back(su.s); nodes.push_back({idx, su.action, level + 1});
              nextf.push_back((int64_t)store.size() - 1);
              r.act_distinct[su.action]++;
              if (dump) std::fprintf(dump, "%s\n", sp.dump_line(su.s).c_str());
              // debugging aid: ORACLE_FIND=<state text> prints that state's parent and action
              static const char* find_text = std::getenv("ORACLE_FIND");
              if (find_text && sp.dump_line(su.s) == find_text)
                std::fprintf(stderr, "FOUND via %s from\n%s\n", sp.action_names()[su.action].c_str(), sp.dump_line(cur).c_str());
            }
          }
          if (isnew || (!im && o.inv_out_of_model)) {
            std::string bad;
            try { bad = check_inv(su.s); } catch (const EvalError& e) {   // error evaluating an invariant
              r.verdict = "EVAL_ERROR"; r.error = e.what();
              if (isnew) build_trace((int64_t)store.size() - 1, -1, nullptr);
              else build_trace(idx, su.action, &su.s);
              r.depth = level + 1;
              r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
              goto finish;
            }
            if (!bad.empty()) {
              r.verdict = "INVARIANT_VIOLATION"; r.violated = bad;
              if (isnew) build_trace((int64_t)store.size() - 1, -1, nullptr);
              else build_trace(idx, su.action, &su.s);
              r.depth = level + 1;
              r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
              goto finish;
            }
          }
          if (o.max_states && (int64_t)seen.size() >= o.max_states) {
            r.verdict = "SAMPLE_LIMIT"; r.left_on_queue = (int64_t)(frontier.size() - fi - 1 + nextf.size());
            goto finish;
          }
        }
      }
      if (!nextf.empty()) { level++; r.depth = level; r.level_sizes.push_back((int64_t)nextf.size()); }
      frontier.swap(nextf);
    }
  finish:
    r.distinct = (int64_t)seen.size();
  } catch (const EvalError& e) {
    r.verdict = "EVAL_ERROR"; r.error = e.what(); r.distinct = (int64_t)seen.size();
  }
done:
  if (dump) std::fclose(dump);
  r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

// ----------------------------------------------------------------- lean BFS (full-size counts)
// The same search as bfs() with its workers > 1 merge (parents in frontier order, successors in
// Next order, so every count — per-action distinct ones included — is the single-worker FIFO
// one), for state spaces whose canonical texts and value trees do not fit in memory: the seen-set
// holds a 128-bit hash of each canonical key (two independent 64-bit hashes of the text; for
// 1e8 keys the chance of any collision is ~1e-23), and only the current and next level's states
// are kept, so there are no traces (a violation reports the verdict, the invariant and TLC's
// counters at the stop point).  Used for the full-size raft_original C2 fixture.
inline uint64_t text_hash(const std::string& k, uint64_t seed) {
  uint64_t h = seed ^ (k.size() * 0x9E3779B97F4A7C15ull);
  size_t i = 0;
  auto mix = [](uint64_t x) { x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x; };
  for (; i + 8 <= k.size(); i += 8) { uint64_t w; std::memcpy(&w, k.data() + i, 8); h = mix(h ^ w) * 0x100000001B3ull + i; }
  uint64_t w = 0; std::memcpy(&w, k.data() + i, k.size() - i);
  return mix(h ^ w ^ (0xA5ull << 56));
}

struct Key128 { uint64_t a, b; };
struct Key128Set {   // open addressing, linear probing; {0,0} = empty
  std::vector<Key128> t; uint64_t mask = 0, n = 0;
  explicit Key128Set(int log2) : t(1ull << log2, Key128{0, 0}), mask((1ull << log2) - 1) {}
  bool insert(Key128 k) {
    if (!k.a && !k.b) k.b = 1;
    if (2 * (n + 1) > t.size()) grow();
    for (uint64_t i = k.a & mask;; i = (i + 1) & mask) {
      if (!t[i].a && !t[i].b) { t[i] = k; ++n; return true; }
      if (t[i].a == k.a && t[i].b == k.b) return false;
    }
  }
  void grow() {
    std::vector<Key128> old; old.swap(t);
    t.assign(old.size() * 2, Key128{0, 0}); mask = t.size() - 1; n = 0;
    for (auto& k : old) if (k.a || k.b) insert(k);
  }
};

inline Result bfs_lean(const Spec& sp, const Cfg& cfg, const Options& o) {
  auto t0 = std::chrono::steady_clock::now();
  Result r;
  auto an = sp.action_names();
  r.act_generated.assign(an.size(), 0); r.act_distinct.assign(an.size(), 0);
  auto perms = cfg.symmetry.empty() ? std::vector<std::vector<int>>{} : sp.symmetry_perms(cfg.symmetry);
  auto vv = cfg.view.empty() ? std::vector<int>{} : sp.view_vars(cfg.view);
  Key128Set seen(20);
  auto key_of = [&](const State& s) {
    const std::string k = canon_key(sp, cfg, o, s, perms, vv);
    return Key128{text_hash(k, 0x243F6A8885A308D3ull), text_hash(k, 0x13198A2E03707344ull)};
  };
  auto in_model = [&](const State& s) {
    for (auto& c : cfg.constraints) if (!sp.constraint(c, s)) return false;
    return true;
  };
  auto in_actions = [&](const State& s, const State& t) {
    for (auto& c : cfg.action_constraints) if (!sp.action_constraint(c, s, t)) return false;
    return true;
  };
  auto check_inv = [&](const State& s) -> std::string {
    for (auto& inv : cfg.invariants) if (!sp.invariant(inv, s)) return inv;
    return "";
  };
  const int W = std::max(1, o.workers);
  try {
    std::vector<State> frontier;
    for (auto& s : sp.init()) {
      r.generated++;
      const bool im = in_model(s);
      const bool isnew = im && seen.insert(key_of(s));
      if (isnew) frontier.push_back(s);
      if (isnew || (!im && o.inv_out_of_model)) {
        auto bad = check_inv(s);
        if (!bad.empty()) { r.verdict = "INVARIANT_VIOLATION"; r.violated = bad; r.depth = 1; goto finish; }
      }
    }
    r.level_sizes.push_back((int64_t)frontier.size());
    r.depth = frontier.empty() ? 0 : 1;
    for (int32_t level = 1; !frontier.empty();) {
      if (o.max_depth && level >= o.max_depth) { r.left_on_queue = (int64_t)frontier.size(); break; }
      std::vector<State> nextf;
      struct SRec { int action; bool im; Key128 key; std::string bad, bad_err; State s; };
      struct PRec { std::vector<SRec> succ; bool err = false; std::string errmsg; };
      const size_t B = 8192;
      for (size_t b0 = 0; b0 < frontier.size(); b0 += B) {
        const size_t b1 = std::min(frontier.size(), b0 + B);
        std::vector<PRec> recs(b1 - b0);
        std::atomic<size_t> next_i{b0};
        auto work = [&]() {
          std::vector<Succ> ss;
          for (size_t i; (i = next_i.fetch_add(1)) < b1;) {
            PRec& pr = recs[i - b0];
            const State& cur = frontier[i];
            try {
              ss.clear();
              sp.next(cur, ss);
              for (auto& su : ss) {
                SRec sr;
                sr.action = su.action;
                sr.im = in_model(su.s) && in_actions(cur, su.s);
                sr.key = sr.im ? key_of(su.s) : Key128{0, 0};
                if (sr.im || o.inv_out_of_model) {
                  try { sr.bad = check_inv(su.s); } catch (const EvalError& e) { sr.bad_err = e.what(); }
                }
                if (sr.im) sr.s = std::move(su.s);
                pr.succ.push_back(std::move(sr));
              }
            } catch (const EvalError& e) { pr.err = true; pr.errmsg = e.what(); }
          }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < W; ++t) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
        for (size_t fi = b0; fi < b1; ++fi) {
          PRec& pr = recs[fi - b0];
          auto left = [&]() { return (int64_t)(frontier.size() - fi - 1 + nextf.size()); };
          if (pr.err) { r.verdict = "EVAL_ERROR"; r.error = pr.errmsg; r.left_on_queue = left(); goto finish; }
          r.generated += (int64_t)pr.succ.size();
          if (pr.succ.empty() && o.check_deadlock) { r.verdict = "DEADLOCK"; r.left_on_queue = left(); goto finish; }
          for (auto& su : pr.succ) {
            r.act_generated[su.action]++;
            const bool isnew = su.im && seen.insert(su.key);
            if (isnew) { r.act_distinct[su.action]++; nextf.push_back(std::move(su.s)); }
            if (isnew || (!su.im && o.inv_out_of_model)) {
              if (!su.bad_err.empty() || !su.bad.empty()) {
                if (su.bad_err.empty()) { r.verdict = "INVARIANT_VIOLATION"; r.violated = su.bad; }
                else { r.verdict = "EVAL_ERROR"; r.error = su.bad_err; }
                r.depth = level + 1; r.left_on_queue = left();
                goto finish;
              }
            }
          }
        }
        if (o.progress) std::fprintf(stderr, "level %d: %zu/%zu parents, %llu distinct, %.0f s\n", level, b1, frontier.size(),
                                     (unsigned long long)seen.n,
                                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      }
      if (!nextf.empty()) { level++; r.depth = level; r.level_sizes.push_back((int64_t)nextf.size()); }
      frontier.swap(nextf);
    }
  } catch (const EvalError& e) {
    r.verdict = "EVAL_ERROR"; r.error = e.what();
  }
finish:
  r.distinct = (int64_t)seen.n;
  r.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

}  // namespace oracle
