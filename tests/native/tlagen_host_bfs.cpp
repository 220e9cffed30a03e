// TEST INFRASTRUCTURE: a sequential host BFS over the front end's generated C++ (compiled with
// -DTLG_FILE="x.gen.h"), checking the generated semantics on the CPU against the oracle's counts
// (tests/test_tlagen.py).  It is the same code the GPU path compiles for gfx950; the GPU engine
// is raft-tla_amd/csrc/tlagen/tlagen_kernels.h.
//
//   tlagen_host_bfs [--max-depth D] [--no-deadlock] [--trace] [--dump FILE]
// prints {"verdict", "generated", "distinct", "depth", "levels", "actions", "violated", "err"}
// (--trace: and "trace", the counterexample to a violating new state, one line per state, in the
// format of the library's trace printer; --dump: every kept state's text, one per line)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

#include TLG_FILE

using tlv::u32;

struct WordsHash {
  size_t operator()(const std::vector<u32>& w) const { return (size_t)tlv::fp_words(w.data(), (u32)w.size(), 7); }
};

struct Succ { std::vector<u32> w, key; int act; bool im, cerr; };   // key: the view's words (TLC VIEW) or w

struct Emit {
  std::vector<Succ>* out;
  bool init;   // initial states: no transition, no action constraints
  void operator()(tlg::Cx& c) {
    tlv::Ar& A = *c.A;
    const u32 t0 = A.top;
    tlg::Cx d = c;
    for (int i = 0; i < tlg::NV; ++i) d.cur[i] = c.nxt[i];
    Succ s;
    const u32 e0 = A.err;
    s.im = tlg::constraints(d) && (init || tlg::action_constraints(c));
    s.cerr = A.err != e0;   // a constraint could not be evaluated: TLC's evaluation error
    A.err = e0;
    for (int i = 0; i < tlg::NV; ++i) { const u32 h = c.nxt[i]; s.w.insert(s.w.end(), A.w + h, A.w + h + tlv::sz(A, h)); }
    if ((tlg::HAS_VIEW || tlg::HAS_SYMMETRY) && s.im && !s.cerr) {   // TLC's VIEW / SYMMETRY: states told apart by canon_view
      const u32 vh = tlg::canon_view(d);
      s.key.assign(A.w + vh, A.w + vh + tlv::sz(A, vh));
      if (A.err != e0) { s.cerr = true; A.err = e0; }
    } else {
      s.key = s.w;
    }
    s.act = c.act;
    out->push_back(std::move(s));
    A.top = t0;
  }
};

// one-line text of a value / state (raft-tla_amd/csrc/tlagen/tlagen_backend.cpp Printer)
static std::string vtext(const u32* w) {
  const u32 tag = w[0] & 7u, n = w[1];
  switch (tag) {
    case 1: return w[1] ? "TRUE" : "FALSE";
    case 2: return std::to_string((long long)(int)(w[1] ^ 0x80000000u));
    case 3: return tlg::kAtomNames[w[1]];
    case 4: case 6: {   // set elements sorted by their text (the oracle's print rule, oracle/tla.h show)
      std::vector<std::string> el;
      const u32* e = w + 2;
      for (u32 i = 0; i < n; ++i) { el.push_back(vtext(e)); e += e[0] >> 3; }
      if (tag == 6) std::sort(el.begin(), el.end());
      std::string o = tag == 4 ? "<<" : "{";
      for (u32 i = 0; i < n; ++i) o += (i ? ", " : "") + el[i];
      return o + (tag == 4 ? ">>" : "}");
    }
    default: {
      bool rec = true;
      const u32* e = w + 2;
      for (u32 i = 0; i < n; ++i) {
        if ((e[0] & 7u) != 3 || tlg::kAtomNames[e[1]][0] != '"') rec = false;
        e += e[0] >> 3; e += e[0] >> 3;
      }
      std::vector<std::pair<std::string, std::string>> fs;   // fields / pairs sorted by text
      e = w + 2;
      for (u32 i = 0; i < n; ++i) {
        const u32* val = e + (e[0] >> 3);
        if (rec) { std::string k = tlg::kAtomNames[e[1]]; fs.push_back({k.substr(1, k.size() - 2), vtext(val)}); }
        else fs.push_back({vtext(e), vtext(val)});
        e = val + (val[0] >> 3);
      }
      std::sort(fs.begin(), fs.end());
      std::string o = rec ? "[" : "(";
      for (u32 i = 0; i < n; ++i) o += (i ? (rec ? ", " : " @@ ") : "") + fs[i].first + (rec ? " |-> " : " :> ") + fs[i].second;
      return o + (rec ? "]" : ")");
    }
  }
}
static std::string state_text(const std::vector<u32>& w) {
  std::string o;
  const u32* p = w.data();
  for (int i = 0; i < tlg::NV; ++i) { o += (i ? " " : "") + std::string("/\\ ") + tlg::kVarNames[i] + " = " + vtext(p); p += p[0] >> 3; }
  return o;
}

static void load(tlg::Cx& c, const std::vector<u32>& w) {
  u32 off = 0;
  for (int i = 0; i < tlg::NV; ++i) { c.cur[i] = tlv::copy_in(*c.A, w.data() + off); off += w[off] >> 3; }
}

int main(int argc, char** argv) {
  long long max_depth = 0;
  bool deadlock = true, want_trace = false;
  const char* dump_path = nullptr;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--max-depth") && i + 1 < argc) max_depth = std::atoll(argv[++i]);
    else if (!std::strcmp(argv[i], "--no-deadlock")) deadlock = false;
    else if (!std::strcmp(argv[i], "--trace")) want_trace = true;
    else if (!std::strcmp(argv[i], "--dump") && i + 1 < argc) dump_path = argv[++i];
  }
  const int succ_debug = std::getenv("TLG_SUCC_DEBUG") ? std::atoi(std::getenv("TLG_SUCC_DEBUG")) : 0;
  static u32 words[1 << 22], hs[1 << 16];
  tlv::Ar A;
  tlv::init(A, words, 1 << 22, hs, 1 << 16);
  tlg::Cx c;
  c.A = &A;
  tlg::init_consts(c);
  const u32 floor = A.top;
  std::unordered_set<std::vector<u32>, WordsHash> seen;
  std::vector<std::vector<u32>> all;      // every kept state, in FIFO order
  std::vector<long long> par;              // its parent's index (-1: initial)
  std::vector<long long> frontier, next;   // indices into all
  std::vector<std::string> trace;
  auto trace_to = [&](long long i, const std::vector<u32>* extra) {
    std::vector<long long> chain;
    for (; i >= 0; i = par[i]) chain.push_back(i);
    for (size_t q = chain.size(); q-- > 0;) trace.push_back(state_text(all[chain[q]]));
    if (extra) trace.push_back(state_text(*extra));
  };
  std::vector<long long> levels;
  std::vector<long long> gen_act(tlg::NACT + 1, 0), dist_act(tlg::NACT + 1, 0);
  long long generated = 0;
  std::string verdict = "OK", violated;
  int depth = 0;
  unsigned err = 0;
  // invariant index that fails, -1 if all hold; an evaluation error sets `inv_err` (TLC's
  // "Evaluating invariant X failed": an EVAL_ERROR verdict, not a violation)
  bool inv_err = false;
  auto check = [&](const std::vector<u32>& w) -> int {
    A.top = floor; A.err = 0; load(c, w);
    const int bad = tlg::invariants(c);
    if (A.err) { err |= A.err; inv_err = true; }
    return bad;
  };
  auto report = [&](int bad) {
    if (inv_err) { verdict = "EVAL_ERROR"; violated = tlg::kInvariantNames[bad]; }
    else { verdict = "INVARIANT_VIOLATION"; violated = tlg::kInvariantNames[bad]; }
  };
  {
    std::vector<Succ> init;
    Emit em{&init, true};
    A.top = floor;
    tlg::init_states(c, em);
    err |= A.err;
    for (auto& s : init) {
      ++generated;
      if (!s.im) continue;
      if (!seen.insert(s.key).second) continue;
      const int bad = check(s.w);
      all.push_back(s.w); par.push_back(-1);
      if (bad >= 0) { report(bad); trace_to((long long)all.size() - 1, nullptr); }
      frontier.push_back((long long)all.size() - 1);
    }
    if (!frontier.empty()) { depth = 1; levels.push_back((long long)frontier.size()); }
  }
  while (!frontier.empty() && verdict == "OK" && !err) {
    if (max_depth && depth >= max_depth) { verdict = "DEPTH_LIMIT"; break; }
    next.clear();
    for (size_t fi = 0; fi < frontier.size() && verdict == "OK"; ++fi) {
      std::vector<Succ> succ;
      Emit em{&succ, false};
      A.top = floor;
      A.err = 0;
      load(c, all[frontier[fi]]);
      tlg::next_states(c, em);
      if (A.err) { err |= A.err; verdict = (A.err & tlv::E_OVF) ? "CAPACITY" : "EVAL_ERROR"; break; }
      generated += (long long)succ.size();
      if (succ_debug && depth >= succ_debug)   // (debugging aid: every parent and its successor count, stderr)
        std::fprintf(stderr, "P\t%d\t%s\t%zu\n", depth, state_text(all[frontier[fi]]).c_str(), succ.size());
      if (succ.empty() && deadlock) { verdict = "DEADLOCK"; break; }
      for (auto& s : succ) {
        if (s.cerr) { verdict = "EVAL_ERROR"; break; }
        gen_act[s.act]++;
        bool isnew = false;
        if (s.im) {
          isnew = seen.insert(s.key).second;
          if (isnew) {
            all.push_back(s.w); par.push_back(frontier[fi]);
            next.push_back((long long)all.size() - 1); dist_act[s.act]++;
          }
        }
        if (isnew || !s.im) {
          const int bad = check(s.w);
          if (bad >= 0) {
            report(bad);
            if (isnew) trace_to((long long)all.size() - 1, nullptr); else trace_to(frontier[fi], &s.w);
            break;
          }
        }
      }
    }
    if (!next.empty()) { ++depth; levels.push_back((long long)next.size()); }
    frontier.swap(next);
  }
  if (dump_path) {
    if (std::FILE* f = std::fopen(dump_path, "w")) {
      for (auto& w : all) std::fprintf(f, "%s\n", state_text(w).c_str());
      std::fclose(f);
    }
  }
  size_t nwords = 0;
  for (auto& w : seen) nwords += w.size();
  std::printf("{\"verdict\": \"%s\", \"violated\": \"%s\", \"generated\": %lld, \"distinct\": %zu, \"depth\": %d, \"err\": %u, "
              "\"words_per_state\": %.1f, \"levels\": [", verdict.c_str(), violated.c_str(), generated, seen.size(), depth, err,
              seen.empty() ? 0.0 : (double)nwords / seen.size());
  for (size_t q = 0; q < levels.size(); ++q) std::printf("%s%lld", q ? ", " : "", levels[q]);
  std::printf("], \"actions\": {");
  for (int k = 0; k < tlg::NACT; ++k) std::printf("%s\"%s\": [%lld, %lld]", k ? ", " : "", tlg::kActionNames[k], gen_act[k], dist_act[k]);
  std::printf("}");
  if (want_trace) {
    std::printf(", \"trace\": [");
    for (size_t q = 0; q < trace.size(); ++q) {
      std::string e;
      for (char ch : trace[q]) { if (ch == '"' || ch == '\\') e += '\\'; e += ch; }
      std::printf("%s\"%s\"", q ? ", " : "", e.c_str());
    }
    std::printf("]");
  }
  std::printf("}\n");
  return 0;
}
