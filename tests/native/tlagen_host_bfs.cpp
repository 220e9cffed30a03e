// TEST INFRASTRUCTURE: a sequential host BFS over the front end's generated C++ (compiled with
// -DTLG_FILE="x.gen.h"), checking the generated semantics on the CPU against the oracle's counts
// (tests/test_tlagen.py).  It is the same code the GPU path compiles for gfx950; the GPU engine
// is raft-tla_amd/csrc/tlagen/tlagen_kernels.h.
//
//   tlagen_host_bfs [--max-depth D] [--no-deadlock]
// prints {"verdict", "generated", "distinct", "depth", "levels", "actions", "violated", "err"}
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

struct Succ { std::vector<u32> w; int act; bool im, cerr; };

struct Emit {
  std::vector<Succ>* out;
  void operator()(tlg::Cx& c) {
    tlv::Ar& A = *c.A;
    const u32 t0 = A.top;
    tlg::Cx d = c;
    for (int i = 0; i < tlg::NV; ++i) d.cur[i] = c.nxt[i];
    Succ s;
    const u32 e0 = A.err;
    s.im = tlg::constraints(d);
    s.cerr = A.err != e0;   // a constraint could not be evaluated: TLC's evaluation error
    A.err = e0;
    for (int i = 0; i < tlg::NV; ++i) { const u32 h = c.nxt[i]; s.w.insert(s.w.end(), A.w + h, A.w + h + tlv::sz(A, h)); }
    s.act = c.act;
    out->push_back(std::move(s));
    A.top = t0;
  }
};

static void load(tlg::Cx& c, const std::vector<u32>& w) {
  u32 off = 0;
  for (int i = 0; i < tlg::NV; ++i) { c.cur[i] = tlv::copy_in(*c.A, w.data() + off); off += w[off] >> 3; }
}

int main(int argc, char** argv) {
  long long max_depth = 0;
  bool deadlock = true;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--max-depth") && i + 1 < argc) max_depth = std::atoll(argv[++i]);
    else if (!std::strcmp(argv[i], "--no-deadlock")) deadlock = false;
  }
  static u32 words[1 << 22], hs[1 << 16];
  tlv::Ar A;
  tlv::init(A, words, 1 << 22, hs, 1 << 16);
  tlg::Cx c;
  c.A = &A;
  tlg::init_consts(c);
  const u32 floor = A.top;
  std::unordered_set<std::vector<u32>, WordsHash> seen;
  std::vector<std::vector<u32>> frontier, next;
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
    Emit em{&init};
    A.top = floor;
    tlg::init_states(c, em);
    err |= A.err;
    for (auto& s : init) {
      ++generated;
      A.top = floor; load(c, s.w);
      if (!tlg::constraints(c)) continue;
      if (!seen.insert(s.w).second) continue;
      const int bad = check(s.w);
      if (bad >= 0) report(bad);
      frontier.push_back(s.w);
    }
    if (!frontier.empty()) { depth = 1; levels.push_back((long long)frontier.size()); }
  }
  while (!frontier.empty() && verdict == "OK" && !err) {
    if (max_depth && depth >= max_depth) { verdict = "DEPTH_LIMIT"; break; }
    next.clear();
    for (size_t fi = 0; fi < frontier.size() && verdict == "OK"; ++fi) {
      std::vector<Succ> succ;
      Emit em{&succ};
      A.top = floor;
      A.err = 0;
      load(c, frontier[fi]);
      tlg::next_states(c, em);
      if (A.err) { err |= A.err; verdict = (A.err & tlv::E_OVF) ? "CAPACITY" : "EVAL_ERROR"; break; }
      generated += (long long)succ.size();
      if (succ.empty() && deadlock) { verdict = "DEADLOCK"; break; }
      for (auto& s : succ) {
        if (s.cerr) { verdict = "EVAL_ERROR"; break; }
        gen_act[s.act]++;
        bool isnew = false;
        if (s.im) {
          isnew = seen.insert(s.w).second;
          if (isnew) { next.push_back(s.w); dist_act[s.act]++; }
        }
        if (isnew || !s.im) {
          const int bad = check(s.w);
          if (bad >= 0) { report(bad); break; }
        }
      }
    }
    if (!next.empty()) { ++depth; levels.push_back((long long)next.size()); }
    frontier.swap(next);
  }
  size_t nwords = 0;
  for (auto& w : seen) nwords += w.size();
  std::printf("{\"verdict\": \"%s\", \"violated\": \"%s\", \"generated\": %lld, \"distinct\": %zu, \"depth\": %d, \"err\": %u, "
              "\"words_per_state\": %.1f, \"levels\": [", verdict.c_str(), violated.c_str(), generated, seen.size(), depth, err,
              seen.empty() ? 0.0 : (double)nwords / seen.size());
  for (size_t q = 0; q < levels.size(); ++q) std::printf("%s%lld", q ? ", " : "", levels[q]);
  std::printf("], \"actions\": {");
  for (int k = 0; k < tlg::NACT; ++k) std::printf("%s\"%s\": [%lld, %lld]", k ? ", " : "", tlg::kActionNames[k], gen_act[k], dist_act[k]);
  std::printf("}}\n");
  return 0;
}
