// ============================================================================
// TEST INFRASTRUCTURE ONLY.  This is the CPU *oracle* of raftmc: a literal
// restatement of the reference TLA+ specs over an explicit TLA+ value model.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// build, link or execute anything under oracle/.  The product (raft-tla_amd/)
// never includes this file.
//
// tla.h — a minimal TLA+ value model: BOOLEAN, Int, strings, model values,
// sequences, finite sets and finite functions (records are functions whose
// domain is a set of strings).  Semantics follow TLC's value equality:
//   * a function whose domain is 1..n (n >= 0) IS the sequence of its values
//     (TLC: FcnRcdValue over 1..n == TupleValue), so [x \in {} |-> v] = <<>>;
//   * sets are canonical (sorted, duplicate-free) so structural equality is
//     TLA+ equality.
// The total order used to canonicalise sets/functions is an implementation
// order, not TLC's Value.compareTo (see DESIGN.md "symmetry compare order").
// ============================================================================
#pragma once
#include <algorithm>
#include <cassert>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <shared_mutex>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace tla {

enum class K : uint8_t { Bool = 0, Int = 1, Str = 2, MV = 3, Seq = 4, Set = 5, Fcn = 6 };

struct Val;
using V = std::shared_ptr<const Val>;

struct EvalError : std::runtime_error {
  explicit EvalError(const std::string& m) : std::runtime_error(m) {}
};

// ---- interning of strings and model values (ids are stable per process) ----
// Thread-safe for the parallel BFS (engine.h, --workers): lookups take a shared lock,
// insertions an exclusive one, and the name vectors are reserved up front so an
// insertion never moves the strings other threads are reading by id.
struct Names {
  std::vector<std::string> str, mv;
  std::unordered_map<std::string, int> str_id, mv_id;
  std::shared_mutex mu;
  Names() { str.reserve(1 << 16); mv.reserve(1 << 12); }
  static Names& get() { static Names n; return n; }
  int intern(std::vector<std::string>& names, std::unordered_map<std::string, int>& ids, const std::string& s) {
    {
      std::shared_lock<std::shared_mutex> lk(mu);
      auto it = ids.find(s);
      if (it != ids.end()) return it->second;
    }
    std::unique_lock<std::shared_mutex> lk(mu);
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    if (names.size() == names.capacity()) throw EvalError("too many distinct names");
    int id = (int)names.size(); names.push_back(s); ids[s] = id; return id;
  }
  // per-thread memo in front of the shared table: no shared cache line on the hot path
  int intern_str(const std::string& s) {
    thread_local std::unordered_map<std::string, int> memo;
    auto it = memo.find(s);
    if (it != memo.end()) return it->second;
    return memo[s] = intern(str, str_id, s);
  }
  int intern_mv(const std::string& s) {
    thread_local std::unordered_map<std::string, int> memo;
    auto it = memo.find(s);
    if (it != memo.end()) return it->second;
    return memo[s] = intern(mv, mv_id, s);
  }
};

struct Val {
  K k;
  int64_t i = 0;            // Bool (0/1), Int, Str id, MV id
  std::vector<V> a;         // Seq elements | Set elements (sorted) | Fcn domain (sorted)
  std::vector<V> b;         // Fcn values (parallel to a)
  size_t h = 0;             // structural hash
};

int cmp(const V& x, const V& y);
inline bool eq(const V& x, const V& y) { return x.get() == y.get() || cmp(x, y) == 0; }
struct Less { bool operator()(const V& x, const V& y) const { return cmp(x, y) < 0; } };

inline size_t mix(size_t h, size_t v) {
  h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
  return h;
}

inline V mk(K k, int64_t i) {
  auto p = std::make_shared<Val>(); p->k = k; p->i = i;
  p->h = mix((size_t)k * 1315423911u, (size_t)i);
  return p;
}
inline V Bool(bool b) { static V t = mk(K::Bool, 1), f = mk(K::Bool, 0); return b ? t : f; }
inline V Int(int64_t i) { return mk(K::Int, i); }
inline V Str(const std::string& s) { return mk(K::Str, Names::get().intern_str(s)); }
inline V MV(const std::string& s) { return mk(K::MV, Names::get().intern_mv(s)); }

inline V seq(std::vector<V> xs) {
  auto p = std::make_shared<Val>(); p->k = K::Seq;
  size_t h = 77;
  for (auto& x : xs) h = mix(h, x->h);
  p->a = std::move(xs); p->h = h; return p;
}
inline V set(std::vector<V> xs) {
  std::sort(xs.begin(), xs.end(), Less());
  xs.erase(std::unique(xs.begin(), xs.end(), [](const V& x, const V& y) { return eq(x, y); }), xs.end());
  auto p = std::make_shared<Val>(); p->k = K::Set;
  size_t h = 991;
  for (auto& x : xs) h = mix(h, x->h);
  p->a = std::move(xs); p->h = h; return p;
}
// Function from parallel key/value vectors (keys need not be sorted; must be unique).
inline V fcn(std::vector<V> ks, std::vector<V> vs) {
  std::vector<size_t> idx(ks.size());
  for (size_t t = 0; t < idx.size(); ++t) idx[t] = t;
  std::sort(idx.begin(), idx.end(), [&](size_t x, size_t y) { return cmp(ks[x], ks[y]) < 0; });
  std::vector<V> a, b;
  a.reserve(ks.size()); b.reserve(ks.size());
  for (size_t t : idx) {
    if (!a.empty() && eq(a.back(), ks[t])) throw EvalError("duplicate function domain element");
    a.push_back(ks[t]); b.push_back(vs[t]);
  }
  // TLC: a function with domain 1..n is the n-tuple of its values.
  bool is_seq = true;
  for (size_t t = 0; t < a.size(); ++t)
    if (a[t]->k != K::Int || a[t]->i != (int64_t)t + 1) { is_seq = false; break; }
  if (is_seq) return seq(std::move(b));
  auto p = std::make_shared<Val>(); p->k = K::Fcn;
  size_t h = 4241;
  for (size_t t = 0; t < a.size(); ++t) h = mix(mix(h, a[t]->h), b[t]->h);
  p->a = std::move(a); p->b = std::move(b); p->h = h; return p;
}
// Record [f1 |-> v1, ...]
inline V rec(std::initializer_list<std::pair<const char*, V>> fs) {
  std::vector<V> ks, vs;
  for (auto& f : fs) { ks.push_back(Str(f.first)); vs.push_back(f.second); }
  return fcn(std::move(ks), std::move(vs));
}

inline int cmp(const V& x, const V& y) {
  if (x.get() == y.get()) return 0;
  if (x->k != y->k) {
    // an empty Fcn never exists (normalised to <<>>), so kinds are decisive
    return (int)x->k < (int)y->k ? -1 : 1;
  }
  switch (x->k) {
    case K::Bool: case K::Int: case K::MV:
      return x->i < y->i ? -1 : (x->i > y->i ? 1 : 0);
    case K::Str: {
      if (x->i == y->i) return 0;
      const auto& n = Names::get().str;
      int c = n[x->i].compare(n[y->i]);
      return c < 0 ? -1 : (c > 0 ? 1 : 0);
    }
    case K::Seq: case K::Set: {
      if (x->h == y->h && x->a.size() == y->a.size()) {
        bool same = true;
        for (size_t t = 0; t < x->a.size(); ++t) if (!eq(x->a[t], y->a[t])) { same = false; break; }
        if (same) return 0;
      }
      if (x->a.size() != y->a.size()) return x->a.size() < y->a.size() ? -1 : 1;
      for (size_t t = 0; t < x->a.size(); ++t) { int c = cmp(x->a[t], y->a[t]); if (c) return c; }
      return 0;
    }
    case K::Fcn: {
      if (x->a.size() != y->a.size()) return x->a.size() < y->a.size() ? -1 : 1;
      for (size_t t = 0; t < x->a.size(); ++t) { int c = cmp(x->a[t], y->a[t]); if (c) return c; }
      for (size_t t = 0; t < x->b.size(); ++t) { int c = cmp(x->b[t], y->b[t]); if (c) return c; }
      return 0;
    }
  }
  return 0;
}

// ---------------------------------------------------------------- accessors
inline int64_t as_int(const V& v) { if (v->k != K::Int) throw EvalError("expected integer"); return v->i; }
inline bool as_bool(const V& v) { if (v->k != K::Bool) throw EvalError("expected boolean"); return v->i != 0; }

// DOMAIN f
inline V domain(const V& f) {
  if (f->k == K::Seq) { std::vector<V> d; for (size_t t = 0; t < f->a.size(); ++t) d.push_back(Int((int64_t)t + 1)); return set(d); }
  if (f->k == K::Fcn) { auto p = std::make_shared<Val>(); p->k = K::Set; p->a = f->a; size_t h = 991; for (auto& x : p->a) h = mix(h, x->h); p->h = h; return p; }
  throw EvalError("DOMAIN of non-function");
}
inline std::vector<V> domain_elems(const V& f) {
  if (f->k == K::Seq) { std::vector<V> d; for (size_t t = 0; t < f->a.size(); ++t) d.push_back(Int((int64_t)t + 1)); return d; }
  if (f->k == K::Fcn) return f->a;
  throw EvalError("DOMAIN of non-function");
}
inline int find_key(const V& f, const V& x) {   // index into f->a, -1 if absent (Fcn only)
  auto it = std::lower_bound(f->a.begin(), f->a.end(), x, Less());
  if (it != f->a.end() && eq(*it, x)) return (int)(it - f->a.begin());
  return -1;
}
inline bool in_domain(const V& f, const V& x) {
  if (f->k == K::Seq) return x->k == K::Int && x->i >= 1 && x->i <= (int64_t)f->a.size();
  if (f->k == K::Fcn) return find_key(f, x) >= 0;
  throw EvalError("DOMAIN of non-function");
}
// f[x]
inline V ap(const V& f, const V& x) {
  if (f->k == K::Seq) {
    if (x->k != K::Int || x->i < 1 || x->i > (int64_t)f->a.size())
      throw EvalError("sequence index out of domain");
    return f->a[x->i - 1];
  }
  if (f->k == K::Fcn) {
    int t = find_key(f, x);
    if (t < 0) throw EvalError("function applied outside its domain");
    return f->b[t];
  }
  throw EvalError("application of non-function");
}
inline V ap(const V& f, const char* field) { return ap(f, Str(field)); }
inline V ap(const V& f, int64_t i) { return ap(f, Int(i)); }

// [f EXCEPT ![x] = v]
inline V except(const V& f, const V& x, const V& v) {
  if (f->k == K::Seq) {
    if (x->k != K::Int || x->i < 1 || x->i > (int64_t)f->a.size()) return f;  // TLC: EXCEPT outside domain is a no-op
    std::vector<V> xs = f->a; xs[x->i - 1] = v; return seq(std::move(xs));
  }
  if (f->k == K::Fcn) {
    int t = find_key(f, x);
    if (t < 0) return f;
    std::vector<V> ks = f->a, vs = f->b; vs[t] = v;
    return fcn(std::move(ks), std::move(vs));
  }
  throw EvalError("EXCEPT on non-function");
}
inline V except(const V& f, const char* field, const V& v) { return except(f, Str(field), v); }

// f @@ g  (TLC module: left-biased union of functions)
inline V at_at(const V& f, const V& g) {
  std::vector<V> ks = domain_elems(f), vs;
  for (auto& k : ks) vs.push_back(ap(f, k));
  for (auto& k : domain_elems(g)) if (!in_domain(f, k)) { ks.push_back(k); vs.push_back(ap(g, k)); }
  return fcn(std::move(ks), std::move(vs));
}
// x :> y
inline V colon_gt(const V& x, const V& y) { return fcn({x}, {y}); }

// ---------------------------------------------------------------- sets
inline bool in_set(const V& x, const V& s) {
  if (s->k != K::Set) throw EvalError("\\in of non-set");
  return std::binary_search(s->a.begin(), s->a.end(), x, Less());
}
inline V cup(const V& s, const V& t) { std::vector<V> xs = s->a; xs.insert(xs.end(), t->a.begin(), t->a.end()); return set(xs); }
inline V setminus(const V& s, const V& t) { std::vector<V> xs; for (auto& x : s->a) if (!in_set(x, t)) xs.push_back(x); return set(xs); }
inline V cap(const V& s, const V& t) { std::vector<V> xs; for (auto& x : s->a) if (in_set(x, t)) xs.push_back(x); return set(xs); }
inline V empty_set() { static V e = set({}); return e; }
inline int64_t card(const V& s) { if (s->k != K::Set) throw EvalError("Cardinality of non-set"); return (int64_t)s->a.size(); }
inline bool subseteq(const V& s, const V& t) { for (auto& x : s->a) if (!in_set(x, t)) return false; return true; }
inline V range_set(int64_t lo, int64_t hi) { std::vector<V> xs; for (int64_t t = lo; t <= hi; ++t) xs.push_back(Int(t)); return set(xs); }
// SUBSET s (power set), used only for tiny server sets
inline std::vector<V> subsets(const V& s) {
  std::vector<V> out; size_t n = s->a.size();
  if (n > 20) throw EvalError("SUBSET too large");
  for (size_t m = 0; m < ((size_t)1 << n); ++m) {
    std::vector<V> xs; for (size_t t = 0; t < n; ++t) if (m >> t & 1) xs.push_back(s->a[t]);
    out.push_back(set(xs));
  }
  return out;
}
inline int64_t set_max(const V& s) {   // Max(s) == CHOOSE x \in s : \A y \in s : x >= y
  if (s->a.empty()) throw EvalError("CHOOSE from empty set (Max({}))");
  int64_t m = as_int(s->a[0]); for (auto& x : s->a) m = std::max(m, as_int(x)); return m;
}
inline int64_t set_min(const V& s) {
  if (s->a.empty()) throw EvalError("CHOOSE from empty set (Min({}))");
  int64_t m = as_int(s->a[0]); for (auto& x : s->a) m = std::min(m, as_int(x)); return m;
}

// ---------------------------------------------------------------- sequences
inline int64_t len(const V& s) {
  if (s->k != K::Seq) throw EvalError("Len of non-sequence");
  return (int64_t)s->a.size();
}
inline V append(const V& s, const V& x) { if (s->k != K::Seq) throw EvalError("Append to non-sequence"); std::vector<V> xs = s->a; xs.push_back(x); return seq(std::move(xs)); }
inline V concat(const V& s, const V& t) { if (s->k != K::Seq || t->k != K::Seq) throw EvalError("\\o of non-sequences"); std::vector<V> xs = s->a; xs.insert(xs.end(), t->a.begin(), t->a.end()); return seq(std::move(xs)); }
// SubSeq(s, m, n) == [i \in 1..(1+n-m) |-> s[i+m-1]]
inline V subseq(const V& s, int64_t m, int64_t n) {
  if (s->k != K::Seq) throw EvalError("SubSeq of non-sequence");
  std::vector<V> xs;
  for (int64_t t = m; t <= n; ++t) {
    if (t < 1 || t > (int64_t)s->a.size()) throw EvalError("SubSeq index out of domain");
    xs.push_back(s->a[t - 1]);
  }
  return seq(std::move(xs));
}
inline V empty_seq() { static V e = seq({}); return e; }
// SequencesExt.tla:134-140 IsPrefix(s, t) == DOMAIN s \subseteq DOMAIN t /\ \A i \in DOMAIN s: s[i] = t[i]
inline bool is_prefix(const V& s, const V& t) {
  if (len(s) > len(t)) return false;
  for (size_t q = 0; q < s->a.size(); ++q) if (!eq(s->a[q], t->a[q])) return false;
  return true;
}

// ---------------------------------------------------------------- printing
// Canonical text: records print fields alphabetically; set elements and
// general-function keys print sorted by their own canonical text (bytewise).
// The product's decoder prints with the same rule so state dumps compare as
// sets of strings.
std::string show(const V& v);
inline bool is_record(const V& v) {
  if (v->k != K::Fcn || v->a.empty()) return false;
  for (auto& k : v->a) if (k->k != K::Str) return false;
  return true;
}
inline std::string show(const V& v) {
  const auto& N = Names::get();
  switch (v->k) {
    case K::Bool: return v->i ? "TRUE" : "FALSE";
    case K::Int: return std::to_string(v->i);
    case K::Str: return "\"" + N.str[v->i] + "\"";
    case K::MV: return N.mv[v->i];
    case K::Seq: {
      std::string s = "<<";
      for (size_t t = 0; t < v->a.size(); ++t) { if (t) s += ", "; s += show(v->a[t]); }
      return s + ">>";
    }
    case K::Set: {
      std::vector<std::string> el; for (auto& x : v->a) el.push_back(show(x));
      std::sort(el.begin(), el.end());
      std::string s = "{";
      for (size_t t = 0; t < el.size(); ++t) { if (t) s += ", "; s += el[t]; }
      return s + "}";
    }
    case K::Fcn: {
      if (is_record(v)) {
        std::vector<std::pair<std::string, std::string>> fs;
        for (size_t t = 0; t < v->a.size(); ++t) fs.push_back({N.str[v->a[t]->i], show(v->b[t])});
        std::sort(fs.begin(), fs.end());
        std::string s = "[";
        for (size_t t = 0; t < fs.size(); ++t) { if (t) s += ", "; s += fs[t].first + " |-> " + fs[t].second; }
        return s + "]";
      }
      std::vector<std::pair<std::string, std::string>> fs;
      for (size_t t = 0; t < v->a.size(); ++t) fs.push_back({show(v->a[t]), show(v->b[t])});
      std::sort(fs.begin(), fs.end());
      std::string s = "(";
      for (size_t t = 0; t < fs.size(); ++t) { if (t) s += " @@ "; s += fs[t].first + " :> " + fs[t].second; }
      return s + ")";
    }
  }
  return "?";
}

// ---------------------------------------------------------------- permutation of model values
// Applies a permutation of model values (map mv id -> mv id) everywhere inside v.
inline V permute(const V& v, const std::vector<int>& perm) {
  switch (v->k) {
    case K::MV: return (v->i < (int64_t)perm.size() && perm[v->i] >= 0) ? mk(K::MV, perm[v->i]) : v;
    case K::Bool: case K::Int: case K::Str: return v;
    case K::Seq: { std::vector<V> xs; for (auto& x : v->a) xs.push_back(permute(x, perm)); return seq(std::move(xs)); }
    case K::Set: { std::vector<V> xs; for (auto& x : v->a) xs.push_back(permute(x, perm)); return set(std::move(xs)); }
    case K::Fcn: {
      std::vector<V> ks, vs;
      for (auto& x : v->a) ks.push_back(permute(x, perm));
      for (auto& x : v->b) vs.push_back(permute(x, perm));
      return fcn(std::move(ks), std::move(vs));
    }
  }
  return v;
}

}  // namespace tla
