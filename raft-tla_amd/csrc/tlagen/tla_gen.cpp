// tla_gen.cpp — TLA+ (SANY subset) to C++ over tlv.h; see tla_gen.h for the semantics.
#include "tla_gen.h"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <functional>
#include <map>
#include <set>
#include <sstream>

#include "../../../include/raftmc.h"

namespace rmc {
namespace tlagen {

namespace {

struct Sym {
  enum Kind { Val, LetOp, RecFn } kind = Val;
  std::string cxx;                 // Val: handle expression; LetOp: lambda name; RecFn: how to call it (see rec_call)
  std::shared_ptr<Def> def;        // LetOp
  std::shared_ptr<std::vector<std::pair<std::string, Sym>>> scope;   // LetOp: scope at its definition
};
typedef std::vector<std::pair<std::string, Sym>> Scope;

const Sym* find(const Scope& sc, const std::string& n) {
  for (auto it = sc.rbegin(); it != sc.rend(); ++it) if (it->first == n) return &it->second;
  return nullptr;
}

std::string cstr(const std::string& s) {
  std::string o = "\"";
  for (char ch : s) { if (ch == '"' || ch == '\\') o += '\\'; if (ch == '\n') { o += "\\n"; continue; } o += ch; }
  return o + "\"";
}

struct Gen {
  const Program& P;
  const CfgFile& cfg;
  std::map<std::string, int> var_idx, const_idx;
  std::map<std::string, int> atom_ids;
  std::vector<std::string> atoms;
  std::vector<std::string> actions;
  std::map<std::string, int> action_ids;
  std::map<std::string, std::string> op_fn;       // global op -> C++ function name
  std::vector<std::string> fn_protos, fn_bodies;
  std::map<std::string, int> level_memo;          // 0 pure, 1 action
  std::map<std::string, int> free_memo;           // 1: the definition reads no state variable
  std::map<std::string, int> cache_slot;          // state-free 0-arity definitions: c.k slot
  std::vector<std::string> cache_init;            // their evaluation, in dependency order
  int uid = 0;
  bool init_mode = false;

  Gen(const Program& p, const CfgFile& c) : P(p), cfg(c) {
    for (size_t i = 0; i < P.variables.size(); ++i) var_idx[P.variables[i]] = (int)i;
    for (size_t i = 0; i < P.constants.size(); ++i) const_idx[P.constants[i]] = (int)i;
  }

  std::string fresh(const char* p) { return std::string(p) + std::to_string(uid++); }
  [[noreturn]] void unsup(const Node& n, const std::string& what) {
    throw CfgError(MC_E_UNSUPPORTED, node_where(n) + ": " + what + " is outside the front end's subset");
  }
  int atom(const std::string& key, const std::string& text) {
    auto it = atom_ids.find(key);
    if (it != atom_ids.end()) return it->second;
    const int id = (int)atoms.size();
    atoms.push_back(text);
    atom_ids[key] = id;
    return id;
  }
  int str_atom(const std::string& s) { return atom("s:" + s, "\"" + s + "\""); }
  int mv_atom(const std::string& s) { return atom("m:" + s, s); }
  int action_id(const std::string& n) {
    auto it = action_ids.find(n);
    if (it != action_ids.end()) return it->second;
    action_ids[n] = (int)actions.size();
    actions.push_back(n);
    return (int)actions.size() - 1;
  }
  std::shared_ptr<Def> global(const std::string& n) {
    auto it = P.defs.find(n);
    return it == P.defs.end() ? nullptr : it->second;
  }
  const Def& body_of(const std::shared_ptr<Def>& d, const Node& at) {
    if (!d->body) throw CfgError(MC_E_UNSUPPORTED, node_where(at) + ": definition " + d->name + " does not parse: " + d->error);
    return *d;
  }

  static int arity_of(const Def& d, size_t i) { return i < d.arity.size() ? d.arity[i] : 0; }
  static bool higher_order(const Def& d) {
    for (size_t i = 0; i < d.params.size(); ++i) if (arity_of(d, i)) return true;
    return false;
  }

  // ---- level: does a definition (transitively) contain primes / UNCHANGED?
  bool has_action(const NP& e, std::set<std::string>& visiting) {
    if (!e) return false;
    if (e->k == K::Prime || e->k == K::Unchanged) return true;
    if (e->k == K::Ident || e->k == K::OpApp) {
      auto d = global(e->s);
      if (d && d->body && is_action(d, visiting)) return true;
    }
    for (auto& c : e->a) if (has_action(c, visiting)) return true;
    for (auto& b : e->binds) if (has_action(b.set, visiting)) return true;
    for (auto& u : e->ups) { if (has_action(u.rhs, visiting)) return true; for (auto& s : u.path) if (has_action(s.idx, visiting)) return true; }
    for (auto& d : e->defs) if (has_action(d->body, visiting)) return true;
    return false;
  }
  bool is_action(const std::shared_ptr<Def>& d, std::set<std::string>& visiting) {
    auto it = level_memo.find(d->name);
    if (it != level_memo.end()) return it->second != 0;
    if (visiting.count(d->name)) return false;
    visiting.insert(d->name);
    const bool r = has_action(d->body, visiting);
    visiting.erase(d->name);
    level_memo[d->name] = r;
    return r;
  }
  bool is_action(const std::shared_ptr<Def>& d) { std::set<std::string> v; return d->body && is_action(d, v); }

  // a definition that reads no state variable (transitively) has one value per model: it is
  // evaluated once per lane (init_consts) instead of at every use (raft's Quorum: SUBSET Server)
  bool reads_state(const NP& e, std::set<std::string>& visiting) {
    if (!e) return false;
    if (e->k == K::Prime || e->k == K::Unchanged || e->k == K::Enabled || e->k == K::Temporal) return true;
    if (e->k == K::Ident || e->k == K::OpApp || e->k == K::Binary) {
      if (var_idx.count(e->s)) return true;
      auto d = global(e->s);
      if (d && (!d->body || !state_free(d, visiting))) return true;
    }
    for (auto& c : e->a) if (reads_state(c, visiting)) return true;
    for (auto& b : e->binds) if (reads_state(b.set, visiting)) return true;
    for (auto& u : e->ups) { if (reads_state(u.rhs, visiting)) return true; for (auto& st : u.path) if (reads_state(st.idx, visiting)) return true; }
    for (auto& d : e->defs) if (reads_state(d->body, visiting)) return true;
    return false;
  }
  bool state_free(const std::shared_ptr<Def>& d, std::set<std::string>& visiting) {
    auto it = free_memo.find(d->name);
    if (it != free_memo.end()) return it->second != 0;
    if (visiting.count(d->name)) return false;
    visiting.insert(d->name);
    const bool r = d->body && !reads_state(d->body, visiting);
    visiting.erase(d->name);
    free_memo[d->name] = r;
    return r;
  }

  // the state variables an expression reads, a bit per variable, transitively through the
  // definitions it uses; all bits for anything the analysis does not follow (primes, temporal
  // operators, a definition without a body).  Names are matched without scopes, so a bound name
  // that shadows a variable or definition only adds bits (conservative).  The kernels skip a
  // constraint or invariant whose variables a successor left unchanged: its parent, which is in
  // the model and satisfies every invariant, gives the same value.
  std::map<std::string, unsigned long long> mask_memo;
  bool mask_cycle = false;
  unsigned long long var_mask(const NP& e, std::set<std::string>& visiting) {
    if (!e) return 0;
    if (e->k == K::Prime || e->k == K::Unchanged || e->k == K::Enabled || e->k == K::Temporal) return ~0ull;
    unsigned long long m = 0;
    if (e->k == K::Ident || e->k == K::OpApp || e->k == K::Binary) {
      auto v = var_idx.find(e->s);
      if (v != var_idx.end()) m |= 1ull << v->second;
      else if (auto d = global(e->s)) {
        if (!d->body) return ~0ull;
        m |= def_mask(d, visiting);
      }
    }
    for (auto& c : e->a) m |= var_mask(c, visiting);
    for (auto& b : e->binds) m |= var_mask(b.set, visiting);
    for (auto& u : e->ups) { m |= var_mask(u.rhs, visiting); for (auto& st : u.path) m |= var_mask(st.idx, visiting); }
    for (auto& d : e->defs) m |= var_mask(d->body, visiting);
    return m;
  }
  unsigned long long def_mask(const std::shared_ptr<Def>& d, std::set<std::string>& visiting) {
    auto it = mask_memo.find(d->name);
    if (it != mask_memo.end()) return it->second;
    if (visiting.count(d->name)) { mask_cycle = true; return 0; }   // the enclosing visit covers the rest
    const bool outer = visiting.empty();
    if (outer) mask_cycle = false;
    visiting.insert(d->name);
    const unsigned long long m = var_mask(d->body, visiting);
    visiting.erase(d->name);
    if (!mask_cycle || outer) mask_memo[d->name] = m;   // a partial mask inside a cycle is not kept
    return m;
  }
  std::string mask_of(const std::shared_ptr<Def>& d) {
    std::set<std::string> visiting;
    mask_cycle = false;
    visiting.insert(d->name);
    const unsigned long long m = var_mask(d->body, visiting);
    char b[32];
    std::snprintf(b, sizeof b, "0x%llxull", m);
    return b;
  }

  // ---- a global operator as a C++ function (emitted once)
  std::string op_function(const std::shared_ptr<Def>& d, const Node& at) {
    auto it = op_fn.find(d->name);
    if (it != op_fn.end()) return it->second;
    body_of(d, at);
    std::string fn = "op_" + std::to_string(op_fn.size()) + "_";
    for (char ch : d->name) fn += std::isalnum((unsigned char)ch) ? ch : '_';
    op_fn[d->name] = fn;
    std::string sig = "TLV_NI u32 " + fn + "(Cx& c";
    Scope sc;
    for (size_t i = 0; i < d->params.size(); ++i) {
      sig += ", u32 p" + std::to_string(i);
      Sym s; s.cxx = "p" + std::to_string(i);
      sc.push_back({d->params[i], s});
    }
    sig += ")";
    const bool save = init_mode;
    init_mode = false;
    const std::string body = ex(d->body, sc);
    init_mode = save;
    fn_protos.push_back(sig + ";");
    if (recursive_op(d))   // a RECURSIVE operator (or one of a mutually recursive group): bounded like TLC's stack
      fn_bodies.push_back(sig + " {\n  Ar& A = *c.A; (void)A;\n  if (A.rdepth >= kMaxRecDepth) { A.err |= E_UNSUP; return 0u; }\n"
                          "  ++A.rdepth; const u32 r_ = " + body + ";\n  --A.rdepth; return r_;\n}\n");
    else
      fn_bodies.push_back(sig + " {\n  Ar& A = *c.A; (void)A;\n  return " + body + ";\n}\n");
    return fn;
  }

  // does a global operator reach itself through the global operators its body applies?
  std::map<std::string, bool> rec_memo;
  void reached(const NP& e, std::set<std::string>& seen) {
    if (!e) return;
    if (e->k == K::Ident || e->k == K::OpApp || e->k == K::Binary) {
      auto d = global(e->s);
      if (d && d->body && seen.insert(d->name).second) reached(d->body, seen);
    }
    for (auto& c : e->a) reached(c, seen);
    for (auto& b : e->binds) reached(b.set, seen);
    for (auto& u : e->ups) { reached(u.rhs, seen); for (auto& st : u.path) reached(st.idx, seen); }
    for (auto& d : e->defs) reached(d->body, seen);
  }
  bool recursive_op(const std::shared_ptr<Def>& d) {
    auto it = rec_memo.find(d->name);
    if (it != rec_memo.end()) return it->second;
    std::set<std::string> seen;
    reached(d->body, seen);
    return rec_memo[d->name] = seen.count(d->name) != 0;
  }

  // ---- recursive function definitions  f[x \in S] == e  whose body applies f (TypedBags' Sum:
  // LET DSum[S \in SUBSET DOMAIN f] == .. DSum[S \ {elt}] ..).  TLC evaluates them lazily, one
  // application at a time (never the whole function over S); so does the generated code: the
  // definition becomes a recursive C++ function of the argument, which checks that the argument
  // lies in the domain (TLC's error otherwise) and evaluates e with x bound to it.
  static bool mentions(const NP& e, const std::string& name) {
    if (!e) return false;
    if ((e->k == K::Ident || e->k == K::OpApp) && e->s == name) return true;
    for (auto& c : e->a) if (mentions(c, name)) return true;
    for (auto& b : e->binds) if (mentions(b.set, name)) return true;
    for (auto& u : e->ups) { if (mentions(u.rhs, name)) return true; for (auto& s : u.path) if (mentions(s.idx, name)) return true; }
    for (auto& d : e->defs) if (d->name != name && mentions(d->body, name)) return true;
    return false;
  }
  static bool recursive_fun(const Def& d) {
    return d.params.empty() && d.body && d.body->k == K::FunCons && mentions(d.body->a[0], d.name);
  }
  // the body of the recursive function as a C++ statement block over the argument `arg`: domain
  // check, then the value of e; `sc` must already map the function's name to its RecFn symbol
  std::string rec_body(const Def& d, Scope& sc, const std::string& arg) {
    const Node& fc = *d.body;
    if (fc.binds.size() != 1 || fc.binds[0].names.size() != 1 || fc.binds[0].tuple) unsup(fc, "recursive function " + d.name + " of more than one argument");
    Scope inner = sc;
    Sym x; x.cxx = arg;
    inner.push_back({fc.binds[0].names[0], x});
    auto in = std::make_shared<Node>(fc);   // arg \in S, by the membership rules of binary()
    in->k = K::Binary; in->s = "\\in"; in->binds.clear();
    auto id = std::make_shared<Node>(fc);
    id->k = K::Ident; id->s = fc.binds[0].names[0]; id->a.clear(); id->binds.clear();
    in->a = {id, fc.binds[0].set};
    return "if (!truth(A, " + ex(in, inner) + ")) { A.err |= E_DOMAIN; return 0u; }\n"
           " if (A.rdepth >= kMaxRecDepth) { A.err |= E_UNSUP; return 0u; }\n"
           " ++A.rdepth; const u32 r_ = " + ex(fc.a[0], inner) + ";\n --A.rdepth; return r_;\n";
  }
  std::string rec_call(const Sym& s, const std::string& arg) {
    return s.cxx + "(" + s.cxx + ", " + arg + ")";   // a generic lambda that receives itself
  }

  std::string rec_fun_function(const std::shared_ptr<Def>& d, const Node& at) {   // a global one, emitted once
    auto it = op_fn.find(d->name);
    if (it != op_fn.end()) return it->second;
    body_of(d, at);
    std::string fn = "rf_" + std::to_string(op_fn.size()) + "_";
    for (char ch : d->name) fn += std::isalnum((unsigned char)ch) ? ch : '_';
    op_fn[d->name] = fn;
    const std::string sig = "TLV_NI u32 " + fn + "(Cx& c, u32 a0)";
    fn_protos.push_back(sig + ";");
    const bool save = init_mode;
    init_mode = false;
    Scope sc;
    const std::string body = rec_body(*d, sc, "a0");
    init_mode = save;
    fn_bodies.push_back(sig + " {\n  Ar& A = *c.A; (void)A;\n  " + body + "}\n");
    return fn;
  }

  std::string let_defs(const NP& e, Scope& sc) {   // C++ lambdas of a LET's definitions
    std::string out;
    for (auto& d : e->defs) {
      if (!d->body) unsup(*e, "LET definition " + d->name + " (" + d->error + ")");
      if (recursive_fun(*d)) {
        Sym s; s.kind = Sym::RecFn; s.def = d; s.cxx = fresh("R");
        sc.push_back({d->name, s});
        Scope inner = sc;
        // inside its own body the function calls itself through the lambda's first parameter
        Sym self = s; self.cxx = fresh("self");
        inner.push_back({d->name, self});
        const std::string arg = fresh("a");
        out += "auto " + s.cxx + " = [&](auto& " + self.cxx + ", u32 " + arg + ") -> u32 {\n " + rec_body(*d, inner, arg) + "};\n";
        continue;
      }
      if (higher_order(*d)) unsup(*e, "LET operator " + d->name + " with an operator parameter");
      Sym s; s.kind = Sym::LetOp; s.def = d; s.cxx = fresh("L");
      s.scope = std::make_shared<Scope>(sc);   // recursion is outside the subset
      Scope inner = sc;
      std::string params;
      for (size_t i = 0; i < d->params.size(); ++i) {
        const std::string pn = fresh("q");
        params += (i ? ", u32 " : "u32 ") + pn;
        Sym ps; ps.cxx = pn;
        inner.push_back({d->params[i], ps});
      }
      out += "auto " + s.cxx + " = [&](" + params + ") -> u32 { return " + ex(d->body, inner) + "; };\n";
      sc.push_back({d->name, s});
    }
    return out;
  }

  std::string set_loop(const std::string& set, const std::string& elem, const std::string& body, bool restore_top) {
    const std::string S = fresh("S"), i = fresh("i"), n = fresh("n"), st = fresh("t");
    return "{ const u32 " + S + " = " + set + ";\n if (tg(A, " + S + ") != T_SET) A.err |= E_TYPE; else { u32 " + elem +
           " = first(" + S + ");\n for (u32 " + i + " = 0, " + n + " = count(A, " + S + "); " + i + " < " + n + "; ++" + i +
           ", " + elem + " = nextv(A, " + elem + ")) {\n" + (restore_top ? " const u32 " + st + " = A.top;\n" : "") + body +
           (restore_top ? " A.top = " + st + ";\n" : "") + " } } }\n";
  }

  // nested loops over binds; `inner` is generated with the bound names in scope
  std::string bind_loops(const std::vector<Bind>& bs, size_t bi, size_t ni, Scope& sc, bool restore,
                         const std::function<std::string(Scope&)>& inner) {
    if (bi == bs.size()) return inner(sc);
    const Bind& b = bs[bi];
    if (b.tuple) {   // <<a, b>> \in S: each element of S is a tuple of exactly that many components
      const std::string el = fresh("e");
      Scope s2 = sc;
      std::string hd = " if (tg(A, " + el + ") != T_SEQ || count(A, " + el + ") != " + std::to_string(b.names.size()) + "u) { A.err |= E_TYPE; } else {\n";
      for (size_t i = 0; i < b.names.size(); ++i) {
        Sym v; v.cxx = fresh("c");
        hd += " const u32 " + v.cxx + " = apply(A, " + el + ", mk_int(A, " + std::to_string(i + 1) + "));\n";
        s2.push_back({b.names[i], v});
      }
      return set_loop(ex(b.set, sc), el, hd + bind_loops(bs, bi + 1, 0, s2, restore, inner) + " }\n", restore);
    }
    // the set of a multi-name bind is evaluated once
    if (ni == 0 && b.names.size() > 1) {
      const std::string sv = fresh("B");
      Scope s2 = sc;
      Sym ss; ss.cxx = sv;
      s2.push_back({"\x01set" + std::to_string(bi), ss});
      return "{ const u32 " + sv + " = " + ex(b.set, sc) + ";\n" + bind_loops_named(bs, bi, 0, s2, restore, inner, sv) + "}\n";
    }
    return bind_loops_named(bs, bi, ni, sc, restore, inner, ex(b.set, sc));
  }
  std::string bind_loops_named(const std::vector<Bind>& bs, size_t bi, size_t ni, Scope& sc, bool restore,
                               const std::function<std::string(Scope&)>& inner, const std::string& setx) {
    const Bind& b = bs[bi];
    const std::string el = fresh("e");
    Scope s2 = sc;
    Sym s; s.cxx = el;
    s2.push_back({b.names[ni], s});
    std::string body;
    if (ni + 1 < b.names.size()) body = bind_loops_named(bs, bi, ni + 1, s2, restore, inner, setx);
    else body = bind_loops(bs, bi + 1, 0, s2, restore, inner);
    return set_loop(setx, el, body, restore);
  }

  // ---- outlining of large constructors: a sequence / set / record literal of many nodes (the
  // golden TLC traces pasted into tlc_membership/raft.tla:1201,1231 are ~2K nodes) built inline
  // would make one function larger than the short-branch range; each element then becomes a
  // function of its own, taking the bound values it reads as arguments
  static size_t node_count(const NP& e) {
    if (!e) return 0;
    size_t k = 1;
    for (auto& c : e->a) k += node_count(c);
    for (auto& b : e->binds) k += node_count(b.set);
    for (auto& u : e->ups) { k += node_count(u.rhs); for (auto& st : u.path) k += node_count(st.idx); }
    for (auto& d : e->defs) k += node_count(d->body);
    return k;
  }
  static bool has_at(const NP& e) {
    if (!e) return false;
    if (e->k == K::At) return true;
    for (auto& c : e->a) if (has_at(c)) return true;
    for (auto& b : e->binds) if (has_at(b.set)) return true;
    for (auto& u : e->ups) { if (has_at(u.rhs)) return true; for (auto& st : u.path) if (has_at(st.idx)) return true; }
    for (auto& d : e->defs) if (has_at(d->body)) return true;
    return false;
  }
  static constexpr size_t kOutlineCtor = 160, kOutlineElem = 8;   // constructor / element node counts
  std::string element(const NP& e, Scope& sc, bool big) {
    if (!big || node_count(e) < kOutlineElem || has_at(e)) return ex(e, sc);
    std::vector<std::pair<std::string, const Sym*>> used;   // innermost binding of each name e reads
    std::set<std::string> seen;
    for (auto it = sc.rbegin(); it != sc.rend(); ++it) {
      if (!seen.insert(it->first).second || !mentions(e, it->first)) continue;
      if (it->second.kind != Sym::Val) return ex(e, sc);   // a LET operator / recursive function: inline
      used.push_back({it->first, &it->second});
    }
    const std::string fn = "lit_" + std::to_string(fn_protos.size());
    std::string sig = "TLV_NI u32 " + fn + "(Cx& c", call = fn + "(c";
    Scope inner;
    for (size_t i = 0; i < used.size(); ++i) {
      Sym v = *used[i].second;
      const std::string q = "q" + std::to_string(i);
      sig += ", u32 " + q;
      call += ", " + v.cxx;
      v.cxx = q;
      inner.push_back({used[i].first, v});
    }
    sig += ")";
    const std::string body = ex(e, inner);
    fn_protos.push_back(sig + ";");
    fn_bodies.push_back(sig + " {\n  Ar& A = *c.A; (void)A;\n  return " + body + ";\n}\n");
    return call + ")";
  }

  // ---- expressions: a C++ expression yielding a value handle
  std::string ex(const NP& e, Scope& sc) {
    const Node& n = *e;
    switch (n.k) {
      case K::Num: return "mk_int(A, " + std::to_string(n.n) + "LL)";
      case K::Str: return "mk_atom(A, " + std::to_string(str_atom(n.s)) + "u)";
      case K::Bool: return n.n ? "2u" : "0u";
      case K::At: {
        const Sym* s = find(sc, "@");
        if (!s) unsup(n, "@ outside EXCEPT");
        return s->cxx;
      }
      case K::Ident: return ident(n, sc, {});
      case K::OpApp: {
        if (n.s == "Cardinality" && n.a.size() == 1 && n.a[0]->k == K::Unary && n.a[0]->s == "DOMAIN" && !find(sc, n.s) && !global(n.s))
          return "mk_int(A, coll_card(A, " + ex(n.a[0]->a[0], sc) + "))";
        if (!find(sc, n.s)) {
          if (auto d = global(n.s)) { if (higher_order(*d)) return apply_higher(n, sc, *d); }
          else if (n.s == "SelectSeq") return select_seq(n, sc);
        }
        std::vector<std::string> args;
        for (auto& a : n.a) args.push_back(ex(a, sc));
        return ident(n, sc, args);
      }
      case K::Lambda: unsup(n, "LAMBDA other than as an operator argument");
      case K::Prime: {
        if (n.a[0]->k != K::Ident || !var_idx.count(n.a[0]->s)) unsup(n, "priming a non-variable expression");
        const std::string X = std::to_string(var_idx[n.a[0]->s]);
        return "(((c.asg >> " + X + ") & 1ull) ? c.nxt[" + X + "] : (A.err |= E_ASSIGN, 0u))";
      }
      case K::Unary: {
        const std::string x = ex(n.a[0], sc);
        if (n.s == "~") return "mk_bool(!truth(A, " + x + "))";
        if (n.s == "-") return "mk_int(A, -ival(A, " + x + "))";
        if (n.s == "DOMAIN") return "dom(A, " + x + ")";
        if (n.s == "SUBSET") return "powerset(A, " + x + ")";
        if (n.s == "UNION") return "union_all(A, " + x + ")";
        unsup(n, "operator " + n.s);
      }
      case K::Binary: return binary(n, sc);
      case K::And: case K::Or: {
        std::string o = "mk_bool(";
        for (size_t i = 0; i < n.a.size(); ++i) o += (i ? (n.k == K::And ? " && " : " || ") : "") + std::string("truth(A, ") + ex(n.a[i], sc) + ")";
        return o + ")";
      }
      case K::If:
        return "(truth(A, " + ex(n.a[0], sc) + ") ? " + ex(n.a[1], sc) + " : " + ex(n.a[2], sc) + ")";
      case K::Case: {
        std::string o, close;
        for (size_t i = 0; i < n.a.size(); i += 2) {
          if (!n.a[i]) { o += ex(n.a[i + 1], sc); close += ""; goto done; }
          o += "(truth(A, " + ex(n.a[i], sc) + ") ? " + ex(n.a[i + 1], sc) + " : ";
          close += ")";
        }
        o += "(A.err |= E_DOMAIN, 0u)";
      done:
        return o + close;
      }
      case K::Let: {
        Scope s2 = sc;
        const std::string defs = let_defs(e, s2);
        return "[&]() -> u32 {\n" + defs + "return " + ex(n.a[0], s2) + ";\n}()";
      }
      case K::Forall: case K::Exists: {
        const bool all = n.k == K::Forall;
        Scope s2 = sc;
        const std::string loops = bind_loops(n.binds, 0, 0, s2, true, [&](Scope& s3) {
          return std::string(" if (") + (all ? "!" : "") + "truth(A, " + ex(n.a[0], s3) + ")) return " + (all ? "0u" : "2u") + ";\n";
        });
        return "[&]() -> u32 {\n" + loops + " return " + (all ? "2u" : "0u") + ";\n}()";
      }
      case K::Choose: {
        Scope s2 = sc;
        const std::string loops = bind_loops(n.binds, 0, 0, s2, true, [&](Scope& s3) {
          return " if (truth(A, " + ex(n.a[0], s3) + ")) return " + find(s3, n.binds[0].names[0])->cxx + ";\n";
        });
        return "[&]() -> u32 {\n" + loops + " A.err |= E_CHOOSE; return 0u;\n}()";
      }
      case K::SetEnum: {
        if (n.a.empty()) return "set_end(A, A.htop)";
        const std::string m = fresh("m");
        const bool big = node_count(e) >= kOutlineCtor;
        std::string o = "[&]() -> u32 { const u32 " + m + " = A.htop;\n";
        for (auto& a : n.a) o += " hpush(A, " + element(a, sc, big) + ");\n";
        return o + " return set_end(A, " + m + ");\n}()";
      }
      case K::Tuple: {
        const std::string m = fresh("m");
        const bool big = node_count(e) >= kOutlineCtor;
        std::string o = "[&]() -> u32 { const u32 " + m + " = A.htop;\n";
        for (auto& a : n.a) o += " hpush(A, " + element(a, sc, big) + ");\n";
        return o + " return seq_end(A, " + m + ");\n}()";
      }
      case K::SetFilter: case K::SetMap: {
        const std::string m = fresh("m");
        Scope s2 = sc;
        const bool filt = n.k == K::SetFilter;
        if (filt && n.binds[0].tuple) unsup(n, "a set filter over a tuple binding");
        const std::string loops = bind_loops(n.binds, 0, 0, s2, false, [&](Scope& s3) {
          if (filt) return " if (truth(A, " + ex(n.a[0], s3) + ")) hpush(A, " + find(s3, n.binds[0].names[0])->cxx + ");\n";
          return " hpush(A, " + ex(n.a[0], s3) + ");\n";
        });
        return "[&]() -> u32 { const u32 " + m + " = A.htop;\n" + loops + " return set_end(A, " + m + ");\n}()";
      }
      case K::FunCons: {
        for (auto& b : n.binds) if (b.tuple) unsup(n, "a function constructor over a tuple binding");
        const std::string m = fresh("m");
        Scope s2 = sc;
        const std::string loops = bind_loops(n.binds, 0, 0, s2, false, [&](Scope& s3) {
          std::vector<std::string> names;
          for (auto& b : n.binds) for (auto& nm : b.names) names.push_back(find(s3, nm)->cxx);
          std::string key = names[0];
          if (names.size() > 1) {
            const std::string km = fresh("m");
            key = "[&]() -> u32 { const u32 " + km + " = A.htop;";
            for (auto& x : names) key += " hpush(A, " + x + ");";
            key += " return seq_end(A, " + km + "); }()";
          }
          const std::string kv = fresh("k");
          return " { const u32 " + kv + " = " + key + "; const u32 v_ = " + ex(n.a[0], s3) + "; hpush(A, " + kv + "); hpush(A, v_); }\n";
        });
        return "[&]() -> u32 { const u32 " + m + " = A.htop;\n" + loops + " return fun_end(A, " + m + ");\n}()";
      }
      case K::FunApp: {
        if (n.a[0]->k == K::Ident) {
          const Sym* s = find(sc, n.a[0]->s);
          if (s && s->kind == Sym::RecFn) return rec_call(*s, ex(n.a[1], sc));
          if (!s) if (auto d = global(n.a[0]->s)) if (recursive_fun(*d)) return rec_fun_function(d, n) + "(c, " + ex(n.a[1], sc) + ")";
        }
        return "apply(A, " + ex(n.a[0], sc) + ", " + ex(n.a[1], sc) + ")";
      }
      case K::Dot: return "apply(A, " + ex(n.a[0], sc) + ", mk_atom(A, " + std::to_string(str_atom(n.s)) + "u))";
      case K::FunSet: return "fun_set(A, " + ex(n.a[0], sc) + ", " + ex(n.a[1], sc) + ")";
      case K::RecordSet: {
        const std::string m = fresh("m");
        std::string o = "[&]() -> u32 { const u32 " + m + " = A.htop;\n";
        for (size_t i = 0; i < n.fields.size(); ++i) {
          const std::string kv = fresh("k");
          o += " { const u32 " + kv + " = mk_atom(A, " + std::to_string(str_atom(n.fields[i])) + "u); const u32 v_ = " + ex(n.a[i], sc) +
               "; hpush(A, " + kv + "); hpush(A, v_); }\n";
        }
        return o + " return rec_set(A, " + m + ");\n}()";
      }
      case K::Record: {
        const std::string m = fresh("m");
        const bool big = node_count(e) >= kOutlineCtor;
        std::string o = "[&]() -> u32 { const u32 " + m + " = A.htop;\n";
        for (size_t i = 0; i < n.fields.size(); ++i) {
          const std::string kv = fresh("k");
          o += " { const u32 " + kv + " = mk_atom(A, " + std::to_string(str_atom(n.fields[i])) + "u); const u32 v_ = " +
               element(n.a[i], sc, big) + "; hpush(A, " + kv + "); hpush(A, v_); }\n";
        }
        return o + " return fun_end(A, " + m + ");\n}()";
      }
      case K::Except: {
        const std::string F = fresh("F");
        std::string o = "[&]() -> u32 { u32 " + F + " = " + ex(n.a[0], sc) + ";\n";
        for (auto& u : n.ups) o += except_update(F, u, 0, sc, F);
        return o + " return " + F + ";\n}()";
      }
      default: break;
    }
    unsup(n, "this expression form");
  }

  // [F EXCEPT !p1..pk = rhs]: F_new = except(F, p1, [F[p1] EXCEPT !p2..pk = rhs]); keys outside the domain leave F unchanged
  std::string except_update(const std::string& F, const Update& u, size_t i, Scope& sc, const std::string& target) {
    const PathStep& st = u.path[i];
    const std::string key = fresh("x"), old = fresh("o");
    std::string o = "{ const u32 " + key + " = " + (st.field ? "mk_atom(A, " + std::to_string(str_atom(st.name)) + "u)" : ex(st.idx, sc)) +
                    ";\n const u32 " + old + " = lookup(A, " + F + ", " + key + ");\n if (" + old + ") {\n";
    if (i + 1 == u.path.size()) {
      Scope s2 = sc;
      Sym at; at.cxx = old;
      s2.push_back({"@", at});
      o += " " + target + " = except(A, " + F + ", " + key + ", " + ex(u.rhs, s2) + ");\n";
    } else {
      const std::string sub = fresh("F");
      o += " u32 " + sub + " = " + old + ";\n" + except_update(old, u, i + 1, sc, sub) + " " + target + " = except(A, " + F + ", " +
           key + ", " + sub + ");\n";
    }
    return o + " } }\n";
  }

  // Sets a membership test should not build: function sets, record sets, Seq(S), Nat / Int, and unions,
  // filters, SUBSET and definitions of them (TypeOK-style predicates: raft_dricketts.tla:482-492)
  bool lazy_set(const NP& r, int depth = 0) {
    if (!r || depth > 32) return false;
    switch (r->k) {
      case K::FunSet: case K::RecordSet: return true;
      case K::Ident:
        if (r->s == "Nat" || r->s == "Int") return !global(r->s);
        if (auto d = global(r->s)) return d->params.empty() && d->body && !recursive_fun(*d) && lazy_set(d->body, depth + 1);
        return false;
      case K::OpApp: return r->s == "Seq" && r->a.size() == 1 && !global(r->s);
      case K::Binary: return r->s == "\\cup" && (lazy_set(r->a[0], depth + 1) || lazy_set(r->a[1], depth + 1));
      case K::SetFilter: return r->binds.size() == 1 && r->binds[0].names.size() == 1 && lazy_set(r->binds[0].set, depth + 1);
      case K::Unary: return r->s == "SUBSET" && lazy_set(r->a[0], depth + 1);
      default: return false;
    }
  }
  // the elements of a set or sequence value xv, one at a time as `el` (a loop statement)
  std::string coll_loop(const std::string& xv, const std::string& el, const std::string& body) {
    const std::string i = fresh("i"), n = fresh("n"), st = fresh("t");
    return "{ u32 " + el + " = first(" + xv + ");\n for (u32 " + i + " = 0, " + n + " = count(A, " + xv + "); " + i + " < " + n + "; ++" +
           i + ", " + el + " = nextv(A, " + el + ")) {\n const u32 " + st + " = A.top;\n" + body + " A.top = " + st + ";\n } }\n";
  }
  // x \in r as a C++ bool expression, x an evaluated value handle (a C++ name).  The lazy_set forms are
  // tested without being built, as TLC evaluates such a membership (x \in [S -> Nat] works although
  // [S -> Nat] is infinite): a function set by its domain and then every value against the range, a
  // record set field by field, Seq(S) element by element, a union by either side, a filter by its base
  // set and predicate, SUBSET S element by element, a definition by its body
  std::string member_of(const std::string& xv, const NP& r, Scope& sc, int depth = 0) {
    if (r->k == K::Ident && !find(sc, r->s) && !global(r->s)) {
      if (r->s == "Nat") return "(tg(A, " + xv + ") == T_INT && ival(A, " + xv + ") >= 0)";
      if (r->s == "Int") return "(tg(A, " + xv + ") == T_INT)";
    }
    if (depth < 32 && lazy_set(r)) {
      if (r->k == K::Ident && !find(sc, r->s)) {   // a definition: its body, in the module's scope
        Scope top;
        return member_of(xv, global(r->s)->body, top, depth + 1);
      }
      if (r->k == K::Binary && r->s == "\\cup")
        return "(" + member_of(xv, r->a[0], sc, depth + 1) + " || " + member_of(xv, r->a[1], sc, depth + 1) + ")";
      if (r->k == K::SetFilter) {
        Scope s2 = sc;
        Sym b; b.cxx = xv;
        s2.push_back({r->binds[0].names[0], b});
        return "(" + member_of(xv, r->binds[0].set, sc, depth + 1) + " && truth(A, " + ex(r->a[0], s2) + "))";
      }
      if (r->k == K::OpApp && r->s == "Seq") {
        const std::string el = fresh("e");
        return "[&]() -> bool { if (tg(A, " + xv + ") != T_SEQ) return false;\n" +
               coll_loop(xv, el, " if (!(" + member_of(el, r->a[0], sc, depth + 1) + ")) return false;\n") + " return true; }()";
      }
      if (r->k == K::Unary && r->s == "SUBSET") {
        const std::string el = fresh("e");
        return "[&]() -> bool { if (tg(A, " + xv + ") != T_SET) return false;\n" +
               coll_loop(xv, el, " if (!(" + member_of(el, r->a[0], sc, depth + 1) + ")) return false;\n") + " return true; }()";
      }
    }
    if (r->k == K::Unary && r->s == "DOMAIN") return "in_dom(A, " + ex(r->a[0], sc) + ", " + xv + ")";
    if (r->k == K::Unary && r->s == "SUBSET") return "(tg(A, " + xv + ") == T_SET && set_subseteq(A, " + xv + ", " + ex(r->a[0], sc) + "))";
    if (r->k == K::Binary && r->s == "..")
      return "[&]() -> bool { if (tg(A, " + xv + ") != T_INT) return false; const i64 v_ = ival(A, " + xv + "); return v_ >= ival(A, " +
             ex(r->a[0], sc) + ") && v_ <= ival(A, " + ex(r->a[1], sc) + "); }()";
    if (r->k == K::FunSet) {   // [S -> T]: a function (or sequence) with domain S and every value in T
      const std::string k = fresh("e"), v = fresh("v");
      const std::string body = " { const u32 " + v + " = apply(A, " + xv + ", " + k + "); if (!(" + member_of(v, r->a[1], sc, depth + 1) +
                               ")) return false; }\n";
      return "[&]() -> bool { const u32 t_ = tg(A, " + xv + "); if (t_ != T_FUN && t_ != T_SEQ) return false;\n"
             " if (!eqv(A, dom(A, " + xv + "), " + ex(r->a[0], sc) + ")) return false;\n" +
             set_loop("dom(A, " + xv + ")", k, body, true) + " return true; }()";
    }
    if (r->k == K::RecordSet) {   // [f1 : S1, ...]: a record with exactly these fields, each in its set
      std::string o = "[&]() -> bool { if (tg(A, " + xv + ") != T_FUN || coll_card(A, " + xv + ") != " +
                      std::to_string(r->fields.size()) + "u) return false;\n";
      for (size_t i = 0; i < r->fields.size(); ++i) {
        const std::string key = "mk_atom(A, " + std::to_string(str_atom(r->fields[i])) + "u)", v = fresh("v");
        o += " { const u32 k_ = " + key + "; if (!in_dom(A, " + xv + ", k_)) return false; const u32 " + v + " = apply(A, " + xv +
             ", k_); if (!(" + member_of(v, r->a[i], sc, depth + 1) + ")) return false; }\n";
      }
      return o + " return true; }()";
    }
    return "set_in(A, " + xv + ", " + ex(r, sc) + ")";
  }

  std::string binary(const Node& n, Scope& sc) {
    const std::string& op = n.s;
    if (op == "\\X") {   // S1 \X .. \X Sk: the set of k-tuples
      std::string o = "[&]() -> u32 {\n";
      std::vector<std::string> sets, els;
      for (auto& a : n.a) { sets.push_back(fresh("S")); els.push_back(fresh("e")); o += " const u32 " + sets.back() + " = " + ex(a, sc) + ";\n"; }
      const std::string m = fresh("m"), tm = fresh("m");
      std::string body = " { const u32 " + tm + " = A.htop;";
      for (auto& e : els) body += " hpush(A, " + e + ");";
      body += " const u32 t_ = seq_end(A, " + tm + "); hpush(A, t_); }\n";
      for (size_t i = sets.size(); i-- > 0;) body = set_loop(sets[i], els[i], body, false);
      return o + " const u32 " + m + " = A.htop;\n" + body + " return set_end(A, " + m + ");\n}()";
    }
    const NP& l = n.a[0];
    const NP& r = n.a[1];
    if (op == "\\subseteq" && lazy_set(r)) {   // x \subseteq S: every element of x in S (S never built)
      const std::string xv = fresh("x"), el = fresh("e");
      return "[&]() -> u32 { const u32 " + xv + " = " + ex(l, sc) + "; if (tg(A, " + xv + ") != T_SET) { A.err |= E_TYPE; return 0u; }\n" +
             coll_loop(xv, el, " if (!(" + member_of(el, r, sc) + ")) return 0u;\n") + " return 2u; }()";
    }
    if ((op == "\\in" || op == "\\notin") && lazy_set(r) && !(r->k == K::Ident && (r->s == "Nat" || r->s == "Int"))) {
      const std::string xv = fresh("x");
      return "[&]() -> u32 { const u32 " + xv + " = " + ex(l, sc) + "; return mk_bool(" + (op == "\\notin" ? "!" : "") +
             member_of(xv, r, sc) + "); }()";
    }
    if (op == "\\in" || op == "\\notin") {
      const std::string neg = op == "\\notin" ? "!" : "";
      if (r->k == K::Ident && !find(sc, r->s) && !global(r->s)) {
        if (r->s == "Nat") return "[&]() -> u32 { const u32 x_ = " + ex(l, sc) + "; return mk_bool(" + neg + "(tg(A, x_) == T_INT && ival(A, x_) >= 0)); }()";
        if (r->s == "Int") return "mk_bool(" + neg + "(tg(A, " + ex(l, sc) + ") == T_INT))";
      }
      if (r->k == K::Unary && r->s == "DOMAIN") return "mk_bool(" + neg + "in_dom(A, " + ex(r->a[0], sc) + ", " + ex(l, sc) + "))";
      if (r->k == K::Unary && r->s == "SUBSET")   // x \in SUBSET S  <=>  x is a set and x \subseteq S (no 2^|S| powerset)
        return "[&]() -> u32 { const u32 x_ = " + ex(l, sc) + "; return mk_bool(" + neg + "(tg(A, x_) == T_SET && set_subseteq(A, x_, " +
               ex(r->a[0], sc) + "))); }()";
      if (r->k == K::Binary && r->s == "..")
        return "[&]() -> u32 { const u32 x_ = " + ex(l, sc) + "; const i64 lo_ = ival(A, " + ex(r->a[0], sc) + "), hi_ = ival(A, " +
               ex(r->a[1], sc) + "); if (tg(A, x_) != T_INT) return mk_bool(" + (neg.empty() ? "false" : "true") +
               "); const i64 v_ = ival(A, x_); return mk_bool(" + neg + "(v_ >= lo_ && v_ <= hi_)); }()";
      return "mk_bool(" + neg + "set_in(A, " + ex(l, sc) + ", " + ex(r, sc) + "))";
    }
    if (op == "=>") return "mk_bool(!truth(A, " + ex(l, sc) + ") || truth(A, " + ex(r, sc) + "))";
    if (op == "<=>") return "mk_bool(truth(A, " + ex(l, sc) + ") == truth(A, " + ex(r, sc) + "))";
    const std::string a = ex(l, sc), b = ex(r, sc);
    if (op == "=") return "mk_bool(eqv(A, " + a + ", " + b + "))";
    if (op == "/=") return "mk_bool(!eqv(A, " + a + ", " + b + "))";
    if (op == "<" || op == ">" || op == "<=" || op == ">=") return "mk_bool(ival(A, " + a + ") " + op + " ival(A, " + b + "))";
    if (op == "+" || op == "-" || op == "*") return "mk_int(A, ival(A, " + a + ") " + op + " ival(A, " + b + "))";
    if (op == "\\div") return "[&]() -> u32 { const i64 x_ = ival(A, " + a + "), y_ = ival(A, " + b + "); if (y_ <= 0) { A.err |= E_ARITH; return 0u; } i64 q_ = x_ / y_; if ((x_ % y_) < 0) --q_; return mk_int(A, q_); }()";
    if (op == "%") return "[&]() -> u32 { const i64 x_ = ival(A, " + a + "), y_ = ival(A, " + b + "); if (y_ <= 0) { A.err |= E_ARITH; return 0u; } i64 m_ = x_ % y_; if (m_ < 0) m_ += y_; return mk_int(A, m_); }()";
    if (op == "..") return "range(A, ival(A, " + a + "), ival(A, " + b + "))";
    if (op == "\\cup") return "set_union(A, " + a + ", " + b + ")";
    if (op == "\\cap") return "set_cap(A, " + a + ", " + b + ")";
    if (op == "\\") return "set_minus(A, " + a + ", " + b + ")";
    if (op == "\\subseteq") return "mk_bool(set_subseteq(A, " + a + ", " + b + "))";
    if (op == ":>") return "colon_gt(A, " + a + ", " + b + ")";
    if (op == "@@") return "atat(A, " + a + ", " + b + ")";
    if (op == "\\o") return "concat(A, " + a + ", " + b + ")";
    if (auto d = global(op)) {   // user-defined infix operator (TypedBags defines its own (+))
      const std::string fn = op_function(d, n);
      return fn + "(c, " + a + ", " + b + ")";
    }
    if (op == "(+)" || op == "(-)") return "bag_op(A, " + a + ", " + b + ", " + (op == "(+)" ? "true" : "false") + ")";   // Bags
    unsup(n, "operator " + op);
  }

  std::string ident(const Node& n, Scope& sc, const std::vector<std::string>& args) {
    const std::string& nm = n.s;
    if (const Sym* s = find(sc, nm)) {
      if (s->kind == Sym::RecFn) unsup(n, "a recursive function (" + nm + ") used other than by application");
      if (s->kind == Sym::Val) {
        if (!args.empty()) unsup(n, "applying a value as an operator");
        return s->cxx;
      }
      if (s->def && s->def->params.size() != args.size()) unsup(n, "operator " + nm + " with " + std::to_string(args.size()) + " arguments");
      std::string o = s->cxx + "(";
      for (size_t i = 0; i < args.size(); ++i) o += (i ? ", " : "") + args[i];
      return o + ")";
    }
    if (auto d = global(nm)) {
      if (recursive_fun(*d)) unsup(n, "a recursive function (" + nm + ") used other than by application");
      if (d->params.size() != args.size()) unsup(n, "operator " + nm + " with " + std::to_string(args.size()) + " arguments");
      std::set<std::string> v;
      if (d->params.empty() && state_free(d, v)) {
        auto it = cache_slot.find(nm);
        if (it != cache_slot.end()) return "c.k[" + std::to_string(it->second) + "]";
        const std::string fn = op_function(d, n);   // dependencies get their slots first
        const int slot = (int)(P.constants.size() + cache_slot.size());
        cache_slot[nm] = slot;
        cache_init.push_back("  c.k[" + std::to_string(slot) + "] = " + fn + "(c);\n");
        return "c.k[" + std::to_string(slot) + "]";
      }
      std::string o = op_function(d, n) + "(c";
      for (auto& a : args) o += ", " + a;
      return o + ")";
    }
    if (var_idx.count(nm)) {
      if (!args.empty()) unsup(n, "applying a variable");
      const std::string X = std::to_string(var_idx[nm]);
      if (init_mode) return "(((c.asg >> " + X + ") & 1ull) ? c.nxt[" + X + "] : (A.err |= E_ASSIGN, 0u))";
      return "c.cur[" + X + "]";
    }
    if (const_idx.count(nm)) {
      if (!args.empty()) unsup(n, "operator constants");
      return "c.k[" + std::to_string(const_idx[nm]) + "]";
    }
    // standard modules
    auto need = [&](size_t k) { if (args.size() != k) unsup(n, nm + " with " + std::to_string(args.size()) + " arguments"); };
    if (nm == "Len") { need(1); return "mk_int(A, fun_len(A, " + args[0] + "))"; }
    if (nm == "Append") { need(2); return "append(A, " + args[0] + ", " + args[1] + ")"; }
    if (nm == "SubSeq") { need(3); return "subseq(A, " + args[0] + ", ival(A, " + args[1] + "), ival(A, " + args[2] + "))"; }
    if (nm == "Head") { need(1); return "head(A, " + args[0] + ")"; }
    if (nm == "Tail") { need(1); return "tail(A, " + args[0] + ")"; }
    if (nm == "Cardinality") { need(1); return "mk_int(A, set_card(A, " + args[0] + "))"; }
    if (nm == "IsFiniteSet") { need(1); return "2u"; }
    if (nm == "Permutations") { need(1); return "permutations(A, " + args[0] + ")"; }   // TLC module (SYMMETRY sets)
    if (nm == "Print" || nm == "PrintT") { return args.back(); }
    if (nm == "Assert") { need(2); return "(truth(A, " + args[0] + ") ? 2u : (A.err |= E_DOMAIN, 0u))"; }
    // Bags
    if (nm == "EmptyBag") { need(0); return "seq_end(A, A.htop)"; }
    if (nm == "SetToBag") { need(1); return "set_to_bag(A, " + args[0] + ")"; }
    if (nm == "BagToSet") { need(1); return "dom(A, " + args[0] + ")"; }
    if (nm == "BagIn") { need(2); return "mk_bool(in_dom(A, " + args[1] + ", " + args[0] + "))"; }
    if (nm == "CopiesIn") { need(2); return "[&]() -> u32 { const u32 o_ = lookup(A, " + args[1] + ", " + args[0] + "); return o_ ? o_ : mk_int(A, 0); }()"; }
    if (nm == "BagCardinality") { need(1); return "mk_int(A, bag_card(A, " + args[0] + "))"; }
    if (nm == "IsABag") { need(1); return "2u"; }
    if (nm == "BOOLEAN") { need(0); return "[&]() -> u32 { const u32 m_ = A.htop; hpush(A, 0u); hpush(A, 2u); return set_end(A, m_); }()"; }
    unsup(n, "identifier " + nm);
  }

  // ---- actions: statements that run `k` once per way the formula is satisfied
  std::string wrap(const std::string& k, std::string& decl) {
    if (k.size() < 160) return k;
    const std::string name = fresh("K");
    decl += "auto " + name + " = [&]() TLG_NOINLINE {\n" + k + "};\n";
    return name + "();\n";
  }

  std::string assign(int X, const std::string& v, const std::string& k) {
    const std::string x = std::to_string(X), vv = fresh("v"), fr = fresh("f");
    return "{ const u32 " + vv + " = " + v + ";\n const bool " + fr + " = !((c.asg >> " + x + ") & 1ull);\n if (" + fr + ") { c.nxt[" + x +
           "] = " + vv + "; c.asg |= 1ull << " + x + "; }\n if (" + fr + " || eqv(A, c.nxt[" + x + "], " + vv + ")) {\n" + k + "}\n if (" +
           fr + ") c.asg &= ~(1ull << " + x + ");\n}\n";
  }

  int target_var(const NP& e) {   // the variable an `x' = ..` (Next) or `x = ..` (Init) determines, or -1
    if (!init_mode && e->k == K::Prime && e->a[0]->k == K::Ident && var_idx.count(e->a[0]->s)) return var_idx[e->a[0]->s];
    if (init_mode && e->k == K::Ident && var_idx.count(e->s)) return var_idx[e->s];
    return -1;
  }

  void unchanged_vars(const NP& e, std::vector<int>& out, int depth = 0) {
    if (depth > 16) unsup(*e, "UNCHANGED nesting");
    if (e->k == K::Tuple) { for (auto& x : e->a) unchanged_vars(x, out, depth + 1); return; }
    if (e->k == K::Ident) {
      if (var_idx.count(e->s)) { out.push_back(var_idx[e->s]); return; }
      if (auto d = global(e->s)) { if (d->params.empty() && d->body) { unchanged_vars(d->body, out, depth + 1); return; } }
    }
    unsup(*e, "UNCHANGED of a non-variable");
  }

  std::string act(const NP& e, Scope& sc, const std::string& k, bool split, int label) {
    const Node& n = *e;
    switch (n.k) {
      case K::And: {
        std::function<std::string(size_t)> chain = [&](size_t i) -> std::string {
          if (i == n.a.size()) return k;
          return act(n.a[i], sc, chain(i + 1), false, label);
        };
        return chain(0);
      }
      case K::Or: {
        std::string decl;
        const std::string kk = wrap(k, decl);
        std::string o = "{\n" + decl;
        for (auto& b : n.a) {
          const std::string sa = fresh("a"), st = fresh("t");
          o += "{ const unsigned long long " + sa + " = c.asg; const u32 " + st + " = A.top;\n";
          if (split) o += " c.act = " + std::to_string(label) + ";\n";
          std::string body = act(b, sc, kk, split, label);
          // a large branch becomes a function of its own: short branches and fewer live registers
          // in the expand kernel (one giant body needs long jumps and spills)
          if (body.size() > 1500) body = "[&]() TLG_NOINLINE {\n" + body + "}();\n";
          o += body + " c.asg = " + sa + "; A.top = " + st + "; }\n";
        }
        return o + "}\n";
      }
      case K::Exists: {
        Scope s2 = sc;
        return bind_loops(n.binds, 0, 0, s2, true, [&](Scope& s3) {
          return std::string(split ? " c.act = " + std::to_string(label) + ";\n" : "") + act(n.a[0], s3, k, split, label);
        });
      }
      case K::Let: {
        Scope s2 = sc;
        const std::string defs = let_defs(e, s2);
        return "{\n" + defs + act(n.a[0], s2, k, split, label) + "}\n";
      }
      case K::If: {
        std::string decl;
        const std::string kk = wrap(k, decl);
        return "{\n" + decl + "if (truth(A, " + ex(n.a[0], sc) + ")) {\n" + act(n.a[1], sc, kk, false, label) + "} else {\n" +
               act(n.a[2], sc, kk, false, label) + "}\n}\n";
      }
      case K::Case: {
        std::string decl;
        const std::string kk = wrap(k, decl);
        std::string o = "{\n" + decl;
        bool other = false;
        for (size_t i = 0; i < n.a.size(); i += 2) {
          if (!n.a[i]) { o += (i ? "else {\n" : "{\n") + act(n.a[i + 1], sc, kk, false, label) + "}\n"; other = true; break; }
          o += std::string(i ? "else " : "") + "if (truth(A, " + ex(n.a[i], sc) + ")) {\n" + act(n.a[i + 1], sc, kk, false, label) + "}\n";
        }
        if (!other) o += "else A.err |= E_DOMAIN;\n";
        return o + "}\n";
      }
      case K::Unchanged: {
        std::vector<int> vs;
        unchanged_vars(n.a[0], vs);
        std::string o = k;
        for (size_t i = vs.size(); i-- > 0;) o = assign(vs[i], "c.cur[" + std::to_string(vs[i]) + "]", o);
        return o;
      }
      case K::Binary: {
        if (n.s == "=") {
          const int X = target_var(n.a[0]);
          if (X >= 0) return assign(X, ex(n.a[1], sc), k);
        }
        if (n.s == "\\in") {
          const int X = target_var(n.a[0]);
          if (X >= 0) {
            const std::string el = fresh("e");
            return set_loop(ex(n.a[1], sc), el, assign(X, el, k), true);
          }
        }
        break;
      }
      case K::Ident: case K::OpApp: {
        if (find(sc, n.s)) {
          const Sym* s = find(sc, n.s);
          if (s->kind == Sym::LetOp && (init_mode || is_action_body(s->def))) return inline_op(n, sc, *s->def, *s->scope, k, split, label, false);
          break;
        }
        if (auto d = global(n.s)) {
          body_of(d, n);
          const bool action = is_action(d);
          if (higher_order(*d)) {
            if (action) unsup(n, "action operator " + d->name + " with an operator parameter");
            break;   // a predicate: evaluated by ex (apply_higher)
          }
          if (action || init_mode) return inline_op(n, sc, *d, Scope(), k, split, split && action ? action_id(d->name) : label, split && action);
        }
        break;
      }
      case K::Temporal: case K::Enabled: unsup(n, "a temporal formula in an action");
      default: break;
    }
    return "if (truth(A, " + ex(e, sc) + ")) {\n" + k + "}\n";
  }

  bool is_action_body(const std::shared_ptr<Def>& d) { std::set<std::string> v; return has_action(d->body, v); }

  // ---- higher-order operators (Op(F(_), x) == .. F(x) ..) and LAMBDA.  An operator argument
  // becomes a C++ lambda of the caller's scope: a LAMBDA (its body over its parameters), a LET
  // operator (its own lambda), or a global / standard-module operator by name (a wrapper calling
  // it).  A global operator with an operator parameter is expanded at each application, as an
  // immediately invoked lambda whose body sees only its parameters (the module scope), with the
  // operator parameters bound to those lambdas (Sym::LetOp).
  std::set<std::string> expanding;   // higher-order operators being expanded (recursion is refused)
  std::shared_ptr<Def> lambda_def(const Node& l) {
    auto d = std::make_shared<Def>();
    d->name = "LAMBDA"; d->params = l.fields; d->arity.assign(l.fields.size(), 0); d->body = l.a[0]; d->module = l.module; d->line = l.line;
    return d;
  }
  Sym op_arg(const NP& a, Scope& sc, int arity, std::string& decl) {
    Sym s; s.kind = Sym::LetOp; s.cxx = fresh("L");
    s.scope = std::make_shared<Scope>(sc);
    std::string params;
    std::vector<std::string> qs;
    for (int i = 0; i < arity; ++i) { qs.push_back(fresh("q")); params += (i ? ", u32 " : "u32 ") + qs.back(); }
    if (a->k == K::Lambda) {
      if ((int)a->fields.size() != arity) unsup(*a, "a LAMBDA of " + std::to_string(a->fields.size()) + " parameters for an operator of " + std::to_string(arity));
      s.def = lambda_def(*a);
      Scope inner = sc;
      for (int i = 0; i < arity; ++i) { Sym v; v.cxx = qs[i]; inner.push_back({a->fields[i], v}); }
      decl += "auto " + s.cxx + " = [&](" + params + ") -> u32 { return " + ex(a->a[0], inner) + "; };\n";
      return s;
    }
    if (a->k != K::Ident) unsup(*a, "an operator argument that is not a name or a LAMBDA");
    if (const Sym* b = find(sc, a->s)) {
      if (b->kind != Sym::LetOp) unsup(*a, "a value (" + a->s + ") passed as an operator argument");
      if (b->def && (int)b->def->params.size() != arity) unsup(*a, "operator " + a->s + " passed for an operator of " + std::to_string(arity) + " arguments");
      return *b;
    }
    if (auto d = global(a->s)) {
      if (higher_order(*d)) unsup(*a, "a higher-order operator (" + a->s + ") passed as an operator argument");
      if ((int)d->params.size() != arity) unsup(*a, "operator " + a->s + " passed for an operator of " + std::to_string(arity) + " arguments");
      s.def = d;
      s.scope = std::make_shared<Scope>();
    } else {
      s.def = std::make_shared<Def>();   // a standard-module operator (Len, Append, ..): its arity is checked by ident
      s.def->name = a->s; s.def->params = qs; s.def->arity.assign(arity, 0);
      s.def->body = std::make_shared<Node>(*a);
      s.def->body->k = K::OpApp;
      for (auto& q : qs) { auto id = std::make_shared<Node>(*a); id->s = q; s.def->body->a.push_back(id); }
    }
    Node call = *a;
    call.k = K::OpApp;
    decl += "auto " + s.cxx + " = [&](" + params + ") -> u32 { return " + ident(call, sc, qs) + "; };\n";
    return s;
  }
  std::string apply_higher(const Node& n, Scope& sc, const Def& d) {
    if (n.a.size() != d.params.size()) unsup(n, "operator " + d.name + " with " + std::to_string(n.a.size()) + " arguments");
    if (!d.body) unsup(n, "definition " + d.name + " does not parse: " + d.error);
    if (expanding.count(d.name)) unsup(n, "recursive higher-order operator " + d.name);
    std::string decl;
    Scope inner;
    for (size_t i = 0; i < d.params.size(); ++i) {
      if (arity_of(d, i)) { inner.push_back({d.params[i], op_arg(n.a[i], sc, arity_of(d, i), decl)}); continue; }
      if (n.a[i]->k == K::Lambda) unsup(*n.a[i], "a LAMBDA for the value parameter " + d.params[i] + " of " + d.name);
      Sym v; v.cxx = fresh("p");
      decl += "const u32 " + v.cxx + " = " + ex(n.a[i], sc) + ";\n";
      inner.push_back({d.params[i], v});
    }
    expanding.insert(d.name);
    const std::string body = ex(d.body, inner);
    expanding.erase(d.name);
    return "[&]() -> u32 {\n" + decl + "return " + body + ";\n}()";
  }
  // SelectSeq(s, Test) (Sequences): the elements of s, in order, for which Test holds
  std::string select_seq(const Node& n, Scope& sc) {
    if (n.a.size() != 2) unsup(n, "SelectSeq with " + std::to_string(n.a.size()) + " arguments");
    std::string decl;
    const Sym t = op_arg(n.a[1], sc, 1, decl);
    const std::string S = fresh("S"), m = fresh("m"), e = fresh("e"), i = fresh("i"), c = fresh("n"), tp = fresh("t"), kp = fresh("k");
    return "[&]() -> u32 {\n" + decl + "const u32 " + S + " = " + ex(n.a[0], sc) + ";\n if (tg(A, " + S + ") != T_SEQ) { A.err |= E_TYPE; return " + S +
           "; }\n const u32 " + m + " = A.htop; u32 " + e + " = first(" + S + ");\n for (u32 " + i + " = 0, " + c + " = count(A, " + S + "); " + i + " < " + c +
           "; ++" + i + ", " + e + " = nextv(A, " + e + ")) {\n  const u32 " + tp + " = A.top; const bool " + kp + " = truth(A, " + t.cxx + "(" + e + ")); A.top = " + tp +
           ";\n  if (" + kp + ") hpush(A, " + e + ");\n }\n return seq_end(A, " + m + ");\n}()";
  }

  std::string inline_op(const Node& n, Scope& sc, const Def& d, const Scope& defscope, const std::string& k, bool split, int label, bool set_label) {
    if (n.a.size() != d.params.size()) unsup(n, "operator " + d.name + " with " + std::to_string(n.a.size()) + " arguments");
    std::string o = "{\n";
    Scope s2 = defscope;
    for (size_t i = 0; i < d.params.size(); ++i) {
      const std::string pn = fresh("p");
      o += " const u32 " + pn + " = " + ex(n.a[i], sc) + ";\n";
      Sym s; s.cxx = pn;
      s2.push_back({d.params[i], s});
    }
    if (set_label) o += " c.act = " + std::to_string(label) + ";\n";
    return o + act(d.body, s2, k, split, label) + "}\n";
  }

  std::string cval(const CVal& v) {
    switch (v.kind) {
      case CVal::Int: return "mk_int(A, " + std::to_string(v.i) + "LL)";
      case CVal::Str: return "mk_atom(A, " + std::to_string(str_atom(v.s)) + "u)";
      case CVal::MV: return "mk_atom(A, " + std::to_string(mv_atom(v.s)) + "u)";
      case CVal::Bool: return v.i ? "2u" : "0u";
      case CVal::Set: {
        std::string o = "[&]() -> u32 { const u32 m_ = A.htop;";
        for (auto& e : v.elems) o += " hpush(A, " + cval(e) + ");";
        return o + " return set_end(A, m_); }()";
      }
    }
    return "0u";
  }

  std::shared_ptr<Def> cfg_def(const std::string& name, const char* what) {
    auto d = global(name);
    if (!d) throw CfgError(MC_E_UNSUPPORTED, std::string("cfg ") + what + " " + name + " is not defined in the module");
    if (!d->body) throw CfgError(MC_E_UNSUPPORTED, std::string("cfg ") + what + " " + name + " does not parse: " + d->error);
    return d;
  }
};

}  // namespace

// What TLC fingerprints for a state (VIEW / SYMMETRY): under SYMMETRY the least state over the
// permutations, variables compared in declaration order in TLC's value order (tlv ocmp; TLC's rule
// as the oracle's --sym tlc restates it), then the VIEW of it, or the tuple of its variables.  One
// value handle; its words are what is fingerprinted (and the host BFS's seen-set key).
static const char* const kCanonView = R"(TLV_NI u32 canon_view(Cx& d) {
  Ar& A = *d.A;
  Cx e = d;
  if (HAS_SYMMETRY) {
    const u32 ps = symmetry(d);
    if (tg(A, ps) != T_SET) { A.err |= E_TYPE; return 0u; }
    u32 pe = first(ps);
    for (u32 q = 0, n = count(A, ps); q < n; ++q, pe = nextv(A, pe)) {
      int c = q == 0 ? -1 : 0;   // the first permutation sets the least state so far
      for (int i = 0; i < NV; ++i) {
        const u32 r = perm_value(A, d.cur[i], pe);
        if (c == 0) { c = ocmp(A, r, e.cur[i]); if (c > 0) break; }
        if (c < 0) e.cur[i] = r;
      }
    }
  }
  if (HAS_VIEW) return view(e);
  const u32 m = A.htop;
  for (int i = 0; i < NV; ++i) hpush(A, e.cur[i]);
  return seq_end(A, m);
}
)";

Generated generate(const Program& prog, const CfgFile& cfg) {
  Gen g(prog, cfg);
  Generated out;
  out.variables = prog.variables;
  if (prog.variables.size() > 64) throw CfgError(MC_E_UNSUPPORTED, "more than 64 state variables");
  // a model with temporal properties must not report "No error has been found" without checking them
  if (!cfg.properties.empty()) throw CfgError(MC_E_UNSUPPORTED, "temporal PROPERTIES are not supported");
  std::ostringstream consts;
  for (size_t i = 0; i < prog.constants.size(); ++i) {
    const std::string& c = prog.constants[i];
    if (!cfg.has(c)) throw CfgError(MC_E_PARSE, "constant " + c + " has no value in the cfg");
    consts << "  c.k[" << i << "] = " << g.cval(cfg.get(c)) << ";\n";
  }
  out.init_name = cfg.init.empty() ? "Init" : cfg.init;
  out.next_name = cfg.next.empty() ? "Next" : cfg.next;
  auto initd = g.cfg_def(out.init_name, "INIT");
  auto nextd = g.cfg_def(out.next_name, "NEXT");
  if (!initd->params.empty() || !nextd->params.empty()) throw CfgError(MC_E_UNSUPPORTED, "INIT / NEXT with parameters");
  const std::string full = prog.variables.size() == 64 ? "~0ull" : "((1ull << " + std::to_string(prog.variables.size()) + ") - 1ull)";

  Scope sc;
  g.init_mode = true;
  const std::string init_body = g.act(initd->body, sc, "if (c.asg == " + full + ") em(c); else A.err |= E_ASSIGN;\n", false, 0);
  g.init_mode = false;
  const int next_label = g.action_id(out.next_name);
  const std::string next_body = g.act(nextd->body, sc, "if (c.asg == " + full + ") em(c); else A.err |= E_ASSIGN;\n", true, next_label);
  // chg: the variables the successor changed (a bit each; all for an initial state): a constraint
  // or invariant reading none of them holds as it held for the parent (Gen::var_mask)
  std::string cons = "TLV_NI bool constraints(Cx& c, unsigned long long chg) {\n  Ar& A = *c.A; (void)A; (void)chg;\n";
  for (auto& n : cfg.constraints) {
    auto d = g.cfg_def(n, "CONSTRAINT");
    Scope s0;
    const std::string mk = d->params.empty() ? g.mask_of(d) : "~0ull";
    cons += "  if ((chg & " + mk + ") && !truth(A, " + g.ex(d->body, s0) + ")) return false;\n";
    out.constraints.push_back(n);
  }
  cons += "  return true;\n}\n";
  // ACTION_CONSTRAINTS: predicates of a transition (c.cur the parent, c.nxt the successor, every
  // variable assigned); a successor is in the model when the state constraints and these hold
  // (the oracle's in_model && in_actions, oracle/engine.h)
  cons += "TLV_NI bool action_constraints(Cx& c) {\n  Ar& A = *c.A; (void)A;\n";
  for (auto& n : cfg.action_constraints) {
    auto d = g.cfg_def(n, "ACTION_CONSTRAINT");
    Scope s0;
    cons += "  if (!truth(A, " + g.ex(d->body, s0) + ")) return false;\n";
    out.constraints.push_back(n);
  }
  cons += "  return true;\n}\n";
  std::string invs = "TLV_NI int invariants(Cx& c, unsigned long long chg) {\n  Ar& A = *c.A; (void)A; (void)chg;\n";
  for (size_t i = 0; i < cfg.invariants.size(); ++i) {
    auto d = g.cfg_def(cfg.invariants[i], "INVARIANT");
    Scope s0;
    // an invariant whose evaluation fails (TLC: "Evaluating invariant X failed") is the one
    // returned, with the error bits set: the caller reports EVAL_ERROR naming it
    const std::string mk = d->params.empty() ? g.mask_of(d) : "~0ull";
    invs += "  if ((chg & " + mk + ") && (!truth(A, " + g.ex(d->body, s0) + ") || A.err)) return " + std::to_string(i) + ";\n";
    out.invariants.push_back(cfg.invariants[i]);
  }
  invs += "  return -1;\n}\n";
  // TLC's SYMMETRY: the set of permutations (of model values) under which states are identified; the
  // kernels fingerprint the least permuted state in TLC's order (tlagen_kernels.h canonical)
  std::string symm = "TLV_NI u32 symmetry(Cx& c) {\n  Ar& A = *c.A; (void)A;\n";
  if (!cfg.symmetry.empty()) {
    auto d = g.cfg_def(cfg.symmetry, "SYMMETRY");
    if (!d->params.empty()) throw CfgError(MC_E_UNSUPPORTED, "SYMMETRY " + cfg.symmetry + " with parameters");
    Node idn;
    idn.k = K::Ident; idn.s = cfg.symmetry; idn.line = d->line; idn.module = d->module;
    Scope s0;
    symm += "  return " + g.ident(idn, s0, {}) + ";\n}\n";
  } else {
    symm += "  return 0u;\n}\n";
  }
  // TLC's VIEW: states are told apart (fingerprinted) by the value of this expression; the state
  // kept for a view class is the first found (TLC's single-worker FIFO order, tlagen_kernels.h)
  std::string view = "TLV_NI u32 view(Cx& c) {\n  Ar& A = *c.A; (void)A;\n";
  if (!cfg.view.empty()) {
    auto d = g.cfg_def(cfg.view, "VIEW");
    if (!d->params.empty()) throw CfgError(MC_E_UNSUPPORTED, "VIEW " + cfg.view + " with parameters");
    Scope s0;
    view += "  return " + g.ex(d->body, s0) + ";\n}\n";
  } else {
    view += "  return 0u;\n}\n";
  }

  std::ostringstream s;
  s << "#ifndef TLG_NOINLINE\n#define TLG_NOINLINE __attribute__((noinline))\n#endif\n";
  s << "namespace tlg {\nusing namespace tlv;\n";
  s << "enum : int { NV = " << prog.variables.size() << ", NK = " << prog.constants.size() << ", NACT = " << g.actions.size()
    << ", NINV = " << cfg.invariants.size() << ", HAS_VIEW = " << (cfg.view.empty() ? 0 : 1)
    << ", HAS_SYMMETRY = " << (cfg.symmetry.empty() ? 0 : 1) << " };\n";
  s << "struct Cx { Ar* A; u32 k[" << std::max<size_t>(1, prog.constants.size() + g.cache_slot.size()) << "]; u32 cur[" << std::max<size_t>(1, prog.variables.size())
    << "]; u32 nxt[" << std::max<size_t>(1, prog.variables.size()) << "]; unsigned long long asg; int act; };\n";
  for (auto& p : g.fn_protos) s << p << "\n";
  s << "TLV_NI bool constraints(Cx& c, unsigned long long chg = ~0ull);\nTLV_NI bool action_constraints(Cx& c);\nTLV_NI int invariants(Cx& c, unsigned long long chg = ~0ull);\nTLV_NI u32 view(Cx& c);\nTLV_NI u32 symmetry(Cx& c);\n";
  for (auto& b : g.fn_bodies) s << b;
  // atoms in TLC's order (tlv ocmp): strings by text, model values by name (s1 < s2 < ..., the
  // declaration order of the cfg's model values), model values after strings
  {
    std::vector<std::pair<std::pair<int, std::string>, size_t>> ord;
    for (size_t i = 0; i < g.atoms.size(); ++i) {
      const std::string& t = g.atoms[i];
      const bool str = !t.empty() && t[0] == '"';
      ord.push_back({{str ? 0 : 1, str ? t.substr(1, t.size() - 2) : t}, i});
    }
    std::sort(ord.begin(), ord.end());
    std::vector<unsigned> key(g.atoms.size());
    for (size_t r = 0; r < ord.size(); ++r) key[ord[r].second] = (unsigned)r | (ord[r].first.first ? (1u << 30) : 0u);
    s << "TLV_CONST u32 kAtomKey[] = {";
    for (size_t i = 0; i < key.size(); ++i) s << (i ? ", " : "") << key[i] << "u";
    s << (key.empty() ? "0u" : "") << "};\n";
  }
  s << "TLV_HD void init_consts(Cx& c) {\n  Ar& A = *c.A; (void)A;\n  A.akey = kAtomKey; A.nakey = " << g.atoms.size() << ";\n" << consts.str();
  for (auto& ci : g.cache_init) s << ci;
  s << "}\n";
  s << "template <class EM> TLV_HD void init_states(Cx& c, EM& em) {\n  Ar& A = *c.A; (void)A;\n  c.asg = 0; c.act = 0;\n" << init_body << "}\n";
  s << "template <class EM> TLV_HD void next_states(Cx& c, EM& em) {\n  Ar& A = *c.A; (void)A;\n  c.asg = 0; c.act = " << next_label << ";\n" << next_body << "}\n";
  s << cons << invs << view << symm << kCanonView << "}  // namespace tlg\n";
  out.source = s.str();
  out.actions = g.actions;
  out.atoms = g.atoms;
  return out;
}

std::string compose_source(const Generated& g, const std::string& tlv_text, const std::string& tail) {
  std::ostringstream s;
  s << "// generated by raftmc's TLA+ front end\n";
  for (auto& v : g.variables) s << "//@var " << v << "\n";
  for (auto& a : g.actions) s << "//@action " << a << "\n";
  for (auto& a : g.invariants) s << "//@invariant " << a << "\n";
  for (auto& a : g.atoms) s << "//@atom " << a << "\n";
  s << tlv_text << "\n" << g.source << "\n";
  s << "namespace tlg {\n";
  s << "static const char* const kActionNames[] = {";
  for (auto& a : g.actions) s << cstr(a) << ", ";
  s << "nullptr};\nstatic const char* const kInvariantNames[] = {";
  for (auto& a : g.invariants) s << cstr(a) << ", ";
  s << "nullptr};\nstatic const char* const kVarNames[] = {";
  for (auto& a : g.variables) s << cstr(a) << ", ";
  s << "nullptr};\nstatic const char* const kAtomNames[] = {";
  for (auto& a : g.atoms) s << cstr(a) << ", ";
  s << "nullptr};\n}  // namespace tlg\n";
  s << tail;
  return s.str();
}

}  // namespace tlagen
}  // namespace rmc
