// ============================================================================
// TEST INFRASTRUCTURE ONLY (see oracle/tla.h header).
// Parser for TLA+ *value* expressions as TLC prints them (records, tuples,
// sets, `:>`/`@@` functions, strings, integers, booleans, model values).
// Used to load golden TLC traces (tests/golden/*.tla_value) into the oracle.
// ============================================================================
#pragma once
#include <cstring>
#include "tla.h"

namespace tla {

struct ValueParser {
  const std::string& s; size_t p = 0;
  explicit ValueParser(const std::string& str) : s(str) {}
  void ws() { while (p < s.size() && isspace((unsigned char)s[p])) ++p; }
  bool lit(const char* t) { ws(); size_t n = strlen(t); if (s.compare(p, n, t) == 0) { p += n; return true; } return false; }
  void expect(const char* t) { if (!lit(t)) throw EvalError(std::string("value parse: expected '") + t + "' at " + std::to_string(p)); }
  std::string ident() {
    ws(); size_t q = p;
    while (p < s.size() && (isalnum((unsigned char)s[p]) || s[p] == '_')) ++p;
    if (q == p) throw EvalError("value parse: identifier expected at " + std::to_string(p));
    return s.substr(q, p - q);
  }
  V primary() {
    ws();
    if (lit("<<")) {
      std::vector<V> xs; ws();
      if (lit(">>")) return seq(xs);
      do { xs.push_back(value()); } while (lit(","));
      expect(">>"); return seq(xs);
    }
    if (lit("[")) {
      std::vector<V> ks, vs; ws();
      if (lit("]")) return fcn(ks, vs);
      do { std::string f = ident(); expect("|->"); ks.push_back(Str(f)); vs.push_back(value()); } while (lit(","));
      expect("]"); return fcn(ks, vs);
    }
    if (lit("{")) {
      std::vector<V> xs; ws();
      if (lit("}")) return set(xs);
      do { xs.push_back(value()); } while (lit(","));
      expect("}"); return set(xs);
    }
    if (lit("(")) { V v = value(); expect(")"); return v; }
    ws();
    if (p < s.size() && s[p] == '"') { size_t q = ++p; while (p < s.size() && s[p] != '"') ++p; std::string t = s.substr(q, p - q); ++p; return Str(t); }
    if (p < s.size() && (isdigit((unsigned char)s[p]) || s[p] == '-')) {
      size_t q = p; ++p; while (p < s.size() && isdigit((unsigned char)s[p])) ++p; return Int(std::stoll(s.substr(q, p - q)));
    }
    std::string id = ident();
    if (id == "TRUE") return Bool(true);
    if (id == "FALSE") return Bool(false);
    return MV(id);
  }
  // a :> b  binds tighter than @@
  V fn_term() { V a = primary(); if (lit(":>")) { V b = primary(); return colon_gt(a, b); } return a; }
  V value() { V v = fn_term(); while (lit("@@")) v = at_at(v, fn_term()); return v; }
};

inline V parse_value(const std::string& text) { ValueParser vp(text); V v = vp.value(); return v; }

}  // namespace tla
