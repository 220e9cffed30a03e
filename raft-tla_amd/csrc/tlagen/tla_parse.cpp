// tla_parse.cpp — lexer, parser and module loader of the SANY-subset front end (tla_ast.h).
//
// TLA+'s layout rule for junction lists (a /\ or \/ bullet at column c owns every following
// line that starts right of c) is implemented with a column fence: while a list is parsed, a
// token that starts a line at or left of the fence ends the current item.  Top-level units end
// at a token in column 0 that starts a line (the convention of every module in the reference).
#include "tla_ast.h"

#include <cctype>
#include <functional>
#include <fstream>
#include <set>
#include <sstream>

namespace rmc {
namespace tlagen {

namespace {

enum class T { Id, Num, Str, Op, Sep, End, Eof };

struct Tok {
  T t;
  std::string s;
  int line, col;
  bool bol;   // first token on its line
};

// operators, longest first
const char* kOps[] = {"<=>", "|->", "(+)", "(-)", "\\/", "/\\", "==", "=>", "=<", "<=", ">=", "/=", "->", "<-",
                      ":>", "@@", "..", "<<", ">>", "[]", "<>", "~>", "::", "=", "#", "<", ">", "+", "-", "*",
                      "%", "^", "'", "!", "@", "(", ")", "[", "]", "{", "}", ",", ":", ".", "~", "|", "&", "$"};

std::vector<Tok> lex(const std::string& src, const std::string& path) {
  std::vector<Tok> out;
  size_t i = 0;
  int line = 1, col = 0;
  bool bol = true;
  auto adv = [&](size_t n) {
    for (size_t q = 0; q < n && i < src.size(); ++q, ++i) {
      if (src[i] == '\n') { ++line; col = 0; bol = true; } else ++col;
    }
  };
  auto push = [&](T t, std::string s, int l, int c) { out.push_back({t, std::move(s), l, c, bol}); bol = false; };
  while (i < src.size()) {
    const char ch = src[i];
    if (ch == '\n' || ch == ' ' || ch == '\t' || ch == '\r') { adv(1); continue; }
    if (ch == '\\' && i + 1 < src.size() && src[i + 1] == '*') {   // line comment
      while (i < src.size() && src[i] != '\n') adv(1);
      continue;
    }
    if (ch == '(' && i + 1 < src.size() && src[i + 1] == '*') {    // nested block comment
      int depth = 0;
      do {
        if (src.compare(i, 2, "(*") == 0) { ++depth; adv(2); }
        else if (src.compare(i, 2, "*)") == 0) { --depth; adv(2); }
        else adv(1);
      } while (depth > 0 && i < src.size());
      continue;
    }
    const int l = line, c = col;
    if (ch == '-' && src.compare(i, 4, "----") == 0) {
      size_t j = i; while (j < src.size() && src[j] == '-') ++j;
      adv(j - i); push(T::Sep, "----", l, c); continue;
    }
    if (ch == '=' && src.compare(i, 4, "====") == 0) {
      size_t j = i; while (j < src.size() && src[j] == '=') ++j;
      adv(j - i); push(T::End, "====", l, c);
      break;                                                  // the rest of the file is not the module
    }
    if (std::isdigit((unsigned char)ch)) {
      size_t j = i; while (j < src.size() && std::isdigit((unsigned char)src[j])) ++j;
      if (j < src.size() && (std::isalpha((unsigned char)src[j]) || src[j] == '_')) {   // identifier like 1a
        while (j < src.size() && (std::isalnum((unsigned char)src[j]) || src[j] == '_')) ++j;
        push(T::Id, src.substr(i, j - i), l, c);
      } else push(T::Num, src.substr(i, j - i), l, c);
      adv(j - i); continue;
    }
    if (std::isalpha((unsigned char)ch) || ch == '_') {
      size_t j = i; while (j < src.size() && (std::isalnum((unsigned char)src[j]) || src[j] == '_')) ++j;
      std::string w = src.substr(i, j - i);
      // WF_vars / SF_vars: temporal fairness, kept as one token
      push(T::Id, w, l, c); adv(j - i); continue;
    }
    if (ch == '"') {
      std::string s; size_t j = i + 1;
      while (j < src.size() && src[j] != '"') {
        if (src[j] == '\\' && j + 1 < src.size()) { ++j; s += src[j] == 'n' ? '\n' : src[j] == 't' ? '\t' : src[j]; }
        else s += src[j];
        ++j;
      }
      push(T::Str, s, l, c); adv(j + 1 - i); continue;
    }
    if (ch == '\\') {
      if (i + 1 < src.size() && std::isalpha((unsigned char)src[i + 1])) {
        size_t j = i + 1; while (j < src.size() && std::isalpha((unsigned char)src[j])) ++j;
        push(T::Op, src.substr(i, j - i), l, c); adv(j - i); continue;
      }
      if (src.compare(i, 2, "\\/") == 0) { push(T::Op, "\\/", l, c); adv(2); continue; }
      push(T::Op, "\\", l, c); adv(1); continue;                       // set difference
    }
    bool found = false;
    for (const char* op : kOps) {
      const size_t n = std::char_traits<char>::length(op);
      if (src.compare(i, n, op) == 0) { push(T::Op, op, l, c); adv(n); found = true; break; }
    }
    if (!found) throw ParseError(path + ":" + std::to_string(l) + ": unexpected character '" + std::string(1, ch) + "'");
  }
  out.push_back({T::Eof, "", line + 1, 0, true});
  return out;
}

std::string canon_op(const std::string& s) {   // synonyms
  if (s == "\\land") return "/\\";
  if (s == "\\lor") return "\\/";
  if (s == "\\lnot" || s == "\\neg") return "~";
  if (s == "\\union") return "\\cup";
  if (s == "\\intersect") return "\\cap";
  if (s == "\\leq" || s == "=<") return "<=";
  if (s == "\\geq") return ">=";
  if (s == "#") return "/=";
  if (s == "\\circ") return "\\o";
  if (s == "\\equiv") return "<=>";
  if (s == "\\times") return "\\X";
  return s;
}

// binary operators: precedence (TLA+ book table 8, low end) and left associativity
int infix_prec(const std::string& s) {
  static const std::map<std::string, int> p = {
      {"=>", 1}, {"<=>", 2}, {"/\\", 3}, {"\\/", 3},
      {"=", 5}, {"/=", 5}, {"<", 5}, {">", 5}, {"<=", 5}, {">=", 5}, {"\\in", 5}, {"\\notin", 5},
      {"\\subseteq", 5}, {"\\subset", 5}, {"\\supseteq", 5}, {"~>", 2},
      {"@@", 6}, {":>", 7}, {"\\cup", 8}, {"\\cap", 8}, {"\\", 8}, {"(+)", 10}, {"(-)", 11},
      {"..", 9}, {"\\X", 10}, {"+", 10}, {"-", 11}, {"%", 11}, {"*", 13}, {"\\div", 13}, {"\\o", 13}, {"^", 14}};
  auto it = p.find(s);
  return it == p.end() ? -1 : it->second;
}

struct Parser {
  std::vector<Tok> tk;
  size_t p = 0;
  std::vector<int> fence{-1};
  std::string path, module;

  bool unit_mode = false;   // parsing a top-level definition's body
  int let_depth = 0;        // inside a LET's definitions

  // a token that starts a new top-level unit: a keyword, `Name ==`, `Name(..) ==`, `f[..] ==`, `a op b ==`
  bool unit_start(size_t i) const {
    const Tok& t = tk[i];
    if (!t.bol) return false;
    if (t.t == T::Sep || t.t == T::End || t.t == T::Eof) return true;
    if (t.t != T::Id) return false;
    static const std::set<std::string> kw = {"CONSTANT", "CONSTANTS", "VARIABLE", "VARIABLES", "ASSUME", "ASSUMPTION",
                                             "THEOREM", "LEMMA", "LOCAL", "INSTANCE", "EXTENDS", "RECURSIVE", "AXIOM"};
    if (kw.count(t.s)) return true;
    const Tok& n1 = tk[i + 1];
    if (n1.t != T::Op) return false;
    if (n1.s == "==") return true;
    if (n1.s == "(" || n1.s == "[") {
      const std::string close = n1.s == "(" ? ")" : "]";
      int d = 0;
      size_t j = i + 1;
      for (; tk[j].t != T::Eof; ++j) {
        if (tk[j].t == T::Op && tk[j].s == n1.s) ++d;
        else if (tk[j].t == T::Op && tk[j].s == close && --d == 0) break;
      }
      return tk[j].t != T::Eof && tk[j + 1].t == T::Op && tk[j + 1].s == "==";
    }
    return i + 3 < tk.size() && tk[i + 2].t == T::Id && tk[i + 3].t == T::Op && tk[i + 3].s == "==";
  }
  bool fenced_at(size_t i) const {
    const Tok& t = tk[i];
    if (t.t == T::Eof) return false;
    if (t.bol && t.col <= fence.back()) return true;
    return unit_mode && let_depth == 0 && unit_start(i);
  }
  const Tok& raw() const { return tk[p]; }
  // the next token as the current expression sees it (Eof past the fence)
  Tok peek() const {
    const Tok& t = tk[p];
    if (fenced_at(p)) return {T::Eof, "", t.line, t.col, true};
    return t;
  }
  bool is(const char* s) const { const Tok t = peek(); return (t.t == T::Op || t.t == T::Id) && canon_op(t.s) == s; }
  [[noreturn]] void fail(const std::string& m) const {
    const Tok& t = tk[p];
    throw ParseError(path + ":" + std::to_string(t.line) + ":" + std::to_string(t.col + 1) + ": " + m +
                     " (at '" + t.s + "')");
  }
  Tok next() { if (fenced_at(p)) fail("unexpected end of expression"); return tk[p++]; }
  void expect(const char* s) { if (!is(s)) fail(std::string("expected '") + s + "'"); ++p; }
  std::string ident() { const Tok t = peek(); if (t.t != T::Id) fail("expected an identifier"); ++p; return t.s; }
  NP mk(K k, const Tok& at, std::string s = "") {
    auto n = std::make_shared<Node>();
    n->k = k; n->s = std::move(s); n->line = at.line; n->col = at.col; n->module = module;
    return n;
  }

  // ---- bindings: x, y \in S, z \in T
  std::vector<Bind> binds() {
    std::vector<Bind> out;
    do {
      Bind b;
      if (is("<<")) {   // \E <<a, b>> \in S : the elements of S are tuples, a and b their components
        ++p;
        b.tuple = true;
        do b.names.push_back(ident()); while (is(",") && (++p, true));
        expect(">>");
      } else {
        b.names.push_back(ident());
        while (is(",")) {
          const size_t save = p; ++p;
          if (peek().t == T::Id && (tk[p + 1].s == "," || canon_op(tk[p + 1].s) == "\\in")) b.names.push_back(ident());
          else { p = save; break; }
        }
      }
      if (!is("\\in")) fail("unbounded quantifiers are outside the subset");
      ++p;
      b.set = expr(0);
      out.push_back(b);
    } while (is(",") && (++p, true));
    return out;
  }

  NP junction(bool conj) {
    const Tok& b = raw();
    const int c = b.col;
    NP n = mk(conj ? K::And : K::Or, b);
    fence.push_back(c);
    while (true) {
      const Tok& t = raw();
      if (!(t.t == T::Op && canon_op(t.s) == (conj ? "/\\" : "\\/") && t.col == c)) break;
      // a bullet that is not first on its line (or is left of an enclosing fence) ends the list
      if (n->a.size() && !t.bol) break;
      if (fence.size() >= 2 && t.bol && t.col <= fence[fence.size() - 2]) break;
      ++p;
      n->a.push_back(expr(0));
    }
    fence.pop_back();
    return n->a.size() == 1 ? n->a[0] : n;
  }

  NP primary() {
    const Tok t = peek();
    if (t.t == T::Eof || t.t == T::Sep || t.t == T::End) fail("unexpected end of expression");
    if (t.t == T::Num) { ++p; NP n = mk(K::Num, t); n->n = std::stoll(t.s); return n; }
    if (t.t == T::Str) { ++p; return mk(K::Str, t, t.s); }
    const std::string s = canon_op(t.s);
    if (t.t == T::Op) {
      if (s == "/\\" || s == "\\/") return junction(s == "/\\");
      if (s == "(") {
        ++p; fence.push_back(-1); NP e = expr(0); expect(")"); fence.pop_back();
        if (e->k == K::Binary && e->s == "\\X") e->n = 0;   // (A \X B) \X C: a pair whose first component is a pair
        return e;
      }
      if (s == "~") { ++p; NP n = mk(K::Unary, t, "~"); n->a.push_back(expr(4)); return n; }
      if (s == "-") { ++p; NP n = mk(K::Unary, t, "-"); n->a.push_back(expr(12)); return n; }
      if (s == "[]" || s == "<>") { ++p; NP n = mk(K::Temporal, t, s); n->a.push_back(expr(4)); return n; }
      if (s == "\\A" || s == "\\E") {
        ++p;
        NP n = mk(s == "\\A" ? K::Forall : K::Exists, t);
        n->binds = binds();
        expect(":");
        n->a.push_back(expr(0));
        return n;
      }
      if (s == "{") return braces();
      if (s == "[") return brackets();
      if (s == "<<") {
        ++p; fence.push_back(-1);
        NP n = mk(K::Tuple, t);
        if (!is(">>")) { n->a.push_back(expr(0)); while (is(",")) { ++p; n->a.push_back(expr(0)); } }
        expect(">>");
        fence.pop_back();
        if (peek().t == T::Id && peek().s[0] == '_') fail("angle-action subscripts are temporal");
        return n;
      }
      if (s == "@") { ++p; return mk(K::At, t); }
      fail("unexpected operator");
    }
    // identifiers and keywords
    if (s == "TRUE" || s == "FALSE") { ++p; NP n = mk(K::Bool, t); n->n = s == "TRUE"; return n; }
    if (s == "IF") {
      ++p; NP n = mk(K::If, t);
      n->a.push_back(expr(0)); expect("THEN"); n->a.push_back(expr(0)); expect("ELSE"); n->a.push_back(expr(0));
      return n;
    }
    if (s == "CASE") {
      ++p; NP n = mk(K::Case, t);
      while (true) {
        if (is("OTHER")) { ++p; expect("->"); n->a.push_back(nullptr); n->a.push_back(expr(0)); break; }
        n->a.push_back(expr(0)); expect("->"); n->a.push_back(expr(0));
        if (is("[]")) { ++p; continue; }
        break;
      }
      return n;
    }
    if (s == "LET") {
      ++p; NP n = mk(K::Let, t);
      ++let_depth;
      while (!is("IN")) n->defs.push_back(definition(true));
      --let_depth;
      ++p;
      n->a.push_back(expr(0));
      return n;
    }
    if (s == "LAMBDA") {   // LAMBDA x, y : e — SequencesExt's Remove (SelectSeq(s, LAMBDA t : t # e))
      ++p; NP n = mk(K::Lambda, t);
      do n->fields.push_back(ident()); while (is(",") && (++p, true));
      expect(":");
      n->a.push_back(expr(0));
      return n;
    }
    if (s == "CHOOSE") {
      ++p; NP n = mk(K::Choose, t);
      n->binds = binds();
      if (n->binds.size() != 1 || n->binds[0].names.size() != 1 || n->binds[0].tuple) fail("CHOOSE binds one identifier");
      expect(":");
      n->a.push_back(expr(0));
      return n;
    }
    if (s == "UNCHANGED") { ++p; NP n = mk(K::Unchanged, t); n->a.push_back(expr(15)); return n; }
    if (s == "ENABLED") { ++p; NP n = mk(K::Enabled, t); n->a.push_back(expr(15)); return n; }
    if (s == "SUBSET" || s == "UNION" || s == "DOMAIN") { ++p; NP n = mk(K::Unary, t, s); n->a.push_back(expr(9)); return n; }
    if (s.rfind("WF_", 0) == 0 || s.rfind("SF_", 0) == 0) {
      ++p; NP n = mk(K::Temporal, t, s); expect("("); n->a.push_back(expr(0)); expect(")"); return n;
    }
    static const std::set<std::string> kw = {"THEN", "ELSE", "IN", "OTHER", "EXCEPT", "MODULE", "EXTENDS",
                                             "CONSTANT", "CONSTANTS", "VARIABLE", "VARIABLES", "ASSUME", "THEOREM"};
    if (kw.count(s)) fail("unexpected keyword");
    ++p;
    if (is("(")) {   // operator application
      ++p; fence.push_back(-1);
      NP n = mk(K::OpApp, t, t.s);
      if (!is(")")) { n->a.push_back(expr(0)); while (is(",")) { ++p; n->a.push_back(expr(0)); } }
      expect(")");
      fence.pop_back();
      return n;
    }
    return mk(K::Ident, t, t.s);
  }

  NP braces() {
    const Tok t = next();
    fence.push_back(-1);
    NP n;
    if (is("}")) n = mk(K::SetEnum, t);
    else {
      // {x \in S : P} filters when the part before ':' is `identifier \in S`
      if (peek().t == T::Id && canon_op(tk[p + 1].s) == "\\in") {
        const size_t save = p;
        const std::string x = ident(); ++p;
        NP set = expr(0);
        if (is(":")) {
          ++p; n = mk(K::SetFilter, t);
          n->binds.push_back({{x}, set});
          n->a.push_back(expr(0));
        } else p = save;
      }
      if (!n) {
        NP e = expr(0);
        if (is(":")) { ++p; n = mk(K::SetMap, t); n->a.push_back(e); n->binds = binds(); }
        else {
          n = mk(K::SetEnum, t); n->a.push_back(e);
          while (is(",")) { ++p; n->a.push_back(expr(0)); }
        }
      }
    }
    expect("}");
    fence.pop_back();
    return n;
  }

  NP brackets() {
    const Tok t = next();
    fence.push_back(-1);
    NP n;
    const Tok a = peek();
    const std::string nx = canon_op(tk[p + 1].s);
    if (a.t == T::Id && nx == "|->") {                   // record
      n = mk(K::Record, t);
      do { n->fields.push_back(ident()); expect("|->"); n->a.push_back(expr(0)); } while (is(",") && (++p, true));
    } else if (a.t == T::Id && nx == ":") {              // record set
      n = mk(K::RecordSet, t);
      do { n->fields.push_back(ident()); expect(":"); n->a.push_back(expr(0)); } while (is(",") && (++p, true));
    } else if (a.t == T::Id && (nx == "\\in" || nx == ",")) {   // function constructor
      n = mk(K::FunCons, t);
      n->binds = binds();
      expect("|->");
      n->a.push_back(expr(0));
    } else {
      NP e = expr(0);
      if (is("EXCEPT")) {
        ++p; n = mk(K::Except, t); n->a.push_back(e);
        do {
          expect("!");
          Update u;
          while (is("[") || is(".")) {
            PathStep st;
            if (is(".")) { ++p; st.field = true; st.name = ident(); }
            else {
              ++p; st.idx = expr(0);
              if (is(",")) {   // ![a, b] = tuple index
                NP tup = mk(K::Tuple, t); tup->a.push_back(st.idx);
                while (is(",")) { ++p; tup->a.push_back(expr(0)); }
                st.idx = tup;
              }
              expect("]");
            }
            u.path.push_back(st);
          }
          if (u.path.empty()) fail("EXCEPT needs a ![..] or !.f path");
          expect("=");
          u.rhs = expr(0);
          n->ups.push_back(u);
        } while (is(",") && (++p, true));
      } else if (is("->")) {
        ++p; n = mk(K::FunSet, t); n->a.push_back(e); n->a.push_back(expr(0));
      } else if (is("]")) {
        fence.pop_back(); ++p;
        if (peek().t == T::Id && peek().s[0] == '_') { ++p; NP tn = mk(K::Temporal, t, "[A]_v"); return tn; }
        fail("unexpected ']'");
      } else fail("unsupported bracket form");
    }
    expect("]");
    fence.pop_back();
    return n;
  }

  NP postfix(NP e) {
    while (true) {
      const Tok t = peek();
      if (t.t != T::Op) break;
      const std::string s = t.s;
      if (s == "'") { ++p; NP n = mk(K::Prime, t); n->a.push_back(e); e = n; continue; }
      if (s == "[" && !t.bol) {
        ++p; fence.push_back(-1);
        NP n = mk(K::FunApp, t); n->a.push_back(e);
        NP arg = expr(0);
        if (is(",")) { NP tup = mk(K::Tuple, t); tup->a.push_back(arg); while (is(",")) { ++p; tup->a.push_back(expr(0)); } arg = tup; }
        n->a.push_back(arg);
        expect("]");
        fence.pop_back();
        e = n; continue;
      }
      if (s == "." && tk[p + 1].t == T::Id && !t.bol) {
        ++p; NP n = mk(K::Dot, t, ident()); n->a.push_back(e); e = n; continue;
      }
      break;
    }
    return e;
  }

  NP expr(int minp) {
    NP lhs = postfix(primary());
    while (true) {
      const Tok t = peek();
      if (t.t != T::Op && !(t.t == T::Id && false)) break;
      const std::string s = canon_op(t.s);
      const int pr = infix_prec(s);
      if (pr < 0 || pr < minp) break;
      // a /\ or \/ that starts a line is a bullet of an enclosing list, never infix here
      ++p;
      NP rhs = expr(pr + 1);
      if (s == "/\\" || s == "\\/") {
        const K k = s == "/\\" ? K::And : K::Or;
        if (lhs->k == k && lhs->s == "infix") { lhs->a.push_back(rhs); continue; }
        NP n = mk(k, t, "infix"); n->a.push_back(lhs); n->a.push_back(rhs); lhs = n; continue;
      }
      if (s == "\\X") {   // A \X B \X C is the set of triples (\X is not associative)
        if (lhs->k == K::Binary && lhs->s == s && lhs->n == 1) { lhs->a.push_back(rhs); continue; }
        NP n = mk(K::Binary, t, s); n->n = 1; n->a.push_back(lhs); n->a.push_back(rhs); lhs = n; continue;
      }
      NP n = mk(K::Binary, t, s); n->a.push_back(lhs); n->a.push_back(rhs); lhs = n;
    }
    return lhs;
  }

  // Name == e | Name(p, q) == e | f[x \in S] == e | a (+) b == e
  std::shared_ptr<Def> definition(bool in_let) {
    auto d = std::make_shared<Def>();
    d->module = module;
    const Tok t = peek();
    d->line = t.line;
    if (t.t != T::Id) fail("expected a definition");
    const std::string first = t.s;
    ++p;
    if (raw().t == T::Op && raw().s != "==" && raw().s != "(" && raw().s != "[" && tk[p + 1].t == T::Id &&
        tk[p + 2].t == T::Op && tk[p + 2].s == "==") {                 // infix definition a (+) b == ...
      d->name = raw().s; ++p; d->params = {first, ident()}; d->arity = {0, 0};
    } else {
      d->name = first;
      if (is("(")) {
        ++p;
        if (!is(")")) {
          do {
            std::string q = ident();
            int k = 0;
            if (is("(")) {   // operator parameter F(_, _)
              ++p;
              while (!is(")")) { if (raw().s == "_") ++k; ++p; }
              ++p;
              if (!k) fail("operator parameter without an argument");
            }
            d->params.push_back(q);
            d->arity.push_back(k);
          } while (is(",") && (++p, true));
        }
        expect(")");
      } else if (is("[")) {                                   // function definition f[x \in S] == e
        const Tok b = next();
        NP fc = mk(K::FunCons, b);
        fc->binds = binds();
        expect("]");
        expect("==");
        fc->a.push_back(body(in_let, d));
        d->body = d->error.empty() ? fc : nullptr;
        return d;
      }
    }
    expect("==");
    d->body = body(in_let, d);
    return d;
  }

  NP body(bool in_let, std::shared_ptr<Def>& d) {
    if (in_let) return expr(0);
    const size_t start = p;
    fence.push_back(0);
    unit_mode = true;
    try {
      NP e = expr(0);
      if (!unit_start(p) && !(raw().bol && raw().col == 0)) fail("trailing tokens after the definition");
      fence.pop_back();
      unit_mode = false;
      return e;
    } catch (const ParseError& e) {
      fence.resize(1);
      unit_mode = false;
      let_depth = 0;
      d->error = e.what();
      p = start;
      skip_unit();
      return nullptr;
    }
  }

  void skip_unit() {   // to the next token that starts a unit
    ++p;
    while (raw().t != T::Eof && raw().t != T::End && !(raw().bol && raw().col == 0) && !unit_start(p)) ++p;
  }
};

}  // namespace

std::string node_where(const Node& n) {
  return n.module + ":" + std::to_string(n.line) + ":" + std::to_string(n.col + 1);
}

Module parse_module(const std::string& text, const std::string& path) {
  Parser ps;
  ps.tk = lex(text, path);
  ps.path = path;
  Module m;
  m.path = path;
  // header: ---- MODULE Name ----
  while (ps.raw().t != T::Eof && !(ps.raw().t == T::Id && ps.raw().s == "MODULE")) ++ps.p;
  if (ps.raw().t == T::Eof) throw ParseError(path + ": no MODULE header");
  ++ps.p;
  m.name = ps.raw().s;
  ps.module = m.name;
  ++ps.p;
  while (true) {
    const Tok& t = ps.raw();
    if (t.t == T::Eof || t.t == T::End) break;
    if (t.t == T::Sep) { ++ps.p; continue; }
    if (t.t != T::Id) { ps.skip_unit(); continue; }
    const std::string w = t.s;
    if (w == "EXTENDS") {
      ++ps.p;
      do { m.extends.push_back(ps.ident()); } while (ps.is(",") && (++ps.p, true));
    } else if (w == "CONSTANT" || w == "CONSTANTS" || w == "VARIABLE" || w == "VARIABLES") {
      ++ps.p;
      auto& dst = w[0] == 'C' ? m.constants : m.variables;
      do {
        dst.push_back(ps.ident());
        if (ps.is("(")) { ++ps.p; while (!ps.is(")")) ++ps.p; ++ps.p; }
      } while (ps.is(",") && (++ps.p, true));
    } else if (w == "ASSUME" || w == "ASSUMPTION" || w == "THEOREM" || w == "LEMMA" || w == "AXIOM" ||
               w == "INSTANCE" || w == "RECURSIVE" || w == "PROOF" || w == "BY" || w == "QED") {
      ps.skip_unit();
    } else if (w == "LOCAL") {
      ++ps.p;
    } else {
      m.defs.push_back(ps.definition(false));
    }
  }
  return m;
}

namespace {
const std::set<std::string> kStandard = {"Naturals", "Integers", "Sequences", "FiniteSets", "TLC", "Bags", "Reals"};

std::string read_file(const std::string& p) {
  std::ifstream f(p);
  if (!f) return "";
  std::stringstream ss; ss << f.rdbuf();
  return ss.str();
}
std::string dir_of(const std::string& p) {
  const size_t s = p.rfind('/');
  return s == std::string::npos ? "." : p.substr(0, s);
}
}  // namespace

Program load_program(const std::string& root_path, const std::vector<std::string>& search_dirs) {
  Program prog;
  std::set<std::string> loaded;
  std::vector<std::string> stack;
  // depth-first: a module's extended modules come before it
  std::function<void(const std::string&, const std::string&)> load = [&](const std::string& path, const std::string& text) {
    Module m = parse_module(text, path);
    if (loaded.count(m.name)) return;
    loaded.insert(m.name);
    // the repo's MC wrappers name their base module's file in a pragma
    std::string base;
    const size_t pr = text.find("raftmc-base:");
    if (pr != std::string::npos) {
      size_t a = pr + 12; while (a < text.size() && text[a] == ' ') ++a;
      size_t b = a; while (b < text.size() && !std::isspace((unsigned char)text[b])) ++b;
      base = text.substr(a, b - a);
    }
    for (const std::string& e : m.extends) {
      if (kStandard.count(e) || loaded.count(e)) continue;
      std::vector<std::string> cands = {dir_of(path) + "/" + e + ".tla"};
      if (!base.empty()) {
        cands.push_back(dir_of(path) + "/" + base);
        for (const auto& d : search_dirs) cands.push_back(d + "/" + base);
      }
      for (const auto& d : search_dirs) cands.push_back(d + "/" + e + ".tla");
      bool ok = false;
      for (const auto& c : cands) {
        const std::string t = read_file(c);
        if (t.empty()) continue;
        load(c, t);
        ok = true;
        break;
      }
      if (!ok) throw ParseError(path + ": EXTENDS " + e + ": module file not found");
    }
    prog.modules.push_back(std::move(m));
  };
  const std::string text = read_file(root_path);
  if (text.empty()) throw ParseError(root_path + ": cannot read");
  load(root_path, text);
  for (const auto& m : prog.modules) {
    for (const auto& c : m.constants) prog.constants.push_back(c);
    for (const auto& v : m.variables) prog.variables.push_back(v);
    for (const auto& d : m.defs) prog.defs[d->name] = d;
  }
  return prog;
}

}  // namespace tlagen
}  // namespace rmc
