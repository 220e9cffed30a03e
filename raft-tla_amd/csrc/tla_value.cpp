// raftmc host: TLA+ constant values and trace-literal lookup (see tla_value.h).
#include "tla_value.h"

#include <algorithm>
#include <cctype>

#include "../../include/raftmc.h"
#include "model.h"

namespace rmc {

const TVal* TVal::field(const std::string& name) const {
  for (auto& f : fields) if (f.first == name) return &f.second;
  return nullptr;
}

std::vector<std::string> TVal::field_names() const {
  std::vector<std::string> n;
  for (auto& f : fields) n.push_back(f.first);
  std::sort(n.begin(), n.end());
  return n;
}

std::string TVal::text() const {
  switch (kind) {
    case Int: return std::to_string(i);
    case Str: return "\"" + s + "\"";
    case MV: return s;
    case Bool: return i ? "TRUE" : "FALSE";
    case Set:
    case Seq: {
      std::string o = kind == Set ? "{" : "<<";
      for (size_t k = 0; k < elems.size(); ++k) o += (k ? ", " : "") + elems[k].text();
      return o + (kind == Set ? "}" : ">>");
    }
    case Fcn: {
      std::string o = "(";
      for (size_t k = 0; k + 1 < elems.size(); k += 2) o += (k ? " @@ " : "") + elems[k].text() + " :> " + elems[k + 1].text();
      return o + ")";
    }
    case Rec: {
      std::string o = "[";
      for (size_t k = 0; k < fields.size(); ++k) o += (k ? ", " : "") + fields[k].first + " |-> " + fields[k].second.text();
      return o + "]";
    }
  }
  return "?";
}

namespace {

struct Reader {
  const std::string& t;
  size_t p = 0;
  explicit Reader(const std::string& text, size_t at = 0) : t(text), p(at) {}
  [[noreturn]] void fail(const std::string& what) const {
    throw CfgError(MC_E_PARSE, "TLA+ value: " + what + " at offset " + std::to_string(p));
  }
  void ws() {
    for (;;) {
      while (p < t.size() && isspace((unsigned char)t[p])) ++p;
      if (t.compare(p, 2, "\\*") == 0) { while (p < t.size() && t[p] != '\n') ++p; continue; }
      if (t.compare(p, 2, "(*") == 0) {
        int depth = 1; p += 2;
        while (p < t.size() && depth) {
          if (t.compare(p, 2, "(*") == 0) { ++depth; p += 2; }
          else if (t.compare(p, 2, "*)") == 0) { --depth; p += 2; }
          else ++p;
        }
        if (depth) fail("unterminated comment");
        continue;
      }
      return;
    }
  }
  bool eat(const char* tok) {
    ws();
    const size_t n = std::char_traits<char>::length(tok);
    if (t.compare(p, n, tok) == 0) { p += n; return true; }
    return false;
  }
  void expect(const char* tok) { if (!eat(tok)) fail(std::string("'") + tok + "' expected"); }
  std::string ident() {
    ws();
    const size_t b = p;
    while (p < t.size() && (isalnum((unsigned char)t[p]) || t[p] == '_')) ++p;
    if (b == p) fail("identifier expected");
    return t.substr(b, p - b);
  }
  // a comma-separated list up to `close`
  template <class F>
  void list(const char* close, F item) {
    if (eat(close)) return;
    for (;;) {
      item();
      if (eat(close)) return;
      expect(",");
    }
  }
  TVal value() {
    ws();
    if (p >= t.size()) fail("value expected");
    TVal v;
    if (eat("<<")) { v.kind = TVal::Seq; list(">>", [&] { v.elems.push_back(value()); }); return v; }
    if (eat("{")) { v.kind = TVal::Set; list("}", [&] { v.elems.push_back(value()); }); return v; }
    if (eat("[")) {
      v.kind = TVal::Rec;
      list("]", [&] {
        std::string f = ident();
        expect("|->");
        v.fields.push_back({f, value()});
      });
      return v;
    }
    if (eat("(")) {   // TLC function literal: k :> v @@ k :> v
      v.kind = TVal::Fcn;
      do {
        v.elems.push_back(value());
        expect(":>");
        v.elems.push_back(value());
      } while (eat("@@"));
      expect(")");
      return v;
    }
    if (t[p] == '"') {
      const size_t e = t.find('"', p + 1);
      if (e == std::string::npos) fail("unterminated string");
      v.kind = TVal::Str; v.s = t.substr(p + 1, e - p - 1); p = e + 1;
      return v;
    }
    const bool neg = t[p] == '-';
    if (neg || isdigit((unsigned char)t[p])) {
      if (neg) ++p;
      const size_t b = p;
      while (p < t.size() && isdigit((unsigned char)t[p])) ++p;
      if (b == p) fail("digits expected");
      v.kind = TVal::Int; v.i = std::stoll(t.substr(b, p - b)); if (neg) v.i = -v.i;
      return v;
    }
    const std::string id = ident();
    if (id == "TRUE" || id == "FALSE") { v.kind = TVal::Bool; v.i = id == "TRUE"; return v; }
    v.kind = TVal::MV; v.s = id;
    return v;
  }
};

std::string dir_of(const std::string& path) {
  const size_t k = path.find_last_of('/');
  return k == std::string::npos ? std::string(".") : path.substr(0, k);
}

// the text of the definition `op == ...` up to the next top-level definition or the module end
std::string definition_of(const std::string& text, const std::string& op) {
  size_t at = 0;
  for (;;) {
    at = text.find(op, at);
    if (at == std::string::npos) return "";
    const bool line_start = at == 0 || text[at - 1] == '\n';
    size_t q = at + op.size();
    while (q < text.size() && (text[q] == ' ' || text[q] == '\t')) ++q;
    if (line_start && text.compare(q, 2, "==") == 0) break;
    at += op.size();
  }
  size_t end = at + op.size(), scan = text.find('\n', at);
  while (scan != std::string::npos) {
    const size_t ls = scan + 1;
    if (ls >= text.size()) { end = text.size(); break; }
    if (isalpha((unsigned char)text[ls]) || text.compare(ls, 4, "====") == 0) { end = ls; break; }
    scan = text.find('\n', ls);
    end = text.size();
  }
  return text.substr(at, end - at);
}

std::vector<std::string> extends_of(const std::string& text) {
  std::vector<std::string> out;
  const size_t at = text.find("EXTENDS");
  if (at == std::string::npos) return out;
  const size_t eol = text.find('\n', at);
  std::string line = text.substr(at + 7, (eol == std::string::npos ? text.size() : eol) - at - 7);
  std::string cur;
  for (char ch : line + ",") {
    if (isalnum((unsigned char)ch) || ch == '_') cur += ch;
    else if (!cur.empty()) { out.push_back(cur); cur.clear(); }
  }
  return out;
}

std::string literal_in(const std::string& def) {
  for (size_t at = def.find('['); at != std::string::npos; at = def.find('[', at + 1)) {
    Reader r(def, at + 1);
    r.ws();
    if (def.compare(r.p, 6, "global") != 0) continue;
    r.p += 6;
    if (!r.eat("|->")) continue;
    Reader v(def, at);
    v.value();
    return def.substr(at, v.p - at);
  }
  return "";
}

}  // namespace

TVal parse_tla_value(const std::string& text) {
  Reader r(text);
  TVal v = r.value();
  r.ws();
  if (r.p != text.size()) r.fail("trailing text");
  return v;
}

std::string find_trace_literal(const std::string& module_path, const std::string& op) {
  std::string text;
  try { text = read_text_file(module_path); } catch (const CfgError&) { return ""; }
  const std::string def = definition_of(text, op);
  if (!def.empty()) return literal_in(def);
  for (const auto& m : extends_of(text)) {
    std::string sub;
    try { sub = read_text_file(dir_of(module_path) + "/" + m + ".tla"); } catch (const CfgError&) { continue; }
    const std::string d = definition_of(sub, op);
    if (!d.empty()) return literal_in(d);
  }
  return "";
}

namespace {

// offset of the first significant character at or after p (skips blanks, `\*` and nested `(* *)` comments)
size_t skip_blank(const std::string& t, size_t p) {
  while (p < t.size()) {
    if (isspace((unsigned char)t[p])) { ++p; continue; }
    if (t.compare(p, 2, "\\*") == 0) { p = t.find('\n', p); if (p == std::string::npos) return t.size(); continue; }
    if (t.compare(p, 2, "(*") == 0) {
      int depth = 0;
      while (p < t.size()) {
        if (t.compare(p, 2, "(*") == 0) { ++depth; p += 2; }
        else if (t.compare(p, 2, "*)") == 0) { p += 2; if (--depth == 0) break; }
        else ++p;
      }
      continue;
    }
    break;
  }
  return p;
}

// offset just past `op` or `op(params)` followed by `==`, for a definition that starts a line
size_t definition_body(const std::string& t, const std::string& op, size_t& head) {
  for (size_t at = t.find(op); at != std::string::npos; at = t.find(op, at + 1)) {
    if (at != 0 && t[at - 1] != '\n') continue;
    size_t q = at + op.size();
    if (q < t.size() && (isalnum((unsigned char)t[q]) || t[q] == '_')) continue;
    while (q < t.size() && (t[q] == ' ' || t[q] == '\t')) ++q;
    if (q < t.size() && t[q] == '(') {
      const size_t close = t.find(')', q);
      if (close == std::string::npos) continue;
      q = close + 1;
      while (q < t.size() && (t[q] == ' ' || t[q] == '\t')) ++q;
    }
    if (t.compare(q, 2, "==") != 0) continue;
    head = at;
    return q + 2;
  }
  return std::string::npos;
}

void line_col(const std::string& t, size_t off, int& line, int& col) {
  line = 1;
  size_t ls = 0;
  for (size_t k = 0; k < off; ++k)
    if (t[k] == '\n') { ++line; ls = k + 1; }
  col = (int)(off - ls) + 1;
}

std::string module_name(const std::string& t) {
  const size_t at = t.find("MODULE");
  if (at == std::string::npos) return "";
  Reader r(t, at + 6);
  try { return r.ident(); } catch (const CfgError&) { return ""; }
}

}  // namespace

std::string action_location(const std::string& module_path, const std::string& op, int depth) {
  std::string t;
  try { t = read_text_file(module_path); } catch (const CfgError&) { return ""; }
  size_t head = 0;
  const size_t eq = definition_body(t, op, head);
  if (eq == std::string::npos) {
    if (depth >= 4) return "";
    for (const auto& m : extends_of(t)) {
      const std::string loc = action_location(dir_of(module_path) + "/" + m + ".tla", op, depth + 1);
      if (!loc.empty()) return loc;
    }
    return "";
  }
  // the unit ends at the next line that starts a definition or a separator
  size_t unit_end = t.size();
  for (size_t nl = t.find('\n', head); nl != std::string::npos; nl = t.find('\n', nl + 1)) {
    const size_t ls = nl + 1;
    if (ls >= t.size()) break;
    if (isalpha((unsigned char)t[ls]) || t.compare(ls, 4, "----") == 0 || t.compare(ls, 4, "====") == 0) { unit_end = ls; break; }
  }
  const size_t begin = skip_blank(t, eq);
  if (begin >= unit_end) return "";
  size_t last = begin;   // last significant character of the body
  for (size_t p = begin; p < unit_end;) {
    const size_t q = skip_blank(t, p);
    if (q >= unit_end) break;
    if (t[q] == '"') {
      size_t e = q + 1;
      while (e < unit_end && t[e] != '"') e += t[e] == '\\' ? 2 : 1;
      last = std::min(e, unit_end - 1);
      p = e + 1;
      continue;
    }
    last = q;
    p = q + 1;
  }
  int l0, c0, l1, c1;
  line_col(t, begin, l0, c0);
  line_col(t, last, l1, c1);
  return "line " + std::to_string(l0) + ", col " + std::to_string(c0) + " to line " + std::to_string(l1) + ", col " +
         std::to_string(c1) + " of module " + module_name(t);
}

const std::vector<TVal>& trace_global(const TVal& v) {
  if (v.kind == TVal::Seq) return v.elems;
  if (v.kind == TVal::Rec) {
    const TVal* g = v.field("global");
    if (g && g->kind == TVal::Seq) return g->elems;
  }
  throw CfgError(MC_E_PARSE, "a history trace is a sequence or a record with a `global` sequence");
}

}  // namespace rmc
