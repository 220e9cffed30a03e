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

const std::vector<TVal>& trace_global(const TVal& v) {
  if (v.kind == TVal::Seq) return v.elems;
  if (v.kind == TVal::Rec) {
    const TVal* g = v.field("global");
    if (g && g->kind == TVal::Seq) return g->elems;
  }
  throw CfgError(MC_E_PARSE, "a history trace is a sequence or a record with a `global` sequence");
}

}  // namespace rmc
