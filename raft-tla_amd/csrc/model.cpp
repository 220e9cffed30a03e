// raftmc host: TLC .cfg reader (see model.h).
#include "model.h"

#include <algorithm>
#include <cctype>
#include <fstream>
#include <sstream>

#include "../../include/raftmc.h"

namespace rmc {

std::string CVal::text() const {
  switch (kind) {
    case Int: return std::to_string(i);
    case Str: return "\"" + s + "\"";
    case MV: return s;
    case Bool: return i ? "TRUE" : "FALSE";
    case Set: {
      std::vector<std::string> t;
      for (auto& e : elems) t.push_back(e.text());
      std::sort(t.begin(), t.end());
      t.erase(std::unique(t.begin(), t.end()), t.end());
      std::string o = "{";
      for (size_t k = 0; k < t.size(); ++k) o += (k ? ", " : "") + t[k];
      return o + "}";
    }
  }
  return "?";
}

bool CfgFile::has(const std::string& n) const {
  for (auto& c : constants) if (c.first == n) return true;
  return false;
}
const CVal& CfgFile::get(const std::string& n) const {
  for (auto& c : constants) if (c.first == n) return c.second;
  throw CfgError(MC_E_UNSUPPORTED, "constant '" + n + "' is not assigned in the cfg");
}

static std::vector<std::string> tokens(const std::string& text) {
  std::vector<std::string> out;
  size_t i = 0, n = text.size();
  while (i < n) {
    char c = text[i];
    if (isspace((unsigned char)c)) { ++i; continue; }
    if (c == '\\' && i + 1 < n && text[i + 1] == '*') { while (i < n && text[i] != '\n') ++i; continue; }
    if (c == '(' && i + 1 < n && text[i + 1] == '*') {
      int depth = 1; i += 2;
      while (i < n && depth) {
        if (text.compare(i, 2, "(*") == 0) { ++depth; i += 2; }
        else if (text.compare(i, 2, "*)") == 0) { --depth; i += 2; }
        else ++i;
      }
      if (depth) throw CfgError(MC_E_PARSE, "cfg: unterminated comment");
      continue;
    }
    if (c == '"') {
      size_t j = text.find('"', i + 1);
      if (j == std::string::npos) throw CfgError(MC_E_PARSE, "cfg: unterminated string");
      out.push_back(text.substr(i, j - i + 1)); i = j + 1; continue;
    }
    if (text.compare(i, 2, "<-") == 0) { out.push_back("<-"); i += 2; continue; }
    if (c == '{' || c == '}' || c == ',' || c == '=' || c == '-') { out.push_back(std::string(1, c)); ++i; continue; }
    size_t j = i;
    while (j < n && (isalnum((unsigned char)text[j]) || text[j] == '_')) ++j;
    if (j == i) throw CfgError(MC_E_PARSE, std::string("cfg: unexpected character '") + c + "'");
    out.push_back(text.substr(i, j - i)); i = j;
  }
  return out;
}

static bool is_section(const std::string& t) {
  static const char* kw[] = {"CONSTANT", "CONSTANTS", "SYMMETRY", "VIEW", "INIT", "NEXT", "SPECIFICATION",
                             "CONSTRAINT", "CONSTRAINTS", "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS",
                             "INVARIANT", "INVARIANTS", "PROPERTY", "PROPERTIES", "CHECK_DEADLOCK", "ALIAS", "POSTCONDITION"};
  for (auto k : kw) if (t == k) return true;
  return false;
}

static CVal value(const std::vector<std::string>& tk, size_t& p) {
  if (p >= tk.size()) throw CfgError(MC_E_PARSE, "cfg: value expected");
  const std::string& t = tk[p];
  CVal v;
  if (t == "{") {
    ++p; v.kind = CVal::Set;
    while (p < tk.size() && tk[p] != "}") {
      v.elems.push_back(value(tk, p));
      if (p < tk.size() && tk[p] == ",") ++p;
    }
    if (p >= tk.size()) throw CfgError(MC_E_PARSE, "cfg: '}' expected");
    ++p; return v;
  }
  if (t == "-") { ++p; v.kind = CVal::Int; v.i = -std::stoll(tk.at(p++)); return v; }
  if (t[0] == '"') { ++p; v.kind = CVal::Str; v.s = t.substr(1, t.size() - 2); return v; }
  if (isdigit((unsigned char)t[0])) { ++p; v.kind = CVal::Int; v.i = std::stoll(t); return v; }
  if (t == "TRUE" || t == "FALSE") { ++p; v.kind = CVal::Bool; v.i = t == "TRUE"; return v; }
  ++p; v.kind = CVal::MV; v.s = t;   // identifiers on the right-hand side are model values
  return v;
}

static bool is_ident(const std::string& t) {
  if (t.empty() || !(isalpha((unsigned char)t[0]) || t[0] == '_')) return false;
  for (char ch : t) if (!(isalnum((unsigned char)ch) || ch == '_')) return false;
  return true;
}

CfgFile parse_cfg_text(const std::string& text) {
  CfgFile c;
  auto tk = tokens(text);
  size_t p = 0;
  std::string sec;
  auto one = [&](std::string& dst) {
    if (!dst.empty()) throw CfgError(MC_E_PARSE, "cfg: " + sec + " given twice");
    dst = tk[p++];
  };
  while (p < tk.size()) {
    const std::string& t = tk[p];
    if (is_section(t)) { sec = t; ++p; continue; }
    if (!is_ident(t)) throw CfgError(MC_E_PARSE, "cfg: identifier expected, found '" + t + "'");
    if (sec == "CONSTANT" || sec == "CONSTANTS") {
      std::string name = tk[p++];
      if (p < tk.size() && tk[p] == "=") { ++p; c.constants.push_back({name, value(tk, p)}); }
      else if (p < tk.size() && tk[p] == "<-") { ++p; c.overrides.push_back({name, tk.at(p++)}); }
      else { CVal v; v.kind = CVal::MV; v.s = name; c.constants.push_back({name, v}); }
    } else if (sec == "SYMMETRY") one(c.symmetry);
    else if (sec == "VIEW") one(c.view);
    else if (sec == "INIT") one(c.init);
    else if (sec == "NEXT") one(c.next);
    else if (sec == "CONSTRAINT" || sec == "CONSTRAINTS") c.constraints.push_back(tk[p++]);
    else if (sec == "ACTION_CONSTRAINT" || sec == "ACTION_CONSTRAINTS") c.action_constraints.push_back(tk[p++]);
    else if (sec == "INVARIANT" || sec == "INVARIANTS") c.invariants.push_back(tk[p++]);
    else if (sec == "PROPERTY" || sec == "PROPERTIES") c.properties.push_back(tk[p++]);
    else if (sec == "SPECIFICATION") throw CfgError(MC_E_UNSUPPORTED, "cfg: SPECIFICATION is not supported; use INIT/NEXT");
    else throw CfgError(MC_E_PARSE, "cfg: token outside any section: " + t);
  }
  if (c.init.empty()) c.init = "Init";
  if (c.next.empty()) c.next = "Next";
  return c;
}

std::string read_text_file(const std::string& path) {
  std::ifstream f(path);
  if (!f) throw CfgError(MC_E_IO, "cannot open " + path);
  std::stringstream ss; ss << f.rdbuf();
  return ss.str();
}

std::string detect_spec_family(const std::string& t) {
  if (t.find("raftmc-base: thirdparty/raft_original.tla") != std::string::npos) return "raft_original";
  if (t.find("raftmc-base: tlc_membership/raft.tla") != std::string::npos) return "tlc_membership";
  if (t.find("VARIABLE elections") != std::string::npos && t.find("VARIABLE allLogs") != std::string::npos) return "raft_original";
  if (t.find("NextAsyncCrash") != std::string::npos && t.find("CatchupRequest") != std::string::npos) return "tlc_membership";
  throw CfgError(MC_E_UNSUPPORTED, "unrecognised spec module (expected raft_original.tla, tlc_membership/raft.tla, or a configs/ MC wrapper)");
}

}  // namespace rmc
