// raftmc host: TLC .cfg reader and spec/model resolution.
//
// Reads the cfg language of tlc_membership/raft.cfg:1-87 (CONSTANT(S) with
// `=` / `<-`, SYMMETRY, VIEW, INIT, NEXT, CONSTRAINT(S), ACTION_CONSTRAINT(S),
// INVARIANT(S), \* and (* *) comments) and identifies the spec module: the
// reference files themselves (by their declarations) or an MC wrapper under
// configs/ carrying a `raftmc-base:` pragma.  The Raft Next relations are
// hand-compiled, so the module text selects the compiled spec; every cfg
// name must resolve to a compiled predicate or mc_open fails.
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace rmc {

struct CfgError : std::runtime_error {
  int code;
  CfgError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// A constant's value as the cfg assigns it (printed with TLC's conventions).
struct CVal {
  enum Kind { Int, Str, MV, Bool, Set } kind = MV;
  long long i = 0;
  std::string s;              // Str contents / MV name
  std::vector<CVal> elems;    // Set elements
  std::string text() const;   // TLA+ text; sets print their elements sorted by text
};

struct CfgFile {
  std::vector<std::pair<std::string, CVal>> constants;
  std::vector<std::pair<std::string, std::string>> overrides;
  std::string init, next, symmetry, view;
  std::vector<std::string> constraints, action_constraints, invariants, properties;
  bool has(const std::string& n) const;
  const CVal& get(const std::string& n) const;
};

CfgFile parse_cfg_text(const std::string& text);
std::string read_text_file(const std::string& path);
std::string detect_spec_family(const std::string& tla_text);   // "raft_original" | "tlc_membership"

}  // namespace rmc
