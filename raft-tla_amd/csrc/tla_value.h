// raftmc host: TLA+ constant values (the subset TLC prints in traces) and the lookup
// of a trace literal inside a spec module.
//
// The punctuated-search constraints of tlc_membership/raft.tla
// (CommitWhenConcurrentLeaders_unique :1198-1204, MajorityOfClusterRestarts_constraint
// :1228-1234) embed a TLC error trace as a constant `[global |-> << ... >>]`.  The GPU
// backend compiles the constraint's logic, and the trace is data: mc_open takes it from
// the operator's definition in the module (or a module it EXTENDS, found next to it as
// TLC would), and mc_set_history_prefix accepts it from the caller.
#pragma once
#include <string>
#include <utility>
#include <vector>

namespace rmc {

struct TVal {
  enum Kind { Int, Str, MV, Bool, Set, Seq, Rec, Fcn } kind = Int;
  long long i = 0;
  std::string s;                                    // Str contents / MV name
  std::vector<TVal> elems;                          // Set / Seq elements; Fcn: key, value, key, value, ...
  std::vector<std::pair<std::string, TVal>> fields; // Rec fields, as written
  const TVal* field(const std::string& name) const;
  std::vector<std::string> field_names() const;     // sorted
  std::string text() const;                         // TLA+ text (atoms as the cfg reader prints them)
};

// Parse one value; throws CfgError(MC_E_PARSE).  Accepts integers, "strings", TRUE/FALSE,
// identifiers (model values), {sets}, <<sequences>>, [records |-> ...], TLC's function
// literals (k1 :> v1 @@ k2 :> v2), and \* / (* *) comments.
TVal parse_tla_value(const std::string& text);

// The `[global |-> <<...>>]` trace literal inside the definition of operator `op` in a module
// text, or in a module it EXTENDS (looked up as <dir>/<name>.tla, one level); "" if absent.
std::string find_trace_literal(const std::string& module_path, const std::string& op);

// TLC's trace-header location of action `op`: the span of the body of its definition
// `op == body` / `op(params) == body`, as "line L1, col C1 to line L2, col C2 of module M"
// (1-based, end inclusive; comments after the last token excluded).  Looked up in the module,
// then in the modules it EXTENDS (<dir>/<name>.tla, as TLC resolves them); "" if absent.
std::string action_location(const std::string& module_path, const std::string& op, int depth = 0);

// The history sequence of a trace value: the value itself if it is a sequence, else its
// `global` field (throws CfgError(MC_E_PARSE) otherwise).
const std::vector<TVal>& trace_global(const TVal& v);

}  // namespace rmc
