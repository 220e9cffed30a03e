// tla_gen.h — code generation of the SANY-subset front end: a TLA+ module + TLC cfg compiled
// into C++ over tlv.h (Init and Next as successor enumerators, constraints, invariants).
//
// Semantics follow TLC's state enumeration (tlc2.tool.Tool getInitStates / getNextStates):
// conjunctions are evaluated left to right, `x' = e` determines x' when it is still free and is
// a test once x' is determined, `x' \in S` and \E enumerate, disjunction branches, UNCHANGED
// determines each variable of its tuple, user operators are expanded at their use; every
// complete assignment of the primed variables is one generated successor.  Action names are
// TLC's split points: the definition whose body the enumeration was in when it stopped
// splitting (disjunctions, \E, LET and operator definitions split; anything else does not).
#pragma once
#include <string>
#include <vector>

#include "../model.h"
#include "tla_ast.h"

namespace rmc {
namespace tlagen {

struct Generated {
  std::string source;                    // C++ (namespace tlg) to be compiled with tlv.h
  std::vector<std::string> variables;    // state variables in word order
  std::vector<std::string> actions;      // action names (Next's split points)
  std::vector<std::string> invariants;   // cfg order
  std::vector<std::string> constraints;
  std::vector<std::string> atoms;        // atom id -> TLA+ text (model values bare, strings quoted)
  std::string init_name, next_name;
};

// Throws ParseError / CfgError(MC_E_UNSUPPORTED) for constructs outside the subset that the
// cfg's definitions reach.
Generated generate(const Program& prog, const CfgFile& cfg);

// One source file for hiprtc / a host compiler: tlv.h's text, the generated spec, and `tail`.
std::string compose_source(const Generated& g, const std::string& tlv_text, const std::string& tail);

}  // namespace tlagen
}  // namespace rmc
