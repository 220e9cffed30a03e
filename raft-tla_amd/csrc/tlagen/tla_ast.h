// tla_ast.h — the SANY-subset front end's syntax tree and module loader.
//
// a general .tla/.cfg front end so specs run without hand-compilation.
// The subset is what the reference's TLC-checked modules use (thirdparty/raft_original.tla:97-464
// first): modules with EXTENDS / CONSTANT(S) / VARIABLE(S) / operator and function definitions,
// junction lists (/\ and \/ bullets aligned by column), LET/IN, IF/THEN/ELSE, CASE, \A / \E /
// CHOOSE over sets, set enumeration / filter / map, SUBSET, UNION, DOMAIN, function constructors
// and application, records, tuples, EXCEPT with ![..] / !.f paths and @, :> and @@, UNCHANGED,
// primes.  Temporal operators are parsed where they appear (Spec == Init /\ [][Next]_vars) and
// rejected only if evaluated.
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace rmc {
namespace tlagen {

struct Node;
typedef std::shared_ptr<Node> NP;

enum class K {
  Num, Str, Bool, Ident, OpApp,       // Ident: s; OpApp: s(args)
  Prime, Unchanged, Enabled, Temporal,
  Unary, Binary,                      // s = operator text ("~", "-", "DOMAIN", "SUBSET", "UNION"; "+", "\\in", ...)
  And, Or,                            // junction lists and infix /\ \/
  If, Case, Let, Forall, Exists, Choose,
  SetEnum, SetFilter, SetMap, FunCons, FunApp, Except, At, Record, RecordSet, FunSet, Tuple, Dot,
  Lambda,                             // LAMBDA x, y : e (fields = parameters, a[0] = body): an operator argument
  Unsupported
};

struct Bind { std::vector<std::string> names; NP set; bool tuple = false; };   // tuple: <<a, b>> \in S
struct PathStep { bool field = false; std::string name; NP idx; };   // ![idx] or !.name
struct Update { std::vector<PathStep> path; NP rhs; };
struct Def;

struct Node {
  K k;
  std::string s;                      // identifier / operator / field / string text
  long long n = 0;                    // Num value, Bool value
  std::vector<NP> a;                  // operands
  std::vector<Bind> binds;            // quantifiers, CHOOSE, filters, maps, constructors
  std::vector<Update> ups;            // EXCEPT
  std::vector<std::string> fields;    // Record / RecordSet field names (a[] holds the values)
  std::vector<std::shared_ptr<Def>> defs;   // LET
  int line = 0, col = 0;
  std::string module;                 // module the node was parsed from (locations in errors)
};

struct Def {
  std::string name;
  std::vector<std::string> params;
  std::vector<int> arity;              // per parameter: 0 for a value, k for an operator parameter F(_, .., _)
  NP body;                            // null if the body failed to parse (error kept in `error`)
  std::string error;
  std::string module;
  int line = 0;
};

struct Module {
  std::string name, path;
  std::vector<std::string> extends, constants, variables;
  std::vector<std::shared_ptr<Def>> defs;   // in text order
};

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Parse one module's text.  Definitions whose bodies fall outside the subset keep their error
// (reported only if the definition is used).  Throws ParseError on a malformed module header.
Module parse_module(const std::string& text, const std::string& path);

// A root module and every non-standard module it EXTENDS (transitively), found next to it as
// TLC does (<dir>/<Name>.tla) or through the `raftmc-base:` pragma of the repo's MC wrappers.
// Standard modules (Naturals, Integers, Sequences, FiniteSets, TLC, Bags) are built in.
struct Program {
  std::vector<Module> modules;                     // extended modules first, root last
  std::map<std::string, std::shared_ptr<Def>> defs; // later modules override earlier ones
  std::vector<std::string> constants, variables;   // in declaration order over all modules
};
Program load_program(const std::string& root_path, const std::vector<std::string>& search_dirs);

std::string node_where(const Node& n);

}  // namespace tlagen
}  // namespace rmc
