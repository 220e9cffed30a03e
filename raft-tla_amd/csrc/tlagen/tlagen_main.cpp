// tlagen — the front end as a command: parse a TLA+ module (+ the modules it EXTENDS) and a TLC
// cfg, and print the generated C++ (tlv.h + namespace tlg) that the GPU path compiles.
//
//   tlagen SPEC.tla CFG.cfg [-I DIR]... [-o OUT] [--parse-only] [--kernels]
//
// --parse-only parses every definition of every module and reports the ones outside the subset
// (what SANY's parse of the module would reject is a parse error here too).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>

#include "../model.h"
#include "tla_gen.h"
#include "tlv_text.h"

int main(int argc, char** argv) {
  using namespace rmc;
  std::string spec, cfgp, out;
  std::vector<std::string> dirs;
  bool parse_only = false, kernels = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-I" && i + 1 < argc) dirs.push_back(argv[++i]);
    else if (a == "-o" && i + 1 < argc) out = argv[++i];
    else if (a == "--parse-only") parse_only = true;
    else if (a == "--kernels") kernels = true;
    else if (spec.empty()) spec = a;
    else cfgp = a;
  }
  if (spec.empty() || (cfgp.empty() && !parse_only)) {
    std::fprintf(stderr, "usage: tlagen SPEC.tla CFG.cfg [-I DIR]... [-o OUT] [--parse-only]\n");
    return 2;
  }
  try {
    tlagen::Program prog = tlagen::load_program(spec, dirs);
    if (parse_only) {
      int bad = 0, total = 0;
      for (auto& m : prog.modules) {
        for (auto& d : m.defs) {
          ++total;
          if (!d->body) { ++bad; std::printf("%s: %s: %s\n", m.name.c_str(), d->name.c_str(), d->error.c_str()); }
        }
        std::printf("module %s: %zu constants, %zu variables, %zu definitions\n", m.name.c_str(), m.constants.size(),
                    m.variables.size(), m.defs.size());
      }
      std::printf("{\"modules\": %zu, \"definitions\": %d, \"unparsed\": %d}\n", prog.modules.size(), total, bad);
      return bad ? 1 : 0;
    }
    CfgFile cfg = parse_cfg_text(read_text_file(cfgp));
    tlagen::Generated g = tlagen::generate(prog, cfg);
    const std::string src = tlagen::compose_source(g, kTlvText, kernels ? kTlgKernelsText : "");
    if (out.empty()) std::cout << src;
    else { std::ofstream f(out); f << src; }
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "tlagen: %s\n", e.what());
    return 1;
  }
}
