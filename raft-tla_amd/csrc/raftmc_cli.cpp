// raftmc — command-line front end mirroring TLC's flags:
//   raftmc [-config F.cfg] [-workers N] [-deadlock] [-depth D] [-device K]
//          [-fptable BYTES] [-store BYTES] [-seed S] [-no-inv-oom] [-no-disjunct-copies] [-dump FILE] [-json]
//          [-checkpoint LEVELS] [-checkpoint-file FILE] [-recover FILE] [-symmetry tlc|orbit]
//          [-gpus N] [-countfinal] F.tla
// (-countfinal, with -depth D and -workers N: the states at depth D are counted and checked, not
// stored; mc_opts.count_final_level)
// (-gpus N: the node's GPUs -device .. -device+N-1 share one search, owner-partitioned fingerprints,
// one host thread per GPU over an in-process RCCL communicator; TLC's -workers keeps its meaning)
// (-checkpoint counts BFS levels where TLC counts minutes; the file defaults to states/raftmc.ckpt)
// Prints TLC-style lines and exits with TLC-like codes (0 ok, 12 safety
// violation, 11 deadlock, 75 error).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include <sys/stat.h>

#include "../../include/raftmc.h"

int main(int argc, char** argv) {
  mc_opts o;
  mc_default_opts(&o);
  std::string tla, cfg, dump, ckpt_file = "states/raftmc.ckpt", recover;
  int ckpt_every = 0;
  bool json = false;
  for (int a = 1; a < argc; ++a) {
    std::string k = argv[a];
    auto val = [&]() -> const char* {
      if (a + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", k.c_str()); std::exit(2); }
      return argv[++a];
    };
    if (k == "-config") cfg = val();
    else if (k == "-workers") o.workers = std::atoi(val());
    else if (k == "-deadlock") o.check_deadlock = 0;   // TLC: -deadlock turns deadlock checking OFF
    else if (k == "-depth") o.max_depth = std::atoll(val());
    else if (k == "-countfinal") o.count_final_level = 1;
    else if (k == "-device") o.device = std::atoi(val());
    else if (k == "-gpus") o.n_gpus = std::atoi(val());
    else if (k == "-frontend") {   // "auto" (default), "generated" (the SANY-subset front end for any module), "hand"
      const std::string v = val();
      o.frontend = v == "generated" ? MC_FRONTEND_GENERATED : v == "hand" ? MC_FRONTEND_HAND : MC_FRONTEND_AUTO;
    }
    else if (k == "-fptable") o.fp_table_bytes = std::strtoull(val(), nullptr, 10);
    else if (k == "-store") o.state_store_bytes = std::strtoull(val(), nullptr, 10);
    else if (k == "-seed") o.seed = std::strtoull(val(), nullptr, 0);
    else if (k == "-no-inv-oom") o.tlc_compat_flags &= ~MC_COMPAT_INV_OUT_OF_MODEL;
    else if (k == "-no-disjunct-copies") o.tlc_compat_flags &= ~MC_COMPAT_DISJUNCT_COPIES;   // a disjunctive guard's successor counted once
    else if (k == "-symmetry") {   // "tlc" (default): TLC's least-permuted-state rule; "orbit": the faster orbit mode
      const std::string v = val();
      if (v == "tlc") o.tlc_compat_flags |= MC_COMPAT_SYM_TLC;
      else if (v == "orbit") o.tlc_compat_flags &= ~MC_COMPAT_SYM_TLC;
      else { std::fprintf(stderr, "-symmetry tlc|orbit\n"); return 2; }
    }
    else if (k == "-dump") dump = val();
    else if (k == "-json") json = true;
    else if (k == "-checkpoint") ckpt_every = std::atoi(val());
    else if (k == "-checkpoint-file") ckpt_file = val();
    else if (k == "-recover") recover = val();
    else if (!k.empty() && k[0] == '-') { std::fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
    else tla = k;
  }
  if (tla.empty()) { std::fprintf(stderr, "usage: raftmc [-config F.cfg] [options] F.tla\n"); return 2; }
  if (cfg.empty()) { cfg = tla.substr(0, tla.size() > 4 ? tla.size() - 4 : tla.size()) + ".cfg"; }
  mc_ctx* c = nullptr;
  int rc = mc_open(tla.c_str(), cfg.c_str(), &o, &c);
  if (rc) { std::fprintf(stderr, "raftmc: %s (code %d)\n", c ? mc_last_error(c) : "open failed", rc); mc_close(c); return 75; }
  if (!rc && ckpt_every > 0) {
    if (ckpt_file == "states/raftmc.ckpt") (void)::mkdir("states", 0755);
    rc = mc_set_checkpoint(c, ckpt_file.c_str(), ckpt_every);
  }
  if (!rc && !recover.empty()) rc = mc_set_recover(c, recover.c_str());
  if (rc) { std::fprintf(stderr, "raftmc: %s (code %d)\n", mc_last_error(c), rc); mc_close(c); return 75; }
  rc = mc_run(c);
  if (rc == 0) {   // TLC prints its fingerprint-based estimate after a completed search
    mc_summary_t s;
    double v = 0;
    if (mc_summary(c, &s) == 0 && s.verdict == MC_VERDICT_OK && o.n_gpus == 1) (void)mc_collision_observed(c, &v);
  }
  if (rc) { std::fprintf(stderr, "raftmc: %s (code %d)\n", mc_last_error(c), rc); mc_close(c); return 75; }
  char* text = nullptr; size_t len = 0;
  mc_report(c, &text, &len);
  std::fwrite(text, 1, len, stdout);
  mc_free(text);
  if (json) {
    mc_summary_t s; mc_summary(c, &s);
    std::printf("{\"verdict\": %d, \"generated\": %lld, \"distinct\": %lld, \"depth\": %lld, \"seconds\": %.6f, \"kernel_seconds\": %.6f}\n",
                s.verdict, (long long)s.generated, (long long)s.distinct, (long long)s.depth, s.seconds_total, s.seconds_kernels);
  }
  if (!dump.empty() && mc_dump_states(c, dump.c_str())) std::fprintf(stderr, "raftmc: dump failed: %s\n", mc_last_error(c));
  int ec = mc_exit_code(c);
  mc_close(c);
  return ec;
}
