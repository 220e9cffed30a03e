// raftmc — C ABI implementation (include/raftmc.h).  Parses the .tla/.cfg,
// picks the compiled spec backend, drives mc_run and renders TLC-style text.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#define RAFTMC_BUILDING_LIBRARY 1   // the header's inline mc_default_opts is for callers
#include "../../include/raftmc.h"
#include "backend.h"
#include "model.h"
#include "rccl_api.h"
#include "shard_transport.h"
#include "tla_value.h"

struct mc_ctx {
  std::unique_ptr<rmc::Backend> be;
  rmc::RunOpts ro;
  rmc::RunResult res;
  bool ran = false;
  bool released = false;   // mc_release_device_memory since the last run
  std::string last_error, tla_path, cfg_path;
  mutable std::map<std::string, std::string> action_loc;   // action name -> TLC location text ("" if none)
  const std::string& location_of(const std::string& act) const {
    auto it = action_loc.find(act);
    if (it == action_loc.end()) it = action_loc.emplace(act, rmc::action_location(tla_path, act)).first;
    return it->second;
  }
  // RCCL communicator of the native sharded loop, kept across runs of the same job
  ncclComm_t comm = nullptr;
  int comm_rank = -1, comm_world = 0;
  char comm_id[sizeof(ncclUniqueId)] = {0};
  // mc_opts.n_gpus > 1: the backends of ranks 1.. (rank 0 is `be`), one per GPU, and their in-process
  // RCCL communicators (ncclCommInitAll, kept across runs)
  int n_gpus = 1;
  bool same_device = false;
  std::vector<std::unique_ptr<rmc::Backend>> peers;
  std::vector<ncclComm_t> local_comms;
  ~mc_ctx() {
    be.reset();
    peers.clear();
    if (comm) (void)rmc::rccl().CommDestroy(comm);
    for (ncclComm_t x : local_comms) if (x) (void)rmc::rccl().CommDestroy(x);
  }
  rmc::Backend* rank_backend(int r) const { return r == 0 ? be.get() : peers[r - 1].get(); }
};

namespace {
char* dup_text(const std::string& s, size_t* len) {
  char* p = (char*)std::malloc(s.size() + 1);
  if (!p) return nullptr;
  std::memcpy(p, s.c_str(), s.size() + 1);
  if (len) *len = s.size();
  return p;
}
const char* verdict_name(int v) {
  switch (v) {
    case MC_VERDICT_OK: return "OK";
    case MC_VERDICT_INVARIANT_VIOLATION: return "INVARIANT_VIOLATION";
    case MC_VERDICT_EVAL_ERROR: return "EVAL_ERROR";
    case MC_VERDICT_CAPACITY_OVERFLOW: return "CAPACITY_OVERFLOW";
    case MC_VERDICT_DEADLOCK: return "DEADLOCK";
    case MC_VERDICT_DEPTH_LIMIT: return "DEPTH_LIMIT";
  }
  return "?";
}
// TLC's header: "State k: <Action line L1, col C1 to line L2, col C2 of module M>" when the
// action's definition is found in the spec module (or a module it EXTENDS), else "<Action>"
std::string trace_text(const mc_ctx* c, const rmc::RunResult& r) {
  std::ostringstream o;
  for (size_t k = 0; k < r.trace.size(); ++k) {
    o << "State " << (k + 1) << ": ";
    if (k == 0) o << "<Initial predicate>";
    else {
      const std::string& loc = c->location_of(r.trace[k].first);
      o << "<" << r.trace[k].first << (loc.empty() ? "" : " " + loc) << ">";
    }
    o << "\n";
    o << r.trace[k].second << "\n\n";
  }
  return o.str();
}
}  // namespace

extern "C" {

namespace {
bool abi_supported(int32_t v) { return v == 2 || v == RAFTMC_ABI_VERSION; }   // 2 and 3 share the layouts
void fill_default_opts(mc_opts* o) {
  std::memset(o, 0, sizeof *o);
  o->n_gpus = 1;
  o->workers = 1;
  o->tlc_compat_flags = MC_COMPAT_INV_OUT_OF_MODEL | MC_COMPAT_SYM_TLC | MC_COMPAT_DISJUNCT_COPIES;   // TLC's: the drop-in semantics
  o->check_deadlock = 1;
  o->block_size = 256;
}
}  // namespace

int mc_opts_init(mc_opts* o, int32_t caller_abi_version) {
  if (!o) return MC_E_INVALID;
  fill_default_opts(o);
  o->abi_version = caller_abi_version;
  return abi_supported(caller_abi_version) ? MC_OK : MC_E_INVALID;
}

// binaries built before ABI 3 call this symbol: their layout is unknown, so the version stays 0 and
// mc_open refuses the opts (include/raftmc.h)
void mc_default_opts(mc_opts* o) {
  if (!o) return;
  fill_default_opts(o);
}

int mc_open(const char* tla_path, const char* cfg_path, const mc_opts* o, mc_ctx** out) {
  if (!tla_path || !cfg_path || !out) return MC_E_INVALID;
  *out = nullptr;
  auto* c = new mc_ctx();
  c->tla_path = tla_path; c->cfg_path = cfg_path;
  mc_opts d; mc_opts_init(&d, RAFTMC_ABI_VERSION);
  if (!o) o = &d;
  if (!abi_supported(o->abi_version)) { delete c; return MC_E_INVALID; }
  if (o->n_gpus < 1 || o->n_gpus > 8) { delete c; return MC_E_INVALID; }
  c->n_gpus = o->n_gpus;
  c->same_device = o->same_device != 0;
  c->ro.device = o->device;
  c->ro.fp_table_bytes = o->fp_table_bytes;
  c->ro.state_store_bytes = o->state_store_bytes;
  c->ro.max_depth = o->max_depth;
  c->ro.seed = o->seed;
  c->ro.inv_out_of_model = (o->tlc_compat_flags & MC_COMPAT_INV_OUT_OF_MODEL) != 0;
  c->ro.sym_tlc = (o->tlc_compat_flags & MC_COMPAT_SYM_TLC) != 0;
  c->ro.disjunct_copies = (o->tlc_compat_flags & MC_COMPAT_DISJUNCT_COPIES) != 0;
  c->ro.check_deadlock = o->check_deadlock != 0;
  c->ro.block_size = o->block_size ? o->block_size : 256;
  c->ro.workers = o->workers;
  c->ro.count_final_level = o->count_final_level != 0;
  try {
    if (o->frontend < MC_FRONTEND_AUTO || o->frontend > MC_FRONTEND_HAND) throw rmc::CfgError(MC_E_INVALID, "bad mc_opts.frontend");
    std::string fam;
    const std::string tla_text = rmc::read_text_file(tla_path);
    if (o->frontend == MC_FRONTEND_GENERATED) fam = "tlagen";
    else {
      try { fam = rmc::detect_spec_family(tla_text); }
      catch (const rmc::CfgError&) { if (o->frontend == MC_FRONTEND_HAND) throw; fam = "tlagen"; }
    }
    rmc::CfgFile cfg = rmc::parse_cfg_text(rmc::read_text_file(cfg_path));
    // count_final_level exists for raft_original's -workers N search with a depth bound (single GPU
    // or sharded): anywhere else it would be silently ignored, so it is refused
    if (o->count_final_level && (fam != "raft_original" || o->workers == 1 || o->max_depth <= 0))
      throw rmc::CfgError(MC_E_UNSUPPORTED, "count_final_level needs thirdparty/raft_original.tla (hand-compiled), workers != 1 "
                                            "and max_depth > 0");
    if (fam == "tlagen" && c->n_gpus > 1) throw rmc::CfgError(MC_E_UNSUPPORTED, "the generated path runs on one GPU (n_gpus = 1)");
    auto make = [&]() -> rmc::Backend* {
      if (fam == "raft_original") return rmc::make_orig_backend(cfg);
      if (fam == "tlc_membership") return rmc::make_memb_backend(cfg);
      if (fam == "tlagen") return rmc::make_tlagen_backend(tla_path, cfg);
      throw rmc::CfgError(MC_E_UNSUPPORTED, "spec family '" + fam + "' has no GPU backend in this build");
    };
    c->be.reset(make());
    for (int r = 1; r < c->n_gpus; ++r) c->peers.emplace_back(make());   // one compiled model per GPU
    // the golden traces of punctuated-search constraints are operator definitions of the module
    // (or of a module it EXTENDS, next to it); the caller may also pass them (mc_set_history_prefix)
    for (const auto& con : c->be->history_prefixes_needed()) {
      const std::string lit = rmc::find_trace_literal(tla_path, con);
      if (lit.empty()) continue;
      std::string err;
      for (int r = 0; r < c->n_gpus; ++r)
        if (int rc = c->rank_backend(r)->set_history_prefix(con, rmc::parse_tla_value(lit), err)) throw rmc::CfgError(rc, con + ": " + err);
    }
  } catch (const rmc::CfgError& e) {
    c->last_error = e.what();
    int code = e.code;
    *out = c;   // handle kept so mc_last_error can explain; caller must mc_close
    return code;
  } catch (const std::exception& e) {
    c->last_error = e.what();
    *out = c;
    return MC_E_PARSE;
  }
  *out = c;
  return MC_OK;
}

int mc_set_history_prefix(mc_ctx* c, const char* constraint, const char* trace_text) {
  if (!c || !constraint || !trace_text) return MC_E_INVALID;
  if (!c->be) return MC_E_STATE;
  try {
    std::string err;
    for (int r = 0; r < c->n_gpus; ++r) {
      const int rc = c->rank_backend(r)->set_history_prefix(constraint, rmc::parse_tla_value(trace_text), err);
      if (rc) { c->last_error = err; return rc; }
    }
  } catch (const rmc::CfgError& e) {
    c->last_error = e.what();
    return e.code;
  }
  return MC_OK;
}

int mc_set_checkpoint(mc_ctx* c, const char* path, int32_t every_levels) {
  if (!c || every_levels < 0) return MC_E_INVALID;
  if (!c->be) return MC_E_STATE;
  if (path && c->ro.count_final_level) {   // a checkpoint must hold every level it names
    c->last_error = "checkpoints store every level: not with count_final_level";
    return MC_E_UNSUPPORTED;
  }
  c->ro.checkpoint_path = path ? path : "";
  c->ro.checkpoint_every = path ? every_levels : 0;
  return MC_OK;
}

int mc_set_recover(mc_ctx* c, const char* path) {
  if (!c) return MC_E_INVALID;
  if (!c->be) return MC_E_STATE;
  c->ro.recover_path = path ? path : "";
  return MC_OK;
}

int mc_set_fault_injection(mc_ctx* c, int32_t rank, int64_t depth) {
  if (!c) return MC_E_INVALID;
  c->ro.test_fail_rank = rank < 0 ? -1 : rank;
  c->ro.test_fail_depth = rank < 0 ? -1 : depth;
  return MC_OK;
}

int mc_set_fp_slice(mc_ctx* c, int32_t entries) {
  if (!c) return MC_E_INVALID;
  c->ro.test_fp_slice = entries < 0 ? -1 : entries;
  return MC_OK;
}

namespace {
// mc_opts.n_gpus > 1: the sharded BFS (owner-partitioned fingerprints) inside this
// process, one host thread per GPU running the backend's native level loop (raft_original:
// orig_backend.hip shard_run_native; tlc_membership: fifo_shard_loop.h) over an in-process RCCL
// communicator (ncclCommInitAll over the devices), or over the loopback of device copies when every
// rank shares one device (same_device) or RCCL cannot be loaded.  The counterexample is
// reassembled by chasing parent pointers across the ranks' stores (gid bits 37..39 = owner rank).
int run_multi(mc_ctx* c) {
  const int W = c->n_gpus;
  std::string err;
  if (!c->ro.checkpoint_path.empty() || !c->ro.recover_path.empty()) {
    c->last_error = "checkpoint/recover apply to single-GPU runs (n_gpus = 1)";
    return MC_E_UNSUPPORTED;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) { c->last_error = "no HIP device available (raftmc has no CPU fallback)"; return MC_E_NO_DEVICE; }
  std::vector<int> dev(W);
  for (int r = 0; r < W; ++r) dev[r] = c->same_device ? c->ro.device : c->ro.device + r;
  if (dev[W - 1] >= ndev) {
    c->last_error = "n_gpus = " + std::to_string(W) + " from device " + std::to_string(c->ro.device) + " needs " +
                    std::to_string(dev[W - 1] + 1) + " HIP devices, this node has " + std::to_string(ndev);
    return MC_E_NO_DEVICE;
  }
  bool use_rccl = !c->same_device && rmc::rccl().load(err) == 0;
  if (use_rccl && (int)c->local_comms.size() != W) {
    for (ncclComm_t x : c->local_comms) if (x) (void)rmc::rccl().CommDestroy(x);
    std::string e;   // non-blocking communicators where RCCL has them (rccl_api.h rccl_init_all)
    if (rmc::rccl_init_all(c->local_comms, dev, e)) { c->local_comms.clear(); use_rccl = false; }
  }
  if (!use_rccl && !c->same_device) {   // loopback between devices: device copies over xGMI peer access
    for (int a = 0; a < W; ++a)
      for (int b = 0; b < W; ++b)
        if (a != b && hipSetDevice(dev[a]) == hipSuccess) (void)hipDeviceEnablePeerAccess(dev[b], 0);
    (void)hipGetLastError();   // "already enabled" is not an error here
  }
  rmc::LoopbackWorld world(W);
  std::vector<int> rcs(W, MC_OK);
  std::vector<std::string> errs(W);
  // A rank that leaves the loop early (shard_open failed, a rank-local capacity error, a transfer
  // error) must not leave its peers blocked in the next collective: the loopback world releases
  // every rendezvous, and on RCCL the communicators are aborted through RcclAbort (which waits for
  // every rank to be outside its RCCL calls first, so no rank uses a freed communicator; ncclCommAbort
  // stops the peers' pending send/recv/all-reduce kernels; an aborted communicator is never reused).
  rmc::RcclAbort ab(W);
  auto rank_main = [&](int r) {
    rmc::Backend* be = c->rank_backend(r);
    rmc::RunOpts o = c->ro;
    o.device = dev[r];
    std::string e;
    int rc = be->shard_open(o, r, W, e);   // selects the device on this thread
    if (!rc) {
      if (use_rccl) { rmc::RcclTransport t(c->local_comms[r], &ab, r); rc = be->shard_run_native(t, e); }
      else { rmc::LoopbackTransport t(world, r); rc = be->shard_run_native(t, e); }
    }
    if (rc) {
      int expect = -1;
      ab.first.compare_exchange_strong(expect, r);   // the first rank to fail reports the cause
      world.abort();
      if (use_rccl) ab.abort_all(r, c->local_comms);
    }
    rcs[r] = rc; errs[r] = e;
  };
  std::vector<std::thread> th;
  for (int r = 1; r < W; ++r) th.emplace_back(rank_main, r);
  rank_main(0);
  for (auto& x : th) x.join();
  if (ab.done) c->local_comms.clear();   // aborted (and freed by the abort): the next run builds fresh communicators
  // report the rank that failed first in its own right (not a peer released by the abort)
  if (ab.first.load() >= 0) {
    const int r = ab.first.load();
    c->last_error = "rank " + std::to_string(r) + ": " + errs[r];
    return rcs[r];
  }
  c->res = *c->be->shard_result();                 // every rank holds the global counts
  for (int r = 0; r < W && c->res.violated.empty(); ++r) c->res.violated = c->rank_backend(r)->shard_result()->violated;
  // the counterexample: the lowest rank holding the stop's head, then the parent chain by owner
  c->res.trace.clear();
  for (int r = 0; r < W; ++r) {
    uint64_t parent = 0;
    std::string act, text;
    if (c->rank_backend(r)->shard_violation(&parent, act, text)) continue;
    std::vector<std::pair<std::string, std::string>> tr{{act, text}};
    uint64_t gid = parent;
    for (int hop = 0; gid != ~0ull && hop < (1 << 20); ++hop) {
      uint64_t meta = 0;
      std::string t2;
      const int owner = (int)((gid >> 37) & 7);
      if (owner >= W || c->rank_backend(owner)->shard_read_state(gid, t2, &meta, err)) { c->last_error = "trace: " + err; return MC_E_STATE; }
      const size_t a = (size_t)((meta >> 16) & 0xFF);
      tr.push_back({meta == ~0ull ? std::string("<Initial predicate>")
                                  : (a < c->res.action_names.size() ? c->res.action_names[a] : std::string("?")), t2});
      gid = meta == ~0ull ? ~0ull : meta >> 24;
    }
    c->res.trace.assign(tr.rbegin(), tr.rend());
    break;
  }
  c->ran = true;
  c->last_error = c->res.error;
  return MC_OK;
}
}  // namespace

int mc_run(mc_ctx* c) {
  if (!c) return MC_E_INVALID;
  if (!c->be) return MC_E_STATE;
  c->released = false;
  if (c->n_gpus > 1) { c->ran = false; return run_multi(c); }
  std::string err;
  int rc = c->be->run(c->ro, c->res, err);
  c->last_error = err.empty() ? c->res.error : err;
  c->ran = rc == 0;
  return rc;
}

int mc_summary(const mc_ctx* c, mc_summary_t* s) {
  if (!c || !s) return MC_E_INVALID;
  if (!c->ran) return MC_E_STATE;
  std::memset(s, 0, sizeof *s);
  const auto& r = c->res;
  s->generated = r.generated; s->distinct = r.distinct; s->left_on_queue = r.left_on_queue; s->depth = r.depth;
  s->verdict = r.verdict; s->n_actions = (int32_t)r.action_names.size();
  s->collision_prob_optimistic = r.collision_optimistic; s->collision_prob_observed = r.collision_observed;
  s->seconds_total = r.seconds_total; s->seconds_kernels = r.seconds_kernels; s->fp_seed = r.seed;
  s->algo_bytes = r.algo_bytes; s->generated_in_model = r.generated_in_model; s->state_bytes = r.state_bytes;
  s->n_launches = r.n_launches;
  s->seen_set_probes = r.seen_set_probes;
  std::snprintf(s->violated, sizeof s->violated, "%s", r.violated.c_str());
  std::snprintf(s->spec, sizeof s->spec, "%s", c->be->family().c_str());
  return MC_OK;
}

int mc_action_stats(const mc_ctx* c, int32_t k, const char** name, int64_t* gen, int64_t* dist) {
  if (!c) return MC_E_INVALID;
  if (!c->ran) return MC_E_STATE;
  if (k < 0 || k >= (int32_t)c->res.action_names.size()) return MC_E_INVALID;
  if (name) *name = c->res.action_names[k].c_str();
  if (gen) *gen = c->res.act_generated[k];
  if (dist) *dist = c->res.act_distinct[k];
  return MC_OK;
}

int mc_level_stats(const mc_ctx* c, int32_t level, int64_t* states, int64_t* gen, double* ms) {
  if (!c) return MC_E_INVALID;
  if (!c->ran) return MC_E_STATE;
  if (level < 0 || level >= (int32_t)c->res.levels.size()) return MC_E_INVALID;
  const auto& l = c->res.levels[level];
  if (states) *states = l.states;
  if (gen) *gen = l.generated;
  if (ms) *ms = l.kernel_ms;
  return MC_OK;
}

int mc_kernel_stats(const mc_ctx* c, int32_t k, const char** name, double* ms, double* algo_bytes, int64_t* launches) {
  if (!c) return MC_E_INVALID;
  if (!c->ran) return MC_E_STATE;
  if (k < 0 || k >= (int32_t)c->res.kernels.size()) return MC_E_INVALID;
  const auto& ks = c->res.kernels[k];
  if (name) *name = ks.name.c_str();
  if (ms) *ms = ks.ms;
  if (algo_bytes) *algo_bytes = ks.algo_bytes;
  if (launches) *launches = ks.launches;
  return MC_OK;
}

int mc_trace(const mc_ctx* c, char** text, size_t* len) {
  if (!c || !text) return MC_E_INVALID;
  if (!c->ran) return MC_E_STATE;
  *text = dup_text(trace_text(c, c->res), len);
  return *text ? MC_OK : MC_E_OOM;
}

int mc_report(const mc_ctx* c, char** text, size_t* len) {
  if (!c || !text) return MC_E_INVALID;
  if (!c->ran) return MC_E_STATE;
  const auto& r = c->res;
  std::ostringstream o;
  o << "raftmc (MI355X/gfx950) checking " << c->tla_path << " with " << c->cfg_path << "\n";
  if (r.verdict == MC_VERDICT_INVARIANT_VIOLATION) {
    o << "Error: Invariant " << r.violated << " is violated.\n";
    o << "Error: The behavior up to this point is:\n" << trace_text(c, r);
  } else if (r.verdict == MC_VERDICT_DEADLOCK) {
    o << "Error: Deadlock reached.\nError: The behavior up to this point is:\n" << trace_text(c, r);
  } else if (r.verdict == MC_VERDICT_EVAL_ERROR) {
    // TLC: the evaluation error, then the behavior up to the state it was evaluating
    o << "Error: " << r.error << "\n";
    if (!r.trace.empty()) o << "Error: The behavior up to this point is:\n" << trace_text(c, r);
  } else if (r.verdict == MC_VERDICT_CAPACITY_OVERFLOW) {
    o << "Error: " << r.error << "\n";
  } else if (r.verdict == MC_VERDICT_OK) {
    o << "Model checking completed. No error has been found.\n";
    o << "  Estimates of the probability that TLC did not check all reachable states\n";
    o << "  because two distinct states had the same fingerprint:\n";
    char buf[160];
    std::snprintf(buf, sizeof buf, "  calculated (optimistic):  val = %.1E\n", r.collision_optimistic);
    o << buf;
    if (r.collision_observed >= 0) {
      std::snprintf(buf, sizeof buf, "  based on the actual fingerprints:  val = %.1E\n", r.collision_observed);
      o << buf;
    }
  }
  o << r.generated << " states generated, " << r.distinct << " distinct states found, " << r.left_on_queue << " states left on queue.\n";
  o << "The depth of the complete state graph search is " << r.depth << ".\n";
  o << "Finished in " << (long long)(r.seconds_total * 1000.0 + 0.5) << "ms\n";
  o << "Verdict: " << verdict_name(r.verdict) << "\n";
  *text = dup_text(o.str(), len);
  return *text ? MC_OK : MC_E_OOM;
}

int mc_action_location(const mc_ctx* c, const char* action, char** text, size_t* len) {
  if (!c || !action || !text) return MC_E_INVALID;
  const std::string& loc = c->location_of(action);
  if (loc.empty()) {
    const_cast<mc_ctx*>(c)->last_error = std::string("no definition of action ") + action + " in " + c->tla_path + " or the modules it EXTENDS";
    return MC_E_INVALID;
  }
  *text = dup_text(loc, len);
  return *text ? MC_OK : MC_E_OOM;
}

int mc_release_device_memory(mc_ctx* c) {
  if (!c) return MC_E_INVALID;
  if (!c->be) return MC_E_STATE;
  c->be->release_device();
  for (auto& p : c->peers) if (p) p->release_device();
  c->released = true;   // the last run's stored states are gone: mc_dump_states / mc_collision_observed refuse
  return MC_OK;
}

int mc_collision_observed(mc_ctx* c, double* val) {
  if (!c || !val) return MC_E_INVALID;
  if (!c->ran || c->released) return MC_E_STATE;
  std::string err;
  double v = -1;
  const int rc = c->be->observed_collision(v, err);
  if (rc) { c->last_error = err; return rc; }
  c->res.collision_observed = v;
  *val = v;
  return MC_OK;
}

int mc_dump_states(const mc_ctx* c, const char* path) {
  if (!c || !path) return MC_E_INVALID;
  if (!c->ran || c->released) return MC_E_STATE;
  std::string err;
  if (c->n_gpus > 1) {
    // every rank's partition of the state space: one file per rank, path.rank<r> (as shard.py writes)
    for (int r = 0; r < c->n_gpus; ++r) {
      const int rc = const_cast<mc_ctx*>(c)->rank_backend(r)->dump_states(std::string(path) + ".rank" + std::to_string(r), err);
      if (rc) { const_cast<mc_ctx*>(c)->last_error = "rank " + std::to_string(r) + ": " + err; return rc; }
    }
    return MC_OK;
  }
  int rc = c->be->dump_states(path, err);
  if (rc) const_cast<mc_ctx*>(c)->last_error = err;
  return rc;
}

int mc_describe(const mc_ctx* c, char** text, size_t* len) {
  if (!c || !text) return MC_E_INVALID;
  if (!c->be) return MC_E_STATE;
  // the model's own description plus the run options that decide TLC semantics
  std::string d = c->be->describe_json();
  if (!d.empty() && d.back() == '}') {
    d.pop_back();
    d += std::string(", \"symmetry_mode\": \"") + (c->ro.sym_tlc ? "tlc" : "orbit") + "\", \"workers\": " +
         std::to_string(c->ro.workers) + ", \"check_deadlock\": " + (c->ro.check_deadlock ? "true" : "false") +
         ", \"n_gpus\": " + std::to_string(c->n_gpus) + "}";
  }
  *text = dup_text(d, len);
  return *text ? MC_OK : MC_E_OOM;
}

int mc_exit_code(const mc_ctx* c) {
  if (!c || !c->ran) return 75;
  switch (c->res.verdict) {
    case MC_VERDICT_OK: case MC_VERDICT_DEPTH_LIMIT: return 0;
    case MC_VERDICT_INVARIANT_VIOLATION: return 12;
    case MC_VERDICT_DEADLOCK: return 11;
    default: return 75;
  }
}

// ------------------------------------------------------------------ sharded BFS
// checkpoint / recover apply to single-GPU runs only: a sharded run refuses them rather than
// silently writing no checkpoint or starting from Init
#define SHARD_GUARD() \
  if (!c) return MC_E_INVALID; \
  if (!c->be) return MC_E_STATE; \
  if (!c->ro.checkpoint_path.empty() || !c->ro.recover_path.empty()) { \
    c->last_error = "checkpoint/recover apply to single-GPU runs (mc_run); a sharded run cannot use them"; \
    return MC_E_UNSUPPORTED; \
  }
#define SHARD_RC(expr)                      \
  do {                                      \
    std::string err;                        \
    int rc_ = (expr);                       \
    if (rc_) c->last_error = err;           \
    return rc_;                             \
  } while (0)

int mc_shard_open(mc_ctx* c, int32_t rank, int32_t world) {
  SHARD_GUARD();
  c->ran = false;
  SHARD_RC(c->be->shard_open(c->ro, rank, world, err));
}
int mc_shard_record_bytes(const mc_ctx* c, int32_t what) {
  if (!c || !c->be) return MC_E_INVALID;
  return c->be->shard_record_bytes(what);
}
int mc_shard_frontier(const mc_ctx* c, int64_t* states, int64_t* chunk) {
  if (!c || !c->be) return MC_E_INVALID;
  return c->be->shard_frontier(states, chunk);
}
int mc_shard_generate(mc_ctx* c, int64_t begin, int64_t count, int64_t* counts) {
  SHARD_GUARD();
  SHARD_RC(c->be->shard_generate(begin, count, counts, err));
}
int mc_shard_fill(mc_ctx* c, int32_t what, void* dst, const int64_t* offsets) {
  SHARD_GUARD();
  SHARD_RC(c->be->shard_fill(what, dst, offsets, err));
}
int mc_shard_dedup(mc_ctx* c, const void* recv, const int64_t* counts, int64_t* reply_counts) {
  SHARD_GUARD();
  SHARD_RC(c->be->shard_dedup(recv, counts, reply_counts, err));
}
int mc_shard_materialize(mc_ctx* c, const void* acks, const int64_t* counts) {
  SHARD_GUARD();
  SHARD_RC(c->be->shard_materialize(acks, counts, err));
}
int mc_shard_store(mc_ctx* c, const void* states, int64_t n) {
  SHARD_GUARD();
  SHARD_RC(c->be->shard_store(states, n, err));
}
int mc_shard_layout(mc_ctx* c, const int64_t* frontier_counts) {
  SHARD_GUARD();
  if (!frontier_counts) return MC_E_INVALID;
  SHARD_RC(c->be->shard_layout(frontier_counts, err));
}
int mc_shard_select(mc_ctx* c, int64_t* reply_counts) {
  SHARD_GUARD();
  if (!reply_counts) return MC_E_INVALID;
  SHARD_RC(c->be->shard_select(reply_counts, err));
}
int mc_shard_event_stats(mc_ctx* c, const int64_t* global_stats, int64_t* stats) {
  SHARD_GUARD();
  if (!global_stats || !stats) return MC_E_INVALID;
  SHARD_RC(c->be->shard_event_stats(global_stats, stats, err));
}
int mc_shard_level_stats(mc_ctx* c, int64_t* stats) {
  SHARD_GUARD();
  SHARD_RC(c->be->shard_level_stats(stats, err));
}
int mc_shard_level_commit(mc_ctx* c, const int64_t* global, int32_t* done) {
  SHARD_GUARD();
  std::string err;
  int d = 0;
  int rc = c->be->shard_level_commit(global, &d, err);
  if (rc) { c->last_error = err; return rc; }
  *done = d;
  if (d) { c->res = *c->be->shard_result(); c->ran = true; c->last_error = c->res.error; }
  return MC_OK;
}
int mc_shard_read_state(const mc_ctx* c, uint64_t gid, char** text, size_t* len, uint64_t* meta) {
  if (!c || !c->be || !text) return MC_E_INVALID;
  std::string t, err;
  int rc = c->be->shard_read_state(gid, t, meta, err);
  if (rc) { const_cast<mc_ctx*>(c)->last_error = err; return rc; }
  *text = dup_text(t, len);
  return *text ? MC_OK : MC_E_OOM;
}
int mc_shard_violation(const mc_ctx* c, uint64_t* parent, char** action, char** text) {
  if (!c || !c->be || !action || !text) return MC_E_INVALID;
  std::string a, t;
  int rc = c->be->shard_violation(parent, a, t);
  if (rc) return rc;
  *action = dup_text(a, nullptr);
  *text = dup_text(t, nullptr);
  return MC_OK;
}

int mc_rccl_unique_id(mc_ctx* c, void* out, size_t len) {
  if (!c || !out || len < sizeof(ncclUniqueId)) return MC_E_INVALID;
  std::string err;
  if (rmc::rccl().load(err)) { c->last_error = err; return MC_E_UNSUPPORTED; }
  ncclUniqueId id;
  ncclResult_t r = rmc::rccl().GetUniqueId(&id);
  if (r != ncclSuccess) { c->last_error = std::string("ncclGetUniqueId: ") + rmc::rccl().GetErrorString(r); return MC_E_NO_DEVICE; }
  std::memcpy(out, &id, sizeof id);
  return MC_OK;
}
int mc_shard_run_rccl(mc_ctx* c, int32_t rank, int32_t world, const void* unique_id, size_t len) {
  SHARD_GUARD();
  if (!unique_id || len < sizeof(ncclUniqueId)) return MC_E_INVALID;
  std::string err;
  if (rmc::rccl().load(err)) { c->last_error = err; return MC_E_UNSUPPORTED; }
  c->ran = false;
  // shard_open selects the device and allocates; the communicator binds to that device
  int rc = c->be->shard_open(c->ro, rank, world, err);
  if (rc) { c->last_error = err; return rc; }
  if (!c->comm || c->comm_rank != rank || c->comm_world != world || std::memcmp(c->comm_id, unique_id, sizeof(ncclUniqueId))) {
    if (c->comm) { (void)rmc::rccl().CommDestroy(c->comm); c->comm = nullptr; }
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof id);
    if (rmc::rccl_init_rank(&c->comm, world, id, rank, err)) { c->comm = nullptr; c->last_error = err; return MC_E_NO_DEVICE; }
    c->comm_rank = rank; c->comm_world = world;
    std::memcpy(c->comm_id, unique_id, sizeof(ncclUniqueId));
  }
  rmc::RcclTransport t(c->comm);
  rc = c->be->shard_run_native(t, err);
  if (rc) {
    // the loop left early (a peer's failure seen through the communicator's asynchronous error, or a
    // local one): abort the communicator, which stops this rank's pending transfers; the next run
    // builds a fresh one
    (void)rmc::rccl().CommAbort(c->comm);
    c->comm = nullptr;
    c->last_error = err;
    return rc;
  }
  c->res = *c->be->shard_result();
  c->ran = true;
  c->last_error = c->res.error;
  return MC_OK;
}

int mc_shard_run_loopback(mc_ctx* const* ctxs, int32_t world) {
  if (!ctxs || world < 1 || world > 8) return MC_E_INVALID;
  for (int r = 0; r < world; ++r) {
    if (!ctxs[r] || !ctxs[r]->be) return MC_E_INVALID;
    for (int q = 0; q < r; ++q) if (ctxs[q] == ctxs[r]) return MC_E_INVALID;
    if (!ctxs[r]->ro.checkpoint_path.empty() || !ctxs[r]->ro.recover_path.empty()) {
      ctxs[r]->last_error = "checkpoint/recover apply to single-GPU runs (mc_run); a sharded run cannot use them";
      return MC_E_UNSUPPORTED;
    }
  }
  rmc::LoopbackWorld w(world);
  std::vector<int> rcs(world, MC_OK);
  auto rank_main = [&](int r) {
    mc_ctx* c = ctxs[r];
    std::string err;
    c->ran = false;
    int rc = c->be->shard_open(c->ro, r, world, err);   // selects the device on this thread
    if (!rc) {
      rmc::LoopbackTransport t(w, r);
      rc = c->be->shard_run_native(t, err);
    }
    if (rc) { c->last_error = err; w.abort(); }
    else { c->res = *c->be->shard_result(); c->ran = true; c->last_error = c->res.error; }
    rcs[r] = rc;
  };
  std::vector<std::thread> th;
  for (int r = 1; r < world; ++r) th.emplace_back(rank_main, r);
  rank_main(0);
  for (auto& x : th) x.join();
  for (int r = 0; r < world; ++r) if (rcs[r]) return rcs[r];
  return MC_OK;
}

#ifndef RAFTMC_SOURCE_HASH
#define RAFTMC_SOURCE_HASH "unknown"
#endif
const char* mc_source_hash(void) { return RAFTMC_SOURCE_HASH; }

void mc_free(void* p) { std::free(p); }
void mc_close(mc_ctx* c) { delete c; }
const char* mc_last_error(const mc_ctx* c) { return c ? c->last_error.c_str() : "null handle"; }

}  // extern "C"
