// raftmc host: the interface between the C ABI (mc_api.cpp) and a compiled
// spec backend (one per spec family; each owns its GPU buffers and kernels).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "model.h"
#include "tla_value.h"

namespace rmc {

struct ShardTransport;   // shard_transport.h

struct RunOpts {
  int device = 0;
  uint64_t fp_table_bytes = 0, state_store_bytes = 0;
  int64_t max_depth = 0;
  uint64_t seed = 0;
  bool inv_out_of_model = true;
  bool sym_tlc = false;   // MC_COMPAT_SYM_TLC
  bool disjunct_copies = true;   // MC_COMPAT_DISJUNCT_COPIES
  // mc_set_fault_injection (tests only): rank test_fail_rank leaves the sharded loop at that depth
  int test_fail_rank = -1;
  int test_fp_slice = -1;        // mc_set_fp_slice (tests only): tlc_membership's LDS bag slice cap
  int64_t test_fail_depth = -1;
  bool check_deadlock = false;
  int block_size = 256;
  // TLC -workers: 1 = TLC's single-worker FIFO order (order-dependent outputs — which parent of a
  // state is kept, per-action distinct counts, which shortest counterexample — are TLC's exactly);
  // otherwise TLC -workers N semantics (every order-independent output exact; a counterexample
  // still is TLC's single-worker one: the search re-runs in FIFO order to the event's level)
  int workers = 1;
  // TLC -checkpoint / -recover analogues (raft_original): write the BFS state every
  // checkpoint_every levels to checkpoint_path; resume the next run from recover_path
  std::string checkpoint_path, recover_path;
  int checkpoint_every = 0;
  // mc_opts.count_final_level: the last level of a depth-bounded -workers N search is counted and
  // checked, not stored (raft_original; ignored elsewhere)
  bool count_final_level = false;
};

struct LevelStat { int64_t states = 0, generated = 0; double kernel_ms = 0; };
struct KernelStat { std::string name; double ms = 0, algo_bytes = 0; int64_t launches = 0; };

struct RunResult {
  int64_t generated = 0, distinct = 0, left_on_queue = 0, depth = 0;
  int verdict = 0;                       // MC_VERDICT_*
  std::string violated, error;
  std::vector<std::string> action_names;
  std::vector<int64_t> act_generated, act_distinct;
  std::vector<LevelStat> levels;
  std::vector<std::pair<std::string, std::string>> trace;   // (action label, multi-line state text)
  double seconds_total = 0, seconds_kernels = 0;
  double collision_optimistic = 0, collision_observed = -1;
  uint64_t seed = 0;
  // algorithmic byte accounting of the expand kernel
  double algo_bytes = 0;                 // F*S + G_in*8 + D*(8+8+S) summed over levels
  int64_t generated_in_model = 0;
  int64_t seen_set_probes = 0;           // fingerprints that probed the seen-set (after workgroup-local dedup)
  int state_bytes = 0;
  int n_launches = 0;
  std::vector<KernelStat> kernels;       // per-kernel HIP-event time and algorithmic bytes
};

struct Backend {
  virtual ~Backend() {}
  virtual std::string family() const = 0;
  virtual std::string describe_json() const = 0;
  virtual int run(const RunOpts& o, RunResult& r, std::string& err) = 0;
  virtual int dump_states(const std::string& path, std::string& err) = 0;
  // mc_release_device_memory: free the device buffers kept between runs (the next run allocates again)
  virtual void release_device() = 0;
  // TLC's "based on the actual fingerprints" estimate: 1 / min gap of the seen-set (fp_gap.h)
  virtual int observed_collision(double& v, std::string& err) { (void)v; err = "not available"; return -4; }
  // punctuated-search prefix constraints whose golden history trace is data (tla_value.h)
  virtual std::vector<std::string> history_prefixes_needed() const { return {}; }
  virtual int set_history_prefix(const std::string& con, const TVal& trace, std::string& err) {
    (void)trace; err = "'" + con + "' is not a constraint of this spec"; return -1;
  }
  // ---- sharded BFS (include/raftmc.h mc_shard_*); rank-local device work only
  virtual int shard_open(const RunOpts& o, int rank, int world, std::string& err) = 0;
  virtual int shard_record_bytes(int what) const = 0;
  virtual int shard_frontier(int64_t* states, int64_t* chunk) const = 0;
  virtual int shard_generate(int64_t begin, int64_t count, int64_t* counts, std::string& err) = 0;
  virtual int shard_fill(int what, void* dst, const int64_t* offsets, std::string& err) = 0;
  virtual int shard_dedup(const void* recv, const int64_t* counts, int64_t* reply_counts, std::string& err) = 0;
  virtual int shard_materialize(const void* acks, const int64_t* counts, std::string& err) = 0;
  virtual int shard_store(const void* states, int64_t n, std::string& err) = 0;
  virtual int shard_level_stats(int64_t* stats, std::string& err) = 0;
  virtual int shard_level_commit(const int64_t* global, int* done, std::string& err) = 0;
  virtual int shard_read_state(uint64_t gid, std::string& text, uint64_t* meta, std::string& err) const = 0;
  virtual int shard_violation(uint64_t* parent, std::string& action, std::string& text) const = 0;
  virtual const RunResult* shard_result() const = 0;
  // FIFO first-found specs (VIEW): level layout, per-level winner selection, stop-point counters
  // the whole sharded level loop natively over an RCCL communicator (after shard_open)
  virtual int shard_run_native(ShardTransport& t, std::string& err) { (void)t; err = "no native sharded loop for this spec"; return -4; }
  virtual int shard_layout(const int64_t* counts, std::string& err) { (void)counts; err = "not a FIFO-ranked spec"; return -4; }
  virtual int shard_select(int64_t* reply_counts, std::string& err) { (void)reply_counts; err = "not a FIFO-ranked spec"; return -4; }
  virtual int shard_event_stats(const int64_t* g, int64_t* st, std::string& err) { (void)g; (void)st; err = "not a FIFO-ranked spec"; return -4; }
};

Backend* make_orig_backend(const CfgFile& cfg);   // throws CfgError
Backend* make_memb_backend(const CfgFile& cfg);   // throws CfgError
// the generated path (csrc/tlagen): any module in the front end's subset, or a .gen.hip source
Backend* make_tlagen_backend(const std::string& tla_path, const CfgFile& cfg);   // throws CfgError

}  // namespace rmc
