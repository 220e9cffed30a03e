/*
 * raftmc — C ABI of the MI355X-native explicit-state model checker for the
 * dranov/raft-tla specs.  This is the drop-in boundary for the hot path.
 *
 * The reference has no FFI: the path sits behind TLC's command-line contract
 * (SURVEY.md §8b), i.e.
 *     java -cp tla2tools.jar tlc2.TLC [-workers N] [-config F.cfg] [-deadlock] F.tla
 * driven by tlc_membership/raft.cfg:1-87 (README.md:5 "passed to TLC").
 * Each entry point below replaces one part of that contract:
 *   mc_open      <- TLC argument parsing + SANY/cfg loading
 *                   (the .tla given as F.tla, the .cfg given by -config; the
 *                   cfg keywords of tlc_membership/raft.cfg:1-87)
 *   mc_run       <- tlc2.TLC model checking (ModelChecker BFS: Init, Next,
 *                   CONSTRAINTS raft.cfg:37-55, INVARIANTS raft.cfg:60-87,
 *                   SYMMETRY raft.cfg:29, VIEW raft.cfg:30)
 *   mc_summary   <- TLC's final lines "N states generated, M distinct states
 *                   found, K states left on queue", "The depth of the complete
 *                   state graph search is D", the fingerprint collision
 *                   probability lines, and the process exit code
 *   mc_trace     <- TLC's "Error: Invariant X is violated." + "State k:" blocks
 *   mc_report    <- the whole TLC-style stdout text
 *
 * Conventions: every function returns 0 or a negative MC_E_* code and never
 * throws.  The library owns all buffers; text returned through an out
 * parameter is freed by the caller with mc_free().  A handle is used by one
 * host thread at a time; distinct handles are independent.  All GPU work runs
 * on the HIP device selected in mc_opts; there is no CPU fallback: on a host
 * without a usable gfx950 device mc_run fails with MC_E_NO_DEVICE.
 */
#ifndef RAFTMC_H
#define RAFTMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: mc_summary_t gained a reserved tail (a caller built against version 1 passes a smaller struct,
 *    so mc_open refuses version-1 opts rather than let mc_summary write past it).
 * 3: the version in mc_opts is the CALLER's: mc_default_opts is an inline wrapper in this header that
 *    passes RAFTMC_ABI_VERSION as the caller was compiled with it to mc_opts_init (version 2's
 *    library-side mc_default_opts stamped the library's own version, so a version-1 caller passed
 *    mc_open's check).  Layouts are unchanged from version 2. */
#define RAFTMC_ABI_VERSION 3

/* error codes */
#define MC_OK 0
#define MC_E_INVALID (-1)      /* bad argument / unusable handle                   */
#define MC_E_IO (-2)           /* cannot read the .tla / .cfg                      */
#define MC_E_PARSE (-3)        /* cfg syntax error                                 */
#define MC_E_UNSUPPORTED (-4)  /* spec / cfg feature or shape not compiled in       */
#define MC_E_NO_DEVICE (-5)    /* no HIP device / HIP runtime failure              */
#define MC_E_OOM (-6)          /* device allocation failed                         */
#define MC_E_STATE (-7)        /* call out of order (e.g. mc_trace before mc_run)  */

/* verdicts (mc_summary_t.verdict) and the TLC-like exit codes mc_exit_code() maps them to */
#define MC_VERDICT_OK 0
#define MC_VERDICT_INVARIANT_VIOLATION 1
#define MC_VERDICT_EVAL_ERROR 2
#define MC_VERDICT_CAPACITY_OVERFLOW 3
#define MC_VERDICT_DEADLOCK 4
#define MC_VERDICT_DEPTH_LIMIT 5

/* tlc_compat_flags: the [ext] TLC-semantics switches */
#define MC_COMPAT_INV_OUT_OF_MODEL 0x1u /* check invariants on !seen successors that fail a constraint (TLC default) */
/* SYMMETRY as TLC applies it (TLCStateMut.fingerPrint): the permutation giving the least full
 * variable tuple (history included) under TLC's value order, then the VIEW of that state.  Set by
 * mc_default_opts (the drop-in default: TLC's counts for a cfg with SYMMETRY, tlc_membership/raft.cfg:29-30);
 * cleared, SYMMETRY + VIEW identify states whose VIEWs lie in one orbit (the opt-in "orbit" mode,
 * CLI -symmetry orbit: faster, fewer distinct states when histories differ).  tlc_membership only. */
#define MC_COMPAT_SYM_TLC 0x2u
/* TLC's getNextStates enumerates every true disjunct of a disjunctive guard inside an action as a branch
 * of its own, so the one successor such a guard admits is GENERATED once per true disjunct
 * (tlc_membership/raft.tla:796 HandleCheckOldConfig, :783-789 HandleCatchupResponse's discard).  Set by
 * mc_default_opts (TLC's counters); cleared, that successor counts once.  Only generated counters (and
 * TLC's counters at a stop point) see it: the state is the same.  raft_original has no overlapping
 * disjuncts (no effect); the generated path follows the text and refuses the flag cleared. */
#define MC_COMPAT_DISJUNCT_COPIES 0x4u

typedef struct mc_ctx mc_ctx;

typedef struct mc_opts {
  int32_t abi_version;        /* RAFTMC_ABI_VERSION                                       */
  int32_t device;             /* HIP device ordinal (one process per GPU)                  */
  int32_t n_gpus;             /* GPUs of this node that mc_run uses (1..8).  > 1: the fingerprints are
                                 owner-partitioned over devices device .. device + n_gpus - 1, one host
                                 thread per GPU inside the library, exchanging over an in-process RCCL
                                 communicator (xGMI); the result (counts, verdict, counterexample) is the
                                 single-GPU one.  One process per GPU instead: mc_shard_run_rccl.      */
  int32_t workers;            /* TLC -workers N: 1 (TLC's default) = TLC's single-worker FIFO order,
                                 so every order-dependent output (kept parent of a state, per-action
                                 distinct counts, counterexample) is TLC's; otherwise TLC -workers N
                                 semantics: order-independent outputs (generated / distinct / depth /
                                 per-action generated) identical, counterexamples still TLC's
                                 single-worker ones (raft_original re-runs FIFO to the event's level) */
  uint64_t fp_table_bytes;    /* seen-set bytes (power of two used; 0 = auto)             */
  uint64_t state_store_bytes; /* bytes for the per-state store (packed states + parents); 0 = auto */
  int64_t max_depth;          /* 0 = unbounded (TLC -dfid/-depth analogue for BFS)        */
  uint64_t seed;              /* fingerprint seed (0 = default)                           */
  uint32_t tlc_compat_flags;  /* MC_COMPAT_* (default INV_OUT_OF_MODEL | SYM_TLC | DISJUNCT_COPIES) */
  int32_t check_deadlock;     /* 1 = report states without successors (TLC default; -deadlock disables) */
  int32_t block_size;         /* expand kernel workgroup size (0 = 256)                   */
  int32_t same_device;        /* n_gpus > 1 only: 1 = every rank on `device` (the ranks exchange through
                                 an in-process loopback of device copies): the multi-GPU level loop on
                                 a one-GPU machine (tests); 0 = one device per rank (default)        */
  int32_t frontend;           /* MC_FRONTEND_*: which compiled form of the module mc_open uses          */
  int32_t count_final_level;  /* with max_depth, raft_original, workers != 1 (single GPU, n_gpus > 1 or
                                 mc_shard_run_rccl): the states of the last level (depth == max_depth,
                                 never expanded) are fingerprinted, counted and invariant-checked but not
                                 written to the state store (sharded: not shipped to their owners either),
                                 so a depth-bounded search holds one more level than the store.  Counts,
                                 levels and verdicts are unchanged; mc_dump_states refuses (MC_E_STATE).
                                 An event on one GPU still re-runs in TLC's FIFO order, which stores every
                                 level: when that does not fit, the verdict is CAPACITY_OVERFLOW and the
                                 error names the event found.  mc_open refuses it (MC_E_UNSUPPORTED) for
                                 any other spec family, workers = 1 or max_depth = 0, and
                                 mc_set_checkpoint refuses a checkpoint path.  0 = off */
  int32_t reserved[4];
} mc_opts;

/* mc_opts.frontend.  AUTO: the hand-compiled kernels for thirdparty/raft_original.tla and
 * tlc_membership/raft.tla (and their configs/ wrappers), the generated path for any other module.
 * GENERATED: the SANY-subset front end for any module (csrc/tlagen: parse, generate C++ over
 * tlv.h, hiprtc to a gfx950 code object cached by source hash; a path ending in .gen.hip is taken
 * as an already generated source); single GPU; SYMMETRY (TLC's rule), VIEW, ACTION_CONSTRAINTS and
 * TLC's single-worker FIFO order (workers = 1) as on the hand path.  HAND: the hand-compiled
 * families only (MC_E_UNSUPPORTED otherwise). */
#define MC_FRONTEND_AUTO 0
#define MC_FRONTEND_GENERATED 1
#define MC_FRONTEND_HAND 2

typedef struct mc_summary_t {
  int64_t generated;          /* "states generated" (initial states included)             */
  int64_t distinct;           /* "distinct states found"                                  */
  int64_t left_on_queue;      /* "states left on queue"                                   */
  int64_t depth;              /* "depth of the complete state graph search" (Init = 1)    */
  int32_t verdict;            /* MC_VERDICT_*                                              */
  int32_t n_actions;          /* per-action statistics available via mc_action_stats      */
  double collision_prob_optimistic;   /* TLC's "calculated (optimistic)" estimate          */
  double collision_prob_observed;     /* from the minimum gap between fingerprints (or -1) */
  double seconds_total;       /* mc_run wall time                                         */
  double seconds_kernels;     /* sum of expand-kernel times (HIP events)                   */
  uint64_t fp_seed;
  double algo_bytes;           /* expand-kernel algorithmic bytes, SURVEY.md §8d: F*S + G_in*8 + D*(16+S) */
  int64_t generated_in_model;  /* successors that passed every state constraint (G_in)  */
  int32_t state_bytes;         /* S: stored bytes per packed state                      */
  int32_t n_launches;          /* expand-kernel launches (BFS levels expanded)          */
  char violated[64];          /* property name for INVARIANT_VIOLATION                     */
  char spec[32];              /* "raft_original" | "tlc_membership"                        */
  int64_t seen_set_probes;    /* fingerprints that probed the seen-set (device counter; the
                                 successors a workgroup's parents produce twice probe once)   */
  int64_t reserved[8];        /* zero; later fields come out of this tail (the size stays)  */
} mc_summary_t;

/* Fill opts with defaults and stamp caller_abi_version (the RAFTMC_ABI_VERSION the caller was built
 * against) into o->abi_version; mc_open refuses versions whose struct layouts this library does not
 * have.  MC_E_INVALID (opts still filled) for such a version, MC_OK otherwise. */
int mc_opts_init(mc_opts* o, int32_t caller_abi_version);
/* Fill opts with defaults (this header's ABI version).  The library also exports a function of this
 * name for binaries built before version 3: it leaves abi_version 0 ("unstated"), which mc_open
 * refuses, since those callers cannot say which layout they were built with. */
#ifndef RAFTMC_BUILDING_LIBRARY
static inline void mc_default_opts(mc_opts* o) { (void)mc_opts_init(o, RAFTMC_ABI_VERSION); }
#endif

/* Load a spec module (.tla) and a TLC model config (.cfg); no GPU work yet. */
int mc_open(const char* tla_path, const char* cfg_path, const mc_opts* o, mc_ctx** out);

/* Golden history trace of a punctuated-search constraint (CommitWhenConcurrentLeaders_unique,
 * MajorityOfClusterRestarts_constraint; tlc_membership/raft.tla:1198-1204, :1228-1234), as
 * TLA+ value text: the `[global |-> << ... >>]` record the operator's definition embeds
 * (raft.tla:1201, :1231) or the sequence alone.  mc_open already takes it from the module (or
 * the module it EXTENDS, next to it) when the definition is there; this call supplies or
 * replaces it.  MC_E_PARSE for malformed text, MC_E_INVALID for another constraint name. */
int mc_set_history_prefix(mc_ctx* ctx, const char* constraint, const char* trace_text);

/* Breadth-first model checking on the GPU until completion, violation or error. */
int mc_run(mc_ctx* ctx);

/* Summary of the last mc_run. */
int mc_summary(const mc_ctx* ctx, mc_summary_t* out);

/* Per-action statistics: name and (generated, distinct) counts, 0 <= k < n_actions. */
int mc_action_stats(const mc_ctx* ctx, int32_t k, const char** name, int64_t* generated, int64_t* distinct);

/* Per-BFS-level statistics of the last run, 0 <= level < depth. */
int mc_level_stats(const mc_ctx* ctx, int32_t level, int64_t* states, int64_t* generated, double* kernel_ms);

/* Per-kernel statistics of the last run (HIP-event time summed over launches, algorithmic
 * bytes per SURVEY.md §8d), 0 <= k < number of kernels; MC_E_INVALID past the last one. */
int mc_kernel_stats(const mc_ctx* ctx, int32_t k, const char** name, double* ms, double* algo_bytes, int64_t* launches);

/* Counterexample (TLC "State k:" blocks) as text; caller frees with mc_free.  Each header is
 * "State k: <Action line L1, col C1 to line L2, col C2 of module M>" when the action's
 * definition is found in the spec module or a module it EXTENDS (else "<Action>"). */
int mc_trace(const mc_ctx* ctx, char** text, size_t* len);

/* TLC's trace-header location of an action (the span of the body of `Action(params) == body`
 * in the spec module, or in a module it EXTENDS found next to it — the part of TLC's
 * "State k: <...>" line after the name, e.g. "line 177, col 15 to line 186, col 58 of module raft").
 * Needs no run.  MC_E_INVALID when no definition is found; caller frees with mc_free. */
int mc_action_location(const mc_ctx* ctx, const char* action, char** text, size_t* len);

/* TLC's second collision estimate, "based on the actual fingerprints": 1 / (minimum distance
 * between two fingerprints of the seen-set) after a single-GPU mc_run (a sort of the seen-set on
 * the device, outside mc_run's time).  Also fills mc_summary_t.collision_prob_observed and the
 * report's estimate line. */
int mc_collision_observed(mc_ctx* ctx, double* val);

/* Checkpoint / recover (both spec families) — TLC's `-checkpoint <minutes>` and `-recover <dir>`
 * (the states/ directory, reference .gitignore:3).  mc_set_checkpoint: every `every_levels`
 * completed BFS levels mc_run writes the search state (stored states, parent pointers, level
 * position, TLC's counters, the model's identity) to `path` (atomically: path.tmp, rename);
 * NULL or 0 disables.  mc_set_recover: the next mc_run resumes from `path` instead of Init
 * (the seen-set is rebuilt on the GPU from the stored states); generated/distinct/depth/per-action
 * counts continue exactly; kernel timings cover the resumed part.  A checkpoint of another
 * model (or of the other SYMMETRY mode, or — raft_original — a -workers N checkpoint for a -workers 1
 * search) is refused (MC_E_INVALID).  Completed levels that do not fit the device store are kept in
 * host memory on save and on recovery (host spill).  Single-GPU runs only: the mc_shard_* calls
 * return MC_E_UNSUPPORTED on a handle with a checkpoint or recover path set. */
int mc_set_checkpoint(mc_ctx* ctx, const char* path, int32_t every_levels);
int mc_set_recover(mc_ctx* ctx, const char* path);

/* Free the device memory the handle keeps between runs (state store, seen-set, work buffers; the
 * generated path keeps its whole working set, up to state_store_bytes, so that a second run of the
 * same model does not pay ~2.5 s of hipMalloc for a 200 GiB store).  The summary, the trace and the
 * report of the last run stay readable; mc_dump_states and mc_collision_observed, which read the
 * device store, return MC_E_STATE until the next mc_run, which allocates again. */
int mc_release_device_memory(mc_ctx* ctx);

/* Full TLC-style report (summary + trace) as text; caller frees with mc_free. */
int mc_report(const mc_ctx* ctx, char** text, size_t* len);

/* Write every distinct state, one canonical TLA+ line each, to path (parity tests). */
int mc_dump_states(const mc_ctx* ctx, const char* path);

/* Resolved model (spec family, constants, shape, compiled predicates) as JSON text; no GPU needed. */
int mc_describe(const mc_ctx* ctx, char** text, size_t* len);

/* TLC-like process exit code for the verdict (0 ok, 12 safety, 11 deadlock, 75 error). */
int mc_exit_code(const mc_ctx* ctx);

void mc_free(void* p);
void mc_close(mc_ctx* ctx);
const char* mc_last_error(const mc_ctx* ctx);

/* ---------------------------------------------------------------------------------------------
 * Sharded BFS (multi-GPU, one process per GPU).  The state space is partitioned by fingerprint
 * owner (owner = (fp >> 32) mod world): a rank expands its local frontier, routes every
 * in-model successor fingerprint to its owner, the owner dedups it against its local seen-set
 * and acknowledges the new ones, the generating rank materialises those states and ships them
 * to the owner, which stores them as its part of the next level.  The CALLER moves the buffers
 * between ranks (RCCL all-to-all through torch.distributed in raft-tla_amd/shard.py): every
 * mc_shard_* call below is rank-local device work.  Records: ROUTE 16 B (fp, slot),
 * REPLY 8 B (slot), STATES 80 B (64 B packed state, parent meta, fp).  Parent pointers carry
 * the rank in bits [37,40) of the global state id.
 * ------------------------------------------------------------------------------------------- */
#define MC_SHARD_ROUTE 0
#define MC_SHARD_REPLY 1
#define MC_SHARD_STATES 2
#define MC_SHARD_NSTAT 72   /* [0] new stored, [1] generated, [2] generated in model, [3] error flags,
                               [4] violation, [5] deadlock, [6] frontier, [7] spare,
                               [8..40) per-action generated, [40..72) per-action distinct          */
int mc_shard_open(mc_ctx* ctx, int32_t rank, int32_t world);
int mc_shard_record_bytes(const mc_ctx* ctx, int32_t what);
int mc_shard_frontier(const mc_ctx* ctx, int64_t* states, int64_t* chunk_states);
int mc_shard_generate(mc_ctx* ctx, int64_t begin, int64_t count, int64_t* route_counts);
int mc_shard_fill(mc_ctx* ctx, int32_t what, void* dst_device, const int64_t* dst_offsets);
int mc_shard_dedup(mc_ctx* ctx, const void* recv_device, const int64_t* recv_counts, int64_t* reply_counts);
int mc_shard_materialize(mc_ctx* ctx, const void* acks_device, const int64_t* ack_counts);
int mc_shard_store(mc_ctx* ctx, const void* states_device, int64_t n);
int mc_shard_level_stats(mc_ctx* ctx, int64_t* stats);
int mc_shard_level_commit(mc_ctx* ctx, const int64_t* global_stats, int32_t* done);
int mc_shard_read_state(const mc_ctx* ctx, uint64_t gid, char** text, size_t* len, uint64_t* meta);
int mc_shard_violation(const mc_ctx* ctx, uint64_t* parent_gid, char** action, char** text);

/* FIFO-ranked sharding (tlc_membership: VIEW vars makes the kept representative depend on TLC's
 * single-worker FIFO order).  Keys are global (global parent rank * slots + slot);
 * the owner's seen-set entry keeps the minimum key of the level, so winners are decided once per
 * level, not per chunk:
 *   mc_shard_layout(counts)        every rank's frontier size (global ranks in rank order)
 *   per chunk: mc_shard_generate -> ROUTE all-to-all -> mc_shard_dedup (no replies yet)
 *   mc_shard_select(reply_counts)  the owner's winning keys per generating rank -> REPLY all-to-all
 *   mc_shard_materialize(acks)     the generator sorts its winners and re-derives them in key order
 *   mc_shard_level_stats, all-reduce; on a stop (stats[4] != 0) mc_shard_event_stats, all-reduce
 *   (sum), merged into the global stats; mc_shard_level_commit
 *   rebalance: STATES records of the level's new states (key order, one run per rank) to equal
 *   contiguous slices of the next level, then mc_shard_store.
 * The driver is raft-tla_amd/shard.py (fifo_sharded_bfs). */
/* Native sharded BFS over RCCL (both spec families).  The same protocols as the caller-driven
 * mc_shard_* loops above, run entirely inside the library with grouped ncclSend/ncclRecv between
 * the kernels' own buffers — raft_original: three exchanges per level chunk on one HIP stream,
 * two host synchronisations per chunk (the record counts) and one per level (all-reduce of the
 * level statistics); tlc_membership: the FIFO-ranked protocol (layout all-gather, ROUTE per
 * chunk, select + REPLY, statistics, rebalance; csrc/fifo_shard_loop.h).  Replaces, like the
 * whole sharded path, TLC's multi-worker BFS (one JVM, shared FPSet).  The
 * same loops run behind mc_run when mc_opts.n_gpus > 1 (one host thread per GPU).
 *   mc_rccl_unique_id   rank 0 creates the communicator id (ncclGetUniqueId, 128 B) which
 *                       the caller broadcasts (torch.distributed in raft-tla_amd/shard.py)
 *   mc_shard_run_rccl   every rank: shard_open + ncclCommInitRank (cached on the handle for
 *                       repeated runs with the same id) + the whole level loop; afterwards
 *                       mc_summary / mc_shard_violation / mc_shard_read_state as usual.
 *   mc_shard_run_loopback  the same level loop for `world` ranks in ONE process (one host
 *                       thread and one handle per rank, every rank on its handle's device —
 *                       typically all on one GPU), the exchanges as device-to-device copies
 *                       between the ranks' buffers: the multi-rank path (routing, self
 *                       segments, all-reduce, counterexample gather) testable on one GPU.
 *                       ctxs[r] is rank r; results per handle as after mc_shard_run_rccl.
 * RCCL is dlopen()ed (librccl.so.1) on first use; MC_E_UNSUPPORTED if it cannot be loaded. */
int mc_rccl_unique_id(mc_ctx* ctx, void* out, size_t len);
int mc_shard_run_rccl(mc_ctx* ctx, int32_t rank, int32_t world, const void* unique_id, size_t len);
int mc_shard_run_loopback(mc_ctx* const* ctxs, int32_t world);

/* Source identity of this build: the first 16 hex digits of the SHA-256 of the library's
 * sources (raft-tla_amd/csrc/ *.h *.cpp *.hip in byte order, then this header), fixed at
 * compile time.  The Python binding compares it with the sources next to the library and refuses
 * a stale build, so a GPU run provably executes the tree it was shipped with. */
const char* mc_source_hash(void);

/* Test support: in the next sharded run (n_gpus > 1, mc_shard_run_*), rank `rank` leaves the native
 * level loop with MC_E_STATE when the search reaches `depth` -- a rank failure at a known point, to test
 * that its peers are released.  rank < 0 disables (the default).  Nothing else reads
 * it, and no environment variable does: a production run cannot trigger it by accident. */
int mc_set_fault_injection(mc_ctx* ctx, int32_t rank, int64_t depth);

/* Test support: tlc_membership's fingerprint kernel in TLC's symmetry rule keeps a parent's bag in a
 * per-lane LDS slice and leaves a parent whose bag could overflow it to a fallback kernel (DESIGN.md
 * §4b); this caps the slice at `entries` (0: every parent to the fallback; < 0: the compiled slice, the
 * default) so a test drives both kernels with a shipped config.  The fingerprints are the same either
 * way; nothing else reads it. */
int mc_set_fp_slice(mc_ctx* ctx, int32_t entries);
int mc_shard_layout(mc_ctx* ctx, const int64_t* frontier_counts);
int mc_shard_select(mc_ctx* ctx, int64_t* reply_counts);
int mc_shard_event_stats(mc_ctx* ctx, const int64_t* global_stats, int64_t* stats);

#ifdef __cplusplus
}
#endif
#endif /* RAFTMC_H */
