"""bench.py — distinct states/sec of the Raft BFS model checker on MI355X.

Workload (BASELINE.json configs[1], `C2`): thirdparty/raft_original.tla with
configs/c2.cfg (3 servers, 2 values, term <= 3, log <= 2, |DOMAIN messages|
<= 5 with counts 0..1), checking ElectionSafety and LogMatching.  One *step*
is one complete breadth-first model-checking run of that model on the GPU
(seen-set re-zeroed, every level expanded; the state store stays allocated
between steps, the inputs are the spec/cfg only).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 (torchrun, one process per GPU): the model is checked ONCE by all
ranks together: fingerprints are owner-partitioned and every level chunk
exchanges candidates, acknowledgements and new states with three RCCL
all-to-alls (raft-tla_amd/shard.py); value = the model's distinct states /
max-over-ranks time of one run, "scaling": "strong" (total work fixed).

Beside the headline, every invocation measures (same N, same path, outside the headline's timed
region; each with its own barrier-bracketed max-over-ranks timing):
  scale_workload  C5v2 to depth 12 (configs/c5v2.cfg: BASELINE configs[4]'s 5-server model,
                  482M distinct states), the workload large enough for a 1/2/4/8-GPU curve
  scale_workload_configs4  C5v2 to depth 13 (2.44e9 distinct, its last level counted, not stored:
                  mc_opts.count_final_level, single GPU and the sharded native loop alike), at every
                  N; at N=8 also scale_workload_configs4_d14, depth 14 (~1e10 distinct: the config's
                  scale, its levels 0-13 stored over the 8 ranks)
  variants        C2 with MaxMsgDomain = 6 (configs/c2_md6.cfg): AppendEntries responses and
                  commits fire, which C2 as frozen (5 messages) never reaches; at N=1 also C2
                  through the generated path (the front end's code for the
                  unmodified raft_original.tla, one run)

The JSON line adds:
  roofline      dominant kernel (the one with the most HIP-event time): SURVEY.md
                §8(d)'s algorithmic bytes of the run, B = F*S + G_in*8 + D*(16+S) (F frontier
                states expanded, S stored state bytes, G_in in-model successors, D new states),
                per launch of that kernel / its average launch time (HIP events on the library's
                stream), against the 8 TB/s HBM peak; traffic = HBM bytes per launch from the
                rocprofv3 PMC passes committed under profiles/ (FETCH_SIZE x2 + WRITE_SIZE,
                MI355X_MICROARCH.md), or null; valu_issue_frac = PMC VALU wave-instructions per
                launch / (launch time x 256 CUs x 2 wave64 issues per CU-cycle x 2.4 GHz); both PMC
                figures only when the summary names the same kernel AND workload; pipeline_frac =
                the same bytes over the whole step time (every kernel and the host between them)
  dedup_set     the BASELINE metric's second half: dedup-set GB/s (G_in*8 + D*16) / (merge +
                probe kernel time), seen-set probes/s (the device's probe count / that time:
                successors the same workgroup produced twice probe once) and the transaction-level
                figure (probes * 64 B / that time, against the 8 TB/s peak)
  cpu_baseline  the builder's multithreaded C++ CPU BFS (oracle/cpu_bfs.cpp: TLC-style workers, a
                lock-free fingerprint set, the product's packed successor function and invariants;
                "port") with threads = the host cores of this job, on the whole C2 (bounded by
                --cpu-states); beside it the value-model oracle (oracle/main.cpp, one thread) on a
                bounded prefix
"""
import argparse
import importlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

TLA = os.path.join(ROOT, "configs", "raft_original_mc.tla")
TLA_MEMB = os.path.join(ROOT, "configs", "raft_membership_mc.tla")
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def cpu_baseline(cfg, max_states, workers, oracle_states):
    """SURVEY.md §8(d)'s CPU baseline: TLC is not available offline, so the builder's multithreaded
    C++ BFS (oracle/cpu_bfs.cpp: TLC-style workers, lock-free fingerprint set, the packed successor
    function) with threads = the host cores this job may use, on the same model; beside it the
    value-model oracle (oracle/main.cpp, the literal restatement, one thread) on a bounded prefix."""
    odir = os.path.join(ROOT, "oracle")
    exe = os.path.join(odir, "_build", "cpu_bfs_c2")
    orc = os.path.join(odir, "_build", "raft_oracle")
    if not (os.path.exists(exe) and os.path.exists(orc)):
        subprocess.run(["make", "-s", "-C", odir], check=True)
    out = subprocess.run([exe, cfg, "--threads", str(workers), "--max-states", str(max_states)], capture_output=True,
                         text=True, check=True, timeout=600)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    whole = r["verdict"] == "OK"
    res = {"value": r["distinct"] / r["seconds"], "unit": "distinct states/s", "cores": r["threads"], "kind": "port",
           "sample": "%s: %d distinct / %d generated states in %.2f s, %d threads (oracle/cpu_bfs.cpp: TLC-style "
                     "multithreaded BFS, lock-free 64-bit fingerprint set, packed states)"
                     % ("the whole C2 state space" if whole else "C2 BFS stopped after %d distinct" % r["distinct"],
                        r["distinct"], r["generated"], r["seconds"], r["threads"])}
    out = subprocess.run([orc, "bfs", "--tla", TLA, "--cfg", cfg, "--max-states", str(oracle_states)],
                         capture_output=True, text=True, check=True, timeout=600)
    o = json.loads(out.stdout.strip().splitlines()[-1])
    res["oracle_value_model"] = {"value": o["distinct"] / o["seconds"], "cores": 1,
                                 "sample": "oracle/main.cpp (literal TLA+ value-model restatement) stopped after %d "
                                           "distinct states, %.1f s" % (o["distinct"], o["seconds"])}
    return res


def workload_name(cfg, max_depth):
    base = os.path.basename(cfg)
    if base == "c2.cfg":
        name = "C2: raft_original.tla + configs/c2.cfg (3 servers, 2 values, term<=3, log<=2, msgs<=5)"
    else:
        name = "raft_original.tla + configs/%s" % base
    return name + (" to depth %d" % max_depth if max_depth else "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=os.path.join(ROOT, "configs", "c2.cfg"))
    # depth-bounded runs of the larger models (configs/c5.cfg: BASELINE configs[4], the 8-GPU workload)
    ap.add_argument("--max-depth", type=int, default=0)
    ap.add_argument("--cpu-states", type=int, default=60000000, help="bound of the multithreaded CPU BFS (C2: 54.4M)")
    ap.add_argument("--oracle-states", type=int, default=300000, help="bound of the value-model oracle's BFS")
    # the host cores this job may use (the GPU box exports OMP_NUM_THREADS = its CPU share)
    ap.add_argument("--cpu-workers", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count())
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fp-table-bytes", type=int, default=0, help="seen-set bytes (0 = library default)")
    # TLC -workers: the CPU reference point is TLC with -workers = host cores (BASELINE north_star), whose
    # order-dependent outputs are nondeterministic; 1 = TLC's single-worker FIFO order (also measured
    # below, as fifo_ms_per_step, when --fifo-steps > 0)
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--fifo-steps", type=int, default=3)
    ap.add_argument("--state-store-bytes", type=int, default=0, help="state store bytes (0 = library default)")
    # committed rocprofv3 summaries of the dominant kernel (default: the one for whichever kernel dominates)
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--valu-json", default=None)
    ap.add_argument("--no-extra", action="store_true", help="skip the scale_workload / variants measurements")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    mod = importlib.import_module("raft-tla_amd")
    shard = importlib.import_module("raft-tla_amd.shard") if world > 1 else None

    def checker(cfg, max_depth, store, table, workers, tla=TLA, count_final=False, seed=0x5EED):
        if world > 1:
            # owner-partitioned fingerprints, 3 RCCL all-to-alls per level chunk (the library's native
            # level loop, raft-tla_amd/shard.py ShardedChecker); raft_original's sharded search has
            # -workers N semantics (count_final_level needs it said: workers != 1)
            return shard.ShardedChecker(tla, cfg, rank, world, device_index=local, seed=seed, fp_table_bytes=table,
                                        state_store_bytes=store, max_depth=max_depth, workers=workers,
                                        count_final_level=count_final)
        return mod.ModelChecker(tla, cfg, device=local, seed=seed, fp_table_bytes=table, state_store_bytes=store,
                                workers=workers, max_depth=max_depth, count_final_level=count_final)

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    def measure(cfg, max_depth, steps, warmup, store, table, workers, tla=TLA, count_final=False, seed=0x5EED):
        """W untimed runs, then K timed runs bracketed by barrier + device sync; max over ranks"""
        mc = checker(cfg, max_depth, store, table, workers, tla, count_final, seed)
        try:
            for _ in range(warmup):
                mc.run()
            barrier_sync()
            t0 = time.perf_counter()
            r = None
            for _ in range(steps):
                r = mc.run()
            barrier_sync()
            elapsed = time.perf_counter() - t0
        finally:
            mc.close()
        assert r.verdict == "OK" or (max_depth and r.verdict == "DEPTH_LIMIT"), (r.verdict, r.error)
        return r, max_over_ranks(elapsed) / steps

    res, per_step = measure(args.config, args.max_depth, args.steps, args.warmup, args.state_store_bytes,
                            args.fp_table_bytes, args.workers)
    # the seen-set probes of one run, counted by the instrumented dedup kernel in a run of its own
    # (RAFTMC_COUNT_PROBES; the timed runs use the uninstrumented one)
    probes_per_run = None
    if world == 1 and args.workers != 1:
        os.environ["RAFTMC_COUNT_PROBES"] = "1"
        try:
            with checker(args.config, args.max_depth, args.state_store_bytes, args.fp_table_bytes, args.workers) as mc:
                probes_per_run = mc.run().seen_set_probes
        finally:
            del os.environ["RAFTMC_COUNT_PROBES"]
    # TLC -workers 1 (FIFO order) on the same model, outside the timed region: its cost is reported
    fifo = None
    if world == 1 and args.workers != 1 and args.fifo_steps > 0:
        r1, t1 = measure(args.config, args.max_depth, args.fifo_steps, 1, args.state_store_bytes, args.fp_table_bytes, 1)
        fifo = {"ms_per_step": t1 * 1e3, "steps": args.fifo_steps, "distinct_per_run": r1.distinct,
                "generated_per_run": r1.generated, "kernels_ms": {k: v["ms"] for k, v in r1.kernels.items() if v["launches"]}}
        assert (r1.distinct, r1.generated, r1.depth) == (res.distinct, res.generated, res.depth)

    def side(cfg, max_depth, store_gib, table_gib, steps, tla=TLA, workers=None, count_final=False, seed=0x5EED,
             split_table=False):
        """a second workload at the same N through the same path; its failure is reported, not fatal.
        store_gib: the whole job's (split over the ranks with a 1.3x margin); table_gib: per rank, or the
        whole job's with split_table (a power of two per rank)"""
        name = workload_name(cfg, max_depth) if tla == TLA else "tlc_membership/raft.tla + configs/%s%s" % (
            os.path.basename(cfg), " to depth %d" % max_depth if max_depth else "")
        if count_final:
            name += ", its last level counted, not stored (count_final_level)"
        try:
            store = int(store_gib * (1 << 30) / world * (1.3 if world > 1 else 1.0))
            table = int(table_gib * (1 << 30))
            if split_table:
                table = 1 << max(24, (table // world - 1).bit_length())
            r, t = measure(cfg, max_depth, steps, 1, store, table, args.workers if workers is None else workers, tla,
                           count_final, seed)
            out = {"workload": name, "value": r.distinct / t, "unit": "distinct states/s",
                   "ms_per_step": t * 1e3, "steps": steps, "distinct_per_run": r.distinct, "generated_per_run": r.generated,
                   "depth": r.depth, "verdict": r.verdict, "seed": seed,
                   "collision_prob_optimistic": r.collision_prob_optimistic,
                   "store_bytes_per_rank": store, "table_bytes_per_rank": table,
                   "kernels_ms": {k: v["ms"] for k, v in r.kernels.items() if v["launches"]}}
            ks = {k: v for k, v in r.kernels.items() if v["launches"]}
            if ks and r.algo_bytes:   # the dominant kernel against the HBM roofline, SURVEY.md 8(d) bytes
                kname, kst = max(ks.items(), key=lambda kv: kv[1]["ms"])
                avg_s = kst["ms"] / kst["launches"] / 1e3
                ach = r.algo_bytes / kst["launches"] / avg_s / 1e9
                out["roofline"] = {"bound": "hbm", "kernel": kname, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": ach / HBM_PEAK_GBS, "avg_launch_ms": avg_s * 1e3}
            return out
        except Exception as e:   # noqa: BLE001 - the headline stands on its own
            return {"workload": name, "error": str(e)[:300]}

    def generated_c2():
        """C2 through the generated path (the SANY-subset front end's code for the unmodified
        thirdparty/raft_original.tla, prebuilt by build(): DESIGN.md §8): one untimed run (it allocates
        the 200 GiB store, as the headline's warmup does), then one timed run"""
        src = os.path.join(ROOT, "raft-tla_amd", "_build", "tlagen_co", "c2.gen.hip")
        try:
            with mod.ModelChecker(src, os.path.join(ROOT, "configs", "c2.cfg"), frontend="generated", workers=0, device=local,
                                  fp_table_bytes=1 << 30, state_store_bytes=200 << 30) as mc:
                r0 = mc.run()
                t0 = time.perf_counter()
                r = mc.run()
                t = time.perf_counter() - t0
                first_s = r0.seconds
            return {"workload": "C2 via the generated path (front end + generic kernels)", "value": r.distinct / t,
                    "unit": "distinct states/s", "ms_per_step": t * 1e3, "steps": 1, "warmup": 1,
                    "first_run_s": round(first_s, 3), "distinct_per_run": r.distinct,
                    "generated_per_run": r.generated, "depth": r.depth, "verdict": r.verdict,
                    "collision_prob_optimistic": r.collision_prob_optimistic}
        except Exception as e:   # noqa: BLE001
            return {"workload": "C2 via the generated path", "error": str(e)[:300]}

    extra = {}
    if not args.no_extra:
        # C5v2 to depth 12: 482M states of 160 B + 8 B parent pointers = 81 GB, and the host spill's
        # 1.5x margin on the next level must not trigger: 128 GiB at N=1 (a 96 GiB store spilled the
        # completed levels to host memory every run, 1.04 s instead of 0.23 s)
        extra["scale_workload"] = side(os.path.join(ROOT, "configs", "c5v2.cfg"), 12, 128, 16, 2)
        # the membership model (C3 without the invariant it violates at depth 21), depth-bounded: TLC's
        # FIFO first-found order under VIEW and SYMMETRY in TLC's rule; at N > 1 the FIFO-ranked sharded
        # level loop (csrc/fifo_shard_loop.h), so the scaling curve covers both spec families
        extra["scale_workload_membership"] = side(os.path.join(ROOT, "configs", "memb_four_scale.cfg"), 20, 64, 8, 2,
                                                  tla=TLA_MEMB, workers=1)
        extra["variants"] = {"c2_md6": side(os.path.join(ROOT, "configs", "c2_md6.cfg"), 0, 64, 8, 2)}
        # BASELINE configs[4] (raft_original, 5 servers, term <= 3, log <= 3): C5v2 to depth 13, 2.44e9
        # distinct states, at every N (the same workload along the 1/2/4/8 curve), its level 13 counted, not
        # stored (mc_opts.count_final_level: single GPU and the sharded native loop), the stores holding
        # levels 0-12 (81 GB over the ranks); seed 1 (0x5EED loses one state of this model to a 64-bit
        # fingerprint collision, tests/test_gpu.py test_c5v2_depth13_count_final_level)
        c5v2 = os.path.join(ROOT, "configs", "c5v2.cfg")
        extra["scale_workload_configs4"] = side(c5v2, 13, 96 if world > 1 else 120, 64, 1, workers=0, count_final=True, seed=1,
                                                split_table=True)
        if world == 8:
            # depth 14 (~1e10 distinct, the config's scale): levels 0-13 stored over the 8 ranks (410 GB)
            extra["scale_workload_configs4_d14"] = side(c5v2, 14, 420, 256, 1, workers=0, count_final=True, seed=1,
                                                        split_table=True)
        if world == 1:
            extra["variants"]["c2_generated"] = generated_c2()

    if rank == 0:
        total_distinct = float(res.distinct)    # the sharded result is global (every rank reports the model's counts)
        kernels = {k: v for k, v in res.kernels.items() if v["launches"] > 0}
        # dominant kernel = the one with the most HIP-event time in the last run
        kname, kst = max(kernels.items(), key=lambda kv: kv[1]["ms"])
        launches = max(1, kst["launches"])
        avg_s = kst["ms"] / launches / 1e3
        # F*S + G_in*8 + D*(16+S) summed over the levels of the run (mc_summary.algo_bytes)
        bytes_per_launch = res.algo_bytes / launches
        achieved = bytes_per_launch / avg_s / 1e9
        wl_key = os.path.basename(args.config) + ("@%d" % args.max_depth if args.max_depth else "")

        # the library's kernel names -> rocprofv3's (orig_merge_probe is the fused orig_dedup_plain)
        rocprof_name = {"orig_merge_probe": "orig_dedup_plain"}.get(kname, kname)
        defaults = {"orig_generate": ("traffic_r06f_c2_generate.json", "valu_r06f_c2_generate.json"),
                    "orig_merge_probe": ("traffic_r06f_c2_dedup.json", None)}.get(kname, (None, None))

        def pmc_summary(path, default):
            """a committed rocprofv3 summary of this kernel on this workload, else None"""
            path = path or (os.path.join(ROOT, "profiles", default) if default else None)
            try:
                doc = json.load(open(path))
            except (OSError, ValueError, TypeError):
                return None
            return doc if doc.get("kernel_name") in (kname, rocprof_name) and doc.get("workload") == wl_key else None

        tj = pmc_summary(args.traffic_json, defaults[0])
        ded = [v for k, v in kernels.items() if k in ("orig_merge_probe", "orig_dedup")]
        ded_s = sum(v["ms"] for v in ded) / 1e3
        line = {
            "metric": "distinct states/sec (node) on Raft BFS",
            "value": total_distinct / per_step,
            "unit": "distinct states/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1000.0,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: the model's own reachable state space (no external data)",
            "config": {"workload": workload_name(args.config, args.max_depth),
                       "tlc_workers": args.workers,
                       "distinct_per_run": res.distinct, "generated_per_run": res.generated, "depth": res.depth,
                       "generated_in_model_per_run": res.generated_in_model,
                       "kernel_ms_per_run": res.kernel_seconds * 1000.0, "launches_per_run": res.n_launches,
                       "state_bytes": res.state_bytes, "seed": 0x5EED,
                       "collision_prob_optimistic": res.collision_prob_optimistic,
                       "parallelism": "single" if world == 1 else "fp-owner-sharded x%d (RCCL all-to-all)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": tj.get("hbm_bytes_per_launch") if tj else None,
                         "kernel": kname, "algo_bytes_per_launch": bytes_per_launch, "avg_launch_ms": avg_s * 1e3,
                         "pipeline_frac": res.algo_bytes / per_step / 1e9 / HBM_PEAK_GBS,
                         "bytes": "SURVEY.md 8(d): F*S + G_in*8 + D*(16+S) of the run / launches of the dominant kernel",
                         "timed": "HIP events around the kernel's launch pair orig_generate + orig_generate_lead (the "
                                  "leader-work pass over the same parents): rocprofv3 lists them as two kernels whose "
                                  "averages add up to avg_launch_ms" if kname == "orig_generate" else "HIP events around the kernel"},
            "kernels": {k: {"ms": v["ms"], "launches": v["launches"],
                            "algo_GBps": v["algo_bytes"] / max(v["ms"], 1e-9) / 1e6} for k, v in kernels.items()},
        }
        if fifo is not None:
            line["tlc_workers_1"] = fifo
        if ded_s > 0:
            # probes: the device's count of fingerprints that reached the seen-set (a successor that the
            # same 256 parents produced before is filtered in LDS and never probes); the transaction-level
            # figure prices each probe at one 64-B HBM line (8 TB/s / 64 B = 125 G/s)
            probes = probes_per_run or 0
            line["dedup_set"] = {"GBps": (res.generated_in_model * 8 + res.distinct * 16) / ded_s / 1e9,
                                 "probes_per_s": probes / ded_s, "probes_per_run": probes,
                                 "successors_per_s": res.generated_in_model / ded_s,
                                 "transaction_GBps": probes * 64 / ded_s / 1e9,
                                 "transaction_frac": probes * 64 / ded_s / 1e9 / HBM_PEAK_GBS, "ms": ded_s * 1e3,
                                 "bytes": "G_in*8 + D*16 (SURVEY.md 8(d) dedup-set metric) / (merge + probe kernel time); "
                                          "transaction: probes * 64 B / the same time; probes_per_run counted in an extra "
                                          "run by the instrumented dedup kernel (RAFTMC_COUNT_PROBES), rates over the timed runs' time"}
        # VALU issue fraction of the dominant kernel: PMC instruction count per launch from profiles/, live
        # launch time; MI355X_MICROARCH.md: 4 SIMD-32 per CU, a wave64 VALU instruction issues in 2 cycles
        vj = pmc_summary(args.valu_json, defaults[1])
        if vj:
            line["roofline"]["valu_issue_frac"] = vj["valu_insts_per_launch"] / (avg_s * 256 * 2 * 2.4e9)
        line.update(extra)
        if not args.no_cpu_baseline and os.path.basename(args.config) == "c2.cfg" and not args.max_depth:
            line["cpu_baseline"] = cpu_baseline(args.config, args.cpu_states, args.cpu_workers, args.oracle_states)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
