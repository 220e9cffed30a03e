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

The JSON line adds:
  roofline      dominant kernel (orig_generate): algorithmic bytes F*S + G_in*8 +
                D*(16+S) / summed HIP-event kernel time,
                against the 8 TB/s HBM peak; traffic from rocprofv3 PMC passes
                when --traffic-json points at their summary (else null); the
                dominant kernel is integer-VALU bound, so valu_issue_frac = its
                PMC VALU wave-instructions per launch (--valu-json) / (live
                launch time x 256 CUs x 2.4 GHz) is reported beside it
  cpu_baseline  the CPU oracle (oracle/, test infrastructure: "port") on a
                bounded sample of the same model (first --cpu-states distinct
                states of its BFS), --cpu-workers threads (successor expansion in
                parallel, merged in FIFO order; identical results to 1 thread)
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
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def cpu_baseline(cfg, max_states, workers):
    exe = os.path.join(ROOT, "oracle", "_build", "raft_oracle")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    t0 = time.time()
    out = subprocess.run([exe, "bfs", "--tla", TLA, "--cfg", cfg, "--max-states", str(max_states),
                          "--workers", str(workers)], capture_output=True, text=True, check=True, timeout=600)
    wall = time.time() - t0
    r = json.loads(out.stdout.strip().splitlines()[-1])
    secs = r["seconds"] or wall
    return {"value": r["distinct"] / secs, "unit": "distinct states/s", "cores": workers, "kind": "port",
            "sample": "oracle BFS of the same model stopped after %d distinct states (%d generated, %.1f s, "
                      "%d threads expanding, merge in FIFO order)" % (r["distinct"], r["generated"], secs, workers)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=os.path.join(ROOT, "configs", "c2.cfg"))
    ap.add_argument("--cpu-states", type=int, default=400000)
    # 1 thread: the oracle's value model shares reference-counted sub-values between states,
    # so its parallel expansion does not scale (MI355X box, 800k-state sample: 16 threads
    # 25.2k distinct/s vs 1 thread 35.6k distinct/s); the fastest configuration is reported
    ap.add_argument("--cpu-workers", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fp-table-bytes", type=int, default=0, help="seen-set bytes (0 = library default)")
    ap.add_argument("--state-store-bytes", type=int, default=0, help="state store bytes (0 = library default)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"))
    ap.add_argument("--valu-json", default=os.path.join(ROOT, "profiles", "valu_r01.json"))
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
    if world > 1:
        # owner-partitioned fingerprints, 3 RCCL all-to-alls per level chunk (raft-tla_amd/shard.py)
        shard = importlib.import_module("raft-tla_amd.shard")
        mc = shard.ShardedChecker(TLA, args.config, rank, world, device_index=local, seed=0x5EED)
    else:
        mc = mod.ModelChecker(TLA, args.config, device=local, seed=0x5EED, fp_table_bytes=args.fp_table_bytes,
                              state_store_bytes=args.state_store_bytes)

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        mc.run()
    barrier_sync()
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = mc.run()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    mc.close()
    assert res.verdict == "OK", (res.verdict, res.error)

    # the sharded result is global (every rank reports the whole model's counts)
    total_distinct = float(res.distinct)
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])

    if rank == 0:
        per_step = elapsed / args.steps
        # dominant kernel = the one with the most HIP-event time in the last run
        kname, kst = max(res.kernels.items(), key=lambda kv: kv[1]["ms"])
        achieved = kst["algo_bytes"] / (kst["ms"] / 1e3) / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("kernel_name") == kname:
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
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
            "config": {"workload": "C2: raft_original.tla + configs/c2.cfg (3 servers, 2 values, term<=3, log<=2, msgs<=5)",
                       "distinct_per_run": res.distinct, "generated_per_run": res.generated, "depth": res.depth,
                       "kernel_ms_per_run": res.kernel_seconds * 1000.0, "launches_per_run": res.n_launches,
                       "state_bytes": res.state_bytes,
                       "parallelism": "single" if world == 1 else "fp-owner-sharded x%d (RCCL all-to-all)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kname, "algo_bytes_per_launch": kst["algo_bytes"] / max(1, kst["launches"]),
                         "avg_launch_ms": kst["ms"] / max(1, kst["launches"])},
            "kernels": {k: {"ms": v["ms"], "launches": v["launches"],
                            "algo_GBps": v["algo_bytes"] / max(v["ms"], 1e-9) / 1e6} for k, v in res.kernels.items()},
        }
        # the dominant kernel is integer-VALU bound: its VALU issue fraction (PMC instruction count per
        # launch from profiles/, live launch time) next to the HBM roofline
        if os.path.exists(args.valu_json):
            try:
                vj = json.load(open(args.valu_json))
                if vj.get("kernel_name") == kname:
                    avg_s = kst["ms"] / max(1, kst["launches"]) / 1e3
                    line["roofline"]["valu_issue_frac"] = vj["valu_insts_per_launch"] / (avg_s * vj["peak_valu_insts_per_s"])
            except Exception:
                pass
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.config, args.cpu_states, args.cpu_workers)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
