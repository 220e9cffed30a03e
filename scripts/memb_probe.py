"""Probe tlc_membership runs on the GPU: state-space growth and throughput.

    python scripts/memb_probe.py CFG [MAX_DEPTH ...] [--trace-out FILE]

Prints one JSON line per run (verdict, counts, seconds, per-kernel ms).  A
development tool: it drives the product through the C ABI only.
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
raftmc = importlib.import_module("raft-tla_amd")

args = sys.argv[1:]
trace_out = None
sym_tlc = "--orbit" not in args          # TLC's SYMMETRY rule by default (the drop-in); --orbit: the orbit mode
args = [a for a in args if a != "--orbit"]
if "--trace-out" in args:
    k = args.index("--trace-out")
    trace_out = args[k + 1]
    del args[k:k + 2]
cfg = args[0]
depths = [int(x) for x in args[1:]] or [0]
for d in depths:
    t0 = time.time()
    with raftmc.ModelChecker(os.path.join(ROOT, "configs", "raft_membership_mc.tla"), os.path.join(ROOT, "configs", cfg + ".cfg"),
                             max_depth=d, deadlock=False, sym_tlc=sym_tlc) as mc:
        r = mc.run()
    if trace_out and r.trace_text:
        # one state per line (the oracle's check-trace format)
        with open(trace_out, "w") as f:
            for blk in r.trace_text.strip().split("\n\n"):
                f.write(" ".join(blk.split("\n")[1:]) + "\n")
    print(json.dumps({"cfg": cfg, "max_depth": d, "symmetry": "tlc" if sym_tlc else "orbit", "verdict": r.verdict, "error": r.error[:200], "generated": r.generated,
                      "distinct": r.distinct, "depth": r.depth, "violated": r.violated, "left": r.left_on_queue, "wall_s": round(time.time() - t0, 3),
                      "run_s": round(r.seconds, 3), "kernel_s": round(r.kernel_seconds, 3),
                      "distinct_per_s": r.distinct / max(r.seconds, 1e-9),
                      "kernels_ms": {k: round(v["ms"], 2) for k, v in r.kernels.items()},
                      "levels": [lv[0] for lv in r.levels]}), flush=True)
