"""Probe raft_original (C2 by default) on the GPU: per-kernel time vs seen-set size.

    python scripts/orig_probe.py [CFG] [--table-gb 0.5,1,2,4,8] [--runs 3]

Prints one JSON line per table size.  A development tool: it drives the product through the
C ABI only."""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
raftmc = importlib.import_module("raft-tla_amd")

ap = argparse.ArgumentParser()
ap.add_argument("cfg", nargs="?", default="c2")
ap.add_argument("--table-gb", default="0.5,1,2,4,8")
ap.add_argument("--runs", type=int, default=3)
a = ap.parse_args()
for gb in [float(x) for x in a.table_gb.split(",")]:
    with raftmc.ModelChecker(os.path.join(ROOT, "configs", "raft_original_mc.tla"), os.path.join(ROOT, "configs", a.cfg + ".cfg"),
                             fp_table_bytes=int(gb * (1 << 30))) as mc:
        mc.run()
        t0 = time.perf_counter()
        for _ in range(a.runs):
            r = mc.run()
        wall = (time.perf_counter() - t0) / a.runs
    print(json.dumps({"table_gb": gb, "distinct": r.distinct, "ms_per_run": wall * 1e3,
                      "kernels_ms": {k: round(v["ms"], 2) for k, v in r.kernels.items()}}), flush=True)
