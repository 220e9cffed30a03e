"""The reference's one count-like claim (tlc_membership/raft.tla:1188-1191): "there are over 1.2
million traces of length 20 that satisfy CommitWhenConcurrentLeaders_constraint".  Runs the shipped
model (raft.cfg: 3 servers, NextAsyncCrash, SYMMETRY perms in TLC's rule, VIEW vars, the 12 shipped
constraints) with CommitWhenConcurrentLeaders_constraint added (configs/cwcl_count.cfg) on the GPU to
depth D and prints the distinct states per BFS level (TLC's depth: Init = 1).  Reading used in DESIGN.md
§2: a "trace of length 20" is a state at TLC depth 20 (a behaviour of 20 states) or 21 (20 steps).

    python scripts/cwcl_count.py [MAX_DEPTH]
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
raftmc = importlib.import_module("raft-tla_amd")
depth = int(sys.argv[1]) if len(sys.argv) > 1 else 22
t0 = time.time()
r = raftmc.check(os.path.join(ROOT, "configs", "raft_membership_mc.tla"), os.path.join(ROOT, "configs", "cwcl_count.cfg"),
                 max_depth=depth, deadlock=False)
print(json.dumps({"verdict": r.verdict, "depth": r.depth, "distinct": r.distinct, "generated": r.generated,
                  "levels": [lv[0] for lv in r.levels], "seconds": round(time.time() - t0, 2), "error": r.error}), flush=True)
