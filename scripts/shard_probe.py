"""Time the sharded raft_original pipeline at world 1 (no communication) against the single-GPU
pipeline on C2: the per-rank cost of the sharded kernels.  A development tool (C ABI only).

    python scripts/shard_probe.py [CFG]
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
raftmc = importlib.import_module("raft-tla_amd")
shard = importlib.import_module("raft-tla_amd.shard")
cfg = os.path.join(ROOT, "configs", (sys.argv[1] if len(sys.argv) > 1 else "c2") + ".cfg")
tla = os.path.join(ROOT, "configs", "raft_original_mc.tla")
sc = shard.ShardedChecker(tla, cfg, 0, 1, seed=0x5EED)
sc.run()
t0 = time.perf_counter()
r = sc.run()
ms = (time.perf_counter() - t0) * 1e3
sc.close()
print(json.dumps({"mode": "sharded_w1", "distinct": r.distinct, "generated": r.generated, "ms": ms,
                  "kernels_ms": {k: round(v["ms"], 2) for k, v in r.kernels.items()}}), flush=True)
with raftmc.ModelChecker(tla, cfg, seed=0x5EED) as mc:
    mc.run()
    t0 = time.perf_counter()
    r = mc.run()
    ms = (time.perf_counter() - t0) * 1e3
print(json.dumps({"mode": "single", "distinct": r.distinct, "generated": r.generated, "ms": ms,
                  "kernels_ms": {k: round(v["ms"], 2) for k, v in r.kernels.items()}}), flush=True)
