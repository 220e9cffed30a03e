"""C5 (BASELINE.json configs[4]: raft_original, 5 servers, term <= 3, log <= 3; configs/c5.cfg)
on one MI355X, depth-limited: the full state space needs the 8-GPU node, one GPU holds the
first levels.  Prints one JSON line per depth limit.  A measurement tool (C ABI only).

    python scripts/c5_probe.py [max_depth ...]

Environment: C5_CFG (default c5.cfg), C5_TABLE_GB, C5_STORE_GB, C5_WORKERS (default 1: TLC's FIFO
order), C5_COUNT_FINAL=1 (mc_opts.count_final_level: the last level counted, not stored).
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
raftmc = importlib.import_module("raft-tla_amd")
tla = os.path.join(ROOT, "configs", "raft_original_mc.tla")
cfg = os.path.join(ROOT, "configs", os.environ.get("C5_CFG", "c5.cfg"))
WORKERS = int(os.environ.get("C5_WORKERS", "1"))
COUNT_FINAL = os.environ.get("C5_COUNT_FINAL", "0") == "1"
TABLE = int(os.environ.get("C5_TABLE_GB", "32")) << 30
STORE = int(os.environ.get("C5_STORE_GB", "120")) << 30
for d in [int(x) for x in sys.argv[1:]] or [11, 12]:
    with raftmc.ModelChecker(tla, cfg, max_depth=d, fp_table_bytes=TABLE, state_store_bytes=STORE, seed=0x5EED,
                              workers=WORKERS, count_final_level=COUNT_FINAL) as mc:
        mc.run()                      # first run allocates the HBM buffers (hipMalloc of ~150 GB)
        t0 = time.perf_counter()
        r = mc.run()                  # timed: seen-set re-zeroed, every level re-expanded
        secs = time.perf_counter() - t0
    print(json.dumps({"config": os.path.basename(cfg), "workers": WORKERS, "count_final_level": COUNT_FINAL, "max_depth": d, "verdict": r.verdict, "distinct": r.distinct,
                      "generated": r.generated, "left_on_queue": r.left_on_queue, "seconds": secs, "table_gb": TABLE >> 30, "store_gb": STORE >> 30,
                      "distinct_per_s": r.distinct / secs, "levels": [lv[0] for lv in r.levels],
                      "kernels_ms": {k: round(v["ms"], 2) for k, v in r.kernels.items()},
                      "error": r.error}), flush=True)
