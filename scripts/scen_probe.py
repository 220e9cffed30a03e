"""GPU probe of the C4 scenario configs (configs/scen_*.cfg): verdict, violated property, depth,
counts and time per config, one JSON line each (used to decide which ones the CPU oracle can
reproduce as fixtures).   python scripts/scen_probe.py [name ...]"""
import glob
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mod = importlib.import_module("raft-tla_amd")
TLA = os.path.join(ROOT, "configs", "raft_membership_mc.tla")
names = sys.argv[1:] or sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(ROOT, "configs", "scen_*.cfg"))
                               if "_punct" not in p)
for n in names:
    t0 = time.time()
    try:
        r = mod.check(TLA, os.path.join(ROOT, "configs", n + ".cfg"), deadlock=False, max_depth=60)
        out = {"cfg": n, "verdict": r.verdict, "violated": r.violated, "depth": r.depth, "distinct": r.distinct,
               "generated": r.generated, "seconds": round(time.time() - t0, 2), "error": r.error[:200]}
    except Exception as e:   # noqa: BLE001 - report and go on
        out = {"cfg": n, "exception": str(e)[:300]}
    print(json.dumps(out), flush=True)
