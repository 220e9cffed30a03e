"""Time the generated path on full-size C2 (raft_original.tla through the SANY-subset front end,
prebuilt source) on the GPU box; one JSON line per run.

    python scripts/tlagen_c2_time.py [WAVES[@STORE_GIB][xREPS] ...]     (default 8@200)

Each run reports the wall time of mc_run, its kernel time and the rest (allocation, host work)."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rm = importlib.import_module("raft-tla_amd")
src = os.path.join(ROOT, "raft-tla_amd", "_build", "tlagen_co", "c2.gen.hip")
for spec in sys.argv[1:] or ["8@200"]:
    spec, _, reps = spec.partition("x")
    waves, _, gib = spec.partition("@")
    os.environ["RAFTMC_TLAGEN_WAVES"] = waves
    os.environ["RAFTMC_TLAGEN_TIMING"] = "1"
    with rm.ModelChecker(src, os.path.join(ROOT, "configs", "c2.cfg"), frontend="generated", workers=0,
                         fp_table_bytes=1 << 30, state_store_bytes=int(gib or 200) << 30) as mc:
      for rep in range(int(reps or 1)):   # later runs reuse the first one's device buffers
        r = mc.run()
        print(json.dumps({"rep": rep, "run_s": round(r.seconds, 3), "kernel_s": round(r.kernel_seconds, 3)}), flush=True)
    print(json.dumps({"workload": "C2 via the generated path", "waves_per_cu": int(waves), "verdict": r.verdict,
                      "distinct": r.distinct, "generated": r.generated, "depth": r.depth, "run_s": round(r.seconds, 3),
                      "kernel_s": round(r.kernel_seconds, 3), "other_s": round(r.seconds - r.kernel_seconds, 3),
                      "store_gib": int(gib or 200), "distinct_per_s": r.distinct / r.seconds,
                      "kernels_ms": {k: round(v["ms"], 1) for k, v in r.kernels.items()},
                      "levels": [[lv[0], lv[1], round(lv[2], 1)] for lv in r.levels]}), flush=True)
