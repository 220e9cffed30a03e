"""GPU probe of tlc_membership configs beyond the oracle's BFS reach: verdict, property, depth,
TLC's counters and time per config, one JSON line each, and the counterexample (one state per line,
the format of tests/golden/gpu_traces/*.txt) for the oracle's check-trace.

    python scripts/verdict_probe.py OUTDIR [tlc:]cfg[@depth] ...
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mod = importlib.import_module("raft-tla_amd")
TLA = os.path.join(ROOT, "configs", "raft_membership_mc.tla")
out = sys.argv[1]
os.makedirs(out, exist_ok=True)
for spec in sys.argv[2:]:
    tlc = spec.startswith("tlc:")
    name = spec[4:] if tlc else spec
    name, _, depth = name.partition("@")
    t0 = time.time()
    try:
        r = mod.check(TLA, os.path.join(ROOT, "configs", name + ".cfg"), deadlock=False, sym_tlc=tlc,
                      max_depth=int(depth or 0), state_store_bytes=int(os.environ.get("STORE_GB", "150")) << 30,
                      fp_table_bytes=int(os.environ.get("TABLE_GB", "32")) << 30)
        rec = {"case": spec, "verdict": r.verdict, "violated": r.violated, "depth": r.depth, "distinct": r.distinct,
               "generated": r.generated, "left_on_queue": r.left_on_queue, "exit_code": r.exit_code,
               "levels": [lv[0] for lv in r.levels], "actions": r.actions, "seconds": round(time.time() - t0, 2),
               "error": r.error[:300]}
        if r.trace_text.strip():
            blocks = r.trace_text.strip().split("\n\n")
            rec["trace_actions"] = ["Initial"] + [b.split("\n")[0].split("<", 1)[1].split(" ")[0].rstrip(">") for b in blocks[1:]]
            with open(os.path.join(out, spec.replace(":", "_") + ".txt"), "w") as f:
                f.write("\n".join(" ".join(b.split("\n")[1:]) for b in blocks) + "\n")
    except Exception as e:   # noqa: BLE001 - report and go on
        rec = {"case": spec, "exception": str(e)[:300]}
    print(json.dumps(rec), flush=True)
    with open(os.path.join(out, "probe.jsonl"), "a") as f:
        f.write(json.dumps(rec) + "\n")
