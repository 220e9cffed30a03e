"""Run a config on the GPU and write its counterexample, one state per line (the oracle's
check-trace input format), plus the summary as JSON.
    python scripts/dump_trace.py SPEC.tla CFG OUT_PREFIX [--no-deadlock]"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mod = importlib.import_module("raft-tla_amd")
tla, cfg, out = sys.argv[1:4]
r = mod.check(tla, cfg, deadlock=False)
blocks = r.trace_text.strip().split("\n\n") if r.trace_text.strip() else []
with open(out + ".txt", "w") as f:
    for b in blocks:
        f.write(" ".join(b.split("\n")[1:]) + "\n")
json.dump({"cfg": os.path.basename(cfg), "verdict": r.verdict, "violated": r.violated, "depth": r.depth,
           "distinct": r.distinct, "generated": r.generated, "left_on_queue": r.left_on_queue,
           "actions": [b.split("\n")[0] for b in blocks]}, open(out + ".json", "w"), indent=1)
print(r.verdict, r.violated, r.depth, r.distinct, r.generated)
