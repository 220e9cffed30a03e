"""Re-measure the stop-point counters of tests/golden/gpu_traces cases on the GPU box (after a change
to TLC's counting semantics), and check the traces still match.  One JSON line per (case, mode).

    python scripts/gpu_trace_counts.py CASE [CASE ...]
"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rm = importlib.import_module("raft-tla_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
cases = json.load(open(os.path.join(GOLDEN, "gpu_traces", "index.json")))["cases"]
for case in sys.argv[1:]:
    g = cases[case]
    for mode in ["fixture"] + (["tlc"] if "oracle_pin_tlc" in g else []):
        sym_tlc = g.get("sym") == "tlc" if mode == "fixture" else True
        r = rm.check(os.path.join(ROOT, "configs", "raft_membership_mc.tla"), os.path.join(ROOT, "configs", case + ".cfg"),
                     deadlock=False, sym_tlc=sym_tlc)
        got = [" ".join(b.split("\n")[1:]) for b in r.trace_text.strip().split("\n\n")]
        want = open(os.path.join(GOLDEN, "gpu_traces", case + ".txt")).read().strip().split("\n")
        print(json.dumps({"case": case, "mode": mode, "verdict": r.verdict, "violated": r.violated, "depth": r.depth,
                          "distinct": r.distinct, "generated": r.generated, "left_on_queue": r.left_on_queue,
                          "actions": r.actions, "trace_equal": got == want}), flush=True)
