"""C3 (configs/memb_four.cfg: tlc_membership/raft.tla, 4 servers, NextDynamic, VIEW + SYMMETRY in TLC's
rule) through BOTH compiled forms on the GPU box: the generated path (the unmodified module through the
SANY-subset front end, prebuilt as _build/tlagen_co/memb_four_gen.gen.hip) and the hand-compiled
kernels, at each depth bound given; one JSON line per (path, depth) with the counts and the time, and
a line saying whether the two agree.  A development and cross-validation tool (C ABI only).

    python scripts/tlagen_memb_probe.py DEPTH [DEPTH ...]      (0 = unbounded)
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rm = importlib.import_module("raft-tla_amd")
CFG = os.path.join(ROOT, "configs", "memb_four.cfg")
GEN = os.path.join(ROOT, "raft-tla_amd", "_build", "tlagen_co", "memb_four_gen.gen.hip")
HAND = os.path.join(ROOT, "configs", "raft_membership_mc.tla")


def one(path, frontend, depth):
    t0 = time.time()
    with rm.ModelChecker(path, CFG, frontend=frontend, max_depth=depth, deadlock=False, workers=1,
                         fp_table_bytes=8 << 30, state_store_bytes=(160 << 30) if frontend == "generated" else 0) as mc:
        r = mc.run()
    d = {"path": frontend, "max_depth": depth, "verdict": r.verdict, "violated": r.violated, "distinct": r.distinct,
         "generated": r.generated, "depth": r.depth, "left": r.left_on_queue, "run_s": round(r.seconds, 3),
         "wall_s": round(time.time() - t0, 3), "levels": [lv[0] for lv in r.levels], "error": r.error[:200],
         "actions": r.actions, "trace_states": len(r.trace_text.strip().split("\n\n")) if r.trace_text.strip() else 0}
    print(json.dumps(d), flush=True)
    return d


# the front end labels a successor by the defined operator it came from; the hand kernels by handler
GROUPS = {"ReceiveDirect": ("HandleRequestVoteRequest", "DropStaleResponse", "HandleRequestVoteResponse",
                            "HandleAppendEntriesRequest", "HandleAppendEntriesResponse", "HandleCatchupRequest",
                            "HandleCatchupResponse", "HandleCheckOldConfig"),
          "NextUnreliable": ("DuplicateMessage", "DropMessage")}


def grouped(actions):
    out = {}
    for a, (g, d) in actions.items():
        a = next((k for k, v in GROUPS.items() if a in v), a)
        if g or d:
            out[a] = [out.get(a, [0, 0])[0] + g, out.get(a, [0, 0])[1] + d]
    return out


for depth in [int(x) for x in sys.argv[1:]] or [14]:
    h = one(HAND, "hand", depth)
    g = one(GEN, "generated", depth)
    h["actions"], g["actions"] = grouped(h["actions"]), grouped(g["actions"])
    keys = ("verdict", "violated", "distinct", "generated", "depth", "left", "levels", "actions", "trace_states")
    print(json.dumps({"max_depth": depth, "agree": all(h[k] == g[k] for k in keys),
                      "differ": [k for k in keys if h[k] != g[k]]}), flush=True)
