"""Counterexample fixtures for raft_original with the CPU oracle (test infrastructure).

TLC stops at the FIRST violating successor in its single-worker FIFO order (parents in level
order, each parent's successors in the order of the Next disjuncts and of `\\E m \\in DOMAIN
messages`, raft_original.tla:453-462).  For every config below the oracle (oracle/engine.h bfs,
TLC's contract as named [ext] switches) records the verdict, the violated invariant, TLC's
counters at the stop point (generated = whole successor lists up to the violating parent;
distinct, per-action counts and left-on-queue at the violating successor), the completed level
sizes and the counterexample state by state.  The GPU must reproduce all of it exactly
(tests/test_gpu.py).  TLC itself is unavailable offline: oracle-pinned.

    python tests/golden/make_orig_events.py [name ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, ORIG_MC, run_oracle  # noqa: E402

# scenario_first_leader: NoLeader, 2 servers; c2_noleader: NoLeader on the C2 shape (3 servers,
# request-vote traffic only); pair6_nocommit: NoCommit after a full replication round trip
# (every message type in flight)
EVENTS = ["scenario_first_leader", "c2_noleader", "pair6_nocommit"]
OUT = os.path.join(GOLDEN, "orig_events.json")


def main(names):
    doc = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for n in names:
        r = run_oracle("bfs", ORIG_MC, os.path.join(CONFIGS, n + ".cfg"), "--trace", timeout=100000)
        assert r["verdict"] != "OK", r
        doc[n] = {k: r[k] for k in ("verdict", "violated", "generated", "distinct", "left_on_queue", "depth",
                                    "levels", "actions", "trace")}
        doc[n]["oracle_seconds"] = round(r["seconds"], 2)
        print(n, r["verdict"], r["violated"], r["distinct"], len(r["trace"]), flush=True)
        json.dump(doc, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or EVENTS)
