"""Ricketts' raft (thirdparty/raft_dricketts.tla) fixtures from the CPU oracle's restatement
(oracle/raft_dricketts.h; test infrastructure).

The reference ships no TLC cfg for this TLAPS-proved spec; configs/ricketts_mc.tla bounds it and the
cfgs below choose the invariants.  For each case the oracle's single-worker FIFO search (TLC's
contract, oracle/engine.h) records the verdict, TLC's counters (at the stop point for a violation or
an evaluation error), level sizes and per-action (generated, distinct) counts; the generated path
must reproduce them on the host build of its generated code (tests/test_tlagen.py) and on the GPU
(tests/test_gpu_tlagen.py).

    python tests/golden/make_ricketts_oracle.py [name ...]

ricketts_safety (the whole space of 3 servers, term <= 2, log <= 1, one message in flight:
1,542,177 states, depth 49) takes about 4 minutes on 6 threads.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, run_oracle  # noqa: E402

MC = os.path.join(CONFIGS, "ricketts_mc.tla")
# name -> (cfg, extra oracle arguments)
CASES = {
    "c1_d12": ("ricketts_c1", ["--max-depth", "12"]),                 # LogMatching holds to depth 12
    "noleader": ("ricketts_noleader", ["--trace"]),                   # NoLeader violated (a leader is elected)
    "election_safety": ("ricketts_election_safety", ["--trace"]),     # Max({}) in ElectionSafety: EVAL_ERROR
    "safety": ("ricketts_safety", ["--workers", "6"]),               # LogMatching, LeaderVotesQuorum, CandidateTermNotInLog hold
}
OUT = os.path.join(GOLDEN, "ricketts_oracle.json")


def main(names):
    doc = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for n in names:
        cfg, extra = CASES[n]
        r = run_oracle("bfs", MC, os.path.join(CONFIGS, cfg + ".cfg"), *extra, timeout=100000)
        keep = ["verdict", "violated", "error", "generated", "distinct", "left_on_queue", "depth", "levels", "actions"]
        if "--trace" in extra:
            keep.append("trace")
        doc[n] = {k: r[k] for k in keep}
        doc[n]["cfg"] = cfg
        doc[n]["max_depth"] = int(extra[1]) if extra[:1] == ["--max-depth"] else 0
        doc[n]["oracle_seconds"] = round(r["seconds"], 2)
        print(n, r["verdict"], r["violated"], r["error"], r["distinct"], r["depth"], flush=True)
        json.dump(doc, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or list(CASES))
