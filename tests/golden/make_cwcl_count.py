"""Fixture for the reference's one count-like claim (test infrastructure).

tlc_membership/raft.tla:1188-1191: "there are over 1.2 million traces of length 20 that satisfy
CommitWhenConcurrentLeaders_constraint".  The oracle (lean mode, TLC's symmetry rule, single-worker
FIFO merge) searches the shipped model with that constraint added (configs/cwcl_count.cfg) to depth 19
-- the depth of the shortest behaviour whose history reaches length 20 (the ConcurrentLeaders witness,
raft.tla:1179-1180, :1201: 18 steps) -- and the fixture keeps its counts; tests/test_gpu_membership.py
test_cwcl_count_claim checks the GPU against them and the claim against the reading of DESIGN.md §2.
About 6 minutes on 5 cores.

    python tests/golden/make_cwcl_count.py
"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, MEMB_MC  # noqa: E402

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(GOLDEN))), "oracle", "_build", "raft_oracle")
OUT = os.path.join(GOLDEN, "cwcl_count.json")
DEPTH = 19


def main():
    cmd = [ORACLE, "bfs", "--tla", MEMB_MC, "--cfg", os.path.join(CONFIGS, "cwcl_count.cfg"), "--max-depth", str(DEPTH),
           "--workers", "5", "--lean"]
    r = json.loads(subprocess.run(cmd, stdout=subprocess.PIPE, text=True, check=True).stdout.strip().splitlines()[-1])
    doc = {k: r[k] for k in ("verdict", "generated", "distinct", "depth", "levels", "actions", "left_on_queue")}
    doc["max_depth"] = DEPTH
    doc["oracle_seconds"] = round(r["seconds"], 1)
    doc["source"] = "oracle bfs --lean (TLC's symmetry rule) on configs/cwcl_count.cfg to depth %d (tests/golden/make_cwcl_count.py)" % DEPTH
    json.dump(doc, open(OUT, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: doc[k] for k in ("generated", "distinct", "depth")}))


if __name__ == "__main__":
    main()
