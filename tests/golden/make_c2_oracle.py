"""Full-size C2 fixture from the CPU oracle (test infrastructure).

BASELINE.json's headline workload (configs/c2.cfg: 54M distinct states) run to completion by the
oracle's restatement of raft_original.tla (oracle/raft_original.h), in its lean mode
(oracle/engine.h bfs_lean: 128-bit hashes of the canonical state text as the seen-set, two levels
of states in memory, parents expanded by T threads and merged in frontier order so the counts —
per-action distinct ones included — are the single-worker FIFO ones).  This replaces the
self-comparison of tests/golden/c2_exact.json (the product's packed relation on the host) as the
pin of tests/test_gpu.py's full-size C2 test.  About two hours on 7 cores.

    python tests/golden/make_c2_oracle.py [--workers T]
"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, ORIG_MC  # noqa: E402

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(GOLDEN))), "oracle", "_build", "raft_oracle")
OUT = os.path.join(GOLDEN, "c2_oracle.json")


def main():
    workers = sys.argv[sys.argv.index("--workers") + 1] if "--workers" in sys.argv else "7"
    cmd = [ORACLE, "bfs", "--tla", ORIG_MC, "--cfg", os.path.join(CONFIGS, "c2.cfg"), "--lean", "--progress",
           "--workers", workers]
    r = json.loads(subprocess.run(cmd, stdout=subprocess.PIPE, text=True, check=True).stdout.strip().splitlines()[-1])
    assert r["verdict"] == "OK", r
    doc = {k: r[k] for k in ("verdict", "generated", "distinct", "depth", "levels", "actions")}
    doc["oracle_seconds"] = round(r["seconds"], 1)
    doc["oracle_workers"] = int(workers)
    doc["source"] = "oracle/engine.h bfs_lean on configs/c2.cfg (tests/golden/make_c2_oracle.py)"
    json.dump(doc, open(OUT, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: doc[k] for k in ("generated", "distinct", "depth", "oracle_seconds")}))


if __name__ == "__main__":
    main()
