"""Exact C2 state-space size for tests/golden/c2_exact.json (test infrastructure).

Builds tests/native/orig_host_bfs.cpp (the product's packed raft_original successor
relation run by a host BFS whose seen-set holds the FULL packed states, so no
fingerprint collision can merge two states) for the C2 shape and runs it on
configs/c2.cfg.  About 8 minutes and 8 GB of RAM on one core.

    python tests/golden/make_c2_exact.py
"""
import json
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    exe = os.path.join(tempfile.gettempdir(), "orig_host_bfs_c2_exact")
    csrc = os.path.join(ROOT, "raft-tla_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-DSHAPE_N=3", "-DSHAPE_NV=2", "-DSHAPE_MT=3", "-DSHAPE_ML=2", "-DSHAPE_MK=5",
                    "-o", exe, os.path.join(ROOT, "tests", "native", "orig_host_bfs.cpp"), os.path.join(csrc, "model.cpp"),
                    os.path.join(csrc, "orig_model.cpp")], check=True)
    r = json.loads(subprocess.run([exe, os.path.join(ROOT, "configs", "c2.cfg")], capture_output=True, text=True,
                                  check=True).stdout)
    doc = {"source": "tests/native/orig_host_bfs.cpp (test harness: the product's packed raft_original successor relation, "
                     "seen-set keyed on the full packed state, no fingerprints) on configs/c2.cfg; ~8 min on one core",
           "cfg": "c2", "generated": r["generated"], "distinct": r["distinct"], "depth": r["depth"],
           "actions_generated": {k: v[0] for k, v in r["actions"].items()},
           "actions_distinct_parent_major_fifo": {k: v[1] for k, v in r["actions"].items()}}
    json.dump(doc, open(os.path.join(ROOT, "tests", "golden", "c2_exact.json"), "w"), indent=1, sort_keys=True)
    print(doc["distinct"], doc["generated"], doc["depth"])


if __name__ == "__main__":
    main()
