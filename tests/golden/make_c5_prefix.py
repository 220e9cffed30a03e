"""Depth-limited C5 fixture (BASELINE.json configs[4]: raft_original, 5 servers,
term <= 3, log <= 3; configs/c5.cfg) from the CPU oracle (test infrastructure).

The full C5 state space is far beyond the oracle (and one GPU), so the fixture
pins the first levels: the oracle's BFS stopped at --max-depth D (TLC's depth
counting, Init = depth 1) records generated / distinct / left-on-queue /
per-level sizes / per-action (generated, distinct) and the SHA-256 of the
sorted canonical text of every distinct state found.  Oracle-pinned, not
TLC-pinned.

    python tests/golden/make_c5_prefix.py [max_depth] [cfg]

`cfg` c5v2.cfg (two values, compact election records) writes tests/golden/c5v2_prefix.json;
c2_md6.cfg (C2 with 6 messages: AppendEntries responses and commits fire) tests/golden/c2_md6_prefix.json.
"""
import hashlib
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, ORIG_MC, run_oracle  # noqa: E402

def main(depth, cfg="c5.cfg"):
    fd, dump = tempfile.mkstemp(suffix=".txt")
    os.close(fd)
    workers = os.environ.get("ORACLE_WORKERS", "1")
    r = run_oracle("bfs", ORIG_MC, os.path.join(CONFIGS, cfg), "--max-depth", str(depth), "--dump", dump,
                   "--workers", workers, timeout=100000)
    lines = sorted(l.rstrip("\n") for l in open(dump))
    os.unlink(dump)
    assert len(lines) == r["distinct"], (len(lines), r["distinct"])
    doc = {"cfg": cfg, "max_depth": depth, "generated": r["generated"], "distinct": r["distinct"],
           "depth": r["depth"], "left_on_queue": r["left_on_queue"], "levels": r["levels"], "actions": r["actions"],
           "states_sha256": hashlib.sha256("\n".join(lines).encode()).hexdigest(),
           "oracle_seconds": round(r["seconds"], 2)}
    out = os.path.join(GOLDEN, cfg.replace(".cfg", "") + "_prefix.json")
    json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(doc)[:300])


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 7, sys.argv[2] if len(sys.argv) > 2 else "c5.cfg")
