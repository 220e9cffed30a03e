"""Generate raft_original parity fixtures with the CPU oracle (test infrastructure).

For every configs/<name>.cfg given (default: the fast parity set) the oracle
(oracle/, a literal restatement of thirdparty/raft_original.tla with TLC BFS
semantics) runs the full BFS and the fixture records generated / distinct /
depth / per-level sizes / per-action (generated, distinct) and the SHA-256 of
the sorted canonical text of every distinct state.  TLC itself is unavailable
offline, so these counts are oracle-pinned, not TLC-pinned.

    python tests/golden/make_orig_parity.py [name ...]
"""
import hashlib
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, ORIG_MC, run_oracle  # noqa: E402

FAST = ["c1", "parity_single", "parity_pair", "parity_pair_neg", "parity_trio", "parity_pair6"]
OUT = os.path.join(GOLDEN, "orig_parity.json")


def digest_lines(path):
    lines = sorted(l.rstrip("\n") for l in open(path))
    return hashlib.sha256("\n".join(lines).encode()).hexdigest(), len(lines)


def main(names):
    doc = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for n in names:
        fd, dump = tempfile.mkstemp(suffix=".txt")
        os.close(fd)
        r = run_oracle("bfs", ORIG_MC, os.path.join(CONFIGS, n + ".cfg"), "--dump", dump, timeout=100000)
        assert r["verdict"] == "OK", r
        sha, cnt = digest_lines(dump)
        assert cnt == r["distinct"]
        os.unlink(dump)
        doc[n] = {"generated": r["generated"], "distinct": r["distinct"], "depth": r["depth"],
                  "levels": r["levels"], "actions": r["actions"], "states_sha256": sha,
                  "oracle_seconds": round(r["seconds"], 2)}
        print(n, doc[n]["distinct"], doc[n]["oracle_seconds"], "s", flush=True)
        json.dump(doc, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or FAST)
