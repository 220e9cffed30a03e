"""apalache_no_membership/raft.tla fixtures from the CPU oracle's restatement (oracle/raft_apalache.h;
test infrastructure).

The reference's Apalache-annotated spec with its own shipped raft.cfg (TLC syntax; configs/apalache_nm.cfg
is the same file for the GPU box, which has no reference checkout).  Its history["global"] grows with
every Send/Receive and is part of the state (no VIEW), so the state space has no bound: the shipped
model is pinned depth-bounded, and the cfg's two commented-out test-case invariants (raft.cfg:22-24,
raft.tla:776-785) give counterexamples.  For each case the oracle's single-worker FIFO search (TLC's
contract, oracle/engine.h) records the verdict, TLC's counters (at the stop point for a violation),
level sizes, per-action (generated, distinct) counts under the generated path's action names, the
SHA-256 of the sorted text of every kept state, and the counterexample.  The generated path must
reproduce them on the host build of its code (tests/test_tlagen.py) and on the GPU
(tests/test_gpu_tlagen.py).

    python tests/golden/make_apalache_oracle.py [--workers T] [name ...]
"""
import hashlib
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, run_oracle  # noqa: E402

REF = os.environ.get("RAFTMC_REFERENCE", "/root/reference")
SPEC = os.path.join(REF, "apalache_no_membership", "raft.tla")
# name -> (cfg, max depth)
CASES = {
    "shipped_d11": ("apalache_nm", 11),                     # the shipped model, 8 invariants holding
    "BoundedTrace": ("apalache_nm_boundedtrace", 0),        # Len(history["global"]) <= 12 (raft.tla:776)
    "FirstBecomeLeader": ("apalache_nm_firstbecomeleader", 0),   # raft.tla:778-785
}
OUT = os.path.join(GOLDEN, "apalache_oracle.json")


def main(names, workers="1"):
    doc = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for n in names:
        cfg, depth = CASES[n]
        fd, dump = tempfile.mkstemp(suffix=".txt")
        os.close(fd)
        args = ["--dump", dump, "--trace", "--workers", workers] + (["--max-depth", depth] if depth else [])
        r = run_oracle("bfs", SPEC, os.path.join(CONFIGS, cfg + ".cfg"), *args, timeout=100000)
        assert r["verdict"] in ("OK", "INVARIANT_VIOLATION", "EVAL_ERROR"), r
        lines = sorted(l.rstrip("\n") for l in open(dump))
        os.unlink(dump)
        doc[n] = {k: r[k] for k in ("verdict", "violated", "error", "generated", "distinct", "left_on_queue", "depth",
                                     "levels", "actions", "trace")}
        doc[n].update(cfg=cfg, max_depth=depth, states_sha256=hashlib.sha256("\n".join(lines).encode()).hexdigest(),
                      states_dumped=len(lines), oracle_seconds=round(r["seconds"], 2))
        print(n, r["verdict"], r["violated"], r["distinct"], r["depth"], doc[n]["oracle_seconds"], "s", flush=True)
        json.dump(doc, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    argv = sys.argv[1:]
    w = "1"
    if "--workers" in argv:
        i = argv.index("--workers")
        w = argv[i + 1]
        del argv[i:i + 2]
    main(argv or list(CASES), w)
