"""Deep tlc_membership fixtures from the CPU oracle's lean mode (test infrastructure).

C3's model (configs/memb_four.cfg: 4 servers, InitServer of 3, NextDynamic, SYMMETRY perms,
VIEW vars) searched by the oracle's restatement of tlc_membership/raft.tla
(oracle/raft_membership.h) in lean mode (oracle/engine.h bfs_lean: 128-bit hashes of the canonical
state text as the seen-set, two levels of states in memory, parents expanded by T threads and
merged in frontier order), so every count — per-action DISTINCT counts included, which depend on
TLC's single-worker FIFO first-found order under VIEW — is the single-worker one.  Both SYMMETRY
modes: "view" (orbit of the VIEW) and "tlc" (TLC's least permuted full state, then VIEW).  Lean mode
keeps no state text, so the fixture holds counts, per-level sizes and per-action counts, not the
state-set digest of tests/golden/memb_parity.json.  Hours on a few cores.

    python tests/golden/make_memb_deep.py MODE DEPTH [--workers T]     (MODE: view | tlc)
"""
import fcntl
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, MEMB_MC, ORACLE_BIN  # noqa: E402

OUT = os.path.join(GOLDEN, "memb_deep.json")


def main():
    mode, depth = sys.argv[1], int(sys.argv[2])
    workers = sys.argv[sys.argv.index("--workers") + 1] if "--workers" in sys.argv else "4"
    cmd = [ORACLE_BIN, "bfs", "--tla", MEMB_MC, "--cfg", os.path.join(CONFIGS, "memb_four.cfg"), "--sym", mode,
           "--lean", "--progress", "--workers", workers, "--max-depth", str(depth)]
    r = json.loads(subprocess.run(cmd, stdout=subprocess.PIPE, text=True, check=True).stdout.strip().splitlines()[-1])
    assert r["verdict"] in ("OK", "INVARIANT_VIOLATION"), r
    case = "%smemb_four@%d" % ("tlc:" if mode == "tlc" else "", depth)
    lock = open(OUT + ".lock", "w")
    fcntl.flock(lock, fcntl.LOCK_EX)   # the two modes run side by side and finish in any order
    doc = json.load(open(OUT)) if os.path.exists(OUT) else {}
    doc[case] = {k: r[k] for k in ("verdict", "violated", "generated", "distinct", "depth", "left_on_queue", "levels", "actions")}
    doc[case].update(cfg="memb_four", sym=mode, max_depth=depth, oracle_seconds=round(r["seconds"], 1), tlc_copies=True,
                     oracle_workers=int(workers),
                     source="oracle/engine.h bfs_lean on configs/memb_four.cfg (tests/golden/make_memb_deep.py)")
    json.dump(doc, open(OUT, "w"), indent=1, sort_keys=True)
    print(case, json.dumps({k: doc[case][k] for k in ("generated", "distinct", "depth", "oracle_seconds")}), flush=True)


if __name__ == "__main__":
    main()
