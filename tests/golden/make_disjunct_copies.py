"""Fixture for TLC's disjunct copies as a named switch (test infrastructure).

oracle/engine.h Options::disjunct_copies ([ext] switch (vi), CLI --no-disjunct-copies): TLC's
getNextStates enumerates each true disjunct of a disjunctive guard inside an action as a branch of its
own, so the one successor that HandleCheckOldConfig's `state[i] /= Leader \\/ m.mterm = currentTerm[i]`
(tlc_membership/raft.tla:796) or HandleCatchupResponse's five-way discard list (:783-789) admits is
generated once per true disjunct.  The oracle runs configs/memb_dynamic3.cfg (NextDynamic: both
handlers fire) to depth 16 both ways; the GPU must reproduce each (tests/test_gpu_membership.py
test_disjunct_copies_switch) and the two must differ only in the generated counters of those two
actions (tests/test_oracle.py test_disjunct_copies_switch_oracle).

    python tests/golden/make_disjunct_copies.py
"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, MEMB_MC  # noqa: E402

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(GOLDEN))), "oracle", "_build", "raft_oracle")
OUT = os.path.join(GOLDEN, "disjunct_copies.json")
CFG, DEPTH = "memb_dynamic3.cfg", 16


def run(*extra):
    cmd = [ORACLE, "bfs", "--tla", MEMB_MC, "--cfg", os.path.join(CONFIGS, CFG), "--max-depth", str(DEPTH),
           "--workers", "4", *extra]
    r = json.loads(subprocess.run(cmd, stdout=subprocess.PIPE, text=True, check=True).stdout.strip().splitlines()[-1])
    return {k: r[k] for k in ("verdict", "generated", "distinct", "depth", "levels", "actions", "left_on_queue")}


def main():
    doc = {"cfg": CFG, "max_depth": DEPTH, "copies": run(), "once": run("--no-disjunct-copies"),
           "source": "oracle bfs (TLC's symmetry rule) on configs/%s, --max-depth %d, with and without "
                     "--no-disjunct-copies (tests/golden/make_disjunct_copies.py)" % (CFG, DEPTH)}
    json.dump(doc, open(OUT, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: (doc[k]["generated"], doc[k]["distinct"]) for k in ("copies", "once")}))


if __name__ == "__main__":
    main()
