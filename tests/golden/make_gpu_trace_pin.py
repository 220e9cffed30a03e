"""Pin a GPU counterexample fixture (tests/golden/gpu_traces/index.json) with the CPU oracle's
lean-mode BFS (test infrastructure; oracle/engine.h bfs_lean: TLC's single-worker FIFO order,
128-bit hashes of the canonical state text as the seen-set): the oracle's stop-point counters
(verdict, violated invariant, depth, distinct, generated, left on queue) are written into the
case's "oracle_pin" and must equal the GPU's.  The trace itself is validated by check-trace
(tests/test_oracle.py).  Minutes to hours on a few cores.

    python tests/golden/make_gpu_trace_pin.py CASE [--workers T] [--sym view|tlc]
"""
import fcntl
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, MEMB_MC, build_oracle  # noqa: E402

INDEX = os.path.join(GOLDEN, "gpu_traces", "index.json")
KEYS = ("verdict", "violated", "depth", "distinct", "generated", "left_on_queue")


def main():
    case = sys.argv[1]
    workers = sys.argv[sys.argv.index("--workers") + 1] if "--workers" in sys.argv else "3"
    sym = sys.argv[sys.argv.index("--sym") + 1] if "--sym" in sys.argv else "view"
    cmd = [build_oracle(), "bfs", "--tla", MEMB_MC, "--cfg", os.path.join(CONFIGS, case + ".cfg"), "--sym", sym,
           "--lean", "--workers", workers]
    r = json.loads(subprocess.run(cmd, stdout=subprocess.PIPE, text=True, check=True).stdout.strip().splitlines()[-1])
    lock = open(INDEX + ".lock", "w")
    fcntl.flock(lock, fcntl.LOCK_EX)   # the two SYMMETRY modes run side by side and finish in any order
    doc = json.load(open(INDEX))
    pin = {k: r[k] for k in KEYS}
    assert pin == {k: doc["cases"][case][k] for k in KEYS}, (pin, doc["cases"][case])
    key = "oracle_pin" if sym == "view" else "oracle_pin_" + sym   # (the test runs "tlc" against oracle_pin_tlc)
    doc["cases"][case][key] = dict(pin, sym=sym, oracle_seconds=round(r["seconds"], 1), oracle_workers=int(workers))
    json.dump(doc, open(INDEX, "w"), indent=1, sort_keys=True)
    print(case, pin)


if __name__ == "__main__":
    main()
