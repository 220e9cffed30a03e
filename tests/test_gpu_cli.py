"""The raftmc command line on the GPU: TLC's summary lines and exit codes, the
hand-compiled path and the generated path (-frontend), as a TLC user would call it."""
import json
import os
import subprocess

import pytest

from oracle_util import CONFIGS, GOLDEN, ORIG_MC

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "raft-tla_amd", "_build", "raftmc")
SMALL = ["-fptable", str(1 << 26), "-store", str(1 << 30)]


def run(*args):
    if not os.path.exists(CLI):
        pytest.skip("raftmc CLI not built")
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("frontend", ["auto", "generated"])
def test_cli_c1_summary(frontend):
    """C1 through the CLI: TLC's final lines with the oracle's counts, exit code 0, both paths
    (the generated one parses thirdparty/raft_original.tla: skipped where the reference is absent)."""
    g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))["c1"]
    spec = ORIG_MC
    if frontend == "generated":
        spec = os.path.join(ROOT, "raft-tla_amd", "_build", "tlagen_co", "c1.gen.hip")
        if not os.path.exists(spec):
            pytest.skip("prebuilt c1.gen.hip absent")
    r = run("-frontend", frontend, "-workers", "0", "-config", os.path.join(CONFIGS, "c1.cfg"), *SMALL, spec)
    assert r.returncode == 0, r.stderr
    assert "%d states generated, %d distinct states found, 0 states left on queue." % (g["generated"], g["distinct"]) in r.stdout
    assert "The depth of the complete state graph search is %d." % g["depth"] in r.stdout


def test_cli_generated_violation_exit_code():
    """The repo's TokenRing.tla (auto: not a hand-compiled module) with a reachable violation: TLC's
    error line, a trace and exit code 12."""
    r = run("-workers", "0", "-config", os.path.join(CONFIGS, "tlagen", "TokenRing_full.cfg"), *SMALL,
            os.path.join(CONFIGS, "tlagen", "TokenRing.tla"))
    assert r.returncode == 12, r.stderr
    assert "Error: Invariant NotAllFull is violated." in r.stdout
    assert r.stdout.count("State ") >= 9


def test_cli_hand_refuses_unknown_module():
    r = run("-frontend", "hand", "-config", os.path.join(CONFIGS, "tlagen", "TokenRing.cfg"), os.path.join(CONFIGS, "tlagen", "TokenRing.tla"))
    assert r.returncode == 75 and "unrecognised spec module" in r.stderr
