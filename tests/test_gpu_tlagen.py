"""The generated path on the GPU: the front end's C++ compiled for
gfx950 (tlagen_kernels.h), run through the C ABI with mc_opts.frontend.

The reference's raft_original.tla is not on the GPU box, so its generated sources are made by
the build in the container (raft-tla_amd/csrc/tlagen/prebuild.py: _build/tlagen_co/<cfg>.gen.hip
plus their code objects) and opened as .gen.hip files; the repo's own TokenRing.tla goes through
the whole front end on the box (parse, generate, code object by source hash).  Counts are order
independent, so they must equal the oracle's exactly (tests/golden/orig_parity.json, the full-size
C2 pin) and the Python model's for TokenRing."""
import json
import os

import pytest

from oracle_util import CONFIGS, GOLDEN
from tlagen_models import token_ring

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "raft-tla_amd", "_build", "tlagen_co")
RING = os.path.join(CONFIGS, "tlagen", "TokenRing.tla")
SMALL = dict(fp_table_bytes=1 << 26, state_store_bytes=1 << 30)


def gen_source(name):
    p = os.path.join(GEN, name + ".gen.hip")
    if not os.path.exists(p):
        pytest.skip(p + " not built (raft-tla_amd/csrc/tlagen/prebuild.py)")
    return p


@pytest.mark.parametrize("name", ["c1", "parity_single", "parity_pair", "parity_trio"])
def test_generated_raft_original_parity(raftmc, name):
    g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))[name]
    with raftmc.ModelChecker(gen_source(name), os.path.join(CONFIGS, name + ".cfg"), frontend="generated", workers=0, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth) == (g["generated"], g["distinct"], g["depth"])
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert r.actions == {"Next": [g["generated"] - 1, g["distinct"] - 1]}


def test_generated_c2_full_size(raftmc):
    """BASELINE configs[1] through the generated path: the oracle's full-size C2 counts."""
    o = json.load(open(os.path.join(GOLDEN, "c2_oracle.json")))
    with raftmc.ModelChecker(gen_source("c2"), os.path.join(CONFIGS, "c2.cfg"), frontend="generated", workers=0,
                             fp_table_bytes=1 << 30, state_store_bytes=200 << 30) as mc:
        r = mc.run()
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth) == (o["generated"], o["distinct"], o["depth"])
    assert [lv[0] for lv in r.levels] == o["levels"]
    print("generated path C2: %.3f s (kernels %.3f s)" % (r.seconds, r.kernel_seconds))


def test_generated_violation_depth(raftmc):
    """NoLeader on C2's constants: the violation lies at depth 10 (tests/golden/orig_events.json);
    the trace ends in a state with a leader."""
    g = json.load(open(os.path.join(GOLDEN, "orig_events.json")))["c2_noleader"]
    with raftmc.ModelChecker(gen_source("c2_noleader"), os.path.join(CONFIGS, "c2_noleader.cfg"), frontend="generated",
                             workers=0, fp_table_bytes=1 << 28, state_store_bytes=16 << 30) as mc:
        r = mc.run()
    assert (r.verdict, r.violated, r.depth) == ("INVARIANT_VIOLATION", "NoLeader", g["depth"])
    assert r.trace_text.count("/\\ state = ") == g["depth"]
    assert "Leader" in r.trace_text.split("/\\ state = ")[-1].splitlines()[0]


def test_token_ring_front_end_on_gpu(raftmc):
    """The repo's TokenRing.tla through the whole front end on the box (auto: not a hand-compiled
    family): counts and per-action generated counts of the Python model (per-action distinct
    counts depend on which producer reaches a state first: first-come here, as with TLC -workers N)."""
    want = token_ring()
    with raftmc.ModelChecker(RING, os.path.join(CONFIGS, "tlagen", "TokenRing.cfg"), workers=0, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth) == (want["generated"], want["distinct"], want["depth"])
    assert [lv[0] for lv in r.levels] == want["levels"]
    for a, v in want["actions"].items():
        assert r.actions[a][0] == v[0], a
    assert sum(v[1] for v in r.actions.values()) == want["distinct"] - 1


def test_token_ring_violation_trace(raftmc):
    want = token_ring(stop_when_all_full=True)
    with raftmc.ModelChecker(RING, os.path.join(CONFIGS, "tlagen", "TokenRing_full.cfg"), workers=0, **SMALL) as mc:
        r = mc.run()
    assert (r.verdict, r.violated, r.depth) == ("INVARIANT_VIOLATION", "NotAllFull", want["depth"])
    last = r.trace_text.split("/\\ logs = ")[-1].splitlines()[0]
    assert last.count("val |->") == 6, last


@pytest.mark.parametrize("cfg,verdict,depth,code", [("Countdown", "DEADLOCK", 4, 11), ("Countdown_evalerr", "EVAL_ERROR", 3, 75)])
def test_generated_deadlock_and_eval_error(raftmc, cfg, verdict, depth, code):
    """TLC's deadlock and evaluation-error reports from the generated kernels: verdict, TLC's exit
    code, and the trace to the state whose successors could not be computed (or did not exist)."""
    with raftmc.ModelChecker(os.path.join(CONFIGS, "tlagen", "Countdown.tla"), os.path.join(CONFIGS, "tlagen", cfg + ".cfg"),
                             workers=0, **SMALL) as mc:
        r = mc.run()
    assert (r.verdict, r.depth, r.distinct, r.exit_code) == (verdict, depth, depth, code)
    assert r.trace_text.count("/\\ x = ") == depth
    assert "/\\ x = %d" % (0 if verdict == "DEADLOCK" else 1) in r.trace_text.split("State %d:" % depth)[1]


def test_ricketts_on_gpu(raftmc):
    """thirdparty/raft_dricketts.tla (Bags module, TLAPS-only in the reference) through the generated
    path to depth 12: the host build's counts (tests/test_tlagen.py, parity unpinned), and NoLeader's
    depth."""
    from test_tlagen import RICKETTS_D12
    with raftmc.ModelChecker(gen_source("ricketts_c1"), os.path.join(CONFIGS, "ricketts_c1.cfg"), frontend="generated",
                             workers=0, max_depth=12, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "DEPTH_LIMIT", r.error
    assert (r.generated, r.distinct, [lv[0] for lv in r.levels]) == (RICKETTS_D12["generated"], RICKETTS_D12["distinct"], RICKETTS_D12["levels"])
    with raftmc.ModelChecker(gen_source("ricketts_noleader"), os.path.join(CONFIGS, "ricketts_noleader.cfg"), frontend="generated",
                             workers=0, **SMALL) as mc:
        r = mc.run()
    assert (r.verdict, r.violated, r.depth) == ("INVARIANT_VIOLATION", "NoLeader", 10)
