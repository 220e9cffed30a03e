"""GPU parity tests for tlc_membership/raft.tla (SYMMETRY perms, VIEW vars,
history summary, scenario properties) through the C ABI against the CPU
oracle's committed fixtures (tests/golden/make_memb_parity.py).

Integer work, so the bar is bit-exact.  With TLC's FIFO first-found order
reproduced on the GPU (memb_backend.hip), even the order-dependent figures
match: per-action DISTINCT counts, the history counters of every kept state
(they are part of the dumped text) and the counterexample trace, state by
state.  The punctuated-search cases (CommitWhenConcurrentLeaders_unique,
MajorityOfClusterRestarts_constraint) take the reference's golden history
traces from the committed fixtures.  SYMMETRY runs in both modes, on the GPU as in the oracle:
TLC's rule (least permuted full state, then VIEW: the drop-in default, fixtures prefixed "tlc:")
and the orbit of the VIEW ("view").
"""
import hashlib
import json
import os
import tempfile

import pytest

from oracle_util import CONFIGS, GOLDEN, MEMB_MC, tla_text

pytestmark = pytest.mark.gpu

SMALL = dict(fp_table_bytes=1 << 26, state_store_bytes=1 << 29)
FIX = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))
EXHAUSTIVE = sorted(k for k, v in FIX.items() if v["verdict"] == "OK")
VIOLATIONS = sorted(k for k, v in FIX.items() if v["verdict"] == "INVARIANT_VIOLATION")
ERRORS = sorted(k for k, v in FIX.items() if v["verdict"] in ("DEADLOCK", "EVAL_ERROR"))
EXIT = {"DEADLOCK": 11, "EVAL_ERROR": 75, "INVARIANT_VIOLATION": 12}


def open_case(raftmc, g, **kw):
    """A handle for a fixture case; punctuated-search cases get their golden history trace
    (the committed TLC trace fixture) through mc_set_history_prefix; "tlc:" cases run SYMMETRY in
    TLC's mode (MC_COMPAT_SYM_TLC, the oracle's --sym tlc)."""
    kw = dict(kw, deadlock=g.get("deadlock", False))   # TLC's deadlock check as the fixture was searched
    mc = raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), sym_tlc=g.get("sym") == "tlc", **kw)
    if g.get("prefix"):
        con, fixture = g["prefix"]
        mc.set_history_prefix(con, tla_text(json.load(open(os.path.join(GOLDEN, fixture)))["value"]))
    return mc


def states_sha(mc):
    fd, path = tempfile.mkstemp(suffix=".txt")
    os.close(fd)
    mc.dump_states(path)
    lines = sorted(l.rstrip("\n") for l in open(path))
    os.unlink(path)
    return hashlib.sha256("\n".join(lines).encode()).hexdigest(), len(lines)


@pytest.mark.parametrize("case", EXHAUSTIVE)
def test_membership_parity(raftmc, case):
    g = FIX[case]
    with open_case(raftmc, g, max_depth=g["max_depth"], **SMALL) as mc:
        r = mc.run()
        sha, n = states_sha(mc)
    assert r.verdict in ("OK", "DEPTH_LIMIT"), r.error
    assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert r.actions == g["actions"]                      # generated AND distinct per action (FIFO first-found)
    assert n == g["distinct"] and sha == g["states_sha256"]


@pytest.mark.parametrize("case", VIOLATIONS)
def test_scenario_shortest_counterexample(raftmc, case):
    """Every scenario property of tlc_membership/raft.tla:1143-1278 (C4, BASELINE configs[3]) as an
    invariant: TLC's shortest counterexample state by state and TLC's counters at the stop point, in
    the orbit mode and (the "tlc:" fixtures, oracle --sym tlc) in TLC's SYMMETRY rule, the drop-in
    default -- NewlyJoinedBecomeLeader, beyond the exact oracle's reach, in
    test_counterexamples_beyond_oracle_reach."""
    g = FIX[case]
    with open_case(raftmc, g, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "INVARIANT_VIOLATION" and r.violated == g["violated"] and r.exit_code == 12, (r, r.error)
    assert (r.depth, r.generated, r.distinct, r.left_on_queue) == (g["depth"], g["generated"], g["distinct"], g["left_on_queue"])
    blocks = r.trace_text.strip().split("\n\n")
    assert len(blocks) == len(g["trace"]) == g["depth"]
    for k, (blk, ref) in enumerate(zip(blocks, g["trace"])):
        head, *body = blk.split("\n")
        assert " ".join(body) == ref["state"], "trace state %d differs" % (k + 1)
        if k:
            assert head == "State %d: <%s>" % (k + 1, ref["action"])


@pytest.mark.parametrize("case", ERRORS)
def test_error_verdicts(raftmc, case):
    """TLC's other two verdict classes, against the oracle's fixtures: "Deadlock reached" (NEXT
    NextUnreliable on its own: Init has no successor) and an evaluation error (Committed(i) ==
    SubSeq(log[i], 1, commitIndex[i]) out of range after HandleCatchupRequest empties a committed
    log, raft.tla:734-736, :969): verdict, TLC's exit code (11 / 75), the counters at the stop point
    and the trace state by state; with TLC's -deadlock (check off) the deadlock case completes."""
    g = FIX[case]
    with open_case(raftmc, g, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == g["verdict"] and r.exit_code == EXIT[g["verdict"]], (r, r.error)
    assert (r.depth, r.generated, r.distinct, r.left_on_queue) == (g["depth"], g["generated"], g["distinct"], g["left_on_queue"])
    assert r.actions == g["actions"]
    blocks = r.trace_text.strip().split("\n\n")
    assert [" ".join(b.split("\n")[1:]) for b in blocks] == [t["state"] for t in g["trace"]]
    if g["verdict"] == "EVAL_ERROR":
        assert "Committed" in r.error and "Error:" in r.report
    else:
        assert "Deadlock reached" in r.report
        with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), deadlock=False, **SMALL) as mc:
            q = mc.run()
        assert (q.verdict, q.exit_code, q.distinct) == ("OK", 0, 1)


def test_deadlock_check_changes_no_count(raftmc):
    """No state of the shipped NEXT relations lacks a successor (Restart is always
    enabled in NextAsyncCrash/NextDynamic; under NextAsync a server of its own config is a Leader
    with ClientRequest or can Timeout): TLC's default deadlock check (check_deadlock = 1) gives
    the oracle's counts exactly."""
    for case in ("membership_shipped@14", "memb_dynamic3@14", "memb_async@16"):
        g = FIX[case]
        with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), max_depth=g["max_depth"],
                                 deadlock=True, sym_tlc=g.get("sym") == "tlc", **SMALL) as mc:
            r = mc.run()
        assert r.verdict == "DEPTH_LIMIT", (case, r.error)
        assert (r.generated, r.distinct, r.actions) == (g["generated"], g["distinct"], g["actions"]), case


def test_membership_seed_independence(raftmc):
    cfg = os.path.join(CONFIGS, "memb_dynamic3.cfg")
    a = raftmc.check(MEMB_MC, cfg, max_depth=12, seed=3, **SMALL)
    b = raftmc.check(MEMB_MC, cfg, max_depth=12, seed=0xFEEDFACE, **SMALL)
    assert (a.generated, a.distinct, a.depth, a.actions) == (b.generated, b.distinct, b.depth, b.actions)


def test_membership_kat_init_expansion(raftmc):
    # SURVEY.md §4 KAT: with the shipped cfg, expanding Init gives generated 7,
    # distinct 2 (Restart successors violate CleanStartUntilFirstRequest; the
    # three Timeouts are one orbit under perms)
    r = raftmc.check(MEMB_MC, os.path.join(CONFIGS, "membership_shipped.cfg"), max_depth=2, **SMALL)
    assert (r.generated, r.distinct, r.verdict) == (7, 2, "DEPTH_LIMIT")


def test_membership_handle_rerun(raftmc):
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, "memb_two.cfg"), max_depth=14, **SMALL) as mc:
        a = mc.run()
        b = mc.run()
    assert (a.generated, a.distinct, a.actions) == (b.generated, b.distinct, b.actions)


# C3's stop point in both SYMMETRY modes (GPU-measured; the deepest oracle pins of this model are
# memb_four@16 in tests/golden/memb_parity.json and tests/golden/memb_deep.json).  Generated counts
# include TLC's copies of disjunctive guards (memb_spec.h tlc_copies; round 5: +4,637,015 / +4,628,184)
C3_STOP = {"orbit": (21, 162883559, 1118039177), "tlc": (21, 163766653, 1123528184)}


@pytest.mark.parametrize("mode", ["tlc", "orbit"])
def test_c3_counterexample_matches_committed_trace(raftmc, mode):
    """C3 (BASELINE configs[2], 4 servers, NextDynamic) to completion, in TLC's SYMMETRY rule (the
    drop-in default) and in the orbit mode: the first violation in TLC FIFO order is
    LeaderVotesQuorum at depth 21 in both; the trace equals the committed one, which the oracle
    validates (tests/test_oracle.py)."""
    r = raftmc.check(MEMB_MC, os.path.join(CONFIGS, "memb_four.cfg"), deadlock=False, sym_tlc=mode == "tlc")
    assert r.verdict == "INVARIANT_VIOLATION" and r.violated == "LeaderVotesQuorum", (r, r.error)
    assert (r.depth, r.distinct, r.generated) == C3_STOP[mode]
    got = [" ".join(b.split("\n")[1:]) for b in r.trace_text.strip().split("\n\n")]
    want = open(os.path.join(GOLDEN, "c3_leader_votes_quorum_trace.txt")).read().strip().split("\n")
    assert got == want


GPU_TRACES = json.load(open(os.path.join(GOLDEN, "gpu_traces", "index.json")))["cases"]


@pytest.mark.parametrize("cfg,mode", [(c, m) for c in sorted(GPU_TRACES)
                                      for m in ["fixture"] + (["tlc"] if "oracle_pin_tlc" in GPU_TRACES[c] else [])])
def test_counterexamples_beyond_oracle_reach(raftmc, cfg, mode):
    """Counterexamples at 3.4M-468M distinct states (tests/golden/gpu_traces/, each validated
    state by state by the oracle's check-trace, tests/test_oracle.py): TLC's single-worker FIFO
    order makes them reproducible — the same trace, depth and stop-point counters on every run.
    Among them the positive controls of the invariant kernels (VotesGrantedInv_false,
    LeaderCompleteness_false), a LogMatching violation of the dynamic-membership model and
    NewlyJoinedBecomeLeader, whose stop point the oracle's lean BFS reaches in both SYMMETRY modes
    ("oracle_pin", "oracle_pin_tlc"; its growing cluster has no SYMMETRY, so the two coincide):
    mode "tlc" runs it in TLC's rule, the drop-in default, against that pin."""
    g = GPU_TRACES[cfg]
    sym_tlc = g.get("sym") == "tlc" if mode == "fixture" else True
    r = raftmc.check(MEMB_MC, os.path.join(CONFIGS, cfg + ".cfg"), deadlock=False, sym_tlc=sym_tlc)
    assert (r.verdict, r.violated) == (g["verdict"], g["violated"]), r.error
    assert (r.depth, r.distinct, r.generated, r.left_on_queue) == (g["depth"], g["distinct"], g["generated"], g["left_on_queue"])
    if mode == "tlc":
        pin = g["oracle_pin_tlc"]
        assert (r.verdict, r.violated, r.depth, r.distinct, r.generated, r.left_on_queue) == (
            pin["verdict"], pin["violated"], pin["depth"], pin["distinct"], pin["generated"], pin["left_on_queue"])
    got = [" ".join(b.split("\n")[1:]) for b in r.trace_text.strip().split("\n\n")]
    assert got == open(os.path.join(GOLDEN, "gpu_traces", cfg + ".txt")).read().strip().split("\n")


def _memb_slot_bytes(raftmc, cfg):
    """device bytes per stored state: packed state + parent pointer"""
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, cfg + ".cfg")) as mc:
        return mc.describe()["state_bytes_stored"] + 8


def _spill_store(raftmc, g, margin=1.6):
    """a state store too small for the search but large enough for two consecutive levels"""
    sizes = g["levels"]
    cap = max(512, int(max(x + y for x, y in zip(sizes, sizes[1:])) * margin))
    assert cap < g["distinct"]
    return cap * _memb_slot_bytes(raftmc, g["cfg"])


@pytest.mark.parametrize("case", ["memb_two@16", "tlc:membership_shipped@16"])
def test_membership_checkpoint_recover(raftmc, case, tmp_path):
    """TLC -checkpoint / -recover for tlc_membership: a search stopped at depth 9 with a
    checkpoint per level, resumed by a fresh handle (seen-set rebuilt on the GPU with the
    checkpoint's seed and SYMMETRY mode), ends exactly like the oracle's uninterrupted search:
    counts, levels, per-action generated AND distinct counts (FIFO first-found), state set."""
    g = FIX[case]
    ck = str(tmp_path / "m.ckpt")
    kw = dict(SMALL)
    with open_case(raftmc, g, max_depth=9, seed=11, **kw) as mc:
        mc.set_checkpoint(ck, 1)
        a = mc.run()
    assert a.verdict == "DEPTH_LIMIT" and os.path.exists(ck), a.error
    with open_case(raftmc, g, max_depth=g["max_depth"], seed=12345, **kw) as mc:   # the checkpoint's seed wins
        mc.set_recover(ck)
        r = mc.run()
        sha, n = states_sha(mc)
    assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"]), r.error
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert r.actions == g["actions"]
    assert n == g["distinct"] and sha == g["states_sha256"]
    # a checkpoint only resumes its own model, in its own SYMMETRY mode
    other = dict(g, sym=None if g.get("sym") == "tlc" else "tlc")
    with open_case(raftmc, other, **kw) as mc:
        mc.set_recover(ck)
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.run()
    assert e.value.code == -1


@pytest.mark.parametrize("case", ["memb_two@16", "tlc:membership_shipped@16"])
def test_membership_spill_completed_levels(raftmc, case, tmp_path):
    """Host spill for tlc_membership: with a store that holds about two levels, the completed
    levels move to host memory and the search still equals the oracle's (counts, per-action
    distinct counts, the state set read across the host/device split); a checkpoint written
    after spills resumes into the same small store."""
    g = FIX[case]
    kw = dict(SMALL, state_store_bytes=_spill_store(raftmc, g, margin=1.05))   # the last two levels are ~95% of the states
    ck = str(tmp_path / "ms.ckpt")
    with open_case(raftmc, g, max_depth=g["max_depth"], **kw) as mc:
        mc.set_checkpoint(ck, g["max_depth"] - 2)
        r = mc.run()
        sha, n = states_sha(mc)
    assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"]), r.error
    assert [lv[0] for lv in r.levels] == g["levels"] and r.actions == g["actions"]
    assert n == g["distinct"] and sha == g["states_sha256"]
    with open_case(raftmc, g, max_depth=g["max_depth"], **kw) as mc:
        mc.set_recover(ck)
        c = mc.run()
        sha2, _ = states_sha(mc)
    assert (c.generated, c.distinct, c.depth, c.actions) == (r.generated, r.distinct, r.depth, r.actions), c.error
    assert sha2 == sha


@pytest.mark.parametrize("case", ["scen_BoundedTrace", "tlc:scen_FirstCommit"])
def test_membership_spill_counterexample(raftmc, case):
    """Trace reconstruction and TLC's stop-point counters across the host/device split: the
    oracle's shortest counterexample, state by state."""
    g = FIX[case]
    # the store must hold the last complete level and the new states the GPU materializes before
    # the stop (the violation is late in its level): between that and the whole search
    s = g["levels"]
    need = max(max(x + y for x, y in zip(s, s[1:])), s[-1] + g["distinct"] - sum(s))
    cap = need + (g["distinct"] - need) * 3 // 4
    with open_case(raftmc, g, **dict(SMALL, state_store_bytes=cap * _memb_slot_bytes(raftmc, g["cfg"]))) as mc:
        r = mc.run()
    assert r.verdict == "INVARIANT_VIOLATION" and r.violated == g["violated"], (r, r.error)
    assert (r.depth, r.generated, r.distinct, r.left_on_queue) == (g["depth"], g["generated"], g["distinct"], g["left_on_queue"])
    blocks = r.trace_text.strip().split("\n\n")
    assert [" ".join(b.split("\n")[1:]) for b in blocks] == [t["state"] for t in g["trace"]]


DEEP_PATH = os.path.join(GOLDEN, "memb_deep.json")
DEEP = json.load(open(DEEP_PATH)) if os.path.exists(DEEP_PATH) else {}


@pytest.mark.parametrize("case", sorted(DEEP) or ["(memb_deep.json not generated)"])
def test_c3_deep_oracle_pin(raftmc, case):
    """C3's model (memb_four: 4 servers, NextDynamic, SYMMETRY) pinned deep by the oracle's lean mode
    (tests/golden/make_memb_deep.py: millions of states, in both SYMMETRY modes): TLC's counts,
    per-level sizes and per-action generated AND distinct counts (the latter depend on TLC's
    single-worker first-found order under VIEW) at the fixture's depth."""
    if case not in DEEP:
        pytest.skip("tests/golden/memb_deep.json not generated")
    g = DEEP[case]
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), sym_tlc=g["sym"] == "tlc",
                             max_depth=g["max_depth"], deadlock=False) as mc:
        r = mc.run()
    assert r.verdict == ("DEPTH_LIMIT" if g["verdict"] == "OK" else g["verdict"]), r.error
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert (r.distinct, r.depth, r.left_on_queue) == (g["distinct"], g["depth"], g["left_on_queue"])
    assert {a: v[1] for a, v in r.actions.items()} == {a: v[1] for a, v in g["actions"].items()}   # distinct per action
    # Generated counters: compared for a pin made by the oracle that counts TLC's copies of disjunctive
    # guards ("tlc_copies") -- every pin since round 6 (the orbit-mode depth-18 pin was
    # re-made then); a pin without the flag would predate that count and keep only its distinct side.
    if g.get("tlc_copies"):
        assert r.generated == g["generated"]
        assert r.actions == g["actions"]


@pytest.mark.parametrize("mode", ["copies", "once"])
def test_disjunct_copies_switch(raftmc, mode):
    """MC_COMPAT_DISJUNCT_COPIES (the default) counts a disjunctive guard's successor once per true
    disjunct as TLC's getNextStates does (raft.tla:796, :783-789); cleared, once.  Either way the GPU
    equals the oracle's run with the same switch (tests/golden/disjunct_copies.json, NextDynamic to
    depth 16): counts, levels and per-action generated and distinct counts."""
    fx = json.load(open(os.path.join(GOLDEN, "disjunct_copies.json")))
    g = fx[mode]
    r = raftmc.check(MEMB_MC, os.path.join(CONFIGS, fx["cfg"]), max_depth=fx["max_depth"], deadlock=False,
                     disjunct_copies=mode == "copies", **SMALL)
    assert r.verdict in ("OK", "DEPTH_LIMIT"), r.error
    assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert r.actions == g["actions"]


@pytest.mark.parametrize("cap", [0, 2])
def test_fp_slice_fallback(raftmc, cap):
    """TLC-mode fingerprints come from memb_fingerprint_lds, which keeps a parent's bag in an LDS slice and
    leaves a parent whose bag could overflow it to memb_fingerprint_list (the register-bag path).  No
    shipped config fills the slice, so mc_set_fp_slice caps it: 0 sends every parent to the fallback, 2 those
    with more than two messages (a mix of both kernels in every chunk).  Counts, levels and per-action
    counts equal the oracle's NextDynamic fixture (tests/golden/disjunct_copies.json) either way."""
    fx = json.load(open(os.path.join(GOLDEN, "disjunct_copies.json")))
    g = fx["copies"]
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, fx["cfg"]), max_depth=fx["max_depth"], deadlock=False, **SMALL) as mc:
        mc.set_fp_slice(cap)
        r = mc.run()
    assert r.verdict in ("OK", "DEPTH_LIMIT"), r.error
    assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert r.actions == g["actions"]


def test_cwcl_count_claim(raftmc):
    """The reference's count claim, tlc_membership/raft.tla:1188-1191: "there are over 1.2 million traces
    of length 20 that satisfy CommitWhenConcurrentLeaders_constraint".  The shipped model with that
    constraint added (configs/cwcl_count.cfg), searched to depth 19 -- the shortest behaviour whose history
    reaches length 20 (the ConcurrentLeaders witness, :1179-1180, :1201: 18 steps) -- equals the oracle's
    search (tests/golden/cwcl_count.json: levels, generated, per-action counts), and the distinct states
    found by then, 1,252,932, are "over 1.2 million" under the reading DESIGN.md §2 states."""
    g = json.load(open(os.path.join(GOLDEN, "cwcl_count.json")))
    r = raftmc.check(MEMB_MC, os.path.join(CONFIGS, "cwcl_count.cfg"), max_depth=g["max_depth"], deadlock=False)
    assert r.verdict == "DEPTH_LIMIT", r.error
    assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert r.actions == g["actions"]
    assert 1_200_000 < r.distinct < 1_300_000
