"""CPU oracle pinned against the reference's own TLC output and derived KATs.

The reference has no tests; its only machine-generated results are the two
TLC traces pasted into tlc_membership/raft.tla:1201 and :1231 (fixtures in
tests/golden/, made by tests/golden/make_golden.py).  Counts of state spaces
are unpinned against TLC (not runnable offline).
"""
import json
import os

import pytest

from oracle_util import CONFIGS, GOLDEN, MEMB_MC, ORIG_MC, golden_file, run_oracle


def test_init_expansion_kat_original():
    # SURVEY.md §4 KAT: from Init only Restart x3 and Timeout x3 are enabled;
    # the three Restarts yield one state (only allLogs changes), so after
    # expanding Init generated = 1 + 6 = 7 and distinct = 1 + 1 + 3 = 5.
    r = run_oracle("bfs", ORIG_MC, os.path.join(CONFIGS, "c1.cfg"), "--max-depth", 2)
    assert (r["generated"], r["distinct"]) == (7, 5)
    assert r["actions"]["Restart"] == [3, 1] and r["actions"]["Timeout"] == [3, 3]


def test_init_expansion_kat_membership():
    # tlc_membership, shipped cfg: Restart successors of Init violate
    # CleanStartUntilFirstRequest; the 3 Timeout successors are one orbit
    # under SYMMETRY perms  =>  generated 7, distinct 2.
    r = run_oracle("bfs", MEMB_MC, os.path.join(CONFIGS, "membership_shipped.cfg"), "--max-depth", 2)
    assert (r["generated"], r["distinct"]) == (7, 2)


def test_concurrent_leaders_trace_replays():
    # raft.tla:1201: TLC's ConcurrentLeaders witness, history["global"] of length 20
    path, doc = golden_file("concurrent_leaders_trace.json")
    r = run_oracle("replay", MEMB_MC, os.path.join(CONFIGS, "membership_shipped.cfg"), "--golden", path)
    assert r["found"] and r["golden_len"] == 20
    # shortest behaviour producing it: 18 transitions (TLC's "State 19"), raft.tla:1179-1180
    assert r["transitions"] == 18
    st = r["state"]
    assert "hadNumLeaders |-> 2" in st and "hadNumClientRequests |-> 0" in st
    assert "s1 :> [restarted |-> 0, timeout |-> 1] @@ s2 :> [restarted |-> 0, timeout |-> 1] @@ s3 :> [restarted |-> 0, timeout |-> 0]" in st


def test_commit_when_concurrent_leaders_trace_replays():
    # raft.tla:1231: TLC's CommitWhenConcurrentLeaders witness, 28 history entries,
    # with two ClientRequests (they add no history entry, G4) and an UpdateTerm.
    path, doc = golden_file("commit_when_concurrent_leaders_trace.json")
    r = run_oracle("replay", MEMB_MC, os.path.join(CONFIGS, "membership_shipped.cfg"), "--golden", path)
    assert r["found"] and r["golden_len"] == 28
    assert r["transitions"] == 27
    assert r["actions"].count("ClientRequest") == 2
    assert "hadNumClientRequests |-> 2" in r["state"]


def test_original_parity_fixtures_reproduce():
    doc = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))
    for name in ("c1", "parity_single", "parity_pair"):
        r = run_oracle("bfs", ORIG_MC, os.path.join(CONFIGS, name + ".cfg"))
        g = doc[name]
        assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"]), name
        assert r["actions"] == g["actions"], name


def test_first_leader_shortest_witness():
    # NoLeader (test-only scenario invariant) on 2 servers: Timeout, RequestVote x2,
    # HandleRequestVoteRequest (self), UpdateTerm (peer), HandleRequestVoteRequest (peer),
    # HandleRequestVoteResponse x2, BecomeLeader = 9 steps, 10 states
    r = run_oracle("bfs", ORIG_MC, os.path.join(CONFIGS, "scenario_first_leader.cfg"), "--trace")
    assert r["verdict"] == "INVARIANT_VIOLATION" and r["violated"] == "NoLeader"
    assert r["trace_len"] == 10
    assert r["trace"][-1]["action"] == "BecomeLeader"


def test_oracle_validates_gpu_c3_counterexample():
    """BASELINE configs[2] (C3, 4 servers, NextDynamic): the GPU found a
    LeaderVotesQuorum violation at depth 21 (162.9M distinct states, beyond the
    oracle's reach).  The oracle replays the committed trace step by step through
    its own Next relation, constraints and invariants (check-trace mode)."""
    from oracle_util import MEMB_MC, run_oracle
    r = run_oracle("check-trace", MEMB_MC, os.path.join(CONFIGS, "memb_four.cfg"), "--golden",
                   os.path.join(GOLDEN, "c3_leader_votes_quorum_trace.txt"))
    assert r["valid"] and r["length"] == 21 and r["violated"] == "LeaderVotesQuorum"
    assert r["actions"].split(",")[-2:] == ["AddNewServer", "UpdateTerm"]


def test_oracle_check_trace_rejects_a_broken_trace(tmp_path):
    from oracle_util import MEMB_MC, run_oracle
    lines = open(os.path.join(GOLDEN, "c3_leader_votes_quorum_trace.txt")).read().strip().split("\n")
    lines[7] = lines[6]
    p = tmp_path / "broken.txt"
    p.write_text("\n".join(lines) + "\n")
    r = run_oracle("check-trace", MEMB_MC, os.path.join(CONFIGS, "memb_four.cfg"), "--golden", str(p))
    assert not r["valid"] and r["bad_step"] == 7


def test_punctuated_search_prefix_fixture_reproduces():
    """MajorityOfClusterRestarts_constraint (raft.tla:1228-1234) with the 28-entry TLC trace of
    :1231 as its golden prefix: the oracle's bounded search reproduces the committed fixture
    (the GPU and the packed host harness are checked against the same fixture)."""
    g = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))["punct_MajorityOfClusterRestarts@30"]
    path, _ = golden_file("commit_when_concurrent_leaders_trace.json")
    r = run_oracle("bfs", MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), "--sym", "view", "--golden-morc", path,
                   "--max-depth", g["max_depth"])
    assert (r["generated"], r["distinct"], r["depth"], r["left_on_queue"]) == \
        (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
    assert r["actions"] == g["actions"]


@pytest.mark.parametrize("tla,cfg,extra", [
    ("orig", "c1.cfg", ()), ("orig", "scenario_first_leader.cfg", ("--trace",)),
    ("memb", "memb_two.cfg", ("--max-depth", "11", "--trace")),
])
def test_oracle_parallel_expansion_is_identical(tla, cfg, extra):
    """--workers N (the bench's CPU baseline) expands a batch of parents on N threads and merges
    in frontier order: the result (counts, per-action counts, levels, traces) equals 1 thread."""
    from oracle_util import MEMB_MC, ORIG_MC, run_oracle
    spec = ORIG_MC if tla == "orig" else MEMB_MC
    a = run_oracle("bfs", spec, os.path.join(CONFIGS, cfg), *extra)
    b = run_oracle("bfs", spec, os.path.join(CONFIGS, cfg), *extra, "--workers", "4")
    a.pop("seconds"), b.pop("seconds")
    assert a == b


GPU_TRACES = json.load(open(os.path.join(GOLDEN, "gpu_traces", "index.json")))["cases"]


@pytest.mark.parametrize("cfg", sorted(GPU_TRACES))
def test_oracle_validates_gpu_counterexamples(cfg):
    """Counterexamples the GPU finds beyond the oracle's BFS reach (tests/golden/gpu_traces/): the
    LogMatching violation of the dynamic-membership model (InitServer = {s1, s2} grows to three
    servers), the known-false VotesGrantedInv_false / LeaderCompleteness_false (positive controls of
    the invariant kernels, raft.tla:1038-1046, :1079-1083), BoundedTrace under
    CommitWhenConcurrentLeaders_constraint (raft.tla:1182-1186) and the scenario
    NewlyJoinedBecomeLeader (raft.tla:1258-1266: a server added by AddNewServer later becomes leader;
    depth 21 on the growing cluster InitServer = {s1}, Server = {s1, s2}, whose stop-point counters
    the oracle's lean BFS also reached: "oracle_pin").  The oracle replays each state by
    state through its own Init, Next, constraints and invariants: valid, and the last state violates
    the named property."""
    from oracle_util import MEMB_MC, run_oracle
    g = GPU_TRACES[cfg]
    r = run_oracle("check-trace", MEMB_MC, os.path.join(CONFIGS, cfg + ".cfg"), "--golden",
                   os.path.join(GOLDEN, "gpu_traces", cfg + ".txt"))
    assert r["valid"] and r["length"] == g["depth"] and r["violated"] == g["violated"], r
    assert r["actions"].split(",") == g["actions"][1:]
    if "oracle_pin" in g:   # the oracle's own lean-mode BFS reached the stop point (make_gpu_trace_pin.py)
        assert {k: g["oracle_pin"][k] for k in ("verdict", "violated", "depth", "distinct", "generated", "left_on_queue")} == \
            {k: g[k] for k in ("verdict", "violated", "depth", "distinct", "generated", "left_on_queue")}


@pytest.mark.parametrize("name", ["parity_pair", "parity_trio", "c2_noleader"])
def test_oracle_lean_mode_is_identical(name):
    """--lean (engine.h bfs_lean: the mode of the full-size C2 fixture, tests/golden/c2_oracle.json)
    keys the seen-set by 128-bit hashes of the canonical text and keeps two levels of states: its
    counts, per-action counts, levels and stop point equal the exact text-keyed search's."""
    a = run_oracle("bfs", ORIG_MC, os.path.join(CONFIGS, name + ".cfg"))
    b = run_oracle("bfs", ORIG_MC, os.path.join(CONFIGS, name + ".cfg"), "--lean", "--workers", "4")
    for k in ("verdict", "violated", "generated", "distinct", "depth", "left_on_queue", "levels", "actions"):
        assert a[k] == b[k], k


def test_oracle_check_trace_of_an_evaluation_error(tmp_path):
    """TLC's evaluation-error verdict (tests/golden/memb_parity.json "eval:memb_eval_single"): a
    duplicated CatchupRequest handled twice empties s2's committed log (raft.tla:734-736), so
    QuorumLogInv's Committed(s2) == SubSeq(log[s2], 1, commitIndex[s2]) is out of range (:969).
    check-trace replays the fixture's trace and reports the error on its last state only."""
    g = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))["eval:memb_eval_single"]
    assert g["verdict"] == "EVAL_ERROR" and len(g["trace"]) == g["depth"]
    p = tmp_path / "eval.txt"
    p.write_text("\n".join(t["state"] for t in g["trace"]) + "\n")
    r = run_oracle("check-trace", MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), "--golden", str(p))
    assert r["valid"] and r["violated"] == "QuorumLogInv" and "SubSeq" in r["eval_error"], r
    assert r["actions"].split(",") == [t["action"] for t in g["trace"][1:]]
    # the same search in the oracle's lean mode stops at the same point
    b = run_oracle("bfs", MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), "--deadlock", "--lean", "--workers", "4")
    for k in ("verdict", "generated", "distinct", "depth", "left_on_queue", "levels", "actions"):
        assert b[k] == g[k], k


def test_deadlock_verdict_and_no_deadlock_in_shipped_next_relations():
    """TLC's deadlock check: NEXT NextUnreliable alone (raft.tla:924-932) has no successor of Init
    (empty bag) — "Deadlock reached" at State 1; the shipped NEXT relations never deadlock (Restart
    is always enabled; under NextAsync a server of its own config can Timeout or is a Leader with
    ClientRequest), so checking deadlock changes no count of their fixtures."""
    fix = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))
    g = fix["deadlock:memb_unreliable"]
    assert (g["verdict"], g["depth"], g["distinct"], len(g["trace"])) == ("DEADLOCK", 1, 1, 1)
    for case in ("membership_shipped@14", "memb_dynamic3@14"):
        f = fix[case]
        r = run_oracle("bfs", MEMB_MC, os.path.join(CONFIGS, f["cfg"] + ".cfg"), "--sym", f.get("sym", "view"), "--deadlock",
                       "--max-depth", f["max_depth"])
        assert (r["verdict"], r["generated"], r["distinct"], r["actions"]) == ("OK", f["generated"], f["distinct"], f["actions"])


def test_disjunct_copies_switch_oracle():
    """[ext] switch (vi), TLC's disjunct copies (oracle/engine.h Options::disjunct_copies, default on,
    --no-disjunct-copies): the committed fixture of both settings (tests/golden/make_disjunct_copies.py)
    differs only in the GENERATED counters of the two handlers whose guards are disjunctions
    (tlc_membership/raft.tla:796 HandleCheckOldConfig, :783-789 HandleCatchupResponse): the state space,
    its levels and every distinct count are the same; and a live run at depth 14 shows the same shape."""
    fx = json.load(open(os.path.join(GOLDEN, "disjunct_copies.json")))
    a, b = fx["copies"], fx["once"]
    copied = {"HandleCheckOldConfig", "HandleCatchupResponse"}
    for x, y in ((a, b), (run_oracle("bfs", MEMB_MC, os.path.join(CONFIGS, fx["cfg"]), "--max-depth", 14),
                         run_oracle("bfs", MEMB_MC, os.path.join(CONFIGS, fx["cfg"]), "--max-depth", 14, "--no-disjunct-copies"))):
        assert (x["distinct"], x["levels"], x["depth"]) == (y["distinct"], y["levels"], y["depth"])
        diff = {k: x["actions"][k][0] - y["actions"][k][0] for k in x["actions"]}
        assert {k for k, v in diff.items() if v} <= copied and min(diff.values()) == 0
        assert x["generated"] - y["generated"] == sum(diff.values()) > 0
        assert all(x["actions"][k][1] == y["actions"][k][1] for k in x["actions"])
    assert {k for k, v in a["actions"].items() if v[0] != b["actions"][k][0]} == copied   # both fire by depth 16
