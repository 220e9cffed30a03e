"""GPU parity tests (MI355X): the HIP path through the C ABI against the CPU
oracle.  Integer/index work, so the bar is bit-exact: identical generated,
distinct, depth, per-level and per-action counts, and the identical set of
reachable states (SHA-256 of the sorted canonical TLA+ text of every state).
"""
import hashlib
import json
import os
import tempfile

import pytest

from oracle_util import CONFIGS, GOLDEN, MEMB_MC, ORIG_MC

pytestmark = pytest.mark.gpu

SMALL = dict(fp_table_bytes=1 << 26, state_store_bytes=1 << 28)
FIXTURES = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))


def states_sha(mc):
    fd, path = tempfile.mkstemp(suffix=".txt")
    os.close(fd)
    mc.dump_states(path)
    lines = sorted(l.rstrip("\n") for l in open(path))
    os.unlink(path)
    return hashlib.sha256("\n".join(lines).encode()).hexdigest(), len(lines)


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_parity_against_oracle(raftmc, name):
    g = FIXTURES[name]
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, name + ".cfg"), **SMALL) as mc:
        r = mc.run()
        sha, n = states_sha(mc)
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth) == (g["generated"], g["distinct"], g["depth"])
    # per-action generated AND distinct counts: distinct ones depend on which successor reaches a
    # state first (TLC: FIFO order of one worker), which the GPU reproduces (min key per state)
    assert r.actions == g["actions"]
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert n == g["distinct"] and sha == g["states_sha256"]


@pytest.mark.parametrize("name", sorted(FIXTURES))
def test_parity_workers_n(raftmc, name):
    """TLC -workers N semantics (mc_opts.workers != 1: first-come seen-set, no FIFO keys): every
    order-independent output is the oracle's — generated, distinct, depth, level sizes, per-action
    generated counts, the set of states; per-action distinct counts only sum right (which producer
    of a state is kept is the workers' race, as in TLC)."""
    g = FIXTURES[name]
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, name + ".cfg"), workers=0, **SMALL) as mc:
        r = mc.run()
        sha, n = states_sha(mc)
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth) == (g["generated"], g["distinct"], g["depth"])
    assert {k: v[0] for k, v in r.actions.items()} == {k: v[0] for k, v in g["actions"].items()}
    assert sum(v[1] for v in r.actions.values()) == g["distinct"] - 1
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert n == g["distinct"] and sha == g["states_sha256"]


def test_depth_limit_kat(raftmc):
    # SURVEY.md §4 KAT: expanding Init gives generated 7, distinct 5
    r = raftmc.check(ORIG_MC, os.path.join(CONFIGS, "c1.cfg"), max_depth=2, **SMALL)
    assert (r.generated, r.distinct, r.verdict) == (7, 5, "DEPTH_LIMIT")


EVENTS = json.load(open(os.path.join(GOLDEN, "orig_events.json")))


def trace_states(r):
    """(action, one-line state) per "State k:" block of a trace"""
    out = []
    for blk in r.trace_text.strip().split("\n\n"):
        head, *body = blk.split("\n")
        act = "Init" if "<Initial predicate>" in head else head.split("<", 1)[1].split(" ")[0].rstrip(">")
        out.append((act, " ".join(body)))
    return out


@pytest.mark.parametrize("name", sorted(EVENTS))
def test_fifo_stop_point_against_oracle(raftmc, name):
    """TLC's stop point (tests/golden/orig_events.json): the first violating successor in TLC's
    single-worker FIFO order, its counterexample state by state, and TLC's counters at that
    point (generated = whole successor lists up to the violating parent; distinct, per-action
    counts and left-on-queue at the violating successor; completed levels).  Deterministic: a
    second run, another fingerprint seed and the TLC -workers N pipeline give the identical report."""
    g = EVENTS[name]
    cfg = os.path.join(CONFIGS, name + ".cfg")
    a = raftmc.check(ORIG_MC, cfg, **SMALL)
    b = raftmc.check(ORIG_MC, cfg, seed=0xC0FFEE, **SMALL)
    c = raftmc.check(ORIG_MC, cfg, workers=0, **SMALL)    # -workers N: re-searched in FIFO order on the event
    for r in (a, b, c):
        assert (r.verdict, r.violated, r.exit_code) == (g["verdict"], g["violated"], 12), r.error
        assert (r.generated, r.distinct, r.left_on_queue, r.depth) == (g["generated"], g["distinct"], g["left_on_queue"],
                                                                       g["depth"])
        assert [lv[0] for lv in r.levels] == g["levels"]
        assert r.actions == g["actions"]
        assert trace_states(r) == [(t["action"], t["state"]) for t in g["trace"]]
    assert a.trace_text == b.trace_text


def test_stop_point_independent_of_chunking_and_spill(raftmc):
    """The counterexample does not depend on chunking: a state store small enough to split the
    levels into several chunks and to spill completed levels reports the same stop point."""
    g = EVENTS["c2_noleader"]
    cfg = os.path.join(CONFIGS, "c2_noleader.cfg")
    cap = max(4 * 4096, 3 * max(g["levels"]))
    r = raftmc.check(ORIG_MC, cfg, fp_table_bytes=1 << 26, state_store_bytes=cap * _slot_bytes(raftmc, cfg))
    assert (r.verdict, r.generated, r.distinct, r.left_on_queue) == (g["verdict"], g["generated"], g["distinct"],
                                                                     g["left_on_queue"]), r.error
    assert r.actions == g["actions"]
    assert trace_states(r) == [(t["action"], t["state"]) for t in g["trace"]]


def test_capacity_overflow_verdicts(raftmc):
    """Compiled-capacity limits are a CAPACITY_OVERFLOW verdict, never a silent clamp: a seen-set
    or a state store too small for the model."""
    cfg = os.path.join(CONFIGS, "parity_pair.cfg")
    r = raftmc.check(ORIG_MC, cfg, fp_table_bytes=1 << 14, state_store_bytes=1 << 26)   # 1024 entries, 20938 states
    assert r.verdict == "CAPACITY_OVERFLOW" and "fingerprint table full" in r.error, (r.verdict, r.error)
    r = raftmc.check(ORIG_MC, cfg, fp_table_bytes=1 << 26, state_store_bytes=3000 * _slot_bytes(raftmc, cfg))
    assert r.verdict == "CAPACITY_OVERFLOW" and "state store full" in r.error, (r.verdict, r.error)
    assert r.exit_code != 0


def test_trace_headers_carry_action_locations(raftmc, tmp_path):
    """TLC's "State k: <Action line L1, col C1 to line L2, col C2 of module M>" headers: with the
    spec module next to the wrapper (as TLC resolves EXTENDS), every step names the span of its
    action's definition body, and the steps are exactly the oracle's counterexample (TLC's FIFO
    first violating state, tests/golden/orig_events.json)."""
    wrapper = tmp_path / "raft_original_mc.tla"
    wrapper.write_text(open(ORIG_MC).read())
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c1.cfg")) as mc:
        names = mc.describe()["actions"]
    body = ["------ MODULE raft ------"]
    for a in names:                                   # action a's body is the whole of line 2k+3
        body += ["\\* %s" % a, "%s(i) == TRUE" % a]
    (tmp_path / "raft.tla").write_text("\n".join(body + ["===="]) + "\n")
    cfg = os.path.join(CONFIGS, "scenario_first_leader.cfg")
    r = raftmc.check(str(wrapper), cfg, **SMALL)
    assert r.verdict == "INVARIANT_VIOLATION"
    heads = [b.split("\n")[0] for b in r.trace_text.strip().split("\n\n")]
    want = [t["action"] for t in EVENTS["scenario_first_leader"]["trace"]]
    assert len(heads) == len(want) == 10
    expect = ["State 1: <Initial predicate>"]
    for k, act in enumerate(want[1:]):
        line, col = 2 * names.index(act) + 3, len(act) + 8   # after "Act(i) == "
        expect.append("State %d: <%s line %d, col %d to line %d, col %d of module raft>" % (k + 2, act, line, col, line, col + 3))
    assert heads == expect
    assert heads[-1] in r.report


def test_seed_independence_c1(raftmc):
    cfg = os.path.join(CONFIGS, "c1.cfg")
    a = raftmc.check(ORIG_MC, cfg, seed=1, **SMALL)
    b = raftmc.check(ORIG_MC, cfg, seed=0xABCDEF, **SMALL)
    assert (a.generated, a.distinct, a.depth) == (b.generated, b.distinct, b.depth)


def test_c2_workers_n_equals_fifo(raftmc):
    """BASELINE configs[1] at full size in both pipelines: TLC -workers 1 (FIFO keys) and -workers N
    give the identical order-independent results; per-action distinct counts sum to the same."""
    cfg = os.path.join(CONFIGS, "c2.cfg")
    a = raftmc.check(ORIG_MC, cfg)
    b = raftmc.check(ORIG_MC, cfg, workers=0)
    assert a.verdict == b.verdict == "OK", (a.error, b.error)
    assert (a.generated, a.distinct, a.depth, a.generated_in_model) == (b.generated, b.distinct, b.depth, b.generated_in_model)
    assert [lv[0] for lv in a.levels] == [lv[0] for lv in b.levels]
    assert {k: v[0] for k, v in a.actions.items()} == {k: v[0] for k, v in b.actions.items()}
    assert sum(v[1] for v in a.actions.values()) == sum(v[1] for v in b.actions.values())


def test_c2_full_size_properties(raftmc):
    """BASELINE configs[1] at full size: order-independent counts (no VIEW in
    raft_original) must not depend on the fingerprint seed or on re-use of
    the handle, and must equal the exact (collision-free) host count; the level
    sizes sum to the distinct count."""
    cfg = os.path.join(CONFIGS, "c2.cfg")
    with raftmc.ModelChecker(ORIG_MC, cfg, seed=7) as mc:
        a = mc.run()
        b = mc.run()
    c = raftmc.check(ORIG_MC, cfg, seed=0x1234567)
    assert a.verdict == "OK", a.error
    assert (a.generated, a.distinct, a.depth) == (b.generated, b.distinct, b.depth) == (c.generated, c.distinct, c.depth)
    # the exact state space (host BFS over full packed states, tests/golden/make_c2_exact.py): a
    # fingerprint collision would show here as missing states, whatever the seed
    exact = json.load(open(os.path.join(GOLDEN, "c2_exact.json")))
    assert (a.generated, a.distinct, a.depth) == (exact["generated"], exact["distinct"], exact["depth"])
    assert {k: v[0] for k, v in a.actions.items()} == exact["actions_generated"]
    assert sum(lv[0] for lv in a.levels) == a.distinct
    assert sum(v[1] for v in a.actions.values()) + 1 == a.distinct
    assert sum(v[0] for v in a.actions.values()) + 1 == a.generated
    # TLC's "calculated (optimistic)" collision estimate: M * (N - M) / 2^64
    assert a.collision_prob_optimistic == pytest.approx(a.distinct * (a.generated - a.distinct) / 2.0 ** 64)
    # the oracle pin (tests/golden/make_c2_oracle.py: the CPU restatement of raft_original.tla run
    # over the whole C2 in its lean mode): counts, depth, level sizes and the per-action generated
    # AND distinct counts of TLC's single-worker FIFO order (the handle's default, -workers 1)
    pin = os.path.join(GOLDEN, "c2_oracle.json")
    if not os.path.exists(pin):
        pytest.skip("tests/golden/c2_oracle.json not generated yet")
    o = json.load(open(pin))
    assert (a.generated, a.distinct, a.depth) == (o["generated"], o["distinct"], o["depth"])
    assert [lv[0] for lv in a.levels] == o["levels"]
    assert {k: list(v) for k, v in a.actions.items()} == {k: list(v) for k, v in o["actions"].items()}


@pytest.mark.parametrize("fixture", ["c5_prefix", "c5v2_prefix", "c2_md6_prefix"])
def test_c5_prefix_parity(raftmc, fixture):
    """BASELINE configs[4] (C5: 5 servers, term <= 3, log <= 3; 87 action instances per
    state, 96-B packed states; c5v2: two values and 8 messages, 104 instances, 160-B states,
    8 messages, compact election records) to the oracle's depth limit: identical counts, per-level sizes,
    per-action generated counts, left-on-queue and the set of states found."""
    path = os.path.join(GOLDEN, fixture + ".json")
    if not os.path.exists(path):
        pytest.skip(fixture + " not generated")
    g = json.load(open(path))
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, g["cfg"]), max_depth=g["max_depth"], **SMALL) as mc:
        r = mc.run()
        sha, n = states_sha(mc)
    assert r.verdict == "DEPTH_LIMIT", r.error
    assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"],
                                                                   g["left_on_queue"])
    assert [lv[0] for lv in r.levels] == g["levels"]
    assert {k: v[0] for k, v in r.actions.items()} == {k: v[0] for k, v in g["actions"].items()}
    assert n == g["distinct"] and sha == g["states_sha256"]


def test_c5_deep_properties(raftmc):
    """C5 five levels past the oracle's reach (~1e8 distinct states): seed-independent
    counts, levels summing to the distinct count, TLC's generated bookkeeping."""
    cfg = os.path.join(CONFIGS, "c5.cfg")
    a = raftmc.check(ORIG_MC, cfg, max_depth=11, seed=3)
    b = raftmc.check(ORIG_MC, cfg, max_depth=11, seed=0xC5C5C5)
    assert a.verdict == b.verdict == "DEPTH_LIMIT", (a.error, b.error)
    assert (a.generated, a.distinct, a.left_on_queue) == (b.generated, b.distinct, b.left_on_queue)
    assert [lv[0] for lv in a.levels] == [lv[0] for lv in b.levels]
    assert sum(lv[0] for lv in a.levels) == a.distinct and a.left_on_queue == a.levels[-1][0]
    assert sum(v[0] for v in a.actions.values()) + 1 == a.generated


def test_c5v2_deep_properties(raftmc):
    """C5v2 (configs/c5v2.cfg: 5 servers, 2 values, 8 messages) three levels past the oracle's
    depth-7 pin: the TLC -workers 1 (FIFO) and -workers N pipelines agree on every
    order-independent count, the counts do not depend on the fingerprint seed, the levels sum to
    the distinct count and the per-action counts to TLC's generated/distinct bookkeeping."""
    cfg = os.path.join(CONFIGS, "c5v2.cfg")
    a = raftmc.check(ORIG_MC, cfg, max_depth=10, seed=3)
    b = raftmc.check(ORIG_MC, cfg, max_depth=10, seed=0xC5C5C5, workers=0)
    assert a.verdict == b.verdict == "DEPTH_LIMIT", (a.error, b.error)
    assert (a.generated, a.distinct, a.left_on_queue) == (b.generated, b.distinct, b.left_on_queue)
    assert [lv[0] for lv in a.levels] == [lv[0] for lv in b.levels]
    assert {k: v[0] for k, v in a.actions.items()} == {k: v[0] for k, v in b.actions.items()}
    assert sum(lv[0] for lv in a.levels) == a.distinct and a.left_on_queue == a.levels[-1][0]
    assert sum(v[0] for v in a.actions.values()) + 1 == a.generated
    assert sum(v[1] for v in a.actions.values()) + 1 == a.distinct


def test_count_final_level(raftmc, tmp_path):
    """mc_opts.count_final_level: the level at depth max_depth is never expanded, so the -workers N
    search fingerprints, counts and invariant-checks its states without writing them to the store.
    Every count equals the storing run's; mc_dump_states refuses; an event in that level re-runs
    TLC's FIFO order (which stores every level) and gives the same counterexample (NoLeader at depth
    10, tests/golden/orig_events.json)."""
    cfg = os.path.join(CONFIGS, "c5v2.cfg")
    a = raftmc.check(ORIG_MC, cfg, max_depth=10, workers=0)
    with raftmc.ModelChecker(ORIG_MC, cfg, max_depth=10, workers=0, count_final_level=True) as mc:
        b = mc.run()
        with pytest.raises(raftmc.RaftMCError):
            mc.dump_states(str(tmp_path / "states.txt"))
    assert a.verdict == b.verdict == "DEPTH_LIMIT", (a.error, b.error)
    assert (a.generated, a.distinct, a.left_on_queue, a.depth) == (b.generated, b.distinct, b.left_on_queue, b.depth)
    assert [lv[0] for lv in a.levels] == [lv[0] for lv in b.levels]
    # per-action distinct counts are first-come under -workers N (order-dependent): their sum is not
    assert {k: v[0] for k, v in a.actions.items()} == {k: v[0] for k, v in b.actions.items()}
    assert sum(v[1] for v in b.actions.values()) + 1 == b.distinct
    ev = os.path.join(CONFIGS, "c2_noleader.cfg")
    c = raftmc.check(ORIG_MC, ev, max_depth=10, workers=0)
    d = raftmc.check(ORIG_MC, ev, max_depth=10, workers=0, count_final_level=True)
    assert c.verdict == d.verdict == "INVARIANT_VIOLATION" and d.violated == "NoLeader" and d.depth == 10
    assert (c.generated, c.distinct, c.left_on_queue, c.trace_text) == (d.generated, d.distinct, d.left_on_queue, d.trace_text)


def test_c5v2_depth13_count_final_level(raftmc):
    """C5v2 to depth 13 on one MI355X: 2.44e9 distinct states, whose level 13 (1.96e9 states, ~329 GB
    at 168 B stored) fits neither HBM nor the host, so it is counted, not stored (count_final_level).
    The levels through 12 are the storing pipeline's (bench.py's scale_workload), the counts do not
    depend on the fingerprint seed, the levels sum to the distinct count and the per-action counts to
    TLC's generated/distinct bookkeeping."""
    cfg = os.path.join(CONFIGS, "c5v2.cfg")
    runs = []
    for seed in (1, 0xC5C5C5):
        with raftmc.ModelChecker(ORIG_MC, cfg, max_depth=13, workers=0, count_final_level=True, seed=seed,
                                 fp_table_bytes=64 << 30, state_store_bytes=120 << 30) as mc:
            runs.append(mc.run())
    a, b = runs
    assert a.verdict == b.verdict == "DEPTH_LIMIT", (a.error, b.error)
    assert (a.generated, a.distinct, a.left_on_queue, a.depth) == (b.generated, b.distinct, b.left_on_queue, b.depth)
    assert [lv[0] for lv in a.levels] == [lv[0] for lv in b.levels]
    assert [lv[0] for lv in a.levels][:12] == [1, 6, 45, 330, 2190, 13761, 82510, 475485, 2648995, 14330920,
                                               75545752, 389107090]
    # both seeds: 2,442,107,060.  Seed 0x5EED (scripts/c5_probe.py, profiles/r04_c5v2_d13.jsonl) finds
    # one fewer in level 13: a 64-bit fingerprint collision, which at 2.44e9 states TLC's optimistic
    # estimate n^2 / 2^65 puts at 0.16 expected
    assert (a.depth, a.distinct, a.generated) == (13, 2442107060, 18179584961)
    assert sum(lv[0] for lv in a.levels) == a.distinct and a.left_on_queue == a.levels[-1][0]
    assert sum(v[0] for v in a.actions.values()) + 1 == a.generated
    assert sum(v[1] for v in a.actions.values()) + 1 == a.distinct


def test_c5_compact_election_records(raftmc, tmp_path):
    """A reachable 5-server election on the GPU: election records of 5 servers with a 341-log universe
    do not fit 64 bits, so the shape stores them compactly (orig_spec.h ECOMPACT: the voterLog row's
    presence bits come from evotes, eterm in bits_for(MaxTerm)).  configs/c5e_noleader.cfg (one
    election term, 6 messages) reaches TLC's single-worker FIFO first election at depth 14 behind
    301.6M states (c5v2.cfg would need ~1e10); NoLeader's counterexample ends in that BecomeLeader,
    its election record printed through the compact decoding, and the oracle's check-trace replays
    the trace state by state through the literal restatement of raft_original.tla.  (Round 2's
    c5v2 variant of this test could not reach an election: its first one lies at depth 14, not 12.)"""
    from oracle_util import run_oracle
    cfg = os.path.join(CONFIGS, "c5e_noleader.cfg")
    with raftmc.ModelChecker(ORIG_MC, cfg, fp_table_bytes=32 << 30, state_store_bytes=112 << 30) as mc:
        d = mc.describe()
        assert (d["N"], d["MaxTerm"], d["MaxLogLen"], d["log_universe"]) == (5, 2, 4, 341)
        r = mc.run()
    assert r.verdict == "INVARIANT_VIOLATION" and r.violated == "NoLeader", (r, r.error)
    assert r.depth == 14 and r.exit_code == 12
    states = [st for _, st in trace_states(r)]
    assert len(states) == 14
    assert "<BecomeLeader" in r.trace_text.strip().split("\n\n")[-1].split("\n")[0]
    assert "evoterLog |-> (" in states[-1] and "evotes |-> {" in states[-1]
    p = tmp_path / "trace.txt"
    p.write_text("\n".join(states) + "\n")
    o = run_oracle("check-trace", ORIG_MC, cfg, "--golden", str(p))
    assert o["valid"] and o["length"] == len(states) and o["violated"] == "NoLeader", o

def test_checkpoint_recover_c1(raftmc, tmp_path):
    """TLC -checkpoint / -recover: a search stopped at depth 6 with a checkpoint per level,
    resumed by a fresh handle, ends exactly like the uninterrupted search (counts, levels,
    per-action generated counts, the set of states)."""
    g = FIXTURES["c1"]
    cfg = os.path.join(CONFIGS, "c1.cfg")
    ck = str(tmp_path / "c1.ckpt")
    with raftmc.ModelChecker(ORIG_MC, cfg, max_depth=6, **SMALL) as mc:
        mc.set_checkpoint(ck, 1)
        a = mc.run()
    assert a.verdict == "DEPTH_LIMIT" and os.path.exists(ck)
    with raftmc.ModelChecker(ORIG_MC, cfg, **SMALL) as mc:
        mc.set_recover(ck)
        b = mc.run()
        sha, n = states_sha(mc)
    assert (b.verdict, b.generated, b.distinct, b.depth) == ("OK", g["generated"], g["distinct"], g["depth"])
    assert {k: v[0] for k, v in b.actions.items()} == {k: v[0] for k, v in g["actions"].items()}
    assert [lv[0] for lv in b.levels] == g["levels"]
    assert n == g["distinct"] and sha == g["states_sha256"]
    # a checkpoint only resumes its own model
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "parity_pair.cfg"), **SMALL) as mc:
        mc.set_recover(ck)
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.run()
    assert e.value.code == -1


def test_checkpoint_search_order_guard(raftmc, tmp_path):
    """A checkpoint records its search order: one written by the TLC -workers N pipeline (first-come
    dedup, kept parents not TLC's) is refused by a -workers 1 search (TLC's single-worker FIFO
    order); the reverse direction and a -workers N resume are accepted and end with the oracle's
    counts."""
    g = FIXTURES["c1"]
    cfg = os.path.join(CONFIGS, "c1.cfg")
    ckn, ck1 = str(tmp_path / "n.ckpt"), str(tmp_path / "one.ckpt")
    for path, workers in ((ckn, 0), (ck1, 1)):
        with raftmc.ModelChecker(ORIG_MC, cfg, max_depth=6, workers=workers, **SMALL) as mc:
            mc.set_checkpoint(path, 1)
            assert mc.run().verdict == "DEPTH_LIMIT"
    with raftmc.ModelChecker(ORIG_MC, cfg, workers=1, **SMALL) as mc:
        mc.set_recover(ckn)
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.run()
    assert e.value.code == -1 and "-workers N" in str(e.value)
    for path, workers in ((ckn, 0), (ck1, 0), (ck1, 1)):
        with raftmc.ModelChecker(ORIG_MC, cfg, workers=workers, **SMALL) as mc:
            mc.set_recover(path)
            r = mc.run()
        assert (r.verdict, r.generated, r.distinct, r.depth) == ("OK", g["generated"], g["distinct"], g["depth"]), (path, workers)


def test_checkpoint_recover_c2(raftmc, tmp_path):
    """BASELINE configs[1]: checkpoint at depth 20 of a full run, resume to the exact count."""
    cfg = os.path.join(CONFIGS, "c2.cfg")
    ck = str(tmp_path / "c2.ckpt")
    with raftmc.ModelChecker(ORIG_MC, cfg) as mc:
        mc.set_checkpoint(ck, 20)
        a = mc.run()
    with raftmc.ModelChecker(ORIG_MC, cfg, seed=99) as mc:   # the checkpoint's seed wins
        mc.set_recover(ck)
        b = mc.run()
    exact = json.load(open(os.path.join(GOLDEN, "c2_exact.json")))
    for r in (a, b):
        assert (r.verdict, r.generated, r.distinct, r.depth) == ("OK", exact["generated"], exact["distinct"], exact["depth"])
        assert {k: v[0] for k, v in r.actions.items()} == exact["actions_generated"]
    assert [lv[0] for lv in a.levels] == [lv[0] for lv in b.levels]


def _slot_bytes(raftmc, cfg):
    """device bytes per stored state: packed state + parent pointer"""
    with raftmc.ModelChecker(ORIG_MC, cfg) as mc:
        return mc.describe()["state_bytes_stored"] + 8


def test_spill_completed_levels_c2(raftmc, tmp_path):
    """A state store too small for the whole search but large enough for two consecutive
    levels: completed levels move to host memory and the search ends exactly like the
    in-HBM one (counts, levels, per-action counts); a checkpoint taken after spills and the
    trace-visible parent pointers keep working."""
    cfg = os.path.join(CONFIGS, "c2.cfg")
    a = raftmc.check(ORIG_MC, cfg)
    sizes = [lv[0] for lv in a.levels]
    cap = int(max(x + y for x, y in zip(sizes, sizes[1:])) * 1.6)
    assert cap < a.distinct                          # the store cannot hold the search
    ck = str(tmp_path / "c2s.ckpt")
    with raftmc.ModelChecker(ORIG_MC, cfg, state_store_bytes=cap * _slot_bytes(raftmc, cfg)) as mc:
        mc.set_checkpoint(ck, 22)
        b = mc.run()
    assert (b.verdict, b.generated, b.distinct, b.depth) == ("OK", a.generated, a.distinct, a.depth), b.error
    assert [lv[0] for lv in b.levels] == sizes
    assert {k: v[0] for k, v in b.actions.items()} == {k: v[0] for k, v in a.actions.items()}
    with raftmc.ModelChecker(ORIG_MC, cfg, state_store_bytes=cap * _slot_bytes(raftmc, cfg)) as mc:   # resume: spilled part on the host
        mc.set_recover(ck)
        c = mc.run()
    assert (c.generated, c.distinct, c.depth) == (a.generated, a.distinct, a.depth), c.error


def test_spill_state_set_c1(raftmc):
    """The host-spilled and device parts together are exactly the oracle's state set."""
    g = FIXTURES["c1"]
    cap = int(max(x + y for x, y in zip(g["levels"], g["levels"][1:])) * 1.3)
    assert cap < g["distinct"]
    cfg = os.path.join(CONFIGS, "c1.cfg")
    with raftmc.ModelChecker(ORIG_MC, cfg, fp_table_bytes=1 << 26, state_store_bytes=cap * _slot_bytes(raftmc, cfg)) as mc:
        r = mc.run()
        sha, n = states_sha(mc)
    assert (r.verdict, r.generated, r.distinct, r.depth) == ("OK", g["generated"], g["distinct"], g["depth"]), r.error
    assert n == g["distinct"] and sha == g["states_sha256"]


def test_spill_violation_trace(raftmc, tmp_path):
    """Trace reconstruction across the host/device split: with a store that forces spills,
    NoLeader's witness is still TLC's FIFO-first one (the oracle's, state by state), and the
    oracle's check-trace replays it step by step."""
    from oracle_util import run_oracle
    g = EVENTS["scenario_first_leader"]
    cfg = os.path.join(CONFIGS, "scenario_first_leader.cfg")
    sizes = g["levels"]
    cap = max(64, int(max(x + y for x, y in zip(sizes, sizes[1:])) * 1.6))
    b = raftmc.check(ORIG_MC, cfg, fp_table_bytes=1 << 26, state_store_bytes=cap * _slot_bytes(raftmc, cfg))
    assert b.verdict == "INVARIANT_VIOLATION"
    assert (b.distinct, b.generated, b.left_on_queue) == (g["distinct"], g["generated"], g["left_on_queue"])
    assert trace_states(b) == [(t["action"], t["state"]) for t in g["trace"]]
    p = tmp_path / "trace.txt"
    p.write_text("\n".join(st for _, st in trace_states(b)) + "\n")
    r = run_oracle("check-trace", ORIG_MC, cfg, "--golden", str(p))
    assert r["valid"] and r["length"] == 10 and r["violated"] == "NoLeader", r


def test_collision_estimates_and_tlc_summary_lines(raftmc):
    """TLC's two collision estimates: the optimistic M*(N-M)/2^64 and the one "based on the
    actual fingerprints" (1 / minimum distance between two fingerprints of the seen-set, from a
    device sort after the run); the report carries TLC's summary lines."""
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c2.cfg")) as mc:
        r = mc.run()
        v = mc.collision_observed()
        r2 = mc.summary()
    # 54.4M uniform 64-bit fingerprints: expected minimum gap ~ 2^64 / M^2 (~6e3)
    assert 1e-7 < v < 1e-1
    assert r2.collision_prob_observed == v
    assert "Model checking completed. No error has been found." in r2.report
    assert "calculated (optimistic):  val = " in r2.report and "based on the actual fingerprints:  val = " in r2.report
    assert "%d states generated, %d distinct states found, 0 states left on queue." % (r.generated, r.distinct) in r2.report
    assert "The depth of the complete state graph search is %d." % r.depth in r2.report
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, "memb_two.cfg"), max_depth=14, deadlock=False) as mc:
        mc.run()
        assert 0 < mc.collision_observed() < 1


@pytest.mark.parametrize("frontend", ["hand", "generated"])
def test_release_device_memory(raftmc, frontend, tmp_path):
    """mc_release_device_memory (a handle keeps its device buffers between runs -- the generated
    path its whole working set): after it the last run's summary and trace stay readable, mc_dump_states is
    refused (MC_E_STATE), and the next run allocates again and gives the same result."""
    cfg = os.path.join(CONFIGS, "parity_pair.cfg")
    spec = ORIG_MC
    if frontend == "generated":   # the front end's prebuilt source (the GPU box has no reference checkout)
        from test_gpu_tlagen import gen_source
        spec = gen_source("parity_pair")
    with raftmc.ModelChecker(spec, cfg, frontend=frontend, fp_table_bytes=1 << 24, state_store_bytes=1 << 28) as mc:
        a = mc.run()
        mc.release_device_memory()
        assert mc.summary().distinct == a.distinct
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.dump_states(str(tmp_path / "x.txt"))
        assert e.value.code == -7
        b = mc.run()
        mc.dump_states(str(tmp_path / "y.txt"))
    assert (a.verdict, a.generated, a.distinct, a.depth) == (b.verdict, b.generated, b.distinct, b.depth)
    assert sum(1 for _ in open(tmp_path / "y.txt")) == b.distinct
