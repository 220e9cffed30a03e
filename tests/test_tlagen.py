"""The SANY-subset front end (raft-tla_amd/csrc/tlagen) on the CPU:
it parses every module of the reference, and the C++ it generates — the code the GPU path
compiles for gfx950 — reproduces the oracle's counts when run by a plain host BFS
(tests/native/tlagen_host_bfs.cpp): thirdparty/raft_original.tla, unmodified, through the
generated path gives C1's and the parity configs' generated / distinct / depth / level sizes
(tests/golden/orig_parity.json); the repo's own TokenRing.tla matches an independent Python
restatement (tests/tlagen_models.py)."""
import json
import os
import subprocess
import tempfile

import pytest

from oracle_util import CONFIGS, GOLDEN, ORIG_MC, run_oracle
from tlagen_models import rec_fun, token_ring

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "raft-tla_amd", "_build", "tlagen")
REF = "/root/reference"
RING = os.path.join(CONFIGS, "tlagen", "TokenRing.tla")

needs_tool = pytest.mark.skipif(not os.path.exists(TOOL), reason="raft-tla_amd/_build/tlagen not built")
needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="the reference checkout is not present")


def generate(spec, cfg):
    fd, out = tempfile.mkstemp(suffix=".gen.h")
    os.close(fd)
    r = subprocess.run([TOOL, spec, cfg, "-I", REF, "-o", out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


def host_bfs(gen, *args):
    exe = gen + ".bin"
    subprocess.run(["g++", "-O2", "-std=c++17", "-w", '-DTLG_FILE="%s"' % gen, "-o", exe,
                    os.path.join(ROOT, "tests", "native", "tlagen_host_bfs.cpp")], check=True)
    out = subprocess.run([exe, *args], capture_output=True, text=True, check=True).stdout
    os.unlink(exe)
    os.unlink(gen)
    return json.loads(out)


@needs_tool
@needs_ref
@pytest.mark.parametrize("module,defs,unparsed", [
    ("thirdparty/raft_original.tla", 38, 0), ("thirdparty/raft_dricketts.tla", 63, 0),
    ("thirdparty/raft_membership.tla", 46, 0), ("tlc_membership/raft.tla", 166, 0),
    ("apalache_no_membership/raft.tla", 103, 0), ("apalache_membership_broken/raft.tla", 75, 0)])
def test_parses_reference_modules(module, defs, unparsed):
    """Every definition of every reference module (and the modules they EXTEND) parses, SequencesExt's
    Remove (a LAMBDA) included."""
    r = subprocess.run([TOOL, os.path.join(REF, module), "--parse-only"], capture_output=True, text=True)
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert (summary["definitions"], summary["unparsed"]) == (defs, unparsed), r.stdout


@needs_tool
@needs_ref
@pytest.mark.parametrize("name", ["c1", "parity_single", "parity_pair", "parity_trio"])
def test_raft_original_generated_matches_oracle(name):
    g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))[name]
    r = host_bfs(generate(ORIG_MC, os.path.join(CONFIGS, name + ".cfg")))
    assert r["verdict"] == "OK" and r["err"] == 0
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == (g["generated"], g["distinct"], g["depth"], g["levels"])
    # raft_original's Next is a conjunction: TLC does not split it, so it is one action
    assert list(r["actions"]) == ["Next"]


@needs_tool
def test_token_ring_matches_python_model():
    want = token_ring()
    r = host_bfs(generate(RING, os.path.join(CONFIGS, "tlagen", "TokenRing.cfg")))
    assert r["verdict"] == "OK" and r["err"] == 0
    for k in ("generated", "distinct", "depth", "levels"):
        assert r[k] == want[k], k
    for a, v in want["actions"].items():
        assert r["actions"][a] == v, a


@needs_tool
def test_token_ring_view_fifo():
    """TLC's VIEW (configs/tlagen/TokenRing_view.cfg: VIEW <<token, logs>>): states are told apart
    by the view and the kept one is the first found in TLC's single-worker FIFO order -- its
    history decides its own successors, so every count is FIFO-sensitive; the host BFS (sequential:
    FIFO) equals the Python restatement."""
    want = token_ring(view=True)
    r = host_bfs(generate(RING, os.path.join(CONFIGS, "tlagen", "TokenRing_view.cfg")))
    assert r["verdict"] == "OK" and r["err"] == 0
    for k in ("generated", "distinct", "depth", "levels"):
        assert r[k] == want[k], k
    for a, v in want["actions"].items():
        assert r["actions"][a] == v, a


@needs_tool
def test_token_ring_violation_depth():
    want = token_ring(stop_when_all_full=True)
    r = host_bfs(generate(RING, os.path.join(CONFIGS, "tlagen", "TokenRing_full.cfg")))
    assert (r["verdict"], r["violated"], r["depth"]) == ("INVARIANT_VIOLATION", "NotAllFull", want["depth"])


@needs_tool
def test_unsupported_construct_fails_loudly(tmp_path):
    """A definition outside the subset that the cfg reaches is an error naming it (never a silent
    fallback); an unreached one is not."""
    (tmp_path / "Prod.tla").write_text(
        "---- MODULE Prod ----\nEXTENDS Naturals\nVARIABLE x\n"
        "Keep(s) == {<<a, b>> \\in s \\X s : a > b}\nInit == x = {1, 2}\nNext == x' = Keep(x)\n"
        "Unused == {<<a, b>> \\in x \\X x : a > b}\n====\n")
    (tmp_path / "Prod.cfg").write_text("INIT Init\nNEXT Next\n")
    r = subprocess.run([TOOL, str(tmp_path / "Prod.tla"), str(tmp_path / "Prod.cfg")], capture_output=True, text=True)
    assert r.returncode == 1 and "Keep" in r.stderr and "does not parse" in r.stderr


REC = os.path.join(CONFIGS, "tlagen", "RecFun.tla")


@needs_tool
def test_recursive_function_definitions():
    """Recursive function definitions (TypedBags' Sum, tlc_membership/TypedBags.tla:73-83: a LET
    DSum[S \\in SUBSET DOMAIN f] that applies itself) evaluated lazily like TLC, one application at
    a time: the counts of configs/tlagen/RecFun.tla equal an independent Python restatement."""
    want = rec_fun()
    r = host_bfs(generate(REC, os.path.join(CONFIGS, "tlagen", "RecFun.cfg")))
    assert r["verdict"] == "OK" and r["err"] == 0
    assert (r["generated"], r["distinct"], r["depth"], r["levels"]) == (want["generated"], want["distinct"], want["depth"], want["levels"])


@needs_tool
@needs_ref
def test_generated_fifo_trace_equals_oracle():
    """The generated code enumerates successors in TLC's order (sets and function domains in TLC's
    value order, tlv.h ocmp; Next's disjuncts and bound variables in text order): a sequential FIFO
    BFS over it (TLC -workers 1) finds the oracle's NoLeader counterexample state by state, with
    TLC's counters at the stop point (tests/golden/orig_events.json, c2_noleader)."""
    g = json.load(open(os.path.join(GOLDEN, "orig_events.json")))["c2_noleader"]
    r = host_bfs(generate(ORIG_MC, os.path.join(CONFIGS, "c2_noleader.cfg")), "--trace")
    assert (r["verdict"], r["violated"], r["distinct"]) == ("INVARIANT_VIOLATION", "NoLeader", g["distinct"])
    assert r["trace"] == [t["state"] for t in g["trace"]]


# the hand-compiled path's action names for what the unmodified spec's ReceiveDirect disjunction
# holds (tlc_membership/raft.tla:842-863): the generated path splits actions where TLC does
# (disjunctions, \E, operator definitions), and `m.mtype = X /\ HandleX(..)` is a conjunction
RECEIVE_DIRECT = ("HandleRequestVoteRequest", "HandleRequestVoteResponse", "DropStaleResponse", "HandleAppendEntriesRequest",
                  "HandleAppendEntriesResponse", "HandleCatchupRequest", "HandleCatchupResponse", "HandleCheckOldConfig")


# NextUnreliable's disjuncts `\E m \in DOMAIN messages : /\ messages[m] = 1 /\ DuplicateMessage(m)`
# (and DropMessage, raft.tla:924-932) are conjunctions under the \E: actions named NextUnreliable
UNRELIABLE = ("DuplicateMessage", "DropMessage")


def memb_actions_as_generated(acts):
    out = {k: v for k, v in acts.items() if k not in RECEIVE_DIRECT + UNRELIABLE and v[0]}
    for name, group in (("ReceiveDirect", RECEIVE_DIRECT), ("NextUnreliable", UNRELIABLE)):
        g = [sum(acts.get(k, [0, 0])[i] for k in group) for i in (0, 1)]
        if g[0]:
            out[name] = g
    return out


@needs_tool
@needs_ref
@pytest.mark.parametrize("case", ["memb_nosym@13", "tlc:membership_shipped@16", "tlc:memb_two@16", "tlc:memb_dynamic3@14",
                                  "tlc:memb_four@13"])
def test_generated_membership_matches_oracle(case):
    """The unmodified tlc_membership/raft.tla (through configs/raft_membership_mc.tla) on the generated
    path with TLC's semantics in full -- VIEW vars, SYMMETRY perms by TLC's rule (the least permuted
    state in TLC's value order, then its VIEW: tla_gen.cpp canon_view), the single-worker FIFO order
    that decides which state of a view class is kept -- against the oracle's fixtures
    (tests/golden/memb_parity.json): counts, level sizes and per-action generated AND distinct
    counts (the handlers inside ReceiveDirect summed under that name)."""
    g = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))[case]
    r = host_bfs(generate(os.path.join(CONFIGS, "raft_membership_mc.tla"), os.path.join(CONFIGS, g["cfg"] + ".cfg")),
                 "--max-depth", str(g["max_depth"]), "--no-deadlock")
    assert r["err"] == 0 and r["verdict"] in ("DEPTH_LIMIT", "OK"), r["verdict"]
    assert (r["distinct"], r["depth"], r["levels"]) == (g["distinct"], g["depth"], g["levels"])
    want = memb_actions_as_generated(g["actions"])
    got = {k: v for k, v in r["actions"].items() if v[0]}
    assert {k: v[1] for k, v in got.items()} == {k: v[1] for k, v in want.items()}   # distinct: FIFO-sensitive
    # generated: the front end enumerates every true disjunct of a disjunction inside an action, as
    # TLC's getNextStates does; since round 5 the oracle emits those copies too
    # (HandleCheckOldConfig :796, HandleCatchupResponse :783-789), so every generated count is equal
    assert r["generated"] == g["generated"]
    assert {k: v[0] for k, v in got.items()} == {k: v[0] for k, v in want.items()}


@needs_tool
@pytest.mark.parametrize("cfg,inv", [("RecFun_fact", "FactNot24"), ("RecFun_sum", "SumNot7")])
def test_recursive_function_violations(cfg, inv):
    want = rec_fun(inv)
    r = host_bfs(generate(REC, os.path.join(CONFIGS, "tlagen", cfg + ".cfg")))
    assert (r["verdict"], r["violated"], r["depth"]) == ("INVARIANT_VIOLATION", inv, want["depth"])


@needs_tool
def test_invariant_evaluation_error():
    """An invariant that cannot be evaluated (Fact applied outside its domain 0..6) is TLC's
    "Evaluating invariant X failed" — an EVAL_ERROR verdict, not a violation."""
    r = host_bfs(generate(REC, os.path.join(CONFIGS, "tlagen", "RecFun_dom.cfg")))
    assert (r["verdict"], r["violated"], r["depth"]) == ("EVAL_ERROR", "OutOfDomain", 7)


# apalache_no_membership/raft.tla with its shipped raft.cfg (TLC syntax): the first spec of SURVEY.md
# 8(f) rank 3 that needs recursive function definitions (TypedBags' Sum via BagCardinality in
# BoundedInFlightMessages).  Pinned by the oracle's hand restatement of the spec
# (oracle/raft_apalache.h; tests/golden/apalache_oracle.json, tests/golden/make_apalache_oracle.py):
# the shipped model to depth 11 and the cfg's two commented-out test-case invariants.
APALACHE = json.load(open(os.path.join(GOLDEN, "apalache_oracle.json")))
APALACHE_D9 = dict(generated=141083, distinct=60955, levels=[1, 2, 6, 28, 120, 520, 2310, 10388, 47580])


@needs_tool
@needs_ref
def test_apalache_no_membership_shipped_cfg():
    """The host build of the generated code to depth 9: the oracle's level sizes (the first 9 levels of
    its depth-11 fixture; levels are order independent), counts, and every kept state (the state set
    of the oracle's own depth-9 run)."""
    spec = os.path.join(REF, "apalache_no_membership", "raft.tla")
    cfg = os.path.join(REF, "apalache_no_membership", "raft.cfg")
    dump = tempfile.mktemp(suffix=".txt")
    r = host_bfs(generate(spec, cfg), "--max-depth", "9", "--dump", dump)
    assert (r["verdict"], r["err"]) == ("DEPTH_LIMIT", 0)
    assert {k: r[k] for k in APALACHE_D9} == APALACHE_D9
    assert r["levels"] == APALACHE["shipped_d11"]["levels"][:9]
    got = sorted(l.rstrip("\n") for l in open(dump))
    os.unlink(dump)
    o = run_oracle("bfs", spec, os.path.join(CONFIGS, "apalache_nm.cfg"), "--max-depth", "9", "--dump", dump)
    want = sorted(l.rstrip("\n") for l in open(dump))
    os.unlink(dump)
    assert (o["generated"], o["distinct"], o["levels"]) == (APALACHE_D9["generated"], APALACHE_D9["distinct"], APALACHE_D9["levels"])
    assert got == want


@needs_tool
@needs_ref
@pytest.mark.parametrize("case", ["BoundedTrace", "FirstBecomeLeader"])
def test_apalache_counterexamples(case):
    """The shipped cfg's test-case invariants (raft.cfg:22-24) on the host build of the generated code:
    TLC's FIFO counterexample and its stop-point counters, as the oracle's restatement finds them."""
    g = APALACHE[case]
    spec = os.path.join(REF, "apalache_no_membership", "raft.tla")
    r = host_bfs(generate(spec, os.path.join(CONFIGS, g["cfg"] + ".cfg")), "--trace")
    assert (r["verdict"], r["violated"], r["depth"], r["distinct"]) == (g["verdict"], g["violated"], g["depth"], g["distinct"])
    assert r["generated"] == g["generated"]
    assert r["trace"] == [t["state"] for t in g["trace"]]


@needs_tool
def test_temporal_properties_refused(tmp_path):
    """A cfg with PROPERTY/PROPERTIES is refused on the generated path (as on the hand-compiled
    ones): the search checks safety only and must not report a liveness property as checked."""
    cfg = open(os.path.join(CONFIGS, "tlagen", "TokenRing.cfg")).read() + "\nPROPERTY Liveness\n"
    (tmp_path / "ring.cfg").write_text(cfg)
    r = subprocess.run([TOOL, RING, str(tmp_path / "ring.cfg")], capture_output=True, text=True)
    assert r.returncode != 0 and "PROPERTIES" in r.stderr, (r.returncode, r.stderr)


@needs_tool
@pytest.mark.parametrize("cfg,verdict,depth", [("Countdown", "DEADLOCK", 4), ("Countdown_evalerr", "EVAL_ERROR", 3)])
def test_countdown_verdicts(cfg, verdict, depth):
    """TLC's other verdict classes on the generated path: a state without successors (deadlock,
    checked by default) and a sequence read past its end while computing successors."""
    r = host_bfs(generate(os.path.join(CONFIGS, "tlagen", "Countdown.tla"), os.path.join(CONFIGS, "tlagen", cfg + ".cfg")))
    assert (r["verdict"], r["depth"], r["distinct"]) == (verdict, depth, depth)


FUNSETS = os.path.join(CONFIGS, "tlagen", "FunSets.tla")


def funsets_model():
    """configs/tlagen/FunSets.tla restated in Python (S = {s1, s2}): TLC's generated / distinct counts and
    level sizes of the whole space, and the BFS depth at which each negative control first fails."""
    def succ(st):
        f, r, q = st
        out = []
        for i in range(2):
            if f[i] < 2:
                out.append((tuple(x + (j == i) for j, x in enumerate(f)), r, q))
        if r[0] < 2:
            out.append((f, (r[0] + 1, r[1]), q))
        out.append(((1, 1), r, q))
        if len(q) < 2:
            out.append((f, r, q + (r,)))
        return out
    ok = {"FBelow2": lambda st: max(st[0]) <= 1, "RBelow2": lambda st: st[1][0] <= 1, "QEmpty": lambda st: not st[2]}
    level = [((0, 0), (0, b), ()) for b in (False, True)]
    seen, gen, levels, first, depth = set(level), len(level), [len(level)], {}, 1
    while level:
        nxt = []
        for st in level:
            for t in succ(st):
                gen += 1
                if t not in seen:
                    seen.add(t)
                    nxt.append(t)
        depth += 1
        for k, f in ok.items():
            if k not in first and any(not f(t) for t in nxt):
                first[k] = depth
        if nxt:
            levels.append(len(nxt))
        level = nxt
    return {"generated": gen, "distinct": len(seen), "depth": len(levels), "levels": levels, "first_violation": first}


@needs_tool
def test_function_and_record_sets():
    """[S -> T] and [f : S, ...] on the generated path: as values (Init's choices, \\E over a function
    set: fun_set / rec_set) and in membership tests that never build the set (TypeOK-style: [S -> Nat],
    Seq([a : 0..2, b : {FALSE, TRUE}]), a filter over Nat, \\subseteq a record set over Nat, \\notin).
    TypeOK holds in every state, and the whole space equals the Python restatement's counts."""
    want = funsets_model()
    r = host_bfs(generate(FUNSETS, os.path.join(CONFIGS, "tlagen", "FunSets.cfg")))
    assert (r["verdict"], r["err"]) == ("OK", 0)
    assert {k: r[k] for k in ("generated", "distinct", "depth", "levels")} == {k: want[k] for k in ("generated", "distinct", "depth", "levels")}


@needs_tool
@pytest.mark.parametrize("inv", ["FBelow2", "RBelow2", "QEmpty"])
def test_function_set_negative_controls(inv):
    """Each negative control (f \\in [S -> 0..1], r \\in [a : 0..1, b : BOOLEAN], q \\in [{} -> Cell]) is
    violated at the first depth where the Python restatement has a state outside it."""
    r = host_bfs(generate(FUNSETS, os.path.join(CONFIGS, "tlagen", "FunSets_%s.cfg" % inv)))
    assert (r["verdict"], r["violated"], r["depth"]) == ("INVARIANT_VIOLATION", inv, funsets_model()["first_violation"][inv])


@needs_tool
@needs_ref
def test_ricketts_type_invariant():
    """Ricketts' full type invariant (raft_dricketts.tla:482-492, the TLAPS proof's TypeOK: [Server -> Nat],
    Seq([term : Nat, value : Value]), [Server -> [Server -> {n \\in Nat : 1 <= n}]], SUBSET Server, and the
    messages' record types under \\subseteq) checked by the generated code: it holds in every state to depth
    12, whose counts stay the oracle's; its negative control BadTerm fails at the first Timeout."""
    r = host_bfs(generate(os.path.join(CONFIGS, "ricketts_mc.tla"), os.path.join(CONFIGS, "ricketts_typeok.cfg")), "--max-depth", "12")
    assert (r["verdict"], r["err"]) == ("DEPTH_LIMIT", 0)
    assert {k: r[k] for k in RICKETTS_D12} == RICKETTS_D12
    r = host_bfs(generate(os.path.join(CONFIGS, "ricketts_mc.tla"), os.path.join(CONFIGS, "ricketts_badterm.cfg")))
    assert (r["verdict"], r["violated"], r["depth"]) == ("INVARIANT_VIOLATION", "BadTerm", 2)


def strip_history_global(state_line):
    """The oracle's membership state text leaves out history["global"] (its dump_line; the record
    it keeps per state is the rank summary, oracle/raft_membership.h): drop the field to compare."""
    a = state_line.index("global |-> ")
    b = state_line.index(", hadNumClientRequests", a)
    return state_line[:a] + state_line[b + 2:]


@needs_tool
@needs_ref
def test_generated_punctuated_search():
    """The reference's punctuated search (tlc_membership/raft.tla:1212-1234): the state constraint
    MajorityOfClusterRestarts_constraint holds history["global"] to a prefix of the golden TLC trace
    pasted into raft.tla itself, evaluated by the generated code from the spec's own text (IsPrefix,
    SubSeq, \\E over three servers).  TLC's counters at the stop point and the counterexample, state by
    state, equal the oracle's (tests/golden/memb_parity.json); the GPU test adds the
    CommitWhenConcurrentLeaders search, whose cfg also has an ACTION_CONSTRAINT."""
    g = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))["punct_MajorityOfClusterRestarts"]
    r = host_bfs(generate(os.path.join(CONFIGS, "raft_membership_mc.tla"), os.path.join(CONFIGS, g["cfg"] + ".cfg")),
                 "--no-deadlock", "--trace")
    assert (r["verdict"], r["violated"], r["generated"], r["distinct"], r["depth"]) == \
        (g["verdict"], g["violated"], g["generated"], g["distinct"], g["depth"])
    assert [strip_history_global(x) for x in r["trace"]] == [t["state"] for t in g["trace"]]


# Ricketts' spec (thirdparty/raft_dricketts.tla, TLAPS-proved, no TLC cfg in the reference) on the
# generated path through configs/ricketts_mc.tla, pinned by the oracle's hand restatement of it
# (oracle/raft_dricketts.h; tests/golden/ricketts_oracle.json, tests/golden/make_ricketts_oracle.py).
RICKETTS = json.load(open(os.path.join(GOLDEN, "ricketts_oracle.json")))
RICKETTS_D12 = {k: RICKETTS["c1_d12"][k] for k in ("generated", "distinct", "levels")}


def generated_actions(acts):
    """The generated path's per-action counts without the never-taken entry "Next" (the action name
    TLC gives a Next with no split point; Ricketts' Next is a disjunction, so it never fires)."""
    return {k: v for k, v in acts.items() if not (k == "Next" and v == [0, 0])}


@needs_tool
@needs_ref
def test_ricketts_depth_limited():
    """To depth 12: generated, distinct, level sizes and per-action (generated, distinct) counts.
    Ricketts' Next is a disjunction: TLC splits it into its actions; inside Receive, UpdateTerm(i, j, m)
    is a disjunct of its own, `m.mtype = .. /\\ Handle..(i, j, m)` is a conjunction (named Receive) --
    the oracle counts its handlers under the same names."""
    g = RICKETTS["c1_d12"]
    r = host_bfs(generate(os.path.join(CONFIGS, "ricketts_mc.tla"), os.path.join(CONFIGS, "ricketts_c1.cfg")), "--max-depth", "12")
    assert (r["verdict"], r["err"]) == ("DEPTH_LIMIT", 0)
    assert {k: r[k] for k in RICKETTS_D12} == RICKETTS_D12
    assert generated_actions(r["actions"]) == g["actions"]


@needs_tool
@needs_ref
@pytest.mark.parametrize("case,verdict,violated", [("noleader", "INVARIANT_VIOLATION", "NoLeader"),
                                                   ("election_safety", "EVAL_ERROR", "ElectionSafety")])
def test_ricketts_stop_points(case, verdict, violated):
    """NoLeader's counterexample, and ElectionSafety's evaluation error (Max({}) = CHOOSE over the
    empty set, raft_dricketts.tla:106-108, once a leader has no entry of its own term,
    :1123-1128): both at the first leader, depth 10, with the oracle's trace state by state and
    distinct count at the stop point."""
    g = RICKETTS[case]
    r = host_bfs(generate(os.path.join(CONFIGS, "ricketts_mc.tla"), os.path.join(CONFIGS, g["cfg"] + ".cfg")), "--trace")
    assert (r["verdict"], r["violated"], r["depth"]) == (verdict, violated, g["depth"])
    assert (g["verdict"], g["distinct"]) == (verdict, r["distinct"])
    assert r["trace"] == [t["state"] for t in g["trace"]]


@needs_tool
def test_generated_source_is_deterministic():
    """The code-object cache is keyed by the generated source: generating twice gives the same text,
    and the build's prebuilt TokenRing code object is the one the library looks up (the GPU box runs
    the front end on TokenRing.tla itself and must hit it)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("prebuild", os.path.join(ROOT, "raft-tla_amd", "csrc", "tlagen", "prebuild.py"))
    pb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pb)
    outs = []
    for _ in range(2):
        fd, out = tempfile.mkstemp(suffix=".gen.hip")
        os.close(fd)
        subprocess.run([TOOL, RING, os.path.join(CONFIGS, "tlagen", "TokenRing.cfg"), "--kernels", "-o", out], check=True)
        outs.append(open(out).read())
        os.unlink(out)
    assert outs[0] == outs[1]
    co = os.path.join(pb.OUT, pb.key_of(outs[0]) + ".hsaco")
    if os.path.isdir(pb.OUT):
        assert os.path.exists(co), co


HIGHER = os.path.join(CONFIGS, "tlagen", "HigherOrder.tla")


def higher_order_model():
    """configs/tlagen/HigherOrder.tla restated in Python: s grows by one of 0..2 up to length 3, or drops
    every copy of its head (Remove) while n accumulates the head mod 3; TLC's generated / distinct counts,
    level sizes, and the depth at which each negative control first fails."""
    def succ(st):
        s, n = st
        out = [(s + (v,), n) for v in range(3)] if len(s) < 3 else []
        if s:
            out.append((tuple(x for x in s if x != s[0]), (n + s[0]) % 3))
        return out
    ok = {"FewZeros": lambda st: st[0].count(0) < 2, "NBelow2": lambda st: st[1] < 2}
    level = [((), 0)]
    seen, gen, levels, first, depth = set(level), 1, [1], {}, 1
    while level:
        nxt = []
        for st in level:
            for t in succ(st):
                gen += 1
                if t not in seen:
                    seen.add(t)
                    nxt.append(t)
        depth += 1
        for k, f in ok.items():
            if k not in first and any(not f(t) for t in nxt):
                first[k] = depth
        if nxt:
            levels.append(len(nxt))
        level = nxt
    return {"generated": gen, "distinct": len(seen), "depth": len(levels), "levels": levels, "first_violation": first}


@needs_tool
def test_higher_order_operators():
    """Operators with operator parameters (Count(q, P(_)), Fold2(F(_, _), x, y)), LAMBDA and SelectSeq on
    the generated path; the operator arguments are a LAMBDA of one and of two parameters, a global
    operator by name, a LET operator, a standard-module operator (Append) and an operator parameter passed
    on.  TypeOK's identities hold in every state, and the whole space equals the Python restatement's."""
    want = higher_order_model()
    r = host_bfs(generate(HIGHER, os.path.join(CONFIGS, "tlagen", "HigherOrder.cfg")))
    assert (r["verdict"], r["err"]) == ("OK", 0)
    assert {k: r[k] for k in ("generated", "distinct", "depth", "levels")} == {k: want[k] for k in ("generated", "distinct", "depth", "levels")}


@needs_tool
@pytest.mark.parametrize("inv", ["FewZeros", "NBelow2"])
def test_higher_order_negative_controls(inv):
    r = host_bfs(generate(HIGHER, os.path.join(CONFIGS, "tlagen", "HigherOrder_%s.cfg" % inv)))
    assert (r["verdict"], r["violated"], r["depth"]) == ("INVARIANT_VIOLATION", inv, higher_order_model()["first_violation"][inv])


@needs_tool
def test_higher_order_refusals(tmp_path):
    """Outside the subset, refused with the definition's location: a LAMBDA as a value, an operator
    argument of the wrong arity, a value passed for an operator parameter, a recursive higher-order
    operator."""
    body = {"lambda_value": "Bad == (LAMBDA x : x) = 1",
            "arity": "Bad == Count(<<1>>, Fold2)",
            "value_arg": "Bad == LET v == 1 IN Count(<<1>>, v)",
            "recursive": "Rec(F(_), k) == IF k = 0 THEN F(0) ELSE Rec(F, k - 1)\nBad == Rec(IsEven, 2)"}
    for name, text in body.items():
        spec = tmp_path / ("Ref_%s.tla" % name)
        spec.write_text("---- MODULE Ref_%s ----\nEXTENDS Naturals, Sequences\nVARIABLE s\n"
                        "Count(q, P(_)) == Len(SelectSeq(q, P))\nFold2(F(_, _), x, y) == F(x, y)\nIsEven(x) == x %% 2 = 0\n"
                        "%s\nInit == s = 0\nNext == s' = s\nInv == Bad\n====\n" % (name, text))
        cfg = tmp_path / "Ref.cfg"
        cfg.write_text("INIT Init\nNEXT Next\nINVARIANT Inv\n")
        r = subprocess.run([TOOL, str(spec), str(cfg), "-o", str(tmp_path / "x.gen.h")], capture_output=True, text=True)
        assert r.returncode != 0 and "outside the front end's subset" in r.stderr, (name, r.stderr)


@needs_tool
@needs_ref
@pytest.mark.parametrize("cfg,verdict,depth,distinct", [("SeqRemove", "OK", 4, 40), ("SeqRemove_NoRepeat", "INVARIANT_VIOLATION", 3, 5)])
def test_sequences_ext_remove(tmp_path, cfg, verdict, depth, distinct):
    """The reference's own SequencesExt Remove (apalache_no_membership/SequencesExt.tla:66-68, a SelectSeq
    over a LAMBDA) through the generated path: sequences over 0..2 of length <= 3 (1 + 3 + 9 + 27 states,
    4 levels), Remove drops every copy of its argument; the negative control fails on <<0, 0>> at depth 3."""
    out = str(tmp_path / "r.gen.h")
    r = subprocess.run([TOOL, os.path.join(CONFIGS, "tlagen", "SeqRemove.tla"), os.path.join(CONFIGS, "tlagen", cfg + ".cfg"),
                        "-I", os.path.join(REF, "apalache_no_membership"), "-o", out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = host_bfs(out)
    assert (r["verdict"], r["depth"], r["distinct"], r["err"]) == (verdict, depth, distinct, 0)


RECURSIVE_OPS = os.path.join(CONFIGS, "tlagen", "Recursive.tla")


def recursive_ops_model():
    """configs/tlagen/Recursive.tla restated in Python: s grows by one of 0..3 up to length 3, then drops
    its head; TLC's generated / distinct counts and level sizes, and SumBelow4's first failing depth."""
    level = [()]
    seen, gen, levels, first, depth = set(level), 1, [1], None, 1
    while level:
        nxt = []
        for st in level:
            for t in ([st + (v,) for v in range(4)] if len(st) < 3 else [st[1:]]):
                gen += 1
                if t not in seen:
                    seen.add(t)
                    nxt.append(t)
        depth += 1
        if first is None and any(sum(t) >= 4 for t in nxt):
            first = depth
        if nxt:
            levels.append(len(nxt))
        level = nxt
    return {"generated": gen, "distinct": len(seen), "depth": len(levels), "levels": levels, "sum_below4": first}


@needs_tool
def test_recursive_operators():
    """RECURSIVE operators: self-recursive (SumSeq over a sequence, Fact) and mutually recursive (IsEven /
    IsOdd) on the generated path; Inv's identities hold in every state and the whole space equals the
    Python restatement's; the negative control fails at its depth; a runaway recursion (Fact(-1)) is an
    evaluation error at the recursion bound (kMaxRecDepth), like TLC's stack overflow, never a hang."""
    want = recursive_ops_model()
    r = host_bfs(generate(RECURSIVE_OPS, os.path.join(CONFIGS, "tlagen", "Recursive.cfg")))
    assert (r["verdict"], r["err"]) == ("OK", 0)
    assert {k: r[k] for k in ("generated", "distinct", "depth", "levels")} == {k: want[k] for k in ("generated", "distinct", "depth", "levels")}
    r = host_bfs(generate(RECURSIVE_OPS, os.path.join(CONFIGS, "tlagen", "Recursive_SumBelow4.cfg")))
    assert (r["verdict"], r["violated"], r["depth"]) == ("INVARIANT_VIOLATION", "SumBelow4", want["sum_below4"])
    r = host_bfs(generate(RECURSIVE_OPS, os.path.join(CONFIGS, "tlagen", "Recursive_Runaway.cfg")))
    assert (r["verdict"], r["violated"], r["depth"]) == ("EVAL_ERROR", "Runaway", 1)


PRODUCT = os.path.join(CONFIGS, "tlagen", "Product.tla")


def product_model():
    """configs/tlagen/Product.tla restated in Python: p a pair of {0, 1} x {0, 1, 2} whose first component
    flips, q a triple over {0, 1} whose sum grows by one; counts, level sizes and QSumBelow2's depth."""
    import itertools

    def succ(st):
        p, q = st
        out = [((a, b), q) for a in (0, 1) for b in (0, 1, 2) if a != p[0]]
        return out + [(p, t) for t in itertools.product((0, 1), repeat=3) if sum(t) == sum(q) + 1]
    level = [((a, b), (0, 0, 0)) for a in (0, 1) for b in (0, 1, 2)]
    seen, gen, levels, first, depth = set(level), len(level), [len(level)], None, 1
    while level:
        nxt = []
        for st in level:
            for t in succ(st):
                gen += 1
                if t not in seen:
                    seen.add(t)
                    nxt.append(t)
        depth += 1
        if first is None and any(sum(t[1]) >= 2 for t in nxt):
            first = depth
        if nxt:
            levels.append(len(nxt))
        level = nxt
    return {"generated": gen, "distinct": len(seen), "depth": len(levels), "levels": levels, "qsum_below2": first}


@needs_tool
def test_cartesian_products_and_tuple_binds():
    """S \\X T (n-ary: A \\X B \\X C is a set of triples, (A \\X B) \\X C of pairs) and tuple-bound
    quantifiers (\\E <<a, b>> \\in S in an action, \\A <<x, y, z>> in an invariant, a map over a tuple
    binding): Inv holds in every state, the whole space equals the Python restatement's, and the
    negative control fails at its depth."""
    want = product_model()
    r = host_bfs(generate(PRODUCT, os.path.join(CONFIGS, "tlagen", "Product.cfg")))
    assert (r["verdict"], r["err"]) == ("OK", 0)
    assert {k: r[k] for k in ("generated", "distinct", "depth", "levels")} == {k: want[k] for k in ("generated", "distinct", "depth", "levels")}
    r = host_bfs(generate(PRODUCT, os.path.join(CONFIGS, "tlagen", "Product_QSumBelow2.cfg")))
    assert (r["verdict"], r["violated"], r["depth"]) == ("INVARIANT_VIOLATION", "QSumBelow2", want["qsum_below2"])
