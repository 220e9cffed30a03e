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


def test_higher_order_operators_on_gpu(raftmc):
    """Operator parameters, LAMBDA and SelectSeq (configs/tlagen/HigherOrder.tla) on the GPU, both
    pipelines: the Python restatement's counts for the whole space, and a negative control's depth."""
    from test_tlagen import higher_order_model
    want = higher_order_model()
    spec = os.path.join(CONFIGS, "tlagen", "HigherOrder.tla")
    for workers in (1, 0):
        with raftmc.ModelChecker(spec, os.path.join(CONFIGS, "tlagen", "HigherOrder.cfg"), workers=workers, **SMALL) as mc:
            r = mc.run()
        assert r.verdict == "OK", r.error
        assert (r.generated, r.distinct, r.depth, [lv[0] for lv in r.levels]) == (want["generated"], want["distinct"], want["depth"], want["levels"])
    with raftmc.ModelChecker(spec, os.path.join(CONFIGS, "tlagen", "HigherOrder_FewZeros.cfg"), workers=1, **SMALL) as mc:
        r = mc.run()
    assert (r.verdict, r.depth) == ("INVARIANT_VIOLATION", want["first_violation"]["FewZeros"])


def test_recursive_operators_on_gpu(raftmc):
    """RECURSIVE operators (configs/tlagen/Recursive.tla: self- and mutually recursive) on the GPU, both
    pipelines: the Python restatement's counts; a runaway recursion ends as an evaluation error."""
    from test_tlagen import recursive_ops_model
    want = recursive_ops_model()
    spec = os.path.join(CONFIGS, "tlagen", "Recursive.tla")
    for workers in (1, 0):
        with raftmc.ModelChecker(spec, os.path.join(CONFIGS, "tlagen", "Recursive.cfg"), workers=workers, **SMALL) as mc:
            r = mc.run()
        assert r.verdict == "OK", r.error
        assert (r.generated, r.distinct, r.depth, [lv[0] for lv in r.levels]) == (want["generated"], want["distinct"], want["depth"], want["levels"])
    with raftmc.ModelChecker(spec, os.path.join(CONFIGS, "tlagen", "Recursive_Runaway.cfg"), workers=1, **SMALL) as mc:
        r = mc.run()
    assert (r.verdict, r.violated, r.depth) == ("EVAL_ERROR", "Runaway", 1)


def test_cartesian_products_on_gpu(raftmc):
    """S \\X T and tuple-bound quantifiers (configs/tlagen/Product.tla) on the GPU, both pipelines: the
    Python restatement's counts for the whole space."""
    from test_tlagen import product_model
    want = product_model()
    for workers in (1, 0):
        with raftmc.ModelChecker(os.path.join(CONFIGS, "tlagen", "Product.tla"), os.path.join(CONFIGS, "tlagen", "Product.cfg"),
                                 workers=workers, **SMALL) as mc:
            r = mc.run()
        assert r.verdict == "OK", r.error
        assert (r.generated, r.distinct, r.depth, [lv[0] for lv in r.levels]) == (want["generated"], want["distinct"], want["depth"], want["levels"])


def test_function_and_record_sets_on_gpu(raftmc):
    """[S -> T] / [f : S, ...] as values and as lazily tested sets (configs/tlagen/FunSets.tla) on the GPU:
    the Python restatement's counts for the whole space (TypeOK holding), a negative control's depth;
    Ricketts' TypeOK to depth 12 with the oracle's counts, and its negative control BadTerm."""
    from test_tlagen import RICKETTS_D12, funsets_model
    want = funsets_model()
    for workers in (1, 0):
        with raftmc.ModelChecker(os.path.join(CONFIGS, "tlagen", "FunSets.tla"), os.path.join(CONFIGS, "tlagen", "FunSets.cfg"),
                                 workers=workers, **SMALL) as mc:
            r = mc.run()
        assert r.verdict == "OK", r.error
        assert (r.generated, r.distinct, r.depth, [lv[0] for lv in r.levels]) == (want["generated"], want["distinct"], want["depth"], want["levels"])
    for inv in ("FBelow2", "QEmpty"):
        with raftmc.ModelChecker(os.path.join(CONFIGS, "tlagen", "FunSets.tla"), os.path.join(CONFIGS, "tlagen", "FunSets_%s.cfg" % inv),
                                 workers=1, **SMALL) as mc:
            r = mc.run()
        assert (r.verdict, r.violated, r.depth) == ("INVARIANT_VIOLATION", inv, want["first_violation"][inv]), r.error
    with raftmc.ModelChecker(gen_source("ricketts_typeok"), os.path.join(CONFIGS, "ricketts_typeok.cfg"), frontend="generated",
                             workers=1, max_depth=12, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "DEPTH_LIMIT", r.error
    assert {"generated": r.generated, "distinct": r.distinct, "levels": [lv[0] for lv in r.levels]} == RICKETTS_D12
    with raftmc.ModelChecker(gen_source("ricketts_badterm"), os.path.join(CONFIGS, "ricketts_badterm.cfg"), frontend="generated",
                             workers=1, **SMALL) as mc:
        r = mc.run()
    assert (r.verdict, r.violated, r.depth) == ("INVARIANT_VIOLATION", "BadTerm", 2), r.error


def test_ricketts_on_gpu(raftmc):
    """thirdparty/raft_dricketts.tla (Bags module, TLAPS-only in the reference) through the generated
    path, pinned by the oracle's restatement (tests/golden/ricketts_oracle.json): to depth 12 with
    per-action counts; NoLeader's counterexample and ElectionSafety's evaluation error (Max({}))
    with TLC's counters at the stop point and the oracle's trace; the whole space of ricketts_safety
    (1,542,177 states, depth 49) with its three election/log invariants holding."""
    from test_gpu import trace_states
    from test_tlagen import RICKETTS, generated_actions
    g = RICKETTS["c1_d12"]
    with raftmc.ModelChecker(gen_source("ricketts_c1"), os.path.join(CONFIGS, "ricketts_c1.cfg"), frontend="generated",
                             workers=1, max_depth=12, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "DEPTH_LIMIT", r.error
    assert (r.generated, r.distinct, [lv[0] for lv in r.levels]) == (g["generated"], g["distinct"], g["levels"])
    assert generated_actions({k: list(v) for k, v in r.actions.items()}) == g["actions"]
    for case, verdict, violated in (("noleader", "INVARIANT_VIOLATION", "NoLeader"), ("election_safety", "EVAL_ERROR", "ElectionSafety")):
        g = RICKETTS[case]
        for workers in (1, 0):   # -workers N: the event is searched again in FIFO order
            with raftmc.ModelChecker(gen_source("ricketts_" + case), os.path.join(CONFIGS, g["cfg"] + ".cfg"), frontend="generated",
                                     workers=workers, **SMALL) as mc:
                r = mc.run()
            assert (r.verdict, r.violated, r.depth) == (verdict, violated, g["depth"]), r.error
            assert (r.generated, r.distinct, r.left_on_queue) == (g["generated"], g["distinct"], g["left_on_queue"])
            assert [x for _, x in trace_states(r)] == [t["state"] for t in g["trace"]]
    g = RICKETTS["safety"]
    with raftmc.ModelChecker(gen_source("ricketts_safety"), os.path.join(CONFIGS, "ricketts_safety.cfg"), frontend="generated",
                             workers=1, fp_table_bytes=1 << 28, state_store_bytes=8 << 30) as mc:
        r = mc.run()
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth, [lv[0] for lv in r.levels]) == (g["generated"], g["distinct"], g["depth"], g["levels"])
    assert generated_actions({k: list(v) for k, v in r.actions.items()}) == g["actions"]


@pytest.mark.parametrize("case,gen", [("punct_MajorityOfClusterRestarts", "memb_morc_gen"),
                                      ("punct_CommitWhenConcurrentLeaders", "memb_cwcl_gen")])
def test_generated_punctuated_search_on_gpu(raftmc, case, gen):
    """The reference's punctuated searches on the unmodified tlc_membership/raft.tla through the
    generated path: the golden-trace prefix constraints of raft.tla:1198-1234 and (CWCL) the
    ACTION_CONSTRAINT CommitWhenConcurrentLeaders_action_constraint, in TLC's FIFO order: TLC's
    counters at the stop point and the counterexample state by state equal the oracle's."""
    from test_gpu import trace_states
    from test_tlagen import strip_history_global
    g = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))[case]
    # states carry history["global"] (up to 28 records): ~6 KB of words each
    with raftmc.ModelChecker(gen_source(gen), os.path.join(CONFIGS, g["cfg"] + ".cfg"), frontend="generated", workers=1,
                             deadlock=False, fp_table_bytes=1 << 26, state_store_bytes=8 << 30) as mc:
        r = mc.run()
    assert (r.verdict, r.violated, r.depth, r.distinct) == (g["verdict"], g["violated"], g["depth"], g["distinct"]), r.error
    assert r.generated == g["generated"]   # TLC's disjunct copies on both sides (MC_COMPAT_DISJUNCT_COPIES)
    assert [strip_history_global(x) for _, x in trace_states(r)] == [t["state"] for t in g["trace"]]


def test_generated_fifo_trace_equals_oracle(raftmc):
    """TLC's single-worker FIFO order on the generated path (workers=1: two passes per level, the
    minimum (parent rank, successor ordinal) key kept per fingerprint, tlagen_kernels.h): the
    NoLeader counterexample of the unmodified raft_original.tla equals the oracle's state by state
    (tests/golden/orig_events.json), and so do TLC's counters at the stop point.  raft_original's
    Next is one conjunction, so every step is the action "Next" (the oracle names the handler)."""
    from test_gpu import trace_states
    g = json.load(open(os.path.join(GOLDEN, "orig_events.json")))["c2_noleader"]
    for workers in (1, 0):   # -workers N: the event is searched again in FIFO order
        with raftmc.ModelChecker(gen_source("c2_noleader"), os.path.join(CONFIGS, "c2_noleader.cfg"), frontend="generated",
                                 workers=workers, fp_table_bytes=1 << 28, state_store_bytes=16 << 30) as mc:
            r = mc.run()
        assert (r.verdict, r.violated, r.depth, r.exit_code) == ("INVARIANT_VIOLATION", "NoLeader", g["depth"], 12), r.error
        assert (r.generated, r.distinct, r.left_on_queue) == (g["generated"], g["distinct"], g["left_on_queue"])
        assert [lv[0] for lv in r.levels] == g["levels"]
        assert [s for _, s in trace_states(r)] == [t["state"] for t in g["trace"]]


@pytest.mark.parametrize("workers", [1, 0])
def test_generated_parity_both_orders(raftmc, workers):
    """raft_original has no VIEW: the FIFO two-pass search and the -workers N one give the oracle's
    counts (parity_pair, tests/golden/orig_parity.json), and the FIFO one its per-level sizes."""
    g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))["parity_pair"]
    with raftmc.ModelChecker(gen_source("parity_pair"), os.path.join(CONFIGS, "parity_pair.cfg"), frontend="generated",
                             workers=workers, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth, [lv[0] for lv in r.levels]) == (g["generated"], g["distinct"], g["depth"], g["levels"])


def test_view_fifo_on_gpu(raftmc):
    """TLC's VIEW on the GPU in TLC's FIFO order (TokenRing_view.cfg): counts, levels and per-action
    generated AND distinct counts of the Python restatement -- which state of a view class is kept
    (the first found) decides its successors."""
    want = token_ring(view=True)
    with raftmc.ModelChecker(gen_source("toy_ring_view"), os.path.join(CONFIGS, "tlagen", "TokenRing_view.cfg"),
                             frontend="generated", workers=1, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth, [lv[0] for lv in r.levels]) == (want["generated"], want["distinct"], want["depth"], want["levels"])
    for a, v in want["actions"].items():
        assert r.actions[a] == v, a


@pytest.mark.parametrize("workers", [1, 0])
def test_recursive_functions_on_gpu(raftmc, workers):
    """Recursive function definitions evaluated on the device (TypedBags' Sum form; RecFun.tla):
    the Python restatement's counts, its violation depths, and TLC's evaluation error for an
    invariant applied outside the function's domain."""
    from tlagen_models import rec_fun
    rec = os.path.join(CONFIGS, "tlagen", "RecFun.cfg")
    want = rec_fun()
    with raftmc.ModelChecker(gen_source("rec_fun"), rec, frontend="generated", workers=workers, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth, [lv[0] for lv in r.levels]) == (want["generated"], want["distinct"], want["depth"], want["levels"])
    for name, inv in (("rec_fun_fact", "FactNot24"), ("rec_fun_sum", "SumNot7")):
        with raftmc.ModelChecker(gen_source(name), os.path.join(CONFIGS, "tlagen", name.replace("rec_fun", "RecFun") + ".cfg"),
                                 frontend="generated", workers=workers, **SMALL) as mc:
            r = mc.run()
        assert (r.verdict, r.violated, r.depth) == ("INVARIANT_VIOLATION", inv, rec_fun(inv)["depth"])
    with raftmc.ModelChecker(gen_source("rec_fun_dom"), os.path.join(CONFIGS, "tlagen", "RecFun_dom.cfg"), frontend="generated",
                             workers=workers, **SMALL) as mc:
        r = mc.run()
    assert (r.verdict, r.violated, r.depth, r.exit_code) == ("EVAL_ERROR", "OutOfDomain", 7, 75)


def test_apalache_no_membership_on_gpu(raftmc):
    """apalache_no_membership/raft.tla with its shipped raft.cfg (recursive Sum in the constraints),
    pinned by the oracle's restatement (oracle/raft_apalache.h, tests/golden/apalache_oracle.json): the
    shipped model to depth 11 (1.3M states of ~800 words, history["global"] included) -- counts, level
    sizes, per-action generated counts in both search orders, per-action distinct counts and the SHA-256
    of the whole kept state set in TLC's FIFO order."""
    import hashlib
    import tempfile
    from test_tlagen import APALACHE
    g = APALACHE["shipped_d11"]
    for workers in (1, 0):
        with raftmc.ModelChecker(gen_source("apalache_nm"), os.path.join(ROOT, "configs", "apalache_nm.cfg"), frontend="generated",
                                 workers=workers, max_depth=11, fp_table_bytes=1 << 28, state_store_bytes=24 << 30) as mc:
            r = mc.run()
            if workers == 1:
                fd, path = tempfile.mkstemp(suffix=".txt")
                os.close(fd)
                mc.dump_states(path)
                lines = sorted(l.rstrip("\n") for l in open(path))
                os.unlink(path)
                assert hashlib.sha256("\n".join(lines).encode()).hexdigest() == g["states_sha256"]
                assert {k: v for k, v in r.actions.items()} == g["actions"]
        assert r.verdict == "DEPTH_LIMIT", r.error
        assert (r.generated, r.distinct, r.left_on_queue, [lv[0] for lv in r.levels]) == (g["generated"], g["distinct"], g["left_on_queue"], g["levels"])
        assert {k: v[0] for k, v in r.actions.items()} == {k: v[0] for k, v in g["actions"].items()}


@pytest.mark.parametrize("case,gen", [("BoundedTrace", "apalache_nm_boundedtrace"), ("FirstBecomeLeader", "apalache_nm_firstbecomeleader")])
def test_apalache_counterexamples_on_gpu(raftmc, case, gen):
    """The shipped cfg's commented-out test-case invariants (raft.cfg:22-24, raft.tla:776-785) on the GPU:
    TLC's FIFO counterexample state by state and TLC's counters at the stop point, as the oracle's
    restatement finds them; -workers N searches the event's level again in FIFO order."""
    from test_gpu import trace_states
    from test_tlagen import APALACHE
    g = APALACHE[case]
    for workers in (1, 0):
        with raftmc.ModelChecker(gen_source(gen), os.path.join(CONFIGS, g["cfg"] + ".cfg"), frontend="generated",
                                 workers=workers, fp_table_bytes=1 << 26, state_store_bytes=4 << 30) as mc:
            r = mc.run()
        assert (r.verdict, r.violated, r.depth, r.exit_code) == (g["verdict"], g["violated"], g["depth"], 12), r.error
        assert (r.generated, r.distinct, r.left_on_queue) == (g["generated"], g["distinct"], g["left_on_queue"])
        assert [s for _, s in trace_states(r)] == [t["state"] for t in g["trace"]]


@pytest.mark.parametrize("case,gen", [("memb_nosym@13", "memb_nosym_gen"), ("tlc:membership_shipped@16", "memb_shipped_gen"),
                                      ("tlc:memb_two@16", "memb_two_gen")])
def test_generated_membership_on_gpu(raftmc, case, gen):
    """The unmodified tlc_membership/raft.tla through the generated path on the GPU, TLC's semantics in
    full (VIEW vars; SYMMETRY perms by TLC's rule; the single-worker FIFO order that decides which
    state of a view class is kept): the oracle's counts, level sizes and per-action distinct counts
    (tests/golden/memb_parity.json; "generated" as tests/test_tlagen.py explains)."""
    from test_tlagen import memb_actions_as_generated
    g = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))[case]
    with raftmc.ModelChecker(gen_source(gen), os.path.join(CONFIGS, g["cfg"] + ".cfg"), frontend="generated", workers=1,
                             deadlock=False, max_depth=g["max_depth"], **SMALL) as mc:
        r = mc.run()
    assert r.verdict in ("DEPTH_LIMIT", "OK"), r.error
    assert (r.distinct, r.depth, [lv[0] for lv in r.levels]) == (g["distinct"], g["depth"], g["levels"])
    want = memb_actions_as_generated(g["actions"])
    assert {k: v[1] for k, v in r.actions.items() if v[0]} == {k: v[1] for k, v in want.items()}
    assert r.generated == g["generated"]   # TLC's disjunct copies on both sides (MC_COMPAT_DISJUNCT_COPIES)
