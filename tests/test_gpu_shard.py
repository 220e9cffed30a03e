"""GPU tests of the sharded (multi-GPU) BFS through the C ABI.

On a one-GPU box the N>1 path runs as several ranks on cuda:0 with the gloo
backend (payloads staged through host memory); on a node, bench.py runs the
same code with RCCL.  The sharded result must equal the single-GPU result:
identical generated / distinct / depth and per-action generated counts, and
on a violation a shortest counterexample reassembled across ranks."""
import importlib
import json
import time
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle_util import CONFIGS, GOLDEN, MEMB_MC, ORIG_MC, tla_text

pytestmark = pytest.mark.gpu

SMALL = dict(fp_table_bytes=1 << 26, state_store_bytes=1 << 28)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = importlib.import_module("raft-tla_amd.shard")
    try:
        r = shard.check_sharded(ORIG_MC, cfg, rank, world, device_index=0, **kw)
        q.put((rank, r.verdict, r.generated, r.distinct, r.depth, {k: v[0] for k, v in r.actions.items()},
               r.violated, getattr(r, "trace_text", "")))
    except Exception as e:   # surface the error instead of hanging the parent
        q.put((rank, "ERROR: %r" % e, 0, 0, 0, {}, "", ""))
    dist.destroy_process_group()


def run_sharded(cfg, world, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, cfg, {**SMALL, **kw}, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return out


def test_sharded_world1_equals_single(raftmc):
    shard = importlib.import_module("raft-tla_amd.shard")
    cfg = os.path.join(CONFIGS, "parity_pair.cfg")
    g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))["parity_pair"]
    r = shard.check_sharded(ORIG_MC, cfg, 0, 1, **SMALL)
    assert (r.verdict, r.generated, r.distinct, r.depth) == ("OK", g["generated"], g["distinct"], g["depth"])
    assert {k: v[0] for k, v in r.actions.items()} == {k: v[0] for k, v in g["actions"].items()}


@pytest.mark.parametrize("name,world", [("parity_pair", 2), ("parity_trio", 2), ("parity_pair_neg", 3)])
def test_sharded_ranks_on_one_gpu(name, world):
    g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))[name]
    out = run_sharded(os.path.join(CONFIGS, name + ".cfg"), world)
    for rank, verdict, gen, dist_, depth, acts, _, _ in out:
        assert verdict == "OK", verdict
        assert (gen, dist_, depth) == (g["generated"], g["distinct"], g["depth"])
        assert acts == {k: v[0] for k, v in g["actions"].items()}


def test_sharded_violation_trace():
    out = run_sharded(os.path.join(CONFIGS, "scenario_first_leader.cfg"), 2)
    rank0 = out[0]
    assert rank0[1] == "INVARIANT_VIOLATION" and rank0[6] == "NoLeader"
    states = rank0[7].strip().split("\n\n")
    assert len(states) == 10                     # same shortest length as the single-GPU / oracle run
    assert states[0].startswith("State 1: <Initial predicate>")
    assert "<BecomeLeader>" in states[-1].split("\n")[0]


def _native_worker(port, q):
    """One rank with the nccl (RCCL) backend: the library's native level loop (mc_shard_run_rccl)
    over a one-rank communicator; RCCL refuses two ranks on one GPU, so N>1 runs only on a node."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    shard = importlib.import_module("raft-tla_amd.shard")
    out = {}
    try:
        for name, kw in (("parity_pair", SMALL), ("scenario_first_leader", SMALL), ("c2", {})):
            sc = shard.ShardedChecker(ORIG_MC, os.path.join(CONFIGS, name + ".cfg"), 0, 1, **kw)
            assert sc.transport == "rccl"
            runs = [sc.run() for _ in range(2)]      # the second run reuses the cached communicator
            sc.close()
            out[name] = [(r.verdict, r.generated, r.distinct, r.depth, {k: v[0] for k, v in r.actions.items()},
                          r.violated, getattr(r, "trace_text", "")) for r in runs]
    except Exception as e:
        out["error"] = repr(e)
    q.put(out)
    dist.destroy_process_group()


def test_native_rccl_loop_world1():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_native_worker, args=(_port(), q))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert "error" not in out, out.get("error")
    g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))["parity_pair"]
    for verdict, gen, dist_, depth, acts, _, _ in out["parity_pair"]:
        assert (verdict, gen, dist_, depth) == ("OK", g["generated"], g["distinct"], g["depth"])
        assert acts == {k: v[0] for k, v in g["actions"].items()}
    exact = json.load(open(os.path.join(GOLDEN, "c2_exact.json")))
    for verdict, gen, dist_, depth, acts, _, _ in out["c2"]:
        assert (verdict, gen, dist_, depth) == ("OK", exact["generated"], exact["distinct"], exact["depth"])
        assert acts == exact["actions_generated"]
    for verdict, _, _, _, _, violated, trace in out["scenario_first_leader"]:
        assert verdict == "INVARIANT_VIOLATION" and violated == "NoLeader"
        states = trace.strip().split("\n\n")
        assert len(states) == 10 and states[0].startswith("State 1: <Initial predicate>")
        assert "<BecomeLeader>" in states[-1].split("\n")[0]


def _slot_bytes(raftmc, cfg):
    with raftmc.ModelChecker(ORIG_MC, cfg) as mc:
        return mc.describe()["state_bytes_stored"] + 8


@pytest.mark.parametrize("name,world,small", [("c1", 2, False), ("parity_pair", 2, False), ("parity_trio", 3, False),
                                              ("parity_pair_neg", 3, True), ("parity_pair_big", 2, True),
                                              ("c2", 2, False), ("c2", 3, False)])
def test_native_loop_loopback(raftmc, name, world, small):
    """The native sharded level loop (the one that runs over RCCL on a node) with W = 2-3 ranks in
    one process on one GPU, the exchanges as device-to-device copies: every W > 1 branch — routing
    by fingerprint owner, the self segments read in place, per-source dedup / materialize / store
    launches, the level all-reduce — must reproduce the single-GPU counts exactly.  `small` stores
    force several chunk rounds per level, with ranks holding different frontier sizes."""
    shard = importlib.import_module("raft-tla_amd.shard")
    cfg = os.path.join(CONFIGS, name + ".cfg")
    if name == "c2":
        g = json.load(open(os.path.join(GOLDEN, "c2_exact.json")))
        want = (g["generated"], g["distinct"], g["depth"], g["actions_generated"])
        kw = dict(fp_table_bytes=2 << 30, state_store_bytes=2 << 30)
    else:
        g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))[name]
        want = (g["generated"], g["distinct"], g["depth"], {k: v[0] for k, v in g["actions"].items()})
        kw = dict(SMALL)
        if small:   # a store just big enough: chunks of a few thousand states, several per level
            kw["state_store_bytes"] = 3 * g["distinct"] * _slot_bytes(raftmc, cfg) // 2
    out = shard.check_loopback(ORIG_MC, cfg, world, **kw)
    assert len(out) == world
    for r in out:
        assert r.verdict == "OK", r.error
        assert (r.generated, r.distinct, r.depth, {k: v[0] for k, v in r.actions.items()}) == want
        assert [lv[0] for lv in r.levels] == [lv[0] for lv in out[0].levels]


def test_native_loop_loopback_counterexample(raftmc):
    """A violation found on one rank: the search stops on every rank at the same level, and the
    counterexample reassembled across the ranks' stores has the single-GPU shortest length."""
    shard = importlib.import_module("raft-tla_amd.shard")
    ev = json.load(open(os.path.join(GOLDEN, "orig_events.json")))["scenario_first_leader"]
    out = shard.check_loopback(ORIG_MC, os.path.join(CONFIGS, "scenario_first_leader.cfg"), 3, **SMALL)
    for r in out:
        assert r.verdict == "INVARIANT_VIOLATION" and r.violated == "NoLeader", r.error
        assert r.depth == ev["depth"]
    states = out[0].trace_text.strip().split("\n\n")
    assert len(states) == len(ev["trace"]) == 10
    assert states[0].startswith("State 1: <Initial predicate>")
    assert "<BecomeLeader>" in states[-1].split("\n")[0]


# ---------------------------------------------------------------- tlc_membership (FIFO-ranked sharding)
MEMB_FIX = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))
MSMALL = dict(fp_table_bytes=1 << 26, state_store_bytes=1 << 29, deadlock=False)


def _memb_worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = importlib.import_module("raft-tla_amd.shard")
    g = MEMB_FIX[case]
    prefixes = {}
    if g.get("prefix"):
        con, fixture = g["prefix"]
        prefixes[con] = tla_text(json.load(open(os.path.join(GOLDEN, fixture)))["value"])
    try:
        sc = shard.ShardedChecker(MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), rank, world, device_index=0,
                                  history_prefixes=prefixes, max_depth=g["max_depth"], sym_tlc=g.get("sym") == "tlc", **MSMALL)
        r = sc.run()
        dump = "%s.rank%d" % (os.environ["RAFTMC_DUMP"], rank)
        sc.mc.dump_states(dump)
        sc.close()
        q.put((rank, r.verdict, r.generated, r.distinct, r.depth, r.left_on_queue, r.actions, r.violated,
               getattr(r, "trace_text", ""), [lv[0] for lv in r.levels]))
    except Exception as e:
        q.put((rank, "ERROR: %r" % e, 0, 0, 0, 0, {}, "", "", []))
    dist.destroy_process_group()


def run_memb_sharded(case, world, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    os.environ["RAFTMC_DUMP"] = str(tmp_path / "dump")
    ps = [ctx.Process(target=_memb_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    lines = []
    for r in range(world):
        lines += [l.rstrip("\n") for l in open(str(tmp_path / "dump") + ".rank%d" % r)]
    return out, lines


@pytest.mark.parametrize("case,world", [("membership_shipped@14", 2), ("memb_dynamic3@14", 3), ("memb_four@10", 2),
                                        ("punct_MajorityOfClusterRestarts@30", 2), ("tlc:membership_shipped@16", 2),
                                        ("tlc:memb_four@13", 3)])
def test_membership_sharded_equals_fifo_fixture(case, world, tmp_path):
    """Sharded BFS with FIFO ranking across ranks: identical counts, per-action generated AND
    distinct counts, level sizes and set of kept states (first-found representatives) as the
    oracle's single-worker fixture."""
    import hashlib
    g = MEMB_FIX[case]
    out, lines = run_memb_sharded(case, world, tmp_path)
    for rank, verdict, gen, dist_, depth, left, acts, _, _, levels in out:
        assert verdict in ("OK", "DEPTH_LIMIT"), verdict
        assert (gen, dist_, depth, left) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
        assert acts == g["actions"]
        assert levels == g["levels"]
    assert len(lines) == g["distinct"]
    assert hashlib.sha256("\n".join(sorted(lines)).encode()).hexdigest() == g["states_sha256"]


@pytest.mark.parametrize("case,world", [("scen_FirstCommit", 2), ("punct_CommitWhenConcurrentLeaders", 3)])
def test_membership_sharded_counterexample(case, world, tmp_path):
    g = MEMB_FIX[case]
    out, _ = run_memb_sharded(case, world, tmp_path)
    for rank, verdict, gen, dist_, depth, left, acts, violated, trace, _ in out:
        assert verdict == "INVARIANT_VIOLATION" and violated == g["violated"], verdict
        assert (gen, dist_, depth, left) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
    blocks = out[0][8].strip().split("\n\n")
    assert len(blocks) == len(g["trace"]) == g["depth"]
    for k, (blk, ref) in enumerate(zip(blocks, g["trace"])):
        head, *body = blk.split("\n")
        assert " ".join(body) == ref["state"], "trace state %d differs" % (k + 1)
        if k:
            assert head == "State %d: <%s>" % (k + 1, ref["action"])


def _memb_prefixes(g):
    if not g.get("prefix"):
        return {}
    con, fixture = g["prefix"]
    return {con: tla_text(json.load(open(os.path.join(GOLDEN, fixture)))["value"])}


@pytest.mark.parametrize("case,world", [("membership_shipped@14", 2), ("memb_dynamic3@14", 3), ("tlc:memb_four@13", 2), ("tlc:memb_four_scale@15", 2),
                                        ("punct_MajorityOfClusterRestarts@30", 3)])
def test_membership_native_loop_loopback(case, world, tmp_path):
    """The FIFO-ranked sharded level loop in C++ (csrc/fifo_shard_loop.h, what mc_shard_run_rccl runs
    for tlc_membership on a node) with W ranks in one process on one GPU: the oracle's single-worker
    counts, per-action generated and distinct counts, level sizes and set of kept states."""
    import hashlib
    shard = importlib.import_module("raft-tla_amd.shard")
    g = MEMB_FIX[case]
    dump = str(tmp_path / "dump")
    out = shard.check_loopback(MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), world, history_prefixes=_memb_prefixes(g),
                               dump=dump, max_depth=g["max_depth"], sym_tlc=g.get("sym") == "tlc", **MSMALL)
    for r in out:
        assert r.verdict in ("OK", "DEPTH_LIMIT"), r.error
        assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
        assert r.actions == g["actions"]
        assert [lv[0] for lv in r.levels] == g["levels"]
    lines = []
    for k in range(world):
        lines += [l.rstrip("\n") for l in open("%s.rank%d" % (dump, k))]
    assert len(lines) == g["distinct"]
    assert hashlib.sha256("\n".join(sorted(lines)).encode()).hexdigest() == g["states_sha256"]


def _trace_blocks_match(trace_text, g):
    blocks = trace_text.strip().split("\n\n")
    assert len(blocks) == len(g["trace"]) == g["depth"]
    for k, (blk, ref) in enumerate(zip(blocks, g["trace"])):
        head, *body = blk.split("\n")
        assert " ".join(body) == ref["state"], "trace state %d differs" % (k + 1)
        if k:
            assert head.startswith("State %d: <%s" % (k + 1, ref["action"]))


@pytest.mark.parametrize("case,world", [("scen_FirstCommit", 3), ("punct_CommitWhenConcurrentLeaders", 2),
                                        ("eval:memb_eval_single", 2)])
def test_membership_native_loop_loopback_stop(case, world):
    """A stop found on some rank (invariant violation / evaluation error): TLC's stop-point counters
    all-reduced across ranks and the counterexample chased across the ranks' stores, state by state."""
    shard = importlib.import_module("raft-tla_amd.shard")
    g = MEMB_FIX[case]
    kw = dict(MSMALL, deadlock=g.get("deadlock", False))   # TLC's deadlock check as the fixture was searched
    out = shard.check_loopback(MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), world, history_prefixes=_memb_prefixes(g),
                               sym_tlc=g.get("sym") == "tlc", **kw)
    for r in out:
        assert r.verdict == g["verdict"], r.error
        assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
        if g["verdict"] == "INVARIANT_VIOLATION":
            assert r.violated == g["violated"]
    _trace_blocks_match(out[0].trace_text, g)


# ---------------------------------------------------------------- mc_opts.n_gpus (one process, one thread per GPU)
@pytest.mark.parametrize("name,world", [("c1", 2), ("parity_pair_neg", 3), ("c2", 2)])
def test_n_gpus_raft_original(raftmc, name, world):
    """mc_opts.n_gpus > 1 through plain mc_open / mc_run: the library's own multi-GPU search (one host
    thread per rank inside the library).  On a one-GPU box every rank shares cuda:0 (same_device,
    loopback device copies); on a node the ranks are GPUs 0..W-1 over an in-process RCCL
    communicator.  The single-GPU counts, every rank's share summed."""
    cfg = os.path.join(CONFIGS, name + ".cfg")
    if name == "c2":
        g = json.load(open(os.path.join(GOLDEN, "c2_exact.json")))
        want = (g["generated"], g["distinct"], g["depth"], g["actions_generated"])
        kw = dict(fp_table_bytes=2 << 30, state_store_bytes=2 << 30)
    else:
        g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))[name]
        want = (g["generated"], g["distinct"], g["depth"], {k: v[0] for k, v in g["actions"].items()})
        kw = dict(SMALL)
    ndev = torch.cuda.device_count()
    same = ndev < world
    with raftmc.ModelChecker(ORIG_MC, cfg, n_gpus=world, same_device=same, **kw) as mc:
        assert mc.describe()["n_gpus"] == world
        r = mc.run()
    assert r.verdict == "OK", r.error
    assert (r.generated, r.distinct, r.depth, {k: v[0] for k, v in r.actions.items()}) == want


def test_n_gpus_raft_original_counterexample(raftmc):
    ev = json.load(open(os.path.join(GOLDEN, "orig_events.json")))["scenario_first_leader"]
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "scenario_first_leader.cfg"), n_gpus=2,
                             same_device=torch.cuda.device_count() < 2, **SMALL) as mc:
        r = mc.run()
    assert r.verdict == "INVARIANT_VIOLATION" and r.violated == "NoLeader" and r.exit_code == 12, r.error
    assert r.depth == ev["depth"]
    states = r.trace_text.strip().split("\n\n")
    assert len(states) == len(ev["trace"]) == 10
    assert states[0].startswith("State 1: <Initial predicate>")
    assert "<BecomeLeader" in states[-1].split("\n")[0]
    assert "Error: Invariant NoLeader is violated." in r.report


@pytest.mark.parametrize("case,world", [("memb_four@10", 2), ("tlc:membership_shipped@16", 3), ("scen_FirstCommit", 2)])
def test_n_gpus_membership(raftmc, case, world):
    """n_gpus > 1 for tlc_membership (FIFO-ranked: TLC's single-worker kept representatives across
    ranks): the oracle fixture's counts and, for a stop, its counterexample."""
    g = MEMB_FIX[case]
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, g["cfg"] + ".cfg"), n_gpus=world,
                             same_device=torch.cuda.device_count() < world, max_depth=g.get("max_depth", 0),
                             sym_tlc=g.get("sym") == "tlc", **dict(MSMALL, deadlock=g.get("deadlock", False))) as mc:
        r = mc.run()
    assert r.verdict == g["verdict"] if g["verdict"] != "OK" or not g.get("max_depth") else r.verdict in ("OK", "DEPTH_LIMIT"), r.error
    assert (r.generated, r.distinct, r.depth, r.left_on_queue) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
    if g["verdict"] == "OK":
        assert r.actions == g["actions"]
        assert [lv[0] for lv in r.levels] == g["levels"]
    else:
        assert r.violated == g["violated"]
        _trace_blocks_match(r.trace_text, g)


# ---------------------------------------------------------------- count_final_level and rank failures in the native loop
def test_native_loop_count_final_level(raftmc, tmp_path):
    """count_final_level in the sharded native loop (BASELINE configs[4]: C5v2 to depth 14 on 8 GPUs):
    the final level's new states are deduplicated by their owners and counted by the generating ranks,
    never shipped or stored.  Two loopback ranks on C5v2 to depth 10 give the single-GPU storing run's
    counts and levels; so does mc_opts.n_gpus = 2, whose dump refuses (the last level is not stored)."""
    shard = importlib.import_module("raft-tla_amd.shard")
    cfg = os.path.join(CONFIGS, "c5v2.cfg")
    a = raftmc.check(ORIG_MC, cfg, max_depth=10, workers=0)
    assert a.verdict == "DEPTH_LIMIT" and a.distinct == sum([1, 6, 45, 330, 2190, 13761, 82510, 475485, 2648995, 14330920])
    want = (a.generated, a.distinct, a.depth, a.left_on_queue, {k: v[0] for k, v in a.actions.items()})
    kw = dict(max_depth=10, workers=0, count_final_level=True, fp_table_bytes=1 << 30, state_store_bytes=1 << 30)
    out = shard.check_loopback(ORIG_MC, cfg, 2, **kw)
    for r in out:
        assert r.verdict == "DEPTH_LIMIT", r.error
        assert (r.generated, r.distinct, r.depth, r.left_on_queue, {k: v[0] for k, v in r.actions.items()}) == want
        assert [lv[0] for lv in r.levels] == [lv[0] for lv in a.levels]
        assert sum(v[1] for v in r.actions.values()) + 1 == r.distinct
    with raftmc.ModelChecker(ORIG_MC, cfg, n_gpus=2, same_device=torch.cuda.device_count() < 2, **kw) as mc:
        r = mc.run()
        with pytest.raises(raftmc.RaftMCError):
            mc.dump_states(str(tmp_path / "s.txt"))
    assert (r.generated, r.distinct, r.depth, r.left_on_queue, {k: v[0] for k, v in r.actions.items()}) == want


def test_native_loop_store_overflow(raftmc):
    """The ranks' stores fill (each holds 12M of C2's 54.4M states; whichever rank overflows first
    raises the flag): the capacity error travels in the level all-reduce, every rank stops at the same
    level with CAPACITY_OVERFLOW naming the full store, the summary counts the completed levels, and
    nothing hangs."""
    shard = importlib.import_module("raft-tla_amd.shard")
    cfg = os.path.join(CONFIGS, "c2.cfg")
    t0 = time.time()
    out = shard.check_loopback(ORIG_MC, cfg, 2, workers=0, fp_table_bytes=1 << 30,
                               state_store_bytes=12_000_000 * _slot_bytes(raftmc, cfg))
    assert time.time() - t0 < 120
    for r in out:
        assert r.verdict == "CAPACITY_OVERFLOW" and "error flags" in r.error, (r.verdict, r.error)
        assert [lv[0] for lv in r.levels] == [lv[0] for lv in out[0].levels]
    assert out[0].distinct == sum(lv[0] for lv in out[0].levels) < 54426066


def test_n_gpus_rank_failure_releases_peers(raftmc):
    """A rank that leaves the native loop early (here an injected failure of rank 1 at depth 5,
    mc_set_fault_injection) releases its peers instead of leaving them in the next collective: mc_run
    returns the failing rank's error, naming it, within seconds; the same handle then runs the model to
    completion (fresh communicators on a node: the aborted ones are never reused)."""
    cfg = os.path.join(CONFIGS, "c2.cfg")
    kw = dict(workers=0, fp_table_bytes=2 << 30, state_store_bytes=2 << 30)
    with raftmc.ModelChecker(ORIG_MC, cfg, n_gpus=2, same_device=torch.cuda.device_count() < 2, **kw) as mc:
        mc.set_fault_injection(1, 5)
        t0 = time.time()
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.run()
        assert time.time() - t0 < 60
        assert "rank 1" in str(e.value) and "injected failure" in str(e.value), str(e.value)
        mc.set_fault_injection(-1, 0)
        r = mc.run()
    g = json.load(open(os.path.join(GOLDEN, "c2_exact.json")))
    assert (r.verdict, r.generated, r.distinct, r.depth) == ("OK", g["generated"], g["distinct"], g["depth"]), r.error
