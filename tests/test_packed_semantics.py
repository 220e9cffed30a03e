"""The product's packed raft_original successor function (raft-tla_amd/csrc/
orig_spec.h, the same header the gfx950 kernels compile) run on the host by a
test-only BFS harness, checked against the oracle fixtures: identical counts,
per-action counts, depth, and the identical set of reachable states (SHA-256
of the sorted canonical TLA+ text of every distinct state)."""
import hashlib
import json
import os
import subprocess
import tempfile

import pytest

from oracle_util import CONFIGS, GOLDEN, ROOT

SHAPES = {"c1": (3, 1, 2, 1, 2), "parity_single": (1, 2, 3, 2, 3), "parity_pair": (2, 1, 2, 1, 5),
          "parity_pair_neg": (2, 1, 2, 1, 5), "parity_trio": (3, 2, 3, 2, 2), "parity_pair6": (2, 1, 2, 1, 6)}


def build_harness(shape):
    out = os.path.join(tempfile.gettempdir(), "orig_host_bfs_%d%d%d%d%d" % shape)
    src = [os.path.join(ROOT, "tests", "native", "orig_host_bfs.cpp"),
           os.path.join(ROOT, "raft-tla_amd", "csrc", "model.cpp"),
           os.path.join(ROOT, "raft-tla_amd", "csrc", "orig_model.cpp")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(p) for p in src + [
            os.path.join(ROOT, "raft-tla_amd", "csrc", "orig_spec.h")]):
        defs = ["-DSHAPE_%s=%d" % (k, v) for k, v in zip(("N", "NV", "MT", "ML", "MK"), shape)]
        tmp = "%s.%d" % (out, os.getpid())    # build aside and rename: parallel workers never run a partial file
        subprocess.run(["g++", "-O2", "-std=c++17", *defs, "-o", tmp, *src], check=True)
        os.replace(tmp, out)
    return out


@pytest.mark.parametrize("name", ["c1", "parity_single", "parity_pair", "parity_trio"])
def test_packed_successors_match_oracle(name):
    g = json.load(open(os.path.join(GOLDEN, "orig_parity.json")))[name]
    exe = build_harness(SHAPES[name])
    fd, dump = tempfile.mkstemp(suffix=".txt")
    os.close(fd)
    r = json.loads(subprocess.run([exe, os.path.join(CONFIGS, name + ".cfg"), dump],
                                  capture_output=True, text=True, check=True).stdout)
    assert r["err"] == 0
    assert (r["generated"], r["distinct"], r["depth"]) == (g["generated"], g["distinct"], g["depth"])
    assert r["actions"] == g["actions"]
    lines = sorted(l.rstrip("\n") for l in open(dump))
    os.unlink(dump)
    assert hashlib.sha256("\n".join(lines).encode()).hexdigest() == g["states_sha256"]


EVENT_SHAPES = {"scenario_first_leader": (2, 1, 2, 1, 5), "c2_noleader": (3, 2, 3, 2, 5), "pair6_nocommit": (2, 1, 2, 1, 6)}


@pytest.mark.parametrize("name", sorted(EVENT_SHAPES))
def test_packed_fifo_stop_point_matches_oracle(name):
    """TLC's single-worker FIFO order with the product's packed successor function: the bag slot
    order of the order-preserving message codes is the enumeration order of `\\E m \\in DOMAIN
    messages`, so a sequential BFS over instance order reproduces the oracle's first violating
    state, its counterexample and TLC's counters at the stop point exactly
    (tests/golden/orig_events.json)."""
    g = json.load(open(os.path.join(GOLDEN, "orig_events.json")))[name]
    exe = build_harness(EVENT_SHAPES[name])
    r = json.loads(subprocess.run([exe, os.path.join(CONFIGS, name + ".cfg"), "-"],
                                  capture_output=True, text=True, check=True).stdout)
    for k in ("verdict", "violated", "generated", "distinct", "left_on_queue", "depth", "levels", "actions"):
        assert r[k] == g[k], k
    assert [(t["action"], t["state"]) for t in r["trace"]] == [(t["action"], t["state"]) for t in g["trace"]]


@pytest.mark.parametrize("fixture,shape", [("c5_prefix", (5, 1, 3, 3, 4)), ("c5v2_prefix", (5, 2, 3, 3, 8)),
                                           ("c2_md6_prefix", (3, 2, 3, 2, 6))])
def test_packed_c5_prefix_matches_oracle(fixture, shape):
    """The 5-server shapes (one and two values; the two-value one stores election records in
    the compact form, orig_spec.h ECOMPACT) against the oracle's depth-limited fixtures:
    counts and the identical set of states (SHA-256 of the sorted canonical text)."""
    path = os.path.join(GOLDEN, fixture + ".json")
    if not os.path.exists(path):
        pytest.skip(fixture + " not generated")
    g = json.load(open(path))
    exe = build_harness(shape)
    fd, dump = tempfile.mkstemp(suffix=".txt")
    os.close(fd)
    r = json.loads(subprocess.run([exe, os.path.join(CONFIGS, g["cfg"]), dump, "--max-depth", str(g["max_depth"])],
                                  capture_output=True, text=True, check=True).stdout)
    lines = sorted(l.rstrip("\n") for l in open(dump))
    os.unlink(dump)
    assert r["err"] == 0
    assert (r["generated"], r["distinct"], r["left_on_queue"]) == (g["generated"], g["distinct"], g["left_on_queue"])
    assert hashlib.sha256("\n".join(lines).encode()).hexdigest() == g["states_sha256"]


def test_compact_election_records_replayed_by_oracle():
    """5 servers with two values (configs/c5v2.cfg) store election records in the compact form
    (orig_spec.h ECOMPACT: evoterLog without its presence bits, eterm in bits_for(MaxTerm)).
    A seeded walk over the product's packed successor function (tests/native/orig_walk.cpp,
    pack/unpack checked at every step) runs until a state holds an election record and an
    entry with the second value; the oracle's check-trace replays every step of its canonical
    text (records decoded from the compact form) through the literal restatement."""
    from oracle_util import ORIG_MC, run_oracle
    shape = (5, 2, 3, 3, 8)
    out = os.path.join(tempfile.gettempdir(), "orig_walk_%d%d%d%d%d" % shape)
    src = [os.path.join(ROOT, "tests", "native", "orig_walk.cpp"), os.path.join(ROOT, "raft-tla_amd", "csrc", "model.cpp"),
           os.path.join(ROOT, "raft-tla_amd", "csrc", "orig_model.cpp")]
    tmp = "%s.%d" % (out, os.getpid())
    subprocess.run(["g++", "-O2", "-std=c++17", "-DSHAPE_N=%d" % shape[0], "-DSHAPE_NV=%d" % shape[1], "-DSHAPE_MT=%d" % shape[2],
                    "-DSHAPE_ML=%d" % shape[3], "-DSHAPE_MK=%d" % shape[4], "-o", tmp, *src], check=True)
    os.replace(tmp, out)
    cfg = os.path.join(CONFIGS, "c5v2.cfg")
    walk = subprocess.run([out, cfg, "1", "200000", "1"], capture_output=True, text=True, check=True, timeout=300).stdout
    lines = walk.strip().split("\n")
    assert "eleader" in lines[-1] and "v2" in lines[-1]
    fd, path = tempfile.mkstemp(suffix=".txt")
    with os.fdopen(fd, "w") as f:
        f.write(walk)
    r = run_oracle("check-trace", ORIG_MC, cfg, "--golden", path)
    os.unlink(path)
    # every step replayed (no invariant of the cfg is violated, so "valid" - which asks the last
    # state to violate one - stays false)
    assert r["bad_step"] == -1 and len(r["actions"].split(",")) == len(lines) - 1, r
    assert "BecomeLeader" in r["actions"] and "ClientRequest" in r["actions"]
