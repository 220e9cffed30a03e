"""The product's packed tlc_membership spec (raft-tla_amd/csrc/memb_spec.h: the
successor relation, constraints, invariants, history summary and symmetric
fingerprint that the gfx950 kernels compile) run on the host by a test-only
FIFO BFS harness (tests/native/memb_host_bfs.cpp), checked against the oracle
fixtures: identical counts, per-action (generated, distinct) counts, depth,
states left on queue and the identical set of kept states (SHA-256 of the
sorted canonical text, history counters included)."""
import hashlib
import json
import os
import subprocess
import tempfile

import pytest

from oracle_util import CONFIGS, GOLDEN, ROOT, golden_file

SHAPES = {"membership_shipped": (3, 2), "memb_dynamic3": (3, 2), "memb_nosym": (3, 2), "memb_two": (2, 1),
          "memb_four": (4, 2), "memb_four_scale": (4, 2), "memb_async": (3, 2), "scen_CommitWhenConcurrentLeaders_punct": (3, 2),
          "scen_MajorityOfClusterRestarts_punct": (3, 2)}
FIX = json.load(open(os.path.join(GOLDEN, "memb_parity.json")))


def build_harness(shape):
    out = os.path.join(tempfile.gettempdir(), "memb_host_bfs_%d%d" % shape)
    csrc = os.path.join(ROOT, "raft-tla_amd", "csrc")
    src = [os.path.join(ROOT, "tests", "native", "memb_host_bfs.cpp"), os.path.join(csrc, "model.cpp"),
           os.path.join(csrc, "memb_model.cpp"), os.path.join(csrc, "tla_value.cpp")]
    deps = src + [os.path.join(csrc, f) for f in ("memb_spec.h", "memb_text.h", "memb_prefix.h", "tla_value.h", "common.h")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(p) for p in deps):
        tmp = "%s.%d" % (out, os.getpid())    # build aside and rename: parallel workers never run a partial file
        subprocess.run(["g++", "-O2", "-std=c++17", "-DSHAPE_N=%d" % shape[0], "-DSHAPE_NV=%d" % shape[1], "-o", tmp, *src],
                       check=True)
        os.replace(tmp, out)
    return out


def sym_env(g):
    """SYMMETRY in TLC's mode for the "tlc:" fixtures (the oracle's --sym tlc)."""
    return dict(os.environ, SYM_TLC="1") if g.get("sym") == "tlc" else None


def prefix_args(g):
    """--prefix CONSTRAINT FILE for punctuated-search cases (golden trace from the committed fixture)."""
    if not g.get("prefix"):
        return []
    con, fixture = g["prefix"]
    return ["--prefix", con, golden_file(fixture)[0]]


@pytest.mark.parametrize("case", sorted(k for k, v in FIX.items() if v["verdict"] == "OK"))
def test_packed_membership_matches_oracle(case):
    g = FIX[case]
    exe = build_harness(SHAPES[g["cfg"]])
    fd, dump = tempfile.mkstemp(suffix=".txt")
    os.close(fd)
    r = json.loads(subprocess.run([exe, os.path.join(CONFIGS, g["cfg"] + ".cfg"), str(g["max_depth"]), dump, *prefix_args(g)],
                                  capture_output=True, text=True, check=True, env=sym_env(g)).stdout)
    assert r["err"] == 0 and r["verdict"] == "OK"
    assert (r["generated"], r["distinct"], r["depth"], r["left_on_queue"]) == (g["generated"], g["distinct"], g["depth"], g["left_on_queue"])
    assert r["actions"] == g["actions"]
    lines = sorted(l.rstrip("\n") for l in open(dump))
    os.unlink(dump)
    assert hashlib.sha256("\n".join(lines).encode()).hexdigest() == g["states_sha256"]


@pytest.mark.parametrize("case", ["scen_FirstBecomeLeader", "punct_CommitWhenConcurrentLeaders",
                                  "punct_MajorityOfClusterRestarts", "tlc:scen_FirstCommit"])
def test_packed_membership_first_violation(case):
    g = FIX[case]
    exe = build_harness(SHAPES.get(g["cfg"], (3, 2)))
    r = json.loads(subprocess.run([exe, os.path.join(CONFIGS, g["cfg"] + ".cfg"), "0", "-", *prefix_args(g)],
                                  capture_output=True, text=True, check=True, env=sym_env(g)).stdout)
    assert (r["verdict"], r["violated"], r["depth"], r["generated"], r["distinct"], r["left_on_queue"]) == \
        (g["verdict"], g["violated"], g["depth"], g["generated"], g["distinct"], g["left_on_queue"])


def test_refined_symmetric_fingerprint_equals_brute_force_orbits():
    """The GPU's symmetric fingerprint hashes only the permutations that respect the servers'
    invariant signatures (memb_spec.h fingerprint, partition refinement).  On every distinct state
    of the 4-server model without SYMMETRY to depth 15 (all symmetric copies kept, >= 1e5 states),
    it must induce exactly the partition of the brute-force min over all 4! permuted views: same
    number of classes, and no refined class maps to two brute-force classes or vice versa."""
    exe = build_harness((4, 2))
    r = json.loads(subprocess.run([exe, os.path.join(CONFIGS, "memb_four_nosym.cfg"), "15"], capture_output=True,
                                  text=True, check=True, env=dict(os.environ, SYMCHECK="1")).stdout)
    states, refined, brute, bad = r["symcheck"]
    assert states >= 100000 and bad == 0 and refined == brute, r
    assert refined < states / 4      # symmetry really merges (24 permutations)
