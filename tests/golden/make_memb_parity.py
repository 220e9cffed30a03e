"""Generate tlc_membership parity fixtures with the CPU oracle (test infrastructure).

For each (cfg, max depth) case the oracle (oracle/raft_membership.h, a literal
restatement of tlc_membership/raft.tla with TLC BFS semantics) runs BFS with
SYMMETRY in orbit ("view") mode and FIFO single-worker order, and the fixture
records generated / distinct / depth / left on queue / per-level sizes /
per-action (generated, distinct), the verdict, the counterexample trace, and
the SHA-256 of the sorted canonical text of every distinct state (the VIEW
plus every history counter; history["global"] is summarised, see
raft-tla_amd/csrc/memb_spec.h).  TLC itself is unavailable offline
(SURVEY.md §8c): the counts are oracle-pinned; the oracle is pinned by the
reference's two TLC traces (tests/test_oracle.py).

Punctuated-search cases take the golden history trace of their prefix
constraint from the committed trace fixtures (tests/golden/*_trace.json, the
TLC traces of tlc_membership/raft.tla:1201 and :1231).

    python tests/golden/make_memb_parity.py [--workers T] [--out FILE] [case ...]

--workers T expands each batch of parents on T threads with the frontier-order merge (results
identical to one worker, oracle/engine.h); --out writes the cases into FILE instead of
memb_parity.json (to run several cases in parallel and merge them afterwards).
"""
import hashlib
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle_util import CONFIGS, GOLDEN, MEMB_MC, golden_file, run_oracle  # noqa: E402

# prefix constraint -> (oracle flag, trace fixture)
PREFIXES = {"CommitWhenConcurrentLeaders_unique": ("--golden-cwcl", "concurrent_leaders_trace.json"),
            "MajorityOfClusterRestarts_constraint": ("--golden-morc", "commit_when_concurrent_leaders_trace.json")}

CASES = {
    "membership_shipped@14": ("membership_shipped", 14),
    "memb_two@16": ("memb_two", 16),
    "memb_dynamic3@14": ("memb_dynamic3", 14),
    "memb_nosym@13": ("memb_nosym", 13),
    "memb_four@10": ("memb_four", 10),
    "memb_four@16": ("memb_four", 16),   # >= 1e5 states: signature ties in the 4-server refinement
    "scen_FirstBecomeLeader": ("scen_FirstBecomeLeader", 0),
    "scen_FirstCommit": ("scen_FirstCommit", 0),
    "scen_EntryCommitted": ("scen_EntryCommitted", 0),
    "punct_CommitWhenConcurrentLeaders@24": ("scen_CommitWhenConcurrentLeaders_punct", 24, "CommitWhenConcurrentLeaders_unique"),
    "punct_CommitWhenConcurrentLeaders": ("scen_CommitWhenConcurrentLeaders_punct", 0, "CommitWhenConcurrentLeaders_unique"),
    "punct_MajorityOfClusterRestarts@30": ("scen_MajorityOfClusterRestarts_punct", 30, "MajorityOfClusterRestarts_constraint"),
    "punct_MajorityOfClusterRestarts": ("scen_MajorityOfClusterRestarts_punct", 0, "MajorityOfClusterRestarts_constraint"),
    # C4: every scenario property the oracle reaches in minutes (raft.tla:1143-1278)
    "scen_ConcurrentLeaders": ("scen_ConcurrentLeaders", 0),
    "scen_LeadershipChange": ("scen_LeadershipChange", 0),
    "scen_BoundedTrace": ("scen_BoundedTrace", 0),
    "scen_FirstRestart": ("scen_FirstRestart", 0),
    "scen_MembershipChange": ("scen_MembershipChange", 0),
    "scen_MultipleMembershipChanges": ("scen_MultipleMembershipChanges", 0),
    "scen_AddSucessful": ("scen_AddSucessful", 0),
    "scen_MembershipChangeCommits": ("scen_MembershipChangeCommits", 0),
    "scen_AddCommits": ("scen_AddCommits", 0),
    # on the smallest growing cluster (InitServer = {s1}, Server = {s1, s2}; configs/scen_*.cfg headers)
    "scen_MultipleMembershipChangesCommit": ("scen_MultipleMembershipChangesCommit", 0),
    "scen_LeaderChangesDuringConfChange": ("scen_LeaderChangesDuringConfChange", 0),
    # SYMMETRY in TLC's mode (oracle --sym tlc, MC_COMPAT_SYM_TLC): least permuted full state, then VIEW
    "tlc:membership_shipped@16": ("membership_shipped", 16),
    "tlc:memb_two@16": ("memb_two", 16),
    "tlc:memb_dynamic3@14": ("memb_dynamic3", 14),
    "tlc:memb_four@13": ("memb_four", 13),
    # bench.py's membership scale workload (C3's model without LeaderVotesQuorum), depth-bounded
    "tlc:memb_four_scale@15": ("memb_four_scale", 15),
    "tlc:scen_FirstCommit": ("scen_FirstCommit", 0),
    # C4 in TLC's SYMMETRY rule (the drop-in default): every scenario property of raft.tla:1143-1278
    # the oracle's exact search reaches (NewlyJoinedBecomeLeader: tests/golden/gpu_traces, lean mode)
    "tlc:scen_FirstBecomeLeader": ("scen_FirstBecomeLeader", 0),
    "tlc:scen_EntryCommitted": ("scen_EntryCommitted", 0),
    "tlc:scen_ConcurrentLeaders": ("scen_ConcurrentLeaders", 0),
    "tlc:scen_LeadershipChange": ("scen_LeadershipChange", 0),
    "tlc:scen_BoundedTrace": ("scen_BoundedTrace", 0),
    "tlc:scen_FirstRestart": ("scen_FirstRestart", 0),
    "tlc:scen_MembershipChange": ("scen_MembershipChange", 0),
    "tlc:scen_MultipleMembershipChanges": ("scen_MultipleMembershipChanges", 0),
    "tlc:scen_AddSucessful": ("scen_AddSucessful", 0),
    "tlc:scen_MembershipChangeCommits": ("scen_MembershipChangeCommits", 0),
    "tlc:scen_AddCommits": ("scen_AddCommits", 0),
    "tlc:scen_MultipleMembershipChangesCommit": ("scen_MultipleMembershipChangesCommit", 0),
    "tlc:scen_LeaderChangesDuringConfChange": ("scen_LeaderChangesDuringConfChange", 0),
    "tlc:punct_CommitWhenConcurrentLeaders": ("scen_CommitWhenConcurrentLeaders_punct", 0, "CommitWhenConcurrentLeaders_unique"),
    "tlc:punct_MajorityOfClusterRestarts": ("scen_MajorityOfClusterRestarts_punct", 0, "MajorityOfClusterRestarts_constraint"),
    "tlc:punct_MajorityOfClusterRestarts@30": ("scen_MajorityOfClusterRestarts_punct", 30, "MajorityOfClusterRestarts_constraint"),
    # the NEXT relations on their own (raft.tla:909-916, :924-932) and the other verdict classes
    "memb_async@16": ("memb_async", 16),
    "tlc:memb_async@16": ("memb_async", 16),
    "deadlock:memb_unreliable": ("memb_unreliable", 0),        # Init has no successor: TLC's deadlock, exit 11
    "eval:memb_eval_single": ("memb_eval_single", 0),          # Committed(i) out of range: TLC's evaluation error, exit 75
}
# cases searched with TLC's deadlock check on (the oracle's --deadlock; the GPU's default check_deadlock = 1)
DEADLOCK = {"deadlock:memb_unreliable", "eval:memb_eval_single", "memb_async@16", "tlc:memb_async@16"}
OUT = os.path.join(GOLDEN, "memb_parity.json")


def digest_lines(path):
    lines = sorted(l.rstrip("\n") for l in open(path))
    return hashlib.sha256("\n".join(lines).encode()).hexdigest(), len(lines)


def main(names, out=OUT, workers=1):
    doc = json.load(open(out)) if os.path.exists(out) else {}
    for n in names:
        cfg, depth = CASES[n][:2]
        prefix = CASES[n][2] if len(CASES[n]) > 2 else None
        fd, dump = tempfile.mkstemp(suffix=".txt")
        os.close(fd)
        sym = "tlc" if n.startswith("tlc:") else "view"
        args = ["--sym", sym, "--dump", dump, "--trace", "--workers", workers] + (["--deadlock"] if n in DEADLOCK else [])
        if prefix:
            flag, fixture = PREFIXES[prefix]
            args += [flag, golden_file(fixture)[0]]
        if depth:
            args += ["--max-depth", depth]
        r = run_oracle("bfs", MEMB_MC, os.path.join(CONFIGS, cfg + ".cfg"), *args, timeout=100000)
        assert r["verdict"] in ("OK", "INVARIANT_VIOLATION", "DEADLOCK", "EVAL_ERROR"), r
        sha, cnt = digest_lines(dump)
        os.unlink(dump)
        doc[n] = {"cfg": cfg, "max_depth": depth, "sym": sym, "verdict": r["verdict"], "violated": r["violated"],
                  "deadlock": n in DEADLOCK, "error": r["error"],
                  "prefix": [prefix, PREFIXES[prefix][1]] if prefix else None,
                  "generated": r["generated"], "distinct": r["distinct"], "depth": r["depth"],
                  "left_on_queue": r["left_on_queue"], "levels": r["levels"], "actions": r["actions"],
                  "states_sha256": sha, "states_dumped": cnt,
                  "trace": r.get("trace", []), "oracle_seconds": round(r["seconds"], 2)}
        print(n, r["verdict"], r["distinct"], doc[n]["oracle_seconds"], "s", flush=True)
        json.dump(doc, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    argv = sys.argv[1:]
    kw = {}
    for flag, key in (("--workers", "workers"), ("--out", "out")):
        if flag in argv:
            i = argv.index(flag)
            kw[key] = argv[i + 1]
            del argv[i:i + 2]
    main(argv or list(CASES), **kw)
