"""Build step: generated sources and gfx950 code objects for the repo's generated-path test
specs, so the GPU box (which has no /root/reference) runs them without the front end or hiprtc.

For each (name, module, cfg): `_build/tlagen <module> <cfg> --kernels` writes
_build/tlagen_co/<name>.gen.hip (skipped when the module's base file is absent and the source
already exists), and hipcc --genco compiles it to _build/tlagen_co/<key>.hsaco, where <key> is the
library's cache key (FNV-1a 64 of the source and the hiprtc options, tlagen_backend.cpp)."""
import concurrent.futures
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(os.path.dirname(HERE))
ROOT = os.path.dirname(PKG)
OUT = os.path.join(PKG, "_build", "tlagen_co")
OPTS = ["--offload-arch=gfx950", "-O2", "-std=c++17"]
REF = os.environ.get("RAFTMC_REFERENCE", "/root/reference")

SPECS = [(n, "configs/raft_original_mc.tla", "configs/%s.cfg" % n)
         for n in ("c1", "parity_single", "parity_pair", "parity_trio", "c2", "c2_noleader")]
SPECS += [("toy_ring", "configs/tlagen/TokenRing.tla", "configs/tlagen/TokenRing.cfg"),
          ("toy_ring_full", "configs/tlagen/TokenRing.tla", "configs/tlagen/TokenRing_full.cfg"),
          ("countdown", "configs/tlagen/Countdown.tla", "configs/tlagen/Countdown.cfg"),
          ("countdown_evalerr", "configs/tlagen/Countdown.tla", "configs/tlagen/Countdown_evalerr.cfg"),
          ("ricketts_c1", "configs/ricketts_mc.tla", "configs/ricketts_c1.cfg"),
          ("ricketts_noleader", "configs/ricketts_mc.tla", "configs/ricketts_noleader.cfg"),
          ("ricketts_election_safety", "configs/ricketts_mc.tla", "configs/ricketts_election_safety.cfg"),
          ("ricketts_safety", "configs/ricketts_mc.tla", "configs/ricketts_safety.cfg"),
          ("toy_ring_view", "configs/tlagen/TokenRing.tla", "configs/tlagen/TokenRing_view.cfg"),
          ("funsets", "configs/tlagen/FunSets.tla", "configs/tlagen/FunSets.cfg"),
          ("funsets_fbelow2", "configs/tlagen/FunSets.tla", "configs/tlagen/FunSets_FBelow2.cfg"),
          ("funsets_qempty", "configs/tlagen/FunSets.tla", "configs/tlagen/FunSets_QEmpty.cfg"),
          ("ricketts_typeok", "configs/ricketts_mc.tla", "configs/ricketts_typeok.cfg"),
          ("ricketts_badterm", "configs/ricketts_mc.tla", "configs/ricketts_badterm.cfg"),
          ("higher_order", "configs/tlagen/HigherOrder.tla", "configs/tlagen/HigherOrder.cfg"),
          ("higher_order_fewzeros", "configs/tlagen/HigherOrder.tla", "configs/tlagen/HigherOrder_FewZeros.cfg"),
          ("recursive_ops", "configs/tlagen/Recursive.tla", "configs/tlagen/Recursive.cfg"),
          ("recursive_ops_runaway", "configs/tlagen/Recursive.tla", "configs/tlagen/Recursive_Runaway.cfg"),
          ("product", "configs/tlagen/Product.tla", "configs/tlagen/Product.cfg"),
          ("rec_fun", "configs/tlagen/RecFun.tla", "configs/tlagen/RecFun.cfg"),
          ("rec_fun_fact", "configs/tlagen/RecFun.tla", "configs/tlagen/RecFun_fact.cfg"),
          ("rec_fun_sum", "configs/tlagen/RecFun.tla", "configs/tlagen/RecFun_sum.cfg"),
          ("rec_fun_dom", "configs/tlagen/RecFun.tla", "configs/tlagen/RecFun_dom.cfg"),
          # the unmodified tlc_membership/raft.tla with VIEW vars and SYMMETRY perms (TLC's rule)
          ("memb_nosym_gen", "configs/raft_membership_mc.tla", "configs/memb_nosym.cfg"),
          ("memb_shipped_gen", "configs/raft_membership_mc.tla", "configs/membership_shipped.cfg"),
          ("memb_two_gen", "configs/raft_membership_mc.tla", "configs/memb_two.cfg"),
          # C3 (BASELINE configs[2]): 4 servers, NextDynamic -- the hand path's full-size run cross-checked
          ("memb_four_gen", "configs/raft_membership_mc.tla", "configs/memb_four.cfg"),
          # the punctuated searches: golden-trace prefix constraints, an ACTION_CONSTRAINT
          ("memb_morc_gen", "configs/raft_membership_mc.tla", "configs/scen_MajorityOfClusterRestarts_punct.cfg"),
          ("memb_cwcl_gen", "configs/raft_membership_mc.tla", "configs/scen_CommitWhenConcurrentLeaders_punct.cfg"),
          # the reference's Apalache spec with its own shipped cfg (TLC syntax): recursive Sum
          ("apalache_nm", REF + "/apalache_no_membership/raft.tla", REF + "/apalache_no_membership/raft.cfg"),
          # ... and with its commented-out test-case invariants (pinned by oracle/raft_apalache.h)
          ("apalache_nm_boundedtrace", REF + "/apalache_no_membership/raft.tla", "configs/apalache_nm_boundedtrace.cfg"),
          ("apalache_nm_firstbecomeleader", REF + "/apalache_no_membership/raft.tla", "configs/apalache_nm_firstbecomeleader.cfg")]


def key_of(src):
    h = 1469598103934665603
    for b in (src + "".join("\n" + o for o in OPTS)).encode():
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return "%016x" % h


def one(spec):
    name, mod, cfg = spec
    gen = os.path.join(OUT, name + ".gen.hip")
    tool = os.path.join(PKG, "_build", "tlagen")
    r = subprocess.run([tool, os.path.join(ROOT, mod), os.path.join(ROOT, cfg), "-I", REF, "--kernels", "-o", gen + ".tmp"],   # (absolute paths stay)
                       capture_output=True, text=True)
    if r.returncode == 0:
        if not os.path.exists(gen) or open(gen).read() != open(gen + ".tmp").read():
            os.replace(gen + ".tmp", gen)
        else:
            os.remove(gen + ".tmp")
    elif not os.path.exists(gen):
        return name, "skipped (%s)" % r.stderr.strip()[:200]
    src = open(gen).read()
    co = os.path.join(OUT, key_of(src) + ".hsaco")
    if not os.path.exists(co):
        c = subprocess.run(["/opt/rocm/bin/hipcc", "--genco", *OPTS, "-o", co + ".tmp", "-x", "hip", gen], capture_output=True, text=True)
        if c.returncode != 0:
            raise RuntimeError("hipcc %s: %s" % (name, c.stderr[-2000:]))
        os.replace(co + ".tmp", co)
    return name, key_of(src)


def main():
    os.makedirs(OUT, exist_ok=True)
    keys = set()
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        for name, res in ex.map(one, SPECS):
            print("tlagen prebuild %s: %s" % (name, res))
            keys.add(res)
    for f in os.listdir(OUT):   # code objects of sources no longer generated (they travel to the GPU box)
        if f.endswith(".hsaco") and f[:-6] not in keys:
            os.remove(os.path.join(OUT, f))


if __name__ == "__main__":
    sys.exit(main())
