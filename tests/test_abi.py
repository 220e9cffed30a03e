"""C-ABI boundary: the library loads, exports every symbol include/raftmc.h
declares, resolves cfgs (no GPU needed) and fails loudly without a device."""
import os
import re

import pytest

from oracle_util import CONFIGS, MEMB_MC, ORIG_MC, ROOT, cfg_variant

HEADER = os.path.join(ROOT, "include", "raftmc.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:static inline )?(?:int|void|const char\*)\s+(mc_\w+)\s*\(", text, re.M)))


def test_header_and_python_mirror_agree(raftmc):
    assert declared_functions() == sorted(raftmc.EXPORTS)


def test_library_exports_every_declared_symbol(raftmc):
    lib = raftmc.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name


def _c_layout(struct, fields, tmp):
    """sizeof / offsetof of a struct of include/raftmc.h as the C compiler lays it out (gcc)"""
    import subprocess
    src = tmp / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "raftmc.h"\nint main(void) {\n'
                   '  printf("%%zu", sizeof(%s));\n' % struct +
                   "".join('  printf(" %%zu", offsetof(%s, %s));\n' % (struct, f) for f in fields) +
                   '  printf("\\n");\n  return 0;\n}\n')
    exe = tmp / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), "-o", str(exe), str(src)], check=True)
    return [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]


@pytest.mark.parametrize("struct,mirror", [("mc_summary_t", "McSummary"), ("mc_opts", "McOpts")])
def test_struct_layout_matches_ctypes_mirror(raftmc, struct, mirror, tmp_path):
    """The ctypes mirrors of mc_summary_t / mc_opts (raftmc.py) have the C header's size and field
    offsets: mc_summary writes sizeof(mc_summary_t) bytes into the caller's struct."""
    import importlib
    rm = importlib.import_module("raft-tla_amd.raftmc")
    cls = getattr(rm, mirror)
    names = [f[0] for f in cls._fields_]
    got = _c_layout(struct, names, tmp_path)
    assert got[0] == __import__("ctypes").sizeof(cls)
    assert got[1:] == [getattr(cls, n).offset for n in names]


def test_abi_version_mismatch_refused(raftmc):
    """an mc_opts of another ABI version (e.g. a caller built against version 1, whose mc_summary_t
    is smaller) is refused by mc_open"""
    import ctypes
    lib = raftmc.load_library()
    rm = __import__("importlib").import_module("raft-tla_amd.raftmc")
    o = rm.McOpts()
    assert lib.mc_opts_init(ctypes.byref(o), raftmc.ABI_VERSION) == 0
    assert o.abi_version == raftmc.ABI_VERSION == 3
    o.abi_version = 1
    h = ctypes.c_void_p()
    rc = lib.mc_open(ORIG_MC.encode(), os.path.join(CONFIGS, "c2.cfg").encode(), ctypes.byref(o), ctypes.byref(h))
    assert rc == -1 and not h


def test_default_opts_path_stamps_the_callers_version(raftmc, tmp_path):
    """the version in mc_opts is the caller's, also through the documented
    mc_default_opts -> mc_open sequence.  A C caller compiled against include/raftmc.h gets the header's
    version from the inline mc_default_opts and is accepted; a caller built against an older header,
    which reaches the library's exported mc_default_opts symbol, gets version 0 and is refused; the
    version-1 layout is refused by mc_opts_init itself.  (mc_open only parses: no GPU work.)"""
    import ctypes
    lib = raftmc.load_library()
    rm = __import__("importlib").import_module("raft-tla_amd.raftmc")
    cfg = os.path.join(CONFIGS, "c2.cfg").encode()
    o = rm.McOpts()
    lib.mc_default_opts(ctypes.byref(o))            # the pre-v3 symbol
    assert o.abi_version == 0 and o.workers == 1 and o.n_gpus == 1
    h = ctypes.c_void_p()
    assert lib.mc_open(ORIG_MC.encode(), cfg, ctypes.byref(o), ctypes.byref(h)) == -1 and not h
    o = rm.McOpts()
    assert lib.mc_opts_init(ctypes.byref(o), 1) == -1 and o.abi_version == 1
    # a C caller through the header's inline wrapper
    src = tmp_path / "caller.c"
    src.write_text('#include <stdio.h>\n#include "raftmc.h"\n'
                   'int main(int argc, char** argv) {\n  mc_opts o; mc_default_opts(&o);\n  mc_ctx* c = 0;\n'
                   '  int rc = mc_open(argv[1], argv[2], &o, &c);\n  printf("%d %d\\n", o.abi_version, rc);\n'
                   '  if (c) mc_close(c);\n  return 0;\n}\n')
    import subprocess
    libdir = os.path.join(ROOT, "raft-tla_amd", "_build")
    exe = tmp_path / "caller"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), "-o", str(exe), str(src), "-L", libdir, "-lraftmc",
                    "-Wl,-rpath," + libdir], check=True)
    out = subprocess.run([str(exe), ORIG_MC, os.path.join(CONFIGS, "c2.cfg")], capture_output=True, text=True, check=True)
    assert out.stdout.split() == [str(raftmc.ABI_VERSION), "0"], out


@pytest.mark.parametrize("spec,cfg,kw", [
    (ORIG_MC, "c2.cfg", dict(workers=1, max_depth=5)),          # TLC's FIFO order stores every level
    (ORIG_MC, "c2.cfg", dict(workers=0, max_depth=0)),          # no final level without a depth bound
    (MEMB_MC, "membership_shipped.cfg", dict(workers=0, max_depth=5)),   # raft_original only
])
def test_count_final_level_refused_where_unsupported(raftmc, spec, cfg, kw):
    """count_final_level is refused (MC_E_UNSUPPORTED) wherever it would be ignored"""
    with pytest.raises(raftmc.RaftMCError) as e:
        raftmc.ModelChecker(spec, os.path.join(CONFIGS, cfg), count_final_level=True, **kw)
    assert e.value.code == -4


def test_count_final_level_refuses_checkpoint(raftmc, tmp_path):
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c2.cfg"), workers=0, max_depth=5, count_final_level=True) as mc:
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.set_checkpoint(str(tmp_path / "x.ckpt"), 1)
    assert e.value.code == -4


def test_describe_c2(raftmc):
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c2.cfg")) as mc:
        d = mc.describe()
    assert d["spec"] == "raft_original" and (d["N"], d["NV"], d["MaxTerm"], d["MaxLogLen"], d["MaxMsgDomain"]) == (3, 2, 3, 2, 5)
    assert d["invariants"] == ["ElectionSafety", "LogMatching"]
    assert d["state_bytes_stored"] % 16 == 0


@pytest.mark.parametrize("edit,code", [
    ((("    ElectionSafety\n", "    ElectionSafety\n    NotAnInvariant\n"),), -4),
    ((("    BoundedLogs\n", ""),), -4),                       # unbounded logs: refused
    ((("MaxMsgDomain = 5", "MaxMsgDomain = 9"),), -4),        # shape not compiled in
    ((("INIT Init", "INIT Init\nSYMMETRY perms"),), -4),
    ((("CONSTANTS", "CONSTANTS {"),), -3),
])
def test_open_rejects_unsupported(raftmc, edit, code):
    cfg = cfg_variant(os.path.join(CONFIGS, "c2.cfg"), edit)
    with pytest.raises(raftmc.RaftMCError) as e:
        raftmc.ModelChecker(ORIG_MC, cfg)
    assert e.value.code == code


def test_describe_membership_shipped(raftmc):
    from oracle_util import MEMB_MC
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, "membership_shipped.cfg")) as mc:
        d = mc.describe()
    assert d["spec"] == "tlc_membership" and (d["N"], d["NV"], d["MK"]) == (3, 2, 18)
    assert d["symmetry"] is True and d["permutations"] == 6 and d["next"] == "NextAsyncCrash"
    assert d["init_server_mask"] == 7 and d["invariants"][:3] == ["LeaderVotesQuorum", "CandidateTermNotInLog", "ElectionSafety"]
    assert d["state_bytes_stored"] % 16 == 0


def test_describe_membership_four_servers(raftmc):
    from oracle_util import MEMB_MC
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, "memb_four.cfg")) as mc:
        d = mc.describe()
    assert (d["N"], d["MK"], d["permutations"], d["next"], d["init_server_mask"]) == (4, 32, 24, "NextDynamic", 7)


@pytest.mark.parametrize("edit,code", [
    ((("VIEW vars\n", ""),), -4),                                           # history would be fingerprinted
    ((("    BoundedLogSize\n", ""),), -4),                                  # unbounded logs
    ((("    LogMatching\n", "    LogMatching\n    NotAnInvariant\n"),), -4),
    ((("NEXT NextAsyncCrash", "NEXT NextFoo"),), -4),
    ((("    Server = {s1, s2, s3}", "    Server = {s1, s2, s3, s4, s5}"),), -4),   # shape not compiled in
    ((("    Server = {s1, s2, s3}", "    Server = {s1, s2, s3, s4}"),     # two prefix masks of 24 bindings
      ("    CleanStartUntilTwoLeaders\n", "    CleanStartUntilTwoLeaders\n    MajorityOfClusterRestarts_constraint\n"
                                        "    CommitWhenConcurrentLeaders_unique\n")), -4),
])
def test_membership_open_rejects_unsupported(raftmc, edit, code):
    from oracle_util import MEMB_MC
    cfg = cfg_variant(os.path.join(CONFIGS, "membership_shipped.cfg"), edit)
    with pytest.raises(raftmc.RaftMCError) as e:
        raftmc.ModelChecker(MEMB_MC, cfg)
    assert e.value.code == code


def test_run_without_device_fails_loudly(raftmc):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c1.cfg")) as mc:
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.run()
    assert e.value.code == -5


def test_kernels_short_branch_and_no_scratch():
    """Every gfx950 kernel in libraftmc.so stays within the short-branch range
    (no s_getpc/s_setpc long-branch sequences) and uses no scratch: round 1
    found a membership kernel that outgrew the branch range computing wrong
    fingerprints and faulting; and no vector store / atomic issues while a scalar
    load of device memory is outstanding (round 3: a counter store overtook the scalar load of the
    same counter and the GPU intermittently lost a chunk's new states)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_isa.py")], capture_output=True, text=True)
    import json
    ks = json.loads(r.stdout)
    assert len(ks) > 40 and any("memb_fingerprint" in k for k in ks) and any("orig_generate" in k for k in ks)
    bad = {k: v for k, v in ks.items() if v["long_branches"] or v["scratch_bytes"] or v["smem_store_hazards"]}
    assert not bad, bad


def test_fingerprint_kernels_keep_two_waves_per_simd():
    """The symmetric-fingerprint kernels hold their bag in 64 KB of LDS per workgroup, so a CU runs
    two workgroups = two waves per SIMD, which needs <= 256 VGPRs + AGPRs per lane: one more
    register and the kernel drops to one wave per SIMD (round 4: a per-message ConfigEntry mask
    took TLC-mode C3 from 1.27 to 1.90 s of fingerprint time)."""
    import json
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_isa.py")], capture_output=True, text=True)
    ks = {k: v for k, v in json.loads(r.stdout).items() if "memb_fingerprint" in k}
    assert ks
    over = {k: (v.get("vgprs"), v.get("agprs")) for k, v in ks.items() if (v.get("vgprs") or 0) + (v.get("agprs") or 0) > 256}
    assert not over, over


def test_generated_code_objects_short_branch_and_ordered_stores():
    """The same check over the generated path's prebuilt code objects (`_build/tlagen_co/*.hsaco`,
    hiprtc output for every spec `prebuild.py` compiles), kernels and the device functions the
    front end outlines: no long branches, no store issued under an outstanding scalar load.  They
    may use scratch (a call stack and each lane's variable-handle array)."""
    import glob
    import json
    import subprocess
    import sys
    cos = sorted(glob.glob(os.path.join(ROOT, "raft-tla_amd", "_build", "tlagen_co", "*.hsaco")))
    assert len(cos) >= 10, "build() prebuilds the generated specs' code objects"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_isa.py"), *cos], capture_output=True, text=True)
    ks = json.loads(r.stdout)
    assert sum(k.endswith(":tlg_expand_k") for k in ks) == len(cos)
    bad = {k: v for k, v in ks.items() if v["long_branches"] or v["smem_store_hazards"]}
    assert not bad and r.returncode == 0, bad


def test_isa_check_refuses_an_unprovided_dynamic_stack(tmp_path):
    """The stack rule of scripts/check_isa.py (round 4's illegal-address fault): a code
    object whose kernel recurses (dynamic stack) but whose generated source lacks the recursion marker
    runs with the runtime's default per-lane stack, so the check fails it; the same code with the
    marker (the backend then raises the stack to 16 KB per lane) passes."""
    import json
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(ROOT, "raft-tla_amd", "csrc", "tlagen"))
    from prebuild import OPTS, key_of
    body = ("#include <hip/hip_runtime.h>\n"
            "__device__ __attribute__((noinline)) int walk(int n, int* p) { if (n <= 0) return p[0]; int a[8]; "
            "for (int k = 0; k < 8; ++k) a[k] = p[k] + n; return walk(n - 1, a) + a[n & 7]; }\n"
            "extern \"C\" __global__ void tlg_expand_k(int* p, int n) { p[threadIdx.x] = walk(n, p); }\n")
    rcs = {}
    for marked in (False, True):
        d = tmp_path / ("m" if marked else "u")
        d.mkdir()
        src = body + ("// guard: if (depth > tlv::kMaxRecDepth) { ... }\n" if marked else "")
        (d / "x.gen.hip").write_text(src)
        co = d / (key_of(src) + ".hsaco")
        subprocess.run(["/opt/rocm/bin/hipcc", "--genco", *OPTS, "-o", str(co), "-x", "hip", str(d / "x.gen.hip")], check=True)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_isa.py"), str(co)], capture_output=True, text=True)
        k = json.loads(r.stdout)["tlg_expand_k"]
        assert k["dynamic_stack"] and k["raised_stack"] == marked
        rcs[marked] = r.returncode
    assert rcs == {False: 1, True: 0}


PUNCT_CWCL = os.path.join(CONFIGS, "scen_CommitWhenConcurrentLeaders_punct.cfg")


def trace_fixture_text(name):
    import json
    from oracle_util import GOLDEN, tla_text
    return tla_text(json.load(open(os.path.join(GOLDEN, name)))["value"])


def test_prefix_constraint_without_trace_is_refused(raftmc):
    """configs/ holds no raft.tla, so the wrapper's punctuated-search constraint has no
    golden trace: mc_run refuses before touching a device (no silent 'always true')."""
    from oracle_util import MEMB_MC
    with raftmc.ModelChecker(MEMB_MC, PUNCT_CWCL) as mc:
        assert mc.describe()["history_prefixes"] == {"CommitWhenConcurrentLeaders_unique": -1}
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.run()
    assert e.value.code == -4 and "golden history trace" in str(e.value)


def test_set_history_prefix(raftmc):
    from oracle_util import MEMB_MC
    with raftmc.ModelChecker(MEMB_MC, PUNCT_CWCL) as mc:
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.set_history_prefix("BoundedTerms", "<<>>")
        assert e.value.code == -1
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.set_history_prefix("CommitWhenConcurrentLeaders_unique", '<<[action |-> "Timeout", executedOn |-> s1')
        assert e.value.code == -3
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.set_history_prefix("CommitWhenConcurrentLeaders_unique", "[local |-> <<>>]")
        assert e.value.code == -3
        mc.set_history_prefix("CommitWhenConcurrentLeaders_unique", trace_fixture_text("concurrent_leaders_trace.json"))
        d = mc.describe()
    assert d["history_prefixes"] == {"CommitWhenConcurrentLeaders_unique": 20} and d["prefix_bindings"] == 6


def test_prefix_taken_from_extended_module(raftmc, tmp_path):
    """As TLC resolves EXTENDS: the wrapper's `EXTENDS raft` finds raft.tla next to it, and
    the constraint's trace literal comes from the operator's definition there."""
    from oracle_util import MEMB_MC
    wrapper = tmp_path / "raft_membership_mc.tla"
    wrapper.write_text(open(MEMB_MC).read())
    trace = trace_fixture_text("commit_when_concurrent_leaders_trace.json")
    (tmp_path / "raft.tla").write_text(
        "---- MODULE raft ----\n"
        "MajorityOfClusterRestarts_constraint ==\n"
        "    \\E s1, s2, s3 \\in Server :\n"
        "        /\\ Cardinality({s1, s2, s3}) = 3\n"
        "        /\\ LET  CommitWhenConcurrentLeaders_trace == " + trace + "\n"
        "                maxLen == Min({Len(CommitWhenConcurrentLeaders_trace[\"global\"]), Len(history[\"global\"])})\n"
        "            IN IsPrefix(SubSeq(CommitWhenConcurrentLeaders_trace[\"global\"], 1, maxLen), history[\"global\"])\n"
        "\n"
        "Next == TRUE\n"
        "====\n")
    with raftmc.ModelChecker(str(wrapper), os.path.join(CONFIGS, "scen_MajorityOfClusterRestarts_punct.cfg")) as mc:
        assert mc.describe()["history_prefixes"] == {"MajorityOfClusterRestarts_constraint": 28}


def test_checkpoint_api_scope(raftmc):
    """Checkpoints exist for both spec families (TLC -checkpoint / -recover); a negative
    interval is refused."""
    lib = raftmc.load_library()
    with raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, "membership_shipped.cfg")) as mc:
        assert lib.mc_set_checkpoint(mc.h, b"/tmp/x.ckpt", 1) == 0
        assert lib.mc_set_checkpoint(mc.h, b"/tmp/x.ckpt", -1) == -1
        assert lib.mc_set_recover(mc.h, b"/tmp/x.ckpt") == 0
        mc.set_recover(None)
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c1.cfg")) as mc:
        assert lib.mc_set_checkpoint(mc.h, b"/tmp/x.ckpt", -1) == -1
        mc.set_checkpoint("/tmp/x.ckpt", 2)
        mc.set_checkpoint(None)
        mc.set_recover(None)


def test_action_location_in_extended_module(raftmc, tmp_path):
    """TLC's trace header names the action and the span of its definition body
    ("line L1, col C1 to line L2, col C2 of module M"): found through the wrapper's
    `EXTENDS raft`, parameters and `==` skipped, comments after the last token excluded."""
    wrapper = tmp_path / "raft_original_mc.tla"
    wrapper.write_text(open(ORIG_MC).read())
    (tmp_path / "raft.tla").write_text(
        "------ MODULE raft ------\n"                                  # 1
        "\\* Server i times out.\n"                                     # 2
        "Timeout(i) == /\\ state[i] = Follower\n"                       # 3
        "              \\* a comment inside the body\n"                 # 4
        "              /\\ UNCHANGED <<log>> \\* trailing comment\n"    # 5
        "\n"                                                            # 6
        "\\* next unit\n"                                               # 7
        "Restart(i) ==\n"                                               # 8
        "    /\\ state' = [state EXCEPT ![i] = Follower]\n"             # 9
        "    (* block\n"                                                # 10
        "       comment *)\n"                                           # 11
        "----\n"                                                        # 12
        "RestartAll == \\A i \\in Server : Restart(i)\n"                # 13
        "====\n")
    with raftmc.ModelChecker(str(wrapper), os.path.join(CONFIGS, "c1.cfg")) as mc:
        assert mc.action_location("Timeout") == "line 3, col 15 to line 5, col 34 of module raft"
        assert mc.action_location("Restart") == "line 9, col 5 to line 9, col 46 of module raft"
        assert mc.action_location("RestartAll") == "line 13, col 15 to line 13, col 42 of module raft"
        assert mc.action_location("Rest") is None            # a prefix of a defined name is not a definition
        assert mc.action_location("BoundedTerms") == "line 17, col 17 to line 17, col 59 of module raft_original_mc"


def test_action_location_without_module(raftmc):
    """configs/ holds no raft.tla: headers stay "<Action>" and the lookup reports absence."""
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c1.cfg")) as mc:
        assert mc.action_location("Timeout") is None
        assert "Timeout" in mc.lib.mc_last_error(mc.h).decode()


def test_library_is_built_from_this_tree():
    """mc_source_hash (compiled in by raft-tla_amd/Makefile) equals the hash of the sources next to
    the package: a stale libraftmc.so is refused at load time, so a GPU run executes HEAD's sources."""
    import importlib
    rm = importlib.import_module("raft-tla_amd.raftmc")
    lib = rm.load_library()
    assert lib.mc_source_hash().decode() == rm.source_hash()


REF_MEMB = "/root/reference/tlc_membership"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_MEMB, "raft.tla")), reason="the reference exists only in the build container")
def test_open_reference_tlc_membership_unmodified(raftmc):
    """The drop-in claim on the reference's own files: mc_open takes the unmodified
    tlc_membership/raft.tla and raft.cfg (as `tlc2.TLC -config raft.cfg raft.tla` would) and resolves
    the shipped model — 3 servers, Value {1, 2}, SYMMETRY perms in TLC's rule (the default), VIEW
    vars, NEXT NextAsyncCrash, the 12 constraints and 8 invariants of raft.cfg:37-87.  Container-only
    (the reference is not on the GPU box); reads nothing but the reference's text, runs no GPU work."""
    with raftmc.ModelChecker(os.path.join(REF_MEMB, "raft.tla"), os.path.join(REF_MEMB, "raft.cfg")) as mc:
        d = mc.describe()
    assert d["spec"] == "tlc_membership" and (d["N"], d["NV"]) == (3, 2) and d["init_server_mask"] == 7
    assert d["symmetry"] is True and d["permutations"] == 6 and d["symmetry_mode"] == "tlc"
    assert d["next"] == "NextAsyncCrash" and d["check_deadlock"] is True and d["workers"] == 1
    assert d["invariants"] == ["LeaderVotesQuorum", "CandidateTermNotInLog", "ElectionSafety", "LogMatching",
                               "VotesGrantedInv", "QuorumLogInv", "MoreUpToDateCorrect", "LeaderCompleteness"]
    assert len(d["constraints"]) == 12


def test_sharded_runs_refuse_checkpoints(raftmc, tmp_path):
    """Checkpoint/recover are single-GPU features: a sharded run on a handle that has either set
    fails with MC_E_UNSUPPORTED before any device work, instead of silently ignoring them."""
    import ctypes
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c1.cfg")) as mc:
        mc.set_checkpoint(str(tmp_path / "x.ckpt"), 1)
        mc.lib.mc_shard_open.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        assert mc.lib.mc_shard_open(mc.h, 0, 2) == -4
        assert b"single-GPU" in mc.lib.mc_last_error(mc.h)
        mc.set_checkpoint(None)
        mc.set_recover(str(tmp_path / "x.ckpt"))
        hs = (ctypes.c_void_p * 1)(mc.h)
        mc.lib.mc_shard_run_loopback.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32]
        assert mc.lib.mc_shard_run_loopback(hs, 1) == -4


def test_n_gpus_options(raftmc):
    """mc_opts.n_gpus: 1..8 GPUs of the node for one search (no GPU work at mc_open); out of range
    is MC_E_INVALID; a multi-GPU handle refuses checkpoints (single-GPU runs only) when it runs."""
    for n in (0, 9):
        with pytest.raises(raftmc.RaftMCError) as e:
            raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c1.cfg"), n_gpus=n)
        assert e.value.code == -1
    for tla, cfg in ((ORIG_MC, "c1.cfg"), (MEMB_MC, "membership_shipped.cfg")):
        with raftmc.ModelChecker(tla, os.path.join(CONFIGS, cfg), n_gpus=4) as mc:
            assert mc.describe()["n_gpus"] == 4
