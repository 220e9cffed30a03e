"""C-ABI boundary: the library loads, exports every symbol include/raftmc.h
declares, resolves cfgs (no GPU needed) and fails loudly without a device."""
import os
import re

import pytest

from oracle_util import CONFIGS, ORIG_MC, ROOT, cfg_variant

HEADER = os.path.join(ROOT, "include", "raftmc.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(mc_\w+)\s*\(", text, re.M)))


def test_header_and_python_mirror_agree(raftmc):
    assert declared_functions() == sorted(raftmc.EXPORTS)


def test_library_exports_every_declared_symbol(raftmc):
    lib = raftmc.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name


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


def test_membership_has_no_gpu_backend_yet(raftmc):
    from oracle_util import MEMB_MC
    with pytest.raises(raftmc.RaftMCError) as e:
        raftmc.ModelChecker(MEMB_MC, os.path.join(CONFIGS, "membership_shipped.cfg"))
    assert e.value.code == -4


def test_run_without_device_fails_loudly(raftmc):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with raftmc.ModelChecker(ORIG_MC, os.path.join(CONFIGS, "c1.cfg")) as mc:
        with pytest.raises(raftmc.RaftMCError) as e:
            mc.run()
    assert e.value.code == -5
