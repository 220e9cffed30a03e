"""raftmc: MI355X-native explicit-state BFS model checker for the dranov/raft-tla specs.

The product is libraftmc.so (HIP/gfx950 kernels behind the C ABI in
include/raftmc.h); `raftmc` is the host-side mirror of TLC's contract.
"""
from .raftmc import (ABI_VERSION, EXPORTS, LIB_PATH, ModelChecker, RaftMCError, Result, check,  # noqa: F401
                     load_library, tlc_main)
