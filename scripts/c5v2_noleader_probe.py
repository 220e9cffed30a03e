"""Probe: C5v2 NoLeader FIFO search to the first election (depth 12), with per-phase timestamps and a
stack dump every 30 s (so a slow phase is visible before the box's silence limit)."""
import faulthandler
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
faulthandler.dump_traceback_later(30, repeat=True)
os.environ["RAFTMC_PROGRESS"] = "1"
rm = importlib.import_module("raft-tla_amd")
cfg = os.path.join(ROOT, "configs", sys.argv[1] if len(sys.argv) > 1 else "c5e_noleader.cfg")
workers = int(sys.argv[2]) if len(sys.argv) > 2 else 1
store = int(float(sys.argv[3]) * (1 << 30)) if len(sys.argv) > 3 else 112 << 30
table = int(float(sys.argv[4]) * (1 << 30)) if len(sys.argv) > 4 else 32 << 30
t0 = time.time()
with rm.ModelChecker(os.path.join(ROOT, "configs", "raft_original_mc.tla"), cfg, fp_table_bytes=table,
                     state_store_bytes=store, workers=workers) as mc:
    print("open %.1f s" % (time.time() - t0), mc.describe(), flush=True)
    r = mc.run()
    print("run %.1f s" % (time.time() - t0), r, r.error, flush=True)
    print([lv for lv in r.levels], flush=True)
    print(r.kernels, flush=True)
    print(r.trace_text[-3000:] if getattr(r, "trace_text", None) else "", flush=True)
