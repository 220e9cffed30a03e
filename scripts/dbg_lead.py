"""Debug probe: level sizes of small / C2 searches in both pipelines, repeated (nondeterminism check)."""
import importlib, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rm = importlib.import_module("raft-tla_amd")
TLA = os.path.join(ROOT, "configs", "raft_original_mc.tla")
tag = os.environ.get("TAG", "")
for rep in range(3):
    for cfg, depth in (("c2", 3), ("c2", 12)):
        for workers in (1, 0):
            r = rm.check(TLA, os.path.join(ROOT, "configs", cfg + ".cfg"), workers=workers, max_depth=depth,
                         fp_table_bytes=1 << 28, state_store_bytes=4 << 30)
            print(tag, rep, cfg, workers, r, [lv[0] for lv in r.levels][-3:], flush=True)
