import importlib, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
m = importlib.import_module("raft-tla_amd")
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
r = m.check(R + "/configs/raft_original_mc.tla", R + "/configs/c2.cfg")
print(r)
for k, lv in enumerate(r.levels): print(k + 1, lv)
print(r.actions)
