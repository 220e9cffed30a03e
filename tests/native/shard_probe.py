# GPU probe: sharded world=1 timing on C2 vs the single-GPU pipeline, and the C2 K=6 size.
import importlib, os, sys, time
R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo"); sys.path.insert(0, R)
m = importlib.import_module("raft-tla_amd"); sh = importlib.import_module("raft-tla_amd.shard")
tla = R + "/configs/raft_original_mc.tla"; cfg = R + "/configs/c2.cfg"
sc = sh.ShardedChecker(tla, cfg, 0, 1, seed=0x5EED)
sc.run(); t = time.time(); r = sc.run(); print("sharded w1", r, "%.1f ms" % ((time.time() - t) * 1e3), {k: round(v["ms"], 2) for k, v in r.kernels.items()}, flush=True)
sc.close()
import tempfile
c6 = open(cfg).read().replace("MaxMsgDomain = 5", "MaxMsgDomain = 6"); p = tempfile.mktemp(suffix=".cfg"); open(p, "w").write(c6)
mc = m.ModelChecker(tla, p, seed=0x5EED, fp_table_bytes=1 << 34, state_store_bytes=120 << 30)
t = time.time(); r = mc.run(); print("K6", r, "%.1f ms" % ((time.time() - t) * 1e3), {k: round(v["ms"], 2) for k, v in r.kernels.items()}, r.error, flush=True)
