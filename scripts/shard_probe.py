"""Time the sharded raft_original pipeline at world 1 against the single-GPU pipeline on C2: the
per-rank cost of the sharded kernels, with the Python level loop (torch transport, no
communication at world 1) and with the library's native RCCL loop (a one-rank communicator:
self-exchanges are device copies).  A development tool.

    python scripts/shard_probe.py [CFG] [--lib LIBRAFTMC]     (--lib: an experiment build, RAFTMC_LIB)
"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--lib" in sys.argv:
    k = sys.argv.index("--lib")
    os.environ["RAFTMC_LIB"] = os.path.join(ROOT, sys.argv[k + 1])
    del sys.argv[k:k + 2]
raftmc = importlib.import_module("raft-tla_amd")
shard = importlib.import_module("raft-tla_amd.shard")
cfg = os.path.join(ROOT, "configs", (sys.argv[1] if len(sys.argv) > 1 else "c2") + ".cfg")
tla = os.path.join(ROOT, "configs", "raft_original_mc.tla")
sc = shard.ShardedChecker(tla, cfg, 0, 1, seed=0x5EED)
sc.run()
t0 = time.perf_counter()
r = sc.run()
ms = (time.perf_counter() - t0) * 1e3
sc.close()
print(json.dumps({"mode": "sharded_w1", "distinct": r.distinct, "generated": r.generated, "ms": ms,
                  "kernels_ms": {k: round(v["ms"], 2) for k, v in r.kernels.items()}}), flush=True)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
sc = shard.ShardedChecker(tla, cfg, 0, 1, seed=0x5EED, transport="rccl")
sc.run()
t0 = time.perf_counter()
r = sc.run()
ms = (time.perf_counter() - t0) * 1e3
sc.close()
dist.destroy_process_group()
print(json.dumps({"mode": "sharded_w1_rccl_native", "distinct": r.distinct, "generated": r.generated, "ms": ms,
                  "kernels_ms": {k: round(v["ms"], 2) for k, v in r.kernels.items()}}), flush=True)
with raftmc.ModelChecker(tla, cfg, seed=0x5EED) as mc:
    mc.run()
    t0 = time.perf_counter()
    r = mc.run()
    ms = (time.perf_counter() - t0) * 1e3
print(json.dumps({"mode": "single", "distinct": r.distinct, "generated": r.generated, "ms": ms,
                  "kernels_ms": {k: round(v["ms"], 2) for k, v in r.kernels.items()}}), flush=True)
