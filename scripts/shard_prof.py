"""Time the native sharded level loop on one GPU (in-process loopback ranks) beside the
single-GPU search on the same config: wall time per run and the per-kernel HIP-event times.

    python scripts/shard_prof.py [CFG] [--worlds 1,2] [--runs 3]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
TLA = os.path.join(ROOT, "configs", "raft_original_mc.tla")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg", nargs="?", default=os.path.join(ROOT, "configs", "c2.cfg"))
    ap.add_argument("--worlds", default="1,2")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--table", type=int, default=4 << 30)
    ap.add_argument("--store", type=int, default=8 << 30)
    args = ap.parse_args()
    mod = importlib.import_module("raft-tla_amd")
    shard = importlib.import_module("raft-tla_amd.shard")
    with mod.ModelChecker(TLA, args.cfg, seed=0x5EED) as mc:
        mc.run()
        t0 = time.perf_counter()
        for _ in range(args.runs):
            r = mc.run()
        ms = (time.perf_counter() - t0) / args.runs * 1e3
    print(json.dumps({"mode": "single", "ms": ms, "distinct": r.distinct,
                      "kernels": {k: round(v["ms"], 3) for k, v in r.kernels.items()}}), flush=True)
    for w in [int(x) for x in args.worlds.split(",")]:
        kw = dict(fp_table_bytes=args.table // w, state_store_bytes=args.store // w, seed=0x5EED)
        shard.check_loopback(TLA, args.cfg, w, **kw)
        t0 = time.perf_counter()
        for _ in range(args.runs):
            out = shard.check_loopback(TLA, args.cfg, w, **kw)
        ms = (time.perf_counter() - t0) / args.runs * 1e3
        print(json.dumps({"mode": "loopback", "world": w, "ms_incl_open": ms, "distinct": out[0].distinct,
                          "generated": out[0].generated, "seconds": [round(o.seconds * 1e3, 3) for o in out],
                          "kernels": [{k: (round(v["ms"], 3), v["launches"]) for k, v in o.kernels.items()} for o in out]}),
              flush=True)


if __name__ == "__main__":
    main()
