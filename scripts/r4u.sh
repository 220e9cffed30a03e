#!/bin/bash
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_nar2.jsonl 2>&1 || exit 1
for v in nar0 nar1 nar4; do
  RAFTMC_LIB=raft-tla_amd/_build_var/$v/libraftmc.so timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_$v.jsonl 2>&1 || exit 1
done
for f in nar0 nar1 nar2 nar4; do python3 -c "
import json; d=json.loads(open('$O/c3_$f.jsonl').read().strip().splitlines()[-1]); print('$f', d['distinct'], d['run_s'], d['kernels_ms']['memb_fingerprint'])"; done
