#!/bin/bash
O=gpurun_out/r4x; mkdir -p $O
RAFTMC_LIB=raft-tla_amd/_build_var/fpprof/libraftmc.so timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_prof.jsonl 2>&1 || exit 1
grep FP_PROF $O/c3_prof.jsonl; cut -c1-400 $O/c3_prof.jsonl | tail -1
