#!/bin/bash
# C3 TLC mode with the stage-cycle profile build, and the product build for comparison
O=gpurun_out/r4m; mkdir -p $O
RAFTMC_LIB=raft-tla_amd/_build_var/fpprof/libraftmc.so timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_prof.jsonl 2>&1 || exit 1
cut -c1-600 $O/c3_prof.jsonl; grep FP_PROF $O/c3_prof.jsonl
timeout -k 10 200 python -u scripts/memb_probe.py memb_four --orbit > $O/c3_orbit.jsonl 2>&1 || exit 1
cut -c1-600 $O/c3_orbit.jsonl
