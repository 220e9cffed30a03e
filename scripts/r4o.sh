#!/bin/bash
O=${OUT:-gpurun_out/r4o}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_membership.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_tlc.jsonl 2>&1 || exit 1
cut -c1-600 $O/c3_tlc.jsonl
timeout -k 10 200 python -u scripts/memb_probe.py memb_four --orbit > $O/c3_orbit.jsonl 2>&1 || exit 1
cut -c1-600 $O/c3_orbit.jsonl
RAFTMC_LIB=raft-tla_amd/_build_var/fpprof/libraftmc.so timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_prof.jsonl 2>&1 || exit 1
grep FP_PROF $O/c3_prof.jsonl
