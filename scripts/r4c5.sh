#!/bin/bash
# count_final_level: GPU tests, then c5v2 to depth 13 on one MI355X (the last level counted, not stored)
O=${OUT:-gpurun_out/r4c5}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "count_final_level or c5v2_deep" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
C5_CFG=c5v2.cfg C5_WORKERS=0 C5_COUNT_FINAL=1 C5_TABLE_GB=64 C5_STORE_GB=120 RAFTMC_PROGRESS=1 \
  timeout -k 10 400 python -u scripts/c5_probe.py 12 13 > $O/c5v2_d13.jsonl 2> $O/c5v2_d13.err
rc=$?; echo "probe rc=$rc"; cut -c1-1200 $O/c5v2_d13.jsonl; tail -5 $O/c5v2_d13.err
exit $rc
