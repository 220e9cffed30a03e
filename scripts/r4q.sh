#!/bin/bash
O=${OUT:-gpurun_out/r4q}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_tlagen.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/tlagen_c2_time.py 8 16 > $O/tlagen_c2.jsonl 2>&1 || exit 1
cat $O/tlagen_c2.jsonl
