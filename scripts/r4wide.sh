#!/bin/bash
# 16-B arena moves on the generated path: GPU tlagen tests, then C2 timing
O=${OUT:-gpurun_out/r4wide}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tlagen.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u scripts/tlagen_c2_time.py 8 > $O/tlagen_c2.jsonl 2>&1 || exit 1
cut -c1-400 $O/tlagen_c2.jsonl
