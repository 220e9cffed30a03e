#!/bin/bash
# the raft_original GPU suite (count_final_level included, c5v2 to depth 13)
O=${OUT:-gpurun_out/r4c5b}; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED" $O/pytest.log | grep -E "count_final|depth13|FAILED"; tail -3 $O/pytest.log
exit $rc
