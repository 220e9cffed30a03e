#!/bin/bash
# GPU suite; C3 in TLC's SYMMETRY mode; the generated path on C2; the bench
O=${OUT:-gpurun_out/r4k}; mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_tlc.jsonl 2>&1 || exit 1
cut -c1-700 $O/c3_tlc.jsonl
timeout -k 10 300 python -u scripts/tlagen_c2_time.py 8 > $O/tlagen_c2.jsonl 2>&1 || exit 1
cat $O/tlagen_c2.jsonl
timeout -k 10 600 python -u bench.py > $O/bench.jsonl 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-800 $O/bench.jsonl
exit $rc
