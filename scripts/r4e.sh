#!/bin/bash
# full GPU suite, C3 in both SYMMETRY modes (TLC's rule: the closed-form first message stage), bench
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/memb_probe.py memb_four > $O/c3_tlc.jsonl 2>&1 && timeout -k 10 300 python -u scripts/memb_probe.py memb_four --orbit > $O/c3_orbit.jsonl 2>&1
rc=$?; echo "c3 rc=$rc"; cut -c1-600 $O/c3_tlc.jsonl $O/c3_orbit.jsonl
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-3000 $O/bench.jsonl
exit $rc
