#!/bin/bash
# Round-4 GPU session: the GPU parity suite, the NewlyJoinedBecomeLeader scenario probe and a bench
# line.  Every GPU step has its own time limit and the steps are chained: the first failure ends it.
OUT=${1:-gpurun_out/r4a}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/steps.txt"; tail -3 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/scen_probe.py scen_NewlyJoinedBecomeLeader > "$OUT/njbl.jsonl" 2>&1
rc=$?; echo "njbl rc=$rc" | tee -a "$OUT/steps.txt"; cat "$OUT/njbl.jsonl"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/steps.txt"; cut -c1-1500 "$OUT/bench.jsonl"
exit $rc
