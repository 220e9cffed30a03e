#!/bin/bash
# One GPU session on the box: parity tests, a short bench, optionally a rocprofv3 kernel-stats pass.
# Every GPU step has its own time limit; a step that ends by a signal / timeout (rc >= 124) ends
# the session.
OUT=${1:-gpurun_out/s}
TESTS=${2:-tests/test_gpu.py tests/test_gpu_shard.py tests/test_gpu_membership.py}
PROF=${3:-0}
mkdir -p "$OUT"
if [ "$TESTS" != "none" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?
  echo "pytest rc=$rc" | tee -a "$OUT/steps.txt"
  tail -4 "$OUT/pytest.log"
  if [ $rc -ge 124 ]; then exit $rc; fi
fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > "$OUT/bench.jsonl" 2> "$OUT/bench.err"
rc=$?
echo "bench rc=$rc" | tee -a "$OUT/steps.txt"
cut -c1-1800 "$OUT/bench.jsonl"
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "$PROF" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
  rc=$?
  echo "rocprof rc=$rc" | tee -a "$GRAFT_REPO_ROOT/$OUT/steps.txt"
  find "$GRAFT_REPO_ROOT/$OUT/prof" -name "*kernel_stats.csv" -exec head -20 {} \;
fi
exit $rc
