#!/bin/bash
# Round-4 GPU session: the GPU parity suite, the NewlyJoinedBecomeLeader scenario probe, then
# bench A/B variants (scripts/ab_env.sh specs).  Every GPU step has its own time limit and the
# steps are chained: the first failure ends the session.
OUT=${1:-gpurun_out/r4a}; shift
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/steps.txt"; tail -3 "$OUT/pytest.log"
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${NJBL:-0}" = "1" ]; then
  timeout -k 10 300 python -u scripts/scen_probe.py scen_NewlyJoinedBecomeLeader > "$OUT/njbl.jsonl" 2>&1
  rc=$?; echo "njbl rc=$rc" | tee -a "$OUT/steps.txt"; cat "$OUT/njbl.jsonl"
  [ $rc -ne 0 ] && exit $rc
fi
[ $# -gt 0 ] && bash scripts/ab_env.sh "$OUT" "$@"
