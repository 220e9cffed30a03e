#!/bin/bash
# Round-3 measurement, part 1: GPU test suite, the default bench line, C3 in both symmetry modes.
set -u
OUT=${1:-gpurun_out/r3m}
mkdir -p $OUT
PYT="python -u -m pytest -v --timeout 170 --timeout-method thread"
bash scripts/r3_session.sh $OUT "step pytest 720 $PYT tests -m gpu --durations=40" || exit $?
bash scripts/r3_session.sh $OUT "step bench 420 python -u bench.py" "step c3 200 python -u scripts/memb_probe.py memb_four" "step c3orbit 200 python -u scripts/memb_probe.py memb_four --orbit"
