#!/bin/bash
# Round measurement pass on one MI355X (run through gpurun from the repo root):
# GPU test suite, smoke, bench, rocprofv3 kernel stats and PMC HBM-traffic passes.
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
OUT=${OUT:-gpurun_out/round}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_stats" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > "$OUT/prof_stats.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra > "$OUT/pmc_write.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU -d "$OUT/pmc_valu" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra > "$OUT/pmc_valu.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_memb" -o run -- python3 scripts/memb_probe.py memb_four 0 > "$OUT/prof_memb.log" 2>&1
rc=$?
[ $rc -eq 0 ] && timeout -k 10 200 python3 scripts/shard_probe.py > "$OUT/shard_probe.jsonl" 2> "$OUT/shard_probe.err"
rc2=$?
echo "exit $rc $rc2"
