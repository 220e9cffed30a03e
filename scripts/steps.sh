#!/bin/bash
# One GPU session as a list of named steps (run through gpurun from the repo root):
#   bash scripts/steps.sh OUT STEP [STEP ...]
# Every step has its own time limit and writes under OUT; the first failing step ends the session
# (after a GPU fault, abort, timeout or hang nothing else touches the GPU in that call).
#   tests[=EXPR]        pytest -m gpu -x (optionally -k EXPR); testsall[=EXPR]: without -x
#   smoke               __graft_entry__.smoke()
#   bench               bench.py with its defaults (the driver's line)
#   c2[=NAME[=LIB]]     bench.py C2 only (no extras, no CPU baseline) with library LIB (default: the
#                       in-tree build), 8 timed steps; prints ms/step, kernels, seen-set probes
#   c2f[=NAME[=LIB]]    the C2 line and the FIFO (-workers 1) run beside it
#   c2t=GIB             the C2 line with a GIB-GiB seen-set (--fp-table-bytes), 8 timed steps
#   memb[=NAME[=LIB]]   scripts/memb_probe.py memb_four (C3, TLC's symmetry rule) with library LIB, twice
#   prof                rocprofv3 --kernel-trace --stats of a short C2 bench
#   c2_prof[=TAG]       rocprofv3 stats + FETCH/WRITE/SQ passes of C2, summarised (scripts/c2_prof.sh)
#   memb_prof           rocprofv3 stats + PMC passes of C3 (scripts/memb_prof.sh)
#   py=SCRIPT ARGS..    python3 SCRIPT with its arguments (':' separates them: py=scripts/x.py:a:b)
set -o pipefail
O=${1:?OUT}; shift
mkdir -p "$O"
export TMPDIR=/tmp
R=$(pwd)
pyn=0
for step in "$@"; do
  name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
  echo "== $step ($(date +%T))"
  case $name in
    tests|testsall)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      x=(-x); [ "$name" = testsall ] && x=()   # testsall: every test, not stopping at the first failure
      timeout -k 10 1500 python -u -m pytest tests -m gpu "${x[@]}" -v --timeout 300 --timeout-method thread "${k[@]}" > "$O/pytest.log" 2>&1
      rc=$?; tail -3 "$O/pytest.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      rc=$?; tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
      rc=$?; cut -c1-600 "$O/bench.json" ;;
    c2)
      n=${arg%%=*}; lib=${arg#*=}; [ "$lib" = "$arg" ] && lib=""; n=${n:-base}
      timeout -k 10 200 env ${lib:+RAFTMC_LIB=$lib} python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extra --fifo-steps 0 \
        > "$O/c2_$n.json" 2> "$O/c2_$n.err"
      rc=$?
      [ $rc -eq 0 ] && python3 -c "
import json
d = json.loads(open('$O/c2_$n.json').read().strip().splitlines()[-1])
print('$n', round(d['ms_per_step'], 2), {k: round(v['ms'], 2) for k, v in d['kernels'].items()}, d['config']['distinct_per_run'],
      'probes', d.get('dedup_set', {}).get('probes_per_run'))" ;;
    c2f)   # c2f[=NAME[=LIB]]: the C2 line and TLC -workers 1 (FIFO order) beside it
      n=${arg%%=*}; lib=${arg#*=}; [ "$lib" = "$arg" ] && lib=""; n=${n:-base}
      timeout -k 10 300 env ${lib:+RAFTMC_LIB=$lib} python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extra --fifo-steps 3 \
        > "$O/c2f_$n.json" 2> "$O/c2f_$n.err"
      rc=$?
      [ $rc -eq 0 ] && python3 -c "
import json
d = json.loads(open('$O/c2f_$n.json').read().strip().splitlines()[-1])
f = d['tlc_workers_1']
print('$n', round(d['ms_per_step'], 2), 'fifo', round(f['ms_per_step'], 2), {k: round(v, 2) for k, v in f['kernels_ms'].items()})" ;;
    c2t)
      timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extra --fifo-steps 0 \
        --fp-table-bytes $((arg << 30)) > "$O/c2t_$arg.json" 2> "$O/c2t_$arg.err"
      rc=$?
      [ $rc -eq 0 ] && python3 -c "
import json
d = json.loads(open('$O/c2t_$arg.json').read().strip().splitlines()[-1])
print('table $arg GiB', round(d['ms_per_step'], 2), {k: round(v['ms'], 2) for k, v in d['kernels'].items()}, d['config']['distinct_per_run'],
      'probes', d.get('dedup_set', {}).get('probes_per_run'))" ;;
    memb)
      n=${arg%%=*}; lib=${arg#*=}; [ "$lib" = "$arg" ] && lib=""; n=${n:-base}
      timeout -k 10 200 env ${lib:+RAFTMC_LIB=$lib} python3 scripts/memb_probe.py memb_four 0 0 > "$O/memb_$n.json" 2> "$O/memb_$n.err"
      rc=$?
      [ $rc -eq 0 ] && python3 -c "
import json
for l in open('$O/memb_$n.json').read().strip().splitlines():
    d = json.loads(l)
    print('$n', d['verdict'], d['distinct'], d['depth'], d['run_s'], d['kernels_ms'])" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_stats" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --fifo-steps 0 > "$O/prof_stats.log" 2>&1
      rc=$? ;;
    gaps)   # gaps[=EXTRA]: a C2 kernel trace (csv) and the device's idle time per run (scripts/kernel_gaps.py)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/gaps" -o run -- python3 bench.py --steps 3 --warmup 1 \
        --no-cpu-baseline --no-extra --fifo-steps 0 > "$O/gaps.log" 2>&1
      rc=$?
      if [ $rc -eq 0 ]; then
        f=$(find "$O/gaps" -name '*kernel_trace.csv' | sort | tail -n 1)
        python3 scripts/kernel_gaps.py "$f" "$O/kernel_gaps.json"; rc=$?
      fi ;;
    c2_prof)
      bash scripts/c2_prof.sh "${O#$R/}/c2_prof" "${arg:-r05}"; rc=$? ;;
    memb_prof)
      bash scripts/memb_prof.sh "${O#$R/}/memb_prof" "${arg:-r05}"; rc=$? ;;
    py)
      IFS=':' read -r -a a <<< "$arg"
      pyn=$((pyn + 1)); lg="$O/py_$(basename "${a[0]}" .py).log"
      [ "$pyn" -gt 1 ] && lg="$O/py_$(basename "${a[0]}" .py)_$pyn.log"   # (later py steps: _2, _3, ...)
      timeout -k 10 900 python3 -u "${a[@]}" > "$lg" 2>&1
      rc=$?; tail -3 "$lg" ;;
    *) echo "unknown step $name"; rc=2 ;;
  esac
  echo "== $step rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
