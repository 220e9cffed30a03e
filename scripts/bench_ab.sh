#!/bin/bash
# A/B of bench.py runs on one box (C2, no CPU baseline), optionally after a GPU test file:
#   bash scripts/bench_ab.sh OUT "TESTS|none" "name|bench args" ...
set -o pipefail
O=$1; T=$2; shift 2; mkdir -p $O
if [ "$T" != "none" ]; then
  timeout -k 10 500 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -ge 124 ] && exit $rc
fi
for spec in "$@"; do
  IFS='|' read -r name args <<< "$spec"
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $args > $O/$name.jsonl 2> $O/$name.err || { tail -3 $O/$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$name.jsonl').read().strip().splitlines()[-1])
f=d.get('tlc_workers_1',{}).get('ms_per_step')
print('$name', round(d['ms_per_step'],2), {k:round(v['ms'],2) for k,v in d['kernels'].items()}, round(d['config']['kernel_ms_per_run'],2), f and round(f,2))
"
done
