#!/bin/bash
# A/B of bench.py runs (C2, no CPU baseline) on one box, each variant with its own environment:
#   bash scripts/ab_env.sh OUT "name|ENV=1 ENV2=x|bench args" ...
# Every run has its own time limit; the first failure ends the session.
O=$1; shift; mkdir -p $O
for spec in "$@"; do
  IFS='|' read -r name envs args <<< "$spec"
  env $envs timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $args > $O/$name.jsonl 2> $O/$name.err
  rc=$?
  if [ $rc -ne 0 ]; then tail -3 $O/$name.err; exit $rc; fi
  python3 -c "
import json
d=json.loads(open('$O/$name.jsonl').read().strip().splitlines()[-1])
f=d.get('tlc_workers_1',{}).get('ms_per_step')
print('$name', round(d['ms_per_step'],2), {k:round(v['ms'],2) for k,v in d['kernels'].items()}, round(d['config']['kernel_ms_per_run'],2), f and round(f,2), d.get('dedup_set'))
"
done
