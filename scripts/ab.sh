# A/B timing of library variants / env knobs on one box (C2 bench, no CPU baseline):
#   bash scripts/ab.sh OUT "name|ENV=1|lib" ...     (empty lib = the in-tree build)
set -o pipefail
O=$1; shift; mkdir -p $O
for spec in "$@"; do
  IFS='|' read -r name envs lib <<< "$spec"
  lib=${lib:-raft-tla_amd/_build/libraftmc.so}
  timeout -k 10 150 env $envs RAFTMC_LIB=$lib python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --fifo-steps 0 > $O/$name.jsonl 2> $O/$name.err || { tail -3 $O/$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$name.jsonl').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],2), {k:round(v['ms'],2) for k,v in d['kernels'].items()}, d['config']['distinct_per_run'])
"
done
