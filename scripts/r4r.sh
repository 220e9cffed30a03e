#!/bin/bash
# C2 bench at three seen-set sizes (the library default is 8 GiB)
O=gpurun_out/r4r; mkdir -p $O
for tb in 2147483648 4294967296 0; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --fp-table-bytes $tb > $O/t$tb.jsonl 2> $O/t$tb.err || exit 1
  python3 -c "
import json; d=json.loads(open('$O/t$tb.jsonl').read().strip().splitlines()[-1]); print($tb, round(d['ms_per_step'],2), {k:round(v['ms'],2) for k,v in d['kernels'].items()}, d.get('dedup_set',{}).get('probes_per_s'))"
done
