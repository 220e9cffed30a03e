#!/bin/bash
# the default bench (with its side workloads) and smoke
O=${OUT:-gpurun_out/r4bench}; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/bench.jsonl 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 $O/bench.err; python3 -c "
import json; b=json.loads(open('$O/bench.jsonl').read().splitlines()[-1])
print(b['value'], b['ms_per_step']); v=b.get('variants') or b.get('extra',{}).get('variants'); print(json.dumps(v)[:1500])"
exit $rc
