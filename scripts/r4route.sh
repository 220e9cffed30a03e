#!/bin/bash
# wave-aggregated route offsets: sharded GPU tests, then the world-1 shard probe
O=${OUT:-gpurun_out/r4route}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 scripts/shard_probe.py > $O/shard_probe.jsonl 2> $O/shard_probe.err || exit 1
grep -v "version\|Hostname\|path" $O/shard_probe.jsonl | cut -c1-300
