#!/bin/bash
# full GPU suite; C3 (TLC's SYMMETRY mode) with the fingerprint's parts duplicated one at a time;
# the sharded loop at world 1; the bench
O=${OUT:-gpurun_out/r4i}; mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_base.jsonl 2>&1 || exit 1
for v in dupmin dupview dupapply; do
  RAFTMC_LIB=raft-tla_amd/_build_var/$v/libraftmc.so timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_$v.jsonl 2>&1 || exit 1
done
for f in base dupmin dupview dupapply; do python3 -c "
import json; d=json.loads(open('$O/c3_$f.jsonl').read().strip().splitlines()[-1]); print('$f', d['distinct'], d['run_s'], d['kernels_ms'])"; done
timeout -k 10 300 python3 scripts/shard_probe.py > $O/shard_probe.jsonl 2> $O/shard_probe.err || exit 1
cat $O/shard_probe.jsonl
timeout -k 10 600 python -u bench.py > $O/bench.jsonl 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-1500 $O/bench.jsonl
exit $rc
