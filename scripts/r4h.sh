#!/bin/bash
# full GPU suite; C3 in TLC's SYMMETRY mode with the fingerprint's parts duplicated one at a time
# (scripts/build_variant_memb.sh: the time a duplicated part adds is that part's cost)
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_base.jsonl 2>&1 || exit 1
for v in dupmin dupview dupapply; do
  RAFTMC_LIB=raft-tla_amd/_build_var/$v/libraftmc.so timeout -k 10 200 python -u scripts/memb_probe.py memb_four > $O/c3_$v.jsonl 2>&1 || exit 1
done
for f in base dupmin dupview dupapply; do python3 -c "
import json; d=json.loads(open('$O/c3_$f.jsonl').read().strip().splitlines()[-1]); print('$f', d['distinct'], d['run_s'], d['kernels_ms'])"; done
