#!/bin/bash
# Round-end evidence on one box: the GPU parity suite, the default bench line (with the CPU
# baseline), then scripts/prof_session.sh (rocprofv3 kernel stats + FETCH/WRITE/SQ passes).
#   bash scripts/final_session.sh OUT TAG
set -o pipefail
O=${1:-gpurun_out/final}; TAG=${2:-r02}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu.py tests/test_gpu_shard.py tests/test_gpu_membership.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.jsonl
bash scripts/prof_session.sh $O/prof $TAG
