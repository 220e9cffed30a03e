#!/bin/bash
# kernel stats of c5v2 to depth 13 (count_final_level) under rocprofv3
set -o pipefail
O=$GRAFT_REPO_ROOT/${OUT:-gpurun_out/r4c5prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export C5_CFG=c5v2.cfg C5_WORKERS=0 C5_COUNT_FINAL=1 C5_TABLE_GB=64 C5_STORE_GB=120
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/c5_probe.py 13 > $O/probe.jsonl 2> $O/probe.err
rc=$?; echo rc=$rc; cut -c1-600 $O/probe.jsonl; exit $rc
