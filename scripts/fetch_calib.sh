#!/bin/bash
# FETCH_SIZE calibration for 8-B random loads: the seen-set
# microbenchmark's probe mode on a 4 GiB table (past the 256 MiB Infinity Cache) issues exactly
# 2^28 random 8-B loads per launch; rocprofv3's FETCH_SIZE per dispatch over that count is the
# bytes the counter charges one such probe.  Each counter pass is a run of its own.
set -o pipefail
O=$GRAFT_REPO_ROOT/${1:-gpurun_out/calib}; mkdir -p $O
B=$GRAFT_REPO_ROOT/scripts/_build/seen_set_bench
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $B calib > $O/plain.jsonl 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- $B calib > $O/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum -d $O/rdreq -o run -- $B calib > $O/rdreq.log 2>&1
rc=$?; cat $O/plain.jsonl; echo rc=$rc; exit $rc
