#!/bin/bash
# generated-path GPU tests, the NewlyJoinedBecomeLeader counterexample dump, dedup A/B
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tlagen.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python -u scripts/dump_trace.py configs/raft_membership_mc.tla configs/scen_NewlyJoinedBecomeLeader.cfg $O/njbl > $O/njbl.log 2>&1
rc=$?; echo "njbl rc=$rc"; cat $O/njbl.log
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_env.sh $O "base||--no-extra" "dprobe|RAFTMC_LIB=raft-tla_amd/_build_var/dprobe/libraftmc.so|--no-extra" "r03|RAFTMC_LIB=raft-tla_amd/_build_var/r03/libraftmc.so|--no-extra" "queue|RAFTMC_DEDUP_QUEUE=1|--no-extra" "base2||--no-extra"
