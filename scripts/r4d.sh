#!/bin/bash
# generated-path GPU tests, the membership counterexample fixtures, dedup A/B
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tlagen.py tests/test_gpu_membership.py -k "tlagen or generated or view or recursive or apalache or beyond" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/pytest.log
[ $rc -ge 124 ] && exit $rc
bash scripts/ab_env.sh $O "base||--no-extra" "dprobe|RAFTMC_LIB=raft-tla_amd/_build_var/dprobe/libraftmc.so|--no-extra" "r03|RAFTMC_LIB=raft-tla_amd/_build_var/r03/libraftmc.so|--no-extra" "base2||--no-extra"
