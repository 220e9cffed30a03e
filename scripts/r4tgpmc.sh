#!/bin/bash
# PMC passes over the generated path on C2 (where the ~10 ns per generated successor goes)
set -o pipefail
O=$GRAFT_REPO_ROOT/${OUT:-gpurun_out/r4tgpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/tlagen_c2_time.py 8"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES -d $O/sq -o run -- $B > $O/sq.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM -d $O/sq2 -o run -- $B > $O/sq2.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $O/ta -o run -- $B > $O/ta.log 2>&1
rc=$?; echo rc=$rc; tail -3 $O/*.log; exit $rc
