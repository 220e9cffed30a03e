#!/bin/bash
# rocprofv3 evidence for the tlc_membership kernels on C3 (memb_four: 4 servers, NextDynamic,
# SYMMETRY in TLC's mode): kernel-trace stats, then FETCH_SIZE / WRITE_SIZE / SQ passes in runs of
# their own.   scripts/memb_prof.sh OUTDIR TAG
set -o pipefail
O=$GRAFT_REPO_ROOT/${1:-gpurun_out/memb_prof}; TAG=${2:-r03}
mkdir -p $O
R=$GRAFT_REPO_ROOT
P="$R/scripts/memb_probe.py memb_four"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 $P > $O/stats.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 $P > $O/fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 $P > $O/write.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES -d $O/sq -o run -- python3 $P > $O/sq.log 2>&1
rc=$?
echo "rc=$rc"
[ $rc -ne 0 ] && exit $rc
db() { find $1 -name "*.db" | head -1; }
cd $R
python3 scripts/rocpd_summary.py stats $(db $O/stats) $O/${TAG}_c3_memb_kernel_stats.csv &&
python3 scripts/rocpd_summary.py traffic $(db $O/fetch) $(db $O/write) memb_fingerprint $O/traffic_${TAG}_c3_fingerprint.json memb_four.cfg &&
python3 scripts/rocpd_summary.py traffic $(db $O/fetch) $(db $O/write) memb_dedup $O/traffic_${TAG}_c3_dedup.json memb_four.cfg --random &&
python3 scripts/rocpd_summary.py valu $(db $O/sq) memb_fingerprint $O/valu_${TAG}_c3_fingerprint.json memb_four.cfg &&
python3 scripts/rocpd_summary.py valu $(db $O/sq) memb_expand $O/valu_${TAG}_c3_expand.json memb_four.cfg &&
python3 scripts/pmc_table.py $(db $O/sq) > $O/${TAG}_c3_sq_table.txt
rc=$?
rm -rf $O/stats $O/fetch $O/write $O/sq   # (gpurun copies back at most 64 MiB)
exit $rc
