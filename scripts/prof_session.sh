#!/bin/bash
# rocprofv3 evidence for profiles/ (run on the GPU box): kernel-trace stats of the bench, then PMC
# passes in runs of their own (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE separately; one SQ
# group), summarised by scripts/rocpd_summary.py.   scripts/prof_session.sh OUTDIR TAG
set -o pipefail
O=$GRAFT_REPO_ROOT/${1:-gpurun_out/prof}; TAG=${2:-r03}
mkdir -p $O
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --fifo-steps 0 --no-extra"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --fifo-steps 0 --no-extra > $O/stats.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 $B > $O/write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1
rc=$?
echo "rc=$rc"
[ $rc -ne 0 ] && exit $rc
db() { find $1 -name "*.db" | head -1; }
cd $R
python3 scripts/rocpd_summary.py stats $(db $O/stats) $O/${TAG}_c2_kernel_stats.csv &&
python3 scripts/rocpd_summary.py traffic $(db $O/fetch) $(db $O/write) orig_generate $O/traffic_${TAG}.json &&
python3 scripts/rocpd_summary.py traffic $(db $O/fetch) $(db $O/write) orig_dedup_plain $O/traffic_${TAG}_dedup.json &&
python3 scripts/rocpd_summary.py valu $(db $O/sq) orig_generate $O/valu_${TAG}.json &&
python3 scripts/pmc_table.py $(db $O/sq) > $O/${TAG}_sq_table.txt
