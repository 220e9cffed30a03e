#!/bin/bash
# rocprofv3 evidence for the raft_original kernels on C2 (bench.py's headline workload): kernel-trace
# stats, then FETCH_SIZE / WRITE_SIZE / two SQ passes in runs of their own, each summarised into the
# small files kept under profiles/ (the SQLite databases are deleted: gpurun copies back at most 64 MiB).
#   scripts/c2_prof.sh OUTDIR TAG
set -o pipefail
O=$GRAFT_REPO_ROOT/${1:-gpurun_out/c2_prof}; TAG=${2:-r05}
mkdir -p $O
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extra --fifo-steps 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra --fifo-steps 0 > $O/stats.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 $B > $O/write.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES -d $O/sq -o run -- python3 $B > $O/sq.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA -d $O/sq2 -o run -- python3 $B > $O/sq2.log 2>&1
rc=$?
echo "rc=$rc"
[ $rc -ne 0 ] && exit $rc
db() { find $1 -name "*.db" | head -1; }
cd $R
python3 scripts/rocpd_summary.py stats $(db $O/stats) $O/${TAG}_c2_kernel_stats.csv &&
python3 scripts/rocpd_summary.py traffic $(db $O/fetch) $(db $O/write) orig_generate $O/traffic_${TAG}_c2_generate.json c2.cfg &&
python3 scripts/rocpd_summary.py traffic $(db $O/fetch) $(db $O/write) orig_dedup_plain $O/traffic_${TAG}_c2_dedup.json c2.cfg --random &&
python3 scripts/rocpd_summary.py valu $(db $O/sq) orig_generate $O/valu_${TAG}_c2_generate.json c2.cfg &&
python3 scripts/pmc_table.py $(db $O/sq) $(db $O/sq2) > $O/${TAG}_c2_sq_table.txt
rc=$?
rm -rf $O/stats $O/fetch $O/write $O/sq $O/sq2
exit $rc
