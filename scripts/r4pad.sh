#!/bin/bash
# generated path on C2: lane arena stride padding (RAFTMC_TLAGEN_PAD words; 0 = power-of-two stride)
O=${OUT:-gpurun_out/r4pad}; mkdir -p $O
for p in ${PADS:-0 32 96}; do
  RAFTMC_TLAGEN_PAD=$p timeout -k 10 240 python -u scripts/tlagen_c2_time.py 8 > $O/pad_$p.jsonl 2>&1 || { echo "pad $p failed"; tail -5 $O/pad_$p.jsonl; exit 1; }
  echo "pad $p: $(cut -c1-420 $O/pad_$p.jsonl)"
done
