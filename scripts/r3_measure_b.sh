#!/bin/bash
# Round-3 measurement, part 2: rocprofv3 evidence for C2 (bench) and C3 (memb_four).
set -u
OUT=${1:-gpurun_out/r3m}
mkdir -p $OUT
bash scripts/r3_session.sh $OUT "step prof 500 bash scripts/prof_session.sh $OUT/prof r03" "step membprof 500 bash scripts/memb_prof.sh $OUT/memb_prof r03"
