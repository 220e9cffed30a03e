# A/B of orig_generate's waves-per-SIMD hint (scripts/build_variant.sh builds under scripts/_build/var)
set -o pipefail
mkdir -p gpurun_out/r3w2
for n in base w2 w4; do
  RAFTMC_LIB=scripts/_build/var/$n/libraftmc.so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --fifo-steps 0 --no-extra > gpurun_out/r3w2/$n.jsonl 2> gpurun_out/r3w2/$n.err || exit $?
done
