set -o pipefail
mkdir -p gpurun_out/r3x
for n in base dbl_recv dbl_dd dbl_low; do
  RAFTMC_LIB=scripts/_build/var/$n/libraftmc.so timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --fifo-steps 0 --no-extra > gpurun_out/r3x/$n.jsonl 2> gpurun_out/r3x/$n.err || exit $?
done
