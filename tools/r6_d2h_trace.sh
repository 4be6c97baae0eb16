# kernel + memory-copy trace of host -> host steps of the metric bench (the result stream's gaps:
# python3 tools/d2h_gaps.py gpurun_out/r6d2h/tr/b --step 2)
set -e
OUT=gpurun_out/r6d2h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr -o b -- python3 bench.py --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link --no-hbm --no-write --steps 4 --warmup 1 > $OUT/b.log 2>&1
