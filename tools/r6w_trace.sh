# kernel statistics of the metric bench and the templated circuit at the current tree (the round's profile)
set -e
OUT=gpurun_out/round6t
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- $B --steps 5 --warmup 2 > $OUT/trace_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_t -o tmpl -- python3 tools/config_bench.py --reps 3 templated10M > $OUT/trace_tmpl.log 2>&1
