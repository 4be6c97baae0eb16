# kernel + memory-copy trace of the templated circuit host -> host (tools/step_timeline.py / d2h_gaps.py)
set -e
OUT=gpurun_out/r6tt
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tr -o t -- python3 tools/config_bench.py --reps 3 templated10M > $OUT/t.log 2>&1
RS_PROF=1 timeout -k 10 200 python3 tools/config_bench.py --reps 2 templated10M > $OUT/prof.out 2> $OUT/prof.err
