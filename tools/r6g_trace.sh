# kernel + copy traces of the metric bench with pooled streams, torch first (fast) vs not (slow):
# which streams share a hardware queue (Queue_Id per Stream_Id) and the timeline of one call
set -o pipefail
mkdir -p gpurun_out/r6g
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m"
RS_POOLED_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6g/t -o t -- $B > gpurun_out/r6g/t.log 2>&1 || exit 1
RS_POOLED_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6g/n -o n -- $B --no-link > gpurun_out/r6g/n.log 2>&1 || exit 1
