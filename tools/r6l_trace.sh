# kernel + copy trace of the metric bench (current code, /opt/rocm runtime) for the timeline, and the
# kernel statistics of `bench.py --steps 5` (the round's profile)
set -o pipefail
mkdir -p gpurun_out/r6l
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6l/tl -o tl -- $B --steps 3 --warmup 1 > gpurun_out/r6l/tl.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6l/st -o st -- $B --steps 5 --warmup 2 > gpurun_out/r6l/st.log 2>&1 || exit 1
