set -o pipefail
mkdir -p gpurun_out/r6e
B="python -u bench.py --steps 6 --warmup 2 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m"
RS_PROF=1 timeout -k 10 200 $B --no-link > gpurun_out/r6e/b.json 2> gpurun_out/r6e/b.err || exit 1
RS_PROF=1 timeout -k 10 200 $B > gpurun_out/r6e/a.json 2> gpurun_out/r6e/a.err || exit 1
