# the round's bench line (default bench.py) and the single-step PMC passes + writer bench
set -o pipefail
mkdir -p gpurun_out/r6v
timeout -k 10 600 python -u bench.py > gpurun_out/r6v/bench.json 2> gpurun_out/r6v/bench.err || exit 1
bash tools/r6r_pmc.sh
