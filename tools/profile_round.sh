#!/bin/bash
# Profiles the bench workload on the GPU box: kernel trace + stats, the two PMC passes for the
# dominant kernel's HBM traffic, then the contract bench line with that traffic filled in.
# usage (on the box, from the repo root): bash tools/profile_round.sh <tag> <kernel>
set -e
TAG=${1:-round1}
KER=${2:-k_big_main}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/trace_bench.log 2>&1
echo "trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o f -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/pmc_fetch.log 2>&1
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o w -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/pmc_write.log 2>&1
echo "write done"
TRAFFIC=$(python3 tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $KER 2> $OUT/pmc_traffic.txt)
echo "traffic per launch: $TRAFFIC"
if [ "$TRAFFIC" != "null" ]; then export RS_PMC_TRAFFIC_BYTES=$TRAFFIC; fi
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
