#!/bin/bash
# Profiles the bench workloads on the GPU box (from the repo root):
#   1. kernel trace + stats of `bench.py --steps 5 --warmup 2 --no-cpu` (the metric circuit)
#   2. kernel trace + stats of the template-replicated circuit (tools/config_bench.py templated10M)
#   3. FETCH_SIZE pass, 4. WRITE_SIZE pass of the metric bench (separate runs: the two do not fit one pass)
#   5. write-request sizes (TCC_EA0_WRREQ / _64B) of the same kernels
#   6. FETCH_SIZE and WRITE_SIZE passes of the templated circuit (config_bench, one call)
#   7. the counters' calibration on known byte counts in this library's access patterns (pmc_calib)
# The metric PMC passes run `bench.py --steps 1 --warmup 0 --no-hbm --no-write`: the one timed host -> host
# step and nothing else, so a kernel's dispatch count there is its launches per step (pmc_traffic.py --steps 1).
# Outputs land in gpurun_out/<tag>/; tools/pmc_calib.py and tools/pmc_traffic.py turn them into
# profiles/<tag>_pmc_calib.json, <tag>_pmc_traffic.json and <tag>_templated_pmc_traffic.json on the CPU side.
# usage: bash tools/profile_round.sh <tag>
set -e
TAG=${1:-round4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  $B --steps 5 --warmup 2 > $OUT/trace_bench.log 2>&1
echo "trace done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_t -o tmpl -- \
  python3 tools/config_bench.py --reps 3 templated10M > $OUT/trace_tmpl.log 2>&1
echo "templated trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o f -- \
  $B --steps 1 --warmup 0 --no-hbm --no-write > $OUT/pmc_fetch.log 2>&1
echo "fetch done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o w -- \
  $B --steps 1 --warmup 0 --no-hbm --no-write > $OUT/pmc_write.log 2>&1
echo "write done"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_wrreq -o q -- \
  $B --steps 1 --warmup 0 --no-hbm --no-write > $OUT/pmc_wrreq.log 2>&1
echo "wrreq done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_tfetch -o f -- \
  python3 tools/config_bench.py --reps 1 templated10M > $OUT/pmc_tfetch.log 2>&1
echo "templated fetch done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_twrite -o w -- \
  python3 tools/config_bench.py --reps 1 templated10M > $OUT/pmc_twrite.log 2>&1
echo "templated write done"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calf -o f -- tools/micro/pmc_calib > $OUT/calib.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/calw -o w -- tools/micro/pmc_calib > $OUT/calib_w.txt 2>&1
echo "calibration done"
