#!/bin/bash
# Profiles the bench workloads on the GPU box (from the repo root):
#   1. kernel trace + stats of `bench.py --steps 5 --warmup 2 --no-cpu` (the metric circuit)
#   2. kernel trace + stats of the template-replicated circuit (tools/config_bench.py templated10M)
#   3. FETCH_SIZE pass, 4. WRITE_SIZE pass (separate runs: the two do not fit one pass)
#   5. write-request sizes (TCC_EA0_WRREQ / _64B) of the same kernels
# The PMC passes run `bench.py --steps 1 --warmup 0`: one timed step plus the HBM-resident leg's one
# run, so a kernel's dispatch count there is twice its launches per step (pmc_traffic.py --steps 2).  Outputs land in gpurun_out/<tag>/; tools/pmc_traffic.py turns 3-5 into
# profiles/<tag>_pmc_traffic.json on the CPU side.
# usage: bash tools/profile_round.sh <tag>
set -e
TAG=${1:-round3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu --no-flatten --no-templated > $OUT/trace_bench.log 2>&1
echo "trace done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_t -o tmpl -- \
  python3 tools/config_bench.py --reps 3 templated10M > $OUT/trace_tmpl.log 2>&1
echo "templated trace done"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o f -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --no-flatten --no-templated > $OUT/pmc_fetch.log 2>&1
echo "fetch done"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o w -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --no-flatten --no-templated > $OUT/pmc_write.log 2>&1
echo "write done"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_wrreq -o q -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --no-flatten --no-templated > $OUT/pmc_wrreq.log 2>&1
echo "wrreq done"
