#!/bin/bash
# speculative head loop: smoke, elimination parity tests, then the metric / templated timings
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_full.py > gpurun_out/r3b/tests.log 2>&1
echo tests done
RS_PROF=1 timeout -k 10 200 python3 tools/config_bench.py --reps 2 mixed10M templated10M > gpurun_out/r3b/prof.log 2>&1
echo prof done
RS_SPEC_NW=4 timeout -k 10 200 python3 tools/config_bench.py --reps 3 mixed10M templated10M > gpurun_out/r3b/nw4.log 2>&1
timeout -k 10 200 python3 tools/config_bench.py --reps 3 mixed10M templated10M > gpurun_out/r3b/nw8.log 2>&1
echo nw done
