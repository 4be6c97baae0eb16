#!/bin/bash
# speculative head loop checks: parity tests (short per-test limits), then timings
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c/smoke.log 2>&1
echo smoke done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 100 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_full.py > gpurun_out/r3c/tests.log 2>&1
echo tests done
RS_PROF=1 timeout -k 10 200 python3 tools/config_bench.py --reps 2 mixed10M templated10M > gpurun_out/r3c/prof.log 2>&1
echo prof done
timeout -k 10 200 python3 tools/config_bench.py --reps 3 mixed10M templated10M > gpurun_out/r3c/nw8.log 2>&1
echo nw done
