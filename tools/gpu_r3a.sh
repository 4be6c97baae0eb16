#!/bin/bash
# round-3 checkpoint: changed GPU tests, then kernel traces of the templated and metric circuits
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_flatten.py tests/test_gpu_writer.py tests/test_gpu_configs.py > gpurun_out/r3a/tests.log 2>&1
echo tests done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3a/tmpl -o t -- python3 tools/config_bench.py --reps 3 templated10M > gpurun_out/r3a/tmpl.log 2>&1
echo tmpl done
RS_PROF=1 timeout -k 10 200 python3 tools/config_bench.py --reps 2 mixed10M templated10M > gpurun_out/r3a/prof.log 2>&1
echo prof done
