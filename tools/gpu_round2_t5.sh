# round 2: the templated circuit's per-phase breakdown (RS_PROF marks), the parity tests of the
# rounds bookkeeping and the elimination routing, and a short bench (run from the repo root on the
# GPU box)
set -o pipefail
mkdir -p gpurun_out/t5
RS_PROF=1 timeout -k 10 200 python -u tools/kind_stats.py 5 10000000 > gpurun_out/t5/prof.log 2>&1 || exit 1
echo prof done
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_log.py tests/test_gpu_sharded.py tests/test_gpu_edge.py tests/test_gpu_configs.py -k "not bls12381 and not every_prime" -x -v --timeout 300 --timeout-method thread > gpurun_out/t5/tests.log 2>&1 || exit 1
echo tests done
timeout -k 10 200 python -u bench.py --steps 40 --no-cpu --no-flatten > gpurun_out/t5/bench.log 2>&1
