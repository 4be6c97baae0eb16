# round-2 A/B of the one-word field path against the pre-change library (RS_LIB), goldilocks
# parity, and the per-phase profile of the templated circuit (run from the repo root on the GPU box)
set -o pipefail
mkdir -p gpurun_out/ab gpurun_out/t5
B="python -u bench.py --steps 40 --no-cpu --no-flatten --no-templated"
for i in 1 2; do
  timeout -k 10 150 $B > gpurun_out/ab/w64_$i.log 2>&1 || exit 1
  RS_LIB=circom_cvm_amd/_build/librs_now64.so timeout -k 10 150 $B > gpurun_out/ab/now64_$i.log 2>&1 || exit 1
done
echo ab done
timeout -k 10 400 python -u -m pytest tests -m gpu -k "goldilocks or 257 or 97" -x -v --timeout 300 --timeout-method thread > gpurun_out/w64_tests.log 2>&1 || exit 1
echo tests done
timeout -k 10 200 python -u tools/kind_stats.py 5 10000000 > gpurun_out/t5/stats.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t5/trace -o t5 -- python3 tools/kind_stats.py 5 10000000 > gpurun_out/t5/trace.log 2>&1
