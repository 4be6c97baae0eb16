# the speculative loop's DPP reductions: parity, then the head loop's time A/B against the previous build
set -o pipefail
mkdir -p gpurun_out/r6t
timeout -k 10 500 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hosthost.py tests/test_gpu_giant.py > gpurun_out/r6t/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/config_bench.py --check --reps 2 mixed10M templated10M > gpurun_out/r6t/check.log 2>&1 || exit 1
A="--steps 30 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link"
for i in 1 2; do
  RS_LIB=circom_cvm_amd/librs_simplify_base.so timeout -k 10 200 python -u bench.py $A > gpurun_out/r6t/base_$i.json 2> gpurun_out/r6t/base_$i.err || exit 1
  timeout -k 10 200 python -u bench.py $A > gpurun_out/r6t/dpp_$i.json 2> gpurun_out/r6t/dpp_$i.err || exit 1
done
