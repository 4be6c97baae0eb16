# lazily fetched map-list batches: the multi-round parity cases, then templated host -> host A/B
set -o pipefail
mkdir -p gpurun_out/r6y
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/r6y/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/config_bench.py --check --reps 2 templated10M > gpurun_out/r6y/check.log 2>&1 || exit 1
for i in 1 2; do
  RS_LIB=circom_cvm_amd/librs_simplify_base.so timeout -k 10 200 python -u tools/config_bench.py --reps 6 templated10M > gpurun_out/r6y/base_$i.json 2> gpurun_out/r6y/base_$i.err || exit 1
  timeout -k 10 200 python -u tools/config_bench.py --reps 6 templated10M > gpurun_out/r6y/lazy_$i.json 2> gpurun_out/r6y/lazy_$i.err || exit 1
done
