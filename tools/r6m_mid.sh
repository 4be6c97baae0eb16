# the tail's largest clusters on the speculative loop (RS_MID_SPEC = how many): parity, then host -> host
set -o pipefail
mkdir -p gpurun_out/r6m
RS_MID_SPEC=128 timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_hosthost.py tests/test_gpu_parity.py > gpurun_out/r6m/tests.log 2>&1 || exit 1
RS_MID_SPEC=128 timeout -k 10 300 python -u tools/config_bench.py --check --reps 2 mixed10M templated10M > gpurun_out/r6m/check.log 2>&1 || exit 1
A="--steps 30 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link"
for i in 1 2; do
  for m in 0 64 128 256; do
    RS_MID_SPEC=$m timeout -k 10 200 python -u bench.py $A > gpurun_out/r6m/m${m}_$i.json 2> gpurun_out/r6m/m${m}_$i.err || exit 1
  done
  echo "round $i"
done
