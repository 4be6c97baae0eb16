set -o pipefail
mkdir -p gpurun_out/r6d
B="python -u bench.py --steps 20 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m"
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_hosthost.py > gpurun_out/r6d/tests.log 2>&1 || exit 1
for v in a b c d; do
  case $v in
    a) E=""; X="";; b) E=""; X="--no-link";; c) E="RS_POOLED_STREAMS=1"; X="";; d) E="RS_POOLED_STREAMS=1"; X="--no-link";;
  esac
  env $E timeout -k 10 200 $B $X > gpurun_out/r6d/bench_$v.json 2> gpurun_out/r6d/bench_$v.err || exit 1
  echo "$v done"
done
