# the input's H2D over 1 / 2 / 4 copy streams (RS_UP_STREAMS): host -> host A/B, plus the host -> host tests
set -o pipefail
mkdir -p gpurun_out/r6o
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_hosthost.py > gpurun_out/r6o/tests.log 2>&1 || exit 1
timeout -k 10 60 tools/micro/linkpar > gpurun_out/r6o/linkpar.txt 2>&1 || exit 1
A="--steps 30 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m"
for i in 1 2; do
  for u in 1 2 4; do
    RS_UP_STREAMS=$u timeout -k 10 200 python -u bench.py $A > gpurun_out/r6o/u${u}_$i.json 2> gpurun_out/r6o/u${u}_$i.err || exit 1
  done
  echo "round $i"
done
