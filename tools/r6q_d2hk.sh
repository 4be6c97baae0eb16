# the result stream copied by a kernel (RS_D2H_KERNEL=1) vs the runtime's copy engine: parity + host -> host A/B
set -o pipefail
mkdir -p gpurun_out/r6q
RS_D2H_KERNEL=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_hosthost.py > gpurun_out/r6q/tests.log 2>&1 || exit 1
A="--steps 30 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m"
for i in 1 2; do
  for v in sdma kern; do
    case $v in sdma) E="RS_X=1";; kern) E="RS_D2H_KERNEL=1";; esac
    env $E timeout -k 10 200 python -u bench.py $A > gpurun_out/r6q/${v}_$i.json 2> gpurun_out/r6q/${v}_$i.err || exit 1
  done
done
RS_D2H_KERNEL=1 RS_PROF=1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m > gpurun_out/r6q/kprof.json 2> gpurun_out/r6q/kprof.err || exit 1
