# alternating A/B/C of the stream layouts, 4 processes each (bench.py, no torch, /opt/rocm runtime)
set -o pipefail
mkdir -p gpurun_out/r6i
B="python -u bench.py --steps 30 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link"
for i in 1 2 3 4; do
  for v in def all pool; do
    case $v in def) E="RS_X=1";; pool) E="RS_POOLED_STREAMS=1";; all) E="RS_CUMASK_STREAMS=1";; esac
    env $E timeout -k 10 200 $B > gpurun_out/r6i/${v}_$i.json 2> gpurun_out/r6i/${v}_$i.err || exit 1
  done
  echo "round $i done"
done
