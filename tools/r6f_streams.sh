# A/B of the engine's stream -> hardware-queue layouts (bench.py, metric circuit), each with and without
# torch initialising HIP first (the link probe): default = the copy stream on a dedicated queue
set -o pipefail
mkdir -p gpurun_out/r6f
B="python -u bench.py --steps 40 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m"
for v in def_t def_n pool_t pool_n all_t all_n; do
  case $v in
    def_*) E="RS_X=1";; pool_*) E="RS_POOLED_STREAMS=1";; all_*) E="RS_CUMASK_STREAMS=1";;
  esac
  case $v in *_n) X="--no-link";; *) X="";; esac
  env $E timeout -k 10 200 $B $X > gpurun_out/r6f/$v.json 2> gpurun_out/r6f/$v.err || exit 1
  echo "$v done"
done
