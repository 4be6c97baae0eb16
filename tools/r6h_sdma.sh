# the HIP runtime's D2H engine (SDMA vs blit kernels: HSA_ENABLE_SDMA=0) x the stream layouts, bench.py
# on /opt/rocm's runtime (no torch at N = 1)
set -o pipefail
mkdir -p gpurun_out/r6h
B="python -u bench.py --steps 30 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m"
for v in def pool all def_nosdma pool_nosdma all_nosdma; do
  case $v in
    def) E="RS_X=1";; pool) E="RS_POOLED_STREAMS=1";; all) E="RS_CUMASK_STREAMS=1";; def_nosdma) E="HSA_ENABLE_SDMA=0";;
    pool_nosdma) E="RS_POOLED_STREAMS=1 HSA_ENABLE_SDMA=0";; all_nosdma) E="RS_CUMASK_STREAMS=1 HSA_ENABLE_SDMA=0";;
  esac
  env $E timeout -k 10 200 $B > gpurun_out/r6h/$v.json 2> gpurun_out/r6h/$v.err || exit 1
  echo "$v done"
done
