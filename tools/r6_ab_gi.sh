set -e
mkdir -p gpurun_out/pf2
L=$PWD/circom_cvm_amd
for v in ${VARIANTS:-base new giclk_base giclk}; do
  case $v in base) lib=$L/librs_simplify_base.so;; new) lib=$L/librs_simplify.so;; *) lib=$L/librs_simplify_$v.so;; esac
  RS_LIB=$lib RS_PROF=1 timeout -k 10 200 python tools/config_bench.py --reps 1 linear1M > gpurun_out/pf2/$v.out 2> gpurun_out/pf2/$v.err
done
