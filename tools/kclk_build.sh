#!/bin/bash
# Diagnostic variants of librs_simplify with shader clocks inside a kernel:
#   bash tools/kclk_build.sh            -> librs_simplify_kclk.so  (RS_KCLOCKS: phases of k_big_main's loop)
#   bash tools/kclk_build.sh RS_FWCLK fwclk -> librs_simplify_fwclk.so (stages of k_frames_wave, both passes)
# then: RS_LIB=$PWD/circom_cvm_amd/librs_simplify_<suffix>.so RS_PROF=1 python3 tools/config_bench.py ...
# The clocks split the kernels' schedules, so absolute times are inflated; the counts are exact.
set -e
cd "$(dirname "$0")/.."
DEF=${1:-RS_KCLOCKS}
SUF=${2:-kclk}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared --gpu-max-threads-per-block=256 -D$DEF \
  -o circom_cvm_amd/librs_simplify_$SUF.so circom_cvm_amd/csrc/engine.hip circom_cvm_amd/csrc/r1cs_io.cpp \
  circom_cvm_amd/csrc/synth.cpp circom_cvm_amd/csrc/host_common.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
