#!/bin/bash
# Diagnostic variant of librs_simplify with per-phase clocks inside k_big_main's loop (RS_KCLOCKS):
#   bash tools/kclk_build.sh && RS_LIB=$PWD/circom_cvm_amd/librs_simplify_kclk.so RS_PROF=1 python3 tools/quick_bench.py
# The clocks split the loop's schedule, so absolute times are inflated; the path counts are exact.
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared --gpu-max-threads-per-block=256 -DRS_KCLOCKS \
  -o circom_cvm_amd/librs_simplify_kclk.so circom_cvm_amd/csrc/engine.hip circom_cvm_amd/csrc/r1cs_io.cpp \
  circom_cvm_amd/csrc/synth.cpp circom_cvm_amd/csrc/host_common.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
