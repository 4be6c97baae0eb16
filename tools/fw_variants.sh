#!/bin/bash
# kernel traces of the metric circuit for library variants (diagnostic): tools/fw_variants.sh tag=lib ...
set -e
export TMPDIR=/tmp
for tv in "$@"; do
  tag=${tv%%=*}; lib=${tv#*=}
  RS_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwv_$tag -o t -- \
    python3 tools/quick_bench.py 10000000 > gpurun_out/fwv_$tag.log 2>&1
  echo "$tag done"
done
