#!/bin/bash
# k_frames_wave grid sizes on the metric circuit: kernel trace per RS_FW_BLOCKS value (diagnostic)
set -e
export TMPDIR=/tmp
for b in "$@"; do
  RS_FW_BLOCKS=$b timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwk_$b -o t -- \
    python3 tools/quick_bench.py 10000000 > gpurun_out/fwk_$b.log 2>&1
  echo "blocks $b done"
done
