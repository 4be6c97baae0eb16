#!/bin/bash
# A/B of kernel times under environment knobs (GPU box, repo root): for each "TAG:ENV=V,ENV=V" argument,
# rocprofv3 --kernel-trace --stats of tools/config_bench.py on CONFIGS (default mixed10M), then
# tools/kstats.py prints the per-step time of the main kernels side by side.
# usage: CONFIGS="mixed10M" REPS=4 bash tools/ab_kernels.sh base: prof:RS_PROF=1
set -e
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
for arg in "$@"; do
  tag=${arg%%:*}
  envs=${arg#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    unset IFS
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o k -- \
      python3 tools/config_bench.py --reps ${REPS:-4} ${CONFIGS:-mixed10M} > $OUT/$tag.log 2>&1 )
  echo "$tag done"
done
python3 tools/kstats.py $OUT "$@"
