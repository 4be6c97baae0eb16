# result-stream chunking A/B on the metric circuit, host -> host (alternating processes):
# chunk MiB x chunks in flight
set -e
OUT=gpurun_out/r6snap
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-hbm --no-write --steps 20 --warmup 2"
for rep in 1 2; do
  for v in "32 2" "32 8" "64 2" "128 2" "256 1"; do
    set -- $v
    RS_SNAP_CHUNK_MB=$1 RS_SNAP_DEPTH=$2 timeout -k 10 200 $B > $OUT/c$1_d$2_r$rep.json 2> $OUT/c$1_d$2_r$rep.err
  done
done
