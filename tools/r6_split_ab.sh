# the tail's split between the main stream (its largest clusters) and the side stream: host -> host A/B
set -e
OUT=gpurun_out/r6split
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-hbm --no-write --no-link --steps 20 --warmup 2"
for rep in 1 2; do
  for v in 1024 512 256 2048; do
    RS_TAIL_SPLIT=$v timeout -k 10 200 $B > $OUT/s${v}_r$rep.json 2> $OUT/s${v}_r$rep.err
  done
done
