set -e
for h in 0 4 16 64 256; do
  env TAG=head$h RS_HEAD=$h timeout -k 10 120 python tools/knob_bench.py
done
