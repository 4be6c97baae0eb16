set -e
for cfg in "base::::" "m90:92000:::" "f100::100000::" "m90f100:92000:100000::" "gm256::::256:" "gm512::::512:" "gf256:::::256"; do
  IFS=: read tag xm xf gm gf <<< "$cfg"
  env TAG=$tag ${xm:+RS_XM=$xm} ${xf:+RS_XF=$xf} ${gm:+RS_GM=$gm} ${gf:+RS_GF=$gf} timeout -k 10 120 python tools/knob_bench.py
done
