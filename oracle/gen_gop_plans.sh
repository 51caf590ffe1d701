#!/bin/bash
# TEST INFRASTRUCTURE: tests/golden/gop_plans.json -- HM-16.5rc1's own slice set-up of every picture of a
# closed LDP (17 pictures) and RA (33 pictures) encode at QP 32, recorded by the compressCtu capture
# harness (oracle/cu_capture.cpp) on a 64x64 texture sequence (the structure does not depend on the
# content; the cabac_init choices do).  Needs /root/reference (this container only).
set -euo pipefail
cd "$(dirname "$0")"
make -s -j8 ref
cd ..
ORC=oracle/_ref
CFG=/root/reference/hm-16.5rc1/cfg
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
python3 oracle/make_yuv.py texture 64 64 33 "$TMP/tex.yuv"
for spec in ldp:encoder_lowdelay_P_main.cfg:17 ra:encoder_randomaccess_main.cfg:33; do
  IFS=: read -r kind cfg n <<< "$spec"
  HVX_CAPTURE="$TMP/cu.bin" $ORC/TAppEncoder_cucap -c $CFG/$cfg -i "$TMP/tex.yuv" -wdt 64 -hgt 64 -fr 30 -f $n -q 32 \
    -b "$TMP/str.bin" -o "$TMP/rec.yuv" > "$TMP/log.txt"
  python3 oracle/compact_ctu.py "$TMP/cu.bin" "$TMP/$kind.bin"
done
python3 oracle/gop_plans.py tests/golden/gop_plans.json ldp="$TMP/ldp.bin" ra="$TMP/ra.bin"
