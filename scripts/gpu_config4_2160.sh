# BASELINE config 4 at its own resolution: 120 closed RA segments of 3840x2160 random 4:2:0 (30 per base
# QP 22 / 27 / 32 / 37), I then POC 8 and 4 of the first GOP8, decided with the stvssim encoder's
# distortionstVSSIM over each segment's device history; two CTU rows per slice (17 chains per picture,
# 2040 chains), 24 CTUs per chain per launch; a restatement parity sample per QP (3 chains of its
# first segment's POC 4).  ~10 minutes on one MI355X.  Output: gpurun_out/config4_2160.json.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1080 python -u -c "
import json, bench
from video_codecs_amd import hvx
hvx.context()
print(json.dumps(bench.config4_measure(16, W=3840, H=2160, rows=2, ctus_step=24)))" > gpurun_out/config4_2160.json 2> gpurun_out/config4_2160.err; rc=$?
tail -c 3000 gpurun_out/config4_2160.json; tail -3 gpurun_out/config4_2160.err; exit $rc
