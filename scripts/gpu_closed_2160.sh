# closed LDP segments at the headline's resolution (bench.closed_loop_measure): 120 segments of
# 3840x2160 I + P + P, two CTU rows per slice (17 equal chains of 120 CTUs per picture, the partial
# bottom row inside the last slice), 8 CTUs per chain per launch; restatement parity on one P picture
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -c "
import json, bench
from video_codecs_amd import hvx
hvx.context()
print(json.dumps(bench.closed_loop_measure(3840, 2160, segs=120, pics=3, ctus_step=8, rows=2)))" > gpurun_out/closed_2160.json 2> gpurun_out/closed_2160.err; rc=$?; tail -c 2500 gpurun_out/closed_2160.json; tail -3 gpurun_out/closed_2160.err; exit $rc
