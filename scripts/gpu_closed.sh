# the closed-loop LDP segment side figure (bench.closed_loop_measure): a small case with parity first,
# then the full 120-segment 1920x1088 figure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -c "
import json, bench
from video_codecs_amd import hvx
hvx.context()
print(json.dumps(bench.closed_loop_measure(256, 192, 2, 3, 32, 2, 4)))" > gpurun_out/closed_small.json 2> gpurun_out/closed_small.err; rc=$?; tail -c 1500 gpurun_out/closed_small.json; tail -3 gpurun_out/closed_small.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -c "
import json, bench
from video_codecs_amd import hvx
hvx.context()
print(json.dumps(bench.closed_loop_measure()))" > gpurun_out/closed_full.json 2> gpurun_out/closed_full.err; rc=$?; tail -c 3000 gpurun_out/closed_full.json; tail -3 gpurun_out/closed_full.err; exit $rc
