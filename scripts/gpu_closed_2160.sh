# Closed LDP segments at the headline's resolution and reference count (bench.ClosedWorkload): 120
# segments of 3840x2160 I + P1..P4 (HM's encoder_lowdelay_P_main structure: POC 4 searches 4 device-made
# references), two CTU rows per slice (17 equal chains of 120 CTUs per picture, the partial bottom row
# inside the last slice; 2040 chains), 24 CTUs per chain per launch; every picture deblocked, SAO'd,
# written and turned into references on the device; restatement parity on segment 0's POC 4 (3 chains).
# ~13 minutes on one MI355X.  Output: gpurun_out/closed_2160.json (progress in closed_2160.err).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1080 python -u -c "
import json, bench
from video_codecs_amd import hvx
hvx.context()
w = bench.ClosedWorkload(3840, 2160, [32] * 120, 5, rank=0, kind='ldp', rows=2, ctus_step=24)
par = {'seg0_poc4': bench.ClosedParity(w, 4, 0, [0, 8, 16])}
print(json.dumps(bench.closed_figure(w, 16, par)))" > gpurun_out/closed_2160.json 2> gpurun_out/closed_2160.err; rc=$?
tail -c 3000 gpurun_out/closed_2160.json; tail -3 gpurun_out/closed_2160.err; exit $rc
