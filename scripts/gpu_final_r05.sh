# Round-5 final evidence on one box: the bench as the driver runs it (N=1, 20 steps, 5 warmup), then
# the GPU suite with durations + smoke (scripts/gpu_full_tests.sh)
set -o pipefail
mkdir -p gpurun_out
(time timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r05_final.out 2> gpurun_out/bench_r05_final.err) 2> gpurun_out/bench_r05_final.time || exit 1
head -c 600 gpurun_out/bench_r05_final.out; echo; cat gpurun_out/bench_r05_final.time
bash scripts/gpu_full_tests.sh
