# Round-5 final bench on one box, as the driver runs it (N=1, default side figures incl. the
# closed-loop segments), 20 timed steps after 5 warmup
set -o pipefail
mkdir -p gpurun_out
(time timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r05_final2.out 2> gpurun_out/bench_r05_final2.err) 2> gpurun_out/bench_r05_final2.time || exit 1
head -c 600 gpurun_out/bench_r05_final2.out; echo; cat gpurun_out/bench_r05_final2.time
