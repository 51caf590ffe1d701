# kernel-trace statistics of every kernel the default bench run launches (headline, slice writer,
# config 4 with the stVSSIM history sums, SliceMode 0, 1080p, the closed-loop segments with their
# deblocking / SAO / reference builds)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_all -o all --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-ref > gpurun_out/prof_all.log 2>&1
rc=$?
cut -d, -f1-4 gpurun_out/prof_all/all_kernel_stats.csv | head -30
exit $rc
