# Round profile of the bench step: rocprofv3 kernel-trace stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) for the HBM traffic per launch, then the full default bench run.
# usage: bash scripts/gpu_profile.sh TAG     (outputs under gpurun_out/prof_TAG_*)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); TAG=${1:-r02}
B="--no-cpu --no-intra --no-ssim --no-1080p --no-sao --no-cabac"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 $B > gpurun_out/prof_${TAG}_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${TAG}_fetch -o f --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 $B > gpurun_out/prof_${TAG}_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${TAG}_write -o w --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 $B > gpurun_out/prof_${TAG}_write.log 2>&1 &&
timeout -k 10 600 python3 bench.py > gpurun_out/bench_${TAG}.log 2>&1
rc=$?
grep '^{' gpurun_out/bench_${TAG}.log | cut -c1-400
exit $rc
