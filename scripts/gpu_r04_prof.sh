# round 4: parity of the tree's build (HM captures, refusals, SSIM cost), then the profiles of the headline
# (rocprofv3 kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes, SQ passes) under gpurun_out/
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); T=${TAG:-r04}
B="--no-cpu --no-cpu-ref --no-ra --no-slice0"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread -m gpu -k "hm_" \
  > gpurun_out/${T}_parity.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > gpurun_out/prof_${T}_kt.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${T}_fetch -o f --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > gpurun_out/prof_${T}_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${T}_write -o w --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > gpurun_out/prof_${T}_write.log 2>&1 &&
bash scripts/gpu_hm_pmc.sh
rc=$?
grep '^{' gpurun_out/prof_${T}_kt.log | cut -c1-300
exit $rc
