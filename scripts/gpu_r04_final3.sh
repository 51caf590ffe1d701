# round-end evidence on the final engine: the default bench line, then the rocprof kernel stats +
# FETCH/WRITE + SQ passes (r04c); outputs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd); T=r04c
B="--no-cpu --no-cpu-ref --no-ra --no-slice0 --no-1080p"
timeout -k 10 1000 python -u bench.py > gpurun_out/final_bench.log 2> gpurun_out/final_bench.err || exit $?
grep '^{' gpurun_out/final_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > gpurun_out/prof_${T}_kt.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${T}_fetch -o f --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > gpurun_out/prof_${T}_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${T}_write -o w --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > gpurun_out/prof_${T}_write.log 2>&1 &&
bash scripts/gpu_hm_pmc.sh
rc=$?
grep '^{' gpurun_out/prof_${T}_kt.log | cut -c1-200
exit $rc
