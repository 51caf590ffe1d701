# Profiles of the headline (k_hm_compress): rocprofv3 kernel-trace stats, FETCH_SIZE and
# WRITE_SIZE passes (HBM traffic), the SQ passes (scripts/gpu_hm_pmc.sh); outputs under gpurun_out/
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); T=${T:-r06}
B="--no-cpu --no-cpu-ref --no-ra --no-1080p --no-closed"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $B > gpurun_out/prof_${T}_kt.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${T}_fetch -o f --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > gpurun_out/prof_${T}_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${T}_write -o w --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > gpurun_out/prof_${T}_write.log 2>&1 &&
bash scripts/gpu_hm_pmc.sh
rc=$?
grep '^{' gpurun_out/prof_${T}_kt.log | cut -c1-300
exit $rc
