# round-3 final: profiles of the headline kernel on this tree, then the default bench line
set -o pipefail
bash scripts/gpu_profile_r03.sh > gpurun_out/final_prof.txt 2>&1 || { tail -5 gpurun_out/final_prof.txt; exit 1; }
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r03_final.log 2> gpurun_out/bench_r03_final.err; rc=$?
grep '^{' gpurun_out/bench_r03_final.log | cut -c1-400
exit $rc
