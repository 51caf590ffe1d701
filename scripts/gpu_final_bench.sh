# Round-end evidence, part 3: the default bench line (headline + cpu_baseline + side figures)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py > gpurun_out/final_bench.log 2> gpurun_out/final_bench.err; rc=$?
grep '^{' gpurun_out/final_bench.log | cut -c1-600; tail -3 gpurun_out/final_bench.err
exit $rc
