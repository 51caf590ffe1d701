# rocprofv3 kernel-trace summary + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the bench command.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_kt.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o f --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu > gpurun_out/prof_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o w --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu > gpurun_out/prof_write.log 2>&1
rc=$?
find gpurun_out/prof_* -name "*.csv" | head -20
exit $rc
