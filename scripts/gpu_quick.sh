# quick GPU iteration: the named parity tests, then one short bench run (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
K=${1:-"decide or coeff_bits or ctu_pass"}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "$K" > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -15 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/quick_bench.log 2>&1
rc=$?; tail -2 gpurun_out/quick_bench.log | cut -c1-3000; exit $rc
