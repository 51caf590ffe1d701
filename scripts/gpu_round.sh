# full GPU check of the tree: parity suite (without the HM seam encodes), smoke, bench (with CPU
# baseline), rocprof kernel stats + separate FETCH_SIZE / WRITE_SIZE PMC passes of the bench
# command, then the HM seam encodes (encoder progress under gpurun_out/seam/)
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/seam
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=10 --deselect tests/test_hm_seam.py::test_hm_encoder_with_hvx_seams > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-400 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o f --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu > gpurun_out/prof_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o w --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu > gpurun_out/prof_write.log 2>&1
rc=$?
find gpurun_out/prof_* -name "*.csv" | head -20
[ $rc -eq 0 ] || exit $rc
[ "${1:-}" = "noseam" ] && exit 0
HVX_SEAM_LOG_DIR=$R/gpurun_out/seam timeout -k 10 700 python -u -m pytest tests/test_hm_seam.py -m gpu -x -v --timeout-method thread --durations=0 > gpurun_out/seam_tests.log 2>&1
rc=$?; tail -12 gpurun_out/seam_tests.log; exit $rc
