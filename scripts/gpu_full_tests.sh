# the round-end GPU test suite (pytest -m gpu), as the driver runs it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/ -x -v --timeout 900 --timeout-method thread -m gpu > gpurun_out/full_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/full_tests.log | tail -60 | cut -c1-160
exit $rc
