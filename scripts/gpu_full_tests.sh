# the round-end GPU test suite (pytest -m gpu) as the driver runs it, with per-test durations,
# then __graft_entry__.smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -x -v --durations=0 --timeout 600 --timeout-method thread -m gpu > gpurun_out/full_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/full_tests.log | tail -70 | cut -c1-160
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log
exit $rc
