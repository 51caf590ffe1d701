# Round-end evidence, part 1: the whole GPU parity file (kernels + HM engine + loop + SAO) and smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py -v --timeout 600 --timeout-method thread -m gpu \
  > gpurun_out/final_parity.log 2>&1; rc=$?; tail -4 gpurun_out/final_parity.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1; rc=$?; tail -3 gpurun_out/final_smoke.log
exit $rc
