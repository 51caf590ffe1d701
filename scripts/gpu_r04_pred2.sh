# the whole GPU parity file on the tree's libhvx.so, then the A/B bench of RDOQ round-count variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread -m gpu \
  > gpurun_out/parity_pred.log 2>&1; rc=$?; tail -3 gpurun_out/parity_pred.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh "$@"
