# the whole GPU parity file on the tree's libhvx.so, then the A/B bench against variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread -m gpu > gpurun_out/parity_full.log 2>&1; rc=$?; tail -3 gpurun_out/parity_full.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh "$@"
