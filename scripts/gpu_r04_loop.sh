# the device reference loop tests (hvx_hm_finish_picture), then the variant parity + A/B (gpu_r04_ab2.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "finish_picture" > gpurun_out/loop_tests.log 2>&1; rc=$?; tail -6 gpurun_out/loop_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_ab2.sh "$@"
