# HM engine parity on every capture (modes 0/1, resume, multislice, SSIM, closed loop) with the tree's
# libhvx.so, then the A/B bench against variants.  Stops at the first fatal step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread -m gpu \
  -k "hm_ or sao_decide" > gpurun_out/parity_hm.log 2>&1; rc=$?; tail -3 gpurun_out/parity_hm.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh "$@"
