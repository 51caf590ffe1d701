# the variant's HM engine parity (every CTU capture) and the A/B bench against the tree's libhvx.so
# usage: bash scripts/gpu_r04_pred.sh video_codecs_amd/_variants/libhvx_X.so
set -o pipefail
mkdir -p gpurun_out
HVX_LIB_PATH=$(pwd)/$1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread -m gpu \
  -k "hm_ctu_golden or ssim_rdo or closed_loop" > gpurun_out/parity_var.log 2>&1; rc=$?; tail -3 gpurun_out/parity_var.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh "$@"
