# parity (HM engine + CABAC kernels) on the tree's libhvx.so, the A/B bench, the HM_PROFILE profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread -m gpu \
  -k "hm_ctu_golden or cabac or coeff or ssim_rdo or sao_decide" > gpurun_out/parity_esc.log 2>&1; rc=$?; tail -3 gpurun_out/parity_esc.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh "$@" || exit $?
HVX_LIB_PATH=$(pwd)/video_codecs_amd/_variants/libhvx_prof.so timeout -k 10 300 python -u -m tests.hm_profile bench 62 1 > gpurun_out/hprof.log 2>&1 || exit $?
tail -34 gpurun_out/hprof.log
