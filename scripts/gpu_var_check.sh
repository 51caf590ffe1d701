# HM-engine variant: parity on two captures (P + B, both modes), then the A/B bench against the tree's build
# usage: bash scripts/gpu_var_check.sh video_codecs_amd/_variants/libhvx_NAME.so
set -o pipefail
mkdir -p gpurun_out
V=$(pwd)/$1; n=$(basename "$1" .so)
HVX_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "hm_ctu_golden and (ldp_rand or ra_q22)" > gpurun_out/var_$n.log 2>&1; rc=$?; tail -2 gpurun_out/var_$n.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh "$@"
