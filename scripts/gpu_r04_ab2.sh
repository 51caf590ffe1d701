# parity of the tree's libhvx.so and one variant on two captures (P + B), then the A/B bench
# usage: bash scripts/gpu_r04_ab2.sh VARIANT.so [MORE.so ...]
set -o pipefail
mkdir -p gpurun_out
K="hm_ctu_golden and (ldp_rand or ra_q22)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "$K" > gpurun_out/par_tree.log 2>&1; rc=$?; tail -2 gpurun_out/par_tree.log; [ $rc -eq 0 ] || exit $rc
HVX_LIB_PATH=$(pwd)/$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "$K" > gpurun_out/par_var.log 2>&1; rc=$?; tail -2 gpurun_out/par_var.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh "$@"
