# HM engine: golden CTU parity (HM captures, per-CTU / chained / resumed) + the headline bench step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "hm_ctu" > gpurun_out/q_tests.log 2>&1; rc=$?; tail -2 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh "$@" > gpurun_out/q_ab.txt 2>&1; cat gpurun_out/q_ab.txt
