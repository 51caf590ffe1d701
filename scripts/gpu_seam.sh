# the HM drop-in encodes alone (every seam of integration/, counters + MD5 vs the stock encoder)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/seam
HVX_SEAM_LOG_DIR=$R/gpurun_out/seam timeout -k 10 800 python -u -m pytest tests/test_hm_seam.py -m gpu -x -v --timeout-method thread --durations=0 > gpurun_out/seam_tests.log 2>&1
rc=$?; tail -12 gpurun_out/seam_tests.log; exit $rc
