# The HM seam encodes (unchanged TAppEncoder with libhvx seams) incl. the compressCtu seam
set -o pipefail
mkdir -p gpurun_out/seam_logs
export HVX_SEAM_LOG_DIR=$(pwd)/gpurun_out/seam_logs
timeout -k 10 1100 python -u -m pytest tests/test_hm_seam.py -v --timeout 900 --timeout-method thread -m gpu ${K:+-k "$K"} > gpurun_out/seam.log 2>&1; rc=$?; tail -12 gpurun_out/seam.log; exit $rc
