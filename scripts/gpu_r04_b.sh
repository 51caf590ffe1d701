# round 4: the HM engine with B slices on every CTU capture (LDP + RA), then the RA encode through the CU seam
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "hm_ctu" \
  > gpurun_out/r04_hmctu.log 2>&1; rc=$?; tail -15 gpurun_out/r04_hmctu.log; [ $rc -eq 0 ] || exit $rc
HVX_SEAM_LOG_DIR=gpurun_out timeout -k 10 900 python -u -m pytest tests/test_hm_seam.py -x -v --timeout 850 --timeout-method thread -m gpu \
  -k "cu_seam and ra_texture" > gpurun_out/r04_seam_ra.log 2>&1; rc=$?; tail -6 gpurun_out/r04_seam_ra.log; exit $rc
