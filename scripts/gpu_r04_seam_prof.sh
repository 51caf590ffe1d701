# the batched compressCtu seam (1080p + RA), the RA smooth per-CTU seam, then the HM_PROFILE profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_hm_seam.py -x -v --timeout 900 --timeout-method thread -m gpu \
  -k "cu_seam_batched or (cu_seam and ra_smooth)" > gpurun_out/seam_batched.log 2>&1; rc=$?; tail -6 gpurun_out/seam_batched.log
HVX_LIB_PATH=$(pwd)/video_codecs_amd/_variants/libhvx_prof.so timeout -k 10 300 python -u -m tests.hm_profile bench 62 1 > gpurun_out/hprof.log 2>&1; rc2=$?; tail -34 gpurun_out/hprof.log
[ $rc -eq 0 ] && [ $rc2 -eq 0 ]
