# the batched compressCtu seam (1080p + RA) and the RA smooth per-CTU seam; the RDOQ-round A/B;
# the HM_PROFILE profile.  Stops at the first step that times out, faults or aborts.
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
timeout -k 10 1000 python -u -m pytest tests/test_hm_seam.py -x -v --timeout 900 --timeout-method thread -m gpu \
  -k "cu_seam_batched or (cu_seam and ra_smooth)" > gpurun_out/seam_batched.log 2>&1; rc=$?; tail -6 gpurun_out/seam_batched.log
fatal $rc && exit $rc
bash scripts/gpu_hm_ab.sh "$@" || exit $?
HVX_LIB_PATH=$(pwd)/video_codecs_amd/_variants/libhvx_prof.so timeout -k 10 300 python -u -m tests.hm_profile bench 62 1 > gpurun_out/hprof.log 2>&1 || exit $?
tail -34 gpurun_out/hprof.log
exit $rc
