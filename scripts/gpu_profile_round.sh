# This round's profiles of the headline (k_hm_compress): rocprofv3 kernel-trace stats, the FETCH_SIZE /
# WRITE_SIZE passes and the SQ counter passes (scripts/gpu_profile_bench.sh), then the per-category
# s_memtime split of an HM_PROFILE build (gpurun_extra/libhvx_prof.so, scripts/build_variant.sh prof
# -DHM_PROFILE) on the same workload (tests/hm_profile.py bench).  Outputs under gpurun_out/.
# Before the call (here; video_codecs_amd/_variants does not travel):
#   bash scripts/build_variant.sh prof -DHM_PROFILE && mkdir -p gpurun_extra && cp video_codecs_amd/_variants/libhvx_prof.so gpurun_extra/
set -o pipefail
T=${T:-r06} bash scripts/gpu_profile_bench.sh &&
HVX_LIB_PATH=$PWD/gpurun_extra/libhvx_prof.so timeout -k 10 400 python3 -u -m tests.hm_profile bench 62 2 > gpurun_out/hm_profile_r06.log 2>&1
rc=$?
tail -40 gpurun_out/hm_profile_r06.log | cut -c1-150
exit $rc
