# per-category cycle profile of the engine (HM_PROFILE build) on the headline workload
set -o pipefail
mkdir -p gpurun_out
HVX_LIB_PATH=$(pwd)/video_codecs_amd/_variants/libhvx_prof.so timeout -k 10 300 python -u -m tests.hm_profile bench ${PICS:-60} 1 > gpurun_out/hprof.log 2>&1; rc=$?; tail -34 gpurun_out/hprof.log; exit $rc
