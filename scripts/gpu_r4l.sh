# one-lane 4x4 RDOQ in the engine: headline A/B against the previous build, the per-category
# profile, then the HM parity tests
set -o pipefail
mkdir -p gpurun_out
V=video_codecs_amd/_variants
STEPS=4 bash scripts/gpu_hm_ab.sh $V/libhvx_rq3.so $V/libhvx_r4l.so $V/libhvx_rq3.so > gpurun_out/ab_r4l.txt 2>&1; rc=$?; cat gpurun_out/ab_r4l.txt; [ $rc -eq 0 ] || exit 2
HVX_LIB_PATH=$(pwd)/$V/libhvx_prof_r4l.so timeout -k 10 300 python -u -m tests.hm_profile bench 62 2 > gpurun_out/hprof_r4l.log 2>&1 || exit 3
tail -34 gpurun_out/hprof_r4l.log | head -20
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "hm_ or tu_" > gpurun_out/r4l_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4l_tests.log; exit $rc
