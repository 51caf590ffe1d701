# the whole GPU parity file + smoke on the tree's libhvx.so, one headline bench, the HM_PROFILE breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py -q --timeout 600 --timeout-method thread -m gpu \
  > gpurun_out/final_parity.log 2>&1; rc=$?; tail -2 gpurun_out/final_parity.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/final_smoke.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_hm_ab.sh || exit $?
HVX_LIB_PATH=$(pwd)/video_codecs_amd/_variants/libhvx_prof.so timeout -k 10 300 python -u -m tests.hm_profile bench 62 1 > gpurun_out/hprof.log 2>&1 || exit $?
grep -E "bench step|rdoq|TUF |COEF |C.walk|ME  " gpurun_out/hprof.log
