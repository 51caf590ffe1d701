# RDOQ phase profile, then the -O2 HM_CHECKS build on one captured picture (last: it may fault)
set -o pipefail
bash scripts/gpu_hm_prof.sh > /dev/null 2>&1; grep -E "bench step|rdoq|TUF4|C.walk" gpurun_out/hprof.log
HVX_LIB_PATH=$(pwd)/video_codecs_amd/_variants/libhvx_o2chk.so timeout -k 10 120 python -u -m tests.hm_debug ctu_ldp_rand.bin 0 1 > gpurun_out/o2dbg.log 2>&1; echo "o2dbg rc $?"; tail -12 gpurun_out/o2dbg.log
