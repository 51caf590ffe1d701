# round 5: the product (LDS record + chain state zeroed) on the HM parity tests and an A/B against
# the previous build, then the -O2 engine with the same zeroing once on a captured picture set
set -o pipefail
mkdir -p gpurun_out
V=$(pwd)/video_codecs_amd/_variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k hm_ > gpurun_out/z_tests.log 2>&1; rc=$?; tail -2 gpurun_out/z_tests.log; [ $rc -eq 0 ] || exit 2
STEPS=4 bash scripts/gpu_hm_ab.sh video_codecs_amd/_variants/libhvx_rq3.so video_codecs_amd/_variants/libhvx_rq3.so > gpurun_out/ab_z.txt 2>&1; rc=$?; cat gpurun_out/ab_z.txt; [ $rc -eq 0 ] || exit 3
HVX_LIB_PATH=$V/libhvx_o2z.so timeout -k 10 150 python -u -m tests.hm_debug ctu_ldp_rand.bin 0 > gpurun_out/o2z.log 2>&1; rc=$?; tail -4 gpurun_out/o2z.log; [ $rc -eq 0 ] || exit 4
STEPS=4 bash scripts/gpu_hm_ab.sh video_codecs_amd/_variants/libhvx_o2z.so > gpurun_out/ab_o2z.txt 2>&1; cat gpurun_out/ab_o2z.txt
