# -O2 engine: checks build on the captures first; only if clean, the plain -O2 build's parity + A/B
set -o pipefail
V=$(pwd)/video_codecs_amd/_variants
for m in 0 1; do
  HVX_LIB_PATH=$V/libhvx_o2chk.so timeout -k 10 150 python -u -m tests.hm_debug ctu_ldp_rand.bin $m > gpurun_out/o2chk_$m.log 2>&1 || exit 3
  tail -3 gpurun_out/o2chk_$m.log
  grep -q " 0 with a failed check" gpurun_out/o2chk_$m.log && grep -q "^0 mismatching" gpurun_out/o2chk_$m.log || exit 4
done
HVX_LIB_PATH=$V/libhvx_o2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "hm_ctu" > gpurun_out/o2_tests.log 2>&1; rc=$?; tail -2 gpurun_out/o2_tests.log; [ $rc -eq 0 ] || exit 5
bash scripts/gpu_hm_ab.sh video_codecs_amd/_variants/libhvx_o2.so > gpurun_out/o2_ab.txt 2>&1; cat gpurun_out/o2_ab.txt
