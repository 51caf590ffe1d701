set -o pipefail
V=video_codecs_amd/_variants
HVX_LIB_PATH=$(pwd)/$V/libhvx_o2nsa.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -m gpu -k "hm_ctu" > gpurun_out/o2nsa_tests.log 2>&1; echo O2NSA_TESTS rc $?
bash scripts/gpu_hm_ab.sh $V/libhvx_ldscoder.so $V/libhvx_o2nsa.so > gpurun_out/ab1.txt 2>&1; cat gpurun_out/ab1.txt
HVX_LIB_PATH=$(pwd)/$V/libhvx_prof.so timeout -k 10 200 python -u -m tests.hm_profile bench 60 1 > gpurun_out/hprof60.log 2>&1
bash scripts/gpu_hm_pmc.sh; echo PMC rc $?
