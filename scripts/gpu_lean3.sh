# three waves per SIMD (HM_LEAN_LDS, HM_WAVES_PER_EU=3): parity on the HM captures, then the headline
# at 90 pictures (3060 chains) against the tree's build at 60 (2040 chains)
set -o pipefail
V=$(pwd)/video_codecs_amd/_variants/libhvx_lean3.so
HVX_LIB_PATH=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "hm_ctu" > gpurun_out/lean3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/lean3_tests.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --steps 2 --warmup 1 --no-cpu --no-cpu-ref --no-ra --no-slice0 --no-1080p"
show() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], 'CTUs/s', d['ms_per_step'], 'ms/step')"; }
timeout -k 10 300 $B > gpurun_out/l3_orig.log 2>&1 && show gpurun_out/l3_orig.log "orig60" || exit 1
HVX_LIB_PATH=$V timeout -k 10 300 $B --pics 90 > gpurun_out/l3_90.log 2>&1 && show gpurun_out/l3_90.log "lean3_90" || exit 1
HVX_LIB_PATH=$V timeout -k 10 300 $B --pics 60 > gpurun_out/l3_60.log 2>&1 && show gpurun_out/l3_60.log "lean3_60" || exit 1
