# 3 waves per SIMD (HM_LEAN_LDS, 168 VGPRs) with 93 pictures (3069 chains), then the HM_PROFILE category profile
set -o pipefail
mkdir -p gpurun_out
show() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], 'CTUs/s', d['ms_per_step'], 'ms/step', d['config']['slice_chains_per_gpu'], 'chains')"; }
HVX_LIB_PATH=$(pwd)/video_codecs_amd/_variants/libhvx_w3lean.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-cpu-ref --no-ra --no-slice0 --no-1080p --pics 93 > gpurun_out/hab_w3_93.log 2>&1 && show gpurun_out/hab_w3_93.log w3lean_93 || exit 1
PICS=62 bash scripts/gpu_hm_prof.sh
