# one wave per SIMD (504 VGPRs, no spills) on 1020 chains vs the tree's two waves on 2040
set -o pipefail
V=$(pwd)/video_codecs_amd/_variants/libhvx_w1.so
B="python -u bench.py --steps 2 --warmup 1 --no-cpu --no-cpu-ref --no-ra --no-slice0 --no-1080p"
show() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], 'CTUs/s', d['ms_per_step'], 'ms/step')"; }
HVX_LIB_PATH=$V timeout -k 10 300 $B --pics 30 > gpurun_out/w1_30.log 2>&1 && show gpurun_out/w1_30.log "w1_30" || exit 1
timeout -k 10 300 $B --pics 30 > gpurun_out/w2_30.log 2>&1 && show gpurun_out/w2_30.log "orig_30" || exit 1
