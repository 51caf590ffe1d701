set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-cpu --no-ssim --no-intra --no-1080p --no-sao"
show() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_step']; print('$2', d['ms_per_step'], p['me_d2'], p['me_d3'])"; }
timeout -k 10 200 $B > gpurun_out/abB.log 2>&1 && show gpurun_out/abB.log B &&
cp video_codecs_amd/libhvx.so /tmp/libB.so && cp video_codecs_amd/libhvx_a.so video_codecs_amd/libhvx.so &&
timeout -k 10 200 $B > gpurun_out/abA.log 2>&1 && show gpurun_out/abA.log A &&
cp video_codecs_amd/libhvx_c.so video_codecs_amd/libhvx.so &&
timeout -k 10 200 $B > gpurun_out/abC.log 2>&1 && show gpurun_out/abC.log C &&
cp /tmp/libB.so video_codecs_amd/libhvx.so &&
timeout -k 10 200 $B > gpurun_out/abB2.log 2>&1 && show gpurun_out/abB2.log B2
