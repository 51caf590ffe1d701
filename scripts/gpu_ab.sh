# Per-phase times of several libhvx builds on one box; SERIAL=1 (default) puts every branch on one
# stream (isolated kernels), SERIAL=0 keeps the concurrent stream plan.  usage: bash scripts/gpu_ab.sh lib_a.so ...
set -o pipefail
mkdir -p gpurun_out
export HVX_SERIAL_STREAMS=${SERIAL:-1}
B="python bench.py --steps 30 --warmup 5 --no-cpu --no-ssim --no-intra --no-1080p --no-sao --no-cabac"
show() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_step']; print('$2', d['ms_per_step'], ' '.join('%s=%.3f' % kv for kv in p.items()))"; }
cp -p video_codecs_amd/libhvx.so /tmp/libhvx_orig.so || exit 1
restore() { cp -p /tmp/libhvx_orig.so video_codecs_amd/libhvx.so || rm -f video_codecs_amd/libhvx.so; }
trap restore EXIT
timeout -k 10 200 $B > gpurun_out/abs_orig.log 2>&1 && show gpurun_out/abs_orig.log orig || exit 1
for v in "$@"; do
  cp "$v" video_codecs_amd/libhvx.so || exit 1
  timeout -k 10 200 $B > "gpurun_out/abs_$(basename "$v").log" 2>&1 && show "gpurun_out/abs_$(basename "$v").log" "$v" || exit 1
done
