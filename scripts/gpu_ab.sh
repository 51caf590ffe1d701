# A/B of library builds on one box: python bench.py (step only) with each given libhvx variant
# copied over video_codecs_amd/libhvx.so in turn, then the original restored.
# usage (variants built beforehand, in-tree): bash scripts/gpu_ab.sh video_codecs_amd/libhvx_a.so ...
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-cpu --no-ssim --no-intra --no-1080p --no-sao"
show() { tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phase_ms_per_step']; print('$2', d['ms_per_step'], p['me_d2'], p['me_d3'])"; }
cp -p video_codecs_amd/libhvx.so /tmp/libhvx_orig.so || exit 1
# restore the original on every exit path, failures included; if that copy fails, remove the
# variant so the next build() rebuilds libhvx.so from source instead of trusting its mtime
restore() { cp -p /tmp/libhvx_orig.so video_codecs_amd/libhvx.so || rm -f video_codecs_amd/libhvx.so; }
trap restore EXIT
timeout -k 10 200 $B > gpurun_out/ab_orig.log 2>&1 && show gpurun_out/ab_orig.log orig || exit 1
for v in "$@"; do
  cp "$v" video_codecs_amd/libhvx.so || exit 1
  timeout -k 10 200 $B > "gpurun_out/ab_$(basename "$v").log" 2>&1 && show "gpurun_out/ab_$(basename "$v").log" "$v" || exit 1
done
