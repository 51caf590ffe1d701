# A/B of HM-engine builds on one box: the headline step (60 pictures, 2040 chains) per variant.
# usage: bash scripts/gpu_hm_ab.sh lib_a.so ...   (the tree's libhvx.so runs first as "orig")
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu --no-cpu-ref --no-ra --no-1080p --no-closed ${EXTRA:-}"
show() { grep '^{' "$1" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], 'CTUs/s', d['ms_per_step'], 'ms/step', d['roofline']['avg_launch_ms'])"; }
timeout -k 10 300 $B > gpurun_out/hab_orig.log 2>&1 && show gpurun_out/hab_orig.log orig || exit 1
for v in "$@"; do
  n=$(basename "$v" .so)
  HVX_LIB_PATH=$(pwd)/$v timeout -k 10 300 $B > "gpurun_out/hab_$n.log" 2>&1 && show "gpurun_out/hab_$n.log" "$n" || exit 1
done
