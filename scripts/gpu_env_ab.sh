# Bench ms/step under several values of one environment variable (concurrent stream plan).
# usage: bash scripts/gpu_env_ab.sh VAR v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
VAR=$1; shift
B="python bench.py --steps 30 --warmup 5 --no-cpu --no-intra --no-ssim --no-1080p --no-sao"
for v in "$@"; do
  env "$VAR=$v" timeout -k 10 200 $B > gpurun_out/envab_$v.log 2>&1 || exit 1
  echo "$VAR=$v $(grep '^{' gpurun_out/envab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")"
done
