# One GPU iteration: the named parity tests (pytest -k), then a short bench run of the step only
# (no CPU baseline / side measurements).  usage: bash scripts/gpu_iter.sh "<pytest -k expr>" TAG
set -o pipefail
mkdir -p gpurun_out
K=${1:-"tu or ctu"}
TAG=${2:-iter}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "$K" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu --no-intra --no-ssim --no-1080p --no-sao --no-cabac > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_bench.log | cut -c1-1500; exit $rc
