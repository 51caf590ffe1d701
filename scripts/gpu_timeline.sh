# Kernel-trace timeline of one concurrent bench step (rocprofv3 --kernel-trace + scripts/timeline.py).
# usage: bash scripts/gpu_timeline.sh TAG   -> gpurun_out/tl_TAG.txt
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); TAG=${1:-tl}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/tl_${TAG} -o kt --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-intra --no-ssim --no-1080p --no-sao > gpurun_out/tl_${TAG}.log 2>&1 || exit 1
f=$(find gpurun_out/tl_${TAG} -name '*kernel_trace.csv' | head -1)
python3 scripts/timeline.py "$f" > gpurun_out/tl_${TAG}.txt && cat gpurun_out/tl_${TAG}.txt
