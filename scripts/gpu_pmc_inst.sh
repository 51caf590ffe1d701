# Dynamic instruction mix per kernel (one SQ pass on the serial-stream bench step) for the tree's
# libhvx.so and each variant given.  usage: bash scripts/gpu_pmc_inst.sh [lib.so ...]
set -o pipefail
export TMPDIR=/tmp HVX_SERIAL_STREAMS=1
R=$(pwd)
mkdir -p gpurun_out
cp -p video_codecs_amd/libhvx.so /tmp/libhvx_orig.so || exit 1
restore() { cp -p /tmp/libhvx_orig.so video_codecs_amd/libhvx.so; }
trap restore EXIT
run() {
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU -d $R/gpurun_out/inst_$1 -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-intra --no-ssim --no-1080p --no-sao > gpurun_out/inst_$1.log 2>&1
}
run orig || exit 1
for v in "$@"; do
  cp "$v" video_codecs_amd/libhvx.so || exit 1
  run "$(basename "$v" .so)" || exit 1
done
