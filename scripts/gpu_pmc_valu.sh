# One SQ pass on the serial-stream bench step: VALU / SALU issue cycles per kernel (quad-cycles)
# and the GPU busy clock, to tell issue-bound kernels from latency-bound ones.
set -o pipefail
export TMPDIR=/tmp HVX_SERIAL_STREAMS=1
R=$(pwd); TAG=${1:-valu}
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $R/gpurun_out/pmc_$TAG -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-intra --no-ssim --no-1080p --no-sao > gpurun_out/pmc_$TAG.log 2>&1
