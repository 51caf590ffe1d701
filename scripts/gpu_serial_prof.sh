# Isolated per-kernel view of the bench step: every branch on one stream (HVX_SERIAL_STREAMS=1),
# rocprofv3 kernel-trace stats, then one SQ instruction-mix PMC pass.  usage: bash scripts/gpu_serial_prof.sh TAG
set -o pipefail
export TMPDIR=/tmp
export HVX_SERIAL_STREAMS=1
TAG=${1:-serial}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_kt -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-intra --no-ssim --no-1080p --no-sao > gpurun_out/prof_${TAG}_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $R/gpurun_out/prof_${TAG}_sq -o sq --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-intra --no-ssim --no-1080p --no-sao > gpurun_out/prof_${TAG}_sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH -d $R/gpurun_out/prof_${TAG}_sq2 -o sq2 --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-intra --no-ssim --no-1080p --no-sao > gpurun_out/prof_${TAG}_sq2.log 2>&1
rc=$?
tail -2 gpurun_out/prof_${TAG}_kt.log | cut -c1-600
exit $rc
