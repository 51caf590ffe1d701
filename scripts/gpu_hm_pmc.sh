# SQ counters of k_hm_compress on the headline step (one launch, 2040 chains), in separate passes.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
B="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-cpu-ref --no-ra --no-1080p --no-closed ${EXTRA:-}"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $R/gpurun_out/hpmc_a -o a --output-format csv -- python3 $B > gpurun_out/hpmc_a.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d $R/gpurun_out/hpmc_b -o b --output-format csv -- python3 $B > gpurun_out/hpmc_b.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/hpmc_c -o c --output-format csv -- python3 $B > gpurun_out/hpmc_c.log 2>&1
