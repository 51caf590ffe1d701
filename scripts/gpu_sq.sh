# SQ instruction-mix / stall counters for the bench step (one PMC pass, no trace domains).
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $R/gpurun_out/prof_sq -o sq --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/prof_sq.log 2>&1
rc=$?
tail -3 gpurun_out/prof_sq.log
exit $rc
