# VALU/SALU instruction counts per kernel of several libhvx builds (serial-stream bench step,
# one SQ pass each).  usage: bash scripts/gpu_pmc_ab.sh lib_a.so ...
set -o pipefail
export TMPDIR=/tmp HVX_SERIAL_STREAMS=1
R=$(pwd)
mkdir -p gpurun_out
cp -p video_codecs_amd/libhvx.so /tmp/libhvx_orig.so || exit 1
restore() { cp -p /tmp/libhvx_orig.so video_codecs_amd/libhvx.so; }
trap restore EXIT
for v in "$@"; do
  t=$(basename "$v" .so)
  cp "$v" video_codecs_amd/libhvx.so || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d $R/gpurun_out/pab_$t -o p --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-intra --no-ssim --no-1080p --no-sao > gpurun_out/pab_$t.log 2>&1 || exit 1
done
