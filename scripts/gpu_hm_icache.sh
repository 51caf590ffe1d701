# instruction / scalar cache behaviour of k_hm_compress (one launch); counters listed first so an
# unknown name fails fast
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1; grep -oE "SQC?_[A-Z_0-9]+" gpurun_out/avail.txt | sort -u > gpurun_out/avail_sq.txt; grep -E "ICACHE|IFETCH|DCACHE" gpurun_out/avail_sq.txt | head -20
B="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-cpu-ref --no-ra --no-slice0 --no-1080p"
C=$(grep -xE "SQ_IFETCH|SQC_ICACHE_REQ|SQC_ICACHE_HITS|SQC_ICACHE_MISSES|SQC_DCACHE_REQ|SQC_DCACHE_HITS|SQC_DCACHE_MISSES|SQ_WAVES" gpurun_out/avail_sq.txt | head -8 | tr '\n' ' ')
echo "counters: $C"
[ -n "$C" ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/hpmc_i -o i --output-format csv -- python3 $B > gpurun_out/hpmc_i.log 2>&1
