# instruction cache behaviour of k_hm_compress (one launch): SQ_IFETCH and the SQC instruction-cache
# hits / misses, one pass (4 counters); names checked against the profiler's list first
set -o pipefail
export TMPDIR=/tmp
R=$(pwd); mkdir -p gpurun_out
rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1; grep -oE "SQC?_[A-Z_0-9]+" gpurun_out/avail.txt | sort -u > gpurun_out/avail_sq.txt; grep -E "ICACHE|IFETCH" gpurun_out/avail_sq.txt | head -20
B="$R/bench.py --steps 1 --warmup 0 --no-cpu --no-cpu-ref --no-ra --no-1080p --no-closed"
C=$(grep -xE "SQ_IFETCH|SQC_ICACHE_HITS|SQC_ICACHE_MISSES|SQ_WAVES" gpurun_out/avail_sq.txt | head -4 | tr '\n' ' ')
echo "counters: $C"
[ -n "$C" ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/hpmc_i -o i --output-format csv -- python3 $B > gpurun_out/hpmc_i.log 2>&1
rc=$?
python3 - <<'PY'
import csv, collections, glob
d = collections.defaultdict(float)
for f in glob.glob("gpurun_out/hpmc_i/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_hm_compress" in r["Kernel_Name"]:
            d[r["Counter_Name"]] += float(r["Counter_Value"])
print(dict(d))
PY
exit $rc
