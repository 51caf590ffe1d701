"""Per-kernel instruction counts per wave from scripts/gpu_pmc_inst.sh runs, side by side.
usage: python scripts/inst_cmp.py gpurun_out/inst_orig gpurun_out/inst_<variant> [...]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "").strip()
            acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
    return acc


runs = [load(d) for d in sys.argv[1:]]
keys = sorted(runs[0], key=lambda k: -runs[0][k]["SQ_INSTS_VALU"])[:14]
for k in keys:
    cols = []
    for r in runs:
        c = r.get(k, {})
        w = max(c.get("SQ_WAVES", 0), 1)
        cols.append("%7.0f %7.0f" % (c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_SALU", 0) / w))
    print("%-28s %s" % (k[:28], " | ".join(cols)))
