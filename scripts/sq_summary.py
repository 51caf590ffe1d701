"""Per-kernel SQ instruction mix / stall split from a rocprofv3 PMC pass (scripts/gpu_sq.sh).
Values per wave: VALU/SALU/LDS instructions, cycles; WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY
as a share of SQ_WAVE_CYCLES.  usage: python scripts/sq_summary.py <sq_counter_collection.csv>"""
import csv
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
for row in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "").strip()
    acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
print(f"{'kernel':34s} {'waves':>9s} {'cyc/wave':>9s} {'VALU':>7s} {'SALU':>7s} {'LDS':>6s} {'wait':>5s} {'winst':>5s} {'activ':>5s}")
for k, c in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    w = max(c["SQ_WAVES"], 1)
    cyc = c["SQ_WAVE_CYCLES"]
    if cyc == 0:
        continue
    print(f"{k[:34]:34s} {w:9.0f} {cyc / w:9.0f} {c['SQ_INSTS_VALU'] / w:7.0f} {c['SQ_INSTS_SALU'] / w:7.0f} "
          f"{c['SQ_INSTS_LDS'] / w:6.0f} {c['SQ_WAIT_ANY'] / cyc:5.2f} {c['SQ_WAIT_INST_ANY'] / cyc:5.2f} "
          f"{c['SQ_ACTIVE_INST_ANY'] / cyc:5.2f}")
