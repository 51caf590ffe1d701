"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) per kernel.

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section) and
cdna_hip_programming.md section 7: counters are KiB; on gfx950 FETCH_SIZE reads half the
bytes of wide coalesced streaming reads, so it is doubled (the guide's correction; byte-wide
gather reads as in k_me are uncalibrated -- see DESIGN.md).
usage: python scripts/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
"""
import csv
import json
import re
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0.0, 0])
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = re.sub(r"\(.*", "", row["Kernel_Name"]).replace("void ", "").strip()
        name = re.sub(r"<.*>", lambda m: m.group(0).replace(" ", ""), name)
        acc[name][0] += float(row["Counter_Value"])
        acc[name][1] += 1
    return acc


def main():
    fetch, write, out = sys.argv[1:4]
    f, w = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fk, fn = f.get(k, [0.0, 0])
        wk, wn = w.get(k, [0.0, 0])
        n = max(fn, wn, 1)
        fetch_b = fk / max(fn, 1) * 1024 * 2
        write_b = wk / max(wn, 1) * 1024
        res[k] = {"launches": n, "fetch_kib_raw_per_launch": fk / max(fn, 1), "write_kib_per_launch": wk / max(wn, 1),
                  "bytes_per_launch": fetch_b + write_b, "correction": "FETCH_SIZE x2 (gfx950), KiB x1024"}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:40s} launches={v['launches']:3d} bytes/launch={v['bytes_per_launch']:.3e}")


if __name__ == "__main__":
    main()
