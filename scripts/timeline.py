"""Per-dispatch timeline of one bench step from a rocprofv3 kernel trace (--kernel-trace, csv):
start/end of every kernel of the LAST complete step relative to that step's first dispatch, with
its queue, so the critical chain of the multi-stream step can be read off.
usage: python scripts/timeline.py <kernel_trace.csv> [first_kernel_of_step]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "k_set_ptr"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(first)]
i0 = starts[-2] if len(starts) > 1 else starts[0]
i1 = starts[-1]
step = rows[i0:i1]
t0 = int(step[0]["Start_Timestamp"])
tend = max(int(r["End_Timestamp"]) for r in step)
print(f"step: {len(step)} dispatches, {(tend - t0) / 1e6:.3f} ms")
for r in step:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:32]
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    print(f"q{q:>3s} {s:7.3f} {e:7.3f} {e - s:6.3f}  {name}")
