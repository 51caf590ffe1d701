"""Debugging aid: the bench's HM-exact workload (bench.HmWorkload, one picture) at several picture
sizes, decided on the GPU for `steps` steps and checked CTU by CTU against the oracle's
hvxo_hm_chains.  python -m tests.hm_bench_check WxH[,WxH...] [steps]"""
import json
import sys

import torch

import bench
from video_codecs_amd import hvx

if __name__ == "__main__":
    sizes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1].split(",")]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    variants = [(int(v[0]), v[1] == "c") for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [(4, True)]
    hvx.context()
    for (W, H) in sizes:
        for nref, col in variants:
            w = bench.HmWorkload(W, H, 1, nref, 32, 1, 0, col=col)
            rec = torch.zeros(w.slots * 6144, dtype=torch.uint8, device="cuda")
            for _ in range(steps):
                w.step(rec)
            torch.cuda.synchronize()
            r = bench.hm_cpu_port(w, 16)
            print(json.dumps({"size": f"{W}x{H}", "nref": nref, "col": col, "ctus": r["gpu_parity_ctus"],
                              "mismatches": r["gpu_parity_mismatches"], "first": r["first_mismatches"]}), flush=True)
            del w, rec
