#!/usr/bin/env python3
"""Benchmark: 64x64 CTUs/s of the CTU analysis pass (ME + transform + RDOQ) on 2160p random YUV.

One step = hvx_ctu_analyze over one 3840x2160 picture (2040 CTUs): for each of the 85 CUs
of every CTU, TZ integer + half/quarter motion search against 4 reference pictures, luma MC
of the best reference, then transform + RDOQ + dequant + inverse transform + SSE of every
TU (DESIGN.md "CTU analysis pass").  Inputs are resident in HBM before timing starts.

Multi-GPU (torch.distributed.run): one rank per GPU, each rank analyses its own independent
GOP segment (different synthetic frames) -- no data-path collective; weak scaling.

Contract: python bench.py --gpus N --steps K --warmup W  -> one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MI355X_HBM_PEAK_GBS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--nref", type=int, default=4)
    p.add_argument("--qp", type=int, default=32)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    return p.parse_args()


def luma_plane(w, h, index):
    from oracle import make_yuv  # synthetic-input recipe
    y = make_yuv.random_frame(w, h, index)[: w * h].reshape(h, w)
    return np.pad(y, 80, mode="edge")


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local_rank)

    from video_codecs_amd import _abi, hvx

    W, H, nref = args.width, args.height, args.nref
    # independent GOP segment per rank: frames base .. base+nref (refs, then the current picture)
    base = rank * (nref + 1)
    planes = [luma_plane(W, H, base + i) for i in range(nref + 1)]
    cur_t = torch.from_numpy(planes[nref]).cuda()
    ref_t = [torch.from_numpy(p).cuda() for p in planes[:nref]]
    ref_ptrs = torch.tensor([hvx.plane_origin_ptr(t, W) for t in ref_t], dtype=torch.int64).cuda()
    an = hvx.CtuAnalyzer(W, H, nref, args.qp)
    nctu = an.nctu

    for _ in range(args.warmup):
        an.run(cur_t, ref_ptrs)
    torch.cuda.synchronize()
    hvx.set_timing(True)
    hvx.phase_times(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        an.run(cur_t, ref_ptrs)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    phases = hvx.phase_times(reset=True)
    hvx.set_timing(False)
    gpu_res = an.results()

    if rank == 0:
        ctus = nctu * args.steps * world
        value = ctus / elapsed
        # roofline of the dominant kernel: k_me_int_ctu (4 launches per step, one per CU depth)
        me_ms_step = sum(phases[f"me_d{d}"] for d in range(4)) / args.steps
        launch_ms = me_ms_step / 4.0
        bytes_per_launch = nctu * 4096 * (1 + nref)  # each luma sample of cur + refs once
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        traffic = None
        tr_path = os.path.join(ROOT, "profiles", "hbm_traffic_r01.json")
        if os.path.exists(tr_path):
            tr = json.load(open(tr_path)).get("k_me_int_ctu")
            if tr:
                traffic = tr["bytes_per_launch"]
        out = {
            "metric": "64x64 CTUs/s (ME+transform+RDOQ) on 2160p YUV, 1->8 MI355X; bit-exact vs HM",
            "value": round(value, 2),
            "unit": "CTUs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: splitmix64 uniform random 8-bit luma (BASELINE.md sec. 3), independent segment per rank",
            "config": {"workload": "CTU analysis pass: 85 CUs x TZ+frac ME vs %d refs, MC, TU RDOQ/dequant/IT/SSE" % nref,
                       "resolution": f"{W}x{H}", "ctus_per_frame": nctu, "qp": args.qp, "search_range": 64,
                       "n_ref": nref, "parallelism": f"segments x{world}"},
            "phase_ms_per_step": {k: round(v / args.steps, 3) for k, v in phases.items()},
            "roofline": {"bound": "hbm", "kernel": "k_me_int_ctu", "achieved": round(achieved, 3),
                         "peak": MI355X_HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / MI355X_HBM_PEAK_GBS,
                         "traffic": traffic, "bytes_per_launch": bytes_per_launch,
                         "avg_launch_ms": round(launch_ms, 3)},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(planes, an, gpu_res, args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(planes, an, gpu_res, args):
    """The oracle (scalar C port of the same pass, 1 core) on a bounded sample of the same
    picture's CTUs in raster order; also checks the GPU result of every sampled CTU."""
    import oracle
    from video_codecs_amd import _abi
    nref = args.nref
    est = _abi.load_estbits_p_luma()
    ncx = (args.width + 63) // 64
    n_done, mismatches = 0, 0
    t0 = time.perf_counter()
    for c in range(an.nctu):
        r = oracle.ctu_analyze(planes[nref], planes[:nref], an.params, est, c % ncx, c // ncx)
        if r.tobytes() != gpu_res[c].tobytes():
            mismatches += 1
        n_done += 1
        if time.perf_counter() - t0 > args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n_done / dt, 3), "unit": "CTUs/s", "cores": 1, "kind": "port",
            "sample": f"first {n_done} CTUs (raster) of the same 2160p picture, {dt:.1f} s, oracle/hvx_oracle.c",
            "gpu_parity_ctus": n_done, "gpu_parity_mismatches": mismatches}


if __name__ == "__main__":
    main()
