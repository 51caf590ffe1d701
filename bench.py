#!/usr/bin/env python3
"""Benchmark: 64x64 CTUs/s of HM-16.5rc1's CU mode decision on 2160p random YUV, bit-exact vs HM.

One step = one launch of hvx_hm_compress (include/hvx.h) over every SliceMode=1 slice of P
pictures in flight: a 3840x2160 4:2:0 picture has 34 CTU rows, each row a slice; with 22 pictures
per GPU that is 748 slice chains, one wave each, and a step advances every chain by --ctus CTUs
(default 1), each CTU TEncCu::compressCtu + encodeCtu exactly as HM decides it: merge/skip, AMVP
+ TZ search + fractional refinement against 4 references, 2NxN/Nx2N/AMP, the RQT with RDOQ and
transform skip, intra-in-inter, the CABAC context carry.  The chains' CABAC
state and CTU data stay in HBM between steps (HVX_HM_RESUME).  Inputs are resident in HBM before
timing starts; each picture's reference frames are the previous synthetic frames.

Multi-GPU (torch.distributed.run): one rank per GPU, each rank decides its own pictures (different
synthetic frames); per step every rank's reconstructed CTUs are gathered to rank 0's shared DPB
(video_codecs_amd/dpb.py, RCCL over xGMI, asynchronous, double-buffered); weak scaling.

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
METRIC = "64\u00d764 CTUs/s (ME+transform+RDOQ) on 2160p YUV, 1\u21928 MI355X; bit-exact vs HM"
# the bench picture: GOP position 2 of tests/hm_seam/ldp.cfg's LDP GOP at base QP 32 -> QP 34,
# QPFactor 0.4624, GOP depth 1 (TEncSlice.cpp:320-374)
HM_QP_OFFSET, HM_QP_FACTOR = 2, 0.4624


T_START = time.perf_counter()


def progress(msg):
    """A progress line on stderr (the JSON result is the only stdout line)."""
    print("bench[%6.1fs]: %s" % (time.perf_counter() - T_START, msg), file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--pics", type=int, default=62, help="P pictures in flight per GPU (33 slice chains each at 2160p: "
                                                        "62 -> 2046 chains, two waves per SIMD)")
    p.add_argument("--ctus", type=int, default=1, help="CTUs each slice chain advances per step")
    p.add_argument("--cpu-ref-procs", type=int, default=0, help="HM TAppEncoder processes for the reference "
                                                                  "baseline (0: the host's CPU share)")
    p.add_argument("--no-cpu-ref", action="store_true", help="skip the reference HM timing")
    p.add_argument("--no-ra", action="store_true", help="skip the config-4 side figure (RA B pictures, SSIM cost)")
    p.add_argument("--no-slice0", action="store_true", help="skip the SliceMode 0 side figure")
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--nref", type=int, default=4)
    p.add_argument("--qp", type=int, default=32)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-1080p", action="store_true", help="skip the 1080p side measurement")
    p.add_argument("--no-closed", action="store_true", help="skip the closed-loop LDP segment side figure (config 5: "
                                                            "120 segments of 1920x1088 I + 2 P pictures, ~2 minutes)")
    return p.parse_args()


def b_ctu(nref):
    """SURVEY.md 8(d) algorithmic bytes per CTU, B = S(1 + N_ref + 1) + 2S + 16(64*64/16), with
    S = 64*64*1.5 (4:2:0): read the original and N_ref references once, write the reconstruction,
    int16 levels and the 16 B-per-4x4 MV/mode field (53,248 B at N_ref = 4)."""
    S = 64 * 64 * 3 // 2
    return S * (1 + nref + 1) + 2 * S + 16 * (64 * 64 // 16)


def timed_steps(step, steps, warmup, world, device, sync, before=None):
    """W untimed warmup steps, then EXACTLY `steps` steps bracketed by barrier + device sync on
    both sides; returns the MAX elapsed seconds over ranks (all ranks receive it)."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        step()
    sync()
    if before is not None:
        before()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def aggregate(units_per_step, steps, world, elapsed):
    """Whole-job throughput: the units ALL ranks processed / the max-over-ranks time."""
    return units_per_step * steps * world / elapsed


def yuv_split(flat, w, h):
    """Planar Y | Cb | Cr bytes -> the three 2-D planes."""
    ysz, csz = w * h, w * h // 4
    return (flat[:ysz].reshape(h, w), flat[ysz:ysz + csz].reshape(h // 2, w // 2),
            flat[ysz + csz:ysz + 2 * csz].reshape(h // 2, w // 2))


def synthetic_col_field(nctu, seed):
    """The collocated picture's motion field (hvx_hm_picture.col_field: per 16x16 block mode,
    ref idx L0/L1, MV L0/L1): synthetic, seeded -- 70% inter blocks with an L0 reference 0-3 and a
    quarter-sample MV within +-32 samples, 30% intra -- so the TMVP candidate (TComDataCU::
    getColMVP) is exercised with scaling."""
    rng = np.random.default_rng(seed)
    f = np.zeros((nctu * 16, 8), np.int16)
    inter = rng.random(nctu * 16) < 0.7
    f[:, 0] = np.where(inter, 0, 1)
    f[:, 1] = np.where(inter, rng.integers(0, 4, nctu * 16), -1)
    f[:, 2] = -1
    f[:, 3:5] = np.where(inter[:, None], rng.integers(-128, 129, (nctu * 16, 2)), 0)
    return f


class HmPlan:
    """The headline workload's host-side plan (no device): `pics` P pictures of W x H random 4:2:0
    YUV per rank, picture p (POC nref + p) predicted from the nref previous frames of the rank's own
    frame range (frames base .. base + nref + pics - 1, base = 1000 + rank * (pics + nref): disjoint
    across ranks), every CTU row a SliceMode=1 slice decided by one chain -- a partial
    bottom row continues the chain of the row above it (HVX_HM_SLICE_CTUS) -- with the slice
    parameters of GOP position 2 of the LDP GOP (hm.slice_params)."""

    def __init__(self, W, H, pics, nref, base_qp, ctus, rank, col=True):
        from video_codecs_amd import _abi, hm
        self.W, self.H, self.pics, self.nref, self.ctus, self.col = W, H, pics, nref, ctus, col
        self.wc, self.hc = (W + 63) // 64, (H + 63) // 64
        assert self.wc % ctus == 0, "--ctus must divide the CTUs per row"
        self.qp = base_qp + HM_QP_OFFSET
        self.base = rank * (pics + nref) + 1000
        self.params = hm.slice_params(1, self.qp, HM_QP_FACTOR)
        self.entry = _abi.load_ctx_init_states()[1, self.qp]
        # the chains of a picture: one per CTU row slice, except that a partial bottom row (2160 =
        # 33 x 64 + 48) is chained after the row above it -- its first CTU is a picture-boundary CTU
        # whose searches read TEncSearch::m_integerMv2Nx2N as the row above's last CTU left it
        # (HVX_HM_SLICE_CTUS: the coder restarts at the slice, the search state carries on)
        self.merge_last = H % 64 != 0 and self.hc >= 2
        self.rows = self.hc - 1 if self.merge_last else self.hc
        self.n_jobs = pics * self.rows
        self.slots = self.n_jobs * ctus

    def frames(self):
        """The synthetic frame indices this rank reads (references and current pictures)."""
        return list(range(self.base, self.base + self.nref + self.pics))

    def col_field(self, p):
        return synthetic_col_field(self.wc * self.hc, self.base + p) if self.col else None

    def picture_params(self, p):
        poc, nref = self.nref + p, self.nref
        q = dict(self.params)
        q.update(poc=poc, nref=[nref, 0], ref_poc=np.array([[poc - 1 - k for k in range(4)], [0] * 4]),
                 ref_plane=np.array([list(range(nref)) + [0] * (4 - nref), [0] * 4]), max_merge=5, tmvp=1, check_ldc=1,
                 col_from_l0=1, col_valid=int(self.col), col_poc=poc - 1,
                 col_ref_poc=np.array([[poc - 2 - k for k in range(4)], [0] * 4]), search_range=64, amp=1)
        return q

    def host_inputs(self, p):
        """Picture p's arrays in the oracle's (cu_capture.cpp) layout: pic_i32, pic_f64, org,
        reference frames, collocated field."""
        from video_codecs_amd import synth
        prm = self.picture_params(p)
        pi, pf = host_pic_arrays(self.W, self.H, prm, self.qp, col_nref=(4, 0) if self.col else (0, 0))
        org = synth.random_frame(self.W, self.H, self.base + self.nref + p)
        refs = np.concatenate([synth.random_frame(self.W, self.H, self.base + self.nref + p - 1 - k)
                               for k in range(self.nref)])
        return pi, pf, org, refs, self.col_field(p)


def host_pic_arrays(W, H, prm, qp, col_nref=(4, 0)):
    """A picture's slice parameters (hm.DevicePicture's params dict) as the restatement's pic_i32 /
    pic_f64 arrays (oracle/cu_capture.cpp layout: hm_cases.P_* fields)."""
    pi = np.zeros(46, np.int32)
    nref = prm["nref"]
    pi[0:7] = [W, H, prm["poc"], prm["slice_type"], qp, nref[0], nref[1]]
    pi[7:11] = [int(prm["ref_poc"][0][k]) if k < nref[0] else -1 for k in range(4)]
    pi[11:15] = [int(prm["ref_poc"][1][k]) if k < nref[1] else -1 for k in range(4)]
    pi[15:19] = [int(prm["ref_plane"][0][k]) if k < nref[0] else -1 for k in range(4)]
    pi[19:23] = [int(prm["ref_plane"][1][k]) if k < nref[1] else -1 for k in range(4)]
    pi[23:29] = [prm["col_from_l0"], 0, prm["check_ldc"], prm["tmvp"], prm["max_merge"], prm["col_poc"]]
    pi[29:31] = col_nref
    pi[31:35] = prm["col_ref_poc"][0]
    pi[35:39] = prm["col_ref_poc"][1]
    pi[39:41] = prm["chroma_qp"]
    pi[41:43] = [0, ((W + 63) // 64) * ((H + 63) // 64)]
    pi[43] = np.array(prm["lambda_motion"], np.uint32).view(np.int32)
    pi[45] = int(prm["col_valid"])
    pf = np.array([prm["lambda"], prm["sqrt_lambda"], *prm["chroma_weight"], *prm["tq_lambda"]], np.float64)
    return pi, pf


class HmWorkload(HmPlan):
    """The headline workload on one GPU (HmPlan's pictures and chains, resident in HBM).  Step k
    advances every chain by `ctus` CTUs from where step k-1 left it (HVX_HM_RESUME); a chain that
    reaches its row's end starts the row again as a new slice."""

    def __init__(self, W, H, pics, nref, base_qp, ctus, rank, col=True):
        import torch
        from video_codecs_amd import _abi, hm, synth
        super().__init__(W, H, pics, nref, base_qp, ctus, rank, col)
        eb = _abi.load_entropy_bits()
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(8) as ex:
            host = list(ex.map(lambda i: synth.random_frame(W, H, self.base + i), range(nref + pics)))
        frames = [hm.DeviceFrame(yuv_split(f, W, H)) for f in host]
        del host
        self.pictures = []
        for p in range(pics):
            self.pictures.append(hm.DevicePicture(frames[nref + p], [frames[nref + p - 1 - k] for k in range(nref)],
                                                  self.picture_params(p), eb,
                                                  col_field=self.col_field(p)))
        self.eng = hm.Engine(self.pictures)
        self.stream = torch.cuda.Stream()
        torch.cuda.synchronize()  # inputs resident before any launch on the workload's stream
        self.eng.reserve(self.n_jobs)
        # one device job array per step position (the step's first CTU of every chain); the period
        # is two rows when the last chain spans two
        self.phase_jobs = []
        period = 2 * self.wc if self.merge_last else self.wc
        for pos in range(0, period, ctus):
            j = np.zeros(self.n_jobs, hm.HM_JOB)
            for p in range(pics):
                for r in range(self.rows):
                    k = p * self.rows + r
                    j[k]["pic"], j[k]["n_ctus"], j[k]["chained"], j[k]["out"] = p, ctus, 1, k * ctus
                    j[k]["entry"]["st"] = self.entry
                    if self.merge_last and r == self.rows - 1:
                        j[k]["first_ctu"] = r * self.wc + pos
                        j[k]["flags"] = _abi.hm_slice_ctus(self.wc) | (_abi.HM_RESUME if pos else 0)
                    else:
                        q = pos % self.wc
                        j[k]["first_ctu"] = r * self.wc + q
                        j[k]["slice_start"], j[k]["slice_end"] = r * self.wc, r * self.wc + self.wc - 1
                        j[k]["flags"] = _abi.HM_RESUME if q else 0
            self.phase_jobs.append(torch.from_numpy(j.view(np.uint8).reshape(-1).copy()).cuda())
        self.out_ctu = torch.zeros(self.slots * hm.HM_CTU.itemsize, dtype=torch.uint8, device="cuda")
        self.step_idx = 0
        # picture 0's chains (slots 0 .. rows*ctus-1): every step's CTU records + reconstruction
        # kept for the parity check against the oracle after the timed region
        self.keep_steps = []
        self.keep_n = self.rows * ctus

    def step(self, out_rec, events=None):
        """One launch: every chain advances `ctus` CTUs; reconstructed CTUs go to out_rec.  The
        launch, its HIP events and the copies of its records are ordered on the workload's own
        stream (the library launches on torch's current stream when that is not the null stream)."""
        import torch
        pos = self.step_idx % len(self.phase_jobs)
        with torch.cuda.stream(self.stream):
            if events is not None:
                events[0].record()
            self.eng.launch(self.phase_jobs[pos], self.n_jobs, self.out_ctu, out_rec)
            if events is not None:
                events[1].record()
            self.keep_steps.append((pos * self.ctus, self.out_ctu[:self.keep_n * 22544].clone(),
                                    out_rec[:self.keep_n * 6144].clone()))
        self.step_idx += 1


def _chain_jobs(specs, entry):
    """HM_JOB records: specs = [(pic, first_ctu, n_ctus, slice_start, slice_end, resume)]."""
    from video_codecs_amd import _abi, hm
    j = np.zeros(len(specs), hm.HM_JOB)
    for k, (pic, first, n, s0, s1, resume) in enumerate(specs):
        j[k]["pic"], j[k]["first_ctu"], j[k]["n_ctus"], j[k]["chained"], j[k]["out"] = pic, first, n, 1, k * n
        j[k]["slice_start"], j[k]["slice_end"] = s0, s1
        j[k]["flags"] = _abi.HM_RESUME if resume else 0
        j[k]["entry"]["st"] = entry
    return j


def _time_chains(eng, job_steps, n_out, warmup, keep=0):
    """Launch warmup + timed steps of chain jobs on a private stream; returns (seconds per timed
    step from HIP events, wall seconds per timed step, kept) -- kept: per step, copies of the first
    `keep` output slots (HM_CTU records, reconstructions) for a parity check after the timing."""
    import torch
    from video_codecs_amd import hm
    stream = torch.cuda.Stream()
    out_ctu = torch.zeros(n_out * hm.HM_CTU.itemsize, dtype=torch.uint8, device="cuda")
    out_rec = torch.zeros(n_out * 6144, dtype=torch.uint8, device="cuda")
    dev_jobs = [torch.from_numpy(j.view(np.uint8).reshape(-1).copy()).cuda() for j in job_steps]
    n_jobs = len(job_steps[0])
    torch.cuda.synchronize()
    ev, kept = [], []
    t0 = None
    with torch.cuda.stream(stream):
        for k, jt in enumerate(dev_jobs):
            if k == warmup:
                stream.synchronize()
                t0 = time.perf_counter()
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            e[0].record()
            eng.launch(jt, n_jobs, out_ctu, out_rec)
            e[1].record()
            ev.append(e)
            e[1].synchronize()
            progress("side-figure step %d/%d: %.1f ms" % (k + 1, len(dev_jobs), e[0].elapsed_time(e[1])))
            if keep:
                kept.append((out_ctu[:keep * hm.HM_CTU.itemsize].clone(), out_rec[:keep * 6144].clone()))
    stream.synchronize()
    wall = (time.perf_counter() - t0) / (len(dev_jobs) - warmup)
    ms = sum(a.elapsed_time(b) for a, b in ev[warmup:]) / (len(dev_jobs) - warmup)
    return ms * 1e-3, wall, kept


def compare_chain_ctus(port, dev_parts, dev_coef, dev_rec, dev_cost, dev_bd):
    """Mismatches between the restatement's outputs (hm_ctu.chains, CTU o) and the device's records
    of the same CTUs (arrays indexed o): partitions, coefficients, reconstruction, totals."""
    from video_codecs_amd import hm
    mism, first = 0, []
    for o in range(len(dev_parts)):
        what = None
        if not np.array_equal(port["parts"][o], dev_parts[o]):
            d = np.argwhere(port["parts"][o] != dev_parts[o])
            z, f = int(d[0][0]), int(d[0][1])
            what = "part z=%d %s port=%d gpu=%d (%d fields differ)" % (z, hm.PART_FIELDS[f], port["parts"][o][z, f],
                                                                      dev_parts[o][z, f], len(d))
        elif not np.array_equal(port["coef"][o].astype(np.int16), dev_coef[o]):
            what = "coef"
        elif not np.array_equal(port["recon"][o], dev_rec[o]):
            what = "recon"
        elif port["cost"][o] != dev_cost[o] or not np.array_equal(port["bits_dist"][o], dev_bd[o]):
            what = "totals port=(%s,%r) gpu=(%s,%r)" % (list(port["bits_dist"][o]), port["cost"][o], list(dev_bd[o]),
                                                      dev_cost[o])
        if what:
            mism += 1
            if len(first) < 4:
                first.append("ctu %d: %s" % (o, what))
    return mism, first


def stv_history_frames(W, H, n=25, seed=8000):
    """A synthetic stVSSIM history (hvx_hm_picture.hist) of n previous pictures, most recent first: random
    4:2:0 originals and reconstructions = original + a seeded +-3 perturbation (clipped)."""
    from video_codecs_amd import synth
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        org = yuv_split(synth.random_frame(W, H, seed + k), W, H)
        rec = [np.clip(p.astype(np.int16) + rng.integers(-3, 4, p.shape, dtype=np.int16), 0, 255).astype(np.uint8)
               for p in org]
        out.append(tuple(np.ascontiguousarray(p) for p in (*org, *rec)))
    return out


def ra_ssim_measure(W, H, pics=62, distinct=12, qps=(22, 27, 32, 37), warmup=1, steps=10, parity_threads=16):
    """BASELINE config 4 (side figure): 2160p random-access B pictures with the stvssim encoder's active
    stVSSIM cost in the decision (hvx_hm_compress, HVX_RD_STVSSIM: distortionstVSSIM stvssim.c:831 over a
    full 25-picture history + the current picture, the direction map from the collocated field, eta 1)
    at QP 22 / 27 / 32 / 37.  The picture is GOP position 2 of encoder_randomaccess_main.cfg in the
    fourth GOP (POC 28, coding index 26, TId 1: QP offset 2, QPFactor 0.3536, L0 = {24, 32}, L1 = {32,
    24}, TMVP from L1[0], BipredSearchRange 4), `pics` pictures in flight (over `distinct` synthetic frame
    triples, one shared synthetic history), every CTU row a slice (the partial bottom row chained after
    the row above); one step = every chain one CTU, `steps` timed steps after `warmup`.  The B-slice
    decision is pinned to HM by the RA captures (tests/golden/ctu_ra_q*.bin); here every CTU of picture
    0's chains the GPU decided is re-decided by the restatement with the same cost and history
    (oracle/hvx_oracle_cu.c hvxo_hm_chains_stv) and compared bit for bit."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    import oracle  # noqa: F401  (test infrastructure: the parity checker, after the timing)
    from oracle import hm_ctu
    from video_codecs_amd import _abi, hm, synth
    wc, hc = (W + 63) // 64, (H + 63) // 64
    eb = _abi.load_entropy_bits()
    with ThreadPoolExecutor(8) as ex:
        host = list(ex.map(lambda i: synth.random_frame(W, H, 7000 + i), range(3 * distinct)))
    frames = [hm.DeviceFrame(yuv_split(f, W, H)) for f in host]
    col_h = synthetic_col_field(wc * hc, 77)
    col = torch.from_numpy(col_h).cuda()
    hist = stv_history_frames(W, H)
    dirs = hm.stv_direction_map(col_h, W, H)
    stv = hm.StvHistory(hist, dirs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stv.prepare(W, H)  # the history sums, once per history (once per picture in an encode)
    torch.cuda.synchronize()
    prep_ms = (time.perf_counter() - t0) * 1e3
    rows = hc - 1 if H % 64 else hc  # the partial bottom row chained after the row above (HmWorkload)
    res = {}
    for base_qp in qps:
        qp = base_qp + 2
        prm = hm.slice_params(0, qp, 0.3536)
        entry = _abi.load_ctx_init_states()[0, qp]
        prm.update(poc=28, nref=[2, 2], ref_poc=np.array([[24, 32, 0, 0], [32, 24, 0, 0]]),
                   ref_plane=np.array([[0, 1, 0, 0], [1, 0, 0, 0]]), max_merge=5, tmvp=1, check_ldc=0, col_from_l0=0,
                   col_valid=1, col_poc=32, col_ref_poc=np.array([[24, 16, 8, 0], [0] * 4]), search_range=64, amp=1,
                   rd_metric=_abi.RD_STVSSIM, lambda_ssim=hm.lambda_ssim(qp))
        pictures = []
        for p in range(pics):
            k = p % distinct
            pictures.append(hm.DevicePicture(frames[3 * k + 2], [frames[3 * k], frames[3 * k + 1]], prm, eb, col_field=col,
                                             stv=stv))
        eng = hm.Engine(pictures)
        job_steps = []
        for pos in range(warmup + steps):
            specs = [(p, r * wc + pos, 1, r * wc, r * wc + wc - 1, pos > 0) for p in range(pics) for r in range(rows)]
            j = _chain_jobs(specs, entry)
            if rows < hc:
                j["flags"][rows - 1::rows] |= _abi.hm_slice_ctus(wc)
            job_steps.append(j)
        sec, wall, kept = _time_chains(eng, job_steps, pics * rows, warmup, keep=rows)
        del eng, pictures
        torch.cuda.empty_cache()
        # parity: picture 0's `rows` chains, CTUs 0 .. warmup + steps - 1 of each, on the restatement
        done = warmup + steps
        pi, pf = host_pic_arrays(W, H, prm, qp, col_nref=(4, 0))
        t0 = time.perf_counter()
        progress("config 4 QP %d: restatement parity (%d chains x %d CTUs)" % (base_qp, rows, done))
        port = hm_ctu.chains(pi, pf, host[2], np.concatenate([host[0], host[1]]), entry,
                             np.arange(rows, dtype=np.int32) * wc, done, wc, threads=parity_threads, col_field=col_h,
                             rd_metric=_abi.RD_STVSSIM, lambda_ssim=prm["lambda_ssim"], stv=(hist, dirs))
        port_s = time.perf_counter() - t0
        dev = [(ct.cpu().numpy().view(hm.HM_CTU), rc.cpu().numpy().reshape(rows, 6144)) for ct, rc in kept]
        order = [(k, s) for k in range(rows) for s in range(done)]  # the port's CTU order: chain-major
        mism, first = compare_chain_ctus(
            port, np.stack([hm.unpack_parts(dev[s][0][k]["p"]) for k, s in order]),
            np.stack([dev[s][0][k]["coef"] for k, s in order]), np.stack([dev[s][1][k] for k, s in order]),
            np.array([dev[s][0][k]["cost"] for k, s in order]),
            np.array([[dev[s][0][k]["bits"], dev[s][0][k]["dist"]] for k, s in order], np.uint32))
        res[str(base_qp)] = {"slice_qp": qp, "ctus_per_s": round(pics * rows / sec, 2), "ms_per_step": round(sec * 1e3, 1),
                             "wall_ms_per_step": round(wall * 1e3, 1), "lambda_ssim": prm["lambda_ssim"],
                             "gpu_parity_ctus": len(order), "gpu_parity_mismatches": mism, "first_mismatches": first,
                             "port_ctus_per_s": round(len(order) / port_s, 2)}
    return {"workload": "2160p RA B pictures (GOP position 2 of the fourth GOP: POC 28, L0 {24,32} / L1 {32,24}, bi-pred "
                        "+ bBi refinement), stVSSIM cost (distortionstVSSIM over a 25-picture history, direction map from "
                        "the collocated field) in TEncCu's decisions, eta 1, %d pictures x %d row-slice chains, %d timed "
                        "steps after %d warmup; parity: picture 0's chains re-decided by oracle/hvx_oracle_cu.c on %d host "
                        "threads" % (pics, rows, steps, warmup, parity_threads),
            "rd_metric": "HVX_RD_STVSSIM", "hist_n": len(hist), "stv_prepare_ms": round(prep_ms, 1), "per_qp": res}


def slice_mode0_measure(W, H, chains=2040, distinct=16, nref=4, base_qp=32, warmup=1, steps=10):
    """Side figure: the headline's P pictures coded with HM's default SliceMode 0 (one slice per
    picture, encoder_lowdelay_P_main.cfg:63) -- `chains` independent single-slice 2160p pictures in
    flight, one chain each (its own CTU array and reconstruction; the synthetic frames are shared by
    `distinct` picture contents), every chain deciding its picture's CTUs in raster order from CTU 0.
    Shows whether the headline rate depends on the row slices: it depends on the number of
    independent chains, not on how a picture is sliced."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from video_codecs_amd import _abi, hm, synth
    wc, hc = (W + 63) // 64, (H + 63) // 64
    qp = base_qp + HM_QP_OFFSET
    eb = _abi.load_entropy_bits()
    with ThreadPoolExecutor(8) as ex:
        host = list(ex.map(lambda i: synth.random_frame(W, H, 9000 + i), range(distinct + nref)))
    frames = [hm.DeviceFrame(yuv_split(f, W, H)) for f in host]
    del host
    col = torch.from_numpy(synthetic_col_field(wc * hc, 99)).cuda()
    prm = hm.slice_params(1, qp, HM_QP_FACTOR)
    poc = nref + 1
    prm.update(poc=poc, nref=[nref, 0], ref_poc=np.array([[poc - 1 - k for k in range(4)], [0] * 4]),
               ref_plane=np.array([list(range(nref)) + [0] * (4 - nref), [0] * 4]), max_merge=5, tmvp=1, check_ldc=1,
               col_from_l0=1, col_valid=1, col_poc=poc - 1, col_ref_poc=np.array([[poc - 2 - k for k in range(4)], [0] * 4]),
               search_range=64, amp=1)
    entry = _abi.load_ctx_init_states()[1, qp]
    pictures = []
    for c in range(chains):
        k = c % distinct
        pictures.append(hm.DevicePicture(frames[nref + k], [frames[nref + k - 1 - r] for r in range(nref)], prm, eb,
                                         col_field=col))
    eng = hm.Engine(pictures)
    n = wc * hc
    job_steps = [_chain_jobs([(c, pos, 1, 0, n - 1, pos > 0) for c in range(chains)], entry) for pos in range(warmup + steps)]
    sec, wall, _ = _time_chains(eng, job_steps, chains, warmup)
    del eng, pictures
    torch.cuda.empty_cache()
    return {"workload": "%d single-slice (SliceMode 0) 2160p P pictures, one chain each, QP %d, %d refs" % (chains, qp, nref),
            "ctus_per_s": round(chains / sec, 2), "ms_per_step": round(sec * 1e3, 1), "wall_ms_per_step": round(wall * 1e3, 1)}


# encoder_lowdelay_P_main.cfg:24-27: Frame1..4 QP offset and QPFactor; GOP position 4 has depth 0
LDP_GOP = {1: (3, 0.4624, 2), 2: (2, 0.4624, 1), 3: (3, 0.4624, 2), 4: (1, 0.578, 0)}
LDP_SAO_LAYER = {0: 0, 1: 2, 2: 1, 3: 2, 4: 0}


def closed_loop_geometry(W, H, rows, ctus_step):
    """The closed-loop figure's slicing: (CTUs per row, CTU rows, chains per picture, CTUs per chain).
    One chain per slice of `rows` CTU rows; a partial bottom row must share its slice with the row
    above (its picture-boundary CTUs read TEncSearch::m_integerMv2Nx2N as the CTU before them left it,
    DESIGN.md section 5)."""
    assert W % 64 == 0 and (H % 64 == 0 or rows >= 2), "a partial bottom row needs a slice of >= 2 rows"
    wc, hc = W // 64, (H + 63) // 64
    assert hc % rows == 0, "equal slices"
    nch, cl = hc // rows, rows * wc
    assert cl % ctus_step == 0, "whole launches per chain"
    return wc, hc, nch, cl


def closed_loop_specs(segs, nch, cl, launch, ctus_step):
    """_chain_jobs specs of launch `launch` of a closed-loop picture set: every segment's chains,
    `ctus_step` CTUs each from CTU launch * ctus_step of its slice, resumed after the first launch."""
    return [(s, c * cl + launch * ctus_step, ctus_step, c * cl, c * cl + cl - 1, launch > 0)
            for s in range(segs) for c in range(nch)]


def closed_loop_measure(W=1920, H=1088, segs=120, pics=3, base_qp=32, ctus_step=6, threads=16, parity=True, rows=1):
    """Side figure (config 5): closed LDP segments decided entirely on the device --
    `segs` segments in flight (W x H random 4:2:0 originals, `rows` CTU rows per slice, one chain
    per slice), each an I picture and then P pictures decided against references the device made
    (hvx_hm_compress -> hvx_hm_finish_picture: deblocking with device boundary strengths and the
    collocated motion field -> hm.sao_picture -> the padded reference planes), the LDP GOP's QP
    offsets / QPFactors / reference lists (encoder_lowdelay_P_main.cfg:24-27, first GOP).  Each
    picture's chains advance `ctus_step` CTUs per launch until their rows are done; then every
    segment's picture is finished into its next reference.  Reported: the P pictures' CTUs per second
    over their decision launches plus their loop filters / SAO / reference builds (wall clock), and a
    restatement parity sample: segment 0's last P picture re-decided by the restatement on 16 host
    threads against the device-made references and collocated field, every CTU compared."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    from video_codecs_amd import _abi, hm, synth
    wc, hc, nch, cl = closed_loop_geometry(W, H, rows, ctus_step)  # chains per picture, CTUs per chain
    n = wc * hc
    eb = _abi.load_entropy_bits()
    init = _abi.load_ctx_init_states()
    dbk = _abi.deblock_params(W, H)
    with ThreadPoolExecutor(8) as ex:
        orgs = list(ex.map(lambda i: synth.random_frame(W, H, 30000 + i), range(segs * pics)))
    org_frames = [hm.DeviceFrame(yuv_split(f, W, H)) for f in orgs]
    refs = [[] for _ in range(segs)]  # per segment: device-made reference frames, most recent first
    cols = [None] * segs
    rates = [np.zeros((3, 7)) for _ in range(segs)]
    stream = torch.cuda.Stream()
    out_ctu = torch.zeros(segs * nch * ctus_step * hm.HM_CTU.itemsize, dtype=torch.uint8, device="cuda")
    out_rec = torch.zeros(segs * nch * ctus_step * 6144, dtype=torch.uint8, device="cuda")
    per_pic, kept, last = [], {}, None
    t_p = 0.0
    for t in range(pics):
        if t == 0:
            qp, st_idx = base_qp, 2
            prm = hm.slice_params(2, qp, 0.57 * (1.0 - min(0.5, 0.05 * 3)), gop_depth=0)  # I: 0.57 * dLambda_scale
            prm.update(poc=0, nref=[0, 0], ref_poc=np.zeros((2, 4), int), ref_plane=np.zeros((2, 4), int), max_merge=5,
                       tmvp=1, check_ldc=1, col_from_l0=1, col_valid=0, col_poc=0, col_ref_poc=np.zeros((2, 4), int),
                       search_range=64, amp=1)
            col_nref = (0, 0)
        else:
            off, fac, depth = LDP_GOP[t]
            qp, st_idx = base_qp + off, 1
            nr = min(t, 4)
            prm = hm.slice_params(1, qp, fac, gop_depth=depth)
            prm.update(poc=t, nref=[nr, 0], ref_poc=np.array([[t - 1 - k if k < nr else 0 for k in range(4)], [0] * 4]),
                       ref_plane=np.array([[k if k < nr else 0 for k in range(4)], [0] * 4]), max_merge=5, tmvp=1,
                       check_ldc=1, col_from_l0=1, col_valid=1, col_poc=t - 1,
                       col_ref_poc=np.array([[t - 2 - k if k < min(t - 1, 4) else 0 for k in range(4)], [0] * 4]),
                       search_range=64, amp=1)
            col_nref = (min(t - 1, 4), 0)
        entry = init[st_idx, qp]
        col_read = cols[0]  # the collocated field segment 0's picture reads (the parity sample's)
        pictures = [hm.DevicePicture(org_frames[s * pics + t], refs[s][:4], prm, eb, col_field=cols[s]) for s in range(segs)]
        eng = hm.Engine(pictures)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        launch_s = 0.0
        with torch.cuda.stream(stream):
            for L in range(cl // ctus_step):
                specs = closed_loop_specs(segs, nch, cl, L, ctus_step)
                jt = torch.from_numpy(_chain_jobs(specs, entry).view(np.uint8).reshape(-1).copy()).cuda()
                e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                e[0].record()
                eng.launch(jt, len(specs), out_ctu, out_rec)
                e[1].record()
                e[1].synchronize()
                launch_s += e[0].elapsed_time(e[1]) * 1e-3
                if t == pics - 1 and parity:  # segment 0's chains (jobs 0 .. hc-1): the pre-loop-filter records
                    kept[L] = (out_ctu[:nch * ctus_step * hm.HM_CTU.itemsize].cpu().numpy().view(hm.HM_CTU).reshape(nch, ctus_step),
                               out_rec[:nch * ctus_step * 6144].cpu().numpy().reshape(nch, ctus_step, 6144))
                progress("closed loop: picture %d launch %d/%d %.1f s" % (t, L + 1, cl // ctus_step, e[0].elapsed_time(e[1]) * 1e-3))
            t1 = time.perf_counter()
            for s in range(segs):  # deblocking (device boundary strengths) and the collocated field
                _, cols[s] = hm.finish_picture(pictures[s], dbk, col_field=True)
            # SAO: every segment's decision in one launch (one wave per picture)
            sao = hm.sao_pictures(pictures, [LDP_SAO_LAYER[t]] * segs, rates, [int(prm["slice_type"])] * segs, [qp] * segs,
                                  sao_states=[(entry[hm.SAO_CTX_MERGE], entry[hm.SAO_CTX_TYPE])] * segs)
            for s in range(segs):  # the padded reference planes the next picture searches
                rates[s] = sao[s][0]
                ref = hm.DeviceFrame.blank(W, H)
                hm.finish_picture(pictures[s], None, ref_frame=ref)
                refs[s].insert(0, ref)
        stream.synchronize()
        t2 = time.perf_counter()
        per_pic.append({"poc": t, "slice": "I" if t == 0 else "P", "qp": qp, "decision_s": round(launch_s, 3),
                        "decision_wall_s": round(t1 - t0, 3), "loop_s": round(t2 - t1, 3),
                        "ctus_per_s": round(segs * n / (t2 - t0), 1)})
        progress("closed loop: picture %d done (%d CTUs, decision %.1f s, loop filters + SAO + references %.1f s)" % (
            t, segs * n, launch_s, t2 - t1))
        if t > 0:
            t_p += t2 - t0
        if t == pics - 1:
            last = (prm, qp, col_nref, entry, col_read)
        del eng
    res = {"workload": "%d closed LDP segments (I + %d P pictures, %dx%d random 4:2:0 originals, %d CTU row(s) per slice: "
                       "%d chains), every P picture decided against device-made references (deblocked + SAO) and the "
                       "device's collocated field; %d CTUs per chain per launch" % (segs, pics - 1, W, H, rows, segs * nch,
                                                                                   ctus_step),
           "ctus_per_s": round(segs * n * (pics - 1) / t_p, 2), "basis": "P pictures: decision launches + loop filters / "
           "SAO / reference builds, wall clock", "pictures": per_pic}
    if parity:
        import oracle  # noqa: F401  (test infrastructure: the checker)
        from oracle import hm_ctu
        prm, qp, col_nref, entry, col_read = last
        pi, pf = host_pic_arrays(W, H, prm, qp, col_nref=col_nref)
        ref_host = []
        for ref in refs[0][1:1 + prm["nref"][0]]:  # the references the last picture read (refs[0][0] is its own)
            y8, _, cb16, cr16 = (x.cpu().numpy() for x in ref.planes())
            m8 = hm.DeviceFrame.M8
            ref_host.append(np.concatenate([y8[m8:m8 + H, m8:m8 + W].reshape(-1), cb16[40:40 + H // 2, 40:40 + W // 2]
                                            .astype(np.uint8).reshape(-1), cr16[40:40 + H // 2, 40:40 + W // 2].astype(np.uint8).reshape(-1)]))
        col_host = col_read.cpu().numpy() if col_read is not None else None
        t0 = time.perf_counter()
        progress("closed loop: restatement parity (%d chains x %d CTUs)" % (nch, cl))
        port = hm_ctu.chains(pi, pf, orgs[pics - 1], np.concatenate(ref_host), entry, np.arange(nch, dtype=np.int32) * cl,
                             cl, cl, threads=threads, col_field=col_host)
        got = {}
        for L, (ct, rc) in kept.items():
            for k in range(nch):
                for i in range(ctus_step):
                    got[(k, L * ctus_step + i)] = (hm.unpack_parts(ct[k, i]["p"]), ct[k, i]["coef"], rc[k, i], ct[k, i]["cost"],
                                                  (ct[k, i]["bits"], ct[k, i]["dist"]))
        mism, first = _compare_port(port, got, [(k, i) for k in range(nch) for i in range(cl)])
        res.update(gpu_parity_ctus=nch * cl, gpu_parity_mismatches=mism, first_mismatches=first,
                   parity_s=round(time.perf_counter() - t0, 1))
    del pictures, refs, org_frames
    torch.cuda.empty_cache()
    return res


def hm_1080p_measure(pics=128, nref=4, base_qp=32, warmup=1, steps=10):
    """Side figure (BASELINE configs 2/3 size): the headline's decision on 1080p random 4:2:0 P
    pictures -- HmWorkload at 1920x1080, `pics` pictures x 16 chains (17 CTU rows, the partial 17th
    chained after the 16th) = 2048 chains, one CTU per chain per step."""
    import torch
    work = HmWorkload(1920, 1080, pics, nref, base_qp, 1, rank=0)
    out_rec = torch.zeros(work.slots * 6144, dtype=torch.uint8, device="cuda")
    for _ in range(warmup):
        work.step(out_rec)
    torch.cuda.synchronize()
    evs = []
    t0 = time.perf_counter()
    for _ in range(steps):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        work.step(out_rec, ev)
        evs.append(ev)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    sec = sum(a.elapsed_time(b) for a, b in evs) / steps * 1e-3
    n = work.n_jobs
    del work, out_rec
    torch.cuda.empty_cache()
    return {"workload": "%d 1080p P pictures x %d row-slice chains, QP %d, %d refs (HM-exact decision, as the headline)" % (
        pics, n // pics, base_qp + HM_QP_OFFSET, nref), "ctus_per_s": round(n / sec, 2), "ms_per_step": round(sec * 1e3, 1),
        "wall_ms_per_step": round(wall * 1e3, 1)}


def slice_writer_measure(work, done, cap=1 << 18):
    """Side figure: the slice data of the headline's decided CTUs written on the device
    (hvx_hm_write_slices: TEncSlice::encodeSlice's CTU loop, every CTU's CU syntax through
    TEncBinCABAC, one wave per slice) -- every chain's first `done` CTUs as one slice from the
    slice-start context states, all 2046 slices in one launch, timed with HIP events."""
    import torch
    from video_codecs_amd import hm
    wc = work.wc
    n = work.n_jobs
    out = torch.zeros(n * cap, dtype=torch.uint8, device="cuda")
    sl = np.zeros(n, hm.HM_SLICE)
    for p in range(work.pics):
        for r in range(work.rows):
            k = p * work.rows + r
            sl[k]["pic"], sl[k]["first_ctu"], sl[k]["n_ctus"], sl[k]["out_cap"] = p, r * wc, done, cap
            sl[k]["out"] = out.data_ptr() + k * cap
            sl[k]["entry"]["st"] = work.entry
    sl_t = torch.from_numpy(sl.view(np.uint8).reshape(-1).copy()).cuda()
    res_t = torch.zeros(n * hm.HM_SLICE_RESULT.itemsize, dtype=torch.uint8, device="cuda")
    ms = []
    with torch.cuda.stream(work.stream):
        for rep in range(3):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
            work.eng.write_slices_launch(sl_t, n, res_t)
            ev[1].record()
            ev[1].synchronize()
            ms.append(ev[0].elapsed_time(ev[1]))
    res = res_t.cpu().numpy().view(hm.HM_SLICE_RESULT)
    assert (res["status"] == 0).all() and (res["n_bytes"] <= cap).all(), "hvx_hm_write_slices refused a slice"
    t = min(ms) * 1e-3
    nbytes = int(res["n_bytes"].sum())
    return {"workload": "%d slices x %d decided CTUs of the headline's pictures (CU syntax + coefficients through "
                        "TEncBinCABAC, no SAO), one launch, best of 3" % (n, done),
            "ctus_per_s": round(n * done / t, 1), "launch_ms": round(t * 1e3, 2), "bytes": nbytes,
            "bits_per_ctu": round(8.0 * nbytes / (n * done), 1), "bins_per_ctu": round(float(res["bins"].sum()) / (n * done), 1)}


def _kept_records(work, positions):
    """The GPU's records of picture 0's chains from HmWorkload.keep_steps: {(chain, position):
    (parts, coef, recon, cost, (bits, dist))} for the chain positions in `positions` (first pass)."""
    from video_codecs_amd import hm
    got = {}
    for pos, ct, rc in work.keep_steps:
        c = ct.cpu().numpy().view(hm.HM_CTU).reshape(work.rows, work.ctus)
        r = rc.cpu().numpy().reshape(work.rows, work.ctus, 6144)
        for k in range(work.rows):
            for i in range(work.ctus):
                key = (k, pos + i)
                if pos + i in positions[k] and key not in got:
                    got[key] = (hm.unpack_parts(c[k, i]["p"]), c[k, i]["coef"], r[k, i], c[k, i]["cost"],
                                (c[k, i]["bits"], c[k, i]["dist"]))
    return got


def _compare_port(port, got, order):
    recs = [got[key] for key in order]
    return compare_chain_ctus(port, np.stack([g[0] for g in recs]), np.stack([g[1] for g in recs]),
                              np.stack([g[2] for g in recs]), np.array([g[3] for g in recs]),
                              np.array([g[4] for g in recs], np.uint32))


def hm_cpu_port(work, threads):
    """The oracle's restatement (oracle/hvx_oracle_cu.c hvxo_hm_chains) on picture 0's slice
    chains -- the same CTUs the GPU decided in its warmup + timed steps, on `threads` host threads
    -- and the bit-exact comparison of every one of them with the GPU's records."""
    import oracle  # noqa: F401  (test infrastructure: the checker and the port baseline)
    from oracle import hm_ctu
    pi, pf, org, refs, col = work.host_inputs(0)
    wc, hc = work.wc, work.rows  # the picture's chains (the last may continue into the partial bottom row)
    done = min(work.step_idx * work.ctus, wc)  # CTUs of each row decided by the GPU (first pass)
    chain_first = np.arange(hc, dtype=np.int32) * wc
    hm_ctu.chains(pi, pf, org, refs, work.entry, chain_first[:1], 1, wc, threads=1, col_field=col)  # tables
    t0 = time.perf_counter()
    out = hm_ctu.chains(pi, pf, org, refs, work.entry, chain_first, done, wc, threads=threads, col_field=col)
    dt = time.perf_counter() - t0
    n = hc * done
    got = _kept_records(work, [set(range(done))] * hc)
    mism, first = _compare_port(out, got, [(k, i) for k in range(hc) for i in range(done)])
    return {"value": round(n / dt, 3), "unit": "CTUs/s", "cores": threads, "kind": "port",
            "sample": f"picture 0's {hc} slice chains x {done} CTUs ({n} CTUs) through oracle/hvx_oracle_cu.c "
                      f"hvxo_hm_chains on {threads} host threads, {dt:.1f} s",
            "gpu_parity_ctus": n, "gpu_parity_mismatches": mism, "first_mismatches": first}


def hm_merged_chain_parity(threads, W=256, H=176, nref=4, base_qp=32):
    """The headline's chain layout to the end of a picture, which its timed window does not reach:
    a small picture (W/64 CTUs per row, a 48-line partial bottom row) stepped by HmWorkload until
    every chain is done -- the full rows, and the last full row's chain continuing into the partial
    row through HVX_HM_SLICE_CTUS + HVX_HM_RESUME -- every CTU compared with the restatement."""
    import torch
    from oracle import hm_ctu
    work = HmWorkload(W, H, 1, nref, base_qp, 1, rank=0)
    out_rec = torch.zeros(work.slots * 6144, dtype=torch.uint8, device="cuda")
    for _ in range(2 * work.wc):
        work.step(out_rec)
    torch.cuda.synchronize()
    pi, pf, org, refs, col = work.host_inputs(0)
    wc, rows = work.wc, work.rows
    full = hm_ctu.chains(pi, pf, org, refs, work.entry, np.arange(rows - 1, dtype=np.int32) * wc, wc, wc, threads=threads,
                         col_field=col)
    last = hm_ctu.chains(pi, pf, org, refs, work.entry, np.array([(rows - 1) * wc], np.int32), 2 * wc, wc, threads=1,
                         col_field=col)
    port = {k: np.concatenate([full[k], last[k]]) for k in full}
    positions = [set(range(wc))] * (rows - 1) + [set(range(2 * wc))]
    got = _kept_records(work, positions)
    order = [(k, i) for k in range(rows - 1) for i in range(wc)] + [(rows - 1, i) for i in range(2 * wc)]
    mism, first = _compare_port(port, got, order)
    del work, out_rec
    torch.cuda.empty_cache()
    return {"picture": f"{W}x{H}", "chains": rows, "ctus": len(order), "partial_row_ctus": wc,
            "gpu_parity_mismatches": mism, "first_mismatches": first}


def physical_cores():
    """Physical cores of the host (unique (physical id, core id) pairs of /proc/cpuinfo)."""
    cores, phys, core = set(), None, None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                core = line.split(":", 1)[1].strip()
            elif not line.strip() and phys is not None and core is not None:
                cores.add((phys, core))
                phys = core = None
        if phys is not None and core is not None:
            cores.add((phys, core))
    except OSError:
        pass
    return len(cores) or (os.cpu_count() or 1)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


REF_W, REF_H, REF_FRAMES, REF_POCS = 512, 256, 7, (5, 6)


def hm_cpu_reference(procs, tmpdir):
    """HM-16.5rc1's own encoder (oracle/_ref/TAppEncoder_cutime: the unchanged TAppEncoder with
    every TEncCu::compressCtu timed, oracle/cu_timer.cpp) on the host cores, on the GPU's workload:
    `procs` concurrent single-threaded encodes of 512x256 random 4:2:0 YUV (the bench's synthetic
    recipe; 8x4 whole CTUs) with oracle/hm_ref_bench.cfg and one row per slice (SliceArgument 8):
    P pictures predicted from the 4 previous frames at the bench picture's slice parameters (QP 34,
    QPFactor 0.4624, GOP depth > 0: the same lambda), TZ SR 64, RDOQ, AMP, FEN.  The timed pictures
    are POC 5 and 6 (4 active references each; POCs 0-4 are the pre-roll); their compressCtu time
    is summed per encode.  value = procs / mean seconds per CTU."""
    import subprocess
    from video_codecs_amd import synth
    exe = os.path.join(ROOT, "oracle", "_ref", "TAppEncoder_cutime")
    cfg = os.path.join(ROOT, "oracle", "hm_ref_bench.cfg")
    if not os.path.exists(exe):
        return None
    per_ctu = []
    t0 = time.perf_counter()
    ps = []
    for k in range(procs):
        yuv = os.path.join(tmpdir, f"hvx_hm_ref{k}.yuv")
        with open(yuv, "wb") as f:
            for i in range(REF_FRAMES):
                f.write(synth.random_frame(REF_W, REF_H, 5000 + 100 * k + i).tobytes())
        ps.append(subprocess.Popen([exe, "-c", cfg, "-i", yuv, "-wdt", str(REF_W), "-hgt", str(REF_H), "-fr", "30",
                                    "-f", str(REF_FRAMES), "--SliceArgument=%d" % (REF_W // 64),
                                    "-b", os.path.join(tmpdir, f"hvx_hm_ref{k}.bin"), "-o", "/dev/null"],
                                   stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True))
    for p in ps:
        _, err = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("TAppEncoder_cutime failed: " + err[-500:])
        secs = ctus = 0
        for line in err.splitlines():
            f = line.split()
            if len(f) == 13 and f[0] == "cu_time" and int(f[2]) in REF_POCS:
                assert int(f[4]) == 1 and int(f[6]) == 34 and int(f[8]) == 4, line  # P, QP 34, 4 refs
                ctus += int(f[10])
                secs += float(f[12])
        per_ctu.append(secs / ctus)
    wall = time.perf_counter() - t0
    s = float(np.mean(per_ctu))
    return {"value": round(procs / s, 3), "unit": "CTUs/s", "cores": procs, "kind": "reference",
            "sample": f"{procs} concurrent HM-16.5rc1 TAppEncoder encodes (oracle/_ref/TAppEncoder_cutime, compressCtu "
                      f"timed) of {REF_W}x{REF_H} random YUV, oracle/hm_ref_bench.cfg with one row per slice: POC "
                      f"{REF_POCS[0]}-{REF_POCS[-1]} ({len(REF_POCS) * (REF_W // 64) * (REF_H // 64)} whole CTUs per "
                      f"encode, P, QP 34, 4 refs) after a 5-frame pre-roll; {wall:.0f} s wall",
            "s_per_ctu_per_core": round(s, 4), "cpu_model": cpu_model(), "cores_present": os.cpu_count(),
            # the whole host at the measured per-core rate (an estimate: the job's CPU share is 16 threads,
            # so all physical cores are not run here; shared caches / memory bandwidth are not modelled)
            "whole_host_estimate": {"physical_cores": physical_cores(),
                                    "ctus_per_s": round(physical_cores() / s, 1),
                                    "basis": "physical_cores / s_per_ctu_per_core"}}


def build_provenance():
    """The libhvx.so this run loaded against the sources in the tree: the stamp build_hip()
    wrote (source digest + library sha256) re-checked here (fresh = the library was built from
    exactly these sources and is the file that was stamped)."""
    import hashlib
    import __graft_entry__ as ge
    from video_codecs_amd import hvx
    lib = hvx.LIB_PATH
    rec = {"lib": os.path.relpath(lib, ROOT), "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]}
    stamp_path = os.path.join(ROOT, "video_codecs_amd", "libhvx.build.json")
    if os.path.exists(stamp_path):
        st = json.load(open(stamp_path))
        rec["built_utc"] = st.get("built_utc")
        rec["fresh"] = st.get("source_digest") == ge.source_digest() and \
            st.get("lib_sha256", "")[:16] == rec["lib_sha256"]
    else:
        rec["fresh"] = None
    return rec


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
    from video_codecs_amd import hvx
    from video_codecs_amd.dpb import DpbGather

    W, H, nref = args.width, args.height, args.nref
    hvx.context()
    work = HmWorkload(W, H, args.pics, nref, args.qp, args.ctus, rank)
    dpb = DpbGather(world, rank, (work.slots * 6144,), "cuda")
    events = []

    def step():
        ev = None
        if timing[0]:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            events.append(ev)
        with torch.cuda.stream(work.stream):  # the gather reads what this step's launch wrote
            work.step(dpb.buffer(), ev)
            dpb.send()
        if rank == 0:  # a progress line per launch queued (the queue runs at most a step or two ahead)
            progress("headline step %d queued" % work.step_idx)

    def sync():
        dpb.drain()
        torch.cuda.synchronize()

    timing = [False]
    elapsed = timed_steps(step, args.steps, args.warmup, world, "cuda", sync,
                          before=lambda: timing.__setitem__(0, True))
    timing[0] = False
    launch_ms = sum(a.elapsed_time(b) for a, b in events) / max(1, len(events))
    own, gathered = dpb.last()
    dpb_ok = None
    if gathered is not None:
        dpb_ok = bool(torch.equal(gathered[0], own))
    if rank == 0:
        units = work.n_jobs * args.ctus
        value = aggregate(units, args.steps, world, elapsed)
        bpc = b_ctu(nref)
        bytes_per_launch = bpc * units
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        traffic = None
        tr_path = os.path.join(ROOT, "profiles", "hbm_traffic_r05.json")  # PMC passes of this round's tree
        if os.path.exists(tr_path):
            tr = json.load(open(tr_path)).get("k_hm_compress")
            if tr:
                traffic = tr["bytes_per_launch"] * units / tr.get("ctus_per_launch", units)
        # the engine's real limiter, from the SQ counter passes of the same kernel on this round's
        # tree (scripts/gpu_hm_pmc.sh + scripts/hm_pmc_summary.py): issue fractions of the SIMDs
        issue = {}
        pmc_path = os.path.join(ROOT, "profiles", "hm_pmc_r05.json")
        if os.path.exists(pmc_path):
            pm = json.load(open(pmc_path))
            issue = {"simd_issue_frac": pm["simd_issue_frac"], "valu_frac": pm["valu_frac"],
                     "wave_cycle_split": pm["wave_cycle_split"], "pmc_file": "profiles/hm_pmc_r05.json"}
        out = {
            "metric": METRIC,
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
            "data": "synthetic: splitmix64 uniform random 8-bit 4:2:0 YUV (BASELINE.md sec. 3), the previous 4 frames "
                    "as references, seeded synthetic collocated motion field; own pictures per rank",
            "config": {"workload": "HM-16.5rc1 TEncCu::compressCtu + encodeCtu, bit-exact: merge/skip, AMVP+TMVP, TZ "
                                   "SR64 + frac ME vs %d refs, 2NxN/Nx2N/AMP, RQT + RDOQ + transform skip, "
                                   "intra-in-inter, CABAC context carry; SliceMode=1 row slices" % nref,
                       "resolution": f"{W}x{H}", "ctus_per_frame": work.wc * work.hc, "pictures_per_gpu": args.pics,
                       "slice_chains_per_gpu": work.n_jobs, "ctus_per_chain_per_step": args.ctus,
                       "slice": "P, QP %d (base %d + GOP offset %d), QPFactor %g, lambda %.6f" % (
                           work.qp, args.qp, HM_QP_OFFSET, HM_QP_FACTOR, work.params["lambda"]),
                       "n_ref": nref, "parallelism": f"pictures x{world}",
                       "dpb": "gather of every rank's reconstructed CTUs to rank 0 per step" if world > 1 else "local"},
            # priced against HBM (integer work); the limiter is the serial RD decision
            # chain inside each wave (latency), not bandwidth -- frac << 1
            "roofline": {"bound": "hbm", "limiter": "instruction latency of the serial decision chain (issue + "
                                                    "dependency waits; see simd_issue_frac / wave_cycle_split)",
                         "kernel": "k_hm_compress",
                         "achieved": round(achieved, 4), "peak": MI355X_HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / MI355X_HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_launch": bytes_per_launch, "avg_launch_ms": round(launch_ms, 3), "b_ctu": bpc,
                         **issue},
            "cpu_baseline": None,
        }
        if dpb_ok is not None:
            out["dpb_gather_ok"] = dpb_ok
        out["build"] = build_provenance()
        if world == 1:
            threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)))
            if not args.no_cpu_ref:
                progress("reference HM on the host cores")
                try:
                    out["cpu_baseline"] = hm_cpu_reference(args.cpu_ref_procs or threads,
                                                           os.environ.get("TMPDIR", "/tmp"))
                except Exception as e:  # noqa: BLE001  (the port figure below stands in)
                    progress("reference HM timing failed: %s: %s" % (type(e).__name__, e))
            def side(key, what, fn):
                # a side figure that raises is reported as such; the headline line is never lost
                progress(what)
                try:
                    out[key] = fn()
                except Exception as e:  # noqa: BLE001
                    out[key] = {"error": "%s: %s" % (type(e).__name__, e)}
                    progress("%s failed: %s" % (what, out[key]["error"]))

            side("slice_writer", "slice writer side figure", lambda: slice_writer_measure(work, args.warmup + args.steps))
            if not args.no_cpu:
                def port_figure():
                    progress("restatement parity of the headline's CTUs")
                    port = hm_cpu_port(work, threads)
                    progress("merged bottom chain parity")
                    port["merged_chain"] = hm_merged_chain_parity(threads)
                    return port
                side("cpu_port", "the restatement's port figure", port_figure)
                if out["cpu_baseline"] is None and "error" not in out["cpu_port"]:
                    out["cpu_baseline"] = out["cpu_port"]
            del work, dpb
            torch.cuda.empty_cache()
            if not args.no_ra:
                side("config4_ra_ssim", "config 4 (RA, stVSSIM cost)", lambda: ra_ssim_measure(W, H))
            if not args.no_slice0:
                side("slice_mode0", "SliceMode 0 side figure", lambda: slice_mode0_measure(W, H))
            if not args.no_1080p:
                side("hm_1080p", "1080p side figure", hm_1080p_measure)
            if not args.no_closed:
                side("closed_loop", "closed-loop LDP segments (config 5)",
                     lambda: closed_loop_measure(threads=threads, parity=not args.no_cpu))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
