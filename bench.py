#!/usr/bin/env python3
"""Benchmark: 64x64 CTUs/s of HM-16.5rc1's CU mode decision on 2160p random YUV, bit-exact vs HM.

N = 1 (the headline, `--workload steady`): one step = one launch of hvx_hm_compress (include/hvx.h)
over every SliceMode=1 slice of P pictures in flight: a 3840x2160 4:2:0 picture has 34 CTU rows
(33 slice chains: the partial bottom row continues the chain above it); with 62 pictures per GPU
that is 2046 slice chains, one wave each, and a step advances every chain by --ctus CTUs (default 1),
each CTU TEncCu::compressCtu + encodeCtu exactly as HM decides it: merge/skip, AMVP + TZ search +
fractional refinement against 4 references, 2NxN/Nx2N/AMP, the RQT with RDOQ and transform skip,
intra-in-inter, the CABAC context carry.  The chains' CABAC state and CTU data
stay in HBM between steps (HVX_HM_RESUME).  Inputs are resident in HBM before timing starts; each
picture's reference frames are the previous synthetic frames.

N > 1 (torch.distributed.run; `--workload closed`, BASELINE config 5): one rank per GPU, each rank
encodes its own closed LDP GOP segments (gop.ClosedSegments: disjoint frame indices, references made
by each segment's own loop on the device); after every picture each rank's finished (deblocked + SAO)
pictures are gathered to rank 0's shared DPB (video_codecs_amd/dpb.py, RCCL over xGMI, asynchronous,
double-buffered); weak scaling.  The same per-GPU workload at N = 1 is the N = 1 line's
`config5_closed_segments` figure.

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
    p.add_argument("--workload", choices=("auto", "steady", "closed"), default="auto",
                   help="steady: the 2160p steady-state P pictures (the N=1 headline); closed: BASELINE config 5 -- "
                        "closed LDP segments per rank with the DPB gather of finished pictures (the N>1 default)")
    p.add_argument("--pics", type=int, default=62, help="steady: P pictures in flight per GPU (33 slice chains each at "
                                                        "2160p: 62 -> 2046 chains, two waves per SIMD)")
    p.add_argument("--ctus", type=int, default=1, help="steady: CTUs each slice chain advances per step")
    p.add_argument("--segs", type=int, default=120, help="closed: segments per GPU (17 row-slice chains each at 1088p)")
    p.add_argument("--closed-ctus", type=int, default=6, help="closed: CTUs each chain advances per step (launch)")
    p.add_argument("--cpu-ref-procs", type=int, default=0, help="HM TAppEncoder processes for the reference "
                                                                  "baseline (0: the host's CPU share)")
    p.add_argument("--no-cpu-ref", action="store_true", help="skip the reference HM timing")
    p.add_argument("--no-ra", action="store_true", help="skip the config-4 side figure (closed RA segments, stVSSIM cost)")
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--nref", type=int, default=4)
    p.add_argument("--qp", type=int, default=32)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-1080p", action="store_true", help="skip the 1080p side measurement")
    p.add_argument("--no-closed", action="store_true", help="skip the config-5 side figure (closed LDP segments: "
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
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if dist.get_backend() != "gloo" else "cpu")
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
    from video_codecs_amd import gop
    return gop.host_pic_arrays(W, H, prm, qp, col_nref)


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


def closed_seed(rank, segs, s, poc):
    """The synthetic frame index of segment s's picture `poc` on `rank`: disjoint across segments and
    ranks (BASELINE.md sec. 3 recipe, synth.random_frame)."""
    return 30000 + (rank * segs + s) * 64 + poc


class ClosedWorkload:
    """Closed GOP segments on one GPU (BASELINE config 5's unit; config 4 with the stVSSIM cost):
    `len(base_qps)` segments of W x H random 4:2:0 originals made on the device (synth.random_frame_torch,
    frame indices closed_seed: distinct per segment and rank), the first `n_pics` pictures of HM's
    `kind` ('ldp' / 'ra') segment structure, every picture decided by hvx_hm_compress against the
    references its own segment's loop made on the device (video_codecs_amd/gop.py ClosedSegments:
    deblocking + SAO + slice writer + cabac_init choice + padded references), chains of `rows` CTU rows
    stepping `ctus_step` CTUs per launch.  dpb: a DpbGather -- after every picture each segment's
    finished (deblocked + SAO) reconstruction is gathered to rank 0.  One step() = one launch (and, after
    a picture's last launch, its loop)."""

    def __init__(self, W, H, base_qps, n_pics, rank, kind="ldp", rows=1, ctus_step=6, rd_metric=0, dpb=None,
                 device="cuda", segments_cls=None):
        import torch
        from video_codecs_amd import gop, synth
        self.W, self.H, self.rank, self.kind = W, H, rank, kind
        segs = len(base_qps)
        self.plan = gop.load_plan(kind, n_pics)
        self.frames = {}
        for s in range(segs):
            for g in self.plan:
                f = synth.random_frame_torch(W, H, closed_seed(rank, segs, s, g.poc), device)
                ysz, csz = W * H, W * H // 4
                self.frames[(s, g.poc)] = (f[:ysz].view(H, W), f[ysz:ysz + csz].view(H // 2, W // 2),
                                           f[ysz + csz:].view(H // 2, W // 2))
        self.dpb, self.gathered = dpb, []
        self.cs = (segments_cls or gop.ClosedSegments)(
            self.plan, W, H, list(base_qps), lambda s, poc: self.frames[(s, poc)], rows=rows, ctus_step=ctus_step,
            rd_metric=rd_metric, on_finished=self._finished if dpb is not None else None, device=device)
        self.cs.launch_events = []
        self.stream = torch.cuda.Stream() if device != "cpu" else None
        self.units_per_step = segs * self.cs.nch * self.cs.ctus_step
        if device != "cpu":
            torch.cuda.synchronize()

    def _finished(self, t, recs):
        """The DPB gather of picture t: every segment's final reconstruction into the rank's send buffer,
        then one asynchronous gather to rank 0 (video_codecs_amd/dpb.py)."""
        buf = self.dpb.buffer()
        W, H = self.W, self.H
        psz, ysz, csz = W * H * 3 // 2, W * H, W * H // 4
        for s, (y, cb, cr) in enumerate(recs):
            o = s * psz
            buf[o:o + ysz].copy_(y.reshape(-1))
            buf[o + ysz:o + ysz + csz].copy_(cb.reshape(-1))
            buf[o + ysz + csz:o + psz].copy_(cr.reshape(-1))
        self.dpb.send()
        self.gathered.append(t)

    def step(self):
        import contextlib
        import torch
        with torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext():
            self.cs.step()

    def launch_seconds(self, first=0):
        """(seconds, CTUs, algorithmic bytes) of the decision launches from launch `first` on (HIP events)."""
        from video_codecs_amd import gop
        sec = ctus = byt = 0
        for t, n, (a, b) in self.cs.launch_events[first:]:
            sec += a.elapsed_time(b) * 1e-3
            ctus += n
            g = self.plan[t]
            byt += n * b_ctu(len(g.ref_pocs()) if g.slice_type != gop.I_SLICE else 0)
        return sec, ctus, byt

    def workload(self):
        cs = self.cs
        cost = ""
        if cs.rd_metric == _abi_mod().RD_STVSSIM:
            cost = ("; cost: the stvssim encoder's distortionstVSSIM over each segment's own device history (its "
                    "originals and final reconstructions in coding order)")
        return ("%d closed %s segments (HM's %s structure: %s; %dx%d random 4:2:0 originals, %d CTU row(s) per slice: "
                "%d chains) decided entirely on the device: every picture against the references its own segment's "
                "loop made (deblocking + SAO + slice writer + cabac_init choice), %d CTUs per chain per launch%s" % (
                    len(cs.segs), self.kind.upper(), "encoder_lowdelay_P_main" if self.kind == "ldp" else
                    "encoder_randomaccess_main", "POC " + ",".join(str(g.poc) for g in self.plan), self.W, self.H,
                    cs.rows, len(cs.segs) * cs.nch, cs.ctus_step, cost))


def _abi_mod():
    from video_codecs_amd import _abi
    return _abi


class ClosedParity:
    """A restatement parity sample of a ClosedWorkload: segment `seg`'s picture `t` -- its inputs (the
    device-made references, collocated field, history, slice parameters) captured when the picture is set
    up, the device's CTU records of `chains` captured after each launch -- re-decided by
    oracle/hvx_oracle_cu.c after the run (test infrastructure: the checker, outside any timed region)."""

    def __init__(self, work, t, seg, chains):
        self.work, self.t, self.seg, self.chains = work, t, seg, chains
        self.inputs, self.got = None, {}
        cs = work.cs
        begin, after = cs.begin, cs.after_launch

        def hooked_begin():
            begin()
            if cs.t == self.t:
                self._capture_inputs()

        def hooked_after(L):
            after(L)
            if cs.t == self.t:
                from video_codecs_amd import hm
                ct = cs.out_ctu.cpu().numpy().view(hm.HM_CTU)
                rc = cs.out_rec.cpu().numpy().reshape(-1, 6144)
                for c in self.chains:
                    k = self.seg * cs.nch + c
                    for i in range(cs.ctus_step):
                        self.got[(c, L * cs.ctus_step + i)] = (ct[k * cs.ctus_step + i], rc[k * cs.ctus_step + i])
        cs.begin, cs.after_launch = hooked_begin, hooked_after

    def _capture_inputs(self):
        from video_codecs_amd import _abi, gop, hm
        cs, s, W, H = self.work.cs, self.seg, self.work.W, self.work.H
        prm, qp, entry, table, planes, col_nref = cs.picture_params(s, self.t)
        seg = cs.segs[s]
        refs = []
        m8 = hm.DeviceFrame.M8
        for p in planes:
            y8, _, cb16, cr16 = (x.cpu().numpy() for x in seg.dpb[p].planes())
            refs.append(np.concatenate([y8[m8:m8 + H, m8:m8 + W].reshape(-1), cb16[40:40 + H // 2, 40:40 + W // 2]
                                        .astype(np.uint8).reshape(-1), cr16[40:40 + H // 2, 40:40 + W // 2].astype(np.uint8).reshape(-1)]))
        g = self.work.plan[self.t]
        col = seg.cols[g.col_poc].cpu().numpy() if g.col_poc is not None else None
        stv = None
        if cs.rd_metric == _abi.RD_STVSSIM:
            stv = ([tuple(x.cpu().numpy() for x in fr) for fr in seg.hist[:_abi.STV_HIST]], gop.stv_direction_map(col, W, H))
        org = np.concatenate([x.cpu().numpy().reshape(-1) for x in self.work.frames[(s, g.poc)]])
        self.inputs = (prm, qp, entry, col_nref, refs, col, stv, org)

    def check(self, threads):
        """Re-decide the sampled chains on the host and compare every CTU: (ctus, mismatches, first, seconds)."""
        import oracle  # noqa: F401  (test infrastructure: the checker, after the timing)
        from oracle import hm_ctu
        from video_codecs_amd import gop
        prm, qp, entry, col_nref, refs, col, stv, org = self.inputs
        cs, W, H = self.work.cs, self.work.W, self.work.H
        pi, pf = gop.host_pic_arrays(W, H, prm, qp, col_nref=col_nref)
        t0 = time.perf_counter()
        port = hm_ctu.chains(pi, pf, org, np.concatenate(refs) if refs else np.zeros(1, np.uint8), entry,
                             np.array(self.chains, np.int32) * cs.cl, cs.cl, cs.cl, threads=threads, col_field=col,
                             rd_metric=prm.get("rd_metric", 0), lambda_ssim=prm.get("lambda_ssim", 0.0), stv=stv)
        from video_codecs_amd import hm
        got = {k: (hm.unpack_parts(v[0]["p"]), v[0]["coef"], v[1], v[0]["cost"], (v[0]["bits"], v[0]["dist"]))
               for k, v in self.got.items()}
        order = [(c, i) for c in self.chains for i in range(cs.cl)]
        mism, first = _compare_port(port, got, order)
        return len(order), mism, first, round(time.perf_counter() - t0, 1)


def closed_figure(work, threads, parity=None, first_timed_pic=1):
    """Run every launch of a ClosedWorkload; report the pictures from `first_timed_pic` on (decision
    launches by HIP events + their loops, wall clock) and the parity samples."""
    import torch
    t_run = 0.0
    per_pic = []
    nl = work.cs.launches
    for t in range(len(work.plan)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(nl):
            work.step()
            progress("closed %s: picture %d (POC %d) launch %d/%d" % (work.kind, t, work.plan[t].poc, work.cs.L or nl, nl))
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        sec = sum(a.elapsed_time(b) * 1e-3 for tt, _, (a, b) in work.cs.launch_events if tt == t)
        log = work.cs.log[t]
        n = len(work.cs.segs) * work.cs.nch * work.cs.cl
        per_pic.append(dict(log, decision_s=round(sec, 3), wall_s=round(wall, 3), ctus=n, ctus_per_s=round(n / wall, 1)))
        if t >= first_timed_pic:
            t_run += wall
    n_timed = sum(p["ctus"] for p in per_pic[first_timed_pic:])
    res = {"workload": work.workload(), "ctus_per_s": round(n_timed / t_run, 2) if t_run else None,
           "basis": "pictures %s: decision launches + loop filters / SAO / slice writer / reference builds, wall clock" % (
               ",".join(str(p["poc"]) for p in per_pic[first_timed_pic:])), "pictures": per_pic}
    for key, par in (parity or {}).items():
        progress("closed %s: restatement parity %s" % (work.kind, key))
        n, mism, first, secs = par.check(threads)
        res.setdefault("parity", {})[key] = {"ctus": n, "mismatches": mism, "first_mismatches": first, "seconds": secs}
    return res


def config5_measure(threads, W=1920, H=1088, segs=120, pics=3, base_qp=32, ctus_step=6, parity=True):
    """Side figure, BASELINE config 5's unit on one GPU: the same ClosedWorkload the multi-GPU bench times
    per rank (LDP, 120 segments of 1920x1088, I + P pictures); parity: segment 0's last picture."""
    work = ClosedWorkload(W, H, [base_qp] * segs, pics, rank=0, kind="ldp", ctus_step=ctus_step)
    par = {"seg0_poc%d" % work.plan[-1].poc: ClosedParity(work, pics - 1, 0, list(range(work.cs.nch)))} if parity else None
    res = closed_figure(work, threads, par)
    del work
    return res


def config4_measure(threads, W=1920, H=1088, segs_per_qp=30, qps=(22, 27, 32, 37), pics=3, ctus_step=6, parity=True,
                    rows=1):
    """Side figure, BASELINE config 4 as an encode: closed random-access segments (HM's
    encoder_randomaccess_main structure: I, then POC 8, 4, ... of the first GOP8) decided with the
    stvssim encoder's active cost (HVX_RD_STVSSIM: distortionstVSSIM over the segment's own history of
    originals and final reconstructions in coding order, lambda_2(QP) * eta^0.85 with eta 1), the four
    base QPs' segments side by side in the same launches; per QP a restatement parity sample of its first
    segment's last picture (3 of its slice chains)."""
    from video_codecs_amd import _abi
    base = [q for q in qps for _ in range(segs_per_qp)]
    work = ClosedWorkload(W, H, base, pics, rank=0, kind="ra", rows=rows, ctus_step=ctus_step, rd_metric=_abi.RD_STVSSIM)
    nch = work.cs.nch
    par = {"qp%d" % q: ClosedParity(work, pics - 1, k * segs_per_qp, sorted({0, nch // 2, nch - 1}))
           for k, q in enumerate(qps)} if parity else None
    res = closed_figure(work, threads, par)
    # per base QP: the B pictures' rate (every segment of one QP decides the same CTUs per picture)
    res["rd_metric"] = "HVX_RD_STVSSIM"
    res["history_pictures"] = [min(t, _abi.STV_HIST) for t in range(pics)]
    del work
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


def closed_main(args, rank, world, device="cuda", segments_cls=None, size=(1920, 1088)):
    """The closed-segment workload timed by the contract (BASELINE config 5; the N>1 default): every rank
    encodes its own `segs` closed LDP segments of 1920x1088 random originals (ClosedWorkload, frame
    indices disjoint across ranks), one step = one decision launch (`closed_ctus` CTUs per chain, the
    picture's loop after its last launch), and after every picture each segment's finished picture is
    gathered to rank 0's DPB over RCCL.  W warmup steps, K timed steps, max over ranks; value = the CTUs
    all ranks decided in the timed steps / that time (weak scaling)."""
    import math
    import torch
    from video_codecs_amd.dpb import DpbGather
    (W, H), segs = size, args.segs
    launches = W // 64 // args.closed_ctus  # one CTU row per slice: launches per picture
    n_pics = math.ceil((args.warmup + args.steps) / launches) + 1
    dpb = DpbGather(world, rank, (segs * W * H * 3 // 2,), device)
    work = ClosedWorkload(W, H, [args.qp] * segs, n_pics, rank, kind="ldp", ctus_step=args.closed_ctus, dpb=dpb,
                          device=device, segments_cls=segments_cls)
    marks = {}

    def sync():
        if device != "cpu":
            torch.cuda.synchronize()
        dpb.drain()
        if device != "cpu":
            torch.cuda.synchronize()

    def step():
        work.step()
        if rank == 0:
            progress("closed step %d (picture %d launch %d/%d)" % (len(work.cs.launch_events), work.cs.t - (work.cs.L == 0),
                                                                    work.cs.L or launches, launches))
    elapsed = timed_steps(step, args.steps, args.warmup, world, device, sync,
                          before=lambda: marks.__setitem__("first", len(work.cs.launch_events)))
    sec, ctus, byt = work.launch_seconds(marks["first"])
    # per picture of the timed launches: the decision launches' HIP-event time and CTUs (rank 0's)
    per = {}
    for t, n, (a, b) in work.cs.launch_events[marks["first"]:]:
        d = per.setdefault(t, [0, 0.0, 0])
        d[0] += 1
        d[1] += a.elapsed_time(b) * 1e-3
        d[2] += n
    work.timed_pictures = [{"poc": work.plan[t].poc, "slice": "IPB"[(2, 1, 0).index(work.plan[t].slice_type)],
                            "refs": len(work.plan[t].ref_pocs()), "launches": d[0], "ctus": d[2],
                            "decision_s": round(d[1], 3), "decision_ctus_per_s": round(d[2] / d[1], 1)}
                           for t, d in sorted(per.items())]
    own, gathered = dpb.last()
    dpb_ok = bool(torch.equal(gathered[0], own)) if gathered is not None else None
    return work, elapsed, sec, ctus, byt, dpb_ok, len(work.gathered)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # RCCL over xGMI; HVX_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU
        dist.init_process_group(os.environ.get("HVX_DIST_BACKEND", "nccl"), init_method="env://")
    torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    from video_codecs_amd import hvx
    hvx.context()
    kind = args.workload if args.workload != "auto" else ("closed" if world > 1 else "steady")
    W, H, nref = args.width, args.height, args.nref
    if kind == "steady":
        work = HmWorkload(W, H, args.pics, nref, args.qp, args.ctus, rank)
        out_rec = torch.zeros(work.slots * 6144, dtype=torch.uint8, device="cuda")
        events = []

        def step():
            ev = None
            if timing[0]:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                events.append(ev)
            work.step(out_rec, ev)
            if rank == 0:  # a progress line per launch queued (the queue runs at most a step or two ahead)
                progress("headline step %d queued" % work.step_idx)

        timing = [False]
        elapsed = timed_steps(step, args.steps, args.warmup, world, "cuda", torch.cuda.synchronize,
                              before=lambda: timing.__setitem__(0, True))
        launch_ms = sum(a.elapsed_time(b) for a, b in events) / max(1, len(events))
        units_per_step = work.n_jobs * args.ctus
        bytes_per_launch = b_ctu(nref) * units_per_step
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        config = {"workload": "HM-16.5rc1 TEncCu::compressCtu + encodeCtu, bit-exact: merge/skip, AMVP+TMVP, TZ "
                              "SR64 + frac ME vs %d refs, 2NxN/Nx2N/AMP, RQT + RDOQ + transform skip, "
                              "intra-in-inter, CABAC context carry; SliceMode=1 row slices; steady state (synthetic "
                              "references)" % nref,
                  "resolution": f"{W}x{H}", "ctus_per_frame": work.wc * work.hc, "pictures_per_gpu": args.pics,
                  "slice_chains_per_gpu": work.n_jobs, "ctus_per_chain_per_step": args.ctus,
                  "slice": "P, QP %d (base %d + GOP offset %d), QPFactor %g, lambda %.6f" % (
                      work.qp, args.qp, HM_QP_OFFSET, HM_QP_FACTOR, work.params["lambda"]),
                  "n_ref": nref, "parallelism": f"pictures x{world}", "dpb": "local"}
        data = ("synthetic: splitmix64 uniform random 8-bit 4:2:0 YUV (BASELINE.md sec. 3), the previous 4 frames as "
                "references, seeded synthetic collocated motion field; own pictures per rank")
        dpb_ok = None
    else:
        work, elapsed, sec, ctus, byt, dpb_ok, n_gathered = closed_main(args, rank, world)
        units_per_step = work.units_per_step
        launch_ms = sec / args.steps * 1e3
        bytes_per_launch = byt / args.steps
        achieved = byt / sec / 1e9
        W, H = work.W, work.H
        config = {"workload": "BASELINE config 5: " + work.workload() + "; after every picture each segment's finished "
                              "(deblocked + SAO) picture is gathered to rank 0's DPB (RCCL over xGMI)",
                  "resolution": f"{W}x{H}", "segments_per_gpu": len(work.cs.segs),
                  "slice_chains_per_gpu": len(work.cs.segs) * work.cs.nch, "ctus_per_chain_per_step": work.cs.ctus_step,
                  "pictures": [dict(p) for p in work.cs.log], "timed_pictures": work.timed_pictures,
                  "parallelism": f"closed segments x{world}",
                  "dpb": "each finished picture of every segment gathered to rank 0 (%d pictures x %d segments per "
                         "rank)" % (n_gathered, len(work.cs.segs)) if world > 1 else "local",
                  "n1_comparable": "the N=1 line's config5_closed_segments figure (the same per-GPU workload; compare "
                                   "timed_pictures' per-POC rates with its pictures' -- the reference count grows "
                                   "with the POC); this exact line at N=1 (--workload closed --steps 20 --warmup 5): "
                                   "1412.3 CTUs/s, profiles/bench_closed_r06c.log -- scaling efficiency at N is "
                                   "value / (N x that), not value / (N x the steady-state headline)"}
        data = ("synthetic: splitmix64 uniform random 8-bit 4:2:0 originals made on the device (BASELINE.md sec. 3), "
                "frame indices disjoint per segment and rank; references made by each segment's own loop")
    if rank == 0:
        value = aggregate(units_per_step, args.steps, world, elapsed)
        traffic, issue = None, {}
        tr_path = os.path.join(ROOT, "profiles", "hbm_traffic_r06.json")  # PMC passes of this round's tree
        if kind == "steady" and os.path.exists(tr_path):
            tr = json.load(open(tr_path)).get("k_hm_compress")
            if tr:
                traffic = tr["bytes_per_launch"] * units_per_step / tr.get("ctus_per_launch", units_per_step)
        pmc_path = os.path.join(ROOT, "profiles", "hm_pmc_r06.json")
        if os.path.exists(pmc_path):
            pm = json.load(open(pmc_path))
            issue = {"simd_issue_frac": pm["simd_issue_frac"], "valu_frac": pm["valu_frac"],
                     "wave_cycle_split": pm["wave_cycle_split"], "pmc_file": "profiles/hm_pmc_r06.json"}
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
            "data": data,
            "config": config,
            # priced against HBM (integer work); the limiter is the serial RD decision
            # chain inside each wave (latency), not bandwidth -- frac << 1
            "roofline": {"bound": "hbm", "limiter": "instruction latency of the serial decision chain (issue + "
                                                    "dependency waits; see simd_issue_frac / wave_cycle_split)",
                         "kernel": "k_hm_compress",
                         "achieved": round(achieved, 4), "peak": MI355X_HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / MI355X_HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_launch": bytes_per_launch, "avg_launch_ms": round(launch_ms, 3),
                         "b_ctu": b_ctu(nref) if kind == "steady" else "per picture: b_ctu(distinct refs)",
                         **issue},
            "cpu_baseline": None,
        }
        if dpb_ok is not None:
            out["dpb_gather_ok"] = dpb_ok
        out["build"] = build_provenance()
        if world == 1 and kind == "steady":
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
            del work, out_rec
            torch.cuda.empty_cache()
            if not args.no_ra:
                side("config4_ra_stvssim", "config 4 (closed RA segments, stVSSIM cost)",
                     lambda: config4_measure(threads, parity=not args.no_cpu))
                torch.cuda.empty_cache()
            if not args.no_closed:
                side("config5_closed_segments", "config 5 unit (closed LDP segments)",
                     lambda: config5_measure(threads, parity=not args.no_cpu))
                torch.cuda.empty_cache()
            if not args.no_1080p:
                side("hm_1080p", "1080p side figure", hm_1080p_measure)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
