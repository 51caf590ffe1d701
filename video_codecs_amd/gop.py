"""Closed GOP segments on the device: the per-picture loop around the CU decision.

The reference encodes a segment picture by picture (hm-16.5rc1 TEncGOP::compressGOP, TEncGOP.cpp:994):
slice set-up (reference lists, lambdas, slice-start CABAC states), compressSlice (the CU decision,
TEncSlice.cpp:727-828), loopFilterPic (:1465), SAOProcess (:1500), encodeSlice (:1570, which also
picks the next slice's cabac_init table), and the picture becomes a reference.  ClosedSegments runs
that loop for many independent segments at once on one GPU, entirely on the device:

- decision: hvx_hm_compress, one wave per slice chain, `ctus_step` CTUs per chain per launch;
- hvx_hm_finish_picture: deblocking with device boundary strengths, the compressed motion field;
- SAO statistics / RD decision / offsets (hm.sao_pictures: one decision launch for all segments);
- hvx_hm_write_slices: every slice's syntax through TEncBinCABAC (SAO + CU syntax), the context
  states it ends with -> determineCabacInitIdx (cabac_init.py) -> the next picture's table;
- the padded reference planes (hvx_hm_finish_picture) the next pictures search, and for the stvssim
  cost (rd_metric HVX_RD_STVSSIM) the segment's own history of originals and final reconstructions in
  coding order (storeRefAndEncFrames, stvssim.c:362, called after every coded frame, image.c:563).

The segment structure (coding order, reference lists, collocated picture, QP offsets) is HM's own for
the encoder_lowdelay_P_main / encoder_randomaccess_main configurations: recorded from the compiled
reference's TEncGOP (tests/golden/gop_plans.json, oracle/gen_gop_plans.sh), because HM builds the
first GOPs' reference sets with TAppEncCfg's extra-RPS search and temporal-layer rules
(TAppEncCfg.cpp:1847-2050); the QP offsets / QPFactors / GOP depths are the cfg's (checked against the
recorded lambdas by tests/test_gop_cpu.py).  Scope: this is the harness of the path (config 4 / 5),
not a general encoder -- one slice type per picture, no rate control, no NAL / header writing.
"""
import json
import os

import numpy as np

from . import _abi, cabac_init, hm

I_SLICE, P_SLICE, B_SLICE = 2, 1, 0
# cfg Frame entries: POC % GOPSize -> (QP offset, QPFactor) (encoder_lowdelay_P_main.cfg:24-27,
# encoder_randomaccess_main.cfg:24-31)
CFG = {
    "ldp": {"gop": 4, "frames": {1: (3, 0.4624), 2: (2, 0.4624), 3: (3, 0.4624), 0: (1, 0.578)}},
    "ra": {"gop": 8, "frames": {0: (1, 0.442), 4: (2, 0.3536), 2: (3, 0.3536), 6: (3, 0.3536), 1: (4, 0.68), 3: (4, 0.68),
                                5: (4, 0.68), 7: (4, 0.68)}},
}


def gop_depth(poc, gop_size):
    """TEncSlice::initEncSlice's GOP depth of a picture (TEncSlice.cpp:233-252): 0 for POC % GOPSize == 0,
    else the level of the dyadic hierarchy the position falls on."""
    p = poc % gop_size
    if p == 0:
        return 0
    step, depth = gop_size, 0
    i = step >> 1
    while i >= 1:
        found = False
        for j in range(i, gop_size, step):
            if j == p:
                found = True
                break
        step >>= 1
        depth += 1
        if found:
            break
        i >>= 1
    return depth


class GopPicture:
    """One picture of a segment in coding order: POC, slice type, QP offset / QPFactor / GOP depth,
    reference POC lists, collocated picture (TComSlice after TEncGOP's set-up)."""

    def __init__(self, rec, kind):
        self.poc, self.slice_type = int(rec["poc"]), int(rec["slice_type"])
        self.nref = [int(x) for x in rec["nref"]]
        self.refs = [[int(p) for p in rec["ref_poc"][l][:self.nref[l]]] for l in range(2)]
        self.col_from_l0, self.check_ldc = int(rec["col_from_l0"]), int(rec["check_ldc"])
        self.tmvp, self.max_merge = int(rec["tmvp"]), int(rec["max_merge"])
        cfg = CFG[kind]
        self.depth = gop_depth(self.poc, cfg["gop"])
        if self.slice_type == I_SLICE:
            self.qp_offset = 0
            nb = cfg["gop"] - 1  # TEncSlice.cpp:255: dLambda_scale from the number of B frames
            self.qp_factor = 0.57 * (1.0 - min(0.5, 0.05 * nb))
        else:
            self.qp_offset, self.qp_factor = cfg["frames"][self.poc % cfg["gop"]]

    @property
    def col_poc(self):
        l = 0 if (self.slice_type == P_SLICE or self.col_from_l0) else 1
        return self.refs[l][0] if self.nref[l] else None

    def ref_pocs(self):
        """The distinct reference POCs of both lists, in first-use order (the picture's ref planes)."""
        out = []
        for l in range(2):
            for p in self.refs[l]:
                if p not in out:
                    out.append(p)
        return out


def load_plan(kind, n_pics, path=None):
    """The first n_pics pictures (coding order) of a closed segment of configuration `kind` ('ldp' or
    'ra') as HM's TEncGOP sets them up (tests/golden/gop_plans.json)."""
    path = path or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                                "gop_plans.json")
    recs = json.load(open(path))[kind]
    assert n_pics <= len(recs), "the recorded plan has %d pictures" % len(recs)
    return [GopPicture(r, kind) for r in recs[:n_pics]]


def host_pic_arrays(W, H, prm, qp, col_nref=(4, 0)):
    """A picture's slice parameters (hm.DevicePicture's params dict) as the restatement's pic_i32 /
    pic_f64 arrays (oracle/cu_capture.cpp layout: tests/hm_cases.P_* fields)."""
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


def stv_direction_map(col_field, w, h):
    """hm.stv_direction_map vectorised: per 16x16 block of the collocated field its (at most two)
    motion votes, getOrientation'd (stvssim.c:1317, float32 as the reference; memoised per distinct
    vector) and chosen by chooseOrient (:1347: the first maximum of the 16 two-bin counts, i.e. with
    two different votes the lower bin)."""
    f = np.float32
    pi = f(3.1415926)
    bw, bh = w // 4, h // 4
    out = np.zeros((bh, bw), np.float32)
    if col_field is None:
        return out
    col = np.asarray(col_field).reshape(-1, 16, 8).astype(np.int32)
    memo = {}

    def orient(x, y):
        k = (x, y)
        if k not in memo:
            memo[k] = hm.stv_orientation(x, y) // 2
        return memo[k]
    inter = col[:, :, 0] >= 0
    idx = np.full(col.shape[:2], 16, np.int32)
    for l in range(2):
        has = inter & (col[:, :, 1 + l] >= 0)
        for a, b in zip(*np.nonzero(has)):
            v = orient(int(col[a, b, 3 + 2 * l]), int(col[a, b, 4 + 2 * l]))
            idx[a, b] = min(idx[a, b], v)
    idx[idx == 16] = 0
    table = np.array([f(0)] + [f(f(pi * f(i)) / f(16)) for i in range(1, 16)], np.float32)
    vals = table[idx]
    wc = (w + 63) // 64
    z = np.arange(16)
    bx, by = (z & 1) | ((z >> 1) & 2), ((z >> 1) & 1) | ((z >> 2) & 2)
    for a in range(col.shape[0]):
        for b in range(16):
            x0, y0 = ((a % wc) * 64 + bx[b] * 16) // 4, ((a // wc) * 64 + by[b] * 16) // 4
            if x0 < bw and y0 < bh:
                out[y0:min(y0 + 4, bh), x0:min(x0 + 4, bw)] = vals[a, b]
    return out


def chain_jobs(specs):
    """HM_JOB records: specs = [(pic, first_ctu, n_ctus, slice_start, slice_end, resume, entry_states)]."""
    j = np.zeros(len(specs), hm.HM_JOB)
    for k, (pic, first, n, s0, s1, resume, entry) in enumerate(specs):
        j[k]["pic"], j[k]["first_ctu"], j[k]["n_ctus"], j[k]["chained"], j[k]["out"] = pic, first, n, 1, k * n
        j[k]["slice_start"], j[k]["slice_end"] = s0, s1
        j[k]["flags"] = _abi.HM_RESUME if resume else 0
        j[k]["entry"]["st"] = entry
    return j


class Segment:
    """One closed segment's encoder state between pictures."""

    def __init__(self, base_qp, seed):
        self.base_qp, self.seed = base_qp, seed
        self.dpb, self.cols, self.lists = {}, {}, {}   # POC -> reference frame / motion field / (nref, ref POCs)
        self.rates = np.zeros((3, 7))                   # SAO-off rates per temporal layer (decidePicParams)
        self.enc_table = I_SLICE                        # TEncSlice::m_encCABACTableIdx
        self.hist = []                                  # stVSSIM history, most recent first
        self.tables, self.bytes = [], []                # per coded picture: CABAC table used, slice data bytes


class ClosedSegments:
    """`len(base_qps)` closed segments of `plan` (load_plan) with W x H originals from org_fn(seg, poc) ->
    (Y, Cb, Cr), decided on the device picture by picture: every picture's chains (one per slice of
    `rows` CTU rows) advance `ctus_step` CTUs per launch (step()); after a picture's last launch every
    segment's picture is finished on the device (finish()).  on_finished(t, [(Y, Cb, Cr) final
    reconstruction per segment]) is called after each picture (the DPB gather of the multi-GPU bench).

    rd_metric HVX_RD_STVSSIM: the decision's cost is the stvssim encoder's (lambda_ssim(QP) * eta^0.85),
    over the segment's own history.  write: the slice writer runs per picture and picks the next
    picture's cabac_init table as HM does (else every slice uses its own type's table)."""

    def __init__(self, plan, W, H, base_qps, org_fn, rows=1, ctus_step=None, sao=True, write=True,
                 rd_metric=_abi.RD_SSE, eta=1.0, on_finished=None, seeds=None, device="cuda"):
        assert W % 8 == 0 and H % 8 == 0
        self.plan, self.W, self.H = plan, W, H
        self.wc, self.hc = (W + 63) // 64, (H + 63) // 64
        assert H % 64 == 0 or rows >= 2, "a partial bottom row shares its slice with the row above"
        assert self.hc % rows == 0, "equal slices of `rows` CTU rows"
        self.rows, self.nch, self.cl = rows, self.hc // rows, rows * self.wc
        self.ctus_step = ctus_step or self.cl
        assert self.cl % self.ctus_step == 0, "whole launches per picture"
        self.launches = self.cl // self.ctus_step
        self.segs = [Segment(q, (seeds or list(range(len(base_qps))))[s]) for s, q in enumerate(base_qps)]
        self.org_fn, self.sao, self.write = org_fn, sao, write
        self.rd_metric, self.eta, self.on_finished = rd_metric, eta, on_finished
        self.device = device
        self.eb = _abi.load_entropy_bits()
        self.t, self.L = 0, 0          # next picture (coding index) and launch within it
        self.pictures = None
        self.log = []                  # per finished picture: timings, bytes, CABAC tables
        self.ctus_decided = 0
        self.launch_events = None      # a list: (picture, CTUs, (start, end) HIP events) per launch
        self.finished_log = None       # a list: every picture's loop() results (kept when set)
        self.last_slices = None        # the last picture's slice writes: (bytes, results, capacity, tables
                                       # each slice was written with, the result index of each slice)

    # ---- picture set-up (TEncGOP / TEncSlice::initEncSlice) --------------------------------------
    def picture_params(self, s, t):
        """(params dict for hm.DevicePicture, slice QP, entry states, ref POCs in plane order, col nref)."""
        g, seg = self.plan[t], self.segs[s]
        qp = seg.base_qp + g.qp_offset
        prm = hm.slice_params(g.slice_type, qp, g.qp_factor, gop_depth=g.depth)
        planes = g.ref_pocs()
        ref_poc = np.zeros((2, 4), int)
        ref_plane = np.zeros((2, 4), int)
        for l in range(2):
            for k, p in enumerate(g.refs[l]):
                ref_poc[l, k], ref_plane[l, k] = p, planes.index(p)
        col_ref_poc, col_nref = np.zeros((2, 4), int), (0, 0)
        col_poc = g.col_poc
        if col_poc is not None:
            cn, cr = seg.lists[col_poc]
            col_nref = tuple(cn)
            for l in range(2):
                for k in range(cn[l]):
                    col_ref_poc[l, k] = cr[l][k]
        prm.update(poc=g.poc, nref=list(g.nref), ref_poc=ref_poc, ref_plane=ref_plane, max_merge=g.max_merge,
                   tmvp=g.tmvp, check_ldc=g.check_ldc, col_from_l0=g.col_from_l0,
                   col_valid=int(col_poc is not None and bool(g.tmvp)), col_poc=col_poc or 0, col_ref_poc=col_ref_poc,
                   search_range=64, amp=1)
        if self.rd_metric != _abi.RD_SSE:
            prm.update(rd_metric=self.rd_metric, lambda_ssim=hm.lambda_ssim(qp, self.eta))
        table = cabac_init.resolve_table(g.slice_type, seg.enc_table)
        entry = cabac_init.slice_start_states(table, qp)
        return prm, qp, entry, table, planes, col_nref

    def begin(self):
        """Set up picture t of every segment: originals, references, motion field, slice parameters."""
        import torch
        t = self.t
        self.cur = []
        pictures = []
        for s, seg in enumerate(self.segs):
            prm, qp, entry, table, planes, col_nref = self.picture_params(s, t)
            g = self.plan[t]
            org = hm.DeviceFrame.original(self.org_fn(s, g.poc), self.device)
            stv = None
            if self.rd_metric == _abi.RD_STVSSIM:
                col_h = seg.cols[g.col_poc].cpu().numpy() if g.col_poc is not None else None
                dirs = stv_direction_map(col_h, self.W, self.H)
                stv = hm.StvHistory(seg.hist[:_abi.STV_HIST], dirs, device=self.device).prepare(self.W, self.H)
            pic = hm.DevicePicture(org, [seg.dpb[p] for p in planes], prm, self.eb,
                                   col_field=seg.cols.get(g.col_poc) if g.col_poc is not None else None,
                                   device=self.device, stv=stv)
            pictures.append(pic)
            self.cur.append(dict(prm=prm, qp=qp, entry=entry, table=table, planes=planes, col_nref=col_nref,
                                 org=org, stv=stv))
        self.pictures = pictures
        self.eng = hm.Engine(pictures, self.device)
        n_out = len(self.segs) * self.nch * self.ctus_step
        if getattr(self, "_n_out", None) != n_out:
            self.out_ctu = torch.zeros(n_out * hm.HM_CTU.itemsize, dtype=torch.uint8, device=self.device)
            self.out_rec = torch.zeros(n_out * 6144, dtype=torch.uint8, device=self.device)
            self._n_out = n_out

    def launch_jobs(self, L):
        specs = []
        for s in range(len(self.segs)):
            for c in range(self.nch):
                first = c * self.cl + L * self.ctus_step
                specs.append((s, first, self.ctus_step, c * self.cl, c * self.cl + self.cl - 1, L > 0, self.cur[s]["entry"]))
        return chain_jobs(specs)

    # ---- one step: one launch (and the picture's loop after its last launch) -------------------
    def step(self):
        """Launch L of picture t; after the picture's last launch, finish() it.  Returns the CTUs
        this launch decided.  Every allocation and kernel of the step is ordered on one stream
        (torch's current stream, or the segments' own when that is the null stream), so no buffer is
        released to the caching allocator while a kernel of another stream still reads it."""
        import contextlib
        ctx = contextlib.nullcontext()
        if self.device != "cpu":
            import torch
            if torch.cuda.current_stream().cuda_stream == 0:
                if getattr(self, "_stream", None) is None:
                    self._stream = torch.cuda.Stream()
                ctx = torch.cuda.stream(self._stream)
        with ctx:
            if self.L == 0:
                self.begin()
            self.launch(self.L)
            self.after_launch(self.L)
            n = len(self.segs) * self.nch * self.ctus_step
            self.ctus_decided += n
            self.L += 1
            if self.L == self.launches:
                self.finish()
                self.L = 0
                self.t += 1
        return n

    def launch(self, L):
        """Decision launch L of picture t: every segment's chains advance ctus_step CTUs."""
        import torch
        jt = torch.from_numpy(self.launch_jobs(L).view(np.uint8).reshape(-1).copy()).to(self.device)
        ev = None
        if self.launch_events is not None:  # HIP events around the decision launch on its stream
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        self.eng.launch(jt, len(self.segs) * self.nch, self.out_ctu, self.out_rec)
        self._jobs = jt  # held until the next launch (the kernel reads it asynchronously)
        if ev is not None:
            ev[1].record()
            self.launch_events.append((self.t, len(self.segs) * self.nch * self.ctus_step, ev))

    def after_launch(self, L):
        """Hook: the launch's outputs (self.out_ctu / out_rec) are on the stream (parity samples)."""

    def finish(self):
        """Picture t's reference loop (loop()), then the segments' bookkeeping: the DPB, motion fields,
        reference lists, stVSSIM history, the pictures no later picture needs released, on_finished."""
        import time
        t0 = time.perf_counter()
        t, g = self.t, self.plan[self.t]
        results = self.loop()
        if self.finished_log is not None:
            self.finished_log.append(results)
        for seg, r in zip(self.segs, results):
            seg.dpb[g.poc], seg.cols[g.poc] = r["ref"], r["col"]
            seg.lists[g.poc] = (tuple(g.nref), [list(g.refs[0]), list(g.refs[1])])
            seg.tables.append(r["table"])
            seg.bytes.append(r["bytes"])
            if self.rd_metric == _abi.RD_STVSSIM:
                seg.hist.insert(0, (*r["org"], *r["rec"]))
                del seg.hist[_abi.STV_HIST:]
        later = set()
        for q in self.plan[t + 1:]:
            later.update(q.ref_pocs())
            if q.col_poc is not None:
                later.add(q.col_poc)
        for seg in self.segs:
            for p in [p for p in seg.dpb if p not in later]:
                del seg.dpb[p]
                seg.cols.pop(p, None)
        if self.on_finished is not None:
            self.on_finished(t, [r["rec"] for r in results])
        self.log.append({"poc": g.poc, "slice": "IPB"[{I_SLICE: 0, P_SLICE: 1, B_SLICE: 2}[g.slice_type]],
                         "qp_offset": g.qp_offset, "slice_data_bytes": int(sum(r["bytes"] for r in results)),
                         "loop_s": round(time.perf_counter() - t0, 3)})

    def loop(self):
        """The reference loop of picture t of every segment on the device (TEncGOP.cpp:1465-1570):
        deblocking + motion field, SAO, the slice writer, the padded reference planes.  Returns per
        segment dict(ref, col, rec = final (Y, Cb, Cr), org, bytes, table)."""
        import torch
        g = self.plan[self.t]
        segs, pics = self.segs, self.pictures
        dbk = _abi.deblock_params(self.W, self.H)
        cols = [hm.finish_picture(p, dbk, col_field=True)[1] for p in pics]
        slice_ctus = self.cl if self.nch > 1 else 0
        if self.sao:
            sao = hm.sao_pictures(pics, [g.depth] * len(segs), [s.rates for s in segs], [g.slice_type] * len(segs),
                                  [c["qp"] for c in self.cur], slice_ctus=slice_ctus,
                                  sao_states=[(c["entry"][hm.SAO_CTX_MERGE], c["entry"][hm.SAO_CTX_TYPE]) for c in self.cur])
        nbytes = [0] * len(segs)
        if self.write:
            nbytes = self.write_slices(sao if self.sao else None)
        out = []
        for s, (seg, pic) in enumerate(zip(segs, pics)):
            if self.sao:
                seg.rates = sao[s][0]
            ref = hm.DeviceFrame.blank(self.W, self.H, self.device)
            hm.finish_picture(pic, None, ref_frame=ref)
            rec = tuple(r[:(self.H >> (1 if c else 0)), :(self.W >> (1 if c else 0))] for c, r in enumerate(pic.rec_t))
            out.append(dict(ref=ref, col=cols[s], rec=rec, org=tuple(self.cur[s]["org"].org), bytes=nbytes[s],
                            table=self.cur[s]["table"]))
        torch.cuda.current_stream().synchronize()
        self.last_pictures = pics
        return out

    def write_slices(self, sao):
        """encodeSlice of every slice of picture t (hvx_hm_write_slices, one launch for all segments):
        the slice data bytes per segment, and each segment's next cabac_init table.

        HM writes a picture's slices one after another, and each encodeSlice ends with
        determineCabacInitIdx (TEncSlice.cpp:1096-1099) over that slice's final states and coded
        contexts; slice k > 0 is written with the table the slice before it chose (TEncGOP.cpp:1559
        takes m_encCABACTableIdx for every slice header, TEncSbac::resetEntropy initialises from it)
        while the decision used the previous picture's choice for all of them (TEncGOP.cpp:1246).  A
        slice's data depends only on its own CTUs and the table it starts from, and a P / B slice can
        start from two tables (B's or P's), so every slice after the first is written from both in the
        same launch and the chain of choices is then followed on the host: the first slice from the
        picture's table, each next one from what the slice before it chose."""
        import torch
        n_seg = len(self.segs)
        st = self.plan[self.t].slice_type
        cands = [cabac_init.B_SLICE, cabac_init.P_SLICE] if st != I_SLICE else [I_SLICE]
        jobs = []  # (segment, slice, table)
        for s in range(n_seg):
            for c in range(self.nch):
                for tab in ([self.cur[s]["table"]] if c == 0 else cands):
                    jobs.append((s, c, tab))
        n = len(jobs)
        cap = max(1 << 16, self.cl * 12288)
        out = torch.zeros(n * cap, dtype=torch.uint8, device=self.device)
        sl = np.zeros(n, hm.HM_SLICE)
        keep, en, coded = [], [], []
        for s in range(n_seg):
            coded_t = None
            e3 = [0, 0, 0]
            if sao is not None:
                coded_t = torch.from_numpy(np.ascontiguousarray(sao[s][1], np.int32)).to(self.device)
                keep.append(coded_t)
                # the slice header carries one chroma flag, Cb's (TEncGOP.cpp:1504-1508): when the rates
                # of decidePicParams disabled only one chroma component, Cr's offsets are applied but
                # not written
                e = [int(x) for x in sao[s][3]]
                e3 = [e[0], e[1], e[1]]
            en.append(e3)
            coded.append(coded_t.data_ptr() if coded_t is not None else 0)
        for k, (s, c, tab) in enumerate(jobs):
            sl[k]["pic"], sl[k]["first_ctu"], sl[k]["n_ctus"], sl[k]["out_cap"] = s, c * self.cl, self.cl, cap
            sl[k]["out"] = out.data_ptr() + k * cap
            sl[k]["sao_enabled"] = en[s]
            sl[k]["sao_coded"] = coded[s]
            sl[k]["entry"]["st"] = cabac_init.slice_start_states(cabac_init.resolve_table(st, tab), self.cur[s]["qp"])
        sl_t = torch.from_numpy(sl.view(np.uint8).reshape(-1).copy()).to(self.device)
        res_t = torch.zeros(n * hm.HM_SLICE_RESULT.itemsize, dtype=torch.uint8, device=self.device)
        self.eng.write_slices_launch(sl_t, n, res_t)
        res = res_t.cpu().numpy().view(hm.HM_SLICE_RESULT)
        assert (res["status"] == 0).all() and (res["n_bytes"] <= cap).all(), "hvx_hm_write_slices refused a slice"
        at = {j: k for k, j in enumerate(jobs)}
        nbytes, used, final = [], [], []
        for s, seg in enumerate(self.segs):
            tab, tabs, nb, ks = self.cur[s]["table"], [], 0, []
            for c in range(self.nch):
                k = at[(s, c, tab if c == 0 else cabac_init.resolve_table(st, tab))]
                tabs.append(tab)
                ks.append(k)
                nb += int(res[k]["n_bytes"])
                tab = cabac_init.determine_cabac_init_idx(st, res[k]["states"][:202], cabac_init.coded_flags(res[k]["coded"]),
                                                          self.cur[s]["qp"], self.eb)
            seg.enc_table = tab
            nbytes.append(nb)
            used.append(tabs)
            final.append(ks)
        self.last_slices = (out, res, cap, used, final)
        return nbytes
