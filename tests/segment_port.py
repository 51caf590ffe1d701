"""TEST INFRASTRUCTURE: video_codecs_amd/gop.py's ClosedSegments with the device replaced by the CPU
restatement (oracle/hvx_oracle_cu.c), so the closed-segment orchestration -- picture set-up, reference
lists, DPB bookkeeping, stepping, the multi-GPU bench's DPB gather -- runs under pytest without a GPU.

Per picture: every slice chain decided by hvxo_hm_chains (at the picture's last launch), the boundary
strengths (hvxo_hm_boundary_strength), loopFilterPic (oracle.deblock) and compressMotion
(hvxo_hm_col_field).  SAO and the slice writer are not restated here (sao=False, write=False: each
slice starts from its own type's table); the device loop's SAO / writer are pinned on the GPU
(tests/test_gop_gpu.py)."""
import time

import numpy as np

from video_codecs_amd import _abi, gop


class _Wall:
    """A stand-in for a HIP event pair: elapsed_time in ms from the host clock."""

    def __init__(self):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class PortSegments(gop.ClosedSegments):
    def __init__(self, *a, threads=1, **k):
        k.update(sao=False, write=False, device="cpu")
        super().__init__(*a, **k)
        self.threads = threads
        self.decided = None
        self.finished_log = []

    def begin(self):
        self.cur = []
        for s, seg in enumerate(self.segs):
            prm, qp, entry, table, planes, col_nref = self.picture_params(s, self.t)
            g = self.plan[self.t]
            org = tuple(np.ascontiguousarray(np.asarray(p), np.uint8) for p in self.org_fn(s, g.poc))
            refs = np.concatenate([seg.dpb[p] for p in planes]) if planes else np.zeros(1, np.uint8)
            col = seg.cols.get(g.col_poc) if g.col_poc is not None else None
            self.cur.append(dict(prm=prm, qp=qp, entry=entry, table=table, col_nref=col_nref, org=org, refs=refs, col=col))
        self.decided = None

    def launch(self, L):
        from oracle import hm_ctu
        a = _Wall()
        if L == self.launches - 1:  # the whole picture on the host, at its last launch
            self.decided = []
            for c in self.cur:
                pi, pf = gop.host_pic_arrays(self.W, self.H, c["prm"], c["qp"], col_nref=c["col_nref"])
                org = np.concatenate([p.reshape(-1) for p in c["org"]])
                self.decided.append((pi, hm_ctu.chains(pi, pf, org, c["refs"], c["entry"],
                                                       np.arange(self.nch, dtype=np.int32) * self.cl, self.cl, self.cl,
                                                       threads=self.threads, col_field=c["col"])))
        if self.launch_events is not None:
            self.launch_events.append((self.t, len(self.segs) * self.nch * self.ctus_step, (a, _Wall())))

    def loop(self):
        import oracle
        import torch
        from oracle import hm_ctu
        W, H, wc = self.W, self.H, self.wc
        out = []
        for c, (pi, r) in zip(self.cur, self.decided):
            rec = [np.zeros((H >> (1 if k else 0), W >> (1 if k else 0)), np.uint8) for k in range(3)]
            for a in range(wc * self.hc):
                ax, ay = a % wc, a // wc
                t = r["recon"][a]
                yy, xx = min(64, H - ay * 64), min(64, W - ax * 64)
                rec[0][ay * 64:ay * 64 + yy, ax * 64:ax * 64 + xx] = t[:4096].reshape(64, 64)[:yy, :xx]
                for k in (1, 2):
                    cpl = t[4096 + (k - 1) * 1024:4096 + k * 1024].reshape(32, 32)
                    rec[k][ay * 32:ay * 32 + yy // 2, ax * 32:ax * 32 + xx // 2] = cpl[:yy // 2, :xx // 2]
            bv, bh, qp = hm_ctu.boundary_strength(W, H, r["parts"], np.asarray(pi[7:15]).reshape(2, 4),
                                                  int(pi[3]) == gop.B_SLICE)
            fin = oracle.deblock(*rec, bv.reshape(-1), bh.reshape(-1), qp.reshape(-1), _abi.deblock_params(W, H))
            fin = tuple(np.ascontiguousarray(p, np.uint8) for p in fin)
            out.append(dict(ref=np.concatenate([p.reshape(-1) for p in fin]), col=hm_ctu.col_field(W, H, r["parts"]),
                            rec=tuple(torch.from_numpy(p) for p in fin), org=c["org"], bytes=0, table=c["table"],
                            parts=r["parts"]))
        self.last_results = out
        return out
