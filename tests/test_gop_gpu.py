"""Closed GOP segments on the device (video_codecs_amd/gop.py ClosedSegments) against the reference.

- test_closed_ra_segments_vs_hm: two closed random-access segments (encoder_randomaccess_main.cfg: I +
  two GOP8s, 128x64, QP 27 and 37, SAO on) encoded concurrently, every picture decided against the
  references, collocated field and slice-start states the device loop made (deblocking, SAO, the slice
  writer's cabac_init choice): every CTU of all 34 pictures equals HM-16.5rc1's own encode of the same
  YUV (tests/golden/ctu_ra_closed_q*.bin), and so does every picture's CABAC initialisation table.
- test_closed_ldp_segment_vs_hm: the LDP configuration (I, P, P at 416x240, one slice per picture, SAO on)
  against HM's encode (tests/golden/ctu_ldp_rand.bin).
- test_closed_ldp_row_slices_vs_hm / test_closed_ra_row_slices_vs_hm: closed LDP (448x256, four slices
  per picture) and RA (192x128, I + GOP8, two slices per picture) segments with one slice per CTU row
  (SliceMode 1), SAO on: every CTU, finished picture and CABAC table equals HM's encode
  (tests/golden/ctu_{ldp,ra}_closed_slices.bin).  Each slice after the first is written with the table
  the slice before it chose, as HM writes them (gop.ClosedSegments.write_slices).
- test_closed_ldp_four_refs_vs_hm: LDP I + 8 P pictures (128x64, QP 32), four device-made references
  from POC 4 on, against HM's encode (tests/golden/ctu_ldp_closed_4ref.bin).
- test_closed_ra_stvssim_full_history: config 4 as an encode -- a closed RA segment decided with the
  stvssim encoder's active cost (HVX_RD_STVSSIM) over the segment's own history of originals and final
  reconstructions, up to the full 25 pictures (POC 28, coding index 26): every picture re-decided by the
  restatement (oracle/hvx_oracle_cu.c) from the device's references, field and history, bit-exact.
"""
import numpy as np
import pytest

from tests import golden_cases as gc
from tests import hm_cases


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("needs a GPU")
    return t


def _capture_org_fn(gs):
    """org_fn(seg, poc) -> the capture's original of that POC (segment s reads capture gs[s])."""
    def fn(s, poc):
        g = gs[s]
        for k, pi in enumerate(g["pic_i32"]):
            if int(pi[hm_cases.P_POC]) == poc:
                w, h = int(pi[hm_cases.P_W]), int(pi[hm_cases.P_H])
                psz = w * h * 3 // 2
                return hm_cases.yuv_split(g["org"][k * psz:(k + 1) * psz], w, h)
        raise KeyError(poc)
    return fn


class Kept:
    """after_launch hook: the launch's CTU records and reconstructions, per (picture, segment, chain)."""

    def __init__(self, cs):
        self.cs, self.out = cs, {}
        cs.after_launch = self

    def __call__(self, L):
        from video_codecs_amd import hm
        cs = self.cs
        ct = cs.out_ctu.cpu().numpy().view(hm.HM_CTU).reshape(len(cs.segs), cs.nch, cs.ctus_step)
        rc = cs.out_rec.cpu().numpy().reshape(len(cs.segs), cs.nch, cs.ctus_step, 6144)
        for s in range(len(cs.segs)):
            for c in range(cs.nch):
                for i in range(cs.ctus_step):
                    self.out[(cs.t, s, c * cs.cl + L * cs.ctus_step + i)] = (ct[s, c, i].copy(), rc[s, c, i].copy())


def _compare_with_capture(g, kept, t_of_pic, s, n):
    bad = []
    for pic in range(g["pic_i32"].shape[0]):
        first = int(g["pic_i32"][pic][hm_cases.P_FIRST_CTU])
        ctus = np.stack([kept[(t_of_pic[pic], s, a)][0] for a in range(n)])
        rec = np.stack([kept[(t_of_pic[pic], s, a)][1] for a in range(n)])
        for b in hm_cases.compare(g, [(pic, first, n, 0)], (ctus, rec, None)):
            bad.append((s, int(g["pic_i32"][pic][hm_cases.P_POC])) + b[1:])
    return bad


@pytest.mark.gpu
def test_closed_ra_segments_vs_hm(torch):
    from video_codecs_amd import cabac_init, gop, hvx
    hvx.context()
    gs = [gc.load("ctu_ra_closed_q27.bin"), gc.load("ctu_ra_closed_q37.bin")]
    plan = gop.load_plan("ra", 17)
    finals = {}

    def finished(t, recs):  # every finished (deblocked + SAO) picture, for the reference-picture check
        for s, r in enumerate(recs):
            finals[(s, plan[t].poc)] = np.concatenate([x.cpu().numpy().reshape(-1) for x in r])
    cs = gop.ClosedSegments(plan, 128, 64, [27, 37], _capture_org_fn(gs), on_finished=finished)
    kept = Kept(cs)
    while cs.t < len(plan):
        cs.step()
    torch.cuda.synchronize()
    pocs = [g.poc for g in plan]
    bad, tables = [], []
    for s, g in enumerate(gs):
        t_of_pic = [pocs.index(int(pi[hm_cases.P_POC])) for pi in g["pic_i32"]]
        bad += _compare_with_capture(g, kept.out, t_of_pic, s, 2)
        psz = 128 * 64 * 3 // 2
        for k, q in enumerate(int(p) for p in g["refpic_poc"]):  # HM's reference pictures (after SAO)
            if not np.array_equal(finals[(s, q)], g["refpic"][k * psz:(k + 1) * psz]):
                bad.append((s, q, "finished picture"))
        # the CABAC initialisation table of every picture (cabac_init_flag from the device writer's states)
        want = [cabac_init.resolve_table(int(pi[hm_cases.P_SLICE_TYPE]), int(pi[hm_cases.P_CABAC_TABLE])) for pi in g["pic_i32"]]
        got = [cs.segs[s].tables[t] for t in t_of_pic]
        if got != want:
            tables.append((s, got, want))
        assert all(b > 0 for b in cs.segs[s].bytes)
    assert not bad and not tables, ([b for b in bad if b[2] == "finished picture"], bad[:6], tables)


@pytest.mark.gpu
def test_closed_ldp_segment_vs_hm(torch):
    from video_codecs_amd import gop, hvx
    hvx.context()
    g = gc.load("ctu_ldp_rand.bin")
    plan = gop.load_plan("ldp", 3)
    cs = gop.ClosedSegments(plan, 416, 240, [32], _capture_org_fn([g]), rows=4)  # SliceMode 0: one slice
    kept = Kept(cs)
    while cs.t < len(plan):
        cs.step()
    torch.cuda.synchronize()
    bad = _compare_with_capture(g, kept.out, [0, 1, 2], 0, 28)
    assert not bad, bad[:6]


def _closed_vs_capture(torch, name, kind, W, H, qp):
    """A closed segment with one slice per CTU row (one slice when the picture is one row) against HM's
    encode of the same YUV (capture `name`): every CTU, finished picture and CABAC table; returns the
    tables each picture's slices were written with."""
    from video_codecs_amd import cabac_init, gop, hvx
    hvx.context()
    g = gc.load(name)
    n_pic = g["pic_i32"].shape[0]
    plan = gop.load_plan(kind, n_pic)
    finals, chains = {}, []

    def finished(t, recs):
        finals[plan[t].poc] = np.concatenate([x.cpu().numpy().reshape(-1) for x in recs[0]])
    cs = gop.ClosedSegments(plan, W, H, [qp], _capture_org_fn([g]), rows=1, on_finished=finished)
    assert cs.nch == H // 64 and cs.cl == W // 64
    kept = Kept(cs)
    while cs.t < len(plan):
        cs.step()
        if cs.L == 0 and cs.last_slices is not None:  # the table each slice of the picture was written with
            chains.append([int(x) for x in cs.last_slices[3][0]])
    torch.cuda.synchronize()
    pocs = [p.poc for p in plan]
    t_of_pic = [pocs.index(int(pi[hm_cases.P_POC])) for pi in g["pic_i32"]]
    bad = _compare_with_capture(g, kept.out, t_of_pic, 0, cs.nch * cs.cl)
    psz = W * H * 3 // 2
    for k, q in enumerate(int(p) for p in g["refpic_poc"]):
        if not np.array_equal(finals[q], g["refpic"][k * psz:(k + 1) * psz]):
            bad.append((0, q, "finished picture"))
    want = [cabac_init.resolve_table(int(pi[hm_cases.P_SLICE_TYPE]), int(pi[hm_cases.P_CABAC_TABLE])) for pi in g["pic_i32"]]
    got = [cs.segs[0].tables[t] for t in t_of_pic]
    assert not bad and got == want, (bad[:6], got, want, chains)
    assert len(chains) == n_pic and all(len(c) == cs.nch for c in chains)
    return chains


@pytest.mark.gpu
def test_closed_ldp_row_slices_vs_hm(torch):
    _closed_vs_capture(torch, "ctu_ldp_closed_slices.bin", "ldp", 448, 256, 30)


@pytest.mark.gpu
def test_closed_ra_row_slices_vs_hm(torch):
    """RA (I + one GOP8, B slices) at 192x128 with two row slices per picture, QP 32
    (tests/golden/ctu_ra_closed_slices.bin)."""
    _closed_vs_capture(torch, "ctu_ra_closed_slices.bin", "ra", 192, 128, 32)


@pytest.mark.gpu
def test_closed_ldp_four_refs_vs_hm(torch):
    """LDP I + 8 P pictures at 128x64, QP 32: from POC 4 on every P picture searches four references the
    device made (tests/golden/ctu_ldp_closed_4ref.bin) -- the headline's reference count in a closed loop."""
    _closed_vs_capture(torch, "ctu_ldp_closed_4ref.bin", "ldp", 128, 64, 32)


@pytest.mark.gpu
def test_closed_ra_stvssim_full_history(torch):
    from oracle import hm_ctu
    from oracle import make_yuv
    from video_codecs_amd import _abi, gop, hm, hvx
    hvx.context()
    W, H, n = 64, 64, 27
    frames = [hm_cases.yuv_split(make_yuv.texture_frame(W, H, i), W, H) for i in range(33)]
    plan = gop.load_plan("ra", n)
    cs = gop.ClosedSegments(plan, W, H, [30], lambda s, poc: frames[poc], rd_metric=_abi.RD_STVSSIM)
    kept = Kept(cs)
    checked = []
    while cs.t < n:
        t = cs.t
        # the restatement's inputs for picture t, from the device's own loop (before it decides t)
        seg = cs.segs[0]
        prm, qp, entry, table, planes, col_nref = cs.picture_params(0, t)
        refs = []
        for p in planes:
            y8, _, cb16, cr16 = (x.cpu().numpy() for x in seg.dpb[p].planes())
            m8 = hm.DeviceFrame.M8
            refs.append(np.concatenate([y8[m8:m8 + H, m8:m8 + W].reshape(-1), cb16[40:40 + H // 2, 40:40 + W // 2]
                                        .astype(np.uint8).reshape(-1), cr16[40:40 + H // 2, 40:40 + W // 2].astype(np.uint8).reshape(-1)]))
        g = plan[t]
        col = seg.cols[g.col_poc].cpu().numpy() if g.col_poc is not None else None
        hist = [tuple(x.cpu().numpy() for x in fr) for fr in seg.hist[:_abi.STV_HIST]]
        dirs = gop.stv_direction_map(col, W, H)
        cs.step()
        pi, pf = gop.host_pic_arrays(W, H, prm, qp, col_nref=col_nref)
        org = np.concatenate([p.reshape(-1) for p in frames[g.poc]])
        port = hm_ctu.chains(pi, pf, org, np.concatenate(refs) if refs else np.zeros(1, np.uint8), entry,
                             np.array([0], np.int32), 1, 1, col_field=col, rd_metric=_abi.RD_STVSSIM,
                             lambda_ssim=prm["lambda_ssim"], stv=(hist, dirs))
        ct, rc = kept.out[(t, 0, 0)]
        assert np.array_equal(port["parts"][0], hm.unpack_parts(ct["p"][None])[0]), (t, g.poc)
        assert np.array_equal(port["coef"][0].astype(np.int16), ct["coef"]) and np.array_equal(port["recon"][0], rc), t
        assert port["cost"][0] == ct["cost"] and (int(port["bits_dist"][0][0]), int(port["bits_dist"][0][1])) == \
            (int(ct["bits"]), int(ct["dist"])), t
        checked.append(len(hist))
    assert checked[-1] == _abi.STV_HIST and plan[n - 1].slice_type == gop.B_SLICE  # POC 28 over 25 pictures
