"""GPU-vs-oracle parity cases shared by tests/test_gpu_parity.py and __graft_entry__.smoke().

Every function runs the HIP path (video_codecs_amd.hvx -> libhvx.so) and checks it
against the CPU oracle (test infrastructure) and/or the reference goldens; it raises
AssertionError on the first mismatch.
"""
import numpy as np

import oracle
from oracle import make_yuv
from tests import golden_cases as gc
from video_codecs_amd import _abi, hvx

M = _abi.PLANE_MARGIN


def _torch():
    import torch
    return torch


def padded_plane(img):
    """uint8 HxW -> padded plane (H+2M)x(W+2M) with replicated borders (extendPicBorder)."""
    return np.pad(img, M, mode="edge")


def device_planes(planes):
    """list of padded uint8 planes (same shape) -> (device tensors, int64 device tensor of origin pointers)."""
    torch = _torch()
    ts = [torch.from_numpy(np.ascontiguousarray(p)).cuda() for p in planes]
    W = planes[0].shape[1] - 2 * M
    ptrs = torch.tensor([hvx.plane_origin_ptr(t, W) for t in ts], dtype=torch.int64).cuda()
    return ts, ptrs


def run_me(planes_cur, planes_ref, jobs):
    torch = _torch()
    cur_t, cur_p = device_planes(planes_cur)
    ref_t, ref_p = device_planes(planes_ref)
    stride = planes_cur[0].shape[1]
    jd = hvx.to_device(jobs)
    out = torch.zeros(len(jobs) * _abi.ME_RESULT.itemsize, dtype=torch.uint8, device="cuda")
    hvx.me_batch(cur_p, ref_p, stride, jd, len(jobs), out)
    torch.cuda.synchronize()
    del cur_t, ref_t
    return hvx.from_device(out, _abi.ME_RESULT)


def me_jobs_random(rng, n, W, H, n_planes=1):
    jobs = np.zeros(n, _abi.ME_JOB)
    shapes = [(64, 64), (32, 32), (16, 16), (8, 8), (64, 32), (32, 64), (16, 8), (8, 16), (64, 16), (64, 48),
              (16, 64), (48, 64), (32, 8), (32, 24), (8, 32), (24, 32), (16, 4), (16, 12), (4, 16), (12, 16), (8, 4), (4, 8)]
    for i in range(n):
        w, h = shapes[rng.integers(len(shapes))]
        cu = max(w, h)
        cu = 64 if cu > 32 else 32 if cu > 16 else 16 if cu > 8 else 8
        cux = rng.integers(0, (W - cu) // cu + 1) * cu
        cuy = rng.integers(0, (H - cu) // cu + 1) * cu
        pux = cux + (rng.integers(0, (cu - w) // 4 + 1) * 4 if w < cu else 0)
        puy = cuy + (rng.integers(0, (cu - h) // 4 + 1) * 4 if h < cu else 0)
        lam = 0.57 * 2.0 ** ((int(rng.integers(22, 38)) - 12) / 3.0)
        j = jobs[i]
        j["pic_w"], j["pic_h"], j["max_cu"] = W, H, 64
        j["cu_x"], j["cu_y"], j["pu_x"], j["pu_y"], j["w"], j["h"] = cux, cuy, pux, puy, w, h
        j["pred_x"], j["pred_y"] = rng.integers(-60, 61), rng.integers(-60, 61)
        if i % 6 == 1:
            j["pred_x"], j["pred_y"] = rng.integers(-900, 900), rng.integers(-600, 600)
        j["use_int2nx2n"] = i % 3 == 0
        j["i2_x"], j["i2_y"] = rng.integers(-20, 21), rng.integers(-20, 21)
        j["bits_in"] = rng.integers(0, 8)
        j["search_range"] = 64
        j["lambda_motion"] = _abi.lambda_motion_sad(lam)
        j["flags"] = _abi.ME_FEN | _abi.ME_HADME | _abi.ME_SMOOTHMV
        j["cur_idx"] = j["ref_idx"] = rng.integers(0, n_planes)
    return jobs


def check_me_random(seed, n_jobs, width, height):
    rng = np.random.default_rng(seed)
    cur, ref = [], []
    for p in range(2):
        if p == 0:
            a = make_yuv.random_frame(width, height, seed)[:width * height].reshape(height, width)
            b = make_yuv.random_frame(width, height, seed + 1)[:width * height].reshape(height, width)
        else:
            a = make_yuv.smooth_frame(width, height, 3)[:width * height].reshape(height, width)
            b = make_yuv.smooth_frame(width, height, 2)[:width * height].reshape(height, width)
        cur.append(padded_plane(a))
        ref.append(padded_plane(b))
    jobs = me_jobs_random(rng, n_jobs, width, height, n_planes=2)
    got = run_me(cur, ref, jobs)
    for i in range(n_jobs):
        exp = oracle.motion_estimation(cur[jobs["cur_idx"][i]], ref[jobs["ref_idx"][i]], jobs[i])
        assert tuple(got[i]) == tuple(exp), (i, jobs[i], got[i], exp)
    return True


def check_me_golden():
    g = gc.load("me.bin")
    planes, jobs, exp = gc.me_jobs(g)
    cur = [planes[p, 0] for p in range(planes.shape[0])]
    ref = [planes[p, 1] for p in range(planes.shape[0])]
    got = run_me(cur, ref, jobs)
    for i in range(len(jobs)):
        assert [int(x) for x in got[i]] == [int(x) for x in exp[i]], (i, jobs[i], got[i], exp[i])
    return len(jobs)


# ------------------------------------------------------------------------------------------ TUs
def run_tu(descs, ests, residuals, mode="forward", levels_in=None):
    """descs: TU_DESC array; ests: [n, 224] int32; residuals/levels_in: list of arrays (w*h)."""
    torch = _torch()
    n = len(descs)
    sizes = [int(d["width"]) * int(d["height"]) for d in descs]
    off = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    total = int(sum(sizes))
    d_desc = hvx.to_device(descs)
    d_off = torch.from_numpy(off).cuda()
    if mode == "inverse":
        lev = torch.from_numpy(np.concatenate([np.asarray(x, np.int32).reshape(-1) for x in levels_in])).cuda()
        res_out = torch.zeros(total, dtype=torch.int16, device="cuda")
        hvx.tu_inverse_batch(d_desc, d_off, n, lev, res_out)
        torch.cuda.synchronize()
        r = res_out.cpu().numpy()
        return [r[o:o + s] for o, s in zip(off, sizes)]
    d_est = torch.from_numpy(np.ascontiguousarray(ests, np.int32).reshape(-1)).cuda()
    res = torch.from_numpy(np.concatenate([np.asarray(x, np.int16).reshape(-1) for x in residuals])).cuda()
    lev = torch.zeros(total, dtype=torch.int32, device="cuda")
    absum = torch.zeros(n, dtype=torch.int32, device="cuda")
    if mode == "forward":
        temp = torch.zeros(total, dtype=torch.int32, device="cuda")
        arl = torch.zeros(total, dtype=torch.int32, device="cuda")
        hvx.tu_forward_batch(d_desc, d_est, None, d_off, n, res, temp, lev, arl, absum)
        torch.cuda.synchronize()
        t, l, a = temp.cpu().numpy(), lev.cpu().numpy(), absum.cpu().numpy()
        return [(t[o:o + s], l[o:o + s], int(a[i])) for i, (o, s) in enumerate(zip(off, sizes))]
    res_out = torch.zeros(total, dtype=torch.int16, device="cuda")
    sse = torch.zeros(n, dtype=torch.int32, device="cuda")
    hvx.tu_pipeline_batch(d_desc, d_est, None, d_off, n, res, lev, absum, res_out, sse)
    torch.cuda.synchronize()
    l, a, r, s_ = lev.cpu().numpy(), absum.cpu().numpy(), res_out.cpu().numpy(), sse.cpu().numpy().view(np.uint32)
    return [(l[o:o + s], int(a[i]), r[o:o + s], int(s_[i])) for i, (o, s) in enumerate(zip(off, sizes))]


def golden_estbits_pool():
    pool = []
    for f in gc.TU_FILES:
        g = gc.load(f)
        pool.append(g["fwd_estbits"])
    return np.concatenate(pool)


def random_tus(rng, n, est_pool):
    descs = np.zeros(n, _abi.TU_DESC)
    ests, res = [], []
    for i in range(n):
        d = descs[i]
        log2 = int(rng.integers(2, 6))
        comp = int(rng.integers(0, 3)) if log2 < 5 else 0
        qp = int(rng.integers(0, 52))
        d["comp"], d["width"], d["height"], d["log2_size"] = comp, 1 << log2, 1 << log2, log2
        d["is_intra"] = int(rng.integers(0, 2))
        d["scan_type"] = int(rng.integers(0, 3)) if (d["is_intra"] and log2 <= 3) else 0
        d["use_dst"] = int(d["is_intra"] and comp == 0 and log2 == 2)
        d["transform_skip"] = int(log2 == 2 and rng.integers(0, 4) == 0)
        d["tr_idx"] = int(rng.integers(0, 2))
        d["ctx_qt_cbf"] = int(rng.integers(0, 3 if comp == 0 else 5))
        d["slice_type"] = int(rng.integers(0, 3))
        d["qp_per"], d["qp_rem"] = qp // 6, qp % 6
        d["sign_hiding"] = int(rng.integers(0, 4) != 0)
        mode = int(rng.integers(0, 5))
        d["use_rdoq"] = int(mode != 0)
        d["use_rdoq_ts"] = int(mode != 0)
        d["selective_rdoq"] = int(mode == 4)
        d["max_log2_tr_range"], d["bit_depth"] = 15, 8
        d["golomb_rice_stat"] = 0
        d["lambda"] = 0.57 * 2.0 ** ((qp - 12) / 3.0) * (1.0 if comp == 0 else 0.8)
        ests.append(est_pool[int(rng.integers(0, len(est_pool)))])
        amp = [255, 60, 12, 3][int(rng.integers(0, 4))]
        res.append(rng.integers(-amp, amp + 1, size=(1 << log2) * (1 << log2)).astype(np.int16))
    return descs, np.stack(ests), res


def check_tu_random(seed, n):
    rng = np.random.default_rng(seed)
    descs, ests, res = random_tus(rng, n, golden_estbits_pool())
    got = run_tu(descs, ests, res, "pipeline")
    for i in range(n):
        w = int(descs[i]["width"])
        t, l, _, a = oracle.transform_nxn(descs[i], ests[i], res[i].reshape(w, w))
        rr = oracle.inv_transform_nxn(descs[i], l)
        gl, ga, gr, gs = got[i]
        np.testing.assert_array_equal(gl, l, err_msg=f"levels tu {i} {descs[i]}")
        assert ga == a, (i, ga, a)
        np.testing.assert_array_equal(gr, rr.reshape(-1), err_msg=f"recon residual tu {i}")
        sse = int(((res[i].astype(np.int64) - rr.reshape(-1)) ** 2).sum())
        assert gs == sse, (i, gs, sse)
    return True


def mc_planes(rng, W, H, n_ref):
    """HM-like int16 4:2:0 reference planes (margins 80 luma / 40 chroma, borders replicated),
    smooth random content.  Returns [(array, origin_offset)] * 3*n_ref, strides."""
    out = []
    ML, MC = 80, 40
    for _ in range(n_ref):
        for c in range(3):
            w, h, m = (W, H, ML) if c == 0 else (W // 2, H // 2, MC)
            base = rng.integers(0, 256, size=(h // 4 + 2, w // 4 + 2)).astype(np.float64)
            img = np.kron(base, np.ones((4, 4)))[:h, :w] + rng.normal(0, 12, size=(h, w))
            img = np.clip(np.rint(img), 0, 255).astype(np.int16)
            p = np.pad(img, m, mode="edge")
            out.append((p, m * p.shape[1] + m))
    return out, W + 2 * ML, W // 2 + 2 * MC


def mc_jobs_random(rng, n, W, H, n_ref):
    shapes = [(64, 64), (32, 32), (16, 16), (8, 8), (64, 32), (32, 64), (16, 8), (8, 16), (64, 16), (64, 48),
              (16, 64), (32, 8), (8, 32), (16, 12), (12, 16), (8, 4), (4, 8), (24, 32), (32, 24)]
    jobs = np.zeros(n, _abi.MC_JOB)
    off = 0
    for i in range(n):
        w, h = shapes[rng.integers(len(shapes))]
        cu = 64 if max(w, h) > 32 else 32 if max(w, h) > 16 else 16 if max(w, h) > 8 else 8
        cux = int(rng.integers(0, (W - cu) // cu + 1)) * cu
        cuy = int(rng.integers(0, (H - cu) // cu + 1)) * cu
        j = jobs[i]
        j["pic_w"], j["pic_h"], j["max_cu"], j["cu_x"], j["cu_y"] = W, H, 64, cux, cuy
        j["pu_x"] = cux + (int(rng.integers(0, (cu - w) // 4 + 1)) * 4 if w < cu else 0)
        j["pu_y"] = cuy + (int(rng.integers(0, (cu - h) // 4 + 1)) * 4 if h < cu else 0)
        j["w"], j["h"] = w, h
        kind = i % 6  # 0/1 uni L0/L1, 2/3 bi, 4 identical (B), 5 identical motion in a P-style job (no shortcut)
        big = i % 7 == 0  # far MVs exercise clipMv
        for l in range(2):
            j["ref"][l] = int(rng.integers(0, n_ref))
            j["poc"][l] = int(j["ref"][l]) * 2
            j["mv_x"][l] = int(rng.integers(-700, 701)) if big else int(rng.integers(-96, 97))
            j["mv_y"][l] = int(rng.integers(-700, 701)) if big else int(rng.integers(-96, 97))
        if kind == 0:
            j["ref"][1] = -1
        elif kind == 1:
            j["ref"][0] = -1
        elif kind in (4, 5):
            j["ref"][1], j["poc"][1] = j["ref"][0], j["poc"][0]
            j["mv_x"][1], j["mv_y"][1] = j["mv_x"][0], j["mv_y"][0]
        j["flags"] = _abi.MC_B_SLICE if kind != 5 else 0
        j["dst_offset"] = off
        off += w * h + 2 * (w // 2) * (h // 2)
    return jobs, off


def check_mc_random(seed, n, W=320, H=192, n_ref=2):
    torch = _torch()
    rng = np.random.default_rng(seed)
    planes, ls, cs = mc_planes(rng, W, H, n_ref)
    jobs, total = mc_jobs_random(rng, n, W, H, n_ref)
    dev = [torch.from_numpy(p.reshape(-1).copy()).cuda() for p, _ in planes]
    ptrs = torch.tensor([t.data_ptr() + 2 * o for t, (_, o) in zip(dev, planes)], dtype=torch.int64).cuda()
    dst = torch.zeros(total, dtype=torch.int16, device="cuda")
    hvx.mc_batch(ptrs, ls, cs, hvx.to_device(jobs), n, dst)
    torch.cuda.synchronize()
    got = dst.cpu().numpy()
    for i in range(n):
        exp = oracle.mc(planes, ls, cs, jobs[i])
        o = int(jobs[i]["dst_offset"])
        np.testing.assert_array_equal(got[o:o + exp.size], exp, err_msg=f"mc job {i}: {jobs[i]}")
    return True


def check_me_full_golden():
    """hvx_me_full_batch vs the reference's xPatternSearch / bi refinement (me_full.bin)."""
    torch = _torch()
    g = gc.load("me_full.bin")
    planes, jobs, tg, exp = gc.me_full_jobs(g)
    n = len(jobs)
    ref_t, ref_p = device_planes([planes[p, 1] for p in range(planes.shape[0])])
    stride = planes.shape[-1]
    d_tg = torch.from_numpy(np.ascontiguousarray(tg).reshape(-1)).cuda()
    base = d_tg.data_ptr()
    # one virtual int16 plane per job whose (pu_x, pu_y) is the job's 64x64 pattern block
    tptr = [base + 2 * (i * 4096 - (int(jobs[i]["pu_y"]) * 64 + int(jobs[i]["pu_x"]))) for i in range(n)]
    d_tp = torch.tensor(tptr, dtype=torch.int64).cuda()
    out = torch.zeros(n * _abi.ME_RESULT.itemsize, dtype=torch.uint8, device="cuda")
    hvx.me_full_batch(d_tp, 64, ref_p, stride, hvx.to_device(jobs), n, out)
    torch.cuda.synchronize()
    got = hvx.from_device(out, _abi.ME_RESULT)
    for i in range(n):
        assert [int(x) for x in got[i]] == [int(x) for x in exp[i]], (i, jobs[i], got[i], exp[i])
    del ref_t
    return n


def random_coeff_tus(seed, n):
    """Random TUs for the coefficient-rate counter: sizes 4-32, both channels, all scans,
    sparse to dense levels with large escape values, random (valid) context states."""
    rng = np.random.default_rng(seed)
    descs = np.zeros(n, _abi.TU_DESC)
    levels, states = [], np.zeros((n, _abi.NUM_CTX), np.uint8)
    for i in range(n):
        w = int(rng.choice([4, 8, 16, 32]))
        d = descs[i:i + 1]
        d["width"] = d["height"] = w
        d["log2_size"] = int(np.log2(w))
        d["comp"] = int(rng.integers(0, 3))
        d["scan_type"] = int(rng.integers(0, 3)) if w <= 8 else 0
        d["pps_tskip"] = int(rng.integers(0, 2))
        d["transform_skip"] = int(rng.integers(0, 2)) if w == 4 else 0
        d["sign_hiding"] = int(rng.integers(0, 2))
        d["transquant_bypass"] = int(rng.random() < 0.1)
        d["ts_context"] = int(rng.random() < 0.2)
        d["persistent_rice"] = int(rng.integers(0, 2))
        d["golomb_rice_stat"] = int(rng.integers(0, 16)) if d["persistent_rice"][0] else 0
        d["extended_precision"] = int(rng.random() < 0.2)
        d["max_log2_tr_range"] = 15
        d["bit_depth"] = 8
        dens = rng.choice([0.0, 0.02, 0.1, 0.4, 1.0])
        mag = rng.choice([2, 4, 40, 2000, 32767])
        lv = (rng.random(w * w) < dens) * rng.integers(1, mag + 1, w * w)
        lv = np.where(rng.random(w * w) < 0.5, -lv, lv).astype(np.int32)
        if not lv.any() and rng.random() < 0.7:
            lv[int(rng.integers(0, w * w))] = int(rng.integers(-3, 4)) or 1
        levels.append(lv)
        states[i] = rng.integers(0, 126, _abi.NUM_CTX)
    return descs, levels, states


def check_coeff_bits_random(seed, n):
    import torch
    descs, levels, states = random_coeff_tus(seed, n)
    eb = gc.load("cabac.bin")["entropy_bits"].astype(np.int32)
    off = np.concatenate([[0], np.cumsum([len(l) for l in levels])[:-1]]).astype(np.int64)
    d_st = torch.from_numpy(states.reshape(-1).copy()).cuda()
    out = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    hvx.coeff_bits_batch(hvx.to_device(descs), hvx.to_device(off), n, hvx.to_device(np.concatenate(levels)),
                         hvx.to_device(eb), d_st, out)
    torch.cuda.synchronize()
    r = out.cpu().numpy().view(_abi.COEFF_BITS)
    st_gpu = d_st.cpu().numpy().reshape(n, -1)
    for i in range(n):
        fb, rice, ns, st = oracle.coeff_bits(descs[i], levels[i], states[i], eb)
        got = (int(r["frac_bits"][i]), int(r["rice_stat"][i]), int(r["num_sig"][i]))
        assert got == (fb, rice, ns), (i, descs[i], got, (fb, rice, ns))
        np.testing.assert_array_equal(st_gpu[i], st, err_msg=f"TU {i}")
    return True


def run_coeff_write(descs, levels, stream_first, states, regs, cap):
    """hvx_coeff_write_batch on host arrays: stream k = TUs [stream_first[k], stream_first[k+1]).
    Returns (list of byte arrays, regs after, states after)."""
    import torch
    ns = len(stream_first) - 1
    off = np.concatenate([[0], np.cumsum([len(l) for l in levels])[:-1]]).astype(np.int64)
    flat = np.concatenate(levels).astype(np.int32) if levels else np.zeros(1, np.int32)
    d_st = torch.from_numpy(np.ascontiguousarray(states, np.uint8).reshape(-1).copy()).cuda()
    d_rg = torch.from_numpy(np.ascontiguousarray(regs, _abi.CABAC_REGS).view(np.uint8).copy()).cuda()
    out = torch.zeros(ns * cap, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(ns, dtype=torch.int32, device="cuda")
    hvx.coeff_write_batch(hvx.to_device(descs), hvx.to_device(off), hvx.to_device(flat),
                          hvx.to_device(np.asarray(stream_first, np.int32)), ns, d_st, d_rg, out,
                          hvx.to_device(np.arange(ns, dtype=np.int64) * cap), cap, d_len)
    torch.cuda.synchronize()
    lens = d_len.cpu().numpy()
    o = out.cpu().numpy().reshape(ns, cap)
    assert (lens >= 0).all(), lens[lens < 0]
    return [o[k, :lens[k]].copy() for k in range(ns)], d_rg.cpu().numpy().view(_abi.CABAC_REGS), \
        d_st.cpu().numpy().reshape(ns, -1)


def check_coeff_write_golden():
    """Every record of cabac_write.bin as a one-TU run from its captured registers and states."""
    g = gc.load("cabac_write.bin")
    descs, levels = gc.cabac_cases(g)
    n = len(levels)
    regs = np.zeros(n, _abi.CABAC_REGS)
    for k, f in enumerate(("low", "range", "bits_left", "num_buffered", "buffered_byte")):
        regs[f] = g["regs"][:, k]
    got, r, st = run_coeff_write(descs, levels, np.arange(n + 1), g["states_before"], regs, 4096)
    bo = g["byte_off"]
    for i in range(n):
        np.testing.assert_array_equal(got[i], g["bytes"][bo[i]:bo[i + 1]], err_msg=f"record {i}")
        assert tuple(int(r[i][f]) for f in ("low", "range", "bits_left", "num_buffered", "buffered_byte")) == \
            tuple(int(x) for x in g["regs"][i, 5:]), (i, r[i], g["regs"][i])
    np.testing.assert_array_equal(st, g["states_after"])
    return n


def check_coeff_write_random(seed, n_streams, max_tus):
    """Random runs of random TUs (random_coeff_tus) from TEncBinCABAC::start() and random context
    states; the oracle writes each run TU by TU carrying registers and states."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, max_tus + 1, n_streams)
    first = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    descs, levels, _ = random_coeff_tus(seed + 1, int(first[-1]))
    # the writer refuses persistent Rice adaptation (its statistic would have to carry across the
    # TUs of a run; include/hvx.h): those runs are checked for the refusal separately
    descs["persistent_rice"] = 0
    descs["golomb_rice_stat"] = 0
    states = rng.integers(0, 126, (n_streams, _abi.NUM_CTX)).astype(np.uint8)
    regs = np.zeros(n_streams, _abi.CABAC_REGS)
    regs[:] = _abi.CABAC_START
    got, r, st = run_coeff_write(descs, levels, first, states, regs, 1 << 16)
    total = 0
    for k in range(n_streams):
        rk, sk, exp = tuple(_abi.CABAC_START), states[k].copy(), []
        for t in range(first[k], first[k + 1]):
            b, rk, sk = oracle.coeff_write(descs[t], levels[t], sk, rk)
            exp.append(b)
        exp = np.concatenate(exp) if exp else np.zeros(0, np.uint8)
        np.testing.assert_array_equal(got[k], exp, err_msg=f"run {k}")
        fields = ("low", "range", "bits_left", "num_buffered", "buffered_byte", "bins")
        assert tuple(int(r[k][f]) for f in fields) == \
            tuple(int(rk[f]) if isinstance(rk, np.void) else int(rk[i]) for i, f in enumerate(fields)), (k, r[k], rk)
        if isinstance(rk, np.void):  # the contexts the run coded (setBinsCoded)
            np.testing.assert_array_equal(r[k]["coded"], rk["coded"], err_msg=f"run {k} coded")
        np.testing.assert_array_equal(st[k], sk, err_msg=f"run {k}")
        total += len(exp)
    return int(first[-1]), total


# ----------------------------------------------------------------------------------------- intra
INTRA_TILE = 144  # a block at (8, 8) of its tile: above-right / below-left reach 8 + 128


def intra_planes(n_tiles, seed):
    """org + rec planes (random bytes, HVX_PLANE_MARGIN border) holding n_tiles INTRA_TILE tiles."""
    g = int(np.ceil(np.sqrt(max(n_tiles, 1))))
    W = H = g * INTRA_TILE
    rng = np.random.default_rng(seed)
    M = _abi.PLANE_MARGIN
    org = rng.integers(0, 256, (H + 2 * M, W + 2 * M), dtype=np.uint8)
    rec = rng.integers(0, 256, (H + 2 * M, W + 2 * M), dtype=np.uint8)
    return org, rec, g, W


def intra_tile_origin(i, g):
    M = _abi.PLANE_MARGIN
    return M + (i // g) * INTRA_TILE + 8, M + (i % g) * INTRA_TILE + 8  # (row, col) in the padded plane


def put_border(rec, r, c, n, raw):
    """write border-layout samples (corner, above row, left column) around the block at (r, c)."""
    raw = np.asarray(raw, np.int64) & 0xFF
    rec[r - 1, c - 1] = raw[0]
    rec[r - 1, c:c + 2 * n] = raw[1:2 * n + 1]
    rec[r:r + 2 * n, c - 1] = raw[2 * n + 1:4 * n + 1]


def run_intra_pred(org_or_none, rec, W, jobs):
    """hvx_intra_pred_batch over `jobs` (structured INTRA_JOB, x/y relative to the plane origin)
    -> (list of n x n predictions, ref borders [n, 2, 257])."""
    torch = _torch()
    n = len(jobs)
    sizes = [1 << int(j["log2_size"]) for j in jobs]
    off = np.concatenate([[0], np.cumsum([s * s for s in sizes])]).astype(np.int64)
    rec_t = torch.from_numpy(rec).cuda()
    jobs_t = hvx.to_device(jobs)
    off_t = torch.from_numpy(off[:-1].copy()).cuda()
    pred_t = torch.zeros(int(off[-1]), dtype=torch.uint8, device="cuda")
    ref_t = torch.zeros(n * 2 * 257, dtype=torch.int16, device="cuda")
    stride = rec.shape[1]
    hvx.intra_pred_batch(hvx.plane_origin_ptr(rec_t, W), stride, jobs_t, n, pred_t, off_t, ref_t)
    torch.cuda.synchronize()
    pred = pred_t.cpu().numpy()
    preds = [pred[off[i]:off[i + 1]].reshape(sizes[i], sizes[i]) for i in range(n)]
    return preds, ref_t.cpu().numpy().reshape(n, 2, 257)


def run_intra_search(org, rec, W, jobs):
    torch = _torch()
    n = len(jobs)
    org_t, rec_t = torch.from_numpy(org).cuda(), torch.from_numpy(rec).cuda()
    jobs_t = hvx.to_device(jobs)
    eb_t = torch.from_numpy(_abi.load_entropy_bits().copy()).cuda()
    out_t = torch.zeros(n * _abi.INTRA_RESULT.itemsize, dtype=torch.uint8, device="cuda")
    hvx.intra_search_batch(hvx.plane_origin_ptr(org_t, W), hvx.plane_origin_ptr(rec_t, W), org.shape[1], jobs_t, n,
                           eb_t, out_t)
    torch.cuda.synchronize()
    return hvx.from_device(out_t, _abi.INTRA_RESULT)


def check_intra_ref_golden():
    """initIntraPatternChType goldens through hvx_intra_pred_batch's border output: the raw samples
    placed around each block (unavailable positions hold random bytes, which must not leak)."""
    from tests import golden_cases as gc
    cases = gc.intra_ref_cases(gc.load("intra.bin"))
    org, rec, g, W = intra_planes(len(cases), 21)
    M = _abi.PLANE_MARGIN
    jobs = np.zeros(len(cases), _abi.INTRA_JOB)
    for i, (n, luma, ul, _f, raw, flags, _u, _ff) in enumerate(cases):
        r, c = intra_tile_origin(i, g)
        put_border(rec, r, c, n, raw)
        jobs[i]["x"], jobs[i]["y"] = c - M, r - M
        jobs[i]["log2_size"], jobs[i]["ch_type"], jobs[i]["unit_log2"] = n.bit_length() - 1, 0 if luma else 1, ul
        jobs[i]["avail"] = oracle.avail_words(flags)
        jobs[i]["flags"] = _abi.INTRA_STRONG
        jobs[i]["mode"] = 1
    _, refs = run_intra_pred(None, rec, W, jobs)
    for i, (n, luma, _ul, filt, _raw, _fl, unf, exp_filt) in enumerate(cases):
        np.testing.assert_array_equal(refs[i, 0, :4 * n + 1], unf, err_msg=f"unfiltered border, record {i}")
        if filt and luma:
            np.testing.assert_array_equal(refs[i, 1, :4 * n + 1], exp_filt, err_msg=f"filtered border, record {i}")
    return len(cases)


def check_intra_first_pass_golden():
    """estIntraPredLumaQT first-pass goldens through hvx_intra_search_batch."""
    from tests import golden_cases as gc
    cases = gc.intra_fp_cases(gc.load("intra.bin"))
    org, rec, g, W = intra_planes(len(cases), 22)
    M = _abi.PLANE_MARGIN
    jobs = np.zeros(len(cases), _abi.INTRA_JOB)
    for i, (job, o, raw, _exp) in enumerate(cases):
        n = 1 << int(job["log2_size"])
        r, c = intra_tile_origin(i, g)
        org[r:r + n, c:c + n] = np.asarray(o).reshape(n, n)
        put_border(rec, r, c, n, raw)
        jobs[i] = job
        jobs[i]["x"], jobs[i]["y"] = c - M, r - M
    res = run_intra_search(org, rec, W, jobs)
    bad = [i for i, (_j, _o, _r, exp) in enumerate(cases) if not gc.intra_fp_matches(res[i], exp)]
    assert not bad, (len(bad), bad[:5])
    return len(cases)


def random_intra_jobs(rng, n_jobs, g):
    """random luma/chroma blocks of every size with random neighbour availability (incl. none/all)."""
    M = _abi.PLANE_MARGIN
    jobs = np.zeros(n_jobs, _abi.INTRA_JOB)
    for i in range(n_jobs):
        ch = int(rng.integers(0, 2))
        log2 = int(rng.integers(2, 6 if ch else 7))
        ul = 1 if ch else 2
        nunits = ((4 << log2) >> ul) + 1
        kind = int(rng.integers(0, 4))
        flags = np.zeros(nunits, np.uint8) if kind == 0 else np.ones(nunits, np.uint8) if kind == 1 else \
            (rng.random(nunits) < (0.3 if kind == 2 else 0.8)).astype(np.uint8)
        r, c = intra_tile_origin(i, g)
        jobs[i]["x"], jobs[i]["y"], jobs[i]["log2_size"], jobs[i]["ch_type"] = c - M, r - M, log2, ch
        jobs[i]["unit_log2"], jobs[i]["avail"] = ul, oracle.avail_words(flags)
        jobs[i]["mode"] = int(rng.integers(0, 35))
        jobs[i]["flags"] = int(rng.integers(0, 4))
        jobs[i]["left_dir"], jobs[i]["above_dir"] = int(rng.integers(0, 35)), int(rng.integers(0, 35))
        jobs[i]["ctx_state"], jobs[i]["frac_bits"] = int(rng.integers(0, 126)), int(rng.integers(0, 32768))
        jobs[i]["sqrt_lambda"] = float(rng.uniform(2.0, 40.0))
    return jobs


def _raw_border(plane, r, c, n):
    return np.concatenate([[plane[r - 1, c - 1]], plane[r - 1, c:c + 2 * n], plane[r:r + 2 * n, c - 1]]).astype(np.int16)


def _flags_of(job):
    n = 1 << int(job["log2_size"])
    nunits = ((4 * n) >> int(job["unit_log2"])) + 1
    a = job["avail"]
    return np.array([(int(a[i >> 5]) >> (i & 31)) & 1 for i in range(nunits)], np.uint8)


def check_intra_random(seed, n_jobs):
    """random jobs: borders + prediction (hvx_intra_pred_batch) and the first pass
    (hvx_intra_search_batch, luma jobs) vs the oracle, bit-exact."""
    rng = np.random.default_rng(seed)
    org, rec, g, W = intra_planes(n_jobs, seed)
    jobs = random_intra_jobs(rng, n_jobs, g)
    preds, refs = run_intra_pred(None, rec, W, jobs)
    luma = np.nonzero(jobs["ch_type"] == 0)[0]
    res = run_intra_search(org, rec, W, jobs[luma])
    eb = _abi.load_entropy_bits()
    M = _abi.PLANE_MARGIN
    for i, j in enumerate(jobs):
        n, is_luma = 1 << int(j["log2_size"]), int(j["ch_type"]) == 0
        r, c = int(j["y"]) + M, int(j["x"]) + M
        raw = _raw_border(rec, r, c, n)
        unf = oracle.intra_fill(raw, _flags_of(j), n, int(j["unit_log2"]))
        np.testing.assert_array_equal(refs[i, 0, :4 * n + 1], unf, err_msg=f"job {i}")
        filt = oracle.intra_filter(unf, n, is_luma, bool(j["flags"] & _abi.INTRA_STRONG)) if is_luma else unf
        if is_luma:
            np.testing.assert_array_equal(refs[i, 1, :4 * n + 1], filt, err_msg=f"job {i}")
        m = int(j["mode"])
        exp = oracle.intra_pred(filt if oracle.intra_use_filter(m, n, is_luma) else unf, n, is_luma, m)
        np.testing.assert_array_equal(preds[i], exp, err_msg=f"job {i} mode {m} n {n}")
    for k, i in enumerate(luma):
        j = jobs[i]
        n = 1 << int(j["log2_size"])
        r, c = int(j["y"]) + M, int(j["x"]) + M
        exp = oracle.intra_search(org[r:r + n, c:c + n], _raw_border(rec, r, c, n), j, eb)
        assert res[k].tobytes() == exp.tobytes(), (i, res[k], exp)
    return n_jobs, len(luma)


# ------------------------------------------------------------------------------------ deblocking
def run_deblock(y, cb, cr, bs_ver, bs_hor, qp, params, margin=16):
    """hvx_deblock on padded device copies of the planes (borders hold random bytes that must stay
    untouched); returns the filtered (y, cb, cr) and whether every border byte survived."""
    torch = _torch()
    rng = np.random.default_rng(5)
    outs, keep = [], True
    pads = []
    for a in (y, cb, cr):
        pa = rng.integers(0, 256, (a.shape[0] + 2 * margin, a.shape[1] + 2 * margin), dtype=np.uint8)
        pa[margin:-margin, margin:-margin] = a
        pads.append(pa)
    dev = [torch.from_numpy(pa.copy()).cuda() for pa in pads]
    org = lambda t, w: t.data_ptr() + margin * (w + 2 * margin) + margin  # noqa: E731
    hvx.deblock(org(dev[0], y.shape[1]), dev[0].shape[1], org(dev[1], cb.shape[1]), org(dev[2], cr.shape[1]),
                dev[1].shape[1], hvx.to_device(np.asarray(bs_ver, np.uint8)), hvx.to_device(np.asarray(bs_hor, np.uint8)),
                hvx.to_device(np.asarray(qp, np.int8)), params)
    torch.cuda.synchronize()
    for pa, d in zip(pads, dev):
        got = d.cpu().numpy()
        inner = got[margin:-margin, margin:-margin].copy()
        got[margin:-margin, margin:-margin] = pa[margin:-margin, margin:-margin]
        keep &= np.array_equal(got, pa)
        outs.append(inner)
    return outs, keep


def check_deblock_golden():
    cases = gc.deblock_cases(gc.load("deblock.bin"))
    for k, (params, pre, post, bv, bh, qp) in enumerate(cases):
        got, keep = run_deblock(*pre, bv, bh, qp, params)
        assert keep, k
        for c in range(3):
            np.testing.assert_array_equal(got[c], post[c], err_msg=f"picture {k} plane {c}")
    return len(cases)


def check_deblock_random(seed, w=1920, h=1080):
    """random pictures, BS maps (0/1/2 on the edge grid), QP maps 0..51 and offsets vs the oracle."""
    rng = np.random.default_rng(seed)
    h8 = h - h % 8
    y = rng.integers(0, 256, (h8, w), dtype=np.uint8)
    # smooth-ish content so the filters actually fire: blocks of a ramp plus small noise
    base = (np.add.outer(np.arange(h8), np.arange(w)) // 3 % 256).astype(np.int32)
    y = np.clip(base + rng.integers(-3, 4, base.shape) + (rng.integers(0, 2, base.shape) * (y % 8)), 0, 255).astype(np.uint8)
    cb = (y[::2, ::2] // 2 + 64).astype(np.uint8)
    cr = (255 - y[::2, ::2]).astype(np.uint8)
    uw, uh = w // 4, h8 // 4
    bs_ver = rng.integers(0, 3, (uh, uw)).astype(np.uint8)
    bs_hor = rng.integers(0, 3, (uh, uw)).astype(np.uint8)
    bs_ver[:, 1::2] = 0
    bs_ver[:, 0] = 0
    bs_hor[1::2, :] = 0
    bs_hor[0, :] = 0
    qp = rng.integers(0, 52, (uh, uw)).astype(np.int8)
    params = _abi.deblock_params(w, h8, int(rng.integers(-6, 7)), int(rng.integers(-6, 7)), int(rng.integers(-12, 13)),
                                 int(rng.integers(-12, 13)))
    exp = oracle.deblock(y, cb, cr, bs_ver.ravel(), bs_hor.ravel(), qp.ravel(), params)
    got, keep = run_deblock(y, cb, cr, bs_ver.ravel(), bs_hor.ravel(), qp.ravel(), params)
    assert keep
    for c in range(3):
        np.testing.assert_array_equal(got[c], exp[c], err_msg=f"plane {c}")
    return int((exp[0] != y).sum())


def _padded_dev(planes, margin, rng):
    """padded device copies of planes (random border bytes); returns (tensors, [(origin, stride)])."""
    torch = _torch()
    devs, views = [], []
    for a in planes:
        pa = rng.integers(0, 256, (a.shape[0] + 2 * margin, a.shape[1] + 2 * margin), dtype=np.uint8)
        pa[margin:-margin, margin:-margin] = a
        t = torch.from_numpy(pa).cuda()
        devs.append(t)
        views.append((t.data_ptr() + margin * pa.shape[1] + margin, pa.shape[1]))
    return devs, views


def run_sao(org, pre, params, w, h, margin=8, luma_only=False):
    """hvx_sao_stats + hvx_sao_apply on padded device planes: (stats [nctu,3,5] SAO_STAT, applied
    planes, destination borders untouched)."""
    torch = _torch()
    rng = np.random.default_rng(9)
    k = 1 if luma_only else 3
    keep_org, ov = _padded_dev(org[:k], margin, rng)  # the tensors must outlive the launches
    keep_pre, pv = _padded_dev(pre[:k], margin, rng)
    dst_init = [rng.integers(0, 256, (p.shape[0] + 2 * margin, p.shape[1] + 2 * margin), dtype=np.uint8) for p in pre[:k]]
    dd = [torch.from_numpy(d.copy()).cuda() for d in dst_init]
    dv = [(t.data_ptr() + margin * t.shape[1] + margin, t.shape[1]) for t in dd]
    if luma_only:
        ov, pv, dv = ov + [(0, 0)] * 2, pv + [(0, 0)] * 2, dv + [(0, 0)] * 2
    nctu = ((w + 63) // 64) * ((h + 63) // 64)
    stats = torch.full((nctu * 15 * _abi.SAO_STAT.itemsize,), 0x5A, dtype=torch.uint8, device="cuda")
    hvx.sao_stats(ov, pv, w, h, stats)
    prm = hvx.to_device(np.ascontiguousarray(params, _abi.SAO_CTU))
    hvx.sao_apply(pv, dv, w, h, prm)
    torch.cuda.synchronize()
    del keep_org, keep_pre
    st = stats.cpu().numpy().view(_abi.SAO_STAT).reshape(nctu, 3, 5)
    outs, keep = [], True
    for d, init in zip(dd, dst_init):
        got = d.cpu().numpy()
        outs.append(got[margin:-margin, margin:-margin].copy())
        got[margin:-margin, margin:-margin] = init[margin:-margin, margin:-margin]
        keep &= np.array_equal(got, init)
    return st, outs, keep


def check_sao_golden():
    cases = gc.sao_cases(gc.load("sao.bin"))
    for k, (w, h, syn, org, pre, post, st, params) in enumerate(cases):
        got_st, got, keep = run_sao(org, pre, params, w, h)
        assert keep, k
        assert got_st.tobytes() == np.ascontiguousarray(st).tobytes(), f"record {k}: statistics"
        for c in range(3):
            np.testing.assert_array_equal(got[c], post[c], err_msg=f"record {k} plane {c}")
    return len(cases)


def sao_random_params(rng, nctu):
    rows = np.zeros((nctu, 3, 6), np.int32)
    rows[:, :, 0] = rng.integers(-1, 5, (nctu, 3))
    rows[:, :, 1] = rng.integers(0, 32, (nctu, 3))
    rows[:, :, 2:4] = rng.integers(0, 8, (nctu, 3, 2))
    rows[:, :, 4:6] = rng.integers(-7, 1, (nctu, 3, 2))
    bo = rows[:, :, 0] == 4
    rows[:, :, 2:6][bo] = rng.integers(-7, 8, (int(bo.sum()), 4))
    return _abi.sao_ctu_params(rows)


def check_sao_random(seed, w=1920, h=1080, luma_only=False):
    """random pictures (blocky, so every edge class occurs) and parameters vs the oracle."""
    rng = np.random.default_rng(seed)
    y = np.clip(np.kron(rng.integers(0, 256, (h // 4, w // 4)), np.ones((4, 4), np.int64))
                + rng.integers(-2, 3, (h, w)), 0, 255).astype(np.uint8)
    org = [np.clip(y.astype(np.int32) + rng.integers(-9, 10, y.shape), 0, 255).astype(np.uint8)]
    pre = [y, (y[::2, ::2] // 2 + 64).astype(np.uint8), (255 - y[::2, ::2]).astype(np.uint8)]
    org += [np.clip(p.astype(np.int32) + rng.integers(-5, 6, p.shape), 0, 255).astype(np.uint8) for p in pre[1:]]
    nctu = ((w + 63) // 64) * ((h + 63) // 64)
    params = sao_random_params(rng, nctu)
    st, got, keep = run_sao(org, pre, params, w, h, luma_only=luma_only)
    assert keep
    for c in range(1 if luma_only else 3):
        exp = oracle.sao_stats(org[c], pre[c], c)
        assert st[:, c].tobytes() == exp.tobytes(), f"plane {c} statistics"
        np.testing.assert_array_equal(got[c], oracle.sao_apply(pre[c], c, params), err_msg=f"plane {c}")
    return nctu


def check_coeff_write_refusals(seed):
    """Runs holding a TU the writer does not support (persistent Rice, a non-square or 64-wide TU)
    come back with length -2 and their registers and context states untouched, whatever TUs
    precede the refused one in the run; the other runs of the launch are written normally."""
    import torch
    rng = np.random.default_rng(seed)
    descs, levels, _ = random_coeff_tus(seed + 1, 12)
    descs["persistent_rice"] = 0
    descs["golomb_rice_stat"] = 0
    descs[5]["persistent_rice"] = 1   # run 1 (TUs 4..7): its second TU is refused
    descs[10]["height"] = descs[10]["width"] * 2 if descs[10]["width"] < 32 else 16  # run 2: non-square
    first = np.array([0, 4, 8, 12], np.int32)
    ns = 3
    states = rng.integers(0, 126, (ns, _abi.NUM_CTX)).astype(np.uint8)
    regs = np.zeros(ns, _abi.CABAC_REGS)
    regs[:] = _abi.CABAC_START
    off = np.concatenate([[0], np.cumsum([len(l) for l in levels])[:-1]]).astype(np.int64)
    flat = np.concatenate(levels).astype(np.int32)
    d_st = torch.from_numpy(states.reshape(-1).copy()).cuda()
    d_rg = torch.from_numpy(regs.view(np.uint8).copy()).cuda()
    cap = 1 << 16
    out = torch.zeros(ns * cap, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(ns, dtype=torch.int32, device="cuda")
    hvx.coeff_write_batch(hvx.to_device(descs), hvx.to_device(off), hvx.to_device(flat), hvx.to_device(first), ns, d_st,
                          d_rg, out, hvx.to_device(np.arange(ns, dtype=np.int64) * cap), cap, d_len)
    torch.cuda.synchronize()
    lens, r, st = d_len.cpu().numpy(), d_rg.cpu().numpy().view(_abi.CABAC_REGS), d_st.cpu().numpy().reshape(ns, -1)
    assert lens[0] >= 0 and lens[1] == -2 and lens[2] == -2, lens
    for k in (1, 2):
        assert r[k].tobytes() == regs[k].tobytes(), (k, r[k])
        np.testing.assert_array_equal(st[k], states[k], err_msg=f"run {k}")
    return True
