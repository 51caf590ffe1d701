"""The HM-exact CTU engine (video_codecs_amd.hm -> libhvx.so hvx_hm_compress) against the
reference's own compressCtu decisions (tests/golden/ctu_ldp_*.bin, oracle/cu_capture.cpp).

Test infrastructure shared by tests/test_gpu_parity.py, __graft_entry__.smoke() and bench.py's
parity check.  Layouts of the capture arrays: oracle/cu_capture.cpp.
"""
import numpy as np

from tests import golden_cases as gc
from video_codecs_amd import _abi
from video_codecs_amd import hm

CAPTURES = ("ctu_ldp_rand.bin", "ctu_ldp_smooth.bin", "ctu_ldp_slices.bin", "ctu_ra_q22.bin", "ctu_ra_q27.bin",
            "ctu_ra_q32.bin", "ctu_ra_q37.bin")
# captures encoded with SliceMode=1 SliceArgument=<CTUs per row>: every CTU row is a slice
ROW_SLICES = {"ctu_ldp_slices.bin"}
LAST_ENGINE = [None]
# cu_capture.cpp pic_i32 / pic_f64 fields
(P_W, P_H, P_POC, P_SLICE_TYPE, P_QP, P_NREF0, P_NREF1) = range(7)
P_REFPOC0, P_REFPOC1, P_REFPIC0, P_REFPIC1 = 7, 11, 15, 19
P_COL_FROM_L0, P_COL_REF_IDX, P_CHECK_LDC, P_TMVP, P_MAX_MERGE, P_COL_POC = 23, 24, 25, 26, 27, 28
P_COL_REFPOC0, P_COL_REFPOC1 = 31, 35
P_CHROMA_QP_CB, P_CHROMA_QP_CR, P_FIRST_CTU, P_NCTU, P_LAMBDA_MOTION, P_CABAC_TABLE, P_COL_VALID = 39, 40, 41, 42, 43, 44, 45


def yuv_split(flat, w, h):
    ysz, csz = w * h, w * h // 4
    return (flat[:ysz].reshape(h, w), flat[ysz:ysz + csz].reshape(h // 2, w // 2),
            flat[ysz + csz:ysz + 2 * csz].reshape(h // 2, w // 2))


def pic_params(pi, pf):
    return {
        "poc": int(pi[P_POC]), "slice_type": int(pi[P_SLICE_TYPE]), "qp": int(pi[P_QP]),
        "nref": [int(pi[P_NREF0]), int(pi[P_NREF1])],
        "ref_poc": np.array([pi[P_REFPOC0:P_REFPOC0 + 4], pi[P_REFPOC1:P_REFPOC1 + 4]]),
        "ref_plane": np.maximum(np.array([pi[P_REFPIC0:P_REFPIC0 + 4], pi[P_REFPIC1:P_REFPIC1 + 4]]), 0),
        "chroma_qp": [int(pi[P_CHROMA_QP_CB]), int(pi[P_CHROMA_QP_CR])],
        "max_merge": int(pi[P_MAX_MERGE]), "tmvp": int(pi[P_TMVP]), "check_ldc": int(pi[P_CHECK_LDC]),
        "col_from_l0": int(pi[P_COL_FROM_L0]), "col_valid": int(pi[P_COL_VALID]), "col_poc": int(pi[P_COL_POC]),
        "col_ref_poc": np.array([pi[P_COL_REFPOC0:P_COL_REFPOC0 + 4], pi[P_COL_REFPOC1:P_COL_REFPOC1 + 4]]),
        "search_range": 64, "amp": 1, "lambda_motion": int(pi[P_LAMBDA_MOTION]) & 0xffffffff,
        "lambda": float(pf[0]), "sqrt_lambda": float(pf[1]), "chroma_weight": [float(pf[2]), float(pf[3])],
        "tq_lambda": [float(pf[4]), float(pf[5]), float(pf[6])],
    }


def hm_ctus(g, first, n):
    """The reference's final CTU data of CTUs first..first+n-1 as HM_CTU records."""
    ct = np.zeros(n, hm.HM_CTU)
    ct["p"] = hm.pack_parts(g["ctu_parts"][first:first + n])
    ct["coef"] = g["ctu_coef"][first:first + n].astype(np.int16)
    ct["bits"] = g["ctu_meta"][first:first + n, 2]
    ct["dist"] = g["ctu_meta"][first:first + n, 3]
    ct["cost"] = g["ctu_cost"][first:first + n]
    return ct


def hm_recon(g, first, w, h):
    """The reference's pre-loop-filter reconstruction of a picture (whole CTUs) from ctu_recon."""
    wc, hc = (w + 63) // 64, (h + 63) // 64
    planes = [np.zeros((hc * 64, wc * 64), np.uint8), np.zeros((hc * 32, wc * 32), np.uint8),
              np.zeros((hc * 32, wc * 32), np.uint8)]
    for a in range(wc * hc):
        r = g["ctu_recon"][first + a]
        ax, ay = a % wc, a // wc
        planes[0][ay * 64:ay * 64 + 64, ax * 64:ax * 64 + 64] = r[:4096].reshape(64, 64)
        for c in (1, 2):
            planes[c][ay * 32:ay * 32 + 32, ax * 32:ax * 32 + 32] = r[4096 + (c - 1) * 1024:4096 + c * 1024].reshape(32, 32)
    return planes


RA_CODING_ORDER = (0, 8, 4, 2, 1, 3, 6, 5, 7)  # encoder_randomaccess_main.cfg GOP8, first GOP


def stv_history(g, pic):
    """The stVSSIM history of an RA capture's picture (hvx_hm_picture.hist): the pictures coded before it
    (RA_CODING_ORDER), most recent first, each (org Y, Cb, Cr, rec Y, Cb, Cr) -- originals regenerated
    (oracle/make_yuv.py texture, the captures' input, gen_goldens.sh), reconstructions = the capture's
    final reference pictures, or for a non-reference picture the capture's own pre-loop-filter
    reconstruction (its original when the capture holds neither) -- and the direction map from the picture's collocated field (hm.stv_direction_map)."""
    from oracle import make_yuv
    pi = g["pic_i32"][pic]
    w, h = int(pi[P_W]), int(pi[P_H])
    psz = w * h * 3 // 2
    poc = int(pi[P_POC])
    order = list(RA_CODING_ORDER)
    prev = order[:order.index(poc)][::-1][:_abi.STV_HIST]
    refpoc = [int(q) for q in g["refpic_poc"]]
    cap = [int(q) for q in g["pic_i32"][:, P_POC]]
    frames = []
    for q in prev:
        org = yuv_split(np.asarray(make_yuv.texture_frame(w, h, q), np.uint8), w, h)
        if q in refpoc:
            r = refpoc.index(q)
            rec = yuv_split(g["refpic"][r * psz:(r + 1) * psz], w, h)
        elif q in cap:
            k = cap.index(q)
            full = hm_recon(g, int(g["pic_i32"][k][P_FIRST_CTU]), w, h)
            rec = (full[0][:h, :w], full[1][:h // 2, :w // 2], full[2][:h // 2, :w // 2])
        else:  # a picture the capture holds no reconstruction of: its original stands in
            rec = org
        frames.append(tuple(np.ascontiguousarray(p) for p in (*org, *rec)))
    col = None
    if int(pi[P_COL_VALID]):
        n = int(pi[P_NCTU])
        k = sum(1 for q in range(pic) if int(g["pic_i32"][q][P_COL_VALID]))
        col = g["col_field"][k * n * 16:(k + 1) * n * 16]
    return frames, hm.stv_direction_map(col, w, h)


def device_picture(g, pic, chained, entropy_bits, rd_metric=0, eta=1.0, stv_prepare=True):
    pi, pf = g["pic_i32"][pic], g["pic_f64"][pic]
    w, h = int(pi[P_W]), int(pi[P_H])
    psz = w * h * 3 // 2
    org = yuv_split(g["org"][pic * psz:(pic + 1) * psz], w, h)
    nref = len(g["refpic_poc"])
    refs = [yuv_split(g["refpic"][r * psz:(r + 1) * psz], w, h) for r in range(nref)]
    first, n = int(pi[P_FIRST_CTU]), int(pi[P_NCTU])
    col = None
    if int(pi[P_COL_VALID]):
        k = sum(1 for q in range(pic) if int(g["pic_i32"][q][P_COL_VALID]))
        col = g["col_field"][k * n * 16:(k + 1) * n * 16]
    rec = None if chained else hm_recon(g, first, w, h)
    ctus = None if chained else hm_ctus(g, first, n)
    params = pic_params(pi, pf)
    stv = None
    if rd_metric:
        params["rd_metric"], params["lambda_ssim"] = rd_metric, hm.lambda_ssim(int(pi[P_QP]), eta)
        if rd_metric == _abi.RD_STVSSIM:
            stv = hm.StvHistory(*stv_history(g, pic))
            if stv_prepare:  # the history sums precomputed (hvx_hm_stv_prepare), else summed per window
                stv.prepare(w, h)
    return hm.DevicePicture(org, refs, params, entropy_bits, rec=rec, ctus=ctus, col_field=col, stv=stv)


def run_capture(name, mode, pics=None, stage=0, rd_metric=0, eta=1.0, serial=False, stv_prepare=True):
    """Decide the captured pictures on the device.  mode 0: every CTU as its own job from the
    reference's entry state and neighbourhood; mode 1: one chained job per picture (per row slice
    for the row-sliced capture); mode 2: one chained job per picture across its row slices.  Returns
    (g, list of (pic, first, n, out_slot0), (ctus, rec, coders))."""
    g = gc.load(name)
    g["_row_slices"] = name in ROW_SLICES
    eb = _abi.load_entropy_bits()
    pics = range(g["pic_i32"].shape[0]) if pics is None else pics
    dps, jobs, plan, slot = [], [], [], 0
    for pi_idx, pic in enumerate(pics):
        pi = g["pic_i32"][pic]
        first, n = int(pi[P_FIRST_CTU]), int(pi[P_NCTU])
        dps.append(device_picture(g, pic, mode == 1, eb, rd_metric, eta, stv_prepare))
        plan.append((pic, first, n, slot))
        wc = (int(pi[P_W]) + 63) // 64
        rows = name in ROW_SLICES
        if mode == 0:
            ctus = [(a, 1) for a in range(n)]
        elif mode == 2:  # one chain over the whole picture, across its row slices (HVX_HM_SLICE_CTUS)
            ctus = [(0, n)]
        else:
            ctus = [(r, wc) for r in range(0, n, wc)] if rows else [(0, n)]
        for a, cnt in ctus:
            j = np.zeros(1, hm.HM_JOB)
            j["pic"], j["first_ctu"], j["n_ctus"], j["chained"], j["out"] = pi_idx, a, cnt, mode, slot + a
            j["entry"]["st"] = g["ctu_states"][first + a]
            j["entry"]["frac"] = np.uint64(int(g["ctu_frac"][first + a]))
            j["int2n"] = g["ctu_int2n"][first + a]
            j["flags"] = stage << 8
            if rows and mode == 2:
                j["flags"] |= _abi.hm_slice_ctus(wc)
            if rows:
                j["slice_start"], j["slice_end"] = a - a % wc, a - a % wc + wc - 1
            else:
                j["slice_start"], j["slice_end"] = 0, n - 1
            jobs.append(j)
        slot += n
    eng = hm.Engine(dps)
    LAST_ENGINE[:] = [eng]
    if serial:  # debugging aid: one launch per job, so that a faulting job is the last one announced
        for i, j in enumerate(jobs):
            print("hm_cases: launching job %d of %d" % (i, len(jobs)), flush=True)
            out = eng.compress(j, slot)
        return g, plan, out
    out = eng.compress(np.concatenate(jobs), slot)
    return g, plan, out


def run_capture_resumed(name, split):
    """The row-sliced capture decided in two launches per picture set: CTUs 0..split-1 of every
    row, then (HVX_HM_RESUME, same job slots) CTUs split..end -- the bench's stepping.  Returns
    (g, plan, out) like run_capture(mode=1)."""
    import torch
    g = gc.load(name)
    g["_row_slices"] = True
    eb = _abi.load_entropy_bits()
    npic = g["pic_i32"].shape[0]
    dps, plan, slot, rows = [], [], 0, []
    for pic in range(npic):
        pi = g["pic_i32"][pic]
        first, n = int(pi[P_FIRST_CTU]), int(pi[P_NCTU])
        wc = (int(pi[P_W]) + 63) // 64
        dps.append(device_picture(g, pic, True, eb))
        plan.append((pic, first, n, slot))
        rows += [(pic, first, r, wc, slot) for r in range(0, n, wc)]
        slot += n
    eng = hm.Engine(dps)
    LAST_ENGINE[:] = [eng]
    out_ctu = torch.zeros(slot * hm.HM_CTU.itemsize, dtype=torch.uint8, device="cuda")
    out_rec = torch.zeros(slot * 6144, dtype=torch.uint8, device="cuda")
    out_cod = torch.zeros(slot * hm.HM_CODER.itemsize, dtype=torch.uint8, device="cuda")
    for phase in (0, 1):
        j = np.zeros(len(rows), hm.HM_JOB)
        for k, (pic, first, r, wc, s0) in enumerate(rows):
            a = r if phase == 0 else r + split
            j[k]["pic"], j[k]["first_ctu"], j[k]["chained"], j[k]["out"] = pic, a, 1, s0 + a
            j[k]["n_ctus"] = split if phase == 0 else wc - split
            j[k]["slice_start"], j[k]["slice_end"] = r, r + wc - 1
            j[k]["flags"] = _abi.HM_RESUME if phase else 0
            if phase == 0:
                j[k]["entry"]["st"] = g["ctu_states"][first + r]
                j[k]["entry"]["frac"] = np.uint64(int(g["ctu_frac"][first + r]))
                j[k]["int2n"] = g["ctu_int2n"][first + r]
        jobs_t = torch.from_numpy(j.view(np.uint8).reshape(-1).copy()).cuda()
        eng.launch(jobs_t, len(rows), out_ctu, out_rec, out_cod)
    torch.cuda.synchronize()
    return g, plan, (out_ctu.cpu().numpy().view(hm.HM_CTU), out_rec.cpu().numpy().reshape(slot, 6144),
                     out_cod.cpu().numpy().view(hm.HM_CODER))


def compare_outputs(plan, out, ref_outs):
    """Mismatches (pic, ctu, what) of the engine's outputs against per-picture restatement outputs
    (oracle.hm_ctu.replay dicts, one per plan entry): every field, bit for bit (costs included)."""
    ctus, rec, _ = out
    bad = []
    for (pic, first, n, slot), ro in zip(plan, ref_outs):
        parts = hm.unpack_parts(ctus["p"][slot:slot + n])
        for a in range(n):
            c = ctus[slot + a]
            if not np.array_equal(ro["parts"][a], parts[a]):
                bad.append((pic, a, "parts"))
            elif not np.array_equal(ro["coef"][a].astype(np.int16), c["coef"]):
                bad.append((pic, a, "coef"))
            elif not np.array_equal(ro["recon"][a], rec[slot + a]):
                bad.append((pic, a, "recon"))
            elif (int(ro["bits_dist"][a][0]), int(ro["bits_dist"][a][1])) != (int(c["bits"]), int(c["dist"])):
                bad.append((pic, a, "bits/dist"))
            elif float(ro["cost"][a]) != float(c["cost"]):
                bad.append((pic, a, "cost %r vs %r" % (float(ro["cost"][a]), float(c["cost"]))))
    return bad


def name_rows(g):
    return bool(g.get("_row_slices", False))


def compare(g, plan, out):
    """Mismatches (pic, ctu, what) of the engine's outputs against the reference's CTUs (and, when
    the coders after encodeCtu are given, the context states each CTU hands the next)."""
    ctus, rec, cod = out
    bad = []
    for pic, first, n, slot in plan:
        parts = hm.unpack_parts(ctus["p"][slot:slot + n])
        for a in range(n):
            k = first + a
            hp = g["ctu_parts"][k]
            if not np.array_equal(hp, parts[a]):
                d = np.argwhere(hp != parts[a])
                z, f = int(d[0][0]), int(d[0][1])
                bad.append((pic, a, "part z=%d %s hm=%d dev=%d (%d diffs; fields %s)" % (
                    z, hm.PART_FIELDS[f], hp[z, f], parts[a][z, f], len(d), sorted({hm.PART_FIELDS[i] for i in d[:, 1]}))))
                continue
            if not np.array_equal(g["ctu_coef"][k].astype(np.int16), ctus["coef"][slot + a]):
                i = int(np.argwhere(g["ctu_coef"][k] != ctus["coef"][slot + a])[0][0])
                bad.append((pic, a, "coef idx %d" % i))
                continue
            if not np.array_equal(g["ctu_recon"][k], rec[slot + a]):
                i = int(np.argwhere(g["ctu_recon"][k] != rec[slot + a])[0][0])
                bad.append((pic, a, "recon idx %d" % i))
                continue
            c = ctus[slot + a]
            hb, hd = int(g["ctu_meta"][k][2]), int(g["ctu_meta"][k][3])
            if (hb, hd) != (int(c["bits"]), int(c["dist"])) or float(g["ctu_cost"][k]) != float(c["cost"]):
                bad.append((pic, a, "totals hm=(%d,%d,%r) dev=(%d,%d,%r)" % (hb, hd, g["ctu_cost"][k], c["bits"], c["dist"],
                                                                           c["cost"])))
                continue
            wc = (int(g["pic_i32"][pic][P_W]) + 63) // 64
            if cod is not None and a + 1 < n and not (name_rows(g) and (a + 1) % wc == 0):
                if (not np.array_equal(g["ctu_states"][k + 1], cod[slot + a]["st"])
                        or int(g["ctu_frac"][k + 1]) != int(cod[slot + a]["frac"])):
                    bad.append((pic, a, "encodeCtu state"))
    return bad


# deblocking captures of the same encodes as the CTU captures (oracle/deblock_capture.cpp,
# oracle/gen_goldens.sh): per recorded POC the picture before / after loopFilterPic, the boundary
# strengths it used and the QP map
LOOP_CAPTURES = (("ctu_ldp_rand.bin", "dbk_ldp_rand.bin"), ("ctu_ldp_smooth.bin", "dbk_ldp_smooth.bin"),
                 ("ctu_ra_q32.bin", "dbk_ra_q32.bin"))


def loop_cases(ctu_name, dbk_name):
    """Per recorded picture: dict(pic = index in the CTU capture, poc, w, h, params (hvx_deblock_params),
    pre / post (Y, Cb, Cr), bs_ver / bs_hor / qp [h/4, w/4], ref_poc [2, 4], is_b, parts [nctu, 256, 29])."""
    g, d = gc.load(ctu_name), gc.load(dbk_name)
    out, po, pu = [], 0, 0
    for i, poc in enumerate(d["poc"]):
        w, h, beta, tc, cbo, cro, bypass = (int(v) for v in d["meta"][i])
        n, nu = w * h * 3 // 2, (w // 4) * (h // 4)
        pic = [k for k in range(g["pic_i32"].shape[0]) if int(g["pic_i32"][k][P_POC]) == int(poc)][0]
        pi = g["pic_i32"][pic]
        first, nctu = int(pi[P_FIRST_CTU]), int(pi[P_NCTU])
        out.append({"pic": pic, "poc": int(poc), "w": w, "h": h,
                    "params": _abi.deblock_params(w, h, beta, tc, cbo, cro),
                    "pre": yuv_split(d["pre"][po:po + n], w, h), "post": yuv_split(d["post"][po:po + n], w, h),
                    "bs_ver": d["bs_ver"][pu:pu + nu].reshape(h // 4, w // 4),
                    "bs_hor": d["bs_hor"][pu:pu + nu].reshape(h // 4, w // 4),
                    "qp": d["qp"][pu:pu + nu].reshape(h // 4, w // 4),
                    "ref_poc": np.array([pi[P_REFPOC0:P_REFPOC0 + 4], pi[P_REFPOC1:P_REFPOC1 + 4]]),
                    "is_b": int(pi[P_SLICE_TYPE]) == 0, "parts": g["ctu_parts"][first:first + nctu]})
        po += n
        pu += nu
    return g, out


def captured_col_fields(g):
    """{poc of the collocated picture: its captured compressed motion field [nctu*16, 8]} for every
    recorded picture that reads one (cu_capture.cpp col_field)."""
    out, k = {}, 0
    for pi in g["pic_i32"]:
        if not int(pi[P_COL_VALID]):
            continue
        n = int(pi[P_NCTU])
        out[int(pi[P_COL_POC])] = g["col_field"][k * n * 16:(k + 1) * n * 16]
        k += 1
    return out


if __name__ == "__main__":  # debugging aid: python -m tests.hm_cases [mode]
    import sys
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    per_pic = len(sys.argv) > 2 and sys.argv[2] == "per_pic"
    if len(sys.argv) > 2 and sys.argv[2] == "stage":  # debugging: one picture up to one stage
        name, pic, stage = sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
        import torch
        g, plan, out = run_capture(name, mode, [pic], stage)
        dbg = LAST_ENGINE[0].last_debug
        print("stage %d ok; checks:" % stage, [(j, *dbg[j, :3]) for j in np.nonzero(dbg[:, 0])[0][:8]], flush=True)
        sys.exit(0)
    for name in CAPTURES:
        npic = gc.load(name)["pic_i32"].shape[0]
        for pics in ([[p] for p in range(npic)] if per_pic else [None]):
            print("running %s mode %d pics %s" % (name, mode, pics), flush=True)
            g, plan, out = run_capture(name, mode, pics)
            bad = compare(g, plan, out)
            n = sum(p[2] for p in plan)
            print("%s mode %d: %d/%d CTUs match" % (name, mode, n - len(bad), n), flush=True)
            for b in bad[:12]:
                print("  pic %d ctu %d: %s" % b)
            dbg = LAST_ENGINE[0].last_debug
            for j in np.nonzero(dbg[:, 0])[0][:12]:
                print("  job %d check %d a=%d b=%d" % (j, dbg[j, 0], dbg[j, 1], dbg[j, 2]))
