"""HIP path (libhvx.so via the C-ABI) vs reference goldens and the CPU oracle.  MI355X only."""
import numpy as np
import pytest

import oracle
from tests import golden_cases as gc
from tests import gpu_cases
from tests import hm_cases
from video_codecs_amd import _abi, hvx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_dist_golden_gpu(torch):
    g = gc.load("dist.bin")
    meta, org, cur, wgt, out = g["meta"], g["org"], g["cur"], g["weight"], g["out"]
    n = meta.shape[0]
    jobs = np.zeros(n, hvx.DIST_JOB)
    kind_map = {0: hvx.DIST_SAD_ME, 1: hvx.DIST_SAD_ME, 2: hvx.DIST_SATD, 3: hvx.DIST_SSE, 4: hvx.DIST_SSE_W, 5: hvx.DIST_SAD}
    for i in range(n):
        k, w, h, sub = (int(x) for x in meta[i])
        jobs[i] = (kind_map[k], w, h, sub, i * 4096, i * 4096, 64, 64, wgt[i])
    d_org = torch.from_numpy(org.astype(np.int16).reshape(-1)).cuda()
    d_cur = torch.from_numpy(cur.astype(np.int16).reshape(-1)).cuda()
    d_out = torch.zeros(n, dtype=torch.int32, device="cuda")
    hvx.dist_batch(d_org, d_cur, hvx.to_device(jobs), n, d_out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_out.cpu().numpy().view(np.uint32), out)


def test_interp_golden_gpu(torch):
    g = gc.load("interp.bin")
    meta, src, out = g["meta"], g["src"], g["out"]
    n = meta.shape[0]
    jobs = np.zeros(n, hvx.INTERP_JOB)
    for i in range(n):
        is_luma, d, frac, first, last, w, h = (int(x) for x in meta[i])
        jobs[i] = (is_luma, d, frac, first, last, w, h, 0, i * 6400 + 8 * 80 + 8, i * 6400, 80, 80)
    d_src = torch.from_numpy(src.reshape(-1).copy()).cuda()
    d_dst = torch.zeros(n * 6400, dtype=torch.int16, device="cuda")
    hvx.interp_batch(d_src, d_dst, hvx.to_device(jobs), n)
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy().reshape(n, 80, 80)
    for i in range(n):
        w, h = int(meta[i][5]), int(meta[i][6])
        np.testing.assert_array_equal(got[i][:h, :w], out[i][:h, :w], err_msg=str(meta[i]))


@pytest.mark.parametrize("name", gc.TU_FILES)
def test_tu_forward_golden_gpu(torch, name):
    recs = list(gc.fwd_records(gc.load(name)))
    descs = np.concatenate([r[0] for r in recs])
    ests = np.stack([r[1] for r in recs])
    got = gpu_cases.run_tu(descs, ests, [r[2] for r in recs], "forward")
    for i, (desc, _, _, temp, lev, absum) in enumerate(recs):
        t, l, a = got[i]
        if not desc["transquant_bypass"][0]:
            np.testing.assert_array_equal(t, temp, err_msg=f"{name} {i} transform")
        np.testing.assert_array_equal(l, lev, err_msg=f"{name} {i} levels {desc}")
        assert a == absum, (name, i)


@pytest.mark.parametrize("name", gc.TU_FILES)
def test_tu_inverse_golden_gpu(torch, name):
    recs = list(gc.inv_records(gc.load(name)))
    descs = np.concatenate([r[0] for r in recs])
    got = gpu_cases.run_tu(descs, None, None, "inverse", levels_in=[r[1] for r in recs])
    for i, (_, _, res) in enumerate(recs):
        np.testing.assert_array_equal(got[i], res.reshape(-1), err_msg=f"{name} {i}")


def test_tu_pipeline_random_gpu(torch):
    assert gpu_cases.check_tu_random(seed=1234, n=600)


def test_me_golden_gpu(torch):
    assert gpu_cases.check_me_golden() > 300


def test_me_random_gpu(torch):
    assert gpu_cases.check_me_random(seed=99, n_jobs=300, width=640, height=384)


def test_me_edge_pictures_gpu(torch):
    # tiny / non-CTU-multiple pictures exercise clipMv and the border extension margins
    assert gpu_cases.check_me_random(seed=5, n_jobs=80, width=136, height=72)


def test_ssim_golden_gpu(torch):
    g = gc.load("ssim.bin")
    meta, oh, rh, dirs, out = g["meta"], g["org_hist"], g["rec_hist"], g["dirs"], g["out"]
    n = meta.shape[0]
    B = oh.shape[-1]
    jobs = np.zeros(n, hvx.SSIM_JOB)
    for i in range(n):
        w, h, wint, ov, gama, comp = (int(x) for x in meta[i])
        base = (i * 26 + 25) * B * B
        jobs[i] = (w, h, wint, ov, base, base, B, B)
    d_o = torch.from_numpy(oh.reshape(-1).copy()).cuda()
    d_r = torch.from_numpy(rh.reshape(-1).copy()).cuda()
    d_out = torch.zeros(n, dtype=torch.float32, device="cuda")
    hvx.ssim_batch(d_o, d_r, hvx.to_device(jobs), n, d_out)
    # stVSSIM
    sj = np.zeros(n, hvx.STVSSIM_JOB)
    po, pr = [], []
    for i in range(n):
        w, h, wint, ov, gama, comp = (int(x) for x in meta[i])
        used = min(gama, 26)
        sj[i] = (w, h, wint, ov, gama, comp, B, 2 * B, i * 4 * B * B)
        frames = list(range(used - 1)) + [25] + [25] * (26 - used)
        po += [d_o.data_ptr() + (i * 26 + f) * B * B for f in frames]
        pr += [d_r.data_ptr() + (i * 26 + f) * B * B for f in frames]
    d_po = torch.tensor(po, dtype=torch.int64).cuda()
    d_pr = torch.tensor(pr, dtype=torch.int64).cuda()
    d_dirs = torch.from_numpy(dirs.reshape(-1).copy()).cuda()
    d_out4 = torch.zeros(n * 4, dtype=torch.float32, device="cuda")
    hvx.stvssim_batch(d_po, d_pr, d_dirs, hvx.to_device(sj), n, d_out4)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_out.cpu().numpy(), out[:, 0])
    np.testing.assert_array_equal(d_out4.cpu().numpy().reshape(n, 4), out[:, 1:])


def test_plane_from_pel_gpu(torch):
    rng = np.random.default_rng(3)
    W, H, stride = 200, 120, 224
    pel = rng.integers(0, 256, size=(H, stride)).astype(np.int16)
    d_pel = torch.from_numpy(pel.reshape(-1).copy()).cuda()
    M = _abi.PLANE_MARGIN
    plane = torch.zeros((H + 2 * M) * (W + 2 * M), dtype=torch.uint8, device="cuda")
    hvx.plane_from_pel(d_pel, stride, W, H, plane)
    torch.cuda.synchronize()
    exp = np.pad(pel[:, :W].astype(np.uint8), M, mode="edge")
    np.testing.assert_array_equal(plane.cpu().numpy().reshape(H + 2 * M, W + 2 * M), exp)


def test_estbits_batch_golden_gpu(torch):
    g = gc.load("estbit.bin")
    meta, states, rice, before, after, eb = g["meta"], g["states"], g["rice"], g["before"], g["after"], g["entropy_bits"]
    n = meta.shape[0]
    jobs = np.zeros(n, hvx.ESTBIT_JOB)
    jobs["width"], jobs["height"], jobs["ch_type"] = meta[:, 0], meta[:, 1], meta[:, 2]
    st = np.ascontiguousarray(states[:, :hvx.NUM_CTX])
    d_st = torch.from_numpy(st.reshape(-1).copy()).cuda()
    d_eb = torch.from_numpy(eb.copy()).cuda()
    d_rc = torch.from_numpy(rice.astype(np.int32).reshape(-1).copy()).cuda()
    d_io = torch.from_numpy(before.astype(np.int32).reshape(-1).copy()).cuda()
    hvx.estbits_batch(d_st, d_eb, d_rc, hvx.to_device(jobs), n, d_io)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_io.cpu().numpy().reshape(n, -1), after)


def test_mc_random_gpu(torch):
    # uni L0/L1, bi (addAvg), identical motion with and without the B-slice shortcut, AMP and
    # 4xN/Nx4 PUs (2-wide chroma), far MVs through clipMv, every luma/chroma fractional phase
    assert gpu_cases.check_mc_random(seed=17, n=240)


def test_me_full_golden_gpu(torch):
    assert gpu_cases.check_me_full_golden() == 120


def test_coeff_bits_golden_gpu(torch):
    # codeCoeffNxN rate on the device, one TU per lane: the 3154 captured reference calls
    g = gc.load("cabac.bin")
    descs, levels = gc.cabac_cases(g)
    n = len(levels)
    off = np.asarray(g["coef_off"][:n], np.int64)
    flat = np.concatenate(levels).astype(np.int32)
    d_st = torch.from_numpy(np.ascontiguousarray(g["states_before"]).reshape(-1).copy()).cuda()
    out = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    hvx.coeff_bits_batch(hvx.to_device(descs), hvx.to_device(off), n, hvx.to_device(flat),
                         hvx.to_device(g["entropy_bits"].astype(np.int32)), d_st, out)
    torch.cuda.synchronize()
    r = out.cpu().numpy().view(hvx._abi.COEFF_BITS)
    np.testing.assert_array_equal(r["frac_bits"].astype(np.int64), g["frac"][:, 1] - g["frac"][:, 0])
    np.testing.assert_array_equal(r["rice_stat"], g["rice_after"].astype(np.uint32))
    np.testing.assert_array_equal(r["num_sig"], [np.count_nonzero(l) for l in levels])
    np.testing.assert_array_equal(d_st.cpu().numpy().reshape(n, -1), g["states_after"])


def test_coeff_bits_random_gpu(torch):
    # random levels (sparse, dense, large escapes; every size / scan / channel / transform skip,
    # persistent Rice adaptation on and off) and random context states vs the oracle
    assert gpu_cases.check_coeff_bits_random(seed=23, n=700)


def test_coeff_write_golden_gpu(torch):
    # the CABAC residual writer (TEncBinCABAC) on the device: the 2623 captured reference calls,
    # each from its captured registers and context states -> bytes, registers, states
    assert gpu_cases.check_coeff_write_golden() == 2623


def test_coeff_write_random_gpu(torch):
    # 200 runs of 0..12 random TUs (every size / scan / channel, transform skip, bypass, sign
    # hiding, extended-precision escapes) from start() vs the oracle, TU by TU, with the
    # contexts each run coded (hvx_cabac_regs.coded)
    n_tu, n_bytes = gpu_cases.check_coeff_write_random(seed=41, n_streams=200, max_tus=12)
    assert n_tu > 1000 and n_bytes > 100000


def test_coeff_write_refusals_gpu(torch):
    # a run holding an unsupported TU (persistent Rice, non-square) is refused before anything is
    # coded: length -2, registers and context states untouched
    assert gpu_cases.check_coeff_write_refusals(seed=5)


def test_intra_reference_samples_golden_gpu(torch):
    # initIntraPatternChType: 1188 captured reference borders (unfiltered + smoothed), every size
    # and availability pattern; unavailable neighbour positions hold random bytes
    assert gpu_cases.check_intra_ref_golden() == 1188


def test_intra_first_pass_golden_gpu(torch):
    # estIntraPredLumaQT's first pass: 642 captured PUs (SATD of 35 modes, rates, ranking, MPMs)
    assert gpu_cases.check_intra_first_pass_golden() == 642


def test_intra_random_gpu(torch):
    # random luma/chroma blocks 4..64, random availability (none / all / sparse / dense), every mode
    n, n_luma = gpu_cases.check_intra_random(seed=31, n_jobs=600)
    assert n == 600 and n_luma > 200


def test_deblock_golden_gpu(torch):
    # loopFilterPic: 9 captured reference pictures (intra, LDP, LDB, random P, offsets), Y/Cb/Cr
    assert gpu_cases.check_deblock_golden() == 9


def test_deblock_random_gpu(torch):
    # 1080p random BS / QP maps and offsets vs the oracle; plane borders must stay untouched
    assert gpu_cases.check_deblock_random(seed=41) > 10000


def test_sao_golden_gpu(torch):
    # SAOProcess: 8 records (5 encoder-decided pictures, 3 random parameter sets through the
    # reference's offsetCTU), statistics of every CTU / component / type + Y/Cb/Cr after SAO
    assert gpu_cases.check_sao_golden() == 8


def test_sao_random_gpu(torch):
    # 1080p and 1000x600 (partial CTUs on both axes) blocky pictures, random parameters vs the
    # oracle; luma-only form; destination borders untouched
    assert gpu_cases.check_sao_random(seed=51) == 510
    assert gpu_cases.check_sao_random(seed=52, w=1000, h=600) == 160
    assert gpu_cases.check_sao_random(seed=53, w=512, h=256, luma_only=True) == 32


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("name", hm_cases.CAPTURES)
def test_hm_ctu_golden_gpu(torch, name, mode):
    """hvx_hm_compress vs the reference's compressCtu + encodeCtu on every captured CTU: mode 0 each
    CTU from HM's entry state and neighbourhood, mode 1 whole pictures chained on the device."""
    g, plan, out = hm_cases.run_capture(name, mode)
    bad = hm_cases.compare(g, plan, out)
    assert not bad, bad[:5]


@pytest.mark.gpu
def test_hm_ctu_multislice_gpu(torch):
    """HVX_HM_SLICE_CTUS: one chain per picture over its row slices (each slice restarting from the
    slice-start states, m_integerMv2Nx2N carried across slice boundaries as in TAppEncoder);
    bit-exact vs HM on every CTU of the row-sliced capture."""
    g, plan, out = hm_cases.run_capture("ctu_ldp_slices.bin", 2)
    bad = hm_cases.compare(g, plan, out)
    assert not bad, bad[:5]


@pytest.mark.gpu
def test_hm_ctu_resume_gpu(torch):
    """HVX_HM_RESUME (the bench's stepping): every row slice decided in two launches, the second
    continuing from the CABAC state and m_integerMv2Nx2N the first left in the job's state slot;
    bit-exact vs HM."""
    g, plan, out = hm_cases.run_capture_resumed("ctu_ldp_slices.bin", 3)
    bad = hm_cases.compare(g, plan, out)
    assert not bad, bad[:5]


@pytest.mark.gpu
@pytest.mark.parametrize("name,eta", [("ctu_ra_q37.bin", 1.3)])  # the active cost's sweep: test_hm_ctu_stvssim_rdo_gpu
def test_hm_ctu_ssim_rdo_gpu(torch, name, eta):
    """BASELINE config 4's cost inside the real decision: hvx_hm_compress with HVX_RD_SSIM (TEncCu's
    mode / split comparisons on J = D_ssim + lambda_2(QP) * eta^0.85 * max(0.5, R), stvssim.c:567,
    :1805, rdopt.c:1631) on the RA B pictures at QP 22 / 27 / 32 / 37, chained per picture, against
    the restatement with the same cost (oracle/hvx_oracle_cu.c cu_dssim / cu_cost): every decision,
    coefficient, reconstruction sample, bit count, distortion and cost bit-exact (the SSIM floats
    and the double cost included, tighter than north_star's 1e-6); and the cost changes decisions
    against HM's SSE cost."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import hm_ctu
    from video_codecs_amd import hm
    g, plan, out = hm_cases.run_capture(name, 1, rd_metric=1, eta=eta)

    def ref(p):
        qp = int(g["pic_i32"][p[0]][hm_cases.P_QP])
        return hm_ctu.replay(g, p[0], 1, rd_metric=1, lambda_ssim=hm.lambda_ssim(qp, eta))
    with ThreadPoolExecutor(max_workers=8) as ex:
        refs = list(ex.map(ref, plan))
    bad = hm_cases.compare_outputs(plan, out, refs)
    assert not bad, bad[:5]
    assert hm_cases.compare(g, plan, out), "the SSIM cost decided exactly as HM's SSE cost"


@pytest.mark.gpu
@pytest.mark.parametrize("name,eta,prep", [("ctu_ra_q22.bin", 1.0, True), ("ctu_ra_q27.bin", 0.7, True),
                                           ("ctu_ra_q32.bin", 1.0, True), ("ctu_ra_q37.bin", 1.3, False)])
def test_hm_ctu_stvssim_rdo_gpu(torch, name, eta, prep):
    """BASELINE config 4 with the reference's ACTIVE cost (att_stv.h:5 -> distortionstVSSIM,
    stvssim.c:831-855): hvx_hm_compress with HVX_RD_STVSSIM on the RA B pictures at QP 22 / 27 / 32 / 37,
    each with its stVSSIM history (the pictures coded before it, tests/hm_cases.stv_history: up to 4
    previous frames here) and direction map, chained per picture, against the restatement (cu_dstv
    through the pinned hvxo_stvssim): every decision, coefficient, reconstruction sample, bit count,
    distortion and double cost bit-exact; and the cost decides differently from HM's SSE cost.  prep:
    the history part of the window sums precomputed per picture (hvx_hm_stv_prepare), else summed by
    the engine per window."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import hm_ctu
    from video_codecs_amd import _abi, hm
    g, plan, out = hm_cases.run_capture(name, 1, rd_metric=_abi.RD_STVSSIM, eta=eta, stv_prepare=prep)

    def ref(p):
        qp = int(g["pic_i32"][p[0]][hm_cases.P_QP])
        return hm_ctu.replay(g, p[0], 1, rd_metric=_abi.RD_STVSSIM, lambda_ssim=hm.lambda_ssim(qp, eta),
                             stv=hm_cases.stv_history(g, p[0]))
    with ThreadPoolExecutor(max_workers=8) as ex:
        refs = list(ex.map(ref, plan))
    bad = hm_cases.compare_outputs(plan, out, refs)
    assert not bad, bad[:5]
    assert hm_cases.compare(g, plan, out), "the stVSSIM cost decided exactly as HM's SSE cost"


@pytest.mark.gpu
def test_hm_compress_refuses_bad_jobs(torch):
    """hvx_hm_compress's device-side preconditions (include/hvx.h): jobs with a picture index, CTU
    range, slice range or output slot out of range are skipped with their HVX_HM_BAD_* status --
    nothing of theirs is written -- while a valid job of the same launch runs bit-exactly."""
    import numpy as np
    from tests import golden_cases as gc
    from video_codecs_amd import _abi, hm
    g = gc.load("ctu_ldp_rand.bin")
    pic = 1
    pi = g["pic_i32"][pic]
    first = int(pi[hm_cases.P_FIRST_CTU])
    eb = _abi.load_entropy_bits()
    eng = hm.Engine([hm_cases.device_picture(g, pic, False, eb)])
    n = 28

    def job(**kw):
        j = np.zeros(1, hm.HM_JOB)
        j["pic"], j["first_ctu"], j["n_ctus"], j["chained"], j["out"] = 0, 5, 1, 0, 0
        j["slice_start"], j["slice_end"] = 0, n - 1
        j["entry"]["st"] = g["ctu_states"][first + 5]
        j["entry"]["frac"] = np.uint64(int(g["ctu_frac"][first + 5]))
        j["int2n"] = g["ctu_int2n"][first + 5]
        for k, v in kw.items():
            j[k] = v
        return j
    jobs = np.concatenate([job(out=0), job(pic=1, out=1), job(first_ctu=n, out=2), job(n_ctus=0, out=3),
                           job(slice_start=6, out=4), job(slice_end=n, out=5), job(out=6), job(first_ctu=-1, out=0)])
    out_ctu, out_rec, _ = eng.compress(jobs, 6)  # 6 output slots: job 6 (out=6) is out of range
    st = eng.job_status(len(jobs))
    assert list(st) == [0, -1, -5, -5, -5, -5, -6, -5], list(st)
    # the valid job's CTU equals the reference's; the refused jobs' slots stay untouched (zero)
    parts = hm.unpack_parts(out_ctu["p"][0:1])
    assert np.array_equal(parts[0], g["ctu_parts"][first + 5])
    assert not out_rec[1:6].any() and not out_ctu["coef"][1:6].any()


@pytest.mark.gpu
@pytest.mark.parametrize("ctu_name,dbk_name", hm_cases.LOOP_CAPTURES)
def test_hm_finish_picture_gpu(torch, ctu_name, dbk_name):
    """The reference loop on the device: every picture of the capture decided by hvx_hm_compress
    (chained), then hvx_hm_finish_picture -- boundary strengths + QP map derived from the engine's own
    CTU data, loopFilterPic in place, compressMotion, the border-extended reference planes -- against
    the same encode's loopFilterPic capture (BS maps, filtered picture), the restatement's field and the
    padded planes the next picture would read: all bit-exact, for I, P and B pictures."""
    from oracle import hm_ctu
    from video_codecs_amd import hm
    g, plan, out = hm_cases.run_capture(ctu_name, 1)
    assert not hm_cases.compare(g, plan, out)
    eng = hm_cases.LAST_ENGINE[0]
    _, cases = hm_cases.loop_cases(ctu_name, dbk_name)
    fields = hm_cases.captured_col_fields(g)
    for c in cases:
        w, h = c["w"], c["h"]
        dp = eng.pictures[c["pic"]]
        ref = hm.DeviceFrame.blank(w, h)
        work, col = hm.finish_picture(dp, c["params"], col_field=True, ref_frame=ref)
        torch.cuda.synchronize()
        wk = work.cpu().numpy()
        np.testing.assert_array_equal(wk[0], c["bs_ver"], err_msg="poc %d bs_ver" % c["poc"])
        np.testing.assert_array_equal(wk[1], c["bs_hor"], err_msg="poc %d bs_hor" % c["poc"])
        np.testing.assert_array_equal(wk[2].view(np.int8), c["qp"].astype(np.int8))
        for k in range(3):
            sh = 1 if k else 0
            rec = dp.rec_t[k].cpu().numpy()[:h >> sh, :w >> sh]
            np.testing.assert_array_equal(rec, c["post"][k], err_msg="poc %d plane %d" % (c["poc"], k))
        want = hm_ctu.col_field(w, h, c["parts"])
        np.testing.assert_array_equal(col.cpu().numpy(), want)
        if c["poc"] in fields:
            np.testing.assert_array_equal(col.cpu().numpy(), fields[c["poc"]])
        y8, y16, cb16, cr16 = (t.cpu().numpy() for t in ref.planes())
        m8 = hm.DeviceFrame.M8
        np.testing.assert_array_equal(y8, np.pad(c["post"][0], m8, mode="edge"))
        np.testing.assert_array_equal(y16, np.pad(c["post"][0], 80, mode="edge").astype(np.int16))
        np.testing.assert_array_equal(cb16, np.pad(c["post"][1], 40, mode="edge").astype(np.int16))
        np.testing.assert_array_equal(cr16, np.pad(c["post"][2], 40, mode="edge").astype(np.int16))


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(200, 176), (136, 184)])
def test_hm_partial_ctus_gpu(torch, w, h):
    """Pictures whose right CTU column and bottom CTU row are both partial (8 / 56 px wide, 48 / 56
    lines high), decided the bench's way (HmWorkload: one chain per row slice, the partial bottom row
    continuing the chain of the row above) to the end of the picture: every CTU equal to the
    restatement's (boundary-forced splits, clipped search windows and MVs, TMVP at the edges)."""
    import bench
    hvx.context()
    r = bench.hm_merged_chain_parity(4, W=w, H=h)
    assert r["gpu_parity_mismatches"] == 0, r["first_mismatches"]
    assert r["ctus"] == ((w + 63) // 64) * ((h + 63) // 64)


@pytest.mark.gpu
@pytest.mark.parametrize("base_qp", [0, 49])
def test_hm_extreme_qp_gpu(torch, base_qp):
    """The decision at the ends of the QP range (slice QP 2 and 51: the bench picture's GOP offset on
    base QP 0 / 49) on random content: at QP 2 the levels run into the thousands (escape codes with
    the Rice parameter at its cap, RDOQ's max / max-1 candidates far from 0), at QP 51 almost every
    level is 0 -- a 256x176 picture decided to the end, every CTU equal to the restatement's."""
    import bench
    hvx.context()
    r = bench.hm_merged_chain_parity(4, base_qp=base_qp)
    assert r["gpu_parity_mismatches"] == 0, r["first_mismatches"]


@pytest.mark.gpu
def test_closed_loop_segments_gpu(torch):
    """The bench's closed-segment figures in miniature (bench.ClosedWorkload, the per-rank workload of the
    multi-GPU bench): config 5 -- two LDP segments of 256x192 random pictures (I, P, P), every P picture
    decided against the references, collocated field and cabac_init table the device loop made
    (deblocking + SAO + slice writer), the chains stepped 2 CTUs per launch -- and config 4 -- two RA
    segments of 128x64 (I, POC 8, POC 4) with the stVSSIM cost over their own history; each figure's last
    picture re-decided by the restatement from the device's references, field and history: every CTU equal."""
    import bench
    hvx.context()
    r = bench.config5_measure(4, W=256, H=192, segs=2, pics=3, ctus_step=2)
    assert [p["slice"] for p in r["pictures"]] == ["I", "P", "P"]
    assert all(p["slice_data_bytes"] > 0 for p in r["pictures"])
    par = r["parity"]["seg0_poc2"]
    assert par["ctus"] == 12 and par["mismatches"] == 0, par["first_mismatches"]
    r = bench.config4_measure(4, W=128, H=64, segs_per_qp=1, qps=(27, 37), pics=3, ctus_step=1)
    assert [p["poc"] for p in r["pictures"]] == [0, 8, 4] and [p["slice"] for p in r["pictures"]] == ["I", "B", "B"]
    for q in ("qp27", "qp37"):
        assert r["parity"][q]["ctus"] == 2 and r["parity"][q]["mismatches"] == 0, r["parity"][q]


@pytest.mark.gpu
def test_hm_closed_loop_gpu(torch):
    """A GOP segment run entirely on the device (SAO off, tests/golden/ctu_ldp_nosao.bin): the I
    picture decided by hvx_hm_compress, finished by hvx_hm_finish_picture (deblocking from the
    engine's own CTU data, compressMotion, padded reference planes); each P picture then decided
    against the references and the collocated field the device produced -- no reference-encoder
    data enters after the first picture except the originals and the slice-start states.  Every
    CTU of every picture bit-exact vs HM, and each device reference plane equals the reference
    picture HM handed the next pictures."""
    from video_codecs_amd import _abi, hm
    g = gc.load("ctu_ldp_nosao.bin")
    g["_row_slices"] = False
    eb = _abi.load_entropy_bits()
    refs_by_poc, cols_by_poc = {}, {}
    for pic, pi in enumerate(g["pic_i32"]):
        poc, w, h = int(pi[hm_cases.P_POC]), int(pi[hm_cases.P_W]), int(pi[hm_cases.P_H])
        first, n = int(pi[hm_cases.P_FIRST_CTU]), int(pi[hm_cases.P_NCTU])
        psz = w * h * 3 // 2
        org = hm_cases.yuv_split(g["org"][pic * psz:(pic + 1) * psz], w, h)
        params = hm_cases.pic_params(pi, g["pic_f64"][pic])
        nref0 = int(pi[hm_cases.P_NREF0])
        refs = [refs_by_poc[int(p)] for p in g["refpic_poc"] if int(p) in refs_by_poc]
        assert all(int(g["refpic_poc"][params["ref_plane"][0][i]]) in refs_by_poc for i in range(nref0))
        col = cols_by_poc[int(pi[hm_cases.P_COL_POC])] if int(pi[hm_cases.P_COL_VALID]) else None
        dp = hm.DevicePicture(org, refs, params, eb, col_field=col)
        job = np.zeros(1, hm.HM_JOB)
        job["pic"], job["first_ctu"], job["n_ctus"], job["chained"], job["out"] = 0, 0, n, 1, 0
        job["entry"]["st"] = g["ctu_states"][first]
        job["entry"]["frac"] = np.uint64(int(g["ctu_frac"][first]))
        job["int2n"] = g["ctu_int2n"][first]
        job["slice_start"], job["slice_end"] = 0, n - 1
        out = hm.Engine([dp]).compress(job, n)
        bad = hm_cases.compare(g, [(pic, first, n, 0)], out)
        assert not bad, (poc, bad[:4])
        ref = hm.DeviceFrame.blank(w, h)
        _, col_t = hm.finish_picture(dp, _abi.deblock_params(w, h), col_field=True, ref_frame=ref)
        torch.cuda.synchronize()
        refs_by_poc[poc], cols_by_poc[poc] = ref, col_t
        if poc in list(g["refpic_poc"]):
            k = list(g["refpic_poc"]).index(poc)
            want = hm_cases.yuv_split(g["refpic"][k * psz:(k + 1) * psz], w, h)
            y8, y16, cb16, cr16 = (t.cpu().numpy() for t in ref.planes())
            m8 = hm.DeviceFrame.M8
            np.testing.assert_array_equal(y8[m8:m8 + h, m8:m8 + w], want[0])
            np.testing.assert_array_equal(y16[80:80 + h, 80:80 + w], want[0].astype(np.int16))
            np.testing.assert_array_equal(cb16[40:40 + h // 2, 40:40 + w // 2], want[1].astype(np.int16))
            np.testing.assert_array_equal(cr16[40:40 + h // 2, 40:40 + w // 2], want[2].astype(np.int16))
    assert len(refs_by_poc) == 3


@pytest.mark.gpu
def test_sao_decide_gpu(torch):
    """hvx_sao_decide (SAO's RD decision, one wave per picture) on all 25 captured SAOProcess
    decisions at once: every CTU's coded mode / type / band / offsets, the merge-resolved parameters
    (vs the restatement), the slice-enabled flags after the picture-level test, and the total cost
    bit for bit."""
    import oracle
    cases = gc.saodec_cases(gc.load("saodec.bin"))
    eb = torch.from_numpy(_abi.load_entropy_bits().astype(np.int32)).cuda()
    keep, jobs = [], np.zeros(len(cases), _abi.SAO_DECIDE_JOB)
    for i, c in enumerate(cases):
        en = oracle.sao_pic_params(c["layer"], c["rates_before"], c["rate"], c["rate_chroma"])
        st = torch.from_numpy(np.ascontiguousarray(c["stats"].astype(np.int64))).cuda()
        coded = torch.zeros((c["nctu"], 3, 8), dtype=torch.int32, device="cuda")
        recon = torch.zeros(c["nctu"] * _abi.SAO_CTU.itemsize, dtype=torch.uint8, device="cuda")
        en_out = torch.zeros(3, dtype=torch.int32, device="cuda")
        tot = torch.zeros(1, dtype=torch.float64, device="cuda")
        keep.append((st, coded, recon, en_out, tot, en))
        j = jobs[i]
        j["pic_w"], j["pic_h"], j["slice_ctus"], j["test_off"] = c["w"], c["h"], c["slice_ctus"], c["test_off"]
        j["slice_enabled"], j["frac_lo"], j["sao_states"], j["lambda"] = en, c["frac_lo"], c["sao_states"], c["lambdas"]
        j["stats"], j["entropy_bits"], j["coded"] = st.data_ptr(), eb.data_ptr(), coded.data_ptr()
        j["recon"], j["slice_enabled_out"], j["total_cost"] = recon.data_ptr(), en_out.data_ptr(), tot.data_ptr()
    jobs_t = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    hvx.sao_decide(jobs_t, len(cases))
    torch.cuda.synchronize()
    for c, (st, coded, recon, en_out, tot, en) in zip(cases, keep):
        np.testing.assert_array_equal(coded.cpu().numpy(), c["params"])
        assert list(en_out.cpu().numpy()) == c["enabled_out"]
        o_coded, o_recon, o_en, o_tot = oracle.sao_decide(c["w"], c["h"], c["stats"], c["lambdas"], en, c["sao_states"],
                                                          c["frac_lo"], c["slice_ctus"], c["test_off"])
        assert recon.cpu().numpy().tobytes() == o_recon.tobytes()
        assert float(tot.cpu().numpy()[0]) == o_tot
