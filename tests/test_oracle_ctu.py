"""Pin the HM-exact CTU restatement (oracle/hvx_oracle_cu.c) against TEncCu::compressCtu
decisions captured from the reference's own LDP encodes (oracle/cu_capture.cpp ->
tests/golden/ctu_ldp_*.bin; oracle/gen_goldens.sh).  CPU only.

Every captured CTU must match HM bit for bit: the per-partition TComDataCU fields (depth,
part size, pred mode, skip/merge/merge index, inter dir, ref idx, MV, MVD, MVP idx, intra
dirs, TU depth, transform skip, cbf, QP), the quantised levels, the pre-loop-filter
reconstruction, the RD totals (bits, distortion, cost) and the context state encodeCtu
leaves for the next CTU.
"""
import pytest

from oracle import hm_ctu
from tests import golden_cases as gc
from tests import hm_cases

CAPTURES = ["ctu_ldp_rand.bin", "ctu_ldp_smooth.bin"]


def _load(name):
    import os
    return hm_ctu.load(os.path.join(os.path.dirname(__file__), "golden", name))


@pytest.mark.parametrize("name", CAPTURES)
def test_ctu_chained_vs_hm(name):
    """mode 1: the CTUs of each picture in raster order, each from the restatement's own
    encodeCtu context state (TEncSlice.cpp:727-764 carry) -- no HM state after CTU 0."""
    g = _load(name)
    for pic in range(g["pic_i32"].shape[0]):
        bad = hm_ctu.compare(g, pic, hm_ctu.replay(g, pic, mode=1), verbose=False)
        assert not bad, (name, pic, bad[:3])


def test_ctu_entry_state_vs_hm():
    """mode 0: every CTU from HM's own entry state (one P picture with skip/merge/AMP/intra)."""
    g = _load("ctu_ldp_smooth.bin")
    bad = hm_ctu.compare(g, 2, hm_ctu.replay(g, 2, mode=0), verbose=False)
    assert not bad, bad[:3]


def test_ctu_capture_covers_modes():
    """The fixtures exercise every decision branch the restatement has."""
    import numpy as np
    g = _load("ctu_ldp_smooth.bin")
    p = g["ctu_parts"].reshape(-1, 29)
    f = {n: i for i, n in enumerate(hm_ctu.PART_FIELDS)}
    assert set(np.unique(p[:, f["part"]])) >= {0, 1, 2, 4, 6, 7}  # 2Nx2N 2NxN Nx2N 2NxnU nLx2N nRx2N
    assert (p[:, f["skip"]] == 1).any() and (p[:, f["merge"]] == 1).any()
    assert (p[:, f["pred"]] == 1).any()          # intra CUs inside P pictures
    assert (p[:, f["tr_idx"]] > 0).any()         # RQT splits
    assert set(np.unique(p[:, f["depth"]])) >= {0, 1, 2, 3}


def test_ctx_init_states_vs_hm():
    """The library's slice-start states (video_codecs_amd/cabac_init.py, derived from the
    initialisation values) equal HM's own resetEntropy output for every slice type / QP
    (tests/golden/ctx_init_states.bin, oracle/ctx_init_dump.cpp) and the slice-start states the
    captures recorded."""
    import numpy as np
    from video_codecs_amd import _abi
    import os
    init = _abi.load_ctx_init_states()
    hm_dump = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", "ctx_init_states.bin"), np.uint8)
    np.testing.assert_array_equal(init, hm_dump.reshape(3, 52, 202))
    for name in CAPTURES + ["ctu_ldp_slices.bin"]:
        g = _load(name)
        wc = (int(g["pic_i32"][0][0]) + 63) // 64
        for pic in range(g["pic_i32"].shape[0]):
            pi = g["pic_i32"][pic]
            first, n, st, qp = int(pi[41]), int(pi[42]), int(pi[3]), int(pi[4])
            starts = range(0, n, wc) if name == "ctu_ldp_slices.bin" else [0]
            for a in starts:
                np.testing.assert_array_equal(g["ctu_states"][first + a], init[st, qp], err_msg=(name, pic, a))


def test_ctu_slices_vs_hm():
    """SliceMode=1 slices of one CTU row each (neighbours across the slice boundary unavailable,
    no end_of_slice bin at a slice's last CTU): chained per slice from HM's slice-start state."""
    g = _load("ctu_ldp_slices.bin")
    wc = (int(g["pic_i32"][0][0]) + 63) // 64
    for pic in range(g["pic_i32"].shape[0]):
        out = hm_ctu.replay(g, pic, mode=1, slice_ctus=wc)
        bad = hm_ctu.compare(g, pic, out, verbose=False, slice_ctus=wc)
        assert not bad, (pic, bad[:3])


def test_slice_params_vs_hm():
    """video_codecs_amd.hm.slice_params (TEncSlice::initEncSlice / setUpLambda) reproduces every
    captured picture's lambda, sqrt lambda, lambda_motion, chroma QPs / weights and TrQuant lambdas
    bit for bit (LDP GOP: QPFactor 0.4624 at POC % 4 = 1-3, 0.578 at 0; I: 0.57 * (1 - 0.05 * 3))."""
    from tests import hm_cases as hc
    from video_codecs_amd import hm
    for name in CAPTURES + ["ctu_ldp_slices.bin"]:
        g = _load(name)
        for pic in range(g["pic_i32"].shape[0]):
            pi, pf = g["pic_i32"][pic], g["pic_f64"][pic]
            st, qp, poc = int(pi[3]), int(pi[4]), int(pi[2])
            fac = 0.57 * (1 - 0.05 * 3) if st == 2 else (0.578 if poc % 4 == 0 else 0.4624)
            mine = hm.slice_params(st, qp, fac, gop_depth=0 if st == 2 else 1)
            ref = hc.pic_params(pi, pf)
            for k in ("lambda", "sqrt_lambda", "lambda_motion"):
                assert mine[k] == ref[k], (name, pic, k)
            for k in ("chroma_qp", "chroma_weight", "tq_lambda"):
                assert list(mine[k]) == list(ref[k]), (name, pic, k)


def test_hm_chains_vs_hm():
    """hvxo_hm_chains (the bench's CPU port: independent row-slice chains on host threads) on
    the sliced capture's QP 32 picture: 4 chains x 3 CTUs on 4 threads equal HM's CTUs."""
    import numpy as np
    g = _load("ctu_ldp_slices.bin")
    pic = 2
    pi, pf = g["pic_i32"][pic], g["pic_f64"][pic]
    w, h = int(pi[0]), int(pi[1])
    psz = w * h * 3 // 2
    first, n = int(pi[41]), int(pi[42])
    wc = (w + 63) // 64
    col = g["col_field"][n * 16:2 * n * 16]  # pictures 1 and 2 carry a col field; this is picture 2's
    chain_first = [r * wc for r in range(4)]
    out = hm_ctu.chains(pi, pf, g["org"][pic * psz:(pic + 1) * psz], g["refpic"], g["ctu_states"][first],
                        chain_first, 3, wc, threads=4, col_field=col)
    for k, c in enumerate(chain_first):
        for i in range(3):
            a, o = first + c + i, k * 3 + i
            np.testing.assert_array_equal(out["parts"][o], g["ctu_parts"][a], err_msg=(k, i))
            np.testing.assert_array_equal(out["coef"][o], g["ctu_coef"][a], err_msg=(k, i))
            np.testing.assert_array_equal(out["recon"][o], g["ctu_recon"][a], err_msg=(k, i))
            assert out["cost"][o] == g["ctu_cost"][a]


def test_hm_chains_rejects_bad_layout():
    g = _load("ctu_ldp_slices.bin")
    pi, pf = g["pic_i32"][2], g["pic_f64"][2]
    psz = int(pi[0]) * int(pi[1]) * 3 // 2
    with pytest.raises(ValueError):  # a chain past the picture's last CTU
        hm_ctu.chains(pi, pf, g["org"][2 * psz:3 * psz], g["refpic"], g["ctu_states"][56], [26], 3, 7,
                      col_field=g["col_field"][448:896])
    with pytest.raises(ValueError):  # TMVP on without a collocated field
        hm_ctu.chains(pi, pf, g["org"][2 * psz:3 * psz], g["refpic"], g["ctu_states"][56], [0], 1, 7)


RA_CAPTURES = ["ctu_ra_q22.bin", "ctu_ra_q27.bin", "ctu_ra_q32.bin", "ctu_ra_q37.bin"]


@pytest.mark.parametrize("name", RA_CAPTURES)
def test_ctu_ra_chained_vs_hm(name):
    """B slices (encoder_randomaccess_main.cfg, QP 22/27/32/37, textured content in motion): the
    chained restatement bit-exact on every captured B picture -- uni-L0 / uni-L1 / bi AMVP with
    the bBi refinement (TEncSearch.cpp:3096-3251), FastMEForGenBLowDelay list-1 reuse, the GPB
    picture's MvdL1Zero path, combined-bi merge candidates, L1 TMVP."""
    _replay_all(_load(name), 1, name)


def _replay_all(g, mode, name):
    """Replay every picture of a capture, the pictures on parallel threads (ctypes drops the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    npic = g["pic_i32"].shape[0]
    with ThreadPoolExecutor(max_workers=min(npic, 8)) as ex:
        outs = list(ex.map(lambda pic: hm_ctu.replay(g, pic, mode=mode), range(npic)))
    for pic, out in enumerate(outs):
        bad = hm_ctu.compare(g, pic, out, verbose=False)
        assert not bad, (name, pic, bad[:3])


def test_ctu_ra_entry_state_vs_hm():
    """mode 0 on the B pictures of the QP 22 capture: every CTU from HM's own entry state."""
    _replay_all(_load("ctu_ra_q22.bin"), 0, "ctu_ra_q22.bin")


def test_ctu_ra_capture_covers_b_modes():
    """The RA fixtures exercise the B-slice branches: every inter direction chosen by AMVP (not
    merge), bi PUs with a coded L1 MVD and GPB pictures (L1 = L0: MvdL1ZeroFlag), lists that
    share pictures (FastMEForGenB) and disjoint ones (uni-L1 candidates)."""
    import numpy as np
    f = {n: i for i, n in enumerate(hm_ctu.PART_FIELDS)}
    dirs, mvd1, gpb, shared, disjoint = set(), 0, 0, 0, 0
    for name in RA_CAPTURES:
        g = _load(name)
        p = g["ctu_parts"].reshape(-1, 29)
        amvp = (p[:, f["pred"]] == 0) & (p[:, f["merge"]] == 0)
        dirs |= set(np.unique(p[amvp, f["inter_dir"]]).tolist())
        mvd1 += int((amvp & (p[:, f["inter_dir"]] == 3) & ((p[:, f["mvd1x"]] != 0) | (p[:, f["mvd1y"]] != 0))).sum())
        for pi in g["pic_i32"]:
            n0, n1 = int(pi[5]), int(pi[6])
            l0, l1 = list(pi[7:7 + n0]), list(pi[11:11 + n1])
            gpb += int(l0 == l1)
            shared += int(bool(set(l0) & set(l1)) and l0 != l1)
            disjoint += int(any(x not in l0 for x in l1))
    assert dirs == {1, 2, 3} and mvd1 > 0 and gpb and shared and disjoint, (dirs, mvd1, gpb, shared, disjoint)


def test_slice_params_ra_vs_hm():
    """hm.slice_params for the random-access B pictures: every RA capture's lambdas, chroma QPs /
    weights and TrQuant lambdas bit for bit (encoder_randomaccess_main.cfg QPFactors: 0.442 at
    POC 8 (GOP depth 0), 0.3536 at POC 4 / 2 / 6, 0.68 at odd POCs; depth > 0 below POC 8)."""
    from tests import hm_cases as hc
    from video_codecs_amd import hm
    fac = {8: 0.442, 4: 0.3536, 2: 0.3536, 6: 0.3536, 1: 0.68, 3: 0.68, 5: 0.68, 7: 0.68}
    for name in RA_CAPTURES:
        g = _load(name)
        for pic in range(g["pic_i32"].shape[0]):
            pi, pf = g["pic_i32"][pic], g["pic_f64"][pic]
            st, qp, poc = int(pi[3]), int(pi[4]), int(pi[2])
            assert st == 0, (name, pic, st)
            mine = hm.slice_params(st, qp, fac[poc % 8 if poc % 8 else 8], gop_depth=0 if poc % 8 == 0 else 1)
            ref = hc.pic_params(pi, pf)
            for k in ("lambda", "sqrt_lambda", "lambda_motion"):
                assert mine[k] == ref[k], (name, pic, k, mine[k], ref[k])
            for k in ("chroma_qp", "chroma_weight", "tq_lambda"):
                assert list(mine[k]) == list(ref[k]), (name, pic, k)


def test_ctx_init_states_ra_vs_hm():
    """The RA captures' slice-start states are ctx_init_states.bin rows too: the B slice's own
    table, or the P table where HM's encoder set cabac_init_flag (TEncSlice::getEncCABACTableIdx,
    TEncSbac::resetEntropy swaps the B / P initialisation; the capture's table index 2 = no swap)."""
    import numpy as np
    from video_codecs_amd import _abi
    init = _abi.load_ctx_init_states()
    swapped = 0
    for name in RA_CAPTURES:
        g = _load(name)
        for pic in range(g["pic_i32"].shape[0]):
            pi = g["pic_i32"][pic]
            first, st, qp, tab = int(pi[41]), int(pi[3]), int(pi[4]), int(pi[44])
            eff = st if tab == 2 else tab
            swapped += eff != st
            np.testing.assert_array_equal(g["ctu_states"][first], init[eff, qp], err_msg=(name, pic))
    assert swapped > 0


def test_hm_chains_across_slices_vs_hm():
    """One chain over consecutive row slices (rows 1-3 of the sliced capture's QP 32 picture, 21
    CTUs): each slice restarts from the slice-start states while m_integerMv2Nx2N carries across
    the slice boundary as in TAppEncoder -- every CTU equals HM's, including the partial bottom
    row, whose boundary CTUs read the carried integer MVs."""
    import numpy as np
    g = _load("ctu_ldp_slices.bin")
    pic = 2
    pi, pf = g["pic_i32"][pic], g["pic_f64"][pic]
    w, h = int(pi[0]), int(pi[1])
    psz = w * h * 3 // 2
    first, n = int(pi[41]), int(pi[42])
    wc = (w + 63) // 64
    col = g["col_field"][n * 16:2 * n * 16]
    # the chain starts at row 0 from a zero m_integerMv2Nx2N (HM carries the previous picture's, but
    # a whole CTU's depth-0 2Nx2N searches set it before any search reads it) and runs all 4 rows
    out = hm_ctu.chains(pi, pf, g["org"][pic * psz:(pic + 1) * psz], g["refpic"], g["ctu_states"][first], [0], n, wc,
                        threads=1, col_field=col)
    for a in range(n):
        np.testing.assert_array_equal(out["parts"][a], g["ctu_parts"][first + a], err_msg=a)
        np.testing.assert_array_equal(out["coef"][a], g["ctu_coef"][first + a], err_msg=a)
        np.testing.assert_array_equal(out["recon"][a], g["ctu_recon"][first + a], err_msg=a)
        assert out["cost"][a] == g["ctu_cost"][first + a], a


def test_stv_orientation_known_answers():
    """getOrientation (stvssim.c:1317) bins of the stVSSIM direction map: x == 0 -> pi/2 (bin 16),
    y == 0 -> 0, diagonals pi/4 (bin 8) and 3pi/4 (bin 24, atan < 0 + pi), and a shallow vector."""
    from video_codecs_amd import hm
    assert hm.stv_orientation(0, 0) == 16 and hm.stv_orientation(0, -7) == 16
    assert hm.stv_orientation(5, 0) == 0 and hm.stv_orientation(-5, 0) == 0
    assert hm.stv_orientation(3, 3) == 8 and hm.stv_orientation(-3, -3) == 8
    assert hm.stv_orientation(-2, 2) == 24
    assert hm.stv_orientation(10, 1) == 1  # atan(0.1) = 0.0997 rad, nearest pi/32 = 0.0982


def test_stv_direction_map_layout():
    """hm.stv_direction_map: the z-order 16x16 blocks of a col field land on their 4x4 luma blocks;
    chooseOrient's vote (bin / 2, first maximum); intra / outside / no-motion blocks map to 0."""
    import numpy as np
    from video_codecs_amd import hm
    w, h = 128, 72
    wc, hc = 2, 2
    col = np.zeros((wc * hc * 16, 8), np.int16)
    col[:, 0] = 1  # intra everywhere
    col[:, 1:3] = -1
    # CTU 1, z-order block 3 (bx 1, by 1): L0 (0, 5) vertical -> bin 16 -> orients2[8] = pi/2
    r = 1 * 16 + 3
    col[r, 0], col[r, 1], col[r, 3], col[r, 4] = 0, 0, 0, 5
    # CTU 2 (x 0, y 64), block 0: L0 (4, 4) and L1 (-4, 4): one vote each, bins 4 and 12 -> first max = 4
    r = 2 * 16
    col[r, 0], col[r, 1], col[r, 2], col[r, 3:7] = 0, 0, 0, (4, 4, -4, 4)
    m = hm.stv_direction_map(col, w, h)
    assert m.shape == (18, 32) and m.dtype == np.float32
    f = np.float32
    assert np.all(m[4:8, 20:24] == f(f(f(3.1415926) * f(8)) / f(16)))
    assert m[16, 0] == f(f(f(3.1415926) * f(4)) / f(16))
    assert m[17, 3] == m[16, 0]  # the bottom CTU row is cut at h / 4
    m[4:8, 20:24] = 0
    m[16:18, 0:4] = 0
    assert not m.any()


def test_ctu_stvssim_cost_reads_history_and_map():
    """The restatement's stVSSIM cost (rd_metric 2, oracle cu_dstv) on an RA B picture with a 4-frame
    history: it decides differently from the plain SSIM cost, and both the history and the direction map
    change its costs (the 3-D terms read them), while a rerun is identical."""
    import numpy as np
    from oracle import hm_ctu
    from video_codecs_amd import hm
    g = gc.load("ctu_ra_q32.bin")
    pic = 1
    qp = int(g["pic_i32"][pic][hm_cases.P_QP])
    lam = hm.lambda_ssim(qp, 1.0)
    frames, dirs = hm_cases.stv_history(g, pic)
    assert len(frames) == 4 and dirs.any()
    a = hm_ctu.replay(g, pic, 1, rd_metric=2, lambda_ssim=lam, stv=(frames, dirs))
    assert np.array_equal(a["cost"], hm_ctu.replay(g, pic, 1, rd_metric=2, lambda_ssim=lam, stv=(frames, dirs))["cost"])
    s = hm_ctu.replay(g, pic, 1, rd_metric=1, lambda_ssim=lam)
    assert (a["parts"] != s["parts"]).any()
    flat = [tuple(np.zeros_like(p) for p in f) for f in frames]
    assert not np.array_equal(a["cost"], hm_ctu.replay(g, pic, 1, rd_metric=2, lambda_ssim=lam, stv=(flat, dirs))["cost"])
    assert not np.array_equal(a["cost"], hm_ctu.replay(g, pic, 1, rd_metric=2, lambda_ssim=lam,
                                                       stv=(frames, np.zeros_like(dirs)))["cost"])
