"""The picture-level loop after compressSlice, CPU restatement (oracle/hvx_oracle_cu.c
hvxo_hm_boundary_strength / hvxo_hm_col_field) against the reference's own encodes: the boundary
strengths and QP map TComLoopFilter::loopFilterPic uses on each decided picture, the deblocked
picture they produce, and TComPic::compressMotion's field the next picture's TMVP reads.

Inputs are the reference's CTU data (tests/golden/ctu_*.bin); expected values come from the SAME
encodes' deblocking captures (tests/golden/dbk_*.bin, oracle/deblock_capture.cpp)."""
import numpy as np
import pytest

import oracle
from oracle import hm_ctu
from tests import hm_cases


@pytest.mark.parametrize("ctu_name,dbk_name", hm_cases.LOOP_CAPTURES)
def test_boundary_strength_vs_reference(ctu_name, dbk_name):
    """BS maps (vertical + horizontal, 8x8 grid) and QP map bit-exact on every recorded picture (I, P
    and B slices); the reference's pre-deblocking picture equals the CTU capture's reconstruction
    (the two captures are one encode), and the oracle's deblocking with the derived maps gives the
    reference's filtered picture."""
    g, cases = hm_cases.loop_cases(ctu_name, dbk_name)
    seen = set()
    for c in cases:
        w, h = c["w"], c["h"]
        bv, bh, qp = hm_ctu.boundary_strength(w, h, c["parts"], c["ref_poc"], c["is_b"])
        np.testing.assert_array_equal(bv, c["bs_ver"], err_msg="poc %d bs_ver" % c["poc"])
        np.testing.assert_array_equal(bh, c["bs_hor"], err_msg="poc %d bs_hor" % c["poc"])
        np.testing.assert_array_equal(qp, c["qp"].astype(np.int8), err_msg="poc %d qp" % c["poc"])
        rec = hm_cases.hm_recon(g, int(g["pic_i32"][c["pic"]][hm_cases.P_FIRST_CTU]), w, h)
        for k in range(3):
            sh = 1 if k else 0
            np.testing.assert_array_equal(rec[k][:h >> sh, :w >> sh], c["pre"][k])
        got = oracle.deblock(*[p.copy() for p in c["pre"]], bv.reshape(-1), bh.reshape(-1), qp.reshape(-1), c["params"])
        for k in range(3):
            np.testing.assert_array_equal(got[k], c["post"][k], err_msg="poc %d plane %d" % (c["poc"], k))
        seen |= set(np.unique(bv)) | set(np.unique(bh))
    assert seen >= ({0, 2} if ctu_name == "ctu_ldp_rand.bin" else {0, 1, 2})


@pytest.mark.parametrize("ctu_name", ["ctu_ldp_rand.bin", "ctu_ldp_smooth.bin"])
def test_col_field_vs_reference(ctu_name):
    """compressMotion of a recorded picture == the collocated field the reference hands the next
    recorded picture's TMVP (every 16x16 block of every CTU, outside-picture blocks included)."""
    g, _ = hm_cases.loop_cases(ctu_name, dict(hm_cases.LOOP_CAPTURES)[ctu_name])
    fields = hm_cases.captured_col_fields(g)
    n_checked = 0
    for k, pi in enumerate(g["pic_i32"]):
        poc = int(pi[hm_cases.P_POC])
        if poc not in fields:
            continue
        w, h, first, n = int(pi[hm_cases.P_W]), int(pi[hm_cases.P_H]), int(pi[hm_cases.P_FIRST_CTU]), int(pi[hm_cases.P_NCTU])
        np.testing.assert_array_equal(hm_ctu.col_field(w, h, g["ctu_parts"][first:first + n]), fields[poc])
        n_checked += 1
    assert n_checked >= 2


def test_closed_loop_references_vs_reference():
    """With SAO off (tests/golden/ctu_ldp_nosao.bin) a reference picture is the deblocked
    reconstruction: the restatement's boundary strengths from each decided picture's CTU data,
    applied by the oracle's loopFilterPic to its reconstruction, give exactly the reference
    picture the reference encoder hands the next pictures (the capture's refpic of that POC)."""
    from tests import golden_cases as gc
    from video_codecs_amd import _abi
    g = gc.load("ctu_ldp_nosao.bin")
    checked = 0
    for pic, pi in enumerate(g["pic_i32"]):
        poc, w, h = int(pi[hm_cases.P_POC]), int(pi[hm_cases.P_W]), int(pi[hm_cases.P_H])
        if poc not in list(g["refpic_poc"]):
            continue
        first, n = int(pi[hm_cases.P_FIRST_CTU]), int(pi[hm_cases.P_NCTU])
        rp = np.array([pi[hm_cases.P_REFPOC0:hm_cases.P_REFPOC0 + 4], pi[hm_cases.P_REFPOC1:hm_cases.P_REFPOC1 + 4]])
        bv, bh, qp = hm_ctu.boundary_strength(w, h, g["ctu_parts"][first:first + n], rp, int(pi[hm_cases.P_SLICE_TYPE]) == 0)
        rec = [p[:h >> (1 if c else 0), :w >> (1 if c else 0)].copy() for c, p in enumerate(hm_cases.hm_recon(g, first, w, h))]
        got = oracle.deblock(*rec, bv.reshape(-1), bh.reshape(-1), qp.reshape(-1), _abi.deblock_params(w, h))
        k = list(g["refpic_poc"]).index(poc)
        psz = w * h * 3 // 2
        want = hm_cases.yuv_split(g["refpic"][k * psz:(k + 1) * psz], w, h)
        for c in range(3):
            np.testing.assert_array_equal(got[c], want[c])
        checked += 1
    assert checked == 2
