"""The closed-segment harness's host logic (video_codecs_amd/gop.py, cabac_init.py) on CPU: the picture
set-up it gives every picture of a closed LDP / RA segment equals the set-up HM-16.5rc1's TEncGOP gave the
same picture (tests/golden/gop_plans.json, recorded by oracle/gen_gop_plans.sh): slice QP, lambdas,
reference lists, collocated picture and its lists."""
import numpy as np
import pytest

from video_codecs_amd import cabac_init, gop, hm


def _plans():
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "gop_plans.json")))


def test_gop_depth_matches_initencslice():
    # TEncSlice.cpp:203-244: GOP 8 -> POC 8k: 0, 4: 1, 2 / 6: 2, odd: 3; GOP 4 (LDP) -> 4k: 0, 2: 1, odd: 2
    assert [gop.gop_depth(p, 8) for p in range(9)] == [0, 3, 2, 3, 1, 3, 2, 3, 0]
    assert [gop.gop_depth(p, 4) for p in range(5)] == [0, 2, 1, 2, 0]


@pytest.mark.parametrize("kind", ["ldp", "ra"])
def test_picture_setup_matches_hm(kind):
    recs = _plans()[kind]
    plan = gop.load_plan(kind, len(recs))
    cs = gop.ClosedSegments(plan, 64, 64, [32], org_fn=None)
    seg = cs.segs[0]
    for t, (g, r) in enumerate(zip(plan, recs)):
        prm, qp, entry, table, planes, col_nref = cs.picture_params(0, t)
        assert qp == r["qp"], (kind, t)
        assert prm["lambda"] == r["lambda"] and prm["lambda_motion"] == r["lambda_motion"], (kind, t, prm["lambda"], r["lambda"])
        assert list(prm["chroma_qp"]) == r["chroma_qp"]
        for l in range(2):
            assert list(prm["ref_poc"][l][:g.nref[l]]) == r["ref_poc"][l][:g.nref[l]]
        if r["col_valid"]:
            assert prm["col_valid"] == 1 and prm["col_poc"] == r["col_poc"], (kind, t)
            assert list(col_nref) == r["col_nref"]
            for l in range(2):
                assert list(prm["col_ref_poc"][l][:col_nref[l]]) == r["col_ref_poc"][l][:col_nref[l]]
        assert prm["check_ldc"] == r["check_ldc"] and prm["col_from_l0"] == r["col_from_l0"]
        # the slice-start states of the table the encoder chose (cabac_init_flag) are the library's
        np.testing.assert_array_equal(cabac_init.slice_start_states(cabac_init.resolve_table(g.slice_type, r["cabac_table"]), qp),
                                      cabac_init.ctx_init_states()[cabac_init.resolve_table(g.slice_type, r["cabac_table"]), qp])
        seg.lists[g.poc] = (tuple(g.nref), [list(g.refs[0]), list(g.refs[1])])  # what finish() records
    if kind == "ra":  # the recorded segment spans I, three GOP8s and the next intra picture (POC 32)
        assert [g.poc for g in plan[:9]] == [0, 8, 4, 2, 1, 3, 6, 5, 7] and plan[25].slice_type == gop.I_SLICE


def test_cabac_init_choice_basics():
    eb = hm._abi.load_entropy_bits()
    st = cabac_init.slice_start_states(1, 30)
    none = np.zeros(202, np.uint8)
    assert cabac_init.determine_cabac_init_idx(gop.I_SLICE, st, none, 30, eb) == gop.I_SLICE
    assert cabac_init.determine_cabac_init_idx(gop.P_SLICE, st, none, 30, eb) == gop.B_SLICE  # equal costs: B first
    allc = np.ones(202, np.uint8)
    # states equal to a table's own initial states cost less under that table
    for t in (0, 1):
        st = cabac_init.slice_start_states(t, 30)
        assert cabac_init.determine_cabac_init_idx(gop.B_SLICE, st, allc, 30, eb) == t
    assert list(cabac_init.coded_flags([1, 0, 0, 0, 0, 0, 1 << 9])[[0, 1, 201]]) == [1, 0, 1]


def test_cabac_init_choice_equals_hm():
    """determine_cabac_init_idx == HM's TEncSbac::determineCabacInitIdx (TEncSbac.cpp:162) on 3000 seeded
    writer states / coded-context sets over every QP, B and P slices (tests/golden/cabac_init_choice.bin,
    oracle/cabac_init_choice.cpp run on HM-16.5rc1's own library)."""
    import os
    rec = np.dtype([("qp", "<i4"), ("st", "<i4"), ("states", "u1", 202), ("coded", "u1", 202), ("choice", "<i4")])
    g = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", "cabac_init_choice.bin"), rec)
    assert len(g) == 3000 and set(np.unique(g["choice"])) == {gop.B_SLICE, gop.P_SLICE}
    eb = hm._abi.load_entropy_bits()
    got = [cabac_init.determine_cabac_init_idx(int(r["st"]), r["states"], r["coded"], int(r["qp"]), eb) for r in g]
    np.testing.assert_array_equal(np.array(got), g["choice"])


def test_stv_direction_map_vectorised_equals_reference_form():
    rng = np.random.default_rng(5)
    for w, h in ((128, 64), (200, 136)):
        n = ((w + 63) // 64) * ((h + 63) // 64)
        col = np.zeros((n * 16, 8), np.int16)
        col[:, 0] = np.where(rng.random(n * 16) < 0.8, 0, -1)
        col[:, 1] = np.where(rng.random(n * 16) < 0.8, rng.integers(0, 3, n * 16), -1)
        col[:, 2] = np.where(rng.random(n * 16) < 0.5, rng.integers(0, 3, n * 16), -1)
        col[:, 3:7] = rng.integers(-40, 41, (n * 16, 4))
        col[rng.random(n * 16) < 0.1, 3:5] = 0
        np.testing.assert_array_equal(gop.stv_direction_map(col, w, h), hm.stv_direction_map(col, w, h))
