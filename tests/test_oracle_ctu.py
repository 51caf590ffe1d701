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
    """video_codecs_amd/data/ctx_init_states.bin (TEncSbac::resetEntropy of every slice type / QP,
    oracle/ctx_init_dump.cpp) equals the slice-start states the captures recorded."""
    import numpy as np
    from video_codecs_amd import _abi
    init = _abi.load_ctx_init_states()
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
