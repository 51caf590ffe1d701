"""SAO's RD decision, CPU restatement (oracle/hvx_oracle.c hvxo_sao_decide / hvxo_sao_pic_params /
hvxo_sao_update_rates) against the reference's own SAOProcess decisions (tests/golden/saodec.bin,
oracle/saodec_capture.cpp): LDP / RA / intra encodes of smooth, textured and random content at QP
22-37, temporal layers 0-3 (slice-level enables from the earlier pictures' SAO-off rates), six
row-sliced pictures with TestSAODisableAtPictureLevel."""
import numpy as np

import oracle
from tests import golden_cases as gc


def test_sao_decision_vs_reference():
    cases = gc.saodec_cases(gc.load("saodec.bin"))
    assert len(cases) == 25
    modes = np.zeros(3, np.int64)
    types = np.zeros(5, np.int64)
    for c in cases:
        en = oracle.sao_pic_params(c["layer"], c["rates_before"], c["rate"], c["rate_chroma"])
        out, recon, en_out, _ = oracle.sao_decide(c["w"], c["h"], c["stats"], c["lambdas"], en, c["sao_states"], c["frac_lo"],
                                                 c["slice_ctus"], c["test_off"])
        np.testing.assert_array_equal(out, c["params"])  # every CTU's coded mode, type, band, offsets
        assert list(en_out) == c["enabled_out"]
        np.testing.assert_array_equal(oracle.sao_update_rates(c["layer"], recon, c["rate"], c["rate_chroma"],
                                                              c["rates_before"]), c["rates_after"])
        modes += np.bincount(c["params"][:, :, 0].ravel(), minlength=3)
        p = c["params"][:, :, :2].reshape(-1, 2)
        types += np.bincount(p[p[:, 0] == 1, 1], minlength=5)
    assert (modes > 50).all() and (types > 3).all(), (modes, types)


def test_sao_picture_logic_host_vs_reference():
    """The product's host side of the SAO decision (video_codecs_amd.hm: decidePicParams' slice
    enables, the SAO-off rate update) against the captures, and the context indices of the two SAO
    contexts against the captured picture-start states (resetEntropy)."""
    from video_codecs_amd import _abi, hm
    cases = gc.saodec_cases(gc.load("saodec.bin"))
    init = _abi.load_ctx_init_states()
    for c in cases:
        en = hm.sao_slice_enabled(c["layer"], c["rates_before"], c["rate"], c["rate_chroma"])
        assert en == list(oracle.sao_pic_params(c["layer"], c["rates_before"], c["rate"], c["rate_chroma"]))
        _, recon, _, _ = oracle.sao_decide(c["w"], c["h"], c["stats"], c["lambdas"], en, c["sao_states"], c["frac_lo"],
                                           c["slice_ctus"], c["test_off"])
        np.testing.assert_array_equal(hm.sao_update_rates(c["layer"], recon, c["rates_before"], c["rate"], c["rate_chroma"]),
                                      c["rates_after"])
        # the picture-start SAO states are resetEntropy's for some slice type and QP
        assert any(init[t, q, hm.SAO_CTX_MERGE] == c["sao_states"][0] and init[t, q, hm.SAO_CTX_TYPE] == c["sao_states"][1]
                   for t in range(3) for q in range(52))
