"""End-to-end drop-in check: the UNCHANGED reference TAppEncoder (HM-16.5rc1), with every
TComTrQuant::transformNxN / invTransformNxN call (integration/hm_tu_seam.cpp), every
TComPrediction::motionCompensation call (hm_mc_seam.cpp) and every TEncSearch::xMotionEstimation
call (hm_me_seam.cpp), every residual the slice writer codes (TEncSbac::codeCoeffNxN through
TEncBinCABAC, hm_cabac_seam.cpp), every picture's TComLoopFilter::loopFilterPic (hm_lf_seam.cpp) and SAO
statistics + offsets (hm_sao_seam.cpp, TEncSampleAdaptiveOffset::SAOProcess) and, in the
intra encodes, every TComPrediction::predIntraAng call (hm_intra_seam.cpp) served by
libhvx.so on the MI355X, must produce the same bitstream and
reconstruction MD5 as the reference CPU build (tests/hm_seam/expected_md5.json, recorded by
make_expected.py)."""
import re
import json
import os
import subprocess
import tempfile

import pytest

from tests.hm_seam import make_expected as mk

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "TAppEncoder_hvx")
EXPECTED = json.load(open(os.path.join(ROOT, "tests", "hm_seam", "expected_md5.json")))


# The leaf seams make ~1M synchronous per-call offloads per encode (correctness, not speed), and
# every leaf kernel they serve is pinned by the golden tests of test_gpu_parity.py: one intra encode
# (the intra prediction seam) and one B-slice encode (bi-prediction MC, B-slice ME, every other
# leaf seam) keep the end-to-end check inside the GPU suite's time budget.
LEAF_SEAM_CASES = ("intra_rand_qp32", "ldb_smooth_qp32")


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", LEAF_SEAM_CASES)
def test_hm_encoder_with_hvx_seams(case, monkeypatch):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.skip("TAppEncoder_hvx not built (needs /root/reference at build time)")
    intra = case.startswith("intra")
    # the intra prediction seam (hm_intra_seam.cpp) serves the intra-only encodes
    monkeypatch.setenv("HVX_SEAM_INTRA", "1" if intra else "0")
    log = []
    with tempfile.TemporaryDirectory() as tmp:
        got = mk.encode(EXE, case, tmp, log)
    print(log[0][-600:])
    assert got == EXPECTED[case], (case, got, EXPECTED[case])
    m = re.search(r"hm_me_seam: (\d+) xMotionEstimation calls served .* (\d+) fell through", log[0])
    assert m, log[0][-2000:]
    served, fell = int(m.group(1)), int(m.group(2))
    assert fell == 0
    if not case.startswith("intra"):
        assert served > 0
    # every picture's deblocking ran on the device (hm_lf_seam.cpp, hvx_deblock)
    m = re.search(r"hm_lf_seam: (\d+) pictures deblocked by libhvx, (\d+) fell through", log[0])
    assert m and int(m.group(1)) == mk.CASES[case][2] and int(m.group(2)) == 0, log[0][-2000:]
    # every picture's SAO statistics and offsets ran on the device (hm_sao_seam.cpp)
    m = re.search(r"hm_sao_seam: (\d+) pictures through libhvx SAO, (\d+) fell through", log[0])
    assert m and int(m.group(1)) == mk.CASES[case][2] and int(m.group(2)) == 0, log[0][-2000:]
    # the slice writer's residual syntax (TEncSbac::codeCoeffNxN through TEncBinCABAC) was written
    # by the device (hm_cabac_seam.cpp, hvx_coeff_write_batch): the same bitstream MD5 as above
    m = re.search(r"hm_cabac_seam: (\d+) codeCoeffNxN calls written by libhvx \((\d+) bytes\), (\d+) fell through", log[0])
    assert m and int(m.group(1)) > 100 and int(m.group(3)) == 0, log[0][-2000:]
    if intra:  # every intra prediction of the encode ran on the device
        m = re.search(r"hm_intra_seam: (\d+) predIntraAng calls served by libhvx, (\d+) fell through", log[0])
        assert m and int(m.group(1)) > 100000 and int(m.group(2)) == 0, log[0][-2000:]


def slices_of(case):
    """slices per encode: SliceMode=1 slices of SliceArgument CTUs, or one per picture"""
    frames = mk.CASES[case][2]
    w, h = mk.case_size(case)
    ctus = ((w + 63) // 64) * ((h + 63) // 64)
    extra = mk.CASES[case][6] if len(mk.CASES[case]) > 6 else []
    arg = [int(a.split("=")[1]) for a in extra if a.startswith("--SliceArgument=")]
    return frames * (-(-ctus // arg[0]) if arg else 1)


def check_slice_seam(case, log):
    """every slice of the encode was written by the device slice writer (hm_slice_seam.cpp ->
    hvx_hm_write_slices): SAO + CU syntax through the device TEncBinCABAC, 0 fall-throughs"""
    m = re.search(r"hm_slice_seam: (\d+) slices written by libhvx \((\d+) bytes\), (\d+) fell through", log)
    assert m and int(m.group(1)) == slices_of(case) and int(m.group(2)) > 0 and int(m.group(3)) == 0, log[-2000:]


DECODER = os.path.join(ROOT, "oracle", "_ref", "TAppDecoder")


def conformance(case, tmp):
    """SURVEY 4's conformance check: the reference decoder (HM-16.5rc1 TAppDecoder, built from the
    reference sources) decodes the device-written bitstream to exactly the encoder's reconstruction."""
    if not os.path.exists(DECODER):
        pytest.fail("oracle/_ref/TAppDecoder missing: the conformance check cannot run")
    dec = os.path.join(tmp, case + ".dec.yuv")
    p = subprocess.run([DECODER, "-b", os.path.join(tmp, case + ".bin"), "-o", dec], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[-2000:]
    rec = open(os.path.join(tmp, case + ".rec.yuv"), "rb").read()
    assert open(dec, "rb").read() == rec, (case, "decoded pictures differ from the encoder's reconstruction")


def test_expected_md5_cases_present():
    assert set(EXPECTED) == set(mk.CASES)


@pytest.mark.gpu
@pytest.mark.timeout(600)  # one synchronous single-CTU launch per compressCtu call: correctness, not speed
# the RA B pictures go through the batched form below (ra_texture_qp32); this synchronous form keeps
# one intra and one LDP encode inside the GPU suite's budget
@pytest.mark.parametrize("case", ["intra_rand_qp32", "ldp_rand_qp32"])
def test_hm_encoder_with_cu_seam(case, monkeypatch):
    """The L3 boundary: every TEncCu::compressCtu of an unchanged TAppEncoder encode (LDP: I + P
    pictures; RA: I + hierarchical GOP8 B pictures) served by the HM-exact CTU engine (integration/hm_cu_seam.cpp -> hvx_hm_compress),
    HM's own encodeCtu / loop filters / SAO / slice writer (with the device deblocking, SAO and
    residual-writer seams) downstream: the bitstream and reconstruction MD5 of the reference."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.skip("TAppEncoder_hvx not built (needs /root/reference at build time)")
    monkeypatch.setenv("HVX_SEAM_CU", "1")
    monkeypatch.setenv("HVX_SEAM_SLICE", "1")
    monkeypatch.setenv("HVX_SEAM_INTRA", "0")
    log = []
    with tempfile.TemporaryDirectory() as tmp:
        got = mk.encode(EXE, case, tmp, log)
        conformance(case, tmp)
    print(log[0][-600:])
    m = re.search(r"hm_cu_seam: (\d+) compressCtu calls served by libhvx \((\d+) pictures\), (\d+) fell through", log[0])
    assert m, log[0][-2000:]
    frames = mk.CASES[case][2]
    w, h = mk.case_size(case)
    ctus = ((w + 63) // 64) * ((h + 63) // 64)
    assert int(m.group(1)) == frames * ctus and int(m.group(2)) == frames and int(m.group(3)) == 0, m.group(0)
    assert got == EXPECTED[case], (case, got, EXPECTED[case])
    check_slice_seam(case, log[0])
    # with every CTU decided on the device, HM's own motion search is never reached
    m = re.search(r"hm_me_seam: (\d+) xMotionEstimation calls served .* (\d+) fell through", log[0])
    assert m is None or (int(m.group(1)) == 0 and int(m.group(2)) == 0), m.group(0)


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", ["ldp_smooth_1080p_qp32", "ra_texture_qp32", "ra_smooth_qp27", "ldp_smooth_qp32",
                                  "intra_smooth_qp22",
                                  "ldp_rand_qp4", "ldp_rand_qp51", "ldp_rand_sr16_noamp_qp32", "foreman_ldp_qp27",
                                  "foreman_ldb_qp32", "foreman_intra_qp22"])
def test_hm_encoder_with_cu_seam_batched(case, monkeypatch):
    """The throughput form of the CTU seam (HVX_SEAM_CU_BATCH=1): at each picture's first
    compressCtu call every slice of the picture is decided by ONE hvx_hm_compress launch (one chain
    per slice; the 1080p encode's CTU-row slices, its partial bottom row continuing the chain of
    the row above), and the unchanged TAppEncoder's later compressCtu calls take the kept results.
    The bitstream and reconstruction MD5 of the reference at BASELINE's 1080p size (configs 2/3)
    and on the random-access B pictures, 0 fall-throughs, one launch per picture, and the entry
    coder HM holds before every CTU equal to the state the device chain carried into it."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.skip("TAppEncoder_hvx not built (needs /root/reference at build time)")
    monkeypatch.setenv("HVX_SEAM_CU", "1")
    monkeypatch.setenv("HVX_SEAM_CU_BATCH", "1")
    monkeypatch.setenv("HVX_SEAM_SLICE", "1")
    monkeypatch.setenv("HVX_SEAM_INTRA", "0")
    log = []
    with tempfile.TemporaryDirectory() as tmp:
        got = mk.encode(EXE, case, tmp, log)
        conformance(case, tmp)
    print(log[0][-600:])
    frames = mk.CASES[case][2]
    w, h = mk.case_size(case)
    ctus = ((w + 63) // 64) * ((h + 63) // 64)
    m = re.search(r"hm_cu_seam: (\d+) compressCtu calls served by libhvx \((\d+) pictures\), (\d+) fell through", log[0])
    assert m and int(m.group(1)) == frames * ctus and int(m.group(3)) == 0, log[0][-2000:]
    m = re.search(r"hm_cu_seam batched: (\d+) CTUs from (\d+) launches, (\d+) entry-state mismatches", log[0])
    assert m and int(m.group(1)) == frames * ctus and int(m.group(2)) == frames and int(m.group(3)) == 0, log[0][-2000:]
    assert got == EXPECTED[case], (case, got, EXPECTED[case])
    check_slice_seam(case, log[0])



@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_hm_seams_fall_through_unsupported_tools(monkeypatch):
    """An encode with a tool the device path does not implement (SignHideFlag=0): the CTU seam's and
    the slice seam's tool checks refuse every picture / slice, HM's own compressCtu and encodeSlice run,
    and the bitstream and reconstruction are the reference's."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(EXE):
        pytest.skip("TAppEncoder_hvx not built (needs /root/reference at build time)")
    case = "ldp_rand_nosbh_qp32"
    monkeypatch.setenv("HVX_SEAM_CU", "1")
    monkeypatch.setenv("HVX_SEAM_CU_BATCH", "1")
    monkeypatch.setenv("HVX_SEAM_SLICE", "1")
    monkeypatch.setenv("HVX_SEAM_INTRA", "0")
    log = []
    with tempfile.TemporaryDirectory() as tmp:
        got = mk.encode(EXE, case, tmp, log)
        conformance(case, tmp)
    assert got == EXPECTED[case], (case, got, EXPECTED[case])
    m = re.search(r"hm_slice_seam: (\d+) slices written by libhvx \((\d+) bytes\), (\d+) fell through", log[0])
    assert m and int(m.group(1)) == 0 and int(m.group(3)) == slices_of(case), log[0][-2000:]
    m = re.search(r"hm_cu_seam: (\d+) compressCtu calls served by libhvx \((\d+) pictures\), (\d+) fell through", log[0])
    assert m and int(m.group(1)) == 0 and int(m.group(3)) > 0, log[0][-2000:]
