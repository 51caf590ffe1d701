"""CPU-side checks of the drop-in boundary: libhvx.so loads and exports every symbol that
include/hvx.h declares; the ABI struct mirrors match the C layouts; no compute calls."""
import ctypes
import os
import re
import subprocess

import numpy as np

from video_codecs_amd import _abi, hvx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "hvx.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void \*|const char \*)\s*(hvx_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    L = hvx.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert L.hvx_version() == 1


def test_no_gpu_is_a_loud_error():
    import torch
    if torch.cuda.is_available():
        return
    p = ctypes.c_void_p()
    rc = hvx.lib().hvx_create(0, ctypes.byref(p))
    assert rc != 0
    try:
        hvx.context()
    except hvx.HvxError:
        pass
    else:
        raise AssertionError("hvx.context() must raise without a GPU")


def test_struct_layouts_match_c():
    # compile a tiny C program printing sizeof/offsetof of the ABI structs
    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "hvx.h"
int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(hvx_tu_desc), offsetof(hvx_tu_desc, lambda),
 sizeof(hvx_estbits), sizeof(hvx_me_job), sizeof(hvx_me_result), sizeof(hvx_dist_job), sizeof(hvx_interp_job),
 sizeof(hvx_ssim_job), sizeof(hvx_stvssim_job), offsetof(hvx_me_job, lambda_motion)); return 0;}
"""
    tmp = "/tmp/hvx_layout_check"
    with open(tmp + ".c", "w") as f:
        f.write(prog)
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), tmp + ".c", "-o", tmp])
    vals = [int(x) for x in subprocess.check_output([tmp]).split()]
    assert vals == [_abi.TU_DESC.itemsize, _abi.TU_DESC.fields["lambda"][1], _abi.ESTBITS_INTS * 4,
                    _abi.ME_JOB.itemsize, _abi.ME_RESULT.itemsize, hvx.DIST_JOB.itemsize, hvx.INTERP_JOB.itemsize,
                    hvx.SSIM_JOB.itemsize, hvx.STVSSIM_JOB.itemsize, _abi.ME_JOB.fields["lambda_motion"][1]]


def test_golden_estbits_layout():
    from tests import golden_cases as gc
    g = gc.load("tu_ldp.bin")
    assert g["fwd_estbits"].shape[1] == _abi.ESTBITS_INTS


def test_estbits_update_host_golden():
    # the library's host form of TEncSbac::estBit (product code, no device) vs the reference
    from tests import golden_cases as gc
    g = gc.load("estbit.bin")
    meta, states, rice, before, after, eb = g["meta"], g["states"], g["rice"], g["before"], g["after"], g["entropy_bits"]
    for i in range(meta.shape[0]):
        w, h, ch = (int(x) for x in meta[i, :3])
        got = hvx.estbits_update(states[i], eb, rice[i], w, h, ch, before[i])
        np.testing.assert_array_equal(got, after[i], err_msg=f"record {i}")
    # invalid geometry is an error, not a silent result
    import pytest
    with pytest.raises(hvx.HvxError):
        hvx.estbits_update(states[0], eb, rice[0], 64, 64, 0, before[0])
